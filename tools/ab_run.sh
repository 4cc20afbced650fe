set -e
bash tools/gpu_check.sh r04
for c in c5 c2 c3; do bash tools/ab_env.sh $c staged="SPHRT_TABLE_STAGED=1" compact="SPHRT_TABLE_STAGED=0"; done
python tools/ab_table.py gpurun_out/ab "trace_kernel|local_table|compact|screen|exact_wave" c3 c5 c2
