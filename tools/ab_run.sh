set -e
bash tools/gpu_check.sh r04
for c in c3 c5 c2; do bash tools/ab_variants.sh $c "trace_kernel" mpath; done
python tools/ab_table.py gpurun_out/ab "trace_kernel|local_table_radix|compact|screen|exact_wave" c3 c5 c2
