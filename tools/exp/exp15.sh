set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests15.log 2>&1 || { tail -40 gpurun_out/gpu_tests15.log; exit 1; }
tail -1 gpurun_out/gpu_tests15.log
for c in c2 c5; do
rm -rf gpurun_out/tb_$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tb_$c -o tb --output-format csv -- python tools/trace_bench.py $c > gpurun_out/tb_$c.log 2>&1
grep -v amdgpu gpurun_out/tb_$c.log
for f in $(find gpurun_out/tb_$c -name "*kernel_stats.csv"); do grep -E "trace_kernel|screen|exact" "$f" | cut -d, -f1,2,4 | sed 's/(sphrt::GridDev[^"]*//'; done
done
