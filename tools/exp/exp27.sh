set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests27.log 2>&1 || { tail -40 gpurun_out/gpu_tests27.log; exit 1; }
tail -1 gpurun_out/gpu_tests27.log
for c in c3 c5 c2; do
rm -rf gpurun_out/tb_$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tb_$c -o tb --output-format csv -- python tools/trace_bench.py $c > gpurun_out/tb_$c.log 2>&1
grep operator gpurun_out/tb_$c.log
done
