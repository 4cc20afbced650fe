set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests16.log 2>&1 || { tail -40 gpurun_out/gpu_tests16.log; exit 1; }
tail -1 gpurun_out/gpu_tests16.log
for c in c2 c5; do
rm -rf gpurun_out/tb_$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tb_$c -o tb --output-format csv -- python tools/trace_bench.py $c > gpurun_out/tb_$c.log 2>&1
done
rm -rf gpurun_out/tpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/tpmc -o p --output-format csv -- python tools/trace_bench.py c2 --reps 1 > gpurun_out/tpmc.log 2>&1
