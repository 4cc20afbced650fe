set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests30.log 2>&1 || { tail -40 gpurun_out/gpu_tests30.log; exit 1; }
tail -1 gpurun_out/gpu_tests30.log
timeout -k 10 300 python bench.py --config c4 --steps 50 --warmup 5 --cpu-sample-views 2 --cpu-reps 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
cut -c1-300 gpurun_out/bench_c4.json
