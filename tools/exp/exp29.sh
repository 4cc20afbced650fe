set -e
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c4 --steps 50 --warmup 5 --cpu-sample-views 2 --cpu-reps 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
