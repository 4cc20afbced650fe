set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp7/gpu_tests.log 2>&1 || { tail -30 gpurun_out/exp7/gpu_tests.log; exit 1; }
tail -1 gpurun_out/exp7/gpu_tests.log
timeout -k 10 120 python tools/host_overhead.py
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp7/bench.json 2> gpurun_out/exp7/bench.err
cut -c1-400 gpurun_out/exp7/bench.json
