set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests23.log 2>&1 || { tail -40 gpurun_out/gpu_tests23.log; exit 1; }
tail -1 gpurun_out/gpu_tests23.log
timeout -k 10 300 python tools/retrieval_bench.py --out gpurun_out/r01_retrieval_c5.json 2>&1 | grep -v amdgpu
rm -rf gpurun_out/rprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rprof -o r --output-format csv -- python tools/retrieval_bench.py --iters 20 > /dev/null 2>&1
