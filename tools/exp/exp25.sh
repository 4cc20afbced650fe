set -e
export TMPDIR=/tmp
timeout -k 10 300 python tools/retrieval_bench.py --out gpurun_out/r01_retrieval_c5.json 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -q -k gd --timeout 120 --timeout-method thread 2>&1 | tail -1
