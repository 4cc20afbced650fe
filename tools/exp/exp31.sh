set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests31.log 2>&1 || { tail -40 gpurun_out/gpu_tests31.log; exit 1; }
tail -1 gpurun_out/gpu_tests31.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
