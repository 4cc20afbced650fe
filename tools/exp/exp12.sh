set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests12.log 2>&1 || { tail -40 gpurun_out/gpu_tests12.log; exit 1; }
tail -1 gpurun_out/gpu_tests12.log
for c in c2 c5; do timeout -k 10 200 python tools/cold_breakdown.py --config $c 2>&1 | grep -v amdgpu; done
timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | cut -c1-300
