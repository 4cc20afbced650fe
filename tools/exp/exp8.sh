set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp8/gpu_tests.log 2>&1 || { tail -40 gpurun_out/exp8/gpu_tests.log; exit 1; }
tail -1 gpurun_out/exp8/gpu_tests.log
for c in c2 c5 c3; do timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 > gpurun_out/exp8/apply_$c.log 2>&1; grep -v amdgpu.ids gpurun_out/exp8/apply_$c.log | cut -c1-120; done
