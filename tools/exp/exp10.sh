set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests10.log 2>&1 || { tail -40 gpurun_out/gpu_tests10.log; exit 1; }
tail -1 gpurun_out/gpu_tests10.log
for c in c2 c5 c3; do
echo "== $c"; timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 2>&1 | grep -v amdgpu | grep -v atomic | cut -c1-100
done
