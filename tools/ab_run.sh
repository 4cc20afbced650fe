set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log
for r in 1 2; do for c in c2 c3 c5; do for v in 0 1; do SPHRT_PINNED_UPLOAD=$v timeout -k 10 120 python tools/operator_time.py --config $c --reps 9; done; done; done
