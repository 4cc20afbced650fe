set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log
for c in c5 c4 c5; do timeout -k 10 120 python tools/operator_time.py --config $c --reps 9; done
timeout -k 10 120 python tools/prelude_time.py c5
