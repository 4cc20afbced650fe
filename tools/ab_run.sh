set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log
timeout -k 10 120 python tools/bound_check.py
bash tools/ab_variants.sh c3 "screen|local_table|trace_kernel"
bash tools/ab_variants.sh c5 "screen|local_table|trace_kernel"
