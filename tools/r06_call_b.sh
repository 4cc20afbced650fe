#!/bin/bash
# Round 6: compact closes (dense ranges) + the reference-mode register sort: parity tests, the
# dense A/B, C4 adjoint stats, reference-mode C2 times (ftype=float32 / invalid / default).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_golden.py tests/test_gpu_reference_suite.py -x -q --timeout 300 --timeout-method thread > $O/refmode_tests.log 2>&1
tail -1 $O/refmode_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py tests/test_gpu_pins.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4 or dense or time" > $O/compact2_tests.log 2>&1
tail -1 $O/compact2_tests.log
timeout -k 10 120 python tools/dense_ab.py --config c4 > $O/r06_dense_ab_c4.json 2> $O/dense_ab.err
cat $O/r06_dense_ab_c4.json
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/r06_refmode_trace_times_net.jsonl 2>/dev/null
done
cut -c1-250 $O/r06_refmode_trace_times_net.jsonl
