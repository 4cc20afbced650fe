#!/bin/bash
# Round 6: invalid=True through the infinite-distance ranges of the emulated introsort and the
# register sort: reference-mode tests, C2 times, kernel stats of the invalid=True construction.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_reference_suite.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/infrange_tests.log 2>&1
tail -1 $O/infrange_tests.log
for m in "--invalid" "--ftype float32"; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/r06_refmode_trace_times_infrange.jsonl 2>/dev/null
done
cut -c1-300 $O/r06_refmode_trace_times_infrange.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_inv_inf -o run --output-format csv -- python tools/operator_time.py --config c2 --reps 5 --invalid > $O/op_inv_inf.json 2> $O/op_inv_inf.err
cp $(find $O/op_inv_inf -name "*kernel_stats.csv" | head -1) $O/r06_operator_c2_invalid_kernel_stats_infrange.csv
head -6 $O/r06_operator_c2_invalid_kernel_stats_infrange.csv | cut -c1-150
