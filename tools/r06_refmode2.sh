#!/bin/bash
# Round 6: reference-mode screen as its own kernel (ray list, one wave per listed ray): tests,
# C2 times, kernel stats of the float32 construction.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_reference_suite.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/refmode_tests3.log 2>&1
tail -1 $O/refmode_tests3.log
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/r06_refmode_trace_times_screen.jsonl 2>/dev/null
done
cut -c1-200 $O/r06_refmode_trace_times_screen.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_ref2_f32 -o run --output-format csv -- python tools/operator_time.py --config c2 --reps 5 --ftype float32 > $O/op_ref2_f32.json 2> $O/op_ref2_f32.err
cp $(find $O/op_ref2_f32 -name "*kernel_stats.csv" | head -1) $O/r06_operator_c2_f32_kernel_stats_screen.csv
head -8 $O/r06_operator_c2_f32_kernel_stats_screen.csv | cut -c1-150
