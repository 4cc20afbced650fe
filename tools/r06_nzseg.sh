#!/bin/bash
# Round 6: the staged table build reading each block's rows as (start, slot offset) pairs:
# construction parity, then the C3 Operator kernel stats.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_construct.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/nzseg_tests.log 2>&1
tail -1 $O/nzseg_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_c3_nzseg -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 5 > $O/r06_operator_c3_nzseg.json 2> /dev/null
cp $(find $O/op_c3_nzseg -name "*kernel_stats.csv" | head -1) $O/r06_operator_c3_nzseg_kernel_stats.csv
grep -i "table\|trace_kernel" $O/r06_operator_c3_nzseg_kernel_stats.csv | cut -c1-140
