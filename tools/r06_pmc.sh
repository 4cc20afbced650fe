#!/bin/bash
# Round 6: PMC records of the forward kernels (C2-C5) and of the C4 time-paired adjoint on the
# current tree (the bench roofline's `traffic`), the reference-mode trace times at C2 and the
# Operator-construction kernel stats at C3.  Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_properties.py -x -q --timeout 100 --timeout-method thread -k "side_stream or concurrent_streams" > $O/side_stream_test.log 2>&1
tail -1 $O/side_stream_test.log
for c in c2 c3 c4 c5; do
  timeout -k 10 400 python tools/pmc_forward.py --config $c --out $O/r06_forward_${c}_pmc.json --workdir $O/pmc_$c > $O/pmc_$c.log 2>&1
done
timeout -k 10 400 python tools/pmc_forward.py --config c4 --adjoint --out $O/r06_adjoint_c4_pmc.json --workdir $O/pmc_adj > $O/pmc_adj.log 2>&1
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/r06_refmode_trace_times.jsonl 2>/dev/null
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_c3 -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 5 > $O/r06_operator_c3.json 2> $O/operator_c3.err
cp $(find $O/op_c3 -name "*kernel_stats.csv" | head -1) $O/r06_operator_c3_kernel_stats.csv
