#!/bin/bash
# Round 6: the dense time-paired transposed CSR's block order — dispatch order (tree) against one
# contiguous block range per XCD (order bit 1): C4 adjoint kernel, alternating.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2 3; do
  for o in 0 2; do
    timeout -k 10 120 python tools/adjoint_stats.py --config c4 --or-order $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'or_order': $o, 'r': $r, 'order': d['order'], 'adjoint_kernel_us': d['adjoint_kernel_us'], 'adjoint_call_us': d['adjoint_call_us_events']}))" >> $O/r06_dorder_ab.jsonl
  done
done
cat $O/r06_dorder_ab.jsonl
