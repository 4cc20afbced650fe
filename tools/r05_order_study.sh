#!/bin/bash
# C3 trace-order study: forward / transposed-adjoint kernel times (tools/prof_forward.py) with the
# rays traced in geometry order and row-interleaved across groups of G views (SPHRT_RAY_ORDER=
# views:G), two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/order; mkdir -p $O; rm -f $O/times.jsonl
for i in 1 2; do
  for m in natural views:16 views:64 views:128; do
    SPHRT_RAY_ORDER=$m timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 \
      | sed "s/^{/{\"order\": \"$m\", /" >> $O/times.jsonl
  done
done
cut -c1-200 $O/times.jsonl
# native construction timeline at C2 (kernel trace; gaps = host turns between launches)
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c2 -o run -- python tools/operator_time.py --config c2 --reps 5 > $O/prof_c2.log 2>&1
