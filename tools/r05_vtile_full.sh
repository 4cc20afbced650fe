#!/bin/bash
# C3 with the rays traced in tiles across views: forward and transposed adjoint kernels
# (tools/prof_forward.py) and Operator + first forward (tools/operator_time.py), natural order
# against vtile:64,1,2 / vtile:32,1,2, two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vtile2; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for m in natural vtile:64,1,2 vtile:32,1,2; do
    SPHRT_RAY_ORDER=$m timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 \
      | sed "s/^{/{\"order\": \"$m\", /" >> $O/kernels.jsonl
    SPHRT_RAY_ORDER=$m timeout -k 10 120 python tools/operator_time.py --config c3 --reps 5 \
      | sed "s/^{/{\"order\": \"$m\", /" >> $O/operator.jsonl
  done
done
