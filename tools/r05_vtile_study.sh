#!/bin/bash
# C3 forward with the rays traced in tiles across views (SPHRT_RAY_ORDER=vtile:V,R,C: V views x R
# rows x C columns per tile) against the geometry order, two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vtile; mkdir -p $O; rm -f $O/times.jsonl
for i in 1 2; do
  for m in natural vtile:16,1,4 vtile:32,1,2 vtile:32,1,4 vtile:64,1,1 vtile:64,1,2 vtile:128,1,1 vtile:128,1,2; do
    SPHRT_RAY_ORDER=$m timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 \
      | grep forward | sed "s/^{/{\"config\": \"c3\", \"order\": \"$m\", /" >> $O/times.jsonl
  done
done
cut -c1-160 $O/times.jsonl
