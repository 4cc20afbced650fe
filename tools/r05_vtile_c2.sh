#!/bin/bash
# C2 (the headline) forward kernel by view tile (SPHRT_RAY_ORDER=vtile:tv,1,tw; default (50, 2)),
# three interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vtc2; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2 3; do
  for m in vtile:50,1,2 vtile:10,1,4 vtile:25,1,4 vtile:50,1,4 vtile:10,1,2 vtile:5,1,4 vtile:10,1,5 vtile:25,1,2 vtile:50,1,1; do
    SPHRT_RAY_ORDER=$m timeout -k 10 180 python tools/prof_forward.py --config c2 --rounds 3 | grep forward \
      | sed "s/^{/{\"order\": \"$m\", /" >> $O/k.jsonl
  done
done
