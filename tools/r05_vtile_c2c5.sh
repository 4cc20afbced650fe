#!/bin/bash
# Cross-view tile orders at C2 (single-wave grid, the headline) and C5 (ConeCirc, wedge order by
# default): forward kernels, two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vtile3; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for m in default vtile:50,1,2 vtile:25,1,2 vtile:10,1,4 vtile:5,1,8 vtile:50,1,1; do
    e=$m; [ $m = default ] && e=auto
    SPHRT_RAY_ORDER=$e timeout -k 10 180 python tools/prof_forward.py --config c2 --rounds 3 \
      | grep -v atomic | sed "s/^{/{\"config\": \"c2\", \"order\": \"$m\", /" >> $O/kernels.jsonl
  done
  for m in default natural vtile:64,1,2 vtile:32,1,2 vtile:16,1,4 vtile:64,1,1; do
    e=$m; [ $m = default ] && e=auto
    SPHRT_RAY_ORDER=$e timeout -k 10 180 python tools/prof_forward.py --config c5 --rounds 3 \
      | grep -v atomic | sed "s/^{/{\"config\": \"c5\", \"order\": \"$m\", /" >> $O/kernels.jsonl
  done
done
