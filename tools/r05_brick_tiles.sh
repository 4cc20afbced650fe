#!/bin/bash
# Density brick (SPHRT_BRICK = r,e,a voxels) of the multi-wave forward under the view-tile order:
# C3 and C5 forward kernels, two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/bricktiles; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for c in c3 c5; do
    for b in 4,2,4 2,4,4 4,4,2 8,2,2 2,2,8 4,4,4 2,8,2 off; do
      SPHRT_BRICK=$b timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | grep forward \
        | sed "s/^{/{\"config\": \"$c\", \"brick\": \"$b\", /" >> $O/k.jsonl
    done
  done
done
