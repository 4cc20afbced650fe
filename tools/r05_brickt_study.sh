#!/bin/bash
# With the transposed rows in voxel bricks: the ray-side brick staging of the transposed CSR
# (SPHRT_BRICK_T = views,rows,cols per brick; off = none, the default) at C3, two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/brickt; mkdir -p $O; rm -f $O/times.jsonl
for i in 1 2; do
  for m in off 4,2,4 8,2,4 8,1,4 16,1,4 4,1,8 8,2,8 4,4,4; do
    SPHRT_BRICK_T=$m timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 \
      | grep adjoint_T | sed "s/^{/{\"config\": \"c3\", \"brick_t\": \"$m\", /" >> $O/times.jsonl
  done
done
cut -c1-160 $O/times.jsonl
