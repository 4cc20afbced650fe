#!/bin/bash
# Under the view tiles: float64 half tables on / off (SPHRT_FWD_HALF) at C5 / C3 / C2, and the
# transposed rows' voxel brick (SPHRT_TROWS) at C5 / C3; two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/misc; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for c in c5 c3 c2; do
    for h in 1 0; do
      SPHRT_FWD_HALF=$h timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | grep _f64 | grep -v atomic \
        | sed "s/^{/{\"config\": \"$c\", \"half\": $h, /" >> $O/half.jsonl
    done
  done
  for c in c5 c3; do
    for t in auto 8,8,4 4,4,4 2,4,4 8,4,4; do
      SPHRT_TROWS=$t timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | grep adjoint_T \
        | sed "s/^{/{\"config\": \"$c\", \"trows\": \"$t\", /" >> $O/trows.jsonl
    done
  done
done
