#!/bin/bash
# Row order of the transposed CSR (SPHRT_TROWS: off = linear voxels, b0,b1,b2 = voxel bricks):
# adjoint kernel times (tools/prof_forward.py, HIP events over graph replay) at C3 / C5 / C2, two
# interleaved rounds; then the whole gpu suite on the default.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/trows; mkdir -p $O; rm -f $O/times.jsonl
for i in 1 2; do
  for c in c3 c5 c2; do
    for m in off 4,2,4 2,4,4 4,4,4 8,8,4; do
      SPHRT_TROWS=$m timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 \
        | grep adjoint_T | sed "s/^{/{\"config\": \"$c\", \"trows\": \"$m\", /" >> $O/times.jsonl
    done
  done
done
cut -c1-150 $O/times.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
