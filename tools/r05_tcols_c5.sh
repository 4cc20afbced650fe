#!/bin/bash
# C5 transposed adjoint kernel by column order / ray brick: trace-row columns, geometry columns
# with SPHRT_BRICK_T off / 8,1,4 / 8,1,2 / 16,1,2 / 4,1,2 / 32,1,2 (tools/prof_forward.py), two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tcols5; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  SPHRT_TCOLS=trace timeout -k 10 180 python tools/prof_forward.py --config c5 --rounds 3 | grep adjoint_T | sed 's/^{/{"variant": "trace", /' >> $O/k.jsonl
  for b in off 8,1,4 8,1,2 16,1,2 4,1,2 32,1,2; do
    SPHRT_TCOLS=geom SPHRT_BRICK_T=$b timeout -k 10 180 python tools/prof_forward.py --config c5 --rounds 3 | grep adjoint_T | sed "s/^{/{\"variant\": \"geom $b\", /" >> $O/k.jsonl
  done
done
