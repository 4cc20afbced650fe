#!/bin/bash
# Same-box A/B of the forward / static adjoint kernels: this tree against the round-start
# apply.hip (variant head), C2 / C5 / C3, interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
for r in 1 2; do
 for c in c2 c5 c3; do
  for v in tree head; do
   lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
   SPHRT_LIB=$lib timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | sed "s/^/{\"v\": \"$v\", \"c\": \"$c\", \"r\": $r, \"x\": /; s/$/}/" >> $O/ab_head.jsonl
  done
 done
done
