#!/bin/bash
# XCD run length of the multi-wave forward (fwd_chunk: 64 blocks; variants 32 / 128 / 256) with
# the view-tile trace order: forward and transposed adjoint kernels at C3 / C5, two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/chunk; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for c in c3 c5; do
    for k in 64 32 128 256; do
      lib=""; [ $k != 64 ] && lib=sph_raytracer_amd/lib/variants/libsphrt_chunk$k.so
      SPHRT_LIB=$lib timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | grep -v atomic \
        | sed "s/^{/{\"config\": \"$c\", \"chunk\": $k, /" >> $O/k.jsonl
    done
  done
done
