#!/bin/bash
# Under the view tiles (tiles row-major outermost): one contiguous block range per XCD (variant
# contig: each XCD a band of detector rows, i.e. a horizontal slab of the volume) against runs of
# 64 blocks dealt round-robin (product), C3 / C5 forward and adjoint kernels, two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/contig; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for c in c3 c5; do
    for v in product contig; do
      lib=""; [ $v != product ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
      SPHRT_LIB=$lib timeout -k 10 180 python tools/prof_forward.py --config $c --rounds 3 | grep -v atomic \
        | sed "s/^{/{\"config\": \"$c\", \"variant\": \"$v\", /" >> $O/k.jsonl
    done
  done
done
