#!/bin/bash
# Block order of one-wave forwards (C2): one contiguous range per XCD (product) against dispatch
# order (sw0) and runs of 64 / 16 blocks (sw64 / sw16), with the view-tile trace order; 3 rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sw; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2 3; do
  for v in product sw0 sw64 sw16; do
    lib=""; [ $v != product ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 180 python tools/prof_forward.py --config c2 --rounds 3 | grep -v atomic \
      | sed "s/^{/{\"variant\": \"$v\", /" >> $O/k.jsonl
  done
done
