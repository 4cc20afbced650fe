#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
for r in 1 2; do
 for v in tree nolrow; do
  lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
  SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['forward_us'][0], d['adjoint_kernel_us'][0], d['adjoint_call_us_events'])" >> $O/ab_lrow.txt
 done
done
