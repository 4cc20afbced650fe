#!/bin/bash
# Wall-clock A/B of Operator construction + first forward (tools/operator_time.py, no profiler):
# the in-tree library against variants of tools/build_ab.py, two alternating rounds.
#   bash tools/ab_wall.sh "c3 c4" VARIANT...
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/abw; mkdir -p $O
CFGS=$1; shift
for r in 1 2; do
  for c in $CFGS; do
    for v in tree "$@"; do
      lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
      echo "$v $(SPHRT_LIB=$lib timeout -k 10 200 python tools/operator_time.py --config $c --reps 7 2>/dev/null)" | tee -a $O/wall.txt
    done
  done
done
