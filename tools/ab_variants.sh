#!/bin/bash
# Kernel A/B of Operator construction: rocprofv3 kernel stats of tools/operator_time.py for the
# in-tree library and each variant built by tools/build_ab.py (sph_raytracer_amd/lib/variants).
#   bash tools/ab_variants.sh CONFIG PATTERN VARIANT...
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
C=$1; P=$2; shift 2
O=gpurun_out/ab; mkdir -p $O
for v in tree "$@"; do
  lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
  SPHRT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${C}_$v -o run --output-format csv -- python tools/operator_time.py --config $C --reps 5 $OPT_ARGS > $O/op_${C}_$v.json 2>$O/op_${C}_$v.err
  f=$(find $O/prof_${C}_$v -name "*kernel_stats.csv"); cp $f $O/${C}_${v}_kernel_stats.csv
  echo "== $v $(cat $O/op_${C}_$v.json)"; grep -iE "$P" $f | cut -d, -f1-4 | cut -c1-150 || true
done
