#!/bin/bash
# Trace-kernel phase split by ablation builds (tools/build_variants.py abl1..abl4 =
# -DSPHRT_TRACE_ABL=1..4) and the product build: one PMC pass each (tools/pmc_trace.py).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${1:-c3}
TAG=${2:-r04}
OUT=gpurun_out/abl
mkdir -p $OUT
for v in full abl11 abl12 abl1 abl2 abl3 abl4; do
  if [ $v = full ]; then LIB=""; else LIB=sph_raytracer_amd/lib/variants/libsphrt_$v.so; fi
  SPHRT_LIB=$LIB timeout -k 10 120 python tools/pmc_trace.py --config $CFG --out $OUT/${TAG}_trace_${CFG}_pmc_$v.json > $OUT/pmc_$v.log 2>&1
  python -c "import json,sys;d=json.load(open('$OUT/${TAG}_trace_${CFG}_pmc_$v.json'));[print('$v',k,v.get('median_s'),v['per_launch'].get('SQ_INSTS_VALU'),v['per_launch'].get('SQ_INSTS_SALU'),v['per_launch'].get('SQ_INSTS_LDS')) for k,v in d['kernels'].items()]"
done
