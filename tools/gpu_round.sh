#!/bin/bash
# One GPU call: parity tests, PMC passes, bench, rocprofv3 kernel stats. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
TAG=${1:-r01}
STEPS=${STEPS:-tests,pmc,bench,prof}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -3 $OUT/gpu_tests.log
fi
if [[ $STEPS == *pmc* ]]; then
  timeout -k 10 300 python tools/pmc_forward.py --out $OUT/${TAG}_forward_c2_pmc.json > $OUT/pmc.log 2>&1
  cp $OUT/${TAG}_forward_c2_pmc.json profiles/
  tail -c 600 $OUT/pmc.log
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
if [[ $STEPS == *prof* ]]; then
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
  for f in $(find $OUT/prof -name "*kernel_stats.csv"); do head -12 "$f"; done
fi
