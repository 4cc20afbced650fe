#!/bin/bash
# One GPU call: gpu suite + smoke, Operator-construction A/B against variants, then the round's
# bench records (C2 with rocprofv3 legs, C3/C4/C5 lines) and Operator kernel stats at C2-C5.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/round; mkdir -p $O
STEPS=tests bash tools/gpu_round.sh $TAG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
if [ -n "$AB" ]; then bash tools/ab_variants.sh c3 "table|compact" $AB; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
cut -c1-200 $O/bench_driver.json
STEPS=bench,prof,configs bash tools/gpu_round.sh $TAG
for c in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_$c -o run --output-format csv -- python tools/operator_time.py --config $c --reps 5 > $O/operator_$c.json 2> $O/operator_$c.err
  cp $(find $O/op_$c -name "*kernel_stats.csv") $O/${TAG}_operator_${c}_kernel_stats.csv
  cat $O/operator_$c.json
done
