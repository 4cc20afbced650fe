#!/bin/bash
# One GPU call refreshing the round's evidence: parity tests, PMC passes (C2, C3), the C2 bench,
# rocprofv3 kernel stats of the bench, C3/C5 bench lines and the apply-kernel study.  Every GPU
# step has its own time limit and the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
TAG=${1:-r03}
STEPS=${STEPS:-tests,pmc,bench,prof,configs,apply,retrieval}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -3 $OUT/gpu_tests.log
fi
if [[ $STEPS == *pmc* ]]; then
  for c in c2 c3 c4 c5; do
    timeout -k 10 300 python tools/pmc_forward.py --config $c --reps 5 --out $OUT/${TAG}_forward_${c}_pmc.json > $OUT/pmc_$c.log 2>&1
    cp $OUT/${TAG}_forward_${c}_pmc.json profiles/
    for p in fetch_size write_size sq_waves_sq_insts_valu sq_wait_any_sq_wait_inst_any; do
      cp gpurun_out/pmc/$p/pmc_counter_collection.csv $OUT/${TAG}_forward_${c}_pmc_$p.csv
    done
  done
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
fi
if [[ $STEPS == *prof* ]]; then
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-strong-legs > $OUT/prof_bench.json 2> $OUT/prof.err
  for f in $(find $OUT/prof -name "*kernel_stats.csv"); do head -6 "$f"; cp "$f" $OUT/${TAG}_bench_c2_kernel_stats.csv; done
  python tools/rocprof_legs.py $OUT/prof $OUT/prof.err > $OUT/${TAG}_bench_c2_rocprof_legs.json
  cat $OUT/${TAG}_bench_c2_rocprof_legs.json
fi
if [[ $STEPS == *configs* ]]; then
  for c in c3 c4 c5; do
    v=10; [ $c = c3 ] && v=4
    timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --cpu-sample-views $v --cpu-reps 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err
    cut -c1-200 $OUT/bench_$c.json
  done
fi
if [[ $STEPS == *apply* ]]; then
  rm -f $OUT/apply_kernels.jsonl
  for c in c2 c5 c3; do
    timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 2>/dev/null | sed "s/}$/, \"config\": \"$c\"}/" >> $OUT/apply_kernels.jsonl
  done
  wc -l $OUT/apply_kernels.jsonl
fi
if [[ $STEPS == *retrieval* ]]; then
  timeout -k 10 300 python tools/retrieval_bench.py --out $OUT/${TAG}_retrieval_c5.json > $OUT/retrieval.log 2>&1
  head -c 400 $OUT/${TAG}_retrieval_c5.json
fi
