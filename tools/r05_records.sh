#!/bin/bash
# Round-5 records in one GPU call: forward PMC at C2-C5 (the bench's roofline traffic), the round
# record (gpu suite, smoke, driver-shaped bench, bench + rocprofv3 legs, C3/C4/C5 lines,
# Operator kernel stats), trace-kernel PMC at C2/C3/C5, the C5 retrieval, exact-path counters,
# Operator + first forward medians (tools/operator_time.py, the record the docs quote), and
# two-rank strong-scaling rehearsals of C4 / C5.  Stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
STEPS=pmc bash tools/gpu_round.sh r05
TAG=r05 bash tools/record_round.sh
mkdir -p gpurun_out/tpmc
for c in c2 c3 c5; do
  timeout -k 10 120 python tools/pmc_trace.py --config $c --out gpurun_out/tpmc/r05_trace_${c}_pmc.json > gpurun_out/tpmc/pmc_$c.log 2>&1
done
O=gpurun_out/round
timeout -k 10 300 python tools/retrieval_bench.py --out $O/r05_retrieval_c5.json > $O/retrieval.log 2>&1
head -c 400 $O/r05_retrieval_c5.json
timeout -k 10 120 python tools/exact_stats.py > $O/r05_exact_stats.jsonl 2>&1
rm -f $O/r05_operator_times.jsonl
for c in c2 c3 c4 c5; do
  timeout -k 10 120 python tools/operator_time.py --config $c --reps 9 >> $O/r05_operator_times.jsonl
done
cat $O/r05_operator_times.jsonl
for c in c4 c5; do
  SPHRT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --config $c --scaling strong --steps 20 --warmup 3 --no-cpu-baseline > $O/r05_strong_${c}_2rank_rehearsal.json 2> $O/strong_$c.err
  cut -c1-300 $O/r05_strong_${c}_2rank_rehearsal.json
  timeout -k 10 300 python bench.py --config $c --scaling strong --steps 20 --warmup 3 > $O/r05_strong_${c}_1gpu.json 2> $O/strong1_$c.err
  cut -c1-300 $O/r05_strong_${c}_1gpu.json
done
