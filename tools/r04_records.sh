#!/bin/bash
# Round-4 records in one GPU call: forward PMC (profiles the bench's roofline traffic reads), the
# round record (gpu suite, smoke, driver-shaped bench, bench + rocprofv3, C3/C4/C5 lines, Operator
# kernel stats), then trace-kernel PMC at C2/C3/C5.  Stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
STEPS=pmc bash tools/gpu_round.sh r04
TAG=r04 bash tools/record_round.sh
mkdir -p gpurun_out/tpmc
for c in c2 c3 c5; do
  timeout -k 10 120 python tools/pmc_trace.py --config $c --out gpurun_out/tpmc/r04_trace_${c}_pmc.json > gpurun_out/tpmc/pmc_$c.log 2>&1
done
ls gpurun_out/tpmc
timeout -k 10 300 python tools/retrieval_bench.py --out gpurun_out/round/r04_retrieval_c5.json > gpurun_out/round/retrieval.log 2>&1
head -c 400 gpurun_out/round/r04_retrieval_c5.json
timeout -k 10 120 python tools/exact_stats.py > gpurun_out/round/r04_exact_stats.jsonl 2>&1
cat gpurun_out/round/r04_exact_stats.jsonl
timeout -k 10 120 python tools/bound_check.py > gpurun_out/round/r04_bound_check.jsonl 2>&1
cat gpurun_out/round/r04_bound_check.jsonl
