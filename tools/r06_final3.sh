#!/bin/bash
# Round 6 closing records from the final tree (r06_final.sh without its PMC passes: bench.py
# reads the PMC records it wrote into profiles/), one GPU call: the gpu suite and smoke(); the
# default bench line, the
# driver-shaped one and the C2 bench under rocprofv3 split into legs; C3 / C4 / C5 lines; the
# strong C4 / C5 legs and their two-rank rehearsals; reference-mode and Operator times; the first
# dynamic construction; the C5 retrieval.  Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final3; mkdir -p $O
T=r06
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench_c2.json 2> $O/bench.err
cut -c1-160 $O/${T}_bench_c2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench_c2_driver_steps20.json 2> $O/bench20.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-strong-legs > $O/${T}_bench_c2_prof.json 2> $O/prof.err
python tools/rocprof_legs.py $O/prof $O/prof.err > $O/${T}_bench_c2_rocprof_legs.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/${T}_bench_c2_kernel_stats.csv
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/${T}_bench_$c.json 2> $O/bench_$c.err
done
timeout -k 10 300 python bench.py --config c4 --scaling strong --no-cpu-baseline --steps 100 > $O/${T}_strong_c4_1gpu.json 2> $O/strong_c4.err
timeout -k 10 300 python bench.py --config c5 --scaling strong --no-cpu-baseline --steps 100 > $O/${T}_strong_c5_1gpu.json 2> $O/strong_c5.err
SPHRT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --config c4 --scaling strong --no-cpu-baseline --steps 50 > $O/${T}_strong_c4_2rank_rehearsal.json 2> $O/reh_c4.err
SPHRT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --config c5 --scaling strong --no-cpu-baseline --steps 50 > $O/${T}_strong_c5_2rank_rehearsal.json 2> $O/reh_c5.err
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/${T}_refmode_trace_times.jsonl 2>/dev/null
done
for c in c2 c3 c4 c5; do
  timeout -k 10 200 python tools/operator_time.py --config $c --reps 9 >> $O/${T}_operator_times.jsonl 2>/dev/null
done
timeout -k 10 120 python tools/first_construct.py --warm none --config c4 > $O/${T}_first_c4.json 2>&1
timeout -k 10 300 python tools/retrieval_bench.py --out $O/${T}_retrieval_c5.json > $O/retrieval.log 2>&1
echo final-done
