#!/bin/bash
# Round 6 closing records, second call (after the construction fix): gpu suite, smoke, the C2
# bench lines and rocprofv3 legs, Operator and reference-mode times.  Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final2; mkdir -p $O
T=r06
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench_c2.json 2> $O/bench.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench_c2_driver_steps20.json 2> $O/bench20.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-strong-legs > $O/${T}_bench_c2_prof.json 2> $O/prof.err
python tools/rocprof_legs.py $O/prof $O/prof.err > $O/${T}_bench_c2_rocprof_legs.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/${T}_bench_c2_kernel_stats.csv
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/${T}_bench_c4.json 2> $O/bench_c4.err
for c in c2 c3 c4 c5; do
  timeout -k 10 200 python tools/operator_time.py --config $c --reps 9 >> $O/${T}_operator_times.jsonl 2>/dev/null
done
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/${T}_refmode_trace_times.jsonl 2>/dev/null
done
echo final2-done
