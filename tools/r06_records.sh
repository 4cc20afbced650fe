#!/bin/bash
# Round 6 records from the current tree, one GPU call: the gpu suite, smoke(), the default bench
# line and the driver-shaped one, the C2 bench under rocprofv3 --kernel-trace --stats (split into
# legs), the C3 / C4 / C5 lines, the strong C4 leg and the C4 first construction.
# Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
T=${TAG:-r06}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1
  tail -1 $O/${T}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
  tail -1 $O/${T}_smoke.log
fi
timeout -k 10 300 python bench.py > $O/${T}_bench_c2.json 2> $O/bench.err
cut -c1-200 $O/${T}_bench_c2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench_c2_driver_steps20.json 2> $O/bench20.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-strong-legs > $O/${T}_bench_c2_prof.json 2> $O/prof.err
python tools/rocprof_legs.py $O/prof $O/prof.err > $O/${T}_bench_c2_rocprof_legs.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/${T}_bench_c2_kernel_stats.csv
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/${T}_bench_$c.json 2> $O/bench_$c.err
  cut -c1-160 $O/${T}_bench_$c.json
done
timeout -k 10 300 python bench.py --config c4 --scaling strong --no-cpu-baseline --steps 100 > $O/${T}_strong_c4_1gpu.json 2> /dev/null
timeout -k 10 120 python tools/first_construct.py --warm none --config c4 > $O/${T}_first_c4.json 2>&1
