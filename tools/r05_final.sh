#!/bin/bash
# Closing records of round 5 from the final tree, one GPU call: the gpu suite, smoke(), the C5
# retrieval (median of 5 gd calls), the default bench line and the driver-shaped one (--steps 20
# --warmup 5), and the bench under rocprofv3 --kernel-trace --stats.  Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05_gpu_tests.log 2>&1
tail -1 $O/r05_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05_smoke.log 2>&1
tail -1 $O/r05_smoke.log
timeout -k 10 300 python tools/retrieval_bench.py --out $O/r05_retrieval_c5.json > $O/retrieval.log 2>&1
timeout -k 10 300 python bench.py > $O/r05_bench_c2.json 2> $O/bench.err
cut -c1-200 $O/r05_bench_c2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r05_bench_c2_driver_steps20.json 2> $O/bench20.err
cut -c1-200 $O/r05_bench_c2_driver_steps20.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-strong-legs > $O/prof_bench.json 2> $O/prof.err
