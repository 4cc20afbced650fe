#!/bin/bash
# Round 6: confirmation on the closing tree — the gpu suite, smoke(), the default bench line and
# the driver-shaped one.  Stops at the first failure.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/confirm; mkdir -p $O
T=r06
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench_c2_confirm.json 2> $O/bench.err
cut -c1-200 $O/${T}_bench_c2_confirm.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/${T}_bench_c2_driver_steps20_confirm.json 2> $O/bench20.err
cut -c1-200 $O/${T}_bench_c2_driver_steps20_confirm.json
echo confirm-done
