#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_fullsize.py tests/test_gpu_properties.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4" > $O/dense_tests.log 2>&1
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_lrow.json 2> $O/adjstats_c4.err
timeout -k 10 300 python bench.py --no-strong-legs --no-cpu-baseline > $O/bench_c2_check.json 2> /dev/null
