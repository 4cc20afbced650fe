#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_fullsize.py tests/test_gpu_properties.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4" > $O/dyn_tests6.log 2>&1
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 100 > $O/bench_c4_6.json 2> /dev/null
timeout -k 10 300 python bench.py --config c4 --scaling strong --no-cpu-baseline --steps 100 > $O/strong_c4_6.json 2> /dev/null
