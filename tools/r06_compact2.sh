#!/bin/bash
# Round 6: compact closes for every dense range up to kOutRange: tests, same-process A/B against
# row_ray closes, C4 adjoint stats.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py tests/test_gpu_pins.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4 or dense or time" > $O/compact2_tests.log 2>&1
tail -1 $O/compact2_tests.log
timeout -k 10 120 python tools/dense_ab.py --config c4 > $O/r06_dense_ab_c4.json 2> $O/dense_ab.err
cat $O/r06_dense_ab_c4.json
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_compact2.json 2> $O/adjstats4.err
cut -c 600-1200 $O/adjstats_c4_compact2.json
