#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4.json 2> $O/adjstats_c4.err
SPHRT_TCOLS=geom timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_geom.json 2>> $O/adjstats_c4.err
timeout -k 10 120 python tools/adjoint_stats.py --config c5 > $O/adjstats_c5.json 2>> $O/adjstats_c4.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "c4" > $O/c4_full_tests.log 2>&1
