#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_call5.log 2>&1
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_g.json 2> $O/adjstats.err
timeout -k 10 120 python tools/adjoint_stats.py --config c5 > $O/adjstats_c5_g.json 2>> $O/adjstats.err
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o calib --output-format csv -- tools/fetch_calib > $O/calib.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o calib --output-format csv -- tools/fetch_calib >> $O/calib.log 2>&1
timeout -s KILL 60 rocprofv3 --kernel-trace -d $O/calib_trace -o calib --output-format csv -- tools/fetch_calib >> $O/calib.log 2>&1
