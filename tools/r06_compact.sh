#!/bin/bash
# Round 6: compact closes of the dense output ranges (occupancy bitmap) + geometry columns for
# the time-paired adjoint: dynamic parity tests, C4 adjoint stats, C4 bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py tests/test_gpu_pins.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4 or dense or side_stream or time" > $O/compact_tests.log 2>&1
tail -1 $O/compact_tests.log
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_compact.json 2> $O/adjstats3.err
cat $O/adjstats_c4_compact.json
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4_compact.json 2> /dev/null
cut -c1-300 $O/bench_c4_compact.json
