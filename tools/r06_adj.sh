#!/bin/bash
# Round 6: C4 time-paired adjoint statistics and kernel times (trace-row vs geometry columns).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4.json 2> $O/adjstats.err
SPHRT_TCOLS=geom timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_geom.json 2>> $O/adjstats.err
timeout -k 10 120 python tools/adjoint_stats.py --config c5 > $O/adjstats_c5.json 2>> $O/adjstats.err
timeout -k 10 120 python tools/adjoint_stats.py --config c3 > $O/adjstats_c3.json 2>> $O/adjstats.err
cat $O/adjstats_c4.json $O/adjstats_c4_geom.json $O/adjstats_c5.json $O/adjstats_c3.json
