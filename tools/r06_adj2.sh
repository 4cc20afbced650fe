#!/bin/bash
# Round 6: C4 time-paired adjoint with geometry columns and no ray bricks (no per-call gather, no pack).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
SPHRT_TCOLS=geom SPHRT_BRICK_T=off timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_geom_nobrick.json 2> $O/adjstats2.err
timeout -k 10 120 python tools/adjoint_stats.py --config c4 > $O/adjstats_c4_b.json 2>> $O/adjstats2.err
cat $O/adjstats_c4_geom_nobrick.json $O/adjstats_c4_b.json
