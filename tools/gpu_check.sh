#!/bin/bash
# GPU suite, then the C3 cold-path timing (tools/cold_c3.sh); stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -40 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log
bash tools/cold_c3.sh ${1:-r04}
