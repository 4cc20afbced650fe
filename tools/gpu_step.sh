#!/bin/bash
# One GPU call: selected pytest files (-m gpu), then optional bench runs; stops at the first failure.
#   bash tools/gpu_step.sh <out-dir> "<pytest targets>" ["<bench args>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p "$out"
tests=$1; shift
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -v --timeout 400 --timeout-method thread \
      > "$out/tests.log" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$out/tests.log" | tail -60
  if [ $rc -ne 0 ]; then echo "pytest failed (rc $rc)"; tail -60 "$out/tests.log"; exit 1; fi
fi
i=0
for b in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py $b > "$out/bench$i.json" 2> "$out/bench$i.err" \
      || { echo "bench $i ($b) failed"; tail -30 "$out/bench$i.err"; exit 1; }
  echo "bench $i ($b):"; cat "$out/bench$i.json"
done
