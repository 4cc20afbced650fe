#!/bin/bash
# Round 6: reference-mode one-pass + screen (tests, C2 times), then the C4 records (r06_c4.sh).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api_surface.py -x -q --timeout 120 --timeout-method thread > $O/api_surface_tests.log 2>&1
for m in "--ftype float32" "--invalid" ""; do
  timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 $m >> $O/refmode_times.jsonl 2>/dev/null
done
bash tools/r06_c4.sh
