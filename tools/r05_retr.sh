#!/bin/bash
# Retrieval A/B (C5 gd ms/iteration, this tree vs _ab_base) and the gd-related GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-retr}; mkdir -p "$out"
for rep in 1 2 3; do
  timeout -k 10 120 python tools/retrieval_bench.py --pkg _ab_base --no-autograd >> "$out/retr_ab.jsonl" || exit 1
  timeout -k 10 120 python tools/retrieval_bench.py >> "$out/retr_ab.jsonl" || exit 1
done
cat "$out/retr_ab.jsonl"
