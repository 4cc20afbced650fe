#!/bin/bash
# rocprofv3 kernel trace of the C5 retrieval loop on this tree: one iteration's kernels and the
# mean span / busy time per iteration (tools/retrieval_iteration.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-rtrace2}; mkdir -p "$out"
timeout -k 10 180 rocprofv3 --kernel-trace -d "$out/prof" -o run --output-format csv -- python tools/retrieval_bench.py --iters 50 --no-autograd > "$out/rb.json" 2> "$out/rb.err" || exit 1
python tools/retrieval_iteration.py "$out/prof" > "$out/iter.json" || exit 1
cat "$out/iter.json"
