#!/bin/bash
# rocprofv3 kernel traces of the C5 retrieval loop (this tree and _ab_base): one iteration's
# kernels and the mean span / busy time per iteration (tools/retrieval_iteration.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-rtrace}; mkdir -p "$out"
for v in base tree; do
  pkg=""; [ $v = base ] && pkg="--pkg _ab_base"
  timeout -k 10 180 rocprofv3 --kernel-trace -d "$out/prof_$v" -o run --output-format csv -- python tools/retrieval_bench.py --iters 50 --no-autograd $pkg > "$out/rb_$v.json" 2> "$out/rb_$v.err" || exit 1
  python tools/retrieval_iteration.py "$out/prof_$v" > "$out/iter_$v.json" || exit 1
  cat "$out/iter_$v.json"
done
