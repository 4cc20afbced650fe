#!/bin/bash
# Round 6: C4 time-paired adjoint with the dense closes' later rows prefetched with the first ones
# (2 or 6 more rows per thread, variants) against the tree (rows past the second read at the close).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2 3; do
  for v in tree more2 more6; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_morerows_ab.jsonl
  done
done
cat $O/r06_morerows_ab.jsonl
