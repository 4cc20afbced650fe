#!/bin/bash
# Round 6: C4 time-paired adjoint with a 2560-output stage (variant) against 2048 (tree).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2 3; do
  for v in tree o2560; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_o2560_ab.jsonl
  done
done
cat $O/r06_o2560_ab.jsonl
