#!/bin/bash
# Round 6: C4 time-paired adjoint against the dense output stage size (kOutStage 2048 in the
# tree, 4096 / 6144 variants), interleaved, same box.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2; do
  for v in tree o4096 o6144; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'forward_us': d['forward_us'], 'adjoint_kernel_us': d['adjoint_kernel_us'], 'adjoint_call_us': d['adjoint_call_us_events']}))" >> $O/r06_ostage_ab.jsonl
  done
done
cat $O/r06_ostage_ab.jsonl
