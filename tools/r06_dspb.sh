#!/bin/bash
# Round 6: blocks of 1920 row starts for dense output ranges (the tree) — the gpu suite on the
# tree, then the C4 time-paired adjoint (and the C4 forward, C5 adjoint as controls) against
# dense blocks of 1792 (the previous layout), 1984 and 2016 (variants), alternating.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/dspb_gpu_tests.log 2>&1
tail -1 $O/dspb_gpu_tests.log
for r in 1 2 3; do
  for v in tree d1792 d1984 d2016; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    for c in c4 c5; do
      SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config $c 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': '$c', 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_dspb_ab.jsonl
    done
  done
done
cat $O/r06_dspb_ab.jsonl
