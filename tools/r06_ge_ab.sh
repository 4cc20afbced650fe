#!/bin/bash
# Round 6: early granule DMA rounds sized to the largest table (tree) against a fixed 3 (ge3):
# parity, then forward / adjoint kernels at C2-C5 and the C4 time-paired adjoint, interleaved.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/ge_tests.log 2>&1
tail -1 $O/ge_tests.log
for r in 1 2; do
  for c in c2 c5 c3; do
    for v in tree ge3; do
      lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
      SPHRT_LIB=$lib timeout -k 10 120 python tools/prof_forward.py --config $c --rounds 3 2>/dev/null | sed "s/^/{\"v\": \"$v\", \"c\": \"$c\", \"r\": $r, \"x\": /; s/$/}/" >> $O/r06_ge_ab.jsonl
    done
  done
  for v in tree ge3; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'c': 'c4', 'r': $r, 'x': {'kernel': 'c4_adjoint', 'us_median': d['adjoint_kernel_us'][1], 'forward_us': d['forward_us'][1], 'tab_stride': d['tab_stride']}}))" >> $O/r06_ge_ab.jsonl
  done
done
echo done
