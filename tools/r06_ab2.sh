#!/bin/bash
# Round 6: (1) 32-bit keys in the full-network sorts only (tree) against 64-bit keys (k64):
# CSR parity, then the count-pass A/B; (2) the C4 time-paired adjoint against the LDS it takes
# (tree: 3 early granule rounds + a 2048-output stage; g2: 2 early rounds; o1536 / o1024: smaller
# stages), interleaved, same box.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_construct.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/k32b_tests.log 2>&1
tail -1 $O/k32b_tests.log
bash tools/trace_ab.sh r06/k32b_ab k64 c2 c5 c3
for r in 1 2; do
  for v in tree g2 o1536 o1024; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'forward_us': d['forward_us'], 'adjoint_kernel_us': d['adjoint_kernel_us'], 'adjoint_call_us': d['adjoint_call_us_events']}))" >> $O/r06_adj_lds_ab.jsonl
  done
done
cat $O/r06_adj_lds_ab.jsonl
