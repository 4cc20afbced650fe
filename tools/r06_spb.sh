#!/bin/bash
# Round 6: segments per block (row starts per workgroup) 1536 / 1664 / 1920 (variants) against
# 1792 (tree): C4 time-paired adjoint, C5 transposed adjoint, C2 forward (graph replay).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2 3; do
  for v in tree spb1536 spb1664 spb1920; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    for c in c4 c5; do
      SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config $c 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': '$c', 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_spb_ab.jsonl
    done
    SPHRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-strong-legs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': 'c2', 'graph_us': d['roofline']['kernel_ms_graph_replay']*1e3, 'ms_per_step': d['ms_per_step']}))" >> $O/r06_spb_ab.jsonl
  done
done
cat $O/r06_spb_ab.jsonl
