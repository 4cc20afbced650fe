#!/bin/bash
# Round 6: dense output stage zeroed and flushed in 16-byte vectors, no empty-list load in dense
# launches (variant vflush) against the tree: parity of the variant (full-size and property
# tests), then C4 / C5 adjoints and the C2 forward (graph replay), alternating.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_vflush.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_properties.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/vflush_tests.log 2>&1
tail -1 $O/vflush_tests.log
for r in 1 2 3; do
  for v in tree vflush; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    for c in c4 c5; do
      SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config $c 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': '$c', 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_vflush_ab.jsonl
    done
    SPHRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-strong-legs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': 'c2', 'graph_us': d['roofline']['kernel_ms_graph_replay']*1e3, 'ms_per_step': d['ms_per_step']}))" >> $O/r06_vflush_ab.jsonl
  done
done
cat $O/r06_vflush_ab.jsonl
