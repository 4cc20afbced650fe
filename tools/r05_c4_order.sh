#!/bin/bash
# C4 (dynamic, view i <-> slice i: no tiles across views) per-view trace orders: the wedge order
# (default) against detector tiles (SPHRT_RAY_ORDER=tile:rows,cols) and the natural order;
# bench forward step and gradient leg, two rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c4order; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for m in auto natural tile:4,4 tile:8,2 tile:2,8 tile:16,2 tile:8,4 tile:4,8; do
    SPHRT_RAY_ORDER=$m timeout -k 10 300 python bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --no-strong-legs > $O/b.json 2>/dev/null
    python -c "import json;r=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'order':'$m','forward_us':r['ms_per_step']*1e3,'kernel_us':r['roofline']['kernel_ms']*1e3,'gradient_us':r['adjoint']['ms_per_step']*1e3}))" >> $O/c4.jsonl
  done
done
cat $O/c4.jsonl
