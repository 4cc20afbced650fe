#!/bin/bash
# Columns of the transposed CSR of a reordered trace: geometry rays (SPHRT_TCOLS=geom, y read as
# given and brick-staged) vs trace rows (=trace, y permuted per call): bench adjoint legs C2 / C3
# / C5 and the C5 retrieval, two interleaved rounds; then the gpu suite on the default.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tcols; mkdir -p $O; rm -f $O/*.jsonl
for i in 1 2; do
  for m in trace geom; do
    for c in c2 c3 c5; do
      SPHRT_TCOLS=$m timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-strong-legs > $O/b.json 2>/dev/null
      python -c "import json;r=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'tcols':'$m','config':'$c','adjoint_us':r['adjoint']['ms_per_step']*1e3,'forward_us':r['ms_per_step']*1e3}))" >> $O/bench.jsonl
    done
    SPHRT_TCOLS=$m timeout -k 10 300 python tools/retrieval_bench.py --out $O/retr.json > /dev/null 2>&1
    python -c "import json;r=json.load(open('$O/retr.json'));print(json.dumps({'tcols':'$m','ms_per_iteration':r['ms_per_iteration']}))" >> $O/retr.jsonl
  done
done
cat $O/bench.jsonl $O/retr.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
