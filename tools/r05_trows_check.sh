#!/bin/bash
# The brick row order of the transposed CSRs: full gpu suite, then C4 (dynamic gradient leg) and
# C5 retrieval with SPHRT_TROWS=off / default, two interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/trows2; mkdir -p $O; rm -f $O/*.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for m in off auto; do
    SPHRT_TROWS=$m timeout -k 10 300 python bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline --no-strong-legs > $O/c4_$m.json 2>/dev/null
    python -c "import json;r=json.loads(open('$O/c4_$m.json').read().splitlines()[-1]);print(json.dumps({'trows':'$m','c4_adjoint_us':r['adjoint']['ms_per_step']*1e3,'c4_forward_us':r['ms_per_step']*1e3}))" >> $O/c4.jsonl
    SPHRT_TROWS=$m timeout -k 10 300 python tools/retrieval_bench.py --out $O/retr_$m.json > /dev/null 2>&1
    python -c "import json;r=json.load(open('$O/retr_$m.json'));print(json.dumps({'trows':'$m','ms_per_iteration':r['ms_per_iteration']}))" >> $O/retr.jsonl
  done
done
cat $O/c4.jsonl $O/retr.jsonl
