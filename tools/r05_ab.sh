#!/bin/bash
# Same-box A/B against _ab_base (the previous revision's package): C5 retrieval ms/iteration and
# Operator + first forward at C2-C5, interleaved.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-ab}; mkdir -p "$out"
for rep in 1 2 3; do
  timeout -k 10 120 python tools/retrieval_bench.py --pkg _ab_base --no-autograd >> "$out/retr_ab.jsonl" || exit 1
  timeout -k 10 120 python tools/retrieval_bench.py --no-autograd >> "$out/retr_ab.jsonl" || exit 1
done
for rep in 1 2; do
  for c in c2 c3 c5 c4; do
    timeout -k 10 120 python tools/cold_ab.py --config $c --pkg _ab_base >> "$out/cold_ab.jsonl" || exit 1
    timeout -k 10 120 python tools/cold_ab.py --config $c >> "$out/cold_ab.jsonl" || exit 1
  done
done
python - "$out" <<'PY'
import json, sys, collections
d = sys.argv[1]
r = collections.defaultdict(list)
for l in open(f'{d}/retr_ab.jsonl'):
    j = json.loads(l); r[('retr', j['pkg'])].append(round(j['ms_per_iteration'], 4))
for l in open(f'{d}/cold_ab.jsonl'):
    j = json.loads(l); r[(j['config'], j['pkg'], j['module'])].append(round(j['operator_ms_median'], 3))
for k, v in sorted(r.items()): print(k, v)
PY
