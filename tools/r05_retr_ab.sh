#!/bin/bash
# Same-box A/B of the C5 retrieval against _ab_base (the previous revision's package),
# interleaved: median of 5 gd(100) calls per run.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-retr_ab}; mkdir -p "$out"
for rep in 1 2 3; do
  timeout -k 10 150 python tools/retrieval_bench.py --pkg _ab_base --no-autograd >> "$out/retr_ab.jsonl" || exit 1
  timeout -k 10 150 python tools/retrieval_bench.py --no-autograd >> "$out/retr_ab.jsonl" || exit 1
done
python - "$out" <<'PY'
import json, sys, collections
r = collections.defaultdict(list)
for l in open(f'{sys.argv[1]}/retr_ab.jsonl'):
    j = json.loads(l); r[j['pkg']].append(round(j['ms_per_iteration'], 4))
for k, v in sorted(r.items()): print(k, v)
PY
