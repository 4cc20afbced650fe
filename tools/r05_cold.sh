#!/bin/bash
# Round-5 cold-path records: same-box A/B of Operator + first forward against _ab_base (the
# previous revision's package), the reference-mode trace's throughput, and the C3 table kernel's
# HBM counters.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-cold}; mkdir -p "$out"
for rep in 1 2; do
  for c in c2 c3 c5 c4; do
    timeout -k 10 120 python tools/cold_ab.py --config $c --pkg _ab_base >> "$out/cold_ab.jsonl" || exit 1
    timeout -k 10 120 python tools/cold_ab.py --config $c >> "$out/cold_ab.jsonl" || exit 1
  done
done
for c in c1 c2; do
  timeout -k 10 120 python tools/operator_time.py --config $c --reps 5 >> "$out/refmode.jsonl" || exit 1
  timeout -k 10 120 python tools/operator_time.py --config $c --reps 5 --ftype float32 >> "$out/refmode.jsonl" || exit 1
  timeout -k 10 120 python tools/operator_time.py --config $c --reps 5 --invalid >> "$out/refmode.jsonl" || exit 1
done
timeout -k 10 120 python tools/pmc_trace.py --config c3 --match local_table_radix --counters FETCH_SIZE --out "$out/table_c3_pmc_fetch.json" > "$out/pmc1.log" 2>&1 || exit 1
timeout -k 10 120 python tools/pmc_trace.py --config c3 --match local_table_radix --counters WRITE_SIZE --out "$out/table_c3_pmc_write.json" > "$out/pmc2.log" 2>&1 || exit 1
cat "$out/cold_ab.jsonl" "$out/refmode.jsonl"
for f in "$out"/table_c3_pmc_*.json; do python -c "import json;d=json.load(open('$f'));[print('$f',k,v.get('median_s'),{c:round(x/1e6,2) for c,x in v['per_launch'].items()}) for k,v in d['kernels'].items()]"; done
