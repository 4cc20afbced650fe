#!/bin/bash
# Round 6 study: C3 forward kernel against super-tiled trace orders (SPHRT_SUPERTILE, Python
# construction) — the hierarchical per-XCD order DESIGN proposed; baseline = the product order.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
for r in 1 2; do
  for st in none 4,4,A 2,8,A 8,2,A 4,8,B 8,4,B 2,16,B; do
    if [ $st = none ]; then
      timeout -k 10 120 python tools/prof_forward.py --config c3 --rounds 3 2>/dev/null | sed "s/^/{\"st\": \"$st\", \"r\": $r, \"x\": /; s/$/}/" >> $O/r06_supertile_c3.jsonl
    else
      SPHRT_SUPERTILE=$st timeout -k 10 120 python tools/prof_forward.py --config c3 --rounds 3 2>/dev/null | sed "s/^/{\"st\": \"$st\", \"r\": $r, \"x\": /; s/$/}/" >> $O/r06_supertile_c3.jsonl
    fi
  done
done
cut -c1-220 $O/r06_supertile_c3.jsonl
