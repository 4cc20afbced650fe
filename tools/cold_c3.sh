#!/bin/bash
# C3 cold path: Operator construction + first forward wall time (median of 7) and its kernel
# split under rocprofv3 (kernel trace + stats).  Every GPU step has its own time limit.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r04}
OUT=gpurun_out/cold
mkdir -p $OUT
timeout -k 10 300 python tools/operator_time.py --config c3 --reps 7 > $OUT/${TAG}_operator_times.json 2> $OUT/optime.err
cat $OUT/${TAG}_operator_times.json
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 3 > $OUT/prof.out 2> $OUT/prof.err
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/${TAG}_operator_c3_kernel_stats.csv
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6/4:9.3f} ms/rep  calls {int(r['Calls'])/4:5.1f}  {r['Name'][:90]}")
print('total per rep', tot / 1e6 / 4)
PY
