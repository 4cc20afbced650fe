#!/usr/bin/env python3
"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (the host stalls of a cold
Operator construction: syncs, host work, allocations).

    python tools/kernel_gaps.py gpurun_out/ab/prof_c3_tree [min_gap_us]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
rows = []
for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                     r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]))
rows.sort()
busy = sum(e - s for s, e, _ in rows)
span = rows[-1][1] - rows[0][0]
print(f'{len(rows)} kernels, busy {busy / 1e3:.1f} us over {span / 1e3:.1f} us')
prev_end, prev_name = rows[0][1], rows[0][2]
for s, e, name in rows[1:]:
    gap = (s - prev_end) / 1e3
    if gap >= min_gap:
        print(f'{gap:9.1f} us  after {prev_name:60s} before {name}')
    prev_end, prev_name = max(prev_end, e), name
