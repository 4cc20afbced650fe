#!/usr/bin/env python3
"""Per-kernel average durations (us) from tools/ab_variants.sh's kernel-stats CSVs:
    python tools/ab_table.py gpurun_out/ab PATTERN [CONFIG ...]"""
import csv
import glob
import os
import re
import sys

d, pat = sys.argv[1], re.compile(sys.argv[2])
cfgs = sys.argv[3:] or sorted({os.path.basename(f).split('_')[0] for f in glob.glob(f'{d}/*_kernel_stats.csv')})
for c in cfgs:
    for f in sorted(glob.glob(f'{d}/{c}_*_kernel_stats.csv')):
        v = os.path.basename(f)[len(c) + 1:-len('_kernel_stats.csv')]
        for r in csv.DictReader(open(f)):
            if pat.search(r['Name']):
                print(f"{c:4s} {v:8s} {float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>3s}  {r['Name'][:70]}")
