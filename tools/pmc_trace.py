#!/usr/bin/env python3
"""rocprofv3 PMC pass over the trace kernels (Operator construction, tools/trace_bench.py): VALU
instruction mix per launch, FP64 split, and the executed FP64 rate next to the algorithmic one
(~1064 FLOP per ray at C2).  Runs rocprofv3 as a child process.

    python tools/pmc_trace.py --config c2 --out profiles/r01_trace_c2_pmc.json
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ['SQ_WAVES', 'SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VALU_FMA_F64',
            'SQ_INSTS_VALU_MUL_F64', 'SQ_INSTS_VALU_ADD_F64', 'SQ_INSTS_VALU_TRANS_F64']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--out', required=True)
    ap.add_argument('--counters', default=None, help='comma-separated SQ counters (one pass)')
    ap.add_argument('--count-pass', action='store_true',
                    help='profile tools/trace_time.py (the two-pass COUNT kernel) instead of '
                         'trace_bench.py')
    ap.add_argument('--match', default='trace_kernel',
                    help='kernels whose name contains this (e.g. screen_kernel)')
    args = ap.parse_args()
    counters = args.counters.split(',') if args.counters else COUNTERS
    d = os.path.join(ROOT, 'gpurun_out', 'pmc_trace')
    shutil.rmtree(d, ignore_errors=True)
    subprocess.run(['rocprofv3', '--pmc', *counters, '--kernel-trace', '-d', d, '-o', 'p',
                    '--output-format', 'csv', '--', sys.executable,
                    *([os.path.join(ROOT, 'tools', 'trace_time.py'), args.config] if args.count_pass
                      else [os.path.join(ROOT, 'tools', 'trace_bench.py'), args.config, '--reps',
                            '1'])],
                   check=True, cwd=ROOT, stdout=subprocess.DEVNULL)
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r['Kernel_Name'].split('(')[0].replace('void ', '')
            if args.match in name:
                vals[name][r['Counter_Name']].append(float(r['Counter_Value']))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r['Kernel_Name'].split('(')[0].replace('void ', '')
            if args.match in name:
                dur[name].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
    rec = {'config': args.config, 'counters': counters, 'lib': os.environ.get('SPHRT_LIB'),
           'kernels': {}}
    for k, v in vals.items():
        per = {c: sum(x) / len(x) for c, x in v.items()}
        t = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else None
        if counters is not COUNTERS:
            rec['kernels'][k] = {'per_launch': per, 'median_s': t}
            continue
        f64_flop = 64 * (2 * per['SQ_INSTS_VALU_FMA_F64'] + per['SQ_INSTS_VALU_MUL_F64'] +
                         per['SQ_INSTS_VALU_ADD_F64'] + per['SQ_INSTS_VALU_TRANS_F64'])
        t = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else None
        rec['kernels'][k] = {'per_launch': per, 'median_s': t,
                             'f64_flop_executed': f64_flop,
                             'f64_tflops_executed': f64_flop / t / 1e12 if t else None,
                             'f64_valu_share': (per['SQ_INSTS_VALU_FMA_F64'] + per['SQ_INSTS_VALU_MUL_F64']
                                                + per['SQ_INSTS_VALU_ADD_F64'] + per['SQ_INSTS_VALU_TRANS_F64'])
                             / per['SQ_INSTS_VALU']}
    with open(args.out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
