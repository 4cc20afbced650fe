#!/usr/bin/env python3
"""profiles/rNN_operator_times.json from a round's records: the Operator + first forward medians
(tools/operator_time.py lines, rNN_operator_times_c2_c5.jsonl) and the per-kernel device time of
the same construction under rocprofv3 (rNN_operator_cN_kernel_stats.csv, tools/record_round.sh).

    python tools/operator_record.py r05 [--reps 6]
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, 'profiles')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('tag')
    ap.add_argument('--reps', type=int, default=6,
                    help='constructions in the profiled run (record_round.sh: 1 warm-up + 5)')
    a = ap.parse_args()
    out = {'what': 'Operator construction + first forward (tools/operator_time.py: median and min '
                   'of 9 warm repetitions, float64 trace, the bench density dtype) and the device '
                   'time per construction of every kernel under rocprofv3 --kernel-trace --stats '
                   f'({a.reps} constructions per profiled run)',
           'source': f'profiles/{a.tag}_operator_times_c2_c5.jsonl, '
                     f'profiles/{a.tag}_operator_cN_kernel_stats.csv',
           'configs': {}}
    for line in open(os.path.join(P, f'{a.tag}_operator_times_c2_c5.jsonl')):
        r = json.loads(line)
        c = r['config']
        ks = {}
        path = os.path.join(P, f'{a.tag}_operator_{c}_kernel_stats.csv')
        if os.path.exists(path):
            for row in csv.DictReader(open(path)):
                name = row['Name'].split('(')[0].replace('void ', '').replace('sphrt::', '')
                ks[name] = ks.get(name, 0) + float(row['TotalDurationNs']) / a.reps / 1e3
        top = dict(sorted(((k, round(v, 1)) for k, v in ks.items()), key=lambda kv: -kv[1])[:8])
        out['configs'][c] = {'operator_ms_median': round(r['operator_ms_median'], 3),
                             'operator_ms_min': round(r['operator_ms_min'], 3), 'rays': r['rays'],
                             'env': r.get('env', {}),
                             'device_busy_us_per_construction': round(sum(ks.values()), 1),
                             'top_kernels_us': top}
    dst = os.path.join(P, f'{a.tag}_operator_times.json')
    with open(dst, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(dst)


if __name__ == '__main__':
    main()
