#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of ``bench.py`` into the bench's legs (first call, warm-up,
timed steps, cold operators, host-tensor calls, graph replays) and give the forward kernel's mean
duration per leg, so the rocprofv3 average of the timed steps can be set beside the bench's own
HIP-event kernel time.

    rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python bench.py ... 2> err
    python tools/rocprof_legs.py DIR err [--kernel forward_kernel]
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace_dir')
    ap.add_argument('bench_stderr')
    ap.add_argument('--kernel', default='forward_kernel')
    args = ap.parse_args()
    legs = None
    for line in open(args.bench_stderr):
        if line.startswith('legs '):
            legs = json.loads(line[5:])
    if legs is None:
        raise SystemExit('no "legs" line in the bench stderr')
    files = glob.glob(os.path.join(args.trace_dir, '**', '*kernel_trace.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no kernel_trace.csv under {args.trace_dir}')
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if args.kernel in r['Kernel_Name']:
                    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    rows.sort()
    want = sum(n for _, n in legs)
    out = {'kernel': args.kernel, 'launches': len(rows), 'expected': want, 'legs': {}}
    if len(rows) < want:
        out['warning'] = 'fewer launches than the bench legs; legs not split'
        legs = [['all', len(rows)]]
    elif len(rows) > want:      # launches after the legs (the strong C4 / C5 legs of a C2 run)
        legs = legs + [['after_legs', len(rows) - want]]
    i = 0
    for name, n in legs:
        d = [(e - s) / 1e3 for s, e in rows[i:i + n]]
        i += n
        if d:
            ds = sorted(d)
            out['legs'][name] = {'n': n, 'mean_us': round(sum(d) / len(d), 3),
                                 'median_us': round(ds[len(ds) // 2], 3),
                                 'min_us': round(ds[0], 3), 'max_us': round(ds[-1], 3)}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
