#!/usr/bin/env python3
"""One retrieval iteration from a rocprofv3 kernel trace of tools/retrieval_bench.py: each
kernel's start offset and duration (us), plus the mean span and busy time per iteration over
20 iterations of the direct loop (iterations are delimited by the Adam launch that ends each).

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/retrieval_bench.py --iters 50
    python tools/retrieval_iteration.py DIR > profiles/rNN_retrieval_c5_iteration_trace.json
"""
import csv
import glob
import json
import sys


def main():
    f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
    ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows]
    ends = [i for i, k in enumerate(ks) if 'adam_neg' in k[2]]
    if len(ends) < 42:
        raise SystemExit(f'{len(ends)} Adam launches in the trace; run --iters 50')
    win = ks[ends[20] + 1:ends[40] + 1]
    span = (win[-1][1] - win[0][0]) / 1e3 / 20
    busy = sum(e - s for s, e, _ in win) / 1e3 / 20
    it = ks[ends[30] + 1:ends[31] + 1]
    t0 = it[0][0]
    print(json.dumps({
        'what': 'one C5 retrieval iteration (retrieval._gd_direct) from a rocprofv3 kernel trace of '
                'tools/retrieval_bench.py --iters 50: start offset and duration (us) per kernel; '
                'span / busy: means over 20 iterations',
        'iteration_us': round((it[-1][1] - t0) / 1e3, 3),
        'span_us_per_iteration': round(span, 3), 'busy_us_per_iteration': round(busy, 3),
        'kernels': [[round((s - t0) / 1e3, 2), round((e - s) / 1e3, 2), n[:100]] for s, e, n in it],
    }, indent=1))


if __name__ == '__main__':
    main()
