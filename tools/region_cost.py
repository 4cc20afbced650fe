#!/usr/bin/env python3
"""Fixed cost of bench.py's timed region (C2): where the ~15-20 µs of a 20-step region beyond
its kernels go. Times K back-to-back op(x) calls bracketed as bench.py does, with the closing
bracket in several forms, and the idle costs of each synchronisation call on its own.

    python tools/region_cost.py [--reps 41] [--steps 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=41)
    ap.add_argument('--steps', type=int, default=20)
    a = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS['c2']
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    x = torch.rand(cfg[0], device=dev)
    for _ in range(20):
        op(x)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)

    def idle(fn, reps=200):
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e6

    out = {'idle_us': {
        'torch.cuda.synchronize(dev)': idle(lambda: torch.cuda.synchronize(dev)),
        'stream.synchronize()': idle(stream.synchronize),
        'event.record()': idle(lambda: torch.cuda.Event().record()),
        'op(x) issue (one call, idle queue)': idle(lambda: op(x), 50),
    }}

    K = a.steps

    def region(close):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(K):
            op(x)
        t1 = time.perf_counter()
        close()
        return (time.perf_counter() - t0) * 1e6, (t1 - t0) * 1e6

    ev = torch.cuda.Event()

    def ev_close():
        ev.record()
        ev.synchronize()

    closes = {
        'sync + sync (bench at N=1)': lambda: (torch.cuda.synchronize(dev), torch.cuda.synchronize(dev)),
        'sync': lambda: torch.cuda.synchronize(dev),
        'stream.synchronize': stream.synchronize,
        'event record + synchronize': ev_close,
    }
    res = {k: [] for k in closes}
    issue = {k: [] for k in closes}
    for _ in range(a.reps):                      # interleaved, so drift hits every form alike
        for k, c in closes.items():
            w, i = region(c)
            res[k].append(w)
            issue[k].append(i)
    out['region_us'] = {k: {'median': statistics.median(v), 'min': min(v),
                            'issue_median': statistics.median(issue[k])} for k, v in res.items()}
    # the kernels alone: HIP events around the same K launches
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    spans = []
    for _ in range(a.reps):
        torch.cuda.synchronize(dev)
        e0.record()
        for _ in range(K):
            op(x)
        e1.record()
        torch.cuda.synchronize(dev)
        spans.append(e0.elapsed_time(e1) * 1e3)
    out['event_span_us'] = statistics.median(spans)
    out['steps'] = K
    print(json.dumps(out))


if __name__ == '__main__':
    main()
