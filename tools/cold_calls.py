#!/usr/bin/env python3
"""Cold path (Operator construction + first forward) attributed per C entry point: every
``_lib.check`` (called right after each libsphrt call) synchronises the device and stamps the
time, so each entry's time is the host work since the previous call plus the call's own GPU
work.  The unsynchronised cold time is printed next to it (median of --reps).

    python tools/cold_calls.py [--config c2] [--reps 7]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=7)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    grid, geom = bench.build_geometry(cfg, 0, 1)

    def cold():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op = Operator(grid, geom, device=dev)
        op(x)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3

    for _ in range(2):
        cold()
    plain = sorted(cold() for _ in range(args.reps))[args.reps // 2]

    orig = _lib.check
    log = []

    def check(status, what):
        torch.cuda.synchronize(dev)
        log.append((what, time.perf_counter()))
        return orig(status, what)

    _lib.check = check
    per = {}
    try:
        for _ in range(args.reps):
            log.clear()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            op = Operator(grid, geom, device=dev)
            log.append(('(construction tail)', time.perf_counter()))
            op(x)
            torch.cuda.synchronize(dev)
            log.append(('(first forward tail)', time.perf_counter()))
            prev = t0
            seen = {}
            for what, t in log:
                k = what
                seen[k] = seen.get(k, 0) + 1
                if seen[k] > 1:
                    k = f'{what} #{seen[k]}'
                per.setdefault(k, []).append((t - prev) * 1e3)
                prev = t
    finally:
        _lib.check = orig
    rec = {k: round(sorted(v)[len(v) // 2], 4) for k, v in per.items()}
    rec = dict(sorted(rec.items(), key=lambda kv: -kv[1]))
    print(json.dumps({'config': args.config, 'cold_ms': round(plain, 4),
                      'synced_sum_ms': round(sum(rec.values()), 4), 'per_call_ms': rec}),
          flush=True)


if __name__ == '__main__':
    main()
