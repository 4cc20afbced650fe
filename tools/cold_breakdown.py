#!/usr/bin/env python3
"""Where the cold path (geometry + Operator trace + first forward) spends its time: each stage of
Operator._trace re-enacted with a device sync after it (so stages do not overlap; the sum is a
little above the bench's `cold`).  Median of 5 warm repetitions.

    python tools/cold_breakdown.py [--config c2]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, raytracer as rt
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    stages = {}

    def tick(name, t0):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        stages.setdefault(name, []).append((t1 - t0) * 1e3)
        return t1

    # instrumented copies of the pieces Operator._trace calls
    orig = {k: getattr(rt, k) for k in ('_Plan', '_geom_rays', '_RayBatch', '_local_tables')}

    def wrap(name, fn):
        def inner(*a, **k):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            r = fn(*a, **k)
            tick(name, t0)
            return r
        return inner

    for k, fn in orig.items():
        setattr(rt, k, wrap(k, fn))
    for i in range(args.reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        grid, geom = bench.build_geometry(cfg, 0, 1)
        t1 = tick('build_geometry', t0)
        op = Operator(grid, geom, device=dev)
        t2 = tick('Operator(...)', t1)
        _, g2 = bench.build_geometry(cfg, 0, 1)
        t2b = time.perf_counter()
        g2._ray_spec()
        tick('(geom._ray_spec, host part of _geom_rays)', t2b)
        t2 = time.perf_counter()
        op(x)
        t3 = tick('first forward', t2)
        stages.setdefault('total', []).append((t3 - t0) * 1e3)
        if i == 0:
            stages = {}
    for k, fn in orig.items():
        setattr(rt, k, fn)
    rec = {k: sorted(v)[len(v) // 2] for k, v in stages.items()}
    rec['config'] = args.config
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
