#!/usr/bin/env python3
"""Host time of Operator construction's steps (the cold path's host side between kernels):
wraps the construction's Python steps with timers and reports the mean per Operator, plus the
host time until the first kernel launch.

    python tools/prelude_time.py [c3] [--reps 10]
"""
import argparse
import collections
import functools
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ACC = collections.defaultdict(float)


def wrap(owner, name, label=None):
    f = getattr(owner, name)
    label = label or f'{getattr(owner, "__name__", owner)}.{name}'

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t0
    setattr(owner, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('config', nargs='?', default='c3')
    ap.add_argument('--reps', type=int, default=10)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, raytracer as rt
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    for _ in range(3):
        Operator(grid, geom, device=dev)(x)
    torch.cuda.synchronize()
    for owner, name in [(rt._Plan, '__init__'), (rt._ConeRays, 'of'), (rt._RayBatch, 'host_starts'),
                        (rt._Staging, 'upload'), (rt._Plan, 'attach'), (rt._ConeRays, 'launch'),
                        (rt, '_trace_order'), (rt, '_permute_rays'), (rt._RayBatch, '__init__'),
                        (rt, '_trace_csr'), (rt, '_local_tables'), (rt.Operator, '_index'),
                        (torch.cuda, 'mem_get_info'), (rt, '_workspace')]:
        wrap(owner, name)
    first = []
    lib = rt._lib.load()
    names = ('sphrt_rays_cone', 'sphrt_rays_cone_ordered')   # the first kernel launched
    origs = {nm: getattr(lib, nm) for nm in names}

    class Probe:
        def __init__(self, f):
            self.f = f

        def __call__(self, *a):
            first.append(time.perf_counter())
            return self.f(*a)
    for nm in names:
        setattr(lib, nm, Probe(origs[nm]))
    starts, walls = [], []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        starts.append(t0)
        Operator(grid, geom, device=dev)(x)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    for nm in names:
        setattr(lib, nm, origs[nm])
    n = args.reps
    out = {'config': args.config, 'wall_ms': 1e3 * sorted(walls)[n // 2],
           'host_until_first_kernel_ms': (1e3 * sum(f - s for f, s in zip(first, starts)) / n
                                          if len(first) == n else None),
           'per_operator_ms': {k: round(1e3 * v / n, 4) for k, v in
                               sorted(ACC.items(), key=lambda kv: -kv[1])}}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
