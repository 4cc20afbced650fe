#!/usr/bin/env python3
"""Operator construction + first forward (bench.py's `operator_seconds`), median of --reps, for the
package in this tree or in another directory (--pkg DIR: a copy of an earlier revision's
sph_raytracer_amd with its built libraries), for same-box A/B of cold-path changes.

    python tools/cold_ab.py --config c3 [--pkg _ab_base] [--reps 9] [--dtype float64]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    ap.add_argument('--pkg', default=None)
    ap.add_argument('--reps', type=int, default=9)
    ap.add_argument('--dtype', default=None, choices=(None, 'float32', 'float64'))
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    import torch
    import bench            # (puts ROOT first on sys.path: --pkg goes in front of it after)
    if args.pkg:
        sys.path.insert(0, os.path.abspath(os.path.join(ROOT, args.pkg)))
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    dtype = getattr(torch, args.dtype) if args.dtype else cfg[4]
    x = torch.rand(cfg[0], dtype=dtype, device=dev)
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    op(x)
    del op
    times = []
    for _ in range(args.reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        grid, geom = bench.build_geometry(cfg, 0, 1)
        t1 = time.perf_counter()
        op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
        op(x)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t1)
        del op
    times.sort()
    import sph_raytracer_amd
    print(json.dumps({'config': args.config, 'pkg': args.pkg or '.', 'dtype': str(dtype),
                      'operator_ms_median': 1e3 * times[len(times) // 2],
                      'operator_ms_min': 1e3 * times[0], 'reps': args.reps,
                      'peak_gb': torch.cuda.max_memory_allocated(dev) / 1e9,
                      'module': os.path.relpath(sph_raytracer_amd.__file__, ROOT)}))


if __name__ == '__main__':
    main()
