#!/usr/bin/env python3
"""cProfile of Operator construction + first forward (the cold path's host side) on a bench
config, after a warm-up: where the wall time above the kernels goes.

    python tools/host_profile.py --config c2 [--reps 20]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    for _ in range(3):
        Operator(grid, geom, device=dev)(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        Operator(grid, geom, device=dev)(x)
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.reps):
        Operator(grid, geom, device=dev)(x)
        torch.cuda.synchronize()
    pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats('tottime').print_stats(30)
    print(f'wall per Operator + first forward: {wall * 1e3:.3f} ms (unprofiled)')
    print(out.getvalue()[:8000])


if __name__ == '__main__':
    main()
