#!/usr/bin/env python3
"""Host profile of the cold path (Operator construction + first forward): cProfile over --reps
warm repetitions, the top entries by internal and cumulative time.

    python tools/cold_pyprof.py [--config c2] [--reps 30]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=30)
    ap.add_argument('--top', type=int, default=40)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    grid, geom = bench.build_geometry(cfg, 0, 1)
    for _ in range(3):
        Operator(grid, geom, device=dev)(x)
    torch.cuda.synchronize(dev)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.reps):
        Operator(grid, geom, device=dev)(x)
        torch.cuda.synchronize(dev)
    pr.disable()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(args.top)
        print(s.getvalue())


if __name__ == '__main__':
    main()
