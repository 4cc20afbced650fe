#!/usr/bin/env python3
"""Trace-path timings on a bench config: Operator construction (count + scan + fill + CSR index +
granule tables) and the fused no-store forward (line_integrals), several times each.  Run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations.

    python tools/trace_bench.py [c2] [--reps 3]
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
    ap.add_argument('config', nargs='?', default='c2')
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    from sph_raytracer_amd.raytracer import line_integrals
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    Operator(grid, geom, device=dev)(x)
    line_integrals(grid, geom, x)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (('operator_init', lambda: Operator(grid, geom, device=dev)),
                     ('line_integrals', lambda: line_integrals(grid, geom, x))):
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res[name + '_ms'] = sorted(ts)[len(ts) // 2]
    print(json.dumps(res))


if __name__ == '__main__':
    main()
