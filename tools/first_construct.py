#!/usr/bin/env python3
"""Where the FIRST Operator of a config in a process spends its time (the
first dynamic C4 Operator + first forward took 0.7-0.95 s against ~1 ms for later ones).

    python tools/first_construct.py [--warm c2] [--config c4] [--profile]

Phases, each bracketed by torch.cuda.synchronize: the warm-up config's Operator + forward (HIP,
allocator, library loading), then for --config: geometry, Operator(...), first forward, second
forward, a second Operator + first forward.  --profile adds a cProfile of the first Operator +
first forward (top entries by cumulative time) to the JSON line.
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--warm', default='c2', help="config built first ('none': skip)")
    ap.add_argument('--config', default='c4')
    ap.add_argument('--profile', action='store_true')
    ap.add_argument('--top', type=int, default=25)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    rec = {'config': args.config, 'warm': args.warm}

    def sync_time(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize(dev)
        return r, (time.perf_counter() - t0) * 1e3

    t_start = time.perf_counter()
    torch.cuda.init()
    torch.zeros(1, device=dev)
    rec['cuda_init_ms'] = (time.perf_counter() - t_start) * 1e3
    if args.warm != 'none':
        cw = bench.CONFIGS[args.warm]
        gw, geow = bench.build_geometry(cw, 0, 1)
        xw = torch.rand(cw[0], dtype=cw[4], device=dev)
        _, rec['warm_operator_forward_ms'] = sync_time(
            lambda: Operator(gw, geow, device=dev, dynamic=gw.dynamic)(xw))
    cfg = bench.CONFIGS[args.config]
    (grid, geom), rec['geometry_ms'] = sync_time(lambda: bench.build_geometry(cfg, 0, 1))
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    pr = cProfile.Profile() if args.profile else None
    if pr:
        pr.enable()
    op, rec['first_operator_ms'] = sync_time(
        lambda: Operator(grid, geom, device=dev, dynamic=grid.dynamic))
    _, rec['first_forward_ms'] = sync_time(lambda: op(x))
    if pr:
        pr.disable()
    _, rec['second_forward_ms'] = sync_time(lambda: op(x))
    if grid.dynamic:
        y = torch.rand(tuple(geom.shape), dtype=cfg[4], device=dev)
        _, rec['first_gradient_ms'] = sync_time(
            lambda: op._apply_adjoint(y, tuple(x.shape), x.dtype, dev))
        _, rec['second_gradient_ms'] = sync_time(
            lambda: op._apply_adjoint(y, tuple(x.shape), x.dtype, dev))
    del op
    _, rec['second_operator_forward_ms'] = sync_time(
        lambda: Operator(grid, geom, device=dev, dynamic=grid.dynamic)(x))
    if pr:
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats('cumulative').print_stats(args.top)
        rec['profile_cumulative'] = s.getvalue().splitlines()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(args.top)
        rec['profile_tottime'] = s.getvalue().splitlines()
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
