#!/usr/bin/env python3
"""Operator construction + first forward (the reference's cold definition, as bench.py's
`operator_seconds`) on a bench config, median of --reps warm repetitions; for A/B runs of
environment switches (e.g. SPHRT_TABLE_SORT=radix) and under rocprofv3 for the kernel split.

    python tools/operator_time.py --config c3 [--reps 7] [--ftype float32] [--invalid]

--ftype float32 / --invalid time the reference-mode trace (sphrt_trace_reference: every ray
through the exact path, count then fill; raytracer.py:48-173 with those options).
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
    ap.add_argument('--config', default='c3')
    ap.add_argument('--reps', type=int, default=7)
    ap.add_argument('--adjoint', action='store_true',
                    help='also the first op.T(y) of each Operator (builds the transposed CSR)')
    ap.add_argument('--ftype', default='float64', choices=('float64', 'float32'))
    ap.add_argument('--invalid', action='store_true')
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    kw = dict(ftype=getattr(torch, args.ftype), invalid=args.invalid)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # the first Operator of the process (recorded beside the warm median;
    # it also pays HIP's loading of the library's code objects and torch's first-use costs)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic, **kw)
    y = op(x)
    if args.adjoint:
        op.T(y)
    torch.cuda.synchronize(dev)
    t_first = time.perf_counter() - t0
    del op
    times = []
    for _ in range(args.reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op = Operator(grid, geom, device=dev, dynamic=grid.dynamic, **kw)
        y = op(x)
        if args.adjoint:
            op.T(y)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
        op_n = op._csr['n']
        del op
    times.sort()
    env = {k: v for k, v in os.environ.items() if k.startswith('SPHRT_')}
    med = times[len(times) // 2]
    n = int(op_n)
    print(json.dumps({'config': args.config, 'adjoint': args.adjoint, 'ftype': args.ftype,
                      'invalid': args.invalid, 'operator_ms_median': 1e3 * med,
                      'operator_ms_min': 1e3 * times[0], 'operator_ms_first': 1e3 * t_first,
                      'rays': n,
                      'rays_per_s_median': n / med, 'reps': args.reps, 'env': env}))


if __name__ == '__main__':
    main()
