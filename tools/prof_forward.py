#!/usr/bin/env python3
"""Apply-kernel study on a bench workload: mean per-launch time of the forward (f32, f64) and the
adjoint, from HIP events around graph-replayed launches, interleaved rounds in one process
(guide §5.4 rule 24).

    python tools/prof_forward.py [--config c2] [--rounds 5] [--reps 50]
    python tools/prof_forward.py --only [--reps 20] [--dtype f64]   # bare forwards, for rocprofv3 --pmc
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def graph_time_us(fn, reps):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        for _ in range(3):
            g.replay()
        e1.record(side)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--config', default='c2')
    ap.add_argument('--only', action='store_true')
    ap.add_argument('--dtype', default='f32', choices=['f32', 'f64'], help='--only: forward dtype')
    ap.add_argument('--adjoint', action='store_true',
                    help='--only: the adjoint instead (op.T, or the time-paired gradient of a '
                         'dynamic grid): the transposed CSR\'s forward kernel')
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    n, total = op._csr['n'], op._csr['total']
    x32 = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    x64 = x32.double()
    n_chan, div, _ = op._layout(x32.shape)      # (a dynamic grid: view i <-> time slice i)
    o32 = torch.empty(n * (n_chan if div == 0 else 1), dtype=torch.float32, device=dev)
    o64 = torch.empty(o32.shape, dtype=torch.float64, device=dev)
    if args.only:
        xo, oo = (x32, o32) if args.dtype == 'f32' else (x64, o64)
        if args.adjoint:
            yo = torch.rand(tuple(geom.shape), dtype=xo.dtype, device=dev)
            op._apply_adjoint(yo, tuple(xo.shape), xo.dtype, dev)     # builds the transpose
            torch.cuda.synchronize()
            for _ in range(args.reps):
                op._apply_adjoint(yo, tuple(xo.shape), xo.dtype, dev)
            torch.cuda.synchronize()
            return
        for _ in range(args.reps):
            op._launch_forward(xo, oo, n_chan, div)
        torch.cuda.synchronize()
        return
    if grid.dynamic:
        for name, xo, oo in (('forward_f32', x32, o32), ('forward_f64', x64, o64)):
            us = sorted(graph_time_us(lambda: op._launch_forward(xo, oo, n_chan, div), args.reps)
                        for _ in range(args.rounds))
            print(json.dumps({'kernel': name, 'rays': n, 'segments': total,
                              'us_median': us[len(us) // 2], 'us_min': us[0]}))
        return
    y = torch.rand(n, dtype=torch.float64, device=dev)
    acc = torch.zeros(math.prod(cfg[0]), dtype=torch.float64, device=dev)
    lib = _lib.load()

    def adjoint():
        _lib.check(lib.sphrt_adjoint_accumulate(op._csr['desc'], _lib.ptr(y), 1, 1, n, 0,
                                                 _lib.ptr(acc), acc.numel(),
                                                 _lib.stream_of(dev)), 'adjoint')

    T = op._transposed()['desc']
    nvox = acc.numel()
    a64 = torch.empty(nvox, dtype=torch.float64, device=dev)
    a32 = torch.empty(nvox, dtype=torch.float32, device=dev)
    y32 = y.float()

    from sph_raytracer_amd.raytracer import _call_forward

    def adjoint_t(yy, out):     # through _call_forward: a staged T (SPHRT_BRICK_T) gets its stage
        fn = lib.sphrt_forward_f32 if yy.dtype == torch.float32 else lib.sphrt_forward_f64
        _call_forward(fn, T, yy, 1, n, 0, out, nvox, dev)

    variants = {
        'forward_f32': (lambda: op._launch_forward(x32, o32, 1, 0), n * 8 + total * 12),
        'forward_f64': (lambda: op._launch_forward(x64, o64, 1, 0), n * 12 + total * 20),
        'adjoint_T_f32': (lambda: adjoint_t(y32, a32), nvox * 8 + total * 12),
        'adjoint_T_f64': (lambda: adjoint_t(y, a64), nvox * 12 + total * 20),
        'adjoint_atomic_f64': (adjoint, n * 12 + total * (4 + 8 + 16)),
    }
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, (fn, _) in variants.items():
            res[k].append(graph_time_us(fn, args.reps))
    for k, v in res.items():
        v.sort()
        med = v[len(v) // 2]
        print(json.dumps({'kernel': k, 'rays': n, 'segments': total, 'us_median': med,
                          'us_min': v[0], 'alg_GBps': variants[k][1] / (med * 1e-6) / 1e9}))


if __name__ == '__main__':
    main()
