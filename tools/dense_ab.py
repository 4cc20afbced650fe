#!/usr/bin/env python3
"""Same-process A/B of the dense-range closes of a time-paired adjoint (C4): the occupancy
bitmap (compact closes, sphrt_csr.out_bits set) against row_ray closes (out_bits cleared),
alternating rounds of dispatch-timed kernel launches.

    python tools/dense_ab.py [--config c4] [--rounds 6] [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c4')
    ap.add_argument('--rounds', type=int, default=6)
    ap.add_argument('--reps', type=int, default=50)
    args = ap.parse_args()
    import bench
    from adjoint_stats import dispatch_us
    from sph_raytracer_amd import Operator, _lib
    from sph_raytracer_amd.raytracer import _call_forward
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    y = torch.rand(tuple(geom.shape), dtype=cfg[4], device=dev)
    g0 = op._apply_adjoint(y, tuple(x.shape), x.dtype, dev)
    n_chan, div, _ = op._layout(x.shape)
    c = op._paired(x.shape[0], div)['transposed']['desc']
    bits = c.out_bits
    res = torch.empty(x.numel(), dtype=x.dtype, device=dev)
    fn = lib.sphrt_forward_f32 if x.dtype == torch.float32 else lib.sphrt_forward_f64
    yv = y.reshape(-1)

    def launch():
        _call_forward(fn, c, yv, 1, op._csr['n'], 0, res, res.numel(), dev)
    out = {'config': args.config, 'bitmap': [], 'row_ray': []}
    for r in range(args.rounds):
        for name, b in (('bitmap', bits), ('row_ray', None)) if r % 2 == 0 else \
                (('row_ray', None), ('bitmap', bits)):
            c.out_bits = b
            launch()
            out[name].append(dispatch_us(launch, args.reps, lib)[0])
            assert torch.equal(res.view(x.shape), g0)
    c.out_bits = bits
    for k in ('bitmap', 'row_ray'):
        v = sorted(out[k])
        out[k + '_median_us'] = v[len(v) // 2]
    print(json.dumps(out))


if __name__ == '__main__':
    main()
