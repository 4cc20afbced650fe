#!/usr/bin/env python3
"""Forward-kernel study on a bench workload: granule-table statistics and the per-launch time of
the table mode against the per-segment gather mode (same CSR, desc.loc cleared), f32 and f64.

    python tools/fwd_study.py [--config c3] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prof_forward import graph_time_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    c = op._csr
    n, total, nb = c['n'], c['total'], c['nblocks']
    blocks = c['blocks'].view(nb, 6).cpu()
    segs = (blocks[:, 3] - blocks[:, 2]).double()
    ntab = blocks[:, 5].double()
    ok = ntab >= 0
    stats = {'config': args.config, 'rays': n, 'segments': total, 'blocks': nb,
             'tab_stride': c['desc'].tab_stride, 'n_fallback': c['desc'].n_fallback,
             'seg_per_block_mean': segs.mean().item(), 'seg_per_block_max': segs.max().item(),
             'gran_per_block_mean': ntab[ok].mean().item(), 'gran_per_block_max': ntab[ok].max().item(),
             'segments_per_granule': (segs[ok].sum() / ntab[ok].sum()).item(),
             'volume_granules': (torch.tensor(cfg[0]).prod().item() + 3) // 4}
    print(json.dumps(stats), flush=True)
    x32 = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    x64 = x32.double()
    o32 = torch.empty(n, dtype=torch.float32, device=dev)
    o64 = torch.empty(n, dtype=torch.float64, device=dev)
    res = {}
    for mode in ('table', 'gather'):
        loc = c['desc'].loc
        if mode == 'gather':
            c['desc'].loc = None
        try:
            for name, x, o in (('f32', x32, o32), ('f64', x64, o64)):
                res[f'{mode}_{name}'] = graph_time_us(lambda: op._launch_forward(x, o, 1, 0), args.reps)
                res[f'{mode}_{name}_out'] = o.double().sum().item()
        finally:
            c['desc'].loc = loc
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
