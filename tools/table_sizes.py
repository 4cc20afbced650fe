#!/usr/bin/env python3
"""Distribution of the per-workgroup granule-table sizes (blocks field n_tab) of a bench config's
trace CSR (and its transpose): the table stride, i.e. the LDS image every forward workgroup
reserves, is set by the largest table.

    python tools/table_sizes.py [c5]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(blocks, stride, what):
    n_tab = blocks.view(-1, 6)[:, 5].cpu().numpy()
    t = n_tab[n_tab >= 0]
    q = np.percentile(t, [50, 90, 95, 99, 99.9]).round(1).tolist()
    return {'what': what, 'blocks': int(len(n_tab)), 'fallback_blocks': int((n_tab < 0).sum()),
            'tab_stride': int(stride), 'mean': round(float(t.mean()), 1),
            'p50_p90_p95_p99_p999': q, 'max': int(t.max())}


def main():
    import bench
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    name = sys.argv[1] if len(sys.argv) > 1 else 'c5'
    cfg = bench.CONFIGS[name]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    c = op._csr
    out = [stats(c['blocks'], c['desc'].tab_stride, f'{name} trace')]
    if not grid.dynamic:
        x = torch.rand(grid.shape, dtype=cfg[4], device=dev, requires_grad=True)
        op(x).sum().backward()
        t = op._transposed()
        out.append(stats(t['keep'][6], t['desc'].tab_stride, f'{name} transposed'))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
