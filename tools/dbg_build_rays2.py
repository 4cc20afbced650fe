#!/usr/bin/env python3
"""Debug: build_rays with broadcast (1, 1, 3) rays against the same rays expanded."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sph_raytracer_amd import ParallelGeom, SphericalGrid, _lib, Operator
    torch.zeros(1, device='cuda')
    grid = SphericalGrid(shape=(20, 18, 22))
    geom = ParallelGeom((40, 30), pos=(2, 1.5, 0.4), size=(1.5, 1.2))
    fc = _lib.load_construct()
    g = grid
    for tag, rays in (('bcast', geom.rays), ('full', geom.rays.expand(geom.ray_starts.shape).contiguous()),
                      ('bcast_clone', geom.rays.clone())):
        c = _lib.CSR()
        res = fc.build_rays(geom.ray_starts, rays, g.r_b, g.e_b, g.a_b, 20, 18, 22, 20 * 18 * 22,
                            ctypes.addressof(c))
        rp = res[0].cpu()
        print(tag, tuple(rays.shape), rays.stride(), res[13], (rp[1:] - rp[:-1])[:8].tolist(), flush=True)
    os.environ['SPHRT_CONSTRUCT'] = 'python'
    op = Operator(grid, geom, device='cuda')
    rp = op._csr['row_ptr'].cpu()
    print('python', op._csr['total'], (rp[1:] - rp[:-1])[:8].tolist())


if __name__ == '__main__':
    main()
