#!/usr/bin/env python3
"""Debug: native build_rays against the Python construction for the generic-geometry cases."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import test_construct as t
    from sph_raytracer_amd import Operator, _lib
    from sph_raytracer_amd import raytracer as R
    dev = torch.device('cuda', 0)
    for name in ('parallel_single', 'parallel_orbit', 'viewgeom_rays', 'parallel_dynamic'):
        grid, geom = t.GPU_CASES[name]()
        os.environ.pop('SPHRT_CONSTRUCT', None)
        a = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
        os.environ['SPHRT_CONSTRUCT'] = 'python'
        b = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
        os.environ.pop('SPHRT_CONSTRUCT', None)
        print(name, 'native' if isinstance(a._batch, R._NativeBatch) else 'python', a._ray_shape,
              b._ray_shape, a._csr['total'], b._csr['total'], flush=True)
        if isinstance(a._batch, R._NativeBatch):
            xs = a._batch.xs.cpu()
            print('  xs', tuple(xs.shape), bool(torch.equal(xs, geom.ray_starts.expand(xs.shape))),
                  flush=True)
        fc = _lib.load_construct()
        c = _lib.CSR()
        import ctypes
        g = grid
        res = fc.build_rays(geom.ray_starts, geom.rays, g.r_b, g.e_b, g.a_b, g.shape.r, g.shape.e,
                            g.shape.a, 16 * 18 * 20, ctypes.addressof(c))
        print('  direct', None if res is None else (res[13], res[15]), flush=True)


if __name__ == '__main__':
    main()
