#!/usr/bin/env python3
"""Host-side cost of a steady-state Operator call (C2): op(x) issue rate (CPython fast path, and
the ctypes-only path) vs the bare C launch."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rate(fn, reps=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6


def main():
    import bench
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS['c2']
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    x = torch.rand(cfg[0], device=dev)
    n = op._csr['n']
    out = torch.empty(n, device=dev)
    op(x)
    lib = _lib.load()
    desc = op._csr['desc']
    st = torch.cuda.current_stream(dev).cuda_stream
    n_vox = x.numel()
    fc = op._fastc
    op_ct = Operator(grid, geom, device=dev)      # the same call through ctypes only
    op_ct(x)
    op_ct._fastc = None
    for name, fn in [
        ('op(x)', lambda: op(x)),
        ('op(x) ctypes', lambda: op_ct(x)),
        ('torch.empty', lambda: torch.empty(n, device=dev)),
        ('current_stream', lambda: torch.cuda.current_stream(dev).cuda_stream),
        ('bare C launch', lambda: lib.sphrt_forward_f32(desc, x.data_ptr(), 1, n_vox, 0,
                                                         out.data_ptr(), n, st)),
    ]:
        issue, total = rate(fn)
        print(f'{name:16s} issue {issue:7.2f} us/call   issue+drain {total:7.2f} us/call', flush=True)


if __name__ == '__main__':
    main()
