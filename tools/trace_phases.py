#!/usr/bin/env python3
"""Trace-kernel phase split from a stamped build: s_memtime cycles per hit ray and phase.

    python tools/build_variants.py tstamps=-DSPHRT_TRACE_STAMPS
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so python tools/trace_phases.py [c2]
"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sph_raytracer_amd import _lib
    from sph_raytracer_amd.raytracer import line_integrals
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c2']
    grid, geom = bench.build_geometry(cfg, 0, 1)
    lib = _lib.load()
    lib.sphrt_diag_trace_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    x = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    Operator(grid, geom, device=dev)          # warm-up (count + fill)
    torch.cuda.synchronize()
    rec = {}
    for name, fn in (('operator (count+fill)', lambda: Operator(grid, geom, device=dev)),
                     ('fused line_integrals', lambda: line_integrals(grid, geom, x))):
        lib.sphrt_diag_trace_cycles(None, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        buf = (ctypes.c_ulonglong * 24)()
        lib.sphrt_diag_trace_cycles(ctypes.cast(buf, ctypes.c_void_p), 0)
        n = max(buf[5], 1)
        ne = max(buf[8], 1)
        rec[name] = {'rays_traced': buf[5], 'mean_F': buf[6] / n, 'wall_ms': wall * 1e3,
                     'cycles_per_ray': {k: buf[i] / n for i, k in enumerate(
                         ['solve', 'sort', 'ties', 'fill', 'emit'])},
                     'exact_rays': buf[8],
                     'exact_cycles_per_ray': {k: buf[9 + i] / ne for i, k in enumerate(
                         ['candidates', 'partition', 'leaf_ranks', 'walk'])}}
    print(json.dumps(rec, indent=1))


if __name__ == '__main__':
    main()
