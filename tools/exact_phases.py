#!/usr/bin/env python3
"""exact_wave_kernel phase split (deferred exact-tie rays) from a stamped build: s_memtime
cycles per deferred ray for the candidate solve, the partition phase, the leaf ranks and the walk.

    python tools/build_variants.py tstamps=-DSPHRT_TRACE_STAMPS
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so python tools/exact_phases.py [c5]
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
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c5']
    grid, geom = bench.build_geometry(cfg, 0, 1)
    lib = _lib.load()
    lib.sphrt_diag_trace_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    Operator(grid, geom, device=dev)
    torch.cuda.synchronize()
    lib.sphrt_diag_trace_cycles(None, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Operator(grid, geom, device=dev)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    buf = (ctypes.c_ulonglong * 24)()
    lib.sphrt_diag_trace_cycles(ctypes.cast(buf, ctypes.c_void_p), 0)
    n = max(buf[8], 1)
    print(json.dumps({'deferred_rays_both_passes': buf[8], 'wall_ms': wall * 1e3, 'cycles_per_ray': {
        k: buf[9 + i] / n for i, k in enumerate(['candidates', 'partitions', 'leaf_ranks', 'walk'])},
        'max_ray_cycles': buf[13], 'max_partition_cycles': buf[14], 'heap_sorted_ranges': buf[15],
        'wave_partitions_per_ray': buf[16] / n, 'cycles_per_partition': buf[17] / max(buf[16], 1),
        'cycles_per_heap_range': buf[18] / max(buf[15], 1)}))


if __name__ == '__main__':
    main()
