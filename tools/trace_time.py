#!/usr/bin/env python3
"""Time the trace count pass (screen + trace + exact kernels) and the fused forward on a bench
config with HIP events; for A/B builds (SPHRT_LIB=...).

    python tools/trace_time.py [c2]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sph_raytracer_amd import _lib
    from sph_raytracer_amd.raytracer import _Plan, _RayBatch, _geom_rays, _workspace
    dev = torch.device('cuda', 0)
    name = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    cfg = bench.CONFIGS[name]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    lib = _lib.load()
    plan = _Plan(grid, dev)
    batch = _RayBatch(grid, geom.ray_starts, _geom_rays(geom, dev), dev)
    n = batch.n
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    ws = _workspace(lib, plan, n, dev)
    st = _lib.stream_of(dev)
    x = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)

    def count():
        _lib.check(lib.sphrt_trace_count(plan.handle, batch.desc, _lib.ptr(counts), _lib.ptr(ws),
                                         ws.numel(), st), 'count')

    def fused():
        _lib.check(lib.sphrt_trace_integrate_f32(plan.handle, batch.desc, _lib.ptr(x), 1,
                                                 x.numel(), 0, _lib.ptr(out), n, _lib.ptr(ws),
                                                 ws.numel(), st), 'integrate')
    res = {'lib': os.path.basename(os.environ.get('SPHRT_LIB', 'libsphrt.so')), 'config': name}
    for k, fn in (('count_us', count), ('fused_us', fused)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[k] = e0.elapsed_time(e1) * 100
        if k == 'count_us':       # rays sent to the exact path (the workspace's first word)
            res['deferred'] = int(ws[:8].cpu().view(torch.int64)[0])
    print(json.dumps(res))


if __name__ == '__main__':
    main()
