#!/usr/bin/env python3
"""One-pass trace bounds against the true segment counts on a bench configuration: every bound
must hold (else the emit pass overflows and the trace falls back to two passes); prints the
staging size the bounds reserve.

    python tools/bound_check.py [c2 c3 c5]
"""
import json
import os
import sys

import torch as tr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(cfgs):
    import bench
    from sph_raytracer_amd import _lib, raytracer as rt
    dev = tr.device('cuda', 0)
    lib = _lib.load()
    st = _lib.stream_of(dev)
    for name in cfgs:
        grid, geom = bench.build_geometry(bench.CONFIGS[name], 0, 1)
        plan = rt._Plan(grid, dev)
        batch = rt._RayBatch(grid, geom.ray_starts, rt._geom_rays(geom, dev), dev)
        n = batch.n
        bound = tr.empty(n, dtype=tr.int32, device=dev)
        count = tr.empty(n, dtype=tr.int32, device=dev)
        tws = rt._workspace(lib, plan, n, dev)
        _lib.check(lib.sphrt_trace_bound(plan.handle, batch.desc, _lib.ptr(bound), _lib.ptr(tws),
                                         tws.numel(), st), 'sphrt_trace_bound')
        _lib.check(lib.sphrt_trace_count(plan.handle, batch.desc, _lib.ptr(count), _lib.ptr(tws),
                                         tws.numel(), st), 'sphrt_trace_count')
        b, c = bound.long(), count.long()
        print(json.dumps({'config': name, 'rays': n, 'violations': int((b < c).sum()),
                          'bound_sum': int(b.sum()), 'count_sum': int(c.sum()),
                          'slack': float(b.sum()) / max(float(c.sum()), 1.0)}))


if __name__ == '__main__':
    main(sys.argv[1:] or ['c2', 'c3', 'c5'])
