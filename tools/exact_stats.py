#!/usr/bin/env python3
"""Exact-path counters of a count pass over a bench configuration: deferred rays and depth-limit
ranges rank-sorted in parallel / heap-sorted by one lane (trace.hip exact_heap_range); hit rays.

    python tools/exact_stats.py [c2 c3 c4 c5]
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
    for name in cfgs:
        grid, geom = bench.build_geometry(bench.CONFIGS[name], 0, 1)
        plan = rt._Plan(grid, dev)
        batch = rt._RayBatch(grid, geom.ray_starts, rt._geom_rays(geom, dev), dev)
        counts = tr.empty(max(batch.n, 1), dtype=tr.int32, device=dev)
        tws = rt._workspace(lib, plan, batch.n, dev)
        _lib.check(lib.sphrt_trace_count(plan.handle, batch.desc, _lib.ptr(counts), _lib.ptr(tws),
                                         tws.numel(), _lib.stream_of(dev)), 'sphrt_trace_count')
        head = tws[:256].cpu().view(tr.int64)
        print(json.dumps({'config': name, 'rays': batch.n, 'deferred': int(head[0]),
                          'heap_rank_sorted': int(head[16]), 'heap_serial': int(head[17]),
                          'hit_rays': int(tws[64:68].cpu().view(tr.int32)[0])}))


if __name__ == '__main__':
    main(sys.argv[1:] or ['c2', 'c3', 'c4', 'c5'])
