#!/usr/bin/env python3
"""Calibrate oracle/ref_trace.py (the cold-path CPU baseline) against the reference itself.

Runs in the survey container only (it imports /root/reference through tests/golden/refshim.py):
for each workload, the reference's trace_indices and ref_trace.trace_dense on the same rays —
outputs compared bit for bit, wall times (median of 3 after a warm-up, torch's thread count) side
by side.  SURVEY §8(d) asks for identical output and wall time within +-20 %.

    python tools/calibrate_ref_trace.py [--threads 8] [--out profiles/r03_ref_trace_calibration.json]
"""
import argparse
import json
import os
import sys
import time

import torch as tr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))


def med(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    tr.set_num_threads(args.threads)
    import refshim
    from oracle import ref_trace
    R = refshim.load()
    G, RT = R.geometry, R.raytracer

    def orbit(n_obs, views, mk):
        th = tr.linspace(0, 2 * tr.pi, n_obs)[list(views)]
        return sum(mk((5 * tr.cos(t), 5 * tr.sin(t), 1)) for t in th)

    cases = {
        'C1': (G.SphericalGrid(shape=(50, 50, 50)),
               G.ConeRectGeom((50, 100), pos=(5, 0, 0), fov=(45, 45))),
        'C2': (G.SphericalGrid(shape=(50, 50, 50)),
               orbit(50, range(50), lambda p: G.ConeRectGeom((50, 100), pos=p, fov=(45, 45)))),
        'C5 (8 of 64 views)': (G.SphericalGrid(shape=(64, 64, 64)),
                               orbit(64, range(0, 64, 8),
                                     lambda p: G.ConeCircGeom(shape=(100, 50), pos=p, fov=(0, 45)))),
    }
    res = {'threads': tr.get_num_threads(), 'cpus': os.cpu_count(), 'cases': {}}
    for name, (grid, geom) in cases.items():
        xs, rays = geom.ray_starts, geom.rays
        xb = xs.broadcast_to(rays.shape).reshape(-1, 3).clone()
        rb = rays.reshape(-1, 3).clone()
        starts = RT.find_starts(grid, xb)

        def ref():
            return RT.trace_indices(grid, xb.clone(), rb.clone())

        def mine():
            return ref_trace.trace_dense(grid.r_b, grid.e_b, grid.a_b, xb, rb, starts)

        t_ref, (regs_r, lens_r) = med(ref)
        t_mine, (regs_m, lens_m) = med(mine)
        same = bool(tr.equal(regs_r, regs_m) and tr.equal(lens_r, lens_m))
        rec = {'rays': len(xb), 'K': lens_r.shape[-1], 'reference_s': t_ref, 'restatement_s': t_mine,
               'ratio': t_mine / t_ref, 'bitwise_identical': same}
        res['cases'][name] = rec
        print(name, json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
