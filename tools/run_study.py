#!/usr/bin/env python3
"""Study (CPU, oracle solves): how many ascending runs a hit ray's candidate list splits into
when every family is listed in an order that follows the ray — sphere entries by descending
shell, exits by ascending shell; cone roots and half-planes in the ray's sweep direction.  Decides
whether a run merge can replace the bitonic sort of the trace kernel.

    python tools/run_study.py [c2] [--rays 20000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('config', nargs='?', default='c2')
    ap.add_argument('--rays', type=int, default=20000)
    args = ap.parse_args()
    import bench
    from oracle import oracle
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3)
    d = geom.rays.numpy().reshape(-1, 3)
    rng = np.random.default_rng(0)
    pick = rng.choice(len(d), size=min(args.rays, len(d)), replace=False)
    xs, d = np.ascontiguousarray(xs[pick]), np.ascontiguousarray(d[pick])
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ts, _, _ = oracle.solve(g, 0, xs, d)
    te, _, _ = oracle.solve(g, 1, xs, d)
    ta, _, _ = oracle.solve(g, 2, xs, d)
    nbr = g.nr + 1
    nbe = g.ne + 1
    u = d / np.linalg.norm(d, axis=1, keepdims=True)
    tc = -(xs * u).sum(1)
    dd2 = (xs * xs).sum(1) - tc * tc
    R = grid.r_b.numpy()[-1]
    t1c = np.sqrt(np.maximum(R * R - dd2, -1))
    hit = R * R - dd2 > 0
    t_lo, t_hi = tc - t1c, tc + t1c
    sweep_up = (xs[:, 0] * u[:, 1] - xs[:, 1] * u[:, 0]) > 0      # azimuth increases along t
    runs, fams, F = [], {'s': [], 'c': [], 'a': []}, []
    for i in np.nonzero(hit)[0]:
        lo = max(t_lo[i], 0.0)

        def keep(t):
            return t[np.isfinite(t) & (t >= lo) & (t <= t_hi[i])]
        s_in = keep(ts[i, :nbr][::-1])
        s_out = keep(ts[i, nbr:])
        c_a, c_b = keep(te[i, :nbe]), keep(te[i, nbe:])
        pl = keep(ta[i] if sweep_up[i] else ta[i][::-1])
        seq = np.concatenate([s_in, s_out, c_a, c_b, pl])
        F.append(len(seq))
        runs.append(1 + int(np.sum(seq[1:] < seq[:-1])) if len(seq) else 0)
        for k, parts in (('s', [s_in, s_out]), ('c', [c_a, c_b]), ('a', [pl])):
            fams[k].append(sum(1 + int(np.sum(p[1:] < p[:-1])) for p in parts if len(p)))
    runs = np.array(runs)
    print(f'{args.config}: {len(runs)} hit rays of {len(d)} sampled; mean F {np.mean(F):.1f}')
    print('runs: mean %.2f  p50 %d  p90 %d  p99 %d  max %d' % (
        runs.mean(), *np.percentile(runs, [50, 90, 99]), runs.max()))
    for k, v in fams.items():
        v = np.array(v)
        print(f'  family {k}: runs mean {v.mean():.2f} max {v.max()}  '
              f'hist {np.bincount(v)[:12].tolist()}')


if __name__ == '__main__':
    main()
