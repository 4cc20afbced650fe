#!/usr/bin/env python3
"""The fixed cost of one `gd` call on C5 (retrieval._gd_direct): wall time of gd at several
iteration counts (slope = per-iteration time, intercept = the call's fixed cost) and the host
pieces of that fixed cost measured one by one.

    python tools/gd_fixed.py [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS['c5']
    torch.manual_seed(0)
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    truth = torch.zeros(grid.shape, dtype=torch.float64, device=dev)
    truth[:, 32:, :32] = 1
    truth[:, :32, 32:] = 1
    y = op(truth)
    model = FullyDenseModel(grid)
    losses = [SquareLoss(), NegRegularizer()]

    def gd(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = retrieval.gd(op, y, model, num_iterations=n, loss_fns=losses, lr=1e-1,
                           progress_bar=False)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, out

    gd(3)
    rec = {'gd_ms': {}}
    for n in (1, 11, 101):
        rec['gd_ms'][n] = statistics.median(gd(n)[0] for _ in range(a.reps)) * 1e3
    slope = (rec['gd_ms'][101] - rec['gd_ms'][1]) / 100
    rec['per_iteration_ms'] = slope
    rec['fixed_ms'] = rec['gd_ms'][1] - slope

    def piece(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e3

    coeffs = torch.ones(model.coeffs_shape, requires_grad=True, device=dev, dtype=torch.float64)
    rec['pieces_ms'] = {
        'torch.optim.Adam(...)': piece(lambda: torch.optim.Adam([coeffs], lr=1e-1)),
        '_direct_plan': piece(lambda: retrieval._direct_plan(op, y, model, coeffs, losses, [coeffs])),
        'f(model(best)) (the return value)': piece(lambda: op(model(coeffs.detach()))),
        'sync only': piece(lambda: None),
    }
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
