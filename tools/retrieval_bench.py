#!/usr/bin/env python3
"""The C5 retrieval (BASELINE configs[4], examples/static_retrieval.py shape): 64^3 grid, 64-view
ConeCirc (100,50) orbit, FullyDenseModel, SquareLoss + NegRegularizer, Adam lr 0.1, float64
coefficients, `gd` unchanged.  Reports the Operator construction, the measurement forward and the
per-iteration time of `gd` (forward + adjoint + Adam on the GPU), both the autograd-free loop gd
takes for this configuration and the same loop through autograd (the iterates are compared).

    python tools/retrieval_bench.py [--iters 100] [--out profiles/r01_retrieval_c5.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=100)
    ap.add_argument('--out', default=None)
    ap.add_argument('--pkg', default=None,
                    help='directory holding another revision\'s sph_raytracer_amd (A/B)')
    ap.add_argument('--no-autograd', action='store_true', help='skip the autograd comparison')
    ap.add_argument('--reps', type=int, default=5,
                    help='timed gd calls of each loop (the median is reported)')
    args = ap.parse_args()
    import bench            # (puts ROOT first on sys.path: --pkg goes in front of it after)
    if args.pkg:
        sys.path.insert(0, os.path.abspath(os.path.join(ROOT, args.pkg)))
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS['c5']
    torch.manual_seed(0)
    grid, geom = bench.build_geometry(cfg, 0, 1)
    Operator(grid, geom, device=dev)            # warm-up (kernels loaded, allocator primed)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    op = Operator(grid, geom, device=dev)
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t0
    truth = torch.zeros(grid.shape, dtype=torch.float64, device=dev)   # static_retrieval.py:47-49
    truth[:, 32:, :32] = 1
    truth[:, :32, 32:] = 1
    y = op(truth)
    model = FullyDenseModel(grid)
    losses = [SquareLoss(), NegRegularizer()]
    def run():
        # one warm-up call, then the median of `reps` whole gd calls (each the example's
        # num_iterations, its set-up and the final forward of its return value included)
        retrieval.gd(op, y, model, num_iterations=3, loss_fns=losses, lr=1e-1, progress_bar=False)
        ts = []
        for _ in range(max(args.reps, 1)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = retrieval.gd(op, y, model, num_iterations=args.iters, loss_fns=losses, lr=1e-1,
                               progress_bar=False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        run.times = ts
        return out, sorted(ts)[len(ts) // 2]

    (coeffs, y_hat, hist), t_gd = run()          # the autograd-free loop (retrieval._gd_direct)
    gd_ms_all = [v * 1e3 for v in run.times]
    if args.no_autograd:
        (c_ag, hist_ag, t_ag) = (coeffs, hist, float('nan'))
    else:
        plan = retrieval._direct_plan
        retrieval._direct_plan = lambda *a: None     # the same loop through autograd
        (c_ag, _, hist_ag), t_ag = run()
        retrieval._direct_plan = plan
    fid = hist[losses[0]]
    rec = {'pkg': args.pkg or '.', 'config': 'C5 retrieval: 64^3 grid, 64-view ConeCirc (100,50) orbit, FullyDenseModel, '
                     'SquareLoss + NegRegularizer, Adam lr 0.1, float64',
           'rays': op._csr['n'], 'segments': op._csr['total'], 'iterations': args.iters,
           'operator_init_ms': t_init * 1e3, 'gd_total_ms': t_gd * 1e3,
           'gd_total_ms_all': gd_ms_all, 'gd_timing': f'median of {len(gd_ms_all)} gd calls',
           'ms_per_iteration': t_gd / args.iters * 1e3,
           'ms_per_iteration_autograd': t_ag / args.iters * 1e3,
           'direct_iterates_equal_autograd': bool(torch.equal(coeffs, c_ag)),
           'direct_loss_max_rel_diff': max(
               abs(a - b) / max(abs(b), 1e-300) for k in hist for a, b in zip(hist[k], hist_ag[k])),
           'fidelity_first': fid[0], 'fidelity_last': fid[-1],
           'reference_cpu_s_per_iteration': 1.64,
           'speedup_vs_reference_cpu': 1.64 / (t_gd / args.iters),
           'peak_gb_resident': torch.cuda.max_memory_allocated(dev) / 1e9}
    print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            json.dump(rec, f, indent=1)


if __name__ == '__main__':
    main()
