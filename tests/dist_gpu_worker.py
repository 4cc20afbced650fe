"""One rank of tests/test_gpu_distributed.py: ShardedOperator over the real HIP Operator.

Launched as a plain child process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment), every rank on cuda:0 over gloo (a one-GPU box cannot give two RCCL ranks one
device), or — SPHRT_DIST_BACKEND=nccl, world size 1 — over RCCL with device tensors, so the
all_gather_into_tensor / device all_reduce branches of distributed.py run (counted, and required).  Each rank checks its results itself (a failed check exits non-zero) and rank 0 writes
the measured differences to $SPHRT_DIST_OUT as JSON.
"""
import json
import os
import sys

import torch as tr
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def orbit(n_views, det, grid_shape, kind):
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, SphericalGrid
    grid = SphericalGrid(shape=grid_shape)
    mk = (lambda p: ConeRectGeom(det, pos=p, fov=(45, 45))) if kind == 'rect' else \
        (lambda p: ConeCircGeom(shape=det, pos=p, fov=(0, 45)))
    return grid, sum(mk((5 * tr.cos(t), 5 * tr.sin(t), 1)) for t in tr.linspace(0, 2 * tr.pi, n_views))


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def main():
    dev = tr.device('cuda', 0)
    tr.cuda.set_device(dev)
    backend = os.environ.get('SPHRT_DIST_BACKEND', 'gloo')
    seen = {'all_gather_into_tensor': 0, 'all_reduce_cuda': 0}
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=dev)
        # count the device-side collectives the RCCL path issues (distributed.py)
        agit, ar = dist.all_gather_into_tensor, dist.all_reduce

        def agit_spy(out, inp, *a, **k):
            seen['all_gather_into_tensor'] += int(inp.is_cuda)
            return agit(out, inp, *a, **k)

        def ar_spy(t, *a, **k):
            seen['all_reduce_cuda'] += int(t.is_cuda)
            return ar(t, *a, **k)

        dist.all_gather_into_tensor, dist.all_reduce = agit_spy, ar_spy
    else:
        dist.init_process_group('gloo')
    rank = dist.get_rank()
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.distributed import ShardedOperator, gd as dgd
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    res = {}
    g = tr.Generator().manual_seed(0)

    # static grid: full stack, multichannel, adjoint
    grid, geom = orbit(7, (32, 40), (30, 28, 32), 'rect')
    sop = ShardedOperator(grid, geom, device=dev)
    single = Operator(grid, geom, device=dev)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g).to(dev)
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, generator=g).to(dev)
    for dt in (tr.float64, tr.float32):
        got, want = sop.forward_full(x.to(dt)), single(x.to(dt))
        assert got.shape == want.shape and got.dtype == dt
        res[f'fwd_{dt}'] = rel(got, want)
        res[f'fwd_bitwise_{dt}'] = bool(tr.equal(got, want))
    xc = tr.stack([x, 2 * x, x * x])
    res['fwd_mc'] = rel(sop.forward_full(xc), single(xc))
    res['T'] = rel(sop.T(y), single.T(y))
    # the sharded results for the parent's oracle comparison (rank 0; every rank holds them)
    sharded = {'x': x.cpu(), 'y': y.cpu(), 'fwd': sop.forward_full(x).cpu(), 'T': sop.T(y).cpu()}

    # dynamic grid: view i <-> time slice i; forward, autograd gradient, adjoint
    dgrid, dgeom = orbit(6, (16, 12), (6, 12, 10, 14), 'circ')
    dop = ShardedOperator(dgrid, dgeom, device=dev)
    dsingle = Operator(dgrid, dgeom, device=dev)
    xd = tr.rand(dgrid.shape, dtype=tr.float64, generator=g).to(dev)
    yd = tr.rand(tuple(dgeom.shape), dtype=tr.float64, generator=g).to(dev)
    res['dyn_fwd'] = rel(dop.forward_full(xd), dsingle(xd))
    xg = xd.clone().requires_grad_()
    (dop(xg) * yd[dop.lo:dop.hi]).sum().backward()
    grad = dop.all_reduce(xg.grad)          # each rank's slices -> the full gradient
    xs = xd.clone().requires_grad_()
    (dsingle(xs) * yd).sum().backward()
    res['dyn_grad'] = rel(grad, xs.grad)
    res['dyn_T'] = rel(dop.T(yd), xs.grad)

    # data-parallel retrieval (the static_retrieval.py loop) vs the single-GPU loop
    cgrid, cgeom = orbit(12, (20, 16), (16, 16, 16), 'circ')
    cop = ShardedOperator(cgrid, cgeom, device=dev)
    csingle = Operator(cgrid, cgeom, device=dev)
    truth = tr.zeros(cgrid.shape, dtype=tr.float64, device=dev)
    truth[:, 8:, :8] = 1
    truth[:, :8, 8:] = 1
    meas = csingle(truth)
    calls = []
    direct = retrieval._gd_direct

    def spy(*a, **k):
        calls.append(1)
        return direct(*a, **k)

    retrieval._gd_direct = spy
    fns = [SquareLoss(), NegRegularizer()]
    c_d, stack, l_d = dgd(cop, meas[cop.lo:cop.hi].clone(), FullyDenseModel(cgrid),
                          num_iterations=25, lr=0.1, loss_fns=fns)
    fns1 = [SquareLoss(), NegRegularizer()]
    c_s, y_s, l_s = retrieval.gd(csingle, meas.clone(), FullyDenseModel(cgrid), num_iterations=25,
                                 lr=0.1, loss_fns=fns1, progress_bar=False)
    retrieval._gd_direct = direct
    assert calls == [1, 1], calls               # both took the autograd-free loop
    res['gd_coeffs_abs'] = float((c_d - c_s).abs().max())
    res['gd_stack'] = rel(stack, y_s)
    a, b = tr.tensor(l_d[fns[0]]), tr.tensor(l_s[fns1[0]])
    res['gd_sqloss'] = float(((a - b).abs() / b.abs()).max())
    res['gd_negloss_abs'] = float((tr.tensor(l_d[fns[1]]) - tr.tensor(l_s[fns1[1]])).abs().max())
    res['gd_drop'] = float(a[-1] / a[0])

    tol = {'fwd_torch.float64': 1e-13, 'fwd_torch.float32': 1e-6, 'fwd_mc': 1e-13, 'T': 1e-12,
           'dyn_fwd': 1e-13, 'dyn_grad': 1e-12, 'dyn_T': 1e-12, 'gd_coeffs_abs': 1e-12,
           'gd_stack': 1e-12, 'gd_sqloss': 1e-12, 'gd_negloss_abs': 1e-15}
    bad = {k: res[k] for k, t in tol.items() if not res[k] <= t}
    res['rank'] = rank
    res['backend'] = backend
    res['collectives'] = dict(seen)
    if backend == 'nccl' and not (seen['all_gather_into_tensor'] and seen['all_reduce_cuda']):
        bad['rccl_path_not_taken'] = dict(seen)
    if rank == 0 and os.environ.get('SPHRT_DIST_OUT'):
        tr.save(sharded, os.environ['SPHRT_DIST_OUT'] + '.pt')
        with open(os.environ['SPHRT_DIST_OUT'], 'w') as fh:
            json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        print(f'rank {rank}: out of tolerance {bad}', file=sys.stderr)
        sys.exit(1)


if __name__ == '__main__':
    main()
