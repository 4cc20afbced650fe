"""ShardedOperator on 2 (and 3) CPU ranks over gloo, against the single-process result.

The local operators are the oracle-backed CPU stand-in (tests/cpu_operator.py), so these tests
cover exactly the distributed logic — view sharding, the padded all-gather of the image stack,
the all_reduce of the static adjoint, the communication-free dynamic split and the
data-parallel gd — that runs unchanged over RCCL with the HIP Operator on GPUs.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch as tr
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _geometry(n_obs, dynamic=False):
    from sph_raytracer_amd import ConeCircGeom, SphericalGrid
    grid = SphericalGrid(shape=(n_obs, 6, 5, 7) if dynamic else (6, 5, 7))
    geoms = [ConeCircGeom(shape=(6, 5), pos=(5 * tr.cos(t), 5 * tr.sin(t), 1), fov=(0, 45))
             for t in tr.linspace(0, 2 * tr.pi, n_obs)]
    return grid, sum(geoms)


def _worker(rank, world, port, n_obs, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from cpu_operator import CpuOperator
        from sph_raytracer_amd.distributed import ShardedOperator, gd as dgd
        from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
        from sph_raytracer_amd.model import FullyDenseModel
        res = {}
        # static grid: full stack, adjoint, multichannel
        grid, geom = _geometry(n_obs)
        sop = ShardedOperator(grid, geom, operator_factory=lambda g, lg, d: CpuOperator(g, lg))
        g = tr.Generator().manual_seed(0)
        x = tr.rand(grid.shape, dtype=tr.float64, generator=g)
        y = tr.rand(geom.shape, dtype=tr.float64, generator=g)
        res['fwd'] = sop.forward_full(x).numpy()
        res['fwd_mc'] = sop.forward_full(tr.stack([x, 2 * x])).numpy()
        res['adj'] = sop.T(y).numpy()
        # dynamic grid: view i <-> time slice i
        dgrid, dgeom = _geometry(n_obs, dynamic=True)
        dop = ShardedOperator(dgrid, dgeom, operator_factory=lambda g, lg, d: CpuOperator(g, lg))
        xd = tr.rand(dgrid.shape, dtype=tr.float64, generator=g)
        res['dyn'] = dop.forward_full(xd).numpy()
        yd = tr.rand(dgeom.shape, dtype=tr.float64, generator=g)
        res['dyn_T'] = dop.T(yd).numpy()          # each rank's slices, all-gathered
        # data-parallel retrieval, 5 Adam steps
        meas = sop.forward_full(x)
        y_loc = meas[sop.lo:sop.hi].clone()
        coeffs, _, losses = dgd(sop, y_loc, FullyDenseModel(grid), num_iterations=5, lr=1e-1,
                                loss_fns=[SquareLoss(), NegRegularizer()])
        res['gd'] = coeffs.detach().numpy()
        res['gd_loss'] = np.array(list(losses.values())[0])
        if rank == 0:
            out_q.put(res)
    except Exception as exc:   # surface worker failures instead of waiting for the queue
        import traceback
        out_q.put({'error': f'rank {rank}: {exc!r}\n{traceback.format_exc()}'})
        raise
    finally:
        dist.destroy_process_group()


def _single(n_obs):
    from cpu_operator import CpuOperator
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    from sph_raytracer_amd.retrieval import gd
    grid, geom = _geometry(n_obs)
    op = CpuOperator(grid, geom)
    g = tr.Generator().manual_seed(0)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g)
    y = tr.rand(geom.shape, dtype=tr.float64, generator=g)
    res = {'fwd': op(x).numpy(), 'fwd_mc': op(tr.stack([x, 2 * x])).numpy(), 'adj': op.T(y).numpy()}
    dgrid, dgeom = _geometry(n_obs, dynamic=True)
    xd = tr.rand(dgrid.shape, dtype=tr.float64, generator=g)
    dop = CpuOperator(dgrid, dgeom)
    res['dyn'] = dop(xd).numpy()
    yd = tr.rand(dgeom.shape, dtype=tr.float64, generator=g)
    res['dyn_T'] = dop._adj(yd, tuple(dgrid.shape)).numpy()
    meas = op(x).detach()
    coeffs, _, losses = gd(op, meas.clone(), FullyDenseModel(grid), num_iterations=5, lr=1e-1,
                           loss_fns=[SquareLoss(), NegRegularizer()], progress_bar=False)
    res['gd'] = coeffs.detach().numpy()
    res['gd_loss'] = np.array(list(losses.values())[0])
    return res


@pytest.mark.parametrize('world,n_obs', [(2, 6), (3, 7)])
def test_sharded_matches_single_process(world, n_obs):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_obs, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert 'error' not in got, got.get('error')
    assert all(p.exitcode == 0 for p in procs)
    ref = _single(n_obs)
    for k in ('fwd', 'fwd_mc', 'dyn'):
        assert got[k].shape == ref[k].shape, k
        assert np.array_equal(got[k], ref[k]), k        # same per-ray sums, just regrouped
    assert np.allclose(got['adj'], ref['adj'], rtol=1e-12, atol=1e-14)
    assert np.array_equal(got['dyn_T'], ref['dyn_T'])   # disjoint time slices: no reduction
    assert np.allclose(got['gd_loss'], ref['gd_loss'], rtol=1e-10)
    assert np.allclose(got['gd'], ref['gd'], rtol=1e-9, atol=1e-12)


def test_shard_bounds():
    from sph_raytracer_amd.distributed import shard_bounds
    for n in (1, 7, 50, 128):
        for w in (1, 2, 3, 8):
            if n < w:
                continue
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            sizes = [h - l for l, h in b]
            assert max(sizes) - min(sizes) <= 1
