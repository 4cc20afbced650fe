"""GPU parity against reference fixtures for the rows the trace fixtures leave open:
the dynamic adjoint (autograd through the time-indexed gather, raytracer.py:705-712), the
multichannel static forward and its gradient (raytracer.py:708-712; plotting.py:280-297's
preview3d shape), and a whole gd() retrieval (retrieval.py:84-116, loss.py:92-95,153-155).
Fixtures: tests/golden/make_golden.py pins (generated from the reference in this container).

Tolerances (written here): forwards 1e-10 relative in float64 and 1e-5 in float32;
gradients 1e-10 (float64) / 1e-5 (float32) relative to the gradient's largest magnitude; the gd()
run: coefficients within 1e-9 absolute, SquareLoss within 1e-9 relative and NegRegularizer
within 1e-12 absolute at every iteration.  The reference run itself moves by 1.2e-12
(coefficients) and 1.4e-14 (SquareLoss, relative) when its measurement is perturbed by one ulp
(make_golden.py gd_case), so 1e-9 leaves three decades for the difference in summation order.
"""
import numpy as np
import pytest
import torch as tr

import golden_cases as gc

pytestmark = pytest.mark.gpu

FWD = {tr.float64: gc.F64_RTOL, tr.float32: gc.F32_RTOL}
GRAD = {tr.float64: 1e-10, tr.float32: 1e-5}


def _grad_check(case, op, gpu, name):
    i = 0
    while f'density{i}' in case:
        for dt, tag in ((tr.float64, '64'), (tr.float32, '32')):
            x = tr.from_numpy(case[f'density{i}']).to(gpu, dt).requires_grad_()
            y = tr.from_numpy(case[f'gy{i}']).to(gpu, dt)
            res = op(x)
            assert res.dtype == dt and tuple(res.shape) == case[f'fwd{tag}_{i}'].shape, name
            err = gc.rel_close(res.detach().cpu().numpy(), case[f'fwd{tag}_{i}'], FWD[dt])
            assert err <= FWD[dt], f'{name} pair {i} f{tag} forward rel err {err:.3g}'
            (res * y).sum().backward()
            ref = case[f'grad{tag}_{i}']
            got = x.grad.cpu().numpy()
            assert got.shape == ref.shape and x.grad.dtype == dt
            err = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300))
            assert err <= GRAD[dt], f'{name} pair {i} f{tag} gradient rel err {err:.3g}'
        i += 1
    assert i > 0


@pytest.mark.parametrize('name', ['dynamic_grad', 'dynamic_single_grad'])
def test_dynamic_gradient_vs_reference(name, gpu):
    """Row f1: the dynamic forward and its gradient (the reference's autograd backward of
    density[t, r, e, a]) — views paired with time slices (time-paired CSR, transposed adjoint),
    and one detector integrated at every time step (channels of one CSR)."""
    from sph_raytracer_amd import Operator
    case = gc.load(name)
    grid = gc.make_grid(case)
    assert grid.dynamic
    op = Operator(grid, gc.FixtureGeom(case), device=gpu)
    _grad_check(case, op, gpu, name)


def test_dynamic_gradient_atomic_mode_vs_reference(gpu):
    """The same gradient through the float64-atomic adjoint (adjoint_mode='atomic')."""
    from sph_raytracer_amd import Operator
    case = gc.load('dynamic_grad')
    op = Operator(gc.make_grid(case), gc.FixtureGeom(case), device=gpu)
    op.adjoint_mode = 'atomic'
    _grad_check(case, op, gpu, 'dynamic_grad (atomic)')


def test_multichannel_vs_reference(gpu):
    """Row f4: static densities with leading channel dimensions — 3 channels, preview3d's
    (Na, Nr, Ne, Na) stack of 14 and a (2, 2) lead — forward and gradient, float64 and float32,
    one CSR streamed for all channels."""
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    case = gc.load('multichannel')
    geom = ConeRectGeom((24, 20), pos=(5, 0.3, 1), fov=(45, 45))
    assert tr.equal(geom.rays, tr.from_numpy(case['rays']))     # the reference's rays, bitwise
    op = Operator(SphericalGrid(shape=(12, 10, 14)), geom, device=gpu)
    _grad_check(case, op, gpu, 'multichannel')


@pytest.mark.parametrize('case_name,n,n_views,det,optim_kw', [
    ('gd_circ16', 16, 12, (20, 16), {}), ('gd_circ16', 16, 12, (20, 16), {'fused': True}),
    ('gd_circ32', 32, 32, (50, 40), {})])
def test_gd_vs_reference(case_name, n, n_views, det, optim_kw, gpu):
    """Row f2: gd() with the reference's arguments (FullyDenseModel, [SquareLoss(),
    NegRegularizer()], lr 0.1; 16^3 x 12 views x 25 iterations, and 32^3 x 32 views (50, 40) x 20
    iterations, closer to C5) against the reference's own run on the same
    measurement: every iteration's loss values and the final coefficients and reconstruction.
    The default optimiser is the reference's (torch's default Adam); fused=True, the caller's
    choice, stays inside the same tolerance.  Both take the autograd-free loop (_gd_direct)."""
    from sph_raytracer_amd import ConeCircGeom, Operator, SphericalGrid, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    case = gc.load(case_name)
    grid = SphericalGrid(shape=(n, n, n))
    th = tr.linspace(0, 2 * tr.pi, n_views)
    geom = sum(ConeCircGeom(shape=det, pos=(5 * tr.cos(t), 5 * tr.sin(t), 1), fov=(0, 45))
               for t in th)
    assert tr.equal(geom.rays, tr.from_numpy(case['rays']))
    op = Operator(grid, geom, device=gpu)
    meas = tr.from_numpy(case['meas']).to(gpu)
    calls = []
    direct = retrieval._gd_direct

    def spy(*a, **k):
        calls.append(1)
        return direct(*a, **k)

    retrieval._gd_direct = spy
    try:
        sq, neg = SquareLoss(), NegRegularizer()
        coeffs, y_res, losses = retrieval.gd(op, meas, FullyDenseModel(grid), lr=0.1,
                                             num_iterations=int(case['iterations']),
                                             loss_fns=[sq, neg], progress_bar=False, **optim_kw)
    finally:
        retrieval._gd_direct = direct
    assert calls == [1]
    l_sq, l_neg = np.array(losses[sq]), np.array(losses[neg])
    assert len(l_sq) == len(case['loss_sq']) == int(case['iterations'])
    err = np.abs(l_sq - case['loss_sq']) / case['loss_sq']
    assert err.max() <= 1e-9, f'SquareLoss history rel err {err.max():.3g} at {err.argmax()}'
    err = np.abs(l_neg - case['loss_neg'])
    assert err.max() <= 1e-12, f'NegRegularizer history abs err {err.max():.3g}'
    err = float(np.abs(coeffs.detach().cpu().numpy() - case['coeffs']).max())
    assert err <= 1e-9, f'final coefficients differ by {err:.3g}'
    err = gc.rel_close(y_res.detach().cpu().numpy(), case['y_result'], 1e-9)
    assert err <= 1e-9, f'reconstruction rel err {err:.3g}'
    assert l_sq[-1] < 0.05 * l_sq[0]
