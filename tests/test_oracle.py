"""The CPU oracle (oracle/) pinned against the reference: golden fixtures + torch.sort itself.

With sqrt bound to MKL vdSqrt (the routine torch CPU uses) the oracle must reproduce the
reference bit for bit; with IEEE sqrt (what the GPU uses) it must satisfy the parity contract.
"""
import os
import sys

import numpy as np
import pytest
import torch as tr

import golden_cases as gc

sys.path.insert(0, os.path.join(gc.GOLDEN, '..', '..'))
from oracle import oracle  # noqa: E402


def _grid(case):
    return oracle.Grid.from_boundaries(case['r_b'], case['e_b'], case['a_b'])


@pytest.fixture(params=[True, False], ids=['mkl_sqrt', 'ieee_sqrt'])
def sqrt_mode(request):
    if request.param and not oracle.use_mkl_sqrt(True):
        pytest.skip('vdSqrt not exported by this torch build')
    if not request.param:
        oracle.use_mkl_sqrt(False)
    yield request.param
    oracle.use_mkl_sqrt(False)


def test_introsort_matches_torch_sort():
    """torch.sort (CPU, unstable) == libstdc++ introsort over (value, index): the permutation of
    tie-heavy rows (±0, ±inf, repeated values) must match exactly for sizes 1..700."""
    rng = np.random.default_rng(0)
    pool = np.array([-np.inf, np.inf, 0.0, -0.0, 1.0, 2.0, -1.0, 0.5])
    for trial in range(600):
        n = int(rng.integers(1, 700))
        kind = trial % 3
        if kind == 0:
            x = rng.choice(pool, n)
        elif kind == 1:
            x = np.where(rng.random(n) < 0.5, np.inf, rng.choice(pool, n))
        else:
            x = np.where(rng.random(n) < 0.3, rng.normal(size=n), rng.choice(pool, n))
        _, ref = tr.from_numpy(x).sort()
        _, got = oracle.introsort(x)
        assert np.array_equal(ref.numpy(), got), f'trial {trial} n={n}'
    # realistic candidate rows: a reference-shaped mix of +inf misses, negatives and crossings
    for trial in range(200):
        n = 256
        x = np.full(n, np.inf)
        k = int(rng.integers(0, n))
        x[rng.choice(n, k, replace=False)] = np.round(rng.normal(2, 2, k), 1)
        _, ref = tr.from_numpy(x).sort()
        _, got = oracle.introsort(x)
        assert np.array_equal(ref.numpy(), got)


def test_solvers_vs_reference(sqrt_mode):
    z = gc.load('solvers')
    g = oracle.Grid.from_boundaries(z['r_b'], z['e_b'], z['a_b'])
    for fam, key in enumerate('rea'):
        t, reg, neg = oracle.solve(g, fam, z['xs'], z['rays'])
        rt = z[f'{key}_t']
        fin = np.isfinite(rt)
        assert np.array_equal(np.isinf(t), np.isinf(rt))
        assert np.array_equal(reg[fin], z[f'{key}_reg'][fin])
        assert np.array_equal(neg[fin], z[f'{key}_neg'][fin])
        if sqrt_mode:
            assert np.array_equal(t[fin], rt[fin]), f'{key}: not bit-exact with MKL sqrt'
            assert np.array_equal(reg, z[f'{key}_reg'])
        else:
            d = np.abs(t[fin] - rt[fin])
            assert d.max() <= 1e-9
            assert np.mean(d <= 4 * np.spacing(np.abs(rt[fin])) + 1e-13) >= 0.999


@pytest.mark.parametrize('i', range(5))
def test_dense_trace_bitexact(i, sqrt_mode):
    """The reference's own (regs, lens) for test_raytracer.py's rays, entry for entry."""
    case = gc.load(f'optest_{i}')
    regs, lens = oracle.trace_dense(_grid(case), case['xs'], case['rays'], case['starts'])
    if sqrt_mode:
        assert np.array_equal(lens, case['dense_lens'])
        assert np.array_equal(regs, case['dense_regs'])
    else:
        assert np.allclose(lens, case['dense_lens'], rtol=1e-12, atol=1e-12 * gc.scale_of(case))


@pytest.mark.parametrize('name', gc.CASES)
def test_segments_vs_reference(name, sqrt_mode):
    case = gc.load(name)
    got = oracle.trace_segments(_grid(case), case['xs'], case['rays'], case['starts'])
    ref = (case['seg_ptr'], case['seg_vox'], case['seg_len'])
    if sqrt_mode:
        for a, b in zip(ref, got):
            assert np.array_equal(a, b), f'{name}: not bit-exact with MKL sqrt'
    msg = gc.compare_segments(ref, got, gc.scale_of(case), name)
    assert msg is None, msg


@pytest.mark.parametrize('name', gc.CASES)
def test_forward_adjoint_vs_reference(name):
    case = gc.load(name)
    ptr, vox, seg = oracle.trace_segments(_grid(case), case['xs'], case['rays'], case['starts'])
    shape = tuple(int(s) for s in case['shape'])
    n_vox = int(np.prod(shape[-3:]))
    R = tuple(int(s) for s in case['ray_shape'])
    i = 0
    while f'density{i}' in case:
        dens = case[f'density{i}']
        div = int(np.prod(R[1:])) if bool(case['dynamic']) else 0
        out = oracle.forward(ptr, vox, seg, dens, n_vox, ray_chan_div=div)
        ref = case[f'fwd64_{i}']
        assert gc.rel_close(out.reshape(ref.shape), ref, gc.F64_RTOL) <= gc.F64_RTOL
        i += 1
    if 'y0' in case:
        adj = oracle.adjoint(ptr, vox, seg, case['y0'], n_vox).reshape(case['adj64_0'].shape)
        ref = case['adj64_0']
        assert np.abs(adj - ref).max() <= 1e-10 * np.abs(ref).max()


# ---- the reference's known-answer solver tests (test_all.py:18-173), against the oracle -------

def _fam(fam, bounds, xs, rays):
    b = np.asarray(bounds, np.float64)
    unit = np.array([0.0, 1.0])
    g = oracle.Grid.from_boundaries(*(b if i == fam else unit for i in range(3)))
    t, reg, _ = oracle.solve(g, fam, np.asarray(xs, np.float64), np.asarray(rays, np.float64))
    return t, reg


def check(a, b):
    return np.allclose(np.asarray(a, np.float32).ravel(), np.asarray(b, np.float32).ravel(),
                       atol=1e-2)


def test_known_answers_r():
    from known_answers import R_CASES
    for bounds, xs, rays, t_exp, reg_exp in R_CASES:
        t, reg = _fam(0, bounds, xs, rays)
        if t_exp == 'inf':
            assert np.all(np.isinf(t))
            continue
        assert check(t, t_exp)
        if reg_exp is not None:
            assert check(reg, reg_exp)


def test_known_answers_e():
    from known_answers import E_CASES, e_boundaries
    for spec, xs, rays, t_exp, reg_exp in E_CASES:
        bounds = e_boundaries(spec)
        t, reg = _fam(1, bounds, xs, rays)
        assert check(t, t_exp), (bounds, xs, rays, t)
        if reg_exp is not None:
            assert check(reg, reg_exp)


def test_known_answers_a():
    from known_answers import A_CASES
    for bounds, xs, rays, t_exp, reg_exp in A_CASES:
        t, reg = _fam(2, bounds, xs, rays)
        if t_exp == 'absinf':
            assert check(np.abs(t), [np.inf])
            continue
        assert check(t, t_exp)
        if reg_exp is not None:
            assert check(reg, reg_exp)


# ---- reference-mode options: ftype=float32 and invalid=True (make_golden.py api fixtures) -----

def test_solvers_f32_vs_reference(sqrt_mode):
    """The float32 solvers (raytracer.py:248-552 with ftype=float32) bit for bit with MKL vsSqrt.
    With IEEE sqrt (the GPU's) ~3 % of sphere / cone distances differ: torch's float32 sqrt is
    not correctly rounded on ~0.6 % of its inputs, and t = tc -+ sqrt(R^2 - d^2) resp.
    (-b +- sqrt(delta)) / 2a amplify that ulp near grazing incidence (up to ~64 / ~200 ulp of t,
    < 1e-4 absolute here); regions and crossing signs are unaffected."""
    z = gc.load('solvers_f32')
    g = oracle.Grid.from_boundaries(z['r_b'], z['e_b'], z['a_b'], ftype='float32')
    for fam, key in enumerate('rea'):
        t, reg, neg = oracle.solve(g, fam, z['xs'], z['rays'])
        assert t.dtype == np.float32
        rt = z[f'{key}_t']
        assert np.array_equal(np.isfinite(t), np.isfinite(rt)), key
        assert np.array_equal(reg, z[f'{key}_reg']), key
        assert np.array_equal(neg, z[f'{key}_neg']), key
        fin = np.isfinite(rt)
        if sqrt_mode:
            assert np.array_equal(t, rt), f'{key}: not bit-exact with MKL sqrt'
        else:
            assert np.abs(t[fin].astype(np.float64) - rt[fin]).max() <= 1e-4, key
            assert np.array_equal(t[~fin], rt[~fin])


@pytest.mark.parametrize('name', gc.F32_CASES + gc.INVALID_CASES)
def test_reference_mode_trace_vs_reference(name, sqrt_mode):
    """Operator(..., ftype=float32) / Operator(..., invalid=True) traces: the reference's dense
    (regs, lens), entry for entry with MKL sqrt (float32: the solvers each normalise their own
    float32 copy of the float64 rays, raytracer.py:276,360,500); with IEEE sqrt the same regions
    and lengths within float32 resolution (float64: 1e-12)."""
    case = gc.load(name)
    f32 = name in gc.F32_CASES
    g = oracle.Grid.from_boundaries(case['r_b'], case['e_b'], case['a_b'],
                                    ftype='float32' if f32 else 'float64')
    regs, lens = oracle.trace_dense(g, case['xs'], case['rays'], gc.ref_mode_starts(case, f32),
                                    invalid=not f32)
    rr, rl = case['dense_regs'], case['dense_lens']
    regs, lens = regs.reshape(rr.shape), lens.reshape(rl.shape)
    assert np.array_equal(regs, rr), name
    if sqrt_mode:
        assert np.array_equal(lens, rl, equal_nan=True), f'{name}: not bit-exact with MKL sqrt'
    else:
        fin = np.isfinite(rl)
        assert np.array_equal(np.isfinite(lens), fin)
        tol = (1e-6 if f32 else 1e-12) * gc.scale_of(case)
        assert np.abs(lens[fin] - rl[fin]).max() <= tol
