"""Seeded random grids and rays against the C oracle (parity fuzz).

Each case draws a grid from explicit boundary vectors (`SphericalGrid(r_b=, e_b=, a_b=)`,
geometry.py): random spacing, hollow radial ranges, partial elevation and azimuth ranges next
to full ones, 3-40 voxels per axis; and 3000 lines as a `ViewGeom`: half from outside the grid
aimed at random points of it, half from random points around it in random directions.  Every
ray's segments are checked against the C oracle's restatement of the reference's trace
(raytracer.py:48-173, IEEE square roots), then the float64 / float32 line integrals
(raytracer.py:703-713) and the adjoint (the autograd backward of :710) against the oracle on the
oracle's segments.  The reference-mode options (`ftype=float32`, `invalid=True`) are checked bit
for bit for `ftype=float32`; for `invalid=True` the non-finite segments (the infinite last one,
the NaN ones between infinite distances: their voxels follow the emulated introsort's order of
tied distances) exactly, the finite ones like the default trace.  Tolerances: voxel sequences
exact after dropping segments under 1e-12 x the scale (gc.compare_segments: a near-tie can leave
an ulp-long segment on one side only); lengths 1e-12 relative + 1e-12 x the scale (invalid=True
keeps the segments beyond the grid, up to ~1000 long, whose distances the device and the oracle
give 1-2 ulp apart: 1.8e-10 absolute at 1028); float64 integrals and the adjoint 1e-10 relative,
float32 integrals 1e-5 relative.
"""
import math

import numpy as np
import pytest
import torch as tr

import golden_cases as gc

pytestmark = pytest.mark.gpu


def _bounds(rng, n, lo, hi):
    """n + 1 ascending boundaries from lo to hi, gaps random but at least (hi - lo) / (8 n)."""
    w = rng.uniform(1.0, 8.0, n)
    w = w / w.sum() * (hi - lo)
    return np.concatenate([[lo], lo + np.cumsum(w)[:-1], [hi]])


def _case(seed):
    rng = np.random.default_rng(seed)
    nr, ne, na = (int(v) for v in rng.integers(3, 41, 3))
    r0 = 0.0 if rng.random() < 0.5 else float(rng.uniform(0.1, 0.5))
    r1 = float(rng.uniform(0.8, 1.5))
    if rng.random() < 0.5:
        e_lo, e_hi = 0.0, math.pi
    else:
        e_lo, e_hi = sorted(rng.uniform(0.0, math.pi, 2))
    u = rng.random()
    if u < 0.4:
        a_lo, a_hi = -math.pi, math.pi
    else:
        a_lo, a_hi = sorted(rng.uniform(-math.pi, math.pi, 2))
    r_b, e_b, a_b = _bounds(rng, nr, r0, r1), _bounds(rng, ne, e_lo, e_hi), _bounds(rng, na, a_lo, a_hi)
    n = 3000
    xs = np.empty((n, 3))
    d = np.empty((n, 3))
    h = n // 2
    v = rng.normal(size=(h, 3))
    xs[:h] = v / np.linalg.norm(v, axis=1, keepdims=True) * rng.uniform(1.6, 4.0, (h, 1))
    w = rng.normal(size=(h, 3))
    tgt = w / np.linalg.norm(w, axis=1, keepdims=True) * r1 * rng.uniform(0, 1, (h, 1)) ** (1 / 3)
    d[:h] = tgt - xs[:h]
    xs[h:] = rng.uniform(-1.2, 1.2, (n - h, 3)) * r1
    d[h:] = rng.normal(size=(n - h, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return r_b, e_b, a_b, xs, d


def _split_nonfinite(ptr, vox, seg):
    """(finite CSR, (ray, voxel, kind) of the non-finite segments: +1 inf, -1 -inf, 0 NaN)."""
    n = len(ptr) - 1
    ray = np.repeat(np.arange(n), np.diff(ptr))
    fin = np.isfinite(seg)
    fptr = np.concatenate([[0], np.cumsum(np.bincount(ray[fin], minlength=n))])
    kind = np.where(np.isnan(seg[~fin]), 0, np.sign(seg[~fin]))
    return (fptr, vox[fin], seg[fin]), (ray[~fin], vox[~fin], kind)


def _oracle():
    from oracle import oracle
    oracle.use_mkl_sqrt(False)
    return oracle


@pytest.mark.parametrize('seed', range(10))
def test_random_grid_and_rays_vs_oracle(seed, gpu):
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    from sph_raytracer_amd.raytracer import find_starts
    ora = _oracle()
    r_b, e_b, a_b, xs, d = _case(seed)
    grid = SphericalGrid(r_b=tr.from_numpy(r_b), e_b=tr.from_numpy(e_b), a_b=tr.from_numpy(a_b))
    geom = ViewGeom(tr.from_numpy(xs), tr.from_numpy(d))
    op = Operator(grid, geom, device=gpu)
    starts = find_starts(grid, tr.from_numpy(xs)).numpy()
    g = ora.Grid.from_boundaries(r_b, e_b, a_b)
    ref = ora.trace_segments(g, xs, d, starts)
    got = tuple(t.cpu().numpy() for t in op.segments())
    msg = gc.compare_segments(ref, got, 4.0, f'seed {seed}')
    assert msg is None, msg
    assert len(ref[1]) > 1000, 'the case should cross the grid'
    n_vox = math.prod(grid.shape)
    gen = tr.Generator().manual_seed(seed)
    x = tr.rand(tuple(grid.shape), dtype=tr.float64, generator=gen)
    want = np.asarray(ora.forward(*ref, x.numpy(), n_vox)).reshape(-1)
    have = op(x.to(gpu)).cpu().numpy().reshape(-1)
    assert gc.rel_close(have, want, 1e-10) <= 1e-10
    have32 = op(x.to(gpu, tr.float32)).cpu().numpy().reshape(-1)
    assert gc.rel_close(have32, want, 1e-5) <= 1e-5
    y = tr.rand(len(xs), dtype=tr.float64, generator=gen)
    want_t = np.asarray(ora.adjoint(*ref, y.numpy(), n_vox)).reshape(-1)
    have_t = op.T(y.to(gpu)).cpu().numpy().reshape(-1)
    scale = max(float(np.abs(want_t).max()), 1e-300)
    assert float(np.abs(have_t - want_t).max()) <= 1e-10 * scale


@pytest.mark.parametrize('mode, seed', [('float32', 20), ('float32', 21), ('invalid', 22),
                                        ('invalid', 23)])
def test_random_grid_reference_modes_vs_oracle(mode, seed, gpu):
    """`ftype=float32` and `invalid=True` on random grids against the oracle's restatement of
    the same options: float32 bit for bit; invalid=True's non-finite segments (whose voxels follow
    the emulated introsort's order of tied infinite distances) exactly, its finite ones within
    the module's tolerances."""
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    from sph_raytracer_amd.raytracer import find_starts
    ora = _oracle()
    f32 = mode == 'float32'
    r_b, e_b, a_b, xs, d = _case(seed)
    grid = SphericalGrid(r_b=tr.from_numpy(r_b), e_b=tr.from_numpy(e_b), a_b=tr.from_numpy(a_b))
    geom = ViewGeom(tr.from_numpy(xs), tr.from_numpy(d))
    kw = dict(ftype=tr.float32) if f32 else dict(invalid=True)
    op = Operator(grid, geom, device=gpu, **kw)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    g = ora.Grid.from_boundaries(r_b, e_b, a_b, ftype='float32' if f32 else 'float64')
    starts = find_starts(grid, tr.from_numpy(xs), ftype=tr.float32 if f32 else tr.float64).numpy()
    optr, ovox, oseg = ora.trace_segments(g, xs, d, starts, invalid=not f32)
    if f32:
        assert np.array_equal(ptr, optr), f'{mode} seed {seed}: segment counts differ'
        assert np.array_equal(vox, ovox), f'{mode} seed {seed}: voxels differ'
        assert np.array_equal(seg, oseg), f'{mode} seed {seed}: lengths differ'
        return
    got_f, got_n = _split_nonfinite(ptr, vox, seg)
    ref_f, ref_n = _split_nonfinite(optr, ovox, oseg)
    for a, b, what in zip(got_n, ref_n, ('rays', 'voxels', 'kinds')):
        assert np.array_equal(a, b), f'{mode} seed {seed}: non-finite segments differ ({what})'
    assert len(ref_n[0]) >= len(xs), 'every list ends in an infinite segment'
    msg = gc.compare_segments(ref_f, got_f, 4.0, f'{mode} seed {seed}')
    assert msg is None, msg
