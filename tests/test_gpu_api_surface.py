"""GPU parity for the Operator options traced in reference mode and for ParallelGeom, against
fixtures the reference itself produced (tests/golden/make_golden.py api) and against the oracle's
restatement of the same options with IEEE sqrt (oracle/sphrt_oracle_body.inc, float32 build),
which test_oracle.py pins bit for bit to those fixtures with MKL sqrt:

  - ftype=torch.float32 (raytracer.py:48-246 in float32; isclose threshold 0.01; each solver
    normalising its own float32 copy of the float64 rays): the per-family solvers and the trace
    bit for bit the oracle's; against the reference regions exact, voxel sequences exact under
    the canonical form, lengths at float32 resolution; forwards (float32 1e-5; float64 1e-10 vs
    the oracle, 1e-6 vs the reference) and adjoints;
  - invalid=True (raytracer.py:155: nothing masked): every non-zero entry of the reference's
    dense trace per ray, in order — voxels (wrapped as the reference's forward indexes them),
    finite lengths within 1e-12, and the inf / NaN entries at the same places — and the
    reference's forward and adjoint, which are non-finite exactly where the reference's are;
  - ParallelGeom (geometry.py:607-655: one direction broadcast over a plane of starts) through
    Operator directly, which the reference's own Operator refuses, against the
    reference's ViewGeom(pg.ray_starts, pg.rays.expand(...).clone()) fixture.
"""
import numpy as np
import pytest
import torch as tr

import golden_cases as gc

pytestmark = pytest.mark.gpu
F32_TINY = 1e-6          # float32 resolution: length / tiny-segment scale of a float32 trace
F32_LEN_RTOL = 4e-7      # 2-3 ulp of float32


def _op(case, gpu, **kw):
    from sph_raytracer_amd import Operator
    return Operator(gc.make_grid(case), gc.FixtureGeom(case), device=gpu, **kw)


def _oracle():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(gc.GOLDEN) + '/..')
    from oracle import oracle
    oracle.use_mkl_sqrt(False)
    return oracle


def _oracle_segments(case, f32, invalid=False, fresh=None):
    """The oracle's trace of a fixture with IEEE sqrt (the GPU's arithmetic): (ptr, vox, len)."""
    ora = _oracle()
    g = ora.Grid.from_boundaries(case['r_b'], case['e_b'], case['a_b'],
                                 ftype='float32' if f32 else 'float64')
    return ora.trace_segments(g, case['xs'], case['rays'], gc.ref_mode_starts(case, f32),
                              invalid=invalid, fresh=fresh)


def _same_bits(got, ref):
    got, ref = np.asarray(got), np.asarray(ref)
    return got.shape == ref.shape and bool(np.all((got == ref) | (np.isnan(got) & np.isnan(ref))))


@pytest.mark.parametrize('family', ['r', 'e', 'a'])
def test_solvers_f32(family, gpu):
    """float32 solvers: bit for bit the oracle's float32 restatement with IEEE sqrt (distances,
    regions, signs; inf included), and the reference's regions, signs and finite pattern.  The
    oracle with MKL vsSqrt equals the fixture bit for bit (test_oracle.py); torch's float32 sqrt
    is not correctly rounded, so the reference's distances themselves differ from any IEEE
    evaluation by up to ~200 ulp near grazing incidence."""
    from sph_raytracer_amd.raytracer import a_torch, e_torch, r_torch
    case = gc.load('solvers_f32')
    fam = 'rea'.index(family)
    fn = (r_torch, e_torch, a_torch)[fam]
    b = tr.from_numpy(case[f'{family}_b'])
    t, reg, _, neg = fn(b, tr.from_numpy(case['xs']), tr.from_numpy(case['rays']),
                        ftype=tr.float32, device=gpu)
    assert t.dtype == tr.float32
    t, reg, neg = t.cpu().numpy(), reg.cpu().numpy(), neg.cpu().numpy()
    ora = _oracle()
    g = ora.Grid.from_boundaries(case['r_b'], case['e_b'], case['a_b'], ftype='float32')
    ot, oreg, oneg = ora.solve(g, fam, case['xs'], case['rays'])
    assert _same_bits(t, ot), f'{family}: {int((t != ot).sum())} distances differ from the oracle'
    assert np.array_equal(reg, oreg) and np.array_equal(neg, oneg), family
    t_ref = case[f'{family}_t']
    assert np.array_equal(np.isfinite(t), np.isfinite(t_ref)), family
    assert np.array_equal(reg, case[f'{family}_reg']), family
    assert np.array_equal(neg, case[f'{family}_neg']), family


@pytest.mark.parametrize('name', gc.F32_CASES)
def test_f32_trace(name, gpu):
    """Operator(..., ftype=float32): the CSR bit for bit the oracle's float32 trace (IEEE sqrt),
    and the reference's trace under the segment contract at float32 resolution."""
    case = gc.load(name)
    op = _op(case, gpu, ftype=tr.float32)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    # float32 lengths: exactly float32 values
    assert np.array_equal(seg.astype(np.float32).astype(np.float64), seg)
    optr, ovox, oseg = _oracle_segments(case, True)
    assert np.array_equal(ptr, optr), f'{name}: segment counts differ from the oracle'
    assert np.array_equal(vox, ovox), f'{name}: voxels differ from the oracle'
    assert np.array_equal(seg, oseg), f'{name}: lengths differ from the oracle'
    shape = tuple(int(v) for v in case['shape'])[-3:]
    ref = gc.dense_to_segments(case['dense_regs'], case['dense_lens'], shape)
    msg = gc.compare_segments(ref, (ptr, vox, seg), gc.scale_of(case), name, tiny=F32_TINY,
                              len_rtol=F32_LEN_RTOL, len_atol=F32_TINY)
    assert msg is None, msg
    assert op.lens.dtype == tr.float32


@pytest.mark.parametrize('name', gc.F32_CASES)
def test_f32_forward_adjoint(name, gpu):
    case = gc.load(name)
    op = _op(case, gpu, ftype=tr.float32)
    d64 = tr.from_numpy(case['density0']).to(gpu)
    got = op(d64.float())
    assert got.dtype == tr.float32
    err = gc.rel_close(got.cpu().numpy(), case['fwd32_0'], gc.F32_RTOL)
    assert err <= gc.F32_RTOL, f'{name} f32 forward rel err {err:.3g}'
    # float64 density on float32 lengths (the reference promotes): against the oracle's float32
    # trace to float64 accumulation order, against the reference to the lengths' IEEE-vs-MKL sqrt
    # difference (<= 4.1e-7 over these fixtures, tests/test_oracle.py)
    got = op(d64).cpu().numpy()
    ptr, vox, seg = _oracle_segments(case, True)
    ora = _oracle()
    n_vox = int(np.prod(case['shape'][-3:]))
    ref = ora.forward(ptr, vox, seg, case['density0'], n_vox).reshape(got.shape)
    assert gc.rel_close(got, ref, gc.F64_RTOL) <= gc.F64_RTOL, f'{name} f64 forward vs oracle'
    err = gc.rel_close(got, case['fwd64_0'], 1e-6)
    assert err <= 1e-6, f'{name} f64 forward rel err {err:.3g}'
    y = tr.from_numpy(case['y0']).to(gpu)
    for yy, key, tol in ((y, 'adj64_0', 1e-6), (y.float(), 'adj32_0', 1e-5)):
        got = op.T(yy).cpu().numpy()
        ref = case[key]
        err = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300))
        assert err <= tol, f'{name} {key} rel err {err:.3g}'


def test_fresh_rays_float64(gpu):
    """float32 rays in a float64 trace: tr.asarray copies them per solver (raytracer.py:276,360,
    500), so r_torch and e_torch normalise their own copy once and a_torch takes them as they are
    (SPHRT_TRACE_FRESH_RAYS) — bit for bit the oracle's trace with fresh copies, and different from
    the twice-normalised in-place chain of float64 rays."""
    case = gc.load('f32_inside')
    case = dict(case, rays=(case['rays'] * 1.5).astype(np.float32).astype(np.float64))

    class Geom32:
        ray_starts = tr.from_numpy(case['xs'])
        rays = tr.from_numpy(case['rays']).float()
        shape = tuple(int(s) for s in case['ray_shape'])

    from sph_raytracer_amd import Operator
    op = Operator(gc.make_grid(case), Geom32(), device=gpu)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    optr, ovox, oseg = _oracle_segments(case, False, fresh=True)
    assert np.array_equal(ptr, optr) and np.array_equal(vox, ovox)
    assert np.array_equal(seg, oseg), 'lengths differ from the fresh-copy oracle'
    _, _, chained = _oracle_segments(case, False, fresh=False)
    assert len(chained) != len(oseg) or not np.array_equal(chained, oseg)


def _same_nonfinite(got, ref):
    return np.array_equal(np.isnan(got), np.isnan(ref)) and \
        np.array_equal(np.isposinf(got), np.isposinf(ref)) and \
        np.array_equal(np.isneginf(got), np.isneginf(ref))


@pytest.mark.parametrize('name', gc.INVALID_CASES)
def test_invalid_trace(name, gpu):
    case = gc.load(name)
    op = _op(case, gpu, invalid=True)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    optr, ovox, oseg = _oracle_segments(case, False, invalid=True)
    assert np.array_equal(ptr, optr) and np.array_equal(vox, ovox), f'{name}: oracle structure'
    assert _same_bits(seg, oseg), f'{name}: lengths differ from the oracle'
    shape = tuple(int(v) for v in case['shape'])[-3:]
    rp, rv, rl = gc.dense_to_segments(case['dense_regs'], case['dense_lens'], shape, invalid=True)
    assert np.array_equal(ptr, rp), f'{name}: segment counts differ'
    assert np.array_equal(vox, rv), f'{name}: voxels differ'
    assert _same_nonfinite(seg, rl), f'{name}: inf / NaN lengths at other places'
    fin = np.isfinite(rl)
    err = np.abs(seg[fin] - rl[fin])
    tol = gc.LEN_RTOL * np.abs(rl[fin]) + gc.LEN_ATOL * gc.scale_of(case)
    assert np.all(err <= tol), f'{name}: finite lengths differ by {err.max():.3g}'
    assert int(fin.sum()) > 0 and int((~fin).sum()) > 0


@pytest.mark.parametrize('name', gc.INVALID_CASES)
def test_invalid_forward_adjoint(name, gpu):
    """The reference's forward with invalid=True is non-finite for every ray (each ray's list
    holds an inf - inf = NaN length); ours is non-finite in the same places, and so is T."""
    case = gc.load(name)
    op = _op(case, gpu, invalid=True)
    d64 = tr.from_numpy(case['density0']).to(gpu)
    for dt, key in ((tr.float64, 'fwd64_0'), (tr.float32, 'fwd32_0')):
        got = op(d64.to(dt)).cpu().numpy()
        ref = case[key]
        assert _same_nonfinite(got, ref), f'{name} {key}: non-finite pattern differs'
        fin = np.isfinite(ref)
        if fin.any():
            assert gc.rel_close(got[fin], ref[fin], 1e-5) <= 1e-5
    got = op.T(tr.from_numpy(case['y0']).to(gpu)).cpu().numpy()
    ref = case['adj64_0']
    assert _same_nonfinite(got, ref), f'{name} T: non-finite pattern differs'
    fin = np.isfinite(ref)
    if fin.any():
        err = float(np.abs(got[fin] - ref[fin]).max() / max(np.abs(ref[fin]).max(), 1e-300))
        assert err <= 1e-10


def test_parallel_geom_operator(gpu):
    """ParallelGeom straight into Operator (its (1, 1, 3) rays broadcast over the starts, as
    trace_indices broadcasts them, raytracer.py:77-80) equals the reference's trace and forward
    of the same rays materialised per start."""
    from sph_raytracer_amd import Operator, ParallelGeom, SphericalGrid
    case = gc.load('parallel_geom')
    pg = ParallelGeom((30, 40), pos=(5, 0.5, 1), size=(2.2, 2.2))
    assert tuple(pg.rays.shape) == (1, 1, 3)
    assert tr.equal(pg.ray_starts, tr.from_numpy(case['xs']))
    assert tr.equal(pg.rays.expand(pg.ray_starts.shape), tr.from_numpy(case['rays']))
    op = Operator(SphericalGrid(shape=(20, 18, 24)), pg, device=gpu)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    msg = gc.compare_segments((case['seg_ptr'], case['seg_vox'], case['seg_len']),
                              (ptr, vox, seg), gc.scale_of(case), 'parallel_geom')
    assert msg is None, msg
    d = tr.from_numpy(case['density0']).to(gpu)
    got = op(d)
    assert tuple(got.shape) == (30, 40)
    err = gc.rel_close(got.cpu().numpy(), case['fwd64_0'], gc.F64_RTOL)
    assert err <= gc.F64_RTOL, f'parallel_geom forward rel err {err:.3g}'
    got = op.T(tr.from_numpy(case['y0']).to(gpu)).cpu().numpy()
    ref = case['adj64_0']
    assert float(np.abs(got - ref).max() / np.abs(ref).max()) <= 1e-10


@pytest.mark.parametrize('mode', ['float32', 'invalid'])
def test_reference_mode_orbit_sample(mode, gpu):
    """The reference-mode trace at an orbit's size class (3 views of the C2 orbit: 15,000 rays,
    50^3 grid): one pass into slots of K segments plus the compaction (sphrt_trace_reference_emit)
    and, for float32, the screen that skips rays starting outside every shell and crossing no
    sphere (~80 % of them: no kept segment) — the CSR bit for bit the oracle's restatement of the
    same options (IEEE sqrt), misses included."""
    import math
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    from sph_raytracer_amd.raytracer import find_starts
    f32 = mode == 'float32'
    grid = SphericalGrid(shape=(50, 50, 50))
    thetas = tr.linspace(0, 2 * math.pi, 50)[[0, 17, 33]]
    geom = sum(ConeRectGeom((50, 100), pos=(5 * tr.cos(t), 5 * tr.sin(t), 1), fov=(45, 45))
               for t in thetas)
    kw = dict(ftype=tr.float32) if f32 else dict(invalid=True)
    op = Operator(grid, geom, device=gpu, **kw)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    ora = _oracle()
    g = ora.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy(),
                                 ftype='float32' if f32 else 'float64')
    xs = geom.ray_starts.broadcast_to(geom.rays.shape)
    starts = find_starts(grid, xs, ftype=tr.float32 if f32 else tr.float64).numpy()
    optr, ovox, oseg = ora.trace_segments(g, xs.numpy(), geom.rays.numpy(), starts,
                                          invalid=not f32)
    assert np.array_equal(ptr, optr), f'{mode}: segment counts differ from the oracle'
    assert np.array_equal(vox, ovox), f'{mode}: voxels differ from the oracle'
    assert _same_bits(seg, oseg), f'{mode}: lengths differ from the oracle'
    empty = float((np.diff(ptr) == 0).mean())
    assert (empty > 0.5) if f32 else (empty == 0.0), empty
