"""GPU parity against the reference's golden vectors (tests/golden, made by make_golden.py).

Every case runs the HIP trace -> CSR, the HIP forward (float64 and float32) and the HIP adjoint,
and compares with the reference outputs captured in this repo's fixtures:
  - voxel sequences bit-exact per ray (canonical form, golden_cases.compare_segments),
  - segment lengths within 1e-12 relative,
  - line integrals within 1e-10 (float64) / 1e-5 (float32) relative,
  - adjoint volumes within 1e-10 relative to the volume's max.
"""
import numpy as np
import pytest
import torch as tr

import golden_cases as gc

pytestmark = pytest.mark.gpu


def _op(case, gpu, **kw):
    from sph_raytracer_amd import Operator
    return Operator(gc.make_grid(case), gc.FixtureGeom(case), device=gpu, **kw)


@pytest.mark.parametrize('name', gc.CASES)
def test_trace_segments(name, gpu):
    case = gc.load(name)
    op = _op(case, gpu)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    msg = gc.compare_segments((case['seg_ptr'], case['seg_vox'], case['seg_len']),
                              (ptr, vox, seg), gc.scale_of(case), name)
    assert msg is None, msg


@pytest.mark.parametrize('name', gc.CASES)
def test_forward(name, gpu):
    case = gc.load(name)
    op = _op(case, gpu)
    i = 0
    while f'density{i}' in case:
        d64 = tr.from_numpy(case[f'density{i}']).to(gpu)
        got64 = op(d64)
        assert got64.dtype == tr.float64 and tuple(got64.shape) == case[f'fwd64_{i}'].shape
        err = gc.rel_close(got64.cpu().numpy(), case[f'fwd64_{i}'], gc.F64_RTOL)
        assert err <= gc.F64_RTOL, f'{name} density{i} f64 rel err {err:.3g}'
        got32 = op(d64.float())
        assert got32.dtype == tr.float32
        err = gc.rel_close(got32.cpu().numpy(), case[f'fwd32_{i}'], gc.F32_RTOL)
        assert err <= gc.F32_RTOL, f'{name} density{i} f32 rel err {err:.3g}'
        i += 1


@pytest.mark.parametrize('name', [c for c in gc.CASES if c != 'dynamic_obs'])
def test_adjoint(name, gpu):
    case = gc.load(name)
    if 'y0' not in case:
        pytest.skip('no adjoint vector in this fixture')
    op = _op(case, gpu)
    y = tr.from_numpy(case['y0']).to(gpu)
    got = op.T(y).cpu().numpy()
    ref = case['adj64_0']
    err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300)
    assert err <= 1e-10, f'{name}: adjoint rel err {err:.3g}'


@pytest.mark.parametrize('name', ['c1_single_vantage', 'circ_orbit', 'inside_starts',
                                  'dynamic_obs'])
def test_fused_no_store(name, gpu):
    """Trace+integrate in one pass (nothing persisted) equals the reference forward."""
    from sph_raytracer_amd.raytracer import line_integrals
    case = gc.load(name)
    grid, geom = gc.make_grid(case), gc.FixtureGeom(case)
    i = 0
    while f'density{i}' in case:
        d64 = tr.from_numpy(case[f'density{i}']).to(gpu)
        got = line_integrals(grid, geom, d64)
        err = gc.rel_close(got.cpu().numpy(), case[f'fwd64_{i}'], gc.F64_RTOL)
        assert err <= gc.F64_RTOL, f'{name} fused density{i} rel err {err:.3g}'
        got32 = line_integrals(grid, geom, d64.float())
        err = gc.rel_close(got32.cpu().numpy(), case[f'fwd32_{i}'], gc.F32_RTOL)
        assert err <= gc.F32_RTOL, f'{name} fused f32 density{i} rel err {err:.3g}'
        i += 1


def test_solvers_bitlevel(gpu):
    """Per-family crossing solves vs the reference's r_torch/e_torch/a_torch on 4000 random rays:
    regions and negative_crossing exact; distances equal up to the IEEE-vs-MKL sqrt ulp."""
    from sph_raytracer_amd.raytracer import r_torch, e_torch, a_torch
    z = gc.load('solvers')
    xs, rays = tr.from_numpy(z['xs']), tr.from_numpy(z['rays'])
    for key, fn in (('r', r_torch), ('e', e_torch), ('a', a_torch)):
        t, reg, _, neg = fn(tr.from_numpy(z[f'{key}_b']), xs, rays)
        t, reg, neg = t.numpy(), reg.numpy(), neg.numpy()
        rt = z[f'{key}_t']
        assert np.array_equal(np.isinf(t), np.isinf(rt)), f'{key}: inf pattern differs'
        fin = np.isfinite(rt)
        d = np.abs(t[fin] - rt[fin])
        # IEEE sqrt (GPU) vs MKL vdSqrt (reference) differ by <= 1 ulp on ~1% of inputs; in the
        # cone roots (-b +- q) / 2a that ulp of q is amplified by 1/|a| when a is small.  So:
        # (almost) every distance within 4 ulp, none off by more than 1e-9 absolute.
        tol = 4 * np.spacing(np.abs(rt[fin])) + 1e-13
        frac_exact = float(np.mean(d == 0))
        frac_ulp = float(np.mean(d <= tol))
        assert d.max() <= 1e-9, f'{key}: distance error {d.max():.3g}'
        assert frac_ulp >= 0.999, f'{key}: only {frac_ulp:.4f} of distances within 4 ulp'
        assert frac_exact > 0.95, f'{key}: only {frac_exact:.3f} of distances bit-exact'
        # regions are only meaningful for finite distances (inf entries never update a row)
        assert np.array_equal(reg[fin], z[f'{key}_reg'][fin]), f'{key}: regions differ'
        assert np.array_equal(neg[fin], z[f'{key}_neg'][fin]), f'{key}: negative_crossing differs'


def test_solvers_match_ieee_oracle(gpu):
    """GPU crossing solves vs the oracle with IEEE sqrt: same arithmetic, same rounding, so every
    distance, region and negative_crossing must be identical (all entries, inf/NaN included)."""
    import os, sys
    sys.path.insert(0, os.path.dirname(gc.GOLDEN) + '/..')
    from oracle import oracle
    from sph_raytracer_amd.raytracer import a_torch, e_torch, r_torch
    z = gc.load('solvers')
    xs, rays = tr.from_numpy(z['xs']), tr.from_numpy(z['rays'])
    oracle.use_mkl_sqrt(False)
    g = oracle.Grid.from_boundaries(z['r_b'], z['e_b'], z['a_b'])
    for fam, (key, fn) in enumerate((('r', r_torch), ('e', e_torch), ('a', a_torch))):
        t, reg, _, neg = fn(tr.from_numpy(z[f'{key}_b']), xs, rays)
        ot, oreg, oneg = oracle.solve(g, fam, z['xs'], z['rays'])
        t = t.numpy()
        same = (t == ot) | (np.isnan(t) & np.isnan(ot))
        assert same.all(), f'{key}: {int((~same).sum())} distances differ from the IEEE oracle, ' \
                           f'first {t[~same][:3]} vs {ot[~same][:3]}'
        assert np.array_equal(reg.numpy(), oreg), f'{key}: regions differ'
        assert np.array_equal(neg.numpy(), oneg), f'{key}: negative_crossing differs'


def test_gpu_sqrt_div_correctly_rounded(gpu):
    """FP64 sqrt and division on gfx950 as compiled here must be IEEE correctly rounded (the
    solver's bit-exactness against the IEEE oracle rests on it)."""
    from sph_raytracer_amd.raytracer import r_torch
    rng = np.random.default_rng(5)
    # r_torch with start on the z axis and direction +x: tc = 0, d = |x| ... t = +-sqrt(R^2 - d^2)
    R = np.sort(rng.uniform(1.0, 3.0, 2000))
    x = np.zeros((2000, 3))
    x[:, 2] = rng.uniform(0.0, 0.999, 2000)
    t, _, _, _ = r_torch(tr.from_numpy(R), tr.from_numpy(x[:1]), tr.tensor([[1.0, 0.0, 0.0]]))
    d = x[0, 2]
    ref = np.sqrt(R * R - d * d)
    assert np.array_equal(t.numpy()[0, len(R):], ref)


def test_device_rays_bit_identical(gpu):
    """On-device cone-beam rays (sphrt_rays_cone) equal the torch CPU rays bit
    for bit: ConeRect / ConeCirc (lin and log radial spacing), orbit collections, one-pixel axes,
    explicit look/up directions."""
    import torch as tr
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    from sph_raytracer_amd.raytracer import _device_rays
    th = tr.linspace(0, 2 * tr.pi, 7)
    cases = [
        ConeRectGeom((50, 100), pos=(5, 0, 0), fov=(45, 45)),
        ConeRectGeom((1, 5), pos=(3, 1, 2), fov=(10, 30)),
        ConeRectGeom((4, 1), pos=(3, 1, 2)),
        ConeRectGeom((6, 7), (1, 0, 0), (-1, 0, 0), (0, 1, 0), fov=(23, 45)),
        sum(ConeRectGeom((50, 100), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(45, 45)) for a in th),
        sum(ConeCircGeom((30, 24), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(0, 45)) for a in th),
        ConeCircGeom((9, 13), pos=(2, 3, 4), fov=(5, 40), spacing='log'),
    ]
    for g in cases:
        got = _device_rays(g, gpu)
        assert got is not None
        assert tr.equal(got.cpu(), g.rays), type(g).__name__


def test_device_rays_in_trace_order(gpu):
    """sphrt_rays_cone_ordered: each view's rays generated in a per-view pixel order equal the
    geometry's rays gathered in that order, bit for bit, and every row's ray id is its geometry
    ray (the ConeCirc wedge order of the Operator's trace, and a random permutation)."""
    import torch as tr
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    from sph_raytracer_amd.raytracer import _ConeRays, _wedge_order
    th = tr.linspace(0, 2 * tr.pi, 5)
    cases = [
        sum(ConeCircGeom((30, 24), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(0, 45)) for a in th),
        ConeCircGeom((9, 13), pos=(2, 3, 4), fov=(5, 40), spacing='log'),
        sum(ConeRectGeom((12, 20), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1)) for a in th),
    ]
    gen = tr.Generator().manual_seed(5)
    for g in cases:
        cone = _ConeRays.of(g)
        h, w = cone.h, cone.w
        for perm in (_wedge_order(h, w), tr.randperm(h * w, generator=gen)):
            rays, ray_id = cone.launch(gpu, order=perm.to(gpu))
            flat = g.rays.reshape(cone.n_views, h * w, 3)
            assert tr.equal(rays.cpu().reshape(cone.n_views, h * w, 3), flat[:, perm])
            want = (tr.arange(cone.n_views)[:, None] * (h * w) + perm).reshape(-1).to(tr.int32)
            assert tr.equal(ray_id.cpu(), want)


def test_device_rays_in_view_tiles(gpu):
    """sphrt_rays_cone_tiled: the rays in the (h, w / tw, V / tv, tv, tw) view-tile layout equal
    the geometry's rays rearranged that way, bit for bit, and every row's ray id is its geometry
    ray (the Operator's trace order for orbits, raytracer._view_tiles)."""
    import torch as tr
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    from sph_raytracer_amd.raytracer import _ConeRays, _Staging, _launch_tiled
    th = tr.linspace(0, 2 * tr.pi, 6)
    cases = [
        sum(ConeCircGeom((30, 24), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(0, 45)) for a in th),
        sum(ConeRectGeom((12, 20), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1)) for a in th),
    ]
    for g in cases:
        cone = _ConeRays.of(g)
        v, h, w = cone.n_views, cone.h, cone.w
        stg = _Staging()
        cone.stage(stg)
        stg.upload(gpu)
        for tv, tw in ((6, 2), (3, 4), (2, 1), (1, 2)):
            rays, ray_id = _launch_tiled(cone, gpu, stg, (tv, tw))
            want = g.rays.reshape(v // tv, tv, h, w // tw, tw, 3).permute(2, 3, 0, 1, 4, 5)
            assert tr.equal(rays.cpu(), want), (tv, tw)
            idx = tr.arange(v * h * w).reshape(v // tv, tv, h, w // tw, tw).permute(2, 3, 0, 1, 4)
            assert tr.equal(ray_id.cpu(), idx.reshape(-1).to(tr.int32))


def _csr(op):
    c = op._csr
    return (c['row_ptr'].cpu(), c['vox'][:c['total']].cpu(), c['len'][:c['total']].cpu())


@pytest.mark.parametrize('name', gc.CASES)
def test_onepass_trace_equals_twopass(name, gpu, monkeypatch):
    """The one-pass trace (geometric segment bounds -> staging slots -> compaction) builds the
    same CSR as the two-pass count + fill, bit for bit; so does its fallback when bounds fail
    (forced by halving every bound: the emit pass overflows, the counts stay exact and only the
    fill pass runs)."""
    from sph_raytracer_amd import raytracer as rt
    case = gc.load(name)
    monkeypatch.setenv('SPHRT_TRACE', 'twopass')
    ref = _csr(_op(case, gpu))
    monkeypatch.setenv('SPHRT_TRACE', 'onepass')
    got = _csr(_op(case, gpu))
    for a, b in zip(ref, got):
        assert tr.equal(a, b), name
    monkeypatch.setattr(rt, '_bound_hook', lambda b: b.div_(2, rounding_mode='floor'))
    got = _csr(_op(case, gpu))
    for a, b in zip(ref, got):
        assert tr.equal(a, b), name + ' (fallback)'
