"""Size-independent properties of the HIP path at the BASELINE sizes (C1, C2 full; C5 geometry),
plus oracle spot checks on rays sampled from the full-size traces.

Tolerances: float64 identities within 1e-12 relative (1e-11 for sums over 10^5+ terms);
segment voxels exact, lengths 1e-12 relative (golden_cases.compare_segments)."""
import math
import os
import sys

import numpy as np
import pytest
import torch as tr

import golden_cases as gc

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pytestmark = pytest.mark.gpu


def _orbit(n_views, det, kind='rect', grid_shape=(50, 50, 50)):
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, SphericalGrid
    grid = SphericalGrid(shape=grid_shape)
    geoms = []
    for th in tr.linspace(0, 2 * tr.pi, n_views):
        pos = (5 * tr.cos(th), 5 * tr.sin(th), 1)
        geoms.append(ConeRectGeom(det, pos=pos, fov=(45, 45)) if kind == 'rect'
                     else ConeCircGeom(shape=det, pos=pos, fov=(0, 45)))
    return grid, sum(geoms)


@pytest.fixture(scope='module')
def c2(gpu):
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(50, (50, 100))
    return grid, geom, Operator(grid, geom, device=gpu)


def test_adjoint_identity_and_determinism(c2, gpu):
    grid, geom, op = c2
    g = tr.Generator(device=gpu).manual_seed(0)
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu, generator=g)
    y = tr.rand(geom.shape, dtype=tr.float64, device=gpu, generator=g)
    ax = op(x)
    aty = op.T(y)
    lhs, rhs = float((ax * y).sum()), float((x * aty).sum())
    assert abs(lhs - rhs) <= 1e-12 * abs(lhs), (lhs, rhs)
    assert tr.equal(op(x), ax), 'forward not bitwise reproducible'
    assert tr.equal(op.T(y), aty), 'adjoint not bitwise reproducible'
    # deterministic transposed adjoint == float64-atomic adjoint (up to summation order)
    op.adjoint_mode = 'atomic'
    at2 = op.T(y)
    op.adjoint_mode = 'transpose'
    assert tr.allclose(at2, aty, rtol=1e-12, atol=1e-12 * float(aty.abs().max()))
    # float32 forward/adjoint against float64
    ax32 = op(x.float())
    assert float(((ax32.double() - ax).abs() / ax.abs().clamp_min(1e-12)).max()) <= 1e-5
    aty32 = op.T(y.float())
    assert aty32.dtype == tr.float32
    assert float((aty32.double() - aty).abs().max()) <= 1e-5 * float(aty.abs().max())


def test_linearity_and_channels(c2, gpu):
    grid, geom, op = c2
    g = tr.Generator(device=gpu).manual_seed(1)
    x1 = tr.rand(grid.shape, dtype=tr.float64, device=gpu, generator=g)
    x2 = tr.rand(grid.shape, dtype=tr.float64, device=gpu, generator=g) - 0.5
    lhs = op(2.5 * x1 - 3.0 * x2)
    rhs = 2.5 * op(x1) - 3.0 * op(x2)
    assert float((lhs - rhs).abs().max()) <= 1e-12 * float(rhs.abs().max())
    # multichannel static input == per-channel calls (preview3d-style batching)
    xc = tr.stack([x1, x2, x1 * x2])
    out = op(xc)
    assert out.shape == (3,) + tuple(geom.shape)
    for i in range(3):
        assert tr.equal(out[i], op(xc[i]))
    yc = tr.rand((3,) + tuple(geom.shape), dtype=tr.float64, device=gpu, generator=g)
    grad = tr.autograd.grad((op(xc.requires_grad_()) * yc).sum(), xc)[0]
    for i in range(3):
        assert tr.allclose(grad[i], op.T(yc[i]), rtol=1e-12, atol=1e-14)


def test_chord_lengths(c2, gpu):
    """With every voxel = 1, a ray's line integral is its chord through the outer sphere."""
    grid, geom, op = c2
    out = op(tr.ones(grid.shape, dtype=tr.float64, device=gpu)).cpu().numpy().reshape(-1)
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3)
    d = geom.rays.numpy().reshape(-1, 3)
    tc = -(xs * d).sum(1)
    dd2 = (xs * xs).sum(1) - tc * tc
    chord = 2 * np.sqrt(np.clip(1.0 - dd2, 0, None))
    assert np.allclose(out, chord, rtol=1e-9, atol=1e-9)
    assert (out > 0).mean() > 0.15


def test_fused_equals_csr(c2, gpu):
    from sph_raytracer_amd.raytracer import line_integrals
    grid, geom, op = c2
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu)
    a = op(x)
    b = line_integrals(grid, geom, x)
    assert float((a - b).abs().max()) <= 1e-12 * float(a.abs().max())


def test_granule_tables(c2, gpu):
    """Per-workgroup granule tables (sphrt_csr_local, LDS-bitmap build at 50^3): each table
    ascending and distinct, every segment's slot names its voxel's granule and lane and carries
    its row-head flag; the table forward equals the per-segment-gather forward bitwise, for the
    forward and the transposed adjoint."""
    _check_granule_tables(*c2, gpu, tab_bytes=2)


def test_granule_tables_radix_build(gpu):
    """The same checks on a grid above 2^19 voxels, whose tables come from the block radix sort
    (and have 32-bit entries)."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(3, (48, 64), grid_shape=(96, 80, 90))
    _check_granule_tables(grid, geom, Operator(grid, geom, device=gpu), gpu, tab_bytes=4)


def test_granule_tables_big_blocks(gpu):
    """A narrow bundle of lines through the centre of a grid above 2^19 voxels: rows of ~400
    segments give blocks of more than 2048 segments (the last row's overhang), whose tables come
    from the separate 16-key launch (local_table_big_kernel); the same checks, and such blocks
    exist."""
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    grid = SphericalGrid(shape=(96, 80, 90))
    rng = np.random.default_rng(11)
    xs = np.tile([1.5, 0.01, 0.02], (20000, 1))
    d = rng.normal(size=(20000, 3)) * 0.03 - xs
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    geom = ViewGeom(tr.from_numpy(xs), tr.from_numpy(d))
    op = Operator(grid, geom, device=gpu)
    blk = op._csr['blocks'].cpu().numpy().reshape(-1, 6)
    n = blk[:, 3] - blk[:, 2]
    assert ((n > 2048) & (n <= 4096) & (blk[:, 5] >= 0)).sum() > 0
    _check_granule_tables(grid, geom, op, gpu, tab_bytes=4)


def test_granule_tables_partial_last_granule(gpu):
    """Voxel and ray counts that are not multiples of 4 (the last granule is partial): the table
    forward / transposed adjoint take the chunk-first order with the partial tail copied lane by
    lane (no early DMA) and still equal the per-segment gathers bitwise."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(6, (23, 29), grid_shape=(21, 17, 23))
    assert math.prod(grid.shape) % 4 == 3 and math.prod(geom.shape) % 4 == 2
    op = Operator(grid, geom, device=gpu)
    assert ', false, 8,' in op._forward_kernel_name(tr.rand(grid.shape, device=gpu))
    _check_granule_tables(grid, geom, op, gpu, tab_bytes=2)


def _stage_col(v, shape, brick):
    """Natural voxel -> brick-staged column (apply.hip stage_col), numpy."""
    (nr, ne, na), (br, be, ba) = shape, brick
    r, e, a = v // (ne * na), (v // na) % ne, v % na
    nbe, nba = -(-ne // be), -(-na // ba)
    blk = ((r // br) * nbe + e // be) * nba + a // ba
    return blk * (br * be * ba) + ((r % br) * be + e % be) * ba + a % ba


def test_brick_staged_tables(gpu, monkeypatch):
    """Brick staging forced on a grid no brick divides (padded staging, 3 channels growing the
    stage): tables and loc address the staged columns, and the staged table forward equals the
    per-segment gather forward bitwise (_check_granule_tables), for three bricks (4,2,4: the
    default, r padded 30 -> 32)."""
    from sph_raytracer_amd import Operator
    for brick in ('4,2,4', '2,4,4', '4,4,2'):
        monkeypatch.setenv('SPHRT_BRICK', brick)
        monkeypatch.setenv('SPHRT_BRICK_T', '1,2,8')     # transposed: rays, 30 columns padded
        grid, geom = _orbit(4, (24, 30), grid_shape=(30, 21, 26))
        op = Operator(grid, geom, device=gpu)
        d = op._csr['desc']
        assert tuple(d.stage_brick) == tuple(int(b) for b in brick.split(','))
        assert d.stage_cols == math.prod(-(-s // b) * b for s, b in zip((30, 21, 26), d.stage_brick))
        _check_granule_tables(grid, geom, op, gpu, tab_bytes=2)
        t = op._transposed()['desc']
        assert tuple(t.stage_brick) == (1, 2, 8) and tuple(t.stage_shape) == (4, 24, 30)
        x = tr.rand((3,) + tuple(grid.shape), dtype=tr.float64, device=gpu)
        out = op(x)
        assert op._csr['desc'].stage_bytes == 0 and not op._csr['desc'].stage   # per call
        for i in range(3):
            assert tr.equal(out[i], op(x[i]))
        # a density 4 bytes off 16-byte alignment (the pack's scalar path), float32
        x32 = x[0].float()
        big = tr.empty(x32.numel() + 1, dtype=tr.float32, device=gpu)
        off = big[1:].view(grid.shape)
        off.copy_(x32)
        assert off.data_ptr() % 16 != 0
        assert tr.equal(op(off), op(x32))


def _check_granule_tables(grid, geom, op, gpu, tab_bytes):
    from sph_raytracer_amd import _lib
    csr = op._csr
    blocks = csr['blocks'].cpu().numpy().reshape(-1, _lib.BLOCK_FIELDS)
    vox = csr['vox'].cpu().numpy().view(np.uint32)[:csr['total']]
    loc = csr['loc'].cpu().numpy().view(np.uint16)[:csr['total']]
    tab = csr['tab'].cpu().numpy()
    assert csr['desc'].tab_bytes == tab_bytes
    tab = tab.view(np.uint16).astype(np.int64) if tab_bytes == 2 else tab.astype(np.int64)
    s0, s1, n_tab = blocks[:, 2], blocks[:, 3], blocks[:, 5]
    assert (n_tab >= 0).all() and (n_tab <= s1 - s0).all() and csr['desc'].n_fallback == 0
    owner = np.repeat(np.arange(len(blocks)), s1 - s0)
    off = (loc & 0x7fff).astype(np.int64)   # byte offset in the float LDS image (zero granule first)
    assert (off % 4 == 0).all() and (off >= 16).all()
    slot = off // 4 - 4
    assert (slot // 4 < n_tab[owner]).all()
    v = (vox & 0x7fffffff).astype(np.int64)
    d = csr['desc']
    if d.stage_shape[0] > 0:                 # brick staging: tables address the staged columns
        v = _stage_col(v, tuple(d.stage_shape), tuple(d.stage_brick))
    stride = csr['desc'].tab_stride
    assert stride >= n_tab.max() and stride % 64 == 0
    assert np.array_equal(tab[owner * stride + slot // 4], v >> 2)
    assert np.array_equal(slot % 4, v % 4)
    assert np.array_equal(loc >> 15, vox >> 31)
    for b in range(0, len(blocks), 97):
        t0 = b * stride
        assert (np.diff(tab[t0:t0 + n_tab[b]]) > 0).all()
    g = tr.Generator(device=gpu).manual_seed(3)
    for dt in (tr.float32, tr.float64):
        x = tr.rand(grid.shape, dtype=dt, device=gpu, generator=g)
        y = tr.rand(geom.shape, dtype=dt, device=gpu, generator=g)
        xc = tr.rand((2,) + tuple(grid.shape), dtype=dt, device=gpu, generator=g)
        a, at, ac = op(x), op.T(y), op(xc)
        descs = [csr['desc'], op._transposed()['desc']]
        saved = [(d.loc, d.tab) for d in descs]
        try:
            for d in descs:
                d.loc, d.tab = None, None
            assert tr.equal(op(x), a)
            assert tr.equal(op.T(y), at)
            assert tr.equal(op(xc), ac)
        finally:
            for d, (lc, tb) in zip(descs, saved):
                d.loc, d.tab = lc, tb


@pytest.mark.parametrize('runs', ['auto', 'on'])
def test_long_rows_fall_back_to_per_segment_gather(runs, gpu, monkeypatch):
    """Rays of ~3300 segments through 1650 shells: their workgroups exceed the granule table
    (n_tab = -1) and use the per-segment gather, and the workgroups inside a long row own no
    row; results against the C oracle's trace + forward, with and without run records."""
    from oracle import oracle
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid, _lib
    from sph_raytracer_amd.raytracer import find_starts
    monkeypatch.setenv('SPHRT_RUNS', runs)
    grid = SphericalGrid(shape=(1650, 2, 3))
    geom = ConeRectGeom((4, 5), pos=(3, 0.01, 0.02), fov=(2, 2))
    op = Operator(grid, geom, device=gpu)
    assert bool(op._csr['desc'].runs) == (runs == 'on')
    blocks = op._csr['blocks'].cpu().numpy().reshape(-1, _lib.BLOCK_FIELDS)
    assert (blocks[:, 5] == -1).any()
    assert op._csr['desc'].n_fallback == int((blocks[:, 5] == -1).sum())
    x = tr.rand(grid.shape, dtype=tr.float64)
    got = op(x.to(gpu)).cpu().numpy().reshape(-1)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3).copy()
    d = geom.rays.numpy().reshape(-1, 3).copy()
    ptr, vox, seg = oracle.trace_segments(g, xs, d, find_starts(grid, tr.from_numpy(xs)).numpy())
    assert np.diff(ptr).max() > 3000
    ref = oracle.forward(ptr, vox, seg, x.numpy(), math.prod(grid.shape))
    assert np.allclose(got, np.asarray(ref).reshape(-1), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('nr', [2500, 6000])
def test_large_k_trace_vs_oracle(nr, gpu):
    """K = 2(Nr+1)+... beyond what four per-wave LDS lists fit (K 5013 -> 2 waves per workgroup,
    K 12013 -> 1): segments and line integrals against the C oracle."""
    from oracle import oracle
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    from sph_raytracer_amd.raytracer import find_starts
    grid = SphericalGrid(shape=(nr, 2, 3))
    geom = ConeRectGeom((2, 3), pos=(3, 0.01, 0.02), fov=(2, 2))
    op = Operator(grid, geom, device=gpu)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3).copy()
    d = geom.rays.numpy().reshape(-1, 3).copy()
    ptr, vox, seg = oracle.trace_segments(g, xs, d, find_starts(grid, tr.from_numpy(xs)).numpy())
    row_ptr, gvox, glen = (t.cpu().numpy() for t in op.segments())
    msg = gc.compare_segments((ptr, vox, seg), (row_ptr, gvox, glen), scale=1.0, what=f'nr={nr}')
    assert msg is None, msg
    x = tr.rand(grid.shape, dtype=tr.float64)
    ref = np.asarray(oracle.forward(ptr, vox, seg, x.numpy(), math.prod(grid.shape))).reshape(-1)
    got = op(x.to(gpu)).cpu().numpy().reshape(-1)
    assert np.allclose(got, ref, rtol=1e-10, atol=1e-12)


def test_full_size_trace_vs_oracle_sample(c2, gpu):
    """2000 rays sampled from the full C2 trace, each checked against the C oracle."""
    from oracle import oracle
    from sph_raytracer_amd.raytracer import find_starts
    grid, geom, op = c2
    rng = np.random.default_rng(0)
    n = math.prod(geom.shape)
    pick = np.sort(rng.choice(n, 2000, replace=False))
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3)[pick]
    rays = geom.rays.numpy().reshape(-1, 3)[pick]
    starts = find_starts(grid, tr.from_numpy(xs)).numpy()
    oracle.use_mkl_sqrt(False)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ref = oracle.trace_segments(g, xs, rays, starts)
    rp, vx, ln = (t.cpu().numpy() for t in op.segments())
    cnt = rp[pick + 1] - rp[pick]
    ptr = np.concatenate([[0], np.cumsum(cnt)])
    idx = np.concatenate([np.arange(rp[i], rp[i + 1]) for i in pick]).astype(np.int64)
    msg = gc.compare_segments(ref, (ptr, vx[idx], ln[idx]), 5.1, 'C2 sample')
    assert msg is None, msg


def test_c5_geometry_vs_oracle_sample(gpu):
    """C5 geometry (64^3, 64 ConeCirc views incl. rays through the origin) sampled vs oracle."""
    from oracle import oracle
    from sph_raytracer_amd import Operator
    from sph_raytracer_amd.raytracer import find_starts
    grid, geom = _orbit(64, (100, 50), kind='circ', grid_shape=(64, 64, 64))
    op = Operator(grid, geom, device=gpu)
    rng = np.random.default_rng(1)
    n = math.prod(geom.shape)
    pick = np.sort(rng.choice(n, 3000, replace=False))
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3)[pick]
    rays = geom.rays.numpy().reshape(-1, 3)[pick]
    starts = find_starts(grid, tr.from_numpy(xs)).numpy()
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ref = oracle.trace_segments(g, xs, rays, starts)
    rp, vx, ln = (t.cpu().numpy() for t in op.segments())
    cnt = rp[pick + 1] - rp[pick]
    ptr = np.concatenate([[0], np.cumsum(cnt)])
    idx = np.concatenate([np.arange(rp[i], rp[i + 1]) for i in pick]).astype(np.int64)
    msg = gc.compare_segments(ref, (ptr, vx[idx], ln[idx]), 5.1, 'C5 sample')
    assert msg is None, msg


@pytest.mark.parametrize('case', ['c3_orbit', 'inside_starts', 'hemisphere'])
def test_wide_families_vs_oracle(case, gpu):
    """Grids of more than 64 boundaries per family, where the trace solves only the chunks whose
    boundaries can cross (sphere_may_cross / cone_may_cross): the C3 grid (129 per family) seen
    by an orbit, random rays starting inside a (100, 90, 130) grid (every family listed behind
    the start), and a hemisphere / half-azimuth grid of 97 x 70 x 80 — every ray against the C
    oracle (IEEE sqrt), segments and f64 line integrals."""
    from oracle import oracle
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid, ViewGeom
    from sph_raytracer_amd.raytracer import find_starts
    if case == 'c3_orbit':
        grid, geom = _orbit(6, (32, 64), grid_shape=(128, 128, 128))
    elif case == 'inside_starts':
        grid = SphericalGrid(shape=(100, 90, 130))
        gen = tr.Generator().manual_seed(7)
        xs = (tr.rand((4000, 3), generator=gen, dtype=tr.float64) - 0.5) * 1.2
        d = tr.randn((4000, 3), generator=gen, dtype=tr.float64)
        geom = ViewGeom(xs, d / d.norm(dim=-1, keepdim=True))
    else:
        grid = SphericalGrid(shape=(97, 70, 80), size_e=(0, tr.pi / 2), size_a=(0, tr.pi))
        geom = sum(ConeRectGeom((24, 40), pos=p, fov=(40, 40))
                   for p in ((3, 1, 2), (-2, 2.5, 0.5), (0.3, -4, -1)))
    op = Operator(grid, geom, device=gpu)
    xs = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape).reshape(-1, 3).copy()
    rays = geom.rays.numpy().reshape(-1, 3).copy()
    starts = find_starts(grid, tr.from_numpy(xs)).numpy()
    oracle.use_mkl_sqrt(False)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ref = oracle.trace_segments(g, xs, rays, starts)
    got = tuple(t.cpu().numpy() for t in op.segments())
    msg = gc.compare_segments(ref, got, 1.0, case)
    assert msg is None, msg
    x = tr.rand(grid.shape, dtype=tr.float64, generator=tr.Generator().manual_seed(3))
    want = np.asarray(oracle.forward(*ref, x.numpy(), math.prod(grid.shape))).reshape(-1)
    have = op(x.to(gpu)).cpu().numpy().reshape(-1)
    assert np.allclose(have, want, rtol=1e-10, atol=1e-12)


def _wedge_rays(n, seed):
    """Lines from outside the unit ball: aimed at random points of it, at points 1e-12..1e-3 off
    the z axis, nearly vertical, from the azimuth seam (x on the negative x axis), and with
    their closest approach to the z axis around the 1e-6 threshold of the half-plane wedge."""
    rng = np.random.default_rng(seed)
    xs = np.empty((n, 3))
    d = np.empty((n, 3))
    for i in range(n):
        u = rng.normal(size=3)
        start = u / np.linalg.norm(u) * rng.uniform(1.05, 8)
        kind = i % 5
        eps = 10.0 ** rng.uniform(-12, -3)
        if kind == 0:
            v = rng.normal(size=3)
            tgt = v / np.linalg.norm(v) * rng.uniform(0, 1) ** (1 / 3)
        elif kind == 1:
            tgt = np.array([eps, eps * rng.uniform(-1, 1), rng.uniform(-0.9, 0.9)])
        elif kind == 2:
            start = np.array([rng.uniform(-0.6, 0.6), rng.uniform(-0.6, 0.6), rng.choice([-3, 3])])
            tgt = start + np.array([eps, eps * rng.uniform(-1, 1), -np.sign(start[2])])
        elif kind == 3:
            start = np.array([-rng.uniform(1.5, 6), 0.0, rng.uniform(-1, 1)])
            tgt = np.array([0.0, rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5)])
        else:
            rho = 1e-6 * rng.uniform(0.5, 2)
            phi = rng.uniform(-np.pi, np.pi)
            tgt = np.array([rho * np.cos(phi), rho * np.sin(phi), rng.uniform(-0.5, 0.5)])
            start = tgt + 3 * np.array([-np.sin(phi), np.cos(phi), rng.uniform(-0.3, 0.3)])
        xs[i] = start
        d[i] = tgt - start
    return xs, d


@pytest.mark.parametrize('shape, size_a', [((30, 40, 150), None), ((20, 70, 100), (-1.0, 2.5)),
                                           ((20, 30, 90), (-3.0, 3.0)), ((128, 128, 128), None),
                                           ((64, 64, 64), None)])
def test_plane_wedge_exact(shape, size_a, gpu, monkeypatch):
    """The half-plane wedge (trace.hip: only the cyclic run of half-planes inside the azimuth
    range a line sweeps over [0, t_hi] is solved) changes nothing: the CSR with it equals the CSR
    without it (SPHRT_TRACE_WEDGE=0) bit for bit, and the voxel sequences equal the oracle's —
    full and partial azimuth ranges (one across the +-pi seam); near-axis, vertical, seam and
    threshold lines.  Lengths against the oracle within 1e-9: ill-conditioned cone roots (lines
    near the z axis, or nearly parallel to a generator) differ between the device and the C
    oracle by up to ~1e-11 with or without the wedge, an ulp of a square root amplified."""
    from oracle import oracle
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    from sph_raytracer_amd.raytracer import find_starts
    kw = {} if size_a is None else {'size_a': size_a}
    grid = SphericalGrid(shape=shape, **kw)
    xs, d = _wedge_rays(5000, sum(shape))
    geom = ViewGeom(tr.from_numpy(xs), tr.from_numpy(d))
    got = tuple(t.cpu().numpy() for t in Operator(grid, geom, device=gpu).segments())
    monkeypatch.setenv('SPHRT_TRACE_WEDGE', '0')
    full = tuple(t.cpu().numpy() for t in Operator(grid, geom, device=gpu).segments())
    for a, b in zip(got, full):
        assert np.array_equal(a, b)
    oracle.use_mkl_sqrt(False)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ref = oracle.trace_segments(g, xs, d, find_starts(grid, tr.from_numpy(xs)).numpy())
    assert np.array_equal(np.asarray(ref[0]), got[0])
    assert np.array_equal(np.asarray(ref[1]), got[1])
    lr = np.asarray(ref[2])
    err = np.abs(got[2] - lr)
    k = int(np.argmax(err))
    ray = int(np.searchsorted(np.asarray(ref[0]), k, side='right') - 1)
    assert err[k] <= 1e-9, (f'ray {ray} (kind {ray % 5}) x {xs[ray].tolist()} d {d[ray].tolist()}'
                            f': segment {k - ref[0][ray]} {lr[k]!r} vs {got[2][k]!r}')


def test_half_tables_float64(gpu, monkeypatch):
    """C5 geometry (granule tables of up to 1512 entries: float64 forwards stage them in two
    halves, apply.hip HALF): float64 forward and transposed adjoint against the C oracle on the
    GPU's own trace, bitwise equal to whole tables (SPHRT_FWD_HALF=0), and two channels (the
    first half staged again per channel) equal to one channel each."""
    from oracle import oracle
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(64, (100, 50), kind='circ', grid_shape=(64, 64, 64))
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'natural')    # (the wedge order's tables are smaller)
    op = Operator(grid, geom, device=gpu)
    monkeypatch.delenv('SPHRT_RAY_ORDER')
    assert 1279 < op._csr['desc'].tab_stride <= 1536
    gen = tr.Generator().manual_seed(5)
    x = tr.rand((2,) + tuple(grid.shape), dtype=tr.float64, generator=gen)
    xg = x.to(gpu)
    assert op._forward_kernel_name(xg[0]).endswith('true, true, false, 3>')   # (half, not dense)
    y = op(xg[0])
    rp, vx, ln = (t.cpu().numpy() for t in op.segments())
    nv = math.prod(grid.shape)
    ref = np.asarray(oracle.forward(rp, vx, ln, x[0].numpy(), nv)).reshape(-1)
    assert np.allclose(y.cpu().numpy().reshape(-1), ref, rtol=1e-10, atol=1e-12)
    y2 = op(xg)
    assert tr.equal(y2[0], y) and tr.equal(y2[1], op(xg[1]))
    yt = tr.rand(geom.shape, dtype=tr.float64, generator=gen)
    a = op.T(yt.to(gpu))
    aref = np.asarray(oracle.adjoint(rp, vx, ln, yt.numpy().reshape(-1), nv)).reshape(-1)
    assert np.allclose(a.cpu().numpy().reshape(-1), aref, rtol=1e-10, atol=1e-12)
    monkeypatch.setenv('SPHRT_FWD_HALF', '0')
    assert tr.equal(op(xg[0]), y) and tr.equal(op(xg), y2) and tr.equal(op.T(yt.to(gpu)), a)


def test_gd_retrieval_decreases_loss(gpu):
    """static_retrieval.py's loop (FullyDenseModel, SquareLoss + NegRegularizer, Adam) on a small
    grid: runs unchanged on the HIP operator and the fidelity loss drops."""
    from sph_raytracer_amd import Operator
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    from sph_raytracer_amd.retrieval import gd
    grid, geom = _orbit(12, (20, 16), kind='circ', grid_shape=(16, 16, 16))
    x = tr.zeros(grid.shape, device=gpu)
    x[:, 8:, :8] = 1
    x[:, :8, 8:] = 1
    op = Operator(grid, geom, device=x.device)
    meas = op(x)
    coeffs, y, losses = gd(op, meas, FullyDenseModel(grid), lr=1e-1, num_iterations=30,
                           loss_fns=[1 * SquareLoss(), 1 * NegRegularizer()], progress_bar=False)
    fid = list(losses.values())[0]
    assert fid[-1] < 0.2 * fid[0]
    assert y.shape == meas.shape


def _deferred_count(grid, geom, gpu):
    """Rays the wave trace defers to the exact (emulated introsort) path: the trace workspace's
    counter after a count pass (trace.hip launch_trace)."""
    return _exact_stats(grid, geom, gpu)[0]


def _exact_stats(grid, geom, gpu):
    """(deferred rays, depth-limit ranges rank-sorted, ranges heap-sorted by one lane) of a count
    pass: the trace workspace's counters (trace.hip launch_trace, exact_heap_range)."""
    from sph_raytracer_amd import _lib, raytracer as rt
    lib = _lib.load()
    plan = rt._Plan(grid, gpu)
    batch = rt._RayBatch(grid, geom.ray_starts, rt._geom_rays(geom, gpu), gpu)
    counts = tr.empty(max(batch.n, 1), dtype=tr.int32, device=gpu)
    tws = rt._workspace(lib, plan, batch.n, gpu)
    _lib.check(lib.sphrt_trace_count(plan.handle, batch.desc, _lib.ptr(counts), _lib.ptr(tws),
                                     tws.numel(), _lib.stream_of(gpu)), 'sphrt_trace_count')
    head = tws[:256].cpu().view(tr.int64)
    return int(head[0]), int(head[16]), int(head[17])


@pytest.mark.parametrize('shape,a_full', [((64, 64, 64), False), ((17, 9, 30), False),
                                          ((12, 20, 7), True), ((40, 3, 100), True),
                                          ((900, 4, 30), False)])   # K 1844: serial exact kernel
def test_exact_tie_rays_vs_oracle(shape, a_full, gpu):
    """Rays that hit exact ties (through the origin: every cone and half-plane crossed at one
    distance; starts on the a = 0 half-plane) take the exact path, whose emulated introsort
    decides the voxel after each tie group.  Compared with the IEEE-sqrt C oracle under the
    parity contract (golden_cases.compare_segments: voxel sequences exact, lengths 1e-12)."""
    from oracle import oracle
    from sph_raytracer_amd import ConeCircGeom, Operator, SphericalGrid, ViewGeom
    from sph_raytracer_amd.raytracer import find_starts
    size_a = (0, 2 * tr.pi) if a_full else (-tr.pi, tr.pi)
    grid = SphericalGrid(shape=shape, size_a=size_a)
    geoms = [ConeCircGeom(shape=(6, 16), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(0, 40))
             for th in tr.linspace(0, 2 * tr.pi, 7)]
    rng = np.random.default_rng(3)
    pos = tr.from_numpy(rng.normal(size=(40, 3)) * 2.0)
    geoms.append(ViewGeom(pos[:, None, :], -pos[:, None, :]))           # aimed at the origin
    xs_in = tr.from_numpy(np.c_[rng.uniform(0.1, 0.9, 30), np.zeros(30), rng.uniform(-.5, .5, 30)])
    geoms.append(ViewGeom(xs_in[:, None, :], tr.from_numpy(rng.normal(size=(30, 1, 3)))))
    for gm in geoms:
        op = Operator(grid, gm, device=gpu)
        oracle.use_mkl_sqrt(False)
        g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
        xs = np.broadcast_to(gm.ray_starts.numpy(), gm.rays.shape).reshape(-1, 3).copy()
        d = gm.rays.numpy().reshape(-1, 3).copy()
        ptr, vox, seg = oracle.trace_segments(g, xs, d, find_starts(grid, tr.from_numpy(xs)).numpy())
        got = tuple(t.cpu().numpy() for t in op.segments())
        msg = gc.compare_segments((ptr, vox, seg), got, 5.1, f'{shape} {type(gm).__name__}')
        assert msg is None, msg
    # the geometry really exercises the exact path (rays through the origin, starts on a = 0)
    stats = [_exact_stats(grid, gm, gpu) for gm in geoms]
    print('(deferred rays, heap ranges rank-sorted, heap-sorted) per view:', stats)
    assert sum(st[0] for st in stats) > 0
    if shape == (64, 64, 64):     # the depth limit runs out (reference heapsort): rank-sorted
        assert sum(st[1] for st in stats) > 0


def test_fast_path_matches_general_path(c2, gpu):
    """Steady-state calls go through the CPython entry (csrc/fastpath.cpp) once a shape is bound:
    bitwise the same result as the general path, fresh output tensors, and inputs it does not
    serve (grad, non-contiguous, other shapes) still take the general path."""
    grid, geom, op = c2
    assert op._fastc is not None or op._fast == {}
    for dt in (tr.float32, tr.float64):
        x = tr.rand(grid.shape, dtype=dt, device=gpu)
        y0 = op(x)                       # binds
        y1 = op(x)                       # fast path
        y2 = op(x)
        assert op._fastc is not None
        assert y1.shape == y0.shape == tuple(geom.shape) and y1.dtype == dt
        assert tr.equal(y0, y1) and tr.equal(y1, y2) and y1.data_ptr() != y2.data_ptr()
        xg = x.clone().requires_grad_(True)
        yg = op(xg)
        assert yg.requires_grad and tr.equal(yg.detach(), y0)
        xt = x.transpose(0, 2).contiguous().transpose(0, 2)     # same values, not contiguous
        assert tr.equal(op(xt), y0)
        x2 = tr.stack([x, 2 * x])
        y3 = op(x2)
        assert y3.shape == (2,) + tuple(geom.shape) and tr.equal(y3[0], y0)


def test_float32_accuracy_vs_float64(c2, gpu):
    """float32 forward and transposed adjoint (products, runs and cross-thread stitching in
    float32, like the reference's float32 sums) stay within 1e-6 relative of the float64 results
    on the same float32 inputs (measured <= 2.5e-7 at C2-C5; the parity bound is 1e-5)."""
    grid, geom, op = c2
    g = tr.Generator(device='cpu').manual_seed(11)
    x = tr.rand(grid.shape, dtype=tr.float32, generator=g).to(gpu)
    y = tr.rand(tuple(geom.shape), dtype=tr.float32, generator=g).to(gpu)
    for a32, a64 in ((op(x), op(x.double())), (op.T(y), op.T(y.double()))):
        big = a64.abs() > 1e-3 * a64.abs().max()
        rel = ((a32.double() - a64).abs() / a64.abs())[big]
        assert float(rel.max()) < 1e-6, float(rel.max())


def test_adjoint_fast_path_matches_general_path(c2, gpu):
    """op.T on a bound shape/dtype goes through the CPython entry as one transposed-CSR forward
    (the input read through the trace's ray ids when the trace has another ray order: the C2
    orbit's view tiles, a single ConeCirc view's wedges): bitwise the general path's result,
    fresh outputs."""
    from sph_raytracer_amd import Operator
    grid, geom, op = c2
    for dt in (tr.float32, tr.float64):
        y = tr.rand(tuple(geom.shape), dtype=dt, device=gpu)
        a0 = op.T(y)                     # general path, binds
        a1 = op.T(y)                     # fast path
        a2 = op.T(y)
        assert op._fastc_T is not None
        assert a1.shape == a0.shape == tuple(grid.shape) and a1.dtype == dt
        assert tr.equal(a0, a1) and tr.equal(a1, a2) and a1.data_ptr() != a2.data_ptr()
        assert tr.equal(op.T(y.cpu()).to(gpu), a0)            # host input: general path
    assert op._csr['ray_id'] is not None                       # (view tiles)
    from sph_raytracer_amd import ConeCircGeom, SphericalGrid
    cgrid = SphericalGrid(shape=(12, 12, 12))
    cop = Operator(cgrid, ConeCircGeom((12, 16), pos=(3, 1, 1)), device=gpu)
    assert cop._csr['ray_id'] is not None                      # (wedges)
    yc = tr.rand((12, 16), dtype=tr.float64, device=gpu)
    c0 = cop.T(yc)
    assert tr.equal(cop.T(yc), c0) and cop._fastc_T is not None and tr.equal(cop.T(yc), c0)


@pytest.mark.parametrize('dt', [tr.float64, tr.float32])
def test_dynamic_operator_T_time_slices(gpu, dt):
    """Operator.T on a dynamic grid: raises like the reference (raytracer.py:733-734) unless
    time_slices=True, which gives the native time-indexed adjoint — equal to the gradient
    autograd gives the forward (bitwise: the same transposed time-paired CSR), and for one
    geometry over every time step, to the static adjoint of each step's image."""
    from sph_raytracer_amd import ConeCircGeom, Operator, SphericalGrid
    T = 5
    grid = SphericalGrid(shape=(T, 12, 10, 16))
    geom = sum(ConeCircGeom(shape=(24, 16), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(0, 45))
               for th in tr.linspace(0, 2 * tr.pi, T))
    op = Operator(grid, geom, dynamic=True, device=gpu)
    g = tr.Generator(device=gpu).manual_seed(3)
    x = tr.rand(grid.shape, dtype=dt, device=gpu, generator=g)
    y = tr.rand(geom.shape, dtype=dt, device=gpu, generator=g)
    with pytest.raises(NotImplementedError):
        op.T(y)
    got = op.T(y, time_slices=True)
    assert got.shape == grid.shape and got.dtype == dt
    xg = x.clone().requires_grad_(True)
    (op(xg) * y).sum().backward()
    assert tr.equal(got, xg.grad)
    # the steady-state binding (csrc/fastpath.cpp: gather into trace order + transposed forward)
    # serves the later calls: the same bits
    assert op._fastc_A is not None
    assert tr.equal(op.T(y, time_slices=True), got)
    assert tr.equal(op._apply_adjoint(y, tuple(grid.shape), dt, gpu), got)
    # one geometry seen at every time step: slice t = the static adjoint of image t
    single = geom.geoms[0]
    op1 = Operator(grid, single, device=gpu)
    st = Operator(SphericalGrid(shape=grid.shape[1:]), single, device=gpu)
    ys = tr.rand((T,) + tuple(single.shape), dtype=dt, device=gpu, generator=g)
    got1 = op1.T(ys, time_slices=True)
    want = tr.stack([st.T(ys[t]) for t in range(T)])
    tol = 1e-12 if dt == tr.float64 else 1e-5
    assert tr.allclose(got1, want, rtol=tol, atol=tol * float(want.abs().max()))


def test_dynamic_pairing_forward_and_adjoint(gpu):
    """View i <-> time slice i (dynamic grid, a collection of T views): the forward runs on the
    time-paired CSR (granule tables over the flattened (T, vol) density) and the adjoint on its
    transpose.  Forward equals the per-segment time-slice gather of the trace's CSR bitwise in
    float64 up to summation order (1e-12), the adjoint equals the float64-atomic adjoint, and
    <A x, y> = <x, A^T y>."""
    from sph_raytracer_amd import ConeCircGeom, Operator, SphericalGrid
    T = 6
    grid = SphericalGrid(shape=(T, 20, 18, 24))
    geom = sum(ConeCircGeom(shape=(30, 20), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(0, 45))
               for th in tr.linspace(0, 2 * tr.pi, T))
    op = Operator(grid, geom, dynamic=True, device=gpu)
    g = tr.Generator(device=gpu).manual_seed(7)
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu, generator=g)
    y = tr.rand(geom.shape, dtype=tr.float64, device=gpu, generator=g)
    fx = op(x)
    n_chan, div, _ = op._layout(x.shape)
    assert div > 0 and op._paired(T, div) is not None
    assert op._forward_kernel_name(x).startswith('forward_kernel<double, double, 0')
    # the trace's own CSR with the time-slice gather (kFwdDynamic)
    ref = tr.empty(op._csr['n'], dtype=tr.float64, device=gpu)
    lib = __import__('sph_raytracer_amd._lib', fromlist=['_lib'])
    lib.check(lib.load().sphrt_forward_f64(op._csr['desc'], lib.ptr(x), 1, x[0].numel(), div,
                                           lib.ptr(ref), op._csr['n'], lib.stream_of(gpu)), 'fwd')
    assert tr.allclose(fx.reshape(-1), ref, rtol=1e-12, atol=1e-14)
    xg = x.clone().requires_grad_(True)
    (op(xg) * y).sum().backward()
    atx = xg.grad
    op.adjoint_mode = 'atomic'
    xa = x.clone().requires_grad_(True)
    (op(xa) * y).sum().backward()
    op.adjoint_mode = 'transpose'
    assert tr.allclose(atx, xa.grad, rtol=1e-12, atol=1e-14)
    lhs, rhs = (fx * y).sum().item(), (x * atx).sum().item()
    assert abs(lhs - rhs) <= 1e-12 * abs(lhs)
    xg2 = x.clone().requires_grad_(True)
    (op(xg2) * y).sum().backward()
    assert tr.equal(xg2.grad, atx)                       # deterministic
    # the paired CSR's contiguous-XCD-range hint (order bit 1) changes the block order only
    pd = op._paired(T, div)['desc']
    assert pd.order & 2
    for bits in (pd.order & 1, (pd.order & 1) ^ 1):       # dispatch-order / runs and reversed
        pd.order = bits
        assert tr.equal(op(x), fx)
    pd.order = 2
    f32 = op(x.float())
    assert tr.allclose(f32.double(), fx, rtol=1e-5, atol=1e-6)
    assert op._fastc is not None and tr.equal(op(x), fx)     # bound: the CPython fast path


def test_dense_ranges_need_dense_blocks(gpu):
    """The time-paired transposed CSR (dense output ranges, sphrt_csr.order bit 2) is indexed in
    the blocks of sphrt_csr_index_dense (1984 row starts, apply.hip kDenseSegPerBlock); the
    forward refuses a CSR that claims dense ranges with another block count instead of reading
    the wrong first pass."""
    from sph_raytracer_amd import ConeCircGeom, Operator, SphericalGrid, _lib
    T = 6
    grid = SphericalGrid(shape=(T, 20, 18, 24))
    geom = sum(ConeCircGeom(shape=(30, 20), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(0, 45))
               for th in tr.linspace(0, 2 * tr.pi, T))
    op = Operator(grid, geom, dynamic=True, device=gpu)
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu)
    y = tr.rand(geom.shape, dtype=tr.float64, device=gpu)
    g = op._apply_adjoint(y, tuple(x.shape), x.dtype, x.device)
    n_chan, div, _ = op._layout(x.shape)
    pt = op._paired(T, div)['transposed']['desc']
    lib = _lib.load()
    assert pt.order & 4 and pt.n_blocks == lib.sphrt_csr_blocks_dense(pt.n_segments)
    bad = _lib.CSR.from_buffer_copy(pt)
    bad.n_blocks = lib.sphrt_csr_blocks(pt.n_segments)
    assert bad.n_blocks != pt.n_blocks
    yt = y.reshape(-1).contiguous()
    out = tr.empty(pt.n_rays, dtype=tr.float64, device=gpu)
    rc = lib.sphrt_forward_f64(bad, _lib.ptr(yt), 1, yt.numel(), 0, _lib.ptr(out), pt.n_rays,
                               _lib.stream_of(gpu))
    with pytest.raises(RuntimeError, match='sphrt_csr_index_dense'):
        _lib.check(rc, 'forward')
    rc = lib.sphrt_forward_f64(pt, _lib.ptr(yt), 1, yt.numel(), 0, _lib.ptr(out), pt.n_rays,
                               _lib.stream_of(gpu))
    _lib.check(rc, 'forward')
    assert tr.equal(out.reshape(g.shape), g)


@pytest.mark.parametrize('grid_shape,n_views,det,order', [
    ((128, 128, 128), 6, (128, 128), 'runs'),     # density > 4 MB: runs of 64 blocks per XCD
    ((50, 50, 50), 80, (50, 100), 'dispatch'),    # > 1536 blocks, small density
    ((50, 50, 50), 10, (50, 100), 'range'),       # <= 1536 blocks: one range per XCD
])
def test_workgroup_orders_cover_every_block(grid_shape, n_views, det, order, gpu):
    """The forward's workgroup -> block maps (apply.hip block_of / fwd_chunk) are bijections:
    op(x) and op.T(y) equal a torch index_add over the CSR's own segments for each launch order
    (float64 within 1e-12, float32 within 1e-5 of it)."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(n_views, det, grid_shape=grid_shape)
    op = Operator(grid, geom, device=gpu)
    csr = op._csr
    n, nvox = csr['n'], math.prod(grid_shape)
    total = csr['total']
    ptr = csr['row_ptr']
    rows = tr.arange(n, device=gpu) if csr['ray_id'] is None else csr['ray_id'].long()
    ray = tr.repeat_interleave(rows, ptr[1:] - ptr[:-1])      # (each row's geometry ray)
    vox = (csr['vox'][:total] & 0x7fffffff).long()
    ln = csr['len'][:total]
    nblocks = csr['nblocks']
    assert ray.numel() == total
    if order == 'runs':      # with a ragged tail (blocks past the last whole 8 x 64 keep order)
        assert nblocks > 512 and nblocks % 512 != 0, nblocks
    elif order == 'dispatch':   # (no brick staging: the 50^3 density fits one XCD's L2)
        assert nblocks > 1536 and csr['desc'].stage_shape[0] == 0, nblocks
    else:
        assert 8 < nblocks <= 1536 and nblocks % 8 != 0, nblocks
    g = tr.Generator(device=gpu).manual_seed(7)
    x = tr.rand(grid_shape, dtype=tr.float64, device=gpu, generator=g)
    y = tr.rand(geom.shape, dtype=tr.float64, device=gpu, generator=g)
    ref = tr.zeros(n, dtype=tr.float64, device=gpu).index_add_(0, ray, x.reshape(-1)[vox] * ln)
    got = op(x).reshape(-1)
    assert float((got - ref).abs().max()) <= 1e-12 * float(ref.abs().max())
    got32 = op(x.float()).reshape(-1).double()
    assert float((got32 - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
    reft = tr.zeros(nvox, dtype=tr.float64, device=gpu).index_add_(0, vox, y.reshape(-1)[ray] * ln)
    gott = op.T(y).reshape(-1)
    assert float((gott - reft).abs().max()) <= 1e-12 * float(reft.abs().max())


def test_gd_optimiser_as_the_reference_builds_it(gpu):
    """gd() builds the optimiser exactly as the reference does (retrieval.py:84: no implementation
    chosen for the caller, so torch's default multi-tensor step on GPU tensors); an explicit
    Adam(fused=True) gives the same loss history, coefficients and reconstruction within
    rounding (relative 1e-9 after 30 steps); the masks/weights of 1 that the losses skip change
    nothing."""
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import CheaterLoss, NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    grid, geom = _orbit(12, (20, 16), kind='circ', grid_shape=(16, 16, 16))
    x = tr.zeros(grid.shape, dtype=tr.float64, device=gpu)
    x[:, 8:, :8] = 1
    x[:, :8, 8:] = 1
    op = Operator(grid, geom, device=gpu)
    meas = op(x)
    made = []
    orig = tr.optim.Adam.__init__

    def spy(self, params, **kw):
        made.append(dict(kw))
        orig(self, params, **kw)

    runs = []
    for kw, fns in (({'fused': True}, [0.5 * SquareLoss(), NegRegularizer(), CheaterLoss(x)]),
                    ({}, [SquareLoss(lam=0.5, projection_mask=tr.ones_like(meas)),
                          NegRegularizer(volume_mask=tr.ones_like(x)), CheaterLoss(x)])):
        tr.optim.Adam.__init__ = spy
        try:
            c, yh, hist = retrieval.gd(op, meas, FullyDenseModel(grid), lr=1e-1, num_iterations=30,
                                       loss_fns=fns, progress_bar=False, **kw)
        finally:
            tr.optim.Adam.__init__ = orig
        runs.append((c.detach().clone(), yh.detach().clone(), list(hist.values())))
    assert made == [{'fused': True, 'lr': 1e-1}, {'lr': 1e-1}]     # nothing added to the caller's
    (ca, ya, ha), (cb, yb, hb) = runs
    for a, b in zip(ha, hb):
        assert len(a) == len(b) == 30
        assert np.allclose(a, b, rtol=1e-9, atol=1e-15)
    assert ha[0][-1] < 0.2 * ha[0][0]
    assert tr.allclose(ca, cb, rtol=1e-9, atol=1e-12)
    assert tr.allclose(ya, yb, rtol=1e-9, atol=1e-12)


def test_staged_forward_on_concurrent_streams(gpu, monkeypatch):
    """A brick-staged operator called on two streams at once: each call packs into a stage of its
    own (per-call caching-allocator buffer), so both results equal the sequential
    ones bitwise — forward and transposed adjoint, float32 and float64."""
    from sph_raytracer_amd import Operator
    monkeypatch.setenv('SPHRT_BRICK', '2,4,4')
    grid, geom = _orbit(6, (24, 30), grid_shape=(30, 21, 26))
    op = Operator(grid, geom, device=gpu)
    assert op._csr['desc'].stage_shape[0] > 0
    g = tr.Generator(device=gpu).manual_seed(3)
    for dt in (tr.float32, tr.float64):
        xs = [tr.rand(grid.shape, dtype=dt, device=gpu, generator=g) for _ in range(2)]
        ref = [op(x) for x in xs]
        s1, s2 = tr.cuda.Stream(device=gpu), tr.cuda.Stream(device=gpu)
        tr.cuda.synchronize(gpu)
        outs = [None, None]
        for _ in range(20):
            for i, s in enumerate((s1, s2)):
                s.wait_stream(tr.cuda.current_stream(gpu))
                with tr.cuda.stream(s):
                    outs[i] = op(xs[i])
            tr.cuda.current_stream(gpu).wait_stream(s1)
            tr.cuda.current_stream(gpu).wait_stream(s2)
            tr.cuda.synchronize(gpu)
            assert tr.equal(outs[0], ref[0]) and tr.equal(outs[1], ref[1])


def test_first_float64_use_on_side_stream(gpu):
    """The float64 segment lengths stay in the trace staging until the first float64 use, which
    compacts them on the current stream: an operator whose first float64 forward and
    adjoint run on a side stream — with allocations on the construction stream right after —
    matches one whose first float64 use ran on the default stream, bitwise."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(5, (24, 30), grid_shape=(20, 17, 22))
    g = tr.Generator(device=gpu).manual_seed(11)
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu, generator=g)
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, device=gpu, generator=g)
    ref_op = Operator(grid, geom, device=gpu)
    ref_f, ref_a = ref_op(x), ref_op.T(y)
    for _ in range(3):
        op = Operator(grid, geom, device=gpu)
        op(x.float())                            # float32 first: the lengths stay staged
        s = tr.cuda.Stream(device=gpu)
        s.wait_stream(tr.cuda.current_stream(gpu))
        with tr.cuda.stream(s):
            f = op(x)
            a = op.T(y)
        junk = [tr.full((1 << 20,), 7.0, dtype=tr.float64, device=gpu) for _ in range(8)]
        tr.cuda.current_stream(gpu).wait_stream(s)
        tr.cuda.synchronize(gpu)
        del junk
        assert tr.equal(f, ref_f) and tr.equal(a, ref_a)


def test_operator_device_argument(gpu):
    """Operator(device='cuda:k') traces and computes on GPU k whatever device is current (ADVICE
    r1): the compute device follows `device`; with two GPUs an operator built on cuda:1 while
    cuda:0 is current (and called after the current device changed) matches the cuda:0 one."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(3, (16, 20), grid_shape=(12, 10, 16))
    op0 = Operator(grid, geom, device=gpu)
    assert op0._cdev == tr.device('cuda', 0)
    x = tr.rand(grid.shape, dtype=tr.float64, device=gpu)
    y0 = op0(x)
    assert y0.device == gpu
    if tr.cuda.device_count() < 2:
        pytest.skip('one GPU: the cross-device half needs two')
    dev1 = tr.device('cuda', 1)
    with tr.cuda.device(0):
        op1 = Operator(grid, geom, device=dev1)
    assert op1._cdev == dev1 and op1._csr['row_ptr'].device == dev1
    x1 = x.to(dev1)
    with tr.cuda.device(0):
        y1 = op1(x1)          # current device 0, operator and density on 1
    assert y1.device == dev1 and tr.equal(y1.cpu(), y0.cpu())
    with tr.cuda.device(0):
        g1 = op1.T(y1)
    assert tr.allclose(g1.cpu(), op0.T(y0).cpu(), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('kind, n_views, det, grid_shape', [
    ('rect', 50, (50, 100), (50, 50, 50)),          # C2
    ('circ', 64, (100, 50), (64, 64, 64)),          # C5 geometry: ring 0 through the origin
    ('rect', 8, (64, 96), (40, 70, 33)),
])
def test_onepass_trace_full_size(kind, n_views, det, grid_shape, gpu, monkeypatch):
    """At full size the one-pass trace equals the two-pass one bit for bit and no ray exceeds its
    geometric bound (every bound holds: the fallback is not taken)."""
    from sph_raytracer_amd import Operator, raytracer as rt
    grid, geom = _orbit(n_views, det, kind=kind, grid_shape=grid_shape)
    monkeypatch.setenv('SPHRT_TRACE', 'twopass')
    ref = Operator(grid, geom, device=gpu)._csr
    monkeypatch.setenv('SPHRT_TRACE', 'onepass')
    calls = []
    orig = rt._lib.load().sphrt_trace_fill

    def spy(*a):
        calls.append(1)
        return orig(*a)
    monkeypatch.setattr(rt._lib.load(), 'sphrt_trace_fill', spy)
    got = Operator(grid, geom, device=gpu)._csr
    assert not calls, 'a segment bound failed: the one-pass trace fell back to the fill pass'
    assert ref['total'] == got['total']
    for k in ('row_ptr', 'vox', 'len'):
        assert tr.equal(ref[k][:ref['total'] if k != 'row_ptr' else None],
                        got[k][:got['total'] if k != 'row_ptr' else None]), k


@pytest.mark.parametrize('grid_shape, staged', [((50, 50, 50), 'auto'), ((96, 80, 90), 'auto'),
                                                ((30, 21, 26), '2,4,4'), ((30, 21, 26), '4,2,4')])
def test_onepass_tables_equal_twopass(grid_shape, staged, gpu, monkeypatch):
    """Granule tables built in one pass (wide tables + pack) equal the count + fill ones: block
    records, loc, tables (bitmap build at 50^3, radix build above 2^19 voxels, brick-staged)."""
    from sph_raytracer_amd import Operator
    monkeypatch.setenv('SPHRT_BRICK', staged)
    grid, geom = _orbit(6, (40, 64), grid_shape=grid_shape)
    res = []
    for mode in ('twopass', 'onepass'):
        monkeypatch.setenv('SPHRT_TABLES', mode)
        c = Operator(grid, geom, device=gpu)._csr
        d = c['desc']
        res.append((c['blocks'].cpu(), c['loc'][:c['total']].cpu(), d.tab_stride, d.n_fallback,
                    c['tab'][:c['nblocks'] * d.tab_stride].cpu()))
    (b0, l0, s0, f0, t0), (b1, l1, s1, f1, t1) = res
    assert s0 == s1 and f0 == f1
    assert tr.equal(b0, b1) and tr.equal(l0, l1)
    n_tab = b0.reshape(-1, 6)[:, 5]
    for b in range(len(n_tab)):      # entries past n_tab are unused (uninitialised)
        k = int(n_tab[b])
        assert tr.equal(t0[b * s0:b * s0 + k], t1[b * s1:b * s1 + k])


def _expected_runs(csr, n_blocks_fields):
    """Host restatement of block_runs_kernel: per block, the runs of consecutive rays of its rows
    and of its share of the empty list (None for more than MAX_RUNS)."""
    from sph_raytracer_amd import _lib
    blocks = csr['blocks'].cpu().numpy().reshape(-1, n_blocks_fields)
    row_ray = csr['row_ray'].cpu().numpy()
    empty = csr['empty_ray'].cpu().numpy()
    n_rows = csr['n'] - blocks[-1, 1]

    def runs(v):
        if len(v) == 0:
            return []
        cut = np.nonzero(np.diff(v) != 1)[0] + 1
        starts = np.concatenate(([0], cut))
        ends = np.concatenate((cut, [len(v)]))
        return [(int(a), int(v[a]), int(b - a)) for a, b in zip(starts, ends)]

    out = []
    for b in range(len(blocks)):
        k0 = blocks[b, 4]
        k1 = blocks[b + 1, 4] if b + 1 < len(blocks) else n_rows
        rr = runs(row_ray[k0:k1])
        er = runs(empty[blocks[b, 0]:blocks[b, 1]])
        out.append((rr if len(rr) <= _lib.MAX_RUNS else None,
                    er if len(er) <= _lib.MAX_RUNS else None))
    return out


def test_run_records(c2, gpu, monkeypatch):
    """Row runs / empty ranges (sphrt_csr_runs, forced on at C2): the records equal a numpy
    restatement on the C2 trace and its transpose, the forward and the transposed adjoint with records equal the ones
    reading row_ray / empty_ray bitwise (f32, f64, 3 channels), and a trace whose rows are too
    fragmented for the records (random rays, every other one missing) leaves desc.runs unset and
    still matches the oracle."""
    from sph_raytracer_amd import Operator, ViewGeom, _lib
    grid, geom, op_auto = c2
    if os.environ.get('SPHRT_RUNS', 'auto') == 'auto':
        assert not op_auto._csr['desc'].runs   # auto: a single-wave grid keeps the loads
    monkeypatch.setenv('SPHRT_RUNS', 'on')
    # rows in geometry order: the orbit's view tiles would scatter every row's rays (records
    # overflow, desc.runs unset: their fallback is checked below)
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'natural')
    op = Operator(grid, geom, device=gpu)
    for csr in (op._csr, dict(op._transposed(), n=math.prod(grid.shape))):
        if 'keep' in csr:      # transposed: row_ptr, t_ray, len, len32, vox_list, empty, blocks..
            k = csr['keep']
            csr = dict(n=csr['n'], blocks=k[6], row_ray=k[4], empty_ray=k[5], runs=k[9],
                       desc=csr['desc'])
        assert csr['desc'].runs, 'run records expected at C2'
        rec = csr['runs'].cpu().numpy().reshape(-1, _lib.RUN_FIELDS)
        for b, (rr, er) in enumerate(_expected_runs(csr, _lib.BLOCK_FIELDS)):
            assert rr is not None and er is not None
            assert rec[b, 0] == len(rr) and rec[b, 1] == len(er)
            for i, (off, ray, _) in enumerate(rr):
                assert (rec[b, 2 + 2 * i], rec[b, 3 + 2 * i]) == (off, ray)
            for i, (_, ray, cnt) in enumerate(er):
                assert (rec[b, 16 + 2 * i], rec[b, 17 + 2 * i]) == (ray, cnt)
    g = tr.Generator(device=gpu).manual_seed(11)
    descs = [op._csr['desc'], op._transposed()['desc']]
    for dt in (tr.float32, tr.float64):
        x = tr.rand((3,) + tuple(grid.shape), dtype=dt, device=gpu, generator=g)
        y = tr.rand(geom.shape, dtype=dt, device=gpu, generator=g)
        a, at = op(x), op.T(y)
        tol = 1e-12 if dt == tr.float64 else 1e-6     # (op_auto: view tiles, another sum order)
        for u, v in ((op_auto(x), a), (op_auto.T(y), at)):
            assert float((u - v).abs().max()) <= tol * float(v.abs().max())
        saved = [d.runs for d in descs]
        try:
            for d in descs:
                d.runs = None
            op._fast.clear()
            op._fastc = None
            assert tr.equal(op(x), a) and tr.equal(op.T(y), at)
        finally:
            for d, r in zip(descs, saved):
                d.runs = r
            op._fast.clear()
            op._fastc = None
    # fragmented rows: random directions from inside the grid's bounding box, half of them
    # pointed away from a tiny grid -> more than MAX_RUNS runs per block
    rng = np.random.default_rng(5)
    n = 40000
    d = rng.normal(size=(n, 3))
    d[1::2] = np.array([0.0, 0.0, 1.0])                     # every other ray: straight up ...
    xs = np.tile(np.array([0.0, 0.0, 3.0]), (n, 1))          # ... from above the grid: misses
    xs[0::2] = rng.uniform(-0.4, 0.4, size=(n // 2, 3))      # the others start inside
    geom_f = ViewGeom(tr.from_numpy(xs), tr.from_numpy(d))
    from sph_raytracer_amd import SphericalGrid
    grid_f = SphericalGrid(shape=(6, 5, 8))
    op_f = Operator(grid_f, geom_f, device=gpu)
    assert not op_f._csr['desc'].runs
    xf = tr.rand(grid_f.shape, dtype=tr.float64, device=gpu, generator=g)
    yf = op_f(xf).cpu().numpy().reshape(-1)
    from oracle import oracle
    from sph_raytracer_amd.raytracer import find_starts
    og = oracle.Grid.from_boundaries(grid_f.r_b.numpy(), grid_f.e_b.numpy(), grid_f.a_b.numpy())
    ptr, vox, seg = oracle.trace_segments(og, geom_f.ray_starts.numpy(), geom_f.rays.numpy(),
                                          find_starts(grid_f, geom_f.ray_starts).numpy())
    ref = oracle.forward(ptr, vox, seg, xf.cpu().numpy(), math.prod(grid_f.shape))[0]
    assert np.allclose(yf, ref, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize('kind, grid_shape', [('rect', (20, 20, 20)), ('circ', (96, 96, 96))])
def test_block_order_hint(kind, grid_shape, gpu):
    """sphrt_csr.order = 1 (blocks in reverse order) changes nothing but the order: forward
    (float32, float64) and transposed adjoint bitwise equal to order 0, for a one-wave launch
    (one contiguous range per XCD) and a multi-wave one (dispatch order for float32, runs of 64
    blocks per XCD for float64, brick staging).  Multi-wave CSRs alternate their order from call
    to call on every path (general, ctypes fast path, C++ fast path, adjoint); one-wave CSRs
    keep order 0."""
    from sph_raytracer_amd import Operator
    small = kind == 'rect'
    grid, geom = _orbit(8 if small else 64, (16, 24) if small else (32, 64), kind=kind,
                        grid_shape=grid_shape)
    op = Operator(grid, geom, device=gpu)
    assert (op._csr['desc'].n_blocks > 256 * 6) == (not small)
    g = tr.Generator(device='cpu').manual_seed(5)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g).to(gpu)
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, generator=g).to(gpu)
    fwd, adj = op._csr['desc'], op._transposed()['desc']
    calls = {'f32': (op, x.float(), fwd), 'f64': (op, x, fwd), 'adj': (op.T, y, adj)}
    outs = {}
    for _ in range(4):                       # general path first, then the fast paths
        for name, (fn, arg, dsc) in calls.items():
            before = dsc.order
            outs.setdefault((name, before), []).append(fn(arg))
            assert dsc.order == (before if small else 1 - before)
    for name, (fn, arg, dsc) in calls.items():
        for order in (0, 1):
            dsc.order = order
            outs.setdefault((name, order), []).append(fn(arg))
        ref = outs[(name, 0)][0]
        assert all(tr.equal(ref, o) for k, v in outs.items() if k[0] == name for o in v)


@pytest.mark.parametrize('wd', [0.0, 0.01])
@pytest.mark.parametrize('c_neg', [None, 0.3])
def test_adam_matches_torch_fused(wd, c_neg, gpu):
    """sphrt_adam_neg_f64 (the retrieval loop's one-launch regulariser + Adam step) gives
    torch._fused_adam_'s parameters and moments bitwise over 20 steps of gradients spanning four
    decades, with and without weight decay; with the regulariser folded in, the same as
    sphrt_neg_reg_f64 on the gradient first (gradient and loss partials)."""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    n = 70001                                   # ragged: not a multiple of the workgroup
    gen = tr.Generator(device='cpu').manual_seed(3)
    p0 = tr.randn(n, generator=gen, dtype=tr.float64).to(gpu)
    pa, pb = p0.clone(), p0.clone()
    ma, va, mb, vb = (tr.zeros(n, dtype=tr.float64, device=gpu) for _ in range(4))
    steps = [tr.zeros((), dtype=tr.float32, device=gpu)]
    np_ = lib.sphrt_loss_partials(n)
    stream = _lib.stream_of(gpu)
    for it in range(20):
        g = tr.randn(n, generator=gen, dtype=tr.float64).to(gpu) * 10.0 ** (it % 4 - 2)
        ga = g.clone()
        part_a = tr.empty(np_, dtype=tr.float64, device=gpu)
        part_b = tr.full((np_,), float('nan'), dtype=tr.float64, device=gpu)
        if c_neg is not None:
            _lib.check(lib.sphrt_neg_reg_f64(_lib.ptr(pa), n, c_neg, _lib.ptr(ga),
                                             _lib.ptr(part_a), stream), 'neg_reg')
        tr._foreach_add_(steps, 1)
        tr._fused_adam_([pa], [ga], [ma], [va], [], steps, amsgrad=False, lr=0.01, beta1=0.9,
                        beta2=0.999, weight_decay=wd, eps=1e-8, maximize=False, grad_scale=None,
                        found_inf=None)
        _lib.check(lib.sphrt_adam_neg_f64(
            _lib.ptr(pb), _lib.ptr(g), _lib.ptr(mb), _lib.ptr(vb), n, 0.01, 0.9, 0.999, 1e-8, wd,
            float(it + 1), c_neg or 0.0, _lib.ptr(part_b if c_neg is not None else None), None,
            stream), 'adam_neg')
        assert tr.equal(pa, pb) and tr.equal(ma, mb) and tr.equal(va, vb), it
        if c_neg is not None:
            assert tr.equal(part_a, part_b), it


def test_gd_direct_brick_staged(gpu, monkeypatch):
    """The direct loop on a brick-staged (multi-wave) operator, where the Adam launch writes the
    next forward's staged density instead of the forward packing it: iterates and losses as the
    autograd loop's (bitwise / 1e-13), and the stage the loop leaves equals a fresh pack of the
    final coefficients."""
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    grid, geom = _orbit(64, (50, 100), kind='circ', grid_shape=(64, 64, 64))
    monkeypatch.setenv('SPHRT_BRICK', '4,2,4')        # (a 64^3 density is not staged by default)
    op = Operator(grid, geom, device=gpu)
    assert op._csr['desc'].stage_shape[0] > 0          # brick-staged
    x = tr.zeros(grid.shape, dtype=tr.float64, device=gpu)
    x[:, 32:, :32] = 1
    meas = op(x)
    made = []
    orig = Operator._stage_for_loop

    def spy(self, dtype):
        r = orig(self, dtype)
        made.append(r)
        return r

    monkeypatch.setattr(Operator, '_stage_for_loop', spy)
    runs = []
    for use_direct in (True, False):
        if not use_direct:
            monkeypatch.setattr(retrieval, '_direct_plan', lambda *a: None)
        fns = [SquareLoss(), NegRegularizer()]
        c, yh, hist = retrieval.gd(op, meas.clone(), FullyDenseModel(grid), lr=1e-1,
                                   num_iterations=6, loss_fns=fns, progress_bar=False)
        runs.append((c.detach().clone(), yh.detach().clone(), list(hist.values())))
    (ca, ya, ha), (cb, yb, hb) = runs
    assert len(made) == 1 and made[0] is not None
    for la, lb in zip(ha, hb):
        assert np.allclose(la, lb, rtol=1e-13, atol=0), (la, lb)
    assert tr.equal(ca, cb) and tr.equal(ya, yb)
    # the stage the direct loop left holds the coefficients it ended with (its last Adam launch)
    sd, buf = made[0]
    cols = tr.tensor([_stage_col(v, tuple(grid.shape), tuple(sd.stage_brick))
                      for v in range(0, x.numel(), 997)], device=gpu)
    staged = buf.view(tr.float64)[:sd.stage_cols]
    assert tr.equal(staged[cols], ca.reshape(-1)[::997])


@pytest.mark.parametrize('wd', [0.0, 0.01])
@pytest.mark.parametrize('c_neg', [None, 0.3])
@pytest.mark.parametrize('beta1', [0.9, 0.3])
def test_adam_matches_torch_foreach(wd, c_neg, beta1, gpu):
    """sphrt_adam_foreach_neg_f64 gives torch.optim.Adam's default GPU step (foreach=True, the
    multi-tensor path the reference's `optim(optim_vars)` takes on a ROCm tensor) bitwise over 20
    steps of gradients spanning four decades: parameters and both moments, with and without
    weight decay, both lerp forms (1 - beta1 below / above 0.5), the regulariser folded in as
    sphrt_neg_reg_f64 on the gradient first."""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    n = 70001
    gen = tr.Generator(device='cpu').manual_seed(4)
    p0 = tr.randn(n, generator=gen, dtype=tr.float64).to(gpu)
    pa, pb = p0.clone(), p0.clone()
    mb, vb = (tr.zeros(n, dtype=tr.float64, device=gpu) for _ in range(2))
    opt = tr.optim.Adam([pa], lr=0.01, betas=(beta1, 0.999), eps=1e-8, weight_decay=wd,
                        foreach=True)
    np_ = lib.sphrt_loss_partials(n)
    stream = _lib.stream_of(gpu)
    for it in range(20):
        g = tr.randn(n, generator=gen, dtype=tr.float64).to(gpu) * 10.0 ** (it % 4 - 2)
        ga = g.clone()
        part_a = tr.empty(np_, dtype=tr.float64, device=gpu)
        part_b = tr.full((np_,), float('nan'), dtype=tr.float64, device=gpu)
        if c_neg is not None:
            _lib.check(lib.sphrt_neg_reg_f64(_lib.ptr(pa), n, c_neg, _lib.ptr(ga),
                                             _lib.ptr(part_a), stream), 'neg_reg')
        pa.grad = ga
        opt.step()
        st = float(it + 1)
        _lib.check(lib.sphrt_adam_foreach_neg_f64(
            _lib.ptr(pb), _lib.ptr(g), _lib.ptr(mb), _lib.ptr(vb), n, (0.01 / (1 - beta1 ** st)) * -1,
            beta1, 0.999, 1e-8, wd, (1 - 0.999 ** st) ** 0.5, c_neg or 0.0,
            _lib.ptr(part_b if c_neg is not None else None), None, stream), 'adam_foreach')
        state = opt.state[pa]
        for name, a, b in (('param', pa, pb), ('exp_avg', state['exp_avg'], mb),
                           ('exp_avg_sq', state['exp_avg_sq'], vb)):
            if not tr.equal(a, b):
                k = int((a != b).nonzero()[0])
                pytest.fail(f'step {it}: {name} differs at {int((a != b).sum())} of {n} '
                            f'elements, first {k}: {a[k].item()!r} vs {b[k].item()!r}')
        if c_neg is not None:
            assert tr.equal(part_a, part_b), it


@pytest.mark.parametrize('optim_kw', [{}, {'fused': True}])
@pytest.mark.parametrize('lams, meas_dtype', [((1, 1), tr.float64), ((0.5, 2), tr.float64),
                                              ((1, None), tr.float32)])
def test_gd_direct_matches_autograd(lams, meas_dtype, optim_kw, gpu, monkeypatch):
    """The static_retrieval.py loop without autograd (retrieval._gd_direct: forward, residual,
    adjoint, -lam/N on negative voxels, Adam) gives the autograd loop's iterates bitwise: the
    same coefficients and reconstruction, for unit and non-unit weights, with and without the
    regulariser, and a float32 measurement.  Its loss values are the fused kernels' own
    deterministic means: equal to torch.mean's within 1e-13 relative."""
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    grid, geom = _orbit(12, (20, 16), kind='circ', grid_shape=(16, 16, 16))
    x = tr.zeros(grid.shape, dtype=tr.float64, device=gpu)
    x[:, 8:, :8] = 1
    x[:, :8, 8:] = 1
    op = Operator(grid, geom, device=gpu)
    meas = op(x).to(meas_dtype)
    calls = []
    direct = retrieval._gd_direct

    def spy(*a, **k):
        calls.append(1)
        return direct(*a, **k)

    monkeypatch.setattr(retrieval, '_gd_direct', spy)
    # (a wedge-ordered trace: the loop's forward writes f(d) in trace order)
    rows = []
    orig_rows = Operator._trace_position_rows
    monkeypatch.setattr(Operator, '_trace_position_rows',
                        lambda self, sd: rows.append(orig_rows(self, sd)) or rows[-1])
    runs = []
    for use_direct in (True, False):
        if not use_direct:
            monkeypatch.setattr(retrieval, '_direct_plan', lambda *a: None)
        fns = [lams[0] * SquareLoss()] + ([lams[1] * NegRegularizer()] if lams[1] else [])
        c, yh, hist = retrieval.gd(op, meas.clone(), FullyDenseModel(grid), lr=1e-1,
                                   num_iterations=25, loss_fns=fns, progress_bar=False, **optim_kw)
        runs.append((c.detach().clone(), yh.detach().clone(), list(hist.values())))
    assert len(calls) == 1
    assert len(rows) == 1 and rows[0] is not None
    (ca, ya, ha), (cb, yb, hb) = runs
    assert len(ha) == len(hb) and len(ha[0]) == 25 and ha[0][-1] < 0.3 * ha[0][0]
    for la, lb in zip(ha, hb):
        assert np.allclose(la, lb, rtol=1e-13, atol=0), (la, lb)
    assert tr.equal(ca, cb) and tr.equal(ya, yb)


@pytest.mark.parametrize('n', [1, 2, 7, 100001, 700000])
@pytest.mark.parametrize('ydt', [tr.float64, tr.float32])
@pytest.mark.parametrize('mode', ['in_order', 'order', 'unaligned'])
def test_sq_residual_kernel(n, ydt, mode, gpu):
    """sphrt_sq_residual_f64: r_scaled = (yhat - y) * scale elementwise as torch computes it
    (bitwise), through a ray map or in order (aligned or not, odd lengths), and workgroup partial
    sums of r * r within 1e-13 of torch's sum."""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    g = tr.Generator(device='cpu').manual_seed(n)
    yhat = tr.randn(n + 1, generator=g, dtype=tr.float64).to(gpu)
    y = tr.randn(n + 1, generator=g, dtype=tr.float64).to(ydt).to(gpu)
    order = None
    if mode == 'unaligned':
        yhat, y = yhat[1:], y[1:]
    else:
        yhat, y = yhat[:n], y[:n]
    if mode == 'order':
        order = tr.randperm(n, generator=g).to(tr.int32).to(gpu)
    scale = 0.37
    out = tr.empty(n, dtype=tr.float64, device=gpu)
    part = tr.full((lib.sphrt_loss_partials(n),), float('nan'), dtype=tr.float64, device=gpu)
    _lib.check(lib.sphrt_sq_residual_f64(_lib.ptr(yhat), _lib.ptr(y), int(ydt == tr.float64), n,
                                         scale, _lib.ptr(order), _lib.ptr(out), _lib.ptr(part),
                                         _lib.stream_of(gpu)), 'sq_residual')
    r = yhat - y.to(tr.float64)
    if order is not None:
        r = r[order.long()]
    assert tr.equal(out, r * scale)
    assert not tr.isnan(part).any()
    ref = float((r * r).sum())
    assert abs(float(part.sum()) - ref) <= 1e-13 * abs(ref)


@pytest.mark.parametrize('kind, dtype', [('circ', tr.float64), ('circ', tr.float32),
                                         ('rect', tr.float64)])
@pytest.mark.parametrize('runs', ['auto', 'on'])
def test_forward_in_trace_positions(kind, dtype, runs, gpu, monkeypatch):
    """A loop descriptor whose row lists name trace positions (_trace_position_rows, the direct
    gd loop's forward) writes the integral of trace position j to out[j]: bitwise op(x) gathered
    through the trace's ray map, empty rays included."""
    from sph_raytracer_amd import Operator
    monkeypatch.setenv('SPHRT_RUNS', runs)           # (on: run records in trace positions)
    grid, geom = _orbit(10, (20, 16), kind=kind, grid_shape=(16, 16, 16))
    op = Operator(grid, geom, device=gpu)
    if op._csr['ray_id'] is None:
        pytest.skip('natural trace order')
    x = tr.rand(grid.shape, dtype=dtype, device=gpu)
    ref = op(x).reshape(-1)
    sd = op._loop_descriptor(dtype)
    keep = op._trace_position_rows(sd)
    assert keep is not None and (sd.runs is None) == (keep[2] is None)
    out = tr.full_like(ref, float('nan'))
    op._forward_staged(x, out, sd)
    tr.cuda.synchronize()
    assert tr.equal(out, ref[op._ray_id_long()])


def test_gd_direct_declines_what_it_cannot_run(gpu, monkeypatch):
    """_direct_plan hands the autograd loop every call it does not cover exactly: a
    measurement with an extra leading singleton dimension (the reference's SquareLoss broadcasts
    it) runs and gives the same iterates as the exact-shape call; coefficients on another device
    than the operator's are declined too.  With two GPUs, a direct loop on an operator built on
    cuda:1 while cuda:0 is current equals the cuda:0 one."""
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    grid, geom = _orbit(6, (20, 16), kind='circ', grid_shape=(16, 16, 16))
    x = tr.zeros(grid.shape, dtype=tr.float64, device=gpu)
    x[:, 8:, :8] = 1
    op = Operator(grid, geom, device=gpu)
    meas = op(x)
    calls = []
    direct = retrieval._gd_direct

    def spy(*a, **k):
        calls.append(1)
        return direct(*a, **k)

    monkeypatch.setattr(retrieval, '_gd_direct', spy)
    fns = [SquareLoss(), NegRegularizer()]
    ca, _, ha = retrieval.gd(op, meas.clone(), FullyDenseModel(grid), lr=1e-1, num_iterations=8,
                             loss_fns=fns, progress_bar=False)
    assert len(calls) == 1
    cb, _, hb = retrieval.gd(op, meas.clone()[None], FullyDenseModel(grid), lr=1e-1,
                             num_iterations=8, loss_fns=fns, progress_bar=False)
    assert len(calls) == 1                     # the broadcasting call took the autograd loop
    assert tr.equal(ca, cb)
    for a, b in zip(ha.values(), hb.values()):
        assert np.allclose(a, b, rtol=1e-13, atol=0)
    cpu_coeffs = tr.ones(grid.shape, dtype=tr.float64, requires_grad=True)
    assert retrieval._direct_plan(op, meas, FullyDenseModel(grid), cpu_coeffs, fns,
                                  [cpu_coeffs]) is None
    if tr.cuda.device_count() < 2:
        pytest.skip('one GPU: the cross-device half needs two')
    dev1 = tr.device('cuda', 1)
    with tr.cuda.device(0):
        op1 = Operator(grid, geom, device=dev1)
        c1, _, h1 = retrieval.gd(op1, meas.to(dev1), FullyDenseModel(grid), lr=1e-1,
                                 num_iterations=8, loss_fns=fns, progress_bar=False)
    assert len(calls) == 2 and c1.device == dev1
    assert tr.equal(c1.cpu(), ca.cpu())


@pytest.mark.parametrize('case', ['c3_views', 'long_rows', 'c4_paired', 'c3_adjoint'])
def test_bucket_tables_equal_sorted_tables(case, gpu, monkeypatch):
    """The granule tables from the two-level bucket bitmaps (apply.hip bucket_table) equal the
    block radix sort's bit for bit — blocks, loc, every used table entry (SPHRT_TABLE_BUCKETS=0
    sorts every block): C3-like 20-bit keys (buckets, the 8-bit sort behind), long rows (blocks
    over 2048 segments: the 16-key kernel), C4-like time-paired tables (21-bit keys) and C3-like
    transposed tables (21-bit keys, many blocks past the bucket slots: the 10-bit sort)."""
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, Operator, SphericalGrid
    dynamic = case == 'c4_paired'
    if case in ('c3_views', 'c3_adjoint'):
        grid, geom = _orbit(6, (32, 64), grid_shape=(128, 128, 128))
    elif case == 'long_rows':
        grid = SphericalGrid(shape=(2500, 16, 16))
        geom = ConeRectGeom((6, 8), pos=(3, 0.01, 0.02), fov=(3, 3))
    else:
        th = tr.linspace(0, 2 * tr.pi, 36)      # 36 slices x 50^3: 2^20+ granules, 21-bit keys
        grid = SphericalGrid(shape=(36, 50, 50, 50))
        geom = sum(ConeCircGeom(shape=(20, 30), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(0, 45))
                   for a in th)

    def tables(flag):
        monkeypatch.setenv('SPHRT_TABLE_BUCKETS', flag)
        op = Operator(grid, geom, device=gpu, dynamic=dynamic)
        csr = op._csr
        if case == 'c3_adjoint':
            keep = op._transposed()['keep']
            blocks, loc, tab, stride = keep[6], keep[7], keep[8], op._transposed()['desc'].tab_stride
        elif case == 'c4_paired':
            op(tr.rand(grid.shape, dtype=tr.float32, device=gpu))
            pair = [v for k, v in csr.items() if isinstance(k, tuple) and k[0] == 'paired']
            assert pair and pair[0] is not None
            blocks, loc, tab = pair[0]['keep'][1:4]
            stride = pair[0]['desc'].tab_stride
        else:
            blocks, loc, tab, stride = csr['blocks'], csr['loc'], csr['tab'], csr['desc'].tab_stride
        n_seg = csr['total']
        bl = blocks.cpu().view(-1, 6)
        tab = tab.cpu()
        n_tab = bl[:, 5].tolist()
        used = tr.cat([tab[b * stride:b * stride + k] for b, k in enumerate(n_tab) if k > 0]
                      or [tab[:0]])
        keep = tr.zeros(n_seg, dtype=tr.bool)
        for b, k in enumerate(n_tab):
            if k >= 0:
                keep[int(bl[b, 2]):int(bl[b, 3])] = True
        return bl, used, loc[:n_seg].cpu()[keep]

    a, b = tables('1'), tables('0')
    for name, x, y in zip(('blocks', 'tab', 'loc'), a, b):
        assert tr.equal(x, y), name


@pytest.mark.parametrize('case', ['c3_views', 'long_rows', 'c2_views', 'tiny_grid'])
def test_staged_table_build_equals_compaction(case, gpu, monkeypatch):
    """The one-pass trace's staging moved into the CSR by the table build
    (sphrt_csr_local_build_staged) equals compacting it first (sphrt_trace_compact +
    sphrt_csr_index + sphrt_csr_local_build, SPHRT_TABLE_STAGED=0) bit for bit: row pointers,
    voxels with their head bits, float64 / float32 lengths, blocks, slots and tables; and the
    forwards agree.  long_rows: a radix-table volume (> 2^19 columns) whose rays of ~5000
    segments make blocks over 2048 segments (the big-block kernel) and over 4096 (no table);
    c2_views: bitmap tables, the rows in the bitmap's LDS; tiny_grid: a 4^3 grid whose bitmap LDS
    holds no row table (the rows read from global memory)."""
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    if case == 'c3_views':
        grid, geom = _orbit(6, (32, 64), grid_shape=(128, 128, 128))
    elif case == 'c2_views':
        grid, geom = _orbit(8, (50, 100), grid_shape=(50, 50, 50))
    elif case == 'tiny_grid':
        grid, geom = _orbit(8, (40, 60), grid_shape=(4, 4, 4))
    else:
        grid = SphericalGrid(shape=(2500, 16, 16))
        geom = ConeRectGeom((6, 8), pos=(3, 0.01, 0.02), fov=(3, 3))

    def build(flag):
        monkeypatch.setenv('SPHRT_TABLE_STAGED', flag)
        op = Operator(grid, geom, device=gpu)
        c = op._csr
        n_seg = c['total']
        arrs = {k: c[k][:n_seg].cpu() for k in ('vox', 'len', 'len32', 'loc')}
        arrs.update(row_ptr=c['row_ptr'].cpu(), blocks=c['blocks'].cpu())
        # the tables' used entries (each block's first n_tab at its stride; the rest is padding)
        stride, tab = c['desc'].tab_stride, c['tab'].cpu()
        n_tab = arrs['blocks'].view(-1, 6)[:, 5].tolist()
        arrs['tab'] = tr.cat([tab[b * stride:b * stride + k] for b, k in enumerate(n_tab)
                              if k > 0] or [tab[:0]])
        # slots exist only in blocks with a table (the others gather per segment)
        bl = arrs['blocks'].view(-1, 6)
        keep = tr.zeros(n_seg, dtype=tr.bool)
        for b, k in enumerate(n_tab):
            if k >= 0:
                keep[int(bl[b, 2]):int(bl[b, 3])] = True
        arrs['loc'] = arrs['loc'][keep]
        return op, arrs

    op1, a1 = build('1')
    op0, a0 = build('0')
    for k in a0:
        assert tr.equal(a1[k], a0[k]), k
    if case == 'long_rows':
        blocks = a1['blocks'].numpy().reshape(-1, 6)
        n = blocks[:, 3] - blocks[:, 2]
        assert (n > 2048).any() and (n > 4096).any()
    x = tr.rand(grid.shape, dtype=tr.float32, device=gpu)
    assert tr.equal(op1(x), op0(x))
    assert tr.equal(op1(x.double()), op0(x.double()))


def test_transposed_brick_rows_equal_linear_rows(gpu, monkeypatch):
    """The static transposed CSR's rows in voxel-brick order (_voxel_rows, multi-wave grids) give
    the adjoint of the linear voxel order (SPHRT_TROWS=off) up to summation order — every voxel
    keeps its segments in the same order, but a row's place in its workgroup decides how the
    segmented scan associates its sums (float64 within 1e-13, float32 within 1e-6 relative) — and
    stay deterministic; the rows report their voxel through the index's row ids."""
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(40, (64, 64), kind='circ', grid_shape=(64, 64, 64))
    outs = {}
    for mode in ('auto', 'off', 'auto'):
        monkeypatch.setenv('SPHRT_TROWS', mode)
        op = Operator(grid, geom, device=gpu)
        assert op._csr['nblocks'] > 256 * 6, 'a multi-wave grid'
        g = tr.Generator(device=gpu).manual_seed(3)
        res = []
        for dt in (tr.float32, tr.float64):
            x = tr.rand(grid.shape, dtype=dt, device=gpu, generator=g).requires_grad_(True)
            y = tr.rand(geom.shape, dtype=dt, device=gpu, generator=g)
            (op(x) * y).sum().backward()
            res += [x.grad, op.T(y)]
        if mode in outs:                  # deterministic: the same bits on a fresh Operator
            for a, b in zip(res, outs[mode]):
                assert tr.equal(a, b)
        outs[mode] = res
        rows = op._transposed()['keep'][4][:200]   # the voxels the first rows report:
        assert bool((rows[1:] > rows[:-1]).all()) == (mode == 'off')   # ascending iff linear
    for a, b in zip(outs['auto'], outs['off']):
        tol = 1e-13 if a.dtype == tr.float64 else 1e-6
        assert float((a - b).abs().max()) <= tol * float(b.abs().max()), a.dtype
