"""The native Operator construction (csrc/construct.cpp, _sphrt_fast.build_cone for cone-beam
detectors, build_rays for any other geometry) against the Python construction sequence it
replaces (raytracer.Operator._trace_on).

CPU: the host values the trace reads — detector frames and pixel coordinates (_ConeRays.of), ray
starts and their start voxels (_RayBatch.host_starts), the plan's trigonometric tables (_Plan) —
are bit-identical to the Python path's, and geometries outside the native sequence are declined
(None, nothing done).  GPU: Operators built natively and with SPHRT_CONSTRUCT=python hold the
same CSR, tables, run records and ray ids, and give bit-identical forwards and adjoints.
"""
import math

import numpy as np
import pytest
import torch

from sph_raytracer_amd import (ConeCircGeom, ConeRectGeom, Operator, ParallelGeom, SphericalGrid,
                               ViewGeom, _lib)
from sph_raytracer_amd import raytracer as R


def _fast():
    fc = _lib.load_construct()
    if fc is None:
        pytest.fail('_sphrt_fast.so (csrc/fastpath.cpp + construct.cpp) is not built')
    return fc


def _orbit(kind, n_views, det, radius=5.0, z=1.0, **kw):
    th = torch.linspace(0, 2 * torch.pi, n_views + 1)[:n_views]
    cls = ConeRectGeom if kind == 'rect' else ConeCircGeom
    return sum(cls(det, pos=(radius * torch.cos(t), radius * torch.sin(t), z), **kw) for t in th)


def _cases():
    g50 = SphericalGrid(shape=(50, 50, 50))
    g_dyn = SphericalGrid(shape=(6, 20, 24, 28))
    g_log = SphericalGrid(shape=(12, 10, 16), size_r=(0.1, 3), spacing='log')
    return {
        'rect_orbit': (g50, _orbit('rect', 12, (20, 30), fov=(45, 45))),
        'circ_orbit': (g50, _orbit('circ', 9, (16, 24), fov=(0, 45))),
        'circ_orbit_log': (g_log, _orbit('circ', 5, (8, 12), fov=(5, 40), spacing='log')),
        'rect_single': (g50, ConeRectGeom((24, 16), pos=(3, 1, 0.5), fov=(30, 20))),
        'circ_single': (g50, ConeCircGeom((10, 14), pos=(-2, 2, 1))),
        'rect_one_row': (g50, ConeRectGeom((1, 17), pos=(4, 0, 0))),       # a zero span
        'rect_dynamic': (g_dyn, _orbit('rect', 6, (12, 10))),
        # starts on boundaries: r = 1 (the outer sphere), the +Z axis, the -X half-plane
        'starts_on_bounds': (g50, ConeRectGeom((5, 6), pos=(1, 0, 0)) + ConeRectGeom(
            (5, 6), pos=(0, 0, 0.5)) + ConeRectGeom((5, 6), pos=(-0.5, 0, 0))),
    }


CASES = _cases()


def _bits(t):
    t = t.contiguous()
    return t.view(torch.int64) if t.dtype == torch.float64 else t.view(torch.int32)


@pytest.mark.parametrize('name', sorted(CASES))
def test_cone_host_values_match_python(name):
    grid, geom = CASES[name]
    fc = _fast()
    res = fc.cone_host(geom, grid.r_b, grid.e_b, grid.a_b, grid.shape.r, grid.shape.e,
                       grid.shape.a)
    assert res is not None, name
    circ, frame, row, col, xs, st, tables = res
    cone = R._ConeRays.of(geom)
    assert cone is not None and circ == cone.circ
    blob = torch.cat([frame.reshape(-1), row.reshape(-1), col.reshape(-1)])
    assert torch.equal(_bits(blob), _bits(cone.host))
    xs_h, st_h = R._RayBatch.host_starts(grid, geom.ray_starts)
    assert xs.shape == xs_h.shape and torch.equal(_bits(xs), _bits(xs_h))
    assert torch.equal(st, st_h)
    plan = R._Plan(grid, 'cpu', staging=R._Staging())
    assert torch.equal(tables, plan._host)


def test_start_voxels_on_boundaries():
    """The boundary rules of find_starts (raytracer.py:605-644): a start on the outer sphere is in
    the last shell, one past it in none (-1)."""
    grid = SphericalGrid(shape=(4, 6, 8))
    geom = ConeRectGeom((2, 2), pos=(1, 0, 0)) + ConeRectGeom((2, 2), pos=(2, 0, 0)) + \
        ConeRectGeom((2, 2), pos=(0.3, 0.2, -0.1))
    res = _fast().cone_host(geom, grid.r_b, grid.e_b, grid.a_b, 4, 6, 8)
    st = res[5].reshape(-1, 4)
    assert st[0, 0] == 3 and st[1, 0] == -1
    assert torch.equal(st[:, :3].T.to(torch.int64),
                       R.find_starts(grid, res[4]).reshape(3, -1))


def test_cone_host_declines_other_geometries():
    fc = _fast()
    grid = SphericalGrid(shape=(8, 8, 8))
    args = (grid.r_b, grid.e_b, grid.a_b, 8, 8, 8)
    assert fc.cone_host(ParallelGeom((4, 4), pos=(3, 0, 0)), *args) is None
    mixed = ConeRectGeom((4, 4), pos=(3, 0, 0)) + ConeCircGeom((4, 4), pos=(0, 3, 0))
    assert fc.cone_host(mixed, *args) is None
    fovs = ConeRectGeom((4, 4), pos=(3, 0, 0)) + ConeRectGeom((4, 4), pos=(0, 3, 0), fov=(30, 30))
    assert fc.cone_host(fovs, *args) is None           # views that differ: per-view specs
    far = ConeRectGeom((4, 4), pos=(3, 0, 0)) + ConeRectGeom((4, 4), pos=(0, 3, 0))
    far.geoms[1].pos = torch.tensor([math.inf, 0.0, 0.0], dtype=torch.float64)
    assert fc.cone_host(far, *args) is None            # non-finite start: find_starts
    unsorted = SphericalGrid(r_b=[0, 2, 1, 3], e_b=[0, 1, 2, 3], a_b=[-3, 0, 3])
    assert fc.cone_host(ConeRectGeom((4, 4), pos=(3, 0, 0)), unsorted.r_b, unsorted.e_b,
                        unsorted.a_b, 3, 3, 2) is None


# ---- GPU: the whole construction -------------------------------------------------------------

def _build(grid, geom, dev, monkeypatch, native):
    if native:
        monkeypatch.delenv('SPHRT_CONSTRUCT', raising=False)
    else:
        monkeypatch.setenv('SPHRT_CONSTRUCT', 'python')
    op = Operator(grid, geom, device=dev)
    assert isinstance(op._batch, R._NativeBatch) == native
    return op


GPU_CASES = {
    'c2_like': lambda: (SphericalGrid(shape=(50, 50, 50)), _orbit('rect', 50, (50, 100))),
    'c5_like_wedges': lambda: (SphericalGrid(shape=(64, 64, 64)),
                               _orbit('circ', 64, (100, 50), fov=(0, 45))),
    'c4_like_dynamic': lambda: (SphericalGrid(shape=(50, 50, 50, 50)),
                                _orbit('circ', 50, (100, 50), fov=(0, 45))),
    'multi_wave_runs_brick': lambda: (SphericalGrid(shape=(96, 96, 96)),
                                      _orbit('rect', 40, (128, 128))),
    'single_view': lambda: (SphericalGrid(shape=(30, 40, 50)),
                            ConeRectGeom((64, 48), pos=(3, 1, 0.5), fov=(40, 30))),
    # view tiles (9, 1): an odd view count and an odd detector width
    'odd_tiles': lambda: (SphericalGrid(shape=(24, 20, 28)), _orbit('rect', 9, (17, 41))),
    'few_views': lambda: (SphericalGrid(shape=(24, 20, 28)), _orbit('circ', 7, (20, 30))),
    # build_rays: any other geometry from its host starts and directions (geometry order)
    'parallel_orbit': lambda: (SphericalGrid(shape=(40, 30, 36)), _parallel_orbit(6, (32, 24))),
    'parallel_single': lambda: (SphericalGrid(shape=(20, 18, 22)),
                                ParallelGeom((40, 30), pos=(2, 1.5, 0.4), size=(1.5, 1.2))),
    'viewgeom_rays': lambda: (SphericalGrid(shape=(30, 24, 40)), _random_viewgeom(3, (24, 33))),
    'parallel_dynamic': lambda: (SphericalGrid(shape=(5, 16, 18, 20)), _parallel_orbit(5, (20, 16))),
}


def _parallel_orbit(n_views, det):
    th = torch.linspace(0, 2 * torch.pi, n_views + 1)[:n_views]
    return sum(ParallelGeom(det, pos=(3 * torch.cos(t), 3 * torch.sin(t), 0.3), size=(2, 1.6))
               for t in th)


def _random_viewgeom(n_views, det):
    """Arbitrary ViewGeoms: per-pixel starts on a sphere of radius 2.5 and directions towards
    jittered points of the unit ball."""
    g = torch.Generator().manual_seed(11)
    views = []
    for _ in range(n_views):
        d = torch.randn(det + (3,), generator=g, dtype=torch.float64)
        xs = 2.5 * d / torch.linalg.norm(d, dim=-1, keepdim=True)
        aim = 0.8 * torch.rand(det + (3,), generator=g, dtype=torch.float64) - 0.4
        views.append(ViewGeom(xs, aim - xs))
    return sum(views)


@pytest.mark.gpu
@pytest.mark.parametrize('name', sorted(GPU_CASES))
def test_native_construction_matches_python(gpu, monkeypatch, name):
    grid, geom = GPU_CASES[name]()
    a = _build(grid, geom, gpu, monkeypatch, native=True)
    b = _build(grid, geom, gpu, monkeypatch, native=False)
    ca, cb = a._csr, b._csr
    assert a._ray_shape == b._ray_shape
    for k in ('n', 'total', 'nblocks'):
        assert ca[k] == cb[k], k
    da, db = ca['desc'], cb['desc']
    for f in ('n_rays', 'n_segments', 'n_blocks', 'n_cols', 'n_fallback', 'tab_stride',
              'tab_bytes', 'stage_cols', 'order'):
        assert getattr(da, f) == getattr(db, f), f
    assert list(da.stage_shape) == list(db.stage_shape)
    assert list(da.stage_brick) == list(db.stage_brick)
    assert (da.runs is None) == (db.runs is None)
    total, n = ca['total'], ca['n']
    # rows with segments (row_ray) and without (empty_ray): blocks[b, 1] ends b's empty rays
    n_empty = int(ca['blocks'].view(-1, 6)[:, 1].max())
    assert n_empty == int((ca['row_ptr'][1:] == ca['row_ptr'][:-1]).sum())
    for k, m in (('row_ptr', n + 1), ('vox', total), ('len32', total), ('loc', total),
                 ('row_ray', n - n_empty), ('empty_ray', n_empty), ('blocks', None)):
        x, y = ca[k], cb[k]
        if m is not None:
            x, y = x[:m], y[:m]
        assert torch.equal(x.view(torch.uint8) if x.dtype.is_floating_point else x,
                           y.view(torch.uint8) if y.dtype.is_floating_point else y), k
    # each block's n_tab granules (blocks[b, 5]; the rest of its stride is never read)
    nb, stride = ca['nblocks'], da.tab_stride
    n_tab = ca['blocks'].view(nb, 6)[:, 5]
    valid = torch.arange(stride, device=gpu)[None, :] < n_tab[:, None]
    ta, tb = ca['tab'][:nb * stride].view(nb, stride), cb['tab'][:nb * stride].view(nb, stride)
    assert int(valid.sum()) > 0 and torch.equal(ta[valid], tb[valid])
    if ca['runs'] is not None:   # counts, then the row runs and empty ranges each block uses
        ra, rb = ca['runs'].view(nb, 32), cb['runs'].view(nb, 32)
        assert torch.equal(ra[:, :2], rb[:, :2])
        col = torch.arange(32, device=gpu)[None, :]
        used = ((col >= 2) & (col < 2 + 2 * ra[:, :1])) | ((col >= 16) & (col < 16 + 2 * ra[:, 1:2]))
        assert torch.equal(ra[used], rb[used])
    assert (ca['ray_id'] is None) == (cb['ray_id'] is None)
    if ca['ray_id'] is not None:
        assert torch.equal(ca['ray_id'], cb['ray_id'])
    # the float64 lengths moved out of the staging on first use
    assert torch.equal(ca['len'][:total].view(torch.int64), cb['len'][:total].view(torch.int64))
    g = torch.Generator(device='cpu').manual_seed(5)
    for dt in (torch.float32, torch.float64):
        x = torch.rand(tuple(grid.shape), generator=g, dtype=dt).to(gpu)
        ya, yb = a(x), b(x)
        assert torch.equal(ya, yb), dt
        xa = x.clone().requires_grad_(True)
        xb = x.clone().requires_grad_(True)
        (a(xa) ** 2).sum().backward()
        (b(xb) ** 2).sum().backward()
        assert torch.equal(xa.grad, xb.grad), dt


@pytest.mark.gpu
def test_native_construction_is_the_default(gpu, monkeypatch):
    """float64 traces construct natively unless a construction switch is set: cone detectors
    (build_cone) and every other geometry (build_rays); the reference-mode trace does not."""
    monkeypatch.delenv('SPHRT_CONSTRUCT', raising=False)
    grid = SphericalGrid(shape=(10, 12, 14))
    geom = _orbit('rect', 3, (8, 9))
    assert isinstance(Operator(grid, geom, device=gpu)._batch, R._NativeBatch)
    monkeypatch.setenv('SPHRT_TRACE', 'twopass')
    assert not isinstance(Operator(grid, geom, device=gpu)._batch, R._NativeBatch)
    monkeypatch.delenv('SPHRT_TRACE')
    assert not isinstance(Operator(grid, geom, device=gpu, ftype=torch.float32)._batch,
                          R._NativeBatch)
    assert isinstance(Operator(grid, ParallelGeom((4, 4), pos=(3, 0, 0)), device=gpu)._batch,
                      R._NativeBatch)
    xs = torch.tensor([[2.0, 0.1, 0.2], [0.0, -2.0, 0.3]], dtype=torch.float64)
    assert isinstance(Operator(grid, ViewGeom(xs, -xs), device=gpu)._batch, R._NativeBatch)


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['rect', 'circ'])
def test_view_tiles_match_geometry_order(gpu, monkeypatch, kind):
    """Orbits are traced in view tiles (raytracer._view_tiles): every ray's segments equal those
    of the geometry-order trace (SPHRT_RAY_ORDER=natural) bit for bit, and the forward and adjoint
    agree up to summation order (float64 1e-13, float32 1e-6 relative)."""
    grid = SphericalGrid(shape=(40, 36, 44))
    geom = _orbit(kind, 24, (30, 40), fov=(45, 45) if kind == 'rect' else (0, 45))
    assert R._view_tiles(tuple(geom.shape), False) == (24, 2)
    monkeypatch.delenv('SPHRT_RAY_ORDER', raising=False)
    a = Operator(grid, geom, device=gpu)
    assert isinstance(a._batch, R._NativeBatch) and a._csr['ray_id'] is not None
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'natural')
    b = Operator(grid, geom, device=gpu)
    assert b._csr['ray_id'] is None and a._ray_shape == b._ray_shape == tuple(geom.shape)

    def per_ray(op):          # (ray -> (voxels, length bits)) in geometry order
        c = op._csr
        n = c['n']
        ptr = c['row_ptr'].cpu()
        vox = (c['vox'][:c['total']] & 0x7fffffff).cpu()
        ln = c['len'][:c['total']].cpu().view(torch.int64)
        rid = c['ray_id'].cpu().long() if c['ray_id'] is not None else torch.arange(n)
        order = torch.argsort(rid)
        cnt = (ptr[1:] - ptr[:-1])[order]
        starts = ptr[:-1][order]
        idx = torch.repeat_interleave(starts - (torch.cumsum(cnt, 0) - cnt), cnt) + \
            torch.arange(int(cnt.sum()))
        return cnt, vox[idx], ln[idx]

    for x, y in zip(per_ray(a), per_ray(b)):
        assert torch.equal(x, y)
    g = torch.Generator(device='cpu').manual_seed(2)
    for dt, tol in ((torch.float64, 1e-13), (torch.float32, 1e-6)):
        x = torch.rand(tuple(grid.shape), generator=g, dtype=dt).to(gpu)
        y = torch.rand(tuple(geom.shape), generator=g, dtype=dt).to(gpu)
        fa, fb = a(x), b(x)
        assert float((fa - fb).abs().max()) <= tol * float(fb.abs().max())
        ta, tb = a.T(y), b.T(y)
        assert float((ta - tb).abs().max()) <= tol * float(tb.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['rect', 'circ'])
def test_transposed_columns_geometry_or_trace_order(gpu, monkeypatch, kind):
    """A reordered trace's transposed CSR takes its columns in geometry order (ConeRect orbits:
    y read as given, brick-staged) or in trace-row order (ConeCirc: y gathered per call); either
    choice (SPHRT_TCOLS=geom / trace) gives the same adjoint up to summation order, through the
    general and the steady-state paths, float64 and float32."""
    grid = SphericalGrid(shape=(40, 36, 44))
    geom = _orbit(kind, 16, (30, 40), fov=(45, 45) if kind == 'rect' else (0, 45))
    g = torch.Generator(device='cpu').manual_seed(4)
    ys = [torch.rand(tuple(geom.shape), generator=g, dtype=dt).to(gpu)
          for dt in (torch.float64, torch.float32)]
    out = {}
    for mode in ('auto', 'geom', 'trace'):
        monkeypatch.setenv('SPHRT_TCOLS', mode)
        op = Operator(grid, geom, device=gpu)
        assert op._csr['ray_id'] is not None
        want_geom = mode == 'geom' or (mode == 'auto' and kind == 'rect')
        assert op._tcols_geom() == want_geom
        res = []
        for y in ys:
            a0, a1 = op.T(y), op.T(y)            # general path (binds), steady-state path
            assert torch.equal(a0, a1)
            res.append(a0)
        out[mode] = res
    for mode in ('geom', 'trace'):
        for a, b in zip(out[mode], out['auto']):
            tol = 1e-13 if a.dtype == torch.float64 else 1e-6
            assert float((a - b).abs().max()) <= tol * float(b.abs().max())
