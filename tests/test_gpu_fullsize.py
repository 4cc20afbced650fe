"""Parity at the full BASELINE sizes of C2, C3, C4 and C5, every ray against the C
oracle.

C3: (128,128,128) grid, 128-view orbit x ConeRect (128,256) = 4.19 M rays, ~115 M segments —
the production path of the HBM roofline run: the multi-wave forward with (4,2,4) brick staging,
run records and the alternating block order, its 32-bit-free (uint16) granule tables, and the
transposed adjoint.  C4: dynamic (50,50,50,50) grid, 50-view orbit x ConeCirc (100,50), view i
<-> time slice i: the time-paired CSR over 6.25 M columns (int32 granule tables, one contiguous
block range per XCD) and its transposed adjoint (the gradient).

The oracle traces every ray on the host (16 threads over view chunks; ~3 s at C3), so these are
whole-config comparisons, not samples: per ray the canonical voxel sequence exactly and lengths
within 1e-12 (golden_cases.compare_segments), line integrals within 1e-10 relative (float64) and
1e-5 (float32), the adjoint / gradient volume within 1e-10 (float64) and 1e-5 (float32) of its
largest magnitude.
"""
import math
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch as tr

import golden_cases as gc

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = 16      # the GPU box's CPU share


def _orbit(n_views, det, kind, grid_shape):
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, SphericalGrid
    grid = SphericalGrid(shape=grid_shape)
    geoms = []
    for th in tr.linspace(0, 2 * tr.pi, n_views):
        pos = (5 * tr.cos(th), 5 * tr.sin(th), 1)
        geoms.append(ConeRectGeom(det, pos=pos, fov=(45, 45)) if kind == 'rect'
                     else ConeCircGeom(shape=det, pos=pos, fov=(0, 45)))
    return grid, sum(geoms)


def _oracle_trace(grid, geom):
    """Every ray of `geom` through the C oracle (IEEE sqrt), one view per task -> per view
    (ptr, vox, seg)."""
    from oracle import oracle
    from sph_raytracer_amd.raytracer import find_starts
    oracle.use_mkl_sqrt(False)
    shp = tuple(grid.shape)[-3:]
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    rays = geom.rays.numpy()
    xs = np.broadcast_to(geom.ray_starts.numpy(), rays.shape)
    n_views = rays.shape[0]

    def one(v):
        x = np.ascontiguousarray(xs[v].reshape(-1, 3))
        d = np.ascontiguousarray(rays[v].reshape(-1, 3))
        st = find_starts(grid, tr.from_numpy(x)).numpy()
        return oracle.trace_segments(g, x, d, st)

    oracle.load()
    with ThreadPoolExecutor(THREADS) as pool:
        views = list(pool.map(one, range(n_views)))
    assert all(len(p) - 1 == math.prod(rays.shape[1:-1]) for p, _, _ in views)
    return views, math.prod(shp)


def _gpu_views(op, n_views):
    """The GPU trace split per view (geometry order) on the host."""
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    per = (len(ptr) - 1) // n_views
    out = []
    for v in range(n_views):
        p = ptr[v * per:(v + 1) * per + 1]
        a, b = p[0], p[-1]
        out.append((p - a, vox[a:b], seg[a:b]))
    return out


def _compare_all(ref_views, got_views, scale, what):
    for v, (r, g) in enumerate(zip(ref_views, got_views)):
        msg = gc.compare_segments(r, g, scale, f'{what} view {v}')
        assert msg is None, msg


def _flat(views):
    ptrs, voxs, segs, base = [], [], [], 0
    for p, v, s in views:
        ptrs.append(p[:-1] + base)
        voxs.append(v)
        segs.append(s)
        base += p[-1]
    ptr = np.concatenate(ptrs + [np.array([base])])
    return ptr, np.concatenate(voxs), np.concatenate(segs)


@pytest.fixture(scope='module')
def c3(gpu):
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(128, (128, 256), 'rect', (128, 128, 128))
    op = Operator(grid, geom, device=gpu)
    ref, n_vox = _oracle_trace(grid, geom)
    return grid, geom, op, ref, n_vox


def test_c3_full_trace_vs_oracle(c3):
    """All 4.19 M C3 rays: voxel sequences exact, lengths 1e-12 (the production trace path)."""
    grid, geom, op, ref, _ = c3
    assert op._csr['n'] == 128 * 128 * 256 and op._csr['total'] > 100_000_000
    _compare_all(ref, _gpu_views(op, 128), 5.1, 'C3')


def test_c3_full_forward_and_adjoint_vs_oracle(c3, gpu):
    """C3 forward (float64, float32) and transposed adjoint (float64, float32) over every ray /
    voxel against the oracle's segments, through the product configuration: the orbit traced in
    view tiles, (4,2,4) brick staging, alternating block order (each call below flips it), the
    transposed rows in voxel bricks (its y in trace order: the views interleaved already)."""
    grid, geom, op, ref, n_vox = c3
    desc = op._csr['desc']
    assert tuple(desc.stage_brick) == (4, 2, 4) and desc.n_blocks > 256 * 6
    assert op._csr['ray_id'] is not None
    ptr, vox, seg = _flat(ref)
    ray = np.repeat(np.arange(len(ptr) - 1), np.diff(ptr))
    g = tr.Generator().manual_seed(11)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g)
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, generator=g)
    want = np.bincount(ray, x.numpy().reshape(-1)[vox] * seg, minlength=len(ptr) - 1)
    for dt, tol in ((tr.float64, gc.F64_RTOL), (tr.float32, gc.F32_RTOL)):
        for _ in range(2):                         # both block orders
            got = op(x.to(gpu, dt)).cpu().numpy().reshape(-1)
            err = gc.rel_close(got, want, tol)
            assert err <= tol, f'C3 forward {dt} rel err {err:.3g}'
    want_t = np.bincount(vox, y.numpy().reshape(-1)[ray] * seg, minlength=n_vox)
    scale = np.abs(want_t).max()
    for dt, tol in ((tr.float64, 1e-10), (tr.float32, 1e-5)):
        for _ in range(2):
            got = op.T(y.to(gpu, dt)).cpu().numpy().reshape(-1)
            err = float(np.abs(got - want_t).max() / scale)
            assert err <= tol, f'C3 adjoint {dt} rel err {err:.3g}'


@pytest.fixture(scope='module')
def c4(gpu):
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(50, (100, 50), 'circ', (50, 50, 50, 50))
    op = Operator(grid, geom, device=gpu, dynamic=True)
    ref, n_vox = _oracle_trace(grid, geom)
    return grid, geom, op, ref, n_vox


def test_c4_full_trace_vs_oracle(c4):
    """All 250 k C4 rays (ConeCirc wedge trace order, reordered to geometry order)."""
    grid, geom, op, ref, _ = c4
    assert op._csr['ray_id'] is not None
    _compare_all(ref, _gpu_views(op, 50), 5.1, 'C4')


def test_c4_full_forward_and_gradient_vs_oracle(c4, gpu):
    """C4 dynamic forward (view i reads time slice i) and its gradient (autograd: the transposed
    time-paired CSR), float64 and float32, against the oracle; the time-paired CSR spans 6.25 M
    columns, so its granule tables are int32."""
    grid, geom, op, ref, n_vox = c4
    ptr, vox, seg = _flat(ref)
    n = len(ptr) - 1
    per_view = n // 50
    ray = np.repeat(np.arange(n), np.diff(ptr))
    t_of = ray // per_view
    g = tr.Generator().manual_seed(12)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g)
    # the C4 density pattern plus noise, so every slice differs
    x[:, :, 25:, :25] += 1
    for t in range(50):
        x[t, :, (2 * t) % 50, :] += 1
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, generator=g)
    col = t_of * n_vox + vox
    want = np.bincount(ray, x.numpy().reshape(-1)[col] * seg, minlength=n)
    want_g = np.bincount(col, y.numpy().reshape(-1)[ray] * seg, minlength=50 * n_vox)
    scale = np.abs(want_g).max()
    for dt, tol, gtol in ((tr.float64, gc.F64_RTOL, 1e-10), (tr.float32, gc.F32_RTOL, 1e-5)):
        for _ in range(2):
            xd = x.to(gpu, dt).requires_grad_()
            out = op(xd)
            assert tuple(out.shape) == (50, 100, 50)
            err = gc.rel_close(out.detach().cpu().numpy().reshape(-1), want, tol)
            assert err <= tol, f'C4 forward {dt} rel err {err:.3g}'
            (out * y.to(gpu, dt)).sum().backward()
            err = float(np.abs(xd.grad.cpu().numpy().reshape(-1) - want_g).max() / scale)
            assert err <= gtol, f'C4 gradient {dt} rel err {err:.3g}'
    rec = op._paired(50, per_view)
    assert rec is not None and rec['desc'].n_cols == 50 * n_vox and rec['desc'].tab_bytes == 4
    assert rec['desc'].order & 2          # one contiguous block range per XCD


def _static_forward_adjoint(grid, geom, op, ref, n_vox, gpu, seed, what):
    """Static forward (float64, float32) and adjoint op.T (float64, float32) of every ray /
    voxel against the oracle's segments; each call is made three times (the general path, then
    the steady-state bindings: the C++ fast path and T's transposed-CSR binding)."""
    ptr, vox, seg = _flat(ref)
    ray = np.repeat(np.arange(len(ptr) - 1), np.diff(ptr))
    g = tr.Generator().manual_seed(seed)
    x = tr.rand(grid.shape, dtype=tr.float64, generator=g)
    y = tr.rand(tuple(geom.shape), dtype=tr.float64, generator=g)
    want = np.bincount(ray, x.numpy().reshape(-1)[vox] * seg, minlength=len(ptr) - 1)
    for dt, tol in ((tr.float64, gc.F64_RTOL), (tr.float32, gc.F32_RTOL)):
        xd = x.to(gpu, dt)
        for _ in range(3):
            got = op(xd).cpu().numpy().reshape(-1)
            err = gc.rel_close(got, want, tol)
            assert err <= tol, f'{what} forward {dt} rel err {err:.3g}'
    want_t = np.bincount(vox, y.numpy().reshape(-1)[ray] * seg, minlength=n_vox)
    scale = np.abs(want_t).max()
    for dt, tol in ((tr.float64, 1e-10), (tr.float32, 1e-5)):
        yd = y.to(gpu, dt)
        for _ in range(3):
            got = op.T(yd).cpu().numpy().reshape(-1)
            err = float(np.abs(got - want_t).max() / scale)
            assert err <= tol, f'{what} adjoint {dt} rel err {err:.3g}'


@pytest.fixture(scope='module')
def c2(gpu):
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(50, (50, 100), 'rect', (50, 50, 50))
    op = Operator(grid, geom, device=gpu)
    ref, n_vox = _oracle_trace(grid, geom)
    return grid, geom, op, ref, n_vox


def test_c2_full_trace_vs_oracle(c2):
    """All 250 k rays of the headline config (BASELINE configs[1]): voxel sequences exact,
    lengths 1e-12 — the one-wave path (bitmap granule tables, no brick staging)."""
    grid, geom, op, ref, _ = c2
    assert op._csr['n'] == 50 * 50 * 100 and op._csr['ray_id'] is not None   # (view tiles)
    _compare_all(ref, _gpu_views(op, 50), 5.1, 'C2')


def test_c2_full_forward_and_adjoint_vs_oracle(c2, gpu):
    """C2 forward and adjoint over every ray / voxel, general and steady-state paths."""
    grid, geom, op, ref, n_vox = c2
    assert op._csr['desc'].stage_brick[0] == 0      # one resident wave: natural layout
    _static_forward_adjoint(grid, geom, op, ref, n_vox, gpu, 21, 'C2')


@pytest.fixture(scope='module')
def c5(gpu):
    from sph_raytracer_amd import Operator
    grid, geom = _orbit(64, (100, 50), 'circ', (64, 64, 64))
    op = Operator(grid, geom, device=gpu)
    ref, n_vox = _oracle_trace(grid, geom)
    return grid, geom, op, ref, n_vox


def test_c5_full_trace_vs_oracle(c5):
    """All 320 k rays of the retrieval config (BASELINE configs[4]): the ConeCirc wedge trace
    order (rays generated in trace order on the device), ~2 k exact-path tie rays per trace
    (ring 0 passes through the origin), reordered to geometry order."""
    grid, geom, op, ref, _ = c5
    assert op._csr['n'] == 64 * 100 * 50 and op._csr['ray_id'] is not None
    _compare_all(ref, _gpu_views(op, 64), 5.1, 'C5')


def test_c5_full_forward_and_adjoint_vs_oracle(c5, gpu):
    """C5 forward (float64 half tables, view tiles, alternating block order; no brick staging:
    the 64^3 density fits one XCD's L2) and adjoint (the transposed CSR of a trace-ordered CSR)
    over every ray / voxel."""
    grid, geom, op, ref, n_vox = c5
    desc = op._csr['desc']
    assert tuple(desc.stage_brick) == (0, 0, 0) and desc.n_blocks > 256 * 6
    assert op._csr['ray_id'] is not None
    _static_forward_adjoint(grid, geom, op, ref, n_vox, gpu, 51, 'C5')


def test_large_k_trace_vs_oracle(gpu):
    """A grid whose candidate list (K = 2 (nr + 1) + 2 (ne + 1) + (na + 1) + 1 = 14 017) outgrows one
    wave's LDS list (K <= 13 653): every hit ray goes through the exact path with its list in the
    workspace (the reference materialises any K, raytracer.py:92-173).  Segments of every ray
    against the oracle, the forward against the oracle's line integrals."""
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    grid = SphericalGrid(shape=(7000, 3, 5))
    geom = sum(ConeRectGeom((6, 8), pos=(3 * tr.cos(th), 3 * tr.sin(th), 0.5), fov=(40, 40))
               for th in tr.linspace(0, 2 * tr.pi, 3))
    op = Operator(grid, geom, device=gpu)
    assert op._csr['total'] > 0
    ref, n_vox = _oracle_trace(grid, geom)
    _compare_all(ref, _gpu_views(op, 3), 5.1, 'large K')
    g = tr.Generator().manual_seed(7)
    x = tr.rand(tuple(grid.shape), dtype=tr.float64, generator=g)
    ptr, vox, seg = _flat(ref)
    xv = x.numpy().reshape(-1)
    want = np.array([float(np.sum(xv[vox[a:b]] * seg[a:b])) for a, b in zip(ptr[:-1], ptr[1:])])
    got = op(x.to(gpu)).cpu().numpy().reshape(-1)
    assert np.allclose(got, want, rtol=1e-10, atol=1e-12)
