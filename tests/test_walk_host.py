"""The lane walk (csrc/walk.hpp) replayed on the CPU against the C oracle — no GPU needed.

tests/walk_host.cpp compiles the device walk's source as host C++ (g++ -ffp-contract=off: the
device build's arithmetic), fed the boundary tables sphrt_plan_pack_tables packs for the GPU.
Every ray the walk takes (status 0) must give the oracle's segments bit for bit (voxels and
lengths, IEEE sqrt); rays it hands on (1: an exact tie, 2: a run out of order) are counted — the
GPU sends those to the exact / list trace.  Geometries: the BASELINE orbits (C2, C3, C5 views),
the golden fixtures' grids (hollow, hemisphere, half-azimuth, log-spaced [0, 2 pi] azimuth,
orbit views at azimuth 0), random rays from outside random grids, and near-degenerate lines
(close to the z axis, close to the origin, tangent to cones).
"""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest
import torch as tr

import golden_cases as gc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, 'sph_raytracer_amd', 'csrc')


@pytest.fixture(scope='module')
def walk_lib(tmp_path_factory):
    from sph_raytracer_amd import build
    build.build()          # (the table packing comes from libsphrt.so)
    out = tmp_path_factory.mktemp('walk') / 'libwalk_host.so'
    subprocess.run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off',
                    '-I', os.path.join(HERE, 'walk_host'), '-I', CSRC,
                    os.path.join(HERE, 'walk_host.cpp'), '-o', str(out)], check=True)
    lib = ctypes.CDLL(str(out))
    P = ctypes.c_void_p
    lib.walk_host.argtypes = [ctypes.c_int] * 3 + [P, ctypes.c_int, ctypes.c_double,
                                                   ctypes.c_double, P, P, P, ctypes.c_int64, P,
                                                   P, P, P, ctypes.c_int64]
    return lib


def _walk(lib, grid, xs, rays, starts, cap=None):
    from sph_raytracer_amd.raytracer import _Plan, _Staging
    plan = _Plan(grid, None, staging=_Staging())
    tables = plan._host
    d = plan._desc
    n = len(xs)
    cap = cap or (2 * (d.nr + d.ne) + d.na + 8)
    xs = np.ascontiguousarray(xs, np.float64)
    rays = np.ascontiguousarray(rays, np.float64)
    st = np.ascontiguousarray(np.asarray(starts).reshape(3, -1).T, np.int32)
    status = np.empty(n, np.int32)
    counts = np.empty(n, np.int32)
    vox = np.zeros((n, cap), np.int32)
    ln = np.zeros((n, cap), np.float64)
    lib.walk_host(d.nr, d.ne, d.na, tables.data_ptr(), d.a_wrap, d.close_tol, d.plane_par_tol,
                  xs.ctypes.data, rays.ctypes.data, st.ctypes.data, n, status.ctypes.data,
                  counts.ctypes.data, vox.ctypes.data, ln.ctypes.data, cap)
    assert counts.max(initial=0) <= cap
    return status, counts, vox, ln


def _check(lib, grid, xs, rays, what, min_walked=0.0, max_order=0.01):
    """Walk every ray; status-0 rays must equal the oracle bitwise.  Returns the status counts."""
    from oracle import oracle
    from sph_raytracer_amd.raytracer import find_starts
    xs = np.ascontiguousarray(np.broadcast_to(xs, np.shape(rays)).reshape(-1, 3))
    rays = np.ascontiguousarray(np.asarray(rays).reshape(-1, 3))
    starts = find_starts(grid, tr.from_numpy(xs)).numpy()
    status, counts, vox, ln = _walk(lib, grid, xs, rays, starts)
    oracle.use_mkl_sqrt(False)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    ptr, ov, ol = oracle.trace_segments(g, xs, rays, starts)
    ok = np.flatnonzero(status == 0)
    for i in ok:
        a, b = ptr[i], ptr[i + 1]
        k = counts[i]
        if k != b - a or not np.array_equal(vox[i, :k], ov[a:b]) or \
                not np.array_equal(ln[i, :k], ol[a:b]):
            pytest.fail(f'{what}: ray {i} walked {list(zip(vox[i, :k], ln[i, :k]))[:6]}... '
                        f'({k}) oracle {list(zip(ov[a:b], ol[a:b]))[:6]}... ({b - a})')
    hit = np.diff(ptr) > 0
    n_hit = max(int(hit.sum()), 1)
    frac = {s: float(np.mean(status[hit] == s)) for s in (-1, 0, 1, 2)}
    assert frac[0] >= min_walked, f'{what}: only {frac[0]:.3f} of hit rays walked ({frac})'
    assert frac[2] <= max_order, f'{what}: {frac[2]:.4f} of hit rays out of order'
    print(f'{what}: {n_hit} hit rays; walked {frac[0]:.4f}, not eligible {frac[-1]:.4f}, '
          f'ties {frac[1]:.4f}, out of order {frac[2]:.4f}')
    return frac


def _orbit(grid_shape, views, n_views, det, kind):
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, SphericalGrid
    grid = SphericalGrid(shape=grid_shape)
    th = tr.linspace(0, 2 * tr.pi, n_views)[list(views)]
    mk = (lambda p: ConeRectGeom(det, pos=p, fov=(45, 45))) if kind == 'rect' else \
        (lambda p: ConeCircGeom(shape=det, pos=p, fov=(0, 45)))
    geom = sum(mk((5 * tr.cos(t), 5 * tr.sin(t), 1)) for t in th)
    return grid, geom


@pytest.mark.parametrize('name, grid_shape, views, n_views, det, kind', [
    ('C2', (50, 50, 50), (1, 17, 33, 49), 50, (50, 100), 'rect'),
    ('C5', (64, 64, 64), (0, 5, 20, 47), 64, (100, 50), 'circ'),
    ('C3', (128, 128, 128), (3, 77), 128, (128, 256), 'rect'),
])
def test_walk_orbits_vs_oracle(walk_lib, name, grid_shape, views, n_views, det, kind):
    grid, geom = _orbit(grid_shape, views, n_views, det, kind)
    frac = _check(walk_lib, grid, geom.ray_starts.numpy(), geom.rays.numpy(), name)
    assert frac[0] + frac[1] > 0.99 and frac[2] < 0.005


@pytest.mark.parametrize('name', ['circ_orbit', 'partial_grid', 'log_grid', 'dynamic_obs',
                                  'c2_orbit3', 'c1_single_vantage'])
def test_walk_fixture_grids_vs_oracle(walk_lib, name):
    case = gc.load(name)
    grid = gc.make_grid(case)
    _check(walk_lib, grid, case['xs'], case['rays'], name)


@pytest.mark.parametrize('seed', range(6))
def test_walk_random_grids_vs_oracle(walk_lib, seed):
    """Random grids (odd shapes, hollow, partial elevation / azimuth ranges, log spacing) seen by
    random rays from outside aimed at random points of the ball."""
    from sph_raytracer_amd import SphericalGrid
    rng = np.random.default_rng(seed)
    shape = tuple(int(v) for v in rng.integers(3, 40, size=3))
    kw = {}
    if seed % 2:
        kw['size_r'] = (float(rng.uniform(0.05, 0.5)), 1.0)
    if seed % 3 == 1:
        kw['size_e'] = (float(rng.uniform(0, 1)), float(rng.uniform(2, math.pi)))
    if seed % 3 == 2:
        lo = float(rng.uniform(-math.pi, 0))
        kw['size_a'] = (lo, lo + float(rng.uniform(1, 2 * math.pi)))
    if seed == 4:
        kw['spacing'] = 'log'
        kw['size_r'] = (0.1, 1.0)
    grid = SphericalGrid(shape=shape, **kw)
    n = 6000
    u = rng.normal(size=(n, 3))
    xs = u / np.linalg.norm(u, axis=1, keepdims=True) * rng.uniform(1.05, 8, size=(n, 1))
    tgt = rng.normal(size=(n, 3))
    tgt = tgt / np.linalg.norm(tgt, axis=1, keepdims=True) * rng.uniform(0, 1.1, size=(n, 1)) ** (1 / 3)
    d = tgt - xs
    _check(walk_lib, grid, xs, d, f'random grid {shape} {kw}')


def test_walk_near_degenerate_lines(walk_lib):
    """Lines passing close to the z axis and to the origin, nearly vertical ones, and lines
    grazing cones (their elevation extremum on a cone angle): every walked ray exact."""
    from sph_raytracer_amd import SphericalGrid
    grid = SphericalGrid(shape=(20, 18, 24))
    rng = np.random.default_rng(9)
    n = 4000
    xs = np.empty((n, 3))
    d = np.empty((n, 3))
    for i in range(n):
        start = rng.normal(size=3)
        start = start / np.linalg.norm(start) * rng.uniform(1.5, 5)
        kind = i % 4
        eps = 10.0 ** rng.uniform(-12, -3)
        if kind == 0:    # through a point eps off the z axis
            tgt = np.array([eps, -eps * rng.uniform(), rng.uniform(-0.9, 0.9)])
        elif kind == 1:  # eps off the origin
            tgt = rng.normal(size=3) * eps
        elif kind == 2:  # nearly vertical
            start = np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), 3.0])
            tgt = start + np.array([eps, eps * rng.uniform(), -1.0])
        else:            # tangent to a cone: closest elevation equal to a boundary angle
            e = float(grid.e_b[rng.integers(1, 18)])
            p = np.array([math.sin(e), 0.0, math.cos(e)]) * rng.uniform(0.2, 0.9)
            rot = rng.uniform(0, 2 * math.pi)
            p = np.array([p[0] * math.cos(rot), p[0] * math.sin(rot), p[2]])
            axis = np.cross(p, [0, 0, 1.0])
            axis /= np.linalg.norm(axis)
            start, tgt = p - 3 * axis, p
        xs[i] = start
        d[i] = tgt - start
    _check(walk_lib, grid, xs, d, 'near-degenerate lines', max_order=0.15)
