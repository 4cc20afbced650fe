"""The reference's own test suite, run against sph_raytracer_amd on the GPU.

Ports of sph_raytracer/test_all.py (solver known answers, find_starts) and
sph_raytracer/test_raytracer.py (operator chord lengths, shapes, regression LOS) — same inputs,
same assertions, same check() tolerance (float32 allclose, atol 1e-2).
"""
import numpy as np
import pytest
import torch as tr

from known_answers import A_CASES, E_CASES, R_CASES, e_boundaries

pytestmark = pytest.mark.gpu


def check(a, b):
    return tr.allclose(tr.asarray(a).type(tr.float32).flatten().squeeze(),
                       tr.asarray(b).type(tr.float32).flatten().squeeze(), atol=1e-2)


def test_r(gpu):
    from sph_raytracer_amd.raytracer import r_torch
    for bounds, xs, rays, t_exp, reg_exp in R_CASES:
        t, reg = r_torch(bounds, xs, rays)[:2]
        if t_exp == 'inf':
            assert tr.all(tr.isinf(t))
            continue
        assert check(t, t_exp)
        assert check(reg, reg_exp)


def test_e(gpu):
    from sph_raytracer_amd.raytracer import e_torch
    for spec, xs, rays, t_exp, reg_exp in E_CASES:
        bounds = e_boundaries(spec)
        t, reg = e_torch(tr.from_numpy(bounds), xs, rays)[:2]
        assert check(t, t_exp), (bounds, xs, rays, t)
        if reg_exp is not None:
            assert check(reg, reg_exp)


def test_a(gpu):
    from sph_raytracer_amd.raytracer import a_torch
    for bounds, xs, rays, t_exp, reg_exp in A_CASES:
        t, reg = a_torch(bounds, xs, rays)[:2]
        if t_exp == 'absinf':
            assert check(t.abs(), [float('inf')])
            continue
        assert check(t, t_exp)
        if reg_exp is not None:
            assert check(reg, reg_exp)


# ---- test_raytracer.py:8-116 --------------------------------------------------------------
U = 0.001
STARTS = [[-100, U, U], [U, -100, U], [U, U, -100], [-100, 0, U], [0, -100, U], [0, U, -100],
          [-100, U, 0], [U, -100, 0], [U, 0, -100], [5, 0, 0]]
DIRS = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0],
        [0, 0, 1], [-0.99998629093170166016, 0.00413372274488210678, 0.00321511807851493359]]


def test_operator_static(gpu):
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    grids = [SphericalGrid(shape=(50, 50, 50), size_r=(3, 25), size_e=(0, tr.pi),
                           size_a=(-tr.pi, tr.pi)),
             SphericalGrid(shape=(4, 4, 4)), SphericalGrid(shape=(1, 4, 4)),
             SphericalGrid(shape=(4, 1, 4)), SphericalGrid(shape=(4, 4, 1))]
    for grid in grids:
        op = Operator(grid, ViewGeom(STARTS, DIRS))
        result = op(tr.ones(grid.shape))
        diam = 2 * (grid.size[0][1] - grid.size[0][0])
        ok = tr.isclose(result, tr.tensor(diam, dtype=result.dtype), atol=1e-2)
        assert bool(ok.all()), f'grid={grid} rays {tr.where(~ok)[0].tolist()}: {result}'
    op = Operator(SphericalGrid(shape=(25, 25, 25), size_r=(5, 10)), ViewGeom([-100, 0, 0], [1, 0, 0]))
    result = op(tr.rand((5,) + (25, 25, 25)))
    assert result.shape == (5,), 'Incorrect shape for multi-channel volume'


def test_operator_shape(gpu):
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    cases = [[SphericalGrid((2, 3, 4)), tr.rand((2, 3, 4))],
             [SphericalGrid((2, 3, 4)), tr.rand((10, 2, 3, 4))],
             [SphericalGrid((10, 2, 3, 4)), tr.rand((10, 2, 3, 4))]]
    shape = (64, 64)
    geom = ConeRectGeom(shape, (1, 0, 0))
    for grid, d in cases:
        result = Operator(grid, geom)(d)
        assert result.shape == d.shape[:-3] + shape, f'grid={grid} input={d.shape}'


def test_buggy_los(gpu):
    from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom
    grid = SphericalGrid(shape=(1, 2, 1), size_r=(0, 25))
    d = tr.tensor([[[1.0], [0]]])     # upper hemisphere filled
    op = Operator(grid, ViewGeom([-200, U, U], [1, 0, 0]))
    result = op(d)
    assert tr.isclose(result, tr.tensor(50, dtype=result.dtype), atol=1e-2), result
