"""Parametric volume models — thin counterparts of the reference's model.py (model.py:7-114).

Glue around the hot path, kept so ``gd()`` and the examples run unchanged.
"""
import torch as t

from .geometry import SphericalGrid


class Model:
    """Base class: map coefficients (shape ``coeffs_shape``) to a volume of ``grid.shape``."""

    def __init__(self, grid: SphericalGrid):
        raise NotImplementedError

    def __call__(self, coeffs):
        raise NotImplementedError

    @property
    def coeffs_shape(self):
        raise NotImplementedError

    def __repr__(self):
        return f'{type(self).__name__}({tuple(self.grid.shape)})'


class FullyDenseModel(Model):
    """One coefficient per voxel: the coefficients are the density."""

    def __init__(self, grid: SphericalGrid):
        self.grid = grid

    def __call__(self, coeffs):
        return coeffs

    @property
    def coeffs_shape(self):
        return self.grid.shape


def _frac_index(n, fracs):
    return [int(v) for v in n * t.tensor(fracs)]


class CubesModel(Model):
    """Test phantom: two boxes in (r, e, a) index space (model.py:55-85)."""

    def __init__(self, grid: SphericalGrid):
        self.grid = grid
        self.r0, self.r1 = _frac_index(grid.shape.r, (.333, .666))
        self.e00, self.e01 = _frac_index(grid.shape.e, (.2, .3))
        self.e10, self.e11 = _frac_index(grid.shape.e, (.7, .9))
        self.a0, self.a1 = _frac_index(grid.shape.a, (.4, .6))
        self.volume = t.zeros(grid.shape)
        for e_lo, e_hi in ((self.e00, self.e01), (self.e10, self.e11)):
            self.volume[self.r0:self.r1, e_lo:e_hi, self.a0:self.a1] = 1

    def __call__(self, coeffs):
        return self.volume

    @property
    def coeffs_shape(self):
        return ()


class AxisAlignmentModel(Model):
    """Test phantom marking the +X, +Y and +Z axes, to catch mirrored projections
    (model.py:88-114)."""

    def __init__(self, grid: SphericalGrid):
        self.grid = grid
        s = grid.shape
        self.volume = t.zeros(s)
        self.volume[:s.r // 3, s.e // 2, 0] = 1                 # X axis
        self.volume[:s.r // 2, s.e // 2, (s.a * 3) // 4] = 1    # Y axis
        self.volume[:, 0, :] = 1                                # Z axis

    def __call__(self, coeffs):
        return self.volume

    @property
    def coeffs_shape(self):
        return ()
