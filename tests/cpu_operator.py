"""CPU stand-in for Operator built on the oracle — TEST INFRASTRUCTURE ONLY.

Lets the multi-process (gloo, CPU) tests exercise ShardedOperator's sharding, all-gather and
all-reduce logic without a GPU.  Same call semantics as Operator for static grids and for
dynamic grids paired view-by-view with time slices; differentiable through a torch autograd
Function whose backward is the oracle adjoint.
"""
import math
import os
import sys

import numpy as np
import torch as tr

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from sph_raytracer_amd.raytracer import _layout_for, find_starts  # noqa: E402


class _Fn(tr.autograd.Function):
    @staticmethod
    def forward(ctx, density, op):
        ctx.op = op
        ctx.shape = density.shape
        return op._fwd(density.detach())

    @staticmethod
    def backward(ctx, g):
        return ctx.op._adj(g, ctx.shape), None


class CpuOperator:
    def __init__(self, grid, geom, device='cpu'):
        self.grid, self.geom, self.device = grid, geom, device
        xs, rays = geom.ray_starts, geom.rays
        shape = tuple(tr.broadcast_shapes(xs.shape, rays.shape))[:-1]
        self.ray_shape = shape
        g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
        starts = find_starts(grid, xs).numpy()
        self.ptr, self.vox, self.seg = oracle.trace_segments(g, xs.numpy(), rays.numpy(), starts)
        self.n_vox = math.prod(grid.shape[-3:])

    def __call__(self, density):
        return _Fn.apply(tr.as_tensor(density), self)

    def _fwd(self, density):
        n_chan, div, out_shape = _layout_for(self.grid, self.ray_shape, density.shape)
        out = oracle.forward(self.ptr, self.vox, self.seg, density.numpy(), self.n_vox,
                             ray_chan_div=div)
        return tr.from_numpy(np.ascontiguousarray(out).reshape(out_shape)).to(density.dtype)

    def _adj(self, y, dshape):
        n_chan, div, _ = _layout_for(self.grid, self.ray_shape, dshape)
        dtype = y.dtype
        y = y.detach().numpy().reshape(n_chan if not div else 1, -1)
        n = len(self.ptr) - 1
        ray = np.repeat(np.arange(n), np.diff(self.ptr))
        if div:
            vol = np.zeros((dshape[0], self.n_vox))
            np.add.at(vol, (ray[...] // div, self.vox), y[0][ray] * self.seg)
        else:
            vol = np.stack([np.bincount(self.vox, yc[ray] * self.seg, minlength=self.n_vox)
                            for yc in y])
        return tr.from_numpy(vol.reshape(dshape)).to(dtype)

    def T(self, y):
        return self._adj(tr.as_tensor(y), tuple(self.grid.shape))

    def _apply_adjoint(self, y, dshape, ddtype, ddevice):
        """Operator._apply_adjoint's contract (any grid, dynamic included)."""
        return self._adj(tr.as_tensor(y), tuple(dshape)).to(device=ddevice, dtype=ddtype)
