"""Torch-CPU restatement of the reference's Operator forward / adjoint — CPU BASELINE + TESTS ONLY.

The reference keeps, per operator, the padded trace regs (3, *rays, K) int64 and lens (*rays, K)
float64 (raytracer.py:675-679, 230) and evaluates
    forward  (raytracer.py:703-713): out = (density[t, r, e, a] * lens).sum(-1)
    adjoint  (raytracer.py:725-748): zeros(grid).index_put_((r, e, a), y[..., None] * lens,
                                     accumulate=True)
with torch CPU kernels.  The padded trace itself is produced by the C oracle (oracle.trace_dense,
bit-identical to trace_indices with MKL sqrt), so the timed forward runs on exactly the
reference's arrays.  Only bench.py's cpu_baseline leg and tests/ use this module.
"""
import numpy as np
import torch as tr

from . import oracle


def dense_trace(grid_boundaries, xs, rays, starts, sqrt_mkl=True):
    """-> (regs (3, *rays, K) int64, lens (*rays, K) float64) as torch CPU tensors."""
    if sqrt_mkl:
        oracle.use_mkl_sqrt(True)
    try:
        g = oracle.Grid.from_boundaries(*grid_boundaries)
        regs, lens = oracle.trace_dense(g, xs, rays, starts)
    finally:
        oracle.use_mkl_sqrt(False)
    return tr.from_numpy(regs.astype(np.int64)), tr.from_numpy(lens)


def forward(regs, lens, density, dynamic=False):
    """Operator.__call__ of the reference on its padded trace (raytracer.py:703-713)."""
    r, e, a = regs
    t = tr.arange(len(density))[:, None, None, None] if dynamic else Ellipsis
    out = density[t, r, e, a]
    out *= lens
    return out.sum(axis=-1)


def adjoint(regs, lens, y, grid_shape):
    """Operator.T of the reference (raytracer.py:725-748), static grids."""
    vol = tr.zeros(grid_shape, dtype=y.dtype)
    vol.index_put_(tuple(regs), y[..., None] * lens, accumulate=True)
    return vol
