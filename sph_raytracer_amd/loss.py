"""Retrieval losses — thin counterparts of the reference's loss.py (loss.py:14-162).

A loss is built once, weighted by multiplying with a scalar (``5 * SquareLoss()``), and called
by ``gd()`` as ``loss(f, y, density, coeffs)``; the fidelity losses call the Operator ``f``.
"""
import torch as t


def _scaled(m, x):
    """m * x, skipping the multiply (one kernel, and one more in the backward) when m is the
    scalar 1: x * 1 == x exactly."""
    if isinstance(m, (int, float)) and not isinstance(m, bool) and m == 1:
        return x
    return m * x


class Loss:
    """Base loss: ``compute(f, y, d, c)`` times weight ``lam``.

    Args: projection_mask / volume_mask (multiplied into measurements / densities), lam (weight),
    use_grad (False -> evaluated under no_grad, e.g. for monitoring).
    """

    kind = 'regularizer'

    def __init__(self, *args, projection_mask=1, volume_mask=1, lam=1, use_grad=True, **kwargs):
        self.projection_mask = projection_mask
        self.volume_mask = volume_mask
        self.lam = lam
        self.use_grad = use_grad

    def compute(self, f, y, d, c):
        raise NotImplementedError

    def __call__(self, f, y, d, c):
        if self.use_grad:
            val = self.compute(f, y, d, c)
        else:
            with t.no_grad():
                val = self.compute(f, y, d, c)
        return None if val is None else _scaled(self.lam, val)

    def __mul__(self, other):
        self.lam = other
        return self

    __rmul__ = __mul__

    def __repr__(self):
        return f'{self.lam:.0e} * {type(self).__name__}'


class SquareLoss(Loss):
    """mean((y - f(d))^2) over unmasked pixels."""
    kind = 'fidelity'

    def compute(self, f, y, d, c):
        return t.mean(_scaled(self.projection_mask, (y - f(_scaled(self.volume_mask, d))) ** 2))


class SquareRelLoss(Loss):
    """mean(((y - f(d)) / y)^2), zero where y == 0."""
    kind = 'fidelity'

    def compute(self, f, y, d, c):
        pred = f(_scaled(self.volume_mask, d))
        nz = y != 0
        rel = t.zeros_like(y)
        rel[nz] = (y - pred)[nz] / y[nz]
        return t.mean(_scaled(self.projection_mask, rel) ** 2)


class AbsLoss(Loss):
    """mean(|y - f(d)|)."""
    kind = 'fidelity'

    def compute(self, f, y, d, c):
        return t.mean(_scaled(self.projection_mask, (y - f(_scaled(self.volume_mask, d))).abs()))


class CheaterLoss(Loss):
    """L2 distance to a known ground-truth density (monitoring only)."""
    kind = 'oracle'

    def __init__(self, density_truth, *args, **kwargs):
        self.density_truth = density_truth
        super().__init__(**kwargs)

    def compute(self, f, y, d, c):
        return t.mean(_scaled(self.volume_mask, (d - self.density_truth) ** 2))


class NegRegularizer(Loss):
    """Mean magnitude of negative voxels."""

    def compute(self, f, y, d, c):
        return t.mean(t.abs(_scaled(self.volume_mask, d.clip(max=0))))


class NegSumRegularizer(Loss):
    """Summed magnitude of negative voxels."""

    def compute(self, f, y, d, c):
        return t.sum(t.abs(_scaled(self.volume_mask, d.clip(max=0))))
