"""Gradient-descent retrieval — thin counterpart of the reference's retrieval.py (:24-127).

Every iteration is one Operator forward per fidelity loss plus one backward, i.e. the forward
and adjoint HIP kernels on the cached trace; the optimiser step is plain PyTorch.
"""
import math

import torch as t

from .loss import SquareLoss

try:
    from tqdm import tqdm
except ImportError:    # progress bars are cosmetic
    def tqdm(it, disable=False):
        return it


def detach_loss(loss):
    """Loss value as a float, detached from autograd."""
    return float(loss.detach().cpu()) if isinstance(loss, t.Tensor) else loss


class _Bar:
    def __init__(self, it, enabled):
        self.it = tqdm(it, disable=not enabled)
        self.enabled = enabled

    def __iter__(self):
        return iter(self.it)

    def describe(self, text):
        if self.enabled and hasattr(self.it, 'set_description'):
            self.it.set_description(text)


def gd(f, y, model, coeffs=None, num_iterations=100, loss_fns=[SquareLoss()], optim=t.optim.Adam,
       optim_vars=None, progress_bar=True, device=None, **kwargs):
    """Minimise the weighted sum of ``loss_fns`` over the model coefficients.

    Same contract as the reference: returns (coeffs, f(model(coeffs)), {loss_fn: [values]});
    Ctrl-C stops early.  Like the reference, the coefficients returned are those of the last
    iteration (its best-loss bookkeeping never updates, retrieval.py:112-113).
    """
    if hasattr(f, 'grid') and f.grid != model.grid:
        raise ValueError("f and model must have same grid")
    if y is not None:
        y.requires_grad_()
    if coeffs is None:
        coeffs = t.ones(model.coeffs_shape, requires_grad=True, device=device or f.device,
                        dtype=t.float64)
    if optim_vars is None:
        optim_vars = [coeffs]
    for v in optim_vars:
        v.requires_grad_()
    best_loss, best_coeffs = float('inf'), None
    # A torch optimiser with a fused GPU step (Adam, AdamW, SGD, ...) takes it unless the caller
    # chose an implementation: one kernel per step instead of ~10 multi-tensor launches, with
    # the same update within rounding (C5: 0.42-0.52 -> 0.36 ms per iteration).
    if ('foreach' not in kwargs and 'fused' not in kwargs and 'fused' in _init_args(optim)
            and all(isinstance(v, t.Tensor) and v.is_cuda and v.is_floating_point()
                    for v in optim_vars)):
        kwargs['fused'] = True
    opt = optim(optim_vars, **kwargs)
    losses = {fn: [] for fn in loss_fns}
    o_stat = 0
    bar = _Bar(range(num_iterations), progress_bar)
    # Without a progress bar nothing needs the loss values during the loop: they stay on the
    # device and are read back once at the end (no host sync per iteration; same values, same
    # return contract).  With a bar, every iteration reads them back as the reference does.
    deferred = not progress_bar
    pending = {fn: [] for fn in loss_fns}
    improved = None                       # device flag: some iteration had total < best_loss
    try:
        for _ in bar:
            opt.zero_grad()
            density = model(coeffs)
            total = f_stat = r_stat = 0
            for fn in loss_fns:
                val = fn(f, y, density, coeffs)
                if fn.use_grad and fn.kind != 'oracle':
                    total += val
                if deferred:
                    pending[fn].append(val.detach() if isinstance(val, t.Tensor) else val)
                    continue
                if fn.kind == 'oracle' and not math.isnan(val):
                    o_stat = val
                elif fn.kind == 'fidelity':
                    f_stat += val
                elif fn.kind == 'regularizer':
                    r_stat += val
                losses[fn].append(detach_loss(val))
            if deferred:
                ok = total < best_loss
                improved = ok if improved is None else improved | ok
            else:
                bar.describe(f'F:{f_stat:.1e} R:{r_stat:.1e} O:{o_stat * 100:.0f}')
                if total < best_loss:
                    best_coeffs = coeffs
            total.backward(retain_graph=True)
            opt.step()
            if hasattr(model, 'proj'):
                coeffs.data = model.proj(coeffs)
    except KeyboardInterrupt:
        pass
    if deferred:
        for fn, vals in pending.items():
            tens = [v for v in vals if isinstance(v, t.Tensor)]
            host = iter(t.stack(tens).cpu().tolist()) if tens else iter(())
            losses[fn] = [next(host) if isinstance(v, t.Tensor) else v for v in vals]
        if improved is not None and bool(improved):
            best_coeffs = coeffs    # the same tensor object every iteration (updated in place)
    return best_coeffs, f(model(best_coeffs)), losses



def _init_args(optim):
    import inspect
    try:
        return inspect.signature(optim.__init__).parameters
    except (TypeError, ValueError):
        return {}
