"""Gradient-descent retrieval — thin counterpart of the reference's retrieval.py (:24-127).

Every iteration is one Operator forward per fidelity loss plus one backward, i.e. the forward
and adjoint HIP kernels on the cached trace; the optimiser step is plain PyTorch.  The
examples/static_retrieval.py loop (FullyDenseModel, SquareLoss + NegRegularizer) runs the same
arithmetic without autograd (_gd_direct): the same iterates, a quarter of the launches.
"""
import ctypes
import math

import torch as t

from .loss import NegRegularizer, SquareLoss
from .model import FullyDenseModel

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
    # the optimiser exactly as the reference builds it (retrieval.py:84): torch's own default
    # implementation choice (foreach on GPU tensors) unless the caller passes foreach=/fused=
    opt = optim(optim_vars, **kwargs)
    plan = _direct_plan(f, y, model, coeffs, loss_fns, optim_vars)
    if plan is not None:
        return _gd_direct(f, y, coeffs, loss_fns, opt, plan, num_iterations, progress_bar)
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



def _unit(m):
    return isinstance(m, (int, float)) and not isinstance(m, bool) and m == 1


def _direct_plan(f, y, model, coeffs, loss_fns, optim_vars):
    """The loss terms of a loop `_gd_direct` runs without autograd, or None.  It covers the
    examples/static_retrieval.py loop: a FullyDenseModel (the coefficients are the density) on a
    static Operator, one SquareLoss and at most one NegRegularizer, scalar weights, no masks, the
    coefficients the only optimised variable.  Anything else takes the autograd loop."""
    from .raytracer import Operator
    if not isinstance(f, Operator) or f.dynamic or f._csr is None or y is None:
        return None
    if type(model) is not FullyDenseModel or hasattr(model, 'proj'):
        return None
    if len(optim_vars) != 1 or optim_vars[0] is not coeffs or coeffs.dtype != t.float64:
        return None     # (float64, the reference's coefficients: every scalar below is exact)
    if not (isinstance(y, t.Tensor) and coeffs.is_cuda and coeffs.device == f._cdev
            and y.device == coeffs.device and y.dtype in (t.float32, t.float64)
            and coeffs.is_contiguous() and tuple(coeffs.shape) == tuple(f.grid.shape)
            and tuple(y.shape) == tuple(f._ray_shape)):
        # (other devices, or a y the reference's SquareLoss would broadcast: the autograd loop)
        return None
    sq = neg = None
    for fn in loss_fns:
        if not (fn.use_grad and isinstance(fn.lam, (int, float)) and not isinstance(fn.lam, bool)
                and _unit(fn.projection_mask) and _unit(fn.volume_mask)):
            return None
        if type(fn) is SquareLoss and sq is None:
            sq = fn
        elif type(fn) is NegRegularizer and neg is None:
            neg = fn
        else:
            return None
    if sq is None:
        return None
    return sq, neg


def _gd_direct(f, y, coeffs, loss_fns, opt, plan, num_iterations, progress_bar, reduce=None,
               n_total=None):
    """`gd` for `_direct_plan` loops: the same arithmetic as autograd's, op by op, so the
    iterates are the same (the Operator forward, the adjoint of the SquareLoss residual, the
    NegRegularizer's -lam/N on negative voxels, the optimiser step), without building and walking
    a graph every iteration: one forward, one adjoint, the residual kernel of csrc/loss.hip
    and the optimiser step (for Adam, one csrc/loss.hip launch that also applies the
    regulariser and keeps the forward's brick-staged density current; otherwise the
    regulariser's own kernel, then opt.step()).  The loss values are the fused kernels' partial
    sums, summed for all iterations after the loop: deterministic, within rounding of the
    autograd loop's torch.mean.

    Gradient of lam * mean((y - f(d))^2): autograd's chain gives (lam / N) * (2 * (y - f(d)))
    negated, i.e. (f(d) - y) * (2 * (lam / N)) exactly (scaling by 2 and negation are exact).
    Gradient of lam * mean(|clip(d, max=0)|): -(lam / N) where d < 0, else 0 (sign(0) = 0).
    The two are summed (IEEE addition commutes, so the order autograd accumulates them in does
    not matter) and handed to the optimiser as coeffs.grad.

    Data-parallel use (distributed.gd): `f` is this rank's operator over its share of the views,
    `y` its share of the measurements, `n_total` the size of the whole stack (the SquareLoss
    mean's N) and `reduce` an in-place sum over the ranks, applied to the adjoint's gradient
    before the regulariser and the optimiser step (which are then identical on every rank) and
    to the SquareLoss sums after the loop."""
    from . import _lib
    sq, neg = plan
    losses = {fn: [] for fn in loss_fns}
    y.requires_grad_()                 # (the reference's own side effect on y)
    # y as measured: a float32 y is promoted inside the residual kernel (exactly, as y - f(d)
    # promotes it); anything else is converted to float64 once
    yd = y.detach()
    if yd.dtype not in (t.float32, t.float64):
        yd = yd.to(coeffs.dtype)
    yd = yd.contiguous()
    n_norm = yd.numel() if n_total is None else n_total     # the SquareLoss mean's N
    c_sq = sq.lam / n_norm
    c_neg = neg.lam / coeffs.numel() if neg is not None else 0.0
    step = _split_adam(opt, coeffs)
    bar = _Bar(range(num_iterations), progress_bar)
    lib = _lib.load()
    n_meas, n_vox = yd.numel(), coeffs.numel()
    # Adam keeps the forward's brick-staged density current (no pack launch per iteration)
    staged = f._stage_for_loop(coeffs.dtype) if step is not None else None
    if staged is not None and f._csr['n'] != n_meas:
        staged = None
    order = f._adjoint_trace_order()
    if order is not None and order.numel() != n_meas:
        order = None
    # the loop's own forward descriptor (a copy of the trace's): the staged one above, and with a
    # reordered trace — whose adjoint takes its input in trace order — one that writes f(d) in
    # that order too; the measurements are then permuted once and the residual kernel streams
    # both (the same values in the same order: bitwise the same iterates)
    loop_desc = staged[0] if staged is not None else None
    y_res, res_order, keep_rows = yd, order, None
    if order is not None:
        sd = loop_desc if loop_desc is not None else f._loop_descriptor(coeffs.dtype)
        keep_rows = f._trace_position_rows(sd) if sd is not None else None
        if keep_rows is not None:
            loop_desc = sd
            y_res, res_order = yd.reshape(-1).index_select(0, f._ray_id_long()), None
    yhat_buf = t.empty(n_meas, dtype=coeffs.dtype, device=coeffs.device) \
        if loop_desc is not None else None
    # every iteration's loss as the workgroup partial sums of its fused kernel, one row per
    # iteration, summed once after the loop (no reduction launch, no host sync per iteration)
    ps, pn = lib.sphrt_loss_partials(n_meas), lib.sphrt_loss_partials(n_vox)
    rows = max(num_iterations, 1)
    part_sq = t.empty((rows, ps), dtype=t.float64, device=coeffs.device)
    part_neg = t.empty((rows, pn), dtype=t.float64, device=coeffs.device) if neg is not None else None
    done = 0

    def scaled(sums, n, lam):
        val = sums / n
        return val if _unit(lam) else lam * val

    try:
        # every launch below on the coefficients' GPU, whatever device is current (the C entry
        # points launch on the stream's device; torch's default stream handle is the current
        # device's)
        with t.no_grad(), t.cuda.device(coeffs.device):
            for it in bar:
                opt.zero_grad()
                d = coeffs.detach()
                stream = _lib.stream_of(d.device)
                if loop_desc is not None:
                    # (staged: the forward reads the brick copy the previous Adam launch wrote;
                    # the first one packs it)
                    f._forward_staged(d, yhat_buf, loop_desc)
                    if staged is not None:
                        loop_desc.stage_packed = 1
                    yhat = yhat_buf.view(yd.shape)
                else:
                    yhat = f(d)
                if yhat.shape != yd.shape:
                    raise ValueError(f'measurements {tuple(yd.shape)} do not match the operator '
                                     f'output {tuple(yhat.shape)}')
                # r = f(d) - y, r * (2 lam / N) (the adjoint's input) and the partial sums of
                # r * r (the loss) in one launch (csrc/loss.hip)
                # (in the trace's ray order when the adjoint takes that: no permutation launch)
                r_scaled = t.empty_like(yhat)
                _lib.check(lib.sphrt_sq_residual_f64(
                    _lib.ptr(yhat), _lib.ptr(y_res), int(yd.dtype == t.float64), n_meas,
                    2 * c_sq, _lib.ptr(res_order), _lib.ptr(r_scaled), _lib.ptr(part_sq[it]),
                    stream), 'sphrt_sq_residual_f64')
                g = f._apply_adjoint(r_scaled, tuple(d.shape), d.dtype, d.device,
                                     trace_order=order is not None)
                if reduce is not None:
                    reduce(g)          # data-parallel: the sum of every rank's adjoint
                if step is not None:
                    # the regulariser's gradient term and loss partials inside the Adam launch
                    step(g, c_neg, part_neg[it] if neg is not None else None, stream,
                         staged[0] if staged is not None else None)
                elif neg is not None:
                    # g -= lam/N where d < 0, and the partial sums of |clamp(d, max=0)|
                    _lib.check(lib.sphrt_neg_reg_f64(_lib.ptr(d), n_vox, c_neg, _lib.ptr(g),
                                                     _lib.ptr(part_neg[it]), stream),
                               'sphrt_neg_reg_f64')
                if progress_bar:      # (this rank's share of the SquareLoss when data-parallel)
                    fv = float(scaled(part_sq[it].sum(), n_norm, sq.lam))
                    rv = float(scaled(part_neg[it].sum(), n_vox, neg.lam)) if neg is not None else 0
                    bar.describe(f'F:{fv:.1e} R:{rv:.1e} O:0')
                if step is None:
                    coeffs.grad = g
                    opt.step()
                done = it + 1
    except KeyboardInterrupt:
        if reduce is not None:
            # data-parallel: the other ranks may have stopped at another iteration, and the
            # loss sums below are reduced over equal lengths only — stop every rank loudly
            raise
    sums = part_sq[:done].sum(-1)
    if reduce is not None:
        reduce(sums)
    if neg is not None:
        sums = t.cat([sums, part_neg[:done].sum(-1)])
    # the return value's forward goes out before the readback waits (best is these coefficients
    # unless no iteration's total was finite, below)
    y_best = f(coeffs)
    # one readback for both terms; the scaling in Python floats (the weights are Python
    # numbers, _direct_plan) is the IEEE float64 division and product the tensor ops would do
    host = sums.cpu().tolist()
    losses[sq] = [scaled(v, n_norm, sq.lam) for v in host[:done]]
    if neg is not None:
        losses[neg] = [scaled(v, n_vox, neg.lam) for v in host[done:]]
    # the reference's bookkeeping: the coefficients once some iteration's total was < inf
    totals = [sum(v) for v in zip(*(losses[fn] for fn in loss_fns))]
    best = coeffs if any(v < float('inf') for v in totals) else None
    return best, (y_best if best is not None else f(best)), losses


def _number(v):
    """A plain Python scalar hyper-parameter (torch's defaults mix ints and floats: weight_decay=0)."""
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _split_adam(opt, coeffs):
    """torch.optim.Adam's step on `coeffs` as one csrc/loss.hip launch, or None.

    The launch runs the per-element arithmetic of the implementation torch itself would pick for
    this optimiser, bitwise: torch._fused_adam_ for Adam(fused=True) (sphrt_adam_neg_f64;
    `test_adam_matches_torch_fused`), the multi-tensor foreach step for the default Adam on a GPU
    tensor (sphrt_adam_foreach_neg_f64; `test_adam_matches_torch_foreach`) — the reference's own
    `optim(optim_vars, **kwargs)` (retrieval.py:84).  Either way it is one launch over the whole
    volume with the NegRegularizer's gradient term folded in, where torch runs ~10 foreach
    launches (or a fused step of one workgroup per 65536 elements: a 64^3 volume is 4 workgroups
    on a 256-CU GPU), and given a brick-staged forward descriptor (stage_of) it writes the
    updated coefficients to its stage too.  The optimiser's own state is left untouched (the loop
    owns the moments and the step count).  Anything else (amsgrad, maximize, capturable,
    differentiable, tensor hyper-parameters, the single-tensor path): None, and opt.step() runs."""
    from . import _lib
    if type(opt) is not t.optim.Adam or len(opt.param_groups) != 1:
        return None
    grp = opt.param_groups[0]
    if not (not grp.get('amsgrad') and not grp.get('maximize') and not grp.get('capturable')
            and not grp.get('differentiable') and not grp.get('decoupled_weight_decay')
            and all(_number(grp[k]) for k in ('lr', 'eps', 'weight_decay'))
            and all(_number(b) for b in grp['betas'])
            and len(grp['params']) == 1 and grp['params'][0] is coeffs):
        return None
    fused, foreach = grp.get('fused'), grp.get('foreach')
    if not fused and foreach is None:       # torch's own resolution (Optimizer defaults)
        try:   # a private torch helper: if it moves or changes, the generic opt.step() runs
            from torch.optim.optimizer import _default_to_fused_or_foreach
            _, foreach = _default_to_fused_or_foreach([coeffs], False, use_fused=False)
        except (ImportError, TypeError):
            return None
    if not fused and not foreach:
        return None
    lib = _lib.load()
    flat = coeffs.detach().view(-1)
    m, v = t.zeros_like(flat), t.zeros_like(flat)
    b1, b2 = (float(b) for b in grp['betas'])
    lr, eps, wd = (float(grp[k]) for k in ('lr', 'eps', 'weight_decay'))
    count = [0]

    def step(g, c_neg, part, stream, stage_of=None):
        count[0] += 1
        stage = ctypes.byref(stage_of) if stage_of is not None else None
        if fused:
            _lib.check(lib.sphrt_adam_neg_f64(
                _lib.ptr(flat), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), flat.numel(), lr, b1, b2,
                eps, wd, float(count[0]), c_neg, _lib.ptr(part), stage, stream),
                'sphrt_adam_neg_f64')
            return
        # the foreach step's bias corrections, as torch computes them (Python floats of the
        # float32 step count)
        st = float(count[0])
        step_size = (lr / (1 - b1 ** st)) * -1
        bc2_sqrt = (1 - b2 ** st) ** 0.5
        _lib.check(lib.sphrt_adam_foreach_neg_f64(
            _lib.ptr(flat), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), flat.numel(), step_size, b1, b2,
            eps, wd, bc2_sqrt, c_neg, _lib.ptr(part), stage, stream), 'sphrt_adam_foreach_neg_f64')
    return step
