"""Multi-GPU operator: observations sharded across the ranks of one node.

One process per GPU (torchrun), torch.distributed with the "nccl" backend (RCCL over xGMI).
Rays are independent, so each rank traces and integrates only its own contiguous block of views
— no data-path communication — and the path's only exchanges are:
  - forward: the image stack, gathered with one all_gather (padded to the largest shard);
  - static adjoint / gradient: one all_reduce(sum) of the volume (1-17 MB);
  - dynamic grids: view i pairs with time slice i, so every rank owns disjoint time slices and
    its adjoint needs no reduction at all (the full adjoint is one all-gather of the slices);
  - data-parallel retrieval: one all_reduce(sum) of the coefficient gradient per iteration.

The reference has no distributed code; the single-GPU semantics are Operator's (raytracer.py).
"""
import math

import torch as tr
import torch.distributed as dist

from .geometry import ViewGeomCollection


def shard_bounds(n_items, world, rank):
    """Contiguous block of `n_items` for `rank`: sizes differ by at most one (remainder spread
    over the first ranks)."""
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedOperator:
    """Operator over a ViewGeomCollection whose views are split across a process group.

    Args:
        grid: SphericalGrid (static, or dynamic with one time slice per view).
        geom: ViewGeomCollection of n_obs views (the full set; every rank passes the same).
        group: process group (default: WORLD).
        device: this rank's GPU.
        operator_factory: callable(grid, local_geom, device) -> local operator; defaults to
            sph_raytracer_amd.Operator (tests substitute a CPU stand-in to exercise the
            communication on gloo).
    Calling returns this rank's images (differentiable); ``gather`` assembles the full stack.
    """

    def __init__(self, grid, geom, group=None, device=None, operator_factory=None, **op_kwargs):
        if not isinstance(geom, ViewGeomCollection):
            raise TypeError('ShardedOperator shards a ViewGeomCollection by observation')
        self.grid, self.geom, self.group = grid, geom, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.n_obs = len(geom)
        if self.n_obs < self.world:
            raise ValueError(f'{self.n_obs} views cannot be sharded over {self.world} ranks')
        self.bounds = [shard_bounds(self.n_obs, self.world, r) for r in range(self.world)]
        self.lo, self.hi = self.bounds[self.rank]
        local = ViewGeomCollection(*geom.geoms[self.lo:self.hi])
        if operator_factory is None:
            from .raytracer import Operator
            operator_factory = lambda g, lg, dev: Operator(g, lg, device=dev, **op_kwargs)  # noqa: E731
        self.local = operator_factory(grid, local, device)
        self.device = getattr(self.local, 'device', device)
        self.view_shape = tuple(geom.shape[1:])

    # -- collectives (RCCL for GPU tensors; gloo — CPU runs and one-GPU rehearsals — through host
    #    copies, since gloo's GPU support is partial) ---------------------------------------------
    def _host_staged(self, t):
        return t.is_cuda and dist.get_backend(self.group) != 'nccl'

    def all_reduce(self, t):
        """In-place sum over the group (one RCCL all_reduce on GPUs)."""
        if self._host_staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def _all_gather_rows(self, local, lead):
        """Every rank's `local` (lead..., n_local, P) -> (lead..., n_obs, P) on every rank: one
        all-gather of blocks padded to the largest shard (RCCL all_gather_into_tensor)."""
        n_loc = self.hi - self.lo
        width = max(h - l for l, h in self.bounds)
        pad = tr.zeros(lead + (width, local.shape[-1]), dtype=local.dtype, device=local.device)
        pad[..., :n_loc, :] = local
        pad = pad.movedim(len(lead), 0).contiguous()          # (width, *lead, P)
        out = tr.empty((self.world,) + tuple(pad.shape), dtype=pad.dtype, device=pad.device)
        if self._host_staged(pad):
            ho = out.cpu()
            dist.all_gather(list(ho.unbind(0)), pad.cpu(), group=self.group)
            out.copy_(ho)
        elif dist.get_backend(self.group) == 'nccl':
            dist.all_gather_into_tensor(out, pad, group=self.group)     # one RCCL all-gather
        else:
            dist.all_gather(list(out.unbind(0)), pad, group=self.group)
        parts = [out[r, :h - l] for r, (l, h) in enumerate(self.bounds)]
        return tr.cat(parts, dim=0).movedim(0, len(lead))         # (*lead, n_obs, P)

    # -- forward ---------------------------------------------------------------------------------
    def _local_density(self, density):
        if self.grid.dynamic:     # view i sees time slice i: keep this rank's slices
            if density.shape[0] != self.n_obs:
                raise ValueError('dynamic density must have one time slice per view')
            return density[self.lo:self.hi]
        return density

    def __call__(self, density):
        """This rank's line integrals: (C..., n_local, *view) static / (n_local, *view) dynamic.
        Differentiable: the gradient reaches this rank's share (all of a static density, its own
        time slices of a dynamic one); sum it over ranks (all_reduce) for the full gradient."""
        return self.local(self._local_density(density))

    def gather(self, y_local):
        """All-gather the per-rank image stacks -> (C..., n_obs, *view) on every rank."""
        lead = tuple(y_local.shape[:-1 - len(self.view_shape)])
        flat = y_local.detach().reshape(lead + (self.hi - self.lo, -1))
        full = self._all_gather_rows(flat, lead)
        return full.reshape(lead + (self.n_obs,) + self.view_shape)

    def forward_full(self, density):
        """Full image stack (n_obs views) on every rank: local forward + one all-gather."""
        return self.gather(self(density))

    # -- adjoint ---------------------------------------------------------------------------------
    def T_local(self, y_local):
        """Back-projection of this rank's own views (n_local, *view), no communication: a
        partial volume (static grid; summed over ranks it is T of the whole stack) or this rank's
        own time slices (n_local, nr, ne, na) (dynamic grid)."""
        y = tr.as_tensor(y_local)
        if not self.grid.dynamic:
            return self.local.T(y)
        dshape = (self.hi - self.lo,) + tuple(self.grid.shape[1:])
        return self.local._apply_adjoint(y, dshape, y.dtype, y.device)

    def T(self, line_integrations):
        """Back-projection of the full (n_obs, *view) stack on every rank.  Static grid: each
        rank back-projects its views, then one all_reduce(sum) of the volume.  Dynamic grid
        (view i <-> time slice i; the reference's Operator.T raises for it, raytracer.py:733):
        each rank back-projects its views into its own slices, then one all-gather of the
        slices."""
        y = tr.as_tensor(line_integrations)
        vol = self.T_local(y[self.lo:self.hi])
        if not self.grid.dynamic:
            return self.all_reduce(vol)
        g3 = tuple(self.grid.shape[1:])
        full = self._all_gather_rows(vol.reshape(self.hi - self.lo, -1), ())
        return full.reshape((self.n_obs,) + g3)

    def reduce_grad(self, grad):
        """Sum a replicated parameter's gradient over ranks (data-parallel retrieval)."""
        return self.all_reduce(grad)

    @property
    def n_measurements(self):
        """Values in the whole (n_obs, *view) stack."""
        return self.n_obs * math.prod(self.view_shape)


def gd(f, y_local, model, coeffs=None, num_iterations=100, loss_fns=None, optim=tr.optim.Adam,
       progress_bar=False, device=None, **kwargs):
    """Data-parallel counterpart of retrieval.gd for a ShardedOperator (static grids).

    Every rank holds replicated coefficients and its own measurement shard ``y_local`` (its
    views of the stack).  Each iteration: local forward, local adjoint, one all_reduce(sum) of
    the coefficient gradient, the identical optimiser step on every rank; the losses are those of
    the whole stack (SquareLoss: the mean over all n_obs views).

    The static_retrieval.py loop (retrieval._direct_plan: FullyDenseModel, SquareLoss +
    NegRegularizer, Adam, ...) runs autograd-free as on one GPU (retrieval._gd_direct) with the
    all_reduce between its adjoint and its Adam launch; anything else takes the autograd loop,
    where fidelity losses are weighted by the rank's share of the views so the summed gradient
    equals the single-GPU gradient of the full-stack mean and regulariser gradients are divided
    by the world size (every rank computes them).
    Returns (coeffs, the full reconstructed stack, {loss_fn: [values]}).
    """
    from .loss import SquareLoss
    from .retrieval import _direct_plan, _gd_direct, detach_loss
    loss_fns = [SquareLoss()] if loss_fns is None else loss_fns
    share = (f.hi - f.lo) / f.n_obs
    if coeffs is None:
        coeffs = tr.ones(model.coeffs_shape, dtype=tr.float64, device=device or f.device)
    coeffs.requires_grad_()
    opt = optim([coeffs], **kwargs)
    plan = _direct_plan(f.local, y_local, model, coeffs, loss_fns, [coeffs]) \
        if hasattr(f.local, '_csr') else None
    # the two loops issue different collectives: every rank takes the direct loop or none does
    flag = tr.tensor([1.0 if plan is not None else 0.0], dtype=tr.float64, device=coeffs.device)
    if f._host_staged(flag):
        h = flag.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MIN, group=f.group)
        flag.copy_(h)
    else:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=f.group)
    if plan is not None and flag.item() == 1.0:
        best, y_best, losses = _gd_direct(f.local, y_local, coeffs, loss_fns, opt, plan,
                                          num_iterations, progress_bar, reduce=f.all_reduce,
                                          n_total=f.n_measurements)
        # this rank's forward of the returned coefficients is already computed: gather it
        return best, f.gather(y_best), losses
    losses = {fn: [] for fn in loss_fns}
    for _ in range(num_iterations):
        opt.zero_grad()
        density = model(coeffs)
        total = 0
        for fn in loss_fns:
            val = fn(f, y_local, density, coeffs)
            w = share if fn.kind == 'fidelity' else 1.0 / f.world
            if fn.use_grad and fn.kind != 'oracle':
                total = total + w * val
            v = tr.as_tensor(detach_loss(val) * (share if fn.kind == 'fidelity' else 1.0),
                             dtype=tr.float64, device=coeffs.device)
            if fn.kind == 'fidelity':
                f.all_reduce(v)
            losses[fn].append(float(v))
        total.backward(retain_graph=True)
        f.reduce_grad(coeffs.grad)
        opt.step()
        if hasattr(model, 'proj'):
            coeffs.data = model.proj(coeffs)
    return coeffs, f.gather(f(model(coeffs))), losses
