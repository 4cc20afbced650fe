"""Multi-GPU operator: observations sharded across the ranks of one node.

One process per GPU (torchrun), torch.distributed with the "nccl" backend (RCCL over xGMI).
Rays are independent, so each rank traces and integrates only its own contiguous block of views
— no data-path communication — and the path's only exchanges are:
  - forward: the image stack, gathered with one all_gather (padded to the largest shard);
  - static adjoint / gradient: one all_reduce(sum) of the volume (1-17 MB);
  - dynamic grids: view i pairs with time slice i, so every rank owns disjoint time slices and
    its adjoint needs no reduction at all.

The reference has no distributed code; the single-GPU semantics are Operator's (raytracer.py).
"""
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

    # -- forward ---------------------------------------------------------------------------------
    def _local_density(self, density):
        if self.grid.dynamic:     # view i sees time slice i: keep this rank's slices
            if density.shape[0] != self.n_obs:
                raise ValueError('dynamic density must have one time slice per view')
            return density[self.lo:self.hi]
        return density

    def __call__(self, density):
        """This rank's line integrals: (C..., n_local, *view) static / (n_local, *view) dynamic."""
        return self.local(self._local_density(density))

    def gather(self, y_local):
        """All-gather the per-rank image stacks -> (C..., n_obs, *view) on every rank."""
        lead = tuple(y_local.shape[:-1 - len(self.view_shape)])
        n_loc = self.hi - self.lo
        width = max(h - l for l, h in self.bounds)
        flat = y_local.detach().reshape(lead + (n_loc, -1))
        pad = tr.zeros(lead + (width, flat.shape[-1]), dtype=flat.dtype, device=flat.device)
        pad[..., :n_loc, :] = flat
        pad = pad.movedim(len(lead), 0).contiguous()          # (width, *lead, P)
        out = tr.empty((self.world,) + tuple(pad.shape), dtype=pad.dtype, device=pad.device)
        if dist.get_backend(self.group) == 'nccl':
            dist.all_gather_into_tensor(out, pad, group=self.group)     # one RCCL all-gather
        else:
            dist.all_gather(list(out.unbind(0)), pad, group=self.group)
        parts = [out[r, :h - l] for r, (l, h) in enumerate(self.bounds)]
        full = tr.cat(parts, dim=0).movedim(0, len(lead))      # (*lead, n_obs, P)
        return full.reshape(lead + (self.n_obs,) + self.view_shape)

    def forward_full(self, density):
        """Full image stack (n_obs views) on every rank: local forward + one all-gather."""
        return self.gather(self(density))

    # -- adjoint ---------------------------------------------------------------------------------
    def T(self, line_integrations):
        """Back-projection of the full (n_obs, *view) stack: each rank back-projects its views,
        then one all_reduce(sum) of the volume (static grids)."""
        if self.grid.dynamic:
            raise NotImplementedError('use T_local: dynamic shards own disjoint time slices')
        y = tr.as_tensor(line_integrations)
        vol = self.local.T(y[self.lo:self.hi])
        dist.all_reduce(vol, op=dist.ReduceOp.SUM, group=self.group)
        return vol

    def reduce_grad(self, grad):
        """Sum a replicated parameter's gradient over ranks (data-parallel retrieval)."""
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=self.group)
        return grad


def gd(f, y_local, model, coeffs=None, num_iterations=100, loss_fns=None, optim=tr.optim.Adam,
       progress_bar=False, device=None, **kwargs):
    """Data-parallel counterpart of retrieval.gd for a ShardedOperator (static grids).

    Every rank holds replicated coefficients and its own measurement shard ``y_local``.  Each
    iteration: local forward + local losses, backward, one all_reduce(sum) of the coefficient
    gradient, identical optimiser step everywhere.  Fidelity losses are weighted by the rank's
    share of the views so the summed gradient equals the single-GPU gradient of the full-stack
    mean; regulariser gradients are divided by the world size (every rank computes them).
    """
    from .loss import SquareLoss
    from .retrieval import detach_loss
    loss_fns = [SquareLoss()] if loss_fns is None else loss_fns
    share = (f.hi - f.lo) / f.n_obs
    if coeffs is None:
        coeffs = tr.ones(model.coeffs_shape, dtype=tr.float64, device=device or f.device)
    coeffs.requires_grad_()
    opt = optim([coeffs], **kwargs)
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
                dist.all_reduce(v, group=f.group)
            losses[fn].append(float(v))
        total.backward(retain_graph=True)
        f.reduce_grad(coeffs.grad)
        opt.step()
        if hasattr(model, 'proj'):
            coeffs.data = model.proj(coeffs)
    return coeffs, f.gather(f(model(coeffs))), losses
