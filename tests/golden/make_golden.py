"""Generate golden vectors from the real reference (this container only; needs /root/reference).

    python tests/golden/make_golden.py          # trace / forward / adjoint fixtures
    python tests/golden/make_golden.py pins     # dynamic gradients, multichannel, gd() run

Every case stores its INPUTS (grid boundaries, ray starts, ray directions as the reference
geometry produced them, densities, adjoint inputs) and the reference's OUTPUTS (non-zero trace
segments in ray order, forward line integrals in float64 and float32, the adjoint T(y)), so the
GPU tests never regenerate rays and never need the reference.  Files: tests/golden/<case>.npz.
"""
import os
import sys

import numpy as np
import torch as tr

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

R = refshim.load()
G, RT = R.geometry, R.raytracer


def segments_from_dense(regs, lens, grid_shape):
    """Reference (3, *rays, K) regs + (*rays, K) lens -> non-zero segments per ray (in order)."""
    nr, ne, na = grid_shape
    K = lens.shape[-1]
    regs = regs.reshape(3, -1, K).numpy()
    lens = lens.reshape(-1, K).numpy()
    keep = lens > 0
    ray_ptr = np.zeros(lens.shape[0] + 1, np.int64)
    ray_ptr[1:] = np.cumsum(keep.sum(1))
    r, e, a = (regs[i][keep] for i in range(3))
    vox = ((r * ne + e) * na + a).astype(np.int32)
    return ray_ptr, vox, lens[keep]


def orbit(n_obs, maker):
    geoms = []
    for th in tr.linspace(0, 2 * tr.pi, n_obs):
        geoms.append(maker((5 * tr.cos(th), 5 * tr.sin(th), 1)))
    return sum(geoms)


def grid_arrays(grid):
    return dict(r_b=grid.r_b.numpy(), e_b=grid.e_b.numpy(), a_b=grid.a_b.numpy(),
                shape=np.array(tuple(grid.shape)), dynamic=np.array(grid.dynamic))


def save_case(name, grid, geom, densities=(), ys=(), note='', keep_dense=False):
    tr.manual_seed(1234)
    xs = geom.ray_starts.clone()
    rays = geom.rays.clone()     # as the reference geometry produced them (before tracing)
    op = RT.Operator(grid, geom)
    gshape = tuple(grid.shape)[-3:]
    ray_ptr, vox, seglen = segments_from_dense(op.regs, op.lens, gshape)
    out = dict(grid_arrays(grid), xs=xs.numpy(), rays=rays.numpy(), ray_shape=np.array(op.lens.shape[:-1]),
               seg_ptr=ray_ptr, seg_vox=vox, seg_len=seglen, note=np.array(note))
    starts = RT.find_starts(grid, xs)
    out['starts'] = starts.numpy()
    for i, d in enumerate(densities):
        d64 = d.to(tr.float64)
        out[f'density{i}'] = d64.numpy()
        out[f'fwd64_{i}'] = op(d64).numpy()
        out[f'fwd32_{i}'] = op(d64.to(tr.float32)).numpy()
    for i, y in enumerate(ys):
        y64 = y.to(tr.float64)
        out[f'y{i}'] = y64.numpy()
        out[f'adj64_{i}'] = op.T(y64).numpy()
    if keep_dense:
        out['dense_regs'] = op.regs.numpy().astype(np.int32)
        out['dense_lens'] = op.lens.numpy()
    path = os.path.join(HERE, f'{name}.npz')
    np.savez_compressed(path, **out)
    print(f'{name}: rays={int(np.prod(op.lens.shape[:-1]))} K={op.lens.shape[-1]} '
          f'segments={len(vox)} -> {os.path.getsize(path) / 1e3:.0f} kB')


def solver_case():
    """Raw per-family solver outputs on random rays (bit-level check of the crossing solves)."""
    g = tr.Generator().manual_seed(7)
    n = 4000
    xs = (tr.rand(n, 3, generator=g, dtype=tr.float64) - 0.5) * 6
    xs[: n // 4] = (tr.rand(n // 4, 3, generator=g, dtype=tr.float64) - 0.5) * 1.2   # inside
    rays = tr.randn(n, 3, generator=g, dtype=tr.float64)
    rays /= tr.linalg.norm(rays, axis=-1)[..., None]
    r_b = tr.linspace(0, 1, 11, dtype=tr.float64)
    e_b = tr.linspace(0, tr.pi, 11, dtype=tr.float64)
    a_b = tr.linspace(-tr.pi, tr.pi, 11, dtype=tr.float64)
    out = dict(xs=xs.numpy(), rays=rays.numpy(), r_b=r_b.numpy(), e_b=e_b.numpy(),
               a_b=a_b.numpy())
    for key, fn, b in (('r', RT.r_torch, r_b), ('e', RT.e_torch, e_b), ('a', RT.a_torch, a_b)):
        t, reg, _, neg = fn(b, xs.clone(), rays.clone())
        out[f'{key}_t'] = t.numpy()
        out[f'{key}_reg'] = reg.numpy().astype(np.int32)
        out[f'{key}_neg'] = neg.numpy().astype(np.int8)
    path = os.path.join(HERE, 'solvers.npz')
    np.savez_compressed(path, **out)
    print(f'solvers: {n} rays -> {os.path.getsize(path) / 1e3:.0f} kB')


def save_grad_case(name, grid, geom, pairs, note=''):
    """Reference forward and autograd gradient of (op(x) * y).sum() for each (x, y) in `pairs`,
    float64 and float32 (the backward gd() runs: raytracer.py:705-712 through autograd), with the
    inputs (rays as the reference geometry produced them)."""
    xs, rays = geom.ray_starts.clone(), geom.rays.clone()
    op = RT.Operator(grid, geom)
    out = dict(grid_arrays(grid), xs=xs.numpy(), rays=rays.numpy(),
               ray_shape=np.array(op.lens.shape[:-1]), note=np.array(note))
    for i, (d, y) in enumerate(pairs):
        out[f'density{i}'] = d.to(tr.float64).numpy()
        out[f'gy{i}'] = y.to(tr.float64).numpy()
        for dt, tag in ((tr.float64, '64'), (tr.float32, '32')):
            x = d.to(dt).clone().requires_grad_()
            res = op(x)
            (res * y.to(dt)).sum().backward()
            out[f'fwd{tag}_{i}'] = res.detach().numpy()
            out[f'grad{tag}_{i}'] = x.grad.numpy()
    path = os.path.join(HERE, f'{name}.npz')
    np.savez_compressed(path, **out)
    print(f'{name}: rays={int(np.prod(op.lens.shape[:-1]))} pairs={len(pairs)} '
          f'-> {os.path.getsize(path) / 1e3:.0f} kB')


def gd_case(name='gd_circ16', n_iter=25, n=16, n_views=12, det=(20, 16)):
    """A reference gd() run: examples/static_retrieval.py's loop (FullyDenseModel, [SquareLoss(),
    NegRegularizer()], lr 0.1, the reference's default Adam: retrieval.py:84-116, loss.py:92-95,
    153-155) on a 16^3 grid seen by 12 ConeCirc views; stores the inputs, the measurement, every
    iteration's loss values and the final coefficients.  Also prints how far the same run moves
    when the measurement is perturbed by one ulp per value (the run's own rounding sensitivity,
    which bounds any two correct implementations' agreement)."""
    L, M, RET = R.loss, R.model, R.retrieval
    grid = G.SphericalGrid(shape=(n, n, n))
    geom = orbit(n_views, lambda p: G.ConeCircGeom(shape=det, pos=p, fov=(0, 45)))
    xs, rays = geom.ray_starts.clone(), geom.rays.clone()
    op = RT.Operator(grid, geom)
    truth = tr.zeros(grid.shape, dtype=tr.float64)
    h = n // 2
    truth[:, h:, :h] = 1
    truth[:, :h, h:] = 1
    meas = op(truth).detach()

    def run(y):
        fns = [L.SquareLoss(), L.NegRegularizer()]
        c, yres, losses = RET.gd(op, y.clone(), M.FullyDenseModel(grid), lr=1e-1,
                                 num_iterations=n_iter, loss_fns=fns, progress_bar=False)
        return c.detach(), yres.detach(), [np.array(losses[f]) for f in fns]

    coeffs, yres, (l_sq, l_neg) = run(meas)
    g = np.random.default_rng(1)
    m = meas.numpy()
    pert = np.where(g.random(m.shape) < 0.5, np.nextafter(m, np.inf), np.nextafter(m, -np.inf))
    c2, _, (s2, n2) = run(tr.from_numpy(pert))
    print(f'{name}: 1-ulp measurement perturbation moves coeffs by '
          f'{float((c2 - coeffs).abs().max()):.3g}, SquareLoss by '
          f'{float(np.max(np.abs(s2 - l_sq) / np.abs(l_sq))):.3g} rel, NegRegularizer by '
          f'{float(np.max(np.abs(n2 - l_neg))):.3g} abs')
    out = dict(grid_arrays(grid), xs=xs.numpy(), rays=rays.numpy(),
               ray_shape=np.array(op.lens.shape[:-1]), truth=truth.numpy(), meas=meas.numpy(),
               loss_sq=l_sq, loss_neg=l_neg, coeffs=coeffs.numpy(), y_result=yres.numpy(),
               lr=np.array(0.1), iterations=np.array(n_iter),
               note=np.array(f'reference gd(): {n}^3, {n_views} ConeCirc {det}, SquareLoss + '
                             f'NegRegularizer, Adam lr 0.1 (default implementation), {n_iter} '
                             'iterations'))
    path = os.path.join(HERE, f'{name}.npz')
    np.savez_compressed(path, **out)
    print(f'{name}: final SquareLoss {l_sq[-1]:.4g} (from {l_sq[0]:.4g}) -> '
          f'{os.path.getsize(path) / 1e3:.0f} kB')


def pins():
    """Fixtures pinning the rows the trace fixtures do not: the dynamic adjoint (autograd through
    the time-indexed gather), multichannel forwards, and a whole gd() retrieval."""
    g = tr.Generator().manual_seed(21)
    # dynamic: 6 views paired with 6 time slices (the dynamic_obs geometry) ...
    grid = G.SphericalGrid(shape=(6, 12, 10, 14))
    geom = orbit(6, lambda p: G.ConeCircGeom(shape=(16, 12), pos=p, fov=(0, 45)))
    save_grad_case('dynamic_grad', grid, geom,
                   [(tr.rand(grid.shape, generator=g, dtype=tr.float64),
                     tr.rand(geom.shape, generator=g, dtype=tr.float64))],
                   note='dynamic (6,12,10,14), 6 ConeCirc (16,12) views, view i <-> time i')
    # ... and one detector seen at every time step (t = arange(T)[:, None, None, None])
    grid = G.SphericalGrid(shape=(4, 12, 10, 14))
    geom = G.ConeRectGeom((18, 22), pos=(4, 2, 1.5), fov=(40, 40))
    save_grad_case('dynamic_single_grad', grid, geom,
                   [(tr.rand(grid.shape, generator=g, dtype=tr.float64),
                     tr.rand((4, 18, 22), generator=g, dtype=tr.float64))],
                   note='dynamic (4,12,10,14), one ConeRect (18,22): every time step, every ray')
    # multichannel static forwards: 3 channels, (2, 2) channels, and the preview3d shape
    # (plotting.py:280-297: one channel per azimuth rotation, (Na, Nr, Ne, Na))
    grid = G.SphericalGrid(shape=(12, 10, 14))
    geom = G.ConeRectGeom((24, 20), pos=(5, 0.3, 1), fov=(45, 45))
    pairs = [(tr.rand((C,) + tuple(grid.shape), generator=g, dtype=tr.float64),
              tr.rand(tuple(C) + tuple(geom.shape) if isinstance(C, tuple) else
                      (C,) + tuple(geom.shape), generator=g, dtype=tr.float64))
             for C in (3, 14)]
    pairs.append((tr.rand((2, 2) + tuple(grid.shape), generator=g, dtype=tr.float64),
                  tr.rand((2, 2) + tuple(geom.shape), generator=g, dtype=tr.float64)))
    save_grad_case('multichannel', grid, geom, pairs,
                   note='static (12,10,14), ConeRect (24,20); channels 3, 14 (preview3d), (2,2)')
    gd_case()


def save_api_case(name, grid, geom, densities=(), ys=(), note='', **op_kw):
    """An Operator(..., **op_kw) case (ftype=float32, invalid=True): inputs, the reference's dense
    (regs, lens) exactly as it returns them (lens in the trace's ftype, invalid entries kept), its
    forward on float32 and float64 densities and its adjoint T(y)."""
    xs, rays = geom.ray_starts.clone(), geom.rays.clone()
    op = RT.Operator(grid, geom, **op_kw)
    out = dict(grid_arrays(grid), xs=xs.numpy(), rays=rays.numpy(),
               ray_shape=np.array(op.lens.shape[:-1]), note=np.array(note),
               dense_regs=op.regs.numpy().astype(np.int32), dense_lens=op.lens.numpy())
    for i, d in enumerate(densities):
        out[f'density{i}'] = d.to(tr.float64).numpy()
        out[f'fwd64_{i}'] = op(d.to(tr.float64)).numpy()
        out[f'fwd32_{i}'] = op(d.to(tr.float32)).numpy()
    for i, y in enumerate(ys):
        out[f'y{i}'] = y.to(tr.float64).numpy()
        out[f'adj64_{i}'] = op.T(y.to(tr.float64)).numpy()
        try:   # (the reference's T raises for a float32 y on float64 lengths: index_put_ dtypes)
            out[f'adj32_{i}'] = op.T(y.to(tr.float32)).numpy()
        except RuntimeError as exc:
            out[f'adj32_{i}_error'] = np.array(str(exc))
    path = os.path.join(HERE, f'{name}.npz')
    np.savez_compressed(path, **out)
    lens = op.lens
    print(f'{name}: rays={int(np.prod(lens.shape[:-1]))} K={lens.shape[-1]} lens {lens.dtype} '
          f'finite non-zero {int((lens.isfinite() & (lens != 0)).sum())} nan '
          f'{int(lens.isnan().sum())} inf {int(lens.isinf().sum())} -> '
          f'{os.path.getsize(path) / 1e3:.0f} kB')


def api_surface():
    """Fixtures for the Operator options the GPU build once refused: ftype=float32 traces
    (raytracer.py:48-173 and the solvers in float32, isclose threshold 0.01), invalid=True (the
    un-masked lengths, raytracer.py:155-173), and ParallelGeom through ViewGeom (SURVEY App. C.2:
    the reference's own Operator raises on ParallelGeom's broadcast rays)."""
    g = tr.Generator().manual_seed(41)
    f32 = tr.float32
    # float32 solvers on random rays (as solvers.npz, ftype=float32)
    n = 3000
    xs = (tr.rand(n, 3, generator=g, dtype=tr.float64) - 0.5) * 6
    xs[: n // 4] = (tr.rand(n // 4, 3, generator=g, dtype=tr.float64) - 0.5) * 1.2
    rays = tr.randn(n, 3, generator=g, dtype=tr.float64)
    rays /= tr.linalg.norm(rays, axis=-1)[..., None]
    r_b = tr.linspace(0, 1, 11, dtype=tr.float64)
    e_b = tr.linspace(0, tr.pi, 11, dtype=tr.float64)
    a_b = tr.linspace(-tr.pi, tr.pi, 11, dtype=tr.float64)
    out = dict(xs=xs.numpy(), rays=rays.numpy(), r_b=r_b.numpy(), e_b=e_b.numpy(),
               a_b=a_b.numpy())
    for key, fn, b in (('r', RT.r_torch, r_b), ('e', RT.e_torch, e_b), ('a', RT.a_torch, a_b)):
        t, reg, _, neg = fn(b, xs.clone(), rays.clone(), ftype=f32)
        out[f'{key}_t'] = t.numpy()
        out[f'{key}_reg'] = reg.numpy().astype(np.int32)
        out[f'{key}_neg'] = neg.numpy().astype(np.int8)
    np.savez_compressed(os.path.join(HERE, 'solvers_f32.npz'), **out)
    print('solvers_f32: done')
    # float32 traces: a ConeRect view, a ConeCirc pair (ring 0 through the origin), inside starts
    grid = G.SphericalGrid(shape=(16, 14, 18))
    geom = G.ConeRectGeom((30, 40), pos=(5, 0.3, 1), fov=(45, 45))
    save_api_case('f32_rect', grid, geom, densities=[tr.rand(grid.shape, generator=g)],
                  ys=[tr.rand(geom.shape, generator=g, dtype=tr.float64)],
                  note='ftype=float32: 16x14x18, ConeRect (30,40)', ftype=f32)
    geom = orbit(2, lambda p: G.ConeCircGeom(shape=(24, 20), pos=p, fov=(0, 45)))
    save_api_case('f32_circ', grid, geom, densities=[tr.rand(grid.shape, generator=g)],
                  ys=[tr.rand(geom.shape, generator=g, dtype=tr.float64)],
                  note='ftype=float32: 16x14x18, 2 ConeCirc (24,20)', ftype=f32)
    grid = G.SphericalGrid(shape=(12, 10, 14))
    n = 2000
    xs = (tr.rand(n, 3, generator=g, dtype=tr.float64) - 0.5) * 1.6
    rays = tr.randn(n, 3, generator=g, dtype=tr.float64)
    save_api_case('f32_inside', grid, G.ViewGeom(xs, rays),
                  densities=[tr.rand(grid.shape, generator=g)],
                  ys=[tr.rand((n,), generator=g, dtype=tr.float64)],
                  note='ftype=float32: random starts in/around the unit grid', ftype=f32)
    # invalid=True: nothing masked (float64)
    grid = G.SphericalGrid(shape=(16, 14, 18))
    geom = G.ConeRectGeom((20, 24), pos=(5, 0.3, 1), fov=(45, 45))
    save_api_case('invalid_rect', grid, geom, densities=[tr.rand(grid.shape, generator=g)],
                  ys=[tr.rand(geom.shape, generator=g, dtype=tr.float64)],
                  note='invalid=True: 16x14x18, ConeRect (20,24)', invalid=True)
    grid = G.SphericalGrid(shape=(12, 10, 14))
    n = 1000
    xs = (tr.rand(n, 3, generator=g, dtype=tr.float64) - 0.5) * 1.6
    rays = tr.randn(n, 3, generator=g, dtype=tr.float64)
    save_api_case('invalid_inside', grid, G.ViewGeom(xs, rays),
                  densities=[tr.rand(grid.shape, generator=g)],
                  ys=[tr.rand((n,), generator=g, dtype=tr.float64)],
                  note='invalid=True: random starts in/around the unit grid', invalid=True)
    # ParallelGeom (geometry.py:607-655) through ViewGeom with the broadcast rays materialised
    grid = G.SphericalGrid(shape=(20, 18, 24))
    pg = G.ParallelGeom((30, 40), pos=(5, 0.5, 1), size=(2.2, 2.2))
    vg = G.ViewGeom(pg.ray_starts, pg.rays.expand(pg.ray_starts.shape).clone())
    save_case('parallel_geom', grid, vg, densities=[tr.rand(grid.shape, generator=g)],
              ys=[tr.rand(vg.shape, generator=g, dtype=tr.float64)],
              note='ParallelGeom (30,40) at (5,0.5,1), size 2.2: ViewGeom(ray_starts, rays '
                   'expanded) (SURVEY App. C.2)')


def main():
    tr.manual_seed(0)
    # C1: examples/single_vantage.py geometry at the BASELINE (50, 100) detector
    grid = G.SphericalGrid(shape=(50, 50, 50))
    geom = G.ConeRectGeom((50, 100), pos=(5, 0, 0), fov=(45, 45))
    shells = tr.zeros(grid.shape)
    shells[-1] += 1
    shells[-10] += 1
    save_case('c1_single_vantage', grid, geom,
              densities=[shells, tr.rand(grid.shape)], ys=[tr.rand(geom.shape, dtype=tr.float64)],
              note='C1 50^3, ConeRect (50,100) at (5,0,0)')

    # C2 subset: 3 orbit observations of the BASELINE config
    grid = G.SphericalGrid(shape=(50, 50, 50))
    geoms = [G.ConeRectGeom((50, 100), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(45, 45))
             for th in tr.linspace(0, 2 * tr.pi, 50)[[0, 17, 33]]]
    geom = sum(geoms)
    save_case('c2_orbit3', grid, geom, densities=[tr.rand(grid.shape)],
              ys=[tr.rand(geom.shape, dtype=tr.float64)], note='3 of the 50 C2 orbit views')

    # ConeCirc orbit (static_retrieval.py geometry, smaller detector); ring 0 passes the origin
    grid = G.SphericalGrid(shape=(24, 20, 28))
    geom = orbit(5, lambda p: G.ConeCircGeom(shape=(30, 24), pos=p, fov=(0, 45)))
    x = tr.zeros(grid.shape)
    x[:, 10:, :14] = 1
    x[:, :10, 14:] = 1
    save_case('circ_orbit', grid, geom, densities=[x, tr.rand(grid.shape)],
              ys=[tr.rand(geom.shape, dtype=tr.float64)], note='ConeCirc orbit, 24x20x28 grid')

    # starts inside the grid: behind-start integration in the start voxel
    g = tr.Generator().manual_seed(3)
    grid = G.SphericalGrid(shape=(12, 10, 14))
    n = 3000
    xs = (tr.rand(n, 3, generator=g, dtype=tr.float64) - 0.5) * 1.6
    rays = tr.randn(n, 3, generator=g, dtype=tr.float64)
    save_case('inside_starts', grid, G.ViewGeom(xs, rays), densities=[tr.rand(grid.shape)],
              ys=[tr.rand((n,), dtype=tr.float64)], note='random starts in/around the unit grid')

    # hollow / log-spaced / partial-angle grids with ConeRect views
    grid = G.SphericalGrid(shape=(10, 12, 16), size_r=(0.3, 1), size_e=(0, tr.pi / 2),
                           size_a=(-tr.pi / 2, tr.pi / 2))
    geom = orbit(3, lambda p: G.ConeRectGeom((24, 20), pos=p, fov=(40, 40)))
    save_case('partial_grid', grid, geom, densities=[tr.rand(grid.shape)],
              ys=[tr.rand(geom.shape, dtype=tr.float64)], note='hollow, hemisphere, half azimuth')

    grid = G.SphericalGrid(shape=(9, 11, 13), size_r=(0.1, 1), spacing='log',
                           size_a=(0, 2 * tr.pi))
    geom = orbit(3, lambda p: G.ConeRectGeom((20, 22), pos=p, fov=(45, 45)))
    save_case('log_grid', grid, geom, densities=[tr.rand(grid.shape)],
              ys=[tr.rand(geom.shape, dtype=tr.float64)], note='log radial, a in [0, 2pi] (no wrap)')

    # dynamic grid: T views paired with T time slices (dynamic_measurements.py shape, small)
    grid = G.SphericalGrid(shape=(6, 12, 10, 14))
    geom = orbit(6, lambda p: G.ConeCircGeom(shape=(16, 12), pos=p, fov=(0, 45)))
    x = tr.zeros(grid.shape)
    x[:, :, 5:, :7] = 1
    x[:, :, :5, 7:] = 1
    for t in range(6):
        x[t, :, (2 * t) % 10, :] += 1
    save_case('dynamic_obs', grid, geom, densities=[x, tr.rand(grid.shape)],
              note='dynamic (6,12,10,14), 6 ConeCirc views')

    # the reference's own operator tests (test_raytracer.py:8-60), dense outputs kept
    u = 0.001
    starts = [[-100, u, u], [u, -100, u], [u, u, -100], [-100, 0, u], [0, -100, u],
              [0, u, -100], [-100, u, 0], [u, -100, 0], [u, 0, -100], [5, 0, 0]]
    dirs = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0],
            [0, 1, 0], [0, 0, 1],
            [-0.99998629093170166016, 0.00413372274488210678, 0.00321511807851493359]]
    grids = [G.SphericalGrid(shape=(50, 50, 50), size_r=(3, 25)), G.SphericalGrid(shape=(4, 4, 4)),
             G.SphericalGrid(shape=(1, 4, 4)), G.SphericalGrid(shape=(4, 1, 4)),
             G.SphericalGrid(shape=(4, 4, 1))]
    for i, grid in enumerate(grids):
        save_case(f'optest_{i}', grid, G.ViewGeom(starts, dirs),
                  densities=[tr.ones(grid.shape), tr.rand(grid.shape)], keep_dense=True,
                  note='test_raytracer.py:8-60 rays')
    solver_case()


if __name__ == '__main__':
    # `make_golden.py`: the trace fixtures; `make_golden.py pins`: dynamic_grad,
    # dynamic_single_grad, multichannel, gd_circ16
    # `make_golden.py api`: solvers_f32, f32_*, invalid_*, parallel_geom;
    # `make_golden.py gd32`: gd_circ32 (32^3, 32 ConeCirc views, 20 iterations)
    arg = sys.argv[1:]
    if arg == ['pins']:
        pins()
    elif arg == ['api']:
        api_surface()
    elif arg == ['gd32']:
        gd_case('gd_circ32', n_iter=20, n=32, n_views=32, det=(50, 40))
    else:
        main()
