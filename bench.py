#!/usr/bin/env python3
"""Benchmark: steady-state forward Operator throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5]
                    [--scaling weak|strong] [--no-cpu-baseline] [--no-strong-legs]

Workload (default, BASELINE configs[1] = SURVEY §8(d) C2): a (50,50,50) SphericalGrid seen by a
circular orbit of 50 ConeRectGeom((50,100), fov=(45,45)) views, 250,000 rays, float32 density.
A step is one ``op(x)`` forward call on the cached trace (the reference's Operator.__call__,
raytracer.py:692-713) — the drop-in call including its host overhead.  With N GPUs (one process
each, torchrun or this script's own launcher) every rank traces its own 50-view slice of a
50*N-view orbit (weak scaling); views are independent, so the step has no collective, and the
image stack is all-gathered over RCCL once after the loop.

Strong scaling (BASELINE configs[3] and [4] as defined): ``--scaling strong --config c4`` shards
ONE 50-view / 50-slice dynamic volume over the ranks (each rank its own time slices; a step is
its forward + dynamic gradient), ``--config c5`` times the static_retrieval.py gd loop with the
64 views sharded (one gradient all_reduce per iteration; a step is one iteration).  The default
C2 run reports both legs too (``strong``), each checked against one GPU over the whole orbit.

One JSON line on rank 0: value = rays/s over all ranks; roofline of the forward kernel
(algorithmic bytes per launch, and the bytes it must stream, over its mean duration back to back
in a HIP graph between HIP events — what the committed rocprofv3 trace's graph leg reports; the
dispatch-bound HIP events and the timed steps' span / K beside it); cpu_baseline = the reference's forward (torch CPU on the reference's padded trace,
oracle/ref_forward.py) on a bounded sample, timed on this host.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
METRIC = ('rays/sec (forward Operator) + peak GB resident, 50³ grid, 50×(50,100) sensor')

CONFIGS = {
    # name: (grid shape, views per GPU, detector, geometry kind, dtype, description)
    'c2': ((50, 50, 50), 50, (50, 100), 'rect', torch.float32,
           'C2: (50,50,50) grid, 50-view orbit x ConeRect (50,100), fp32 forward, trace cached'),
    'c1': ((50, 50, 50), 1, (50, 100), 'rect1', torch.float32,
           'C1: (50,50,50) grid, single ConeRect (50,100) view at (5,0,0), fp32 forward'),
    'c3': ((128, 128, 128), 128, (128, 256), 'rect', torch.float32,
           'C3: (128,128,128) grid, 128-view orbit x ConeRect (128,256), fp32 forward'),
    'c5': ((64, 64, 64), 64, (100, 50), 'circ', torch.float64,
           'C5: (64,64,64) grid, 64-view orbit x ConeCirc (100,50), fp64 forward'),
    # dynamic grid: view i sees time slice i (Operator(..., dynamic=True), raytracer.py:703-712)
    'c4': ((50, 50, 50, 50), 50, (100, 50), 'circ', torch.float32,
           'C4: dynamic (50,50,50,50) grid, 50-view orbit x ConeCirc (100,50), view i <-> time i, '
           'fp32 forward'),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_geometry(cfg, rank, world):
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, SphericalGrid
    shape, n_views, det, kind, _, _ = cfg
    grid = SphericalGrid(shape=shape)
    if kind == 'rect1':
        return grid, ConeRectGeom(det, pos=(5, 0, 0), fov=(45, 45))
    thetas = torch.linspace(0, 2 * torch.pi, n_views * world)[rank * n_views:(rank + 1) * n_views]
    geoms = []
    for th in thetas:
        pos = (5 * torch.cos(th), 5 * torch.sin(th), 1)
        if kind == 'rect':
            geoms.append(ConeRectGeom(det, pos=pos, fov=(45, 45)))
        else:
            geoms.append(ConeCircGeom(shape=det, pos=pos, fov=(0, 45)))
    return grid, sum(geoms)


def kernel_time_ms(op, x, reps=50):
    """Mean duration of the forward kernel: `reps` launches captured in one HIP graph, replayed
    between two HIP events on the launch stream (no host gaps)."""
    n_chan, div, _ = op._layout(x.shape)
    out = torch.empty(op._csr['n'], dtype=x.dtype, device=x.device)
    op._lengths(x.dtype)
    side = torch.cuda.Stream(device=x.device)
    side.wait_stream(torch.cuda.current_stream(x.device))
    try:
        with torch.cuda.stream(side):
            op._launch_forward(x, out, n_chan, div)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                for _ in range(reps):
                    op._launch_forward(x, out, n_chan, div)
            g.replay()
            torch.cuda.synchronize(x.device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            for _ in range(3):
                g.replay()
            e1.record(side)
        torch.cuda.synchronize(x.device)
        return e0.elapsed_time(e1) / (3 * reps), 'hip-graph replay, HIP events'
    except Exception as exc:   # capture unsupported: back-to-back launches, events around them
        log(f'graph capture failed ({exc}); timing back-to-back launches')
        torch.cuda.synchronize(x.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            op._launch_forward(x, out, n_chan, div)
        e1.record()
        torch.cuda.synchronize(x.device)
        return e0.elapsed_time(e1) / reps, 'back-to-back launches, HIP events'


def cpu_cold_baseline(cfg, sample_views):
    """The reference's cold path — Operator init (trace_indices, raytracer.py:48-230) + the first
    forward (:703-713) — restated in torch CPU (oracle/ref_trace.py: the same materialised
    solves, cat, sort, forward fill, diff and masks, calibrated bitwise and within +-20 % of the
    reference's wall time, profiles/r03_ref_trace_calibration.json) and timed on this host's
    cores on a bounded sample of the workload's views."""
    from oracle import ref_forward, ref_trace
    from sph_raytracer_amd.raytracer import find_starts
    shape, n_views, det, kind, dtype, _ = cfg
    grid, geom = _cpu_sample(cfg, sample_views)
    views = geom.rays.shape[0] if geom.rays.dim() == 4 else 1
    xs = geom.ray_starts.broadcast_to(geom.rays.shape).reshape(-1, 3).clone()
    rays = geom.rays.reshape(-1, 3).clone()
    dyn = grid.dynamic
    x = torch.rand((views,) + tuple(shape[1:]) if dyn else shape, dtype=dtype)
    t0 = time.perf_counter()
    starts = find_starts(grid, xs)
    regs, lens = ref_trace.trace_dense(grid.r_b, grid.e_b, grid.a_b, xs, rays, starts)
    hw = geom.rays.shape[-3:-1] if geom.rays.dim() >= 3 else ()
    regs = regs.reshape((3, views) + tuple(hw) + (-1,)) if dyn else regs
    lens = lens.reshape((views,) + tuple(hw) + (-1,)) if dyn else lens
    ref_forward.forward(regs, lens, x, dynamic=dyn)
    dt = time.perf_counter() - t0
    n = len(xs)
    return {'value': n / dt, 'unit': 'rays/s', 'seconds': dt, 'cores': torch.get_num_threads(),
            'kind': 'port',
            'sample': f'{views} of {n_views} views ({n} rays, K={lens.shape[-1]}): find_starts + '
                      f'trace_indices restated in torch CPU (oracle/ref_trace.py) + the '
                      f'reference forward, once (cold)'}


def _cpu_sample(cfg, sample_views):
    from sph_raytracer_amd import ConeRectGeom, ConeCircGeom, SphericalGrid
    shape, n_views, det, kind, dtype, _ = cfg
    grid = SphericalGrid(shape=shape)
    views = min(sample_views, n_views)
    if kind == 'rect1':
        return grid, ConeRectGeom(det, pos=(5, 0, 0), fov=(45, 45))
    # evenly spread over the orbit (views differ in hit fraction)
    idx = torch.linspace(0, n_views - 1, views).round().long()
    thetas = torch.linspace(0, 2 * torch.pi, n_views)[idx]
    mk = (lambda p: ConeRectGeom(det, pos=p, fov=(45, 45))) if kind.startswith('rect') else \
        (lambda p: ConeCircGeom(shape=det, pos=p, fov=(0, 45)))
    return grid, sum(mk((5 * torch.cos(t), 5 * torch.sin(t), 1)) for t in thetas)


def cpu_baseline(cfg, sample_views, reps):
    """Reference forward (torch CPU on the reference's padded trace) on a bounded sample."""
    from oracle import ref_forward
    from sph_raytracer_amd.raytracer import find_starts
    shape, n_views, det, kind, dtype, _ = cfg
    grid, geom = _cpu_sample(cfg, sample_views)
    views = geom.rays.shape[0] if geom.rays.dim() == 4 else 1
    xs, rays = geom.ray_starts, geom.rays
    starts = find_starts(grid, xs)
    t0 = time.perf_counter()
    regs, lens = ref_forward.dense_trace((grid.r_b, grid.e_b, grid.a_b), xs.numpy(), rays.numpy(),
                                         starts.numpy())
    t_trace = time.perf_counter() - t0
    dyn = grid.dynamic          # view i <-> time i: the sample's views take the first slices
    x = torch.rand((views,) + tuple(shape[1:]) if dyn else shape, dtype=dtype)
    ref_forward.forward(regs, lens, x, dynamic=dyn)           # warm-up
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ref_forward.forward(regs, lens, x, dynamic=dyn)
        times.append(time.perf_counter() - t0)
    n = lens.numel() // lens.shape[-1]
    med = sorted(times)[len(times) // 2]
    return {'value': n / med, 'unit': 'rays/s', 'cores': torch.get_num_threads(),
            'kind': 'port',
            'sample': f'{views} of {n_views} views ({n} rays, K={lens.shape[-1]}), reference '
                      f'forward (raytracer.py:703-713) in torch CPU on the padded trace, median '
                      f'of {reps}; padded trace built by the C oracle in {t_trace:.2f} s',
            'host_cpus': os.cpu_count()}


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


class _Ranks:
    """This process's place in the job: the process group (None at N=1), its GPU, and the
    collective helpers every leg shares (a barrier + device sync; the max of host floats over
    ranks)."""

    def __init__(self, dist, dev, world, rank):
        self.dist, self.dev, self.world, self.rank = dist, dev, world, rank

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()
        torch.cuda.synchronize(self.dev)

    def max_over_ranks(self, vals):
        if self.dist is None:
            return list(vals)
        on = self.dev if self.dist.get_backend() == 'nccl' else 'cpu'
        tt = torch.tensor(vals, dtype=torch.float64, device=on)
        self.dist.all_reduce(tt, op=self.dist.ReduceOp.MAX)
        return tt.tolist()

    def close(self):
        """The closing bracket of a timed region: device sync, then the barrier (with one rank the
        barrier is nothing, and a second idle synchronize would add ~2 µs to every region:
        profiles/r05_region_cost.json)."""
        torch.cuda.synchronize(self.dev)
        if self.dist is not None:
            self.dist.barrier()
            torch.cuda.synchronize(self.dev)

    def timed(self, fn, reps):
        """Run fn() `reps` times between barrier + sync brackets -> max seconds over ranks."""
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        self.close()
        return self.max_over_ranks([time.perf_counter() - t0])[0]


def strong_c4(rk, steps, warmup, check=True):
    """BASELINE configs[3], strong-scaled: ONE dynamic (50,50,50,50) volume seen by a 50-view
    ConeCirc (100,50) orbit with view i <-> time slice i (examples/dynamic_measurements.py:18-48,
    raytracer.py:703-712), its 50 views and their time slices sharded over the ranks (7,7,6,...
    at N=8: SURVEY §8(e)) through ShardedOperator.  A step is this rank's forward of its slices
    plus its gradient of 0.5*||A x - m||^2 (the residual, then the dynamic adjoint through the
    time-paired transposed CSR): no communication inside the step, every rank owns disjoint
    slices.  The image stack is all-gathered once after the loop.  Outside the timed region every
    rank checks the gathered stack and the gathered gradient against a single-GPU Operator of the
    whole orbit (the same rays; float32 sums grouped by other workgroup blocks: ~1e-7)."""
    from sph_raytracer_amd import Operator
    cfg = CONFIGS['c4']
    grid, geom = build_geometry(cfg, 0, 1)          # the whole orbit, on every rank
    g = torch.Generator().manual_seed(4)
    x = torch.rand(tuple(grid.shape), dtype=torch.float32, generator=g).to(rk.dev)
    m = torch.rand(tuple(geom.shape), dtype=torch.float32, generator=g).to(rk.dev)
    n_views = int(geom.shape[0])
    rk.barrier()
    t0 = time.perf_counter()
    if rk.dist is None:
        op = Operator(grid, geom, device=rk.dev, dynamic=True)
        lo, hi, sop = 0, n_views, None
        fwd = op
        dshape = tuple(x.shape)

        def adj(r):
            return op._apply_adjoint(r, dshape, r.dtype, r.device)
    else:
        from sph_raytracer_amd.distributed import ShardedOperator
        sop = ShardedOperator(grid, geom, device=rk.dev, dynamic=True)
        op, lo, hi = sop.local, sop.lo, sop.hi
        fwd, adj = sop, sop.T_local
    y0 = fwd(x)
    torch.cuda.synchronize(rk.dev)
    t_op = time.perf_counter() - t0
    m_loc = m[lo:hi]

    def step():
        r = fwd(x)
        r.sub_(m_loc)
        return adj(r)

    for _ in range(max(warmup, 2)):     # (the first adjoint builds the time-paired transpose)
        grad = step()
    dt = rk.timed(step, steps)
    t_op, = rk.max_over_ranks([t_op])
    out = {'workload': 'C4 strong: ONE dynamic (50,50,50,50) volume, 50-view ConeCirc (100,50) '
                       'orbit, view i <-> time i; views/slices sharded over the ranks',
           'scaling': 'strong', 'rays': int(math.prod(geom.shape)), 'views': n_views,
           'views_this_rank': hi - lo, 'steps': steps, 'ms_per_step': dt / steps * 1e3,
           'rays_per_s': math.prod(geom.shape) * steps / dt,
           'operator_first_forward_ms': t_op * 1e3,
           'what': 'step = forward of this rank\'s time slices + the gradient of '
                   '0.5*||A x - m||^2 for them (residual, dynamic adjoint); float32'}
    grad = step()
    y_loc = fwd(x)
    if sop is not None:
        rk.barrier()
        t0 = time.perf_counter()
        stack = sop.gather(y_loc)
        torch.cuda.synchronize(rk.dev)
        out['final_gather_ms'] = rk.max_over_ranks([time.perf_counter() - t0])[0] * 1e3
        out['backend'] = rk.dist.get_backend()
        g_full = sop._all_gather_rows(grad.reshape(hi - lo, -1), ()).reshape(x.shape)
    else:
        stack, g_full = y_loc, grad
    out['stack_shape'] = list(stack.shape)
    if check:       # against one GPU over the whole orbit (outside the timed region)
        single = Operator(grid, geom, device=rk.dev, dynamic=True)
        ys = single(x)
        gs = single._apply_adjoint(ys - m, tuple(x.shape), x.dtype, x.device)
        out['stack_rel_diff_vs_1gpu'] = _rel(stack, ys)
        out['grad_rel_diff_vs_1gpu'] = _rel(g_full, gs)
        out['matches_1gpu'] = bool(out['stack_rel_diff_vs_1gpu'] <= 1e-5 and
                                   out['grad_rel_diff_vs_1gpu'] <= 1e-5)
        del single
    out['_op'], out['_x'] = op, (x[lo:hi] if sop is not None else x)
    del y0
    return out


C5_ITERATIONS = 100     # examples/static_retrieval.py:57


def strong_c5(rk, iterations, check=True):
    """BASELINE configs[4], strong-scaled: the static_retrieval.py loop (examples/
    static_retrieval.py:42-57, retrieval.py:88-120) on C5 (64^3 grid, 64-view ConeCirc (100,50)
    orbit; FullyDenseModel, SquareLoss + NegRegularizer, Adam lr 0.1, float64 coefficients), the
    64 views sharded over the ranks: distributed.gd, i.e. per iteration the local forward, the
    residual, the local adjoint, one all_reduce(sum) of the 64^3 gradient (RCCL), the identical
    Adam step on every rank.  Timed: one whole gd call of `iterations` iterations (plan set-up,
    the final forward and the stack's all-gather included), after a 3-iteration warm-up call.
    Checked (outside the timing) against retrieval.gd on one GPU over the whole orbit with the
    same gathered measurements: only the gradient's summation order differs."""
    from sph_raytracer_amd import Operator, retrieval
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    cfg = CONFIGS['c5']
    grid, geom = build_geometry(cfg, 0, 1)
    truth = torch.zeros(tuple(grid.shape), dtype=torch.float64, device=rk.dev)
    truth[:, 32:, :32] = 1                       # static_retrieval.py:22-24 at 64^3
    truth[:, :32, 32:] = 1
    model = FullyDenseModel(grid)
    rk.barrier()
    t0 = time.perf_counter()
    if rk.dist is None:
        op = sop = Operator(grid, geom, device=rk.dev)
        y_loc = op(truth)

        def run(k):
            return retrieval.gd(op, y_loc.clone(), model, num_iterations=k, lr=1e-1,
                                loss_fns=[SquareLoss(), NegRegularizer()], progress_bar=False)
    else:
        from sph_raytracer_amd.distributed import ShardedOperator, gd as dgd
        sop = ShardedOperator(grid, geom, device=rk.dev)
        op = sop.local
        y_loc = sop(truth)

        def run(k):
            return dgd(sop, y_loc.clone(), model, num_iterations=k, lr=1e-1,
                       loss_fns=[SquareLoss(), NegRegularizer()])
    torch.cuda.synchronize(rk.dev)
    t_op = time.perf_counter() - t0
    run(3)                          # warm-up: the transposed CSR, the kernels' first launches
    rk.barrier()
    res = []
    dt = rk.timed(lambda: res.append(run(iterations)), 1)
    t1 = rk.timed(lambda: run(1), 1)
    t_op, = rk.max_over_ranks([t_op])
    coeffs, stack, losses = res[0]
    fid = losses[next(iter(losses))]
    n_rays = int(math.prod(geom.shape))
    out = {'workload': 'C5 strong: static_retrieval.py loop, (64,64,64) grid, 64-view ConeCirc '
                       '(100,50) orbit, FullyDenseModel, SquareLoss + NegRegularizer, Adam lr 0.1, '
                       'f64; views sharded over the ranks, one gradient all_reduce per iteration',
           'scaling': 'strong', 'rays': n_rays, 'views': int(geom.shape[0]),
           'views_this_rank': int(y_loc.shape[0]), 'iterations': iterations,
           'ms_per_iteration': dt / iterations * 1e3,
           'ms_per_iteration_marginal': (dt - t1) / max(iterations - 1, 1) * 1e3,
           'gd_call_ms': dt * 1e3, 'gd_1_iteration_call_ms': t1 * 1e3,
           'rays_per_s': n_rays * iterations / dt,
           'operator_first_forward_ms': t_op * 1e3,
           'fidelity_first': fid[0], 'fidelity_last': fid[-1],
           'what': 'one gd call of `iterations` iterations (forward + residual + adjoint + '
                   'gradient all_reduce + Adam each), plan set-up and final forward/all-gather '
                   'included; marginal = (t(K) - t(1)) / (K - 1)'}
    if rk.dist is not None:
        out['backend'] = rk.dist.get_backend()
    if check and rk.dist is not None:    # (at N=1 the timed run is the single-GPU loop itself)
        single = Operator(grid, geom, device=rk.dev)
        fns = [SquareLoss(), NegRegularizer()]
        c1, _, l1 = retrieval.gd(single, sop.gather(y_loc), model, num_iterations=iterations,
                                 lr=1e-1, loss_fns=fns, progress_bar=False)
        a, b = torch.tensor(fid), torch.tensor(l1[fns[0]])
        out['coeffs_max_abs_diff_vs_1gpu'] = float((coeffs - c1).abs().max())
        out['sqloss_max_rel_diff_vs_1gpu'] = float(((a - b).abs() / b.abs()).max())
        out['matches_1gpu'] = bool(out['coeffs_max_abs_diff_vs_1gpu'] <= 1e-9 and
                                   out['sqloss_max_rel_diff_vs_1gpu'] <= 1e-9)
        del single
    out['_op'], out['_x'] = op, truth
    return out


def _public(leg):
    return {k: v for k, v in leg.items() if not k.startswith('_')}


def kernel_dispatch_ms(op, x, reps):
    """Mean duration of the forward kernel over `reps` back-to-back launches on the launch stream,
    each launch's own dispatch bracketed by a pair of HIP events (sphrt_time_next_forward:
    hipExtLaunchKernelGGL binds the events to the kernel's start and end) — the kernel's duration
    as rocprofv3's kernel trace reports it, whatever the host's issue rate (a timed region's span
    / K also counts the gaps between launches, and under the profiler the host can fall behind
    the GPU).  -> (mean ms, median ms)."""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    n_chan, div, _ = op._layout(x.shape)
    out = torch.empty(op._csr['n'] * (n_chan if div == 0 else 1), dtype=x.dtype, device=x.device)
    op._lengths(x.dtype)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:            # (torch creates the HIP events on their first record)
        a.record()
        b.record()
    torch.cuda.synchronize(x.device)
    try:
        for a, b in evs:
            _lib.check(lib.sphrt_time_next_forward(ctypes.c_void_p(a.cuda_event),
                                                   ctypes.c_void_p(b.cuda_event)),
                       'sphrt_time_next_forward')
            op._launch_forward(x, out, n_chan, div)
    finally:
        lib.sphrt_time_next_forward(None, None)
    torch.cuda.synchronize(x.device)
    d = sorted(a.elapsed_time(b) for a, b in evs)
    return sum(d) / len(d), d[len(d) // 2]


def must_move_bytes(op, x):
    """Bytes the forward kernel must stream from HBM per launch, beside
    SURVEY §8(d)'s algorithmic count: per segment its 2-byte granule slot (`loc`; 4-byte `vox`
    for the per-segment gather modes) and its length in the density's precision; the granule
    table entries its workgroups read (sum of n_tab over blocks, the tables' entry width); the
    row metadata (48-byte block records, plus 128-byte run records or 4 B of row / empty-ray list
    per ray); the outputs; the density once per resident copy (the distinct granules the tables
    name, at most the whole array).  Density re-reads served by L2/MALL are not counted: this is
    the floor a kernel could reach at full HBM bandwidth."""
    n_chan, div, _ = op._layout(x.shape)
    desc, k_chan, cs, k_div = op._launch_args(x, n_chan, div)
    es = x.element_size()
    csr = op._csr
    n, total = csr['n'], csr['total']
    blocks = csr['blocks']
    if div > 0:
        rec = op._paired(x.shape[0], div)
        if rec is not None:
            blocks = rec['keep'][1]
    table = bool(desc.loc) and bool(desc.tab) and desc.tab_stride > 0 and k_div == 0
    n_tab = int(blocks.view(-1, 6)[:, 5].sum()) if table else 0
    seg = total * ((2 if table else 4) + es)
    tabs = n_tab * int(desc.tab_bytes)
    meta = desc.n_blocks * 48 + (desc.n_blocks * 128 if desc.runs else 4 * n)
    outs = n * es * (k_chan if k_div == 0 else 1)
    cols = desc.stage_cols if desc.stage_shape[0] > 0 else desc.n_cols
    dens = k_chan * es * (min(cols, 4 * n_tab) if table else cols)
    return {'bytes': seg + tabs + meta + outs + dens, 'segments': seg, 'tables': tabs,
            'metadata': meta, 'outputs': outs, 'density_once': dens}


def _pmc_traffic(op, x, config, kname):
    """HBM traffic per launch of the newest committed rocprofv3 --pmc record of this kernel and
    config (profiles/rNN_forward_<config>_pmc.json), when it was taken on the same CSR: records
    carry their ray and segment counts (round 6 on); a record without them is taken to be the
    single-GPU config, so a shard (a strong-scaled rank) of another size gets none."""
    for tag in ('r06', 'r05', 'r04', 'r03', 'r02', 'r01'):
        pmc = os.path.join(ROOT, 'profiles', f'{tag}_forward_{config}_pmc.json')
        if not os.path.exists(pmc):
            continue
        rec = json.load(open(pmc))
        if rec.get('kernel') != kname or rec.get('config') != config:
            continue
        if 'segments' in rec:
            same = rec['segments'] == op._csr['total'] and rec.get('rays') == op._csr['n']
        else:
            full = CONFIGS[config]
            same = op._csr['n'] == math.prod(full[2]) * full[1]
        if not same:
            return None, f'{os.path.relpath(pmc, ROOT)} was taken on another CSR (not this shard)'
        return rec['traffic_bytes_per_launch'], os.path.relpath(pmc, ROOT)
    return None, None


def roofline(op, x, config, k_ms, k_method):
    """The forward kernel's roofline.  achieved = ALGORITHMIC bytes per launch (SURVEY §8(d):
    s_y + 4 + S*(4 + s_len + s_rho) per ray; f32 path s_len = s_rho = 4) over its mean launch
    duration `k_ms`; `must_move` = the same over the bytes the kernel must stream (must_move_bytes);
    `traffic` = HBM bytes per launch of the committed PMC record of this kernel on this CSR.
    SURVEY's basis counts every density gather as HBM although the volume is L2-resident, so it
    can exceed the peak where gathers repeat (C5: the view tiles); must_move cannot."""
    kname = op._forward_kernel_name(x)
    traffic, traffic_src = _pmc_traffic(op, x, config, kname)
    es = x.element_size()
    n_chan, div, _ = op._layout(x.shape)
    n_out = n_chan if div == 0 else 1
    alg_bytes = op._csr['n'] * n_out * (es + 4) + op._csr['total'] * n_out * (4 + es + es)
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    mm = must_move_bytes(op, x)
    mm_gbs = mm['bytes'] / (k_ms * 1e-3) / 1e9
    mm.update({'achieved': mm_gbs, 'frac': mm_gbs / HBM_PEAK_GBS})
    return {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
            'achieved_basis': 'algorithmic bytes (SURVEY 8(d): s_y + 4 + S*(4 + s_len + '
                              's_rho) per ray; density gathers counted as HBM)',
            'must_move': mm,
            'traffic_gbs': traffic / (k_ms * 1e-3) / 1e9 if traffic else None,
            'traffic_frac': traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
            'traffic_source': traffic_src, 'kernel': kname,
            'kernel_ms': k_ms, 'bytes_per_launch': alg_bytes, 'timing': k_method}


def strong_legs(rk, steps, warmup):
    """The strong-scaled C4 and C5 legs the default run reports beside its headline, so that
    every `bench.py --gpus N` run (the driver's N = 1, 2, 4, 8 scaling runs included) also
    records BASELINE configs[3] and configs[4] as they are defined.  A leg that raises is
    reported as its error (identically on every rank: the legs issue the same collectives)."""
    legs = {}
    for name, fn in (('c4', lambda: strong_c4(rk, max(steps, 20), warmup)),
                     ('c5_retrieval', lambda: strong_c5(rk, C5_ITERATIONS))):
        try:
            legs[name] = _public(fn())
        except Exception as exc:      # informative legs: never lose the headline line to them
            log(f'strong leg {name} failed: {exc!r}')
            legs[name] = {'error': repr(exc)}
        torch.cuda.empty_cache()
    return legs


def strong_main(args, rk):
    """`--scaling strong --config c4|c5`: the JSON line's value is the strong-scaled leg's
    rays/s (C4: forward + dynamic gradient steps; C5: gd iterations, each a forward and an
    adjoint of all 320,000 rays), over all ranks."""
    cfg = CONFIGS[args.config]
    torch.cuda.reset_peak_memory_stats(rk.dev)
    if args.config == 'c4':
        leg = strong_c4(rk, args.steps, args.warmup)
        ms, dtype = leg['ms_per_step'], torch.float32
    else:
        leg = strong_c5(rk, args.steps)
        ms, dtype = leg['ms_per_iteration'], torch.float64
    peak_gb = torch.cuda.max_memory_allocated(rk.dev) / 1e9
    op, x = leg['_op'], leg['_x']
    k_ms, k_method = kernel_time_ms(op, x, reps=50)
    k_disp, k_med = kernel_dispatch_ms(op, x, reps=max(args.steps, 50))
    rec = {
        'metric': METRIC,
        'value': leg['rays_per_s'],
        'unit': 'rays/s',
        'n_gpus': rk.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms,
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'f32' if dtype == torch.float32 else 'f64',
        'data': 'synthetic (torch.rand density / the static_retrieval.py phantom, reference '
                'geometry)',
        'config': {'workload': leg['workload'], 'grid': list(cfg[0]), 'views': leg['views'],
                   'detector': list(cfg[2]), 'rays': leg['rays'],
                   'views_this_rank': leg['views_this_rank'],
                   'parallelism': f'obs/time-sharded x{rk.world} (strong)'},
        'peak_gb_resident': peak_gb,
        'strong': _public(leg),
        'roofline': roofline(op, x, args.config, k_ms, k_method),
    }
    rec['roofline']['kernel_ms_dispatch_events'] = k_disp
    rec['roofline']['kernel_ms_dispatch_events_median'] = k_med
    rec['roofline']['scope'] = 'this rank\'s local forward kernel'
    if rk.rank == 0 and rk.world == 1 and not args.no_cpu_baseline:
        try:
            rec['cpu_baseline'] = cpu_baseline(cfg, args.cpu_sample_views, args.cpu_reps)
            rec['cpu_baseline']['scope'] = 'the forward only'
        except Exception as exc:
            rec['cpu_baseline'] = {'value': None, 'error': repr(exc)}
    else:
        rec['cpu_baseline'] = None
    if rk.rank == 0:
        print(json.dumps(rec), flush=True)


def spawn_ranks(n):
    """Run this script as `n` child ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one
    GPU each), as torch.distributed.run would; rank 0 prints the JSON line.  Returns the exit
    status: non-zero as soon as any rank fails (the others are then stopped).  The parent never
    initialises the GPU (torch.cuda.device_count() does not, on this image)."""
    import socket
    import subprocess
    one_dev = os.environ.get('SPHRT_BENCH_ONE_DEVICE') == '1'
    have = torch.cuda.device_count()
    if not one_dev and have < n:
        log(f'bench.py --gpus {n}: only {have} GPU(s) visible; run on a node with {n} GPUs '
            f'(or set SPHRT_BENCH_ONE_DEVICE=1 to rehearse {n} gloo ranks on cuda:0)')
        return 2
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        if one_dev:
            env.setdefault('SPHRT_BENCH_BACKEND', 'gloo')   # one device cannot hold 2 RCCL ranks
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    status = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                rc = p.poll()
                if rc is None:
                    continue
                pending.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 1
                    log(f'bench.py: rank {procs.index(p)} exited with {rc}; stopping the others')
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='c2', choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample-views', type=int, default=10)
    ap.add_argument('--cpu-reps', type=int, default=10)
    ap.add_argument('--cpu-cold-views', type=int, default=None,
                    help='views of the cold CPU sample (default: 10, C3: 2)')
    ap.add_argument('--scaling', default='weak', choices=('weak', 'strong'),
                    help='weak (default): every rank its own views of a views*N orbit; strong '
                         '(c4, c5): ONE workload sharded over the ranks (c4: forward + dynamic '
                         'gradient per step; c5: the static_retrieval.py gd loop, one step = one '
                         'iteration)')
    ap.add_argument('--no-strong-legs', action='store_true',
                    help='skip the strong-scaled C4 / C5 legs the default run reports beside '
                         'the headline')
    args = ap.parse_args()
    if args.scaling == 'strong' and args.config not in ('c4', 'c5'):
        ap.error('--scaling strong is defined for --config c4 and c5')

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks here, before this
        # process touches the GPU (a process that has initialised HIP must never be replaced)
        sys.exit(spawn_ranks(args.gpus))

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.gpus != world:
        log(f'note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE')
    # rehearsal knobs for a one-GPU box (never set by the driver): all ranks on cuda:0, gloo
    same_dev = os.environ.get('SPHRT_BENCH_ONE_DEVICE') == '1'
    dev = torch.device('cuda', 0 if same_dev else local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get('SPHRT_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    from sph_raytracer_amd import Operator, build
    build.build()
    cfg = CONFIGS[args.config]
    shape, n_views, det, kind, dtype, desc = cfg
    torch.manual_seed(0)
    rk = _Ranks(dist, dev, world, rank)
    barrier, max_over_ranks = rk.barrier, rk.max_over_ranks
    if args.scaling == 'strong':
        strong_main(args, rk)
        if dist is not None:
            dist.destroy_process_group()
        return

    # ---- cold: geometry + trace + first forward ----------------------------------------------
    torch.cuda.reset_peak_memory_stats(dev)
    barrier()
    t0 = time.perf_counter()
    if dist is None:
        grid, geom = build_geometry(cfg, 0, 1)
        sop = op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    else:   # every rank sees the whole 50*N-view orbit and keeps its contiguous 50-view shard
        from sph_raytracer_amd.distributed import ShardedOperator
        grid, geom = build_geometry((shape, n_views * world) + cfg[2:], 0, 1)
        sop = ShardedOperator(grid, geom, device=dev)
        op = sop.local
    x = torch.rand(shape, dtype=dtype, device=dev)
    y = op(x)
    torch.cuda.synchronize(dev)
    t_cold = time.perf_counter() - t0
    n_rays = op._csr['n']
    total_seg = op._csr['total']

    def step():
        # one forward Operator call on this rank's shard of views: the path has no exchange step
        # (views are independent), so no collective inside the step (weak scaling)
        return op(x)

    for _ in range(args.warmup):
        step()
    # HIP events on the launch stream (the current stream: op(x) launches there) bracket the
    # timed steps: their span / K is the forward's average launch duration over the timed region
    # (it includes the short gaps between back-to-back launches)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ev1.record()
    rk.close()
    dt = time.perf_counter() - t0
    k_ms_timed = ev0.elapsed_time(ev1) / args.steps
    # the forward kernel's own duration over K more launches, each dispatch bracketed by its HIP
    # event pair
    k_ms_disp, k_med_disp = kernel_dispatch_ms(op, x, args.steps)
    gather = None
    if dist is not None:
        dt, t_cold = max_over_ranks([dt, t_cold])
        # the final image stack: one RCCL all-gather over xGMI, after the loop (north_star), timed
        # on its own; the gathered stack is checked against this rank's own shard
        y_loc = op(x)
        barrier()
        t0 = time.perf_counter()
        full = sop.gather(y_loc)
        torch.cuda.synchronize(dev)
        t_g = time.perf_counter() - t0
        t_g, = max_over_ranks([t_g])
        ok = bool(torch.equal(full[sop.lo:sop.hi], y_loc))
        gather = {'ms': t_g * 1e3, 'bytes': full.numel() * full.element_size(),
                  'stack_shape': list(full.shape), 'matches_local_shard': ok,
                  'backend': dist.get_backend(),
                  'what': 'one all-gather of the image stack after the timed loop (RCCL '
                          'all_gather_into_tensor; gloo rehearsals: host-staged)'}
    peak_gb = torch.cuda.max_memory_allocated(dev) / 1e9

    # cold path again in a warm process (the reference's 34k rays/s was also taken after
    # warm-up): new geometry objects + Operator (trace) + first forward
    colds, op_colds = [], []
    for _ in range(3):
        barrier()
        t0 = time.perf_counter()
        grid2, geom2 = build_geometry(cfg, rank, world)
        t1 = time.perf_counter()
        op2 = Operator(grid2, geom2, device=dev, dynamic=grid2.dynamic)
        op2(x)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        colds.append(t2 - t0)
        op_colds.append(t2 - t1)     # the reference's cold: Operator init + first call
        del op2
    t_warm_cold = sorted(colds)[1]
    t_op_cold = sorted(op_colds)[1]
    if dist is not None:
        t_warm_cold, t_op_cold = max_over_ranks([t_warm_cold, t_op_cold])

    # drop-in use with host tensors (the reference's device='cpu' default): H2D density, D2H image
    x_host = x.cpu()
    for _ in range(3):
        op(x_host)
    t0 = time.perf_counter()
    reps_h = 20
    for _ in range(reps_h):
        op(x_host)
    t_host = (time.perf_counter() - t0) / reps_h

    k_reps = 50
    adj_steps = min(args.steps, 50)      # the adjoint leg below
    k_ms_graph, _ = kernel_time_ms(op, x, reps=k_reps)
    # launch order of the forward kernel in this process, for tools/rocprof_legs.py (splits a
    # rocprofv3 kernel trace of this command into these legs)
    log('legs ' + json.dumps([['first', 1], ['warmup', args.warmup], ['steps', args.steps],
                              ['dispatch', args.steps]] +
                             ([['final_gather_fwd', 1]] if dist is not None else []) +
                             [['cold', 3], ['pcie', 3 + reps_h], ['graph', 1 + 4 * k_reps]] +
                             [['adjoint', 3 + adj_steps]]))
    # the adjoint (op.T, static grids; BASELINE configs[2] is a forward + adjoint run): the
    # transposed CSR is built by the first call (untimed), then `adj_steps` calls are timed
    adjoint = None
    if grid.dynamic:
        # the dynamic gradient (the autograd backward of raytracer.py:710, which
        # the reference's Operator.T refuses): the time-paired transposed CSR through the same
        # table kernel, built by the first of 3 untimed calls
        y_adj = torch.rand(tuple(op.geom.shape), dtype=dtype, device=dev)
        dshape = tuple(x.shape)

        def adj_step():
            return op._apply_adjoint(y_adj, dshape, dtype, dev)
        for _ in range(3):
            adj_step()
        t_adj = rk.timed(adj_step, adj_steps) / adj_steps
        n_vox = math.prod(shape)
        adj_bytes = n_vox * (x.element_size() + 4) + total_seg * (4 + 2 * x.element_size())
        adjoint = {'ms_per_step': t_adj * 1e3, 'rays_per_s': n_rays * world / t_adj,
                   'alg_GBps_per_gpu': adj_bytes / t_adj / 1e9, 'steps': adj_steps,
                   'what': 'dynamic gradient: the adjoint of the view <-> time pairing (the '
                           'time-paired CSR transposed once, then the same table kernel); '
                           'per-step wall time incl. launch; bytes as SURVEY 8(d) with voxels '
                           '(T x vol) as rows'}
    if not grid.dynamic:
        y_adj = torch.rand(tuple(op.geom.shape), dtype=dtype, device=dev)
        for _ in range(3):
            op.T(y_adj)
        barrier()
        t0 = time.perf_counter()
        for _ in range(adj_steps):
            op.T(y_adj)
        rk.close()
        t_adj = (time.perf_counter() - t0) / adj_steps
        if dist is not None:
            t_adj, = max_over_ranks([t_adj])
        n_vox = math.prod(shape[-3:])
        adj_bytes = n_vox * (x.element_size() + 4) + total_seg * (4 + 2 * x.element_size())
        adjoint = {'ms_per_step': t_adj * 1e3, 'rays_per_s': n_rays * world / t_adj,
                   'alg_GBps_per_gpu': adj_bytes / t_adj / 1e9, 'steps': adj_steps,
                   'what': 'op.T(y), y = torch.rand(geom.shape): the transposed CSR (built by the '
                           'first of 3 untimed calls) through the same table kernel; per-step '
                           'wall time incl. launch; bytes as SURVEY 8(d) with voxels as rows'}
    # the roofline's denominator: the kernel back to back in a HIP graph (no host issue between
    # launches) between HIP events on its stream — the quantity the committed rocprofv3 trace
    # of this command reports for its graph leg (tools/rocprof_legs.py: C2 5.88 against 5.88 us,
    # profiles/r06_bench_c2_rocprof_legs.json); launches under the profiler's per-dispatch
    # interception read 10-15 % longer, so the dispatch-bound events are reported beside it
    roof = roofline(op, x, args.config, k_ms_graph,
                    f'HIP-graph replay of {k_reps} launches x 3 between HIP events on the launch '
                    f'stream (the rocprofv3 graph leg)')
    roof['kernel_ms_graph_replay'] = k_ms_graph
    # each launch's own dispatch bracketed by HIP events (sphrt_time_next_forward), K launches
    roof['kernel_ms_dispatch_events'] = k_ms_disp
    roof['kernel_ms_dispatch_events_median'] = k_med_disp
    roof['frac_dispatch_events'] = roof['bytes_per_launch'] / (k_ms_disp * 1e-3) / 1e9 / HBM_PEAK_GBS
    # the timed steps' span / K on the launch stream (kernel + the gaps between launches)
    roof['kernel_ms_timed_span'] = k_ms_timed
    roof['frac_timed_span'] = roof['bytes_per_launch'] / (k_ms_timed * 1e-3) / 1e9 / HBM_PEAK_GBS

    rec = {
        'metric': METRIC,
        'value': n_rays * world * args.steps / dt,
        'unit': 'rays/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': dt / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32' if dtype == torch.float32 else 'f64',
        'data': 'synthetic (torch.rand density, reference geometry)',
        'config': {'workload': desc, 'grid': list(shape), 'views_per_gpu': n_views,
                   'detector': list(det), 'rays_per_gpu': n_rays, 'segments_per_gpu': total_seg,
                   'parallelism': f'obs-sharded x{world}' + (' (final stack: one RCCL all-gather)' if world > 1 else '')},
        'peak_gb_resident': peak_gb,
        'final_gather': gather,
        'adjoint': adjoint,
        'pcie_inclusive': {'rays_per_s': n_rays / t_host, 'ms_per_call': t_host * 1e3,
                           'what': 'op(x) with x and the result in host memory (per rank)'},
        'cold': {'rays_per_s': n_rays * world / t_warm_cold, 'seconds': t_warm_cold,
                 'operator_rays_per_s': n_rays * world / t_op_cold, 'operator_seconds': t_op_cold,
                 'first_in_process_seconds': t_cold,
                 'what': 'geometry + Operator trace + first forward (median of 3, warm process; '
                         'operator_*: Operator init + first forward only, the reference\'s cold '
                         'definition; first_in_process includes HIP/torch initialisation)'},
        'roofline': roof,
    }
    if not args.no_strong_legs and args.config == 'c2':
        rec['strong'] = strong_legs(rk, args.steps, args.warmup)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            rec['cpu_baseline'] = cpu_baseline(cfg, args.cpu_sample_views, args.cpu_reps)
        except Exception as exc:   # the baseline is informative; never fail the GPU bench on it
            rec['cpu_baseline'] = {'value': None, 'error': repr(exc)}
        try:
            cold_views = args.cpu_cold_views or (2 if args.config == 'c3' else 10)
            cold = cpu_cold_baseline(cfg, cold_views)
            cold['gpu_ratio'] = rec['cold']['operator_rays_per_s'] / cold['value']
            rec['cpu_baseline']['cold'] = cold
        except Exception as exc:
            rec['cpu_baseline']['cold'] = {'value': None, 'error': repr(exc)}
    else:
        rec['cpu_baseline'] = None
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
