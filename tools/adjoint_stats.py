#!/usr/bin/env python3
"""Statistics of an operator's adjoint CSR (the transposed CSR; a dynamic grid's time-paired
one) and the per-launch durations of its kernels, from HIP events bound to each dispatch.

    python tools/adjoint_stats.py [--config c4] [--reps 50]

Prints one JSON line: rows, empty rows, segments, blocks, granule-table stride and entries,
dense-range sizes, forward / adjoint kernel means (us) and the adjoint's per-call gather of y.
"""
import argparse
import ctypes
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dispatch_us(fn, reps, lib):
    """Mean / median duration (us) of the forward kernel `fn` launches, dispatch-bound events."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        b.record()
    torch.cuda.synchronize()
    for a, b in evs:
        lib.sphrt_time_next_forward(ctypes.c_void_p(a.cuda_event), ctypes.c_void_p(b.cuda_event))
        fn()
    lib.sphrt_time_next_forward(None, None)
    torch.cuda.synchronize()
    d = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return sum(d) / len(d), d[len(d) // 2]


def events_us(fn, reps):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c4')
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--or-order', type=int, default=0,
                    help='bits OR-ed into the adjoint CSR\'s order (block-order hints) before timing')
    args = ap.parse_args()
    import bench
    from sph_raytracer_amd import Operator, _lib
    from sph_raytracer_amd.raytracer import _call_forward
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev, dynamic=grid.dynamic)
    x = torch.rand(cfg[0], dtype=cfg[4], device=dev)
    y = torch.rand(tuple(geom.shape), dtype=cfg[4], device=dev)
    op(x)
    op._apply_adjoint(y, tuple(x.shape), x.dtype, dev)
    n_chan, div, _ = op._layout(x.shape)
    tr_rec = op._paired(x.shape[0], div)['transposed'] if div else op._transposed()
    c = tr_rec['desc']
    c.order |= args.or_order
    keep = tr_rec['keep']
    col_ptr, blocks = keep[0], keep[6]
    b = blocks.view(-1, 6)
    rows_nz = int((col_ptr[1:] > col_ptr[:-1]).sum())
    rec = {'config': args.config, 'rows': int(c.n_rays), 'rows_nonempty': rows_nz,
           'segments': int(c.n_segments), 'blocks': int(c.n_blocks),
           'tab_stride': int(c.tab_stride), 'tab_bytes': int(c.tab_bytes),
           'n_tab_sum': int(b[:, 5].clamp_min(0).sum()), 'n_fallback': int(c.n_fallback),
           'order': int(c.order), 'runs': bool(c.runs), 'n_cols': int(c.n_cols),
           'adjoint_kernel': op._adjoint_kernel_name(x)}
    if c.order & 4:
        span = (b[:, 1] - b[:, 0]).float()
        rec['dense_range_mean'] = float(span.mean())
        rec['dense_range_p99'] = float(span.quantile(0.99))
        rec['dense_range_max'] = float(span.max())
        rec['dense_ranges_over_stage'] = int((span > 2048).sum())
    seg = (b[:, 3] - b[:, 2]).clamp_min(0)
    rec['segments_per_row'] = rec['segments'] / max(rows_nz, 1)
    out = torch.empty(op._csr['n'], dtype=x.dtype, device=dev)
    res = torch.empty(math.prod(x.shape), dtype=x.dtype, device=dev)
    yv = y.reshape(-1)
    if op._csr['ray_id'] is not None and not op._tcols_geom():
        yv = yv.index_select(0, op._ray_id_long())
    fn = lib.sphrt_forward_f32 if x.dtype == torch.float32 else lib.sphrt_forward_f64
    rec['forward_us'] = dispatch_us(lambda: op._launch_forward(x, out, n_chan, div), args.reps,
                                    lib)
    rec['adjoint_kernel_us'] = dispatch_us(
        lambda: _call_forward(fn, c, yv, 1, op._csr['n'], 0, res, res.numel(), dev), args.reps, lib)
    rid = op._ray_id_long() if op._csr['ray_id'] is not None else None
    if rid is not None:
        from sph_raytracer_amd.raytracer import _gather
        rec['index_select_y_us_events'] = events_us(lambda: y.reshape(-1).index_select(0, rid),
                                                    args.reps)
        rec['gather_y_us_events'] = events_us(
            lambda: _gather(y.reshape(-1), op._csr['ray_id'], op._csr['n'], dev), args.reps)
    rec['adjoint_call_us_events'] = events_us(
        lambda: op._apply_adjoint(y, tuple(x.shape), x.dtype, dev), args.reps)
    rec['forward_call_us_events'] = events_us(lambda: op(x), args.reps)
    rec['env'] = {k: v for k, v in os.environ.items() if k.startswith('SPHRT_')}
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
