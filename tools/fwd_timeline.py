#!/usr/bin/env python3
"""Per-workgroup phase timeline of the forward kernel from a stamped diagnostic build.

    python tools/build_variants.py stamps=-DSPHRT_FWD_STAMPS
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_stamps.so python tools/fwd_timeline.py

Stamps (s_memrealtime, 100 MHz, wave 0 of each workgroup): 0 entry, 1 first window loaded and
masked, 2 granule DMA issued, 3 count scan done (granules landed), 4 segmented scan done, 5 exit.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c2']
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    x = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    out = torch.empty(op._csr['n'], device=dev)
    for _ in range(20):
        op._launch_forward(x, out, 1, 0)
    torch.cuda.synchronize()
    nb = min(op._csr['nblocks'], 1 << 17)
    lib = _lib.load()
    lib.sphrt_diag_fwd_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(8 * nb, dtype=np.uint64)
    assert lib.sphrt_diag_fwd_stamps(buf.ctypes.data_as(ctypes.c_void_p), 8 * nb) == 0
    st = buf.reshape(nb, 8)[:, :6].astype(np.int64)
    ok = (st > 0).all(1)
    st = st[ok]
    t0 = st[:, 0].min()
    ns = (st - t0) * 10.0            # 100 MHz -> ns
    rec = {'blocks': int(ok.sum()), 'kernel_span_us': float((ns[:, 5].max()) / 1e3)}
    for i, name in enumerate(['entry', 'loaded', 'dma_issued', 'count_scan', 'seg_scan', 'exit']):
        rec[name + '_us'] = {'min': float(ns[:, i].min() / 1e3), 'median': float(np.median(ns[:, i]) / 1e3),
                             'max': float(ns[:, i].max() / 1e3)}
    for i in range(1, 6):
        d = (ns[:, i] - ns[:, i - 1]) / 1e3
        rec[f'phase{i - 1}->{i}_us'] = {'median': float(np.median(d)), 'p90': float(np.percentile(d, 90)),
                                        'max': float(d.max())}
    blk = op._csr['blocks'].cpu().numpy().reshape(-1, _lib.BLOCK_FIELDS)[:nb][ok]
    rows = np.diff(np.append(blk[:, 4], op._csr['row_ray'].numel()))
    dur = ns[:, 5] - ns[:, 0]
    worst = np.argsort(-ns[:, 5])[:12]
    rec['slowest'] = [{'block': int(np.nonzero(ok)[0][i]), 'entry': float(ns[i, 0] / 1e3),
                       'exit': float(ns[i, 5] / 1e3), 'phases': [float(x) for x in np.diff(ns[i]) / 1e3],
                       'segs': int(blk[i, 3] - blk[i, 2]), 'n_tab': int(blk[i, 5]),
                       'empty': int(blk[i, 1] - blk[i, 0])} for i in worst]
    segs = blk[:, 3] - blk[:, 2]
    rec['corr_exit_vs_entry'] = float(np.corrcoef(ns[:, 0], ns[:, 5])[0, 1])
    rec['corr_dur_vs_segs'] = float(np.corrcoef(segs, dur)[0, 1])
    rec['corr_dur_vs_empty'] = float(np.corrcoef(blk[:, 1] - blk[:, 0], dur)[0, 1])
    rec['dur_us'] = {'median': float(np.median(dur) / 1e3), 'p90': float(np.percentile(dur, 90) / 1e3),
                     'max': float(dur.max() / 1e3)}
    print(json.dumps(rec, indent=1))


if __name__ == '__main__':
    main()
