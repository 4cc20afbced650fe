#!/usr/bin/env python3
"""Time the forward-kernel ablation stages (tools/fwd_ablate.hip) on a bench workload.

    python tools/fwd_ablate.py [--config c2]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
ABL = os.path.join(ROOT, 'sph_raytracer_amd', 'lib', 'variants', 'libablate.so')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--stages', default='0,1,2,3,8,9,10,11,12,13,14,4,5,6,7')
    ap.add_argument('--rounds', type=int, default=2)
    args = ap.parse_args()
    import bench
    from prof_forward import graph_time_us
    from sph_raytracer_amd import Operator, _lib
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    x = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    o = torch.empty(op._csr['n'], dtype=torch.float32, device=dev)
    op._launch_forward(x, o, 1, 0)
    abl = ctypes.CDLL(ABL)
    abl.sphrt_ablate.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p]
    sink = torch.empty(op._csr['nblocks'] * 256, dtype=torch.float32, device=dev)
    desc = ctypes.addressof(op._csr['desc'])
    tag = os.path.basename(os.environ.get('SPHRT_LIB', 'libsphrt.so'))
    for _round in range(args.rounds):
        for stage in [int(x) for x in args.stages.split(',')]:
            desc_c = op._csr['desc']
            if stage == 6:
                fn = lambda: op._launch_forward(x, o, 1, 0)  # noqa: E731
            elif stage == 7:
                def fn():
                    keep = (desc_c.loc, desc_c.tab)
                    desc_c.loc, desc_c.tab = None, None
                    op._launch_forward(x, o, 1, 0)
                    desc_c.loc, desc_c.tab = keep
            else:
                def fn(s=stage):
                    assert abl.sphrt_ablate(s, desc, x.data_ptr(), sink.data_ptr(),
                                            _lib.stream_of(dev)) == 0
            print(json.dumps({'lib': tag, 'stage': stage, 'us': graph_time_us(fn, args.reps)}),
                  flush=True)


if __name__ == '__main__':
    main()
