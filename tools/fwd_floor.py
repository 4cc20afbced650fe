#!/usr/bin/env python3
"""Floors of the C2 forward (tools/fwd_floor.hip, same grid as forward_kernel): an empty launch,
the per-segment byte stream alone, and stream + one store per ray, against the product kernel,
all graph-replayed back to back (so each includes the dependent-launch boundary).

    python tools/fwd_floor.py [--config c2]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
LIB = os.path.join(ROOT, 'sph_raytracer_amd', 'lib', 'variants', 'libfloor.so')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=50)
    args = ap.parse_args()
    if not os.path.exists(LIB):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared',
                        os.path.join(ROOT, 'tools', 'fwd_floor.hip'), '-o', LIB], check=True)
    import bench
    from prof_forward import graph_time_us
    from sph_raytracer_amd import Operator
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    x = torch.rand(cfg[0], dtype=torch.float32, device=dev)
    c = op._csr
    o = torch.empty(c['n'], dtype=torch.float32, device=dev)
    op._launch_forward(x, o, 1, 0)
    lib = ctypes.CDLL(LIB)
    lib.sphrt_floor.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 3 + \
        [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    d = c['desc']
    res = {'config': args.config, 'blocks': c['nblocks']}
    for stage, name in ((0, 'empty'), (1, 'segment_stream'), (2, 'stream_and_store')):
        def fn(stage=stage):
            lib.sphrt_floor(stage, d.loc, d.len32, d.tab, c['total'], d.tab_stride, c['nblocks'],
                            o.data_ptr(), c['n'], torch.cuda.current_stream().cuda_stream)
        res[name + '_us'] = graph_time_us(fn, args.reps)
    res['product_us'] = graph_time_us(lambda: op._launch_forward(x, o, 1, 0), args.reps)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
