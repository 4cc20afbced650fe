#!/usr/bin/env python3
"""Multichannel forward timing: one launch over C = 1 and 8 channels (f32, f64) on the C2 and C5
workloads, HIP-event graph replay (prof_forward.graph_time_us).

    python tools/multichannel_time.py
"""
import os, sys, json
import torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tools'))
import bench
from prof_forward import graph_time_us
from sph_raytracer_amd import Operator
dev = torch.device('cuda', 0)
for cname in ('c2', 'c5'):
    cfg = bench.CONFIGS[cname]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    op = Operator(grid, geom, device=dev)
    n = op._csr['n']
    for C in (1, 8):
        for dt in (torch.float32, torch.float64):
            x = torch.rand((C,) + tuple(cfg[0]), dtype=dt, device=dev)
            out = torch.empty(C * n, dtype=dt, device=dev)
            op(x)
            t = graph_time_us(lambda: op._launch_forward(x, out, C, 0), 20)
            print(json.dumps({'config': cname, 'channels': C, 'dtype': str(dt), 'us': round(t, 1), 'us_per_channel': round(t / C, 2)}))
