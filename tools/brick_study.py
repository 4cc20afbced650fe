"""CPU study: distinct 16-B granules and 128-B lines per 1792-segment block under the natural
(r, e, a) layout and brick layouts, on views of the C3 / C5 traces (oracle trace)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from oracle import oracle  # noqa: E402
from sph_raytracer_amd.raytracer import find_starts  # noqa: E402


def brick_index(vox, shape, b):
    nr, ne, na = shape
    br, be, ba = b
    r = vox // (ne * na)
    e = (vox // na) % ne
    a = vox % na
    nbe, nba = ne // be, na // ba
    blk = ((r // br) * nbe + e // be) * nba + a // ba
    inner = ((r % br) * be + e % be) * ba + a % ba
    return blk * (br * be * ba) + inner


def study(cfg_name, views, seg_per_block=1792):
    cfg = bench.CONFIGS[cfg_name]
    grid, geom = bench.build_geometry(cfg, 0, 1)
    shape = tuple(grid.shape)
    g = oracle.Grid.from_boundaries(grid.r_b.numpy(), grid.e_b.numpy(), grid.a_b.numpy())
    xs_all = np.broadcast_to(geom.ray_starts.numpy(), geom.rays.shape)
    d_all = geom.rays.numpy()
    vox_list = []
    for v in views:
        xs = xs_all[v].reshape(-1, 3).copy()
        d = d_all[v].reshape(-1, 3).copy()
        ptr, vox, seg = oracle.trace_segments(g, xs, d, find_starts(grid, torch.from_numpy(xs)).numpy())
        vox_list.append(np.asarray(vox))
    vox = np.concatenate(vox_list).astype(np.int64)
    nb = len(vox) // seg_per_block
    print(cfg_name, shape, 'segments', len(vox), 'blocks', nb)
    layouts = {'natural': None}
    for b in [(1, 2, 2), (1, 1, 4), (2, 2, 8), (1, 4, 8), (2, 4, 4), (4, 4, 2), (2, 2, 2), (1, 2, 16)]:
        if all(s % x == 0 for s, x in zip(shape, b)):
            layouts[str(b)] = b
    for name, b in layouts.items():
        idx = vox if b is None else brick_index(vox, shape, b)
        gran, lines = [], []
        for k in range(nb):
            blk = idx[k * seg_per_block:(k + 1) * seg_per_block]
            gran.append(len(np.unique(blk >> 2)))
            lines.append(len(np.unique(blk >> 5)))
        print(f'  {name:12s} granules/block {np.mean(gran):7.1f}  lines/block {np.mean(lines):7.1f}')


if __name__ == '__main__':
    study('c3', [0, 40])
    study('c5', [0, 20])
    study('c2', [0, 20])
