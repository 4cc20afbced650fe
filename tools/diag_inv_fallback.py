"""Diagnostic (diagnostic build only): how many invalid=True rays of the C2 orbit leave the
register sort for the whole emulation.  The diagnostic build counts, in the trace workspace's head,
lists with an infinite distance (counter 3) and fallbacks (counter 2)."""
import sys
import torch as tr
sys.path.insert(0, '.')
import bench  # noqa: E402
from sph_raytracer_amd import raytracer as rt, Operator  # noqa: E402
cap = []
orig = rt._workspace


def ws(lib, plan, n, dev):
    t = orig(lib, plan, n, dev)
    cap.append(t)
    return t


rt._workspace = ws
grid, geom = bench.build_geometry(bench.CONFIGS['c2'], 0, 1)
op = Operator(grid, geom, device='cuda', invalid=True)
tr.cuda.synchronize()
head = cap[-1][:256].cpu().view(tr.int64).tolist()
print({'rays': int(geom.rays.shape[:-1].numel()), 'heap_rank': head[16], 'heap_sorted': head[17],
       'fallbacks': head[18], 'inf_lists': head[19], 'K': int(op._plan.K)})
