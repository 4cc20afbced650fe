import sys, json, torch
sys.path.insert(0, '.')
import bench
from sph_raytracer_amd import Operator
dev = torch.device('cuda', 0)
for c in ('c2', 'c3', 'c5'):
    grid, geom = bench.build_geometry(bench.CONFIGS[c], 0, 1)
    op = Operator(grid, geom, device=dev)
    cs = op._csr; d = cs['desc']
    nt = cs['blocks'].view(-1, 6)[:, 5].double()
    print(json.dumps({'config': c, 'nblocks': cs['nblocks'], 'total': cs['total'], 'tab_bytes': d.tab_bytes, 'tab_stride': d.tab_stride,
                      'n_tab_mean': float(nt[nt >= 0].mean()), 'n_tab_max': float(nt.max()), 'fallback': int((nt < 0).sum()),
                      'table_MB': float(nt[nt >= 0].sum()) * d.tab_bytes / 1e6, 'stage': list(d.stage_brick)}))
