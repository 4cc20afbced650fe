import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['SPHRT_TCOLS'] = 'trace'
from sph_raytracer_amd import Operator, SphericalGrid, ConeRectGeom
from sph_raytracer_amd.raytracer import _gather
dev = torch.device('cuda', 0)
grid = SphericalGrid(shape=(40, 36, 44))
th = torch.linspace(0, 2 * torch.pi, 16)
geom = sum(ConeRectGeom((30, 40), pos=(5 * torch.cos(t), 5 * torch.sin(t), 1), fov=(45, 45)) for t in th)
op = Operator(grid, geom, device=dev)
y = torch.rand(tuple(geom.shape), dtype=torch.float64, device=dev)
rid = op._csr['ray_id']
print('rid', rid.dtype, rid.shape, rid.is_contiguous(), rid.min().item(), rid.max().item())
g1 = _gather(y.reshape(-1), rid, op._csr['n'], dev)
g2 = y.reshape(-1).index_select(0, rid.long())
print('gather eq', torch.equal(g1, g2), (g1 - g2).abs().max().item())
a0 = op.T(y); a1 = op.T(y); a2 = op.T(y)
print('a0 a1', torch.equal(a0, a1), (a0 - a1).abs().max().item(), torch.equal(a1, a2))
x = torch.rand(tuple(grid.shape), dtype=torch.float64, device=dev)
lhs = float((op(x) * y).sum())
print('dot', lhs, float((x * a0).sum()), float((x * a1).sum()))
op2 = Operator(grid, geom, device=dev)
b0 = op2.T(y.clone()); b1 = op2.T(y)
print('op2', torch.equal(b0, b1), float((x * b0).sum()), float((x * b1).sum()))
os.environ['SPHRT_TCOLS'] = 'geom'
op3 = Operator(grid, geom, device=dev)
c0 = op3.T(y); print('geom', float((x * c0).sum()))
