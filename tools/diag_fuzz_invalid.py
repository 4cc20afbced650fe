"""Diagnostic: the GPU's invalid=True CSR for the fuzz cases of tests/test_gpu_fuzz.py (seeds
given on the command line), saved as npz under gpurun_out/ for a comparison on the host."""
import os
import sys
import numpy as np
import torch as tr
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import test_gpu_fuzz as fz  # noqa: E402
from sph_raytracer_amd import Operator, SphericalGrid, ViewGeom  # noqa: E402
os.makedirs(os.path.join(ROOT, 'gpurun_out', 'r06'), exist_ok=True)
for s in sys.argv[1:]:
    seed = int(s)
    r_b, e_b, a_b, xs, d = fz._case(seed)
    grid = SphericalGrid(r_b=tr.from_numpy(r_b), e_b=tr.from_numpy(e_b), a_b=tr.from_numpy(a_b))
    op = Operator(grid, ViewGeom(tr.from_numpy(xs), tr.from_numpy(d)), device='cuda', invalid=True)
    ptr, vox, seg = (t.cpu().numpy() for t in op.segments())
    np.savez(os.path.join(ROOT, 'gpurun_out', 'r06', f'fuzz_invalid_{seed}.npz'), ptr=ptr, vox=vox,
             seg=seg)
    print(seed, len(vox))
