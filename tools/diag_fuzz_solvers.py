"""Diagnostic: the per-family crossing solves (r_torch / e_torch / a_torch on the GPU) against the
C oracle with IEEE sqrt on the fuzz cases of tests/test_gpu_fuzz.py: entries that differ and the
largest difference per family."""
import os
import sys
import numpy as np
import torch as tr
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import test_gpu_fuzz as fz  # noqa: E402
from oracle import oracle  # noqa: E402
from sph_raytracer_amd.raytracer import a_torch, e_torch, r_torch  # noqa: E402
oracle.use_mkl_sqrt(False)
for s in sys.argv[1:]:
    seed = int(s)
    r_b, e_b, a_b, xs, d = fz._case(seed)
    g = oracle.Grid.from_boundaries(r_b, e_b, a_b)
    out = {'seed': seed}
    for fam, (key, fn, b) in enumerate((('r', r_torch, r_b), ('e', e_torch, e_b), ('a', a_torch, a_b))):
        t, reg, _, neg = fn(tr.from_numpy(b), tr.from_numpy(xs), tr.from_numpy(d))
        ot, oreg, oneg = oracle.solve(g, fam, xs, d)
        t = t.numpy()
        same = (t == ot) | (np.isnan(t) & np.isnan(ot))
        fin = np.isfinite(t) & np.isfinite(ot)
        diff = np.abs(t - ot)[fin]
        out[key] = {'differ': int((~same).sum()), 'max_abs': float(diff.max()) if diff.size else 0.0,
                    'regions_differ': int((reg.numpy() != oreg).sum())}
        if (~same).any():
            i, j = np.argwhere(~same)[0]
            out[key]['first'] = [int(i), int(j), float(t[i, j]), float(ot[i, j]), float(b[j % len(b)])]
    print(out)
