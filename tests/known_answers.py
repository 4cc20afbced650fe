"""Known-answer vectors of the reference's solver unit tests (sph_raytracer/test_all.py:18-173).

Data only: (boundaries, ray starts, ray directions, expected distances, expected regions); an
expected-region entry of None means the reference asserts nothing about regions there.  The two
assertions the reference leaves as FIXME (test_all.py:119-128, 167-173) are left out, as there.
Compared with the reference's check(): float32 allclose, atol 1e-2.
"""
import math

INF = float('inf')
PI = math.pi
INV3 = 1 / math.sqrt(3)
D = 100

# r_torch (test_all.py:18-53)
R_CASES = [
    ((0.1, 1, 2), [(-3, 0, 0)], [(1, 0, 0)], [2.9, 2, 1, 3.1, 4, 5], [-1, 0, 1, 0, 1, -1]),
    ((0.1, 1, 2), [(-3, 0, 0)], [(-1, 0, 0)], [-3.1, -4, -5, -2.9, -2, -1], [-1, 0, 1, 0, 1, -1]),
    ((0.1, 1, 2), [(-3, 0, 0)], [(0, 0, 1)], 'inf', None),
    ((2,), [(-3, 2, 0), (-3, -2, 0), (-3, -2, 0)], [(1, 0, 0), (1, 0, 0), (-1, 0, 0)],
     [(3, 3), (3, 3), (-3, -3)], [(-1, -1), (-1, -1), (-1, -1)]),
    ((0,), [(-3, 0, 0)], [(1, 0, 0)], [3, 3], [-1, -1]),
]

# e_torch (test_all.py:56-128).  The reference builds its two-cone set as a float32 tensor,
# e = tr.tensor([pi/6, pi/4]) (test_all.py:57), and the single cones as Python lists (float64);
# e_boundaries() reproduces that rounding.
E_CASES = [
    (('f32', PI / 6, PI / 4), [(-1, 0, 0)], [(0, 0, 1)], [math.sqrt(3), 1, INF, INF], [-1, 0, -1, 0]),
    (('f32', PI / 6, PI / 4), [(-D, 0, 1)], [(1, 0, 0)], [D - INV3, D - 1, D + INV3, D + 1],
     [-1, 0, 0, -1]),
    (('pi-f32', PI / 6, PI / 4), [(-D, 0, -1)], [(1, 0, 0)], [D - INV3, D - 1, D + INV3, D + 1],
     [0, -1, -1, 0]),
    (('f32', PI / 6, PI / 4), [(-1, 0, -1)], [(1, 0, 0)], [INF] * 4, [0, -1, -1, 0]),
    (('f64', PI / 4), [(0, 0, 1)], [(1, 0, 1)], [-1 / math.sqrt(2), INF], [-1, -1]),
    (('f64', PI / 4), [(-1, 0, 1)], [(1, 0, -1)], [-INF, -INF], [-1, -1]),
    (('f64', PI / 4), [(1, 1, 1)], [(0, -1, 0)], [1, 1], [-2, -2]),
    (('f32', PI / 6, PI / 4), [(-1, 0, 0)], [(1, 0, 0)], [1, 1, 1, 1], None),
]


def e_boundaries(spec):
    """Cone angles as the reference test passes them to e_torch (as a float64 array)."""
    import numpy as np
    kind, *vals = spec
    if kind == 'f64':
        return np.asarray(vals, np.float64)
    e32 = np.asarray(vals, np.float32)
    if kind == 'pi-f32':             # tr.pi - e, computed in float32 (test_all.py:79)
        e32 = np.float32(PI) - e32
    return e32.astype(np.float64)

# a_torch (test_all.py:131-173)
A_CASES = [
    ((PI / 4, PI / 2), [(-1, 1, 0)], [(1, 0, 0)], [2, 1], [-1, 0]),
    ((PI / 4, PI / 2), [(-1, 1, 0)], [(-1, 0, 0)], [-2, -1], [0, -1]),
    ((PI / 4, PI / 2), [(-1, -1, 0)], [(1, 0, 0)], [INF, INF], None),
    ((0,), [(0, 1, 0)], [(1, 0, 0)], 'absinf', None),
    ((PI / 4, PI / 2), [(-1, 0, 0)], [(1, 0, 0)], [1, 1], [-1, 0]),
]

# find_starts (test_all.py:225-234): (grid shape, start, expected (r, e, a))
START_CASES = [
    ((5, 5, 1), [0, 0, 100], [-1, 0, 0]),
    ((5, 5, 1), [0, 0, -100], [-1, 4, 0]),
    ((5, 5, 5), [100, 0, 0], [-1, 2, 2]),
]
