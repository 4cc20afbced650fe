"""Python handle on the CPU oracle (oracle/sphrt_oracle.c) — TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
or as the timed CPU baseline; never by the product package.  All arrays are numpy, host memory.

    grid = oracle.Grid.from_boundaries(r_b, e_b, a_b)
    ptr, vox, seg = oracle.trace_segments(grid, xs, rays, starts)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')

_lib = None


def build(force=False):
    srcs = [os.path.join(HERE, f) for f in ('sphrt_oracle.c', 'sphrt_oracle_body.inc')]
    if force or not os.path.exists(LIB) or \
            os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(['make', '-s', '-C', HERE], check=True, capture_output=True)
    return LIB


class Grid(ctypes.Structure):
    _fields_ = [('nr', ctypes.c_int), ('ne', ctypes.c_int), ('na', ctypes.c_int),
                ('r_b', ctypes.c_void_p), ('e_b', ctypes.c_void_p), ('a_b', ctypes.c_void_p),
                ('cos_e', ctypes.c_void_p), ('cos2_e', ctypes.c_void_p),
                ('cos_a', ctypes.c_void_p), ('sin_a', ctypes.c_void_p),
                ('a_wrap', ctypes.c_int), ('th', ctypes.c_double), ('par', ctypes.c_double)]

    @classmethod
    def from_boundaries(cls, r_b, e_b, a_b, ftype='float64'):
        """Boundary tables as the reference computes them: tr.asarray(b, ftype) and torch CPU
        trig in that dtype (raytracer.py:277,361,373,501,505).  ftype 'float32' selects the
        float32 solvers / trace (ora_*_f32); the tables travel as float64 (exact)."""
        import torch as tr
        dt = {'float64': tr.float64, 'float32': tr.float32}[str(ftype).replace('torch.', '')]
        rb, eb, ab = (tr.as_tensor(np.asarray(b, np.float64)).to(dt) for b in (r_b, e_b, a_b))
        keep = [np.ascontiguousarray(x.numpy(), np.float64) for x in
                (rb, eb, ab, tr.cos(eb), tr.cos(eb) ** 2, tr.cos(ab), tr.sin(ab))]
        g = cls()
        g.f32 = dt == tr.float32
        g._keep = keep
        g.nr, g.ne, g.na = len(keep[0]) - 1, len(keep[1]) - 1, len(keep[2]) - 1
        (g.r_b, g.e_b, g.a_b, g.cos_e, g.cos2_e, g.cos_a, g.sin_a) = (k.ctypes.data for k in keep)
        g.a_wrap = int(bool(-ab[0] == ab[-1] == tr.pi))
        res = float(np.finfo(np.float32 if g.f32 else np.float64).resolution)
        g.th = res ** (1 / 3)
        g.par = res
        return g

    @property
    def K(self):
        return 2 * (self.nr + 1) + 2 * (self.ne + 1) + (self.na + 1) + 1


def load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        I, N = ctypes.c_int, ctypes.c_int64
        lib.ora_set_sqrt.argtypes = [P]
        lib.ora_set_sqrt_f32.argtypes = [P]
        lib.ora_introsort.argtypes = [P, P, I]
        for sfx in ('', '_f32'):
            getattr(lib, 'ora_solve' + sfx).argtypes = [ctypes.POINTER(Grid), I, P, P, N, P, P, P]
            getattr(lib, 'ora_trace_dense' + sfx).argtypes = [ctypes.POINTER(Grid), P, P, P, N, I,
                                                              I, P, P]
            getattr(lib, 'ora_trace_segments' + sfx).argtypes = [ctypes.POINTER(Grid), P, P, P, N,
                                                                 I, I, P, P, P, P]
        _lib = lib
    return _lib


def use_mkl_sqrt(enable=True):
    """Bind the oracle's sqrt to MKL vdSqrt / vsSqrt from libtorch_cpu.so (what torch.sqrt runs
    on CPU for float64 / float32 tensors), making crossing distances bit-identical to the
    reference.  Returns False if unavailable."""
    lib = load()
    if not enable:
        lib.ora_set_sqrt(None)
        lib.ora_set_sqrt_f32(None)
        return True
    try:
        import torch
        tl = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), 'lib', 'libtorch_cpu.so'))
        fd, fs = tl.vdSqrt, tl.vsSqrt
    except (OSError, AttributeError):
        return False
    lib.ora_set_sqrt(ctypes.cast(fd, ctypes.c_void_p))
    lib.ora_set_sqrt_f32(ctypes.cast(fs, ctypes.c_void_p))
    return True


def _fn(grid, name):
    return getattr(load(), name + ('_f32' if getattr(grid, 'f32', False) else ''))


def _c(a, dt):
    return np.ascontiguousarray(a, dt)


def rays_flat(xs, rays):
    """Broadcast starts and directions like raytracer.py:76-80 -> (shape, xs (n,3), rays (n,3))."""
    xs, rays = np.asarray(xs, np.float64), np.asarray(rays, np.float64)
    shape = np.broadcast_shapes(xs.shape, rays.shape)
    return shape[:-1], _c(np.broadcast_to(xs, shape).reshape(-1, 3), np.float64), \
        _c(np.broadcast_to(rays, shape).reshape(-1, 3), np.float64)


def introsort(values):
    """libstdc++ std::sort of (value, index) pairs by value -> (sorted values, permutation)."""
    t = _c(values, np.float64).copy()
    idx = np.zeros(len(t), np.int32)
    load().ora_introsort(t.ctypes.data, idx.ctypes.data, len(t))
    return t, idx


def solve(grid, family, xs, rays):
    """Per-family crossings (r_torch / e_torch / a_torch semantics): t (in the grid's ftype),
    region, negative."""
    shape, x, d = rays_flat(xs, rays)
    n = len(x)
    w = 2 * (grid.nr + 1) if family == 0 else 2 * (grid.ne + 1) if family == 1 else grid.na + 1
    t = np.empty((n, w), np.float32 if getattr(grid, 'f32', False) else np.float64)
    reg = np.empty((n, w), np.int32)
    neg = np.empty((n, w), np.int8)
    _fn(grid, 'ora_solve')(ctypes.byref(grid), family, x.ctypes.data, d.ctypes.data, n,
                           t.ctypes.data, reg.ctypes.data, neg.ctypes.data)
    return t.reshape(shape + (w,)), reg.reshape(shape + (w,)), neg.reshape(shape + (w,))


def _starts(starts, n):
    s = _c(np.asarray(starts).reshape(3, -1).T, np.int32)
    if len(s) != n:
        s = _c(np.broadcast_to(s, (n, 3)), np.int32)
    return s


def _fresh(grid, fresh):
    # the oracle's rays are float64: a float32 trace copies them per solver (raytracer.py:276)
    return int(getattr(grid, 'f32', False) if fresh is None else fresh)


def trace_dense(grid, xs, rays, starts, invalid=False, fresh=None):
    """Reference-layout trace: regs (3, *rays, K) int32, lens (*rays, K) (float32 grids: float32
    values as float64).  `starts` is the (3, *rays) start-voxel array (find_starts); invalid=True
    leaves the lengths unmasked (raytracer.py:155); fresh: each solver normalises its own copy of
    the rays (default: float32 grids — float64 rays are copied by tr.asarray)."""
    shape, x, d = rays_flat(xs, rays)
    n, K = len(x), grid.K
    s = _starts(np.broadcast_to(np.asarray(starts), (3,) + shape), n)
    regs = np.empty((n, 3, K), np.int32)
    lens = np.empty((n, K), np.float64)
    _fn(grid, 'ora_trace_dense')(ctypes.byref(grid), x.ctypes.data, d.ctypes.data, s.ctypes.data,
                                 n, int(invalid), _fresh(grid, fresh), regs.ctypes.data,
                                 lens.ctypes.data)
    return np.moveaxis(regs, 1, 0).reshape((3,) + shape + (K,)), lens.reshape(shape + (K,))


def trace_segments(grid, xs, rays, starts, invalid=False, fresh=None):
    """Non-zero segments per ray in sorted order: (row_ptr (n+1,), vox int32, len float64).
    invalid=True: every non-zero length, inf / NaN included, negative regions wrapped."""
    shape, x, d = rays_flat(xs, rays)
    n = len(x)
    s = _starts(np.broadcast_to(np.asarray(starts), (3,) + shape), n)
    fn = _fn(grid, 'ora_trace_segments')
    counts = np.empty(n, np.int32)
    fresh = _fresh(grid, fresh)
    fn(ctypes.byref(grid), x.ctypes.data, d.ctypes.data, s.ctypes.data, n, int(invalid), fresh,
       None, counts.ctypes.data, None, None)
    ptr = np.zeros(n + 1, np.int64)
    ptr[1:] = np.cumsum(counts)
    vox = np.empty(max(int(ptr[-1]), 1), np.int32)
    seg = np.empty(max(int(ptr[-1]), 1), np.float64)
    fn(ctypes.byref(grid), x.ctypes.data, d.ctypes.data, s.ctypes.data, n, int(invalid), fresh,
       ptr.ctypes.data, None, vox.ctypes.data, seg.ctypes.data)
    return ptr, vox[:ptr[-1]], seg[:ptr[-1]]


def forward(ptr, vox, seg, density, n_vox, ray_chan_div=0):
    """Line integrals from segments, float64 accumulation.  density: (..., n_vox) flattened to
    (C, n_vox) -> (C, n); with ray_chan_div, ray i reads channel i // ray_chan_div -> (n,)."""
    n = len(ptr) - 1
    ray = np.repeat(np.arange(n), np.diff(ptr))
    dens = np.asarray(density, np.float64).reshape(-1, n_vox)
    if ray_chan_div:
        ch = ray // ray_chan_div
        vals = dens[ch, vox] * seg
        return np.bincount(ray, vals, minlength=n)
    return np.stack([np.bincount(ray, dc[vox] * seg, minlength=n) for dc in dens])


def adjoint(ptr, vox, seg, y, n_vox):
    n = len(ptr) - 1
    ray = np.repeat(np.arange(n), np.diff(ptr))
    return np.bincount(vox, np.asarray(y, np.float64).reshape(-1)[ray] * seg, minlength=n_vox)
