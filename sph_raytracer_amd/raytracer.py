"""Raytracing operator on MI355X: drop-in for the reference's ``sph_raytracer.raytracer``.

``Operator(grid, geom)`` traces every detector ray through the spherical grid once, on the GPU,
into a compact CSR of (linear voxel index, length) segments; ``op(density)`` is the line
integral (forward), ``op.T(y)`` the back-projection (adjoint), and autograd's backward of
``op(density)`` runs the adjoint kernel.  Constructor arguments, attributes and call shapes follow
raytracer.py:647-755.  All compute goes through libsphrt.so (include/sphrt.h); there is no CPU
fallback — without a ROCm GPU every compute entry point raises.

Differences from the reference, by design:
- the trace is stored as a CSR of non-zero segments, not as (3, *rays, K) / (*rays, K) tensors;
  ``op.regs`` / ``op.lens`` rebuild a padded compatibility view on demand;
- crossings at exactly equal distances are ordered as the reference's libstdc++ introsort orders
  them whenever that order can change a voxel (rare rays, replayed by an exact kernel);
- float64 forwards accumulate in float64; float32 forwards multiply and sum in float32 (runs of
  up to 8 segments per thread, stitched across threads), within 2.5e-7 of float64 accumulation;
- the caller's ``geom.rays`` tensor is never normalised in place.
"""
import ctypes
import functools
import math
import os
import weakref

import torch as tr

from . import _lib
from .geometry import ConeCircGeom, ConeRectGeom, ViewGeom, ViewGeomCollection

DEVICE = 'cpu'
PDEVICE = 'cpu'
FTYPE = tr.float64
ITYPE = tr.int64



def isclose(a, b, factor=3):
    """|a - b| < finfo(dtype).resolution ** (1/factor)   (raytracer.py:233-246)."""
    return abs(a - b) < tr.finfo(a.dtype).resolution ** (1 / factor)


# ----- host helpers: start voxels (raytracer.py:555-644) --------------------------------------

def cart2sph(xyz):
    """(x, y, z) -> (radius, elevation from +Z in [0, pi], azimuth from +X in [-pi, pi])."""
    x, y, z = xyz.moveaxis(-1, 0)
    out = tr.empty_like(xyz, dtype=float)
    rho2 = x ** 2 + y ** 2
    out[..., 0] = tr.sqrt(rho2 + z ** 2)
    out[..., 1] = tr.arctan2(tr.sqrt(rho2), z)
    out[..., 2] = tr.arctan2(y, x)
    return out


def sph2cart(rea):
    """(radius, elevation, azimuth) -> (x, y, z)."""
    r, e, a = rea.moveaxis(-1, 0)
    out = tr.empty_like(rea)
    out[..., 0] = r * tr.sin(e) * tr.cos(a)
    out[..., 1] = r * tr.sin(e) * tr.sin(a)
    out[..., 2] = r * tr.cos(e)
    return out


def _region_of(bounds, v, n):
    """Bin of v in `bounds` (searchsorted right - 1); the last boundary belongs to the last bin;
    outside -> -1."""
    idx = tr.searchsorted(bounds, v.contiguous(), right=True) - 1
    idx = tr.where(v == bounds[-1], n - 1, idx)
    idx[idx == n] = -1
    return idx


def find_starts(grid, xs, ftype=FTYPE, device=DEVICE):
    """Voxel (r, e, a) containing each ray start, shape (3, ...).  Evaluated on the host with
    torch — once per *unique* start — so angles and bins are bit-identical to the reference."""
    spec = dict(dtype=ftype, device=device)
    xs = tr.asarray(xs, **spec)
    rb, eb, ab = (tr.asarray(b, **spec) for b in (grid.r_b, grid.e_b, grid.a_b))
    sph = cart2sph(xs)
    shp = grid.shape
    return tr.stack((_region_of(rb, sph[..., 0], shp.r),
                     _region_of(eb, sph[..., 1], shp.e),
                     _region_of(ab, sph[..., 2], shp.a)), axis=0)


def _find_starts_host(grid, xs):
    """find_starts for a float64 host tensor of starts with four torch calls instead of ~35 (C2
    cold path -0.1 ms): only sqrt and arctan2 go through torch — the reference's own routines,
    called on the same layouts (contiguous sums, stride-3 coordinate views), since torch's CPU
    sqrt is MKL vdSqrt and its atan2 path depends on the layout; the squares, sums and the
    binning are exact IEEE operations and comparisons, done in numpy.  Bitwise find_starts
    (tests/test_cpu_api.py::test_find_starts_host).  Non-finite starts take find_starts."""
    import numpy as np
    xt = xs.reshape(-1, 3)
    x = xt.numpy()
    if not np.isfinite(x).all():
        return find_starts(grid, xs)
    x0, x1, x2 = x[:, 0], x[:, 1], x[:, 2]
    rho2 = x0 ** 2 + x1 ** 2
    sph = (tr.sqrt(tr.from_numpy(rho2 + x2 ** 2)).numpy(),
           tr.arctan2(tr.sqrt(tr.from_numpy(rho2)), xt[:, 2]).numpy(),
           tr.arctan2(xt[:, 1], xt[:, 0]).numpy())
    out = np.empty((3, len(x)), np.int64)
    shp = grid.shape
    for k, (b, n) in enumerate(((grid.r_b, shp.r), (grid.e_b, shp.e), (grid.a_b, shp.a))):
        b = np.asarray(b, np.float64)
        idx = np.searchsorted(b, sph[k], side='right') - 1
        idx = np.where(sph[k] == b[-1], n - 1, idx)
        idx[idx == n] = -1
        out[k] = idx
    return tr.from_numpy(out).reshape((3,) + tuple(xs.shape[:-1]))


# ----- device plumbing ------------------------------------------------------------------------

class _Staging:
    """Host byte blobs gathered for one host-to-device copy (the Operator's plan tables, ray
    spec and start bins go over together instead of as three copies)."""

    def __init__(self):
        self._parts, self._offs, self._size = [], [], 0
        self._dev = None

    def add(self, t):
        """Register a contiguous CPU tensor; returns its slot."""
        b = t.contiguous().reshape(-1).view(tr.uint8)
        self._offs.append(self._size)
        self._parts.append(b)
        self._size += -(-b.numel() // 16) * 16              # 16-byte aligned slots
        if b.numel() % 16:
            self._parts.append(tr.zeros(16 - b.numel() % 16, dtype=tr.uint8))
        return len(self._offs) - 1

    def upload(self, dev):
        """One host-to-device copy of the blobs, from pinned memory (torch's caching host
        allocator) so the host goes on to launch the first kernels while it runs."""
        if not self._parts:
            self._dev = None
            return
        if tr.device(dev).type == 'cuda':
            buf = tr.empty(self._size, dtype=tr.uint8, pin_memory=True)
            tr.cat(self._parts, out=buf)
            self._dev = buf.to(dev, non_blocking=True)
        else:
            self._dev = tr.concat(self._parts).to(dev)

    def get(self, slot, like):
        """The device copy of slot `slot` with the dtype and shape of host tensor `like`."""
        o = self._offs[slot]
        nb = like.numel() * like.element_size()
        return self._dev[o:o + nb].view(like.dtype).view(like.shape)


class _Plan:
    """Owner of a libsphrt plan: the grid's boundary tables resident on one GPU.  With a
    `staging`, the tables are packed on the host and go to the device with the staging's copy:
    the plan is created by attach() after the upload, over the caller's device copy (no
    hipMalloc, and no hipFree with its device-wide sync when the plan is destroyed)."""

    def __init__(self, grid, device, boundaries=None, staging=None, ftype=tr.float64):
        lib = _lib.load()
        rb, eb, ab = boundaries if boundaries is not None else (grid.r_b, grid.e_b, grid.a_b)
        # the boundaries in the trace's dtype (r_torch / e_torch / a_torch: tr.asarray(b, ftype))
        rb, eb, ab = (tr.asarray(b, dtype=ftype).contiguous() for b in (rb, eb, ab))
        # trigonometric tables with torch CPU in that dtype — the values the reference solvers
        # use (float32: torch's float32 cos / sin, not rounded float64 values); every table is
        # handed over as float64 (exact for float32 values)
        cos_e = tr.cos(eb)
        cos2_e = tr.cos(eb) ** 2
        cos_a, sin_a = tr.cos(ab), tr.sin(ab)
        a_wrap = bool(-ab[0] == ab[-1] == tr.pi)
        self._keep = [t.to(tr.float64).contiguous() for t in (rb, eb, ab, cos_e, cos2_e, cos_a,
                                                               sin_a)]
        rb, eb, ab, cos_e, cos2_e, cos_a, sin_a = self._keep
        desc = _lib.GridDesc()
        desc.nr, desc.ne, desc.na = len(rb) - 1, len(eb) - 1, len(ab) - 1
        desc.r_b, desc.e_b, desc.a_b = rb.data_ptr(), eb.data_ptr(), ab.data_ptr()
        desc.cos_e, desc.cos2_e = cos_e.data_ptr(), cos2_e.data_ptr()
        desc.cos_a, desc.sin_a = cos_a.data_ptr(), sin_a.data_ptr()
        desc.a_wrap = int(a_wrap)
        res = tr.finfo(ftype).resolution
        desc.close_tol = res ** (1 / 3)
        desc.plane_par_tol = res
        self.shape = (desc.nr, desc.ne, desc.na)
        self.device = device
        self._desc = desc
        self.handle = None
        if staging is not None:
            host = tr.empty(lib.sphrt_plan_table_bytes(desc), dtype=tr.uint8)
            _lib.check(lib.sphrt_plan_pack_tables(desc, host.data_ptr()), 'sphrt_plan_pack_tables')
            self._host, self._slot = host, staging.add(host)
            return
        h = _lib.c_vp()
        _lib.check(lib.sphrt_plan_create(desc, device.index, h), 'sphrt_plan_create')
        self.handle = h
        self.K = lib.sphrt_plan_candidates(h)

    def attach(self, staging):
        """Create the plan over the staged tables' device copy (after staging.upload)."""
        lib = _lib.load()
        self._tables = staging.get(self._slot, self._host)
        h = _lib.c_vp()
        _lib.check(lib.sphrt_plan_create_external(self._desc, self.device.index,
                                                  self._tables.data_ptr(), h),
                   'sphrt_plan_create_external')
        self.handle = h
        self.K = lib.sphrt_plan_candidates(h)

    def __del__(self):
        h = getattr(self, 'handle', None)
        if h is not None and h.value:
            try:
                _lib.load().sphrt_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


def _broadcast_shapes(*shapes):
    """torch.broadcast_shapes in plain Python: the torch function imports torch._refs (and with
    it sympy) on its first call, ~0.8 s that the first dynamic Operator's first forward paid
    (tools/first_construct.py).  Same result and the same error type."""
    nd = max((len(s) for s in shapes), default=0)
    out = [1] * nd
    for s in shapes:
        for i, v in enumerate(s, nd - len(s)):
            v = int(v)
            if v != 1:
                if out[i] not in (1, v):
                    raise RuntimeError(f'Shape mismatch: objects cannot be broadcast to a single '
                                       f'shape.  Mismatch is between {tuple(shapes)}')
                out[i] = v
    return tuple(out)


def _broadcast_pair(xs, rays):
    """Reference broadcasting rule (raytracer.py:76-80) -> (ray shape, xs, rays) un-expanded."""
    xs = tr.asarray(xs, dtype=tr.float64)
    rays = tr.asarray(rays, dtype=tr.float64)
    if xs.numel() > rays.numel():
        shape = _broadcast_shapes(rays.shape, xs.shape)
    else:
        shape = _broadcast_shapes(xs.shape, rays.shape)
    return shape[:-1], xs, rays


class _ConeRays:
    """Generator inputs of a cone detector's ray directions (sphrt_rays_cone, bit-identical to
    ``geom.rays``), staged for the device; of() gives None for other geometries (their rays are
    copied from the host)."""

    @classmethod
    def of(cls, geom):
        spec = geom._ray_spec() if hasattr(geom, '_ray_spec') else None
        if spec is None:
            return None
        circ, frame, row, col = (spec[0],) + tuple(t.to(tr.float64).contiguous() for t in spec[1:])
        shape = tuple(geom.shape)
        n_views = frame.shape[0] if frame.dim() == 2 else 1
        h, w = shape[-2], shape[-1]
        if n_views * h * w != math.prod(shape) or row.shape[-1] != h:
            return None
        self = cls()
        self.circ, self.shape, self.n_views, self.h, self.w = circ, shape, n_views, h, w
        # (frame, row, col) as one blob
        self.host = tr.concat([frame.reshape(-1), row.reshape(-1), col.reshape(-1)])
        self.sizes = [frame.numel(), row.numel(), col.numel()]
        return self

    def stage(self, staging):
        self.slot = staging.add(self.host)

    def launch(self, dev, staging=None, order=None):
        """The rays (*shape, 3) on `dev`, from the staged copy or a copy of their own.  order (a
        device int64 permutation of a view's pixels): each view's rays in that order, returned
        with the geometry ray of every row (int32) — _permute_rays in the generating launch."""
        packed = staging.get(self.slot, self.host) if staging is not None else self.host.to(dev)
        frame_d, row_d, col_d = packed.split(self.sizes)
        rays = tr.empty(self.shape + (3,), dtype=tr.float64, device=dev)
        lib = _lib.load()
        if order is not None:
            ray_id = tr.empty(math.prod(self.shape), dtype=tr.int32, device=dev)
            _lib.check(lib.sphrt_rays_cone_ordered(
                self.n_views, self.h, self.w, int(self.circ), _lib.ptr(frame_d), _lib.ptr(row_d),
                _lib.ptr(col_d), _lib.ptr(order), _lib.ptr(rays), _lib.ptr(ray_id),
                _lib.stream_of(dev)), 'sphrt_rays_cone_ordered')
            return rays, ray_id
        _lib.check(lib.sphrt_rays_cone(
            self.n_views, self.h, self.w, int(self.circ), _lib.ptr(frame_d), _lib.ptr(row_d),
            _lib.ptr(col_d), _lib.ptr(rays), _lib.stream_of(dev)), 'sphrt_rays_cone')
        return rays


def _launch_tiled(cone, dev, staging, tiles):
    """The rays of `cone` (an orbit: n_views > 1) in view tiles (sphrt_rays_cone_tiled): an array
    (h, w / tw, n_views / tv, tv, tw, 3) and the geometry ray of every row (int32)."""
    tv, tw = tiles
    packed = staging.get(cone.slot, cone.host)
    frame_d, row_d, col_d = packed.split(cone.sizes)
    h, w, v = cone.h, cone.w, cone.n_views
    rays = tr.empty((h, w // tw, v // tv, tv, tw, 3), dtype=tr.float64, device=dev)
    ray_id = tr.empty(v * h * w, dtype=tr.int32, device=dev)
    _lib.check(_lib.load().sphrt_rays_cone_tiled(
        v, h, w, int(cone.circ), _lib.ptr(frame_d), _lib.ptr(row_d), _lib.ptr(col_d), tv, tw,
        _lib.ptr(rays), _lib.ptr(ray_id), _lib.stream_of(dev)), 'sphrt_rays_cone_tiled')
    return rays, ray_id


def _device_rays(geom, dev):
    """Cone-detector ray directions generated on the device (sphrt_rays_cone), bit-identical to
    ``geom.rays``; None for other geometries (their rays are copied from the host)."""
    cone = _ConeRays.of(geom)
    return cone.launch(dev) if cone is not None else None


def _geom_rays(geom, dev):
    rays = _device_rays(geom, dev)
    return geom.rays if rays is None else rays


# azimuth columns per wedge of the ConeCirc trace order; measured (C5 forward f64 / transposed
# adjoint f64 / retrieval iteration, C4 forward): 2: 46.5 / 42.5 / 0.157 ms, 21.9; 3: 45.8 /
# 43.5 / 0.157 ms, 21.3; 4: 45.6 / 46.7 / 0.161 ms, 21.1; 5: 45.8 / 47.7 / 0.164 ms, 21.2; 8: 48.0
# / 48.3 / 0.167 ms, 21.5 us.
_WEDGE = 3


# Trace order of orbits (a collection of identical cone detectors, static grids): tiles of tw
# neighbouring pixels of one detector row seen from tv consecutive views, tiles by (row, column
# pair, view group) — a workgroup's rays then cross the volume along one family of nearby lines
# from many directions, whose granules the neighbouring workgroups share in L2.  Forward kernel
# (f32 / f64 us, profiles/r05_vtile_*.jsonl) C2 6.33 / 9.6 -> 5.92 / 8.45 with (50, 2), C3 204.1 /
# 333.3 -> 195.1 / 314.1 with (64, 2), C5 (against the wedge order) 27.7 / 44.2 -> 26.8 / 37.0
# with (64, 2); the transposed adjoints C2 6.2 / 8.6 -> 5.9 / 8.4, C3 192 / 303 -> 187 / 287, C5
# 24.7 / 40.4 -> 24.7 / 35.3.  tv: the largest divisor of the view count in [8, 64]; tw = 2 (1
# for an odd width).  Dynamic grids keep the per-view orders (view i <-> time slice i pairs trace
# rows with slices by position).  SPHRT_RAY_ORDER=natural keeps the geometry order, vtile:tv,1,tw
# forces a tile.
_VIEW_TILE_MAX, _VIEW_TILE_MIN = 64, 8


def _view_tiles(shape, dynamic):
    """(tv, tw) for an orbit of `shape` (views, rows, columns), or None."""
    mode = os.environ.get('SPHRT_RAY_ORDER', 'auto')
    if dynamic or len(shape) != 3 or shape[0] < 2:
        return None
    v, h, w = shape
    if mode.startswith('vtile:'):
        tv, th, tw = (int(x) for x in mode[6:].split(','))
        return (tv, tw) if th == 1 and v % tv == 0 and w % tw == 0 else None
    if mode != 'auto':
        return None
    tv = next((d for d in range(min(v, _VIEW_TILE_MAX), _VIEW_TILE_MIN - 1, -1) if v % d == 0),
              None)
    if tv is None:
        return None
    return tv, (2 if w % 2 == 0 else 1)


def _trace_order(geom, rays, dynamic=False):
    """Per-view order the trace visits a ConeCirc detector's pixels in, or None (geometry order).

    ConeCirc pixels are (radius, azimuth) with the azimuth fastest: ~36 consecutive rays (one
    workgroup block at C5) sweep most of a ring, whose rays part around the view axis.  Wedges of
    _WEDGE azimuth columns, radius-major inside, keep a block's rays together: C5 table stride
    1536 -> 1024, forward f32 33.2 -> 29.5 us, f64 52.7 -> 45.8 us, transposed adjoint f64 53.4
    -> 43.5 us (ConeRect rows are already compact: strips beat every tiling measured).  Only the
    order of the CSR's rows changes: every row reports its geometry ray (sphrt_csr_index ray_ids),
    outputs stay in geometry order.  SPHRT_RAY_ORDER=natural keeps the geometry order.  (The
    orders across views measured in rounds 2-5 — rows of G views, detector tiles, tiles of
    several rows — live in tools/build_src_variant.py's history and the A/B records; only the
    view tiles, _view_tiles, were kept.)"""
    if os.environ.get('SPHRT_RAY_ORDER', 'auto') == 'natural':
        return None
    from .geometry import ConeCircGeom
    geoms = getattr(geom, 'geoms', [geom])
    if not geoms or any(type(g) is not ConeCircGeom for g in geoms):
        return None
    shape = tuple(rays.shape[:-1])
    if len(shape) not in (2, 3) or shape[-1] <= _WEDGE:
        return None
    return _wedge_order(shape[-2], shape[-1])


@functools.lru_cache(maxsize=16)
def _wedge_order(h, w):
    """Pixel order of an (h, w) ConeCirc detector in wedges of _WEDGE azimuth columns."""
    r = tr.arange(h).repeat_interleave(w)
    a = tr.arange(w).repeat(h)
    key = ((a // _WEDGE) * h + r) * _WEDGE + a % _WEDGE
    return tr.argsort(key)


def _permute_rays(rays, perm):
    """Rays (V, H, W, 3) or (H, W, 3) with each view's pixels in trace order `perm` (a device
    index) and the geometry ray of every trace row (int32, on the device)."""
    shape = rays.shape
    v = shape[0] if rays.dim() == 4 else 1
    flat = rays.reshape(v, -1, 3).index_select(1, perm)
    hw = perm.numel()
    ray_id = (tr.arange(v, device=perm.device, dtype=tr.int32) * hw)[:, None] + perm.to(tr.int32)
    return flat.reshape(shape), ray_id.reshape(-1)


class _RayBatch:
    """Device copies of the unique starts / directions + the broadcast descriptor."""

    @staticmethod
    def host_starts(grid, xs):
        """(starts, start voxels) on the host: float64 (..., 3) and int32 (..., 4)."""
        xs_u = tr.asarray(xs, dtype=tr.float64).detach().to('cpu').contiguous()
        st = tr.zeros(xs_u.shape[:-1] + (4,), dtype=tr.int32)
        if grid is not None:
            starts = _find_starts_host(grid, xs_u)             # (3, ...) on the host
            st[..., :3] = starts.moveaxis(0, -1).to(tr.int32)
        return xs_u, st

    def __init__(self, grid, xs, rays, device, staged=None):
        """grid=None: no start voxels (per-family solves only).  staged: the device copies of
        host_starts(grid, xs) (a _Staging's), else they are made here."""
        rshape, xs, rays = _broadcast_pair(xs, rays)
        if len(rshape) > _lib.MAX_DIMS:
            raise ValueError(f'ray batch rank {len(rshape)} > {_lib.MAX_DIMS}')
        self.shape = rshape
        self.n = math.prod(rshape)
        if staged is not None:
            self.xs, self.start = staged
        else:
            xs_u, st = self.host_starts(grid, xs)
            # starts and start voxels in one host-to-device copy
            xb, sb = xs_u.reshape(-1).view(tr.uint8), st.reshape(-1).view(tr.uint8)
            packed = tr.concat([xb, sb]).to(device)
            self.xs = packed[:xb.numel()].view(tr.float64).view(xs_u.shape)
            self.start = packed[xb.numel():].view(tr.int32).view(st.shape)
        self.rays = rays.detach().contiguous().to(device)
        full = rshape + (3,)
        xs_str = self.xs.expand(full).stride()
        ry_str = self.rays.expand(full).stride()
        d = _lib.RayBatch()
        d.ndim = len(rshape)
        for i, s in enumerate(rshape):
            d.shape[i] = s
            d.xs_stride[i] = xs_str[i]
            d.rays_stride[i] = ry_str[i]
        d.xs, d.rays, d.start = self.xs.data_ptr(), self.rays.data_ptr(), self.start.data_ptr()
        self.desc = d


# ----- API-parity solvers (raytracer.py:248-552) ----------------------------------------------

def _check_ftype(ftype):
    if ftype not in (tr.float64, tr.float32):
        raise NotImplementedError(f'sph_raytracer_amd traces in float64 or float32, not {ftype}')


def _solve(family, bounds, xs, rays, ftype, itype, device):
    _check_ftype(ftype)
    dev = _lib.require_gpu(device)
    with tr.cuda.device(dev):
        bounds = tr.asarray(bounds, dtype=tr.float64)
        unit = tr.tensor([0.0, 1.0], dtype=tr.float64)
        grid_b = tuple(bounds if i == family else unit for i in range(3))
        plan = _Plan(None, dev, boundaries=grid_b, ftype=ftype)
        batch = _RayBatch(None, xs, rays, dev)
        nb = len(bounds)
        width = nb if family == 2 else 2 * nb
        t = tr.empty(batch.shape + (width,), dtype=ftype, device=dev)
        reg = tr.empty(batch.shape + (width,), dtype=tr.int32, device=dev)
        neg = tr.empty(batch.shape + (width,), dtype=tr.int8, device=dev)
        lib = _lib.load()
        fn = lib.sphrt_solve if ftype == tr.float64 else lib.sphrt_solve_f32
        _lib.check(fn(plan.handle, batch.desc, family, _lib.ptr(t), _lib.ptr(reg), _lib.ptr(neg),
                      _lib.stream_of(dev)), 'sphrt_solve')
        inds = tr.arange(nb, dtype=itype)
        inds = (inds if family == 2 else tr.cat((inds, inds))).repeat(*batch.shape, 1)
        return t.to(device), reg.to(itype).to(device), inds.to(device), neg.to(device)


def r_torch(r, xs, rays, ftype=FTYPE, itype=ITYPE, device=DEVICE):
    """Crossings of every ray with spheres of radii ``r`` (raytracer.py:248-325).
    Returns (t, regions, inds, negative_crossing), each (*rays, 2*len(r))."""
    return _solve(0, r, xs, rays, ftype, itype, device)


def e_torch(e, xs, rays, ftype=FTYPE, itype=ITYPE, device=DEVICE):
    """Crossings with elevation cones at angles ``e`` (raytracer.py:328-468), (*rays, 2*len(e))."""
    return _solve(1, e, xs, rays, ftype, itype, device)


def a_torch(a_b, xs, rays, ftype=FTYPE, itype=ITYPE, device=DEVICE):
    """Crossings with azimuth half-planes ``a_b`` (raytracer.py:471-552), (*rays, len(a_b))."""
    return _solve(2, a_b, xs, rays, ftype, itype, device)


def _layout_for(grid, ray_shape, shape):
    """-> (n_chan, ray_chan_div, out_shape): the indexing rules of raytracer.py:703-712.

    Static grid: density (C..., nr, ne, na) -> (C..., *rays).  Dynamic grid: density
    (T, nr, ne, na) indexed with t = arange(T)[:, None, None, None], i.e. view i of a (T, H, W)
    collection sees time slice i, while a single detector is integrated for every time step."""
    R = tuple(ray_shape)
    g = tuple(grid.shape)
    if grid.dynamic:
        if len(shape) != 4 or tuple(shape[1:]) != g[1:]:
            raise ValueError(f'dynamic grid expects density (T, {g[1]}, {g[2]}, {g[3]}), '
                             f'got {tuple(shape)}')
        T = shape[0]
        if len(R) > 3:
            raise NotImplementedError('dynamic grids need a detector of rank <= 3')
        out_shape = _broadcast_shapes((T, 1, 1, 1), R + (1,))[:-1]
        if len(R) == 3 and R[0] == T and T > 1:
            return 1, R[1] * R[2], out_shape        # view i sees time slice i
        if len(R) == 3 and R[0] != 1 and T != 1:
            raise ValueError(f'cannot pair {T} time steps with {R[0]} views')
        return T, 0, out_shape                        # every time step sees every ray
    if tuple(shape[-3:]) != g:
        raise ValueError(f'density shape {tuple(shape)} does not end with grid shape {g}')
    lead = tuple(shape[:-3])
    return math.prod(lead), 0, lead + R


try:   # the current HIP stream as an int without building a torch Stream object (~0.3 vs 1.9 us)
    _raw_stream = tr._C._cuda_getCurrentRawStream
    _cur_dev = tr._C._cuda_getDevice
except AttributeError:   # pragma: no cover - older torch
    def _raw_stream(index):
        return tr.cuda.current_stream(index).cuda_stream
    _cur_dev = tr.cuda.current_device


def _seg_alloc(total):
    """Per-segment arrays are allocated to a multiple of 16 entries (the apply kernels read whole
    aligned 8- or 16-segment chunks; entries past the total are masked, never used)."""
    return max((total + 15) // 16 * 16, 16)


# memory gates of the construction (fractions of the free device memory), shared with the native
# construction (csrc/construct.cpp kGate*, pinned by tests/test_cpu_api.py)
_GATE_WIDE_TABLES = 0.3     # one-pass tables: the wide tables' bytes
_GATE_STAGED = 0.5          # staged table build: final CSR + wide tables
_STAGED_SEG_BYTES = 18      # its CSR bytes per segment (vox 4 + len 8 + len32 4 + loc 2)
_GATE_TRACE_STAGING = 0.4   # one-pass trace: its staging
_STAGING_SLOT_BYTES = 12    # per bound slot (vox 4 + len 8)


def _tables_one_pass(desc, nblocks, dev, free=None):
    """Whether _local_tables builds in one pass (wide tables fit comfortably in free memory and
    SPHRT_TABLES is not 'twopass'); decides desc.tab_bytes (16-bit entries when every granule
    index fits: <= 2^18 columns, half the table bytes the forward streams)."""
    cols = desc.stage_cols if desc.stage_shape[0] > 0 else desc.n_cols
    desc.tab_bytes = 2 if (cols + 3) // 4 <= 65536 else 4
    wide_bytes = nblocks * _lib.TAB_WIDE * desc.tab_bytes
    return (os.environ.get('SPHRT_TABLES', 'onepass') != 'twopass' and
            wide_bytes <= _GATE_WIDE_TABLES * (tr.cuda.mem_get_info(dev)[0] if free is None
                                               else free))


def _staged_fits(desc, nblocks, total, free):
    """Whether the staged table build fits: it keeps the one-pass trace's staging (12 B per bound
    slot, allocated already) alive while it writes the final CSR (vox 4 + len 8 + len32 4 + loc 2
    = 18 B per segment) and the wide tables, so its peak is staging + CSR + tables, against the
    compaction path's staging + 12 B per segment (the staging is freed before the tables).  Taken
    only when the CSR and the wide tables fit in half the free memory; otherwise the staging is
    compacted first (C3 peak 3.04 -> 4.60 GB with the staged build)."""
    need = _STAGED_SEG_BYTES * _seg_alloc(total) + nblocks * _lib.TAB_WIDE * desc.tab_bytes
    return need <= _GATE_STAGED * free


def _local_tables(lib, desc, blocks, nblocks, total, dev, stream, staged=None):
    """Per-workgroup granule tables and run records of a CSR; sets desc.loc/.tab/.tab_stride/
    .n_fallback/.runs and returns (loc, tab, runs).  One host sync (the largest table decides
    the stride; the run-record overflow count decides desc.runs).  One pass
    (sphrt_csr_local_build into SPHRT_TAB_WIDE-strided tables, then _pack to the stride) unless
    the wide tables would not fit comfortably in free memory or SPHRT_TABLES=twopass
    (sphrt_csr_local_count, then _fill).  Run records (sphrt_csr_runs) replace the forward's
    row_ray / empty_ray loads in grids of more than one wave of workgroups (SPHRT_RUNS=auto;
    =on: every grid, =off: none).  Measured on MI355X (forward / transposed adjoint, us): C3 f32
    234.4 -> 227.6 / 226.4 -> 225.2, f64 370.3 -> 360.5 / 317.5 -> 305.0; C5 f32 34.8 -> 34.1,
    f64 63.8 -> 63.3; but the single-wave C2 f32 forward 6.90 -> 7.06 (its dependent loads are
    hidden under the one wave's latency chain), so single-wave grids keep the loads."""
    stats = tr.empty(3, dtype=tr.int64, device=dev)
    desc.runs = None
    runs = None
    mode = os.environ.get('SPHRT_RUNS', 'auto')
    want = mode == 'on' or (mode == 'auto' and nblocks > _SINGLE_WAVE_BLOCKS)
    if want and desc.n_rays < 2 ** 31:
        runs = tr.empty(_lib.RUN_FIELDS * nblocks, dtype=tr.int32, device=dev)
        _lib.check(lib.sphrt_csr_runs(desc, _lib.ptr(runs), _lib.ptr(stats[2:]), stream),
                   'sphrt_csr_runs')
    else:
        stats[2:].fill_(1)
    loc = tr.empty(_seg_alloc(total), dtype=tr.int16, device=dev)
    one_pass = staged is not None or _tables_one_pass(desc, nblocks, dev)
    tdt = tr.int16 if desc.tab_bytes == 2 else tr.int32
    if staged is not None:      # (the caller checked one_pass)
        (bound_ptr, svox, slen), nz_row = staged
        wide = tr.empty(nblocks * _lib.TAB_WIDE, dtype=tdt, device=dev)
        _lib.check(lib.sphrt_csr_local_build_staged(desc, _lib.ptr(blocks), _lib.ptr(loc),
                                                    _lib.ptr(wide), _lib.ptr(stats),
                                                    _lib.ptr(bound_ptr), _lib.ptr(nz_row),
                                                    _lib.ptr(svox), _lib.ptr(slen), stream),
                   'sphrt_csr_local_build_staged')
    elif one_pass:
        wide = tr.empty(nblocks * _lib.TAB_WIDE, dtype=tdt, device=dev)
        _lib.check(lib.sphrt_csr_local_build(desc, _lib.ptr(blocks), _lib.ptr(loc), _lib.ptr(wide),
                                             _lib.ptr(stats), stream), 'sphrt_csr_local_build')
    else:
        _lib.check(lib.sphrt_csr_local_count(desc, _lib.ptr(blocks), _lib.ptr(stats), stream),
                   'sphrt_csr_local_count')
    n_fallback, max_tab, runs_over = stats.tolist()
    if runs_over:
        runs = None
    stride = max(64, (max_tab + 63) // 64 * 64)
    tab = tr.empty(nblocks * stride + 3 * 256, dtype=tdt, device=dev)   # + early-fetch pad
    if one_pass:
        _lib.check(lib.sphrt_csr_local_pack(desc, _lib.ptr(blocks), _lib.ptr(wide), _lib.ptr(tab),
                                            stride, stream), 'sphrt_csr_local_pack')
        del wide
    else:
        _lib.check(lib.sphrt_csr_local_fill(desc, _lib.ptr(blocks), _lib.ptr(loc), _lib.ptr(tab),
                                            stride, stream), 'sphrt_csr_local_fill')
    desc.n_fallback, desc.tab_stride = n_fallback, stride
    desc.loc, desc.tab = loc.data_ptr(), tab.data_ptr()
    desc.runs = runs.data_ptr() if runs is not None else None
    return loc, tab, runs


_BRICK = (4, 2, 4)   # (r, e, a) voxels per staging brick: 32 = one 128-byte float line
# (4, 2, 4) over round 1's (2, 4, 4): C3 forward f32 214.5 -> 204.1 us, f64 350.4 -> 333.5 us, C5
# unchanged (27.7 / 45.3 us); 11 shapes swept in profiles/r02_brick_sweep.jsonl.
_SINGLE_WAVE_BLOCKS = 256 * 6   # forward workgroups resident at once (256 CUs x 6)


_HEAD32 = -2 ** 31      # bit 31 of an int32 (the row-head flag of vox)

# Row order of the transposed CSRs (the adjoint's rows are voxels): bricks of (r, e, a) voxels,
# brick by brick in (r, e, a) order and inside a brick in (r, e, a) order, instead of the linear
# voxel order (azimuth fastest).  A workgroup's ~32 voxels are then a compact cluster instead of
# an azimuth arc, and its rays (the gathered columns) compact patches of each view: fewer
# granules and L2 lines per workgroup.  Measured (profiles/r05_trows_ab.json, transposed adjoint
# f32 / f64 us): C3 236.5 / 328.8 -> 208.4 / 310.8 with (4,2,4) bricks ((2,4,4) 221 / 324,
# (4,4,4) 223 / 323, (8,8,4) 233 / 335), C5 27.8 / 44.2 -> 24.9 / 40.6; a one-wave grid (C2) is
# neutral (6.3 / 8.8 -> 6.2 / 9.0) and keeps the linear order (and its row-run records); so
# does the time-paired transpose of a dynamic operator (C4 gradient 37.5 -> 39.6 us with bricks
# inside each slice).  C5 retrieval 0.1272 -> 0.1189 ms per iteration (profiles/r05_trows_ab.json).
# The rows report their voxel through the index's row ids; each voxel's segments keep their
# order (a stable sort), and a row's place in its workgroup sets how the segmented scan
# associates its sum: the same adjoint up to summation order (deterministic, float64 within
# 1e-13 of the linear order: test_transposed_brick_rows_equal_linear_rows).  SPHRT_TROWS=off
# keeps the linear order, =b0,b1,b2 sets the brick.
_TROWS = (4, 2, 4)


def _voxel_rows(shape3, n_cols, dev, nblocks):
    """A _VoxelRows (vpos, vperm: int32 on `dev`): row position of every voxel (column) of a static
    transposed CSR and the voxel of every row position, or None (linear order)."""
    env = os.environ.get('SPHRT_TROWS', 'auto')
    brick = None if env == 'off' else tuple(int(v) for v in env.split(',')) if env != 'auto' \
        else _TROWS if nblocks > _SINGLE_WAVE_BLOCKS else None
    if brick is None or n_cols != math.prod(shape3) or n_cols >= 2 ** 31:
        return None
    key = (shape3, brick, str(dev))
    rows = _VOXEL_ROWS.get(key)
    if rows is None:
        rows = _VoxelRows(*_voxel_rows_make(shape3, brick, dev))
        _VOXEL_ROWS[key] = rows
    return rows


class _VoxelRows:
    """The row maps of one grid shape and device, shared by the transposed CSRs that hold them
    (each keeps a reference in its record) and released with the last of them (ADVICE r05:
    a module-level cache of device tensors outlived every Operator)."""

    def __init__(self, vpos, vperm):
        self.vpos, self.vperm = vpos, vperm


_VOXEL_ROWS = weakref.WeakValueDictionary()


def _voxel_rows_make(shape3, brick, dev):
    nr, ne, na = shape3
    br, be, ba = brick
    idx = tr.arange(nr * ne * na, device=dev, dtype=tr.int64)
    r, e, a = idx // (ne * na), (idx // na) % ne, idx % na
    nbe, nba = -(-ne // be), -(-na // ba)
    key = (((r // br) * nbe + e // be) * nba + a // ba) * (br * be * ba) + \
        ((r % br) * be + e % be) * ba + a % ba
    vperm = tr.argsort(key).to(tr.int32)                  # position -> voxel
    vpos = tr.empty_like(vperm)
    vpos[vperm.long()] = tr.arange(vperm.numel(), device=dev, dtype=tr.int32)
    return vpos, vperm


# Transposed CSRs (columns = rays, when they are the geometry's rays) of multi-wave grids stage
# y in bricks of (views, rows, columns) = (8, 1, 4) rays: with the rows in voxel bricks
# (_TROWS) a workgroup's rays are the same few pixels of many views, which such a brick puts in
# one 128-byte line (C3 transposed adjoint f32 208 -> 193 us, f64 310 -> 304 us; (16,1,4) 194 /
# 302, (4,2,4) 198 / 314, (1,4,8) 234 / 366, (4,4,4) 214 / 340: profiles/r05_brickt_study.jsonl).
# Before the voxel-brick rows, detector tiles lost (C3 f32 229 -> 261 us with (1, 4, 8)).
# SPHRT_BRICK_T=off / b0,b1,b2 overrides.
_BRICK_RAYS = (8, 1, 4)


_L2_BYTES = 4 << 20     # one XCD's L2


def _stage_brick(nblocks, env_name='SPHRT_BRICK', brick=_BRICK, n_cols=None):
    """Brick of the density staging for a trace CSR of `nblocks` workgroup blocks (sphrt.h
    stage_*), or None.  It pays when the forward runs in several waves of workgroups, whose
    granule DMA is bound by L2 requests, over an array larger than one XCD's L2 (n_cols float32
    columns; None: not checked): C3 (8.4 MB) f32 forward 267 -> 241 us in round 1, 206.7 -> 196.1
    us with the view tiles (f64 311 -> 318); a grid that is resident at once (C2: 1473 blocks) is
    latency-bound and would only pay the packing pass, and with the view tiles an array that fits
    the L2 loses too (C5, 1 MB: f32 24.9 -> 26.8 us, f64 33.8 -> 36.7 us with (4,2,4) bricks;
    profiles/r05_brick_tiles_sweep.jsonl).  The environment variable `env_name` (SPHRT_BRICK for
    the trace CSR, SPHRT_BRICK_T for the transposed one, whose columns are rays) set to `off`
    disables it, to `b0,b1,b2` forces that brick."""
    env = os.environ.get(env_name, 'auto')
    if env == 'off':
        return None
    if env != 'auto':
        return tuple(int(v) for v in env.split(','))
    if n_cols is not None and 4 * n_cols <= _L2_BYTES:
        return None
    return brick if brick is not None and nblocks > _SINGLE_WAVE_BLOCKS else None


def _set_stage(desc, shape, brick):
    """Fill the CSR's stage_* fields for `brick` (None: off); True when staging is on.  The
    stage buffer itself is not part of the operator: every forward call gets its own
    (_call_forward), so calls on different streams never share one."""
    _clear_stage(desc)
    if brick is None:
        return False
    cols = math.prod(-(-s // b) * b for s, b in zip(shape, brick))
    if cols >= 2 ** 31 - 1 or math.prod(brick) % 4:    # 32-bit staged columns, whole granules
        return False
    for i in range(3):
        desc.stage_shape[i], desc.stage_brick[i] = shape[i], brick[i]
    desc.stage_cols = cols
    return True


def _stage_bytes(desc, n_chan, elem):
    """Bytes of the brick stage one forward call on `desc` needs (0: not staged)."""
    return n_chan * desc.stage_cols * elem if desc.stage_shape[0] > 0 else 0


# Launches of more blocks than one resident wave (6 workgroups per CU) alternate their block order
# (sphrt_csr.order) from call to call: a CSR that outgrows the memory-side cache then starts each
# launch on the lines the previous launch touched last, which are the ones still cached, instead
# of the ones it evicted first.  Same results.  Measured on repeated forwards (tools/prof, MI355X):
# C3 f32 233 -> 213 us, f64 364 -> 350 us, C5 f32 29.3 -> 28.3 us; one-wave launches (C2) gain
# nothing and keep their order.  The C++ fast path (csrc/fastpath.cpp) applies the same rule.
_ALTERNATE_MIN_BLOCKS = 256 * 6


def _alternate(desc):
    """Flip a multi-wave CSR's block order for its next launch."""
    if desc.n_blocks > _ALTERNATE_MIN_BLOCKS:
        desc.order ^= 1


def _call_forward(fn, desc, d, n_chan, cs, div, out, ocs, dev):
    """sphrt_forward_f32/_f64 on the current stream of `dev`.  A brick-staged CSR gets this
    call's stage buffer from torch's caching allocator on that stream (released to the same
    stream afterwards: stream-ordered reuse, never shared with a call on another stream)."""
    need = _stage_bytes(desc, n_chan, d.element_size())
    stage = None
    if need:
        stage = tr.empty(need, dtype=tr.uint8, device=dev)
        desc = _lib.CSR.from_buffer_copy(desc)
        desc.stage, desc.stage_bytes = stage.data_ptr(), need
    _lib.check(fn(desc, _lib.ptr(d), n_chan, cs, div, _lib.ptr(out), ocs, _lib.stream_of(dev)),
               'sphrt_forward')
    del stage


def _dense_ranges(desc, blocks, row_list, n_out):
    """Dense output ranges (sphrt_csr.order bit 2) for a CSR whose rows are in output order:
    block b owns outputs [first row of b, first row of the next block with rows) — the first
    block from 0, the last to n_out — written into its record's fields 0 / 1 (the empty-list
    share, unused in this mode), and zeroes that range itself before its row closes.  Every
    output line is then written by one workgroup: the time-paired transposed adjoint of C4
    (6.25 M voxel-slice rows, ~70 % of them empty) wrote 47 MB per launch for a 25 MB result
    through the empty-ray list, its zeros and closes landing in the same lines from different
    XCDs (profiles/r06_adjoint_c4_pmc.json).  Run records are dropped (their empty ranges
    describe the list).  (Closing the rows by block-relative index and expanding them through an
    occupancy bitmap instead of reading row_ray — 17 MB less per C4 launch — measured the same:
    26.56 against 26.42 us, profiles/r06_dense_ab_c4.json.)"""
    b = blocks.view(-1, _lib.BLOCK_FIELDS)
    n_rows = max(int(row_list.numel()), 1)
    has = b[:, 2] < b[:, 3]
    k0 = b[:, 4].clamp(0, n_rows - 1)
    first = tr.where(has, row_list[k0].long(), tr.full_like(k0, n_out))
    first = first.flip(0).cummin(0).values.flip(0)     # rowless blocks: the next block's first
    lo = first.clone()
    lo[0] = 0
    hi = tr.cat((first[1:], first.new_full((1,), n_out)))
    b[:, 0], b[:, 1] = lo, hi
    desc.order |= 4
    desc.runs = None


def _gather(src, idx, n, dev):
    """src[idx] (contiguous float32 / float64 src, int32 idx of n entries) on the current stream
    of `dev` through sphrt_gather_* — the adjoint's input in trace order (one launch of 4
    gathers per thread; torch's index_select took 7.5 us for C4's 250,000 rays)."""
    out = tr.empty(n, dtype=src.dtype, device=dev)
    lib = _lib.load()
    fn = lib.sphrt_gather_f32 if src.dtype == tr.float32 else lib.sphrt_gather_f64
    _lib.check(fn(_lib.ptr(src), _lib.ptr(idx), n, _lib.ptr(out), _lib.stream_of(dev)),
               'sphrt_gather')
    return out


def _clear_stage(desc):
    for i in range(3):
        desc.stage_shape[i] = desc.stage_brick[i] = 0
    desc.stage_cols, desc.stage, desc.stage_bytes = 0, None, 0


def _workspace(lib, plan, n, dev):
    return tr.empty(lib.sphrt_trace_workspace_bytes(plan.handle, n), dtype=tr.uint8, device=dev)


_bound_hook = None   # tests only: callable(bounds) run on the one-pass trace's bounds


def _trace_csr(lib, plan, batch, dev, stream, keep_staging=False):
    """Trace every ray of `batch` into the segment CSR -> (row_ptr, vox, len, total, staging).

    One pass (sphrt_trace_bound / _emit / _compact, include/sphrt.h): a geometric upper bound of
    every ray's segment count sizes a staging CSR, every ray is traced once into its slot, and
    the rows are compacted — two host syncs (the bound total; the segment total).  The two-pass
    trace (count, then fill: every ray traced twice, one sync) serves when the staging would
    not fit comfortably in free device memory, when a bound failed (then only the fill pass
    runs: the counts are exact), and on request (SPHRT_TRACE=twopass).  keep_staging: a
    successful one-pass trace returns its staging (bound_ptr, svox, slen) uncompacted, with vox
    and len None — the caller compacts it (_compact_staging) or lets the table build move the
    segments (sphrt_csr_local_build_staged); staging is None otherwise."""
    n = batch.n
    counts = tr.empty(max(n, 1), dtype=tr.int32, device=dev)
    row_ptr = tr.empty(n + 1, dtype=tr.int64, device=dev)
    ws = tr.empty(lib.sphrt_scan_workspace_bytes(n), dtype=tr.uint8, device=dev)
    tws = _workspace(lib, plan, n, dev)
    h, d, tw = plan.handle, batch.desc, (_lib.ptr(tws), tws.numel())

    def scan(src, dst):
        _lib.check(lib.sphrt_scan_counts(_lib.ptr(src), n, _lib.ptr(dst), _lib.ptr(ws), stream),
                   'sphrt_scan_counts')

    def fill(total):
        vox = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
        seg_len = tr.empty(_seg_alloc(total), dtype=tr.float64, device=dev)
        _lib.check(lib.sphrt_trace_fill(h, d, _lib.ptr(row_ptr), _lib.ptr(vox), _lib.ptr(seg_len),
                                        *tw, stream), 'sphrt_trace_fill')
        return vox, seg_len

    if n > 0 and os.environ.get('SPHRT_TRACE', 'onepass') != 'twopass':
        bound_ptr = tr.empty(n + 1, dtype=tr.int64, device=dev)
        _lib.check(lib.sphrt_trace_bound(h, d, _lib.ptr(counts), *tw, stream), 'sphrt_trace_bound')
        if _bound_hook is not None:      # tests: shrink bounds to exercise the fallback
            _bound_hook(counts[:n])
        scan(counts, bound_ptr)          # (counts holds the bounds until the emit pass)
        cap = int(bound_ptr[n].item())   # host sync 1
        if cap * _STAGING_SLOT_BYTES <= _GATE_TRACE_STAGING * tr.cuda.mem_get_info(dev)[0]:
            svox = tr.empty(max(cap, 1), dtype=tr.int32, device=dev)
            slen = tr.empty(max(cap, 1), dtype=tr.float64, device=dev)
            over = tr.empty(1, dtype=tr.int64, device=dev)
            _lib.check(lib.sphrt_trace_emit(h, d, _lib.ptr(bound_ptr), _lib.ptr(counts),
                                            _lib.ptr(svox), _lib.ptr(slen), _lib.ptr(over),
                                            *tw, stream), 'sphrt_trace_emit')
            scan(counts, row_ptr)
            total, n_over = tr.stack((row_ptr[n], over[0])).tolist()   # host sync 2
            if n_over == 0:
                del tws, counts, over
                staging = (bound_ptr, svox, slen)
                if keep_staging:
                    return row_ptr, None, None, total, staging
                return (row_ptr,) + _compact_staging(lib, n, row_ptr, total, staging, dev,
                                                     stream) + (total, None)
            del svox, slen
            return (row_ptr,) + fill(total) + (total, None)
    _lib.check(lib.sphrt_trace_count(h, d, _lib.ptr(counts), *tw, stream), 'sphrt_trace_count')
    scan(counts, row_ptr)
    total = int(row_ptr[n].item())        # the one host sync of the two-pass trace
    return (row_ptr,) + fill(total) + (total, None)


def _compact_staging(lib, n, row_ptr, total, staging, dev, stream):
    """A one-pass trace's staging -> the tight CSR (vox, len) (sphrt_trace_compact: voxels and
    lengths in one pass, one row search per segment for both; peak = staging + 12 B per segment.
    Two passes, freeing the voxel staging in between, peaked 4 B per staging slot lower and cost
    C3 2 x 457 us)."""
    bound_ptr, svox, slen = staging
    vox = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
    seg_len = tr.empty(_seg_alloc(total), dtype=tr.float64, device=dev)
    _lib.check(lib.sphrt_trace_compact(n, _lib.ptr(bound_ptr), _lib.ptr(svox), _lib.ptr(slen),
                                       _lib.ptr(row_ptr), _lib.ptr(vox), _lib.ptr(seg_len), stream),
               'sphrt_trace_compact')
    return vox, seg_len


def line_integrals(grid, geom, density):
    """No-store forward: trace and integrate in one fused pass, nothing persisted.

    Same result as ``Operator(grid, geom)(density)`` (not differentiable), without building the
    segment CSR — the memory-capped / cold path (one kernel, O(output) memory)."""
    density = tr.as_tensor(density)
    dev = _lib.require_gpu(density.device)    # a GPU density computes where it lives
    with tr.cuda.device(dev):
        plan = _Plan(grid, dev)
        batch = _RayBatch(grid, geom.ray_starts, _geom_rays(geom, dev), dev)
        n_chan, div, out_shape = _layout_for(grid, batch.shape, density.shape)
        cdt = density.dtype if density.dtype in (tr.float32, tr.float64) else tr.float32
        d = density.detach().to(device=dev, dtype=cdt).contiguous()
        n = batch.n
        out = tr.empty((n_chan, n) if div == 0 else (n,), dtype=cdt, device=dev)
        lib = _lib.load()
        ws = _workspace(lib, plan, n, dev)
        fn = lib.sphrt_trace_integrate_f32 if cdt == tr.float32 else lib.sphrt_trace_integrate_f64
        _lib.check(fn(plan.handle, batch.desc, _lib.ptr(d), n_chan, math.prod(grid.shape[-3:]),
                      div, _lib.ptr(out), n, _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)),
                   'sphrt_trace_integrate')
        return out.reshape(out_shape).to(device=density.device, dtype=density.dtype)


# switches of the Python construction sequence: any of them set keeps Operator construction in
# Python, as SPHRT_CONSTRUCT=python does (the parity tests and A/B runs)
_NATIVE_OFF = ('SPHRT_TRACE', 'SPHRT_TABLES', 'SPHRT_TABLE_STAGED', 'SPHRT_RUNS',
               'SPHRT_RAY_ORDER', 'SPHRT_BRICK')


class _NativeBatch:
    """What an Operator keeps of its ray batch after a native construction (debug_los prints
    the start)."""

    def __init__(self, xs, shape):
        self.xs, self.shape = xs, shape


class _TraceRecord(dict):
    """The trace's CSR record (row_ptr, vox, len, len32, tables, ...).  After the staged table
    build 'len', the float64 segment lengths, is not written: it stays in the one-pass trace's
    staging (slen at its bound slots) and is moved into the CSR on the first access — the first
    float64 forward, adjoint, time pairing or segments() — by sphrt_trace_compact(lengths only),
    which then frees the staging.  A float32-only Operator never writes it (the table build's
    writes at C3: 18 -> 10 B per segment)."""

    def __getitem__(self, k):
        if k == 'len' and dict.__getitem__(self, 'len') is None:
            self._move_len()
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        return self[k] if k in self else default

    def lengths64(self):
        """The float64 segment lengths (moved out of the trace staging on the first call)."""
        return self['len']

    def _move_len(self):
        row_ptr, bound_ptr, slen, dev = dict.pop(self, 'len_staging')
        total, n = dict.__getitem__(self, 'total'), dict.__getitem__(self, 'n')
        seg_len = tr.empty(_seg_alloc(total), dtype=tr.float64, device=dev)
        with tr.cuda.device(dev):
            stream = tr.cuda.current_stream(dev)
            _lib.check(_lib.load().sphrt_trace_compact(
                n, _lib.ptr(bound_ptr), None, _lib.ptr(slen), _lib.ptr(row_ptr), None,
                _lib.ptr(seg_len), ctypes.c_void_p(stream.cuda_stream)), 'sphrt_trace_compact(len)')
            # the staging was allocated on the construction stream: if this first float64 use
            # runs on another stream, the allocator must not hand the staging back to the
            # construction stream before the compaction has read it
            for t in (bound_ptr, slen, row_ptr):
                t.record_stream(stream)
        dict.__getitem__(self, 'desc').len = seg_len.data_ptr()
        dict.__setitem__(self, 'len', seg_len)


# ----- the operator ---------------------------------------------------------------------------

class _LineIntegral(tr.autograd.Function):
    """y = A x with dA/dx = A^T on the cached CSR; nothing large is saved for backward."""

    @staticmethod
    def forward(ctx, density, op):
        ctx.op = op
        ctx.meta = (density.shape, density.dtype, density.device)
        return op._apply_forward(density)

    @staticmethod
    def backward(ctx, grad):
        shape, dtype, device = ctx.meta
        return ctx.op._apply_adjoint(grad, shape, dtype, device), None


class Operator:
    """Raytracing operator (raytracer.py:647-755).

    Args:
        grid (SphericalGrid), geom (ViewGeom or collection), dynamic (bool or None: infer from
        geom), ftype (float64, or float32: the crossings solved and differenced in float32 as
        the reference does), itype (index dtype of the ``regs`` view), device (where results
        live; compute always runs on the current ROCm GPU), pdevice (accepted for
        compatibility), debug / debug_los (print one ray's segments), invalid (keep the
        unmasked segments, inf / NaN lengths and out-of-grid regions included: the reference's
        forward is then non-finite), _compute (False: skip the trace, for plotting-only
        operators).  float32 and invalid traces take the reference-mode trace
        (sphrt_trace_reference: every ray through the exact path); float64 takes the fast one.
    """

    def __init__(self, grid, geom, dynamic=False, ftype=FTYPE, itype=ITYPE, device=DEVICE,
                 pdevice=PDEVICE, debug=False, debug_los=None, invalid=False, _compute=True):
        self.grid = grid
        self.geom = geom
        if dynamic is None:
            dynamic = isinstance(geom, ViewGeomCollection)
        self.dynamic = dynamic
        self.ftype = ftype
        self.itype = itype
        self.device = device
        _check_ftype(ftype)
        self.invalid = bool(invalid)
        self._csr = None
        self._fast = {}     # (shape, dtype, device) -> bound forward launch (steady-state calls)
        self._fastc = None  # the same bindings inside the CPython entry (csrc/fastpath.cpp)
        self._fastc_T = None  # the adjoint's steady-state bindings (T), same entry
        self._fastc_A = None  # the time-paired adjoint's (dynamic gradient), same entry
        # 'transpose': deterministic voxel-major adjoint (default; a view <-> time pairing
        # transposes its time-paired CSR); 'atomic': float64 atomics (a cross-check, and the
        # fallback when T * vol does not fit 32-bit columns)
        self.adjoint_mode = 'transpose'
        if _compute:
            self._trace()
            if debug:
                self._debug_print(debug_los)

    # -- trace ---------------------------------------------------------------------------------
    def _trace(self):
        """The trace runs on the GPU `device` names (else the current GPU), with that GPU
        current for every allocation and launch; later calls run there too (_cdev)."""
        dev = _lib.require_gpu(self.device)
        self._cdev = dev
        with tr.cuda.device(dev):
            self._trace_on(dev)

    def _fresh_rays(self):
        """True when trace_indices' solvers each get a fresh copy of the rays: tr.asarray(rays,
        ftype) copies when the geometry's rays are not of the trace's dtype
        (raytracer.py:276,360,500), and then r_torch and e_torch normalise their own copy once and
        a_torch takes the rays unnormalised; otherwise the in-place normalisations chain
        (raytracer.py:281,365).  Every geometry class here holds float64 rays, as the
        reference's do (geometry.py:25,285-286)."""
        if isinstance(self.geom, (ViewGeom, ViewGeomCollection)):
            dt = tr.float64
        else:
            rays = self.geom.rays
            dt = rays.dtype if isinstance(rays, tr.Tensor) else tr.asarray(rays).dtype
        return dt != self.ftype

    def _reference_mode(self):
        """The trace options only the reference-mode trace takes (sphrt_trace_reference):
        float32 solves (ftype=float32), unmasked segments (invalid=True), fresh ray copies per
        solver (_fresh_rays)."""
        return self.ftype != tr.float64 or self.invalid or self._fresh_rays()

    def _trace_on(self, dev):
        if self._reference_mode():
            return self._trace_reference(dev)
        if self._trace_native(dev):
            return
        lib = _lib.load()
        # plan tables, cone-ray spec and start bins: one host-to-device copy
        stg = _Staging()
        self._plan = _Plan(self.grid, dev, staging=stg)
        cone = _ConeRays.of(self.geom)
        perm, s_perm, tiles = None, None, None
        if cone is not None:
            cone.stage(stg)
            tiles = _view_tiles(cone.shape, self.grid.dynamic) if cone.n_views > 1 else None
            if tiles is None:
                perm = _trace_order(self.geom, tr.empty(cone.shape + (3,), device='meta'),
                                    self.grid.dynamic)
            if perm is not None and perm.numel() == cone.h * cone.w:   # per view: staged too
                s_perm = stg.add(perm)
        xs_h, st_h = _RayBatch.host_starts(self.grid, self.geom.ray_starts)
        s_xs, s_st = stg.add(xs_h), stg.add(st_h)
        stg.upload(dev)
        self._plan.attach(stg)
        ray_id = None
        xs_d, st_d = stg.get(s_xs, xs_h), stg.get(s_st, st_h)
        if tiles is not None:          # view tiles: the starts broadcast over the tiled layout
            rays, ray_id = _launch_tiled(cone, dev, stg, tiles)
            tshape = (1, 1, cone.n_views // tiles[0], tiles[0], 1, 3)
            xs_h, xs_d = xs_h.reshape(tshape), xs_d.reshape(tshape)
        elif s_perm is not None:       # trace in wedges, generated in that order
            rays, ray_id = cone.launch(dev, stg, order=stg.get(s_perm, perm))
            perm = None
        elif cone is not None:
            rays = cone.launch(dev, stg)
        else:
            rays = self.geom.rays
            perm = _trace_order(self.geom, rays, self.grid.dynamic)
        if perm is not None:           # trace in wedges; rows report their geometry ray
            rays, ray_id = _permute_rays(rays, perm.to(dev, non_blocking=True))
        batch = _RayBatch(self.grid, xs_h, rays, dev, staged=(xs_d, st_d))
        self._ray_shape = cone.shape if tiles is not None else batch.shape
        n = batch.n
        stream = _lib.stream_of(dev)
        row_ptr, vox, seg_len, total, staging = _trace_csr(lib, self._plan, batch, dev, stream,
                                                           keep_staging=True)
        self._index(lib, dev, batch, row_ptr, vox, seg_len, total, ray_id, staging)

    def _trace_native(self, dev):
        """The construction below (cone detectors, float64, default switches) in one C++ call:
        _sphrt_fast.build_cone (csrc/construct.cpp) computes the same host values with the same
        torch CPU operations and runs the same one-pass trace and staged table build, without
        the Python between kernels (C2 0.80 -> see DESIGN.md §4).  False: not applicable, or a
        rare branch (a ray over its bound, a staging that does not fit) the Python sequence
        handles; nothing of the Operator was set."""
        fc = _lib.load_construct()
        if (fc is None or _bound_hook is not None or any(k in os.environ for k in _NATIVE_OFF)
                or os.environ.get('SPHRT_CONSTRUCT', 'native') == 'python'):
            return False
        shape = tuple(self.geom.shape)
        g = self.grid
        perm, tiles = None, _view_tiles(shape, g.dynamic)
        if tiles is None and len(shape) in (2, 3) and shape[-1] > _WEDGE:   # _trace_order
            perm = _wedge_order(shape[-2], shape[-1])                       # (ConeCirc views)
        c = _lib.CSR()
        geoms = getattr(self.geom, 'geoms', [self.geom])
        if all(type(v) in (ConeRectGeom, ConeCircGeom) for v in geoms):   # (type checks only:
            # _ConeRays.of would build the cone spec in Python, the work build_cone does in C++)
            res = fc.build_cone(self.geom, g.r_b, g.e_b, g.a_b, g.shape.r, g.shape.e, g.shape.a,
                                perm, tiles, math.prod(g.shape[-3:]), ctypes.addressof(c))
        else:   # ParallelGeom, ViewGeom, ...: geometry order, the host rays in the one copy
            xs, rays = self.geom.ray_starts, self.geom.rays
            if not (isinstance(xs, tr.Tensor) and isinstance(rays, tr.Tensor)):
                return False
            res = fc.build_rays(xs, rays, g.r_b, g.e_b, g.a_b, g.shape.r, g.shape.e, g.shape.a,
                                math.prod(g.shape[-3:]), ctypes.addressof(c))
        if res is None:
            return False
        (row_ptr, vox, len32, row_ray, empty_ray, blocks, loc, tab, runs, ray_id, bound_ptr, slen,
         xs, total, nblocks, rshape) = res
        self._plan = None
        self._ray_shape = rshape
        self._batch = _NativeBatch(xs, rshape)
        n = math.prod(rshape)
        self._csr = _TraceRecord(row_ptr=row_ptr, vox=vox, len=None, len32=len32, row_ray=row_ray,
                                 empty_ray=empty_ray, blocks=blocks, loc=loc, tab=tab, runs=runs,
                                 nblocks=nblocks, n=n, total=total, desc=c, ray_id=ray_id)
        self._csr['len_staging'] = (row_ptr, bound_ptr, slen, dev)
        return True

    def _trace_reference(self, dev):
        """Trace in reference mode: every ray through the exact path with the reference's own
        rules for this ftype / invalid (raytracer.py:48-173), count then fill; start voxels by
        find_starts in the trace's dtype (raytracer.py:133-137), on the host as the reference."""
        lib = _lib.load()
        stream = _lib.stream_of(dev)
        self._plan = _Plan(self.grid, dev, ftype=self.ftype)
        rays = _geom_rays(self.geom, dev)
        xs_u = tr.asarray(self.geom.ray_starts, dtype=tr.float64).detach().to('cpu').contiguous()
        st = tr.zeros(xs_u.shape[:-1] + (4,), dtype=tr.int32)
        st[..., :3] = find_starts(self.grid, xs_u, ftype=self.ftype).moveaxis(0, -1).to(tr.int32)
        staged = (xs_u.to(dev), st.to(dev))
        batch = _RayBatch(self.grid, xs_u, rays, dev, staged=staged)
        self._ray_shape = batch.shape
        n = batch.n
        flags = (_lib.TRACE_F32 if self.ftype == tr.float32 else 0) | \
            (_lib.TRACE_INVALID if self.invalid else 0) | \
            (_lib.TRACE_FRESH_RAYS if self._fresh_rays() else 0)
        counts = tr.empty(max(n, 1), dtype=tr.int32, device=dev)
        row_ptr = tr.empty(n + 1, dtype=tr.int64, device=dev)
        tws = _workspace(lib, self._plan, n, dev)
        h, d = self._plan.handle, batch.desc
        ws = tr.empty(lib.sphrt_scan_workspace_bytes(n), dtype=tr.uint8, device=dev)
        K = int(self._plan.K)
        # one pass into slots of K segments (the walk keeps at most one per list entry), then a
        # compaction — when the staging fits comfortably; else count, then fill
        if 0 < n and n * K * _STAGING_SLOT_BYTES <= _GATE_TRACE_STAGING * tr.cuda.mem_get_info(dev)[0]:
            bound_ptr = tr.arange(n + 1, dtype=tr.int64, device=dev) * K
            svox = tr.empty(n * K, dtype=tr.int32, device=dev)
            slen = tr.empty(n * K, dtype=tr.float64, device=dev)
            over = tr.empty(1, dtype=tr.int64, device=dev)
            _lib.check(lib.sphrt_trace_reference_emit(
                h, d, flags, _lib.ptr(bound_ptr), _lib.ptr(counts), _lib.ptr(svox),
                _lib.ptr(slen), _lib.ptr(over), _lib.ptr(tws), tws.numel(), stream),
                'sphrt_trace_reference_emit')
            _lib.check(lib.sphrt_scan_counts(_lib.ptr(counts), n, _lib.ptr(row_ptr),
                                             _lib.ptr(ws), stream), 'sphrt_scan_counts')
            total, n_over = tr.stack((row_ptr[n], over[0])).tolist()
            if n_over == 0:
                vox, seg_len = _compact_staging(lib, n, row_ptr, total, (bound_ptr, svox, slen),
                                                dev, stream)
                del tws, counts, ws, svox, slen, bound_ptr
                self._index(lib, dev, batch, row_ptr, vox, seg_len, total, None)
                return
            del svox, slen, bound_ptr
        else:
            _lib.check(lib.sphrt_trace_reference(h, d, flags, _lib.ptr(counts), None, None, None,
                                                 _lib.ptr(tws), tws.numel(), stream),
                       'sphrt_trace_reference(count)')
            _lib.check(lib.sphrt_scan_counts(_lib.ptr(counts), n, _lib.ptr(row_ptr),
                                             _lib.ptr(ws), stream), 'sphrt_scan_counts')
            total = int(row_ptr[n].item())
        vox = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
        seg_len = tr.empty(_seg_alloc(total), dtype=tr.float64, device=dev)
        if n > 0:
            _lib.check(lib.sphrt_trace_reference(h, d, flags, None, _lib.ptr(row_ptr),
                                                 _lib.ptr(vox), _lib.ptr(seg_len), _lib.ptr(tws),
                                                 tws.numel(), stream),
                       'sphrt_trace_reference(fill)')
        del tws, counts, ws
        self._index(lib, dev, batch, row_ptr, vox, seg_len, total, None)

    def _index(self, lib, dev, batch, row_ptr, vox, seg_len, total, ray_id, staging=None):
        """The apply kernels' row index and granule tables over a traced CSR.  With a one-pass
        trace's staging (vox / seg_len None) and one-pass tables, the table build moves the
        segments out of the staging (sphrt_csr_local_build_staged: no compaction pass, C3
        compact_kernel 0.68 ms); otherwise the staging is compacted first."""
        n = batch.n
        stream = _lib.stream_of(dev)
        batch.rays = None        # device ray directions: trace input only (24 B per ray)
        nblocks = lib.sphrt_csr_blocks(total)
        c = _lib.CSR()
        c.n_rays, c.n_segments, c.n_blocks = n, total, nblocks
        c.n_cols = math.prod(self.grid.shape[-3:])
        shape3 = tuple(int(v) for v in self.grid.shape[-3:])
        _set_stage(c, shape3, _stage_brick(nblocks, n_cols=c.n_cols))
        staged = staging is not None and os.environ.get('SPHRT_TABLE_STAGED', '1') != '0'
        if staged:
            free = tr.cuda.mem_get_info(dev)[0]
            staged = (_tables_one_pass(c, nblocks, dev, free) and
                      _staged_fits(c, nblocks, total, free))
        if staging is not None and not staged:
            vox, seg_len = _compact_staging(lib, n, row_ptr, total, staging, dev, stream)
            staging = None
        elif staged:      # (the float64 lengths stay in the staging: _TraceRecord)
            vox = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
            seg_len = None
        # row index for the apply kernels: head bits, non-empty row list, workgroup blocks
        row_ray = tr.empty(max(n, 1), dtype=tr.int32, device=dev)
        empty_ray = tr.empty(n + 1, dtype=tr.int32, device=dev)
        blocks = tr.empty(_lib.BLOCK_FIELDS * nblocks, dtype=tr.int64, device=dev)
        iws = tr.empty(lib.sphrt_csr_index_workspace_bytes(n), dtype=tr.uint8, device=dev)
        nz_row = None
        if staged:      # (head bits and the segments come with the tables)
            nz_row = tr.empty(max(n, 1), dtype=tr.int32, device=dev)
            _lib.check(lib.sphrt_csr_index_staged(_lib.ptr(row_ptr), n, _lib.ptr(row_ray),
                                                  _lib.ptr(empty_ray), _lib.ptr(blocks), nblocks,
                                                  _lib.ptr(ray_id), _lib.ptr(nz_row),
                                                  _lib.ptr(iws), stream),
                       'sphrt_csr_index_staged')
        else:
            _lib.check(lib.sphrt_csr_index(_lib.ptr(row_ptr), n, _lib.ptr(vox), _lib.ptr(row_ray),
                                           _lib.ptr(empty_ray), _lib.ptr(blocks), nblocks,
                                           _lib.ptr(ray_id), _lib.ptr(iws), stream),
                       'sphrt_csr_index')
        del iws
        c.row_ptr, c.vox = row_ptr.data_ptr(), vox.data_ptr()
        c.len = seg_len.data_ptr() if seg_len is not None else None
        # the float32 lengths come with the granule tables (sphrt_csr_local_build writes len32)
        len32 = tr.empty(vox.shape, dtype=tr.float32, device=dev)
        c.row_ray, c.blocks, c.len32 = row_ray.data_ptr(), blocks.data_ptr(), len32.data_ptr()
        c.empty_ray = empty_ray.data_ptr()
        loc, tab, runs = _local_tables(lib, c, blocks, nblocks, total, dev, stream,
                                       staged=(staging, nz_row) if staged else None)
        self._csr = _TraceRecord(row_ptr=row_ptr, vox=vox, len=seg_len, len32=len32,
                                 row_ray=row_ray, empty_ray=empty_ray, blocks=blocks, loc=loc,
                                 tab=tab, runs=runs, nblocks=nblocks, n=n, total=total, desc=c,
                                 ray_id=ray_id)
        if seg_len is None:         # the staging's lengths, kept (its voxels are freed here)
            self._csr['len_staging'] = (row_ptr, staging[0], staging[2], dev)
        del staging, nz_row
        self._batch = batch

    # -- shape logic of raytracer.py:703-712 -----------------------------------------------------
    def _layout(self, shape):
        """-> (n_chan, ray_chan_div, out_shape) for a density of `shape`."""
        return _layout_for(self.grid, self._ray_shape, shape)

    def __call__(self, density):
        """Line integrals of ``density`` along every ray: (C..., *geom.shape) for a static grid,
        (T, H, W) for a dynamic one (raytracer.py:692-713).  Differentiable in ``density``."""
        fc = self._fastc
        if fc is not None:
            # steady state in one C call (bound shapes/dtypes, contiguous, on the GPU, no grad)
            out = self._fastfn(fc, density)
            if out is not None:
                return out
        if self._csr is None:
            raise RuntimeError('Operator was built with _compute=False')
        if type(density) is tr.Tensor and not (density.requires_grad and tr.is_grad_enabled()):
            # steady-state fast path: a density already on the compute device, in a dtype and
            # shape seen before -> one allocation and one C call
            ent = self._fast.get((density.shape, density.dtype, density.device))
            if ent is not None and density.is_contiguous() and \
                    _cur_dev() == density.device.index:
                fn, desc, n_chan, n_vox, div, n, alloc, shape = ent
                out = tr.empty(alloc, dtype=density.dtype, device=density.device)
                st = _raw_stream(density.device.index)
                if fn(desc, density.data_ptr(), n_chan, n_vox, div, out.data_ptr(), n, st):
                    _lib.check(-1, 'sphrt_forward')
                _alternate(desc._obj)
                return out.view(shape)
        density = tr.as_tensor(density)
        if density.requires_grad and tr.is_grad_enabled():
            return _LineIntegral.apply(density, self)
        return self._apply_forward(density)

    def _stage_for_loop(self, dtype):
        """(descriptor copy, its stage buffer) for a loop that keeps the brick-staged density
        current itself (retrieval._gd_direct: the Adam launch writes it), or None when the
        forward CSR is not brick-staged or the grid is dynamic.  The copy's stage_packed starts
        at 0: the first _forward_staged packs."""
        desc = self._csr['desc'] if self._csr is not None else None
        if desc is None or self.grid.dynamic or not _stage_bytes(desc, 1, 1):
            return None
        self._lengths(dtype)
        need = _stage_bytes(desc, 1, tr.finfo(dtype).bits // 8)
        buf = tr.empty(need, dtype=tr.uint8, device=self._cdev)
        sd = _lib.CSR.from_buffer_copy(desc)
        sd.stage, sd.stage_bytes, sd.stage_packed = buf.data_ptr(), need, 0
        return sd, buf

    def _loop_descriptor(self, dtype):
        """A copy of the trace's forward descriptor for a loop's own launches (_forward_staged),
        or None (no trace, a dynamic grid, or a brick-staged CSR: _stage_for_loop)."""
        desc = self._csr['desc'] if self._csr is not None else None
        if desc is None or self.grid.dynamic or _stage_bytes(desc, 1, 1):
            return None
        self._lengths(dtype)            # (the float64 lengths moved into the CSR first)
        return _lib.CSR.from_buffer_copy(desc)

    def _forward_staged(self, d, out, sd):
        """Static single-channel forward of d (contiguous, on the compute device) into the flat
        out on the current stream, through a _stage_for_loop descriptor (its stage_packed says
        whether the stage already holds d)."""
        with tr.cuda.device(self._cdev):
            lib = _lib.load()
            fn = lib.sphrt_forward_f32 if d.dtype == tr.float32 else lib.sphrt_forward_f64
            _lib.check(fn(sd, _lib.ptr(d), 1, math.prod(self.grid.shape[-3:]), 0, _lib.ptr(out),
                          self._csr['n'], _lib.stream_of(self._cdev)), 'sphrt_forward')
            _alternate(sd)

    def _trace_position_rows(self, sd):
        """Point a _stage_for_loop descriptor's row -> ray and empty-ray lists at trace
        positions instead of geometry rays: its forward then writes the integral of trace
        position j to out[j] — the transposed adjoint's column order (_adjoint_trace_order), so
        the loop's residual streams f(d) and the measurements (pre-permuted once) instead of
        gathering both through the ray map, and the forward's row closes store to consecutive
        addresses.  Run records are rebuilt in trace positions (a block's rows are then one run
        but for empty rays) or dropped (list loads).  -> the list tensors (keep them alive with
        the descriptor), or None without a reordered trace."""
        csr = self._csr
        if csr is None or csr['ray_id'] is None:
            return None
        if 'trace_rows' not in csr:          # (once per trace)
            n, rid = csr['n'], self._ray_id_long()
            inv = tr.empty(n, dtype=tr.int32, device=rid.device)
            inv[rid] = tr.arange(n, dtype=tr.int32, device=rid.device)
            # (entries past the lists' lengths are never used; clamped so the gather stays in
            # range)
            rows = inv[csr['row_ray'].long().clamp_(0, n - 1)]
            empty = inv[csr['empty_ray'].long().clamp_(0, n - 1)]
            # run records in trace positions, where a block's rows are consecutive but for
            # empty rays (_local_tables' rule: grids of more than one wave of workgroups)
            runs = None
            mode = os.environ.get('SPHRT_RUNS', 'auto')
            if (mode == 'on' or (mode == 'auto' and csr['nblocks'] > _SINGLE_WAVE_BLOCKS)) \
                    and n < 2 ** 31:
                lib = _lib.load()
                tmp = _lib.CSR.from_buffer_copy(sd)
                tmp.row_ray, tmp.empty_ray = rows.data_ptr(), empty.data_ptr()
                runs = tr.empty(_lib.RUN_FIELDS * csr['nblocks'], dtype=tr.int32,
                                device=rid.device)
                over = tr.empty(1, dtype=tr.int64, device=rid.device)
                _lib.check(lib.sphrt_csr_runs(tmp, _lib.ptr(runs), _lib.ptr(over),
                                              _lib.stream_of(rid.device)), 'sphrt_csr_runs')
                if over.item():
                    runs = None
            csr['trace_rows'] = (rows, empty, runs)
        rows, empty, runs = csr['trace_rows']
        sd.row_ray, sd.empty_ray = rows.data_ptr(), empty.data_ptr()
        sd.runs = runs.data_ptr() if runs is not None else None
        return rows, empty, runs

    def _lengths(self, dtype):
        """Segment lengths as streamed by the forward kernel: the float64 trace, or (float32
        path) its float32 copy — half the bytes, <=6e-8 relative rounding — written by the
        granule-table launch (no pass of its own: C3 f64_to_f32_kernel 0.25 ms)."""
        csr = self._csr
        return csr['len'] if dtype == tr.float64 else csr['len32']

    def _launch_args(self, d, n_chan, div):
        """(csr desc, n_chan, chan_stride, div) of the launch for density d: a view <-> time
        pairing runs as a static single-channel forward over the flattened (T, vol) density on
        the time-paired CSR (its granule tables apply); everything else on the trace's CSR."""
        vol = math.prod(self.grid.shape[-3:])
        if div > 0:
            rec = self._paired(d.shape[0], div)
            if rec is not None:   # (the trace's lengths: the float64 ones once moved, _lengths)
                rec['desc'].len32 = self._csr['desc'].len32
                rec['desc'].len = self._csr['desc'].len
                return rec['desc'], 1, rec['desc'].n_cols, 0
        return self._csr['desc'], n_chan, vol, div

    def _launch_forward(self, d, out, n_chan, div):
        """Enqueue the forward kernel on the current stream: d (contiguous, compute device,
        float32/float64) -> out (preallocated, same dtype).  No host sync; a brick-staged CSR
        allocates its stage for the call from the caching allocator."""
        lib = _lib.load()
        self._lengths(d.dtype)
        desc, n_chan, cs, div = self._launch_args(d, n_chan, div)
        if d.dtype == tr.float64 and not desc.len:
            raise RuntimeError('float64 forward without the float64 segment lengths')
        fn = lib.sphrt_forward_f32 if d.dtype == tr.float32 else lib.sphrt_forward_f64
        _call_forward(fn, desc, d, n_chan, cs, div, out, self._csr['n'], self._cdev)
        _alternate(desc)

    def _forward_kernel_name(self, d):
        """The forward kernel instantiation a launch on `d` runs (sphrt_forward_*'s choice, for
        reports): 0 = granule tables staged in LDS, 1 = per-segment gathers, 2 = time slices;
        the last flag: float64 half tables."""
        n_chan, div, _ = self._layout(d.shape)
        c, n_chan, _, div = self._launch_args(d, n_chan, div)
        return self._kernel_name_for(c, d, n_chan, div)

    def _adjoint_kernel_name(self, d):
        """The instantiation the adjoint of a density like `d` runs (the transposed CSR's
        forward; a dynamic grid's time-paired gradient), after the first adjoint built it."""
        n_chan, div, _ = self._layout(d.shape)
        if div > 0:
            c = self._paired(d.shape[0], div)['transposed']['desc']
        else:
            c = self._transposed()['desc']
        return self._kernel_name_for(c, d, 1, 0)

    @staticmethod
    def _kernel_name_for(c, d, n_chan, div):
        t = 'float, float' if d.dtype == tr.float32 else 'double, double'
        es = d.element_size()
        dense = 'true' if c.order & 4 else 'false'     # (dense output ranges, sphrt.h order)
        aligned = d.data_ptr() % (4 * es) == 0 and (n_chan == 1 or d[0].numel() % 4 == 0)
        extra = 2560 * es if c.order & 4 else 0          # (apply.hip kOutStage)
        table = (c.loc and div == 0 and 0 < c.tab_stride
                 and (max(c.tab_stride, 768) + 1) * 4 * es + extra <= 64 * 1024
                 and (c.stage_shape[0] > 0 or aligned))
        if table:   # early granule DMA whenever the table columns are whole granules
            cols = c.stage_cols if c.stage_shape[0] > 0 else c.n_cols
            edma = 'true' if cols % 4 == 0 else 'false'
            tabt = 'unsigned short' if c.tab_bytes == 2 else 'int'
            runs = 'true' if c.runs else 'false'
            # float64 half tables (apply.hip kHalfTab = 768 granules per phase)
            half = (es == 8 and edma == 'true' and (c.tab_stride + 1) * 32 > 40 * 1024
                    and c.tab_stride <= 1536 and os.environ.get('SPHRT_FWD_HALF', '1') != '0')
            # early DMA rounds: 256-entry chunks of the largest table (apply.hip launch_forward)
            ge = 3 if half or edma == 'false' else min(3, max(1, -(-c.tab_stride // 256)))
            return (f'forward_kernel<{t}, 0, {tabt}, {edma}, 8, {runs}, '
                    f'{"true" if half else "false"}, {dense}, {ge}>')
        return f'forward_kernel<{t}, {2 if div else 1}, int, false, 8, false, false, {dense}, 3>'

    def _apply_forward(self, density):
        with tr.cuda.device(self._cdev):      # launches and allocations on the operator's GPU
            return self._apply_forward_on(density)

    def _apply_forward_on(self, density):
        dev = self._cdev
        n_chan, div, out_shape = self._layout(density.shape)
        in_dtype = density.dtype
        cdt = in_dtype if in_dtype in (tr.float32, tr.float64) else tr.float32
        d = density.detach()
        if d.device != dev or d.dtype != cdt or not d.is_contiguous():
            d = d.to(device=dev, dtype=cdt).contiguous()
        n = self._csr['n']
        alloc = (n_chan, n) if div == 0 else (n,)
        out = tr.empty(alloc, dtype=cdt, device=dev)
        self._launch_forward(d, out, n_chan, div)
        if density.device == dev and density.dtype == cdt and density.is_contiguous():
            lib = _lib.load()
            fn = lib.sphrt_forward_f32 if cdt == tr.float32 else lib.sphrt_forward_f64
            desc, b_chan, b_cs, b_div = self._launch_args(d, n_chan, div)
            stage = _stage_bytes(desc, b_chan, d.element_size())
            if not stage:     # the ctypes fast path has no per-call stage
                self._fast[(density.shape, density.dtype, density.device)] = (
                    fn, ctypes.byref(desc), b_chan, b_cs, b_div, n, alloc, tuple(out_shape))
            fast = _lib.load_fast()
            if fast is not None:
                if self._fastc is None:
                    self._fastfn = fast.forward
                    self._fastc = fast.new(_lib.address(lib.sphrt_last_error))
                fast.add(self._fastc, tuple(density.shape), cdt == tr.float64, dev.index,
                         _lib.address(fn), ctypes.addressof(desc), b_chan, b_cs, b_div, n,
                         tuple(out_shape), stage)
        out = out.view(out_shape)
        if out.device != density.device or cdt != in_dtype:
            out = out.to(device=density.device, dtype=in_dtype)
        return out

    def _transposed(self):
        """Voxel-major copy of the trace (built on the first adjoint): the adjoint then runs the
        forward's segmented gather-reduce with rays and voxels swapped — no atomics,
        bitwise reproducible."""
        csr = self._csr
        if 'T' not in csr:
            csr['T'] = self._transpose_of(csr['desc'], math.prod(self.grid.shape[-3:]),
                                          csr['vox'])
        return csr['T']

    def _ray_shape3(self):
        """The rays' layout as 3 dims (views, rows, columns of the detector) for brick staging of
        a transposed CSR, whose columns are rays."""
        shape = [int(v) for v in self.geom.shape]
        if math.prod(shape) != self._csr['n']:
            return None
        shape = [1] * max(0, 3 - len(shape)) + shape
        return (math.prod(shape[:-2]), shape[-2], shape[-1])

    def _transpose_of(self, src, n_cols, vox, dense=False):
        """Transpose of the CSR `src` (columns < n_cols; `vox` its column tensor) with its own
        index and granule tables; its columns (rays) are brick-staged in detector tiles for
        multi-wave grids.  Its rows (voxels) are ordered brick by brick (_voxel_rows) and report
        their voxel through the index's row ids.  dense (rows in linear order): every workgroup
        owns a contiguous output range and zeroes it itself (_dense_ranges)."""
        csr = self._csr
        lib, dev = _lib.load(), self._cdev
        stream = _lib.stream_of(dev)
        n_vox = n_cols
        total = csr['total']
        csr['len']                       # (the float64 lengths moved out of the staging, if not yet)
        src.len = csr['desc'].len        # (a time-paired CSR shares the trace's lengths)
        rows = _voxel_rows(tuple(int(v) for v in self.grid.shape[-3:]), n_cols, dev,
                           csr['nblocks'])
        if rows is not None:             # the columns renumbered in row order for the sort
            vpos = rows.vpos
            v = vox[:total]
            pos = vpos.index_select(0, v & 0x7fffffff)
            vox_pos = tr.where(v < 0, pos | _HEAD32, pos)
            src = _lib.CSR.from_buffer_copy(src)
            src.vox = vox_pos.data_ptr()
        col_ptr = tr.empty(n_vox + 1, dtype=tr.int64, device=dev)
        t_ray = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
        t_len = tr.empty(_seg_alloc(total), dtype=tr.float64, device=dev)
        ws = tr.empty(lib.sphrt_transpose_workspace_bytes(total, n_vox), dtype=tr.uint8, device=dev)
        _lib.check(lib.sphrt_csr_transpose(src, n_vox, _lib.ptr(col_ptr), _lib.ptr(t_ray),
                                           _lib.ptr(t_len), _lib.ptr(ws), ws.numel(), stream),
                   'sphrt_csr_transpose')
        del ws
        if rows is not None:
            del vox_pos, pos, v
        geom_cols = self._tcols_geom()
        if geom_cols:                    # columns: the rows' geometry rays instead of trace rows
            t_ray[:total] = csr['ray_id'].index_select(0, t_ray[:total])
        # (dense output ranges: the blocks of that layout, sphrt_csr_index_dense)
        ranges = dense and rows is None
        nblocks = (lib.sphrt_csr_blocks_dense if ranges else lib.sphrt_csr_blocks)(total)
        vox_list = tr.empty(n_vox, dtype=tr.int32, device=dev)
        empty_vox = tr.empty(n_vox + 1, dtype=tr.int32, device=dev)
        blocks = tr.empty(_lib.BLOCK_FIELDS * nblocks, dtype=tr.int64, device=dev)
        iws = tr.empty(lib.sphrt_csr_index_workspace_bytes(n_vox), dtype=tr.uint8, device=dev)
        index = lib.sphrt_csr_index_dense if ranges else lib.sphrt_csr_index
        _lib.check(index(_lib.ptr(col_ptr), n_vox, _lib.ptr(t_ray), _lib.ptr(vox_list),
                         _lib.ptr(empty_vox), _lib.ptr(blocks), nblocks,
                         _lib.ptr(rows.vperm) if rows is not None else None, _lib.ptr(iws),
                         stream),
                   'sphrt_csr_index(T)')
        t_len32 = tr.empty(t_len.shape, dtype=tr.float32, device=dev)   # (filled with the tables)
        c = _lib.CSR()
        c.n_rays, c.n_segments, c.n_blocks = n_vox, total, nblocks
        c.row_ptr, c.vox, c.len, c.len32 = (col_ptr.data_ptr(), t_ray.data_ptr(),
                                            t_len.data_ptr(), t_len32.data_ptr())
        c.row_ray, c.blocks = vox_list.data_ptr(), blocks.data_ptr()
        c.empty_ray = empty_vox.data_ptr()
        c.n_cols = csr['n']
        # (columns are trace rows: detector tiles only when they are the geometry's rays; none
        # for the dense time-paired transpose: a pack launch per call for no kernel gain)
        shape3 = (self._ray_shape3() if (csr['ray_id'] is None or geom_cols) and not dense
                  else None)
        _set_stage(c, shape3, _stage_brick(nblocks, 'SPHRT_BRICK_T', _BRICK_RAYS)
                   if shape3 else None)
        loc, tab, runs = _local_tables(lib, c, blocks, nblocks, total, dev, stream)
        if ranges:
            _dense_ranges(c, blocks, vox_list, n_vox)
            runs = None
        return dict(desc=c, keep=(col_ptr, t_ray, t_len, t_len32, vox_list, empty_vox, blocks,
                                  loc, tab, runs, rows))

    def _paired(self, T, div):
        """The trace with time-paired columns (ray r reads slice r // div: column
        (r // div) * vol + voxel), its own blocks and granule tables: a view <-> time pairing is
        then a static forward over the flattened (T, vol) density, and its adjoint the
        transposed forward (deterministic, no atomics).  None when T * vol >= 2^31."""
        csr = self._csr
        key = ('paired', T, div)
        if key in csr:
            return csr[key]
        vol = math.prod(self.grid.shape[-3:])
        if T * vol >= 2 ** 31 - 1 or -(-csr['n'] // div) > T:
            csr[key] = None
            return None
        lib, dev = _lib.load(), self._cdev
        stream = _lib.stream_of(dev)
        total, nblocks = csr['total'], csr['nblocks']
        vox_p = tr.empty(_seg_alloc(total), dtype=tr.int32, device=dev)
        _lib.check(lib.sphrt_csr_time_columns(csr['desc'], div, vol, _lib.ptr(vox_p), stream),
                   'sphrt_csr_time_columns')
        blocks_p = csr['blocks'].clone()            # n_tab (field 5) is per table set
        c = _lib.CSR.from_buffer_copy(csr['desc'])
        _clear_stage(c)                             # time-paired columns are not bricked
        c.vox, c.blocks, c.n_cols = vox_p.data_ptr(), blocks_p.data_ptr(), T * vol
        c.order |= 2        # disjoint slices per view: one contiguous block range per XCD (sphrt.h)
        c.loc, c.tab, c.tab_stride, c.n_fallback = None, None, 0, 0
        l32, c.len32 = c.len32, None                # (the trace's float32 lengths: made already)
        loc, tab, runs = _local_tables(lib, c, blocks_p, nblocks, total, dev, stream)
        c.len32 = l32
        csr[key] = dict(desc=c, keep=(vox_p, blocks_p, loc, tab, runs), n_t=T)
        return csr[key]

    def _apply_adjoint(self, y, dshape, ddtype, ddevice, trace_order=False):
        fa = self._fastc_A
        if fa is not None and not trace_order and y.dtype == ddtype and ddevice == self._cdev:
            # steady state of the time-paired adjoint in one C call (y gathered into trace
            # order and the transposed forward, csrc/fastpath.cpp): the autograd backward of a
            # dynamic forward and Operator.T(y, time_slices=True) land here
            out = self._fastfn(fa, y)
            if out is not None:
                return out
        with tr.cuda.device(self._cdev):
            res = self._apply_adjoint_on(y, dshape, ddtype, ddevice, trace_order)
            if not trace_order:
                self._bind_paired_adjoint(y, dshape, res)
            return res

    def _bind_paired_adjoint(self, y, dshape, res):
        """Register the steady-state binding of the time-paired adjoint for y's shape / dtype
        when the general path ran just the gather and the transposed forward: y contiguous on
        the compute device, float32 / float64, the result there in y's dtype."""
        csr, dev = self._csr, self._cdev
        if not (self.grid.dynamic and type(y) is tr.Tensor and y.device == dev
                and res.device == dev and y.dtype in (tr.float32, tr.float64)
                and res.dtype == y.dtype and y.is_contiguous()
                and self.adjoint_mode == 'transpose' and csr is not None
                and y.numel() == csr['n']):
            return
        n_chan, div, _ = self._layout(dshape)
        paired = csr.get(('paired', dshape[0], div)) if div > 0 else None
        if paired is None or 'transposed' not in paired:
            return
        fast = _lib.load_fast()
        if fast is None:
            return
        tdesc = paired['transposed']['desc']
        lib = _lib.load()
        fn = lib.sphrt_forward_f32 if y.dtype == tr.float32 else lib.sphrt_forward_f64
        gfn = lib.sphrt_gather_f32 if y.dtype == tr.float32 else lib.sphrt_gather_f64
        if self._fastc_A is None:
            self._fastfn = fast.forward
            self._fastc_A = fast.new(_lib.address(lib.sphrt_last_error))
        perm = csr['ray_id'] if csr['ray_id'] is not None and not self._tcols_geom() else None
        fast.add(self._fastc_A, tuple(y.shape), y.dtype == tr.float64, dev.index,
                 _lib.address(fn), ctypes.addressof(tdesc), 1, csr['n'], 0, tdesc.n_rays,
                 tuple(dshape), _stage_bytes(tdesc, 1, y.element_size()), perm,
                 _lib.address(gfn))

    def _tcols_geom(self):
        """Whether the transposed CSRs of a reordered trace (wedges, view tiles) take their
        columns in geometry ray order — their t_ray mapped through ray_id once at transpose
        time: the adjoint reads y as given (no gather per call) and y is brick-staged in
        detector tiles — or in trace-row order (y gathered into trace order per call, or written
        so by the retrieval's residual).  Measured (op.T per step, us; profiles/r05_tcols_*):
        ConeRect orbits take geometry columns (C2 11.7 -> 7.2, C3 214.5 -> 187.2), ConeCirc
        orbits keep trace rows (C5 41.4 against 44.2; its kernel 25.1 / 35.6 us f32 / f64 against
        28.3-30.8 / 39.7-44.0 with geometry columns and any ray brick).  Dynamic grids (the
        time-paired transpose, whose columns are never brick-staged) take geometry columns: C4's
        adjoint call 29.0 -> 25.9 us, the per-call gather of y gone and the kernel unchanged (25.9
        / 25.7 us; profiles/r06_adjstats_c4*.json).  SPHRT_TCOLS=geom / trace overrides."""
        csr = self._csr
        if csr is None or csr['ray_id'] is None:
            return False
        env = os.environ.get('SPHRT_TCOLS', 'auto')
        if env != 'auto':
            return env == 'geom'
        if self.grid.dynamic:
            return True
        geoms = getattr(self.geom, 'geoms', [self.geom])
        return bool(geoms) and all(type(g) is ConeRectGeom for g in geoms)

    def _adjoint_trace_order(self):
        """The row -> geometry ray map (int32, device) when the adjoint takes its input in
        trace order (static, transposed adjoint, a reordered trace with trace-row columns),
        else None."""
        csr = self._csr
        if (self.grid.dynamic or self.adjoint_mode != 'transpose' or csr is None
                or self._tcols_geom()):
            return None
        return csr['ray_id']

    def _apply_adjoint_on(self, y, dshape, ddtype, ddevice, trace_order=False):
        """trace_order: y is already in trace order (_adjoint_trace_order's map applied)."""
        dev = self._cdev
        n_chan, div, out_shape = self._layout(dshape)
        csr = self._csr
        n = csr['n']
        vol = math.prod(self.grid.shape[-3:])
        ydt = y.dtype if y.dtype in (tr.float32, tr.float64) else tr.float32
        yv = y.detach().to(device=dev, dtype=ydt).reshape(-1).contiguous()
        if yv.numel() != n_chan * n:
            raise ValueError(f'adjoint input has {yv.numel()} values, expected {n_chan * n}')
        paired = self._paired(dshape[0], div) if div > 0 else None
        if self.adjoint_mode == 'transpose' and (div == 0 or paired is not None):
            cdt = ddtype if ddtype in (tr.float32, tr.float64) else tr.float32
            yv = yv.to(cdt)
            if csr['ray_id'] is not None and not trace_order and not self._tcols_geom():
                # (its columns are trace rows: y gathered into trace order)
                yv = _gather(yv, csr['ray_id'], n, dev) if yv.numel() == n else \
                    yv.view(-1, n).index_select(1, self._ray_id_long()).reshape(-1)
            if paired is not None:      # columns of the flattened (T, vol) density
                if 'transposed' not in paired:
                    paired['transposed'] = self._transpose_of(paired['desc'],
                                                              paired['desc'].n_cols,
                                                              paired['keep'][0], dense=True)
                tdesc, n_chan, vol = paired['transposed']['desc'], 1, paired['desc'].n_cols
            else:
                tdesc = self._transposed()['desc']
            res = tr.empty(n_chan * vol, dtype=cdt, device=dev)
            lib = _lib.load()
            fn = lib.sphrt_forward_f32 if cdt == tr.float32 else lib.sphrt_forward_f64
            _call_forward(fn, tdesc, yv, n_chan, n, 0, res, vol, dev)
            _alternate(tdesc)
            return res.reshape(dshape).to(device=ddevice, dtype=ddtype)
        acc = tr.zeros(math.prod(dshape), dtype=tr.float64, device=dev)
        csr['len']                       # (the float64 lengths moved out of the staging, if not yet)
        _lib.check(_lib.load().sphrt_adjoint_accumulate(
            csr['desc'], _lib.ptr(yv), int(ydt == tr.float64), n_chan, n, div, _lib.ptr(acc), vol,
            _lib.stream_of(dev)), 'sphrt_adjoint_accumulate')
        if ddtype == tr.float64:
            res = acc
        elif ddtype == tr.float32:
            res = tr.empty(acc.shape, dtype=tr.float32, device=dev)
            _lib.check(_lib.load().sphrt_f64_to_f32(_lib.ptr(acc), _lib.ptr(res), acc.numel(),
                                                     _lib.stream_of(dev)), 'sphrt_f64_to_f32')
        else:
            res = acc.to(ddtype)
        return res.reshape(dshape).to(ddevice)

    def T(self, line_integrations, *, time_slices=False):
        """Back-projection of ``line_integrations`` (geom.shape) into a grid.shape volume
        (raytracer.py:715-748).  Static grids only, like the reference (raytracer.py:733-734
        raises for a dynamic grid) — unless ``time_slices=True``: a dynamic grid's adjoint, y of
        shape (T, H, W) -> (T, nr, ne, na), view i back-projected into time slice i (or every
        time step's image through the one geometry), i.e. the gradient autograd gives the
        forward, natively (the time-paired CSR transposed)."""
        if self.grid.dynamic:
            if not time_slices:
                raise NotImplementedError
            y = tr.as_tensor(line_integrations)
            if self._csr is None:
                raise RuntimeError('Operator was built with _compute=False')
            dshape = (int(y.shape[0]),) + tuple(int(v) for v in self.grid.shape[1:])
            return self._apply_adjoint(y, dshape, y.dtype, tr.device(self.device))
        fc = self._fastc_T
        if fc is not None:
            # steady state in one C call: the transposed CSR's forward (csrc/fastpath.cpp)
            out = self._fastfn(fc, line_integrations)
            if out is not None:
                return out
        y = tr.as_tensor(line_integrations)
        res = self._apply_adjoint(y, tuple(self.grid.shape), y.dtype, tr.device(self.device))
        self._bind_adjoint(y, res)
        return res

    def _bind_adjoint(self, y, res):
        """Register T's steady-state binding for y's shape/dtype when the general path did no
        more than one transposed-CSR forward: y contiguous on the compute device, float32/64, the
        result left there in y's dtype.  A trace in another ray order (wedges, view tiles) reads
        y through its ray ids (index_select in the same call); a brick-staged transpose gets its
        stage buffer per call, as in _call_forward."""
        csr, dev = self._csr, self._cdev
        if not (type(y) is tr.Tensor and y.device == dev and res.device == dev
                and y.dtype in (tr.float32, tr.float64) and res.dtype == y.dtype
                and y.is_contiguous() and self.adjoint_mode == 'transpose'
                and csr is not None and y.numel() == csr['n']):
            return
        tdesc = self._transposed()['desc']
        fast = _lib.load_fast()
        if fast is None:
            return
        lib = _lib.load()
        fn = lib.sphrt_forward_f32 if y.dtype == tr.float32 else lib.sphrt_forward_f64
        if self._fastc_T is None:
            self._fastfn = fast.forward
            self._fastc_T = fast.new(_lib.address(lib.sphrt_last_error))
        vol = math.prod(self.grid.shape[-3:])
        gfn = lib.sphrt_gather_f32 if y.dtype == tr.float32 else lib.sphrt_gather_f64
        fast.add(self._fastc_T, tuple(y.shape), y.dtype == tr.float64, dev.index,
                 _lib.address(fn), ctypes.addressof(tdesc), 1, csr['n'], 0, vol,
                 tuple(res.shape), _stage_bytes(tdesc, 1, y.element_size()),
                 None if self._tcols_geom() else csr['ray_id'], _lib.address(gfn))

    # -- compatibility views -----------------------------------------------------------------------
    def _padded(self):
        csr = self._csr
        row_ptr, seg_vox, seg_len = self.segments()      # geometry order
        seg_len = seg_len.to(self.ftype)                  # (float32 traces: exact)
        counts = (row_ptr[1:] - row_ptr[:-1])
        smax = max(int(counts.max().item()) if csr['n'] else 0, 1)
        n, total = csr['n'], csr['total']
        ray = tr.repeat_interleave(tr.arange(n, device=row_ptr.device), counts)
        pos = tr.arange(total, device=row_ptr.device) - row_ptr[:-1][ray]
        vox = tr.zeros((n, smax), dtype=tr.int64, device=row_ptr.device)
        lens = tr.zeros((n, smax), dtype=self.ftype, device=row_ptr.device)
        vox[ray, pos] = seg_vox.to(tr.int64)
        lens[ray, pos] = seg_len
        _, ne, na = self.grid.shape[-3:]
        regs = tr.stack((vox // (ne * na), (vox // na) % ne, vox % na))
        R = tuple(self._ray_shape)
        return regs.reshape((3,) + R + (smax,)), lens.reshape(R + (smax,))

    @property
    def regs(self):
        """(3, *rays, S_max) voxel indices (padded; compatibility view of the CSR)."""
        return self._padded()[0].to(device=self.device, dtype=self.itype)

    @property
    def lens(self):
        """(*rays, S_max) segment lengths matching ``regs`` (zero padding), in the trace's
        ftype.  invalid=True: every non-zero length of the reference's list, inf and NaN
        included, with ``regs`` holding the wrapped voxel the reference's forward reads (-1 ->
        n - 1)."""
        return self._padded()[1].to(device=self.device)

    def _ray_id_long(self):
        c = self._csr
        if 'ray_id_long' not in c:
            c['ray_id_long'] = c['ray_id'].long()
        return c['ray_id_long']

    def segments(self):
        """The trace itself: (row_ptr int64 (n+1,), linear voxel int32, len float64) on the GPU;
        segment s of ray i is row_ptr[i] <= s < row_ptr[i+1], voxel (r*ne + e)*na + a.  Rays in
        geometry order (a trace made in another order is reordered here)."""
        c = self._csr
        row_ptr, vox = c['row_ptr'], c['vox'][:c['total']] & 0x7FFFFFFF
        seg = c['len'][:c['total']]
        if c['ray_id'] is None:
            return row_ptr, vox, seg
        rid = self._ray_id_long()                     # trace row k -> geometry ray rid[k]
        counts = row_ptr[1:] - row_ptr[:-1]
        g_counts = tr.empty_like(counts)
        g_counts[rid] = counts
        g_ptr = tr.zeros_like(row_ptr)
        g_ptr[1:] = tr.cumsum(g_counts, 0)
        # segment j of trace row k goes to g_ptr[rid[k]] + j
        row = tr.repeat_interleave(tr.arange(c['n'], device=row_ptr.device), counts)
        dst = g_ptr[rid][row] + (tr.arange(c['total'], device=row_ptr.device) - row_ptr[:-1][row])
        g_vox, g_seg = tr.empty_like(vox), tr.empty_like(seg)
        g_vox[dst], g_seg[dst] = vox, seg
        return g_ptr, g_vox, g_seg

    def _debug_print(self, debug_los):
        R = tuple(self._ray_shape)
        if debug_los is None:
            debug_los = (0,) * len(R)
        i = 0
        for k, s in zip(debug_los, R):
            i = i * s + k
        row_ptr, vox, seg = self.segments()
        a, b = int(row_ptr[i]), int(row_ptr[i + 1])
        _, ne, na = self.grid.shape[-3:]
        print('ray_start:', self._batch.xs.reshape(-1, 3)[0].tolist())
        print('  r   e   a      len')
        for v, l in zip(vox[a:b].tolist(), seg[a:b].tolist()):
            print(f'{v // (ne * na):3d} {(v // na) % ne:3d} {v % na:3d}  {l:.6g}')

    def __repr__(self):
        if self.dynamic:
            return f"Operator({(self.geom.shape[0], *self.grid.shape)} → {self.geom.shape})"
        return f"Operator({self.grid.shape} → {self.geom.shape})"

    def plot(self, *args, **kwargs):
        raise NotImplementedError('plotting is out of scope for sph_raytracer_amd')
