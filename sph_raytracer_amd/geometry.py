"""Spherical grid and detector ("view") geometries — host-side inputs of the raytracer.

API-compatible with the reference's ``sph_raytracer.geometry`` (geometry.py:1-681): same
classes, constructor arguments, attributes and properties, and the same torch arithmetic for
boundary vectors and ray directions, so ``Operator`` sees bit-identical rays.  These are O(rays)
host computations, not kernels.  Plotting methods (``plot``) are out of
scope (visualisation); ``_wireframe`` is kept because tests and ``Operator.plot`` callers touch it.
"""
from collections import namedtuple
import math

import torch as tr

__all__ = ['SphericalGrid', 'ConeRectGeom', 'ConeCircGeom',
           'ViewGeomCollection', 'ViewGeom', 'ParallelGeom']

FTYPE = tr.float64

StaticSize = namedtuple('Size', ['r', 'e', 'a'])
StaticShape = namedtuple('Shape', ['r', 'e', 'a'])
DynamicSize = namedtuple('Size', ['t', 'r', 'e', 'a'])
DynamicShape = namedtuple('Shape', ['t', 'r', 'e', 'a'])


def _f64(x):
    return tr.asarray(x, dtype=tr.float64)


def _centers(b):
    return (b[1:] + b[:-1]) / 2


class SphericalGrid:
    """Voxel grid in (r, e, a) = (radius, elevation from +Z, azimuth from +X).

    Mirrors geometry.py:27-252.  Either give ``shape`` (3-D static or 4-D dynamic) plus extents
    ``size_*`` (radial spacing ``'lin'`` or ``'log'``), or give the boundary vectors
    ``r_b, e_b, a_b`` (and optionally sample times ``t``) directly.  Boundaries are float64.
    ``rs_b/phis_b/thetas_b`` are the reference's deprecated aliases.
    """

    def __init__(self, shape=(50, 50, 50), size_t=(0, 1), size_r=(0, 1), size_e=(0, tr.pi),
                 size_a=(-tr.pi, tr.pi), spacing='lin', t=None, r_b=None, e_b=None, a_b=None,
                 timeunit='s', rs_b=None, phis_b=None, thetas_b=None):
        if len(shape) == 3:
            self.dynamic = False
            shape = StaticShape(*shape[-3:])
            size = StaticSize(size_r, size_e, size_a)
        elif len(shape) == 4:
            self.dynamic = True
            shape = DynamicShape(*shape)
            size = DynamicSize(size_t, size_r, size_e, size_a)
        else:
            raise ValueError("shape must be 3D or 4D")

        if rs_b is not None and phis_b is not None and thetas_b is not None:
            r_b, e_b, a_b = rs_b, phis_b, thetas_b

        if r_b is not None and e_b is not None and a_b is not None:
            # explicit boundaries: extents and shape follow from them
            extent = [(float(min(b)), float(max(b))) for b in (r_b, e_b, a_b)]
            if t is None:
                shape = StaticShape(len(r_b) - 1, len(e_b) - 1, len(a_b) - 1)
                size = StaticSize(*extent)
            else:
                t = _f64(t)
                shape = DynamicShape(len(t), len(r_b) - 1, len(e_b) - 1, len(a_b) - 1)
                size = DynamicSize((float(min(t)), float(max(t))), *extent)
                self.dynamic = True
            r_b, e_b, a_b = (_f64(b) for b in (r_b, e_b, a_b))
            r, e, a = (_centers(b) for b in (r_b, e_b, a_b))
        elif shape is not None and size is not None:
            if len(shape) == 4:
                t = tr.linspace(size.t[0], size.t[1], shape.t, dtype=tr.float64)
            if spacing == 'lin':
                r_b = tr.linspace(size.r[0], size.r[1], shape.r + 1, dtype=tr.float64)
                r = _centers(r_b)
            elif spacing == 'log':
                r_b = tr.logspace(math.log10(size.r[0]), math.log10(size.r[1]), shape.r + 1,
                                  dtype=tr.float64)
                r = tr.sqrt(r_b[1:] * r_b[:-1])
            else:
                raise ValueError("Invalid value for spacing")
            e_b = tr.linspace(size.e[0], size.e[1], shape.e + 1, dtype=tr.float64)
            a_b = tr.linspace(size.a[0], size.a[1], shape.a + 1, dtype=tr.float64)
            e, a = _centers(e_b), _centers(a_b)
        else:
            raise ValueError("Must specify either shape or (r, e, a)")

        self.size, self.shape, self.spacing, self.timeunit = size, shape, spacing, timeunit
        self.r_b, self.e_b, self.a_b = r_b, e_b, a_b
        self.t, self.r, self.e, self.a = t, r, e, a
        # deprecated aliases kept by the reference
        self.rs_b, self.phis_b, self.thetas_b = r_b, e_b, a_b
        self.rs, self.phis, self.thetas = r, e, a

    def __repr__(self):
        lines = [f'{type(self).__name__}(', f'shape={tuple(self.shape)},']
        lines += [f'size_{k}=({v[0]:.2f}, {v[1]:.2f}),' for k, v in self.size._asdict().items()]
        return '\n    '.join(lines[:-1] + [lines[-1]]) + '\n)'

    @property
    def coords(self):
        names = ('t', 'r', 'e', 'a') if self.dynamic else ('r', 'e', 'a')
        return {k: getattr(self, k) for k in names}

    @property
    def mesh(self):
        """Dense grid of bin centres, (N_t, N_r, N_e, N_a, 4) dynamic / (N_r, N_e, N_a, 3) static."""
        return tr.stack(tr.meshgrid(list(self.coords.values()), indexing='ij'), dim=-1)

    @property
    def nptime(self):
        return self.t.numpy().astype(f'datetime64[{self.timeunit}]')

    def plot(self, ax=None):
        raise NotImplementedError('plotting is out of scope for sph_raytracer_amd')


# ----- view geometries ------------------------------------------------------------------------

def _frame(pos, lookdir, updir):
    """Detector frame as in geometry.py:474-485: default lookdir points at the origin, default
    updir = lookdir x Z (computed before normalisation); both normalised in place."""
    pos = _f64(pos)
    look = -pos if lookdir is None else _f64(lookdir)
    up = tr.cross(look, _f64((0, 0, 1)), dim=-1) if updir is None else _f64(updir)
    look /= tr.linalg.norm(look, axis=-1)
    up /= tr.linalg.norm(up, axis=-1)
    return pos, look, up


def _unit_rows(v):
    v /= tr.linalg.norm(v, axis=-1)[..., None]
    return v


class ViewGeom:
    """Arbitrary detector: one (start, direction) pair per pixel, any leading shape.

    geometry.py:259-351.  Directions are normalised (on a private copy; the reference divides
    the caller's float64 tensor in place).
    """

    def __init__(self, ray_starts, rays):
        self.ray_starts = _f64(ray_starts)
        self.rays = _unit_rows(_f64(rays).clone())
        self.shape = self.rays.shape[:-1]

    def __add__(self, other):
        if other is None or (not isinstance(other, ViewGeom) and other == 0):
            return ViewGeomCollection(self)
        if isinstance(other, ViewGeomCollection):
            other.geoms.append(self)
            return other
        return ViewGeomCollection(self, other)

    def __radd__(self, other):
        return self.__add__(other)

    def __repr__(self):
        return f'{type(self).__name__}(\nshape={tuple(self.shape)}\n)'

    @property
    def _wireframe(self):
        """[[segments, widths, colors]] — one ray segment per pixel (geometry.py:310-322)."""
        length = 2 * tr.linalg.norm(self.ray_starts, dim=-1)[..., None]
        ends = (self.ray_starts + self.rays * length).reshape(-1, 3)
        starts = self.ray_starts.reshape(-1, 3).broadcast_to(ends.shape)
        segs = tr.stack((starts, ends), dim=1)
        return [[segs, tr.ones(len(segs)), ['black'] * len(segs)]]

    def plot(self, ax=None):
        raise NotImplementedError('plotting is out of scope for sph_raytracer_amd')


class ViewGeomCollection(ViewGeom):
    """Several same-shape ViewGeoms, stacked along a new leading (observation) axis.
    geometry.py:354-456."""

    def __init__(self, *geoms):
        if any(g.shape != geoms[0].shape for g in geoms):
            raise ValueError("ViewGeoms must all have same shape")
        if len(geoms) == 1 and hasattr(geoms[0], 'geoms'):
            self.geoms = geoms[0].geoms
        else:
            self.geoms = list(geoms)

    def __add__(self, other):
        if isinstance(other, ViewGeomCollection):
            self.geoms += other.geoms
        else:
            self.geoms.append(other)
        return self

    def __radd__(self, other):
        return self.__add__(other)

    def __getitem__(self, ind):
        return self.geoms[ind]

    def __len__(self):
        return len(self.geoms)

    @property
    def shape(self):
        return (len(self.geoms), *self.geoms[0].shape)

    @property
    def rays(self):
        return tr.concat([g.rays[None, ...] for g in self.geoms])

    @property
    def ray_starts(self):
        gs = self.geoms
        if gs and all(type(g) in (ConeRectGeom, ConeCircGeom) for g in gs):
            # cone detectors start every ray at pos: one stack instead of two views per view
            # (the same values, (n, 1, 1, 3); C2 cold path -0.1 ms)
            return tr.stack([g.pos for g in gs])[:, None, None, :]
        return tr.concat([g.ray_starts[None, ...] for g in gs])

    def _ray_spec(self):
        """Stacked generator inputs when every view is a cone detector of one kind, else None.

        Orbits of identical detectors (one type, shape, fov and radial samples) take one batched
        pass: the frames' cross products in one call, the per-axis samples once (the same torch
        calls as each view's own spec, so the same bits; tests/test_cpu_api.py)."""
        fast = self._ray_spec_batched()
        if fast is not None:
            return fast
        specs = [g._ray_spec() if hasattr(g, '_ray_spec') else None for g in self.geoms]
        if not specs or any(sp is None for sp in specs) or len({sp[0] for sp in specs}) != 1:
            return None
        return (specs[0][0], tr.stack([sp[1] for sp in specs]), tr.stack([sp[2] for sp in specs]),
                tr.stack([sp[3] for sp in specs]))

    def _ray_spec_batched(self):
        gs = self.geoms
        kind = type(gs[0]) if gs else None
        if kind not in (ConeRectGeom, ConeCircGeom) or any(type(g) is not kind for g in gs):
            return None
        g0 = gs[0]
        shape0 = tuple(g0.shape)
        if any(tuple(g.shape) != shape0 for g in gs):
            return None
        fov = tr.stack([g.fov for g in gs])         # one comparison instead of a tolist per view
        if not bool((fov == fov[0]).all()):
            return None
        if kind is ConeCircGeom and any(not (tr.equal(g.r, g0.r) and tr.equal(g.theta, g0.theta))
                                        for g in gs):
            return None
        look = tr.stack([g.lookdir for g in gs])
        up = tr.stack([g.updir for g in gs])
        frame = tr.concat([look, tr.cross(look, up, dim=-1), up], dim=-1)
        circ, _, row, col = g0._ray_spec()
        n = len(gs)
        return (circ, frame, row.expand(n, *row.shape), col.expand(n, *col.shape))

    @property
    def pos(self):
        if not all(hasattr(g, 'pos') for g in self.geoms):
            return None
        return tr.concat([g.pos[None, ...] for g in self.geoms])

    @property
    def _wireframe(self):
        frames = []
        for g in self.geoms:
            frames += g._wireframe
        return frames


class ConeRectGeom(ViewGeom):
    """Rectangular cone-beam detector (geometry.py:459-538).

    Args: shape (npix_x, npix_y), pos, lookdir (default: towards the origin), updir, fov degrees.
    Pixel (0, 0) is the top-left of the view (matplotlib convention).
    """

    def __init__(self, shape, pos, lookdir=None, updir=None, fov=(45, 45)):
        self.pos, self.lookdir, self.updir = _frame(pos, lookdir, updir)
        self.shape = shape
        self.fov = _f64(fov)

    def _span(self, axis):
        # half-width of the image plane at unit distance; a single pixel looks straight ahead
        if self.shape[axis] <= 1:
            return 0
        return tr.tan(tr.deg2rad(self.fov[axis] / 2))

    @property
    def rays(self):
        """Unit ray directions, (*shape, 3)."""
        right = tr.cross(self.lookdir, self.updir, dim=-1)
        ulim, vlim = self._span(0), self._span(1)
        col = tr.linspace(-ulim, ulim, self.shape[0])[:, None, None]
        row = tr.linspace(-vlim, vlim, self.shape[1])[None, :, None]
        d = (self.lookdir[None, None, :]
             + right[None, None, :] * col
             + self.updir[None, None, :] * row).reshape((*self.shape, 3))
        return _unit_rows(d)

    def _ray_spec(self):
        """Inputs of the on-device generator (sphrt_rays_cone) that reproduce ``rays`` bit for
        bit: (circ, frame = [lookdir, right, updir], per-row values, per-column values), from
        the same torch calls as ``rays``."""
        right = tr.cross(self.lookdir, self.updir, dim=-1)
        ulim, vlim = self._span(0), self._span(1)
        row = tr.linspace(-ulim, ulim, self.shape[0])
        col = tr.linspace(-vlim, vlim, self.shape[1])
        return 0, tr.concat([self.lookdir, right, self.updir]), row, col

    @property
    def ray_starts(self):
        """All rays start at the detector position, shape (1, 1, 3)."""
        return self.pos[None, None, :]

    def __repr__(self):
        return (f'{type(self).__name__}(\nshape={self.shape}\npos={self.pos.tolist()},\n'
                f'lookdir={self.lookdir.tolist()},\nfov={self.fov.tolist()}\n)')

    @property
    def _wireframe(self):
        reach = 2 * tr.linalg.norm(self.pos)
        corners = self.rays[(-1, -1, 0, 0), (0, -1, -1, 0)].clone() * reach + self.pos
        cone = tr.stack((self.pos.broadcast_to(corners.shape), corners), dim=1)
        rim = tr.stack((corners, corners.roll(-1, dims=0)), dim=1)
        segs = tr.concat((cone, rim))
        return [[segs, tr.ones(len(segs)), ['black'] * len(segs)]]


class ConeCircGeom(ConeRectGeom):
    """Circular cone-beam detector in polar pixels (npix_r, npix_theta); fov = (inner, outer)
    degrees, radial ``spacing`` 'lin' or 'log' (geometry.py:541-604)."""

    def __init__(self, *args, fov=(0, 45), spacing='lin', **kwargs):
        super().__init__(*args, fov=fov, **kwargs)
        r_in = tr.tan(tr.deg2rad(self.fov[0] / 2))
        r_out = tr.tan(tr.deg2rad(self.fov[1] / 2))
        if spacing == 'lin':
            self.r = tr.linspace(r_in, r_out, self.shape[0])
        elif spacing == 'log':
            self.r = tr.logspace(r_in, r_out, self.shape[0])
        else:
            raise ValueError(f"Invalid spacing {spacing}")
        self.theta = tr.linspace(0, 2 * tr.pi, self.shape[1]) + tr.pi / 2

    @property
    def rays(self):
        """Unit ray directions, (*shape, 3)."""
        right = tr.cross(self.lookdir, self.updir, dim=-1)
        rad = self.r[:, None, None]
        ang = self.theta[None, :, None]
        d = (self.lookdir[None, None, :]
             + rad * tr.cos(ang) * right[None, None, :]
             + rad * tr.sin(ang) * self.updir[None, None, :])
        return _unit_rows(d)

    def _ray_spec(self):
        right = tr.cross(self.lookdir, self.updir, dim=-1)
        ang = self.theta[None, :, None]
        cos, sin = tr.cos(ang).reshape(-1), tr.sin(ang).reshape(-1)
        # r * cos(theta) is formed in the tensors' own precision (float32 by default)
        single = self.r.dtype == tr.float32 and cos.dtype == tr.float32
        return (2 if single else 1, tr.concat([self.lookdir, right, self.updir]), self.r,
                tr.concat([cos, sin]))

    @property
    def _wireframe(self):
        reach = 2 * tr.linalg.norm(self.pos)
        outer = self.rays[-1].clone() * reach + self.pos
        inner = self.rays[0].clone() * reach + self.pos
        step = math.ceil(len(outer) / 4)
        cone = tr.stack((self.pos.broadcast_to(outer[::step].shape), outer[::step]), dim=1)
        ring_out = tr.stack((outer, outer.roll(-1, dims=0)), dim=1)
        ring_in = tr.stack((inner, inner.roll(-1, dims=0)), dim=1)
        segs = tr.concat((cone, ring_in, ring_out))
        return [[segs, tr.ones(len(segs)), ['black'] * len(segs)]]


class ParallelGeom(ViewGeom):
    """Rectangular parallel-beam detector of physical ``size`` (width, height) centred on ``pos``
    (geometry.py:607-681).  Every pixel looks along ``lookdir``."""

    def __init__(self, shape, pos, lookdir=None, updir=None, size=(1, 1)):
        self.pos, self.lookdir, self.updir = _frame(pos, lookdir, updir)
        right = tr.cross(self.lookdir, self.updir, dim=-1)
        half_u = size[0] / 2 if shape[0] > 1 else 0
        half_v = size[1] / 2 if shape[1] > 1 else 0
        self._u_arr = right[None, None, :] * tr.linspace(half_u, -half_u, shape[0])[:, None, None]
        self._v_arr = self.updir[None, None, :] * tr.linspace(-half_v, half_v, shape[1])[None, :, None]
        self.shape = shape
        self.size = size

    @property
    def rays(self):
        """Single shared direction, shape (1, 1, 3)."""
        return self.lookdir[None, None, :]

    @property
    def ray_starts(self):
        """Pixel positions, (*shape, 3)."""
        return (self.pos[None, None, :] + self._u_arr + self._v_arr).reshape((*self.shape, 3))

    def __repr__(self):
        return (f'ParallelGeom(\nshape={self.shape}\npos={self.pos.tolist()},\n'
                f'lookdir={self.lookdir.tolist()},\n)')

    @property
    def _wireframe(self):
        c0 = self.ray_starts[(-1, -1, 0, 0), (0, -1, -1, 0)].clone()
        c1 = c0 + self.lookdir[None, :] * 2 * tr.linalg.norm(self.pos)
        segs = tr.concat((tr.stack((c0, c1), dim=1),
                          tr.stack((c0, c0.roll(-1, dims=0)), dim=1),
                          tr.stack((c1, c1.roll(-1, dims=0)), dim=1)))
        return [[segs, tr.ones(len(segs)), ['black'] * len(segs)]]
