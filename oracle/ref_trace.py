"""Torch-CPU restatement of the reference's trace pipeline — CPU BASELINE + TESTS ONLY.

The reference builds its Operator with ``trace_indices`` (raytracer.py:48-230): every ray is
solved against all Nr+1 spheres (r_torch, :248-325), Ne+1 cones (e_torch, :328-468) and Na+1
half-planes (a_torch, :471-552) as materialised (rays, boundaries[, 3]) tensors, the K distances
are concatenated with a start entry (:92-122), entries behind the start stop updating (:126), the
rows are sorted (:131) and reordered (:136), forward-filled one of K columns at a time (:17-45,
:140), differenced (:150) and masked (:155-173).  The reference itself cannot travel to the GPU
box, so ``bench.py``'s cold ``cpu_baseline`` leg times this restatement of the same array
pipeline on the box's host cores: the same torch CPU kernels on tensors of the
same shapes, in the same order.

Calibration (tools/calibrate_ref_trace.py, in the survey container against the imported
reference): identical ``regs`` / ``lens`` bit for bit, and wall time within +-20 % of the
reference's (numbers in DESIGN.md).  The arithmetic is SURVEY App. A expressed as torch ops; the
sqrt is torch's (MKL vdSqrt on CPU), so the distances equal the reference's exactly.

Never imported by the product package; only bench.py's cpu_baseline leg and tests/.
"""
import torch as tr

NA = None


def _normalise(v):
    """v / linalg.norm(v) over the last axis (raytracer.py:281, :365)."""
    return v / tr.linalg.norm(v, axis=-1)[..., NA]


def _close(a, b):
    """|a - b| < finfo.resolution ** (1/3) (raytracer.py:233-246)."""
    return abs(a - b) < tr.finfo(a.dtype).resolution ** (1 / 3)


def sphere_crossings(r_b, x, d1):
    """(t, region) of the near / far crossing of every shell, (N, 2 nb) each; d1 unit."""
    nb = len(r_b)
    tc = tr.einsum('...j,...j->...', -x, d1)
    dist = tr.sqrt(tr.einsum('...j,...j->...', x, x) - tc ** 2)
    half = tr.empty((len(x), nb), dtype=x.dtype)
    half[...] = r_b[NA, :] ** 2
    half -= dist[:, NA] ** 2
    half = tr.sqrt(half)
    t = tr.empty((len(x), 2 * nb), dtype=x.dtype)
    t[:, :nb] = tc[:, NA] - half
    t[:, nb:] = tc[:, NA] + half
    pts = tr.empty((len(x), 2 * nb, 3), dtype=x.dtype)
    pts[...] = d1[:, NA, :]
    pts *= t[..., NA]
    pts += x[:, NA, :]
    inward = (tr.einsum('...c,...bc->...b', d1, pts) < 0).to(tr.int8)
    del pts
    region = tr.arange(nb).repeat(2).repeat(len(x), 1) - inward
    region[region == nb - 1] = -1
    t[t.isnan()] = float('inf')
    return t, region


def cone_crossings(e_b, x, d2):
    """(t, region) of both roots of every elevation cone, (N, 2 nb) each; d2 unit."""
    nb = len(e_b)
    zero = tr.tensor(0, dtype=x.dtype)
    c2 = tr.cos(e_b) ** 2
    a = d2[:, 2:] ** 2 - c2[NA, :]
    b = 2 * (d2[:, 2:] * x[:, 2:] - tr.einsum('...j,...j->...', d2, x)[:, NA] * c2[NA, :])
    c = x[:, 2:] ** 2 - (tr.linalg.norm(x, axis=-1) ** 2)[:, NA] * c2[NA, :]
    a[_close(a, zero)] = zero
    disc = b ** 2 - 4 * a * c
    disc[_close(disc, zero)] = zero
    lin = tr.logical_and(_close(a, zero), tr.logical_not(_close(b, zero)))
    t = tr.empty((len(x), 2 * nb), dtype=x.dtype)
    t[:, :nb] = tr.where(lin, -2 * c / b, (-b + tr.sqrt(disc)) / (2 * a))
    t[:, nb:] = tr.where(lin, float('inf'), (-b - tr.sqrt(disc)) / (2 * a))
    lin2 = lin.repeat(1, 2)
    lin_t = tr.empty_like(t)
    lin_t[:, :nb] = -c / b
    lin_t[:, nb:] = float('inf')
    t = tr.where(lin2, lin_t, t)
    del lin_t, lin2
    on_cone = (a == 0) * (b == 0) * (c == 0)
    t[:, :nb][on_cone] = float('inf')
    t[:, nb:][on_cone] = float('inf')
    del a, b, c
    pts = d2[:, NA, :] * t[:, :, NA] + x[:, NA, :]
    normal = tr.cross(pts, tr.stack((-pts[..., 1], pts[..., 0], tr.zeros_like(pts[..., 0])),
                                    axis=-1), dim=-1)
    prod = tr.einsum('...c,...bc->...b', d2, normal)
    del normal
    region = tr.arange(nb).repeat(2).repeat(len(x), 1) - (prod > 0).to(tr.int8)
    region[_close(prod, zero)] = -2
    e2 = e_b.repeat(2)
    shadow = tr.logical_not((pts[..., 2] >= 0) == (tr.cos(e2) >= 0))
    del pts
    shadow[:, _close(tr.tensor(tr.pi / 2, dtype=x.dtype), e2)] = False
    t[shadow] = float('inf')
    region[region == nb - 1] = -1
    t[t.isnan()] = float('inf')
    return t, region


def plane_crossings(a_b, x, d2):
    """(t, region) of every azimuth half-plane, (N, nb) each."""
    nb = len(a_b)
    zero = tr.tensor(0, dtype=x.dtype)
    along = tr.stack((tr.cos(a_b), tr.sin(a_b), tr.zeros_like(a_b)), dim=-1)
    normal = tr.stack((-tr.sin(a_b), tr.cos(a_b), tr.zeros_like(a_b)), dim=-1)
    t = (-tr.einsum('...bc,...jc->...b', normal[NA], x[:, NA, :]) /
         tr.einsum('...bc,...jc->...b', normal[NA], d2[:, NA, :]))
    cz = tr.cross(along[NA], d2[:, NA, :], dim=-1)[..., -1]
    t[..., tr.isclose(cz, zero, atol=tr.finfo(cz.dtype).resolution)] = float('inf')
    region = tr.arange(nb).repeat(len(x), 1) - (cz < 0).to(tr.int8)
    if -a_b[0] == a_b[-1] == tr.pi:
        region = region % (nb - 1)
    else:
        region[region == nb - 1] = -1
    pts = tr.empty((len(x), nb, 3), dtype=x.dtype)
    pts[...] = t[..., NA]
    pts *= d2[:, NA, :]
    pts += x[:, NA, :]
    back = tr.einsum('bc,...bc->...b', along[:, :2], pts[..., :2]) < 0
    del pts
    t[back] = float('inf')
    t[t.isnan()] = float('inf')
    return t, region


def trace_dense(r_b, e_b, a_b, xs, rays, starts):
    """The reference's (regs (3, N, K) int64, lens (N, K) float64) for N rays.

    xs, rays: (N, 3) float64 (rays need not be unit); starts: (3, N) int64, the start voxels
    (find_starts)."""
    r_b, e_b, a_b = (tr.as_tensor(b, dtype=tr.float64) for b in (r_b, e_b, a_b))
    nr, ne, na = len(r_b) - 1, len(e_b) - 1, len(a_b) - 1
    x = tr.as_tensor(xs, dtype=tr.float64)
    d1 = _normalise(tr.as_tensor(rays, dtype=tr.float64))
    t_r, g_r = sphere_crossings(r_b, x, d1)
    d2 = _normalise(d1)
    t_e, g_e = cone_crossings(e_b, x, d2)
    t_a, g_a = plane_crossings(a_b, x, d2)
    n = len(x)
    ts = tr.cat((t_r, t_e, t_a), dim=-1)
    del t_r, t_e, t_a
    blocks = []
    for row, g in enumerate((g_r, g_e, g_a)):
        blk = tr.full((3,) + tuple(g.shape), -2, dtype=tr.int64)
        blk[row] = g
        blocks.append(blk)
    regs = tr.cat(blocks, dim=-1)
    del blocks, g_r, g_e, g_a
    start = tr.as_tensor(starts, dtype=tr.int64).reshape(3, n, 1)
    regs = tr.concat((regs, start), dim=-1)
    ts = tr.concat((ts, tr.zeros_like(ts[..., 0:1])), dim=-1)
    regs[:, ts < 0] = -2
    ts, order = ts.sort(dim=-1)
    regs = tr.take_along_dim(regs, order[NA, ...], dim=-1)
    del order
    # forward fill of the -2 entries along K, one column at a time (raytracer.py:17-45)
    cols = regs.moveaxis(-1, 0)
    last = start[..., 0]
    for k in range(cols.shape[0]):
        cols[k] = cols[k].where(cols[k] != -2, last)
        last = cols[k]
    lens = ts.diff(dim=-1, append=tr.full((n, 1), float('inf'), dtype=tr.float64))
    del ts
    lens[lens.isinf() + lens.isnan()] = 0
    for row, lim in enumerate((nr, ne, na)):
        lens[regs[row] > lim - 1] = 0
    for row in range(3):
        lens[regs[row] < 0] = 0
    return regs, lens
