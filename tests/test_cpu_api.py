"""CPU-side checks: geometry API + bit-identity with the reference geometry, host logic, and the
C ABI library (loads and exports every symbol include/sphrt.h declares; no compute without GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch as tr

import golden_cases as gc
from known_answers import START_CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check(a, b):
    return tr.allclose(tr.asarray(a).type(tr.float32).flatten().squeeze(),
                       tr.asarray(b).type(tr.float32).flatten().squeeze(), atol=1e-2)


# ---- test_all.py:176-302 geometry tests, on this package ---------------------------------------

def test_sphericalgrid_static():
    from sph_raytracer_amd import SphericalGrid
    grid = SphericalGrid(shape=(10, 11, 12))
    assert not grid.dynamic
    assert (len(grid.r_b), len(grid.e_b), len(grid.a_b)) == (11, 12, 13)
    grid = SphericalGrid(r_b=[1, 2], e_b=[1, 2, 3], a_b=[1, 2, 3, 4])
    assert grid.shape == (1, 2, 3) and not grid.dynamic

    def check_bounds(g):
        for c, b in ((g.r, g.r_b), (g.e, g.e_b), (g.a, g.a_b)):
            assert len(c) == len(b) - 1
            assert all(c > b[:-1]) and all(c < b[1:])
    check_bounds(grid)
    check_bounds(SphericalGrid(shape=(10, 11, 12), size_r=(1, 10), size_e=(0, tr.pi),
                               size_a=(0, 2 * tr.pi), spacing='log'))
    for x in (grid.r, grid.e, grid.a):
        assert type(x) is tr.Tensor
    assert grid.mesh.ndim == 4


def test_sphericalgrid_dynamic():
    from sph_raytracer_amd import SphericalGrid
    grid = SphericalGrid(shape=(9, 10, 11, 12))
    assert grid.dynamic
    assert (len(grid.t), len(grid.r_b), len(grid.e_b), len(grid.a_b)) == (9, 11, 12, 13)
    grid = SphericalGrid(t=[1], r_b=[1, 2], e_b=[1, 2, 3], a_b=[1, 2, 3, 4])
    assert grid.shape == (1, 1, 2, 3) and grid.dynamic
    assert len(grid.nptime) == grid.shape.t
    for x in (grid.t, grid.r, grid.e, grid.a):
        assert type(x) is tr.Tensor
    assert grid.mesh.ndim == 5


def test_find_starts():
    from sph_raytracer_amd import SphericalGrid
    from sph_raytracer_amd.raytracer import find_starts
    for shape, x, exp in START_CASES:
        assert check(find_starts(SphericalGrid(shape=shape), x), exp)


def test_find_starts_host():
    """The trace's host start binning (_find_starts_host: numpy sums and binning, torch sqrt and
    arctan2 on the reference's layouts) equals find_starts bitwise: random points inside and
    outside, the origin, points on radius / elevation / azimuth boundaries, the known answers,
    several grids and leading shapes."""
    from sph_raytracer_amd import SphericalGrid
    from sph_raytracer_amd.raytracer import _find_starts_host, find_starts
    gen = tr.Generator().manual_seed(11)
    grids = [SphericalGrid(shape=(50, 50, 50)), SphericalGrid(shape=(7, 9, 12), size_r=(0.2, 1.5),
                                                                size_e=(0, tr.pi / 2), size_a=(0, tr.pi)),
             SphericalGrid(shape=(20, 11, 13), size_r=(0.1, 1), spacing='log'),
             SphericalGrid(shape=(3, 4, 5, 6))]
    for grid in grids:
        pts = [(tr.rand((400, 3), generator=gen, dtype=tr.float64) - 0.5) * 3.5,
               tr.zeros((2, 3), dtype=tr.float64)]
        r, e, a = (tr.as_tensor(b, dtype=tr.float64) for b in (grid.r_b, grid.e_b, grid.a_b))
        for rb in r:                                     # on the spheres, the cones, half-planes
            for eb in e[::3]:
                for ab in a[::4]:
                    pts.append(tr.stack([rb * tr.sin(eb) * tr.cos(ab), rb * tr.sin(eb) * tr.sin(ab),
                                         rb * tr.cos(eb)])[None])
        pts.append(tr.tensor([[1.0, 0.0, 0.0], [-1.0, 0.0, 0.0], [0.0, 0.0, 1.0], [0.0, 0.0, -0.5],
                              [-0.3, -0.0, 0.1], [0.0, 0.5, 0.0]], dtype=tr.float64))
        xs = tr.cat(pts)
        for shaped in (xs, xs[:48].reshape(4, 2, 6, 3), xs[:1].reshape(1, 1, 1, 3)):
            want = find_starts(grid, shaped)
            got = _find_starts_host(grid, shaped.contiguous())
            assert got.dtype == want.dtype and got.shape == want.shape
            assert tr.equal(got, want), np.argwhere((got != want).numpy())[:5]
    for shape, x, exp in START_CASES:
        g = SphericalGrid(shape=shape)
        xt = tr.as_tensor(x, dtype=tr.float64)
        assert tr.equal(_find_starts_host(g, xt), find_starts(g, xt))


def test_trace_order():
    """ConeCirc detectors are traced in wedges of _WEDGE azimuth columns, radius-major inside (a
    permutation of each view's pixels); ConeRect and mixed geometries keep the geometry order."""
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    from sph_raytracer_amd.raytracer import _WEDGE, _trace_order, _wedge_order
    p = _wedge_order(7, 12)
    assert sorted(p.tolist()) == list(range(84))
    w = _WEDGE
    assert p[:w + 2].tolist() == list(range(w)) + [12, 13]   # wedge 0: radius 0, then 1
    assert p[7 * w:7 * w + 2].tolist() == [w, w + 1]         # wedge 1 after 7 x w pixels
    last = 12 - (12 // w) * w or w                            # the last wedge's width
    assert p[-last:].tolist() == list(range(84 - last, 84))
    circ = sum(ConeCircGeom((7, 12), pos=(3, 0, 1)) for _ in range(2))
    assert tr.equal(_trace_order(circ, circ.rays), p)
    rect = ConeRectGeom((7, 12), pos=(3, 0, 1))
    assert _trace_order(rect, rect.rays) is None
    assert _trace_order(rect + ConeCircGeom((7, 12), pos=(3, 0, 1)), circ.rays) is None


def test_staging_round_trip():
    """_Staging (one host-to-device copy for the plan tables, ray spec and start bins): every
    blob comes back with its dtype, shape and values, at 16-byte aligned offsets."""
    from sph_raytracer_amd.raytracer import _Staging
    parts = [tr.arange(7, dtype=tr.uint8), tr.rand(5, 3, dtype=tr.float64),
             tr.arange(12, dtype=tr.int32).reshape(3, 4), tr.rand(3, dtype=tr.float32)]
    stg = _Staging()
    slots = [stg.add(t) for t in parts]
    stg.upload('cpu')
    for slot, t in zip(slots, parts):
        got = stg.get(slot, t)
        assert got.dtype == t.dtype and got.shape == t.shape and tr.equal(got, t)
        assert got.data_ptr() % 16 == stg._dev.data_ptr() % 16


def test_conerectgeom():
    from sph_raytracer_amd import ConeRectGeom
    g = ConeRectGeom((11, 11), (4, 0, 1), fov=(23, 45))
    assert check(tr.dot(g.rays[5, 0], g.rays[5, -1]), tr.cos(tr.deg2rad(g.fov[1])))
    assert check(tr.dot(g.rays[0, 5], g.rays[-1, 5]), tr.cos(tr.deg2rad(g.fov[0])))
    assert check(g.rays[5, 5], g.lookdir)
    g = ConeRectGeom((1, 1), (1, 0, 0), (-1, 0, 0), (0, 1, 0), fov=(23, 45))
    assert check(g.rays[0, 0], g.lookdir)
    g._wireframe


def test_conecircgeom():
    from sph_raytracer_amd import ConeCircGeom
    g = ConeCircGeom((11, 11), (1, 0, 0), (-1, 0, 0), (0, 1, 0), fov=(0, 45))
    assert check(tr.dot(g.rays[-1, 0], g.rays[-1, 5]), tr.cos(tr.deg2rad(g.fov[1])))
    assert check(g.rays[0, 0], g.lookdir)
    g = ConeCircGeom((1, 1), (1, 0, 0), (-1, 0, 0), (0, 1, 0), fov=(0, 45))
    assert check(g.rays[0, 0], g.lookdir)
    g._wireframe


def test_parallelgeom():
    from sph_raytracer_amd import ParallelGeom
    g = ParallelGeom((11, 11), (4, 0, 1), size=(2, 3))
    assert check(tr.linalg.norm(g.ray_starts[5, 0] - g.ray_starts[5, -1]), g.size[1])
    assert check(tr.linalg.norm(g.ray_starts[0, 5] - g.ray_starts[-1, 5]), g.size[0])
    assert all((g.rays == g.lookdir).flatten())
    g = ParallelGeom((1, 1), (1, 0, 0), (-1, 0, 0), (0, 1, 0))
    assert check(g.rays[0, 0], g.lookdir)
    g._wireframe


def test_viewgeom():
    from sph_raytracer_amd import ViewGeom
    rays = tr.rand((4, 4, 3))
    g = ViewGeom(rays=rays, ray_starts=tr.tensor((10, 0, 0)).broadcast_to(rays.shape))
    g._wireframe
    assert g.shape == (4, 4)


def test_ray_spec_availability():
    """Cone detectors (and collections of one kind) expose the on-device generator's inputs;
    arbitrary ViewGeoms and mixed collections keep host rays."""
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom, ViewGeom
    rect = ConeRectGeom((4, 5), pos=(3, 0, 1))
    circ = ConeCircGeom((4, 5), pos=(3, 0, 1))
    circ_, frame, row, col = rect._ray_spec()
    assert circ_ == 0 and frame.shape == (9,) and row.shape == (4,) and col.shape == (5,)
    circ_, frame, row, col = circ._ray_spec()
    assert circ_ == 2 and row.shape == (4,) and col.shape == (10,)   # float32 r, theta
    coll = rect + ConeRectGeom((4, 5), pos=(0, 3, 1))
    assert coll._ray_spec()[1].shape == (2, 9)
    assert (rect + circ)._ray_spec() is None
    rays = tr.rand((4, 5, 3))
    assert not hasattr(ViewGeom(rays=rays, ray_starts=tr.zeros(3)), '_ray_spec')


def test_model_instantiation():
    """test_model.py:7-15."""
    from sph_raytracer_amd import SphericalGrid
    from sph_raytracer_amd.model import AxisAlignmentModel, CubesModel, FullyDenseModel
    g = SphericalGrid()
    for model in (FullyDenseModel, CubesModel, AxisAlignmentModel):
        m = model(g)
        assert m(tr.rand(m.coeffs_shape)).shape == g.shape


# ---- geometry is bit-identical to the reference's (rays are Operator inputs) ----------------

def test_conerect_rays_bit_identical():
    from sph_raytracer_amd import ConeRectGeom
    case = gc.load('c1_single_vantage')
    g = ConeRectGeom((50, 100), pos=(5, 0, 0), fov=(45, 45))
    assert np.array_equal(g.rays.numpy(), case['rays'])
    assert np.array_equal(g.ray_starts.numpy(), case['xs'])


def test_orbit_collections_bit_identical():
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    case = gc.load('circ_orbit')
    geoms = [ConeCircGeom(shape=(30, 24), pos=(5 * tr.cos(th), 5 * tr.sin(th), 1), fov=(0, 45))
             for th in tr.linspace(0, 2 * tr.pi, 5)]
    coll = sum(geoms)
    assert coll.shape == (5, 30, 24)
    assert np.array_equal(coll.rays.numpy(), case['rays'])
    assert np.array_equal(coll.ray_starts.numpy(), case['xs'])
    case = gc.load('c2_orbit3')
    th = tr.linspace(0, 2 * tr.pi, 50)[[0, 17, 33]]
    coll = sum(ConeRectGeom((50, 100), pos=(5 * tr.cos(a), 5 * tr.sin(a), 1), fov=(45, 45))
               for a in th)
    assert np.array_equal(coll.rays.numpy(), case['rays'])


def test_grid_boundaries_bit_identical():
    from sph_raytracer_amd import SphericalGrid
    case = gc.load('log_grid')
    g = SphericalGrid(shape=(9, 11, 13), size_r=(0.1, 1), spacing='log', size_a=(0, 2 * tr.pi))
    for k in ('r_b', 'e_b', 'a_b'):
        assert np.array_equal(getattr(g, k).numpy(), case[k])


# ---- host logic ------------------------------------------------------------------------------

def test_density_layouts():
    """Output shapes / channel rules of raytracer.py:703-712 (no GPU needed)."""
    from sph_raytracer_amd import SphericalGrid
    from sph_raytracer_amd.raytracer import _layout_for
    static, dyn = SphericalGrid((2, 3, 4)), SphericalGrid((10, 2, 3, 4))
    assert _layout_for(static, (64, 64), (2, 3, 4)) == (1, 0, (64, 64))
    assert _layout_for(static, (64, 64), (10, 2, 3, 4)) == (10, 0, (10, 64, 64))
    assert _layout_for(static, (), (5, 2, 3, 4)) == (5, 0, (5,))
    assert _layout_for(dyn, (64, 64), (10, 2, 3, 4)) == (10, 0, (10, 64, 64))
    assert _layout_for(dyn, (10, 8, 6), (10, 2, 3, 4)) == (1, 48, (10, 8, 6))
    assert _layout_for(dyn, (4,), (10, 2, 3, 4)) == (10, 0, (10, 1, 4))   # App. C.5 quirk
    with pytest.raises(ValueError):
        _layout_for(static, (64, 64), (2, 3, 5))


def test_layout_and_broadcast_import_nothing_heavy():
    """The shape rules import no sympy: torch.broadcast_shapes does (torch._refs) on its first
    call, which cost the first dynamic Operator's first forward ~0.8 s.
    The plain-Python broadcast equals torch's, errors included."""
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, %r); import torch; '
            'from sph_raytracer_amd import SphericalGrid; '
            'from sph_raytracer_amd.raytracer import _layout_for, _broadcast_pair; '
            'dyn = SphericalGrid((10, 2, 3, 4)); _layout_for(dyn, (10, 8, 6), (10, 2, 3, 4)); '
            '_layout_for(dyn, (4,), (10, 2, 3, 4)); '
            '_broadcast_pair(torch.zeros(3), torch.ones(5, 4, 3)); '
            'print("sympy" in sys.modules)' % os.path.dirname(os.path.dirname(__file__)))
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, check=True)
    assert out.stdout.strip().splitlines()[-1] == 'False'
    from sph_raytracer_amd.raytracer import _broadcast_shapes
    rng = np.random.default_rng(0)
    for _ in range(500):
        a = tuple(int(v) for v in rng.integers(1, 4, rng.integers(0, 5)))
        b = tuple(int(v) for v in rng.integers(1, 4, rng.integers(0, 5)))
        try:
            want = tuple(tr.broadcast_shapes(a, b))
        except RuntimeError:
            with pytest.raises(RuntimeError):
                _broadcast_shapes(a, b)
            continue
        assert _broadcast_shapes(a, b) == want


def test_no_cpu_fallback():
    """Without a GPU the product path fails loudly instead of computing on the CPU."""
    if tr.cuda.is_available():
        pytest.skip('GPU present')
    from sph_raytracer_amd import ConeRectGeom, Operator, SphericalGrid
    from sph_raytracer_amd.raytracer import line_integrals, r_torch
    grid, geom = SphericalGrid((4, 4, 4)), ConeRectGeom((4, 4), (5, 0, 0))
    with pytest.raises(RuntimeError, match='GPU'):
        Operator(grid, geom)
    with pytest.raises(RuntimeError, match='GPU'):
        line_integrals(grid, geom, tr.ones(grid.shape))
    with pytest.raises(RuntimeError, match='GPU'):
        r_torch([1.0], [(0, 0, 0)], [(1, 0, 0)])


def test_gd_with_linear_stand_in():
    """gd() contract (retrieval.py:24-127) with a dense linear stand-in for f."""
    from sph_raytracer_amd import SphericalGrid
    from sph_raytracer_amd.loss import NegRegularizer, SquareLoss
    from sph_raytracer_amd.model import FullyDenseModel
    from sph_raytracer_amd.retrieval import gd
    grid = SphericalGrid((3, 4, 5))
    A = tr.rand(30, 60, dtype=tr.float64)

    class F:
        device = 'cpu'

        def __init__(self):
            self.grid = grid

        def __call__(self, d):
            return (A @ d.reshape(-1)).reshape(5, 6)
    f = F()
    truth = tr.rand(grid.shape, dtype=tr.float64)
    y = f(truth).detach()
    coeffs, y_res, losses = gd(f, y, FullyDenseModel(grid), num_iterations=20, lr=1e-2,
                               loss_fns=[SquareLoss(), 0.5 * NegRegularizer()], progress_bar=False)
    hist = list(losses.values())[0]
    assert len(hist) == 20 and hist[-1] < hist[0]
    assert y_res.shape == (5, 6)
    assert all(type(v) is float for vals in losses.values() for v in vals)
    # loss values read back once at the end (no bar) == read back every iteration (bar)
    c2, _, l2 = gd(f, y, FullyDenseModel(grid), num_iterations=20, lr=1e-2,
                   loss_fns=[SquareLoss(), 0.5 * NegRegularizer()], progress_bar=True)
    assert tr.equal(c2, coeffs)
    assert [list(v) for v in l2.values()] == [list(v) for v in losses.values()]


# ---- the C ABI library -------------------------------------------------------------------------

def _declared_symbols():
    hdr = open(os.path.join(ROOT, 'include', 'sphrt.h')).read()
    return sorted(set(re.findall(r'\b(sphrt_[a-z0-9_]+)\s*\(', hdr)))


def test_library_builds_and_exports_header():
    from sph_raytracer_amd import _lib, build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), f'{name} declared in include/sphrt.h but not exported'
    assert sorted(_lib.EXPORTED) == declared, 'ctypes bindings out of sync with the header'
    hdr = open(os.path.join(ROOT, 'include', 'sphrt.h')).read()
    for name, val in (('SPHRT_ROW_HEAD', _lib.ROW_HEAD), ('SPHRT_BLOCK_FIELDS', _lib.BLOCK_FIELDS),
                      ('SPHRT_LOC_HEAD', _lib.LOC_HEAD), ('SPHRT_TRACE_F32', _lib.TRACE_F32),
                      ('SPHRT_TRACE_INVALID', _lib.TRACE_INVALID),
                      ('SPHRT_TRACE_FRESH_RAYS', _lib.TRACE_FRESH_RAYS)):
        m = re.search(rf'#define {name} (0x[0-9a-fA-F]+|\d+)', hdr)
        assert m and int(m.group(1).rstrip('u'), 0) == val, name
    lib = _lib.load()
    assert lib.sphrt_version().startswith(b'sph_raytracer_amd')
    assert lib.sphrt_scan_workspace_bytes(10_000) > 0


def test_library_carries_the_tree_hash(tmp_path, monkeypatch):
    """Both libraries embed the hash of the sources + flags they were built from (each its own:
    libsphrt.so its HIP sources, _sphrt_fast.so its C++ ones); it equals this tree's, build()
    decides staleness by it (not by file times), and a library built from other sources is
    refused at load."""
    from sph_raytracer_amd import _lib, build
    build.build()
    want = build.source_hash()
    assert len(want) == 16
    assert build.embedded_hash(build.OUT) == want == _lib.source_hash()
    fast = build.fast_hash()
    assert len(fast) == 16 and fast != want
    assert build.embedded_hash(build.FAST_OUT) == fast
    assert _lib.load_fast().version.endswith(fast)
    assert not build._stale(build.OUT) and not build._stale(build.FAST_OUT)
    fake = tmp_path / 'lib.so'
    fake.write_bytes(b'\0sph_raytracer_amd 0.3 (gfx950) src 0123456789abcdef\0')
    assert build.embedded_hash(str(fake)) == '0123456789abcdef' and build._stale(str(fake))
    with pytest.raises(RuntimeError, match='rebuild'):
        _lib._check_hash('sph_raytracer_amd 0.3 (gfx950) src 0123456789abcdef', 'x.so')
    _lib._check_hash(f'sph_raytracer_amd 0.3 (gfx950) src {want}', 'x.so')
    # a touched (not edited) source does not make the build stale
    src = os.path.join(build.CSRC, 'api.hip')
    st = os.stat(src)
    try:
        os.utime(src, (st.st_atime, st.st_mtime + 100))
        assert not build._stale(build.OUT)
    finally:
        os.utime(src, (st.st_atime, st.st_mtime))


def test_loss_abi_argument_checks():
    """The retrieval entry points reject bad arguments before touching the device: an empty
    problem, null buffers, a step count below 1, a staged CSR whose columns are not the
    coefficients; each with a message in sphrt_last_error.  (No compute call: no GPU here.)"""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    p = ctypes.c_void_p(16)      # never dereferenced: every call below fails its checks first
    none = None

    def adam(param, n, step, stage_of=None):
        return lib.sphrt_adam_neg_f64(param, p, p, p, n, 0.1, 0.9, 0.999, 1e-8, 0.0, step, 0.0,
                                      none, stage_of, none)

    cases = [
        (lambda: adam(p, 0, 1.0), b'empty'),
        (lambda: adam(none, 8, 1.0), b'null'),
        (lambda: adam(p, 8, 0.0), b'step'),
        (lambda: lib.sphrt_sq_residual_f64(p, p, 1, 0, 1.0, none, p, p, none), b'empty'),
        (lambda: lib.sphrt_sq_residual_f64(p, none, 1, 8, 1.0, none, p, p, none), b'null'),
        (lambda: lib.sphrt_neg_reg_f64(p, 0, 0.1, p, p, none), b'empty'),
    ]
    csr = _lib.CSR()          # a brick-staged CSR over 4^3 voxels, without a stage buffer
    csr.stage_shape[:] = [4, 4, 4]
    csr.stage_brick[:] = [2, 4, 4]
    csr.stage_cols, csr.n_cols = 64, 64
    cases += [(lambda: adam(p, 32, 1.0, ctypes.byref(csr)), b'columns'),
              (lambda: adam(p, 64, 1.0, ctypes.byref(csr)), b'stage buffer')]
    for call, word in cases:
        assert call() != 0
        assert word in lib.sphrt_last_error().lower(), lib.sphrt_last_error()


def test_staged_and_reference_trace_argument_checks():
    """The staged one-pass entry points and the reference-mode trace reject bad arguments before
    touching the device (null row list, an incomplete staged CSR, unknown trace flags), with a
    message in sphrt_last_error.  (No compute call: no GPU here.)"""
    from sph_raytracer_amd import _lib
    lib = _lib.load()
    p = ctypes.c_void_p(16)      # never dereferenced: every call below fails its checks first
    csr = _lib.CSR()
    csr.n_rays, csr.n_segments, csr.n_blocks = 10, 20, 1
    cases = [
        (lambda: lib.sphrt_csr_index_staged(p, 10, p, p, p, 1, None, None, p, None), b'nz_row'),
        (lambda: lib.sphrt_csr_local_build_staged(ctypes.byref(csr), p, p, p, p, p, p, p, p,
                                                  None), b'incomplete'),
        (lambda: lib.sphrt_trace_reference(None, None, 8, p, None, None, None, None, 0, None),
         b'plan'),
    ]
    for call, word in cases:
        assert call() != 0
        assert word in lib.sphrt_last_error().lower(), lib.sphrt_last_error()


def test_fastpath_entry_builds_and_declines_foreign_inputs():
    """csrc/fastpath.cpp (the CPython entry for steady-state Operator calls) builds against the
    installed torch, loads, and returns None for anything it has no binding for (CPU tensors,
    non-tensors), so Operator.__call__ falls back to its general path."""
    import torch
    from sph_raytracer_amd import _lib, build
    build.build()
    fast = _lib.load_fast()
    assert fast is not None
    b = fast.new(_lib.address(_lib.load().sphrt_last_error))
    assert fast.forward(b, torch.zeros(4)) is None
    assert fast.forward(b, [1.0]) is None
    with pytest.raises(ValueError):
        fast.add(b, (2, 2), False, 0, 0, 0, 1, 4, 0, 4, (4,), 0)


def test_batched_orbit_spec_matches_per_view():
    """ViewGeomCollection._ray_spec batches uniform orbits (one cross product call, the per-axis
    samples once): bitwise the stack of the views' own specs, for rectangular and circular
    detectors with arbitrary frames; non-uniform collections take the per-view path."""
    from sph_raytracer_amd import ConeCircGeom, ConeRectGeom
    g = tr.Generator().manual_seed(5)
    for kind, kw in ((ConeRectGeom, dict(fov=(30, 50))), (ConeCircGeom, dict(fov=(2, 40)))):
        views = []
        for i in range(40):
            pos = tr.randn(3, generator=g, dtype=tr.float64) * 4
            look = -pos + 0.3 * tr.randn(3, generator=g, dtype=tr.float64) if i % 2 else None
            views.append(kind((7, 9), pos=pos, lookdir=look, **kw))
        coll = sum(views)
        fast = coll._ray_spec()
        assert coll._ray_spec_batched() is not None
        specs = [v._ray_spec() for v in views]
        assert fast[0] == specs[0][0]
        for i in (1, 2, 3):
            ref = tr.stack([sp[i] for sp in specs])
            assert fast[i].shape == ref.shape and tr.equal(fast[i].contiguous(), ref), (kind, i)
    mixed = ConeRectGeom((7, 9), pos=(3, 0, 1), fov=(30, 30)) + ConeRectGeom((7, 9), pos=(0, 3, 1))
    assert mixed._ray_spec_batched() is None and mixed._ray_spec()[1].shape == (2, 9)


def test_brick_stage_fields(monkeypatch):
    """Host side of brick staging (raytracer._stage_brick/_set_stage, sphrt.h stage_*): the
    automatic rule (multi-wave grids only), the environment overrides, the padded column count,
    and the 32-bit / whole-granule guards."""
    from sph_raytracer_amd import _lib
    from sph_raytracer_amd import raytracer as rt
    monkeypatch.delenv('SPHRT_BRICK', raising=False)
    assert rt._stage_brick(1536) is None and rt._stage_brick(1537) == rt._BRICK
    # arrays that fit one XCD's L2 (float32 columns) keep the natural layout
    assert rt._stage_brick(10 ** 6, n_cols=64 ** 3) is None
    assert rt._stage_brick(10 ** 6, n_cols=128 ** 3) == rt._BRICK
    monkeypatch.delenv('SPHRT_BRICK_T', raising=False)
    assert rt._stage_brick(1536, 'SPHRT_BRICK_T', rt._BRICK_RAYS) is None
    assert rt._stage_brick(10 ** 6, 'SPHRT_BRICK_T', rt._BRICK_RAYS) == rt._BRICK_RAYS == (8, 1, 4)
    monkeypatch.setenv('SPHRT_BRICK', 'off')
    assert rt._stage_brick(10 ** 6) is None
    monkeypatch.setenv('SPHRT_BRICK', '4,4,2')
    assert rt._stage_brick(8) == (4, 4, 2)
    c = _lib.CSR()
    assert rt._set_stage(c, (30, 21, 26), (2, 4, 4))
    assert tuple(c.stage_shape) == (30, 21, 26) and tuple(c.stage_brick) == (2, 4, 4)
    assert c.stage_cols == 30 * 24 * 28
    # the operator owns no stage buffer: each forward call allocates its own
    assert not c.stage and c.stage_bytes == 0
    assert rt._stage_bytes(c, 3, 4) == 3 * 4 * c.stage_cols
    assert not rt._set_stage(c, (30, 21, 26), None) and c.stage_shape[0] == 0
    assert rt._stage_bytes(c, 3, 4) == 0
    assert not rt._set_stage(c, (2048, 1024, 1024), (2, 4, 4))   # 2^31 columns
    assert not rt._set_stage(c, (30, 21, 26), (1, 1, 3))          # partial granules
    assert c.stage_cols == 0 and not c.stage


def test_compute_device_resolution():
    """Operator(device=...) computes on the GPU `device` names; 'cpu' / None (results on the
    host) compute on the current GPU (_lib.compute_device)."""
    from sph_raytracer_amd import _lib
    assert _lib.compute_device('cuda:1', current=0) == tr.device('cuda', 1)
    assert _lib.compute_device(tr.device('cuda', 2), current=0) == tr.device('cuda', 2)
    assert _lib.compute_device('cuda', current=3) == tr.device('cuda', 3)
    assert _lib.compute_device('cpu', current=1) == tr.device('cuda', 1)
    assert _lib.compute_device(None, current=0) == tr.device('cuda', 0)


def test_ctypes_structs_match_the_c_header(tmp_path):
    """The ctypes mirrors in _lib (GridDesc, RayBatch, CSR) have the C ABI layout of
    include/sphrt.h: every field at the C offset, same struct size (gcc on the header)."""
    import shutil
    import subprocess
    from sph_raytracer_amd import _lib
    gcc = shutil.which('gcc')
    if gcc is None:
        pytest.skip('gcc not available')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pairs = [('sphrt_grid_desc', _lib.GridDesc), ('sphrt_rays', _lib.RayBatch),
             ('sphrt_csr', _lib.CSR)]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sphrt.h"', 'int main(void) {']
    for cname, py in pairs:
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines += ['return 0;', '}']
    src = tmp_path / 'abi.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'abi'
    subprocess.run([gcc, '-std=c11', '-I', os.path.join(root, 'include'), str(src), '-o', str(exe)],
                   check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True,
                               text=True).stdout.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, py in pairs:
        assert got[(cname, 'sizeof')] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


def test_split_adam_accepts_torch_defaults():
    """retrieval._split_adam takes torch.optim.Adam's own defaults (weight_decay=0 is an int) and
    resolves the implementation torch would pick: fused for fused=True, foreach for a default
    Adam on a GPU tensor (here: a CPU tensor, so the single-tensor path: no split step)."""
    import torch
    from sph_raytracer_amd import retrieval
    c = torch.zeros(4, dtype=torch.float64, requires_grad=True)
    opt = torch.optim.Adam([c], lr=0.1)
    assert opt.param_groups[0]['weight_decay'] == 0 and retrieval._number(0)
    assert retrieval._split_adam(opt, c) is None          # CPU tensor: torch's single-tensor Adam
    assert not retrieval._number(True) and not retrieval._number(torch.tensor(0.1))


def test_view_tiles_rule(monkeypatch):
    """raytracer._view_tiles: orbits of static grids in tiles of tv views (the largest divisor of
    the view count in [8, 64]) x tw pixels of a row (2, or 1 for an odd width); none for single
    views, too few views, dynamic grids, or SPHRT_RAY_ORDER other than auto / vtile:tv,1,tw."""
    from sph_raytracer_amd import raytracer as rt
    monkeypatch.delenv('SPHRT_RAY_ORDER', raising=False)
    assert rt._view_tiles((50, 50, 100), False) == (50, 2)      # C2
    assert rt._view_tiles((128, 128, 256), False) == (64, 2)    # C3
    assert rt._view_tiles((64, 100, 50), False) == (64, 2)      # C5
    assert rt._view_tiles((9, 17, 41), False) == (9, 1)
    assert rt._view_tiles((96, 8, 8), False) == (48, 2)
    assert rt._view_tiles((7, 20, 30), False) is None
    assert rt._view_tiles((50, 100, 50), True) is None          # C4: dynamic
    assert rt._view_tiles((50, 100), False) is None             # a single view
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'natural')
    assert rt._view_tiles((50, 50, 100), False) is None
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'vtile:10,1,4')
    assert rt._view_tiles((50, 50, 100), False) == (10, 4)
    monkeypatch.setenv('SPHRT_RAY_ORDER', 'vtile:4,2,8')       # several rows: the study path
    assert rt._view_tiles((50, 50, 100), False) is None


def test_dense_ranges_partition_the_output():
    """_dense_ranges (sphrt_csr.order bit 2): block b's output range starts at its first row's
    output (0 for the first block), ends where the next block with rows starts (n_out for the
    last), rowless blocks get empty ranges — a partition of [0, n_out) in block order, each
    block's rows inside its own range."""
    from sph_raytracer_amd import _lib
    from sph_raytracer_amd.raytracer import _dense_ranges
    rng = np.random.default_rng(3)
    n_out = 500
    rows = np.sort(rng.choice(n_out, 180, replace=False)).astype(np.int32)   # non-empty outputs
    # blocks over the rows: k0 per block, some blocks without rows (s0 == s1)
    k0 = [0, 0, 17, 60, 60, 61, 120, 179]
    has = [False, True, True, False, True, True, True, True]
    nb = len(k0)
    blocks = tr.zeros((nb, _lib.BLOCK_FIELDS), dtype=tr.int64)
    blocks[:, 4] = tr.tensor(k0)
    blocks[:, 2] = tr.arange(nb) * 10
    blocks[:, 3] = blocks[:, 2] + tr.tensor([10 if h else 0 for h in has])
    desc = _lib.CSR()
    _dense_ranges(desc, blocks.view(-1), tr.from_numpy(rows), n_out)
    lo, hi = blocks[:, 0].tolist(), blocks[:, 1].tolist()
    assert desc.order & 4 and not desc.runs
    assert lo[0] == 0 and hi[-1] == n_out
    assert all(hi[b] == lo[b + 1] for b in range(nb - 1))
    assert all(lo[b] <= hi[b] for b in range(nb))
    k1 = k0[1:] + [len(rows)]
    for b in range(nb):
        if not has[b]:
            assert lo[b] == hi[b] or b == 0
        for k in range(k0[b], k1[b] if has[b] else k0[b]):
            assert lo[b] <= rows[k] < hi[b]


def test_native_construction_constants_match_python():
    """The native cone construction (csrc/construct.cpp) repeats the Python construction's brick,
    L2 and memory-gate rules: every `constexpr` there that names its Python twin in
    its comment (`// _NAME`) equals that twin."""
    from sph_raytracer_amd import raytracer as rt
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            'sph_raytracer_amd', 'csrc', 'construct.cpp')).read()
    pat = re.compile(r'constexpr\s+\w+\s+(k\w+)(\[3\])?\s*=\s*([^;]+);\s*//\s*(_[A-Z0-9_]+)')
    seen = set()
    for cname, arr, val, pyname in pat.findall(src):
        py = getattr(rt, pyname)
        if arr:
            cval = tuple(int(v) for v in val.strip('{} ').split(','))
        else:
            cval = eval(val.replace('int64_t', ''), {})
        assert cval == py, (cname, cval, pyname, py)
        seen.add(pyname)
    assert {'_BRICK', '_L2_BYTES', '_SINGLE_WAVE_BLOCKS', '_GATE_WIDE_TABLES', '_GATE_STAGED',
            '_STAGED_SEG_BYTES', '_GATE_TRACE_STAGING', '_STAGING_SLOT_BYTES'} <= seen
