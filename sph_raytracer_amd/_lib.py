"""ctypes binding of libsphrt.so (the C ABI declared in include/sphrt.h).

The library is built in-tree by ``sph_raytracer_amd.build`` (hipcc, gfx950) and loaded *after*
torch, so it binds to the HIP runtime torch already loaded (same soname ``libamdhip64.so.7``) and
can run on torch's streams and allocations.  There is no fallback: if the library or a GPU is
missing, every compute entry point raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPHRT_LIB selects another build of the same ABI (kernel A/B studies under tools/)
LIB_PATH = os.environ.get('SPHRT_LIB') or os.path.join(_HERE, 'lib', 'libsphrt.so')
MAX_DIMS = 6

c_i32, c_i64, c_dbl, c_vp, c_int = (ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                                    ctypes.c_void_p, ctypes.c_int)


class GridDesc(ctypes.Structure):
    _fields_ = [('nr', c_i32), ('ne', c_i32), ('na', c_i32),
                ('r_b', c_vp), ('e_b', c_vp), ('a_b', c_vp),
                ('cos_e', c_vp), ('cos2_e', c_vp), ('cos_a', c_vp), ('sin_a', c_vp),
                ('a_wrap', c_i32), ('close_tol', c_dbl), ('plane_par_tol', c_dbl)]


class RayBatch(ctypes.Structure):
    _fields_ = [('ndim', c_i32),
                ('shape', c_i64 * MAX_DIMS),
                ('xs_stride', c_i64 * MAX_DIMS),
                ('rays_stride', c_i64 * MAX_DIMS),
                ('xs', c_vp), ('rays', c_vp), ('start', c_vp)]


class CSR(ctypes.Structure):
    _fields_ = [('n_rays', c_i64), ('n_segments', c_i64), ('row_ptr', c_vp), ('vox', c_vp),
                ('len', c_vp), ('len32', c_vp), ('row_ray', c_vp), ('blocks', c_vp),
                ('n_blocks', c_i64), ('loc', c_vp), ('tab', c_vp), ('n_cols', c_i64),
                ('n_fallback', c_i64), ('empty_ray', c_vp), ('tab_stride', c_i64),
                ('tab_bytes', c_i64), ('stage_shape', ctypes.c_int32 * 3),
                ('stage_brick', ctypes.c_int32 * 3), ('stage_cols', c_i64), ('stage', c_vp),
                ('stage_bytes', c_i64), ('runs', c_vp), ('order', c_i64),
                ('stage_packed', c_i64)]


ROW_HEAD = 0x80000000
BLOCK_FIELDS = 6           # SPHRT_BLOCK_FIELDS
LOC_HEAD = 0x8000          # SPHRT_LOC_HEAD
TAB_WIDE = 2048            # SPHRT_TAB_WIDE
RUN_FIELDS = 32            # SPHRT_RUN_FIELDS
MAX_RUNS = 7               # SPHRT_MAX_RUNS

# (name, restype, argtypes) — mirrors include/sphrt.h one to one
_SIGNATURES = [
    ('sphrt_plan_create', c_int, [ctypes.POINTER(GridDesc), c_int, ctypes.POINTER(c_vp)]),
    ('sphrt_plan_table_bytes', ctypes.c_size_t, [ctypes.POINTER(GridDesc)]),
    ('sphrt_plan_pack_tables', c_int, [ctypes.POINTER(GridDesc), c_vp]),
    ('sphrt_plan_create_external', c_int, [ctypes.POINTER(GridDesc), c_int, c_vp,
                                           ctypes.POINTER(c_vp)]),
    ('sphrt_plan_destroy', c_int, [c_vp]),
    ('sphrt_plan_candidates', c_i64, [c_vp]),
    ('sphrt_last_error', ctypes.c_char_p, []),
    ('sphrt_version', ctypes.c_char_p, []),
    ('sphrt_solve', c_int, [c_vp, ctypes.POINTER(RayBatch), c_int, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_solve_f32', c_int, [c_vp, ctypes.POINTER(RayBatch), c_int, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_trace_reference', c_int, [c_vp, ctypes.POINTER(RayBatch), c_int, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, ctypes.c_size_t, c_vp]),
    ('sphrt_trace_reference_emit', c_int, [c_vp, ctypes.POINTER(RayBatch), c_int, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, ctypes.c_size_t, c_vp]),
    ('sphrt_trace_workspace_bytes', ctypes.c_size_t, [c_vp, c_i64]),
    ('sphrt_trace_count', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_vp, ctypes.c_size_t,
                                  c_vp]),
    ('sphrt_scan_workspace_bytes', ctypes.c_size_t, [c_i64]),
    ('sphrt_scan_counts', c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    ('sphrt_trace_fill', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_vp, c_vp, c_vp,
                                 ctypes.c_size_t, c_vp]),
    ('sphrt_trace_bound', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_vp, ctypes.c_size_t,
                                  c_vp]),
    ('sphrt_trace_emit', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, ctypes.c_size_t, c_vp]),
    ('sphrt_trace_compact', c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_rays_cone', c_int, [c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_rays_cone_ordered', c_int, [c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_vp]),
    ('sphrt_rays_cone_tiled', c_int, [c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_i64,
                                      c_vp, c_vp, c_vp]),
    ('sphrt_csr_blocks', c_i64, [c_i64]),
    ('sphrt_csr_index_workspace_bytes', ctypes.c_size_t, [c_i64]),
    ('sphrt_csr_index', c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    ('sphrt_csr_blocks_dense', c_i64, [c_i64]),
    ('sphrt_csr_index_dense', c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                      c_vp]),
    ('sphrt_csr_index_staged', c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                       c_vp]),
    ('sphrt_csr_runs', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp]),
    ('sphrt_csr_local_count', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp]),
    ('sphrt_csr_local_fill', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_i64, c_vp]),
    ('sphrt_csr_local_build', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_csr_local_pack', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_i64, c_vp]),
    ('sphrt_csr_local_build_staged', c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_vp, c_vp,
                                             c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_csr_time_columns', c_int, [ctypes.POINTER(CSR), c_i64, c_i64, c_vp, c_vp]),
    ('sphrt_forward_f32', c_int, [ctypes.POINTER(CSR), c_vp, c_i64, c_i64, c_i64, c_vp, c_i64,
                                  c_vp]),
    ('sphrt_forward_f64', c_int, [ctypes.POINTER(CSR), c_vp, c_i64, c_i64, c_i64, c_vp, c_i64,
                                  c_vp]),
    ('sphrt_time_next_forward', c_int, [c_vp, c_vp]),
    ('sphrt_adjoint_accumulate', c_int, [ctypes.POINTER(CSR), c_vp, c_int, c_i64, c_i64, c_i64,
                                         c_vp, c_i64, c_vp]),
    ('sphrt_transpose_workspace_bytes', ctypes.c_size_t, [c_i64, c_i64]),
    ('sphrt_csr_transpose', c_int, [ctypes.POINTER(CSR), c_i64, c_vp, c_vp, c_vp, c_vp,
                                    ctypes.c_size_t, c_vp]),
    ('sphrt_f64_to_f32', c_int, [c_vp, c_vp, c_i64, c_vp]),
    ('sphrt_gather_f32', c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    ('sphrt_gather_f64', c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    ('sphrt_loss_partials', c_i64, [c_i64]),
    ('sphrt_sq_residual_f64', c_int, [c_vp, c_vp, c_int, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp]),
    ('sphrt_neg_reg_f64', c_int, [c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp]),
    ('sphrt_adam_neg_f64', c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl,
                                   c_dbl, c_dbl, c_vp, ctypes.POINTER(CSR), c_vp]),
    ('sphrt_adam_foreach_neg_f64', c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_dbl, c_dbl,
                                           c_dbl, c_dbl, c_dbl, c_dbl, c_vp, ctypes.POINTER(CSR),
                                           c_vp]),
    ('sphrt_trace_integrate_f32', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_i64, c_i64,
                                          c_i64, c_vp, c_i64, c_vp, ctypes.c_size_t, c_vp]),
    ('sphrt_trace_integrate_f64', c_int, [c_vp, ctypes.POINTER(RayBatch), c_vp, c_i64, c_i64,
                                          c_i64, c_vp, c_i64, c_vp, ctypes.c_size_t, c_vp]),
]
EXPORTED = [s[0] for s in _SIGNATURES]
TRACE_F32, TRACE_INVALID, TRACE_FRESH_RAYS = 1, 2, 4   # sphrt_trace_reference flags (sphrt.h)

_lib = None


def load():
    """Load libsphrt.so (once).  Raises RuntimeError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f'sph_raytracer_amd: HIP library not found at {LIB_PATH}; build it with '
            '`python -m sph_raytracer_amd.build` (hipcc --offload-arch=gfx950). '
            'There is no CPU fallback.')
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    # the source-hash check first: a stale library may lack exports this tree binds, and that
    # must read as "rebuild", not as an AttributeError from the signature loop
    lib.sphrt_version.restype = ctypes.c_char_p
    lib.sphrt_version.argtypes = []
    if not os.environ.get('SPHRT_LIB'):   # an A/B variant may come from other sources
        _check_hash(lib.sphrt_version().decode(), LIB_PATH)
    for name, res, args in _SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            raise RuntimeError(f'sph_raytracer_amd: {LIB_PATH} does not export {name}; rebuild '
                               'with `python -m sph_raytracer_amd.build`') from None
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check_hash(version, path, fast=False):
    """Refuse a library built from other sources than this tree's (build.source_hash, embedded
    as the version's 'src <hash>'): a stale binary shipped next to edited sources would
    otherwise run silently.  Trees without the sources (an installed copy) skip the check."""
    from . import build
    if not build.have_sources():
        return
    want = build.fast_hash() if fast else build.source_hash()
    got = version.rsplit(' src ', 1)[-1] if ' src ' in version else None
    if got != want:
        raise RuntimeError(f'sph_raytracer_amd: {path} was built from sources {got}, this tree is '
                           f'{want}; rebuild with `python -m sph_raytracer_amd.build`')


def source_hash():
    """The hash of the sources the loaded library was built from (sphrt_version)."""
    return load().sphrt_version().decode().rsplit(' src ', 1)[-1]


_fast = None
FAST_PATH = os.path.join(_HERE, 'lib', '_sphrt_fast.so')


def load_fast():
    """The CPython steady-state entry (csrc/fastpath.cpp), or None when it was not built (then
    Operator.__call__ binds through ctypes only: same kernels, more host time per call)."""
    global _fast
    if _fast is None:
        _fast = False
        if os.path.exists(FAST_PATH):
            import importlib.util
            spec = importlib.util.spec_from_file_location('_sphrt_fast', FAST_PATH)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            _check_hash(getattr(mod, 'version', ''), FAST_PATH, fast=True)
            _fast = mod
    return _fast or None


_construct = None


def load_construct():
    """The fast entry bound for Operator construction (csrc/construct.cpp: build_cone over the
    library this module loaded), or None when the entry was not built."""
    global _construct
    if _construct is None:
        _construct = False
        fast = load_fast()
        if fast is not None:
            from .geometry import ConeCircGeom, ConeRectGeom, ViewGeomCollection
            load()
            fast.construct_bind(LIB_PATH, ConeRectGeom, ConeCircGeom, ViewGeomCollection)
            _construct = fast
    return _construct or None


def address(fn):
    """Address of a ctypes-bound C function (for the fast path's bindings)."""
    return ctypes.cast(fn, ctypes.c_void_p).value


def check(status, what):
    if status != 0:
        msg = load().sphrt_last_error().decode(errors='replace')
        raise RuntimeError(f'{what} failed: {msg}')


def compute_device(device=None, current=None):
    """The GPU a call computes on: `device` itself when it names a GPU ('cuda', 'cuda:1',
    torch.device), else (None, 'cpu': results are returned to the host) the current GPU.
    `current` stands in for torch.cuda.current_device() (tests)."""
    if device is not None:
        d = torch.device(device)
        if d.type == 'cuda':
            if d.index is not None:
                return d
            device = None
    idx = torch.cuda.current_device() if current is None else current
    return torch.device('cuda', idx)


def require_gpu(device=None):
    """The device every kernel of a call runs on (compute_device).  No GPU -> loud failure (no
    CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError('sph_raytracer_amd requires a ROCm GPU (MI355X / gfx950); '
                           'torch.cuda.is_available() is False and there is no CPU fallback.')
    load()
    dev = compute_device(device)
    if dev.index >= torch.cuda.device_count():
        raise RuntimeError(f'{dev} does not exist ({torch.cuda.device_count()} GPUs visible)')
    return dev


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
