// construct.cpp — the float64 Operator construction in one C++ call (cone-beam detectors:
// build_cone; any other geometry from its host starts and directions: build_rays).
//
// Host code only (no kernels): part of the CPython entry _sphrt_fast.so (csrc/fastpath.cpp); the
// device work is libsphrt.so's C ABI (include/sphrt.h), resolved from the library the Python
// binding loaded (_lib.LIB_PATH).  Replaces, for ConeRectGeom / ConeCircGeom views, the Python
// sequence of raytracer.Operator._trace_on (the reference's Operator.__init__ ->
// trace_indices, raytracer.py:647-690 / 48-173): at the small configs that sequence spends most
// of the cold time in Python between kernels (C2: 0.8 ms wall for 0.29 ms of kernels,
// profiles/r05_operator_times.json).
//
// Every host value the trace reads comes from the same torch CPU operations as the Python path
// (ViewGeomCollection._ray_spec_batched, ConeRectGeom/ConeCircGeom._ray_spec, _ConeRays.of,
// ViewGeomCollection.ray_starts, _RayBatch.host_starts / _find_starts_host, _Plan), so the
// bits are the same (tests/test_construct.py compares both on the CPU, and the resulting CSRs
// on the GPU).  The device sequence is _trace_csr's one-pass trace followed by _index's staged
// table build with _local_tables' run records, allocations from torch's caching allocator on the
// current stream.
//
// cone_host() / build_cone() return None, with no Python error set, for any input outside that
// sequence (other geometry types, views that differ in shape / fov / radii, non-finite starts,
// unsorted boundaries, no rays) before any device work: the caller takes the Python path.  The
// rare device-side branches — a ray over its bound, a staging or table build that does not fit
// in free memory — also return None (after the device work so far); the caller then constructs
// in Python, which handles them.
#include <Python.h>

#include <ATen/ATen.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/csrc/autograd/python_variable.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "sphrt.h"

namespace sphrt_fast {

namespace {

struct Lib {
    decltype(&sphrt_plan_table_bytes) plan_table_bytes = nullptr;
    decltype(&sphrt_plan_pack_tables) plan_pack_tables = nullptr;
    decltype(&sphrt_plan_create_external) plan_create_external = nullptr;
    decltype(&sphrt_plan_destroy) plan_destroy = nullptr;
    decltype(&sphrt_last_error) last_error = nullptr;
    decltype(&sphrt_rays_cone) rays_cone = nullptr;
    decltype(&sphrt_rays_cone_ordered) rays_cone_ordered = nullptr;
    decltype(&sphrt_rays_cone_tiled) rays_cone_tiled = nullptr;
    decltype(&sphrt_trace_workspace_bytes) trace_workspace_bytes = nullptr;
    decltype(&sphrt_scan_workspace_bytes) scan_workspace_bytes = nullptr;
    decltype(&sphrt_scan_counts) scan_counts = nullptr;
    decltype(&sphrt_trace_bound) trace_bound = nullptr;
    decltype(&sphrt_trace_emit) trace_emit = nullptr;
    decltype(&sphrt_csr_blocks) csr_blocks = nullptr;
    decltype(&sphrt_csr_index_workspace_bytes) csr_index_workspace_bytes = nullptr;
    decltype(&sphrt_csr_index_staged) csr_index_staged = nullptr;
    decltype(&sphrt_csr_runs) csr_runs = nullptr;
    decltype(&sphrt_csr_local_build_staged) csr_local_build_staged = nullptr;
    decltype(&sphrt_csr_local_pack) csr_local_pack = nullptr;
};

Lib g_lib;
bool g_bound = false;
PyObject* g_rect = nullptr;   // geometry.ConeRectGeom
PyObject* g_circ = nullptr;   // geometry.ConeCircGeom
PyObject* g_coll = nullptr;   // geometry.ViewGeomCollection

// raytracer.py constants this sequence follows
constexpr int64_t kSingleWaveBlocks = 256 * 6;          // _SINGLE_WAVE_BLOCKS
constexpr int kBrick[3] = {4, 2, 4};                     // _BRICK
constexpr int64_t kL2Bytes = int64_t(4) << 20;           // _L2_BYTES
constexpr double kGateWideTables = 0.3;                   // _GATE_WIDE_TABLES
constexpr double kGateStaged = 0.5;                       // _GATE_STAGED
constexpr double kStagedSegBytes = 18.0;                  // _STAGED_SEG_BYTES
constexpr double kGateTraceStaging = 0.4;                 // _GATE_TRACE_STAGING
constexpr double kStagingSlotBytes = 12.0;                // _STAGING_SLOT_BYTES
constexpr int64_t kTabWide = SPHRT_TAB_WIDE;
constexpr int64_t kRunFields = SPHRT_RUN_FIELDS;
constexpr int64_t kBlockFields = SPHRT_BLOCK_FIELDS;

struct LibError {
    std::string what;
};

void check(int rc, const char* what) {
    if (rc != 0)
        throw LibError{std::string(what) + " failed: " +
                       (g_lib.last_error ? g_lib.last_error() : "unknown error")};
}

int64_t seg_alloc(int64_t total) { return std::max<int64_t>((total + 15) / 16 * 16, 16); }

// ---- Python attribute helpers (false: attribute missing or not what the sequence expects) ----

// attribute names, interned once (construct_bind)
PyObject* g_names[7];
enum Name { kLookdir, kUpdir, kPos, kFov, kShape, kR, kTheta };
const char* const kNames[7] = {"lookdir", "updir", "pos", "fov", "shape", "r", "theta"};

bool tensor_attr(PyObject* o, Name name, at::Tensor& out) {
    PyObject* a = PyObject_GetAttr(o, g_names[name]);
    if (!a) {
        PyErr_Clear();
        return false;
    }
    const bool ok = THPVariable_Check(a);
    if (ok) out = THPVariable_Unpack(a);
    Py_DECREF(a);
    return ok && out.defined() && out.device().is_cpu();
}

bool int_seq(PyObject* o, std::vector<int64_t>& out) {
    PyObject* seq = PySequence_Fast(o, "sequence");
    if (!seq) {
        PyErr_Clear();
        return false;
    }
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    out.resize(n);
    bool ok = true;
    for (Py_ssize_t i = 0; i < n && ok; ++i) {
        PyObject* it = PySequence_Fast_GET_ITEM(seq, i);
        if (!PyLong_Check(it)) {
            ok = false;
            break;
        }
        out[i] = PyLong_AsLongLong(it);
        if (out[i] == -1 && PyErr_Occurred()) {
            PyErr_Clear();
            ok = false;
        }
    }
    Py_DECREF(seq);
    return ok;
}

bool shape_attr(PyObject* o, std::vector<int64_t>& out) {
    PyObject* a = PyObject_GetAttr(o, g_names[kShape]);
    if (!a) {
        PyErr_Clear();
        return false;
    }
    const bool ok = int_seq(a, out);
    Py_DECREF(a);
    return ok;
}

// ---- the host values of the trace --------------------------------------------------------

struct View {
    at::Tensor look, up, pos, fov, r, theta;
    std::vector<int64_t> shape;
};

bool read_view(PyObject* g, bool circ, View& v) {
    if (!tensor_attr(g, kLookdir, v.look) || !tensor_attr(g, kUpdir, v.up) ||
        !tensor_attr(g, kPos, v.pos) || !tensor_attr(g, kFov, v.fov) || !shape_attr(g, v.shape))
        return false;
    if (circ && (!tensor_attr(g, kR, v.r) || !tensor_attr(g, kTheta, v.theta)))
        return false;
    return true;
}

// torch.stack of same-shape contiguous float64 tensors: a copy of their values
at::Tensor stack_f64(const std::vector<const at::Tensor*>& ts) {
    const int64_t k = ts[0]->numel();
    std::vector<int64_t> shape{(int64_t)ts.size()};
    shape.insert(shape.end(), ts[0]->sizes().begin(), ts[0]->sizes().end());
    at::Tensor out = at::empty(shape, at::kDouble);
    double* o = out.mutable_data_ptr<double>();
    for (size_t i = 0; i < ts.size(); ++i)
        std::memcpy(o + i * k, ts[i]->const_data_ptr<double>(), k * sizeof(double));
    return out;
}

bool f64_vector(const at::Tensor& t, int64_t n) {
    return t.scalar_type() == at::kDouble && t.numel() == n && t.is_contiguous();
}

// torch.equal for same-dtype contiguous tensors, NaN never equal (a NaN takes the Python path)
bool same_values(const at::Tensor& a, const at::Tensor& b) {
    if (a.scalar_type() != b.scalar_type() || !a.sizes().equals(b.sizes()) ||
        !a.is_contiguous() || !b.is_contiguous())
        return false;
    if (a.scalar_type() == at::kDouble) {
        const double *p = a.const_data_ptr<double>(), *q = b.const_data_ptr<double>();
        for (int64_t i = 0; i < a.numel(); ++i)
            if (!(p[i] == q[i])) return false;
        return true;
    }
    if (a.scalar_type() == at::kFloat) {
        const float *p = a.const_data_ptr<float>(), *q = b.const_data_ptr<float>();
        for (int64_t i = 0; i < a.numel(); ++i)
            if (!(p[i] == q[i])) return false;
        return true;
    }
    return false;
}

struct Spec {   // ConeRectGeom / ConeCircGeom._ray_spec()
    int circ = 0;
    at::Tensor frame, row, col;
};

// ConeRectGeom._span
at::Tensor span(const View& v, int axis, bool& is_zero) {
    is_zero = v.shape[axis] <= 1;
    if (is_zero) return at::Tensor();
    return at::tan(at::deg2rad(v.fov.select(0, axis) / 2));
}

// frame: false for the batched call, whose frames come from the stacked views
bool view_spec(const View& v, bool circ, Spec& s, bool frame = true) {
    if (v.shape.size() != 2 || v.look.dim() != 1 || v.up.dim() != 1) return false;
    const at::Tensor right = frame ? at::cross(v.look, v.up, -1) : at::Tensor();
    if (!circ) {
        bool z0, z1;
        const at::Tensor ulim = span(v, 0, z0), vlim = span(v, 1, z1);
        s.circ = 0;
        if (frame) s.frame = at::cat({v.look, right, v.up});
        s.row = z0 ? at::linspace(0, 0, v.shape[0]) : at::linspace(at::neg(ulim), ulim, v.shape[0]);
        s.col = z1 ? at::linspace(0, 0, v.shape[1]) : at::linspace(at::neg(vlim), vlim, v.shape[1]);
        return true;
    }
    if (v.theta.dim() != 1) return false;
    const at::Tensor ang = v.theta.unsqueeze(0).unsqueeze(2);
    const at::Tensor cs = at::cos(ang).reshape(-1), sn = at::sin(ang).reshape(-1);
    const bool single = v.r.scalar_type() == at::kFloat && cs.scalar_type() == at::kFloat;
    s.circ = single ? 2 : 1;
    if (frame) s.frame = at::cat({v.look, right, v.up});
    s.row = v.r;
    s.col = at::cat({cs, sn});
    return true;
}

struct Prelude {
    Spec spec;                  // float64 contiguous frame / row / col
    std::vector<int64_t> shape; // geom.shape
    int64_t n_views = 1, h = 0, w = 0;
    bool circ_kind = false;
    at::Tensor xs, st;          // host starts (..., 3) float64, start voxels (..., 4) int32
    at::Tensor keep[7];         // r_b, e_b, a_b, cos_e, cos2_e, cos_a, sin_a (float64)
    sphrt_grid_desc desc{};
};

// _find_starts_host: sqrt / atan2 through torch on the same layouts, squares / sums / binning
// as the exact IEEE operations numpy does
bool find_starts(const at::Tensor& xs_u, const at::Tensor* bounds, const int64_t* nbins,
                 at::Tensor& st) {
    const at::Tensor xt = xs_u.reshape({-1, 3});
    const int64_t n = xt.size(0);
    const double* x = xt.const_data_ptr<double>();
    for (int64_t i = 0; i < 3 * n; ++i)
        if (!std::isfinite(x[i])) return false;
    at::Tensor rho2 = at::empty({n}, at::kDouble), rr = at::empty({n}, at::kDouble);
    double* p = rho2.mutable_data_ptr<double>();
    double* q = rr.mutable_data_ptr<double>();
    for (int64_t i = 0; i < n; ++i) {
        const double a = x[3 * i] * x[3 * i];
        const double b = x[3 * i + 1] * x[3 * i + 1];
        const double c = x[3 * i + 2] * x[3 * i + 2];
        p[i] = a + b;
        q[i] = p[i] + c;
    }
    const at::Tensor sph[3] = {at::sqrt(rr), at::atan2(at::sqrt(rho2), xt.select(1, 2)),
                               at::atan2(xt.select(1, 1), xt.select(1, 0))};
    std::vector<int64_t> sshape(xs_u.sizes().begin(), xs_u.sizes().end() - 1);
    sshape.push_back(4);
    st = at::zeros(sshape, at::kInt);
    int32_t* o = st.mutable_data_ptr<int32_t>();
    for (int k = 0; k < 3; ++k) {
        const at::Tensor sv = sph[k].contiguous();
        const double* v = sv.const_data_ptr<double>();
        const double* b = bounds[k].const_data_ptr<double>();
        const int64_t nb = bounds[k].numel(), nk = nbins[k];
        for (int64_t i = 0; i < n; ++i) {
            int64_t idx = (std::upper_bound(b, b + nb, v[i]) - b) - 1;   // searchsorted right
            if (v[i] == b[nb - 1]) idx = nk - 1;
            if (idx == nk) idx = -1;
            o[4 * i + k] = (int32_t)idx;
        }
    }
    return true;
}

bool sorted_finite(const at::Tensor& b) {
    const double* p = b.const_data_ptr<double>();
    for (int64_t i = 0; i < b.numel(); ++i)
        if (!std::isfinite(p[i]) || (i && !(p[i - 1] <= p[i]))) return false;
    return b.numel() >= 2;
}

bool grid_prelude(PyObject* const* grid_b, const int64_t* nbins, Prelude& P);

// geom + grid boundaries -> the trace's host values; false (no error set): not this sequence
bool prelude(PyObject* geom, PyObject* const* grid_b, const int64_t* nbins, Prelude& P) {
    std::vector<PyObject*> views;
    const bool coll = (PyObject*)Py_TYPE(geom) == g_coll;
    PyObject* list = nullptr;
    if (coll) {
        list = PyObject_GetAttrString(geom, "geoms");
        if (!list) {
            PyErr_Clear();
            return false;
        }
        if (!PyList_Check(list) || PyList_GET_SIZE(list) == 0) {
            Py_DECREF(list);
            return false;
        }
        for (Py_ssize_t i = 0; i < PyList_GET_SIZE(list); ++i)
            views.push_back(PyList_GET_ITEM(list, i));
    } else {
        views.push_back(geom);
    }
    struct Ref {
        PyObject* o;
        ~Ref() { Py_XDECREF(o); }
    } hold{list};
    PyObject* kind = (PyObject*)Py_TYPE(views[0]);
    if (kind != g_rect && kind != g_circ) return false;
    for (PyObject* g : views)
        if ((PyObject*)Py_TYPE(g) != kind) return false;
    const bool circ = kind == g_circ;
    P.circ_kind = circ;

    std::vector<View> vs(views.size());
    for (size_t i = 0; i < views.size(); ++i)
        if (!read_view(views[i], circ, vs[i])) return false;
    for (const View& v : vs)
        if (!f64_vector(v.look, 3) || !f64_vector(v.up, 3) || !f64_vector(v.pos, 3) ||
            !f64_vector(v.fov, 2))
            return false;

    Spec spec;
    if (coll) {   // ViewGeomCollection._ray_spec_batched
        const View& v0 = vs[0];
        const double* f0 = v0.fov.const_data_ptr<double>();
        for (const View& v : vs) {
            const double* f = v.fov.const_data_ptr<double>();
            if (v.shape != v0.shape || !(f[0] == f0[0]) || !(f[1] == f0[1])) return false;
            if (circ && !(same_values(v.r, v0.r) && same_values(v.theta, v0.theta))) return false;
        }
        std::vector<const at::Tensor*> looks, ups;
        for (const View& v : vs) {
            looks.push_back(&v.look);
            ups.push_back(&v.up);
        }
        const at::Tensor look = stack_f64(looks), up = stack_f64(ups);
        const at::Tensor frame = at::cat({look, at::cross(look, up, -1), up}, -1);
        Spec s0;
        if (!view_spec(v0, circ, s0, false)) return false;
        const int64_t n = (int64_t)vs.size();
        spec.circ = s0.circ;
        spec.frame = frame;
        std::vector<int64_t> rs{n}, cs{n};
        rs.insert(rs.end(), s0.row.sizes().begin(), s0.row.sizes().end());
        cs.insert(cs.end(), s0.col.sizes().begin(), s0.col.sizes().end());
        spec.row = s0.row.expand(rs);
        spec.col = s0.col.expand(cs);
        P.shape = {n};
        P.shape.insert(P.shape.end(), v0.shape.begin(), v0.shape.end());
    } else {
        if (!view_spec(vs[0], circ, spec)) return false;
        P.shape = vs[0].shape;
    }
    // _ConeRays.of
    P.spec.circ = spec.circ;
    P.spec.frame = spec.frame.to(at::kDouble).contiguous();
    P.spec.row = spec.row.to(at::kDouble).contiguous();
    P.spec.col = spec.col.to(at::kDouble).contiguous();
    if (P.shape.size() < 2 || P.shape.size() > SPHRT_MAX_DIMS) return false;
    P.n_views = P.spec.frame.dim() == 2 ? P.spec.frame.size(0) : 1;
    P.h = P.shape[P.shape.size() - 2];
    P.w = P.shape[P.shape.size() - 1];
    int64_t prod = 1;
    for (int64_t s : P.shape) prod *= s;
    if (P.n_views * P.h * P.w != prod || P.spec.row.size(-1) != P.h || prod <= 0) return false;

    // ViewGeomCollection.ray_starts / ConeRectGeom.ray_starts, then _RayBatch.host_starts
    at::Tensor xs;
    if (coll) {
        std::vector<const at::Tensor*> poss;
        for (const View& v : vs) poss.push_back(&v.pos);
        xs = stack_f64(poss).unsqueeze(1).unsqueeze(1);
    } else {
        xs = vs[0].pos.unsqueeze(0).unsqueeze(0);
    }
    P.xs = xs.to(at::kDouble).contiguous();
    return grid_prelude(grid_b, nbins, P);
}

// _Plan and _RayBatch.host_starts for starts P.xs: boundaries in float64 (the fast trace's
// dtype), trig tables with torch CPU, start voxels; false: not this sequence
bool grid_prelude(PyObject* const* grid_b, const int64_t* nbins, Prelude& P) {
    at::Tensor b[3];
    for (int k = 0; k < 3; ++k) {
        if (!THPVariable_Check(grid_b[k])) return false;
        b[k] = THPVariable_Unpack(grid_b[k]);
        if (!b[k].device().is_cpu() || b[k].dim() != 1) return false;
        b[k] = b[k].to(at::kDouble).contiguous();
        if (!sorted_finite(b[k]) || nbins[k] != b[k].numel() - 1) return false;
    }
    if (!find_starts(P.xs, b, nbins, P.st)) return false;
    const at::Tensor& ab = b[2];
    P.keep[0] = b[0];
    P.keep[1] = b[1];
    P.keep[2] = ab;
    P.keep[3] = at::cos(b[1]);
    P.keep[4] = at::pow(at::cos(b[1]), 2);
    P.keep[5] = at::cos(ab);
    P.keep[6] = at::sin(ab);
    const double* a = ab.const_data_ptr<double>();
    const double a_last = a[ab.numel() - 1];
    sphrt_grid_desc& d = P.desc;
    d.nr = (int32_t)(b[0].numel() - 1);
    d.ne = (int32_t)(b[1].numel() - 1);
    d.na = (int32_t)(ab.numel() - 1);
    d.r_b = P.keep[0].const_data_ptr<double>();
    d.e_b = P.keep[1].const_data_ptr<double>();
    d.a_b = P.keep[2].const_data_ptr<double>();
    d.cos_e = P.keep[3].const_data_ptr<double>();
    d.cos2_e = P.keep[4].const_data_ptr<double>();
    d.cos_a = P.keep[5].const_data_ptr<double>();
    d.sin_a = P.keep[6].const_data_ptr<double>();
    d.a_wrap = (-a[0] == a_last) && (a_last == M_PI);
    d.close_tol = std::pow(1e-15, 1.0 / 3.0);   // finfo(float64).resolution ** (1 / 3)
    d.plane_par_tol = 1e-15;
    return true;
}

// ---- the one host-to-device copy (_Staging: 16-byte aligned slots) -------------------------

struct Slots {
    std::vector<std::pair<const void*, int64_t>> parts;
    std::vector<int64_t> offs;
    int64_t size = 0;
    int add(const void* p, int64_t bytes) {
        offs.push_back(size);
        parts.emplace_back(p, bytes);
        size += (bytes + 15) / 16 * 16;
        return (int)offs.size() - 1;
    }
    void write(uint8_t* dst) const {
        std::memset(dst, 0, size);
        for (size_t i = 0; i < parts.size(); ++i)
            if (parts[i].second) std::memcpy(dst + offs[i], parts[i].first, parts[i].second);
    }
};

// The sizes of the staged spec blob pieces
int64_t nbytes(const at::Tensor& t) { return t.numel() * (int64_t)t.element_size(); }

PyObject* wrap(at::Tensor t) {
    if (!t.defined()) Py_RETURN_NONE;
    return THPVariable_Wrap(std::move(t));
}

struct PlanGuard {
    sphrt_plan* p = nullptr;
    ~PlanGuard() {
        if (p) g_lib.plan_destroy(p);
    }
};

// What the common part of a construction starts from: the plan (owned by the guard), the ray
// batch over the staged starts and the device rays, and what the Operator keeps of them.
struct Batch {
    sphrt_rays rd{};
    int64_t n = 0;
    at::Tensor rays;                // device rays (released once traced)
    at::Tensor ray_id;              // the geometry ray of each trace row, or undefined
    at::Tensor xs_keep;             // the staged starts (kept: debug_los)
    std::vector<int64_t> rshape;    // the Operator's ray shape
};

bool prelude_args(PyObject* const* args, int64_t* nbins) {
    for (int k = 0; k < 3; ++k) {
        nbins[k] = PyLong_AsLongLong(args[4 + k]);
        if (nbins[k] == -1 && PyErr_Occurred()) return false;
    }
    return true;
}

}  // namespace

PyObject* build_tail(PlanGuard& guard, Batch& B, const int64_t* nbins, int64_t n_cols,
                     sphrt_csr* c, hipStream_t stream, const at::TensorOptions& on_dev);

// bind(lib_path, ConeRectGeom, ConeCircGeom, ViewGeomCollection)
PyObject* construct_bind(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 4 || !PyUnicode_Check(args[0])) {
        PyErr_SetString(PyExc_TypeError, "construct_bind(lib_path, rect, circ, collection)");
        return nullptr;
    }
    const char* path = PyUnicode_AsUTF8(args[0]);
    void* h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        PyErr_Format(PyExc_RuntimeError, "construct_bind: cannot open %s", path);
        return nullptr;
    }
    Lib L;
    bool ok = true;
#define SPHRT_SYM(field, name)                                                  \
    L.field = reinterpret_cast<decltype(L.field)>(dlsym(h, name));             \
    ok = ok && L.field != nullptr;
    SPHRT_SYM(plan_table_bytes, "sphrt_plan_table_bytes")
    SPHRT_SYM(plan_pack_tables, "sphrt_plan_pack_tables")
    SPHRT_SYM(plan_create_external, "sphrt_plan_create_external")
    SPHRT_SYM(plan_destroy, "sphrt_plan_destroy")
    SPHRT_SYM(last_error, "sphrt_last_error")
    SPHRT_SYM(rays_cone, "sphrt_rays_cone")
    SPHRT_SYM(rays_cone_ordered, "sphrt_rays_cone_ordered")
    SPHRT_SYM(rays_cone_tiled, "sphrt_rays_cone_tiled")
    SPHRT_SYM(trace_workspace_bytes, "sphrt_trace_workspace_bytes")
    SPHRT_SYM(scan_workspace_bytes, "sphrt_scan_workspace_bytes")
    SPHRT_SYM(scan_counts, "sphrt_scan_counts")
    SPHRT_SYM(trace_bound, "sphrt_trace_bound")
    SPHRT_SYM(trace_emit, "sphrt_trace_emit")
    SPHRT_SYM(csr_blocks, "sphrt_csr_blocks")
    SPHRT_SYM(csr_index_workspace_bytes, "sphrt_csr_index_workspace_bytes")
    SPHRT_SYM(csr_index_staged, "sphrt_csr_index_staged")
    SPHRT_SYM(csr_runs, "sphrt_csr_runs")
    SPHRT_SYM(csr_local_build_staged, "sphrt_csr_local_build_staged")
    SPHRT_SYM(csr_local_pack, "sphrt_csr_local_pack")
#undef SPHRT_SYM
    if (!ok) {
        PyErr_Format(PyExc_RuntimeError, "construct_bind: %s lacks an entry point", path);
        return nullptr;
    }
    for (int i = 0; i < 7; ++i)
        if (!g_names[i] && !(g_names[i] = PyUnicode_InternFromString(kNames[i]))) return nullptr;
    for (int i = 1; i < 4; ++i) Py_INCREF(args[i]);
    Py_XDECREF(g_rect);
    Py_XDECREF(g_circ);
    Py_XDECREF(g_coll);
    g_rect = args[1];
    g_circ = args[2];
    g_coll = args[3];
    g_lib = L;
    g_bound = true;
    Py_RETURN_NONE;
}

// cone_host(geom, r_b, e_b, a_b, nr, ne, na) -> (circ, frame, row, col, xs, start, plan_tables)
// | None: the host values build_cone stages (tests compare them with the Python path's)
PyObject* construct_cone_host(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 7 || !g_bound) {
        PyErr_SetString(PyExc_TypeError, "cone_host(geom, r_b, e_b, a_b, nr, ne, na) after bind");
        return nullptr;
    }
    int64_t nbins[3];
    if (!prelude_args(args, nbins)) return nullptr;
    try {
        Prelude P;
        if (!prelude(args[0], args + 1, nbins, P)) {
            if (PyErr_Occurred()) return nullptr;
            Py_RETURN_NONE;
        }
        at::Tensor tables = at::empty({(int64_t)g_lib.plan_table_bytes(&P.desc)}, at::kByte);
        check(g_lib.plan_pack_tables(&P.desc, tables.mutable_data_ptr()), "sphrt_plan_pack_tables");
        return Py_BuildValue("(iNNNNNN)", P.spec.circ, wrap(P.spec.frame), wrap(P.spec.row),
                             wrap(P.spec.col), wrap(P.xs), wrap(P.st), wrap(tables));
    } catch (const LibError& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what.c_str());
    } catch (const std::exception& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    return nullptr;
}

// build_cone(geom, r_b, e_b, a_b, nr, ne, na, perm, tiles, n_cols, csr_address) ->
//   (row_ptr, vox, len32, row_ray, empty_ray, blocks, loc, tab, runs, ray_id, bound_ptr, slen,
//    xs, total, n_blocks, ray_shape) | None
// perm: the ConeCirc wedge order of one view (raytracer._wedge_order, CPU int64) or None; used
// for ConeCirc views only (raytracer._trace_order).  tiles: (tv, tw) view tiles of an orbit
// (raytracer._view_tiles; the trace order then, perm unused) or None.  csr_address: a zeroed
// sphrt_csr the call fills (the Operator's _lib.CSR).  Runs on the current HIP device and
// stream.
PyObject* construct_build_cone(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 11 || !g_bound) {
        PyErr_SetString(PyExc_TypeError, "build_cone(geom, r_b, e_b, a_b, nr, ne, na, perm, "
                                         "tiles, n_cols, csr_address) after bind");
        return nullptr;
    }
    int64_t nbins[3];
    if (!prelude_args(args, nbins)) return nullptr;
    int64_t tv = 0, tw = 0;
    if (args[8] != Py_None) {
        std::vector<int64_t> t;
        if (!int_seq(args[8], t) || t.size() != 2 || t[0] < 1 || t[1] < 1) {
            PyErr_SetString(PyExc_ValueError, "tiles: (tv, tw) or None");
            return nullptr;
        }
        tv = t[0];
        tw = t[1];
    }
    const int64_t n_cols = PyLong_AsLongLong(args[9]);
    auto* c = static_cast<sphrt_csr*>(PyLong_AsVoidPtr(args[10]));
    if (PyErr_Occurred()) return nullptr;
    PlanGuard guard;
    try {
        Prelude P;
        if (!prelude(args[0], args + 1, nbins, P)) {
            if (PyErr_Occurred()) return nullptr;
            Py_RETURN_NONE;
        }
        const bool tiled = tv > 0 && P.n_views > 1;
        if (tiled && (P.n_views % tv != 0 || P.w % tw != 0)) Py_RETURN_NONE;
        at::Tensor perm;
        if (!tiled && P.circ_kind && args[7] != Py_None) {
            if (!THPVariable_Check(args[7])) Py_RETURN_NONE;
            perm = THPVariable_Unpack(args[7]);
            if (perm.scalar_type() != at::kLong || !perm.is_contiguous() ||
                perm.numel() != P.h * P.w || !perm.device().is_cpu())
                Py_RETURN_NONE;
        }
        const int dev = (int)c10::hip::current_device();
        hipStream_t stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
        const at::TensorOptions on_dev = at::TensorOptions().device(at::kCUDA, dev);

        // plan tables, cone spec, wedge order, starts, start voxels: one copy from pinned memory
        const int64_t tbytes = (int64_t)g_lib.plan_table_bytes(&P.desc);
        at::Tensor tables = at::empty({tbytes}, at::kByte);
        check(g_lib.plan_pack_tables(&P.desc, tables.mutable_data_ptr()), "sphrt_plan_pack_tables");
        Slots S;
        const int s_tab = S.add(tables.const_data_ptr(), tbytes);
        const int s_frame = S.add(P.spec.frame.const_data_ptr(), nbytes(P.spec.frame));
        const int s_row = S.add(P.spec.row.const_data_ptr(), nbytes(P.spec.row));
        const int s_col = S.add(P.spec.col.const_data_ptr(), nbytes(P.spec.col));
        const int s_perm = perm.defined() ? S.add(perm.const_data_ptr(), nbytes(perm)) : -1;
        const int s_xs = S.add(P.xs.const_data_ptr(), nbytes(P.xs));
        const int s_st = S.add(P.st.const_data_ptr(), nbytes(P.st));
        at::Tensor host = at::empty({S.size}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
        S.write(host.mutable_data_ptr<uint8_t>());
        const at::Tensor staged = host.to(on_dev.dtype(at::kByte), /*non_blocking=*/true);
        auto dptr = [&](int slot) { return (uint8_t*)staged.data_ptr() + S.offs[slot]; };

        check(g_lib.plan_create_external(&P.desc, dev, dptr(s_tab), &guard.p),
              "sphrt_plan_create_external");
        sphrt_plan* const plan = guard.p;

        // rays on the device (sphrt_rays_cone[_ordered|_tiled]): the geometry shape (..., 3),
        // or the view-tile layout (h, w / tw, n_views / tv, tv, tw, 3)
        const std::vector<int64_t> rshape = P.shape;
        std::vector<int64_t> bshape = tiled ? std::vector<int64_t>{P.h, P.w / tw, P.n_views / tv,
                                                                   tv, tw}
                                            : rshape;
        std::vector<int64_t> full = bshape;
        full.push_back(3);
        const int64_t n = P.n_views * P.h * P.w;
        at::Tensor rays = at::empty(full, on_dev.dtype(at::kDouble));
        at::Tensor ray_id;
        const double* frame_d = (const double*)dptr(s_frame);
        const double* row_d = (const double*)dptr(s_row);
        const double* col_d = (const double*)dptr(s_col);
        if (tiled) {
            ray_id = at::empty({n}, on_dev.dtype(at::kInt));
            check(g_lib.rays_cone_tiled(P.n_views, P.h, P.w, P.spec.circ, frame_d, row_d, col_d,
                                        tv, tw, rays.data_ptr<double>(),
                                        ray_id.data_ptr<int32_t>(), stream),
                  "sphrt_rays_cone_tiled");
        } else if (s_perm >= 0) {
            ray_id = at::empty({n}, on_dev.dtype(at::kInt));
            check(g_lib.rays_cone_ordered(P.n_views, P.h, P.w, P.spec.circ, frame_d, row_d, col_d,
                                          (const int64_t*)dptr(s_perm), rays.data_ptr<double>(),
                                          ray_id.data_ptr<int32_t>(), stream),
                  "sphrt_rays_cone_ordered");
        } else {
            check(g_lib.rays_cone(P.n_views, P.h, P.w, P.spec.circ, frame_d, row_d, col_d,
                                  rays.data_ptr<double>(), stream),
                  "sphrt_rays_cone");
        }
        // _RayBatch over the staged starts (broadcast against the rays, raytracer.py:76-80)
        Batch B;
        B.xs_keep = staged.narrow(0, S.offs[s_xs], nbytes(P.xs)).view(at::kDouble).view(P.xs.sizes());
        const at::Tensor& xs_keep = B.xs_keep;
        // tiles: the view starts (V, 1, 1, 3) as (1, 1, V / tv, tv, 1, 3) over the tile layout
        const at::Tensor xs_b = tiled ? xs_keep.reshape({1, 1, P.n_views / tv, tv, 1, 3}) : xs_keep;
        if ((int64_t)bshape.size() > SPHRT_MAX_DIMS) Py_RETURN_NONE;
        sphrt_rays& rd = B.rd;
        rd.ndim = (int32_t)bshape.size();
        // (the strides copied out: an IntArrayRef of a temporary's strides dangles)
        const std::vector<int64_t> xs_str = xs_b.expand(full).strides().vec();
        const std::vector<int64_t> ry_str = rays.strides().vec();
        for (size_t i = 0; i < bshape.size(); ++i) {
            rd.shape[i] = bshape[i];
            rd.xs_stride[i] = xs_str[i];
            rd.rays_stride[i] = ry_str[i];
        }
        rd.xs = xs_keep.const_data_ptr<double>();
        rd.rays = rays.const_data_ptr<double>();
        rd.start = (const int32_t*)dptr(s_st);

        B.n = n;
        B.rays = rays;
        rays.reset();
        B.ray_id = ray_id;
        B.rshape = rshape;
        return build_tail(guard, B, nbins, n_cols, c, stream, on_dev);
    } catch (const LibError& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what.c_str());
    } catch (const std::exception& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    return nullptr;
}


// _trace_csr's one-pass trace and _index's staged table build over a ray batch (the device
// sequence both constructions share).  Throws LibError; None: a branch the Python path handles.
PyObject* build_tail(PlanGuard& guard, Batch& B, const int64_t* nbins, int64_t n_cols,
                     sphrt_csr* c, hipStream_t stream, const at::TensorOptions& on_dev) {
    const int64_t n = B.n;
    // _trace_csr, one pass: bound -> scan -> [sync] -> emit -> scan -> [sync]
    at::Tensor counts = at::empty({std::max<int64_t>(n, 1)}, on_dev.dtype(at::kInt));
    at::Tensor row_ptr = at::empty({n + 1}, on_dev.dtype(at::kLong));
    at::Tensor ws = at::empty({(int64_t)g_lib.scan_workspace_bytes(n)}, on_dev.dtype(at::kByte));
    at::Tensor tws = at::empty({(int64_t)g_lib.trace_workspace_bytes(guard.p, n)},
                               on_dev.dtype(at::kByte));
    at::Tensor bound_ptr = at::empty({n + 1}, on_dev.dtype(at::kLong));
    check(g_lib.trace_bound(guard.p, &B.rd, counts.data_ptr<int32_t>(), tws.data_ptr(),
                            (size_t)tws.numel(), stream), "sphrt_trace_bound");
    check(g_lib.scan_counts(counts.data_ptr<int32_t>(), n, bound_ptr.data_ptr<int64_t>(),
                            ws.data_ptr(), stream), "sphrt_scan_counts");
    at::Tensor pin = at::empty({4}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    int64_t* hv = pin.mutable_data_ptr<int64_t>();
    auto hip_ok = [](hipError_t e, const char* what) {
        if (e != hipSuccess) throw LibError{std::string(what) + ": " + hipGetErrorString(e)};
    };
    hip_ok(hipMemcpyAsync(hv, bound_ptr.data_ptr<int64_t>() + n, 8, hipMemcpyDeviceToHost,
                          stream), "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(stream), "hipStreamSynchronize");
    const int64_t cap = hv[0];
    size_t free_b = 0, total_b = 0;
    hip_ok(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    if ((double)cap * kStagingSlotBytes > kGateTraceStaging * (double)free_b)   // two-pass trace
        Py_RETURN_NONE;
    at::Tensor svox = at::empty({std::max<int64_t>(cap, 1)}, on_dev.dtype(at::kInt));
    at::Tensor slen = at::empty({std::max<int64_t>(cap, 1)}, on_dev.dtype(at::kDouble));
    at::Tensor over = at::empty({1}, on_dev.dtype(at::kLong));
    check(g_lib.trace_emit(guard.p, &B.rd, bound_ptr.data_ptr<int64_t>(), counts.data_ptr<int32_t>(),
                           svox.data_ptr<int32_t>(), slen.data_ptr<double>(),
                           over.data_ptr<int64_t>(), tws.data_ptr(), (size_t)tws.numel(),
                           stream), "sphrt_trace_emit");
    check(g_lib.scan_counts(counts.data_ptr<int32_t>(), n, row_ptr.data_ptr<int64_t>(),
                            ws.data_ptr(), stream), "sphrt_scan_counts");
    hip_ok(hipMemcpyAsync(hv, row_ptr.data_ptr<int64_t>() + n, 8, hipMemcpyDeviceToHost,
                          stream), "hipMemcpyAsync");
    hip_ok(hipMemcpyAsync(hv + 1, over.data_ptr<int64_t>(), 8, hipMemcpyDeviceToHost, stream),
           "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(stream), "hipStreamSynchronize");
    const int64_t total = hv[0], n_over = hv[1];
    g_lib.plan_destroy(guard.p);    // (the trace has run: the plan is not needed again)
    guard.p = nullptr;
    if (n_over != 0) Py_RETURN_NONE;   // a ray over its bound: the Python path's fill pass
    tws.reset();
    counts.reset();
    over.reset();
    ws.reset();
    B.rays.reset();                 // trace input only

    // Operator._index, staged: blocks, brick staging, table width, memory gates
    const int64_t nblocks = g_lib.csr_blocks(total);
    *c = sphrt_csr{};
    c->n_rays = n;
    c->n_segments = total;
    c->n_blocks = nblocks;
    c->n_cols = n_cols;
    if (nblocks > kSingleWaveBlocks && 4 * n_cols > kL2Bytes) {   // _stage_brick, _set_stage
        int64_t cols = 1;
        for (int i = 0; i < 3; ++i) cols *= (nbins[i] + kBrick[i] - 1) / kBrick[i] * kBrick[i];
        if (cols < (int64_t(1) << 31) - 1) {
            for (int i = 0; i < 3; ++i) {
                c->stage_shape[i] = (int32_t)nbins[i];
                c->stage_brick[i] = kBrick[i];
            }
            c->stage_cols = cols;
        }
    }
    hip_ok(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    const int64_t cols = c->stage_shape[0] > 0 ? c->stage_cols : c->n_cols;   // _tables_one_pass
    c->tab_bytes = (cols + 3) / 4 <= 65536 ? 2 : 4;
    const double wide_bytes = (double)nblocks * kTabWide * (double)c->tab_bytes;
    const double need = kStagedSegBytes * (double)seg_alloc(total) + wide_bytes;  // _staged_fits
    if (!(wide_bytes <= kGateWideTables * (double)free_b) || !(need <= kGateStaged * (double)free_b))
        Py_RETURN_NONE;                          // compaction first: the Python path
    at::Tensor vox = at::empty({seg_alloc(total)}, on_dev.dtype(at::kInt));
    at::Tensor row_ray = at::empty({std::max<int64_t>(n, 1)}, on_dev.dtype(at::kInt));
    at::Tensor empty_ray = at::empty({n + 1}, on_dev.dtype(at::kInt));
    at::Tensor blocks = at::empty({kBlockFields * nblocks}, on_dev.dtype(at::kLong));
    at::Tensor nz_row = at::empty({std::max<int64_t>(n, 1)}, on_dev.dtype(at::kInt));
    {
        at::Tensor iws = at::empty({(int64_t)g_lib.csr_index_workspace_bytes(n)},
                                   on_dev.dtype(at::kByte));
        check(g_lib.csr_index_staged(row_ptr.data_ptr<int64_t>(), n, row_ray.data_ptr<int32_t>(),
                                     empty_ray.data_ptr<int32_t>(), blocks.data_ptr<int64_t>(),
                                     nblocks,
                                     B.ray_id.defined() ? B.ray_id.data_ptr<int32_t>() : nullptr,
                                     nz_row.data_ptr<int32_t>(), iws.data_ptr(), stream),
              "sphrt_csr_index_staged");
    }
    at::Tensor len32 = at::empty({seg_alloc(total)}, on_dev.dtype(at::kFloat));
    c->row_ptr = row_ptr.data_ptr<int64_t>();
    c->vox = vox.data_ptr<int32_t>();
    c->len = nullptr;
    c->len32 = len32.data_ptr<float>();
    c->row_ray = row_ray.data_ptr<int32_t>();
    c->blocks = blocks.data_ptr<int64_t>();
    c->empty_ray = empty_ray.data_ptr<int32_t>();

    // _local_tables, staged: run records, one-pass tables moved out of the staging, pack
    at::Tensor stats = at::empty({3}, on_dev.dtype(at::kLong));
    at::Tensor runs;
    if (nblocks > kSingleWaveBlocks && n < (int64_t(1) << 31)) {
        runs = at::empty({kRunFields * nblocks}, on_dev.dtype(at::kInt));
        check(g_lib.csr_runs(c, runs.data_ptr<int32_t>(), stats.data_ptr<int64_t>() + 2, stream),
              "sphrt_csr_runs");
    } else {
        stats.narrow(0, 2, 1).fill_(1);
    }
    at::Tensor loc = at::empty({seg_alloc(total)}, on_dev.dtype(at::kShort));
    const at::ScalarType tdt = c->tab_bytes == 2 ? at::kShort : at::kInt;
    at::Tensor wide = at::empty({nblocks * kTabWide}, on_dev.dtype(tdt));
    check(g_lib.csr_local_build_staged(c, blocks.data_ptr<int64_t>(),
                                       (uint16_t*)loc.data_ptr(), wide.data_ptr(),
                                       stats.data_ptr<int64_t>(), bound_ptr.data_ptr<int64_t>(),
                                       nz_row.data_ptr<int32_t>(), svox.data_ptr<int32_t>(),
                                       slen.data_ptr<double>(), stream),
          "sphrt_csr_local_build_staged");
    hip_ok(hipMemcpyAsync(hv, stats.data_ptr<int64_t>(), 24, hipMemcpyDeviceToHost, stream),
           "hipMemcpyAsync");
    hip_ok(hipStreamSynchronize(stream), "hipStreamSynchronize");
    const int64_t n_fallback = hv[0], max_tab = hv[1], runs_over = hv[2];
    if (runs_over) runs.reset();
    const int64_t stride = std::max<int64_t>(64, (max_tab + 63) / 64 * 64);
    at::Tensor tab = at::empty({nblocks * stride + 3 * 256}, on_dev.dtype(tdt));
    check(g_lib.csr_local_pack(c, blocks.data_ptr<int64_t>(), wide.data_ptr(), tab.data_ptr(),
                               stride, stream), "sphrt_csr_local_pack");
    wide.reset();
    svox.reset();
    nz_row.reset();
    c->n_fallback = n_fallback;
    c->tab_stride = stride;
    c->loc = (uint16_t*)loc.data_ptr();
    c->tab = tab.data_ptr();
    c->runs = runs.defined() ? runs.data_ptr<int32_t>() : nullptr;

    PyObject* shape_t = PyTuple_New((Py_ssize_t)B.rshape.size());
    for (size_t i = 0; i < B.rshape.size(); ++i)
        PyTuple_SET_ITEM(shape_t, i, PyLong_FromLongLong(B.rshape[i]));
    return Py_BuildValue("(NNNNNNNNNNNNNLLN)", wrap(row_ptr), wrap(vox), wrap(len32),
                         wrap(row_ray), wrap(empty_ray), wrap(blocks), wrap(loc), wrap(tab),
                         wrap(runs), wrap(B.ray_id), wrap(bound_ptr), wrap(slen),
                         wrap(B.xs_keep), (long long)total, (long long)nblocks, shape_t);
}

// build_rays(xs, rays, r_b, e_b, a_b, nr, ne, na, n_cols, csr_address) -> as build_cone | None:
// the same construction for any other geometry (ParallelGeom, an arbitrary ViewGeom, their
// collections) from its float64 host starts and directions (geom.ray_starts / geom.rays,
// broadcast against each other, raytracer.py:76-80): the starts, their voxels, the rays and the
// plan tables in one host-to-device copy, then build_cone's device sequence.  Geometry order
// (the trace orders are for cone detectors): no ray ids.
PyObject* construct_build_rays(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 10 || !g_bound) {
        PyErr_SetString(PyExc_TypeError, "build_rays(xs, rays, r_b, e_b, a_b, nr, ne, na, n_cols, "
                                         "csr_address) after bind");
        return nullptr;
    }
    int64_t nbins[3];
    for (int k = 0; k < 3; ++k) {
        nbins[k] = PyLong_AsLongLong(args[5 + k]);
        if (nbins[k] == -1 && PyErr_Occurred()) return nullptr;
    }
    const int64_t n_cols = PyLong_AsLongLong(args[8]);
    auto* c = static_cast<sphrt_csr*>(PyLong_AsVoidPtr(args[9]));
    if (PyErr_Occurred()) return nullptr;
    if (!THPVariable_Check(args[0]) || !THPVariable_Check(args[1])) Py_RETURN_NONE;
    PlanGuard guard;
    try {
        const at::Tensor xs_in = THPVariable_Unpack(args[0]), ry_in = THPVariable_Unpack(args[1]);
        if (!xs_in.device().is_cpu() || !ry_in.device().is_cpu() ||
            xs_in.scalar_type() != at::kDouble || ry_in.scalar_type() != at::kDouble ||
            xs_in.dim() < 1 || ry_in.dim() < 1 || xs_in.size(-1) != 3 || ry_in.size(-1) != 3)
            Py_RETURN_NONE;
        std::vector<int64_t> full;
        try {
            full = at::infer_size(xs_in.sizes(), ry_in.sizes());
        } catch (const std::exception&) {
            Py_RETURN_NONE;                          // (the Python path raises the error)
        }
        std::vector<int64_t> bshape(full.begin(), full.end() - 1);
        int64_t n = 1;
        for (int64_t v : bshape) n *= v;
        if (bshape.empty() || (int64_t)bshape.size() > SPHRT_MAX_DIMS || n <= 0) Py_RETURN_NONE;
        Prelude P;
        P.xs = xs_in.contiguous();
        if (!grid_prelude(args + 2, nbins, P)) {
            if (PyErr_Occurred()) return nullptr;
            Py_RETURN_NONE;
        }
        const at::Tensor ry_h = ry_in.contiguous();
        const int dev = (int)c10::hip::current_device();
        hipStream_t stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
        const at::TensorOptions on_dev = at::TensorOptions().device(at::kCUDA, dev);
        const int64_t tbytes = (int64_t)g_lib.plan_table_bytes(&P.desc);
        at::Tensor tables = at::empty({tbytes}, at::kByte);
        check(g_lib.plan_pack_tables(&P.desc, tables.mutable_data_ptr()), "sphrt_plan_pack_tables");
        Slots S;
        const int s_tab = S.add(tables.const_data_ptr(), tbytes);
        const int s_xs = S.add(P.xs.const_data_ptr(), nbytes(P.xs));
        const int s_st = S.add(P.st.const_data_ptr(), nbytes(P.st));
        const int s_ry = S.add(ry_h.const_data_ptr(), nbytes(ry_h));
        at::Tensor host = at::empty({S.size}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
        S.write(host.mutable_data_ptr<uint8_t>());
        const at::Tensor staged = host.to(on_dev.dtype(at::kByte), /*non_blocking=*/true);
        auto dptr = [&](int slot) { return (uint8_t*)staged.data_ptr() + S.offs[slot]; };
        check(g_lib.plan_create_external(&P.desc, dev, dptr(s_tab), &guard.p),
              "sphrt_plan_create_external");
        Batch B;
        B.xs_keep = staged.narrow(0, S.offs[s_xs], nbytes(P.xs)).view(at::kDouble).view(P.xs.sizes());
        const at::Tensor rays = staged.narrow(0, S.offs[s_ry], nbytes(ry_h)).view(at::kDouble)
                                    .view(ry_h.sizes());
        const std::vector<int64_t> xs_str = B.xs_keep.expand(full).strides().vec();
        const std::vector<int64_t> ry_str = rays.expand(full).strides().vec();
        B.rd.ndim = (int32_t)bshape.size();
        for (size_t i = 0; i < bshape.size(); ++i) {
            B.rd.shape[i] = bshape[i];
            B.rd.xs_stride[i] = xs_str[i];
            B.rd.rays_stride[i] = ry_str[i];
        }
        B.rd.xs = B.xs_keep.const_data_ptr<double>();
        B.rd.rays = rays.const_data_ptr<double>();
        B.rd.start = (const int32_t*)dptr(s_st);
        B.n = n;
        B.rshape = bshape;
        return build_tail(guard, B, nbins, n_cols, c, stream, on_dev);
    } catch (const LibError& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what.c_str());
    } catch (const std::exception& e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    return nullptr;
}

}  // namespace sphrt_fast
