// fastpath.cpp — CPython entry for the steady-state Operator.__call__ (raytracer.py:692-713).
//
// Host code only (no kernels): the product compute path stays libsphrt.so behind its C ABI
// (include/sphrt.h).  A steady-state forward call from Python — a contiguous density already on
// the GPU, in a shape/dtype seen before, no autograd — costs one C call here instead of ~3 us of
// Python around ctypes: match the density against the operator's bindings, allocate the output
// with torch's caching allocator on the density's device, launch on the current HIP stream via
// the bound sphrt_forward_* entry point, return the tensor.  Anything else returns None and
// Operator.__call__ takes its general path.
#include <Python.h>

#include <ATen/ATen.h>
#include <ATen/core/grad_mode.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <string>
#include <vector>

#include "sphrt.h"

namespace {

using ForwardFn = int (*)(const void* csr, const void* density, int64_t n_chan, int64_t chan_stride,
                          int64_t div, void* out, int64_t ocs, void* stream);
using LastErrorFn = const char* (*)();
using GatherFn = int (*)(const void* src, const int32_t* idx, int64_t n, void* dst, void* stream);

struct Binding {
    std::vector<int64_t> in_sizes;   // density shape this binding serves
    at::ScalarType dtype;
    int device;
    ForwardFn fn;
    const void* csr;
    int64_t n_chan, n_vox, div, n;
    std::vector<int64_t> out_shape;  // the call's result shape (contiguous, n_chan * n or n)
    int64_t stage_bytes;             // > 0: brick-staged CSR, a stage buffer of this size per call
    at::Tensor perm;                 // defined: the input is read as input.view(-1)[perm] (the
                                     // adjoint of a trace in another ray order: y in trace order)
    GatherFn gather = nullptr;       // sphrt_gather_f32/_f64 for perm (else index_select)
};

struct Bindings {
    std::vector<Binding> list;
    LastErrorFn last_error = nullptr;
};

constexpr const char* kCapsule = "sph_raytracer_amd.fastpath";

void destroy(PyObject* cap) {
    delete static_cast<Bindings*>(PyCapsule_GetPointer(cap, kCapsule));
}

bool int_tuple(PyObject* o, std::vector<int64_t>& out) {
    PyObject* seq = PySequence_Fast(o, "expected a sequence of ints");
    if (!seq) return false;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    out.resize(n);
    for (Py_ssize_t i = 0; i < n; ++i) {
        out[i] = PyLong_AsLongLong(PySequence_Fast_GET_ITEM(seq, i));
        if (out[i] == -1 && PyErr_Occurred()) {
            Py_DECREF(seq);
            return false;
        }
    }
    Py_DECREF(seq);
    return true;
}

// new(last_error_fn_address) -> capsule
PyObject* py_new(PyObject*, PyObject* arg) {
    auto* b = new Bindings();
    b->last_error = reinterpret_cast<LastErrorFn>(PyLong_AsVoidPtr(arg));
    if (PyErr_Occurred()) {
        delete b;
        return nullptr;
    }
    return PyCapsule_New(b, kCapsule, destroy);
}

// add(capsule, in_sizes, is_f64, device, fn_address, csr_address, n_chan, n_vox, div, n, out_shape,
//     stage_bytes[, perm[, gather_address]])
PyObject* py_add(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs < 12 || nargs > 14) {
        PyErr_SetString(PyExc_TypeError, "add() takes 12 to 14 arguments");
        return nullptr;
    }
    auto* b = static_cast<Bindings*>(PyCapsule_GetPointer(args[0], kCapsule));
    if (!b) return nullptr;
    Binding x;
    if (!int_tuple(args[1], x.in_sizes)) return nullptr;
    x.dtype = PyObject_IsTrue(args[2]) ? at::kDouble : at::kFloat;
    x.device = (int)PyLong_AsLong(args[3]);
    x.fn = reinterpret_cast<ForwardFn>(PyLong_AsVoidPtr(args[4]));
    x.csr = PyLong_AsVoidPtr(args[5]);
    x.n_chan = PyLong_AsLongLong(args[6]);
    x.n_vox = PyLong_AsLongLong(args[7]);
    x.div = PyLong_AsLongLong(args[8]);
    x.n = PyLong_AsLongLong(args[9]);
    if (PyErr_Occurred() || !int_tuple(args[10], x.out_shape)) return nullptr;
    x.stage_bytes = PyLong_AsLongLong(args[11]);
    if (PyErr_Occurred()) return nullptr;
    if (nargs >= 13 && args[12] != Py_None) {
        if (!THPVariable_Check(args[12])) {
            PyErr_SetString(PyExc_TypeError, "perm: a device index tensor or None");
            return nullptr;
        }
        x.perm = THPVariable_Unpack(args[12]);
        if (nargs == 14 && args[13] != Py_None) {
            x.gather = reinterpret_cast<GatherFn>(PyLong_AsVoidPtr(args[13]));
            if (PyErr_Occurred()) return nullptr;
            if (x.perm.scalar_type() != at::kInt) {
                PyErr_SetString(PyExc_TypeError, "perm: int32 for the gather entry point");
                return nullptr;
            }
        }
    }
    if (!x.fn || !x.csr) {
        PyErr_SetString(PyExc_ValueError, "null forward entry point or CSR");
        return nullptr;
    }
    for (auto& y : b->list)
        if (y.in_sizes == x.in_sizes && y.dtype == x.dtype && y.device == x.device) {
            y = x;
            Py_RETURN_NONE;
        }
    b->list.push_back(std::move(x));
    Py_RETURN_NONE;
}

constexpr int64_t kAlternateMinBlocks = 256 * 6;   // raytracer._ALTERNATE_MIN_BLOCKS

// forward(capsule, density) -> Tensor, or None when no binding applies
PyObject* py_forward(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 2) {
        PyErr_SetString(PyExc_TypeError, "forward() takes 2 arguments");
        return nullptr;
    }
    auto* b = static_cast<Bindings*>(PyCapsule_GetPointer(args[0], kCapsule));
    if (!b) return nullptr;
    PyObject* obj = args[1];
    if (!THPVariable_CheckExact(obj)) Py_RETURN_NONE;
    const at::Tensor& d = THPVariable_Unpack(obj);
    if (!d.is_cuda() || !d.is_contiguous()) Py_RETURN_NONE;
    if (d.requires_grad() && at::GradMode::is_enabled()) Py_RETURN_NONE;
    const at::ScalarType dt = d.scalar_type();
    const int dev = d.get_device();
    // launches go to the current HIP device's streams: another current device takes the general
    // path (which makes the operator's device current)
    if (dev != (int)c10::hip::current_device()) Py_RETURN_NONE;
    const auto sizes = d.sizes();
    for (const Binding& x : b->list) {
        if (x.dtype != dt || x.device != dev || !sizes.equals(x.in_sizes)) continue;
        at::Tensor out = at::empty(x.out_shape, d.options());
        void* stream = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
        at::Tensor src = d;
        if (x.perm.defined() && x.gather && d.numel() == x.perm.numel()) {
            src = at::empty({d.numel()}, d.options());
            if (x.gather(d.const_data_ptr(), x.perm.const_data_ptr<int32_t>(), d.numel(),
                         src.mutable_data_ptr(), stream) != 0) {
                const std::string msg = std::string("sphrt_gather: ") +
                                        (b->last_error ? b->last_error() : "failed");
                PyErr_SetString(PyExc_RuntimeError, msg.c_str());
                return nullptr;
            }
        } else if (x.perm.defined()) {
            src = d.reshape({-1}).index_select(0, x.perm);
        }
        const void* csr = x.csr;
        sphrt_csr staged;
        at::Tensor stage;      // this call's brick stage (caching allocator, current stream)
        if (x.stage_bytes > 0) {
            stage = at::empty({x.stage_bytes}, d.options().dtype(at::kByte));
            staged = *static_cast<const sphrt_csr*>(x.csr);
            staged.stage = stage.mutable_data_ptr();
            staged.stage_bytes = x.stage_bytes;
            csr = &staged;
        }
        const int rc = x.fn(csr, src.const_data_ptr(), x.n_chan, x.n_vox, x.div,
                            out.mutable_data_ptr(), x.n, stream);
        // multi-wave CSRs alternate their block order from call to call (raytracer._alternate)
        if (rc == 0) {
            auto* c = static_cast<sphrt_csr*>(const_cast<void*>(x.csr));
            if (c->n_blocks > kAlternateMinBlocks) c->order ^= 1;
        }
        if (rc != 0) {
            const std::string msg = std::string("sphrt_forward: ") +
                                    (b->last_error ? b->last_error() : "failed");
            PyErr_SetString(PyExc_RuntimeError, msg.c_str());
            return nullptr;
        }
        return THPVariable_Wrap(std::move(out));
    }
    Py_RETURN_NONE;
}

}  // namespace

namespace sphrt_fast {   // csrc/construct.cpp
PyObject* construct_bind(PyObject*, PyObject* const*, Py_ssize_t);
PyObject* construct_cone_host(PyObject*, PyObject* const*, Py_ssize_t);
PyObject* construct_build_cone(PyObject*, PyObject* const*, Py_ssize_t);
PyObject* construct_build_rays(PyObject*, PyObject* const*, Py_ssize_t);
}  // namespace sphrt_fast

namespace {

PyMethodDef methods[] = {
    {"new", (PyCFunction)py_new, METH_O, "new(last_error_address) -> bindings"},
    {"add", (PyCFunction)(void (*)(void))py_add, METH_FASTCALL, "bind a density shape"},
    {"forward", (PyCFunction)(void (*)(void))py_forward, METH_FASTCALL,
     "forward(bindings, density) -> Tensor | None"},
    {"construct_bind", (PyCFunction)(void (*)(void))sphrt_fast::construct_bind, METH_FASTCALL,
     "construct_bind(lib_path, ConeRectGeom, ConeCircGeom, ViewGeomCollection)"},
    {"cone_host", (PyCFunction)(void (*)(void))sphrt_fast::construct_cone_host, METH_FASTCALL,
     "cone_host(geom, r_b, e_b, a_b, nr, ne, na) -> host values of the trace | None"},
    {"build_cone", (PyCFunction)(void (*)(void))sphrt_fast::construct_build_cone, METH_FASTCALL,
     "build_cone(geom, r_b, e_b, a_b, nr, ne, na, perm, n_cols, csr_address) -> CSR | None"},
    {"build_rays", (PyCFunction)(void (*)(void))sphrt_fast::construct_build_rays, METH_FASTCALL,
     "build_rays(xs, rays, r_b, e_b, a_b, nr, ne, na, n_cols, csr_address) -> CSR | None"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_sphrt_fast", nullptr, -1, methods};

}  // namespace

#ifndef SPHRT_SOURCE_HASH
#define SPHRT_SOURCE_HASH "unhashed"
#endif

// the tree this entry was built from (build.source_hash(); checked by _lib.load_fast)
PyMODINIT_FUNC PyInit__sphrt_fast() {
    PyObject* m = PyModule_Create(&module);
    if (m && PyModule_AddStringConstant(m, "version",
                                        "sph_raytracer_amd fastpath src " SPHRT_SOURCE_HASH) < 0) {
        Py_DECREF(m);
        return nullptr;
    }
    return m;
}
