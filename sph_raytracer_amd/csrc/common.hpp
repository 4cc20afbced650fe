// common.hpp — plan object, ray-batch descriptor and error plumbing shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "sphrt.h"
#include "solve.hpp"

struct sphrt_plan {
    int device;
    sphrt::GridDev dev;   // device pointers below
    void* table_mem;      // one hipMalloc holding every boundary table
};

namespace sphrt {

constexpr int kMaxDims = SPHRT_MAX_DIMS;

struct RaysDev {
    int ndim;
    int64_t n;
    int64_t shape[kMaxDims];
    int64_t xs_stride[kMaxDims];
    int64_t rays_stride[kMaxDims];
    const double* xs;
    const double* rays;
    const int32_t* start;
    int fresh;    // reference-mode trace: each solver normalises its own copy (exact_list)
};

int fail(const char* fmt, ...);   // records the message, returns -1
int check_launch(const char* what);

// Makes `dev` the calling thread's current HIP device for the scope (restored afterwards).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        int cur = -1;
        if (dev < 0 || hipGetDevice(&cur) != hipSuccess || cur == dev) return;
        if (hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Device a stream belongs to (the current device for the null stream), -1 on error.
inline int stream_device(void* stream) {
    int dev = -1;
    if (stream == nullptr) return hipGetDevice(&dev) == hipSuccess ? dev : -1;
    hipDevice_t d;
    return hipStreamGetDevice((hipStream_t)stream, &d) == hipSuccess ? (int)d : -1;
}

// Every launching entry point runs on its stream's device, whatever device is current in the
// calling thread (the caller's buffers live on that device too).
struct StreamGuard {
    DeviceGuard g;
    explicit StreamGuard(void* stream) : g(stream_device(stream)) {}
};

// Validate plan + batch and convert to the by-value kernel argument forms.
inline int resolve(const sphrt_plan* plan, const sphrt_rays* rays, GridDev& G, RaysDev& R,
                   void* stream) {
    if (!plan) return fail("null plan");
    const int sdev = stream_device(stream);
    if (sdev != plan->device)
        return fail("stream is on device %d but the plan's tables are on device %d", sdev,
                    plan->device);
    if (!rays) return fail("null ray batch");
    if (rays->ndim < 0 || rays->ndim > kMaxDims) return fail("ray batch rank %d out of range", rays->ndim);
    if (!rays->xs || !rays->rays || !rays->start) return fail("null ray batch pointer");
    G = plan->dev;
    R.ndim = rays->ndim;
    R.n = 1;
    for (int d = 0; d < kMaxDims; ++d) {
        R.shape[d] = d < rays->ndim ? rays->shape[d] : 1;
        R.xs_stride[d] = d < rays->ndim ? rays->xs_stride[d] : 0;
        R.rays_stride[d] = d < rays->ndim ? rays->rays_stride[d] : 0;
        if (d < rays->ndim) {
            if (rays->shape[d] < 0) return fail("negative ray-batch extent");
            R.n *= rays->shape[d];
        }
    }
    R.xs = rays->xs;
    R.rays = rays->rays;
    R.start = rays->start;
    R.fresh = 0;
    return 0;
}

}  // namespace sphrt
