// loss.hip — the elementwise tails of the static_retrieval.py loop (retrieval._gd_direct), fused.
//
// SquareLoss (loss.py:87-110 of the reference: lam * mean((y - f(d))^2)) and NegRegularizer
// (loss.py:140-162: lam * mean(|clamp(d, max=0)|)) need, per iteration, the residual, its scaled
// copy (the adjoint's input) and its mean square (the loss value) and, for the regulariser, the
// mean absolute negative part and -lam/N on the gradient of every negative voxel.  Through torch
// that is ~9 elementwise launches plus two mean reductions (a memset and a reduce each) of
// 5-9 us on a 64^3 problem; here it is two launches, each ending in its own mean.
//
// The elementwise values are single IEEE operations, the ones torch's elementwise ops give (the
// library is built with -ffp-contract=off), so the gradient and hence the iterates stay bitwise
// those of the autograd loop.  The means are deterministic (fixed per-thread strides, a fixed
// reduction tree, the block partials summed in block order by the last block to finish) but
// their order differs from torch.mean's: loss values agree with it to rounding (~1e-16).
#include <stdlib.h>

#include "common.hpp"

namespace sphrt {

constexpr int kLossThreads = 256;
constexpr int kLossMaxBlocks = 2048;    // partials per mean (sphrt_loss_workspace)

__device__ __forceinline__ double block_sum(double v, double* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kLossThreads / 64; ++i) s += sh[i];
    __syncthreads();
    return s;   // thread 0 only
}

// Block partial -> part[blockIdx]; the last block to finish sums the partials in block order and
// writes sum / n to *mean, then re-arms the counter for the next launch.
__device__ void finish_mean(double v, double* part, unsigned* count, double* mean, int64_t n) {
    __shared__ double sh[kLossThreads / 64];
    __shared__ bool last;
    const double s = block_sum(v, sh);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s;
        __threadfence();                                   // publish the partial (agent scope)
        last = atomicAdd(count, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();                                       // every partial is visible
    double acc = 0.0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += kLossThreads)
        acc += part[i];
    const double tot = block_sum(acc, sh);
    if (threadIdx.x == 0) {
        *mean = tot / (double)n;
        atomicExch(count, 0u);
    }
}

// r = yhat - y (y float32 or float64, promoted exactly); r_scaled = r * scale; mean of r * r.
template <typename TY>
__global__ __launch_bounds__(kLossThreads) void sq_residual_kernel(
    const double* __restrict__ yhat, const TY* __restrict__ y, int64_t n, double scale,
    double* __restrict__ r_scaled, double* part, unsigned* count, double* mean) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kLossThreads) {
        const double r = yhat[i] - (double)y[i];
        r_scaled[i] = r * scale;
        acc += r * r;
    }
    finish_mean(acc, part, count, mean, n);
}

// g -= c_neg where d < 0 (g.sub_(d.lt(0), alpha=c): g - c * 0 is g itself, signed zeros
// included); mean of |clamp(d, max=0)| (NaN stays NaN).
__global__ __launch_bounds__(kLossThreads) void neg_reg_kernel(
    const double* __restrict__ d, int64_t n, double c_neg, double* __restrict__ g, double* part,
    unsigned* count, double* mean) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kLossThreads) {
        const double v = d[i];
        const double c = v > 0.0 ? 0.0 : v;                // clamp(max=0): NaN and -0 pass
        acc += __builtin_fabs(c);
        if (v < 0.0) g[i] = g[i] - c_neg;
    }
    finish_mean(acc, part, count, mean, n);
}

// At most 256 workgroups: every workgroup's release fence writes back its XCD's L2 (agent scope on
// a chip of eight L2s), so fewer, longer workgroups win (C5 iteration with 2048 / 512 / 256 / 128
// / 64 / 16 workgroups: 0.229 / 0.202 / 0.192 / 0.193 / 0.199 / 0.253 ms).  SPHRT_LOSS_BLOCKS
// overrides it (A/B studies).
static unsigned loss_grid(int64_t n) {
    static const int64_t cap = [] {
        const char* e = getenv("SPHRT_LOSS_BLOCKS");
        const long v = e ? atol(e) : 256;
        return (int64_t)(v > 0 && v <= kLossMaxBlocks ? v : 256);
    }();
    const int64_t b = (n + kLossThreads - 1) / kLossThreads;
    return (unsigned)(b < cap ? (b > 0 ? b : 1) : cap);
}

struct LossWs {
    double* part;
    unsigned* count;
};
static int loss_ws(void* ws, size_t bytes, LossWs& w) {
    if (!ws || bytes < (size_t)kLossMaxBlocks * sizeof(double) + 64)
        return fail("loss workspace too small (sphrt_loss_workspace_bytes)");
    w.part = (double*)ws;
    w.count = (unsigned*)((char*)ws + (size_t)kLossMaxBlocks * sizeof(double));
    return 0;
}

}  // namespace sphrt

using namespace sphrt;

extern "C" size_t sphrt_loss_workspace_bytes(void) {
    return (size_t)kLossMaxBlocks * sizeof(double) + 64;
}

extern "C" int sphrt_sq_residual_f64(const double* yhat, const void* y, int y_is_f64, int64_t n,
                                     double scale, double* r_scaled, double* mean, void* workspace,
                                     size_t workspace_size, void* stream) {
    if (n <= 0) return fail("sphrt_sq_residual_f64: empty measurement");
    if (!yhat || !y || !r_scaled || !mean) return fail("null buffer");
    LossWs w;
    if (int e = loss_ws(workspace, workspace_size, w)) return e;
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL(sq_residual_kernel<double>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const double*)y, n, scale, r_scaled, w.part, w.count, mean);
    else
        hipLaunchKernelGGL(sq_residual_kernel<float>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const float*)y, n, scale, r_scaled, w.part, w.count, mean);
    return check_launch("sq_residual");
}

extern "C" int sphrt_neg_reg_f64(const double* d, int64_t n, double c_neg, double* g,
                                 double* mean, void* workspace, size_t workspace_size,
                                 void* stream) {
    if (n <= 0) return fail("sphrt_neg_reg_f64: empty volume");
    if (!d || !g || !mean) return fail("null buffer");
    LossWs w;
    if (int e = loss_ws(workspace, workspace_size, w)) return e;
    StreamGuard guard(stream);
    hipLaunchKernelGGL(neg_reg_kernel, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                       (hipStream_t)stream, d, n, c_neg, g, w.part, w.count, mean);
    return check_launch("neg_reg");
}
