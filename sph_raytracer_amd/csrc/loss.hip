// loss.hip — the elementwise tails of the static_retrieval.py loop (retrieval._gd_direct), fused.
//
// SquareLoss (loss.py:87-110 of the reference: lam * mean((y - f(d))^2)) and NegRegularizer
// (loss.py:140-162: lam * mean(|clamp(d, max=0)|)) need, per iteration, the residual, its scaled
// copy (the adjoint's input) and its mean square (the loss value) and, for the regulariser, the
// mean absolute negative part and -lam/N on the gradient of every negative voxel.  Through torch
// that is ~9 elementwise launches plus two mean reductions (a memset and a reduce each) of
// 5-9 us on a 64^3 problem; here it is two launches, each leaving its workgroups' partial sums
// of the loss (summed for every iteration at once after the loop).
//
// The elementwise values are single IEEE operations, the ones torch's elementwise ops give (the
// library is built with -ffp-contract=off), so the gradient and hence the iterates stay bitwise
// those of the autograd loop.  The means are deterministic (fixed per-thread strides, a fixed
// reduction tree, the partials summed in a fixed order) but their order differs from
// torch.mean's: loss values agree with it to rounding (~1e-16).
#include "common.hpp"

namespace sphrt {

constexpr int kLossThreads = 256;
constexpr int kLossMaxBlocks = 256;

// Workgroup sum in a fixed order (wave shuffles, then the four wave totals in order); thread 0
// stores it.  No cross-workgroup step: the partials of every iteration are summed after the loop
// (deterministic; a last-workgroup reduction would need an agent-scope release per workgroup,
// i.e. an L2 write-back on a chip of eight L2s: +6 us per launch at C5).
__device__ __forceinline__ void block_partial(double v, double* out) {
    __shared__ double sh[kLossThreads / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < kLossThreads / 64; ++i) s += sh[i];
        out[blockIdx.x] = s;
    }
}

// r = yhat - y (y float32 or float64, promoted exactly); r_scaled = r * scale; partial sums of
// r * r.
template <typename TY>
__global__ __launch_bounds__(kLossThreads) void sq_residual_kernel(
    const double* __restrict__ yhat, const TY* __restrict__ y, int64_t n, double scale,
    double* __restrict__ r_scaled, double* __restrict__ part) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kLossThreads) {
        const double r = yhat[i] - (double)y[i];
        r_scaled[i] = r * scale;
        acc += r * r;
    }
    block_partial(acc, part);
}

// g -= c_neg where d < 0 (g.sub_(d.lt(0), alpha=c): g - c * 0 is g itself, signed zeros
// included); partial sums of |clamp(d, max=0)| (NaN stays NaN).
__global__ __launch_bounds__(kLossThreads) void neg_reg_kernel(
    const double* __restrict__ d, int64_t n, double c_neg, double* __restrict__ g,
    double* __restrict__ part) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kLossThreads) {
        const double v = d[i];
        const double c = v > 0.0 ? 0.0 : v;                // clamp(max=0): NaN and -0 pass
        acc += __builtin_fabs(c);
        if (v < 0.0) g[i] = g[i] - c_neg;
    }
    block_partial(acc, part);
}

static unsigned loss_grid(int64_t n) {
    const int64_t b = (n + kLossThreads - 1) / kLossThreads;
    return (unsigned)(b < kLossMaxBlocks ? (b > 0 ? b : 1) : kLossMaxBlocks);
}

}  // namespace sphrt

using namespace sphrt;

extern "C" int64_t sphrt_loss_partials(int64_t n) { return n > 0 ? (int64_t)loss_grid(n) : 0; }

extern "C" int sphrt_sq_residual_f64(const double* yhat, const void* y, int y_is_f64, int64_t n,
                                     double scale, double* r_scaled, double* partial_sums,
                                     void* stream) {
    if (n <= 0) return fail("sphrt_sq_residual_f64: empty measurement");
    if (!yhat || !y || !r_scaled || !partial_sums) return fail("null buffer");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL(sq_residual_kernel<double>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const double*)y, n, scale, r_scaled, partial_sums);
    else
        hipLaunchKernelGGL(sq_residual_kernel<float>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const float*)y, n, scale, r_scaled, partial_sums);
    return check_launch("sq_residual");
}

extern "C" int sphrt_neg_reg_f64(const double* d, int64_t n, double c_neg, double* g,
                                 double* partial_sums, void* stream) {
    if (n <= 0) return fail("sphrt_neg_reg_f64: empty volume");
    if (!d || !g || !partial_sums) return fail("null buffer");
    StreamGuard guard(stream);
    hipLaunchKernelGGL(neg_reg_kernel, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                       (hipStream_t)stream, d, n, c_neg, g, partial_sums);
    return check_launch("neg_reg");
}
