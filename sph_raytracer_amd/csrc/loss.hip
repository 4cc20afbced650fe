// loss.hip — the elementwise tails of the static_retrieval.py loop (retrieval._gd_direct), fused.
//
// SquareLoss (loss.py:87-110 of the reference: lam * mean((y - f(d))^2)) and NegRegularizer
// (loss.py:140-162: lam * mean(|clamp(d, max=0)|)) need, per iteration, the residual, its square
// (for the loss value), its scaled copy (the adjoint's input) and, for the regulariser, the
// absolute negative part (the loss value) and -lam/N on the gradient of every negative voxel.
// Through torch those are ~9 elementwise launches of 5-9 us each on a 64^3 problem; here two.
// Every value is the one torch's own elementwise ops produce (single IEEE operations, no
// contraction: the library is built with -ffp-contract=off), so the loss values (torch.mean of
// the squared / absolute arrays written here) and the iterates stay bitwise those of the
// autograd loop.
#include "common.hpp"

namespace sphrt {

// r = yhat - y (y in float32 or float64, promoted exactly); r_sq = r * r; r_scaled = r * scale.
template <typename TY>
__global__ __launch_bounds__(256) void sq_residual_kernel(const double* __restrict__ yhat,
                                                          const TY* __restrict__ y, int64_t n,
                                                          double scale,
                                                          double* __restrict__ r_scaled,
                                                          double* __restrict__ r_sq) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double r = yhat[i] - (double)y[i];
        r_sq[i] = r * r;
        r_scaled[i] = r * scale;
    }
}

// abs_neg = |clamp(d, max=0)| (NaN stays NaN); g -= c_neg where d < 0 (g.sub_(d.lt(0), alpha=c):
// g - c * 0 is g itself, signed zeros included).
__global__ __launch_bounds__(256) void neg_reg_kernel(const double* __restrict__ d, int64_t n,
                                                      double c_neg, double* __restrict__ g,
                                                      double* __restrict__ abs_neg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double v = d[i];
        const double c = v > 0.0 ? 0.0 : v;          // clamp(max=0): NaN and -0 pass through
        abs_neg[i] = __builtin_fabs(c);
        if (v < 0.0) g[i] = g[i] - c_neg;
    }
}

static unsigned elem_grid(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace sphrt

using namespace sphrt;

extern "C" int sphrt_sq_residual_f64(const double* yhat, const void* y, int y_is_f64, int64_t n,
                                     double scale, double* r_scaled, double* r_sq, void* stream) {
    if (n < 0) return fail("negative length");
    if (n == 0) return 0;
    if (!yhat || !y || !r_scaled || !r_sq) return fail("null buffer");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL(sq_residual_kernel<double>, dim3(elem_grid(n)), dim3(256), 0, st, yhat,
                           (const double*)y, n, scale, r_scaled, r_sq);
    else
        hipLaunchKernelGGL(sq_residual_kernel<float>, dim3(elem_grid(n)), dim3(256), 0, st, yhat,
                           (const float*)y, n, scale, r_scaled, r_sq);
    return check_launch("sq_residual");
}

extern "C" int sphrt_neg_reg_f64(const double* d, int64_t n, double c_neg, double* g,
                                 double* abs_neg, void* stream) {
    if (n < 0) return fail("negative length");
    if (n == 0) return 0;
    if (!d || !g || !abs_neg) return fail("null buffer");
    StreamGuard guard(stream);
    hipLaunchKernelGGL(neg_reg_kernel, dim3(elem_grid(n)), dim3(256), 0, (hipStream_t)stream, d, n,
                       c_neg, g, abs_neg);
    return check_launch("neg_reg");
}
