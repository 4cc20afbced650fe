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
#include "stage.hpp"

namespace sphrt {

constexpr int kLossThreads = 256;
constexpr int kLossMaxBlocks = 1024;   // (a 64^3 volume: one element per thread)

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
// r * r.  With `order` (a trace's row -> geometry ray map), r_scaled[j] is the residual of ray
// order[j]: the transposed adjoint's input in trace order, without a separate permutation.
template <typename TY>
__global__ __launch_bounds__(kLossThreads) void sq_residual_kernel(
    const double* __restrict__ yhat, const TY* __restrict__ y, int64_t n, double scale,
    const int32_t* __restrict__ order, double* __restrict__ r_scaled, double* __restrict__ part) {
    double acc = 0.0;
    for (int64_t j = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * kLossThreads) {
        const int64_t i = order ? (int64_t)order[j] : j;
        const double r = yhat[i] - (double)y[i];
        r_scaled[j] = r * scale;
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

// Adam on float64 coefficients, with the NegRegularizer's gradient term and loss partials folded
// in: one launch where the loop made three or more (neg_reg, the step-count add, the optimiser's
// own launches).  Two arithmetics, each the per-element operation sequence of one of torch's
// implementations (amsgrad and maximize off):
//  - FOREACH = false: torch.optim.Adam(fused=True), torch._fused_adam_.  The multiply-adds are
//    the fused ones torch's ROCm build emits for `beta1 * m + (1 - beta1) * g` and
//    `beta2 * v + (1 - beta2) * g * g` (fma of the left product, and of p * weight_decay + g),
//    written out here since this library builds with -ffp-contract=off: measured bitwise equal
//    to torch._fused_adam_ over 20 steps with and without weight decay, where the unfused and the
//    right-product forms differ from step 1 (`test_adam_matches_torch_fused`).  Bias corrections
//    from the device's pow and sqrt, as torch's kernel computes them from its float32 step count.
//  - FOREACH = true: the default Adam on GPU tensors (torch.optim.adam._multi_tensor_adam, what
//    the reference's `optim(optim_vars, **kwargs)`, retrieval.py:84, runs on a CUDA/ROCm device):
//    _foreach_add(g, p, alpha=wd), _foreach_lerp_(m, g, 1 - beta1), _foreach_mul_(v, beta2),
//    _foreach_addcmul_(v, g, g, 1 - beta2), sqrt, / sqrt(1 - beta2^t), + eps,
//    _foreach_addcdiv_(p, m, denom, -lr / (1 - beta1^t)); each functor's `a + s * x` is one
//    fma in torch's ROCm build.  The bias corrections come from the host (Python floats, as
//    torch computes them): `step_size` is the negative step, `bc2s` sqrt(1 - beta2^t).
template <bool FOREACH>
__global__ __launch_bounds__(kLossThreads) void adam_neg_kernel(
    double* __restrict__ param, const double* __restrict__ grad, double* __restrict__ exp_avg,
    double* __restrict__ exp_avg_sq, int64_t n, double lr, double beta1, double beta2, double eps,
    double weight_decay, double step, double c_neg, double* __restrict__ part, StageMap sm,
    double* __restrict__ stage) {
    // the bias corrections once per workgroup (wave 0), under the first element's loads
    __shared__ double bc[2];
    const int64_t i0 = (int64_t)blockIdx.x * kLossThreads + threadIdx.x;
    const bool in0 = i0 < n;
    double p0 = 0.0, g0 = 0.0, m0 = 0.0, v0 = 0.0;
    if (in0) {
        p0 = param[i0];
        g0 = grad[i0];
        m0 = exp_avg[i0];
        v0 = exp_avg_sq[i0];
    }
    double step_size, bc2s;
    if constexpr (FOREACH) {
        step_size = lr;            // (host: -lr / (1 - beta1^t))
        bc2s = step;               // (host: sqrt(1 - beta2^t))
    } else {
        if (threadIdx.x < 64) {
            const double b1 = 1 - pow(beta1, step), b2s = sqrt(1 - pow(beta2, step));
            if (threadIdx.x == 0) {
                bc[0] = b1;
                bc[1] = b2s;
            }
        }
        __syncthreads();
        step_size = lr / bc[0];
        bc2s = bc[1];
    }
    const double ob1 = 1 - beta1, ob2 = 1 - beta2;
    double acc = 0.0;
    for (int64_t i = i0; i < n; i += (int64_t)gridDim.x * kLossThreads) {
        const bool first = i == i0;
        double p = first ? p0 : param[i], g = first ? g0 : grad[i];
        const double mo = first ? m0 : exp_avg[i], vo = first ? v0 : exp_avg_sq[i];
        if (part) {                                        // as neg_reg_kernel
            const double c = p > 0.0 ? 0.0 : p;
            acc += __builtin_fabs(c);
            if (p < 0.0) g = g - c_neg;
        }
        double m, v, pn;
        if constexpr (FOREACH) {
            if (weight_decay != 0) g = fma(weight_decay, p, g);
            // lerp(m, g, w) with w = 1 - beta1 (ATen Lerp.h: the small-weight form below 0.5)
            m = __builtin_fabs(ob1) < 0.5 ? fma(ob1, g - mo, mo) : fma(-(g - mo), 1.0 - ob1, g);
            v = fma(ob2, g * g, vo * beta2);
            double den = sqrt(v);
            den = den / bc2s;
            den = den + eps;
            pn = fma(step_size, m / den, p);
        } else {
            if (weight_decay != 0) g = fma(p, weight_decay, g);
            m = fma(beta1, mo, ob1 * g);
            v = fma(beta2, vo, ob2 * g * g);
            const double denom = sqrt(v) / bc2s + eps;
            pn = p - step_size * m / denom;
        }
        param[i] = pn;
        if (stage) stage[stage_col((uint32_t)i, sm)] = pn;   // the next forward's brick copy
        exp_avg[i] = m;
        exp_avg_sq[i] = v;
    }
    if (part) block_partial(acc, part);
}

static unsigned loss_grid(int64_t n) {
    const int64_t b = (n + kLossThreads - 1) / kLossThreads;
    return (unsigned)(b < kLossMaxBlocks ? (b > 0 ? b : 1) : kLossMaxBlocks);
}

}  // namespace sphrt

using namespace sphrt;

extern "C" int64_t sphrt_loss_partials(int64_t n) { return n > 0 ? (int64_t)loss_grid(n) : 0; }

extern "C" int sphrt_sq_residual_f64(const double* yhat, const void* y, int y_is_f64, int64_t n,
                                     double scale, const int32_t* order, double* r_scaled,
                                     double* partial_sums, void* stream) {
    if (n <= 0) return fail("sphrt_sq_residual_f64: empty measurement");
    if (!yhat || !y || !r_scaled || !partial_sums) return fail("null buffer");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL(sq_residual_kernel<double>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const double*)y, n, scale, order, r_scaled, partial_sums);
    else
        hipLaunchKernelGGL(sq_residual_kernel<float>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           st, yhat, (const float*)y, n, scale, order, r_scaled, partial_sums);
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

static int adam_launch(bool foreach, double* param, const double* grad, double* exp_avg,
                       double* exp_avg_sq, int64_t n, double a, double beta1, double beta2,
                       double eps, double weight_decay, double b, double c_neg,
                       double* partial_sums, const sphrt_csr* stage_of, void* stream,
                       const char* what) {
    if (n <= 0) return fail("%s: empty volume", what);
    if (!param || !grad || !exp_avg || !exp_avg_sq) return fail("null buffer");
    StageMap sm{};
    double* stage = nullptr;
    if (stage_of && staged(stage_of)) {
        if (!stage_map(stage_of, sm)) return fail("inconsistent brick staging fields");
        if (stage_of->n_cols != n)
            return fail("%s: %lld voxels, the CSR has %lld columns", what, (long long)n,
                        (long long)stage_of->n_cols);
        if (!stage_of->stage || (int64_t)sizeof(double) * stage_of->stage_cols > stage_of->stage_bytes)
            return fail("brick stage buffer missing or too small");
        stage = (double*)stage_of->stage;
    }
    StreamGuard guard(stream);
    if (foreach)
        hipLaunchKernelGGL(adam_neg_kernel<true>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq, n, a, beta1,
                           beta2, eps, weight_decay, b, c_neg, partial_sums, sm, stage);
    else
        hipLaunchKernelGGL(adam_neg_kernel<false>, dim3(loss_grid(n)), dim3(kLossThreads), 0,
                           (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq, n, a, beta1,
                           beta2, eps, weight_decay, b, c_neg, partial_sums, sm, stage);
    return check_launch(what);
}

extern "C" int sphrt_adam_neg_f64(double* param, const double* grad, double* exp_avg,
                                  double* exp_avg_sq, int64_t n, double lr, double beta1,
                                  double beta2, double eps, double weight_decay, double step,
                                  double c_neg, double* partial_sums, const sphrt_csr* stage_of,
                                  void* stream) {
    if (!(step >= 1)) return fail("sphrt_adam_neg_f64: step counts from 1");
    return adam_launch(false, param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps,
                       weight_decay, step, c_neg, partial_sums, stage_of, stream,
                       "sphrt_adam_neg_f64");
}

extern "C" int sphrt_adam_foreach_neg_f64(double* param, const double* grad, double* exp_avg,
                                          double* exp_avg_sq, int64_t n, double step_size,
                                          double beta1, double beta2, double eps,
                                          double weight_decay, double bc2_sqrt, double c_neg,
                                          double* partial_sums, const sphrt_csr* stage_of,
                                          void* stream) {
    if (!(bc2_sqrt > 0)) return fail("sphrt_adam_foreach_neg_f64: bias correction must be > 0");
    return adam_launch(true, param, grad, exp_avg, exp_avg_sq, n, step_size, beta1, beta2, eps,
                       weight_decay, bc2_sqrt, c_neg, partial_sums, stage_of, stream,
                       "sphrt_adam_foreach_neg_f64");
}
