// api.hip — plan management, CSR scan/partition, forward and adjoint kernels, error plumbing.
#include <math.h>
#include <string.h>

#include "common.hpp"

#define SPHRT_VERSION "sph_raytracer_amd 0.1 (gfx950)"

namespace sphrt {

static thread_local char g_err[512] = "";

int fail(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return -1;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail("%s launch failed: %s", what, hipGetErrorString(e));
    return 0;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------------------------------------
// exclusive scan of int32 counts -> int64 row pointers (3 launches, 1024 counts per block)
constexpr int kScanPerBlock = 1024;

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int64_t u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    return v;
}

// block-wide exclusive scan of one value per thread (256 threads); returns the block total too
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t& total, int64_t* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    int64_t wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += sh[w];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return wbase + inc - v;
}

__global__ __launch_bounds__(256) void scan_reduce_kernel(const int32_t* counts, int64_t n,
                                                          int64_t* block_sums) {
    __shared__ int64_t sh[4];
    const int64_t b0 = (int64_t)blockIdx.x * kScanPerBlock;
    int64_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int64_t i = b0 + threadIdx.x * 4 + q;
        if (i < n) v += counts[i];
    }
    int64_t tot;
    (void)block_excl_scan(v, tot, sh);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void scan_blocks_kernel(int64_t* block_sums, int64_t nb,
                                                          int64_t* total_out) {
    __shared__ int64_t sh[4];
    const int64_t per = (nb + 255) / 256;
    const int64_t i0 = threadIdx.x * per;
    int64_t v = 0;
    for (int64_t i = i0; i < i0 + per && i < nb; ++i) v += block_sums[i];
    int64_t tot;
    int64_t run = block_excl_scan(v, tot, sh);
    for (int64_t i = i0; i < i0 + per && i < nb; ++i) {
        int64_t x = block_sums[i];
        block_sums[i] = run;
        run += x;
    }
    if (threadIdx.x == 0) *total_out = tot;
}

__global__ __launch_bounds__(256) void scan_apply_kernel(const int32_t* counts, int64_t n,
                                                         const int64_t* block_sums,
                                                         int64_t* row_ptr) {
    __shared__ int64_t sh[4];
    const int64_t b0 = (int64_t)blockIdx.x * kScanPerBlock;
    int64_t c[4];
    int64_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int64_t i = b0 + threadIdx.x * 4 + q;
        c[q] = i < n ? counts[i] : 0;
        v += c[q];
    }
    int64_t tot;
    int64_t run = block_excl_scan(v, tot, sh) + block_sums[blockIdx.x];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int64_t i = b0 + threadIdx.x * 4 + q;
        if (i < n) row_ptr[i] = run;
        run += c[q];
    }
}

// ---------------------------------------------------------------------------------------------
// static partition: block b owns the rays whose row starts in [b*spb, (b+1)*spb)
__global__ __launch_bounds__(256) void partition_kernel(const int64_t* row_ptr, int64_t n,
                                                        int64_t spb, int64_t* block_lo,
                                                        int64_t nblocks) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nblocks) return;
    const int64_t target = b * spb;
    int64_t lo = 0, hi = n;  // first i in [0, n) with row_ptr[i] >= target, else n
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (row_ptr[mid] < target) lo = mid + 1;
        else hi = mid;
    }
    block_lo[b] = lo;
}

// ---------------------------------------------------------------------------------------------
// forward line integral over the CSR.  Per partition block: segment-parallel products staged
// in LDS (balanced gathers, coalesced vox/len streams), then one thread per ray sums its row.
constexpr int kApplyCap = 4096;

// channel of segment s when every observation has its own time slice (ray_chan_div mode)
__device__ __forceinline__ int64_t seg_channel(const int64_t* row_ptr, int64_t s, int64_t lo,
                                               int64_t hi, int64_t div) {
    int64_t o = lo / div;
    const int64_t olast = (hi - 1) / div;
    while (o < olast && row_ptr[(o + 1) * div] <= s) ++o;
    return o;
}

// T: density / image type; L: stored segment length type (float32 copy on the float32 path,
// the float64 trace itself otherwise).  Products and sums are float64 either way.
template <typename T, typename L>
__global__ __launch_bounds__(256) void forward_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ vox,
    const L* __restrict__ len, const int64_t* __restrict__ block_lo,
    const T* __restrict__ density, int64_t n_chan, int64_t chan_stride, int64_t div,
    T* __restrict__ out, int64_t ocs) {
    __shared__ double prod[kApplyCap];
    const int64_t lo = block_lo[blockIdx.x], hi = block_lo[blockIdx.x + 1];
    if (lo >= hi) return;
    const int64_t s0 = row_ptr[lo], s1 = row_ptr[hi];
    const int64_t nsg = s1 - s0;
    const int tid = threadIdx.x;
    for (int64_t c = 0; c < n_chan; ++c) {
        const T* rho = density + c * chan_stride;
        if (nsg <= kApplyCap) {
            for (int64_t s = s0 + tid; s < s1; s += 256) {
                const T* rc = div > 0 ? density + seg_channel(row_ptr, s, lo, hi, div) * chan_stride
                                      : rho;
                prod[s - s0] = (double)rc[vox[s]] * len[s];
            }
            __syncthreads();
            for (int64_t r = lo + tid; r < hi; r += 256) {
                const int64_t a = row_ptr[r] - s0, b = row_ptr[r + 1] - s0;
                double acc = 0.0;
                for (int64_t q = a; q < b; ++q) acc += prod[q];
                out[c * ocs + r] = (T)acc;
            }
            __syncthreads();
        } else {  // a row longer than the LDS stage: direct (rare)
            for (int64_t r = lo + tid; r < hi; r += 256) {
                const T* rc = div > 0 ? density + (r / div) * chan_stride : rho;
                double acc = 0.0;
                for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) acc += (double)rc[vox[q]] * len[q];
                out[c * ocs + r] = (T)acc;
            }
        }
    }
}

// adjoint: acc[chan][vox] += y[chan][ray] * len, float64 atomics.  Per block the ray values are
// spread over their segments in LDS, then segments are streamed in order (coalesced).
template <typename TY>
__global__ __launch_bounds__(256) void adjoint_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ vox,
    const double* __restrict__ len, const int64_t* __restrict__ block_lo,
    const TY* __restrict__ y, int64_t n_chan, int64_t ycs, int64_t div, double* acc,
    int64_t chan_stride) {
    __shared__ double yb[kApplyCap];
    const int64_t lo = block_lo[blockIdx.x], hi = block_lo[blockIdx.x + 1];
    if (lo >= hi) return;
    const int64_t s0 = row_ptr[lo], s1 = row_ptr[hi];
    const int64_t nsg = s1 - s0;
    const int tid = threadIdx.x;
    for (int64_t c = 0; c < n_chan; ++c) {
        const TY* yc = y + c * ycs;
        if (nsg <= kApplyCap) {
            for (int64_t r = lo + tid; r < hi; r += 256) {
                const double v = (double)yc[r];
                for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) yb[q - s0] = v;
            }
            __syncthreads();
            for (int64_t s = s0 + tid; s < s1; s += 256) {
                double* ac = div > 0 ? acc + seg_channel(row_ptr, s, lo, hi, div) * chan_stride
                                     : acc + c * chan_stride;
                atomicAdd(ac + vox[s], yb[s - s0] * len[s]);
            }
            __syncthreads();
        } else {
            for (int64_t r = lo + tid; r < hi; r += 256) {
                double* ac = div > 0 ? acc + (r / div) * chan_stride : acc + c * chan_stride;
                const double v = (double)yc[r];
                for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) atomicAdd(ac + vox[q], v * len[q]);
            }
        }
    }
}

__global__ __launch_bounds__(256) void f64_to_f32_kernel(const double* src, float* dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        dst[i] = (float)src[i];
}

static unsigned grid_for(int64_t n, int64_t per_block, int64_t cap) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

template <typename T, typename L>
static int forward_impl(const int64_t* row_ptr, const int32_t* vox, const L* len, int64_t n,
                        const int64_t* block_lo, int64_t nblocks, int64_t spb, const T* density,
                        int64_t n_chan, int64_t chan_stride, int64_t div, T* out, int64_t ocs,
                        void* stream) {
    if (n == 0) return 0;
    if (nblocks < 1 || nblocks > 0x7fffffff) return fail("bad partition block count %lld", (long long)nblocks);
    if (spb > kApplyCap) return fail("seg_per_block %lld exceeds the LDS stage %d", (long long)spb, kApplyCap);
    if (n_chan < 1) return fail("n_chan must be >= 1");
    if (div > 0 && n_chan != 1) return fail("ray_chan_div requires n_chan == 1");
    hipLaunchKernelGGL((forward_kernel<T, L>), dim3((unsigned)nblocks), dim3(256), 0,
                       (hipStream_t)stream, row_ptr, vox, len, block_lo, density, n_chan,
                       chan_stride, div, out, ocs);
    return check_launch("forward_kernel");
}

}  // namespace sphrt

using namespace sphrt;

extern "C" const char* sphrt_last_error(void) { return g_err; }
extern "C" const char* sphrt_version(void) { return SPHRT_VERSION; }

extern "C" int sphrt_plan_create(const sphrt_grid_desc* gd, int device, sphrt_plan** out) {
    if (!gd || !out) return fail("null argument");
    *out = nullptr;
    // zero-voxel axes are legal for the per-family solves (a single boundary), not for traces
    if (gd->nr < 0 || gd->ne < 0 || gd->na < 0) return fail("grid shape must be non-negative");
    if (gd->nr > 32000 || gd->ne > 32000 || gd->na > 32000)
        return fail("grid extent too large (max 32000 voxels per axis)");
    if (!gd->r_b || !gd->e_b || !gd->a_b || !gd->cos_e || !gd->cos2_e || !gd->cos_a || !gd->sin_a)
        return fail("null boundary table");
    const int nbr = gd->nr + 1, nbe = gd->ne + 1, nba = gd->na + 1;
    for (int j = 1; j < nbr; ++j)
        if (!(gd->r_b[j] >= gd->r_b[j - 1])) return fail("r_b must be ascending");
    const int64_t K = 2LL * nbr + 2LL * nbe + nba + 1;
    if (K >= 65535) return fail("too many boundaries (K=%lld)", (long long)K);
    // table layout: r_b | c2_e | cos_a | sin_a (doubles) | e_flags (bytes)
    const size_t nd = (size_t)nbr + nbe + 2 * (size_t)nba;
    const size_t bytes = nd * sizeof(double) + (size_t)nbe;
    double* host = (double*)malloc(bytes);
    if (!host) return fail("host allocation failed");
    double* h_r = host;
    double* h_c2 = h_r + nbr;
    double* h_ca = h_c2 + nbe;
    double* h_sa = h_ca + nba;
    uint8_t* h_fl = (uint8_t*)(h_sa + nba);
    memcpy(h_r, gd->r_b, nbr * sizeof(double));
    memcpy(h_c2, gd->cos2_e, nbe * sizeof(double));
    memcpy(h_ca, gd->cos_a, nba * sizeof(double));
    memcpy(h_sa, gd->sin_a, nba * sizeof(double));
    const double half_pi = 3.141592653589793 / 2;  // tr.pi / 2 (raytracer.py:457)
    for (int j = 0; j < nbe; ++j) {
        uint8_t f = 0;
        if (gd->cos_e[j] >= 0.0) f |= 1;
        if (fabs(half_pi - gd->e_b[j]) < gd->close_tol) f |= 2;
        h_fl[j] = f;
    }
    DeviceGuard guard(device);
    void* dmem = nullptr;
    hipError_t e = hipMalloc(&dmem, bytes);
    if (e != hipSuccess) {
        free(host);
        return fail("hipMalloc(plan tables) failed: %s", hipGetErrorString(e));
    }
    e = hipMemcpy(dmem, host, bytes, hipMemcpyHostToDevice);
    free(host);
    if (e != hipSuccess) {
        (void)hipFree(dmem);
        return fail("hipMemcpy(plan tables) failed: %s", hipGetErrorString(e));
    }
    sphrt_plan* p = new sphrt_plan;
    p->device = device;
    p->table_mem = dmem;
    GridDev& G = p->dev;
    G.nr = gd->nr; G.ne = gd->ne; G.na = gd->na;
    G.nbr = nbr; G.nbe = nbe; G.nba = nba;
    G.K = (int)K;
    G.a_wrap = gd->a_wrap ? 1 : 0;
    G.close_tol = gd->close_tol;
    G.plane_par_tol = gd->plane_par_tol;
    G.r_outer = gd->r_b[gd->nr];
    double* d = (double*)dmem;
    G.r_b = d;
    G.c2_e = d + nbr;
    G.cos_a = d + nbr + nbe;
    G.sin_a = d + nbr + nbe + nba;
    G.e_flags = (const uint8_t*)(d + nd);
    *out = p;
    return 0;
}

extern "C" int sphrt_plan_destroy(sphrt_plan* plan) {
    if (!plan) return 0;
    DeviceGuard guard(plan->device);
    hipError_t e = hipFree(plan->table_mem);
    delete plan;
    if (e != hipSuccess) return fail("hipFree(plan tables) failed: %s", hipGetErrorString(e));
    return 0;
}

extern "C" int64_t sphrt_plan_candidates(const sphrt_plan* plan) { return plan ? plan->dev.K : -1; }

extern "C" size_t sphrt_scan_workspace_bytes(int64_t n) {
    int64_t nb = (n + kScanPerBlock - 1) / kScanPerBlock;
    return (size_t)(nb + 1) * sizeof(int64_t);
}

extern "C" int sphrt_scan_counts(const int32_t* counts, int64_t n, int64_t* row_ptr,
                                 void* workspace, void* stream) {
    if (n < 0) return fail("negative length");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        if (hipMemsetAsync(row_ptr, 0, sizeof(int64_t), st) != hipSuccess) return fail("memset failed");
        return 0;
    }
    const int64_t nb = (n + kScanPerBlock - 1) / kScanPerBlock;
    if (nb > 0x7fffffff) return fail("too many rays");
    int64_t* bs = (int64_t*)workspace;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(256), 0, st, counts, n, bs);
    if (int e = check_launch("scan_reduce")) return e;
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(256), 0, st, bs, nb, row_ptr + n);
    if (int e = check_launch("scan_blocks")) return e;
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(256), 0, st, counts, n, bs,
                       row_ptr);
    return check_launch("scan_apply");
}

extern "C" int sphrt_partition(const int64_t* row_ptr, int64_t n, int64_t spb, int64_t* block_lo,
                               int64_t nblocks, void* stream) {
    if (spb < 1) return fail("seg_per_block must be >= 1");
    if (nblocks < 1) return fail("nblocks must be >= 1");
    const int64_t m = nblocks + 1;
    hipLaunchKernelGGL(partition_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, row_ptr, n, spb, block_lo, nblocks);
    return check_launch("partition_kernel");
}

extern "C" int sphrt_forward_f32(const int64_t* row_ptr, const int32_t* vox, const float* len,
                                 int64_t n, const int64_t* block_lo, int64_t nblocks,
                                 int64_t spb, const float* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, float* out, int64_t ocs,
                                 void* stream) {
    return forward_impl<float, float>(row_ptr, vox, len, n, block_lo, nblocks, spb, density,
                                      n_chan, chan_stride, div, out, ocs, stream);
}
extern "C" int sphrt_forward_f64(const int64_t* row_ptr, const int32_t* vox, const double* len,
                                 int64_t n, const int64_t* block_lo, int64_t nblocks,
                                 int64_t spb, const double* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, double* out, int64_t ocs,
                                 void* stream) {
    return forward_impl<double, double>(row_ptr, vox, len, n, block_lo, nblocks, spb, density,
                                        n_chan, chan_stride, div, out, ocs, stream);
}

extern "C" int sphrt_adjoint_accumulate(const int64_t* row_ptr, const int32_t* vox,
                                        const double* len, int64_t n, const int64_t* block_lo,
                                        int64_t nblocks, int64_t spb, const void* y, int y_is_f64,
                                        int64_t n_chan, int64_t ycs, int64_t div, double* acc,
                                        int64_t chan_stride, void* stream) {
    if (n == 0) return 0;
    if (nblocks < 1 || nblocks > 0x7fffffff) return fail("bad partition block count");
    if (spb > kApplyCap) return fail("seg_per_block exceeds the LDS stage");
    if (n_chan < 1) return fail("n_chan must be >= 1");
    if (div > 0 && n_chan != 1) return fail("ray_chan_div requires n_chan == 1");
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL((adjoint_kernel<double>), dim3((unsigned)nblocks), dim3(256), 0, st,
                           row_ptr, vox, len, block_lo, (const double*)y, n_chan, ycs, div, acc,
                           chan_stride);
    else
        hipLaunchKernelGGL((adjoint_kernel<float>), dim3((unsigned)nblocks), dim3(256), 0, st,
                           row_ptr, vox, len, block_lo, (const float*)y, n_chan, ycs, div, acc,
                           chan_stride);
    return check_launch("adjoint_kernel");
}

extern "C" int sphrt_f64_to_f32(const double* src, float* dst, int64_t n, void* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(f64_to_f32_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, src, dst, n);
    return check_launch("f64_to_f32");
}
