// api.hip — plan management, the count -> row-pointer scan, conversions, error plumbing.
#include <math.h>
#include <string.h>

#include "common.hpp"

#ifndef SPHRT_SOURCE_HASH   // set by build.py: a hash of the sources and flags (build.source_hash)
#define SPHRT_SOURCE_HASH "unhashed"
#endif
#define SPHRT_VERSION "sph_raytracer_amd 0.3 (gfx950) src " SPHRT_SOURCE_HASH

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

__global__ __launch_bounds__(256) void f64_to_f32_kernel(const double* src, float* dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        dst[i] = (float)src[i];
}

// dst[i] = src[idx[i]]: 4 consecutive outputs per thread (one 16-byte index load, 4 gathers,
// their stores), one pass, no grid-stride loop (the ~1 MB gathers this serves fit one wave of
// workgroups).
template <typename T>
__global__ __launch_bounds__(256) void gather_kernel(const T* __restrict__ src,
                                                     const int32_t* __restrict__ idx, int64_t n,
                                                     T* __restrict__ dst) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 + 4 <= n && ((uintptr_t)(idx + i0) & 15) == 0) {
        const int4 q = *reinterpret_cast<const int4*>(idx + i0);
        const T a = src[q.x], b = src[q.y], c = src[q.z], d = src[q.w];
        dst[i0] = a;
        dst[i0 + 1] = b;
        dst[i0 + 2] = c;
        dst[i0 + 3] = d;
    } else {
        for (int64_t i = i0; i < n && i < i0 + 4; ++i) dst[i] = src[idx[i]];
    }
}

static unsigned grid_for(int64_t n, int64_t per_block, int64_t cap) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace sphrt

using namespace sphrt;

extern "C" const char* sphrt_last_error(void) { return g_err; }
extern "C" const char* sphrt_version(void) { return SPHRT_VERSION; }

// Validate a grid description; K and the table block size on success.
static int plan_check(const sphrt_grid_desc* gd, int64_t& K, size_t& bytes) {
    if (!gd) return fail("null argument");
    // zero-voxel axes are legal for the per-family solves (a single boundary), not for traces
    if (gd->nr < 0 || gd->ne < 0 || gd->na < 0) return fail("grid shape must be non-negative");
    if (gd->nr > 32000 || gd->ne > 32000 || gd->na > 32000)
        return fail("grid extent too large (max 32000 voxels per axis)");
    if (!gd->r_b || !gd->e_b || !gd->a_b || !gd->cos_e || !gd->cos2_e || !gd->cos_a || !gd->sin_a)
        return fail("null boundary table");
    const int nbr = gd->nr + 1, nbe = gd->ne + 1, nba = gd->na + 1;
    for (int j = 1; j < nbr; ++j)
        if (!(gd->r_b[j] >= gd->r_b[j - 1])) return fail("r_b must be ascending");
    K = 2LL * nbr + 2LL * nbe + nba + 1;
    if (K >= 65535) return fail("too many boundaries (K=%lld)", (long long)K);
    // table layout: r_b | c2_e | cos_a | sin_a | e_b | a_b (doubles) | e_flags (bytes)
    const size_t nd = (size_t)nbr + 2 * (size_t)nbe + 3 * (size_t)nba;
    bytes = nd * sizeof(double) + (size_t)nbe;
    return 0;
}

extern "C" size_t sphrt_plan_table_bytes(const sphrt_grid_desc* gd) {
    int64_t K;
    size_t bytes;
    return plan_check(gd, K, bytes) ? 0 : bytes;
}

extern "C" int sphrt_plan_pack_tables(const sphrt_grid_desc* gd, void* host_tables) {
    int64_t K;
    size_t bytes;
    if (int e = plan_check(gd, K, bytes)) return e;
    if (!host_tables) return fail("null table buffer");
    const int nbr = gd->nr + 1, nbe = gd->ne + 1, nba = gd->na + 1;
    double* h_r = (double*)host_tables;
    double* h_c2 = h_r + nbr;
    double* h_ca = h_c2 + nbe;
    double* h_sa = h_ca + nba;
    double* h_eb = h_sa + nba;
    double* h_ab = h_eb + nbe;
    uint8_t* h_fl = (uint8_t*)(h_ab + nba);
    memcpy(h_r, gd->r_b, nbr * sizeof(double));
    memcpy(h_c2, gd->cos2_e, nbe * sizeof(double));
    memcpy(h_ca, gd->cos_a, nba * sizeof(double));
    memcpy(h_sa, gd->sin_a, nba * sizeof(double));
    memcpy(h_eb, gd->e_b, nbe * sizeof(double));
    memcpy(h_ab, gd->a_b, nba * sizeof(double));
    const double half_pi = 3.141592653589793 / 2;  // tr.pi / 2 (raytracer.py:457)
    for (int j = 0; j < nbe; ++j) {
        uint8_t f = 0;
        if (gd->cos_e[j] >= 0.0) f |= 1;
        if (fabs(half_pi - gd->e_b[j]) < gd->close_tol) f |= 2;
        h_fl[j] = f;
    }
    return 0;
}

// The plan over device tables `dmem` (packed by sphrt_plan_pack_tables); owns them if `own`.
static sphrt_plan* plan_over(const sphrt_grid_desc* gd, int device, void* dmem, bool own,
                             int64_t K) {
    sphrt_plan* p = new sphrt_plan;
    p->device = device;
    p->table_mem = own ? dmem : nullptr;
    GridDev& G = p->dev;
    G.nr = gd->nr; G.ne = gd->ne; G.na = gd->na;
    G.nbr = gd->nr + 1; G.nbe = gd->ne + 1; G.nba = gd->na + 1;
    G.K = (int)K;
    G.a_wrap = gd->a_wrap ? 1 : 0;
    G.close_tol = gd->close_tol;
    G.plane_par_tol = gd->plane_par_tol;
    G.r_outer = gd->r_b[gd->nr];
    int e_asc = 1, a_asc = 1;
    for (int j = 1; j < G.nbe; ++j) e_asc &= gd->e_b[j] > gd->e_b[j - 1] ? 1 : 0;
    for (int j = 1; j < G.nba; ++j) a_asc &= gd->a_b[j] > gd->a_b[j - 1] ? 1 : 0;
    G.e_asc = e_asc;
    G.a_asc = a_asc;
    // evenly spaced boundaries (linspace grids): within 1e-9 of a spacing of b0 + i h
    auto even = [](const double* b, int n) {
        if (n < 2 || !(b[n - 1] > b[0])) return 0;
        const double h = (b[n - 1] - b[0]) / (n - 1);
        for (int i = 0; i < n; ++i)
            if (!(fabs(b[i] - (b[0] + i * h)) <= 1e-9 * h)) return 0;
        return 1;
    };
    G.uni = even(gd->r_b, G.nbr) | (even(gd->e_b, G.nbe) << 1) | (even(gd->a_b, G.nba) << 2);
    G.r_b = (const double*)dmem;   // the rest of the block follows it (GridDev accessors)
    return p;
}

extern "C" int sphrt_plan_create(const sphrt_grid_desc* gd, int device, sphrt_plan** out) {
    if (!out) return fail("null argument");
    *out = nullptr;
    int64_t K;
    size_t bytes;
    if (int e = plan_check(gd, K, bytes)) return e;
    void* host = malloc(bytes);
    if (!host) return fail("host allocation failed");
    if (int e = sphrt_plan_pack_tables(gd, host)) {
        free(host);
        return e;
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
    *out = plan_over(gd, device, dmem, true, K);
    return 0;
}

extern "C" int sphrt_plan_create_external(const sphrt_grid_desc* gd, int device,
                                          const void* dev_tables, sphrt_plan** out) {
    if (!out) return fail("null argument");
    *out = nullptr;
    int64_t K;
    size_t bytes;
    if (int e = plan_check(gd, K, bytes)) return e;
    if (!dev_tables || (uintptr_t)dev_tables % 8 != 0)
        return fail("device tables missing or not 8-byte aligned");
    *out = plan_over(gd, device, const_cast<void*>(dev_tables), false, K);
    return 0;
}

extern "C" int sphrt_plan_destroy(sphrt_plan* plan) {
    if (!plan) return 0;
    if (!plan->table_mem) {       // caller-owned tables (sphrt_plan_create_external): no hipFree
        delete plan;
        return 0;
    }
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
    StreamGuard guard(stream);
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

extern "C" int sphrt_f64_to_f32(const double* src, float* dst, int64_t n, void* stream) {
    if (n == 0) return 0;
    StreamGuard guard(stream);
    hipLaunchKernelGGL(f64_to_f32_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, src, dst, n);
    return check_launch("f64_to_f32");
}

template <typename T>
static int gather(const T* src, const int32_t* idx, int64_t n, T* dst, void* stream) {
    if (n < 0) return fail("negative gather length");
    if (n == 0) return 0;
    if (!src || !idx || !dst) return fail("null gather argument");
    StreamGuard guard(stream);
    const int64_t blocks = (n + 1023) / 1024;
    if (blocks > INT32_MAX) return fail("gather too large");
    hipLaunchKernelGGL(gather_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       src, idx, n, dst);
    return check_launch("gather_kernel");
}
extern "C" int sphrt_gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst,
                                void* stream) {
    return gather(src, idx, n, dst, stream);
}
extern "C" int sphrt_gather_f64(const double* src, const int32_t* idx, int64_t n, double* dst,
                                void* stream) {
    return gather(src, idx, n, dst, stream);
}
