// transpose.hip — voxel-major copy of the trace for the deterministic adjoint.
//
// The adjoint (Operator.T, raytracer.py:715-748; autograd backward of raytracer.py:710) scatters
// y[ray] * len into voxels.  Float atomics make that order-dependent and run at the chip's atomic
// rate (MI355X_MICROARCH.md: ~1.3 TB/s of added bytes, far less for scattered adds).  Instead
// the CSR is transposed once — a stable LSD radix sort of (voxel, segment) pairs keeps every
// voxel's contributions in ray order — and the adjoint becomes the same segmented gather-reduce
// as the forward, with rays and voxels swapped: bitwise reproducible, no atomics.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace sphrt {

// Sort keys and values, one thread per segment (coalesced): key = voxel, value = segment.
__global__ __launch_bounds__(256) void seg_keys_kernel(int64_t n_seg, const int32_t* vox,
                                                       int32_t* keys, int32_t* idx) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= n_seg) return;
    keys[s] = vox[s] & 0x7fffffff;
    idx[s] = (int32_t)s;
}

// The ray of every segment: one wave per ray, its lanes over the ray's contiguous segments.
__global__ __launch_bounds__(256) void seg_ray_kernel(const int64_t* row_ptr, int64_t n_rays,
                                                      int32_t* seg_ray) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rays) return;
    const int64_t a = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t s = a + (threadIdx.x & 63); s < e; s += 64) seg_ray[s] = (int32_t)r;
}

// col_ptr from the sorted voxel keys (no per-voxel atomics): at every key change from u to w,
// voxels u+1 .. w start at position i; voxels up to the first key start at 0, those after the
// last key at n.
__global__ __launch_bounds__(256) void col_ptr_kernel(const int32_t* sorted, int64_t n,
                                                      int64_t n_vox, int64_t* col_ptr) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    const int64_t lo = i == 0 ? -1 : (int64_t)sorted[i - 1];
    const int64_t hi = i == n ? n_vox : (int64_t)sorted[i];
    for (int64_t v = lo + 1; v <= hi; ++v) col_ptr[v] = i;
}

__global__ __launch_bounds__(256) void gather_cols_kernel(const int32_t* perm, int64_t n,
                                                          const int32_t* seg_ray,
                                                          const double* len, int32_t* t_ray,
                                                          double* t_len) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int32_t s = perm[i];
    t_ray[i] = seg_ray[s];
    t_len[i] = len[s];
}

struct TWs {
    int32_t *keys, *keys_out, *idx, *perm, *seg_ray, *count;
    void* cub;
    size_t cub_bytes;
    void* scan;
};

static size_t align256(size_t x) { return (x + 255) / 256 * 256; }

static size_t cub_bytes(int64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 31);
    return b;
}

static size_t layout(int64_t n_seg, int64_t n_vox, unsigned char* base, TWs* w) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        unsigned char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    const size_t s4 = (size_t)(n_seg > 0 ? n_seg : 1) * 4;
    TWs t;
    t.keys = (int32_t*)take(s4);
    t.keys_out = (int32_t*)take(s4);
    t.idx = (int32_t*)take(s4);
    t.perm = (int32_t*)take(s4);
    t.seg_ray = (int32_t*)take(s4);
    t.count = (int32_t*)take((size_t)n_vox * 4);
    t.cub_bytes = cub_bytes(n_seg);
    t.cub = take(t.cub_bytes);
    t.scan = take(sphrt_scan_workspace_bytes(n_vox));
    if (w) *w = t;
    return off;
}

}  // namespace sphrt

using namespace sphrt;

extern "C" size_t sphrt_transpose_workspace_bytes(int64_t n_segments, int64_t n_vox) {
    if (n_segments < 0 || n_vox < 1) return 0;
    return layout(n_segments, n_vox, nullptr, nullptr);
}

extern "C" int sphrt_csr_transpose(const sphrt_csr* c, int64_t n_vox, int64_t* col_ptr,
                                   int32_t* t_ray, double* t_len, void* workspace,
                                   size_t workspace_size, void* stream) {
    if (!c || !c->row_ptr || !c->vox || !c->len) return fail("incomplete CSR");
    if (n_vox < 1) return fail("n_vox must be >= 1");
    if (c->n_segments >= 0x7fffffff || c->n_rays >= 0x7fffffff)
        return fail("transpose supports < 2^31 rays and segments");
    if (workspace_size < sphrt_transpose_workspace_bytes(c->n_segments, n_vox))
        return fail("transpose workspace too small");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    TWs w;
    layout(c->n_segments, n_vox, (unsigned char*)workspace, &w);
    const int64_t n = c->n_segments;
    if (n == 0) {
        if (hipMemsetAsync(col_ptr, 0, (size_t)(n_vox + 1) * 8, st) != hipSuccess)
            return fail("memset failed");
        return 0;
    }
    hipLaunchKernelGGL(seg_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                       c->vox, w.keys, w.idx);
    if (int e = check_launch("seg_keys")) return e;
    if (c->n_rays > 0) {
        hipLaunchKernelGGL(seg_ray_kernel, dim3((unsigned)((c->n_rays + 3) / 4)), dim3(256), 0, st,
                           c->row_ptr, c->n_rays, w.seg_ray);
        if (int e = check_launch("seg_ray")) return e;
    }
    int bits = 1;
    while ((1LL << bits) < n_vox) ++bits;
    size_t cb = w.cub_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.keys, w.keys_out, w.idx, w.perm, (int)n, 0,
                                           bits, st) != hipSuccess)
        return fail("radix sort failed");
    hipLaunchKernelGGL(col_ptr_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st,
                       w.keys_out, n, n_vox, col_ptr);
    if (int e = check_launch("col_ptr")) return e;
    hipLaunchKernelGGL(gather_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       w.perm, n, w.seg_ray, c->len, t_ray, t_len);
    return check_launch("gather_cols");
}
