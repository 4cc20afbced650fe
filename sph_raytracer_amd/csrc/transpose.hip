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

__global__ __launch_bounds__(256) void seg_keys_kernel(const int64_t* row_ptr, int64_t n_rays,
                                                       const int32_t* vox, int32_t* keys,
                                                       int32_t* idx, int32_t* seg_ray,
                                                       int32_t* col_count) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n_rays) return;
    for (int64_t s = row_ptr[r]; s < row_ptr[r + 1]; ++s) {
        const int32_t v = vox[s] & 0x7fffffff;
        keys[s] = v;
        idx[s] = (int32_t)s;
        seg_ray[s] = (int32_t)r;
        atomicAdd(col_count + v, 1);
    }
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
    hipcub::DeviceRadixSort::SortPairs(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr,
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
    hipStream_t st = (hipStream_t)stream;
    TWs w;
    layout(c->n_segments, n_vox, (unsigned char*)workspace, &w);
    if (hipMemsetAsync(w.count, 0, (size_t)n_vox * 4, st) != hipSuccess) return fail("memset failed");
    if (c->n_rays > 0) {
        hipLaunchKernelGGL(seg_keys_kernel, dim3((unsigned)((c->n_rays + 255) / 256)), dim3(256), 0,
                           st, c->row_ptr, c->n_rays, c->vox, w.keys, w.idx, w.seg_ray, w.count);
        if (int e = check_launch("seg_keys")) return e;
    }
    if (int e = sphrt_scan_counts(w.count, n_vox, col_ptr, w.scan, stream)) return e;
    const int64_t n = c->n_segments;
    if (n == 0) return 0;
    int bits = 1;
    while ((1LL << bits) < n_vox) ++bits;
    size_t cb = w.cub_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.keys, w.keys_out, w.idx, w.perm, (int)n, 0,
                                           bits, st) != hipSuccess)
        return fail("radix sort failed");
    hipLaunchKernelGGL(gather_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       w.perm, n, w.seg_ray, c->len, t_ray, t_len);
    return check_launch("gather_cols");
}
