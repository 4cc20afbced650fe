// Floors for the forward kernel (study tool, not product code): the same grid and block shape as
// forward_kernel on the same CSR, doing (0) nothing, (1) a coalesced stream of every segment's
// loc + f32 length (the product's per-segment bytes) plus the table read, summed per thread, and
// (2) the same plus one 4-byte store per ray.  Compare with the product kernel's time.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/fwd_floor.hip
//        -o sph_raytracer_amd/lib/variants/libfloor.so
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int STAGE>
__global__ __launch_bounds__(256) void floor_kernel(const uint16_t* __restrict__ loc,
                                                    const float* __restrict__ len,
                                                    const uint16_t* __restrict__ tab,
                                                    int64_t n_seg, int64_t tab_stride,
                                                    float* __restrict__ out, int64_t n_rays) {
    if constexpr (STAGE == 0) {
        if (blockIdx.x == 0x7fffffff) out[0] = 1.f;
        return;
    } else {
        const int64_t base = (int64_t)blockIdx.x * 1792 + threadIdx.x * 8;
        float acc = 0.f;
        if (base + 8 <= n_seg) {
            const uint4 w = *reinterpret_cast<const uint4*>(loc + base);
            const float4 a = *reinterpret_cast<const float4*>(len + base);
            const float4 b = *reinterpret_cast<const float4*>(len + base + 4);
            acc = (float)(w.x + w.y + w.z + w.w) + a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
        }
        for (int j = threadIdx.x; j < tab_stride; j += 256) acc += tab[blockIdx.x * tab_stride + j];
        const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
        if (STAGE == 2 || acc == -1.f) {
            if (r < n_rays) out[r] = acc;
        }
    }
}

extern "C" int sphrt_floor(int stage, const void* loc, const void* len, const void* tab,
                           int64_t n_seg, int64_t tab_stride, int64_t n_blocks, void* out,
                           int64_t n_rays, void* stream) {
    const dim3 g((unsigned)n_blocks), b(256);
    hipStream_t st = (hipStream_t)stream;
    auto a = [&](auto k) {
        hipLaunchKernelGGL(k, g, b, 0, st, (const uint16_t*)loc, (const float*)len,
                           (const uint16_t*)tab, n_seg, tab_stride, (float*)out, n_rays);
    };
    if (stage == 0) a(floor_kernel<0>);
    else if (stage == 1) a(floor_kernel<1>);
    else a(floor_kernel<2>);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
