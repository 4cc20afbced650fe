// Forward-kernel ablation (study tool, not product code): the product forward_kernel's stages
// cut off one at a time on the same CSR and grid, to see where its time goes.
//   0 empty launch  1 +block record  2 +segment stream  3 +density gather  4 +row-head count scan
//   5 +segmented sum scan  (6 = the product kernel, timed through sphrt_forward_f32; 7 = the same
//   without voxel tables)  8/9 = stage 3 with the gather confined to 256/4096 voxels,
//   10 = stage 3 with coalesced loads instead of gathers, 11 = stage 3 reading a 16 KB LDS copy,
//   12-14 = granule-table staging variants (table_ablate)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include
//        -I sph_raytracer_amd/csrc tools/fwd_ablate.hip -o sph_raytracer_amd/lib/variants/libablate.so
#include "../sph_raytracer_amd/csrc/apply.hip"

namespace sphrt {
template <int STAGE>
__global__ __launch_bounds__(kThreads) void ablate_kernel(const int64_t* __restrict__ blocks,
                                                          const int32_t* __restrict__ vox,
                                                          const float* __restrict__ len,
                                                          const float* __restrict__ rho,
                                                          float* __restrict__ sink) {
    __shared__ ScanShared sh;
    __shared__ float tabl[STAGE == 11 ? 4096 : 1];
    if constexpr (STAGE == 11) {             // 16 KB of density staged with 16-byte loads
        const float4* r4 = reinterpret_cast<const float4*>(rho);
        float4* t4 = reinterpret_cast<float4*>(tabl);
#pragma unroll
        for (int q = 0; q < 4; ++q) t4[threadIdx.x + q * kThreads] = r4[threadIdx.x + q * kThreads];
        __syncthreads();
    }
    if constexpr (STAGE == 0) {
        if (blockIdx.x == 0x7fffffff) sink[0] = 1.f;
        return;
    } else {
        const int64_t* m = blocks + kBlockFields * (int64_t)blockIdx.x;
        const int64_t s0 = m[2], s1 = m[3];
        if constexpr (STAGE == 1) {
            if (s0 < 0) sink[blockIdx.x] = (float)s1;
            return;
        } else {
            const int tid = threadIdx.x;
            const int64_t a0 = s0 & ~(int64_t)(kPer - 1);
            double acc = 0.0;
            for (int64_t base = a0; base < s1; base += kPass) {
                uint32_t v[kPer];
                float l[kPer];
                load8(vox + base, len + base, tid * kPer, (int)max<int64_t>(s0 - base, -1),
                      (int)min<int64_t>(s1 - base, (int64_t)kPass + 1), v, l);
                int hc = 0;
                double tail = 0.0;
                bool has = false;
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    float x;
                    if constexpr (STAGE == 8)         // gather confined to 256 voxels (8 lines)
                        x = l[k] != 0.f ? rho[v[k] & 0xff] : 0.f;
                    else if constexpr (STAGE == 9)    // gather confined to 4096 voxels
                        x = l[k] != 0.f ? rho[v[k] & 0xfff] : 0.f;
                    else if constexpr (STAGE == 10)   // coalesced 4-byte loads, same count
                        x = l[k] != 0.f ? rho[threadIdx.x + k * kThreads] : 0.f;
                    else if constexpr (STAGE == 11)   // per-segment read from LDS
                        x = l[k] != 0.f ? tabl[v[k] & 0xfff] : 0.f;
                    else
                        x = STAGE >= 3 ? (l[k] != 0.f ? rho[v[k] & ~kHead] : 0.f)
                                       : (float)(v[k] & 0xff);
                    hc += (v[k] & kHead) ? 1 : 0;
                    if (v[k] & kHead) { has = true; tail = 0.0; }
                    tail += (double)x * (double)l[k];
                }
                acc += tail;
                if constexpr (STAGE >= 4) {
                    int ph;
                    acc += block_excl_count(hc, ph, sh);
                }
                if constexpr (STAGE >= 5) {
                    bool th;
                    double ts;
                    acc += block_excl_segsum(has, tail, th, ts, sh);
                }
            }
            if (acc == -1.0) sink[blockIdx.x * kThreads + tid] = (float)acc;
        }
    }
}
// granule-table staging variants (first pass only, no scans):
//   12 LDS-DMA staging  13 register staging (dwordx4 + ds_write_b128)  14 table loads only
template <int MODE>
__global__ __launch_bounds__(kThreads) void table_ablate(const int64_t* __restrict__ blocks,
                                                         const uint16_t* __restrict__ loc,
                                                         const int32_t* __restrict__ tab,
                                                         const float* __restrict__ len,
                                                         const float* __restrict__ rho,
                                                         float* __restrict__ sink,
                                                         int64_t stride) {
    __shared__ __attribute__((aligned(16))) float dens[4 * kMaxGran];
    const int64_t* m = blocks + kBlockFields * (int64_t)blockIdx.x;
    const int64_t s0 = m[2], s1 = m[3], n_tab = m[5];
    if (n_tab < 0 || s0 >= s1) return;
    const int tid = threadIdx.x;
    const int64_t base = s0 & ~(int64_t)(kPer - 1);
    uint32_t v[kPer];
    float l[kPer];
    load8_loc(loc + base, len + base, tid * kPer, (int)(s0 - base),
              (int)min<int64_t>(s1 - base, (int64_t)kPass + 1), v, l);
    const int32_t* tab_b = tab + (int64_t)blockIdx.x * stride;
    int32_t ti[kGranEarly];
#pragma unroll
    for (int q = 0; q < kGranEarly; ++q) {
        const int j = tid + q * kThreads;
        ti[q] = j < n_tab ? tab_b[j] : 0;
    }
    if constexpr (MODE == 12) {
        stage_granules<float>(rho, ti, tab_b, (int)n_tab, 1 << 30, (int)stride, dens);
    } else if constexpr (MODE == 13) {
#pragma unroll
        for (int q = 0; q < kGranEarly; ++q) {
            const int j = tid + q * kThreads;
            if (j < n_tab)
                reinterpret_cast<float4*>(dens)[j] = reinterpret_cast<const float4*>(rho)[ti[q]];
        }
    } else {
        int acc = 0;
#pragma unroll
        for (int q = 0; q < kGranEarly; ++q) acc += ti[q];
        if (acc == 0x7fffffff) dens[tid] = 1.f;
    }
    __syncthreads();
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) acc += (double)l[k] * (double)dens[v[k] & ~kHead];
    if (acc == -1.0) sink[blockIdx.x * kThreads + tid] = (float)acc;
}
}  // namespace sphrt

extern "C" int sphrt_ablate(int stage, const sphrt_csr* c, const float* rho, float* sink,
                            void* stream) {
    using namespace sphrt;
    const dim3 g((unsigned)c->n_blocks), b(kThreads);
    hipStream_t st = (hipStream_t)stream;
    switch (stage) {
        case 0: hipLaunchKernelGGL(ablate_kernel<0>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 1: hipLaunchKernelGGL(ablate_kernel<1>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 2: hipLaunchKernelGGL(ablate_kernel<2>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 3: hipLaunchKernelGGL(ablate_kernel<3>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 4: hipLaunchKernelGGL(ablate_kernel<4>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 5: hipLaunchKernelGGL(ablate_kernel<5>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 8: hipLaunchKernelGGL(ablate_kernel<8>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 9: hipLaunchKernelGGL(ablate_kernel<9>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 10: hipLaunchKernelGGL(ablate_kernel<10>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 11: hipLaunchKernelGGL(ablate_kernel<11>, g, b, 0, st, c->blocks, c->vox, c->len32, rho, sink); break;
        case 12: hipLaunchKernelGGL(table_ablate<12>, g, b, 0, st, c->blocks, c->loc, c->tab, c->len32, rho, sink, c->tab_stride); break;
        case 13: hipLaunchKernelGGL(table_ablate<13>, g, b, 0, st, c->blocks, c->loc, c->tab, c->len32, rho, sink, c->tab_stride); break;
        case 14: hipLaunchKernelGGL(table_ablate<14>, g, b, 0, st, c->blocks, c->loc, c->tab, c->len32, rho, sink, c->tab_stride); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
