// apply.hip — forward line integral and adjoint back-projection on the segment CSR.
//
// Replaces Operator.__call__ (raytracer.py:692-713) and Operator.T / the autograd backward of
// raytracer.py:710.  The reference gathers density at every one of the K padded candidates of
// every ray and sums over K; here only the non-zero segments are streamed.
//
// Layout built once per trace (sphrt_csr_index):
//   vox[s]     linear voxel index, bit 31 set on the first segment of every non-empty ray
//   row_ray[k] the ray of the k-th non-empty row
//   blocks[b]  {ray_lo, ray_hi, seg_lo, seg_hi, row_lo}: workgroup b owns the rays whose rows
//              start in [b*kSegPerBlock, (b+1)*kSegPerBlock) — whole rows, so no row is ever
//              split between workgroups and the result needs no cross-workgroup combine.
// Forward per workgroup: each thread streams 8 consecutive segments (aligned vector loads),
// gathers the density (a 0.5-8 MB volume, L2/MALL resident), reduces runs between head bits in
// float64, and a block-level segmented scan stitches rows that cross thread chunks.  Balanced
// whatever the row lengths, ~3 dependent global round trips per workgroup, deterministic order.
#include "common.hpp"

namespace sphrt {

constexpr uint32_t kHead = 0x80000000u;
constexpr int kThreads = 256;
constexpr int kPer = 8;                         // segments per thread per pass
constexpr int kPass = kThreads * kPer;          // 2048 segments per pass
constexpr int64_t kSegPerBlock = 1792;          // row starts per workgroup (leaves room for the
                                                // last row's overhang inside one pass)

// ---- index --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mark_rows_kernel(const int64_t* row_ptr, int64_t n,
                                                        int32_t* vox, int32_t* nonempty) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t a = row_ptr[r];
    const bool ne = row_ptr[r + 1] > a;
    nonempty[r] = ne ? 1 : 0;
    if (ne) vox[a] = (int32_t)((uint32_t)vox[a] | kHead);
}

__global__ __launch_bounds__(256) void row_list_kernel(const int64_t* row_ptr,
                                                       const int64_t* row_pre, int64_t n,
                                                       int32_t* row_ray) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    if (row_ptr[r + 1] > row_ptr[r]) row_ray[row_pre[r]] = (int32_t)r;
}

__global__ __launch_bounds__(256) void block_meta_kernel(const int64_t* row_ptr,
                                                         const int64_t* row_pre, int64_t n,
                                                         int64_t nblocks, int64_t* blocks) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblocks) return;
    auto first_at_or_after = [&](int64_t target) {   // first ray r < n with row_ptr[r] >= target
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (row_ptr[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int64_t lo = first_at_or_after(b * kSegPerBlock);
    const int64_t hi = (b + 1 == nblocks) ? n : first_at_or_after((b + 1) * kSegPerBlock);
    int64_t* m = blocks + 5 * b;
    m[0] = lo;
    m[1] = hi;
    m[2] = row_ptr[lo];
    m[3] = row_ptr[hi];
    m[4] = row_pre[lo];
}

// ---- block-level scans (256 threads = 4 waves) -----------------------------------------------
struct ScanShared {
    int cnt[4];
    int has[4];
    double sum[4];
};

// exclusive sum of one int per thread; returns the block total in `total`
__device__ __forceinline__ int block_excl_count(int v, int& total, ScanShared& sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(inc, off);
        if (lane >= off) inc += u;
    }
    if (lane == 63) sh.cnt[wid] = inc;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wid; ++w) base += sh.cnt[w];
    total = sh.cnt[0] + sh.cnt[1] + sh.cnt[2] + sh.cnt[3];
    __syncthreads();
    return base + inc - v;
}

// segmented scan: element (has_head, tail) combines as (h1,s1) o (h2,s2) = (h1|h2, h2 ? s2 : s1+s2).
// Returns the exclusive prefix sum value (the open run entering this thread) and the block total.
__device__ __forceinline__ double block_excl_segsum(bool has, double tail, bool& tot_has,
                                                    double& tot_sum, ScanShared& sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    bool h = has;
    double s = tail;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const bool hu = __shfl_up((int)h, off) != 0;
        const double su = __shfl_up(s, off);
        if (lane >= off) {
            s = h ? s : su + s;
            h = h || hu;
        }
    }
    bool eh = __shfl_up((int)h, 1) != 0;
    double es = __shfl_up(s, 1);
    if (lane == 0) {
        eh = false;
        es = 0.0;
    }
    if (lane == 63) {
        sh.has[wid] = h;
        sh.sum[wid] = s;
    }
    __syncthreads();
    double cs = 0.0;
    for (int w = 0; w < wid; ++w)             // carry of the previous waves, in order
        cs = sh.has[w] ? sh.sum[w] : cs + sh.sum[w];
    tot_has = false;
    tot_sum = 0.0;
    for (int w = 0; w < 4; ++w) {
        tot_sum = sh.has[w] ? sh.sum[w] : tot_sum + sh.sum[w];
        tot_has = tot_has || sh.has[w];
    }
    __syncthreads();
    return eh ? es : cs + es;
}

template <typename L>
__device__ __forceinline__ void load8(const int32_t* __restrict__ vox, const L* __restrict__ len,
                                      int64_t p0, int64_t s0, int64_t s1, uint32_t (&v)[kPer],
                                      L (&l)[kPer]) {
    if (p0 >= s0 && p0 + kPer <= s1) {        // whole chunk inside: 16-byte vector loads
        const uint4* vp = reinterpret_cast<const uint4*>(vox + p0);
        const uint4 a = vp[0], b = vp[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
        for (int k = 0; k < kPer; ++k) l[k] = len[p0 + k];
    } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int64_t s = p0 + k;
            const bool ok = s >= s0 && s < s1;
            v[k] = ok ? (uint32_t)vox[s] : 0u;
            l[k] = ok ? len[s] : (L)0;
        }
    }
}

// ---- forward ------------------------------------------------------------------------------
// Channels: static multichannel -> every ray for every channel c < n_chan; ray_chan_div > 0 ->
// ray i reads channel i / div (a time slice per view) and writes out[i].
template <typename T, typename L>
__global__ __launch_bounds__(kThreads) void forward_kernel(
    const int64_t* __restrict__ blocks, const int64_t* __restrict__ row_ptr,
    const int32_t* __restrict__ vox, const L* __restrict__ len,
    const int32_t* __restrict__ row_ray, const T* __restrict__ density, int64_t n_chan,
    int64_t cs, int64_t div, T* __restrict__ out, int64_t ocs) {
    __shared__ ScanShared sh;
    const int64_t* m = blocks + 5 * (int64_t)blockIdx.x;
    const int64_t lo = m[0], hi = m[1], s0 = m[2], s1 = m[3], k0 = m[4];
    const int tid = threadIdx.x;
    const int64_t nc = div > 0 ? 1 : n_chan;
    // empty rays integrate to zero
    for (int64_t r = lo + tid; r < hi; r += kThreads)
        if (row_ptr[r + 1] == row_ptr[r])
            for (int64_t c = 0; c < nc; ++c) out[c * ocs + r] = (T)0;
    if (s0 >= s1) return;
    const int64_t a0 = s0 & ~(int64_t)(kPer - 1);   // chunk grid aligned to 8 segments (32 B)
    for (int64_t c = 0; c < nc; ++c) {
        double carry = 0.0;      // open run entering the pass
        int64_t heads_done = 0;  // heads in earlier passes
        for (int64_t base = a0; base < s1; base += kPass) {
            const int64_t p0 = base + (int64_t)tid * kPer;
            uint32_t v[kPer];
            L l[kPer];
            load8(vox, len, p0, s0, s1, v, l);
            int hcount = 0;
#pragma unroll
            for (int k = 0; k < kPer; ++k) hcount += (v[k] & kHead) ? 1 : 0;
            T rv[kPer];
            if (div == 0) {           // static: gathers go out before any scan
                const T* rho = density + c * cs;
#pragma unroll
                for (int k = 0; k < kPer; ++k) rv[k] = l[k] != (L)0 ? rho[v[k] & ~kHead] : (T)0;
            }
            int pass_heads;
            const int hb = block_excl_count(hcount, pass_heads, sh);
            if (div > 0) {            // time slice of each segment's ray
                int rank = 0;
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    rank += (v[k] & kHead) ? 1 : 0;
                    T x = (T)0;
                    if (l[k] != (L)0) {
                        const int64_t ray = row_ray[k0 + heads_done + hb + rank - 1];
                        x = density[(ray / div) * cs + (v[k] & ~kHead)];
                    }
                    rv[k] = x;
                }
            }
            // thread-local runs
            double tail = 0.0;
            bool has = false;
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                if (v[k] & kHead) {
                    has = true;
                    tail = 0.0;
                }
                tail += (double)rv[k] * (double)l[k];
            }
            bool tot_has;
            double tot_sum;
            const double ex = block_excl_segsum(has, tail, tot_has, tot_sum, sh);
            // the run open at this thread's start: the segmented prefix of the earlier threads,
            // plus the carry of earlier passes when no earlier thread of this pass saw a head
            double run = hb > 0 ? ex : carry + ex;
            int seen = 0;
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const int64_t s = p0 + k;
                if (s < s0 || s >= s1) continue;
                if (v[k] & kHead) {
                    if (s > s0) {
                        const int64_t ray = row_ray[k0 + heads_done + hb + seen - 1];
                        out[c * ocs + ray] = (T)run;
                    }
                    run = 0.0;
                    ++seen;
                }
                run += (double)rv[k] * (double)l[k];
                if (s == s1 - 1) {
                    const int64_t ray = row_ray[k0 + heads_done + hb + seen - 1];
                    out[c * ocs + ray] = (T)run;
                }
            }
            carry = tot_has ? tot_sum : carry + tot_sum;
            heads_done += pass_heads;
        }
    }
}

// ---- adjoint (float64 atomics into a float64 accumulator) -------------------------------------
template <typename TY>
__global__ __launch_bounds__(kThreads) void adjoint_kernel(
    const int64_t* __restrict__ blocks, const int32_t* __restrict__ vox,
    const double* __restrict__ len, const int32_t* __restrict__ row_ray,
    const TY* __restrict__ y, int64_t n_chan, int64_t ycs, int64_t div, double* acc,
    int64_t cs) {
    __shared__ ScanShared sh;
    const int64_t* m = blocks + 5 * (int64_t)blockIdx.x;
    const int64_t s0 = m[2], s1 = m[3], k0 = m[4];
    if (s0 >= s1) return;
    const int tid = threadIdx.x;
    const int64_t a0 = s0 & ~(int64_t)(kPer - 1);
    const int64_t nc = div > 0 ? 1 : n_chan;
    int64_t heads_done = 0;
    for (int64_t base = a0; base < s1; base += kPass) {
        const int64_t p0 = base + (int64_t)tid * kPer;
        uint32_t v[kPer];
        double l[kPer];
        load8(vox, len, p0, s0, s1, v, l);
        int hcount = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) hcount += (v[k] & kHead) ? 1 : 0;
        int pass_heads;
        const int hb = block_excl_count(hcount, pass_heads, sh);
        int64_t ray[kPer];
        int rank = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            rank += (v[k] & kHead) ? 1 : 0;
            ray[k] = l[k] != 0.0 ? (int64_t)row_ray[k0 + heads_done + hb + rank - 1] : -1;
        }
        for (int64_t c = 0; c < nc; ++c) {
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                if (ray[k] < 0) continue;
                const int64_t ch = div > 0 ? ray[k] / div : c;
                const double yv = div > 0 ? (double)y[ray[k]] : (double)y[c * ycs + ray[k]];
                atomicAdd(acc + ch * cs + (v[k] & ~kHead), yv * l[k]);
            }
        }
        heads_done += pass_heads;
    }
}

}  // namespace sphrt

using namespace sphrt;

extern "C" int64_t sphrt_csr_blocks(int64_t n_segments) {
    return n_segments < 0 ? -1 : n_segments / kSegPerBlock + 1;
}

extern "C" size_t sphrt_csr_index_workspace_bytes(int64_t n_rays) {
    // nonempty flags (int32) | row prefix (int64, n+1) | scan workspace
    const size_t a = (((size_t)n_rays * 4 + 255) / 256) * 256;
    const size_t b = (((size_t)(n_rays + 1) * 8 + 255) / 256) * 256;
    return a + b + sphrt_scan_workspace_bytes(n_rays);
}

extern "C" int sphrt_csr_index(const int64_t* row_ptr, int64_t n_rays, int32_t* vox,
                               int32_t* row_ray, int64_t* blocks, int64_t n_blocks,
                               void* workspace, void* stream) {
    if (n_rays < 0 || n_blocks < 1) return fail("bad CSR index sizes");
    if (n_rays == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    unsigned char* ws = (unsigned char*)workspace;
    int32_t* flags = (int32_t*)ws;
    int64_t* pre = (int64_t*)(ws + (((size_t)n_rays * 4 + 255) / 256) * 256);
    void* scan_ws = (unsigned char*)pre + (((size_t)(n_rays + 1) * 8 + 255) / 256) * 256;
    const unsigned g = (unsigned)((n_rays + 255) / 256);
    hipLaunchKernelGGL(mark_rows_kernel, dim3(g), dim3(256), 0, st, row_ptr, n_rays, vox, flags);
    if (int e = check_launch("mark_rows")) return e;
    if (int e = sphrt_scan_counts(flags, n_rays, pre, scan_ws, stream)) return e;
    hipLaunchKernelGGL(row_list_kernel, dim3(g), dim3(256), 0, st, row_ptr, pre, n_rays, row_ray);
    if (int e = check_launch("row_list")) return e;
    hipLaunchKernelGGL(block_meta_kernel, dim3((unsigned)((n_blocks + 255) / 256)), dim3(256), 0,
                       st, row_ptr, pre, n_rays, n_blocks, blocks);
    return check_launch("block_meta");
}

static int check_csr(const sphrt_csr* c, int64_t n_chan, int64_t div) {
    if (!c || !c->row_ptr || !c->vox || !c->row_ray || !c->blocks) return fail("incomplete CSR");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (n_chan < 1) return fail("n_chan must be >= 1");
    if (div > 0 && n_chan != 1) return fail("ray_chan_div requires n_chan == 1");
    return 0;
}

extern "C" int sphrt_forward_f32(const sphrt_csr* c, const float* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, float* out, int64_t ocs,
                                 void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len32) return fail("the float32 forward needs the float32 length copy (len32)");
    if (c->n_rays == 0) return 0;
    hipLaunchKernelGGL((forward_kernel<float, float>), dim3((unsigned)c->n_blocks), dim3(kThreads),
                       0, (hipStream_t)stream, c->blocks, c->row_ptr, c->vox, c->len32,
                       c->row_ray, density, n_chan, chan_stride, div, out, ocs);
    return check_launch("forward_kernel<f32>");
}

extern "C" int sphrt_forward_f64(const sphrt_csr* c, const double* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, double* out, int64_t ocs,
                                 void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len) return fail("missing segment lengths");
    if (c->n_rays == 0) return 0;
    hipLaunchKernelGGL((forward_kernel<double, double>), dim3((unsigned)c->n_blocks),
                       dim3(kThreads), 0, (hipStream_t)stream, c->blocks, c->row_ptr, c->vox,
                       c->len, c->row_ray, density, n_chan, chan_stride, div, out, ocs);
    return check_launch("forward_kernel<f64>");
}

extern "C" int sphrt_adjoint_accumulate(const sphrt_csr* c, const void* y, int y_is_f64,
                                        int64_t n_chan, int64_t ycs, int64_t div, double* acc,
                                        int64_t chan_stride, void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len) return fail("missing segment lengths");
    if (c->n_rays == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (y_is_f64)
        hipLaunchKernelGGL((adjoint_kernel<double>), dim3((unsigned)c->n_blocks), dim3(kThreads), 0,
                           st, c->blocks, c->vox, c->len, c->row_ray, (const double*)y, n_chan,
                           ycs, div, acc, chan_stride);
    else
        hipLaunchKernelGGL((adjoint_kernel<float>), dim3((unsigned)c->n_blocks), dim3(kThreads), 0,
                           st, c->blocks, c->vox, c->len, c->row_ray, (const float*)y, n_chan,
                           ycs, div, acc, chan_stride);
    return check_launch("adjoint_kernel");
}
