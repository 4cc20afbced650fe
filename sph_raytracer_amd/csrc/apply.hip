// apply.hip — forward line integral and adjoint back-projection on the segment CSR.
//
// Replaces Operator.__call__ (raytracer.py:692-713) and Operator.T / the autograd backward of
// raytracer.py:710.  The reference gathers density at every one of the K padded candidates of
// every ray and sums over K; here only the non-zero segments are streamed.
//
// Layout built once per trace (sphrt_csr_index):
//   vox[s]     linear voxel index, bit 31 set on the first segment of every non-empty ray
//   row_ray[k] the ray of the k-th non-empty row
//   blocks[b]  {empty_lo, empty_hi, seg_lo, seg_hi, row_lo, n_tab}: workgroup b owns the rays whose rows
//              start in [b*kSegPerBlock, (b+1)*kSegPerBlock) — whole rows, so no row is ever
//              split between workgroups and the result needs no cross-workgroup combine.
// Forward per workgroup: each thread streams 8 consecutive segments (aligned vector loads),
// gathers the density (a 0.5-8 MB volume, L2/MALL resident), reduces runs between head bits in
// float64, and a block-level segmented scan stitches rows that cross thread chunks.  Balanced
// whatever the row lengths, ~3 dependent global round trips per workgroup, deterministic order.
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <stdlib.h>

#include "common.hpp"
#include "stage.hpp"

namespace sphrt {

constexpr uint32_t kHead = 0x80000000u;
constexpr int kThreads = 256;
constexpr int kFwdMinB64 = 5;   // resident float64 forward workgroups per CU the registers aim for
constexpr int kFwdMinB32 = 6;   // the same for float32
// Segments per forward thread: 8 (256-thread workgroups).  16 (128-thread ones: half the waves,
// so half the per-wave scan / close / address instructions for the same segments) measured for
// float32: C2 6.7 -> 7.7 us, C5 34.4 -> 37.6 us, C3 236 -> 241 us (the longer serial chain per
// thread costs more than the saved issue slots), so 8 everywhere.
// 64-bit min/max as plain selects (HIP's min<int64_t>/max<int64_t> went through double
// conversions on VALU even for uniform operands).
__host__ __device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ int64_t imax64(int64_t a, int64_t b) { return a > b ? a : b; }
constexpr int kPer = 8;                         // segments per thread per pass
constexpr int kPass = kThreads * kPer;          // 2048 segments per pass
constexpr int64_t kSegPerBlock = 1792;          // row starts per workgroup (leaves room
                                                // for the last row's overhang inside one pass)
// CSRs with dense output ranges (sphrt_csr.order bit 2: the time-paired transposed adjoint, rows
// of ~2 segments, one output per row or empty row) take blocks of 1984 row starts.  Blocks of
// 1920 for every CSR measured C4 adjoint kernel 24.9 -> 23.6 us but the forwards slower (C2 5.86
// -> 6.21 us, C5 34.1 -> 36.3; 1536 / 1664 slower everywhere; profiles/r06_spb_ab.jsonl); for the
// dense CSR alone, C4 adjoint 24.8-24.9 (1792) / 23.8-24.0 (1920) / 23.6-23.7 (1984) / 24.0-24.2
// us (2016), the rest unchanged (r06_dspb_ab.jsonl).  Indexed with sphrt_csr_index_dense /
// sphrt_csr_blocks_dense.
constexpr int64_t kDenseSegPerBlock = 1984;
constexpr int kBlockFields = 6;                 // empty_lo, empty_hi, seg_lo, seg_hi, row_lo, n_tab
constexpr int kLocalMax = 4096;                 // segments per workgroup with a granule table
constexpr int kMaxGran = 2046;                  // granules per table (sphrt_csr_local): loc's
                                                // 15-bit byte offsets reach 16*(2046+1)+12
constexpr int kGranEarly = 3;                   // table chunks of 256 fetched before the record
// Granule-table build modes: kTabCount — n_tab and the fallback decision only (stats); kTabFill —
// the tables of the blocks kTabCount kept, at a caller-chosen stride; kTabBuild — both in one
// pass, tables at the wide stride kTabWide (sphrt_csr_local_build), packed to the final stride
// afterwards (sphrt_csr_local_pack).
enum { kTabCount = 0, kTabFill = 1, kTabBuild = 2 };
constexpr int kTabWide = SPHRT_TAB_WIDE;
static_assert(kTabWide >= kMaxGran, "wide tables hold every table");


// ---- index --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mark_rows_kernel(const int64_t* row_ptr, int64_t n,
                                                        int32_t* vox, int32_t* nonempty) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t a = row_ptr[r];
    const bool ne = row_ptr[r + 1] > a;
    nonempty[r] = ne ? 1 : 0;
    if (ne && vox) vox[a] = (int32_t)((uint32_t)vox[a] | kHead);
}

__global__ __launch_bounds__(256) void row_list_kernel(const int64_t* row_ptr,
                                                       const int64_t* row_pre, int64_t n,
                                                       const int32_t* ray_ids, int32_t* row_ray,
                                                       int32_t* empty_ray, int32_t* nz_row) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int32_t id = ray_ids ? ray_ids[r] : (int32_t)r;   // the ray (output index) of row r
    if (row_ptr[r + 1] > row_ptr[r]) {
        row_ray[row_pre[r]] = id;
        if (nz_row) nz_row[row_pre[r]] = (int32_t)r;          // (staged index: the row itself)
    } else {
        empty_ray[r - row_pre[r]] = id;
    }
}

__global__ __launch_bounds__(256) void block_meta_kernel(const int64_t* row_ptr,
                                                         const int64_t* row_pre, int64_t n,
                                                         int64_t nblocks, int64_t spb,
                                                         int64_t* blocks) {
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
    const int64_t lo = first_at_or_after(b * spb);
    const int64_t hi = (b + 1 == nblocks) ? n : first_at_or_after((b + 1) * spb);
    int64_t* m = blocks + kBlockFields * b;
    // this block's share of the empty-ray list (split evenly, independent of the segments)
    const int64_t n_empty = n - row_pre[n];
    const int64_t e_chunk = (n_empty + nblocks - 1) / nblocks;
    m[0] = imin64(b * e_chunk, n_empty);
    m[1] = imin64((b + 1) * e_chunk, n_empty);
    m[2] = row_ptr[lo];
    m[3] = row_ptr[hi];
    m[4] = row_pre[lo];
    m[5] = -1;                                  // no granule table until sphrt_csr_local
}

// Row runs and empty ranges of block b (sphrt_csr_runs): one thread per block walks its rows'
// rays (row_ray[k0 .. k1)) and its share of the empty list, splitting both where the ray ids stop
// being consecutive.  More than kMaxRuns of either -> -1 and the block counts in stats.
constexpr int kRunFields = SPHRT_RUN_FIELDS;
constexpr int kMaxRuns = SPHRT_MAX_RUNS;
constexpr int kRunEmpty = 2 + 2 * kMaxRuns;           // first empty-range field
static_assert(kRunEmpty + 2 * kMaxRuns <= kRunFields, "run record layout");

__global__ __launch_bounds__(256) void block_runs_kernel(const int64_t* __restrict__ blocks,
                                                         const int32_t* __restrict__ row_ray,
                                                         const int32_t* __restrict__ empty_ray,
                                                         int64_t n_rays, int64_t nblocks,
                                                         int32_t* __restrict__ runs,
                                                         unsigned long long* stats) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblocks) return;
    const int64_t* m = blocks + kBlockFields * b;
    const int64_t n_rows = n_rays - blocks[kBlockFields * (nblocks - 1) + 1];   // all rows
    const int64_t k0 = m[4];
    const int64_t k1 = b + 1 < nblocks ? blocks[kBlockFields * (b + 1) + 4] : n_rows;
    int32_t* r = runs + kRunFields * b;
    bool over = false;
    int n = 0;
    for (int64_t k = k0; k < k1 && !over; ++k) {
        const int32_t ray = row_ray[k];
        if (k == k0 || ray != row_ray[k - 1] + 1) {
            if (n == kMaxRuns) { over = true; break; }
            r[2 + 2 * n] = (int32_t)(k - k0);
            r[3 + 2 * n] = ray;
            ++n;
        }
    }
    r[0] = over ? -1 : n;
    bool over_e = false;
    int ne = 0;
    int32_t start = 0, cnt = 0;
    for (int64_t j = m[0]; j < m[1]; ++j) {
        const int32_t ray = empty_ray[j];
        if (cnt > 0 && ray == start + cnt) { ++cnt; continue; }
        if (cnt > 0) {
            if (ne == kMaxRuns) { over_e = true; break; }
            r[kRunEmpty + 2 * ne] = start;
            r[kRunEmpty + 2 * ne + 1] = cnt;
            ++ne;
        }
        start = ray;
        cnt = 1;
    }
    if (!over_e && cnt > 0) {
        if (ne == kMaxRuns) over_e = true;
        else {
            r[kRunEmpty + 2 * ne] = start;
            r[kRunEmpty + 2 * ne + 1] = cnt;
            ++ne;
        }
    }
    r[1] = over_e ? -1 : ne;
    if (over || over_e) atomicAdd(stats, 1ull);
}

// Raise *p to v.  Most workgroups' values are below the running maximum, so a plain load of it
// (possibly stale, which is safe: the maximum only grows) skips their atomic — every one of the
// table kernels' 64 k workgroups (C3) would otherwise queue an atomic on the same address.
__device__ __forceinline__ void atomic_max_sparse(unsigned long long* p, unsigned long long v) {
    if (v > __atomic_load_n(p, __ATOMIC_RELAXED)) atomicMax(p, v);
}

// ---- block-level scans (256 threads = 4 waves) -----------------------------------------------
struct ScanShared {
    int cnt[4];
    int has[4];
    double sum[4];
};

// Wave-level inclusive scans on DPP lane moves (no LDS crossbar, no lane-index registers):
// row_shr 1, 2, 4, 8 within each row of 16 lanes, then row_bcast 15 (rows 1, 3) and row_bcast 31
// (rows 2, 3).  Lanes without a source read the identity: bound_ctrl zero for the full-row moves
// (no `old` register to clear), `old` = 0 for the row_bcast ones (rows outside ROWS keep it).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp0(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWS, 0xf, ROWS == 0xf);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp0(double x) {
    const uint64_t b = __double_as_longlong(x);
    const int lo = dpp0<CTRL, ROWS>((int)(uint32_t)b), hi = dpp0<CTRL, ROWS>((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
constexpr int kShr1 = 0x111, kShr2 = 0x112, kShr4 = 0x114, kShr8 = 0x118, kBcast15 = 0x142,
              kBcast31 = 0x143, kWaveShr1 = 0x138;

__device__ __forceinline__ int wave_incl_sum(int x) {
    x += dpp0<kShr1>(x);
    x += dpp0<kShr2>(x);
    x += dpp0<kShr4>(x);
    x += dpp0<kShr8>(x);
    x += dpp0<kBcast15, 0xa>(x);
    x += dpp0<kBcast31, 0xc>(x);
    return x;
}

// segmented element (h, s): (h1,s1) o (h2,s2) = (h1|h2, h2 ? s2 : s1+s2)
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ void seg_step(int& h, double& s) {
    const int hu = dpp0<CTRL, ROWS>(h);
    const double su = dpp0<CTRL, ROWS>(s);
    s = h ? s : su + s;
    h |= hu;
}

// exclusive sum of one int per thread; returns the block total in `total`
__device__ __forceinline__ int block_excl_count(int v, int& total, ScanShared& sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int inc = wave_incl_sum(v);
    if (lane == 63) sh.cnt[wid] = inc;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wid; ++w) base += sh.cnt[w];
    total = sh.cnt[0] + sh.cnt[1] + sh.cnt[2] + sh.cnt[3];
    __syncthreads();
    return base + inc - v;
}

// Segmented scan of (has_head, tail) per thread.  Returns the exclusive prefix sum value (the
// open run entering this thread) and the block total.
__device__ __forceinline__ double block_excl_segsum(bool has, double tail, bool& tot_has,
                                                    double& tot_sum, ScanShared& sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int h = has ? 1 : 0;
    double s = tail;
    seg_step<kShr1>(h, s);
    seg_step<kShr2>(h, s);
    seg_step<kShr4>(h, s);
    seg_step<kShr8>(h, s);
    seg_step<kBcast15, 0xa>(h, s);
    seg_step<kBcast31, 0xc>(h, s);
    const int eh = dpp0<kWaveShr1>(h);       // lane 0 reads the identity
    const double es = dpp0<kWaveShr1>(s);
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

// ---- one-barrier block scans for the forward ------------------------------------------------
// The wave totals go to one of two LDS slot sets chosen by the caller's pass parity, so the slots
// a scan reads are rewritten two scans later at the earliest, after barriers every thread has
// passed: no trailing barrier.  `lds_barrier` waits for LDS traffic only, so global loads issued
// before it (row prefetches, per-segment gathers) stay in flight across it.
struct FwdShared {
    alignas(16) int cnt[2][4];
    alignas(16) int has[2][4];
    alignas(16) double sum[2][4];
};

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool kDrain, int W = 4>   // kDrain: a full barrier (also retires LDS-DMA granule loads)
__device__ __forceinline__ int block_excl_count1(int v, int& total, int (&cnt)[4]) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int inc = wave_incl_sum(v);
    if (lane == 63) cnt[wid] = inc;
    if (kDrain) __syncthreads();
    else lds_barrier();
    const int4 c = *reinterpret_cast<const int4*>(cnt);     // one LDS read, no per-wave loop
    if constexpr (W == 2) {                                 // (slots 2, 3 unused)
        total = c.x + c.y;
        return (wid > 0 ? c.x : 0) + inc - v;
    }
    total = c.x + c.y + c.z + c.w;
    const int base = (wid > 0 ? c.x : 0) + (wid > 1 ? c.y : 0) + (wid > 2 ? c.z : 0);
    return base + inc - v;
}

template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp0(float x) {
    return __int_as_float(dpp0<CTRL, ROWS>(__float_as_int(x)));
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ void seg_step(int& h, float& s) {
    const int hu = dpp0<CTRL, ROWS>(h);
    const float su = dpp0<CTRL, ROWS>(s);
    s = h ? s : su + s;
    h |= hu;
}

// float32 forwards stitch a row's runs across threads in float too (the segmented scan's DPP
// steps and wave totals at half the width): C2 forward 6.68 -> 6.37 us, C5 28.3 -> 27.5 us, C3
// unchanged; largest relative difference from float64 accumulation 1.8e-7 -> 2.5e-7 (C2-C5,
// forward and adjoint).
template <int W = 4, typename S = double>
__device__ __forceinline__ S block_excl_segsum1(bool has, S tail, bool& tot_has,
                                                     S& tot_sum, int (&hs)[4],
                                                     double (&sm)[4]) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int h = has ? 1 : 0;
    S s = tail;
    seg_step<kShr1>(h, s);
    seg_step<kShr2>(h, s);
    seg_step<kShr4>(h, s);
    seg_step<kShr8>(h, s);
    seg_step<kBcast15, 0xa>(h, s);
    seg_step<kBcast31, 0xc>(h, s);
    const int eh = dpp0<kWaveShr1>(h);
    const S es = dpp0<kWaveShr1>(s);
    if (lane == 63) {
        hs[wid] = h;
        sm[wid] = (double)s;
    }
    lds_barrier();
    const int4 hv = *reinterpret_cast<const int4*>(hs);   // vector LDS reads, no per-wave loop
    const double2 s01 = *reinterpret_cast<const double2*>(sm);
    const double2 s23 = *reinterpret_cast<const double2*>(sm + 2);
    const int hw[4] = {hv.x, hv.y, W > 2 ? hv.z : 0, W > 2 ? hv.w : 0};   // (W = 2: 2, 3 unused)
    const S sw[4] = {(S)s01.x, (S)s01.y, W > 2 ? (S)s23.x : (S)0, W > 2 ? (S)s23.y : (S)0};
    S t[4];                                        // segmented prefix through wave w
    t[0] = sw[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) t[w] = hw[w] ? sw[w] : t[w - 1] + sw[w];
    const S cs = wid == 0 ? (S)0 : wid == 1 ? t[0] : wid == 2 ? t[1] : t[2];
    tot_sum = t[3];
    tot_has = (hw[0] | hw[1] | hw[2] | hw[3]) != 0;
    return eh ? es : cs + es;
}

// Per-segment arrays are readable up to the next multiple of 8 entries (sphrt.h), so every chunk
// that starts before s1 is one aligned 32-byte (vox) / 32- or 64-byte (len) vector load; entries
// outside [s0, s1) are masked to zero.  Pointers are pass-relative, offsets 32-bit.
template <typename L>
__device__ __forceinline__ void load_len8(const L* __restrict__ len, int p0, L (&l)[kPer]) {
    if constexpr (sizeof(L) == 4) {
        const float4* lp = reinterpret_cast<const float4*>(len + p0);
        const float4 f = lp[0], g = lp[1];
        l[0] = f.x; l[1] = f.y; l[2] = f.z; l[3] = f.w;
        l[4] = g.x; l[5] = g.y; l[6] = g.z; l[7] = g.w;
    } else {
        const double2* lp = reinterpret_cast<const double2*>(len + p0);
#pragma unroll
        for (int k = 0; k < kPer / 2; ++k) {
            const double2 f = lp[k];
            l[2 * k] = f.x;
            l[2 * k + 1] = f.y;
        }
    }
}

template <typename L>
__device__ __forceinline__ void mask8(int p0, int s0, int s1, uint32_t (&v)[kPer], L (&l)[kPer]) {
    const int first = s0 - p0, end = s1 - p0;   // chunk-relative window: compare against k
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (k < first || k >= end) {
            v[k] = 0u;
            l[k] = (L)0;
        }
}

template <typename L>
__device__ __forceinline__ void load8(const int32_t* __restrict__ vox, const L* __restrict__ len,
                                      int p0, int s0, int s1, uint32_t (&v)[kPer], L (&l)[kPer]) {
    if (p0 < s1) {
        const uint4* vp = reinterpret_cast<const uint4*>(vox + p0);
        const uint4 a = vp[0], b = vp[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        load_len8(len, p0, l);
        if (p0 < s0 || p0 + kPer > s1) mask8(p0, s0, s1, v, l);
    } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            v[k] = 0u;
            l[k] = (L)0;
        }
    }
}

// loc entry of a segment whose voxel v sits in granule `rank` of its workgroup's table: the
// byte offset of the voxel in the forward's float LDS image (granule 0 of which is a zero granule
// for masked slots, so table granule r sits at 16*(r+1)), and the row-head flag in bit 15.
__device__ __forceinline__ uint16_t loc_code(int rank, uint32_t v, bool head) {
    return (uint16_t)((16 * (rank + 1) + 4 * (int)(v & 3u)) | (head ? 0x8000 : 0));
}

// Columns the granule tables and the table-mode forward address.
static int64_t table_cols(const sphrt_csr* c) { return staged(c) ? c->stage_cols : c->n_cols; }

// dst[c * stage_cols + p] = src[c * cs + v] for the voxel v staged at column p (0 on pad
// columns).  One thread per brick row: ba voxels contiguous in both layouts (one 16-byte float
// vector when ba = 4 and the rows are 16-byte aligned), 4 integer divisions per row.
template <typename T>
__global__ __launch_bounds__(256) void stage_pack_kernel(const T* __restrict__ src, int64_t cs,
                                                         int64_t n_chan, uint32_t nr, StageMap m,
                                                         int64_t stage_cols, T* __restrict__ dst) {
    const uint32_t rows = m.br * m.be;                        // rows per brick
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= stage_cols / m.ba) return;
    const uint32_t blk = (uint32_t)t / rows, row = (uint32_t)t % rows;
    const uint32_t a0 = (blk % m.nba) * m.ba, q = blk / m.nba;
    const uint32_t e = (q % m.nbe) * m.be + row % m.be;
    const uint32_t r = (q / m.nbe) * m.br + row / m.be;
    const int64_t p0 = (int64_t)t * m.ba;
    const bool real = r < nr && e < m.ne;
    const int64_t v0 = ((int64_t)r * m.ne + e) * m.na + a0;
    const bool vec = m.ba == 4 && a0 + 4 <= m.na && (m.na & 3u) == 0 && (cs & 3) == 0 &&
                     (stage_cols & 3) == 0 && ((uintptr_t)src & 15) == 0;
    for (int64_t c = blockIdx.y; c < n_chan; c += gridDim.y) {
        const T* sr = src + c * cs + v0;
        T* dr = dst + c * stage_cols + p0;
        if (vec && real) {          // 16 (float) or 32 (double) aligned bytes
            const float4* s4 = reinterpret_cast<const float4*>(sr);
            float4* d4 = reinterpret_cast<float4*>(dr);
            d4[0] = s4[0];
            if constexpr (sizeof(T) == 8) d4[1] = s4[1];
        } else {
            for (uint32_t i = 0; i < m.ba; ++i) dr[i] = real && a0 + i < m.na ? sr[i] : (T)0;
        }
    }
}

// ---- per-workgroup granule table ----------------------------------------------------------
// Per-segment density gathers are the forward's bottleneck: every segment is one divergent 4-byte
// lane access, and the load path's per-lane rate, not bytes, bounds the kernel (C2: ~7 of 13 us).
// Built once per trace: for every workgroup b, the sorted distinct 4-voxel granules its segments
// read (tab[b*tab_stride ..+n_tab), granule g = voxels 4g..4g+3) and, per segment, the slot
// 4*rank + (voxel & 3) of its voxel, with the row-head flag in bit 15 (loc).  The forward stages
// the granules into LDS with 16-byte LDS-DMA loads (one lane per granule, ~3x fewer lane accesses
// than segments) and the segments read LDS.  n_tab = -1 marks a workgroup left on the
// per-segment gather (more than kLocalMax segments or kMaxGran granules).

// The float32 lengths (sphrt_csr.len32) written by the table launch that decides the tables
// (count / build), one block's segments per workgroup: the float32 forward's stream without a
// pass of its own over the float64 lengths (C3: f64_to_f32_kernel 0.25 ms).  The common block
// (<= 8 * kThreads segments) issues its eight loads before any store.
__device__ __forceinline__ void copy_len32(const double* __restrict__ len, float* __restrict__ len32,
                                           int64_t s0, int64_t n) {
    const int tid = threadIdx.x;
    if (n <= 8 * kThreads) {
        double v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = i * kThreads + tid;
            v[i] = p < n ? len[s0 + p] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = i * kThreads + tid;
            if (p < n) len32[s0 + p] = (float)v[i];
        }
        return;
    }
    for (int64_t p = tid; p < n; p += kThreads) len32[s0 + p] = (float)len[s0 + p];
}

// A one-pass trace's segments still in their staging slots (sphrt_trace_emit): the table build
// that reads them moves them into the CSR itself (sphrt_csr_local_build_staged) — no separate
// compaction pass (C3 compact_kernel 0.68 ms) and no second read of the voxels.
struct Staged {
    const int64_t* row_ptr;   // CSR row starts (the trace's rows)
    const int64_t* slot;      // staging slot starts (the scanned bounds)
    const int32_t* nz_row;    // the trace row of each non-empty row (sphrt_csr_index_staged)
    int64_t n_rays;           // rows (empty ones included)
    const int32_t* svox;      // staging voxels and lengths
    const double* slen;
    int32_t* vox;             // the CSR: voxels (with the row-head bits), lengths, float32 lengths
    double* len;
    float* len32;
};

// Block b's gather: its rows (non-empty rows [k0, k1), each starting in the block's window) as
// (start - s0, slot - start) in LDS when they fit in lds_cap bytes (else read from nz_row /
// row_ptr / slot in global memory: rare), then segment p of the block reads staging slot
// s0 + p + delta(row of p) (a binary search over the rows).  Thread t takes segments t,
// t + kThreads, ... (striped: every load and store instruction covers consecutive segments;
// thread t taking 8t .. 8t + 7 with one search and a walk measured C3 2.59 ms for gather +
// tables against 1.22 + 0.68 ms for tables + compaction: stride-8 accesses).  Writes vox (head
// bit on each row's first segment), len32 and (when S.len is set) len, and hands the block's voxels to the table
// build in registers when it has at most ITEMS * kThreads segments (xs[i]: segment
// i * kThreads + t; nothing is read back).
template <int ITEMS>
__device__ __forceinline__ void staged_gather(const Staged& S, const int64_t* blocks, int64_t nb,
                                              int64_t b, int64_t s0, int64_t n,
                                              unsigned char* lds, size_t lds_cap,
                                              uint32_t (&xs)[ITEMS]) {
    const int tid = threadIdx.x;
    const int64_t k0 = blocks[kBlockFields * b + 4];
    // (the last block's rows end at the non-empty row count: rays minus the empty list's end)
    const int64_t k1 = b + 1 < nb ? blocks[kBlockFields * (b + 1) + 4]
                                  : S.n_rays - blocks[kBlockFields * (nb - 1) + 1];
    const int nrow = (int)(k1 - k0);
    const size_t rs_bytes = ((size_t)(nrow + 1) * 4 + 7) & ~(size_t)7;
    const bool in_lds = rs_bytes + (size_t)nrow * 8 <= lds_cap;     // (block-uniform)
    int32_t* rs = reinterpret_cast<int32_t*>(lds);
    int64_t* rd = reinterpret_cast<int64_t*>(lds + rs_bytes);
    // grids of several waves of workgroups: each segment's row as a uint16 per segment, written
    // row by row (a wave per row, its lanes over the row's segments) instead of a binary search
    // over the row starts per segment (C3 table kernel 1120 -> 1107 us, C5 198 -> 190 us); a
    // one-wave grid (C2) is bound by each workgroup's chain, which the extra barrier lengthens
    // (35 -> 41 us), and keeps the search (profiles/r05_gather_ab.json)
    const bool rid_ok = nb > 256 * 6 && in_lds &&
                        rs_bytes + (size_t)nrow * 8 + (size_t)n * 2 <= lds_cap;
    uint16_t* rid = reinterpret_cast<uint16_t*>(lds + rs_bytes + (size_t)nrow * 8);
    if (in_lds) {
        for (int t = tid; t < nrow; t += kThreads) {
            const int64_t r = S.nz_row[k0 + t];
            const int64_t a = S.row_ptr[r];
            rs[t] = (int32_t)(a - s0);
            rd[t] = S.slot[r] - a;
        }
        if (tid == 0) rs[nrow] = (int32_t)n;      // sentinel: the end of the last row
    }
    __syncthreads();
    if (rid_ok) {
        const int lane = tid & 63;
        for (int t = tid >> 6; t < nrow; t += kThreads / 64)
            for (int p = rs[t] + lane, e = rs[t + 1]; p < e; p += 64) rid[p] = (uint16_t)t;
        __syncthreads();
    }
    auto start_of = [&](int t) -> int32_t {
        return in_lds ? rs[t] : (int32_t)(S.row_ptr[S.nz_row[k0 + t]] - s0);
    };
    auto row_of = [&](int p) {                    // last row t with start(t) <= p
        if (rid_ok) return (int)rid[p];
        int lo = 0, hi = nrow - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (start_of(mid) <= p) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    auto move = [&](int p, int row) {
        int32_t st;
        int64_t dl;
        if (in_lds) {
            st = rs[row];
            dl = rd[row];
        } else {
            const int64_t r = S.nz_row[k0 + row];
            const int64_t a = S.row_ptr[r];
            st = (int32_t)(a - s0);
            dl = S.slot[r] - a;
        }
        const int64_t src = s0 + p + dl;
        const uint32_t v = (uint32_t)S.svox[src];
        const double l = S.slen[src];
        const uint32_t x = p == st ? (v | kHead) : v;
        S.vox[s0 + p] = (int32_t)x;
        if (S.len) S.len[s0 + p] = l;            // (NULL: the float64 lengths stay in slen)
        S.len32[s0 + p] = (float)l;
        return x;
    };
    if (n <= ITEMS * kThreads) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const int p = i * kThreads + tid;
            xs[i] = p < n ? move(p, row_of(p)) : 0u;
        }
    } else {
        for (int p = tid; p < n; p += kThreads) move(p, row_of(p));
    }
    __syncthreads();                              // (the LDS is reused by the table build)
}

// The tables from a bitmap of the volume's granules in LDS, when the
// bitmap is small (n_cols/4 bits; 128^3 voxels = 64 KiB): set one bit per segment, prefix-popcount
// the words, and a granule's rank is the number of set bits below it.  O(segments + words) per
// workgroup, a handful of barriers.  Identical output to the sort (ascending distinct granules).
template <int TM, typename TabT = int32_t>
__global__ __launch_bounds__(kThreads) void local_table_bitmap_kernel(
    int64_t* __restrict__ blocks, const int32_t* __restrict__ vox, uint16_t* __restrict__ loc,
    TabT* __restrict__ tab, int64_t tab_stride, int n_words, StageMap sm,
    unsigned long long* stats, const double* __restrict__ len, float* __restrict__ len32,
    Staged S = Staged{}, int64_t n_blocks = 0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char bm_lds[];
    uint32_t* bm = reinterpret_cast<uint32_t*>(bm_lds);     // n_words bitmap words
    int32_t* pre = reinterpret_cast<int32_t*>(bm + n_words);  // set bits before each word
    __shared__ ScanShared sh;
    int64_t* m = blocks + kBlockFields * (int64_t)blockIdx.x;
    const int64_t s0 = m[2], s1 = m[3];
    if (TM == kTabFill && m[5] < 0) return;
    const int tid = threadIdx.x;
    const int64_t n = s1 - s0;
    // staged: every block's segments moved out of the staging (rows in the bitmap's LDS when
    // they fit), its table blocks' voxels kept in registers (kLocalMax = 16 * kThreads)
    constexpr int kXs = kLocalMax / kThreads;
    static_assert(kXs * kThreads == kLocalMax, "a table block's voxels fit the registers");
    uint32_t xs[kXs];
    const bool staged = TM == kTabBuild && S.svox;
    if (staged) staged_gather<kXs>(S, blocks, n_blocks, blockIdx.x, s0, n, bm_lds,
                                   (size_t)n_words * 8, xs);
    else if (TM != kTabFill && len32) copy_len32(len, len32, s0, n);
    auto vox_at = [&](int k, int i) {            // segment i = k * kThreads + tid
        return staged ? xs[k] : (uint32_t)vox[s0 + i];
    };
    if (n > kLocalMax) {
        if (TM != kTabFill && tid == 0) {
            m[5] = -1;
            atomicAdd(stats, 1ull);
        }
        return;
    }
    for (int w = tid; w < n_words; w += kThreads) bm[w] = 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kXs; ++k) {
        const int i = k * kThreads + tid;
        if (i < n) {
            const uint32_t g = stage_col(vox_at(k, i) & ~kHead, sm) >> 2;
            atomicOr(&bm[g >> 5], 1u << (g & 31));
        }
    }
    __syncthreads();
    // thread t owns words [t*per, (t+1)*per)
    const int per = (n_words + kThreads - 1) / kThreads;
    const int w0 = min(tid * per, n_words), w1 = min(w0 + per, n_words);
    int cnt = 0;
    for (int w = w0; w < w1; ++w) cnt += __builtin_popcount(bm[w]);
    int n_tab;
    int run = block_excl_count(cnt, n_tab, sh);
    if (TM != kTabFill) {
        if (tid == 0) {
            if (n_tab > kMaxGran) {
                m[5] = -1;
                atomicAdd(stats, 1ull);
            } else {
                m[5] = n_tab;
                atomic_max_sparse(stats + 1, (unsigned long long)n_tab);
            }
        }
        if (TM == kTabCount || n_tab > kMaxGran) return;
    }
    TabT* tab_b = tab + (int64_t)blockIdx.x * tab_stride;
    for (int w = w0; w < w1; ++w) {
        pre[w] = run;
        uint32_t bits = bm[w];
        while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1;
            tab_b[run++] = (TabT)(w * 32 + b);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kXs; ++k) {
        const int i = k * kThreads + tid;
        if (i < n) {
            const uint32_t x = vox_at(k, i);
            const uint32_t v = stage_col(x & ~kHead, sm), g = v >> 2;
            const int rank = pre[g >> 5] + __builtin_popcount(bm[g >> 5] & ((1u << (g & 31)) - 1u));
            loc[s0 + i] = loc_code(rank, v, (x & kHead) != 0);
        }
    }
}

// Large volumes (the bitmap would not fit, or costs more than the segments): the same tables
// from a block radix sort of the workgroup's segments by granule (hipCUB, 16 per thread), value
// = position << 3 | head << 2 | voxel & 3.  O(segments · key bits) per workgroup instead of
// O(volume): at C3 (2 M voxels, 64 k workgroups) 10.6 ms of bitmap work.  Identical output.
// 10 bits per pass (rocprim's match ranking): C3's 19-bit granule keys in 2 passes instead of
// the default 8-bit 3 (local_table_radix_kernel 1324 -> 1240 us; 6 bits: 1404 us).
constexpr int kRadixBits = 10;
// RB: bits per pass.  10 for the grids whose blocks all take the sort; 8 (a third pass, but 8 KB
// of sort storage instead of 33 KB) behind the bucket tables, which leave the sort only the rare
// block of many buckets: the kernel's LDS then fits 7 workgroups per CU instead of 4.
template <int ITEMS, int TM, int RB = kRadixBits>
struct RadixTable {
    // the count pass sorts keys only (its values are dead)
    using Sort = typename std::conditional<
        TM != kTabCount,
        rocprim::block_radix_sort<uint32_t, kThreads, ITEMS, uint16_t, 1, 1, RB>,
        rocprim::block_radix_sort<uint32_t, kThreads, ITEMS, rocprim::empty_type, 1, 1,
                                  RB>>::type;
    using Storage = typename Sort::storage_type;
};

// One block's table from a two-level bitmap of its granules (the sort's result without a sort):
// level 1 marks the occupied buckets of 512 granules (granule >> 9 < 4096: 128 words), its prefix
// popcounts give each occupied bucket a slot; level 2 is one 16-word bitmap per slot.  A thread
// per slot popcounts its bucket, one block scan ranks the buckets, and a granule's rank is its
// bucket's base + the set bits below it.  Ascending distinct granules, the same tables and loc as
// the sort.  A C3 block (1792 segments, ~640 granules) touches ~52 buckets (max ~90 in a traced
// view): blocks with more than kBucketSlots of them, or keys of more than 21 bits, return false
// and take the sort.  At run time SPHRT_TABLE_BUCKETS=0 sorts every block (tests: bucket tables
// == sorted tables), the launch marking key_bits with kSortOnly.
constexpr int kBucketLo = 9;                       // granules per bucket: 512 = 16 words
constexpr int kBucketWords = 1 << (kBucketLo - 5);
constexpr int kBucketL1 = 128;                     // level-1 words: buckets < 4096
constexpr int kBucketSlots = 128;
constexpr int kSortOnly = 256;                     // key_bits flag: no bucket tables
constexpr size_t kBucketLds = (2 * kBucketL1 + 4) * 4 + (size_t)kBucketSlots * kBucketWords * 6;
template <int ITEMS, int TM, typename TabT>
__device__ __forceinline__ bool bucket_table(int64_t* m, const int32_t* __restrict__ vox,
                                             uint16_t* __restrict__ loc, TabT* __restrict__ tab_b,
                                             int64_t s0, int n, int key_bits, const StageMap& sm,
                                             unsigned char* lds, ScanShared& sh,
                                             unsigned long long* stats, const uint32_t* xin) {
    if (key_bits > kBucketLo + 12) return false;
    const int tid = threadIdx.x;
    uint32_t* l1 = reinterpret_cast<uint32_t*>(lds);
    int* pre1 = reinterpret_cast<int*>(l1 + kBucketL1);          // kBucketL1 + 1 (total last)
    uint32_t* l2 = reinterpret_cast<uint32_t*>(pre1 + kBucketL1 + 4);
    uint16_t* pre2 = reinterpret_cast<uint16_t*>(l2 + kBucketSlots * kBucketWords);
    uint32_t gk[ITEMS];                           // granule, or ~0 past the block's segments
    uint32_t va = 0u, hb = 0u;                    // voxel-in-granule (2 bits) and head bit each
    static_assert(ITEMS <= 16, "two bits per item in one dword");
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int p = xin ? i * kThreads + tid : tid * ITEMS + i;
        gk[i] = 0xffffffffu;
        if (p < n) {
            const uint32_t x = xin ? xin[i] : (uint32_t)vox[s0 + p];
            const uint32_t v = stage_col(x & ~kHead, sm);
            gk[i] = v >> 2;
            va |= (v & 3u) << (2 * i);
            hb |= (x >> 31) << i;
        }
    }
    if (tid < kBucketL1) l1[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        if (gk[i] != 0xffffffffu) {
            const uint32_t hi = gk[i] >> kBucketLo;
            atomicOr(&l1[hi >> 5], 1u << (hi & 31));
        }
    }
    __syncthreads();
    if (tid < 64) {                               // wave 0: slots of the occupied buckets
        static_assert(kBucketL1 == 128, "two level-1 words per lane");
        const int a = __builtin_popcount(l1[2 * tid]), c = a + __builtin_popcount(l1[2 * tid + 1]);
        const int inc = wave_incl_sum(c);
        pre1[2 * tid] = inc - c;
        pre1[2 * tid + 1] = inc - c + a;
        if (tid == 63) pre1[kBucketL1] = inc;
    }
    __syncthreads();
    const int nbk = pre1[kBucketL1];
    if (nbk > kBucketSlots) {
        __syncthreads();                          // (the sort reuses the LDS)
        return false;
    }
    for (int w = tid; w < nbk * kBucketWords; w += kThreads) l2[w] = 0u;
    __syncthreads();
    uint32_t slot_w[ITEMS];                       // level-2 word of each segment's granule
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        slot_w[i] = 0u;
        if (gk[i] != 0xffffffffu) {
            const uint32_t hi = gk[i] >> kBucketLo, lo = gk[i] & ((1u << kBucketLo) - 1u);
            const uint32_t w1 = l1[hi >> 5];
            const int slot = pre1[hi >> 5] + __builtin_popcount(w1 & ((1u << (hi & 31)) - 1u));
            slot_w[i] = (uint32_t)slot * kBucketWords + (lo >> 5);
            atomicOr(&l2[slot_w[i]], 1u << (lo & 31));
        }
    }
    __syncthreads();
    int cnt = 0;
    if (tid < nbk) {
#pragma unroll
        for (int j = 0; j < kBucketWords; ++j) cnt += __builtin_popcount(l2[tid * kBucketWords + j]);
    }
    int n_tab;
    int run = block_excl_count(cnt, n_tab, sh);
    if (TM != kTabFill) {
        if (tid == 0) {
            if (n_tab > kMaxGran) {
                m[5] = -1;
                atomicAdd(stats, 1ull);
            } else {
                m[5] = n_tab;
                atomic_max_sparse(stats + 1, (unsigned long long)n_tab);
            }
        }
        if (TM == kTabCount || n_tab > kMaxGran) return true;
    }
    if (tid < nbk) {
        int w = 0;                                // level-1 word holding occupied bucket `tid`
#pragma unroll
        for (int step = kBucketL1 / 2; step > 0; step >>= 1)
            if (w + step < kBucketL1 && pre1[w + step] <= tid) w += step;
        uint32_t bits = l1[w];
        for (int k = tid - pre1[w]; k > 0; --k) bits &= bits - 1;   // its (tid - pre1[w])-th bit
        const uint32_t hi = (uint32_t)w * 32 + (uint32_t)__builtin_ctz(bits);
        for (int j = 0; j < kBucketWords; ++j) {
            pre2[tid * kBucketWords + j] = (uint16_t)run;
            uint32_t b = l2[tid * kBucketWords + j];
            while (b) {
                const int k = __builtin_ctz(b);
                b &= b - 1;
                tab_b[run++] = (TabT)((hi << kBucketLo) | (uint32_t)(j * 32 + k));
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        if (gk[i] != 0xffffffffu) {
            const int p = xin ? i * kThreads + tid : tid * ITEMS + i;
            const uint32_t lo = gk[i] & 31u;
            const int rank = pre2[slot_w[i]] + __builtin_popcount(l2[slot_w[i]] & ((1u << lo) - 1u));
            loc[s0 + p] = loc_code(rank, (va >> (2 * i)) & 3u, ((hb >> i) & 1u) != 0);
        }
    }
    return true;
}

// One block's table from a sort of its n <= ITEMS * kThreads segments (block-uniform call).
// xin: the block's voxels already in registers (xin[i]: segment i * kThreads + t, the staged
// gather's striped order — the sort takes any arrangement, each value carries its position),
// else loaded from vox (segment ITEMS * t + i).
template <int ITEMS, int TM, typename TabT, int RB = kRadixBits>
__device__ __forceinline__ void radix_table(int64_t* m, const int32_t* __restrict__ vox,
                                            uint16_t* __restrict__ loc, TabT* __restrict__ tab_b,
                                            int64_t s0, int n, int key_bits, const StageMap& sm,
                                            unsigned char* ts_raw, uint32_t* last_key,
                                            ScanShared& sh, unsigned long long* stats,
                                            const uint32_t* xin = nullptr) {
    if (bucket_table<ITEMS, TM, TabT>(m, vox, loc, tab_b, s0, n, key_bits, sm, ts_raw, sh, stats,
                                      xin))
        return;
    using RT = RadixTable<ITEMS, TM, RB>;
    auto& ts = *reinterpret_cast<typename RT::Storage*>(ts_raw);
    const int tid = threadIdx.x;
    uint32_t key[ITEMS];
    uint16_t val[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int p = xin ? i * kThreads + tid : tid * ITEMS + i;
        key[i] = 0xffffffffu;                     // padding sorts last
        val[i] = 0;
        if (p < n) {
            const uint32_t x = xin ? xin[i] : (uint32_t)vox[s0 + p];
            const uint32_t v = stage_col(x & ~kHead, sm);
            key[i] = v >> 2;
            val[i] = (uint16_t)((p << 3) | ((x >> 31) << 2) | (v & 3u));
        }
    }
    const int kbits = key_bits & (kSortOnly - 1);
    if constexpr (TM != kTabCount) typename RT::Sort().sort(key, val, ts, 0, kbits);  // blocked:
    else typename RT::Sort().sort(key, ts, 0, kbits);         // thread t: [ITEMS t, ITEMS t + ITEMS)
    last_key[tid] = key[ITEMS - 1];
    __syncthreads();
    uint32_t prev = tid > 0 ? last_key[tid - 1] : 0xffffffffu;
    int first_new = 0;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int p = tid * ITEMS + i;
        const bool fresh = p < n && (p == 0 || key[i] != prev);
        first_new += fresh ? 1 : 0;
        prev = key[i];
    }
    int n_tab;
    int rank = block_excl_count(first_new, n_tab, sh) - 1;
    if (TM != kTabFill) {
        if (tid == 0) {
            if (n_tab > kMaxGran) {
                m[5] = -1;
                atomicAdd(stats, 1ull);
            } else {
                m[5] = n_tab;
                atomic_max_sparse(stats + 1, (unsigned long long)n_tab);
            }
        }
        if (TM == kTabCount || n_tab > kMaxGran) return;
    }
    prev = tid > 0 ? last_key[tid - 1] : 0xffffffffu;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int p = tid * ITEMS + i;
        if (p < n) {
            if (p == 0 || key[i] != prev) {
                ++rank;
                tab_b[rank] = (TabT)key[i];
            }
            const uint32_t w = val[i];
            loc[s0 + (w >> 3)] = loc_code(rank, w & 3u, (w >> 2) & 1u);
        }
        prev = key[i];
    }
}

// Blocks of up to 2048 segments (most: a block owns the rows starting in 1792 segments) sort 8
// keys per thread, larger ones 16: half the sort work for the common case.  (An LDS hash set
// that deduplicated the granules before a smaller sort measured slower at C3, 1268 -> 1503 us,
// and was removed in round 4.)  Blocks of more than 2048 segments (the last row's overhang; few) are left
// to local_table_big_kernel: apart, this kernel is sized for the 8-key sort's registers (72
// VGPRs, 7 waves per SIMD instead of 4 with the 16-key sort inline: C3 1244 -> 1120 us).  With
// the bucket tables (round 4) 8 waves per SIMD: C3 1341 -> 1285 us.
constexpr int kTabWaves = 8;   // minimum waves per SIMD the 8-key table kernel's registers aim for
template <int TM, typename TabT, int ITEMS, int RB = kRadixBits>
constexpr size_t table_lds() {
    const size_t sort = sizeof(typename RadixTable<ITEMS, TM, RB>::Storage);
    return sort > kBucketLds ? sort : kBucketLds;
}
template <int TM, typename TabT = int32_t, int RB = kRadixBits>
__global__ __launch_bounds__(kThreads, kTabWaves) void local_table_radix_kernel(
    int64_t* __restrict__ blocks, const int32_t* __restrict__ vox, uint16_t* __restrict__ loc,
    TabT* __restrict__ tab, int64_t tab_stride, int key_bits, StageMap sm,
    unsigned long long* stats, const double* __restrict__ len, float* __restrict__ len32,
    Staged S = Staged{}, int64_t n_blocks = 0) {
    // (the staged gather's rows share it: up to ~1060 rows per block in LDS, more from global
    // memory — a C3 block has ~13)
    __shared__ __attribute__((aligned(16))) unsigned char ts_raw[table_lds<TM, TabT, 8, RB>()];
    __shared__ uint32_t last_key[kThreads];
    __shared__ ScanShared sh;
    int64_t* m = blocks + kBlockFields * (int64_t)blockIdx.x;
    const int64_t s0 = m[2], s1 = m[3];
    if (TM == kTabFill && m[5] < 0) return;
    const int64_t n = s1 - s0;
    // every block's segments / lengths, whichever launch then builds its table (or none)
    uint32_t xs[8];
    const bool staged = TM == kTabBuild && S.svox;
    if (staged) staged_gather<8>(S, blocks, n_blocks, blockIdx.x, s0, n, ts_raw, sizeof(ts_raw), xs);
    else if (TM != kTabFill && len32) copy_len32(len, len32, s0, n);
    if (n > kLocalMax) {
        if (TM != kTabFill && threadIdx.x == 0) {
            m[5] = -1;
            atomicAdd(stats, 1ull);
        }
        return;
    }
    if (n > 8 * kThreads) return;                 // local_table_big_kernel's
    TabT* tab_b = tab + (int64_t)blockIdx.x * tab_stride;
    radix_table<8, TM, TabT, RB>(m, vox, loc, tab_b, s0, (int)n, key_bits, sm, ts_raw, last_key, sh,
                             stats, staged ? xs : nullptr);
}

// The blocks of 2049..kLocalMax segments: workgroup g looks at blocks [kBigScan g, kBigScan g +
// kBigScan) one per thread and sorts the big ones among them in turn (16 keys per thread).  A
// grid of n_blocks / kBigScan workgroups (C3: ~6 % of the blocks are big; 256 blocks per
// workgroup left ~25 sorts in series per workgroup, 110 us).
constexpr int kBigScan = 32;
template <int TM, typename TabT = int32_t, int RB = kRadixBits>
__global__ __launch_bounds__(kThreads) void local_table_big_kernel(
    int64_t* __restrict__ blocks, int64_t n_blocks, const int32_t* __restrict__ vox,
    uint16_t* __restrict__ loc, TabT* __restrict__ tab, int64_t tab_stride, int key_bits,
    StageMap sm, unsigned long long* stats) {
    __shared__ __attribute__((aligned(16))) unsigned char ts_raw[table_lds<TM, TabT, 16, RB>()];
    __shared__ uint32_t last_key[kThreads];
    __shared__ ScanShared sh;
    __shared__ int n_big;
    __shared__ int32_t big[kBigScan];
    if (threadIdx.x == 0) n_big = 0;
    __syncthreads();
    const int64_t b = (int64_t)blockIdx.x * kBigScan + threadIdx.x;
    if (threadIdx.x < kBigScan && b < n_blocks) {
        const int64_t* m = blocks + kBlockFields * b;
        const int64_t n = m[3] - m[2];
        if (n > 8 * kThreads && n <= kLocalMax && (TM != kTabFill || m[5] >= 0))
            big[atomicAdd(&n_big, 1)] = threadIdx.x;
    }
    __syncthreads();
    const int nb = n_big;
    for (int i = 0; i < nb; ++i) {
        const int64_t bb = (int64_t)blockIdx.x * kBigScan + big[i];
        int64_t* m = blocks + kBlockFields * bb;
        const int64_t s0 = m[2];
        radix_table<16, TM, TabT, RB>(m, vox, loc, tab + bb * tab_stride, s0, (int)(m[3] - s0),
                                  key_bits, sm, ts_raw, last_key, sh, stats);
        __syncthreads();                          // the sort storage is reused by the next one
    }
}

// Wide tables (one-pass build, kTabWide entries per block) -> the final stride.
template <typename TabT>
__global__ __launch_bounds__(kThreads) void table_pack_kernel(const int64_t* __restrict__ blocks,
                                                              const TabT* __restrict__ wide,
                                                              TabT* __restrict__ tab,
                                                              int64_t tab_stride) {
    const int64_t b = blockIdx.x;
    const int64_t n_tab = blocks[kBlockFields * b + 5];
    for (int64_t i = threadIdx.x; i < n_tab; i += kThreads)
        tab[b * tab_stride + i] = wide[b * kTabWide + i];
}

// LDS image of a workgroup's granule table: granule 0 is zero (the read of every masked slot),
// table granule r at granules r+1; float 16 B and double 32 B per granule, contiguous, so a
// segment's loc offset x (bits 0-14) is its voxel's byte offset for float and half of it for
// double.  Each 16-byte LDS-DMA lane carries a whole float granule or half a double one: DMA
// round r of wave w covers table entries gran_entry(r, w, lane) (64/G granules, G lanes each).
template <typename T>
constexpr int kGranLanes = (int)sizeof(T) / 4;        // 16-byte DMA lanes per granule
// Early rounds cover kGranEarly chunks of 256 table entries whatever the workgroup size (THR
// threads: a round moves THR / G granules).
template <typename T, int THR = kThreads, int GE = kGranEarly>
constexpr int kEarlyRounds = GE * (256 / THR) * kGranLanes<T>;

template <typename T, int THR = kThreads>
__device__ __forceinline__ int gran_entry0(int r, int w) {    // first entry of round r (uniform)
    constexpr int G = kGranLanes<T>;
    return (r / G) * THR + w * 64 + (r % G) * (64 / G);
}

template <typename T>
__device__ __forceinline__ T lds_at(const T* dens, uint32_t x) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(dens) + x * (sizeof(T) / 4));
}

// One DMA lane: granule g (its index in the channel; the byte offset is 32-bit: volumes under
// 4 GiB per channel), into the round whose first table entry is e0.
template <typename T>
__device__ __forceinline__ void stage_one(const T* __restrict__ rho, int32_t g, int e0, int lane,
                                          T* dens) {
    constexpr int G = kGranLanes<T>;
    const char* src = reinterpret_cast<const char*>(rho) + (uint32_t)g * (16u * G) +
                      16 * (lane % G);
    __builtin_amdgcn_global_load_lds((const void*)src,
        (__attribute__((address_space(3))) void*)(dens + 4 * (e0 + 1)), 16, 0, 0);
}

// The volume's last granule, if partial (voxel count not a multiple of 4), can only be the
// table's last entry: the DMA skips it (no read past the volume) and one lane copies it here.
template <typename T, typename TabT, int THR = kThreads>
__device__ __forceinline__ void stage_partial_tail(const T* __restrict__ rho,
                                                   const TabT* __restrict__ tab_b, int n_tab,
                                                   int64_t n_cols, T* dens) {
    if ((n_cols & 3) != 0 && n_tab > 0 && (int)threadIdx.x == (n_tab - 1) % THR) {
        const int j = n_tab - 1;
        const int64_t v0 = 4 * (int64_t)tab_b[j];
        if (v0 + 4 > n_cols)
            for (int i = 0; i < 4; ++i) dens[4 * (j + 1) + i] = v0 + i < n_cols ? rho[v0 + i] : (T)0;
    }
}

// DMA rounds [r0, ..) of the table, entries read from memory one round at a time.
template <typename T, typename TabT, int THR = kThreads>
__device__ __forceinline__ void stage_granules_late(const T* __restrict__ rho,
                                                    const TabT* __restrict__ tab_b, int r0,
                                                    int n_tab, int32_t g_full, T* dens) {
    constexpr int G = kGranLanes<T>;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int r = r0; (r / G) * THR < n_tab; ++r) {
        const int e0 = gran_entry0<T, THR>(r, w);
        const int e = e0 + lane / G;
        if (e < n_tab) {
            const int32_t g = (int32_t)tab_b[e];
            if (g < g_full) stage_one<T>(rho, g, e0, lane, dens);
        }
    }
}

// Rounds [0, kEarlyRounds) come from the table entries fetched early (ti); any beyond that
// (large tables) are fetched here.  When the volume's voxel count is not a multiple of 4 its
// last granule is partial: only the table's last entry can be, it is skipped by the DMA (no read
// past the volume) and copied lane by lane at the end.  Writes the zero granule.
template <typename T, typename TabT, int THR = kThreads, int GE = kGranEarly>
__device__ __forceinline__ void stage_granules(const T* __restrict__ rho,
                                               const int32_t (&ti)[kEarlyRounds<T, THR, GE>],
                                               const TabT* __restrict__ tab_b, int n_tab,
                                               int32_t g_full, int64_t n_cols, T* dens) {
    constexpr int G = kGranLanes<T>;
    constexpr int R = kEarlyRounds<T, THR, GE>;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 4) dens[threadIdx.x] = (T)0;
    // every early table entry is consumed before the first DMA goes out (one wait, not one per
    // DMA: the wait-count model serialises VMEM results read after an LDS-DMA)
#pragma unroll
    for (int r = 0; r < R; ++r) asm volatile("" ::"v"(ti[r]));
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e0 = gran_entry0<T, THR>(r, w);
        if (e0 + lane / G < n_tab && ti[r] < g_full) stage_one<T>(rho, ti[r], e0, lane, dens);
    }
    stage_granules_late<T, TabT, THR>(rho, tab_b, R, n_tab, g_full, dens);
    stage_partial_tail<T, TabT, THR>(rho, tab_b, n_tab, n_cols, dens);
}

// Early DMA (forward_kernel<..., EDMA = true>): the early rounds go out as a fixed number of
// unconditional LDS-DMAs right after the table entries arrive, before the first segment chunk is
// decoded — every lane of every round issues (lanes past the table re-read granule 0 into slots
// past the table, inside the LDS image), so the wait-count model knows exactly how many DMAs
// follow the chunk's loads and waits for the chunk alone; the DMA round trip then overlaps the
// chunk's arrival instead of following it.  Needs whole granules (columns % 4 == 0: no partial
// tail granule) and an LDS image of at least kGranEarly * 256 granules.
template <typename T, int THR = kThreads, int GE = kGranEarly>
__device__ __forceinline__ void stage_granules_early(const T* __restrict__ rho,
                                                     const int32_t (&ti)[kEarlyRounds<T, THR, GE>],
                                                     int n_tab, T* dens) {
    constexpr int G = kGranLanes<T>;
    constexpr int R = kEarlyRounds<T, THR, GE>;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 4) dens[threadIdx.x] = (T)0;
#pragma unroll
    for (int r = 0; r < R; ++r) asm volatile("" ::"v"(ti[r]));
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e0 = gran_entry0<T, THR>(r, w);
        const int32_t g = e0 + lane / G < n_tab ? ti[r] : 0;
        stage_one<T>(rho, g, e0, lane, dens);
    }
}

// Segment-stream loads (read once per launch; non-temporal loads measured C3 f64 375 -> 506 us).
__device__ __forceinline__ uint4 stream_load(const uint4* p) { return *p; }

// Segment lengths of one chunk of P segments as aligned 16-byte vectors.
template <typename L, int P>
__device__ __forceinline__ void load_lens(const L* __restrict__ len, L (&l)[P]) {
    constexpr int E = 16 / (int)sizeof(L);      // lengths per 16-byte vector
    const uint4* lp = reinterpret_cast<const uint4*>(len);
#pragma unroll
    for (int k = 0; k < P / E; ++k) {
        const uint4 f = stream_load(lp + k);
        const uint32_t w[4] = {f.x, f.y, f.z, f.w};
        if constexpr (sizeof(L) == 4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) l[4 * k + i] = __uint_as_float(w[i]);
        } else {
            l[2 * k] = __longlong_as_double((long long)(((uint64_t)w[1] << 32) | w[0]));
            l[2 * k + 1] = __longlong_as_double((long long)(((uint64_t)w[3] << 32) | w[2]));
        }
    }
}

// The first pass's loads, issued before anything is known about the workgroup and decoded
// later (raw registers keep the compiler from waiting on them early).  P segments per thread:
// loc half-words (8 per 16-byte vector) or vox words (4 per vector), and their lengths.
template <typename L, bool LOCAL, int P = kPer>
struct RawChunk {
    uint4 ix[LOCAL ? P / 8 : P / 4];
    L l[P];
};

template <typename L, bool LOCAL, int P = kPer>
__device__ __forceinline__ void raw_load(const int32_t* __restrict__ vox,
                                         const uint16_t* __restrict__ loc,
                                         const L* __restrict__ len, int64_t a,
                                         RawChunk<L, LOCAL, P>& r) {
    // unconditional (the caller clamps `a` into the arrays; chunks outside the window are masked
    // by window_chunk): no branch, so no copy of a load result that would wait for it early
    const uint4* ip = LOCAL ? reinterpret_cast<const uint4*>(loc + a)
                            : reinterpret_cast<const uint4*>(vox + a);
#pragma unroll
    for (int k = 0; k < (LOCAL ? P / 8 : P / 4); ++k) r.ix[k] = stream_load(ip + k);
    load_lens<L, P>(len + a, r.l);
}

// Bits [first, end) of a chunk of P segments (chunk-relative segment window).
template <int P = kPer>
__device__ __forceinline__ uint32_t window_bits(int first, int end) {
    const int a = max(first, 0), b = min(end, P);
    return a < b ? (uint32_t)(((1ull << b) - 1ull) & ~((1ull << a) - 1ull)) : 0u;
}

// A chunk's segment columns: table mode keeps the loc half-words packed two per register (head
// bits cleared; slot k = LDS byte offset of its voxel, vslot()), otherwise the vox words.
template <bool LOCAL, int P = kPer>
constexpr int kVW = LOCAL ? P / 2 : P;

template <bool LOCAL, int P = kPer>
__device__ __forceinline__ uint32_t vslot(const uint32_t (&v)[kVW<LOCAL, P>], int k) {
    if constexpr (LOCAL) return (v[k >> 1] >> (16 * (k & 1))) & 0xffffu;
    else return v[k];
}

// Decode a raw chunk; returns the row heads of the chunk (bit k = segment k).
template <typename L, bool LOCAL, int P = kPer>
__device__ __forceinline__ uint32_t decode(const RawChunk<L, LOCAL, P>& r,
                                           uint32_t (&v)[kVW<LOCAL, P>], L (&l)[P]) {
    uint32_t hmask = 0;
    if constexpr (LOCAL) {
#pragma unroll
        for (int q = 0; q < P / 8; ++q) {
            const uint32_t w[4] = {r.ix[q].x, r.ix[q].y, r.ix[q].z, r.ix[q].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * q + j] = w[j] & 0x7ffc7ffcu;
            // bit 15 of half-word k -> bit k: even k to bits 0,2,4,6, odd k to 16,18,20,22,
            // folded
            const uint32_t h = ((w[0] >> 15) & 0x10001u) | ((w[1] >> 13) & 0x40004u) |
                               ((w[2] >> 11) & 0x100010u) | ((w[3] >> 9) & 0x400040u);
            hmask |= ((h | (h >> 15)) & 0xffu) << (8 * q);
        }
    } else {
#pragma unroll
        for (int q = 0; q < P / 4; ++q) {
            v[4 * q] = r.ix[q].x; v[4 * q + 1] = r.ix[q].y;
            v[4 * q + 2] = r.ix[q].z; v[4 * q + 3] = r.ix[q].w;
        }
#pragma unroll
        for (int k = 0; k < P; ++k) hmask |= (v[k] >> 31) << k;
    }
#pragma unroll
    for (int k = 0; k < P; ++k) l[k] = r.l[k];
    return hmask;
}

// Load, decode and window one chunk [p0, p0 + P) of a pass (pass-relative window [lo, hi)):
// masked slots read the zero granule / voxel 0 with length 0 and carry no head.
template <typename L, bool LOCAL, int P = kPer>
__device__ __forceinline__ uint32_t window_chunk(const RawChunk<L, LOCAL, P>& r, int p0, int lo,
                                                 int hi, uint32_t (&v)[kVW<LOCAL, P>],
                                                 L (&l)[P]) {
    uint32_t hmask = decode<L, LOCAL, P>(r, v, l);
    if (p0 < lo || p0 + P > hi) {                   // edge chunks only
        const int first = lo - p0, end = hi - p0;
#pragma unroll
        for (int k = 0; k < P; ++k)
            if (k < first || k >= end) {
                if constexpr (LOCAL) v[k >> 1] &= ~(0xffffu << (16 * (k & 1)));
                else v[k] = 0u;
                l[k] = (L)0;
            }
        hmask &= window_bits<P>(first, end);
    }
    return hmask;
}

// Workgroup -> block of the CSR (ray-major: neighbouring blocks gather neighbouring voxels).
// Workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8 share an L2).  `chunk` > 0 deals
// runs of `chunk` consecutive blocks to each XCD instead (chunk > n/8: one contiguous range per
// XCD), so blocks that gather the same lines share an L2; 0 keeps dispatch order.  Bijective for
// any grid size.  Chosen per launch by fwd_chunk().
__device__ __forceinline__ int64_t block_of(int chunk) {
    const uint32_t n = gridDim.x;
    uint32_t b = blockIdx.x;
    if (chunk < 0) {                 // ~chunk, blocks in reverse order
        chunk = ~chunk;
        b = n - 1 - b;
    }
    if (chunk <= 0) return (int64_t)b;
    const uint32_t q = n / 8, r = n % 8, x = b % 8, i = b / 8, k = (uint32_t)chunk;
    if (k > q) return (int64_t)((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i);
    // chunks of k blocks dealt round-robin over the XCDs; the ragged tail keeps dispatch order
    if (b >= n / (8 * k) * (8 * k)) return (int64_t)b;
    return (int64_t)(((i / k) * 8 + x) * k + i % k);
}

// ---- forward ------------------------------------------------------------------------------
// Channels: static multichannel -> every ray for every channel c < n_chan; ray_chan_div > 0 ->
// ray i reads channel i / div (a time slice per view) and writes out[i].
// Per workgroup: block record -> {segment stream, voxel table, row_ptr of its share of the empty
// rays} -> table gather into LDS -> count scan -> segmented sum scan -> row->ray lookup -> stores.
// Modes (one instantiation each, so each carries only its own registers):
//   kFwdTable    static channels, density staged per workgroup from its granule table; skips the
//                workgroups without a table (n_tab < 0)
//   kFwdGather   static channels, per-segment gathers through vox; with `fallback_only`, only the
//                workgroups a kFwdTable launch skipped (and no empty-ray zeroing)
//   kFwdDynamic  ray i reads channel i / div
enum FwdMode { kFwdTable = 0, kFwdGather = 1, kFwdDynamic = 2 };

// Resident workgroups per CU the register allocation aims for: 6 (<= 80 VGPRs) lets a C2-sized
// launch (~1500 workgroups) be resident at once; float64 stops at 5 (no spills).
template <typename T, int P>
constexpr int fwd_min_blocks() {
    return P == kPer ? (sizeof(T) == 8 ? kFwdMinB64 : kFwdMinB32) : 5;
}

template <typename T>
using AccumOf = typename std::conditional<sizeof(T) == 4, float, double>::type;

// RUNS (table mode, sphrt_csr.runs set): the rows' rays and the empty rays come from the block's
// run record (one dword per lane, loaded with the table entries) instead of row_ray / empty_ray.
// HALF (float64 table mode with early DMA, tables of kHalfTab < n <= 2 kHalfTab granules): the LDS
// image holds half a table — entries [0, kHalfTab), then [kHalfTab, n_tab) — so a workgroup
// reserves 24.6 KB instead of up to 49 KB and five workgroups fit a CU instead of three (C5).
// Every segment reads its density in the phase that holds its granule (the other phase reads
// the zero granule) and keeps that value: the sums are unchanged, bit for bit.
constexpr int kHalfTab = kGranEarly * kThreads;   // = the early DMA rounds' entries (768)
// dense output range staged in LDS (elements).  C4's time-paired adjoint (ranges of 1144 on
// average, p99 2623) with 2-chunk early DMA: 1024 / 1536 / 2048 / 2560 / 4096 / 6144 outputs
// measured 28.0 / 26.8 / 25.4 / 25.0 / 28.5 / 31.5 us (workgroups per CU against ranges staged;
// profiles/r06_ostage_ab.jsonl, r06_adj_lds_ab.jsonl, r06_o2560_ab.jsonl)
constexpr int kOutStage = 2560;

template <typename T, typename L, int MODE, typename TabT = int32_t, bool EDMA = false,
          int P = kPer, bool RUNS = false, bool HALF = false, bool DENSE = false,
          int GE = kGranEarly>
__global__ __launch_bounds__(kPass / P, (fwd_min_blocks<T, P>())) void forward_kernel(
    const int64_t* __restrict__ blocks, const int32_t* __restrict__ vox,
    const uint16_t* __restrict__ loc, const TabT* __restrict__ tab, const L* __restrict__ len,
    const int32_t* __restrict__ row_ray, const int32_t* __restrict__ empty_ray,
    const T* __restrict__ density, int64_t n_chan, int64_t cs, int64_t div, T* __restrict__ out,
    int64_t ocs, int64_t n_rays, int64_t n_seg, int64_t n_cols, int64_t tab_stride,
    int xcd_chunk, int fallback_only, const int32_t* __restrict__ runs) {
    static_assert(!RUNS || MODE == kFwdTable, "run records serve the table mode");
    static_assert(!HALF || (MODE == kFwdTable && EDMA && P == kPer && kPass / P == kThreads),
                  "half tables: table mode, early DMA, 256-thread workgroups");
    static_assert(!HALF || GE == kGranEarly, "half tables: kHalfTab is the early rounds' entries");
    __shared__ FwdShared sh;
    extern __shared__ __attribute__((aligned(16))) unsigned char fwd_dyn_lds[];
    T* dens = reinterpret_cast<T*>(fwd_dyn_lds);   // 4 * tab_stride entries (table mode)
    constexpr bool local = MODE == kFwdTable;
    constexpr int THR = kPass / P;                  // threads (P segments each per pass)
    constexpr int W = THR / 64;
    using A = AccumOf<T>;
    int par = 0;                                    // scan slot parity
    const int tid = threadIdx.x;
    const int o = tid * P;                          // this thread's chunk within a pass
    const int64_t nc = MODE == kFwdDynamic ? 1 : n_chan;
    // Everything addressed by the workgroup index alone goes out before the block record
    // arrives: the first pass (rows of block b start in [b*kSegPerBlock, (b+1)*kSegPerBlock),
    // so its first pass is [b*kSegPerBlock, +kPass)) and the granule table (fixed stride).
    const int64_t blk = block_of(xcd_chunk);
    const int64_t base0 = blk * (DENSE ? kDenseSegPerBlock : kSegPerBlock);
    const int64_t last_chunk = imax64((n_seg + P - 1) / P, 1) - 1;   // clamp for loads
    RawChunk<L, local, P> raw;
    if (!EDMA) raw_load<L, local, P>(vox, loc, len, imin64(base0 + o, last_chunk * P), raw);
    // table chunks beyond the stride read the next workgroup's entries (tab is padded by
    // kGranEarly*kThreads entries); they are never staged (j >= n_tab)
    const TabT* tab_b = tab + blk * tab_stride;
    int32_t ti[kEarlyRounds<T, THR, GE>];
    if (local) {
        const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
        for (int r = 0; r < kEarlyRounds<T, THR, GE>; ++r)
            ti[r] = (int32_t)tab_b[gran_entry0<T, THR>(r, w) + (tid & 63) / kGranLanes<T>];
    }
    // the run record goes out with the table entries, before the chunk (the early-DMA wait below
    // counts only the loads issued after the chunk; issued after the chunk it measured the same)
    int32_t rrec = 0;
    if constexpr (RUNS) rrec = runs[blk * kRunFields + (tid & 31)];
    // early DMA: the table entries first, so waiting for them does not wait for the chunk
    if (EDMA) raw_load<L, local, P>(vox, loc, len, imin64(base0 + o, last_chunk * P), raw);
    __builtin_amdgcn_sched_barrier(0);
    const int64_t* m = blocks + kBlockFields * blk;
    const int64_t s0 = m[2], k0 = m[4], n_tab = m[5];
    int64_t s1 = m[3];
    if (MODE == kFwdTable && n_tab < 0) s1 = s0;      // left to the kFwdGather fallback launch
    // RUNS has no early exit for blocks without rows (below): an empty pass range instead, so
    // no pass runs (a pass over an empty window would still close "the last row" at its end)
    if (RUNS && s0 >= s1) s1 = base0;
    // fallback_only: the per-segment gather launch for the blocks a table launch skipped.
    // DENSE: dense output ranges (sphrt_csr.order bit 2, below) — instantiations of their own,
    // so that the other launches carry none of its code (with it as a run-time switch the
    // forwards measured C2 f32 5.9 -> 6.0 us, C5 f32 24.8 -> 26.7 us on one box)
    static_assert(!DENSE || (!RUNS && MODE != kFwdDynamic), "dense ranges: no runs, no slices");
    const bool fb_only = fallback_only != 0;
    constexpr bool dense = DENSE;
    if (MODE == kFwdGather && fb_only && n_tab >= 0) return;
    // Empty rays integrate to zero: this workgroup's share of the list is fetched now and
    // written at the very end, off the critical path.
    const int64_t e_lo = m[0];
    const int e_n = (fb_only || RUNS || dense) ? 0 : (int)(m[1] - e_lo);
    // Dense output ranges: the rows are in output order and block fields 0 / 1 hold the output
    // range [lo, hi) this workgroup owns (its rows and the empty rows up to the next workgroup's
    // first row): it zeroes the range with contiguous vector stores before any row closes, so
    // every output line is written by one workgroup (no empty-ray list, no partial lines from
    // several XCDs).  The closes of the same workgroup follow after a vmcnt(0) and the count
    // scan's barrier; a block left to the fallback launch zeroes its range here and the later
    // launch writes its rows.
    // Table launches stage a dense range of up to kOutStage outputs in LDS behind the granule
    // image: zeroed, written by the closes, flushed with contiguous stores at the end — each
    // output line is then written once (zeros and values together).  Larger ranges, and the
    // fallback launch, zero the range in global memory first.
    const bool ostaged = MODE == kFwdTable && dense && m[1] - m[0] <= kOutStage;
    T* ost = dens + ((HALF ? kHalfTab : EDMA ? imax64(tab_stride, GE * kThreads)
                                           : tab_stride) + 1) * 4;
    if (ostaged)
        for (int j = tid; j < (int)(m[1] - m[0]); j += THR) ost[j] = (T)0;
    auto put = [&](T* oc, int64_t r, T val) {
        if (ostaged) ost[r - m[0]] = val;
        else oc[r] = val;
    };
    auto zero_range = [&]() {
        const int64_t lo = m[0], hi = m[1];
        constexpr int E = 16 / (int)sizeof(T);             // elements per 16-byte store
        const int64_t a = imin64((lo + E - 1) / E * E, hi), b = imax64(hi / E * E, a);
        if (tid < a - lo) out[lo + tid] = (T)0;
        if (tid < hi - b) out[b + tid] = (T)0;
        uint4* ov = reinterpret_cast<uint4*>(out);
        for (int64_t q = a / E + tid; q < b / E; q += THR) ov[q] = make_uint4(0u, 0u, 0u, 0u);
    };
    // (unconditional load: empty_ray holds n_rays + 1 entries; a predicated load would make
    // the wait-count model drain every load before the granule DMA)
    constexpr int kEmptyLoads = RUNS ? 0 : 1;
    int32_t r_empty = 0;
    if constexpr (!RUNS) r_empty = empty_ray[e_lo + min(tid, max(e_n - 1, 0))];
    auto zero_empty = [&]() {
        if constexpr (RUNS) {      // empty j of the share -> its ray through the ranges
            const int ne = __builtin_amdgcn_readlane(rrec, 1);
            int e_tot = 0;
            for (int i = 0; i < ne; ++i) e_tot += __builtin_amdgcn_readlane(rrec, kRunEmpty + 2 * i + 1);
            for (int j = tid; j < e_tot; j += THR) {   // (one round for shares of <= 256)
                int rem = j;
                int32_t ray = 0;
                for (int i = 0; i < ne; ++i) {
                    const int32_t r0 = __builtin_amdgcn_readlane(rrec, kRunEmpty + 2 * i);
                    const int cnt = __builtin_amdgcn_readlane(rrec, kRunEmpty + 2 * i + 1);
                    ray = (rem >= 0 && rem < cnt) ? r0 + rem : ray;
                    rem -= cnt;
                }
                if (nc == 1) out[ray] = (T)0;
                else
                    for (int64_t c = 0; c < nc; ++c) out[c * ocs + ray] = (T)0;
            }
            return;
        }
        asm volatile("" : "+v"(r_empty));     // keep every use (and its wait) down here
        if (tid < e_n)
            for (int64_t c = 0; c < nc; ++c) out[c * ocs + r_empty] = (T)0;
        for (int j = tid + THR; j < e_n; j += THR) {
            const int64_t r = empty_ray[e_lo + j];
            for (int64_t c = 0; c < nc; ++c) out[c * ocs + r] = (T)0;
        }
    };
    // A block without rows (or left to the fallback launch) zeroes its empty share and leaves.
    // With run records the table kernel runs on instead (its passes are skipped): as a separate
    // exit path, the compiler sank the table-entry and chunk loads below the block record's
    // arrival, serialising one more round trip in front of every workgroup.
    if (!RUNS && s0 >= s1) {
        if (dense) zero_range();
        else zero_empty();
        return;
    }
    const int32_t g_full = (int32_t)imin64(n_cols >> 2, INT32_MAX);   // whole granules
    if (local && EDMA) stage_granules_early<T, THR, GE>(density, ti, (int)n_tab, dens);
    else if (local)
        stage_granules<T, TabT, THR, GE>(density, ti, tab_b, (int)n_tab, g_full, n_cols, dens);
    // pass-relative segment window [lo, hi) of this workgroup (32-bit lane arithmetic)
    auto window = [&](int64_t base, int& lo, int& hi) {
        lo = (int)imax64(s0 - base, -1);
        hi = (int)imin64(s1 - base, (int64_t)kPass + 1);
    };
    uint32_t v[kVW<local, P>];
    L l[P];
    uint32_t hmask;
    if constexpr (local && EDMA) {
        // Loads complete in issue order: the chunk is in once at most the empty-list load and the
        // early DMAs issued after it are outstanding.  Said explicitly: the compiler's model
        // treats LDS-DMA as another event type and would wait for every DMA (vmcnt(0)).
        constexpr int after = kEmptyLoads + kEarlyRounds<T, THR, GE>;
        static_assert(after < 16, "vmcnt field");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((after & 15) | (7 << 4) | (15 << 8));
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        int lo, hi;
        window(base0, lo, hi);
        hmask = window_chunk<L, local, P>(raw, o, lo, hi, v, l);
    }
    if (local && EDMA && !HALF)   // rounds past the early ones (tables of more than 768 granules)
        stage_granules_late<T, TabT, THR>(density, tab_b, kEarlyRounds<T, THR, GE>, (int)n_tab, g_full,
                                          dens);
    if (dense && !ostaged) {      // (uniform) zeros before any close of this workgroup
        zero_range();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    int64_t rbase = 0;                            // rows started in earlier passes
#pragma clang loop unroll(disable)   // (also no peeling: one copy of the pass body)
    for (int64_t c = 0; c < nc; ++c) {
        const T* rho = density + c * cs;
        T* oc = out + c * ocs;
        if (local && c > 0 && !HALF) {
            stage_granules_late<T, TabT, THR>(rho, tab_b, 0, (int)n_tab, g_full, dens);
            stage_partial_tail<T, TabT, THR>(rho, tab_b, (int)n_tab, n_cols, dens);
        }
        using Stitch = typename std::conditional<sizeof(T) == 4, float, double>::type;
        Stitch carry = 0;                   // open run entering the pass
        rbase = 0;
#pragma clang loop unroll(disable)
        for (int64_t base = base0; base < s1; base += kPass) {
            int lo, hi;
            window(base, lo, hi);
            // later channels of a one-pass block reuse the decoded first chunk: the segments
            // are streamed once, only the granules are staged per channel
            if (base != base0 || (c != 0 && s1 > base0 + kPass)) {
                RawChunk<L, local, P> rc;
                raw_load<L, local, P>(vox, loc, len, imin64(base + o, last_chunk * P), rc);
                hmask = window_chunk<L, local, P>(rc, o, lo, hi, v, l);
            }
            const int hcount = __builtin_popcount(hmask);
            T rv[P];
            if constexpr (MODE == kFwdGather) {   // per-segment gathers go out before any scan
#pragma unroll
                for (int k = 0; k < P; ++k)
                    rv[k] = l[k] != (L)0 ? rho[vslot<local, P>(v, k) & ~kHead] : (T)0;
            }
            int pass_heads;
            // HALF: the first half is staged again for each channel, and for every later pass of
            // a two-phase block (its LDS then holds the second half); the previous pass's reads
            // all precede its segmented-scan barrier
            if constexpr (HALF) {
                if ((c > 0 && base == base0) || (n_tab > kHalfTab && base != base0))
                    stage_granules_late<T, TabT, THR>(rho, tab_b, 0, (int)imin64(n_tab, kHalfTab),
                                                      g_full, dens);
            }
            // (table mode: the full barrier also retires the granule LDS-DMA)
            const int hb = block_excl_count1<local, W>(hcount, pass_heads, sh.cnt[par]);
            pass_heads = __builtin_amdgcn_readfirstlane(pass_heads);
            // rows this thread closes: the run open at its start (row hb-1) and its first own row
            // (row hb) are fetched now, under the segmented scan; further ones (rare) at the store
            const int32_t* rows = row_ray + k0 + rbase + hb;
            // unconditional loads (clamped into row_ray's n_rays entries): no branch, so nothing
            // waits for them before the first store
            const int64_t ri = k0 + rbase + hb;
            // RUNS: the ray of block-relative row q from the record's runs (run 0 starts at row 0)
            const int qb = (int)(rbase + hb);
            auto ray_of_row = [&](int q) -> int32_t {
                int32_t r = __builtin_amdgcn_readlane(rrec, 3) + q;
                const int nr = __builtin_amdgcn_readlane(rrec, 0);
                for (int i = 1; i < nr; ++i) {
                    const int off = __builtin_amdgcn_readlane(rrec, 2 + 2 * i);
                    const int32_t ray = __builtin_amdgcn_readlane(rrec, 3 + 2 * i);
                    r = q >= off ? ray + (q - off) : r;
                }
                return r;
            };
            int32_t r_prev, r_first, r_second;
            if constexpr (RUNS) {
                const int32_t r0 = __builtin_amdgcn_readlane(rrec, 3);
                r_prev = r0 + qb - 1;
                r_first = r0 + qb;
                r_second = r0 + qb + 1;
                const int nr = __builtin_amdgcn_readlane(rrec, 0);
                for (int i = 1; i < nr; ++i) {   // uniform: usually 1 or 2 runs
                    const int off = __builtin_amdgcn_readlane(rrec, 2 + 2 * i);
                    const int32_t d = __builtin_amdgcn_readlane(rrec, 3 + 2 * i) - off;
                    r_prev = qb - 1 >= off ? d + qb - 1 : r_prev;
                    r_first = qb >= off ? d + qb : r_first;
                    r_second = qb + 1 >= off ? d + qb + 1 : r_second;
                }
            } else {
                r_prev = row_ray[imax64(ri - 1, 0)];
                r_first = row_ray[imin64(ri, n_rays - 1)];
                r_second = row_ray[imin64(ri + 1, n_rays - 1)];
            }
            auto row_of = [&](int i) -> int64_t {     // ray of the row after i own heads
                if constexpr (RUNS) return i < 0 ? r_prev : i == 0 ? r_first : ray_of_row(qb + i);
                return i < 0 ? r_prev : i == 0 ? r_first : rows[i];
            };
            if constexpr (local && !HALF) {
#pragma unroll
                for (int k = 0; k < P; ++k)
                    rv[k] = lds_at<T>(dens, vslot<local, P>(v, k));   // masked: the zero granule
            }
            if constexpr (HALF) {
                // slots of entries < kHalfTab lie below `lim` (float-unit offsets 16 (r+1) + 4 i);
                // the rest read the zero granule (x & 15) in this phase
                constexpr uint32_t lim = 16u * (kHalfTab + 1);
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    const uint32_t x = vslot<local, P>(v, k);
                    rv[k] = lds_at<T>(dens, x < lim ? x : (x & 15u));
                }
                if (n_tab > kHalfTab) {             // (block-uniform)
                    lds_barrier();                  // every first-half read is done
                    stage_granules_late<T, TabT, THR>(rho, tab_b + kHalfTab, 0,
                                                      (int)n_tab - kHalfTab, g_full, dens);
                    __syncthreads();                // retires the DMA
#pragma unroll
                    for (int k = 0; k < P; ++k) {
                        const uint32_t x = vslot<local, P>(v, k);
                        const T r1 = lds_at<T>(dens, x < lim ? (x & 15u) : x - 16u * kHalfTab);
                        rv[k] = x < lim ? rv[k] : r1;
                    }
                }
            }
            if constexpr (MODE == kFwdDynamic) {   // time slice of each segment's ray
                int rank = 0;
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    rank += (hmask >> k) & 1;
                    T x = (T)0;
                    if (l[k] != (L)0) {
                        const int64_t ray = row_of(rank - 1);
                        x = density[(ray / div) * cs + (vslot<local, P>(v, k) & ~kHead)];
                    }
                    rv[k] = x;
                }
            }
            // Products and thread-local runs in A (float for a float density: the reference's own
            // precision, 4-cycle VALU ops instead of 8-cycle f64 ones); runs that cross threads are
            // stitched in Stitch (A as well).
            A p[P];
#pragma unroll
            for (int k = 0; k < P; ++k) p[k] = (A)rv[k] * (A)l[k];
            // Row closes: at every head except the workgroup's first segment, and at position kPer
            // in the thread holding the workgroup's last segment when this pass reaches it (masked
            // slots carry no head and zero length, so no per-slot window test is needed).  With
            // h1 < h2 < h3 the first three heads of the chunk (kPer when missing), the closes at
            // h1, h2 and h3 store qa (run0 + the chunk's part before h1: the run open at the chunk
            // start, in double), v1 and v2 (the runs [h1,h2), [h2,h3)) to rows hb-1, hb and hb+1;
            // closes past h3 (chunks of 3+ heads) take a second walk.  One walk gives the runs and
            // the thread's tail (its last run, the scan's input).
            const uint32_t hm0 = hmask | (1u << P);
            const uint32_t hm1 = hm0 & (hm0 - 1), hm2 = hm1 & (hm1 - 1);
            const int h1 = __builtin_ctz(hm0);
            const int h2 = __builtin_ctz(hm1 | (1u << P));
            const int h3 = __builtin_ctz(hm2 | (1u << P));
            A tail = (A)0, qa = (A)0, v1 = (A)0, v2 = (A)0;
#pragma unroll
            for (int k = 0; k <= P; ++k) {
                qa = k == h1 ? tail : qa;
                v1 = k == h2 ? tail : v1;
                v2 = k == h3 ? tail : v2;
                if (k < P) tail = ((hmask >> k) & 1 ? (A)0 : tail) + p[k];
            }
            bool tot_has;
            Stitch tot_sum;
            const Stitch ex = block_excl_segsum1<W, Stitch>(hmask != 0, (Stitch)tail, tot_has, tot_sum,
                                                 sh.has[par], sh.sum[par]);
            par ^= 1;
            // the run open at this thread's start: the segmented prefix of the earlier threads,
            // plus the carry of earlier passes when no earlier thread of this pass saw a head
            const Stitch run0 = hb > 0 ? ex : carry + ex;
            uint32_t cmask = hmask;
            {
                const int first = lo - o, end = hi - o;
                if (base == base0 && first >= 0 && first < P) cmask &= ~(1u << first);
                if (base + kPass >= s1 && end > 0 && end <= P) cmask |= 1u << P;
            }
            if ((cmask >> h1) & 1) put(oc, r_prev, (T)(run0 + (Stitch)qa));
            if (h2 != h1 && ((cmask >> h2) & 1)) put(oc, r_first, (T)v1);
            if (h3 != h2 && ((cmask >> h3) & 1)) put(oc, r_second, (T)v2);
            if (hcount > 2) {                         // rare: closes of the fourth and later runs
                A q = (A)0;
                int rank = 0;
#pragma unroll
                for (int k = 0; k <= P; ++k) {
                    if (k > h3 && ((cmask >> k) & 1)) put(oc, row_of(rank - 1), (T)q);
                    if (k < P) {
                        const bool h = (hmask >> k) & 1;
                        rank += h;
                        q = (h ? (A)0 : q) + p[k];
                    }
                }
            }
            carry = tot_has ? tot_sum : carry + tot_sum;
            rbase += pass_heads;
        }
    }
    if (ostaged) {                // the staged range out with contiguous stores
        lds_barrier();
        const int64_t lo = m[0], hi = m[1];
        for (int j = tid; j < (int)(hi - lo); j += THR) out[lo + j] = ost[j];
        return;
    }
    zero_empty();
}

// ---- adjoint (float64 atomics into a float64 accumulator) -------------------------------------
template <typename TY>
__global__ __launch_bounds__(kThreads) void adjoint_kernel(
    const int64_t* __restrict__ blocks, const int32_t* __restrict__ vox,
    const double* __restrict__ len, const int32_t* __restrict__ row_ray,
    const TY* __restrict__ y, int64_t n_chan, int64_t ycs, int64_t div, double* acc,
    int64_t cs) {
    __shared__ ScanShared sh;
    const int64_t* m = blocks + kBlockFields * (int64_t)blockIdx.x;
    const int64_t s0 = m[2], s1 = m[3], k0 = m[4];
    if (s0 >= s1) return;
    const int tid = threadIdx.x;
    const int64_t a0 = s0 & ~(int64_t)(kPer - 1);
    const int64_t nc = div > 0 ? 1 : n_chan;
    int64_t heads_done = 0;
    for (int64_t base = a0; base < s1; base += kPass) {
        uint32_t v[kPer];
        double l[kPer];
        load8(vox + base, len + base, tid * kPer, (int)imax64(s0 - base, -1),
              (int)imin64(s1 - base, (int64_t)kPass + 1), v, l);
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

// Time-paired columns: ray r reads time slice r / div, so its segments' columns become
// (r / div) * vol + voxel (head bit kept).  One wave per ray over its contiguous segments.
__global__ __launch_bounds__(256) void time_columns_kernel(const int64_t* row_ptr, int64_t n_rays,
                                                           const int32_t* vox, int64_t div,
                                                           int64_t vol, int32_t* out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rays) return;
    const int64_t base = (r / div) * vol;
    const int64_t a = row_ptr[r], e = row_ptr[r + 1];
    for (int64_t s = a + (threadIdx.x & 63); s < e; s += 64) {
        const uint32_t x = (uint32_t)vox[s];
        out[s] = (int32_t)((x & kHead) | (uint32_t)(base + (int64_t)(x & ~kHead)));
    }
}

}  // namespace sphrt

using namespace sphrt;

extern "C" int sphrt_csr_time_columns(const sphrt_csr* c, int64_t div, int64_t vol,
                                      int32_t* vox_out, void* stream) {
    if (!c || !c->row_ptr || !c->vox || !vox_out) return fail("incomplete CSR");
    if (div < 1 || vol < 1) return fail("bad time pairing (div, vol)");
    const int64_t n_t = (c->n_rays + div - 1) / div;
    if (n_t * vol >= (int64_t)kHead) return fail("time-paired columns need T * voxels < 2^31");
    if (c->n_rays == 0) return 0;
    StreamGuard guard(stream);
    hipLaunchKernelGGL(time_columns_kernel, dim3((unsigned)((c->n_rays + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, c->row_ptr, c->n_rays, c->vox, div, vol, vox_out);
    return check_launch("time_columns");
}

extern "C" int64_t sphrt_csr_blocks(int64_t n_segments) {
    return n_segments < 0 ? -1 : n_segments / kSegPerBlock + 1;
}

extern "C" int64_t sphrt_csr_blocks_dense(int64_t n_segments) {
    return n_segments < 0 ? -1 : n_segments / kDenseSegPerBlock + 1;
}

extern "C" size_t sphrt_csr_index_workspace_bytes(int64_t n_rays) {
    // nonempty flags (int32) | row prefix (int64, n+1) | scan workspace
    const size_t a = (((size_t)n_rays * 4 + 255) / 256) * 256;
    const size_t b = (((size_t)(n_rays + 1) * 8 + 255) / 256) * 256;
    return a + b + sphrt_scan_workspace_bytes(n_rays);
}

static int csr_index(const int64_t* row_ptr, int64_t n_rays, int32_t* vox, int32_t* row_ray,
                     int32_t* empty_ray, int64_t* blocks, int64_t n_blocks,
                     const int32_t* ray_ids, int32_t* nz_row, void* workspace, void* stream,
                     int64_t spb = kSegPerBlock) {
    if (n_rays < 0 || n_blocks < 1) return fail("bad CSR index sizes");
    if (n_rays == 0) return 0;
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    unsigned char* ws = (unsigned char*)workspace;
    int32_t* flags = (int32_t*)ws;
    int64_t* pre = (int64_t*)(ws + (((size_t)n_rays * 4 + 255) / 256) * 256);
    void* scan_ws = (unsigned char*)pre + (((size_t)(n_rays + 1) * 8 + 255) / 256) * 256;
    const unsigned g = (unsigned)((n_rays + 255) / 256);
    hipLaunchKernelGGL(mark_rows_kernel, dim3(g), dim3(256), 0, st, row_ptr, n_rays, vox, flags);
    if (int e = check_launch("mark_rows")) return e;
    if (int e = sphrt_scan_counts(flags, n_rays, pre, scan_ws, stream)) return e;
    hipLaunchKernelGGL(row_list_kernel, dim3(g), dim3(256), 0, st, row_ptr, pre, n_rays, ray_ids,
                       row_ray, empty_ray, nz_row);
    if (int e = check_launch("row_list")) return e;
    hipLaunchKernelGGL(block_meta_kernel, dim3((unsigned)((n_blocks + 255) / 256)), dim3(256), 0,
                       st, row_ptr, pre, n_rays, n_blocks, spb, blocks);
    return check_launch("block_meta");
}

extern "C" int sphrt_csr_index(const int64_t* row_ptr, int64_t n_rays, int32_t* vox,
                               int32_t* row_ray, int32_t* empty_ray, int64_t* blocks,
                               int64_t n_blocks, const int32_t* ray_ids,
                               void* workspace, void* stream) {
    if (!vox && n_rays > 0) return fail("null vox");
    return csr_index(row_ptr, n_rays, vox, row_ray, empty_ray, blocks, n_blocks, ray_ids, nullptr,
                     workspace, stream);
}

extern "C" int sphrt_csr_index_dense(const int64_t* row_ptr, int64_t n_rays, int32_t* vox,
                                     int32_t* row_ray, int32_t* empty_ray, int64_t* blocks,
                                     int64_t n_blocks, const int32_t* ray_ids, void* workspace,
                                     void* stream) {
    if (!vox && n_rays > 0) return fail("null vox");
    return csr_index(row_ptr, n_rays, vox, row_ray, empty_ray, blocks, n_blocks, ray_ids, nullptr,
                     workspace, stream, kDenseSegPerBlock);
}

extern "C" int sphrt_csr_index_staged(const int64_t* row_ptr, int64_t n_rays, int32_t* row_ray,
                                      int32_t* empty_ray, int64_t* blocks, int64_t n_blocks,
                                      const int32_t* ray_ids, int32_t* nz_row, void* workspace,
                                      void* stream) {
    if (!nz_row && n_rays > 0) return fail("null nz_row");
    // (nz_row and the staged gather index rows as int32)
    if (n_rays > 0x7fffffff) return fail("the staged index needs n_rays < 2^31");
    return csr_index(row_ptr, n_rays, nullptr, row_ray, empty_ray, blocks, n_blocks, ray_ids,
                     nz_row, workspace, stream);
}

extern "C" int sphrt_csr_runs(const sphrt_csr* c, int32_t* runs, int64_t* stats, void* stream) {
    if (!c || !c->row_ray || !c->empty_ray || !c->blocks || !runs || !stats)
        return fail("incomplete CSR for the run records");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (c->n_rays > 0x7fffffff) return fail("run records need ray ids < 2^31");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(stats, 0, sizeof(int64_t), st) != hipSuccess)
        return fail("hipMemsetAsync failed");
    if (c->n_rays == 0) return 0;
    hipLaunchKernelGGL(block_runs_kernel, dim3((unsigned)((c->n_blocks + 255) / 256)), dim3(256),
                       0, st, c->blocks, c->row_ray, c->empty_ray, c->n_rays, c->n_blocks, runs,
                       (unsigned long long*)stats);
    return check_launch("block_runs");
}


// The float32 lengths a count / build launch writes: len32 when the caller set it with len
// (sphrt.h: the table launch then fills the float32 copy), else none.
static float* len32_out(const sphrt_csr* c) {
    return c->len && c->len32 ? const_cast<float*>(c->len32) : nullptr;
}

// bitmap words for a volume of n_cols voxels, or 0 when the bitmap costs more than sorting the
// workgroup's segments (every workgroup clears and scans the whole bitmap: <= 4096 words, i.e.
// volumes up to 2^19 voxels; larger ones take the radix sort)
static int table_bitmap_words(int64_t n_cols) {
    const int64_t words = ((n_cols + 3) / 4 + 31) / 32;
    return n_cols > 0 && words <= 4096 ? (int)words : 0;
}
// Sort bits for the granule keys: strictly more than the largest granule index needs, so the
// padding key (all ones) sorts after every real key whatever the input arrangement (with exactly
// enough bits the last granule of a 2^k-granule volume ties with the padding: C3's 128^3).
static int granule_key_bits(int64_t n_cols) {
    int b = 1;
    while ((1LL << b) <= (n_cols + 3) / 4) ++b;
    return b;
}

// The table kernel's two launches (blocks of <= 2048 segments, then the larger ones).
template <int TM, typename TabT>
static int launch_tables(unsigned nb, hipStream_t st, int64_t* blocks, const int32_t* vox,
                         uint16_t* loc, TabT* tab, int64_t stride, int kb, const StageMap& sm,
                         unsigned long long* stats, const double* len = nullptr,
                         float* len32 = nullptr, const Staged& S = Staged{}) {
    const char* env = getenv("SPHRT_TABLE_BUCKETS");   // (read per build: tests toggle it)
    if (env && env[0] == '0') kb |= kSortOnly;
    // bucket tables, 8-bit sort behind (keys of 21 bits keep the 10-bit one: the transposed
    // tables' rays from every view span more buckets than a block has slots, and sort)
    if (kb <= kBucketLo + 11) {
        hipLaunchKernelGGL((local_table_radix_kernel<TM, TabT, 8>), dim3(nb), dim3(kThreads), 0, st,
                           blocks, vox, loc, tab, stride, kb, sm, stats, len, len32, S, (int64_t)nb);
        hipLaunchKernelGGL((local_table_big_kernel<TM, TabT, 8>), dim3((nb + kBigScan - 1) / kBigScan),
                           dim3(kThreads), 0, st, blocks, (int64_t)nb, vox, loc, tab, stride, kb, sm,
                           stats);
        return check_launch("local_table_radix_kernel");
    }
    hipLaunchKernelGGL((local_table_radix_kernel<TM, TabT>), dim3(nb), dim3(kThreads), 0, st,
                       blocks, vox, loc, tab, stride, kb, sm, stats, len, len32, S, (int64_t)nb);
    hipLaunchKernelGGL((local_table_big_kernel<TM, TabT>), dim3((nb + kBigScan - 1) / kBigScan),
                       dim3(kThreads), 0, st, blocks, (int64_t)nb, vox, loc, tab, stride, kb, sm,
                       stats);
    return check_launch("local_table_radix_kernel");
}

extern "C" int sphrt_csr_local_count(const sphrt_csr* c, int64_t* blocks, int64_t* stats,
                                     void* stream) {
    if (!c || !c->vox || !blocks || !stats) return fail("incomplete CSR for the granule tables");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    StageMap sm;
    if (!stage_map(c, sm)) return fail("inconsistent brick staging fields");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(stats, 0, 2 * sizeof(int64_t), st) != hipSuccess)
        return fail("hipMemsetAsync failed");
    if (c->n_segments == 0) return 0;
    const int64_t cols = table_cols(c);
    if (const int words = table_bitmap_words(cols)) {
        hipLaunchKernelGGL((local_table_bitmap_kernel<kTabCount, int32_t>), dim3((unsigned)c->n_blocks),
                           dim3(kThreads), (size_t)words * 8, st, blocks, c->vox, nullptr, nullptr,
                           0, words, sm, (unsigned long long*)stats, c->len, len32_out(c));
        return check_launch("local_table_bitmap_kernel<count>");
    }
    return launch_tables<kTabCount, int32_t>((unsigned)c->n_blocks, st, blocks,
                                             c->vox, nullptr, nullptr, 0, granule_key_bits(cols),
                                             sm, (unsigned long long*)stats, c->len, len32_out(c));
}

extern "C" int sphrt_csr_local_fill(const sphrt_csr* c, const int64_t* blocks, uint16_t* loc,
                                    void* tab, int64_t tab_stride, void* stream) {
    if (!c || !c->vox || !blocks || !loc || !tab) return fail("incomplete CSR for the granule tables");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (tab_stride < 1 || tab_stride > (kMaxGran + 63) / 64 * 64)
        return fail("bad granule table stride");
    StageMap sm;
    if (!stage_map(c, sm)) return fail("inconsistent brick staging fields");
    const int64_t cols = table_cols(c);
    const bool u16 = c->tab_bytes == 2;
    if (u16 && (cols + 3) / 4 > 65536) return fail("16-bit granule tables need <= 2^18 columns");
    if (c->n_segments == 0) return 0;
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (const int words = table_bitmap_words(cols)) {
        if (u16)
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabFill, uint16_t>), dim3((unsigned)c->n_blocks),
                               dim3(kThreads), (size_t)words * 8, st, (int64_t*)blocks, c->vox, loc,
                               (uint16_t*)tab, tab_stride, words, sm, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabFill, int32_t>), dim3((unsigned)c->n_blocks),
                               dim3(kThreads), (size_t)words * 8, st, (int64_t*)blocks, c->vox, loc,
                               (int32_t*)tab, tab_stride, words, sm, nullptr, nullptr, nullptr);
        return check_launch("local_table_bitmap_kernel<fill>");
    }
    const int kb = granule_key_bits(cols);
    const unsigned nb = (unsigned)c->n_blocks;
    if (u16)
        return launch_tables<kTabFill, uint16_t>(nb, st, (int64_t*)blocks, c->vox, loc,
                                                 (uint16_t*)tab, tab_stride, kb, sm, nullptr);
    return launch_tables<kTabFill, int32_t>(nb, st, (int64_t*)blocks, c->vox, loc,
                                            (int32_t*)tab, tab_stride, kb, sm, nullptr);
}

extern "C" int sphrt_csr_local_build(const sphrt_csr* c, int64_t* blocks, uint16_t* loc,
                                     void* tab_wide, int64_t* stats, void* stream) {
    if (!c || !c->vox || !blocks || !loc || !tab_wide || !stats)
        return fail("incomplete CSR for the granule tables");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    StageMap sm;
    if (!stage_map(c, sm)) return fail("inconsistent brick staging fields");
    const int64_t cols = table_cols(c);
    const bool u16 = c->tab_bytes == 2;
    if (u16 && (cols + 3) / 4 > 65536) return fail("16-bit granule tables need <= 2^18 columns");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(stats, 0, 2 * sizeof(int64_t), st) != hipSuccess)
        return fail("hipMemsetAsync failed");
    if (c->n_segments == 0) return 0;
    const dim3 g((unsigned)c->n_blocks), b(kThreads);
    unsigned long long* s = (unsigned long long*)stats;
    if (const int words = table_bitmap_words(cols)) {
        const size_t lds = (size_t)words * 8;
        if (u16)
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabBuild, uint16_t>), g, b, lds, st,
                               blocks, c->vox, loc, (uint16_t*)tab_wide, kTabWide, words, sm, s,
                               c->len, len32_out(c));
        else
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabBuild, int32_t>), g, b, lds, st,
                               blocks, c->vox, loc, (int32_t*)tab_wide, kTabWide, words, sm, s,
                               c->len, len32_out(c));
        return check_launch("local_table_bitmap_kernel<build>");
    }
    const int kb = granule_key_bits(cols);
    if (u16)
        return launch_tables<kTabBuild, uint16_t>(g.x, st, blocks, c->vox, loc,
                                                  (uint16_t*)tab_wide, kTabWide, kb, sm, s, c->len,
                                                  len32_out(c));
    return launch_tables<kTabBuild, int32_t>(g.x, st, blocks, c->vox, loc,
                                             (int32_t*)tab_wide, kTabWide, kb, sm, s, c->len,
                                             len32_out(c));
}

extern "C" int sphrt_csr_local_build_staged(const sphrt_csr* c, int64_t* blocks, uint16_t* loc,
                                            void* tab_wide, int64_t* stats, const int64_t* slot,
                                            const int32_t* nz_row, const int32_t* svox,
                                            const double* slen,
                                            void* stream) {
    if (!c || !c->row_ptr || !c->vox || !c->len32 || !blocks || !loc || !tab_wide || !stats ||
        !slot || !nz_row || !svox || !slen)
        return fail("incomplete staged CSR for the granule tables");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (c->n_rays > 0x7fffffff) return fail("the staged table build needs n_rays < 2^31");
    StageMap sm;
    if (!stage_map(c, sm)) return fail("inconsistent brick staging fields");
    const int64_t cols = table_cols(c);
    const bool u16 = c->tab_bytes == 2;
    if (u16 && (cols + 3) / 4 > 65536) return fail("16-bit granule tables need <= 2^18 columns");
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(stats, 0, 2 * sizeof(int64_t), st) != hipSuccess)
        return fail("hipMemsetAsync failed");
    if (c->n_segments == 0) return 0;
    const Staged S{c->row_ptr, slot, nz_row, c->n_rays, svox, slen, const_cast<int32_t*>(c->vox),
                   const_cast<double*>(c->len), const_cast<float*>(c->len32)};
    unsigned long long* s = (unsigned long long*)stats;
    const unsigned nb = (unsigned)c->n_blocks;
    if (const int words = table_bitmap_words(cols)) {
        const size_t lds = (size_t)words * 8;
        if (u16)
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabBuild, uint16_t>), dim3(nb),
                               dim3(kThreads), lds, st, blocks, c->vox, loc, (uint16_t*)tab_wide,
                               kTabWide, words, sm, s, nullptr, nullptr, S, (int64_t)nb);
        else
            hipLaunchKernelGGL((local_table_bitmap_kernel<kTabBuild, int32_t>), dim3(nb),
                               dim3(kThreads), lds, st, blocks, c->vox, loc, (int32_t*)tab_wide,
                               kTabWide, words, sm, s, nullptr, nullptr, S, (int64_t)nb);
        return check_launch("local_table_bitmap_kernel<build, staged>");
    }
    const int kb = granule_key_bits(cols);
    if (u16)
        return launch_tables<kTabBuild, uint16_t>(nb, st, blocks, c->vox, loc, (uint16_t*)tab_wide,
                                                  kTabWide, kb, sm, s, nullptr, nullptr, S);
    return launch_tables<kTabBuild, int32_t>(nb, st, blocks, c->vox, loc, (int32_t*)tab_wide,
                                             kTabWide, kb, sm, s, nullptr, nullptr, S);
}

extern "C" int sphrt_csr_local_pack(const sphrt_csr* c, const int64_t* blocks,
                                    const void* tab_wide, void* tab, int64_t tab_stride,
                                    void* stream) {
    if (!c || !blocks || !tab_wide || !tab) return fail("incomplete CSR for the granule tables");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (tab_stride < 1 || tab_stride > (kMaxGran + 63) / 64 * 64)
        return fail("bad granule table stride");
    if (c->n_segments == 0) return 0;
    StreamGuard guard(stream);
    const dim3 g((unsigned)c->n_blocks), b(kThreads);
    if (c->tab_bytes == 2)
        hipLaunchKernelGGL(table_pack_kernel<uint16_t>, g, b, 0, (hipStream_t)stream, blocks,
                           (const uint16_t*)tab_wide, (uint16_t*)tab, tab_stride);
    else
        hipLaunchKernelGGL(table_pack_kernel<int32_t>, g, b, 0, (hipStream_t)stream, blocks,
                           (const int32_t*)tab_wide, (int32_t*)tab, tab_stride);
    return check_launch("table_pack_kernel");
}

static int check_csr(const sphrt_csr* c, int64_t n_chan, int64_t div) {
    if (!c || !c->row_ptr || !c->vox || !c->row_ray || !c->empty_ray || !c->blocks)
        return fail("incomplete CSR");
    if (c->n_blocks < 1 || c->n_blocks > 0x7fffffff) return fail("bad CSR block count");
    if (n_chan < 1) return fail("n_chan must be >= 1");
    if (div > 0 && n_chan != 1) return fail("ray_chan_div requires n_chan == 1");
    return 0;
}

// The granule tables apply to static channels whose granules are 16-byte (float) / 32-byte
// (double) aligned; anything else takes the per-segment gather through vox.
// dynamic LDS for the staged granules, per workgroup (C5 f64, 49 KB: table 64.0 us vs per-segment
// gather 73.3 us)
constexpr size_t kTableLdsMax = 64 * 1024;

// Early granule DMA (forward_kernel EDMA) needs whole granules only: no partial last granule.
// SPHRT_FWD_HALF=0 in the environment at launch keeps whole float64 tables (tests: half tables
// give the whole tables' sums bit for bit).
static bool half_tables_on() {
    const char* e = getenv("SPHRT_FWD_HALF");
    return !(e && e[0] == '0');
}

static bool early_dma(const sphrt_csr* c) {
    return table_cols(c) % 4 == 0 &&
           (size_t)(kGranEarly * kThreads + 1) * 4 * 8 <= kTableLdsMax;
}

template <typename T>
static bool use_tables(const sphrt_csr* c, const T* density, int64_t n_chan, int64_t chan_stride,
                       int64_t div) {
    if (!c->loc || !c->tab || c->n_cols <= 0 || div > 0) return false;
    // (+ the staged output range of dense output ranges, which the granule image leaves room for)
    const size_t extra = (c->order & 4) ? (size_t)kOutStage * sizeof(T) : 0;
    if (c->tab_stride < 1 ||
        (size_t)(imax64(c->tab_stride, kGranEarly * kThreads) + 1) * 4 * sizeof(T) + extra >
            kTableLdsMax)
        return false;
    if ((uintptr_t)density % (4 * sizeof(T)) != 0) return false;
    if (n_chan > 1 && chan_stride % 4 != 0) return false;
    return true;
}

// Workgroup order of a forward launch (block_of).  Measured on MI355X (profiles/r01_apply_kernels):
// when the gathered array (density columns, or the image for a transposed CSR) outgrows one XCD's
// 4 MB L2, runs of 64 blocks per XCD keep its lines L2-resident (C3 forward f32 350 -> 268 us, f64
// 596 -> 366 us; adjoint f64 377 -> 331 us); when the whole grid is resident at once (one wave of
// <= 6 blocks per CU), one contiguous range per XCD cuts the first-touch misses (C2 forward f32
// 7.0 -> 6.7 us); otherwise (the array fits every L2, several waves) dispatch order is as fast or
// faster (C5 f64 64 vs 68 us with runs of 64).  Round 2 (4,2,4 bricks, profiles/r02_xcd_chunk_sweep):
// runs of 64 also win for multi-wave grids whose array is 1-4 MB (C5 f64 forward 45.5 -> 44.0 us;
// C3 keeps 64: f32 204.8 us against 208.3 / 210.1 at 32 / 128); C5 f32 (1 MB) stays in dispatch order.
// A time-paired CSR (sphrt_csr.order bit 1: each view reads its own time slice of T * vol
// columns) takes one contiguous range per XCD, so that an XCD's rays stay on few slices (C4: f32
// 20.3 -> 18.9 us, f64 28.4 -> 26.5 us against runs of 64).
static int fwd_chunk(const sphrt_csr* c, size_t elem) {
    const int64_t bytes = c->n_cols * (int64_t)elem;
    int k = (c->order & 2) ? INT32_MAX
            : bytes > (int64_t)(4 << 20) ? 64
            : c->n_blocks <= 256 * 6 ? INT32_MAX
            : bytes > (int64_t)(1 << 20) ? 64 : 0;
    return (c->order & 1) ? ~k : k;   // (block_of: reversed)
}

// Dispatch timing (sphrt_time_next_forward): the next forward launch on this thread brackets its
// main kernel with these HIP events, recorded by the dispatch itself (hipExtLaunchKernelGGL): the
// kernel's own start and end, as a kernel trace reports them, independent of how fast the host
// issues.  The stage pack and the fallback launch are not bracketed.  Consumed by one launch.
static thread_local hipEvent_t t_fwd_start = nullptr, t_fwd_stop = nullptr;

extern "C" int sphrt_time_next_forward(void* start_event, void* stop_event) {
    t_fwd_start = (hipEvent_t)start_event;
    t_fwd_stop = (hipEvent_t)stop_event;
    return 0;
}

#define FWD_LAUNCH(KERNEL, G, B, LDS, ST, ...)                                                   \
    do {                                                                                          \
        if (t_fwd_start || t_fwd_stop) {                                                          \
            hipEvent_t e0_ = t_fwd_start, e1_ = t_fwd_stop;                                       \
            t_fwd_start = t_fwd_stop = nullptr;                                                   \
            hipExtLaunchKernelGGL(KERNEL, G, B, (uint32_t)(LDS), ST, e0_, e1_, 0u, __VA_ARGS__);   \
        } else {                                                                                  \
            hipLaunchKernelGGL(KERNEL, G, B, LDS, ST, __VA_ARGS__);                               \
        }                                                                                         \
    } while (0)

template <typename T, typename L>
static int launch_forward(const sphrt_csr* c, const L* len, const T* density, int64_t n_chan,
                          int64_t chan_stride, int64_t div, T* out, int64_t ocs, void* stream) {
    constexpr int P = kPer;                         // segments per thread
    const dim3 grid((unsigned)c->n_blocks), block(kPass / P);
    StreamGuard guard(stream);
    hipStream_t st = (hipStream_t)stream;
    const int chunk = fwd_chunk(c, sizeof(T));
    StageMap sm;
    if (!stage_map(c, sm)) return fail("inconsistent brick staging fields");
#define FWD_ARGS(TabT, D, CS, COLS) c->blocks, c->vox, c->loc, (const TabT*)c->tab, len,    \
                       c->row_ray, c->empty_ray, D, n_chan, CS, div, out, ocs, c->n_rays,          \
                       c->n_segments, COLS, c->tab_stride, chunk
    if ((c->order & 4) && (n_chan != 1 || div > 0 || c->runs))
        return fail("dense output ranges need one channel, no time slices and no run records");
    const bool dense = (c->order & 4) != 0;        // (instantiations with DENSE)
    // (dense output ranges read the blocks of sphrt_csr_index_dense: their count at least)
    if (dense && c->n_blocks != c->n_segments / kDenseSegPerBlock + 1)
        return fail("dense output ranges need the blocks of sphrt_csr_index_dense");
    const T* td = sm.on ? (const T*)c->stage : density;      // what the table kernel gathers
    const int64_t tcs = sm.on ? c->stage_cols : chan_stride;
    if (div > 0) {
        FWD_LAUNCH((forward_kernel<T, L, kFwdDynamic, int32_t, false, P>), grid, block, 0, st,
                   FWD_ARGS(int32_t, density, chan_stride, c->n_cols), 0, (const int32_t*)nullptr);
    } else if (use_tables(c, td, n_chan, tcs, div)) {
        if (sm.on && (!c->stage || (int64_t)sizeof(T) * n_chan * c->stage_cols > c->stage_bytes))
            return fail("brick stage buffer missing or too small for this call");
        if (sm.on && !c->stage_packed) {   // natural -> brick layout, every channel
            const int64_t brick_rows = c->stage_cols / c->stage_brick[2];
            const dim3 pg((unsigned)((brick_rows + 255) / 256), (unsigned)imin64(n_chan, 65535));
            hipLaunchKernelGGL(stage_pack_kernel<T>, pg, dim3(256), 0, st, density, chan_stride,
                               n_chan, (uint32_t)c->stage_shape[0], sm, c->stage_cols, (T*)c->stage);
            if (int e = check_launch("stage_pack_kernel")) return e;
        }
        const bool edma = early_dma(c);
        // float64 tables that leave fewer than 4 workgroups per CU (over 40 KB of LDS): half
        // tables, 5 per CU (C5 forward f64 62.1 -> 53.0 us, transposed adjoint 58.8 -> 53.7 us).
        // Not below: C3's 34.8 KB tables (4 per CU) measured 364 -> 383 us with halves (more
        // resident workgroups, more L2 misses; few of its tables even need the second phase).
        // (the half-table kernel exists for the default segments per thread only: P == kPer)
        const bool half = sizeof(T) == 8 && P == kPer && edma &&
                          (size_t)(c->tab_stride + 1) * 32 > 40 * 1024 &&
                          c->tab_stride <= 2 * kHalfTab && half_tables_on();
        // early DMA rounds: as many 256-entry chunks as the largest table needs (at most
        // kGranEarly), so neither the LDS image nor the unconditional early DMAs exceed the
        // tables (C4's time-paired adjoint: 448-entry tables, 3 -> 2 chunks)
        const int ge = c->tab_stride <= kThreads ? 1 : c->tab_stride <= 2 * kThreads ? 2 : 3;
        size_t lds = (size_t)((half ? kHalfTab
                               : edma ? imax64(c->tab_stride, (int64_t)ge * kThreads)
                                      : c->tab_stride) + 1) * 4 * sizeof(T);   // + zero granule
        if (dense) lds += (size_t)kOutStage * sizeof(T);       // the staged output range
#define FWD_TABLE(TabT, E, R, H, D, G)                                                      \
        FWD_LAUNCH((forward_kernel<T, L, kFwdTable, TabT, E, P, R, H, D, G>), grid, block, lds, \
                   st, FWD_ARGS(TabT, td, tcs, table_cols(c)), 0, c->runs)
#define FWD_TABLE_R(TabT, E, H, G)                                                          \
        do {                                                                                      \
            if (dense) FWD_TABLE(TabT, E, false, H, true, G);                               \
            else if (c->runs) FWD_TABLE(TabT, E, true, H, false, G);                        \
            else FWD_TABLE(TabT, E, false, H, false, G);                                    \
        } while (0)
#define FWD_TABLE_E(TabT)                                                                   \
        do {                                                                                      \
            if (half) {                                                                           \
                if constexpr (sizeof(T) == 8 && P == kPer) {                                      \
                    FWD_TABLE_R(TabT, true, true, kGranEarly);                                    \
                }                                                                                 \
            } else if (edma && ge == 1) {                                                         \
                FWD_TABLE_R(TabT, true, false, 1);                                                \
            } else if (edma && ge == 2) {                                                         \
                FWD_TABLE_R(TabT, true, false, 2);                                                \
            } else if (edma) {                                                                    \
                FWD_TABLE_R(TabT, true, false, kGranEarly);                                       \
            } else {                                                                              \
                FWD_TABLE_R(TabT, false, false, kGranEarly);                                      \
            }                                                                                     \
        } while (0)
        if (c->tab_bytes == 2) {
            FWD_TABLE_E(uint16_t);
        } else {
            FWD_TABLE_E(int32_t);
        }
#undef FWD_TABLE_E
#undef FWD_TABLE_R
#undef FWD_TABLE
        if (c->n_fallback > 0) {   // (natural vox, natural density)
            if (int e = check_launch("forward_kernel<table>")) return e;
            if (dense)
                hipLaunchKernelGGL((forward_kernel<T, L, kFwdGather, int32_t, false, P, false, false,
                                                   true>), grid, block, 0, st,
                                   FWD_ARGS(int32_t, density, chan_stride, c->n_cols), 1, nullptr);
            else
                hipLaunchKernelGGL((forward_kernel<T, L, kFwdGather, int32_t, false, P>), grid, block,
                                   0, st, FWD_ARGS(int32_t, density, chan_stride, c->n_cols), 1,
                                   nullptr);
        }
    } else {
        if (dense)
            FWD_LAUNCH((forward_kernel<T, L, kFwdGather, int32_t, false, P, false, false, true>), grid,
                       block, 0, st, FWD_ARGS(int32_t, density, chan_stride, c->n_cols), 0,
                       (const int32_t*)nullptr);
        else
            FWD_LAUNCH((forward_kernel<T, L, kFwdGather, int32_t, false, P>), grid, block, 0, st,
                       FWD_ARGS(int32_t, density, chan_stride, c->n_cols), 0,
                       (const int32_t*)nullptr);
    }
#undef FWD_ARGS
    return check_launch(sizeof(T) == 4 ? "forward_kernel<f32>" : "forward_kernel<f64>");
}

extern "C" int sphrt_forward_f32(const sphrt_csr* c, const float* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, float* out, int64_t ocs,
                                 void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len32) return fail("the float32 forward needs the float32 length copy (len32)");
    if (c->n_rays == 0) return 0;
    return launch_forward(c, c->len32, density, n_chan, chan_stride, div, out, ocs, stream);
}

extern "C" int sphrt_forward_f64(const sphrt_csr* c, const double* density, int64_t n_chan,
                                 int64_t chan_stride, int64_t div, double* out, int64_t ocs,
                                 void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len) return fail("missing segment lengths");
    if (c->n_rays == 0) return 0;
    return launch_forward(c, c->len, density, n_chan, chan_stride, div, out, ocs, stream);
}

extern "C" int sphrt_adjoint_accumulate(const sphrt_csr* c, const void* y, int y_is_f64,
                                        int64_t n_chan, int64_t ycs, int64_t div, double* acc,
                                        int64_t chan_stride, void* stream) {
    if (int e = check_csr(c, n_chan, div)) return e;
    if (!c->len) return fail("missing segment lengths");
    if (c->n_rays == 0) return 0;
    StreamGuard guard(stream);
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
