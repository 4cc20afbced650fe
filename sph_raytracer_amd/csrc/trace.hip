// trace.hip — fused per-ray trace on gfx950 (replaces trace_indices, raytracer.py:48-230).
//
// The reference materialises every ray's K = 2(nr+1)+2(ne+1)+(na+1)+1 candidate crossings,
// sorts them, forward-fills three (K,)-long region rows and differences the distances.  Here a
// tile of 64 rays is screened one ray per lane; every ray that can produce a segment is then
// traced by the whole wave:
//   1. lanes solve disjoint boundaries of each family (solve.hpp) and append the finite,
//      non-negative crossings to a per-wave LDS list (ballot + mbcnt compaction); the most
//      negative finite distance is reduced across the wave (it bounds the behind-start segment);
//   2. the list is sorted by (distance, candidate index) — a total order equal to a stable sort
//      of the reference's concatenation — in registers (<= 512 entries: one 64-bit composite
//      key per entry; the shells' crossings listed as one pre-sorted run and merged with the
//      sorted rest in one bitonic stage) or in LDS (longer lists);
//   3. the sorted list is scanned (forward fill of the r/e/a rows: in registers, lane-major,
//      for lists of <= 512 entries), differenced and the non-zero in-grid segments compacted, in
//      order, back into LDS;
//   4. depending on MODE the segments are counted, copied to the CSR, or integrated against
//      the density right away (no-store mode).
// Nothing of size K ever reaches HBM.
//
// Exact ties.  The reference orders equal distances the way libstdc++'s introsort happens to
// (torch.sort is unstable, raytracer.py:131).  That order only matters when two crossings that
// update the same region row coincide exactly — in practice a ray that starts exactly on a
// boundary (e.g. an orbit view at azimuth 0 with a boundary at 0).  The wave path detects such
// tie groups and defers the ray to exact_kernel, which rebuilds all K candidates in the
// reference's concatenation order, runs the emulated introsort (introsort.hpp) and walks the
// sorted list exactly like trace_indices, one wave per deferred ray with its list in LDS.
#include <climits>

#include "common.hpp"
#include "introsort.hpp"
#include "solve.hpp"

namespace sphrt {

// COUNT / FILL: the two-pass trace (counts, then segments at row_ptr).  BOUND (screen only) and
// EMIT: the one-pass trace — an upper bound of every ray's segment count from its geometry, then
// one pass that writes each ray's segments into its bounded slot of a staging CSR (compacted
// afterwards).  INTEGRATE: the no-store forward.
enum { MODE_COUNT = 0, MODE_FILL = 1, MODE_INTEGRATE = 2, MODE_EMIT = 3, MODE_BOUND = 4 };
constexpr int kNone = 0x7fffffff;  // "no update" in the forward-fill scans
constexpr int kWavesPerBlock = 4;

constexpr size_t kLdsBytes = 160 * 1024;        // LDS per CU; one workgroup may take all of it


__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
// Wave inclusive scans on DPP lane moves: row_shr 1, 2, 4, 8 inside rows of 16, then
// row_bcast 15 (rows 1, 3) and row_bcast 31 (rows 2, 3); lanes without a source read `id`.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp_or(int x, int id) {
    return __builtin_amdgcn_update_dpp(id, x, CTRL, ROWS, 0xf, false);
}
template <typename Op>
__device__ __forceinline__ int wave_scan(int v, int id, Op op) {
    v = op(dpp_or<0x111>(v, id), v);
    v = op(dpp_or<0x112>(v, id), v);
    v = op(dpp_or<0x114>(v, id), v);
    v = op(dpp_or<0x118>(v, id), v);
    v = op(dpp_or<0x142, 0xa>(v, id), v);
    v = op(dpp_or<0x143, 0xc>(v, id), v);
    return v;
}
// inclusive scan with op(a, b) = (b != none) ? b : a  — "last update wins" forward fill
__device__ __forceinline__ int scan_last(int v, int /*lane*/) {
    return wave_scan(v, kNone, [](int a, int b) { return b != kNone ? b : a; });
}

// ---- lane exchanges without the LDS crossbar ------------------------------------------------
// xlane<X>(x): the value x holds in lane (lane ^ X), X a compile-time constant: DPP quad
// permutes and row (half-)mirrors inside 16 lanes, row shifts for xor 4 / 8, a swizzle for
// xor 16 / 31 inside 32 lanes, the gfx950 32-lane swap for xor 32.
// xor 4 / 8 through ds_swizzle (the LDS crossbar, no VALU issue) instead of two row shifts and a
// select (three VALU instructions per dword).  Trace kernel, same box, round 4: C3 3126 -> 3113,
// C5 525 -> 520, C2 124.6 -> 122.4 us (profiles/r04_trace_ab.txt).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
template <int X>
__device__ __forceinline__ uint32_t xlane(uint32_t x, int lane) {
    if constexpr (X == 1) return dpp_mov<0xB1>(x);                 // quad_perm [1,0,3,2]
    else if constexpr (X == 2) return dpp_mov<0x4E>(x);            // quad_perm [2,3,0,1]
    else if constexpr (X == 3) return dpp_mov<0x1B>(x);            // quad_perm [3,2,1,0]
    else if constexpr (X == 7) return dpp_mov<0x141>(x);           // row_half_mirror
    else if constexpr (X == 15) return dpp_mov<0x140>(x);          // row_mirror
    else if constexpr (X == 4 || X == 8 || X == 16 || X == 31) {
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (X << 10) | 0x1F);
    } else if constexpr (X == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return lane < 32 ? (uint32_t)r[1] : (uint32_t)r[0];
    } else if constexpr (X == 63) {
        return xlane<32>(xlane<31>(x, lane), lane);
    } else {
        return (uint32_t)__shfl_xor((int)x, X);
    }
}
template <int X>
__device__ __forceinline__ uint64_t xlane64(uint64_t x, int lane) {
    return (uint64_t)xlane<X>((uint32_t)x, lane) | ((uint64_t)xlane<X>((uint32_t)(x >> 32), lane) << 32);
}

// One compare-exchange layer of the ascending-only ("flip") bitonic network over 64*M keys,
// lane-major: element e = lane*M + i, partner e ^ MASK.  Bits of MASK below M pair registers of
// the same lane (no lane exchange: the 1-, 2-... layers, which every stage ends with); the rest
// is a lane xor.  (The register-major order e = i*64 + lane exchanged lanes in all but the top
// layers: 33 of 36 layers at M = 4 against 21 now.)  The keys are single 64-bit words (the
// composite keys below): one compare and two selects per element and layer.
template <int M>
constexpr int kLogM = M == 1 ? 0 : M == 2 ? 1 : M == 4 ? 2 : 3;
template <int M, int MASK>
__device__ __forceinline__ void cas_layer(uint64_t (&k)[M], int lane) {
    constexpr int IM = MASK & (M - 1);          // register-index xor
    constexpr int LM = MASK >> kLogM<M>;        // lane xor
    if constexpr (LM == 0) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int pi = i ^ IM;
            if (pi < i) continue;                   // each in-lane pair once: lower keeps the min
            const uint64_t ka = k[i], kb = k[pi];
            const bool sw = kb < ka;
            k[i] = sw ? kb : ka;
            k[pi] = sw ? ka : kb;
        }
    } else {
        uint64_t nk[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int pi = i ^ IM;
            const uint64_t ok = xlane64<LM>(k[pi], lane);
            const int e = lane * M + i;
            const int pe = (lane ^ LM) * M + pi;
            // keys are distinct except the identical padding entries
            const bool lt = ok < k[i];
            const bool take = (e < pe) ? lt : !lt;
            nk[i] = take ? ok : k[i];
        }
#pragma unroll
        for (int i = 0; i < M; ++i) k[i] = nk[i];
    }
}

// half-cleaner layers J, J/2, ..., 1 and the stages KK, 2KK, ... P of the network
template <int M, int J>
__device__ __forceinline__ void half_cleaners(uint64_t (&k)[M], int lane) {
    if constexpr (J > 0) {
        cas_layer<M, J>(k, lane);
        half_cleaners<M, J / 2>(k, lane);
    }
}
template <int M, int KK>
__device__ __forceinline__ void sort_stages(uint64_t (&k)[M], int lane) {
    if constexpr (KK <= 64 * M) {
        cas_layer<M, KK - 1>(k, lane);   // flip: mirror partner inside the KK-block
        half_cleaners<M, KK / 4>(k, lane);
        sort_stages<M, KK * 2>(k, lane);
    }
}

// Sorted composite keys k (lane-major, padding ~0 at the end) -> keys[e] / pays[e] hold the
// (distance bits, candidate << 16 | region + 2) pairs, the layout the rest of the trace reads
// (pays[cand] holds the replaced low bits and the region until then).  Composite-key order is
// the (distance, candidate) order unless two different distances agree above the replaced bits —
// e.g. the coinciding half-planes a = -pi and a = pi of a full circle, a few ulps apart, which
// ~5 % of the BASELINE rays cross — or a pre-sorted run held equal distances out of candidate
// order.  The full distances are checked on the way out; true means some adjacent pair is out of
// order (fix_near_ties repairs it).
template <int M>
__device__ __forceinline__ int finish_sort(const uint64_t (&k)[M], uint64_t* keys,
                                           uint32_t* pays, int F, int lane, uint64_t cmask) {
    uint64_t tb[M];
    uint32_t py[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const uint32_t cand = (uint32_t)(k[i] & cmask);
        const uint32_t info = lane * M + i < F ? pays[cand] : 0u;
        tb[i] = (k[i] & ~cmask) | (uint64_t)(info >> 16);
        py[i] = (cand << 16) | (info & 0xffffu);
    }
    bool bad = false, eq = false;
#pragma unroll
    for (int i = 1; i < M; ++i) {
        bad |= lane * M + i < F && tb[i] < tb[i - 1];
        eq |= lane * M + i < F && tb[i] == tb[i - 1];
    }
    const uint64_t prev = (uint64_t)__shfl_up((long long)tb[M - 1], 1);
    bad |= lane > 0 && lane * M < F && tb[0] < prev;
    eq |= lane > 0 && lane * M < F && tb[0] == prev;
    wave_sync();
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        if (e < F) {
            keys[e] = tb[i];
            pays[e] = py[i];
        }
    }
    wave_sync();
    // bit 0: adjacent disorder (fix_near_ties); bit 1: equal adjacent distances (ambiguous_ties
    // has something to look at — after a repair, equal ones may have been apart)
    return (__ballot(bad) != 0 ? 3 : 0) | (__ballot(eq) != 0 ? 2 : 0);
}

// The list trace_one builds (composite keys, see there): the shells' near crossings at
// keys[0, Sn) in shell order — descending distances — then the cone / half-plane / start entries
// up to keys[F - Sf), and the shells' far crossings at keys[cap - 1], keys[cap - 2], ... in shell
// order — ascending distances.
//
// Full sort: the bitonic network over all F <= 64*M entries.
template <int M>
__device__ int sort_regs(uint64_t* keys, uint32_t* pays, int F, int Sf, int cap, int lane,
                          uint64_t cmask) {
    uint64_t k[M];
    const int front = F - Sf;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        k[i] = e < front ? keys[e] : e < F ? keys[cap - 1 - (e - front)] : ~0ull;
    }
    sort_stages<M, 2>(k, lane);
    return finish_sort<M>(k, keys, pays, F, lane, cmask);
}

// Sort + merge: every operation of a shell crossing's distance is monotone in R^2, so the shell
// entries read as near ones outermost-first then far ones innermost-first are one ascending run
// (as composite keys, up to equal distances).  Only the other O entries go through a network
// (64*M2 >= O, a smaller power of two than the whole list's); with them descending behind the
// shell run and the padding between, the list is bitonic and one merge stage (log2(64 M)
// half-cleaner layers) sorts it.  C3 (F ~153, ~88 shell entries): 28 + 8 layers on 2 + 4
// registers instead of 36 on 4.
// Merge path: the shell run A (ascending composite keys: keys[Sn-1] ..
// keys[0], then keys[cap-1], keys[cap-2], ...) and the sorted other entries B (keys[Sn ..
// Sn+O)) merged by rank — lane L finds how many of A precede output L*M (a binary search along
// its diagonal), then takes its M outputs in turn — instead of log2(64 M) half-cleaner layers
// over M registers.  The same sorted sequence whenever A is strictly ascending (merge_sort
// checks that first and keeps the bitonic merge otherwise: equal shell distances, repeated
// radii).
// On for lists of more than 128 entries (M >= 4): trace kernel, same box, C3 3193 -> 3175 us,
// C5 540 -> 530 us; C2's shorter lists (M <= 2) measured 123.5 -> 125.3 us and keep the bitonic
// merge.
__device__ __forceinline__ uint64_t shell_run(const uint64_t* keys, int Sn, int cap, int i) {
    return i < Sn ? keys[Sn - 1 - i] : keys[cap - 1 - (i - Sn)];
}
template <int M>
__device__ __forceinline__ void merge_path(const uint64_t* keys, int F, int Sn, int S, int cap,
                                           int lane, uint64_t (&k)[M]) {
    const int O = F - S;
    const uint64_t* B = keys + Sn;
    const int p0 = lane * M;
    int lo = max(0, p0 - O), hi = min(p0, S);
    while (lo < hi) {                      // first A entry not among the first p0 outputs
        const int mid = (lo + hi) >> 1;
        if (shell_run(keys, Sn, cap, mid) < B[p0 - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int ai = lo, bj = p0 - lo;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        k[i] = ~0ull;
        if (p0 + i < F) {
            const uint64_t a = ai < S ? shell_run(keys, Sn, cap, ai) : ~0ull;
            const uint64_t b = bj < O ? B[bj] : ~0ull;
            const bool ta = ai < S && (bj >= O || a < b);
            k[i] = ta ? a : b;
            ai += ta ? 1 : 0;
            bj += ta ? 0 : 1;
        }
    }
}
__device__ __forceinline__ bool shell_run_ascending(const uint64_t* keys, int Sn, int S, int cap,
                                                    int lane) {
    bool ok = true;
    for (int i = lane + 1; i < S; i += 64)
        ok &= shell_run(keys, Sn, cap, i - 1) < shell_run(keys, Sn, cap, i);
    return __ballot(!ok) == 0;
}

template <int M, int M2>
__device__ int merge_sort(uint64_t* keys, uint32_t* pays, int F, int Sn, int Sf, int cap,
                           int lane, uint64_t cmask) {
    const int S = Sn + Sf, O = F - S;
    {
        uint64_t k[M2];
#pragma unroll
        for (int i = 0; i < M2; ++i) {
            const int e = lane * M2 + i;
            k[i] = e < O ? keys[Sn + e] : ~0ull;
        }
        sort_stages<M2, 2>(k, lane);
        wave_sync();
#pragma unroll
        for (int i = 0; i < M2; ++i) {
            const int e = lane * M2 + i;
            if (e < O) keys[Sn + e] = k[i];
        }
        wave_sync();
    }
    constexpr int P = 64 * M;
    uint64_t k[M];
    if (M >= 4 && shell_run_ascending(keys, Sn, S, cap, lane)) {
        merge_path<M>(keys, F, Sn, S, cap, lane, k);
        return finish_sort<M>(k, keys, pays, F, lane, cmask);
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        k[i] = e < Sn ? keys[Sn - 1 - e]
             : e < S ? keys[cap - 1 - (e - Sn)]
             : e >= P - O ? keys[Sn + (P - 1 - e)] : ~0ull;
    }
    half_cleaners<M, 32 * M>(k, lane);
    return finish_sort<M>(k, keys, pays, F, lane, cmask);
}

__device__ __forceinline__ bool pair_less(uint64_t ka, uint32_t pa, uint64_t kb, uint32_t pb) {
    return ka < kb || (ka == kb && pa < pb);
}

// Odd-even transposition passes over the (distance bits, payload) pairs in LDS until no adjacent
// pair is out of order: after the composite-key sort only entries whose distances agree above
// the candidate bits can be, each inside its (contiguous, small) group, so one or two rounds
// finish it.  The result is the (distance, candidate) order exactly.
__device__ void fix_near_ties(uint64_t* keys, uint32_t* pays, int F, int lane) {
    for (;;) {
        bool swapped = false;
        for (int par = 0; par < 2; ++par) {
            for (int i = 2 * lane + par; i + 1 < F; i += 128) {
                const uint64_t ka = keys[i], kb = keys[i + 1];
                const uint32_t pa = pays[i], pb = pays[i + 1];
                if (pair_less(kb, pb, ka, pa)) {
                    keys[i] = kb; pays[i] = pb;
                    keys[i + 1] = ka; pays[i + 1] = pa;
                    swapped = true;
                }
            }
            wave_sync();
        }
        if (__ballot(swapped) == 0) return;
    }
}
__device__ __forceinline__ void cas_lds(uint64_t* keys, uint32_t* pays, int i, int l) {
    uint64_t ki = keys[i], kl = keys[l];
    uint32_t pi = pays[i], pl = pays[l];
    if (pair_less(kl, pl, ki, pi)) {
        keys[i] = kl; pays[i] = pl;
        keys[l] = ki; pays[l] = pi;
    }
}
// The bitonic network in LDS for long lists (F > 512), on (distance bits, payload) pairs: such
// rays list their crossings a second time in that layout.  Virtual +inf padding beyond F never
// moves (ascending-only comparators), so storage is exactly F entries.
__device__ void sort_lds(uint64_t* keys, uint32_t* pays, int F, int lane) {
    int P = 1;
    while (P < F) P <<= 1;
    for (int kk = 2; kk <= P; kk <<= 1) {
        const int half = kk >> 1;
        for (int q = lane; q < (P >> 1); q += 64) {
            const int blk = q / half, off = q - blk * half;
            const int i = blk * kk + off, l = blk * kk + kk - 1 - off;
            if (l < F) cas_lds(keys, pays, i, l);
        }
        wave_sync();
        for (int j = kk >> 2; j > 0; j >>= 1) {
            for (int q = lane; q < (P >> 1); q += 64) {
                const int i = (q / j) * 2 * j + (q % j), l = i + j;
                if (l < F) cas_lds(keys, pays, i, l);
            }
            wave_sync();
        }
    }
}

// A screened hit ray as the trace kernel reads it: its solve set-up (make_ray, evaluated once by
// the screen lane instead of by all 64 lanes of the tracing wave: six IEEE divisions and four
// square roots per ray), start voxel and ray id — one 128-byte record, read with scalar loads by
// the wave that traces it (no broadcast index arithmetic and no RaysDev in the trace kernel's
// registers).
struct HitRay {
    RayGeo g;
    double t1c_o;       // half the chord of the outer sphere, sqrt(r_outer^2 - dd^2)
    int32_t s[3];
    int32_t ray;
};
static_assert(sizeof(HitRay) == 128, "HitRay is one 128-byte record");

template <typename T>
struct TraceOut {
    int32_t* counts;          // COUNT
    const int64_t* row_ptr;   // FILL
    int32_t* vox;
    double* len;
    const T* density;         // INTEGRATE
    int64_t n_chan, chan_stride, ray_chan_div;
    T* out;
    int64_t out_chan_stride;
    unsigned long long* n_deferred;  // workspace: deferred-ray counter
    int64_t* deferred;               // workspace: deferred ray ids
    unsigned* n_hits;                // workspace: screened hit-ray counter
    HitRay* hits;                    // workspace: hit rays
    unsigned long long* n_over;      // EMIT: rays whose segments exceed their bound
    unsigned long long* n_heap;      // workspace: depth-limit ranges, rank-sorted / heap-sorted
    int wedge;                       // solve only the half-planes of a line's azimuth wedge
};

// EMIT: ray `ray` has `cnt` segments; its staging slot is [row_ptr[ray], row_ptr[ray + 1]) (the
// scanned bounds).  Returns the slot start, or -1 (counted in n_over) when they do not fit.
template <typename T>
__device__ __forceinline__ int64_t emit_slot(const TraceOut<T>& o, int64_t ray, int64_t cnt,
                                             bool leader) {
    return emit_slot(o, ray, cnt, leader, o.row_ptr[ray], o.row_ptr[ray + 1]);
}
// (the same with the slot bounds b0 = row_ptr[ray], b1 = row_ptr[ray + 1] already loaded)
template <typename T>
__device__ __forceinline__ int64_t emit_slot(const TraceOut<T>& o, int64_t ray, int64_t cnt,
                                             bool leader, int64_t b0, int64_t b1) {
    const int64_t cap = b1 - b0;
    if (leader) o.counts[ray] = (int32_t)cnt;
    if (cnt <= cap) return b0;
    if (leader) atomicAdd(o.n_over, 1ull);
    return -1;
}

// region rows a candidate updates: bit0 r, bit1 e, bit2 a (start entry: all)
__device__ __forceinline__ int update_mask(uint32_t pay, int r_lim, int e_lim, int start_c) {
    const int cand = (int)(pay >> 16);
    const int reg = (int)(pay & 0xffffu) - 2;
    if (cand == start_c) return 7;
    if (cand < r_lim) return 1;
    if (reg == -2) return 0;
    return cand < e_lim ? 2 : 4;
}

__device__ __forceinline__ int scan_max(int v, int /*lane*/) {
    return wave_scan(v, INT_MIN, [](int a, int b) { return max(a, b); });
}

// value a candidate writes into region row `row` (0 r, 1 e, 2 a); start entry: the start voxel
__device__ __forceinline__ int row_value(uint32_t pay, int row, int start_c, const int* sv) {
    return (int)(pay >> 16) == start_c ? sv[row] : (int)(pay & 0xffffu) - 2;
}

// Does any group of exactly equal distances hold two crossings that write DIFFERENT values into
// the same region row?  Only then does the reference's tie order change a row's value after the
// group (the segments inside a group have zero length).  Equal-valued ties — a double root of
// the e = pi/2 "cone", a tangent sphere, a boundary crossing that re-enters the start voxel —
// are order-independent and stay on the fast path.
__device__ bool tie_groups_ambiguous(const uint64_t* keys, const uint32_t* pays, int F, int lane,
                                     int r_lim, int e_lim, int start_c, const int* sv);
__device__ bool ambiguous_ties(const uint64_t* keys, const uint32_t* pays, int F, int lane,
                               int r_lim, int e_lim, int start_c, const int* sv) {
    bool any = false;
    for (int c0 = 1; c0 < F; c0 += 64) {
        const int e = c0 + lane;
        any |= __ballot(e < F && keys[e] == keys[e - 1]) != 0;
    }
    if (!any) return false;
    return tie_groups_ambiguous(keys, pays, F, lane, r_lim, e_lim, start_c, sv);
}
// (the analysis itself, for a list known to hold equal adjacent distances)
__device__ bool tie_groups_ambiguous(const uint64_t* keys, const uint32_t* pays, int F, int lane,
                                     int r_lim, int e_lim, int start_c, const int* sv) {
    int grp = 0;                          // start of the current tie group (carried)
    int last[3] = {-1, -1, -1};           // last updater of each row so far (carried)
    bool amb = false;
    for (int c0 = 0; c0 < F; c0 += 64) {
        const int e = c0 + lane;
        const bool real = e < F;
        const uint32_t p = real ? pays[e] : 0u;
        const bool gs = real && (e == 0 || keys[e] != keys[e - 1]);
        const int mask = real ? update_mask(p, r_lim, e_lim, start_c) : 0;
        const int g = max(scan_max(gs ? e : -1, lane), grp);
#pragma unroll
        for (int row = 0; row < 3; ++row) {
            const bool upd = (mask >> row) & 1;
            const int u_inc = max(scan_max(upd ? e : -1, lane), last[row]);
            int u_exc = __shfl_up(u_inc, 1);
            if (lane == 0) u_exc = last[row];
            if (upd && u_exc >= g &&
                row_value(pays[u_exc], row, start_c, sv) != row_value(p, row, start_c, sv))
                amb = true;
            last[row] = __shfl(u_inc, 63);
        }
        grp = __shfl(g, 63);
    }
    return __ballot(amb) != 0;
}

// Forward fill, lengths and compaction (trace_one phase 3) over a sorted list of F <= 64*M
// entries read lane-major — lane L holds entries L*M .. L*M + M - 1: each lane carries the
// region rows through its M entries in registers, and one wave scan per row joins the lanes
// (the chunk loop scans each row once per 64 entries), one prefix sum places the segments.
// The rules are the chunk loop's: an entry updates its family's row (the start entry all
// three), a segment runs to the next entry's distance, and it is kept when its length is
// positive and finite and its voxel inside the grid.
struct FillState {
    int sr, se, sa;        // start voxel (the start entry's update)
    int r0, e0, a0;        // rows before the first entry
    int r_lim, e_lim, start_c;
};
// STORE: kFillNone (count only), kFillLds (the segments compacted into seg_len / seg_vox in LDS,
// for the no-store forward and the LDS-list path), kFillGlobal (straight from the registers into
// the CSR: seg_len / seg_vox are the output arrays, the ray's segments start at gbase; stored only
// when head + count <= gcap — an emit slot that fits; no LDS round trip, no copy loop).
enum { kFillNone = 0, kFillLds = 1, kFillGlobal = 2 };
template <int M, int STORE>
__device__ int fill_regs(const GridDev& G, const uint64_t* keys, const uint32_t* pays, int F,
                         int lane, const FillState& fs, double* seg_len, int32_t* seg_vox,
                         int64_t gbase = 0, int64_t gcap = 0, int head = 0) {
    uint64_t kb[M];
    int ur[M], ue[M], ua[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        kb[i] = e < F ? keys[e] : 0ull;
        const uint32_t p = e < F ? pays[e] : 0u;
        const int cand = (int)(p >> 16);
        const int reg = (int)(p & 0xffffu) - 2;
        ur[i] = ue[i] = ua[i] = kNone;
        if (e < F) {
            if (cand == fs.start_c) {
                ur[i] = fs.sr; ue[i] = fs.se; ua[i] = fs.sa;
            } else if (cand < fs.r_lim) {
                ur[i] = reg;
            } else if (cand < fs.e_lim) {
                if (reg != -2) ue[i] = reg;
            } else {
                if (reg != -2) ua[i] = reg;
            }
        }
        if (i > 0) {
            if (ur[i] == kNone) ur[i] = ur[i - 1];
            if (ue[i] == kNone) ue[i] = ue[i - 1];
            if (ua[i] == kNone) ua[i] = ua[i - 1];
        }
    }
    // rows entering this lane's entries: the last update in the lanes before it
    int pr = __shfl_up(scan_last(ur[M - 1], lane), 1);
    int pe = __shfl_up(scan_last(ue[M - 1], lane), 1);
    int pa = __shfl_up(scan_last(ua[M - 1], lane), 1);
    if (lane == 0 || pr == kNone) pr = fs.r0;
    if (lane == 0 || pe == kNone) pe = fs.e0;
    if (lane == 0 || pa == kNone) pa = fs.a0;
    const uint64_t next0 = (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)kb[0], 1) |
                           ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(kb[0] >> 32), 1) << 32);
    double len[M];
    int vox[M];
    bool ok[M];
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        const int r = ur[i] != kNone ? ur[i] : pr;
        const int ee = ue[i] != kNone ? ue[i] : pe;
        const int a = ua[i] != kNone ? ua[i] : pa;
        const double t = __longlong_as_double((long long)kb[i]);
        const double tn = e + 1 >= F ? kInf
                        : __longlong_as_double((long long)(i + 1 < M ? kb[i + 1] : next0));
        len[i] = tn - t;
        ok[i] = e < F && len[i] > 0.0 && __builtin_isfinite(len[i]) && r >= 0 && r < G.nr &&
                ee >= 0 && ee < G.ne && a >= 0 && a < G.na;
        vox[i] = (r * G.ne + ee) * G.na + a;
        cnt += ok[i] ? 1 : 0;
    }
    const int incl = wave_scan(cnt, 0, [](int x, int y) { return x + y; });
    const int total = __builtin_amdgcn_readlane(incl, 63);
    if (STORE == kFillLds) {
        wave_sync();
        int pos = incl - cnt;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            if (ok[i]) {
                seg_len[pos] = len[i];
                seg_vox[pos] = vox[i];
                ++pos;
            }
        }
        wave_sync();
    } else if (STORE == kFillGlobal && head + total <= gcap) {
        int64_t pos = gbase + (incl - cnt);
#pragma unroll
        for (int i = 0; i < M; ++i) {
            if (ok[i]) {
                seg_len[pos] = len[i];
                seg_vox[pos] = vox[i];
                ++pos;
            }
        }
    }
    return total;
}

__device__ __forceinline__ void load_ray(const RaysDev& R, int64_t i, double* x, double* d,
                                         int* s) {
    int64_t xo = 0, ro = 0;
    if (R.n <= 0x7fffffff) {
        // 32-bit index arithmetic (a 64-bit division is a long software sequence on the GPU)
        uint32_t rem = (uint32_t)i;
#pragma unroll
        for (int dd = kMaxDims - 1; dd >= 0; --dd) {
            if (dd < R.ndim) {
                const uint32_t sz = (uint32_t)R.shape[dd];
                const uint32_t q = rem / sz, c = rem - q * sz;
                rem = q;
                xo += (int64_t)c * R.xs_stride[dd];
                ro += (int64_t)c * R.rays_stride[dd];
            }
        }
    } else {
        int64_t rem = i;
#pragma unroll
        for (int dd = kMaxDims - 1; dd >= 0; --dd) {
            if (dd < R.ndim) {
                const int64_t sz = R.shape[dd];
                const int64_t c = rem % sz;
                rem /= sz;
                xo += c * R.xs_stride[dd];
                ro += c * R.rays_stride[dd];
            }
        }
    }
    x[0] = R.xs[xo]; x[1] = R.xs[xo + 1]; x[2] = R.xs[xo + 2];
    d[0] = R.rays[ro]; d[1] = R.rays[ro + 1]; d[2] = R.rays[ro + 2];
    const int32_t* sp = R.start + 4 * (xo / 3);
    s[0] = sp[0]; s[1] = sp[1]; s[2] = sp[2];
}

// First boundary j < n with ok(j) (n when none), wave-uniform.
template <typename Ok>
__device__ __forceinline__ int first_may_cross(int n, int lane, Ok ok) {
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        const uint64_t m = __ballot(j < n && ok(j));
        if (m) return j0 + __builtin_ctzll(m);
    }
    return n;
}

// Trace ray `ray` (wave-uniform) with the whole wave.  keys/pays: this wave's LDS list.
template <int MODE, typename T>
__device__ void trace_one(const GridDev& G, const RayGeo& g, const double t1c_o,
                          const int sr, const int se,
                          const int sa, const int64_t ray, uint64_t* keys, uint32_t* pays,
                          const int cap, const int lane, const TraceOut<T>& o) {
    // ---- 1. crossings -> LDS list (finite, t >= 0), min finite negative distance ----------
    // the ray's output slot bounds, loaded now: their round trip overlaps the solves instead of
    // following the sort
    int64_t slot0 = 0, slot1 = 0;
    if (MODE == MODE_FILL || MODE == MODE_EMIT) slot0 = o.row_ptr[ray];
    if (MODE == MODE_EMIT) slot1 = o.row_ptr[ray + 1];
    // The list holds composite keys: the distance's bits (t >= 0: ordered as unsigned integers)
    // with the low `cbits` bits replaced by the candidate index, so the sort moves and compares
    // one 64-bit word per entry; pays[candidate] keeps the replaced bits and the region.  A list
    // longer than the register sort takes (F > 512) is listed again as (distance bits, payload)
    // pairs for the LDS network (pair_fmt).
    const int cbits = 32 - __builtin_clz((unsigned)(G.K - 1));
    const uint64_t cmask = (1ull << cbits) - 1ull;
    bool pair_fmt = false;
    int base = 0;       // entries from the front
    int nfar = 0;       // shells' far crossings, from keys[cap - 1] down (composite layout)
    int s_near = 0;     // shells' near crossings: keys[0, s_near)
    double tneg = kInf;
    // the behind-start segment (and so tneg) exists only for a start inside the grid
    const bool start_ok = sr >= 0 && sr < G.nr && se >= 0 && se < G.ne && sa >= 0 && sa < G.na;
    auto note = [&](double t) {
        if (start_ok && t < 0.0 && __builtin_isfinite(t)) tneg = fmin(tneg, t);
    };
    auto push = [&](bool has, double t, int cand, int reg, bool far = false) {
        const uint64_t m = __ballot(has);
        far = far && !pair_fmt;
        if (has) {
            const int rank = __popcll(m & lanemask_lt(lane));
            const int pos = far ? cap - 1 - (nfar + rank) : base + rank;
            const uint64_t tb = (uint64_t)__double_as_longlong(t + 0.0);  // -0 -> +0
            if (pair_fmt) {
                keys[pos] = tb;
                pays[pos] = ((uint32_t)cand << 16) | (uint32_t)(reg + 2);
            } else {
                keys[pos] = (tb & ~cmask) | (uint64_t)cand;
                pays[cand] = ((uint32_t)(tb & cmask) << 16) | (uint32_t)(reg + 2);
            }
        }
        if (far) nfar += __popcll(m);
        else base += __popcll(m);
    };
    // Only crossings inside the outer sphere's span [t_lo, t_hi] are listed and sorted: after
    // the exit every segment lies outside (the r row stays -1: no sphere is crossed again), and
    // for a start outside the outer sphere (t_lo > 0) the e/a rows entering it are those of the
    // last cone / half-plane crossing before t_lo (the start entry's values if none).  That
    // entry state is reduced across the wave below; a tie of different values in its last group
    // defers the ray, exactly as a tie inside the list would.  (C2: 85 -> 62 entries per ray.)
    // t1c_o = sqrt(r_outer^2 - dd^2), sphere nr's half chord (from the hit record)
    const double t_lo = g.tc - t1c_o, t_hi = g.tc + t1c_o;
    const bool clip_lo = t_lo > 0.0;
    auto keep = [&](double t) {
        return __builtin_isfinite(t) && !(t < 0.0) && !(t > t_hi) && !(clip_lo && t < t_lo);
    };
    double pe_t, pa_t;                    // this lane's last e / a update before t_lo
    int pe_v, pa_v;
    bool pe_amb, pa_amb;                  // a second update at that distance, another value
    auto pre = [&](bool v, double t, int reg, double& bt, int& bv, bool& amb) {
        if (v && clip_lo && reg != -2 && !(t < 0.0) && t < t_lo) {
            if (t > bt) {
                bt = t;
                bv = reg;
                amb = false;
            } else if (t == bt && reg != bv) {
                amb = true;
            }
        }
    };

    const int nbr = G.nbr, nbe = G.nbe, nba = G.nba;
    // Half-planes: a line's azimuth turns monotonically, by less than pi, so over [0, t_hi] it
    // sweeps the wedge from A = x_xy to B = (x + t_hi w)_xy (turning with the sign of L, the z
    // of x cross w).  A half-plane outside that wedge has no crossing in [0, t_hi] — only one
    // behind the start or past the exit, or none — so, when the ray has no behind-start segment
    // (start outside the grid: the negative distances are unused), its solve could neither list
    // an entry nor be a pre-entry update.  With ascending angles the half-planes inside the
    // wedge are one cyclic run of indices [p_start, p_start + p_count) (mod nba), and only that
    // run is solved: 1 chunk of 64 instead of 3 at C3 (129 half-planes, a ~150 degree sweep for
    // rays through the ball), 1 instead of 2 at C5.  The wedge is widened by 1e-6 rad and lines
    // passing within 1e-6 of the z axis solve every half-plane: a skipped crossing is then far
    // (> 1e-13) from [0, t_hi] compared with its rounding, and its back-half test is decided by
    // |p_xy| >= 1e-6.  Exact: test_plane_wedge_exact (CSR bitwise the same without the wedge).
    int p_start = 0, p_count = nba;
    {
        const double Lz = g.x0 * g.w1 - g.x1 * g.w0;
        if (o.wedge && nba > 64 && G.a_asc && !start_ok && __builtin_isfinite(t_hi) &&
            Lz * Lz >= 1e-12 * (g.w0 * g.w0 + g.w1 * g.w1)) {
            const double b0 = g.x0 + t_hi * g.w0, b1 = g.x1 + t_hi * g.w1;
            const double tol_a = 1e-12 * (g.x0 * g.x0 + g.x1 * g.x1) * (Lz * Lz);
            const double tol_b = 1e-12 * (b0 * b0 + b1 * b1) * (Lz * Lz);
            int cnt = 0, n_starts = 0, first = -1;
            uint64_t m0 = 0;
            bool prev = false;                      // in(j0 - 1)
            for (int j0 = 0; j0 < nba; j0 += 64) {
                const int j = j0 + lane;
                bool in = false;
                if (j < nba) {
                    // turn * cross >= -1e-6 |.|, turn = sign(Lz), squared: no square roots
                    const double u0 = G.cos_a()[j], u1 = G.sin_a()[j];
                    const double ca = (g.x0 * u1 - g.x1 * u0) * Lz, cb = (u0 * b1 - u1 * b0) * Lz;
                    in = (ca >= 0.0 || ca * ca <= tol_a) && (cb >= 0.0 || cb * cb <= tol_b);
                }
                const uint64_t m = __ballot(in);
                uint64_t st = m & ~((m << 1) | (prev ? 1ull : 0ull));
                if (j0 == 0) {
                    m0 = m;
                    st &= ~1ull;                    // index 0: decided by in(nba - 1) below
                }
                cnt += __popcll(m);
                n_starts += __popcll(st);
                if (st && first < 0) first = j0 + __builtin_ctzll(st);
                prev = (m >> (min(64, nba - j0) - 1)) & 1ull;
            }
            if ((m0 & 1ull) && !prev) {
                ++n_starts;
                first = 0;
            }
            if (cnt == 0) {
                p_count = 0;
            } else if (n_starts == 1) {
                p_start = first;
                p_count = cnt;
            }
        }
    }
    int F;
    for (;;) {
        base = 0;
        nfar = 0;
        tneg = kInf;
        pe_t = pa_t = -1.0;
        pe_v = pa_v = 0;
        pe_amb = pa_amb = false;
        // Families of more than 64 boundaries solve only the 64-wide chunks that can list
        // something: from the first boundary whose solve can give a finite crossing
        // (sphere_may_cross / cone_may_cross: exact, the skipped solves would yield +inf only),
        // and chunks without such a boundary are skipped.  (C5: 65 shells / cones, one chunk
        // instead of two; C3: 129, ~2 instead of 3.)  Families of <= 64 boundaries keep the
        // single chunk (no pre-pass).
        auto sph_ok = [&](int j) { return sphere_may_cross(G, g, j); };
        auto cone_ok = [&](int j) { return cone_may_cross(G, g, j); };
        for (int j0 = nbr > 64 ? first_may_cross(nbr, lane, sph_ok) : 0; j0 < nbr; j0 += 64) {
            const int j = j0 + lane;
            const bool v = j < nbr;
            if (nbr > 64 && __ballot(v && sph_ok(j)) == 0) continue;
            double ti = kInf, to = kInf;
            int ri = 0, ro = 0, ni, no;
            if (v) sphere_solve(G, g, j, ti, ri, to, ro, ni, no);
            note(ti);
            note(to);
            push(v && keep(ti), ti, j, ri);
            // a double root (tangent sphere, the e = pi/2 "cone") writing the same region twice at
            // the same distance changes nothing in the forward fill: keep one entry, so the group is
            // no exact tie (the tie analysis below only runs for real ties)
            push(v && keep(to) && !(to == ti && ro == ri), to, nbr + j, ro, true);
        }
        s_near = base;
        const int ce0 = 2 * nbr;
        for (int j0 = nbe > 64 ? first_may_cross(nbe, lane, cone_ok) : 0; j0 < nbe; j0 += 64) {
            const int j = j0 + lane;
            const bool v = j < nbe;
            ConeQuad q{};
            if (v) q = cone_coeffs(G, g, j);   // once for the chunk test and the solve
            if (nbe > 64 && __ballot(v && cone_q_may_cross(G, q)) == 0) continue;
            double ta = kInf, tb = kInf;
            int ra = 0, rb = 0, na_, nb_;
            if (v) cone_solve_q(G, g, j, q, ta, ra, tb, rb, na_, nb_);
            note(ta);
            note(tb);
            pre(v, ta, ra, pe_t, pe_v, pe_amb);
            pre(v, tb, rb, pe_t, pe_v, pe_amb);
            push(v && keep(ta), ta, ce0 + j, ra);
            push(v && keep(tb) && !(tb == ta && rb == ra), tb, ce0 + nbe + j, rb);
        }
        const int ca0 = 2 * nbr + 2 * nbe;
        for (int k0 = 0; k0 < p_count; k0 += 64) {
            const bool v = k0 + lane < p_count;
            int j = p_start + k0 + lane;
            if (j >= nba) j -= nba;
            double t = kInf;
            int r = 0, ng;
            if (v) plane_solve(G, g, j, t, r, ng);
            note(t);
            pre(v, t, r, pa_t, pa_v, pa_amb);
            push(v && keep(t), t, ca0 + j, r);
        }
        push(lane == 0 && !clip_lo, 0.0, G.K - 1, 0);  // the start entry (raytracer.py:111-122)
        F = base + nfar;
        if (pair_fmt || F <= 512) break;
        pair_fmt = true;
        wave_sync();
    }
    if (start_ok) tneg = wave_min(tneg);
    // rows entering the outer sphere (start outside): the last pre-entry update group per row
    int e_in = se, a_in = sa;
    if (clip_lo) {
        bool amb = false;
        auto entry_row = [&](double bt, int bv, bool bamb, int start_val, int& out) {
            const double m = wave_max(bt);
            if (m < 0.0) return;                    // no update before t_lo: the start's value
            const bool at = bt == m;
            // at t = 0 the group also holds the start entry (sorted last among equals only by
            // candidate index, so any other value there is an ambiguous tie)
            const int v0 = m == 0.0 ? start_val : __shfl(bv, __builtin_ctzll(__ballot(at)));
            amb |= __ballot(at && (bamb || bv != v0)) != 0;
            out = v0;
        };
        entry_row(pe_t, pe_v, pe_amb, se, e_in);
        entry_row(pa_t, pa_v, pa_amb, sa, a_in);
        if (amb) {
            if (lane == 0) {
                const unsigned long long q = atomicAdd(o.n_deferred, 1ull);
                o.deferred[q] = ray;
            }
            wave_sync();
            return;
        }
    }
    wave_sync();

    // ---- 2. sort by (distance, candidate) ------------------------------------------------
    int sflags = 2;          // bit 0: repair the order; bit 1: look for ambiguous ties
    const int n_other = F - s_near - nfar;   // entries outside the shells' sorted run
    if (pair_fmt) sort_lds(keys, pays, F, lane);
    else if (F <= 64) sflags = sort_regs<1>(keys, pays, F, nfar, cap, lane, cmask);
    else if (F <= 128) {
        sflags = n_other <= 64 ? merge_sort<2, 1>(keys, pays, F, s_near, nfar, cap, lane, cmask)
                                 : sort_regs<2>(keys, pays, F, nfar, cap, lane, cmask);
    } else if (F <= 256) {
        sflags = n_other <= 64 ? merge_sort<4, 1>(keys, pays, F, s_near, nfar, cap, lane, cmask)
                 : n_other <= 128 ? merge_sort<4, 2>(keys, pays, F, s_near, nfar, cap, lane, cmask)
                                  : sort_regs<4>(keys, pays, F, nfar, cap, lane, cmask);
    } else {                                                  // C3: 15 % of hit rays
        sflags = n_other <= 128 ? merge_sort<8, 2>(keys, pays, F, s_near, nfar, cap, lane, cmask)
                 : n_other <= 256 ? merge_sort<8, 4>(keys, pays, F, s_near, nfar, cap, lane, cmask)
                                  : sort_regs<8>(keys, pays, F, nfar, cap, lane, cmask);
    }
    if (sflags & 1) fix_near_ties(keys, pays, F, lane);

    const int r_lim = 2 * nbr, e_lim = 2 * nbr + 2 * nbe, start_c = G.K - 1;
    const int start_vals[3] = {sr, se, sa};
    if ((sflags & 2) && ambiguous_ties(keys, pays, F, lane, r_lim, e_lim, start_c, start_vals)) {
        if (lane == 0) {
            const unsigned long long q = atomicAdd(o.n_deferred, 1ull);
            o.deferred[q] = ray;
        }
        wave_sync();
        return;
    }

    // ---- 3. forward fill, lengths, compaction ----------------------------------------------
    // every distance behind the start is integrated in the start voxel (raytracer.py:126,140)
    const int head = (start_ok && tneg < 0.0) ? 1 : 0;
    double* seg_len = reinterpret_cast<double*>(keys);
    int32_t* seg_vox = reinterpret_cast<int32_t*>(pays);
    int cr = sr, cE = e_in, cA = a_in;  // state before the first sorted entry
    int nseg = 0;
    // FILL / EMIT: lists in registers store their segments straight into the CSR slot
    constexpr bool kDirect = MODE == MODE_FILL || MODE == MODE_EMIT;
    constexpr int kStore = MODE == MODE_COUNT ? kFillNone : kDirect ? kFillGlobal : kFillLds;
    const FillState fs{sr, se, sa, sr, e_in, a_in, r_lim, e_lim, start_c};
    if (!pair_fmt) {                    // F <= 512: the list in registers, lane-major
        double* sl = kDirect ? o.len : seg_len;
        int32_t* sv = kDirect ? o.vox : seg_vox;
        const int64_t gcap = MODE == MODE_EMIT ? slot1 - slot0 : (int64_t)INT_MAX;
        const int64_t gb = slot0 + head;
        // (the fill reads the sorted list lane-major at its own width: 3 and 6 entries per lane
        // for F <= 192 / 384 instead of 4 / 8 — count pass C3 2857 -> 2810 us, C5 556 -> 548 us,
        // C2 unchanged, profiles/r05_trace_fillm_ab.jsonl)
        nseg = F <= 64 ? fill_regs<1, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head)
             : F <= 128 ? fill_regs<2, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head)
             : F <= 192 ? fill_regs<3, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head)
             : F <= 256 ? fill_regs<4, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head)
             : F <= 384 ? fill_regs<6, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head)
                        : fill_regs<8, kStore>(G, keys, pays, F, lane, fs, sl, sv, gb, gcap, head);
    }
    for (int c0 = 0; pair_fmt && c0 < F; c0 += 64) {
        const int e = c0 + lane;
        const bool real = e < F;
        uint64_t k = 0;
        uint32_t p = 0;
        double tn = kInf;
        if (real) {
            k = keys[e];
            p = pays[e];
            if (e + 1 < F) tn = __longlong_as_double((long long)keys[e + 1]);
        }
        wave_sync();
        int ur = kNone, ue = kNone, ua = kNone;
        if (real) {
            const int cand = (int)(p >> 16);
            const int reg = (int)(p & 0xffffu) - 2;
            if (cand == start_c) {
                ur = sr; ue = se; ua = sa;
            } else if (cand < r_lim) {
                ur = reg;
            } else if (cand < e_lim) {
                if (reg != -2) ue = reg;
            } else {
                if (reg != -2) ua = reg;
            }
        }
        ur = scan_last(ur, lane);
        ue = scan_last(ue, lane);
        ua = scan_last(ua, lane);
        if (ur == kNone) ur = cr;
        if (ue == kNone) ue = cE;
        if (ua == kNone) ua = cA;
        cr = __builtin_amdgcn_readlane(ur, 63);
        cE = __builtin_amdgcn_readlane(ue, 63);
        cA = __builtin_amdgcn_readlane(ua, 63);
        const double t = __longlong_as_double((long long)k);
        const double len = tn - t;
        const bool ok = real && len > 0.0 && __builtin_isfinite(len) && ur >= 0 && ur < G.nr &&
                        ue >= 0 && ue < G.ne && ua >= 0 && ua < G.na;
        const uint64_t m = __ballot(ok);
        if (MODE != MODE_COUNT && ok) {
            const int pos = nseg + __popcll(m & lanemask_lt(lane));
            seg_len[pos] = len;
            seg_vox[pos] = (ur * G.ne + ue) * G.na + ua;
        }
        nseg += __popcll(m);
        wave_sync();
    }

    // ---- 4. emit ---------------------------------------------------------------------------
    if (MODE == MODE_COUNT) {
        if (lane == 0) o.counts[ray] = head + nseg;
    } else if (MODE == MODE_FILL || MODE == MODE_EMIT) {
        const int64_t r0 = MODE == MODE_FILL ? slot0
                                             : emit_slot(o, ray, head + nseg, lane == 0, slot0,
                                                         slot1);
        if (r0 < 0) {
            wave_sync();
            return;
        }
        if (head && lane == 0) {
            o.vox[r0] = (sr * G.ne + se) * G.na + sa;
            o.len[r0] = -tneg;
        }
        for (int q = lane; pair_fmt && q < nseg; q += 64) {    // (register lists stored already)
            o.vox[r0 + head + q] = seg_vox[q];
            o.len[r0 + head + q] = seg_len[q];
        }
    } else {
        const int svox = (sr * G.ne + se) * G.na + sa;
        int64_t c_lo = 0, c_hi = o.n_chan;
        if (o.ray_chan_div > 0) {
            c_lo = ray / o.ray_chan_div;
            c_hi = c_lo + 1;
        }
        for (int64_t c = c_lo; c < c_hi; ++c) {
            const T* rho = o.density + c * o.chan_stride;
            double acc = 0.0;
            if (head && lane == 0) acc = (double)rho[svox] * (-tneg);
            for (int q = lane; q < nseg; q += 64) acc += (double)rho[seg_vox[q]] * seg_len[q];
            acc = wave_sum(acc);
            const int64_t oc = (o.ray_chan_div > 0) ? 0 : c;
            if (lane == 0) o.out[oc * o.out_chan_stride + ray] = (T)acc;
        }
    }
    wave_sync();
}

// ---- segment-count bounds for the one-pass trace (MODE_BOUND) -------------------------------
// First index of the ascending b[0, n) whose entry is >= v (n when none).
__device__ __forceinline__ int first_ge(const double* b, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (b[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// Evenly spaced b (GridDev::uni): the index range from the spacing, widened by 1e-6 of a spacing
// (a superset of the binary search's: the counts are upper bounds) — no chain of dependent LDS
// loads.  C3 screen 126.5 -> 107.0 us, the same bound totals at C2 / C3 / C5
// (tools/bound_check.py); the bound itself costs ~25 us of it (ablated: 101 us).
__device__ __forceinline__ int first_ge_even(const double* b, int n, double v) {
    const double x = (v - b[0]) * ((n - 1) / (b[n - 1] - b[0])) - 1e-6;
    return x <= 0.0 ? 0 : x >= (double)n ? n : (int)__builtin_ceil(x);
}
// Entries of the ascending b[0, n) inside [lo, hi] (an upper bound when `even`).
__device__ __forceinline__ int count_in(const double* b, int n, double lo, double hi,
                                        bool even = false) {
    if (!(lo <= hi)) return 0;
    if (even) {
        const double ih = (n - 1) / (b[n - 1] - b[0]);
        const double xa = (lo - b[0]) * ih - 1e-6, xz = (hi - b[0]) * ih + 1e-6;
        const int a = xa <= 0.0 ? 0 : xa >= (double)n ? n : (int)__builtin_ceil(xa);
        const int z = xz < 0.0 ? -1 : xz >= (double)(n - 1) ? n - 1 : (int)__builtin_floor(xz);
        return z >= a ? z - a + 1 : 0;
    }
    const int a = first_ge(b, n, lo);
    int l = a, h = n;                                   // first entry > hi
    while (l < h) {
        const int mid = (l + h) >> 1;
        if (b[mid] <= hi) l = mid + 1;
        else h = mid;
    }
    return l - a;
}
__device__ __forceinline__ double polar(double px, double py, double pz) {
    return atan2(hypot(px, py), pz);
}

// Upper bound of the segments trace_one emits for a hit ray: the crossings it lists lie in the
// outer sphere's span [max(t_lo, 0), t_hi] (plus the start entry and the behind-start head), and
// along a line every family's crossings there are countable from the geometry alone:
//   spheres  2 per shell of radius >= the line's distance from the centre;
//   planes   one per half-plane whose azimuth the span's projection sweeps (the sweep is < pi;
//            a projection through the z axis sweeps them all);
//   cones    the elevation along a line has at most one extremum (its cosine's derivative has a
//            linear numerator), so one per cone angle on each monotone stretch.
// Angle margins (1e-6 rad planes, 1e-4 rad cones: the reference snaps |discriminant| < 1e-5 to a
// double root) and +2 / +4 absorb rounding.  A bound that fails anyway only costs time: the ray
// is counted in n_over and the caller falls back to the two-pass trace.  Starts inside a voxel
// get K: the exact (tie) path may split the behind-start stretch at every crossing behind it.
// rb / eb / ab: the grid's boundaries (LDS copies in the screen kernel: the binary searches are
// chains of dependent loads).
__device__ int segment_bound(const GridDev& G, const RayGeo& g, bool start_ok, const double* rb,
                             const double* eb, const double* ab) {
    if (start_ok) return G.K;
    const double R = G.r_outer;
    const double t1c = __builtin_sqrt(R * R - g.dd * g.dd);
    const double ta = fmax(g.tc - t1c, 0.0), tb = g.tc + t1c;
    if (!(tb >= ta)) return 2;                       // (NaN: a miss; behind the start: nothing)
    const double eps = 1e-9;
    const int n_s = G.nbr - ((G.uni & 1)
                                 ? first_ge_even(rb, G.nbr, g.dd * (1.0 - 1e-12))
                                 : first_ge(rb, G.nbr, g.dd * (1.0 - 1e-12)));
    const double ax = g.x0 + ta * g.w0, ay = g.x1 + ta * g.w1, az = g.x2 + ta * g.w2;
    const double bx = g.x0 + tb * g.w0, by = g.x1 + tb * g.w1, bz = g.x2 + tb * g.w2;
    int b_a = G.nba;
    {
        const double na = hypot(ax, ay), nb = hypot(bx, by);
        const double cr = ax * by - ay * bx, dt = ax * bx + ay * by;
        const bool through_axis = na <= eps * R || nb <= eps * R ||
                                  (__builtin_fabs(cr) <= eps * na * nb && dt < 0.0);
        if (G.a_asc && !through_axis) {
            const double pa = atan2(ay, ax), dp = atan2(cr, dt);
            const double lo = fmin(pa, pa + dp) - 1e-6, hi = fmax(pa, pa + dp) + 1e-6;
            const double two_pi = 6.283185307179586;
            // only the shifted windows that can overlap [a_b[0], a_b[nba - 1]] (the others
            // count nothing; one window of margin either side for rounding): three instead of
            // five for the usual [-pi, pi] grid
            const double a_lo = ab[0], a_hi = ab[G.nba - 1];
            const int k0 = max(-2, (int)__builtin_ceil((a_lo - hi) / two_pi) - 1);
            const int k1 = min(2, (int)__builtin_floor((a_hi - lo) / two_pi) + 1);
            int c = 0;
            for (int k = k0; k <= k1; ++k)
                c += count_in(ab, G.nba, lo + k * two_pi, hi + k * two_pi, G.uni & 4);
            if (__builtin_isfinite(lo) && __builtin_isfinite(hi)) b_a = min(c + 2, G.nba);
        }
    }
    int b_e = 2 * G.nbe;
    if (G.e_asc && g.dd > eps * R) {
        const double th_a = polar(ax, ay, az), th_b = polar(bx, by, bz);
        // extremum of cos(elevation) along x + t w: t* = (z0 (x.w) - wz |x|^2) / (wz (x.w) - z0)
        const double ts = (g.x2 * g.wx - g.w2 * g.nx2) / (g.w2 * g.wx - g.x2);
        const double m = 1e-4;
        int c;
        if (ts > ta && ts < tb) {
            const double th_s = polar(g.x0 + ts * g.w0, g.x1 + ts * g.w1, g.x2 + ts * g.w2);
            c = count_in(eb, G.nbe, fmin(th_a, th_s) - m, fmax(th_a, th_s) + m, G.uni & 2) +
                count_in(eb, G.nbe, fmin(th_s, th_b) - m, fmax(th_s, th_b) + m, G.uni & 2);
        } else {
            c = count_in(eb, G.nbe, fmin(th_a, th_b) - m, fmax(th_a, th_b) + m, G.uni & 2);
        }
        if (__builtin_isfinite(th_a) && __builtin_isfinite(th_b)) b_e = min(c + 4, 2 * G.nbe);
    }
    return min(2 * n_s + b_e + b_a + 4, G.K);
}

// Screen one ray per lane: a ray yields a segment only if it reaches the outer sphere or starts
// in a voxel — otherwise every r-row value stays the (invalid) start region (t1c is NaN for every
// shell when it is NaN for the outermost: monotone in R; tangents excluded).  Misses get their
// zero outputs here; hits are appended (wave-aggregated) to the hit list the trace kernel drains.
// The bound screen stages the grid's boundaries in LDS when they fit (screen_lds_bytes): the
// bound's binary searches then wait on LDS instead of global memory.
constexpr int kScreenLdsMax = 4096;   // boundaries (32 KB)
__host__ __device__ __forceinline__ bool screen_lds(const GridDev& G) {
    return G.nbr + G.nbe + G.nba <= kScreenLdsMax;
}
template <int MODE, typename T>
__global__ __launch_bounds__(256) void screen_kernel(GridDev G, RaysDev R, TraceOut<T> o) {
    extern __shared__ double bnd_lds[];
    const double *rb = G.r_b, *eb = G.e_b(), *ab = G.a_b();
    if (MODE == MODE_BOUND && screen_lds(G)) {
        for (int i = threadIdx.x; i < G.nbr; i += 256) bnd_lds[i] = rb[i];
        for (int i = threadIdx.x; i < G.nbe; i += 256) bnd_lds[G.nbr + i] = eb[i];
        for (int i = threadIdx.x; i < G.nba; i += 256) bnd_lds[G.nbr + G.nbe + i] = ab[i];
        __syncthreads();
        rb = bnd_lds;
        eb = bnd_lds + G.nbr;
        ab = bnd_lds + G.nbr + G.nbe;
    }
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool active = ray < R.n;
    double x[3] = {0, 0, 0}, d[3] = {0, 0, 1};
    int s[3] = {-1, -1, -1};
    if (active) load_ray(R, ray, x, d, s);
    const RayGeo g = make_ray(x[0], x[1], x[2], d[0], d[1], d[2]);
    const double t1c_outer = __builtin_sqrt(G.r_outer * G.r_outer - g.dd * g.dd);
    const bool start_r_ok = s[0] >= 0 && s[0] < G.nr;
    const bool hit = active && !(!start_r_ok && __builtin_isnan(t1c_outer));
    if (MODE == MODE_BOUND && active)
        o.counts[ray] = hit ? segment_bound(G, g, start_r_ok && s[1] >= 0 && s[1] < G.ne &&
                                                      s[2] >= 0 && s[2] < G.na, rb, eb, ab)
                            : 0;
    if (active && !hit) {
        if (MODE == MODE_COUNT) o.counts[ray] = 0;
        if (MODE == MODE_INTEGRATE) {
            const int64_t nc = o.ray_chan_div > 0 ? 1 : o.n_chan;
            for (int64_t c = 0; c < nc; ++c) o.out[c * o.out_chan_stride + ray] = (T)0;
        }
    }
    const bool listed = hit;
    const uint64_t m = __ballot(listed);
    unsigned base = 0;
    // one atomic per workgroup on the list's counter instead of one per wave: all waves with a
    // hit queue on that one address (C3 screen 200 -> 127 us, C5 55 -> 31 us)
    __shared__ unsigned wcnt[4], wbase;
    const int wid = threadIdx.x >> 6;
    if (lane == 0) wcnt[wid] = (unsigned)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        wbase = tot ? atomicAdd(o.n_hits, tot) : 0u;
    }
    __syncthreads();
    if (m == 0) return;
    base = wbase;
    for (int w = 0; w < wid; ++w) base += wcnt[w];
    if (listed) {
        HitRay h;
        h.g = g;
        h.t1c_o = t1c_outer;
        h.s[0] = s[0]; h.s[1] = s[1]; h.s[2] = s[2];
        h.ray = (int32_t)ray;
        o.hits[base + __popcll(m & lanemask_lt(lane))] = h;
    }
}

// Trace workgroups of kWavesPerBlock waves (scaled for fewer).  Each wave drains a fixed stride
// of the hit list, so more, shorter-lived workgroups let the dispatcher balance the rays' unequal
// costs: one-pass emit, µs, grid 2048 / 4096 / 8192 / 16384 (same box, rocprofv3): C3 3495 /
// 3317 / 3238 / 3200, C5 579 / 575 / 555 / 534, C4 380 / 358 / 352 / 351, C2 129 / 124 / 124 /
// 127 (profiles/r03_trace_grid_sweep.json).
constexpr int kTraceGrid = 16384;
// Trace the hit rays, one per wave at a time, strided over the list: balanced whatever the
// image looks like.  Every lane evaluates the (wave-uniform) ray set-up itself.
template <int MODE, typename T>
__global__ __launch_bounds__(256, 4) void trace_kernel(GridDev G, TraceOut<T> o,
                                                                            int cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;          // 4, or fewer when K needs the LDS (see launch)
    uint64_t* keys = reinterpret_cast<uint64_t*>(smem) + (size_t)wid * cap;
    uint32_t* pays =
        reinterpret_cast<uint32_t*>(reinterpret_cast<uint64_t*>(smem) + (size_t)waves * cap) +
        (size_t)wid * cap;
    const int64_t n_hits = (int64_t)*o.n_hits;
    for (int64_t h = (int64_t)blockIdx.x * waves + wid; h < n_hits;
         h += (int64_t)gridDim.x * waves) {
        const HitRay& hr = o.hits[__builtin_amdgcn_readfirstlane((int)h)];   // uniform record
        const RayGeo g = hr.g;
        trace_one<MODE, T>(G, g, hr.t1c_o, hr.s[0], hr.s[1], hr.s[2], hr.ray, keys, pays, cap,
                           lane, o);
    }
}

// ---- per-family solves for the r_torch / e_torch / a_torch API ------------------------------
// F: float64, or float32 for ftype=torch.float32 (inputs rounded to float as torch.asarray(...,
// dtype=float32) does, every operation in float).
template <typename F>
__global__ __launch_bounds__(256) void solve_kernel(GridDev G, RaysDev R, int family, F* t,
                                                    int32_t* region, int8_t* neg) {
    const int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ray >= R.n) return;
    double x[3], d[3];
    int s[3];
    load_ray(R, ray, x, d, s);
    const RayGeoT<F> g = make_ray_family<F>((F)x[0], (F)x[1], (F)x[2], (F)d[0], (F)d[1], (F)d[2],
                                            family);
    if (family == 0) {
        const int w = 2 * G.nbr;
        for (int j = 0; j < G.nbr; ++j) {
            F ti, to;
            int ri, ro, ni, no;
            sphere_solve(G, g, j, ti, ri, to, ro, ni, no);
            t[ray * w + j] = ti; region[ray * w + j] = ri; neg[ray * w + j] = (int8_t)ni;
            t[ray * w + G.nbr + j] = to; region[ray * w + G.nbr + j] = ro;
            neg[ray * w + G.nbr + j] = (int8_t)no;
        }
    } else if (family == 1) {
        const int w = 2 * G.nbe;
        for (int j = 0; j < G.nbe; ++j) {
            F ta, tb;
            int ra, rb, na_, nb_;
            cone_solve(G, g, j, ta, ra, tb, rb, na_, nb_);
            t[ray * w + j] = ta; region[ray * w + j] = ra; neg[ray * w + j] = (int8_t)na_;
            t[ray * w + G.nbe + j] = tb; region[ray * w + G.nbe + j] = rb;
            neg[ray * w + G.nbe + j] = (int8_t)nb_;
        }
    } else {
        const int w = G.nba;
        for (int j = 0; j < G.nba; ++j) {
            F tt;
            int r, ng;
            plane_solve(G, g, j, tt, r, ng);
            t[ray * w + j] = tt; region[ray * w + j] = r; neg[ray * w + j] = (int8_t)ng;
        }
    }
}

// ---- exact path for deferred rays: one wave per ray, the reference algorithm verbatim -----
// Candidates in the reference's concatenation order (raytracer.py:92, 117-122), solved by the
// lanes in parallel.  Returns through `put(c, t, region)`.
// F: the solves' precision (double; float for ftype=torch.float32 traces), the distances handed
// to `put` as doubles (exact for float).  gr / ge / ga: the ray as r_torch / e_torch / a_torch see
// it (the same RayGeo unless the rays are fresh copies per solver, exact_list).
template <typename F, class Put>
__device__ __forceinline__ void exact_candidates(const GridDev& G, const RayGeoT<F>& gr,
                                                 const RayGeoT<F>& ge, const RayGeoT<F>& ga,
                                                 int lane, int step, Put put) {
    const int nbr = G.nbr, nbe = G.nbe, nba = G.nba;
    const int r_lim = 2 * nbr, e_lim = 2 * nbr + 2 * nbe;
    for (int j = lane; j < nbr; j += step) {
        F ti, to;
        int ri, ro, ni, no;
        sphere_solve(G, gr, j, ti, ri, to, ro, ni, no);
        put(j, (double)ti, ri);
        put(nbr + j, (double)to, ro);
    }
    for (int j = lane; j < nbe; j += step) {
        F ta, tb;
        int ra, rb, na_, nb_;
        cone_solve(G, ge, j, ta, ra, tb, rb, na_, nb_);
        put(r_lim + j, (double)ta, ra);
        put(r_lim + nbe + j, (double)tb, rb);
    }
    for (int j = lane; j < nba; j += step) {
        F t;
        int r, ng;
        plane_solve(G, ga, j, t, r, ng);
        put(e_lim + j, (double)t, r);
    }
    if (lane == 0) put(G.K - 1, 0.0, 0);
}
// The candidate list of one ray.  trace_indices hands the same `rays` tensor to the three solvers
// and each converts it with tr.asarray(rays, ftype) (raytracer.py:276,360,500): when that is the
// caller's tensor (its dtype is ftype) r_torch and e_torch normalise it in place in turn
// (raytracer.py:281,365) and a_torch sees it normalised twice (make_ray); when the dtype differs
// (R.fresh: sphrt_trace_reference's SPHRT_TRACE_FRESH_RAYS, e.g. float64 rays in a float32 trace)
// every solver gets a fresh copy: r_torch and e_torch normalise theirs once, a_torch not at all.
template <bool ALL, typename F, class Put>
__device__ __forceinline__ void exact_list(const GridDev& G, const RaysDev& R,
                                           const RayGeoT<F>& g, const double* x, const double* d,
                                           int lane, int step, Put put) {
    if (ALL && R.fresh) {
        const RayGeoT<F> ge = make_ray_family<F>((F)x[0], (F)x[1], (F)x[2], (F)d[0], (F)d[1],
                                                 (F)d[2], 1);
        const RayGeoT<F> ga = make_ray_family<F>((F)x[0], (F)x[1], (F)x[2], (F)d[0], (F)d[1],
                                                 (F)d[2], 2);
        exact_candidates(G, g, ge, ga, lane, step, put);
    } else {
        exact_candidates(G, g, g, g, lane, step, put);
    }
}

// A sorted entry's segment under the trace's options: its length (tn - t in F: float32 traces
// difference their float32 distances, raytracer.py:150-151 in the trace's dtype) and whether it
// is kept; its voxel index.  Default (raytracer.py:155-173): kept when positive, finite and inside
// the grid.  INV (Operator(..., invalid=True)): nothing is masked — every non-zero length is kept,
// inf and NaN included, with its regions wrapped as the reference's forward reads them
// (density[r, e, a] with r = -1 is the last shell: Python's negative indexing).
template <typename F>
__device__ __forceinline__ double seg_length(double tn, double t) {
    return (double)((F)tn - (F)t);
}
template <bool INV>
__device__ __forceinline__ bool seg_keep(const GridDev& G, double len, int r, int e, int a) {
    if (INV) return len != 0.0;                // (NaN != 0: kept)
    return len > 0.0 && __builtin_isfinite(len) && r >= 0 && r < G.nr && e >= 0 && e < G.ne &&
           a >= 0 && a < G.na;
}
template <bool INV>
__device__ __forceinline__ int seg_voxel(const GridDev& G, int r, int e, int a) {
    if (INV) {
        r = r < 0 ? r + G.nr : r;
        e = e < 0 ? e + G.ne : e;
        a = a < 0 ? a + G.na : a;
    }
    return (r * G.ne + e) * G.na + a;
}

// Forward fill + diff + masking over the sorted list (raytracer.py:126, 140-173), one lane.
template <int MODE, typename T, typename F, bool INV, class V>
__device__ void exact_walk(const GridDev& G, const TraceOut<T>& o, int64_t ray, const int* s,
                           const V& v) {
    const int K = G.K, r_lim = 2 * G.nbr, e_lim = 2 * G.nbr + 2 * G.nbe;
    int64_t c_lo = 0, c_hi = o.n_chan;
    if (MODE == MODE_INTEGRATE && o.ray_chan_div > 0) {
        c_lo = ray / o.ray_chan_div;
        c_hi = c_lo + 1;
    }
    if (MODE != MODE_INTEGRATE) c_hi = c_lo + 1;
    for (int64_t c = c_lo; c < c_hi; ++c) {
        int cr = s[0], ce = s[1], ca = s[2];
        int64_t nseg = 0;
        double acc = 0.0;
        const int64_t base = MODE == MODE_FILL || MODE == MODE_EMIT ? o.row_ptr[ray] : 0;
        const int64_t cap = MODE == MODE_EMIT ? o.row_ptr[ray + 1] - base : INT64_MAX;
        auto cur = v.get(0);
        for (int k = 0; k < K; ++k) {
            const double t = cur.t;
            const uint32_t p = cur.pay;
            if (!(t < 0.0)) {
                const int cand = (int)(p >> 16);
                const int reg = (int)(p & 0xffffu) - 2;
                if (cand == K - 1) { cr = s[0]; ce = s[1]; ca = s[2]; }
                else if (cand < r_lim) cr = reg;
                else if (cand < e_lim) { if (reg != -2) ce = reg; }
                else if (reg != -2) ca = reg;
            }
            if (k + 1 < K) cur = v.get(k + 1);
            const double tn = k + 1 < K ? cur.t : kInf;
            const double len = seg_length<F>(tn, t);
            if (!seg_keep<INV>(G, len, cr, ce, ca)) continue;
            const int vx = seg_voxel<INV>(G, cr, ce, ca);
            if (MODE == MODE_FILL || (MODE == MODE_EMIT && nseg < cap)) {
                o.vox[base + nseg] = vx;
                o.len[base + nseg] = len;
            } else if (MODE == MODE_INTEGRATE) {
                acc += (double)o.density[c * o.chan_stride + vx] * len;
            }
            ++nseg;
        }
        if (MODE == MODE_COUNT) o.counts[ray] = (int32_t)nseg;
        if (MODE == MODE_EMIT) (void)emit_slot(o, ray, nseg, true);
        if (MODE == MODE_INTEGRATE) {
            const int64_t oc = o.ray_chan_div > 0 ? 0 : c;
            o.out[oc * o.out_chan_stride + ray] = (T)acc;
        }
    }
}

// The same walk, wave-parallel over 64-entry chunks of the sorted list (ts, ps): "last update
// wins" scans for the three region rows, differences, and in-order compaction of the non-zero
// in-grid segments into (seg_vox, seg_len) (LDS, K entries), then count / copy / integrate.
template <int MODE, typename T, typename F, bool INV>
__device__ void exact_walk_wave(const GridDev& G, const TraceOut<T>& o, int64_t ray, const int* s,
                                const double* ts, const uint32_t* ps, int32_t* seg_vox,
                                double* seg_len, int lane) {
    const int K = G.K, r_lim = 2 * G.nbr, e_lim = 2 * G.nbr + 2 * G.nbe;
    int cr = s[0], ce = s[1], ca = s[2];
    int nseg = 0;
    for (int c0 = 0; c0 < K; c0 += 64) {
        const int k = c0 + lane;
        const bool real = k < K;
        const double t = real ? ts[k] : kInf;
        const double tn = k + 1 < K ? ts[k + 1] : kInf;
        const uint32_t p = real ? ps[k] : 0u;
        int ur = kNone, ue = kNone, ua = kNone;
        if (real && !(t < 0.0)) {
            const int cand = (int)(p >> 16);
            const int reg = (int)(p & 0xffffu) - 2;
            if (cand == K - 1) {
                ur = s[0]; ue = s[1]; ua = s[2];
            } else if (cand < r_lim) {
                ur = reg;
            } else if (cand < e_lim) {
                if (reg != -2) ue = reg;
            } else if (reg != -2) {
                ua = reg;
            }
        }
        ur = scan_last(ur, lane);
        ue = scan_last(ue, lane);
        ua = scan_last(ua, lane);
        if (ur == kNone) ur = cr;
        if (ue == kNone) ue = ce;
        if (ua == kNone) ua = ca;
        cr = __builtin_amdgcn_readlane(ur, 63);
        ce = __builtin_amdgcn_readlane(ue, 63);
        ca = __builtin_amdgcn_readlane(ua, 63);
        const double len = seg_length<F>(tn, t);
        const bool ok = real && seg_keep<INV>(G, len, ur, ue, ua);
        const uint64_t m = __ballot(ok);
        if (MODE != MODE_COUNT && ok) {
            const int pos = nseg + __popcll(m & lanemask_lt(lane));
            seg_len[pos] = len;
            seg_vox[pos] = seg_voxel<INV>(G, ur, ue, ua);
        }
        nseg += __popcll(m);
    }
    wave_sync();
    if (MODE == MODE_COUNT) {
        if (lane == 0) o.counts[ray] = nseg;
    } else if (MODE == MODE_FILL || MODE == MODE_EMIT) {
        const int64_t r0 = MODE == MODE_FILL ? o.row_ptr[ray] : emit_slot(o, ray, nseg, lane == 0);
        for (int q = lane; r0 >= 0 && q < nseg; q += 64) {
            o.vox[r0 + q] = seg_vox[q];
            o.len[r0 + q] = seg_len[q];
        }
    } else {
        int64_t c_lo = 0, c_hi = o.n_chan;
        if (o.ray_chan_div > 0) {
            c_lo = ray / o.ray_chan_div;
            c_hi = c_lo + 1;
        }
        for (int64_t c = c_lo; c < c_hi; ++c) {
            const T* rho = o.density + c * o.chan_stride;
            double acc = 0.0;
            for (int q = lane; q < nseg; q += 64) acc += (double)rho[seg_vox[q]] * seg_len[q];
            acc = wave_sum(acc);
            const int64_t oc = (o.ray_chan_div > 0) ? 0 : c;
            if (lane == 0) o.out[oc * o.out_chan_stride + ray] = (T)acc;
        }
    }
}

// Large K (the wave list does not fit kExactLdsMax): lane 0 sorts the ray's list serially in the
// wave's slice of workspace.
// ALL: the reference-mode trace (sphrt_trace_reference): every ray of R, or with a ray list
// (o.deferred set: the rays ref_screen_kernel kept) those; else the fast path's deferred list.
template <bool ALL, typename T>
__device__ __forceinline__ int64_t exact_count(const RaysDev& R, const TraceOut<T>& o) {
    return ALL && !o.deferred ? R.n : (int64_t)*o.n_deferred;
}
template <bool ALL, typename T>
__device__ __forceinline__ int64_t exact_ray(const TraceOut<T>& o, int64_t q) {
    return ALL && !o.deferred ? q : o.deferred[q];
}
template <typename F>
__device__ __forceinline__ RayGeoT<F> exact_geo(const double* x, const double* d) {
    return make_ray<F>((F)x[0], (F)x[1], (F)x[2], (F)d[0], (F)d[1], (F)d[2]);
}

template <int MODE, typename T, typename F = double, bool INV = false, bool ALL = false>
__global__ __launch_bounds__(64) void exact_kernel(GridDev G, RaysDev R, TraceOut<T> o,
                                                   Cand* scratch) {
    const int lane = threadIdx.x;
    const CandList v{scratch + (int64_t)blockIdx.x * G.K};
    const int64_t count = exact_count<ALL>(R, o);
    for (int64_t q = blockIdx.x; q < count; q += gridDim.x) {
        const int64_t ray = exact_ray<ALL>(o, q);
        double x[3], d[3];
        int s[3];
        load_ray(R, ray, x, d, s);
        const RayGeoT<F> g = exact_geo<F>(x, d);
        exact_list<ALL>(G, R, g, x, d, lane, 64, [&](int c, double t, int reg) {
            v.set(c, Cand{t, ((uint32_t)c << 16) | (uint32_t)(reg + 2), 0u});
        });
        __syncthreads();
        if (lane == 0) {
            introsort(v, G.K);
            exact_walk<MODE, T, F, INV>(G, o, ray, s, v);
        }
        __syncthreads();
    }
}

// The emulated introsort, wave-parallel (the list in LDS).  Same result as introsort():
//  * partition: with piv = v[first] after the median-of-three, the left scan's stops are the
//    positions i in (first, last) with !(v[i] < piv), ascending (L[0], L[1], ...), the right
//    scan's the positions j in [first, last) with !(piv < v[j]), descending (R[0], ...).  Swap k
//    exchanges L[k] and R[k] as long as L[k] < R[k]; with k* the first k where that fails
//    (k* = #{left stops i of rank a : #right stops after i > a}), the cut is min(L[k*], R[k*-1])
//    (L[k*] = +inf when there is none; L[0] when k* = 0).  Positions between the pointers are
//    untouched until they cross, so the stop lists of the unswapped array decide everything.
//  * the final insertion sort never moves an element past an equal one, and after the partition
//    phase no element is smaller than one in an earlier leaf: it is a stable sort of each leaf
//    (range of <= 16 left by the loop; heap-sorted ranges are already sorted), computed as ranks.
//  Rays with a NaN distance (none expected: the solvers map NaN to +inf) take the serial sort.
constexpr size_t kExactWaveEntryBytes = 2 * 8 + 5 * 4;   // per candidate, see the layout below
constexpr int kExactStack = 64;                         // partition stack (depth <= 2 log2 K)
constexpr size_t kExactWaveLdsMax = 64 * 1024;
__host__ __device__ constexpr size_t exact_wave_lds(int K, int W) {
    return (size_t)K * kExactWaveEntryBytes + (size_t)W * (3 * kExactStack + 3) * sizeof(int);
}

// One partition of [first, last) by one wave (lane 0 runs the median-of-three), the reference's
// __unguarded_partition_pivot; returns the cut.  lpos / rpos are indexed from `first` (ranks are
// < last - first), so waves partitioning disjoint ranges share them.  Leaves the swaps unsynced.
__device__ __forceinline__ int exact_partition(const SoaList& v, double* tk, uint32_t* pk,
                                               int32_t* lpos, int32_t* rpos, int first, int last,
                                               int lane, uint64_t below) {
    const int mid = first + (last - first) / 2;
    if (lane == 0) move_median_to_first(v, first, first + 1, mid, last - 1);
    wave_sync();
    const double piv = tk[first];
    // stop counts
    int n_l = 0, n_r = 0;
    for (int c0 = first; c0 < last; c0 += 64) {
        const int p = c0 + lane;
        const bool in = p < last;
        const double t = in ? tk[p] : 0.0;
        n_l += __builtin_popcountll(__ballot(in && p > first && !(t < piv)));
        n_r += __builtin_popcountll(__ballot(in && !(piv < t)));
    }
    // ranks, stop lists and k*
    int a0 = 0, r0 = 0, ks = 0;
    for (int c0 = first; c0 < last; c0 += 64) {
        const int p = c0 + lane;
        const bool in = p < last;
        const double t = in ? tk[p] : 0.0;
        const bool is_l = in && p > first && !(t < piv);
        const bool is_r = in && !(piv < t);
        const uint64_t bl = __ballot(is_l), br = __ballot(is_r);
        const int a = a0 + __builtin_popcountll(bl & below);   // left rank
        const int rb = r0 + __builtin_popcountll(br & below);  // right stops before p
        if (is_l) lpos[first + a] = p;
        if (is_r) rpos[first + n_r - 1 - rb] = p;
        const int after = n_r - rb - (is_r ? 1 : 0);          // right stops after p
        ks += __builtin_popcountll(__ballot(is_l && after > a));
        a0 += __builtin_popcountll(bl);
        r0 += __builtin_popcountll(br);
    }
    wave_sync();
    int cut;
    if (ks < n_l) cut = ks > 0 ? min(lpos[first + ks], rpos[first + ks - 1]) : lpos[first];
    else cut = rpos[first + ks - 1];
    for (int k = lane; k < ks; k += 64) {
        const int i = lpos[first + k], j = rpos[first + k];
        const double ti = tk[i], tj = tk[j];
        const uint32_t pi = pk[i], pj = pk[j];
        tk[i] = tj; pk[i] = pj;
        tk[j] = ti; pk[j] = pi;
    }
    return cut;
}

// Whether two list entries with the same distance leave a different state in either order: both
// set one region row (the walk's r / e / a updates; the start entry K - 1 sets all three to the
// start voxel) to different values.
__device__ __forceinline__ int entry_rows(uint32_t p, int K, int r_lim, int e_lim, const int* s,
                                          int* v) {
    const int cand = (int)(p >> 16), reg = (int)(p & 0xffffu) - 2;
    if (cand == K - 1) {
        v[0] = s[0]; v[1] = s[1]; v[2] = s[2];
        return 7;
    }
    v[0] = v[1] = v[2] = reg;
    if (cand < r_lim) return 1;
    if (cand < e_lim) return reg != -2 ? 2 : 0;
    return reg != -2 ? 4 : 0;
}
__device__ __forceinline__ bool entries_conflict(uint32_t pa, uint32_t pb, int K, int r_lim,
                                                 int e_lim, const int* s) {
    int va[3], vb[3];
    const int m = entry_rows(pa, K, r_lim, e_lim, s, va) & entry_rows(pb, K, r_lim, e_lim, s, vb);
    return ((m & 1) && va[0] != vb[0]) || ((m & 2) && va[1] != vb[1]) ||
           ((m & 4) && va[2] != vb[2]);
}

// The depth limit ran out on [first, last): the reference heap-sorts it (std::__partial_sort).
// Heapsort's order among equal distances is its own, but only the walk reads the order, and there
// equal neighbours differ only when both set one region row to different values (the segment
// between them is empty; for INV an infinite one is kept, NaN long).  With no such pair in the
// range a rank sort (ascending, ties by position) gives the same segments — one wave, in
// parallel; otherwise lane 0 runs the heapsort.  ts / ps (free until the leaf ranks) take the
// sorted range; lpos its ranks.
template <bool INV>
__device__ __forceinline__ void exact_heap_range(const SoaList& v, double* tk, uint32_t* pk,
                                                 double* ts, uint32_t* ps, int32_t* lpos,
                                                 int first, int last, int K, int r_lim, int e_lim,
                                                 const int* s, int lane,
                                                 unsigned long long* n_heap) {
    bool amb = false;
    for (int p = first + lane; p < last; p += 64) {
        const double t = tk[p];
        const uint32_t pp = pk[p];
        // ties that can matter: updates (t >= 0) with an empty segment between (finite t;
        // INV keeps the NaN segment between two infinite ones)
        const bool live = t >= 0.0 && (INV || t < kInf);
        int r = first;
        for (int j = first; j < last; ++j) {
            const double u = tk[j];
            r += (u < t || (u == t && j < p)) ? 1 : 0;
            if (u == t && j != p && live) {
                if (INV && t == kInf) amb = true;
                else amb |= entries_conflict(pp, pk[j], K, r_lim, e_lim, s);
            }
        }
        lpos[p] = r;
    }
    if (lane == 0 && n_heap) atomicAdd(n_heap + (__ballot(amb) != 0 ? 1 : 0), 1ull);
    if (__ballot(amb) != 0) {
        wave_sync();
        if (lane == 0) heap_sort(v, first, last);
        wave_sync();
        return;
    }
    for (int p = first + lane; p < last; p += 64) {
        const int r = lpos[p];
        ts[r] = tk[p];
        ps[r] = pk[p];
    }
    wave_sync();
    for (int p = first + lane; p < last; p += 64) {
        tk[p] = ts[p];
        pk[p] = ps[p];
    }
    wave_sync();
}

// Reference mode without invalid=True, lists of <= 64 M candidates: the whole list in
// concatenation order (tk / pk) sorted by (distance, candidate) in registers — composite keys as in
// the fast path, with the distance's bits mapped to an order-preserving unsigned (negative and
// infinite distances included) — into ts / ps.  That is the emulated introsort's order up to the
// order inside groups of equal distances, which the walk reads only where two entries of a group
// set one region row to different values (the segments inside a group are empty, the group's
// state after it is the same in any order) or, from the first infinite distance on, not at all
// (infinite and NaN segments are masked).  False: a NaN distance, two distances the composite
// keys do not separate, or a group that matters — the caller runs the emulated introsort.  (C2
// ftype=float32: ~45 k rays reach the exact path after the miss screen; each sorts 256
// candidates.)  float32 distances never collide in the keys (their low 29 bits are zero).
__device__ __forceinline__ uint64_t order_bits(double t) {
    const uint64_t b = (uint64_t)__double_as_longlong(t + 0.0);      // -0 -> +0
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
template <int M>
__device__ bool network_sort(const GridDev& G, const double* tk, const uint32_t* pk, double* ts,
                             uint32_t* ps, int K, int lane, const int* s) {
    const int cbits = 32 - __builtin_clz((unsigned)(K - 1));
    const uint64_t cmask = (1ull << cbits) - 1ull;
    uint64_t k[M];
    bool nan = false;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        k[i] = ~0ull;
        if (e < K) {
            const double t = tk[e];
            nan |= __builtin_isnan(t);
            k[i] = (order_bits(t) & ~cmask) | (uint64_t)e;
        }
    }
    if (__ballot(nan) != 0) return false;
    sort_stages<M, 2>(k, lane);
    double t[M];
    uint32_t p[M];
    uint64_t kb[M];
    int cand[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
        cand[i] = (int)(k[i] & cmask);
        const bool in = lane * M + i < K;
        t[i] = in ? tk[cand[i]] : kInf;
        p[i] = in ? pk[cand[i]] : 0u;
        kb[i] = order_bits(t[i]);
    }
    // (distance, candidate) strictly ascending, across the lanes too
    bool bad = false;
#pragma unroll
    for (int i = 1; i < M; ++i)
        bad |= lane * M + i < K &&
               (kb[i] < kb[i - 1] || (kb[i] == kb[i - 1] && cand[i] < cand[i - 1]));
    const uint64_t pk_prev = (uint64_t)__shfl_up((long long)kb[M - 1], 1);
    const int pc_prev = __shfl_up(cand[M - 1], 1);
    bad |= lane > 0 && lane * M < K &&
           (kb[0] < pk_prev || (kb[0] == pk_prev && cand[0] < pc_prev));
    if (__ballot(bad) != 0) return false;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const int e = lane * M + i;
        if (e < K) {
            ts[e] = t[i];
            ps[e] = p[i];
        }
    }
    wave_sync();
    const int r_lim = 2 * G.nbr, e_lim = 2 * G.nbr + 2 * G.nbe;
    bool amb = false;
    for (int e = lane; e + 1 < K; e += 64) {
        const double te = ts[e];
        if (!(te >= 0.0 && te < kInf) || ts[e + 1] != te) continue;
        for (int j = e + 1; j < K && ts[j] == te; ++j)
            amb |= entries_conflict(ps[e], ps[j], K, r_lim, e_lim, s);
    }
    return __ballot(amb) == 0;
}
template <bool INV>
__device__ __forceinline__ bool reference_network(const GridDev& G, const double* tk,
                                                  const uint32_t* pk, double* ts, uint32_t* ps,
                                                  int lane, const int* s) {
    if constexpr (INV) {
        return false;       // (every list with two infinite distances is a group that matters)
    } else {
        const int K = G.K;
        if (K <= 64) return network_sort<1>(G, tk, pk, ts, ps, K, lane, s);
        if (K <= 128) return network_sort<2>(G, tk, pk, ts, ps, K, lane, s);
        if (K <= 256) return network_sort<4>(G, tk, pk, ts, ps, K, lane, s);
        if (K <= 512) return network_sort<8>(G, tk, pk, ts, ps, K, lane, s);
        return false;
    }
}

// W waves per ray.  The candidates and the leaf ranks are spread over all 64 W lanes; the
// partitions run breadth-first for log2(W) levels (wave w partitions range w of the level, so
// the two halves of a partition proceed in parallel), then each wave finishes one of the W
// ranges with its own stack: a deferred ray's latency is the partition phase's chain of ~K / 8
// dependent partitions, which W = 4 cuts to about a quarter.  Disjoint ranges give the same
// result in any order.  The walk runs on wave 0.
template <int MODE, typename T, typename F = double, bool INV = false, bool ALL = false, int W = 1>
__global__ __launch_bounds__(64 * W) void exact_wave_kernel(GridDev G, RaysDev R, TraceOut<T> o) {
    extern __shared__ __attribute__((aligned(16))) unsigned char xw_lds[];
    const int K = G.K;
    double* tk = reinterpret_cast<double*>(xw_lds);   // list (distance), current order
    double* ts = tk + K;                              // sorted list
    uint32_t* pk = reinterpret_cast<uint32_t*>(ts + K);
    uint32_t* ps = pk + K;
    int32_t* lpos = reinterpret_cast<int32_t*>(ps + K);   // left stops by rank
    int32_t* rpos = lpos + K;                              // right stops by rank
    uint32_t* leaf = reinterpret_cast<uint32_t*>(rpos + K);   // leaf range lo | hi << 16
    // per wave: the partition stack in LDS (uniform; a private array would live in scratch
    // memory, one global round trip per push or pop); then the W top-level ranges
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int* st_first = reinterpret_cast<int*>(leaf + K) + wid * 3 * kExactStack;
    int* st_last = st_first + kExactStack;
    int* st_depth = st_last + kExactStack;
    int* top = reinterpret_cast<int*>(leaf + K) + W * 3 * kExactStack;   // (first, last, depth)
    const SoaList v{tk, pk};
    const uint64_t below = lanemask_lt(lane);
    const int r_lim = 2 * G.nbr, e_lim = 2 * G.nbr + 2 * G.nbe;
    const int64_t count = exact_count<ALL>(R, o);
    // one ray: its candidate list, the emulated introsort, the walk (uniform over the workgroup)
    auto trace_ray = [&](const int64_t ray) {
        double x[3], d[3];
        int s[3];
        load_ray(R, ray, x, d, s);
        const RayGeoT<F> g = exact_geo<F>(x, d);
        exact_list<ALL>(G, R, g, x, d, tid, 64 * W, [&](int c, double t, int reg) {
            tk[c] = t;
            pk[c] = ((uint32_t)c << 16) | (uint32_t)(reg + 2);
        });
        int nan = 0;
        for (int p = tid; p < K; p += 64 * W) leaf[p] = (uint32_t)p | ((uint32_t)(p + 1) << 16);
        if (tid == 0) {
            top[0] = 0;
            top[1] = K;
            top[2] = 2 * (31 - __builtin_clz((unsigned)max(K, 1)));
        }
        __syncthreads();
        if constexpr (ALL && W == 1 && !INV) {      // reference mode: the register sort first
            if (reference_network<INV>(G, tk, pk, ts, ps, lane, s)) {
                exact_walk_wave<MODE, T, F, INV>(G, o, ray, s, ts, ps, lpos, tk, lane);
                __syncthreads();
                return;
            }
            __syncthreads();
        }
        for (int p = tid; p < K; p += 64 * W) nan |= __builtin_isnan(tk[p]) ? 1 : 0;
        if (__syncthreads_or(nan)) {
            if (tid == 0) {
                introsort(v, K);
                exact_walk<MODE, T, F, INV>(G, o, ray, s, v);
            }
            __syncthreads();
            return;
        }
        // ---- partition phase (uniform control flow per wave) ----
        // the top levels, breadth-first: range w of level l splits into ranges w and w + 2^l
#pragma unroll
        for (int n = 1; n < W; n *= 2) {
            if (wid < n) {
                const int f = top[3 * wid], l = top[3 * wid + 1], dep = top[3 * wid + 2];
                int cut = l, nd = dep;
                if (l - f > kIntroThreshold && dep > 0) {
                    cut = exact_partition(v, tk, pk, lpos, rpos, f, l, lane, below);
                    nd = dep - 1;
                }
                if (lane == 0) {
                    top[3 * wid + 1] = cut;
                    top[3 * wid + 2] = nd;
                    top[3 * (wid + n)] = cut;
                    top[3 * (wid + n) + 1] = l;
                    top[3 * (wid + n) + 2] = nd;
                }
            }
            __syncthreads();
        }
        // then each wave its range, depth first
        int sp = 0;
        int first = top[3 * wid], last = top[3 * wid + 1], depth = top[3 * wid + 2];
        bool have = last - first > 1;
        while (have) {
            while (last - first > kIntroThreshold) {
                if (depth == 0) {                      // the reference's heapsort
                    exact_heap_range<INV>(v, tk, pk, ts, ps, lpos, first, last, K, r_lim, e_lim,
                                          s, lane, o.n_heap);
                    first = last;                      // sorted: no leaf
                    break;
                }
                --depth;
                const int cut = exact_partition(v, tk, pk, lpos, rpos, first, last, lane, below);
                if (lane == 0) {
                    st_first[sp] = cut;
                    st_last[sp] = last;
                    st_depth[sp] = depth;
                }
                ++sp;
                last = cut;
                wave_sync();
            }
            if (last - first > 1) {                    // a leaf: its range, for the final ranks
                const uint32_t code = (uint32_t)first | ((uint32_t)last << 16);
                for (int p = first + lane; p < last; p += 64) leaf[p] = code;
            }
            have = sp > 0;
            if (have) {
                --sp;
                first = st_first[sp];
                last = st_last[sp];
                depth = st_depth[sp];
            }
        }
        __syncthreads();
        // ---- final insertion sort = stable sort inside each leaf, as ranks ----
        for (int p = tid; p < K; p += 64 * W) {
            const uint32_t code = leaf[p];
            const int lo = (int)(code & 0xffffu), hi = (int)(code >> 16);
            const double t = tk[p];
            int r = lo;
            for (int j = lo; j < hi; ++j) {
                const double u = tk[j];
                r += (u < t || (u == t && j < p)) ? 1 : 0;
            }
            ts[r] = t;
            ps[r] = pk[p];
        }
        __syncthreads();
        // (the pre-sort list and the left-stop list are free now: compacted segments go there)
        if (wid == 0) exact_walk_wave<MODE, T, F, INV>(G, o, ray, s, ts, ps, lpos, tk, lane);
        __syncthreads();
    };
    for (int64_t q = blockIdx.x; q < count; q += gridDim.x) trace_ray(exact_ray<ALL>(o, q));
}

// ---- one-pass trace: staging slots -> tight CSR ---------------------------------------------
// Every wave moves the rows of 64 consecutive rays, whose destination is one contiguous range
// [row_ptr[r0], row_ptr[r0 + 64]): lane i holds ray r0 + i's row pointer and slot, and every lane
// copies segments lane, lane + 64, ... of the range, finding its ray by a 6-step binary search
// over the lanes' row pointers — independent loads and stores, no per-row serial loop.
// Workgroups of the compaction (waves stride over the rays past it).  Uncapped by default: one
// step of 64 rays per wave, C3 compact_kernel 774 -> 707 us against a cap of 8192 workgroups on
// one box.  8 chunks of 64 segments per step (loads before stores) instead of 4: C3 699 -> 669,
// 700 -> 660 and 694 -> 688 us on three boxes.
constexpr int kCompactU = 8;   // 64-segment chunks per step, loads before stores
__global__ __launch_bounds__(256) void compact_kernel(int64_t n, const int64_t* __restrict__ slot,
                                                      const int64_t* __restrict__ row_ptr,
                                                      const int32_t* __restrict__ svox,
                                                      const double* __restrict__ slen,
                                                      int32_t* __restrict__ vox,
                                                      double* __restrict__ len) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t r0 = wave * 64; r0 < n; r0 += nw * 64) {
        const int64_t r = r0 + lane;
        const int64_t a = row_ptr[r < n ? r : n];             // rays past n: empty, at the end
        const int64_t b = r < n ? slot[r] : 0;
        const int64_t a0 = __shfl(a, 0);
        const int64_t end = row_ptr[r0 + 64 < n ? r0 + 64 : n];
        const int32_t rel = (int32_t)(a - a0);                // < 2^31: 64 rows of <= K segments
        // uniform trip count: every lane takes part in every shuffle (a shuffle from a lane that
        // left a divergent loop would read nothing); kCompactU chunks of 64 per step, their loads issued
        // before any store (one memory round trip per 64 * kCompactU segments, not per 64)
        const int32_t total = (int32_t)(end - a0);
        const int64_t dl = b - a;                             // slot - row start of lane's ray
        for (int32_t q0 = 0; q0 < total; q0 += 64 * kCompactU) {
            int64_t src[kCompactU];
            int32_t vv[kCompactU];
            double ll[kCompactU];
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const int32_t pos = q0 + 64 * u + lane;
                int lo = 0;
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
                    const int32_t x = __shfl(rel, lo + step);
                    if (x <= pos) lo += step;                 // last lane with rel <= pos
                }
                src[u] = a0 + pos + __shfl(dl, lo);
            }
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const bool in = q0 + 64 * u + lane < total;
                if (vox && in) vv[u] = svox[src[u]];
                if (len && in) ll[u] = slen[src[u]];
            }
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const int32_t pos = q0 + 64 * u + lane;
                if (pos < total) {
                    if (vox) vox[a0 + pos] = vv[u];
                    if (len) len[a0 + pos] = ll[u];
                }
            }
        }
    }
}

// Grids whose K-entry list does not fit a wave's LDS: every screened hit ray goes to the exact
// path (the deferred list; its serial kernel keeps each list in the workspace).
template <typename T>
__global__ __launch_bounds__(256) void defer_hits_kernel(TraceOut<T> o) {
    const int64_t n = (int64_t)*o.n_hits;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        o.deferred[i] = o.hits[i].ray;
    if (blockIdx.x == 0 && threadIdx.x == 0) *o.n_deferred = (unsigned long long)n;
}

// ---- host launchers ----------------------------------------------------------------------
static int trace_cap(const GridDev& G) { return ((G.K + 63) / 64) * 64; }
constexpr int kExactBlocks = 4096;   // one workgroup per deferred ray, 16 per CU
// The serial kernel (grids whose list does not fit LDS) keeps each wave's list in the workspace:
// its grid, and so the workspace, is capped at one wave per CU (deferred rays are rare; the
// waves stride over them) — 256 * K * 16 B, e.g. 56 MB at K = 13653 instead of 0.9 GB.
constexpr int kExactSerialBlocks = 256;
constexpr size_t kWsHead = 256;      // deferred (0), hit (64) and heap-range (128) counters

static bool exact_in_lds(const GridDev& G) {
    return exact_wave_lds(G.K, 1) <= kExactWaveLdsMax;
}
// Waves per deferred ray (exact_wave_kernel's W): 4 unless the list does not fit LDS with their
// stacks.
constexpr int kExactWaves = 4;
static bool exact_multi_wave(const GridDev& G) {
    return kExactWaves > 1 && exact_wave_lds(G.K, kExactWaves) <= kExactWaveLdsMax;
}
static size_t exact_scratch_bytes(const GridDev& G) {   // lists of large-K grids, one per wave
    return exact_in_lds(G) ? 0 : (size_t)kExactSerialBlocks * G.K * sizeof(Cand);
}
static size_t hits_bytes(int64_t n) { return (((size_t)n * sizeof(HitRay) + 255) / 256) * 256; }
static size_t workspace_bytes(const GridDev& G, int64_t n) {
    return kWsHead + (((size_t)n * sizeof(int64_t) + 255) / 256) * 256 + hits_bytes(n) +
           exact_scratch_bytes(G);
}

// The half-plane wedge (trace_one) is on unless SPHRT_TRACE_WEDGE=0 (A/B tests: the CSR is the
// same bit for bit either way).
static bool wedge_enabled() {
    const char* e = getenv("SPHRT_TRACE_WEDGE");
    return !(e && e[0] == '0');
}

// Which launches of a trace a call makes: screen (hit list; counts/zeros/bounds of the misses)
// and trace (the hit rays + the deferred exact ones).  BOUND screens only; EMIT traces the hit
// list an earlier BOUND call left in the same workspace.
enum { kScreen = 1, kTrace = 2 };

template <int MODE, typename T>
static int launch_trace(const GridDev& G, const RaysDev& R, TraceOut<T> o, void* workspace,
                        size_t workspace_size, hipStream_t st, int steps = kScreen | kTrace) {
    if (G.nr < 1 || G.ne < 1 || G.na < 1) return fail("tracing needs at least one voxel per axis");
    if (R.n == 0) return 0;
    if (!workspace || workspace_size < workspace_bytes(G, R.n))
        return fail("trace workspace too small: %zu < %zu bytes", workspace_size,
                    workspace_bytes(G, R.n));
    const int cap = trace_cap(G);
    // one LDS list of K entries per wave: 4 waves per workgroup, fewer for large K (a workgroup
    // may hold all 160 KiB of a CU's LDS), K <= 13653 with one wave; larger K (e.g. ~6800+
    // shells) sends every hit ray through the exact path, its list in the workspace
    const size_t per_wave = (size_t)cap * (sizeof(uint64_t) + sizeof(uint32_t));
    int waves = kWavesPerBlock;
    while (waves > 1 && (size_t)waves * per_wave > kLdsBytes) waves >>= 1;
    const size_t lds = (size_t)waves * per_wave;
    const bool wave_list = lds <= kLdsBytes;
    unsigned char* ws = (unsigned char*)workspace;
    o.n_deferred = (unsigned long long*)ws;
    o.n_hits = (unsigned*)(ws + 64);
    o.n_heap = (unsigned long long*)(ws + 128);
    o.deferred = (int64_t*)(ws + kWsHead);
    o.hits = (HitRay*)(ws + kWsHead + (((size_t)R.n * sizeof(int64_t) + 255) / 256) * 256);
    o.wedge = wedge_enabled();
    Cand* scratch = (Cand*)(ws + workspace_bytes(G, R.n) - exact_scratch_bytes(G));
    if constexpr (MODE == MODE_BOUND) steps = kScreen;
    if constexpr (MODE == MODE_EMIT) steps = kTrace;
    if (steps & kScreen) {
        if (hipMemsetAsync(ws, 0, kWsHead, st) != hipSuccess) return fail("memset failed");
        const size_t slds = MODE == MODE_BOUND && screen_lds(G)
                                ? (size_t)(G.nbr + G.nbe + G.nba) * sizeof(double) : 0;
        hipLaunchKernelGGL((screen_kernel<MODE, T>), dim3((unsigned)((R.n + 255) / 256)), dim3(256),
                           slds, st, G, R, o);
        if (int e = check_launch("screen_kernel")) return e;
    } else if (hipMemsetAsync(o.n_deferred, 0, sizeof(unsigned long long), st) != hipSuccess) {
        return fail("memset failed");
    }
    if constexpr (MODE == MODE_BOUND) return 0;
    if (!(steps & kTrace)) return 0;
    if (wave_list) {
        // enough waves to fill the chip several times over; each drains hits[w], hits[w + W], ...
        const int64_t grid = kTraceGrid * kWavesPerBlock / waves;
        hipLaunchKernelGGL((trace_kernel<MODE, T>), dim3((unsigned)grid), dim3(64 * waves), lds,
                           st, G, o, cap);
        if (int e = check_launch("trace_kernel")) return e;
    } else {
        hipLaunchKernelGGL((defer_hits_kernel<T>), dim3(256), dim3(256), 0, st, o);
        if (int e = check_launch("defer_hits_kernel")) return e;
    }
    if (exact_multi_wave(G))
        hipLaunchKernelGGL((exact_wave_kernel<MODE, T, double, false, false, kExactWaves>),
                           dim3(kExactBlocks), dim3(64 * kExactWaves),
                           exact_wave_lds(G.K, kExactWaves), st, G, R, o);
    else if (exact_in_lds(G))
        hipLaunchKernelGGL((exact_wave_kernel<MODE, T>), dim3(kExactBlocks), dim3(64),
                           exact_wave_lds(G.K, 1), st, G, R, o);
    else
        hipLaunchKernelGGL((exact_kernel<MODE, T>), dim3(kExactSerialBlocks), dim3(64), 0, st, G, R, o,
                           scratch);
    return check_launch("exact_kernel");
}

}  // namespace sphrt

using namespace sphrt;


extern "C" size_t sphrt_trace_workspace_bytes(const sphrt_plan* plan, int64_t n) {
    if (!plan || n < 0) return 0;
    return workspace_bytes(plan->dev, n);
}

extern "C" int sphrt_trace_count(const sphrt_plan* plan, const sphrt_rays* rays, int32_t* counts,
                                 void* workspace, size_t workspace_size, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    TraceOut<double> o{};
    o.counts = counts;
    return launch_trace<MODE_COUNT, double>(G, R, o, workspace, workspace_size,
                                            (hipStream_t)stream);
}

extern "C" int sphrt_trace_bound(const sphrt_plan* plan, const sphrt_rays* rays, int32_t* bounds,
                                 void* workspace, size_t workspace_size, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (!bounds) return fail("null bounds");
    TraceOut<double> o{};
    o.counts = bounds;
    return launch_trace<MODE_BOUND, double>(G, R, o, workspace, workspace_size,
                                            (hipStream_t)stream, kScreen);
}

extern "C" int sphrt_trace_emit(const sphrt_plan* plan, const sphrt_rays* rays,
                                const int64_t* bound_ptr, int32_t* counts, int32_t* svox,
                                double* slen, int64_t* n_over, void* workspace,
                                size_t workspace_size, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (!bound_ptr || !counts || !svox || !slen || !n_over) return fail("null emit argument");
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(n_over, 0, sizeof(int64_t), st) != hipSuccess) return fail("memset failed");
    TraceOut<double> o{};
    o.row_ptr = bound_ptr;
    o.counts = counts;
    o.vox = svox;
    o.len = slen;
    o.n_over = (unsigned long long*)n_over;
    return launch_trace<MODE_EMIT, double>(G, R, o, workspace, workspace_size, st, kTrace);
}

extern "C" int sphrt_trace_compact(int64_t n, const int64_t* bound_ptr, const int32_t* svox,
                                   const double* slen, const int64_t* row_ptr, int32_t* vox,
                                   double* len, void* stream) {
    if (n < 0) return fail("negative ray count");
    if (n == 0) return 0;
    if (!bound_ptr || !row_ptr || (!vox && !len) || (vox && !svox) || (len && !slen))
        return fail("null compact argument");
    StreamGuard guard(stream);
    const int64_t waves = (n + 63) / 64;
    const int64_t cap = (int64_t)1 << 30;
    const int64_t blocks = (waves + 3) / 4 < cap ? (waves + 3) / 4 : cap;
    hipLaunchKernelGGL(compact_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       n, bound_ptr, row_ptr, svox, slen, vox, len);
    return check_launch("compact_kernel");
}

extern "C" int sphrt_trace_fill(const sphrt_plan* plan, const sphrt_rays* rays,
                                const int64_t* row_ptr, int32_t* vox, double* len,
                                void* workspace, size_t workspace_size, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    TraceOut<double> o{};
    o.row_ptr = row_ptr;
    o.vox = vox;
    o.len = len;
    return launch_trace<MODE_FILL, double>(G, R, o, workspace, workspace_size,
                                           (hipStream_t)stream);
}

template <typename T>
static int trace_integrate(const sphrt_plan* plan, const sphrt_rays* rays, const T* density,
                           int64_t n_chan, int64_t chan_stride, int64_t ray_chan_div, T* out,
                           int64_t out_chan_stride, void* workspace, size_t workspace_size,
                           void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (n_chan < 1) return fail("n_chan must be >= 1");
    if (ray_chan_div > 0 && n_chan != 1) return fail("ray_chan_div requires n_chan == 1");
    TraceOut<T> o{};
    o.density = density;
    o.n_chan = n_chan;
    o.chan_stride = chan_stride;
    o.ray_chan_div = ray_chan_div;
    o.out = out;
    o.out_chan_stride = out_chan_stride;
    return launch_trace<MODE_INTEGRATE, T>(G, R, o, workspace, workspace_size,
                                           (hipStream_t)stream);
}

extern "C" int sphrt_trace_integrate_f32(const sphrt_plan* plan, const sphrt_rays* rays,
                                         const float* density, int64_t n_chan,
                                         int64_t chan_stride, int64_t ray_chan_div, float* out,
                                         int64_t out_chan_stride, void* workspace,
                                         size_t workspace_size, void* stream) {
    return trace_integrate<float>(plan, rays, density, n_chan, chan_stride, ray_chan_div, out,
                                  out_chan_stride, workspace, workspace_size, stream);
}
extern "C" int sphrt_trace_integrate_f64(const sphrt_plan* plan, const sphrt_rays* rays,
                                         const double* density, int64_t n_chan,
                                         int64_t chan_stride, int64_t ray_chan_div, double* out,
                                         int64_t out_chan_stride, void* workspace,
                                         size_t workspace_size, void* stream) {
    return trace_integrate<double>(plan, rays, density, n_chan, chan_stride, ray_chan_div, out,
                                   out_chan_stride, workspace, workspace_size, stream);
}

template <typename F>
static int solve(const sphrt_plan* plan, const sphrt_rays* rays, int family, F* t,
                 int32_t* region, int8_t* neg, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (family < 0 || family > 2) return fail("family must be 0 (r), 1 (e) or 2 (a)");
    if (R.n == 0) return 0;
    if (!t || !region || !neg) return fail("null solve output");
    const int64_t grid = (R.n + 255) / 256;
    hipLaunchKernelGGL(solve_kernel<F>, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, G,
                       R, family, t, region, neg);
    return check_launch("solve_kernel");
}
extern "C" int sphrt_solve(const sphrt_plan* plan, const sphrt_rays* rays, int family, double* t,
                           int32_t* region, int8_t* neg, void* stream) {
    return solve<double>(plan, rays, family, t, region, neg, stream);
}
extern "C" int sphrt_solve_f32(const sphrt_plan* plan, const sphrt_rays* rays, int family,
                               float* t, int32_t* region, int8_t* neg, void* stream) {
    return solve<float>(plan, rays, family, t, region, neg, stream);
}

// ---- reference-mode trace (Operator(..., ftype=float32) and / or invalid=True) ---------------
// Every ray takes the exact path — all K candidates in the reference's concatenation order, the
// emulated libstdc++ introsort, the forward fill and diff over the whole list — with the solves
// and the length differences in the trace's precision and, for invalid=True, no masking.  These
// options are outside every fast path (whose pruning — the outer-sphere span, the start-voxel
// rules, the wedge — relies on float64 distances and on the masks).  One pass
// (sphrt_trace_reference_emit: every ray into a slot of K segments, then a compaction) or two
// (count, then fill); without invalid=True the rays that cannot keep a segment are screened out
// (exact_wave_kernel), which at C2 is ~82 % of them.
// The reference-mode screen (without invalid=True), one ray per lane: a ray that starts outside
// every shell (start region r < 0) and crosses no sphere (every sphere_solve distance +inf, in the
// trace's precision) keeps r < 0 for every segment before its first infinite entry, and every
// segment from there on is infinite or NaN: all masked (raytracer.py:155-173), no segment.  The
// others are listed (o.deferred, one atomic per wave) for the exact path, one wave each over the
// whole chip.  (invalid=True keeps those segments: no screen.)  In the exact path's kernel the
// screen took a wave per 64 rays and that wave then traced their ~12 hit rays one after another:
// C2 ftype=float32 exact kernel 628 us.
template <int MODE, typename F>
__global__ __launch_bounds__(256) void ref_screen_kernel(GridDev G, RaysDev R, TraceOut<double> o) {
    const int64_t my = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    bool need = false;
    if (my < R.n) {
        double x[3], d[3];
        int s[3];
        load_ray(R, my, x, d, s);
        need = s[0] >= 0;
        if (!need) {
            const RayGeoT<F> g = exact_geo<F>(x, d);
            for (int j = G.nbr - 1; j >= 0 && !need; --j) {   // (outer shells first: hits stop early)
                F ti, to;
                int ri, ro, ni, no;
                sphere_solve(G, g, j, ti, ri, to, ro, ni, no);
                need = __builtin_isfinite(ti) || __builtin_isfinite(to);
            }
        }
        if (!need) {
            if (MODE == MODE_COUNT) o.counts[my] = 0;
            if (MODE == MODE_EMIT) (void)emit_slot(o, my, 0, true);
        }
    }
    const uint64_t m = __ballot(need);
    unsigned long long base = 0;
    if (lane == 0 && m) base = atomicAdd(o.n_deferred, (unsigned long long)__popcll(m));
    base = (unsigned long long)__shfl((long long)base, 0);
    if (need) o.deferred[base + __popcll(m & lanemask_lt(lane))] = my;
}

template <int MODE, typename F, bool INV>
static int launch_reference(const GridDev& G, const RaysDev& R, TraceOut<double> o,
                            void* workspace, size_t workspace_size, hipStream_t st) {
    if (G.nr < 1 || G.ne < 1 || G.na < 1) return fail("tracing needs at least one voxel per axis");
    if (R.n == 0) return 0;
    if (!workspace || workspace_size < workspace_bytes(G, R.n))
        return fail("trace workspace too small: %zu < %zu bytes", workspace_size,
                    workspace_bytes(G, R.n));
    unsigned char* ws = (unsigned char*)workspace;
    o.n_deferred = (unsigned long long*)ws;
    o.n_heap = (unsigned long long*)(ws + 128);
    if (hipMemsetAsync(ws, 0, kWsHead, st) != hipSuccess) return fail("memset failed");
    if (!INV) {
        o.deferred = (int64_t*)(ws + kWsHead);
        hipLaunchKernelGGL((ref_screen_kernel<MODE, F>), dim3((unsigned)((R.n + 255) / 256)),
                           dim3(256), 0, st, G, R, o);
        if (int e = check_launch("ref_screen_kernel")) return e;
    }
    if (exact_in_lds(G)) {
        const int64_t blocks = R.n < 4 * kExactBlocks ? R.n : 4 * kExactBlocks;
        hipLaunchKernelGGL((exact_wave_kernel<MODE, double, F, INV, true>), dim3((unsigned)blocks),
                           dim3(64), exact_wave_lds(G.K, 1), st, G, R, o);
    } else {
        Cand* scratch = (Cand*)(ws + workspace_bytes(G, R.n) - exact_scratch_bytes(G));
        hipLaunchKernelGGL((exact_kernel<MODE, double, F, INV, true>), dim3(kExactSerialBlocks),
                           dim3(64), 0, st, G, R, o, scratch);
    }
    return check_launch("exact_kernel (reference mode)");
}

extern "C" int sphrt_trace_reference_emit(const sphrt_plan* plan, const sphrt_rays* rays,
                                          int flags, const int64_t* bound_ptr, int32_t* counts,
                                          int32_t* svox, double* slen, int64_t* n_over,
                                          void* workspace, size_t workspace_size, void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (flags & ~(SPHRT_TRACE_F32 | SPHRT_TRACE_INVALID | SPHRT_TRACE_FRESH_RAYS))
        return fail("unknown trace flags %d", flags);
    if (!bound_ptr || !counts || !svox || !slen || !n_over) return fail("null emit argument");
    R.fresh = (flags & SPHRT_TRACE_FRESH_RAYS) != 0;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(n_over, 0, sizeof(int64_t), st) != hipSuccess) return fail("memset failed");
    TraceOut<double> o{};
    o.row_ptr = bound_ptr;
    o.counts = counts;
    o.vox = svox;
    o.len = slen;
    o.n_over = (unsigned long long*)n_over;
    const bool f32 = (flags & SPHRT_TRACE_F32) != 0, inv = (flags & SPHRT_TRACE_INVALID) != 0;
    if (f32)
        return inv ? launch_reference<MODE_EMIT, float, true>(G, R, o, workspace, workspace_size, st)
                   : launch_reference<MODE_EMIT, float, false>(G, R, o, workspace, workspace_size, st);
    return inv ? launch_reference<MODE_EMIT, double, true>(G, R, o, workspace, workspace_size, st)
               : launch_reference<MODE_EMIT, double, false>(G, R, o, workspace, workspace_size, st);
}

extern "C" int sphrt_trace_reference(const sphrt_plan* plan, const sphrt_rays* rays, int flags,
                                     int32_t* counts, const int64_t* row_ptr, int32_t* vox,
                                     double* len, void* workspace, size_t workspace_size,
                                     void* stream) {
    GridDev G;
    RaysDev R;
    if (int e = resolve(plan, rays, G, R, stream)) return e;
    DeviceGuard guard(plan->device);
    if (flags & ~(SPHRT_TRACE_F32 | SPHRT_TRACE_INVALID | SPHRT_TRACE_FRESH_RAYS))
        return fail("unknown trace flags %d", flags);
    R.fresh = (flags & SPHRT_TRACE_FRESH_RAYS) != 0;
    hipStream_t st = (hipStream_t)stream;
    TraceOut<double> o{};
    const bool f32 = (flags & SPHRT_TRACE_F32) != 0, inv = (flags & SPHRT_TRACE_INVALID) != 0;
    if (!row_ptr) {
        if (!counts) return fail("null counts");
        o.counts = counts;
        if (f32)
            return inv ? launch_reference<MODE_COUNT, float, true>(G, R, o, workspace, workspace_size, st)
                       : launch_reference<MODE_COUNT, float, false>(G, R, o, workspace, workspace_size, st);
        return inv ? launch_reference<MODE_COUNT, double, true>(G, R, o, workspace, workspace_size, st)
                   : launch_reference<MODE_COUNT, double, false>(G, R, o, workspace, workspace_size, st);
    }
    if (!vox || !len) return fail("null fill output");
    o.row_ptr = row_ptr;
    o.vox = vox;
    o.len = len;
    if (f32)
        return inv ? launch_reference<MODE_FILL, float, true>(G, R, o, workspace, workspace_size, st)
                   : launch_reference<MODE_FILL, float, false>(G, R, o, workspace, workspace_size, st);
    return inv ? launch_reference<MODE_FILL, double, true>(G, R, o, workspace, workspace_size, st)
               : launch_reference<MODE_FILL, double, false>(G, R, o, workspace, workspace_size, st);
}
