// introsort.hpp — bit-exact device emulation of the reference's unstable sort.
//
// trace_indices sorts every ray's candidate distances with torch.sort (raytracer.py:131), which on
// CPU is libstdc++ std::sort over (value, index) pairs compared by value with operator< (verified
// here against torch on random tie-heavy rows: tests/test_introsort_emulation.py).  When two
// crossings that update the same region row sit at exactly the same distance, their order — and
// with it the voxel of the following segments — is whatever that introsort produces.  This header
// reproduces it step for step (median-of-three pivot, unguarded Hoare partition, depth limit
// 2*floor(log2 n) with heapsort fallback, threshold 16, final insertion sort) on one lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sphrt {

struct Cand {
    double t;      // crossing distance (sort key)
    uint32_t pay;  // candidate index << 16 | (region + 2)
    uint32_t pad;
};

// The sort runs on any list with get/set of one element and operator< on the distance: an array
// of Cand (one lane per list, workspace) or the distance / payload arrays of a wave's LDS list.
struct CandList {
    using E = Cand;
    Cand* v;
    __device__ E get(int i) const { return v[i]; }
    __device__ void set(int i, const E& e) const { v[i] = e; }
};
struct SoaList {
    struct E {
        double t;
        uint32_t pay;
    };
    double* t;
    uint32_t* pay;
    __device__ E get(int i) const { return E{t[i], pay[i]}; }
    __device__ void set(int i, const E& e) const {
        t[i] = e.t;
        pay[i] = e.pay;
    }
};

template <class E>
__device__ __forceinline__ bool eless(const E& a, const E& b) { return a.t < b.t; }
template <class V>
__device__ __forceinline__ bool cless(const V& v, int a, int b) { return eless(v.get(a), v.get(b)); }
template <class V>
__device__ __forceinline__ void cswap(const V& v, int i, int j) {
    const auto x = v.get(i);
    v.set(i, v.get(j));
    v.set(j, x);
}

template <class V>
__device__ inline void move_median_to_first(const V& v, int res, int a, int b, int c) {
    if (cless(v, a, b)) {
        if (cless(v, b, c)) cswap(v, res, b);
        else if (cless(v, a, c)) cswap(v, res, c);
        else cswap(v, res, a);
    } else if (cless(v, a, c)) {
        cswap(v, res, a);
    } else if (cless(v, b, c)) {
        cswap(v, res, c);
    } else {
        cswap(v, res, b);
    }
}

template <class V>
__device__ inline int unguarded_partition(const V& v, int first, int last, int piv) {
    while (true) {
        while (cless(v, first, piv)) ++first;
        --last;
        while (cless(v, piv, last)) --last;
        if (!(first < last)) return first;
        cswap(v, first, last);
        ++first;
    }
}

template <class V, class E>
__device__ inline void adjust_heap(const V& v, int first, int hole, int len, E value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (cless(v, first + child, first + child - 1)) child--;
        v.set(first + hole, v.get(first + child));
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        v.set(first + hole, v.get(first + child - 1));
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && eless(v.get(first + parent), value)) {
        v.set(first + hole, v.get(first + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    v.set(first + hole, value);
}

// std::__partial_sort(first, last, last) = make_heap + sort_heap
template <class V>
__device__ inline void heap_sort(const V& v, int first, int last) {
    const int len = last - first;
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap(v, first, parent, len, v.get(first + parent));
            if (parent == 0) break;
        }
    }
    while (last - first > 1) {
        --last;
        const auto value = v.get(last);
        v.set(last, v.get(first));
        adjust_heap(v, first, 0, last - first, value);
    }
}

template <class V>
__device__ inline void unguarded_linear_insert(const V& v, int last) {
    const auto val = v.get(last);
    int next = last - 1;
    while (eless(val, v.get(next))) {
        v.set(last, v.get(next));
        last = next;
        --next;
    }
    v.set(last, val);
}

template <class V>
__device__ inline void insertion_sort(const V& v, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (cless(v, i, first)) {
            const auto val = v.get(i);
            for (int k = i; k > first; --k) v.set(k, v.get(k - 1));
            v.set(first, val);
        } else {
            unguarded_linear_insert(v, i);
        }
    }
}

constexpr int kIntroThreshold = 16;

template <class V>
__device__ inline void introsort(const V& v, int n) {
    if (n <= 1) return;
    const int lg = 31 - __builtin_clz((unsigned)n);
    // __introsort_loop recurses on [cut, last) and iterates on [first, cut); the two ranges are
    // disjoint, so an explicit stack in any order gives the same final array.
    int st_first[64], st_last[64], st_depth[64];
    int sp = 0;
    st_first[0] = 0; st_last[0] = n; st_depth[0] = 2 * lg; sp = 1;
    while (sp > 0) {
        --sp;
        int first = st_first[sp], last = st_last[sp], depth = st_depth[sp];
        while (last - first > kIntroThreshold) {
            if (depth == 0) {
                heap_sort(v, first, last);
                break;
            }
            --depth;
            const int mid = first + (last - first) / 2;
            move_median_to_first(v, first, first + 1, mid, last - 1);
            const int cut = unguarded_partition(v, first + 1, last, first);
            st_first[sp] = cut; st_last[sp] = last; st_depth[sp] = depth; ++sp;
            last = cut;
        }
    }
    if (n > kIntroThreshold) {
        insertion_sort(v, 0, kIntroThreshold);
        for (int i = kIntroThreshold; i < n; ++i) unguarded_linear_insert(v, i);
    } else {
        insertion_sort(v, 0, n);
    }
}

}  // namespace sphrt
