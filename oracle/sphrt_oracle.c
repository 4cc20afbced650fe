/*
 * sphrt_oracle.c — CPU restatement of the reference raytracer's trace, for TESTS ONLY.
 *
 * TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library, and only as the checker / the timed CPU baseline.  The product path
 * (sph_raytracer_amd) never links, loads or calls it.
 *
 * Precision: the solvers and the trace (sphrt_oracle_body.inc) are compiled twice, in double
 * (ora_*: ftype=torch.float64, the default) and in float (ora_*_f32: ftype=torch.float32).
 *
 * What it restates (file:line in Evidlo/sph_raytracer @ 2025-06-13):
 *   ora_solve_r   <- r_torch        raytracer.py:248-325
 *   ora_solve_e   <- e_torch        raytracer.py:328-468
 *   ora_solve_a   <- a_torch        raytracer.py:471-552
 *   ora_trace     <- trace_indices  raytracer.py:48-230 (concat :92-122, t<0 carry :126,
 *                                   sort :131, take_along_dim :136, forward fill :140 / :17-45,
 *                                   diff :150-151, masking :155-173 unless invalid=True)
 *   ora_introsort <- torch.sort on CPU (raytracer.py:131) = libstdc++ std::sort of
 *                    (value, index) pairs by value (introsort; pinned against torch in
 *                    tests/test_oracle.py)
 * Pinning: tests/test_oracle.py checks every output against the tests/golden npz files, which were
 * captured from the reference itself (tests/golden/make_golden.py).  With sqrt bound to MKL
 * vdSqrt (ora_set_sqrt, the routine torch CPU uses) the crossing distances are bit-identical.
 *
 * Independent of the HIP implementation: one scalar ray at a time, all K candidates materialised
 * per ray exactly as the reference concatenates them, the full introsort, a sequential walk.
 * Build: gcc -O2 -ffp-contract=off -fopenmp -shared -fPIC (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef void (*vsqrt_fn)(int, const double *, double *);
typedef void (*vsqrtf_fn)(int, const float *, float *);
static vsqrt_fn g_vsqrt = NULL;
static vsqrtf_fn g_vsqrtf = NULL;

void ora_set_sqrt(vsqrt_fn fn) { g_vsqrt = fn; }
void ora_set_sqrt_f32(vsqrtf_fn fn) { g_vsqrtf = fn; }

/* torch.sqrt: MKL vdSqrt / vsSqrt on the reference host when bound (neither is correctly rounded
 * on every input), IEEE otherwise */
static double tsqrt(double x) {
    if (g_vsqrt) {
        double r;
        g_vsqrt(1, &x, &r);
        return r;
    }
    return sqrt(x);
}
static float tsqrtf(float x) {
    if (g_vsqrtf) {
        float r;
        g_vsqrtf(1, &x, &r);
        return r;
    }
    return sqrtf(x);
}

typedef struct {
    int nr, ne, na;
    const double *r_b, *e_b, *a_b;      /* boundaries                                  */
    const double *cos_e, *cos2_e;        /* torch.cos(e), torch.cos(e)**2 (host torch)  */
    const double *cos_a, *sin_a;         /* torch.cos(a_b), torch.sin(a_b)              */
    int a_wrap;                          /* -a_b[0] == a_b[-1] == pi                    */
    double th;                           /* finfo.resolution ** (1/3)                   */
    double par;                          /* finfo.resolution                            */
} ora_grid;

/* ---- torch.sort (CPU) == libstdc++ std::sort on (value, index) --------------------------------- */
typedef struct {
    double t;
    int idx;
} ora_item;

static int lt(const ora_item *a, const ora_item *b) { return a->t < b->t; }
static void sw(ora_item *v, int i, int j) {
    ora_item x = v[i];
    v[i] = v[j];
    v[j] = x;
}

static void median_first(ora_item *v, int res, int a, int b, int c) {
    if (lt(&v[a], &v[b])) {
        if (lt(&v[b], &v[c])) sw(v, res, b);
        else if (lt(&v[a], &v[c])) sw(v, res, c);
        else sw(v, res, a);
    } else if (lt(&v[a], &v[c])) sw(v, res, a);
    else if (lt(&v[b], &v[c])) sw(v, res, c);
    else sw(v, res, b);
}

static int hoare(ora_item *v, int first, int last, int piv) {
    for (;;) {
        while (lt(&v[first], &v[piv])) ++first;
        --last;
        while (lt(&v[piv], &v[last])) --last;
        if (!(first < last)) return first;
        sw(v, first, last);
        ++first;
    }
}

static void sift(ora_item *v, int base, int hole, int len, ora_item val) {
    int top = hole, child = hole, parent;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (lt(&v[base + child], &v[base + child - 1])) child--;
        v[base + hole] = v[base + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        v[base + hole] = v[base + child - 1];
        hole = child - 1;
    }
    parent = (hole - 1) / 2;
    while (hole > top && lt(&v[base + parent], &val)) {
        v[base + hole] = v[base + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    v[base + hole] = val;
}

static void heapsort_range(ora_item *v, int first, int last) {
    int len = last - first, parent;
    if (len >= 2)
        for (parent = (len - 2) / 2;; --parent) {
            sift(v, first, parent, len, v[first + parent]);
            if (parent == 0) break;
        }
    while (last - first > 1) {
        ora_item val;
        --last;
        val = v[last];
        v[last] = v[first];
        sift(v, first, 0, last - first, val);
    }
}

static void intro_loop(ora_item *v, int first, int last, int depth) {
    while (last - first > 16) {
        int cut;
        if (depth == 0) {
            heapsort_range(v, first, last);
            return;
        }
        --depth;
        median_first(v, first, first + 1, first + (last - first) / 2, last - 1);
        cut = hoare(v, first + 1, last, first);
        intro_loop(v, cut, last, depth);
        last = cut;
    }
}

static void lin_insert(ora_item *v, int last) {
    ora_item val = v[last];
    int next = last - 1;
    while (lt(&val, &v[next])) {
        v[last] = v[next];
        last = next--;
    }
    v[last] = val;
}

void ora_introsort(double *t, int *idx, int n) {
    ora_item *v = (ora_item *)malloc(sizeof(ora_item) * (n > 0 ? n : 1));
    int i, lg = 0;
    for (i = 0; i < n; ++i) { v[i].t = t[i]; v[i].idx = i; }
    while ((2 << lg) <= n) ++lg;     /* floor(log2(n)) */
    if (n > 1) {
        int lim = n > 16 ? 16 : n;
        intro_loop(v, 0, n, 2 * lg);
        for (i = 1; i < lim; ++i) {
            if (lt(&v[i], &v[0])) {
                ora_item val = v[i];
                memmove(v + 1, v, sizeof(ora_item) * i);
                v[0] = val;
            } else {
                lin_insert(v, i);
            }
        }
        for (i = 16; i < n; ++i) lin_insert(v, i);
    }
    for (i = 0; i < n; ++i) { t[i] = v[i].t; idx[i] = v[i].idx; }
    free(v);
}

int64_t ora_candidates(const ora_grid *g) {
    return 2LL * (g->nr + 1) + 2LL * (g->ne + 1) + (g->na + 1) + 1;
}

/* ---- the solvers and the trace, once per precision -------------------------------------------- */
#define REAL double
#define SFX(name) name
#define RSQRT sqrt
#define RFMA fma
#define RFABS fabs
#define TSQRT tsqrt
#include "sphrt_oracle_body.inc"
#undef REAL
#undef SFX
#undef RSQRT
#undef RFMA
#undef RFABS
#undef TSQRT

#define REAL float
#define SFX(name) name##_f32
#define RSQRT sqrtf
#define RFMA fmaf
#define RFABS fabsf
#define TSQRT tsqrtf
#include "sphrt_oracle_body.inc"
