/*
 * sphrt_oracle.c — CPU restatement of the reference raytracer's trace, for TESTS ONLY.
 *
 * TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library, and only as the checker / the timed CPU baseline.  The product path
 * (sph_raytracer_amd) never links, loads or calls it.
 *
 * What it restates (file:line in Evidlo/sph_raytracer @ 2025-06-13):
 *   ora_solve_r   <- r_torch        raytracer.py:248-325
 *   ora_solve_e   <- e_torch        raytracer.py:328-468
 *   ora_solve_a   <- a_torch        raytracer.py:471-552
 *   ora_trace     <- trace_indices  raytracer.py:48-230 (concat :92-122, t<0 carry :126,
 *                                   sort :131, take_along_dim :136, forward fill :140 / :17-45,
 *                                   diff :150-151, masking :155-173)
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
static vsqrt_fn g_vsqrt = NULL;

void ora_set_sqrt(vsqrt_fn fn) { g_vsqrt = fn; }

/* torch.sqrt: MKL vdSqrt on the reference host when bound, IEEE otherwise */
static double tsqrt(double x) {
    if (g_vsqrt) {
        double r;
        g_vsqrt(1, &x, &r);
        return r;
    }
    return sqrt(x);
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

/* linalg.norm: fused sum of squares + correctly rounded sqrt */
static double lnorm(const double v[3]) { return sqrt(fma(v[2], v[2], fma(v[1], v[1], v[0] * v[0]))); }
/* einsum '...j,...j' : ((a0 b0 + a1 b1) + a2 b2), no fusion */
static double edot(const double a[3], const double b[3]) {
    double s = a[0] * b[0] + a[1] * b[1];
    return s + a[2] * b[2];
}

typedef struct {
    double x[3], d1[3], d2[3];
} ora_ray;

/* rays /= linalg.norm(rays) is applied in place by r_torch and again by e_torch
 * (raytracer.py:281, 365): two successive normalisations */
static void ora_ray_init(ora_ray *R, const double *x, const double *d) {
    double n1, n2;
    int i;
    for (i = 0; i < 3; ++i) R->x[i] = x[i];
    n1 = lnorm(d);
    for (i = 0; i < 3; ++i) R->d1[i] = d[i] / n1;
    n2 = lnorm(R->d1);
    for (i = 0; i < 3; ++i) R->d2[i] = R->d1[i] / n2;
}

/* Called on their own, e_torch normalises its input once (raytracer.py:365) and a_torch not at
 * all: the cone/plane direction d2 is then d/|d| resp. d itself. */
static void ora_ray_init_family(ora_ray *R, const double *x, const double *d, int family) {
    int i;
    ora_ray_init(R, x, d);
    if (family == 1)
        for (i = 0; i < 3; ++i) R->d2[i] = R->d1[i];
    else if (family == 2)
        for (i = 0; i < 3; ++i) R->d2[i] = d[i];
}

/* ---- r_torch: raytracer.py:288-323 ------------------------------------------------------------- */
static void sphere_all(const ora_grid *g, const ora_ray *R, double *t, int *reg, signed char *neg) {
    const int nb = g->nr + 1;
    double mx[3] = {-R->x[0], -R->x[1], -R->x[2]};
    double tc = edot(mx, R->d1);
    double d = tsqrt(edot(R->x, R->x) - tc * tc);
    int j, k;
    for (j = 0; j < nb; ++j) {
        double rr = g->r_b[j] * g->r_b[j];
        double t1c = tsqrt(rr - d * d);
        t[j] = tc - t1c;
        t[nb + j] = tc + t1c;
    }
    for (k = 0; k < 2 * nb; ++k) {
        double p[3];
        int i, ng, r;
        for (i = 0; i < 3; ++i) p[i] = R->d1[i] * t[k] + R->x[i];
        ng = edot(R->d1, p) < 0.0;
        r = (k % nb) - ng;
        if (r == g->nr) r = -1;
        reg[k] = r;
        if (neg) neg[k] = (signed char)ng;
        if (isnan(t[k])) t[k] = INFINITY;
    }
}

/* ---- e_torch: raytracer.py:365-466 ------------------------------------------------------------- */
static void cone_all(const ora_grid *g, const ora_ray *R, double *t, int *reg, signed char *neg) {
    const int nb = g->ne + 1;
    const double *w = R->d2, *x = R->x;
    const double th = g->th;
    double wx = edot(w, x);
    double nx = lnorm(x);
    int j, k;
    for (j = 0; j < nb; ++j) {
        double c2 = g->cos2_e[j];
        double aa = w[2] * w[2] - c2;
        double bb = 2.0 * (w[2] * x[2] - wx * c2);
        double cc = x[2] * x[2] - (nx * nx) * c2;
        double delta, t1, t2;
        if (fabs(aa) < th) aa = 0.0;
        delta = bb * bb - (4.0 * aa) * cc;
        if (fabs(delta) < th) delta = 0.0;
        t1 = (-bb + tsqrt(delta)) / (2.0 * aa);
        t2 = (-bb - tsqrt(delta)) / (2.0 * aa);
        if (fabs(aa) < th && !(fabs(bb) < th)) {   /* parallel to a generator: one root */
            t1 = (-cc) / bb;
            t2 = INFINITY;
        }
        if (aa == 0.0 && bb == 0.0 && cc == 0.0) { /* on the cone */
            t1 = INFINITY;
            t2 = INFINITY;
        }
        t[j] = t1;
        t[nb + j] = t2;
    }
    for (k = 0; k < 2 * nb; ++k) {
        const int j2 = k % nb;
        double p[3], pn[3], prod;
        int i, ng, r, shadow;
        for (i = 0; i < 3; ++i) p[i] = w[i] * t[k] + x[i];
        /* torch.cross(p, (-p1, p0, 0)) */
        pn[0] = fma(p[1], 0.0, -(p[2] * p[0]));
        pn[1] = fma(p[2], -p[1], -(p[0] * 0.0));
        pn[2] = fma(p[0], p[0], -(p[1] * (-p[1])));
        prod = edot(w, pn);
        ng = prod > 0.0;
        r = j2 - ng;
        if (fabs(prod) < th) r = -2;
        shadow = (p[2] >= 0.0) != (g->cos_e[j2] >= 0.0);
        if (fabs(3.141592653589793 / 2 - g->e_b[j2]) < th) shadow = 0;
        if (shadow) t[k] = INFINITY;
        if (r == g->ne) r = -1;
        if (isnan(t[k])) t[k] = INFINITY;
        reg[k] = r;
        if (neg) neg[k] = (signed char)ng;
    }
}

/* ---- a_torch: raytracer.py:505-550 ------------------------------------------------------------- */
static void plane_all(const ora_grid *g, const ora_ray *R, double *t, int *reg, signed char *neg) {
    const int nb = g->na + 1;
    const double *w = R->d2, *x = R->x;
    int j;
    for (j = 0; j < nb; ++j) {
        double ca = g->cos_a[j], sa = g->sin_a[j];
        double nrm[3] = {-sa, ca, 0.0};
        double num = fma(nrm[2], x[2], fma(nrm[1], x[1], nrm[0] * x[0]));
        double den = fma(nrm[2], w[2], fma(nrm[1], w[1], nrm[0] * w[0]));
        double tt = (-num) / den;
        double cz = fma(ca, w[1], -(sa * w[0]));
        double p0, p1;
        int ng, r;
        if (fabs(cz) <= g->par) tt = INFINITY;
        ng = cz < 0.0;
        r = j - ng;
        if (g->a_wrap) {
            r %= g->na;
            if (r < 0) r += g->na;
        } else if (r == g->na) {
            r = -1;
        }
        p0 = tt * w[0] + x[0];
        p1 = tt * w[1] + x[1];
        if (fma(sa, p1, ca * p0) < 0.0) tt = INFINITY;
        if (isnan(tt)) tt = INFINITY;
        t[j] = tt;
        reg[j] = r;
        if (neg) neg[j] = (signed char)ng;
    }
}

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

/* ---- per-family API (test_all.py known answers, solver fixtures) ------------------------------- */
void ora_solve(const ora_grid *g, int family, const double *xs, const double *rays, int64_t n,
               double *t, int *reg, signed char *neg) {
    int64_t i;
    const int w = family == 0 ? 2 * (g->nr + 1) : family == 1 ? 2 * (g->ne + 1) : g->na + 1;
#pragma omp parallel for schedule(static)
    for (i = 0; i < n; ++i) {
        ora_ray R;
        ora_ray_init_family(&R, xs + 3 * i, rays + 3 * i, family);
        if (family == 0) sphere_all(g, &R, t + i * w, reg + i * w, neg + i * w);
        else if (family == 1) cone_all(g, &R, t + i * w, reg + i * w, neg + i * w);
        else plane_all(g, &R, t + i * w, reg + i * w, neg + i * w);
    }
}

int64_t ora_candidates(const ora_grid *g) {
    return 2LL * (g->nr + 1) + 2LL * (g->ne + 1) + (g->na + 1) + 1;
}

/* ---- trace_indices for one ray: K-padded (regs, lens) exactly as the reference ------------------ */
static void trace_one(const ora_grid *g, const double *x, const double *d, const int *start,
                      double *t, int *rows /* 3*K */, int *idx, int *regs_out /* 3*K */,
                      double *lens_out) {
    const int nbr = g->nr + 1, nbe = g->ne + 1, nba = g->na + 1;
    const int K = 2 * nbr + 2 * nbe + nba + 1;
    ora_ray R;
    int *rr = rows, *re = rows + K, *ra = rows + 2 * K;
    int k, cur[3];
    ora_ray_init(&R, x, d);
    /* concatenated candidates and the (3, K) region table, -2 = "no change" (:92-122) */
    for (k = 0; k < K; ++k) rr[k] = re[k] = ra[k] = -2;
    sphere_all(g, &R, t, rr, NULL);
    cone_all(g, &R, t + 2 * nbr, re + 2 * nbr, NULL);
    plane_all(g, &R, t + 2 * nbr + 2 * nbe, ra + 2 * nbr + 2 * nbe, NULL);
    /* sphere_all wrote its regions to rr[0 .. 2nbr) — the other families into their own rows */
    t[K - 1] = 0.0;
    rr[K - 1] = start[0];
    re[K - 1] = start[1];
    ra[K - 1] = start[2];
    for (k = 0; k < K; ++k)            /* behind the start: carry (:126) */
        if (t[k] < 0.0) rr[k] = re[k] = ra[k] = -2;
    ora_introsort(t, idx, K);          /* (:131, :136) */
    cur[0] = start[0]; cur[1] = start[1]; cur[2] = start[2];
    for (k = 0; k < K; ++k) {          /* forward fill (:140), lengths (:150-151), masks (:155-173) */
        const int s = idx[k];
        double len;
        if (rr[s] != -2) cur[0] = rr[s];
        if (re[s] != -2) cur[1] = re[s];
        if (ra[s] != -2) cur[2] = ra[s];
        len = (k + 1 < K ? t[k + 1] : INFINITY) - t[k];
        if (isinf(len) || isnan(len)) len = 0.0;
        if (cur[0] > g->nr - 1 || cur[1] > g->ne - 1 || cur[2] > g->na - 1) len = 0.0;
        if (cur[0] < 0 || cur[1] < 0 || cur[2] < 0) len = 0.0;
        regs_out[k] = cur[0];
        regs_out[K + k] = cur[1];
        regs_out[2 * K + k] = cur[2];
        lens_out[k] = len;
    }
}

/* Dense output: regs (n, 3, K) int32, lens (n, K). */
void ora_trace_dense(const ora_grid *g, const double *xs, const double *rays, const int *starts,
                     int64_t n, int *regs, double *lens) {
    const int K = (int)ora_candidates(g);
    int64_t i;
#pragma omp parallel
    {
        double *t = (double *)malloc(sizeof(double) * K);
        int *rows = (int *)malloc(sizeof(int) * 3 * K);
        int *idx = (int *)malloc(sizeof(int) * K);
#pragma omp for schedule(dynamic, 64)
        for (i = 0; i < n; ++i)
            trace_one(g, xs + 3 * i, rays + 3 * i, starts + 3 * i, t, rows, idx, regs + i * 3 * K,
                      lens + i * K);
        free(t); free(rows); free(idx);
    }
}

/* Compact output, two passes like the GPU path: counts, then (vox, len) of the non-zero entries
 * in sorted order.  vox = (r*ne + e)*na + a. */
static void compact_one(const ora_grid *g, const double *x, const double *d, const int *start,
                        double *t, int *rows, int *idx, int *rg, double *ln, int *cnt,
                        int *vox, double *len) {
    const int K = (int)ora_candidates(g);
    int k, c = 0;
    trace_one(g, x, d, start, t, rows, idx, rg, ln);
    for (k = 0; k < K; ++k) {
        if (ln[k] > 0.0) {
            if (vox) {
                vox[c] = (rg[k] * g->ne + rg[K + k]) * g->na + rg[2 * K + k];
                len[c] = ln[k];
            }
            ++c;
        }
    }
    *cnt = c;
}

void ora_trace_segments(const ora_grid *g, const double *xs, const double *rays,
                        const int *starts, int64_t n, const int64_t *row_ptr, int *counts,
                        int *vox, double *len) {
    const int K = (int)ora_candidates(g);
    int64_t i;
#pragma omp parallel
    {
        double *t = (double *)malloc(sizeof(double) * K);
        int *rows = (int *)malloc(sizeof(int) * 3 * K);
        int *idx = (int *)malloc(sizeof(int) * K);
        int *rg = (int *)malloc(sizeof(int) * 3 * K);
        double *ln = (double *)malloc(sizeof(double) * K);
#pragma omp for schedule(dynamic, 64)
        for (i = 0; i < n; ++i) {
            int c;
            compact_one(g, xs + 3 * i, rays + 3 * i, starts + 3 * i, t, rows, idx, rg, ln, &c,
                        row_ptr ? vox + row_ptr[i] : NULL, row_ptr ? len + row_ptr[i] : NULL);
            if (counts) counts[i] = c;
        }
        free(t); free(rows); free(idx); free(rg); free(ln);
    }
}
