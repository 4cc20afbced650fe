// solve.hpp — per-ray boundary-crossing solves on gfx950, in the trace's precision F: FP64 (the
// reference default and every fast path) or FP32 (Operator(..., ftype=torch.float32): the same
// expressions evaluated in float, as torch runs them on float32 tensors).
//
// Restates the arithmetic of the reference's materialised torch solvers one crossing at a time, in
// registers.  Every expression keeps the reference's operation order; this translation unit is
// compiled with -ffp-contract=off and every fused multiply-add below is an explicit fma(), placed
// where torch's CPU kernels fuse (linalg.norm, cross, the '...bc,...jc->...b' einsum).  The only
// intentional difference is sqrt: torch CPU calls MKL vdSqrt (not correctly rounded), the GPU uses
// IEEE sqrt — a <=1-ulp difference in a small fraction of sphere/cone distances, never in regions
// (SURVEY.md §8(c)).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sphrt {

constexpr double kInf = __builtin_huge_val();

// Boundary tables of one grid, resident in device memory (owned by the plan).
struct GridDev {
    int nr, ne, na;        // voxels per axis
    int nbr, nbe, nba;     // boundaries per axis (n + 1)
    int K;                 // candidates per ray incl. the start entry
    int a_wrap;            // full azimuth circle -> regions wrap mod na
    double close_tol;      // isclose() threshold (raytracer.py:246)
    double plane_par_tol;  // a_torch parallel threshold (raytracer.py:521)
    double r_outer;        // r_b[nr]
    int e_asc, a_asc;      // e_b / a_b strictly ascending (segment bounds may binary-search them)
    int uni;               // bit 0 / 1 / 2: r_b / e_b / a_b evenly spaced (counted arithmetically)
    // One table block: r_b (nbr) | cos(e_b)**2 (nbe) | cos(a_b) (nba) | sin(a_b) (nba) | e_b (nbe)
    // | a_b (nba) as doubles, then e_flags (nbe bytes; bit0: cos(e_b) >= 0, bit1: shadow test
    // exempt, e_b ~ pi/2).  One pointer instead of seven: the trace kernel's arguments stay in
    // fewer SGPRs.
    const double* r_b;
    __device__ __forceinline__ const double* c2_e() const { return r_b + nbr; }
    __device__ __forceinline__ const double* cos_a() const { return r_b + nbr + nbe; }
    __device__ __forceinline__ const double* sin_a() const { return r_b + nbr + nbe + nba; }
    __device__ __forceinline__ const double* e_b() const { return r_b + nbr + nbe + 2 * nba; }
    __device__ __forceinline__ const double* a_b() const { return r_b + nbr + 2 * nbe + 2 * nba; }
    __device__ __forceinline__ const uint8_t* e_flags() const {
        return reinterpret_cast<const uint8_t*>(r_b + nbr + 2 * nbe + 3 * nba);
    }
};

// Everything a crossing solve needs about one ray, in the trace's precision F.
template <typename F>
struct RayGeoT {
    F x0, x1, x2;     // start point
    F u0, u1, u2;     // direction normalised once here (r_torch, raytracer.py:281)
    F w0, w1, w2;     // normalised again (e_torch, raytracer.py:365; a_torch reuses it)
    F tc;             // dot(-x, u)                       (raytracer.py:288)
    F dd;             // sqrt(|x|^2 - tc^2)               (raytracer.py:289)
    F nx2;            // linalg.norm(x)**2                (raytracer.py:375)
    F wx;             // dot(w, x)                        (raytracer.py:374)
};
using RayGeo = RayGeoT<double>;

// Correctly rounded square root and single-rounding fused multiply-add in either precision
// (float: HIP's default correctly rounded sqrtf, as IEEE; torch CPU's float32 sqrt agrees with it
// on all but ~2e-5 of the crossings the f32 fixtures hold, by one ulp).
__device__ __forceinline__ double sq_rt(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ float sq_rt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmad(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fabs_(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float fabs_(float x) { return __builtin_fabsf(x); }

// torch.linalg.norm over the last axis of length 3: fused sum of squares, IEEE sqrt.
template <typename F>
__device__ __forceinline__ F vnorm(F a, F b, F c) {
    return sq_rt(fmad(c, c, fmad(b, b, a * a)));
}
// einsum '...j,...j->...' / '...c,...bc->...b': sequential, unfused.
template <typename F>
__device__ __forceinline__ F dot_seq(F a0, F a1, F a2, F b0, F b1, F b2) {
    F s = a0 * b0 + a1 * b1;
    return s + a2 * b2;
}

template <typename F>
__device__ __forceinline__ RayGeoT<F> make_ray(F x0, F x1, F x2, F d0, F d1, F d2) {
    RayGeoT<F> g;
    g.x0 = x0; g.x1 = x1; g.x2 = x2;
    F n1 = vnorm(d0, d1, d2);
    g.u0 = d0 / n1; g.u1 = d1 / n1; g.u2 = d2 / n1;
    F n2 = vnorm(g.u0, g.u1, g.u2);
    g.w0 = g.u0 / n2; g.w1 = g.u1 / n2; g.w2 = g.u2 / n2;
    g.tc = dot_seq(-x0, -x1, -x2, g.u0, g.u1, g.u2);
    F xx = dot_seq(x0, x1, x2, x0, x1, x2);
    g.dd = sq_rt(xx - g.tc * g.tc);
    F nx = vnorm(x0, x1, x2);
    g.nx2 = nx * nx;
    g.wx = dot_seq(g.w0, g.w1, g.w2, x0, x1, x2);
    return g;
}

// The per-family API: called on their own, e_torch normalises its input once
// (raytracer.py:365) and a_torch not at all (raytracer.py:471-552), so the cone/plane direction
// is u resp. the raw input, not the twice-normalised w that trace_indices hands them.
template <typename F>
__device__ __forceinline__ RayGeoT<F> make_ray_family(F x0, F x1, F x2, F d0, F d1, F d2,
                                                      int family) {
    RayGeoT<F> g = make_ray(x0, x1, x2, d0, d1, d2);
    if (family == 1) {
        g.w0 = g.u0; g.w1 = g.u1; g.w2 = g.u2;
    } else if (family == 2) {
        g.w0 = d0; g.w1 = d1; g.w2 = d2;
    }
    g.wx = dot_seq(g.w0, g.w1, g.w2, x0, x1, x2);
    return g;
}

// ---- spheres (r_torch, raytracer.py:288-323) ------------------------------------------------
// Region entered at distance t on sphere j: j - [u . p(t) < 0], j == nr -> -1 (outside).
template <typename F>
__device__ __forceinline__ int sphere_region(const RayGeoT<F>& g, F t, int j, int nr, int& neg) {
    F p0 = g.u0 * t + g.x0;
    F p1 = g.u1 * t + g.x1;
    F p2 = g.u2 * t + g.x2;
    neg = dot_seq(g.u0, g.u1, g.u2, p0, p1, p2) < F(0) ? 1 : 0;
    int reg = j - neg;
    return reg == nr ? -1 : reg;
}
// Both crossings of sphere j.  NaN distances (no crossing) become +inf.
template <typename F>
__device__ __forceinline__ void sphere_solve(const GridDev& G, const RayGeoT<F>& g, int j,
                                             F& t_in, int& reg_in, F& t_out, int& reg_out,
                                             int& neg_in, int& neg_out) {
    F R = (F)G.r_b[j];
    F t1c = sq_rt(R * R - g.dd * g.dd);
    t_in = g.tc - t1c;
    t_out = g.tc + t1c;
    reg_in = sphere_region(g, t_in, j, G.nr, neg_in);
    reg_out = sphere_region(g, t_out, j, G.nr, neg_out);
    if (__builtin_isnan(t_in)) t_in = (F)kInf;
    if (__builtin_isnan(t_out)) t_out = (F)kInf;
}

// False exactly when sphere_solve(j) yields no finite distance: R*R - dd*dd < 0 (or NaN) makes
// both square roots NaN, i.e. +inf crossings that nothing lists.  (The trace skips such shells.)
__device__ __forceinline__ bool sphere_may_cross(const GridDev& G, const RayGeo& g, int j) {
    const double R = G.r_b[j];
    return R * R - g.dd * g.dd >= 0.0;
}

// ---- cones (e_torch, raytracer.py:373-466) --------------------------------------------------
// The distance part of cone_root: +inf for a root on the opposite (shadow) nappe or NaN.
template <typename F>
__device__ __forceinline__ F cone_root_t(const GridDev& G, const RayGeoT<F>& g, int j, F t) {
    const F p2 = g.w2 * t + g.x2;
    const uint8_t f = G.e_flags()[j];
    const bool cone_up = (f & 1) != 0;
    const bool exempt = (f & 2) != 0;
    if (((p2 >= F(0)) != cone_up) && !exempt) t = (F)kInf;   // opposite (shadow) nappe
    if (__builtin_isnan(t)) t = (F)kInf;
    return t;
}
// Distance/region fix-up of one root t of cone j (region -2 = glancing, keep current region).
template <typename F>
__device__ __forceinline__ void cone_root(const GridDev& G, const RayGeoT<F>& g, int j, F& t,
                                          int& reg, int& neg) {
    F p0 = g.w0 * t + g.x0;
    F p1 = g.w1 * t + g.x1;
    F p2 = g.w2 * t + g.x2;
    // torch.cross(p, (-p1, p0, 0)) with torch CPU's fused pattern
    const F z = F(0);
    F n0 = fmad(p1, z, -(p2 * p0));
    F n1 = fmad(p2, -p1, -(p0 * z));
    F n2 = fmad(p0, p0, -(p1 * (-p1)));
    F prod = dot_seq(g.w0, g.w1, g.w2, n0, n1, n2);
    neg = prod > z ? 1 : 0;
    int r = j - neg;
    if (fabs_(prod) < (F)G.close_tol) r = -2;
    if (r == G.ne) r = -1;
    t = cone_root_t(G, g, j, t);
    reg = r;
}
// Cone j's quadratic coefficients with the reference's snapping (|a|, |delta| < close_tol -> 0;
// the comparison in F, as torch compares a tensor with a Python float in the tensor's dtype).
template <typename F>
struct ConeQuadT {
    F aa, bb, cc, delta;
};
using ConeQuad = ConeQuadT<double>;
template <typename F>
__device__ __forceinline__ ConeQuadT<F> cone_coeffs(const GridDev& G, const RayGeoT<F>& g, int j) {
    const F th = (F)G.close_tol;
    const F c2 = (F)G.c2_e()[j];
    F aa = g.w2 * g.w2 - c2;
    const F bb = F(2) * (g.w2 * g.x2 - g.wx * c2);
    const F cc = g.x2 * g.x2 - g.nx2 * c2;
    if (fabs_(aa) < th) aa = F(0);
    F delta = bb * bb - (F(4) * aa) * cc;
    if (fabs_(delta) < th) delta = F(0);
    return ConeQuadT<F>{aa, bb, cc, delta};
}
// False exactly when cone_solve(j) yields two +inf roots through a NaN square root: the
// (snapped) discriminant is negative or NaN and the ray is not parallel to a generator (the only
// override that makes a root finite).
template <typename F>
__device__ __forceinline__ bool cone_q_may_cross(const GridDev& G, const ConeQuadT<F>& q) {
    const F th = (F)G.close_tol;
    return q.delta >= F(0) || (fabs_(q.aa) < th && !(fabs_(q.bb) < th));
}
__device__ __forceinline__ bool cone_may_cross(const GridDev& G, const RayGeo& g, int j) {
    return cone_q_may_cross(G, cone_coeffs(G, g, j));
}
// The two roots of the quadratic with the reference's overrides, before the per-root fix-up
// (slot j "t1", slot nbe + j "t2").
template <typename F>
__device__ __forceinline__ void cone_roots_q(const GridDev& G, const ConeQuadT<F>& c, F& t1,
                                             F& t2) {
    const F th = (F)G.close_tol;
    const F aa = c.aa, bb = c.bb, cc = c.cc;
    F q = sq_rt(c.delta);
    t1 = (-bb + q) / (F(2) * aa);
    t2 = (-bb - q) / (F(2) * aa);
    if (fabs_(aa) < th && !(fabs_(bb) < th)) {  // ray parallel to a generator
        t1 = (-cc) / bb;
        t2 = (F)kInf;
    }
    if (aa == F(0) && bb == F(0) && cc == F(0)) {   // ray lies on the cone
        t1 = (F)kInf;
        t2 = (F)kInf;
    }
}
// Both roots of cone j: slot j ("t1") and slot nbe + j ("t2"), from its coefficients.
template <typename F>
__device__ __forceinline__ void cone_solve_q(const GridDev& G, const RayGeoT<F>& g, int j,
                                             const ConeQuadT<F>& q, F& ta, int& rega, F& tb,
                                             int& regb, int& nega, int& negb) {
    F t1, t2;
    cone_roots_q(G, q, t1, t2);
    cone_root(G, g, j, t1, rega, nega);
    cone_root(G, g, j, t2, regb, negb);
    ta = t1;
    tb = t2;
}
template <typename F>
__device__ __forceinline__ void cone_solve(const GridDev& G, const RayGeoT<F>& g, int j, F& ta,
                                           int& rega, F& tb, int& regb, int& nega, int& negb) {
    cone_solve_q(G, g, j, cone_coeffs(G, g, j), ta, rega, tb, regb, nega, negb);
}

// ---- azimuth half-planes (a_torch, raytracer.py:505-550) ------------------------------------
template <typename F>
__device__ __forceinline__ void plane_solve(const GridDev& G, const RayGeoT<F>& g, int j, F& t,
                                            int& reg, int& neg) {
    const F ca = (F)G.cos_a()[j], sa = (F)G.sin_a()[j];
    const F msa = -sa, z = F(0);
    // einsum '...bc,...jc->...b' against plane normal (-sin, cos, 0): fused chain
    F num = fmad(z, g.x2, fmad(ca, g.x1, msa * g.x0));
    F den = fmad(z, g.w2, fmad(ca, g.w1, msa * g.w0));
    F tt = (-num) / den;
    F cz = fmad(ca, g.w1, -(sa * g.w0));   // z of cross(plane, ray)
    if (fabs_(cz) <= (F)G.plane_par_tol) tt = (F)kInf;  // parallel to the plane
    int ng = cz < z ? 1 : 0;
    int r = j - ng;
    if (G.a_wrap) {
        // regions % na (raytracer.py:529, Python's modulo) for r = j - ng in [-1, na]: two
        // selects instead of an integer division by a runtime divisor
        if (r == G.na) r = 0;
        if (r < 0) r += G.na;
    } else if (r == G.na) {
        r = -1;
    }
    F p0 = tt * g.w0 + g.x0;
    F p1 = tt * g.w1 + g.x1;
    if (fmad(sa, p1, ca * p0) < z) tt = (F)kInf;   // back half of the plane
    if (__builtin_isnan(tt)) tt = (F)kInf;
    t = tt;
    reg = r;
    neg = ng;
}

}  // namespace sphrt
