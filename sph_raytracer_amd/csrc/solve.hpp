// solve.hpp — per-ray boundary-crossing solves on gfx950, FP64.
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

// Everything a crossing solve needs about one ray.
struct RayGeo {
    double x0, x1, x2;     // start point
    double u0, u1, u2;     // direction normalised once here (r_torch, raytracer.py:281)
    double w0, w1, w2;     // normalised again (e_torch, raytracer.py:365; a_torch reuses it)
    double tc;             // dot(-x, u)                       (raytracer.py:288)
    double dd;             // sqrt(|x|^2 - tc^2)               (raytracer.py:289)
    double nx2;            // linalg.norm(x)**2                (raytracer.py:375)
    double wx;             // dot(w, x)                        (raytracer.py:374)
};

// torch.linalg.norm over the last axis of length 3: fused sum of squares, IEEE sqrt.
__device__ __forceinline__ double vnorm(double a, double b, double c) {
    return __builtin_sqrt(__builtin_fma(c, c, __builtin_fma(b, b, a * a)));
}
// einsum '...j,...j->...' / '...c,...bc->...b': sequential, unfused.
__device__ __forceinline__ double dot_seq(double a0, double a1, double a2,
                                          double b0, double b1, double b2) {
    double s = a0 * b0 + a1 * b1;
    return s + a2 * b2;
}

__device__ __forceinline__ RayGeo make_ray(double x0, double x1, double x2,
                                           double d0, double d1, double d2) {
    RayGeo g;
    g.x0 = x0; g.x1 = x1; g.x2 = x2;
    double n1 = vnorm(d0, d1, d2);
    g.u0 = d0 / n1; g.u1 = d1 / n1; g.u2 = d2 / n1;
    double n2 = vnorm(g.u0, g.u1, g.u2);
    g.w0 = g.u0 / n2; g.w1 = g.u1 / n2; g.w2 = g.u2 / n2;
    g.tc = dot_seq(-x0, -x1, -x2, g.u0, g.u1, g.u2);
    double xx = dot_seq(x0, x1, x2, x0, x1, x2);
    g.dd = __builtin_sqrt(xx - g.tc * g.tc);
    double nx = vnorm(x0, x1, x2);
    g.nx2 = nx * nx;
    g.wx = dot_seq(g.w0, g.w1, g.w2, x0, x1, x2);
    return g;
}

// The per-family API: called on their own, e_torch normalises its input once
// (raytracer.py:365) and a_torch not at all (raytracer.py:471-552), so the cone/plane direction
// is u resp. the raw input, not the twice-normalised w that trace_indices hands them.
__device__ __forceinline__ RayGeo make_ray_family(double x0, double x1, double x2, double d0,
                                                  double d1, double d2, int family) {
    RayGeo g = make_ray(x0, x1, x2, d0, d1, d2);
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
__device__ __forceinline__ int sphere_region(const RayGeo& g, double t, int j, int nr,
                                             int& neg) {
    double p0 = g.u0 * t + g.x0;
    double p1 = g.u1 * t + g.x1;
    double p2 = g.u2 * t + g.x2;
    neg = dot_seq(g.u0, g.u1, g.u2, p0, p1, p2) < 0.0 ? 1 : 0;
    int reg = j - neg;
    return reg == nr ? -1 : reg;
}
// Both crossings of sphere j.  NaN distances (no crossing) become +inf.
__device__ __forceinline__ void sphere_solve(const GridDev& G, const RayGeo& g, int j,
                                             double& t_in, int& reg_in,
                                             double& t_out, int& reg_out,
                                             int& neg_in, int& neg_out) {
    double R = G.r_b[j];
    double t1c = __builtin_sqrt(R * R - g.dd * g.dd);
    t_in = g.tc - t1c;
    t_out = g.tc + t1c;
    reg_in = sphere_region(g, t_in, j, G.nr, neg_in);
    reg_out = sphere_region(g, t_out, j, G.nr, neg_out);
    if (__builtin_isnan(t_in)) t_in = kInf;
    if (__builtin_isnan(t_out)) t_out = kInf;
}

// False exactly when sphere_solve(j) yields no finite distance: R*R - dd*dd < 0 (or NaN) makes
// both square roots NaN, i.e. +inf crossings that nothing lists.  (The trace skips such shells.)
__device__ __forceinline__ bool sphere_may_cross(const GridDev& G, const RayGeo& g, int j) {
    const double R = G.r_b[j];
    return R * R - g.dd * g.dd >= 0.0;
}

// ---- cones (e_torch, raytracer.py:373-466) --------------------------------------------------
// False exactly when cone_solve(j) yields two +inf roots through a NaN square root: the
// (snapped) discriminant is negative or NaN and the ray is not parallel to a generator (the only
// override that makes a root finite).  The coefficients repeat cone_solve's operations.
__device__ __forceinline__ bool cone_may_cross(const GridDev& G, const RayGeo& g, int j) {
    const double th = G.close_tol;
    const double c2 = G.c2_e()[j];
    double aa = g.w2 * g.w2 - c2;
    const double bb = 2.0 * (g.w2 * g.x2 - g.wx * c2);
    const double cc = g.x2 * g.x2 - g.nx2 * c2;
    if (__builtin_fabs(aa) < th) aa = 0.0;
    double delta = bb * bb - (4.0 * aa) * cc;
    if (__builtin_fabs(delta) < th) delta = 0.0;
    const bool parallel = __builtin_fabs(aa) < th && !(__builtin_fabs(bb) < th);
    return delta >= 0.0 || parallel;
}
// The distance part of cone_root: +inf for a root on the opposite (shadow) nappe or NaN.
__device__ __forceinline__ double cone_root_t(const GridDev& G, const RayGeo& g, int j, double t) {
    const double p2 = g.w2 * t + g.x2;
    const uint8_t f = G.e_flags()[j];
    const bool cone_up = (f & 1) != 0;
    const bool exempt = (f & 2) != 0;
    if (((p2 >= 0.0) != cone_up) && !exempt) t = kInf;   // opposite (shadow) nappe
    if (__builtin_isnan(t)) t = kInf;
    return t;
}
// Distance/region fix-up of one root t of cone j (region -2 = glancing, keep current region).
__device__ __forceinline__ void cone_root(const GridDev& G, const RayGeo& g, int j,
                                          double& t, int& reg, int& neg) {
    double p0 = g.w0 * t + g.x0;
    double p1 = g.w1 * t + g.x1;
    double p2 = g.w2 * t + g.x2;
    // torch.cross(p, (-p1, p0, 0)) with torch CPU's fused pattern
    double n0 = __builtin_fma(p1, 0.0, -(p2 * p0));
    double n1 = __builtin_fma(p2, -p1, -(p0 * 0.0));
    double n2 = __builtin_fma(p0, p0, -(p1 * (-p1)));
    double prod = dot_seq(g.w0, g.w1, g.w2, n0, n1, n2);
    neg = prod > 0.0 ? 1 : 0;
    int r = j - neg;
    if (__builtin_fabs(prod) < G.close_tol) r = -2;
    if (r == G.ne) r = -1;
    t = cone_root_t(G, g, j, t);
    reg = r;
}
// Cone j's quadratic coefficients with the reference's snapping (|a|, |delta| < close_tol -> 0).
struct ConeQuad {
    double aa, bb, cc, delta;
};
__device__ __forceinline__ ConeQuad cone_coeffs(const GridDev& G, const RayGeo& g, int j) {
    const double th = G.close_tol;
    const double c2 = G.c2_e()[j];
    double aa = g.w2 * g.w2 - c2;
    const double bb = 2.0 * (g.w2 * g.x2 - g.wx * c2);
    const double cc = g.x2 * g.x2 - g.nx2 * c2;
    if (__builtin_fabs(aa) < th) aa = 0.0;
    double delta = bb * bb - (4.0 * aa) * cc;
    if (__builtin_fabs(delta) < th) delta = 0.0;
    return ConeQuad{aa, bb, cc, delta};
}
// cone_may_cross on coefficients already computed (the trace solves a chunk from the same ones)
__device__ __forceinline__ bool cone_q_may_cross(const GridDev& G, const ConeQuad& q) {
    const double th = G.close_tol;
    return q.delta >= 0.0 || (__builtin_fabs(q.aa) < th && !(__builtin_fabs(q.bb) < th));
}
// The two roots of the quadratic with the reference's overrides, before the per-root fix-up
// (slot j "t1", slot nbe + j "t2").
__device__ __forceinline__ void cone_roots_q(const GridDev& G, const ConeQuad& c, double& t1,
                                             double& t2) {
    const double th = G.close_tol;
    const double aa = c.aa, bb = c.bb, cc = c.cc;
    double q = __builtin_sqrt(c.delta);
    t1 = (-bb + q) / (2.0 * aa);
    t2 = (-bb - q) / (2.0 * aa);
    if (__builtin_fabs(aa) < th && !(__builtin_fabs(bb) < th)) {  // ray parallel to a generator
        t1 = (-cc) / bb;
        t2 = kInf;
    }
    if (aa == 0.0 && bb == 0.0 && cc == 0.0) {                     // ray lies on the cone
        t1 = kInf;
        t2 = kInf;
    }
}
__device__ __forceinline__ void cone_quadratic(const GridDev& G, const RayGeo& g, int j,
                                               double& t1, double& t2) {
    cone_roots_q(G, cone_coeffs(G, g, j), t1, t2);
}
// Both roots of cone j: slot j ("t1") and slot nbe + j ("t2"), from its coefficients.
__device__ __forceinline__ void cone_solve_q(const GridDev& G, const RayGeo& g, int j,
                                             const ConeQuad& q, double& ta, int& rega,
                                             double& tb, int& regb, int& nega, int& negb) {
    double t1, t2;
    cone_roots_q(G, q, t1, t2);
    cone_root(G, g, j, t1, rega, nega);
    cone_root(G, g, j, t2, regb, negb);
    ta = t1;
    tb = t2;
}
__device__ __forceinline__ void cone_solve(const GridDev& G, const RayGeo& g, int j,
                                           double& ta, int& rega, double& tb, int& regb,
                                           int& nega, int& negb) {
    cone_solve_q(G, g, j, cone_coeffs(G, g, j), ta, rega, tb, regb, nega, negb);
}

// ---- azimuth half-planes (a_torch, raytracer.py:505-550) ------------------------------------
__device__ __forceinline__ void plane_solve(const GridDev& G, const RayGeo& g, int j,
                                            double& t, int& reg, int& neg) {
    double ca = G.cos_a()[j], sa = G.sin_a()[j];
    double msa = -sa;
    // einsum '...bc,...jc->...b' against plane normal (-sin, cos, 0): fused chain
    double num = __builtin_fma(0.0, g.x2, __builtin_fma(ca, g.x1, msa * g.x0));
    double den = __builtin_fma(0.0, g.w2, __builtin_fma(ca, g.w1, msa * g.w0));
    double tt = (-num) / den;
    double cz = __builtin_fma(ca, g.w1, -(sa * g.w0));   // z of cross(plane, ray)
    if (__builtin_fabs(cz) <= G.plane_par_tol) tt = kInf;  // parallel to the plane
    int ng = cz < 0.0 ? 1 : 0;
    int r = j - ng;
    if (G.a_wrap) {
        r %= G.na;
        if (r < 0) r += G.na;
    } else if (r == G.na) {
        r = -1;
    }
    double p0 = tt * g.w0 + g.x0;
    double p1 = tt * g.w1 + g.x1;
    if (__builtin_fma(sa, p1, ca * p0) < 0.0) tt = kInf;   // back half of the plane
    if (__builtin_isnan(tt)) tt = kInf;
    t = tt;
    reg = r;
    neg = ng;
}

}  // namespace sphrt
