// walk.hpp — the crossings of one ray in increasing distance, one lane per ray, without a list.
//
// Opt-in (SPHRT_WALK=1): exact, but slower than the list trace on MI355X (trace.hip
// walk_enabled).
// Along a line every boundary family crosses in an order known in advance (SURVEY §7 "merge"):
//   spheres   the near roots tc - t1c(j) for the outermost shell inwards, then the far roots
//             tc + t1c(j) outwards (t1c grows with R, and IEEE rounding keeps that order);
//   cones     the elevation along a line has at most one extremum t* (the derivative of its cosine
//             has a linear numerator), so the cone crossings of [0, t*] come in cone-angle order
//             one way and those of (t*, inf) the other way: two runs;
//   planes    the azimuth is monotone along a line that misses the z axis (d phi / dt = L_z / rho^2,
//             L_z constant), so the half-planes come in cyclic azimuth order from the start's.
// Each run yields its next crossing on demand (one boundary solved per step, solve.hpp, the same
// arithmetic as the list trace), and a four-way merge by distance walks the ray.  Whatever the
// order argument predicts, the walk checks it: a run whose next crossing is nearer than its last
// one makes the caller hand the ray to the sorting (list) trace instead, so a result is only ever
// produced from a verified order.  Runs end early only where the geometry rules out further
// crossings: past the sphere exit, and a plane run at the first half-plane past a crossed one that
// is not crossed (the azimuth's arc along the line has ended).  The cone runs cover index ranges
// found by solving every cone (see ConeRun).
#pragma once
#include "solve.hpp"

namespace sphrt {

// one crossing: distance, candidate index (the reference's concatenation order), region
struct WalkHead {
    double t;
    int cand;
    int reg;
};

__device__ __forceinline__ bool head_less(const WalkHead& a, const WalkHead& b) {
    return a.t < b.t || (a.t == b.t && a.cand < b.cand);
}

// Entries of the ascending b[0, n) that are < v.
__device__ __forceinline__ int count_lt(const double* b, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (b[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// Entries of the ascending b[0, n) that are <= v.
__device__ __forceinline__ int count_le(const double* b, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (b[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ---- spheres: near roots j = nr .. j_lo, then far roots j = j_lo .. nr ------------------------
struct SphereRun {
    int j;
    int phase;          // 0 near, 1 first far root (j_lo), 2 far, 3 done
    double t_lo_in;     // near root of the innermost crossed shell and its region (a tangent
    int r_lo_in;        // shell's identical far root is not listed, as in the list trace)
};

__device__ __forceinline__ void sphere_next(const GridDev& G, const RayGeo& g, SphereRun& s,
                                            WalkHead& h) {
    if (s.phase == 0) {
        if (s.j >= 0 && sphere_may_cross(G, g, s.j)) {
            const double R = G.r_b[s.j];
            const double t1c = __builtin_sqrt(R * R - g.dd * g.dd);
            int neg;
            h.t = g.tc - t1c;
            h.reg = sphere_region(g, h.t, s.j, G.nr, neg);
            h.cand = s.j;
            s.t_lo_in = h.t;
            s.r_lo_in = h.reg;
            --s.j;
            return;
        }
        s.phase = 1;
        ++s.j;
    }
    while (s.phase < 3 && s.j < G.nbr) {
        const double R = G.r_b[s.j];
        const double t1c = __builtin_sqrt(R * R - g.dd * g.dd);
        int neg;
        h.t = g.tc + t1c;
        h.reg = sphere_region(g, h.t, s.j, G.nr, neg);
        h.cand = G.nbr + s.j;
        ++s.j;
        const bool dup = s.phase == 1 && h.t == s.t_lo_in && h.reg == s.r_lo_in;
        s.phase = 2;
        if (!dup) return;
    }
    s.phase = 3;
    h.t = kInf;
    h.cand = INT32_MAX;
    h.reg = 0;
}

// ---- cones: one stretch of the elevation's monotone pieces ---------------------------------
// Every cone is solved up front, all lanes in step, for its roots' distances only
// (cone_quadratic + cone_root_t: the same operations as cone_solve); each stretch run then covers
// exactly the index range of the cones with a root on its side of t*, in its direction.  No cone
// is skipped on geometric grounds — the reference's snapping (|discriminant| < 1e-5 -> 0) gives
// double roots to cones the line does not reach, on a line near the origin to nearly all of
// them (their discriminant is O(dd^2)) — and a run ends exactly at its range's last cone instead
// of searching on, each lane at its own time, through cones that have nothing left for it.
// Where the snapped roots break a stretch's order, the order check sends the ray to the list
// trace.
struct ConeRun {
    int j, dir, end;      // next cone, step (+1: angles ascending), last cone of the range
    int second;           // 0: the stretch [0, split]; 1: (split, inf)
    int done;
    double split;         // t* (+inf: one stretch)
    WalkHead pend;        // the second root of the last cone, when both fall in the stretch
    int has_pend;
};

__device__ __forceinline__ bool cone_in(const ConeRun& c, double t) {
    return __builtin_isfinite(t) && !(t < 0.0) && (c.second ? t > c.split : !(t > c.split));
}

__device__ __forceinline__ void cone_next(const GridDev& G, const RayGeo& g, ConeRun& c,
                                          WalkHead& h) {
    if (c.has_pend) {
        h = c.pend;
        c.has_pend = 0;
        return;
    }
    const int ce0 = 2 * G.nbr;
    while (!c.done) {
        const int j = c.j;
        if (c.dir > 0 ? j > c.end : j < c.end) break;
        c.j = j + c.dir;
        double ta, tb;
        int ra, rb, na_, nb_;
        cone_solve(G, g, j, ta, ra, tb, rb, na_, nb_);
        const bool va = cone_in(c, ta);
        const bool vb = cone_in(c, tb) && !(tb == ta && rb == ra);   // (as the list trace)
        if (!va && !vb) continue;
        const WalkHead a{ta, ce0 + j, ra}, b{tb, ce0 + G.nbe + j, rb};
        if (va && vb) {
            const bool b_first = head_less(b, a);
            h = b_first ? b : a;
            c.pend = b_first ? a : b;
            c.has_pend = 1;
        } else {
            h = va ? a : b;
        }
        return;
    }
    c.done = 1;
    h.t = kInf;
    h.cand = INT32_MAX;
    h.reg = 0;
}

// ---- azimuth half-planes in cyclic order ---------------------------------------------------
struct PlaneRun {
    int j, dir, steps, found, done;
};

__device__ __forceinline__ void plane_next(const GridDev& G, const RayGeo& g, PlaneRun& p,
                                           WalkHead& h) {
    const int ca0 = 2 * G.nbr + 2 * G.nbe;
    while (!p.done && p.steps < G.nba) {
        double t;
        int r, ng;
        plane_solve(G, g, p.j, t, r, ng);
        const int cand = ca0 + p.j;
        p.j += p.dir;
        if (p.j < 0) p.j += G.nba;
        if (p.j >= G.nba) p.j -= G.nba;
        ++p.steps;
        if (__builtin_isfinite(t) && !(t < 0.0)) {
            p.found = 1;
            h.t = t;
            h.cand = cand;
            h.reg = r;
            return;
        }
        if (p.found) break;
    }
    p.done = 1;
    h.t = kInf;
    h.cand = INT32_MAX;
    h.reg = 0;
}

// Can the walk take this ray?  It starts outside the outer sphere (so nothing behind the start
// is ever integrated: the start voxel is invalid) and enters it later; the ray's line keeps
// clear of the origin and of the z axis (dd, |L_z| above 1e-7 of the start's radius: the cone
// and plane orders need a line that does not pass through either); the boundary tables are
// strictly ascending (the runs step through them by index).
__device__ __forceinline__ bool walk_eligible(const GridDev& G, const RayGeo& g, double t1c_outer,
                                              bool start_r_ok) {
    if (!G.e_asc || !G.a_asc || start_r_ok) return false;
    if (!(g.tc - t1c_outer > 0.0)) return false;
    const double sc = __builtin_sqrt(g.nx2);
    const double lz = g.x0 * g.w1 - g.x1 * g.w0;
    return g.dd > 1e-7 * sc && __builtin_fabs(lz) > 1e-7 * sc;
}

// The four runs of a walk-eligible ray.  Sphere and plane runs start at their first possible
// crossing; the cone runs cover the index range of their stretch's cones.
__device__ __forceinline__ void walk_setup(const GridDev& G, const RayGeo& g, SphereRun& s,
                                           ConeRun& c1, ConeRun& c2, PlaneRun& p) {
    s.j = G.nbr - 1;
    s.phase = 0;
    s.t_lo_in = kInf;
    s.r_lo_in = 0;
    // elevation: d cos(theta) / dt is proportional to gd0 + slope * t (segment_bound's t*)
    const double gd0 = g.w2 * g.nx2 - g.x2 * g.wx;
    const double slope = g.w2 * g.wx - g.x2;
    double ts = -gd0 / slope;
    if (!(ts > 0.0) || !__builtin_isfinite(ts)) ts = kInf;
    const double sgn = gd0 != 0.0 ? gd0 : slope;    // cos(theta) rising -> theta falling
    const int dir1 = sgn > 0.0 ? -1 : 1;
    c1 = ConeRun{};
    c1.dir = dir1;
    c1.second = 0;
    c1.split = ts;
    c2 = ConeRun{};
    c2.dir = -dir1;
    c2.second = 1;
    c2.split = ts;
    // the index range of each stretch's cones (distances only, every lane in step)
    int lo1 = G.nbe, hi1 = -1, lo2 = G.nbe, hi2 = -1;
    for (int j = 0; j < G.nbe; ++j) {
        if (!cone_may_cross(G, g, j)) continue;
        double t1, t2;
        cone_quadratic(G, g, j, t1, t2);
        t1 = cone_root_t(G, g, j, t1);
        t2 = cone_root_t(G, g, j, t2);
        const bool in1 = cone_in(c1, t1) || cone_in(c1, t2);
        const bool in2 = cone_in(c2, t1) || cone_in(c2, t2);
        if (in1) {
            lo1 = j < lo1 ? j : lo1;
            hi1 = j;
        }
        if (in2) {
            lo2 = j < lo2 ? j : lo2;
            hi2 = j;
        }
    }
    c1.j = dir1 > 0 ? lo1 : hi1;
    c1.end = dir1 > 0 ? hi1 : lo1;
    c1.done = lo1 > hi1;
    c2.j = dir1 > 0 ? hi2 : lo2;
    c2.end = dir1 > 0 ? lo2 : hi2;
    c2.done = lo2 > hi2;
    // azimuth: increasing when L_z > 0; the start's azimuth brought into the table's range
    const double lz = g.x0 * g.w1 - g.x1 * g.w0;
    const double* ab = G.a_b();
    const int nba = G.nba;
    // The run starts at the first half-plane at or past the start's azimuth (within 1e-9 rad
    // behind it: atan2's rounding) in the sweep's direction and steps cyclically, which is the
    // sweep's own order on a full circle and across a partial table's gap alike.
    double ph = atan2(g.x1, g.x0);
    if (ph < ab[0]) ph += 6.283185307179586;
    p.dir = lz > 0.0 ? 1 : -1;
    int j;
    if (p.dir > 0) {
        j = count_lt(ab, nba, ph - 1e-9);           // first a_b >= ph - eps
        if (j == nba) j = 0;
    } else {
        j = count_le(ab, nba, ph + 1e-9) - 1;       // last a_b <= ph + eps
        if (j < 0) j = nba - 1;
    }
    p.j = j;
    p.steps = 0;
    p.found = 0;
    p.done = 0;
}

// Walk one walk-eligible ray (start voxel s): emit(voxel, length) for every non-zero in-grid
// segment in order, exactly the segments of trace_one's list for the ray.  The merged sequence
// replays trace_one's rules: crossings before the outer sphere's entry t_lo only update the e / a
// rows (the start lies outside, its r row is -1 until the entry), the crossings from t_lo to the
// exit t_hi are the list, and each segment between consecutive list entries takes the rows'
// values after the first.  Returns 0, or 1 when exactly equal distances of two crossings write
// different values into one row (the start entry at t = 0 included: ambiguous_ties'
// condition, the reference's introsort order decides), or 2 when a run is out of order; after a
// non-zero return the emitted segments are void.
template <class Emit>
__device__ __forceinline__ int walk_ray(const GridDev& G, const RayGeo& g, const int* s,
                                        Emit&& emit) {
    constexpr int kNoVal = 0x7fffffff;
    const double t1c_o = __builtin_sqrt(G.r_outer * G.r_outer - g.dd * g.dd);
    const double t_lo = g.tc - t1c_o, t_hi = g.tc + t1c_o;
    // crossings up to this far past the exit are still merged, so their runs' order is checked
    const double margin = 1e-9 * (__builtin_fabs(t_hi) + 1.0);
    SphereRun sr;
    ConeRun c1, c2;
    PlaneRun pr;
    walk_setup(G, g, sr, c1, c2, pr);
    WalkHead hs, h1, h2, hp, hq;            // run heads (named: no indexed array in scratch)
    sphere_next(G, g, sr, hs);
    cone_next(G, g, c1, h1);
    cone_next(G, g, c2, h2);
    // the plane run through a two-entry window: the table's first and last half-planes of a full
    // circle (-pi and pi, or 0 and 2 pi) are one plane whose two crossings differ in the last
    // bits either way; the window yields the nearer first
    plane_next(G, g, pr, hp);
    plane_next(G, g, pr, hq);
    if (head_less(hq, hp)) {
        const WalkHead w = hp;
        hp = hq;
        hq = w;
    }
    int cr = s[0], ce = s[1], ca = s[2];
    double gt = 0.0;                        // the current group of equal distances: the start
    int g0 = s[0], g1 = s[1], g2 = s[2];    // entry's, at t = 0, to begin with
    bool listed = false;
    double tp = 0.0;
    int amb = 0;                            // rows whose last pre-entry group clashed (bits)
    int status = 0;                         // 1: tie (exact kernel), 2: out of order (list trace)
    for (;;) {
        // the nearest head by (distance, candidate)
        int f = 0;
        WalkHead e = hs;
        if (head_less(h1, e)) { e = h1; f = 1; }
        if (head_less(h2, e)) { e = h2; f = 2; }
        if (head_less(hp, e)) { e = hp; f = 3; }
        if (!(e.t <= t_hi + margin)) break;
        double tn;
        if (f == 0) { sphere_next(G, g, sr, hs); tn = hs.t; }
#ifdef SPHRT_WALK_CONE_SHARED
        else if (f != 3) {
            // (A/B variant) both stretches through one call: lanes advancing different stretches
            // share the cone code instead of running it twice under divergence (220 VGPRs)
            ConeRun c = f == 1 ? c1 : c2;
            WalkHead hh;
            cone_next(G, g, c, hh);
            if (f == 1) { c1 = c; h1 = hh; }
            else { c2 = c; h2 = hh; }
            tn = hh.t;
        }
#else
        else if (f == 1) { cone_next(G, g, c1, h1); tn = h1.t; }
        else if (f == 2) { cone_next(G, g, c2, h2); tn = h2.t; }
#endif
        else {
            hp = hq;
            plane_next(G, g, pr, hq);
            if (head_less(hq, hp)) {
                const WalkHead w = hp;
                hp = hq;
                hq = w;
            }
            tn = hp.t;
        }
        if (tn < e.t) {                     // the run's order argument failed for this ray
#ifdef SPHRT_WALK_DIAG
            status = 20 + f;
#else
            status = 2;
#endif
            break;
        }
        if (e.t > t_hi) continue;           // (past the list; kept only for the order check)
        const int row = f == 0 ? 0 : (f == 3 ? 2 : (e.reg == -2 ? -1 : 1));
        if (e.t != gt) {
            gt = e.t;
            g0 = g1 = g2 = kNoVal;
        }
        if (row >= 0) {
            const int gv = row == 0 ? g0 : (row == 1 ? g1 : g2);
            const bool clash = gv != kNoVal && gv != e.reg;
            if (clash && e.t >= t_lo) {
                status = 1;
                break;
            }
            // before the entry a clash only matters if no later group rewrites the row before
            // t_lo (trace_one's entry_row keeps the last pre-entry group per row)
            const int bit = 1 << row;
            if (gv == kNoVal) amb &= ~bit;
            if (clash) amb |= bit;
            if (row == 0) g0 = e.reg;
            else if (row == 1) g1 = e.reg;
            else g2 = e.reg;
        }
        if (e.t >= t_lo) {
            if (amb) {                      // the rows entering the sphere are tie-ambiguous
                status = 1;
                break;
            }
            if (listed) {
                const double len = e.t - tp;
                if (len > 0.0 && __builtin_isfinite(len) && cr >= 0 && cr < G.nr && ce >= 0 &&
                    ce < G.ne && ca >= 0 && ca < G.na) {
                    emit((cr * G.ne + ce) * G.na + ca, len);
                }
            }
            listed = true;
            tp = e.t;
        }
        if (row == 0) cr = e.reg;
        else if (row == 1) ce = e.reg;
        else if (row == 2) ca = e.reg;
    }
    return status;
}

}  // namespace sphrt
