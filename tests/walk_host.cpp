// Host build of the lane walk (csrc/walk.hpp) — TEST INFRASTRUCTURE ONLY.
//
// tests/test_walk_host.py compiles this with g++ -ffp-contract=off (the device build's
// arithmetic rules: no contraction, explicit fma, correctly rounded sqrt and division) against a
// stand-in hip_runtime.h, and checks every walked ray against the C oracle.  The same source
// lines run in walk_kernel on the GPU; this is their CPU replay, not a second implementation.
#define __device__
#define __forceinline__ inline
#include "walk.hpp"

using namespace sphrt;

// tables: the block sphrt_plan_pack_tables packs (r_b | cos^2 e | cos a | sin a | e_b | a_b | flags)
extern "C" int walk_host(int nr, int ne, int na, const double* tables, int a_wrap, double close_tol,
                         double plane_par_tol, const double* xs, const double* rays,
                         const int32_t* starts, int64_t n, int32_t* status, int32_t* counts,
                         int32_t* vox, double* len, int64_t cap) {
    GridDev G;
    G.nr = nr; G.ne = ne; G.na = na;
    G.nbr = nr + 1; G.nbe = ne + 1; G.nba = na + 1;
    G.K = 2 * G.nbr + 2 * G.nbe + G.nba + 1;
    G.a_wrap = a_wrap;
    G.close_tol = close_tol;
    G.plane_par_tol = plane_par_tol;
    G.r_b = tables;
    G.r_outer = tables[nr];
    int e_asc = 1, a_asc = 1;
    for (int j = 1; j < G.nbe; ++j) e_asc &= G.e_b()[j] > G.e_b()[j - 1] ? 1 : 0;
    for (int j = 1; j < G.nba; ++j) a_asc &= G.a_b()[j] > G.a_b()[j - 1] ? 1 : 0;
    G.e_asc = e_asc;
    G.a_asc = a_asc;
    for (int64_t i = 0; i < n; ++i) {
        const double* x = xs + 3 * i;
        const double* d = rays + 3 * i;
        const int s[3] = {starts[3 * i], starts[3 * i + 1], starts[3 * i + 2]};
        const RayGeo g = make_ray(x[0], x[1], x[2], d[0], d[1], d[2]);
        const double t1c_o = __builtin_sqrt(G.r_outer * G.r_outer - g.dd * g.dd);
        const bool start_r_ok = s[0] >= 0 && s[0] < G.nr;
        const bool hit = !(!start_r_ok && __builtin_isnan(t1c_o));
        counts[i] = 0;
        if (!hit || !walk_eligible(G, g, t1c_o, start_r_ok)) {
            status[i] = -1;
            continue;
        }
        int64_t k = 0;
        status[i] = walk_ray(G, g, s, [&](int vx, double l) {
            if (k < cap) {
                vox[i * cap + k] = vx;
                len[i * cap + k] = l;
            }
            ++k;
        });
        counts[i] = (int32_t)k;
    }
    return 0;
}
