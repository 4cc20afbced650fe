// rays.hip — on-device cone-beam ray directions.
//
// Replaces ConeRectGeom.rays (geometry.py:493-508) and ConeCircGeom.rays (geometry.py:570-582)
// for the trace: the per-pixel directions are generated where they are used instead of being
// computed by torch on the host and copied over PCIe (24 B per ray).  Bit-identical to the torch
// CPU expressions: the per-axis values that need transcendental functions (tan of the half field
// of view through linspace, cos/sin of the polar angle) are computed on the host by the same torch
// calls and passed in; the per-pixel arithmetic is restated operation by operation in IEEE double
// (device code is compiled with -ffp-contract=off, fused multiply-adds only where written):
//   rect: d = (look + right * a_i) + up * b_j
//   circ: d = (look + (r_i * cos_j) * right) + (r_i * sin_j) * up, the products r_i * cos_j in
//         the host tensors' precision (float32 by default: torch.linspace of tensor endpoints)
//   ray  = d / sqrt(fma(d2, d2, fma(d1, d1, d0 * d0)))        (torch.linalg.norm, last axis of 3)
#include "common.hpp"

namespace sphrt {

// tv > 0: rays in tiles across views — row i of the (h, w / tw, n_views / tv, tv, tw) layout
// holds pixel (a, cb * tw + cc) of view vg * tv + vi (sphrt_rays_cone_tiled).
__global__ __launch_bounds__(256) void cone_rays_kernel(int64_t n_views, int64_t h, int64_t w,
                                                        int circ, const double* __restrict__ frame,
                                                        const double* __restrict__ row,
                                                        const double* __restrict__ col,
                                                        double* __restrict__ rays,
                                                        const int64_t* __restrict__ order,
                                                        int32_t* __restrict__ ray_id, int64_t tv,
                                                        int64_t tw) {
    const int64_t n = n_views * h * w;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t view, pix;
        if (tv > 0) {
            const int64_t cc = i % tw, vi = (i / tw) % tv, q = i / (tw * tv);
            const int64_t vg = q % (n_views / tv), r = q / (n_views / tv);
            const int64_t cb = r % (w / tw), a = r / (w / tw);
            view = vg * tv + vi;
            pix = a * w + cb * tw + cc;
        } else {
            view = i / (h * w);
            const int64_t slot = i - view * h * w;
            pix = order ? order[slot] : slot;            // the pixel this trace row holds
        }
        if (ray_id) ray_id[i] = (int32_t)(view * h * w + pix);
        const int64_t a = pix / w, b = pix - a * w;
        const double* f = frame + 9 * view;          // look, right, up
        double p, q;                                 // coefficients of right and up
        if (circ == 2) {                             // r, cos, sin are float32 tensors on the host:
            const float r = (float)row[view * h + a];  // their product is rounded to float32
            p = (double)(r * (float)col[view * 2 * w + b]);
            q = (double)(r * (float)col[view * 2 * w + w + b]);
        } else if (circ) {
            const double r = row[view * h + a];
            p = r * col[view * 2 * w + b];           // r_i * cos_j
            q = r * col[view * 2 * w + w + b];       // r_i * sin_j
        } else {
            p = row[view * h + a];
            q = col[view * w + b];
        }
        double d[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double s = f[c] + f[3 + c] * p;
            d[c] = s + f[6 + c] * q;
        }
        const double nrm = __builtin_sqrt(__builtin_fma(d[2], d[2], __builtin_fma(d[1], d[1], d[0] * d[0])));
        double* o = rays + 3 * i;
        o[0] = d[0] / nrm;
        o[1] = d[1] / nrm;
        o[2] = d[2] / nrm;
    }
}

}  // namespace sphrt

using namespace sphrt;

static int rays_cone(int64_t n_views, int64_t h, int64_t w, int circ, const double* frame,
                     const double* row, const double* col, double* rays, const int64_t* order,
                     int32_t* ray_id, void* stream, int64_t tv = 0, int64_t tw = 0) {
    if (n_views < 0 || h < 0 || w < 0) return fail("bad detector shape");
    if (!frame || !row || !col || !rays) return fail("null pointer");
    const int64_t n = n_views * h * w;
    if (n == 0) return 0;
    if (ray_id && n > 0x7fffffff) return fail("too many rays for int32 ray ids");
    StreamGuard guard(stream);
    const int64_t blocks = (n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536;
    hipLaunchKernelGGL(cone_rays_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       n_views, h, w, circ, frame, row, col, rays, order, ray_id, tv, tw);
    return check_launch("cone_rays_kernel");
}

extern "C" int sphrt_rays_cone(int64_t n_views, int64_t h, int64_t w, int circ,
                               const double* frame, const double* row, const double* col,
                               double* rays, void* stream) {
    return rays_cone(n_views, h, w, circ, frame, row, col, rays, nullptr, nullptr, stream);
}

// The same rays in a per-view trace order: row k of view v holds pixel order[k] (a permutation
// of the h * w pixels, on the device), ray_id[v h w + k] = v h w + order[k].  One launch instead
// of generating, gathering (index_select) and numbering the rays in four (C5 Operator: the ray
// ids' torch arithmetic and the gather with their host gaps).
extern "C" int sphrt_rays_cone_ordered(int64_t n_views, int64_t h, int64_t w, int circ,
                                       const double* frame, const double* row, const double* col,
                                       const int64_t* order, double* rays, int32_t* ray_id,
                                       void* stream) {
    if (!order || !ray_id) return fail("null pointer");
    return rays_cone(n_views, h, w, circ, frame, row, col, rays, order, ray_id, stream);
}

// The same rays in tiles across views (the Operator's trace order for orbits of identical cone
// detectors, raytracer._view_tiles): the rays array is laid out (h, w / tw, n_views / tv, tv, tw,
// 3) — a tile is one pair (tw) of pixels of a detector row seen from tv consecutive views — and
// ray_id[i] is the geometry ray of row i (int32).  tv must divide n_views and tw divide w.
extern "C" int sphrt_rays_cone_tiled(int64_t n_views, int64_t h, int64_t w, int circ,
                                     const double* frame, const double* row, const double* col,
                                     int64_t tv, int64_t tw, double* rays, int32_t* ray_id,
                                     void* stream) {
    if (!ray_id) return fail("null pointer");
    if (tv < 1 || tw < 1 || n_views % tv != 0 || w % tw != 0) return fail("bad view tile");
    return rays_cone(n_views, h, w, circ, frame, row, col, rays, nullptr, ray_id, stream, tv, tw);
}
