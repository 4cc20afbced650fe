// stage.hpp — brick staging of a CSR's columns (sphrt_csr.stage_*), shared by the forward
// (csrc/apply.hip: the pack and the granule tables) and the retrieval's Adam step (csrc/loss.hip:
// writing the next forward's staged density).
#pragma once
#include "common.hpp"

namespace sphrt {

// ---- brick staging (sphrt_csr.stage_*) ----------------------------------------------------
// A ray's consecutive voxels step in r, e or a; in the natural (r, e, a) order only steps in a stay
// inside one 128-byte line, so a workgroup's granules spread over as many lines as granules.
// Staged, the columns are bricks of br x be x ba voxels (32 = one float line): the same granules
// fall into 1.7x (C3) to 2.8x (C5) fewer lines, and the granule DMA's L2 requests drop with them
// (C3 f32 forward 267 -> 241 us, C5 41.9 -> 35.2 us with the pack; tools/brick_study.py).  Natural voxel v -> column:
struct StageMap {
    uint32_t on, ne, na, br, be, ba, nbe, nba;
};

__device__ __forceinline__ uint32_t stage_col(uint32_t v, const StageMap& s) {
    if (!s.on) return v;
    const uint32_t a = v % s.na, q = v / s.na, e = q % s.ne, r = q / s.ne;
    const uint32_t blk = ((r / s.br) * s.nbe + e / s.be) * s.nba + a / s.ba;
    return blk * (s.br * s.be * s.ba) + ((r % s.br) * s.be + e % s.be) * s.ba + a % s.ba;
}

static bool staged(const sphrt_csr* c) { return c->stage_shape[0] > 0; }

// Validated map of a CSR (on = 0 when staging is off); false on inconsistent fields.
static bool stage_map(const sphrt_csr* c, StageMap& m) {
    m = StageMap{0, 1, 1, 1, 1, 1, 1, 1};
    if (!staged(c)) return true;
    int64_t cols = 1, vol = 1;
    for (int d = 0; d < 3; ++d) {
        const int64_t n = c->stage_shape[d], b = c->stage_brick[d];
        if (n < 1 || b < 1) return false;
        cols *= (n + b - 1) / b * b;
        vol *= n;
    }
    const int64_t bv = (int64_t)c->stage_brick[0] * c->stage_brick[1] * c->stage_brick[2];
    if (bv % 4 != 0 || cols != c->stage_cols || vol != c->n_cols || cols >= INT32_MAX) return false;
    m.on = 1;
    m.ne = (uint32_t)c->stage_shape[1];
    m.na = (uint32_t)c->stage_shape[2];
    m.br = (uint32_t)c->stage_brick[0];
    m.be = (uint32_t)c->stage_brick[1];
    m.ba = (uint32_t)c->stage_brick[2];
    m.nbe = (m.ne + m.be - 1) / m.be;
    m.nba = (m.na + m.ba - 1) / m.ba;
    return true;
}

}  // namespace sphrt
