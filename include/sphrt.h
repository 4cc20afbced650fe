/*
 * sphrt.h — C ABI of the MI355X-native spherical-grid raytracer (libsphrt.so, gfx950).
 *
 * This is the drop-in boundary for the hot path of Evidlo/sph_raytracer: ray <-> spherical-voxel
 * intersection (sphere / cone / half-plane crossings), per-ray merge + forward fill + segment
 * lengths, and the line-integral forward / adjoint.  The reference has no native boundary; its
 * interface is the Python `Operator` (raytracer.py:647-755).  Each entry point below names the
 * reference code it replaces.  The Python package `sph_raytracer_amd` binds these with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Plain C types only.  Every large buffer is allocated by the caller (PyTorch-ROCm tensors) and
 *    passed as a raw device pointer; the library never frees caller memory.  A plan owns only its
 *    small boundary tables.
 *  - `stream` is a hipStream_t passed as void*.  All work is stream-ordered; the only host sync in
 *    the whole trace is the caller's read of the total segment count between count and fill.
 *    Every call launches on its stream's device, whatever device is current in the calling
 *    thread (a null stream means the current device's); calls with a plan fail when the stream
 *    is not on the plan's device.
 *  - Return value: 0 on success, non-zero on error; sphrt_last_error() gives a message
 *    (thread-local).  Functions never abort the process.
 *  - Geometry is float64 (reference FTYPE = float64, raytracer.py:14).  Densities / images may be
 *    float32 or float64 (float64 densities are accumulated in float64; float32 ones: see
 *    sphrt_forward_f32).
 */
#ifndef SPHRT_H
#define SPHRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPHRT_MAX_DIMS 6

/* Boundary description of a SphericalGrid (geometry.py:107-183).  All pointers are HOST memory;
 * the trigonometric tables are computed by the caller with the same host library the reference
 * uses (torch CPU: raytracer.py:373-375, 505-506), so every table entry is bit-identical. */
typedef struct sphrt_grid_desc {
    int32_t nr, ne, na;       /* voxels per axis: grid.shape.r/e/a                              */
    const double *r_b;        /* nr+1 sphere radii, ascending            (geometry.py:158-161)  */
    const double *e_b;        /* ne+1 cone angles from +Z                (geometry.py:165)      */
    const double *a_b;        /* na+1 half-plane azimuths                (geometry.py:166)      */
    const double *cos_e;      /* torch.cos(e_b)                          (raytracer.py:452)     */
    const double *cos2_e;     /* torch.cos(e_b)**2                       (raytracer.py:373-375) */
    const double *cos_a;      /* torch.cos(a_b)                          (raytracer.py:505)     */
    const double *sin_a;      /* torch.sin(a_b)                          (raytracer.py:506)     */
    int32_t a_wrap;           /* -a_b[0] == a_b[-1] == pi                (raytracer.py:528)     */
    double close_tol;         /* finfo(ftype).resolution ** (1/3)        (raytracer.py:233-246) */
    double plane_par_tol;     /* finfo(ftype).resolution                 (raytracer.py:521)     */
} sphrt_grid_desc;

typedef struct sphrt_plan sphrt_plan;

/* Ray batch: `ndim`-dimensional broadcast shape; xs (...,3) f64 ray starts and rays (...,3) f64
 * directions addressed with per-dim element strides (0 = broadcast dim), last dim contiguous.
 * `start` holds the start voxel of every *unique* start as int32 (r, e, a, pad), addressed as
 * start[4 * (xs_offset / 3)] — i.e. laid out like an un-broadcast, contiguous xs.  It replaces
 * find_starts (raytracer.py:605-644), which the caller evaluates on the host once per unique
 * start. */
typedef struct sphrt_rays {
    int32_t ndim;
    int64_t shape[SPHRT_MAX_DIMS];
    int64_t xs_stride[SPHRT_MAX_DIMS];
    int64_t rays_stride[SPHRT_MAX_DIMS];
    const double *xs;
    const double *rays;
    const int32_t *start;
} sphrt_rays;

/* ---- plan --------------------------------------------------------------------------------- */
/* Replaces the per-call conversion of grid.r_b/e_b/a_b inside r_torch/e_torch/a_torch
 * (raytracer.py:271-277, 353-361, 493-501).  `device` is the HIP device ordinal. */
int sphrt_plan_create(const sphrt_grid_desc *grid, int device, sphrt_plan **out);
/* The same plan over caller-owned device tables (no hipMalloc, no hipFree: the device-wide sync
 * hipFree implies is avoided): sphrt_plan_pack_tables writes sphrt_plan_table_bytes(grid) bytes
 * into host memory, the caller copies them to an 8-byte-aligned device buffer that outlives the
 * plan (stream-ordered before the plan's first use) and passes it here. */
size_t sphrt_plan_table_bytes(const sphrt_grid_desc *grid);
int sphrt_plan_pack_tables(const sphrt_grid_desc *grid, void *host_tables);
int sphrt_plan_create_external(const sphrt_grid_desc *grid, int device, const void *dev_tables,
                               sphrt_plan **out);
int sphrt_plan_destroy(sphrt_plan *plan);
/* Candidates per ray in the reference's concatenation (raytracer.py:92, 117-122):
 * K = 2(nr+1) + 2(ne+1) + (na+1) + 1. */
int64_t sphrt_plan_candidates(const sphrt_plan *plan);
const char *sphrt_last_error(void);
const char *sphrt_version(void);

/* ---- per-family crossing solves (API-parity with r_torch / e_torch / a_torch) -------------- */
/* family 0 = spheres  (r_torch, raytracer.py:248-325): t, region  (n, 2*(nr+1))
 * family 1 = cones    (e_torch, raytracer.py:328-468): t, region  (n, 2*(ne+1))
 * family 2 = planes   (a_torch, raytracer.py:471-552): t, region  (n, na+1)
 * `neg` receives negative_crossing (int8, same shape).  Rays are normalised on private copies
 * (the reference normalises the caller's tensor in place, raytracer.py:281/365). */
int sphrt_solve(const sphrt_plan *plan, const sphrt_rays *rays, int family,
                double *t, int32_t *region, int8_t *neg, void *stream);
/* The same solves in float32 (r_torch / e_torch / a_torch with ftype=torch.float32): starts and
 * directions rounded to float, every operation in float.  The plan must hold the float32 tables
 * (boundaries, cos/sin evaluated by torch in float32, stored exactly as doubles) and the float32
 * thresholds (close_tol = 1e-6 ** (1/3), plane_par_tol = 1e-6: raytracer.py:233-246, 521). */
int sphrt_solve_f32(const sphrt_plan *plan, const sphrt_rays *rays, int family,
                    float *t, int32_t *region, int8_t *neg, void *stream);

/* ---- trace to compact CSR (replaces trace_indices, raytracer.py:48-230) -------------------- */
/* Every trace call takes a caller-allocated device workspace of
 * sphrt_trace_workspace_bytes(plan, n) bytes: it holds the list of rays whose crossings tie
 * exactly in a way that makes the result depend on the reference's (unstable, libstdc++
 * introsort) tie order, and the scratch of the exact kernel that replays that order. */
size_t sphrt_trace_workspace_bytes(const sphrt_plan *plan, int64_t n);
/* Pass 1: number of non-zero-length, in-grid segments of every ray (int32, n = prod(shape)). */
int sphrt_trace_count(const sphrt_plan *plan, const sphrt_rays *rays, int32_t *counts,
                      void *workspace, size_t workspace_size, void *stream);
/* Exclusive scan counts -> row_ptr (n+1, int64).  `workspace` must hold
 * sphrt_scan_workspace_bytes(n) bytes.  row_ptr[n] is the total segment count. */
size_t sphrt_scan_workspace_bytes(int64_t n);
int sphrt_scan_counts(const int32_t *counts, int64_t n, int64_t *row_ptr, void *workspace,
                      void *stream);
/* Pass 2: per-segment linear voxel index ((r*ne + e)*na + a) and length, in ray order and, per
 * ray, in order of increasing distance.  Equivalent to the reference's (regs, lens) with
 * zero-length and invalid entries dropped (raytracer.py:131-173). */
int sphrt_trace_fill(const sphrt_plan *plan, const sphrt_rays *rays, const int64_t *row_ptr,
                     int32_t *vox, double *len, void *workspace, size_t workspace_size,
                     void *stream);

/* Reference-mode trace: the options the fast trace does not take (Operator(..., ftype=float32)
 * and / or invalid=True, raytracer.py:48-173).  Every ray runs the reference algorithm verbatim
 * on the device: all K candidates, its (unstable) introsort order, the forward fill and the
 * length differences.  flags: SPHRT_TRACE_F32 — solves and differences in float32 (a float32
 * plan, as for sphrt_solve_f32; lengths are float32 values stored as doubles);
 * SPHRT_TRACE_INVALID — no masking (raytracer.py:155 `if not invalid`): every non-zero length is
 * kept, inf and NaN included, with its voxel wrapped the way the reference's forward indexes it
 * (region -1 reads the last shell / cone / wedge); SPHRT_TRACE_FRESH_RAYS — the caller's rays are
 * not of the trace's dtype, so tr.asarray(rays, ftype) hands each solver a fresh copy
 * (raytracer.py:276,360,500): r_torch and e_torch normalise theirs once, a_torch uses them
 * unnormalised (without the flag the in-place normalisations of raytracer.py:281,365 chain: e_torch
 * and a_torch see the twice-normalised rays).  row_ptr == NULL: count pass (`counts`, int32 per
 * ray); else fill pass into (vox, len) at row_ptr.  Workspace: sphrt_trace_workspace_bytes. */
#define SPHRT_TRACE_F32 1
#define SPHRT_TRACE_INVALID 2
#define SPHRT_TRACE_FRESH_RAYS 4
int sphrt_trace_reference(const sphrt_plan *plan, const sphrt_rays *rays, int flags,
                          int32_t *counts, const int64_t *row_ptr, int32_t *vox, double *len,
                          void *workspace, size_t workspace_size, void *stream);
/* The reference-mode trace in one pass, as sphrt_trace_emit: every ray's segments into its slot
 * [bound_ptr[i], bound_ptr[i+1]) of (svox, slen) and its exact count into counts; rays whose
 * count exceeds their slot write only the count and are counted in *n_over (device int64).  A
 * slot of K (sphrt_plan_candidates) segments always suffices: the walk keeps at most one segment
 * per list entry.  Compact with sphrt_trace_compact after scanning the counts. */
int sphrt_trace_reference_emit(const sphrt_plan *plan, const sphrt_rays *rays, int flags,
                               const int64_t *bound_ptr, int32_t *counts, int32_t *svox,
                               double *slen, int64_t *n_over, void *workspace,
                               size_t workspace_size, void *stream);

/* One-pass trace (the same CSR as count + fill, tracing every ray once instead of twice):
 *  1. sphrt_trace_bound: screens the rays and writes an upper bound of every ray's segment count
 *     from its geometry alone (int32 `bounds`, 0 for rays that miss the grid); the caller scans
 *     them (sphrt_scan_counts) into bound_ptr (n+1) and allocates a staging CSR of
 *     bound_ptr[n] entries (svox int32, slen float64).
 *  2. sphrt_trace_emit (same workspace: it traces the hit list step 1 left there): every ray's
 *     exact segment count into `counts`, and its segments into staging slot
 *     [bound_ptr[ray], bound_ptr[ray+1]) when they fit.  *n_over (device int64) = rays that did
 *     not fit; if it is non-zero the staging is incomplete and the caller runs sphrt_trace_fill
 *     instead of step 3 (the counts are exact either way).
 *  3. after sphrt_scan_counts(counts) -> row_ptr: sphrt_trace_compact moves the rows into the
 *     tight CSR (vox, len: row_ptr[n] entries).  Either pair (svox, vox) or (slen, len) may be
 *     NULL to move the other one alone: moving them in two calls, freeing each staging array
 *     after its call, caps the peak footprint at staging + 12 B per segment. */
int sphrt_trace_bound(const sphrt_plan *plan, const sphrt_rays *rays, int32_t *bounds,
                      void *workspace, size_t workspace_size, void *stream);
int sphrt_trace_emit(const sphrt_plan *plan, const sphrt_rays *rays, const int64_t *bound_ptr,
                     int32_t *counts, int32_t *svox, double *slen, int64_t *n_over,
                     void *workspace, size_t workspace_size, void *stream);
int sphrt_trace_compact(int64_t n, const int64_t *bound_ptr, const int32_t *svox,
                        const double *slen, const int64_t *row_ptr, int32_t *vox, double *len,
                        void *stream);

/* ---- on-device cone-beam ray directions (replaces ConeRectGeom.rays, geometry.py:493-508, and
 * ConeCircGeom.rays, geometry.py:570-582) ----------------------------------------------------- */
/* rays[v][a][b][0..2] for n_views views of h x w pixels, bit-identical to the torch expressions.
 * frame: per view {lookdir, lookdir x updir, updir} (9 doubles).  circ == 0 (rect): row[v][a] =
 * linspace(-ulim, ulim, h), col[v][b] = linspace(-vlim, vlim, w).  circ == 1: row[v][a] = r,
 * col[v] = {cos(theta) (w values), sin(theta) (w values)}, r*cos and r*sin in double; circ == 2:
 * the same with r*cos and r*sin rounded to float (the host tensors are float32). */
int sphrt_rays_cone(int64_t n_views, int64_t h, int64_t w, int circ, const double *frame,
                    const double *row, const double *col, double *rays, void *stream);
/* The same rays in a per-view trace order (the ConeCirc wedge order of the Operator's trace):
 * rays[v][k] is pixel order[k] of view v (order: a permutation of the h*w pixels, device
 * memory) and ray_id[v*h*w + k] = v*h*w + order[k] (int32; n_views*h*w < 2^31). */
int sphrt_rays_cone_ordered(int64_t n_views, int64_t h, int64_t w, int circ, const double *frame,
                            const double *row, const double *col, const int64_t *order,
                            double *rays, int32_t *ray_id, void *stream);
/* The same rays in tiles across views: rays is laid out (h, w / tw, n_views / tv, tv, tw, 3) —
 * each tile holds tw neighbouring pixels of one detector row seen from tv consecutive views —
 * and ray_id[i] = the geometry ray (v * h * w + pixel) of row i (int32; n_views * h * w < 2^31).
 * tv must divide n_views and tw must divide w.  The Operator traces orbits in this order
 * (raytracer._view_tiles); ray starts broadcast over it with per-dim strides (sphrt_rays). */
int sphrt_rays_cone_tiled(int64_t n_views, int64_t h, int64_t w, int circ, const double *frame,
                          const double *row, const double *col, int64_t tv, int64_t tw,
                          double *rays, int32_t *ray_id, void *stream);

/* ---- row index of the trace, built once (the apply kernels' work partition) ---------------- */
/* A traced operator: the CSR above plus
 *   vox     — bit 31 (SPHRT_ROW_HEAD) set on the first segment of every non-empty ray,
 *   row_ray — ray id of every non-empty row, in order,
 *   empty_ray — the rays without segments, ascending (allocate n_rays + 1 entries),
 *   blocks  — n_blocks x 6 int64 {empty_lo, empty_hi, seg_lo, seg_hi, row_lo, n_tab}: block b
 *             owns the whole rows starting in segments [b*1792, (b+1)*1792) (b*1984 with dense
 *             output ranges: sphrt_csr_index_dense) and zeroes the empty
 *             rays empty_ray[empty_lo .. empty_hi),
 *   tab     — (optional) per block b, its n_tab distinct 4-voxel granules (voxel >> 2) ascending
 *             at tab[b*tab_stride ..) (n_blocks * tab_stride entries),
 *   loc     — (optional) per segment, 16 * (rank of its granule in the block's table + 1) +
 *             4 * (voxel & 3): the voxel's byte offset in the forward's float LDS image, whose
 *             granule 0 is zero; the row-head flag in bit 15 (SPHRT_LOC_HEAD).
 * sphrt_csr_index() fills vox heads, row_ray, empty_ray and blocks from row_ptr (n_tab = -1);
 * n_blocks = sphrt_csr_blocks(n_segments).  sphrt_csr_local_count/_fill then build tab and loc
 * (uint16, n_segments entries) for every block of at most 4096 segments and 2046 granules; with
 * loc/tab/n_cols/tab_stride set, a static forward on a 16-byte-aligned density stages each
 * block's granules in LDS (4 * (tab_stride + 1) elements, up to 64 KB) instead of gathering per
 * segment.
 * Per-segment arrays (vox, len, len32, loc) are read in aligned 8- or 16-entry chunks: allocate
 * them to round_up(n_segments, 16) entries (the entries past n_segments are never used).  `len32` is
 * the float32 copy of `len` used by the float32 forward: sphrt_csr_local_count / _build write it
 * (len32[i] = (float)len[i], every segment) when both len and len32 are set, else the caller makes
 * it (sphrt_f64_to_f32). */
#define SPHRT_ROW_HEAD 0x80000000u
#define SPHRT_BLOCK_FIELDS 6   /* int64 per entry of blocks */
#define SPHRT_LOC_HEAD 0x8000u
typedef struct sphrt_csr {
    int64_t n_rays;
    int64_t n_segments;
    const int64_t *row_ptr;
    const int32_t *vox;
    const double *len;
    const float *len32;
    const int32_t *row_ray;
    const int64_t *blocks;
    int64_t n_blocks;
    const uint16_t *loc;   /* NULL: per-segment gathers through vox */
    const void *tab;       /* int32 entries, or uint16 when tab_bytes == 2 */
    int64_t n_cols;        /* column ids (vox & ~head) are < n_cols: voxels, or rays if transposed */
    int64_t n_fallback;    /* blocks without a granule table (n_tab = -1), from sphrt_csr_local */
    const int32_t *empty_ray;  /* the rays without segments, ascending (n_rays - rows entries) */
    int64_t tab_stride;    /* granule-table entries per block (>= the largest n_tab) */
    int64_t tab_bytes;     /* 2: uint16 table entries (n_cols <= 2^18), else int32 */
    /* Brick staging for the granule-table forward (all zero: off).  The columns are the voxels of
     * an (Nr, Ne, Na) = stage_shape grid; the granule tables and loc address a copy of the
     * density re-laid in bricks of stage_brick = (br, be, ba) voxels (each dim padded up to a
     * multiple of its brick), so one 128-byte line holds a compact 3-D neighbourhood instead of a
     * run along a.  Every table-mode forward first packs the density into `stage` (stage_bytes,
     * >= n_chan * stage_cols * sizeof(T), else the call fails).  The stage is scratch of one call:
     * two calls in flight at once (e.g. on two streams) need two stage buffers; the Python layer
     * passes a fresh stream-ordered allocation with every call.  vox stays in natural order. */
    int32_t stage_shape[3];
    int32_t stage_brick[3];
    int64_t stage_cols;    /* prod over dims of ceil(shape / brick) * brick */
    void *stage;
    int64_t stage_bytes;
    /* (optional, sphrt_csr_runs) per block SPHRT_RUN_FIELDS int32: its rows' rays and its share
     * of the empty rays as ranges; NULL: the forward reads row_ray / empty_ray instead. */
    const int32_t *runs;
    /* Block order of the forward (a performance hint: results are identical).  0: the default
     * order; bit 0 set: reversed; bit 1 set: one contiguous range of blocks per XCD, for CSRs
     * whose rays read disjoint column ranges (the time-paired CSR of a dynamic grid: C4 forward
     * f32 20.3 -> 18.9 us).  The Python layer flips bit 0 after every launch of a CSR of more than one
     * resident wave of blocks, so a CSR (or a forward / adjoint pair) that outgrows the
     * memory-side cache starts each launch on the lines the previous launch left cached instead
     * of the ones it evicted first (C3 forward f32 233 -> 213 us; C5 retrieval 0.138 -> 0.133
     * ms/iteration).  Bit 2 set (not a hint: a layout): dense output ranges — the rows are in
     * output order (row_ray increasing) and each block record's fields 0 / 1 hold the output range
     * [lo, hi) that block writes, its rows and the empty rows up to the next block's first row;
     * the block zeroes the range itself and empty_ray is not read.  One channel, no
     * ray_chan_div, runs NULL. */
    int64_t order;
    /* 1: `stage` already holds this call's density in the brick layout (pad columns zero), e.g.
     * written by sphrt_adam_neg_f64 after an earlier forward packed the same buffer; the forward
     * skips its pack.  0: the forward packs (the default). */
    int64_t stage_packed;
} sphrt_csr;

int64_t sphrt_csr_blocks(int64_t n_segments);
size_t sphrt_csr_index_workspace_bytes(int64_t n_rays);
/* ray_ids: NULL (row r is ray r), or the ray each row reports in row_ray / empty_ray — the
 * output index of a trace made in another ray order than the geometry's (the Operator traces
 * ConeCirc views in wedges of raytracer._WEDGE (3) azimuth columns, raytracer._trace_order). */
int sphrt_csr_index(const int64_t *row_ptr, int64_t n_rays, int32_t *vox, int32_t *row_ray,
                    int32_t *empty_ray, int64_t *blocks, int64_t n_blocks, const int32_t *ray_ids,
                    void *workspace, void *stream);
/* The same index for a CSR that will take dense output ranges (order bit 2: rows in output order,
 * one output per row or empty row — the time-paired transposed adjoint): block b owns the rows
 * starting in segments [b*1984, (b+1)*1984), n_blocks = sphrt_csr_blocks_dense(n_segments).  The
 * forward reads a CSR with order bit 2 set by these blocks, so its index must come from here. */
int64_t sphrt_csr_blocks_dense(int64_t n_segments);
int sphrt_csr_index_dense(const int64_t *row_ptr, int64_t n_rays, int32_t *vox, int32_t *row_ray,
                          int32_t *empty_ray, int64_t *blocks, int64_t n_blocks,
                          const int32_t *ray_ids, void *workspace, void *stream);
/* Granule tables in two passes.  _count sets n_tab in blocks (-1: no table) and writes two
 * device int64 to stats: {blocks without a table, largest n_tab}; the caller copies the first to
 * csr->n_fallback, picks tab_stride >= the second (csr->tab_stride; tab holds n_blocks *
 * tab_stride entries) and runs _fill.  Brick staging (stage_* fields) is decided before _count:
 * both passes and every later forward on the tables use the same stage_* values. */
int sphrt_csr_local_count(const sphrt_csr *csr, int64_t *blocks, int64_t *stats, void *stream);
int sphrt_csr_local_fill(const sphrt_csr *csr, const int64_t *blocks, uint16_t *loc, void *tab,
                         int64_t tab_stride, void *stream);
/* The same tables in one pass: _build decides n_tab (and the fallback blocks) and writes loc and
 * each kept block's table at the fixed wide stride SPHRT_TAB_WIDE (tab_wide: n_blocks *
 * SPHRT_TAB_WIDE entries of tab_bytes each), with stats as in _count; the caller picks tab_stride
 * from stats and _pack copies the tables to that stride.  Same output as _count + _fill. */
#define SPHRT_TAB_WIDE 2048
int sphrt_csr_local_build(const sphrt_csr *csr, int64_t *blocks, uint16_t *loc, void *tab_wide,
                          int64_t *stats, void *stream);
int sphrt_csr_local_pack(const sphrt_csr *csr, const int64_t *blocks, const void *tab_wide,
                         void *tab, int64_t tab_stride, void *stream);
/* The one-pass trace without its compaction pass (one-pass table build).  After sphrt_trace_emit the segments sit in staging slots (svox / slen at
 * slot[row], the scanned bounds); sphrt_csr_index_staged indexes the CSR from row_ptr alone (no
 * head bits: vox is not written yet) and lists the trace row of every non-empty row (nz_row, one
 * int32 per non-empty row: allocate n_rays); sphrt_csr_local_build_staged then moves every block's
 * segments from the staging into csr->vox (with the row-head bits), csr->len and csr->len32 and
 * builds the tables from them — the same CSR, loc and tables as sphrt_trace_compact +
 * sphrt_csr_index + sphrt_csr_local_build (csr->vox/len/len32 are written through the const
 * pointers).  The staging may be freed after it — except with csr->len NULL: the float64
 * lengths then stay in slen (the float32 forward reads len32 only) until
 * sphrt_trace_compact(svox = vox = NULL) moves them into the CSR on the first use that needs
 * them; svox may be freed right away. */
int sphrt_csr_index_staged(const int64_t *row_ptr, int64_t n_rays, int32_t *row_ray,
                           int32_t *empty_ray, int64_t *blocks, int64_t n_blocks,
                           const int32_t *ray_ids, int32_t *nz_row, void *workspace, void *stream);
int sphrt_csr_local_build_staged(const sphrt_csr *csr, int64_t *blocks, uint16_t *loc,
                                 void *tab_wide, int64_t *stats, const int64_t *slot,
                                 const int32_t *nz_row, const int32_t *svox, const double *slen,
                                 void *stream);
/* Row runs (optional).  Block b's rows map to rays in runs of consecutive rays, and its share of
 * the empty rays (empty_ray[empty_lo .. empty_hi)) to ranges of consecutive rays; when both fit
 * in SPHRT_MAX_RUNS entries for every block, the table-mode forward takes them from one 128-byte
 * record per block instead of loading row_ray / empty_ray entries (no dependent row loads, and
 * the empty rays are zeroed by contiguous stores).  runs: n_blocks x SPHRT_RUN_FIELDS int32
 *   [0] row runs, [1] empty ranges (-1: more than SPHRT_MAX_RUNS),
 *   [2 + 2i], [3 + 2i]  run i: first row (relative to the block's row_lo), its ray,
 *   [16 + 2i], [17 + 2i] empty range i: first ray, ray count.
 * Writes one device int64 to stats: the number of blocks with more than SPHRT_MAX_RUNS runs or
 * ranges (the caller sets csr->runs only when it is 0).  Needs row_ray, empty_ray and blocks. */
#define SPHRT_RUN_FIELDS 32
#define SPHRT_MAX_RUNS 7
int sphrt_csr_runs(const sphrt_csr *csr, int32_t *runs, int64_t *stats, void *stream);

/* Time-paired columns for a dynamic operator whose view i sees time slice i (ray r reads slice
 * r / div): vox_out[s] = (r / div) * vol + voxel, head bit kept, for every segment of ray r.  A
 * CSR with these columns (and its own blocks / tables, n_cols = T * vol) is a static CSR over the
 * flattened (T, vol) density: granule-table forward, transposed deterministic adjoint.
 * Requires T * vol < 2^31. */
int sphrt_csr_time_columns(const sphrt_csr *csr, int64_t div, int64_t vol, int32_t *vox_out,
                           void *stream);

/* ---- forward line integral on the CSR (replaces Operator.__call__, raytracer.py:692-713) -- */
/* out[c*out_chan_stride + i] = sum_s density[c*chan_stride + vox[s]] * len[s] over ray i's row.
 * If ray_chan_div > 0, ray i only sees channel c = i / ray_chan_div (dynamic grid paired with a
 * ViewGeomCollection, raytracer.py:705-706) and n_chan must be 1 in the call (the channel is
 * derived); otherwise every ray is integrated for all n_chan channels (static multichannel).
 * float64: products and sums in float64.  float32 (streams `len32`): products and each thread's
 * run of up to 8 consecutive segments of a row in float32 (the reference's own f32 product
 * rounding, raytracer.py:710), the runs of a row stitched across threads in float32 as well
 * (the reference sums in float32 too); measured within 2.5e-7 relative of float64
 * accumulation (C2-C5). */
int sphrt_forward_f32(const sphrt_csr *csr, const float *density, int64_t n_chan,
                      int64_t chan_stride, int64_t ray_chan_div, float *out,
                      int64_t out_chan_stride, void *stream);
int sphrt_forward_f64(const sphrt_csr *csr, const double *density, int64_t n_chan,
                      int64_t chan_stride, int64_t ray_chan_div, double *out,
                      int64_t out_chan_stride, void *stream);

/* Kernel timing for measurement (bench.py's roofline; no reference counterpart): the next
 * sphrt_forward_f32/f64 call on this host thread launches its main forward kernel with these two
 * HIP events (hipEvent_t, created with timing) bound to the dispatch itself, so that
 * hipEventElapsedTime(start, stop) is that kernel's own duration — what a kernel trace reports —
 * whatever the host's issue rate.  Consumed by that one launch; the brick pack and the fallback
 * launch are not bracketed.  Either event may be NULL. */
int sphrt_time_next_forward(void *start_event, void *stop_event);

/* ---- adjoint / back-projection (replaces Operator.T, raytracer.py:715-748, and the autograd
 * backward of raytracer.py:710) ------------------------------------------------------------ */
/* acc[c*chan_stride + vox[s]] += y[c*y_chan_stride + i] * len[s], float64 atomics into a zeroed
 * float64 accumulator `acc` (caller-allocated).  Same channel rules as forward. */
int sphrt_adjoint_accumulate(const sphrt_csr *csr, const void *y, int y_is_f64, int64_t n_chan,
                             int64_t y_chan_stride, int64_t ray_chan_div, double *acc,
                             int64_t chan_stride, void *stream);

/* Deterministic adjoint: the voxel-major transpose of the trace (built once).  col_ptr
 * (n_vox+1), t_ray / t_len (n_segments): for voxel v, the segments col_ptr[v] .. col_ptr[v+1]
 * in ray order (stable radix sort).  Index it with sphrt_csr_index(col_ptr, n_vox, t_ray, ...)
 * and the adjoint is sphrt_forward_f32/f64 on that CSR with y as the "density": no atomics,
 * bitwise reproducible. */
size_t sphrt_transpose_workspace_bytes(int64_t n_segments, int64_t n_vox);
int sphrt_csr_transpose(const sphrt_csr *csr, int64_t n_vox, int64_t *col_ptr, int32_t *t_ray,
                        double *t_len, void *workspace, size_t workspace_size, void *stream);
/* dst[i] = (float)src[i] — rounding the float64 accumulator to a float32 result. */
int sphrt_f64_to_f32(const double *src, float *dst, int64_t n, void *stream);
/* dst[i] = src[idx[i]], i < n (idx int32): the adjoint's input in trace order when the transposed
 * CSR's columns are trace rows (idx = the trace's ray ids), one launch instead of an
 * index_select. */
int sphrt_gather_f32(const float *src, const int32_t *idx, int64_t n, float *dst, void *stream);
int sphrt_gather_f64(const double *src, const int32_t *idx, int64_t n, double *dst, void *stream);

/* ---- retrieval loss tails (csrc/loss.hip; retrieval._gd_direct) ------------------------------
 * SquareLoss: r = yhat - y (y float32 or float64, promoted), r_scaled = r * scale, and the
 * partial sums of r * r; with `order` (NULL: identity), r_scaled[j] is ray order[j]'s (a
 * trace's sphrt_csr_index ray_ids: the transposed adjoint's input in trace order).  NegRegularizer: g -= c_neg where d < 0, and the partial sums of
 * |clamp(d, max=0)|.  The elementwise values are single IEEE operations, the values torch's
 * elementwise ops give (reference loss.py:87-162).  Each call writes sphrt_loss_partials(n)
 * partial sums (fixed partition and order); the loss is their sum / n, within rounding of
 * torch.mean. */
int64_t sphrt_loss_partials(int64_t n);
int sphrt_sq_residual_f64(const double *yhat, const void *y, int y_is_f64, int64_t n, double scale,
                          const int32_t *order, double *r_scaled, double *partial_sums,
                          void *stream);
int sphrt_neg_reg_f64(const double *d, int64_t n, double c_neg, double *g, double *partial_sums,
                      void *stream);
/* One Adam step on float64 coefficients (torch.optim.Adam(fused=True), amsgrad and maximize off:
 * torch._fused_adam_'s per-element arithmetic, bitwise), step = the step count after this step's
 * increment (1, 2, ...).  With partial_sums set, the NegRegularizer is folded in first, as
 * sphrt_neg_reg_f64 on d = param before the step (grad itself is not modified); NULL: no
 * regulariser.  With stage_of (a brick-staged CSR over these n voxels, its `stage` buffer set),
 * the updated coefficients are also written to their staged columns, so the next forward can
 * run with stage_packed = 1 (pad columns are left as they are: zero after a forward's pack);
 * NULL: no stage.  Replaces, per retrieval iteration, the reference's optim.step() after
 * tot_loss.backward() (retrieval.py:115-116; loss.py:140-162 for the regulariser term). */
int sphrt_adam_neg_f64(double *param, const double *grad, double *exp_avg, double *exp_avg_sq,
                       int64_t n, double lr, double beta1, double beta2, double eps,
                       double weight_decay, double step, double c_neg, double *partial_sums,
                       const sphrt_csr *stage_of, void *stream);
/* The same step with the arithmetic of the default Adam on GPU tensors (torch.optim.Adam without
 * fused=: the multi-tensor "foreach" implementation, which the reference's optim(optim_vars,
 * **kwargs), retrieval.py:84, runs on a ROCm device), bitwise.  Its bias corrections come from
 * the host as torch computes them in Python: step_size = -lr / (1 - beta1**t), bc2_sqrt =
 * (1 - beta2**t) ** 0.5.  Regulariser and stage as sphrt_adam_neg_f64. */
int sphrt_adam_foreach_neg_f64(double *param, const double *grad, double *exp_avg,
                               double *exp_avg_sq, int64_t n, double step_size, double beta1,
                               double beta2, double eps, double weight_decay, double bc2_sqrt,
                               double c_neg, double *partial_sums, const sphrt_csr *stage_of,
                               void *stream);

/* ---- fused no-store mode: trace + integrate in one pass (nothing persisted) --------------- */
int sphrt_trace_integrate_f32(const sphrt_plan *plan, const sphrt_rays *rays,
                              const float *density, int64_t n_chan, int64_t chan_stride,
                              int64_t ray_chan_div, float *out, int64_t out_chan_stride,
                              void *workspace, size_t workspace_size, void *stream);
int sphrt_trace_integrate_f64(const sphrt_plan *plan, const sphrt_rays *rays,
                              const double *density, int64_t n_chan, int64_t chan_stride,
                              int64_t ray_chan_div, double *out, int64_t out_chan_stride,
                              void *workspace, size_t workspace_size, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SPHRT_H */
