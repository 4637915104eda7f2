// rt_kparams.h -- what the library's translation units share (not part of the ABI): the
// launch parameters of the render kernels (KParams, KBatch), their feature bits, the heavy-first /
// wide-section constants, the shard deal, and the kernel table rt_kernels.hip / rt_plan.hip export
// to the host code (rt_tracer.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rt_tracer.h"

namespace rtk {

constexpr uint32_t kTile = 16;              // shard / scheduling tile edge (pixels)
constexpr uint32_t kTilePix = kTile * kTile;
constexpr uint32_t kWG = 256;               // lanes per workgroup
constexpr uint32_t kWavesPerWG = kWG / 64u;
// Traversal features, combined into the VAR template argument of the render kernels.
constexpr int kVarWaveGate = 2;             // skip a test's second half when no lane needs it
constexpr int kVarSkipRun = 4;              // wave-uniform proven-empty runs in a tight loop
constexpr int kVarDistSkip = 8;             // L-inf distance field in the empty cells' words
constexpr int kVarBrute = 64;               // RT_ISECT_BRUTE_FORCE (renderer.cpp:157-197)
constexpr int kVarMarch = 128;              // RT_ISECT_RAY_MARCH (renderer.cpp:24-41, 138-155)
constexpr int kVarExhaustive = 256;         // RT_KERNEL_FLAG_EXHAUSTIVE: march without block culling
constexpr int kVarOriginPre = 512;          // per-camera-origin records (frefs, k_origin_pre)
constexpr int kVarFastRcp = 2048;           // Newton-refined exact 1/det (rt_scene::rcp_safe)
constexpr int kVarPackedRem = 4096;         // one packed remaining-cells word (rt_scene::pack_ok)
constexpr int kVarXcdBands = 8192;          // XCD-aware block -> tile order
constexpr int kVarWaveClock = 32768;        // RT_KERNEL_FLAG_WAVE_CLOCK: per-item s_memtime (debug)
constexpr int kVarUniform = 65536;          // scalar loop for wave-uniform cell lists
constexpr int kVarWideHeavy = 524288;       // RT_KERNEL_FLAG_WIDE_HEAVY: heavy items traced wide at the start
constexpr int kVarWideFused = 1048576;      // batch kernel: the wide section's blocks lead the same grid
constexpr int kVarWideG4 = 2097152;         // the wide section at 4 lanes per sample (spp 8-16; else 16)
constexpr int kVarLdsSplit = 4194304;       // the wide section's LDS tier: the waves of a workgroup split one
                                            // item's cell lists, reduced through LDS (wide_section_lds)
// AUTO's traversal: every feature above that is exact for every scene ...
constexpr int kVarAutoCore = kVarWaveGate | kVarDistSkip | kVarOriginPre | kVarXcdBands | kVarUniform;
// ... plus the two that need a scene property (rt_scene::rcp_safe, rt_scene::pack_ok)
constexpr int kVarAuto = kVarAutoCore | kVarFastRcp | kVarPackedRem | kVarSkipRun;
// the wide phase / wide kernel: AUTO's per-ray code, per-lane lists, no empty-run loop
constexpr int kVarWide = kVarWaveGate | kVarDistSkip | kVarOriginPre | kVarFastRcp | kVarPackedRem | kVarXcdBands;
// RT_KERNEL_COMPACT on AUTO's walk (box words present, rcp_safe)
constexpr int kVarCompactBox = kVarWide | kVarSkipRun;
constexpr uint32_t kMarchSteps = 128;       // renderer.cpp:26
constexpr uint32_t kDistBlock = 32;         // triangles per culling block of the distance kernels
constexpr uint32_t kCompactRefill = 48;     // RT_KERNEL_COMPACT default: refill when this many lanes idle

// heavy-first plan (one per list version): blocks listed at each of the two priority levels,
// the maximum block cost, the work items listed for the wide section (kVarWideHeavy) and the
// sum of wave costs of the measured frame
// sum_full: the sum of wave costs of the last measured frame that rendered every item one lane
// per sample (the wide section's span estimate; carried over by the plans of other frames)
// cnt_l: work items listed for the wide section's LDS tier (kVarLdsSplit; the list's second half)
struct HfPlan { uint32_t cnt_hi, cnt_lo, maxc, cnt_w; unsigned long long sum; unsigned long long sum_full; uint32_t cnt_l, pad; };

struct KParams
{
    // camera (per frame)
    float m[9];                 // Matrix44f m_mat[r][c], r,c < 3, row-major
    float fov_xs, aspect;
    float org[3];               // Transf4x4(Vec3f(0)) computed on the host (camera.h:43)
    uint32_t W, H, spp, spp_shift;
    float inv_spp;              // 2^-spp_shift when spp is a power of two (x/spp == x*inv_spp), else 0
    const float2 *smp;          // [spp] sample offsets
    const float *ndcx;          // [W * spp] camera-space x of (column, sample): rtd::cam_x, per frame shape
    const float *ndcy;          // [H * spp] camera-space y of (row, sample): rtd::cam_y
    // grid (grid.h:28-39)
    float bmin[3], bmax[3];
    float cw, icw;
    int dim[3];
    int dxdz;
    uint32_t max_steps;         // bound of the CSR-offset walk: no DDA walk is longer than dx+dy+dz
    const uint32_t *off;
    const uint32_t *cellw;      // packed cell words (start << 11 | count) or null
    const uint32_t *cellwo;     // the dist-skip walks' words: 8 ray-octant copies, or = cellw
    uint32_t oct_stride;        // words per octant copy (ncells), 0 when cellwo == cellw
    const uint32_t *cellwb;     // kVarSkipRun: box-run words, 24 copies (ray octant x major axis)
    uint32_t box_stride;        // words per copy (ncells)
    const float4 *refs;
    const float4 *frefs;        // per camera origin (kVarOriginPre), 3 float4 per reference
    const float4 *shade;
    const float4 *face_n;
    const float4 *tri_mt;       // per triangle {v0, e1, e2} in triangle order (brute force)
    const float4 *tri_dist;     // per triangle distance record (rtd::dist_point_tri), Morton order
    const float4 *dist_blk;     // per kDistBlock records: {aabb min, -}{aabb max, -}
    uint32_t ndist_blk;
    float scene_scale;          // max |vertex coordinate| (error bound of the block cull)
    float smin[3], smax[3];     // vertex AABB (exact float min / max)
    uint32_t ntris;
    uint32_t tri_test;
    uint32_t isect;             // enum rt_intersector
    // work decomposition
    uint32_t rx0, ry0, rw, rh;  // region of the frame rendered by this launch
    uint32_t tiles_x;           // 16x16 tiles across the region
    uint32_t rank, nranks;      // local tile k = row-rotated tile rank + k * nranks (shard_tile_xy)
    uint32_t wg_per_tile;
    uint32_t xcd_chunk;         // kVarXcdBands: consecutive blocks per XCD turn (0 = one band each)
    uint32_t vblocks;           // k_render_lanes_w64: the 256-lane launch blocks its one-wave grid runs
    uint64_t *wave_clk;        // kVarWaveClock: {start, end, uniform tests, lane-loop iterations} per item
    const uint32_t *tile_order; // tile order (position -> local tile) or null = natural order
    // heavy-first block order (AUTO; hf_front == 0: off).  Blocks [0, hf_front) render the blocks
    // the current plan (version hf_ver) lists as heavy, most expensive level first; blocks from
    // hf_front on walk the natural order and skip those.  In a measured frame (every
    // kHfPeriod-th of a launch shape) every wave stores its duration (hf_cost, one plain store)
    // and k_hf_plan writes the plan of version hf_ver + 1 from them.
    uint32_t hf_front;          // front section size (blocks, a multiple of 8)
    uint32_t hf_ver;            // version of the plan this frame uses (0: none yet)
    uint32_t hf_measure;        // 1: this frame records wave costs for the next plan
    uint32_t hf_floor;          // a block is heavy above max(hf_floor, last max >> hf_shift (RT_HF_SHIFT)) cycles
    const uint32_t *hf_mark_in; // per block: == hf_ver when the current plan lists it
    uint32_t *hf_mark_out;      // per block: hf_ver + 1 when the next plan lists it
    const uint32_t *hf_list_in; // the current plan's front: [0, cnt_hi) and [front - cnt_lo, front)
    uint32_t *hf_list_out;      // the next plan's
    const HfPlan *hf_plan_in;   // the current plan (also the previous measurement's max and sum)
    HfPlan *hf_plan_out;        // the next plan (cleared by launch_plans' hipMemsetAsync before k_hf_plan)
    uint32_t *hf_cost;          // per work item: shader cycles of its wave in the measured frame
    uint32_t *hf_ticket;        // k_hf_plan's finished-workgroup count (the last one marks)
                                // (a wide item: the sum over its waves)
    // wide section (kVarWideHeavy; wh_on == 0: off).  k_render_wh's wh_wgs workgroups trace the
    // work items the current plan lists as heavy (wh_list_in, plan->cnt_w of them), wh_g lanes
    // per sample (16 at spp <= 4, 4 at spp 8-16) -- and, in the LDS tier (kVarLdsSplit), the next
    // heaviest one 256-lane workgroup per item, one lane per sample -- and the lane waves skip items whose
    // wh_mark_in == hf_ver; with wh_wgs == 0 (no list seen yet, or a refresh frame) the lane
    // waves render every item.  k_hf_plan lists an item when its lane-mode cost passes
    // max(wh_floor, wh_alpha16 / 16 x the estimated frame span), and keeps the current plan's
    // items (their cost words still hold the lane-mode cost of the last frame that measured
    // them) except in a refresh frame.
    uint32_t wh_on, wh_wgs, wh_refresh, wh_g;
    uint32_t wh_floor, wh_alpha16;
    // kVarLdsSplit (wh_lds = 1): items between wh_beta16 / 16 and wh_alpha16 / 16 of the span estimate are
    // listed for the LDS tier (one 256-lane workgroup per item; the list's second half, wh_list + kWhMax;
    // marks with bit 31), the heavier ones for the wh_g-lane tier
    uint32_t wh_lds, wh_beta16;
    uint32_t wh_wgs_g;          // the first wh_wgs_g of the section's workgroups run the G-lane tier (= wh_wgs
                                // without the LDS tier), the rest the LDS tier
    const uint32_t *wh_mark_in;
    uint32_t *wh_mark_out;
    const uint32_t *wh_list_in;
    uint32_t *wh_list_out;
    uint32_t *wh_host_cnt;      // host-mapped [2]: the newest plan's G-lane waves and LDS items (size the next launches)
    // output
    uint32_t *out;
    uint32_t pitch;             // frame mode: words per row of out
    uint32_t shard_mode;        // 1: out[local_tile * 256 + ty*16 + tx]; 2: the framebuffer's tile buffers
    // shard_mode 2 (rt_render_frame_host_tiled): the fb_tx x fb_ty tile grid of Framebuffer::Resize
    // (framebuffer.cpp:106-117: tiles fb_tw x fb_th, the last column / row absorbs the remainder), each
    // tile's buffer row-major at its own width (framebuffer.h:41-45), the buffers in tile order
    uint32_t fb_tw, fb_th, fb_tx, fb_ty;
    uint32_t fb_mtw, fb_mth;    // ceil(2^32 / fb_tw), ceil(2^32 / fb_th): x / fb_tw as one mul_hi
    uint32_t *hits;             // rt_render_hits_device: per-sample hit triangle, [(y*W + x)*spp + s]
                                // (read after the walk through late_params; NULL in the plain calls)
    rt_sample_rec *recs;        // debug kernel only
    uint32_t rec_x0, rec_y0, rec_w, rec_h;
};

// A frame shape's camera-space tables (KParams::ndcx / ndcy, smp), written on the device by
// k_frame_tables from rtd::cam_x / cam_y (the host's restatement uses the same IEEE operations).
constexpr uint32_t kTabMaxSpp = 64;
struct TabParams
{
    float fx, aspect;               // fov_xs (double tan on the host, H5), width / height
    uint32_t W, H, spp;
    float smp[2 * kTabMaxSpp];      // the sample table (Hammersley or rt_frame.sample_offsets)
};

// Multi-frame launch (rt_render_batch_device): up to kMaxBatch frames -- of different scenes --
// in ONE grid, so one frame's tail overlaps the others' work and the heavy-first order ranks the
// blocks of all of them.  p[0] also carries the batch's heavy-first / wide-section state (its
// block and item indices are the launch's, frame-major); every other field is per frame.
// 10 frames (config 5's whole step) make KBatch ~5.9 KiB of kernel arguments: the runtime passes
// them intact past 4 KiB (tools/probe/kernarg_probe.hip, 8 KiB checked on the MI355X).
constexpr uint32_t kMaxBatch = 10;
struct KBatch
{
    KParams p[kMaxBatch];
    uint32_t nframes;
    uint32_t base[kMaxBatch + 1];   // first launch block of each frame; base[nframes] = all blocks
};

static_assert(sizeof(KBatch) <= 8192, "kernel arguments checked up to 8 KiB");

// Frames in the launch that starts at frame `start` of an n-frame batch: ceil(n / kMaxBatch)
// launches of near-equal size (10 frames: 5 + 5), each with one tail.  Mirrored by the binding's
// batch_chunks().
inline uint32_t batch_chunk_len(uint32_t n, uint32_t start)
{
    const uint32_t left = n - start, k = (left + kMaxBatch - 1u) / kMaxBatch;
    return (left + k - 1u) / k;
}

// XCD-aware block order (kVarXcdBands).  The dispatcher deals workgroups round-robin to the 8
// XCDs (block b runs on XCD b % 8), so consecutive blocks -- the 4 workgroups of one tile and
// the tiles of one row -- land on 8 different L2s, and every XCD's L2 caches the whole visible
// scene.  Remapped, XCD x takes turns of `chunk` consecutive blocks (one tile row): rows x,
// x + 8, x + 16, ... -- compact rows for its L2, and the frame's cost still spread over all
// XCDs.  chunk 0: one contiguous band per XCD (measured: load imbalance, up to 58 % slower).
// A bijection on [0, nblocks) for any grid size (the tail past whole 8-turn rounds keeps its
// order); on a device with another XCD count only the locality changes.
constexpr uint32_t kXcds = 8;
// Heavy-first order (AUTO): front-section capacity and the shape of the heavy threshold.  The
// floor and the smallest launch it is used for are per-scene tunables (rt_scene, read once at
// creation).
constexpr uint32_t kHfFrontMax = 4096;      // blocks (4 waves each): the front list's capacity (hf_front_max)
constexpr uint32_t kWhMax = 4096;           // kVarWideHeavy: work items the wide section can list
constexpr uint32_t kHfPeriod = 16;          // a plan from every kHfPeriod-th frame of a launch shape
// A plan lists blocks only when the slowest block is a real tail: its cost (one wave's
// duration) above kHfTail / 16 of the estimated frame span, sum of wave costs / resident waves
constexpr uint32_t kHfTail = 6;
constexpr uint32_t kHfSlots = 256u * 4u * 8u;   // resident waves: 256 CUs x 4 SIMDs x 8
constexpr int kHfCtxs = 16;                 // launch shapes remembered per scene (a process driving
                                            // the 8 ranks of two scenes' shards keeps all of them)
constexpr uint32_t kHfPlanPer = 8;          // k_hf_plan: blocks per thread

// Shard deal (nranks > 1): tile (tx, ty) has the row-rotated number
// t' = ty * tiles_x + (tx + kShardRot * ty) mod tiles_x, and rank r owns t' = r, r + N, r + 2N, ...
// as its local tiles 0, 1, 2, ...  The rotation turns t mod N's column stripes (1920 / 16 = 120
// columns: every rank held the same columns in every row, so a compact heavy region fell on the
// few ranks owning its columns) into a lattice; a rank's consecutive local tiles still lie in one
// tile row (XCD bands, shard layout and shard sizes are unchanged).  One rank: no rotation.
#ifndef RT_SHARD_ROT
#define RT_SHARD_ROT 3
#endif
constexpr uint32_t kShardRot = RT_SHARD_ROT;

__host__ __device__ __forceinline__ void shard_tile_xy(uint32_t k, uint32_t rank, uint32_t nranks, uint32_t tiles_x,
                                                       uint32_t& tx, uint32_t& ty)
{
    const uint32_t t = rank + k * nranks;
    ty = t / tiles_x;
    tx = t - ty * tiles_x;
    if (nranks > 1u)
    {
        const uint32_t r = (kShardRot * ty) % tiles_x;
        tx = tx >= r ? tx - r : tx + tiles_x - r;
    }
}

// The kernel table: rt_kernels.hip / rt_plan.hip hand the host code (rt_tracer.hip) the kernels it
// launches.  A getter returns nullptr for a variant that is not built.
using kfn_t = void (*)(KParams);
using kbfn_t = void (*)(KBatch);
using kcfn_t = void (*)(KParams, uint32_t, uint32_t);
using knfn_t = void (*)(KParams, uint32_t);
kfn_t lanes_kernel(int tri, int var);          // k_render_lanes<tri, var>
kfn_t lanes_w64_kernel(int var);               // k_render_lanes_w64<MT, var>
kfn_t wide_kernel(uint32_t g, bool lds);       // k_render_wh<g>, g = 4 or 16; k_render_wh_lds<g> (+ the LDS tier)
kfn_t pixel_loop_kernel(int tri, int var);     // k_render_pixel_loop<tri, var>
kcfn_t compact_kernel(int tri, int var);       // k_render_compact<tri, var>(P, n_items, refill)
kbfn_t batch_kernel(int var, bool w64, bool o8 = false);   // k_render_batch / _w64 / _w64_o8<MT, var>
knfn_t trace_records_kernel();                 // k_trace_records(P, n)
knfn_t record_fixup_kernel();                  // k_record_fixup(P, n)
using origin_pre_fn = void (*)(const float4 *, float4 *, uint32_t, float, float, float);
using unshard_fn = void (*)(const uint32_t *, uint32_t *, uint32_t, uint32_t, uint32_t, uint32_t, uint64_t);
using check_fn = void (*)(unsigned long long *);
using primitives_fn = void (*)(int, const float *, uint32_t, float *);
origin_pre_fn origin_pre_kernel();
using tables_fn = void (*)(float *, float2 *, TabParams);
tables_fn frame_tables_kernel();                // k_frame_tables(ndc, smp, T)
unshard_fn unshard_kernel();
check_fn rcp_check_kernel();
check_fn gamma_check_kernel();
primitives_fn primitives_kernel();

} // namespace rtk
