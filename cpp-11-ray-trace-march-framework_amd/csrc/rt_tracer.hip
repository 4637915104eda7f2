// rt_tracer.hip -- HIP kernels + C ABI (include/rt_tracer.h) for gfx950 (MI355X).
//
// One launch renders a whole frame (or one rank's shard): a workgroup of 256 lanes owns
// 256/spp pixels of a 16x16 pixel tile in Morton order, one lane per sample, so a pixel's
// samples sit in adjacent lanes and a wave covers a compact 2^k x 2^k pixel block (coherent
// DDA walks).  Each lane runs the reference's per-sample path (GenerateRay -> Grid::Intersect
// -> IntersectRayTri -> shading, renderer.cpp:88-122); the pixel's samples are then summed IN
// SAMPLE ORDER across lanes (renderer.cpp:87-122, hazard H10), averaged, gamma'd and packed
// (renderer.cpp:124-133).
//
// Scene layout in HBM (built once by rt_scene_create):
//   cellw     u32[C]              packed cell word in GridIdx order (grid.h:41-42): non-empty
//                                 start << 11 | count, empty: L-inf distance to geometry << 11
//   cell_off  u32[C+1]            CSR offsets (scenes whose lists do not fit the packed word)
//   refs      float4[3*R]         one 48-B record per CSR reference, in CSR order:
//                                 {v0.xyz, e1.x} {e1.yz, e2.xy} {e2.z, tri_idx bits, 0, 0}
//   frefs     float4[3*R]         per camera origin (k_origin_pre), one 48-B record per CSR
//                                 reference: {e1.xyz, e2.x} {e2.yz, tvec.xy} {tvec.z, qvec}:
//                                 the origin-only terms of triangle.h:82-90
//   shade     float4[3*T]         per triangle the 3 vertex normals (shading of a hit)
//   face_n    float4[T]           face normal (IntersectRayTriBarycentric only)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rt_tracer.h"
#include "rt_device.h"
#include "rt_internal.h"
#include "rt_box_words.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define RT_HIP(expr)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

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

// heavy-first plan (one per list version): blocks listed at each of the two priority levels,
// the maximum block cost, the work items listed for the wide section (kVarWideHeavy) and the
// sum of wave costs of the measured frame
// sum_full: the sum of wave costs of the last measured frame that rendered every item one lane
// per sample (the wide section's span estimate; carried over by the plans of other frames)
// cnt_w4: work items listed for the wide section's second tier (4 lanes per sample)
struct HfPlan { uint32_t cnt_hi, cnt_lo, maxc, cnt_w; unsigned long long sum; unsigned long long sum_full; uint32_t cnt_w4, pad; };

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
    uint32_t hf_floor;          // a block is heavy above max(hf_floor, last max >> kHfShift) cycles
    const uint32_t *hf_mark_in; // per block: == hf_ver when the current plan lists it
    uint32_t *hf_mark_out;      // per block: hf_ver + 1 when the next plan lists it
    const uint32_t *hf_list_in; // the current plan's front: [0, cnt_hi) and [front - cnt_lo, front)
    uint32_t *hf_list_out;      // the next plan's
    const HfPlan *hf_plan_in;   // the current plan (also the previous measurement's max and sum)
    HfPlan *hf_plan_out;        // the next plan, cleared by the measured frame's first lane
    uint32_t *hf_cost;          // per work item: shader cycles of its wave in the measured frame
    uint32_t *hf_ticket;        // k_hf_plan's finished-workgroup count (the last one marks)
                                // (a wide item: the sum over its waves)
    // wide section (kVarWideHeavy; wh_on == 0: off).  k_render_wh's wh_wgs workgroups trace the
    // work items the current plan lists as heavy (wh_list_in, plan->cnt_w of them), wh_g lanes
    // per sample (16 at spp <= 4, 4 at spp 8-16), and the lane waves skip items whose
    // wh_mark_in == hf_ver; with wh_wgs == 0 (no list seen yet, or a refresh frame) the lane
    // waves render every item.  k_hf_plan lists an item when its lane-mode cost passes
    // max(wh_floor, wh_alpha16 / 16 x the estimated frame span), and keeps the current plan's
    // items (their cost words still hold the lane-mode cost of the last frame that measured
    // them) except in a refresh frame.
    // Two tiers at spp <= 4 (wh_beta16 != 0): items above the alpha threshold take 16 lanes per sample,
    // items between the beta and the alpha thresholds 4 (the list's second half, wh_list + kWhMax;
    // their marks carry bit 31)
    uint32_t wh_on, wh_wgs, wh_refresh, wh_g;
    uint32_t wh_floor, wh_alpha16, wh_beta16;
    const uint32_t *wh_mark_in;
    uint32_t *wh_mark_out;
    const uint32_t *wh_list_in;
    uint32_t *wh_list_out;
    uint32_t *wh_host_cnt;      // host-mapped: the newest plan's wave count (sizes the next launches)
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

// Morton decode of an 8-bit index inside a 16x16 tile: x = even bits, y = odd bits.
__device__ __forceinline__ uint32_t compact_bits(uint32_t v)
{
    v &= 0x55u;
    v = (v | (v >> 1)) & 0x33u;
    v = (v | (v >> 2)) & 0x0Fu;
    return v;
}

// Orders this wave's LDS writes before its later LDS reads of other lanes' data (a wave
// executes its LDS operations in order; this keeps the compiler from reordering them).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// kVarWaveClock debug counters of this wave: [0] records tested in wave-uniform loops,
// [1] iterations of the per-lane list loop
__device__ __forceinline__ uint32_t *wave_counters()
{
    __shared__ uint32_t c[kWavesPerWG * 2u];
    return c + (threadIdx.x >> 6) * 2u;
}

// Wave-uniform "every active lane": the predicate's lane mask against exec.  Pass a single
// compare: a predicate combined from several is materialised in a VGPR and compared back
// (2 VALU per vote, seen in the empty-run loop's ISA), where a compare's mask is the ballot.
__device__ __forceinline__ bool wave_all(bool p)
{
    return __builtin_amdgcn_ballot_w64(p) == __builtin_amdgcn_ballot_w64(true);
}

// The minimum of x over the wave's active lanes (wave-uniform): start from the first active lane's
// value and move to the first lane below it until none is (a few rounds: each takes a strictly
// smaller value).  A NaN x never compares below, so T may stay NaN -- callers only compare x < T.
__device__ __forceinline__ float wave_min_active(float x)
{
    float T = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
    for (;;)
    {
        const uint64_t b = __builtin_amdgcn_ballot_w64(x < T);
        if (b == 0u) break;
        T = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), int(__builtin_ctzll(b))));
    }
    return T;
}

// v of lane (lane & ~3) + J: a DPP quad_perm broadcast within each quad of lanes (every lane of
// the quad must be active, as in process_item's resolve, where the whole wave is)
template <int J>
__device__ __forceinline__ float quad_bcast(float v)
{
    constexpr int ctrl = J | (J << 2) | (J << 4) | (J << 6);
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false));
}
template <int J>
__device__ __forceinline__ uint32_t quad_bcast_u(uint32_t v)
{
    constexpr int ctrl = J | (J << 2) | (J << 4) | (J << 6);
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), ctrl, 0xF, 0xF, false));
}

__device__ __forceinline__ bool first_active_lane()
{
    return (threadIdx.x & 63u) == uint32_t(__ffsll((long long)__ballot(1)) - 1);
}

// The kernel's KParams re-read from the kernarg segment.  Parameters used only after the
// walk (output, shading, tile bookkeeping) are taken from here, so the compiler reloads them
// with s_load after the walk instead of holding ~30 SGPRs of them live across it (the render
// kernels' SGPR budget decides 8 vs 7 waves per SIMD).  The empty asm hides the pointer's
// origin (a register round trip), so these loads cannot be merged with the kernel entry's.
// off: byte offset of the frame's KParams in the kernarg segment (0 for the single-frame
// kernels, whose first argument is the KParams; a frame of KBatch in the batch kernel).
__device__ __forceinline__ const KParams& late_params(const KParams& P, uint32_t off = 0u)
{
    (void)P;
    const uint64_t a = uint64_t(__builtin_amdgcn_kernarg_segment_ptr()) + off;
    uint32_t lo = uint32_t(a), hi = uint32_t(a >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    return *(const KParams *)(const __attribute__((address_space(4))) KParams *)((uint64_t(hi) << 32) | lo);
}

// Multi-frame launch (rt_render_batch_device): up to kMaxBatch frames -- of different scenes --
// in ONE grid, so one frame's tail overlaps the others' work and the heavy-first order ranks the
// blocks of all of them.  p[0] also carries the batch's heavy-first / wide-section state (its
// block and item indices are the launch's, frame-major); every other field is per frame.
// 6 frames keep KBatch (~3.6 KiB) inside the 4 KiB kernarg limit (static_assert below).
constexpr uint32_t kMaxBatch = 6;
struct KBatch
{
    KParams p[kMaxBatch];
    uint32_t nframes;
    uint32_t base[kMaxBatch + 1];   // first launch block of each frame; base[nframes] = all blocks
};

// The batch kernels' KBatch, re-read from the kernarg segment (as late_params).
__device__ __forceinline__ const KBatch& late_batch()
{
    const uint64_t a = uint64_t(__builtin_amdgcn_kernarg_segment_ptr());
    uint32_t lo = uint32_t(a), hi = uint32_t(a >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    return *(const KBatch *)(const __attribute__((address_space(4))) KBatch *)((uint64_t(hi) << 32) | lo);
}

// Frame of launch block b (wave-uniform).
__device__ __forceinline__ uint32_t batch_frame(const KBatch& B, uint32_t b)
{
    uint32_t f = 0;
    for (uint32_t j = 1; j < kMaxBatch; j++) f += (j < B.nframes && b >= B.base[j]) ? 1u : 0u;
    return f;
}

// Frames in the launch that starts at frame `start` of an n-frame batch: ceil(n / kMaxBatch)
// launches of near-equal size (10 frames: 5 + 5), each with one tail.  Mirrored by the binding's
// batch_chunks().
inline uint32_t batch_chunk_len(uint32_t n, uint32_t start)
{
    const uint32_t left = n - start, k = (left + kMaxBatch - 1u) / kMaxBatch;
    return (left + k - 1u) / k;
}

// CSR range of a cell: one u32 load of the packed (start << 11 | count) word when the scene
// fits the packing (every scene of the reference does), else the two CSR offsets.
__device__ __forceinline__ void cell_range(const KParams& P, uint32_t cell, uint32_t& kb, uint32_t& ke)
{
    if (P.cellw)
    {
        const uint32_t w = P.cellw[cell];
        const uint32_t cnt = w & 2047u;
        kb = cnt ? (w >> 11) : 0u;
        ke = kb + cnt;
    }
    else
    {
        kb = P.off[cell];
        ke = P.off[cell + 1];
    }
}

typedef float vf4 __attribute__((ext_vector_type(4)));
// constant address space: uniform loads of memory no store of the render kernels touches (frefs
// are written by k_origin_pre, an earlier launch) select s_load through the scalar cache
typedef const __attribute__((address_space(4))) vf4 cvf4;

// The wide section walks AUTO's box runs with per-lane jumps (1) or the octant cube words (0)
#ifndef RT_WIDE_BOX
#define RT_WIDE_BOX 1
#endif
// The per-lane list loop of the per-camera-record test: this lane's list [kb, ke) in order
// (grid.cpp:243-267), lowering tb on every accepted hit.  The first-half terms (r0..r2) per
// iteration, the second-half terms (r3) only when the gate passes.  Measured against a one-ahead
// prefetch in VGPRs (+12, 6 waves/SIMD) and by LDS-DMA into a per-wave slot
// (global_load_lds_dwordx4; no VGPRs, but four DMA issues per record): both slower on the frame
// and no shorter on the lone heavy waves (profiles/r02e_ab_lane_prefetch.json).
template <bool STATS, int VAR>
__device__ __forceinline__ void lane_list(const KParams& P, rtd::f2v ra, rtd::f2v rc, uint32_t kb, uint32_t ke,
                                          float& tb, float& u, float& v, uint32_t& tri, uint32_t& tests)
{
    constexpr bool F = (VAR & kVarFastRcp) != 0;
    for (uint32_t k = kb; k < ke; k++)
    {
        if constexpr ((VAR & kVarWaveClock) != 0)
            if (first_active_lane()) wave_counters()[1] += 1u;
        if (STATS) tests++;
        const float4 *rp = P.frefs + size_t(k) * 4u;     // one address, immediate offsets
        const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
        float inv, pu;
        const bool ok1 = rtd::mt_rec_first<F>(ra, rc, rtd::f2v{r0.x, r0.y}, rtd::f2v{r0.z, r0.w},
                                              rtd::f2v{r1.x, r1.y}, rtd::f2v{r1.z, r1.w},
                                              rtd::f2v{r2.x, r2.y}, inv, pu);
        if (__any(ok1))
        {
            const float2 r3 = *reinterpret_cast<const float2 *>(rp + 3);
            float pv, pt;
            const bool h = ok1 & rtd::mt_rec_second(ra, rc, rtd::f2v{r2.z, r2.w}, r3.x, r3.y, inv, pu, pv, pt);
            const bool take = h & (pt < tb);
            tb = take ? pt : tb;
            u = take ? pu : u;
            v = take ? pv : v;
            tri = take ? k : tri;
        }
    }
}

// Tests a cell's list [kb, ke) in order (grid.cpp:243-267); true when it produced a hit.
// grid.cpp:258-260 accepts cur_t when cur_t < t && cur_t < next_crossing_t[step_axis].  t is
// FLT_MAX on entry (a hit ends the walk, grid.cpp:270-271) and neither bound is ever NaN, so the
// two compares are one against tb = min(t, nct_ax), which every accepted hit lowers to its t:
// the same hits are taken in the same order (strict '<' keeps the first of equal t, H8).
template <bool STATS, int TRI, int VAR>
__device__ __forceinline__ bool test_cell(const KParams& P, float ox, float oy, float oz, float dx, float dy,
                                          float dz, uint32_t kb, uint32_t ke, float nct_ax, float& t,
                                          float& u, float& v, uint32_t& tri, uint32_t& tests)
{
    constexpr bool PRE = (VAR & kVarOriginPre) != 0 && TRI == RT_TRI_MOLLER_TRUMBORE;
    constexpr bool F = (VAR & kVarFastRcp) != 0;
    const rtd::f2v ra = {dx, dy}, rc = {dy, dz};   // the ray as the record test's register pairs
    // min(t, nct_ax) as a compare and select: neither is ever NaN (and -0 / +0 compare equal in
    // every later '<'), and fminf would canonicalise both operands first (2 more VALU per cell)
    const float tb0 = t < nct_ax ? t : nct_ax;
    // every accepted hit lowers tb strictly, so "some hit was taken" is tb < tb0; u, v and tri
    // are updated in place (the caller's values stand when nothing is taken)
    float tb = tb0;
    bool uniform_done = false;                // wave-uniform
    if constexpr ((VAR & kVarUniform) != 0 && PRE)
    {
        // Wave-uniform list: every lane testing this step sits in the same cell (the common case
        // in dense geometry: a wave is a 4x4-pixel x 4-sample block).  The loop runs on scalar
        // registers and the records arrive through the scalar cache (s_load), off the
        // vector-memory path; results are the same ray/record pairs in the same order.
        const uint32_t kb0 = __builtin_amdgcn_readfirstlane(kb), ke0 = __builtin_amdgcn_readfirstlane(ke);
        // one integer compare for the vote (the empty asm keeps the compiler from splitting it
        // back into two equalities, which materialises the combined predicate in a VGPR)
        uint32_t diff = (kb ^ kb0) | (ke ^ ke0);
        asm volatile("" : "+v"(diff));
        if (wave_all(diff == 0u))
        {
            if constexpr ((VAR & kVarWaveClock) != 0)
                if (first_active_lane()) wave_counters()[0] += ke0 - kb0;
            cvf4 *crefs = (cvf4 *)P.frefs;
            {
                // software pipeline over two register sets in turn: record k + 1 is in flight
                // while record k is tested, with no per-record register copies (scalar loads may
                // return out of order, so each set is waited for where it is first read)
                auto test_rec = [&](const vf4 r0, const vf4 r1, const vf4 r2, const vf4 r3, uint32_t k) {
                    if (STATS) tests++;
                    // the gate skips the record's second half AND the acceptance for the whole
                    // wave when no lane passes det and u (the common case in a dense cell)
                    float inv, cu;
                    const bool ok1 = rtd::mt_rec_first<F>(ra, rc, rtd::f2v{r0.x, r0.y}, rtd::f2v{r0.z, r0.w},
                                                          rtd::f2v{r1.x, r1.y}, rtd::f2v{r1.z, r1.w},
                                                          rtd::f2v{r2.x, r2.y}, inv, cu);
                    if (__any(ok1))
                    {
                        float cv, ct;
                        const bool hit = ok1 & rtd::mt_rec_second(ra, rc, rtd::f2v{r2.z, r2.w}, r3.x, r3.y, inv, cu,
                                                                  cv, ct);
                        const bool take = hit & (ct < tb);
                        tb = take ? ct : tb;
                        u = take ? cu : u;
                        v = take ? cv : v;
                        tri = take ? k : tri;
                    }
                };
                cvf4 *np = crefs + size_t(kb0) * 4u;
                vf4 a0 = np[0], a1 = np[1], a2 = np[2], a3 = np[3];
                for (uint32_t k = kb0;; k += 2u)
                {
                    vf4 b0, b1, b2, b3;
                    const bool more1 = k + 1u < ke0;
                    if (more1)
                    {
                        np = crefs + size_t(k + 1u) * 4u;
                        b0 = np[0];
                        b1 = np[1];
                        b2 = np[2];
                        b3 = np[3];
                    }
                    test_rec(a0, a1, a2, a3, k);
                    if (!more1) break;
                    const bool more2 = k + 2u < ke0;
                    if (more2)
                    {
                        np = crefs + size_t(k + 2u) * 4u;
                        a0 = np[0];
                        a1 = np[1];
                        a2 = np[2];
                        a3 = np[3];
                    }
                    test_rec(b0, b1, b2, b3, k + 1u);
                    if (!more2) break;
                }
            }
            uniform_done = true;
        }
    }
    if constexpr (PRE)
    {
        if (!uniform_done) lane_list<STATS, VAR>(P, ra, rc, kb, ke, tb, u, v, tri, tests);
    }
    else
    for (uint32_t k = kb; k < ke; k++)
    {
        if (STATS) tests++;
        const float4 *rp = P.refs + size_t(k) * 3;          // one address, immediate offsets
        const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
        float ct, cu, cv;
        bool hit;
        const uint32_t id = __float_as_uint(r2.y);
        if (TRI == RT_TRI_BARYCENTRIC)
        {
            const float4 fn = P.face_n[id];
            hit = rtd::ray_tri_bary_pred(ox, oy, oz, dx, dy, dz, r0.x, r0.y, r0.z, r0.w, r1.x,
                                         r1.y, r1.z, r1.w, r2.x, fn.x, fn.y, fn.z, ct, cu, cv);
        }
        else if (VAR & kVarWaveGate)
            hit = rtd::ray_tri_mt_gated(ox, oy, oz, dx, dy, dz, r0.x, r0.y, r0.z, r0.w, r1.x,
                                        r1.y, r1.z, r1.w, r2.x, ct, cu, cv);
        else
            hit = rtd::ray_tri_mt_pred(ox, oy, oz, dx, dy, dz, r0.x, r0.y, r0.z, r0.w, r1.x,
                                       r1.y, r1.z, r1.w, r2.x, ct, cu, cv);
        const bool take = hit & (ct < tb);                     // grid.cpp:258-260
        tb = take ? ct : tb;
        u = take ? cu : u;
        v = take ? cv : v;
        tri = take ? id : tri;
    }
    t = tb < tb0 ? tb : t;
    return t != rtd::kFltMax;                                  // grid.cpp:270-271
}

// One DDA advance over plain local variables (grid.cpp:236-239 + 274-277), exact because
// untouched axes keep their values.  A macro, not a member function or a capturing lambda:
// selecting between struct fields through `this`/references becomes a pointer select, which
// defeats SROA and put the walk state in LDS/scratch (measured).
// Step axis of grid.cpp:236-239 restated: with m = min(nct), the nested strict '<' chain picks
// the HIGHEST axis index among those equal to m (all 7 tie patterns checked), so
// a2 = nct2 == m, a1 = !a2 && nct1 == m, else a0.  nct is never NaN (finite setup, FLT_MAX for
// zero components).  Each crossing time advances as nct_a + (a ? dt_a : 0.0f): the step axis
// gets the reference's single IEEE add (grid.cpp:277), and x + 0.0f == x for every value nct
// takes (finite or +inf, never -0 or NaN: every setup term is >= 0, see dda_setup).  The state
// updates run unconditionally -- when MORE is false the caller breaks and the state is dead --
// so the step has no divergent branch.  Sets NCT_AX to the step axis' crossing t and MORE to
// false when the ray leaves the grid (grid.cpp:275-276).
#define RT_DDA_ADVANCE_ADD(NCT_AX, MORE)                                                       \
    do {                                                                                       \
        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);                   \
        const bool a2_ = nct2 == m_;                                                           \
        const bool a1_ = !a2_ && nct1 == m_;                                                   \
        const bool a0_ = !a2_ && !a1_;                                                         \
        NCT_AX = m_;                                                                           \
        MORE = (a2_ ? rem2 : (a1_ ? rem1 : rem0)) != 0;                                        \
        nct0 += a0_ ? dt0 : 0.0f;                                                              \
        nct1 += a1_ ? dt1 : 0.0f;                                                              \
        nct2 += a2_ ? dt2 : 0.0f;                                                              \
        rem0 -= int(a0_); rem1 -= int(a1_); rem2 -= int(a2_);                                  \
        cell += a2_ ? cs2 : (a1_ ? cs1 : cs0);                                                 \
    } while (0)

// RT_DDA_ADVANCE_ADD with the three remaining-cell counts packed into one word: rem0 in bits
// 0-9, rem1 in 11-20, rem2 in 22-30, guard bits 10, 21, 31 (needs dims <= 512; rt_scene::
// pack_ok).  The step subtracts the axis unit unconditionally; a count that was 0 borrows into
// its guard bit, so MORE = no guard bit set == (rem of the step axis != 0) -- the walk exits
// exactly where RT_DDA_ADVANCE_ADD's does (the borrowed state is dead after the exit).
constexpr int kRemGuards = int((1u << 10) | (1u << 21) | (1u << 31));
#define RT_DDA_ADVANCE_PACKED(NCT_AX, MORE)                                                    \
    do {                                                                                       \
        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);                   \
        const bool a2_ = nct2 == m_;                                                           \
        const bool a1_ = !a2_ && nct1 == m_;                                                   \
        const bool a0_ = !a2_ && !a1_;                                                         \
        NCT_AX = m_;                                                                           \
        remp -= a2_ ? (1 << 22) : (a1_ ? (1 << 11) : 1);                                       \
        MORE = (remp & kRemGuards) == 0;                                                       \
        nct0 += a0_ ? dt0 : 0.0f;                                                              \
        nct1 += a1_ ? dt1 : 0.0f;                                                              \
        nct2 += a2_ ? dt2 : 0.0f;                                                              \
        cell += a2_ ? cs2 : (a1_ ? cs1 : cs0);                                                 \
    } while (0)

// RT_DDA_ADVANCE_PACKED without the exit test: a step inside a proven-empty run (the
// empty-run blocks of grid_intersect read MORE from the packed word after the block).
#define RT_DDA_BARE_STEP()                                                                     \
    do {                                                                                       \
        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);                   \
        const bool a2_ = nct2 == m_;                                                           \
        const bool a1_ = !a2_ && nct1 == m_;                                                   \
        const bool a0_ = !a2_ && !a1_;                                                         \
        remp -= a2_ ? (1 << 22) : (a1_ ? (1 << 11) : 1);                                       \
        nct0 += a0_ ? dt0 : 0.0f;                                                              \
        nct1 += a1_ ? dt1 : 0.0f;                                                              \
        nct2 += a2_ ? dt2 : 0.0f;                                                              \
        cell += a2_ ? cs2 : (a1_ ? cs1 : cs0);                                                 \
    } while (0)

// Empty-run steps in blocks with one vote per block (1) or one vote per step (0, the round-2 loop)
#ifndef RT_SKIP_BLOCKS
#define RT_SKIP_BLOCKS 1
#endif
// spp 4: the pixel's quad resolves one channel per lane (1) or its first lane all three (0)
#ifndef RT_QUAD_RESOLVE
#define RT_QUAD_RESOLVE 1
#endif
// AUTO's empty runs over the box-run words (1, build_box_words) or the octant cube words (0)
#ifndef RT_BOX_RUN
#define RT_BOX_RUN 1
#endif
// AUTO's box runs (grid_intersect): 0 wave-uniform bare steps while every lane is inside its box
// (lock-step), 1 per lane (each lane jumps to just before its own box exit: per-axis add chains),
// 2 time-synchronised (every lane to the wave's lowest exit bound), 3 per lane up to the wave's
// first contact, lock-step after it, 4 as 3 with time-synchronised runs after it, 5 as 3 with a new
// approach whenever the whole wave is inside boxes again
#ifndef RT_LANE_RUNS
#define RT_LANE_RUNS 3
#endif

// The box-run walk's step: RT_DDA_ADVANCE_PACKED, with the step axis' unit also taken from the
// box counts (boxw, build_box_words' empty-cell layout = the packed counts' layout): a count
// that was 0 borrows into its guard bit when the step leaves the box.
#define RT_DDA_ADVANCE_BOX(NCT_AX, MORE)                                                       \
    do {                                                                                       \
        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);                   \
        const bool a2_ = nct2 == m_;                                                           \
        const bool a1_ = !a2_ && nct1 == m_;                                                   \
        const bool a0_ = !a2_ && !a1_;                                                         \
        NCT_AX = m_;                                                                           \
        const int u_ = a2_ ? (1 << 22) : (a1_ ? (1 << 11) : 1);                                \
        remp -= u_;                                                                            \
        boxw -= u_;                                                                            \
        MORE = (remp & kRemGuards) == 0;                                                       \
        nct0 += a0_ ? dt0 : 0.0f;                                                              \
        nct1 += a1_ ? dt1 : 0.0f;                                                              \
        nct2 += a2_ ? dt2 : 0.0f;                                                              \
        cell += a2_ ? cs2 : (a1_ ? cs1 : cs0);                                                 \
    } while (0)
// A step inside a box run: only the crossing times and the box counts move; the run's end
// rebuilds the cell index and the remaining-cell counts from the box counts' difference.
#define RT_DDA_BOX_BARE_STEP()                                                                 \
    do {                                                                                       \
        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);                   \
        const bool a2_ = nct2 == m_;                                                           \
        const bool e1_ = nct1 == m_;                                                           \
        boxw -= a2_ ? (1 << 22) : (e1_ ? (1 << 11) : 1);                                       \
        nct0 += (a2_ | e1_) ? 0.0f : dt0;                                                      \
        nct1 += (e1_ & !a2_) ? dt1 : 0.0f;                                                     \
        nct2 += a2_ ? dt2 : 0.0f;                                                              \
    } while (0)
constexpr int kBoxUnits3 = 3 | (3 << 11) | (3 << 22);   // 3 in every box-count field

// A lower bound of x(f) = the add chain x, fl(x + dt), ... after f steps (a box run's exit crossing
// along one axis; grid_intersect's per-lane runs).  Only compared against crossing times, never part
// of a pixel's arithmetic: its two explicit FMAs (the fused f dt + x, and the margin) are the
// only ones outside rtd::rcp_nr (tests/test_build_guard.py).  A still axis (x = FLT_MAX, dt = 0)
// gives ~FLT_MAX.
__device__ __forceinline__ float box_exit_bound(float x, float dtv, int f)
{
    const float e = __builtin_fmaf(float(f), dtv, x), k = float(f + 2) * 0x1p-23f;
    return e - __builtin_fmaf(__builtin_fabsf(x), k, __builtin_fabsf(e) * k);
}

// Grid entry + per-axis DDA setup of Grid::Intersect (aabb.h:9-83, grid.h:44-51,
// grid.cpp:174-216), axis arrays unrolled into scalars.  Instead of pos/step/out per axis the
// walk keeps the cells left before 'pos == out' (rem) and the signed GridIdx stride of a step
// (cs): grid.cpp:274-277 exits after the same steps.  False when the ray misses the grid.
__device__ __forceinline__ bool dda_setup(const KParams& P, float ox, float oy, float oz, float dx, float dy, float dz,
                                          float& nct0, float& nct1, float& nct2, float& dt0, float& dt1, float& dt2,
                                          int& rem0, int& rem1, int& rem2, int& cs0, int& cs1, int& cs2, int& cell)
{
    float enter_t, leave_t, gx, gy, gz;
    if (rtd::point_in_aabb(ox, oy, oz, P.bmin, P.bmax))
    {
        enter_t = 0.0f;
        gx = ox; gy = oy; gz = oz;
    }
    else if (rtd::ray_aabb(ox, oy, oz, dx, dy, dz, P.bmin, P.bmax, enter_t, leave_t))
    {
        gx = ox + dx * enter_t;
        gy = oy + dy * enter_t;
        gz = oz + dz * enter_t;
    }
    else
        return false;

    // grid.h:44-48 ToVoxel, grid.h:50-51 ToPos, grid.cpp:190-216 per-axis setup
    auto to_voxel = [&](float g, int a) {
        const int vx = rtd::cvt_i32_x86((g - P.bmin[a]) * P.icw);
        const int hi = P.dim[a] - 1;
        return vx < 0 ? 0 : (vx > hi ? hi : vx);
    };
    const int pos0 = to_voxel(gx, 0), pos1 = to_voxel(gy, 1), pos2 = to_voxel(gz, 2);
    dt0 = dt1 = dt2 = 0.0f;
    rem0 = rem1 = rem2 = cs0 = cs1 = cs2 = 0;
    auto setup = [&](float d, float g, int pos, int a, int stride, float& nct, float& dtv, int& rem, int& cs) {
        if (d == 0.0f)
            nct = rtd::kFltMax;
        else if (d > 0.0f)
        {
            nct = enter_t + ((P.bmin[a] + float(pos + 1) * P.cw) - g) / d;
            dtv = P.cw / d;
            rem = P.dim[a] - 1 - pos;           // steps until pos + 1 == dim
            cs = stride;
        }
        else
        {
            nct = enter_t + ((P.bmin[a] + float(pos) * P.cw) - g) / d;
            dtv = -P.cw / d;
            rem = pos;                          // steps until pos - 1 == -1
            cs = -stride;
        }
    };
    setup(dx, gx, pos0, 0, 1, nct0, dt0, rem0, cs0);
    setup(dy, gy, pos1, 1, P.dxdz, nct1, dt1, rem1, cs1);
    setup(dz, gz, pos2, 2, P.dim[0], nct2, dt2, rem2, cs2);
    cell = pos0 + pos2 * P.dim[0] + pos1 * P.dxdz;
    return true;
}

// Offset of the ray's octant copy in P.cellwo (0 when there is one copy).  An axis with d == 0
// never steps, so either sign is right for it (-0.0 counts as +).
__device__ __forceinline__ int oct_offset(const KParams& P, float dx, float dy, float dz)
{
    const uint32_t o = uint32_t(dx < 0.0f) | (uint32_t(dy < 0.0f) << 1) | (uint32_t(dz < 0.0f) << 2);
    return int(o * P.oct_stride);
}

// Offset of the ray's box-run copy in P.cellwb: octant (as oct_offset) x 3 + major axis (the
// largest |d| component; any choice is exact, the copy only shapes the boxes for speed).
__device__ __forceinline__ int box_offset(const KParams& P, float dx, float dy, float dz)
{
    const uint32_t o = uint32_t(dx < 0.0f) | (uint32_t(dy < 0.0f) << 1) | (uint32_t(dz < 0.0f) << 2);
    const float ax = __builtin_fabsf(dx), ay = __builtin_fabsf(dy), az = __builtin_fabsf(dz);
    const uint32_t m = (ax >= ay && ax >= az) ? 0u : (ay >= az ? 1u : 2u);
    return int((o * 3u + m) * P.box_stride);
}

// Records of the product walks (rt_render_records_device): the GridIdx of the last cell walked on a
// miss, from the state the walk ends in.  The exit step along axis a borrowed into the guard bit of
// a's packed remaining-cell count -- the LOWEST set guard, since a borrow only carries upward -- and
// `cell` already includes that step.  The walk itself is unchanged: this runs after it, and only a
// record store reads the result.
constexpr uint32_t kVoxelUnknown = 0xFFFFFFFEu;     // not recoverable from this walk's end state
__device__ __forceinline__ uint32_t exit_voxel(int remp, int cell, int cs0, int cs1, int cs2)
{
    const uint32_t g = uint32_t(remp) & uint32_t(kRemGuards);
    return uint32_t(cell - ((g & (1u << 10)) ? cs0 : ((g & (1u << 21)) ? cs1 : cs2)));
}

// The cell whose CSR list holds reference k: off[c] <= k < off[c + 1] (records of a hit: the walk
// accepts a hit only inside the cell being tested, grid.cpp:258-271, so this is that cell).
__device__ __forceinline__ uint32_t cell_of_ref(const KParams& P, uint32_t k)
{
    uint32_t lo = 0u, hi = uint32_t(P.dim[0]) * uint32_t(P.dim[1]) * uint32_t(P.dim[2]);   // off[hi] = R > k
    while (hi - lo > 1u)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (P.off[mid] <= k) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The colour words of a record (the wide section stores them after its resolve).
__device__ __forceinline__ void store_record_colour(const KParams& Q, uint32_t px, uint32_t py, uint32_t s, float r,
                                                    float g, float b)
{
    const uint32_t rx = px - Q.rec_x0, ry = py - Q.rec_y0;
    if (rx >= Q.rec_w || ry >= Q.rec_h) return;
    volatile uint32_t *o = reinterpret_cast<volatile uint32_t *>(Q.recs + (size_t(ry) * Q.rec_w + rx) * Q.spp + s);
    o[8] = __float_as_uint(r);
    o[9] = __float_as_uint(g);
    o[10] = __float_as_uint(b);
}

// One per-sample record (rt_sample_rec) of a product kernel, for samples inside the requested
// rectangle: rec[((y - y0) * w + (x - x0)) * spp + s], in RAW form -- what the walk leaves, with no
// extra lookups in the product kernels (their register budget decides their occupancy): a hit's CSR
// reference (tri word), a miss's end cell as the walk holds it (voxel word, still inside its copy of
// the cell words).  k_record_fixup then maps the reference to Grid::Intersect's tri_idx and the cell
// it lies in, and moves a raw end cell out of its copy (kRecRaw* in the pad word).  DDA steps and
// tests are not counted by the product walks (0xFFFFFFFF; k_trace_records pins them).
constexpr uint32_t kRecMagic = 0xF1A90000u;     // pad word of a raw record (a -1-filled word is not)
constexpr uint32_t kRecRawCsr = 1u;             // tri word = CSR reference of the hit
constexpr uint32_t kRecRawBox = 2u;             // voxel word = end cell in the ray's box-word copy
constexpr uint32_t kRecRawOct = 4u;             // voxel word = end cell in the ray's octant copy
__device__ __forceinline__ void store_record(const KParams& Q, uint32_t px, uint32_t py, uint32_t s, bool hit,
                                             uint32_t tri, uint32_t voxel, float t, float u, float v, uint32_t raw)
{
    const uint32_t rx = px - Q.rec_x0, ry = py - Q.rec_y0;
    if (rx >= Q.rec_w || ry >= Q.rec_h) return;
    // word by word (volatile: no dwordx4 merging, which needs consecutive VGPRs)
    volatile uint32_t *o = reinterpret_cast<volatile uint32_t *>(Q.recs + (size_t(ry) * Q.rec_w + rx) * Q.spp + s);
    o[0] = hit ? 1u : 0u;
    o[1] = hit ? tri : rtd::kNoTri;
    o[2] = hit ? rtd::kNoTri : voxel;
    o[3] = 0xFFFFFFFFu;
    o[4] = 0xFFFFFFFFu;
    o[5] = hit ? __float_as_uint(t) : 0u;
    o[6] = hit ? __float_as_uint(u) : 0u;
    o[7] = hit ? __float_as_uint(v) : 0u;
    o[11] = kRecMagic | (hit ? (raw & kRecRawCsr) : (raw & ~kRecRawCsr));
}

// grid.cpp:159-281 Grid::Intersect (NEW_GRID_TRAVERSAL), axis arrays unrolled into scalars
// so nothing is runtime-indexed (no scratch).  Counters are compiled in only for records.
template <bool STATS, int TRI, int VAR>
__device__ __forceinline__ bool grid_intersect(const KParams& P, float ox, float oy, float oz,
                                               float dx, float dy, float dz,
                                               float& t, float& u, float& v, uint32_t& tri,
                                               uint32_t& voxel, uint32_t& steps, uint32_t& tests)
{
    float nct0, nct1, nct2, dt0, dt1, dt2;
    int rem0, rem1, rem2, cs0, cs1, cs2, cell;
    if (!dda_setup(P, ox, oy, oz, dx, dy, dz, nct0, nct1, nct2, dt0, dt1, dt2, rem0, rem1, rem2, cs0, cs1, cs2,
                   cell))
        return false;
    t = rtd::kFltMax;

#if RT_BOX_RUN
    if constexpr ((VAR & kVarSkipRun) != 0 && (VAR & kVarPackedRem) != 0)
    {
        // Box runs (AUTO; build_box_words): a looked-up empty cell hands the lane an empty box
        // (its corner at the cell, extending along the ray's octant) as per-axis step counts in
        // the packed counts' layout.  Every step takes its axis unit from both words; while no
        // box count has borrowed, the lane is inside the box and its cell is empty: no lookup,
        // no test.  A non-empty cell's word leaves boxw = 0, so the next step borrows and looks
        // the next cell up.  Same cells in the same order, same tests: only lookups of
        // proven-empty cells are skipped.  Termination as below: every iteration that does not
        // exit decrements a positive remaining-cell count.
        int remp = rem0 | (rem1 << 11) | (rem2 << 22);
        int boxw = kRemGuards;                              // no box yet: look the first cell up
        const int coff = box_offset(P, dx, dy, dz);
        cell += coff;
        constexpr int kLaneRuns = STATS ? 0 : RT_LANE_RUNS;
        bool sync = kLaneRuns < 3;                          // wave-uniform (RT_LANE_RUNS 3-5)
        for (;;)
        {
            if (STATS) { voxel = uint32_t(cell - coff); steps++; }
            uint32_t kb = 0, ke = 0;
            float nct_ax;
            bool more;
            if ((boxw & kRemGuards) != 0)
            {
                const uint32_t w = P.cellwb[uint32_t(cell)];
                const uint32_t ne = uint32_t(int(w) >> 31);           // all ones: a non-empty cell
                kb = (w >> 11) & 0xFFFFFu;
                ke = kb + (w & ne & 2047u);
                boxw = int(w & ~ne);
            }
            if (kLaneRuns >= 3 && !sync)
            {
                // Approach (RT_LANE_RUNS 3-5): per-lane box runs up to each lane's first non-empty
                // cell, where the lane waits (no step, no test; the cell is looked up again)
                // until every active lane of the wave is at its own: from then on the wave walks
                // in lock-step, so rays of a wave that cross the same cells test them together
                // (wave-uniform lists).  Waiting changes no lane's walk, only when it is taken.
                if (wave_all(kb < ke))
                    sync = true;
                else if (kb < ke)
                {
                    boxw = kRemGuards;
                    continue;
                }
            }
            RT_DDA_ADVANCE_BOX(nct_ax, more);
            bool hit = false;
            if (kb < ke) hit = test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests);
            if constexpr (!STATS)
            {
                const bool inside = (uint32_t(boxw) & uint32_t(kRemGuards)) == 0u;
                const bool approach = kLaneRuns == 1 || (kLaneRuns >= 3 && !sync);
                bool lane_run = approach && inside;
                bool wave_run = !approach && wave_all(inside);     // wave-uniform
                if (kLaneRuns == 5 && wave_run)
                {
                    // (5) the whole wave inside boxes again: a new approach
                    lane_run = true;
                    wave_run = false;
                    sync = false;
                }
                constexpr bool kTsync = kLaneRuns == 2 || kLaneRuns == 4;
                if (lane_run || (kTsync && wave_run))
                {
                    // Per-lane box runs (1; 3 before the wave's first contact).  Inside a box the
                    // three crossing-time sequences are independent add chains
                    // x_a(k+1) = fl(x_a(k) + dt_a), and the box is left at the first of the
                    // (f_a + 1)-th crossings E_a = x_a(f_a) (f_a = the box field).  tl is a lower
                    // bound of every E_a: f dt + x fused (one rounding) is within 2^-24 |.| of it, the
                    // chain within f 2^-24 max|x_k| <= f 2^-24 (|x| + |E|) of it, so
                    // E_a >= e_a - (f_a + 2) 2^-23 (|e_a| + |x_a|) with room for the bound's own
                    // roundings.  Each axis then takes its crossings below tl (at most f_a of
                    // them): every taken crossing is < tl <= every untaken one, so these are
                    // exactly the walk's next sum c_a steps, in some order, all inside the box
                    // (empty cells, no test, no exit).  Bare steps then run to the box's exit
                    // (normally one) -- the same cells, crossing times and exits as one step per
                    // cell.  A lane that hit or left the grid holds a borrowed guard.
                    // Time-synchronised runs (2): while every lane is inside its box, all lanes
                    // take their crossings below the wave's lowest bound, then bare steps run
                    // wave-uniformly to the first lane's box exit.
                    const uint32_t b0 = uint32_t(boxw);
                    const int f0 = boxw & 1023, f1 = (boxw >> 11) & 1023, f2 = int(uint32_t(boxw) >> 22);
                    float tl = __builtin_fminf(__builtin_fminf(box_exit_bound(nct0, dt0, f0), box_exit_bound(nct1, dt1, f1)),
                                               box_exit_bound(nct2, dt2, f2));
                    if (kTsync && wave_run) tl = wave_min_active(tl);
                    int c0 = 0, c1 = 0, c2 = 0;
                    while (nct0 < tl && c0 < f0) { nct0 += dt0; c0++; }
                    while (nct1 < tl && c1 < f1) { nct1 += dt1; c1++; }
                    while (nct2 < tl && c2 < f2) { nct2 += dt2; c2++; }
                    boxw -= c0 + (c1 << 11) + (c2 << 22);
                    if (kTsync && wave_run)
                        do
                            RT_DDA_BOX_BARE_STEP();
                        while (wave_all((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u));
                    else
                        do
                            RT_DDA_BOX_BARE_STEP();
                        while ((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u);
                    const uint32_t d = b0 - uint32_t(boxw);
                    remp = int(uint32_t(remp) - d);           // wrapping (d may reach 2^31)
                    cell += int(d & 2047u) * cs0 + int((d >> 11) & 2047u) * cs1 + int(d >> 22) * cs2;
                    more = (remp & kRemGuards) == 0;
                }
                else if (wave_run)
                {
                    // Wave-uniform runs while every active lane is inside its box (the boxes are
                    // clipped to the grid, so inside the box is inside the grid): blocks of 4 bare
                    // steps while every box count of every lane is >= 3 (the first three steps of a
                    // block stay inside; the fourth may leave, which the next vote sees), then
                    // single steps.  A bare step moves only the crossing times and boxw; the run's
                    // end rebuilds the cell index and the remaining-cell counts from the box
                    // counts' difference, which is sum n_a * unit_a over the run's n_a steps along
                    // axis a (n_a <= 1024, 1024, 512: no field of the difference carries).  A lane
                    // that hit holds boxw < 0 (guard set), so runs only start when no lane hit.
                    // (if + do-while: a while loop's exit edge made the compiler copy the whole
                    // walk state every iteration.)
                    const uint32_t b0 = uint32_t(boxw);
                    if (wave_all((uint32_t(boxw - kBoxUnits3) & uint32_t(kRemGuards)) == 0u))
                        do
                        {
                            RT_DDA_BOX_BARE_STEP();
                            RT_DDA_BOX_BARE_STEP();
                            RT_DDA_BOX_BARE_STEP();
                            RT_DDA_BOX_BARE_STEP();
                        } while (wave_all((uint32_t(boxw - kBoxUnits3) & uint32_t(kRemGuards)) == 0u));
                    if (wave_all((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u))
                        do
                            RT_DDA_BOX_BARE_STEP();
                        while (wave_all((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u));
                    const uint32_t d = b0 - uint32_t(boxw);
                    remp = int(uint32_t(remp) - d);           // wrapping (d may reach 2^31)
                    cell += int(d & 2047u) * cs0 + int((d >> 11) & 2047u) * cs1 + int(d >> 22) * cs2;
                    more = (remp & kRemGuards) == 0;
                }
            }
            if (hit | !more) break;
        }
        // records only: the exit cell in the ray's box-word copy (trace_sample removes the copy's
        // offset, so nothing extra is live across the walk)
        if constexpr (!STATS) voxel = exit_voxel(remp, cell, cs0, cs1, cs2);
        return t != rtd::kFltMax;                            // t is only set by a hit
    }
#endif

    if (P.cellw && (VAR & kVarDistSkip))
    {
        // Distance skipping: after an empty cell at L-inf distance d from geometry the next
        // d-1 cells of the walk are provably empty, so they take the DDA step only.
        // Termination: every iteration that does not exit decrements a positive rem (the step
        // axis' count; MORE is false when it is 0), so a walk ends within rem0+rem1+rem2+1
        // iterations whatever nct holds.
        int skip = 0;
        int remp = rem0 | (rem1 << 11) | (rem2 << 22);      // kVarPackedRem only
        const int coff = oct_offset(P, dx, dy, dz);
        cell += coff;
        for (;;)
        {
            if (STATS) { voxel = uint32_t(cell - coff); steps++; }
            uint32_t kb = 0, ke = 0;
            float nct_ax;
            bool more;
            if (skip == 0)
            {
                const uint32_t w = P.cellwo[uint32_t(cell)];
                const uint32_t cnt = w & 2047u;
                kb = w >> 11;
                ke = kb + cnt;
                skip = cnt ? 0 : int(kb) - 1;
            }
            else
                skip--;
            if (VAR & kVarPackedRem)
                RT_DDA_ADVANCE_PACKED(nct_ax, more);
            else
                RT_DDA_ADVANCE_ADD(nct_ax, more);
            // one exit test per iteration (a hit, or the grid's end here or in the empty run
            // below), and the result read from t after the loop: the walk's loop-carried state
            // stays in VGPRs instead of per-exit lane masks (SALU per wave, PMC-measured)
            bool hit = false;
            if (kb < ke) hit = test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests);
            bool done = hit | !more;
            if constexpr ((VAR & kVarSkipRun) != 0 && (VAR & kVarPackedRem) != 0 && !STATS)
            {
                // Wave-uniform empty run: while every active lane is inside a run of cells the
                // distance field proves empty, the wave takes bare DDA steps -- the same advances
                // and the same exits as one iteration per cell, with no cell word or test work.
                // Uniform, so no lane waits on another's run; the run ends when the first lane's
                // does.  (A lane inside a run has no hit and more == true, so done is false.)
                if (wave_all(skip > 0))
                {
#if RT_SKIP_BLOCKS
                    // Blocks of 4, then 2, then 1 bare steps: one vote per block instead of one per
                    // step, and no exit test inside a block.  A lane that leaves the grid inside a
                    // block keeps stepping to the block's end, harmlessly: its state is dead (the
                    // walk ends with no further lookup), and the borrow into a guard bit is sticky
                    // for far more steps than a block holds (a field must count down 2^10 / 2^9
                    // more times to clear it), so MORE read after the block is the exit test.  The
                    // vote also requires every lane inside the grid: a lane with MORE false at the
                    // entry (it left the grid on an empty cell's step) takes no block.
                    auto run_ok = [&](int n) {    // (skip >= n) & more, as ONE integer compare
                        return wave_all(((uint32_t(remp) & uint32_t(kRemGuards)) | (uint32_t(skip - n) & 0x80000000u)) ==
                                        0u);
                    };
                    while (run_ok(4))
                    {
                        RT_DDA_BARE_STEP();
                        RT_DDA_BARE_STEP();
                        RT_DDA_BARE_STEP();
                        RT_DDA_BARE_STEP();
                        skip -= 4;
                    }
                    if (run_ok(2))
                    {
                        RT_DDA_BARE_STEP();
                        RT_DDA_BARE_STEP();
                        skip -= 2;
                    }
                    if (run_ok(1))
                    {
                        RT_DDA_BARE_STEP();
                        skip -= 1;
                    }
                    more = (remp & kRemGuards) == 0;
#else
                    do
                    {
                        skip--;
                        const float m_ = __builtin_fminf(__builtin_fminf(nct0, nct1), nct2);
                        const bool a2_ = nct2 == m_;
                        const bool a1_ = !a2_ && nct1 == m_;
                        const bool a0_ = !a2_ && !a1_;
                        remp -= a2_ ? (1 << 22) : (a1_ ? (1 << 11) : 1);
                        more = (remp & kRemGuards) == 0;
                        nct0 += a0_ ? dt0 : 0.0f;
                        nct1 += a1_ ? dt1 : 0.0f;
                        nct2 += a2_ ? dt2 : 0.0f;
                        cell += a2_ ? cs2 : (a1_ ? cs1 : cs0);
                        // (skip > 0) & more as ONE integer compare (skip >= 0 here)
                    } while (wave_all(((uint32_t(remp) & uint32_t(kRemGuards)) | (uint32_t(skip - 1) & 0x80000000u)) ==
                                      0u));
#endif
                    done = !more;
                }
            }
            if (done) break;
        }
        // a lane leaving the grid inside a block of bare steps stepped on: its last cell is lost
        if constexpr (!STATS)
        {
            if constexpr ((VAR & kVarSkipRun) != 0) voxel = kVoxelUnknown;
            else if constexpr ((VAR & kVarPackedRem) != 0) voxel = exit_voxel(remp, cell - coff, cs0, cs1, cs2);
            else voxel = uint32_t(cell - coff - (rem0 < 0 ? cs0 : (rem1 < 0 ? cs1 : cs2)));   // rem_a went to -1
        }
        return t != rtd::kFltMax;                            // t is only set by a hit
    }

    // One cell per iteration with its CSR range (the plain LANES arm, and scenes whose cell
    // lists do not fit the packed word).  max_steps = dims sum + 3 bounds it redundantly.
    for (uint32_t iter = 0; iter < P.max_steps; iter++)
    {
        if (STATS) { voxel = uint32_t(cell); steps++; }
        // Issue the CSR range loads first; the step's ALU work below overlaps their latency.
        uint32_t kb = 0, ke = 0;
        cell_range(P, uint32_t(cell), kb, ke);
        float nct_ax;
        bool more;
        RT_DDA_ADVANCE_ADD(nct_ax, more);
        if (kb < ke && test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests))
            return true;
        if (!more) break;
    }
    if constexpr (!STATS) voxel = uint32_t(cell - (rem0 < 0 ? cs0 : (rem1 < 0 ? cs1 : cs2)));   // records only
    return false;
}

// Renderer::IntersectBruteForce (renderer.cpp:157-197): every triangle in index order, the
// closest accepted hit wins, ties keep the lower index (strict '<', :187).  All lanes of a wave
// walk the same triangle sequence, so the records arrive through wave-uniform (scalar) loads
// and the wave-gated test skips a triangle's second half when no lane can still hit it.
template <bool STATS>
__device__ __forceinline__ bool brute_intersect(const KParams& P, float ox, float oy, float oz, float dx, float dy,
                                                float dz, float& t, float& u, float& v, uint32_t& tri,
                                                uint32_t& tests)
{
    t = rtd::kFltMax;
    for (uint32_t i = 0; i < P.ntris; i++)
    {
        const float4 a = P.tri_mt[3 * i + 0], b = P.tri_mt[3 * i + 1], c = P.tri_mt[3 * i + 2];
        float ct = 0.0f, cu = 0.0f, cv = 0.0f;
        const bool h = rtd::ray_tri_mt_gated(ox, oy, oz, dx, dy, dz, a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x,
                                             ct, cu, cv);
        if (h && ct < t)
        {
            t = ct;
            u = cu;
            v = cv;
            tri = i;
        }
    }
    if (STATS) tests = P.ntris;
    return t != rtd::kFltMax;
}

// Renderer::RayMarch (renderer.cpp:24-41) over Renderer::DistanceBruteForce (:138-155):
// sphere tracing from the camera, at most 128 steps, hit when a step's distance < 0.001.
//
// DistanceBruteForce is a minimum, and the minimum of a set does not depend on the order it
// is taken in ((d < dist) ? d : dist never selects a NaN, ties have equal values), so any
// triangle whose computed distance is provably above the minimum can be skipped, and any member
// may seed it, without changing a bit.  The records are Morton-sorted into blocks of kDistBlock
// triangles with an exact float AABB.  Error model: every computed DistancePointTri is the
// distance to a point of the triangle (the inside branch's convex combination or a clamped
// segment point) up to ~10 ulp of (|p| + |v|); float box distances are off by a few ulp of the
// same scale.  margin = 1e-5 * (|p|_inf + scene_scale) (>= 166 ulp) therefore gives
//   lb(block) - margin <= every computed distance of the block's triangles.
// Per step and lane: the minimum is seeded with the computed distance to the lane's previous
// nearest triangle, blocks are swept outward from that triangle's block (lane 0's), and a block
// is skipped when lb - margin > running minimum for every active lane (wave-uniform branch).
//
// Miss early-out: once p is outside the vertex AABB with box distance Db, receding from it at a
// rate r = dir . (p - clamp(p)) / Db >= 2e-5, and Db > 1.00001 * (margin + 0.001), every later
// point p' = p + s * dir has Db' >= Db + r s and margin' <= margin + 1e-5 s (|dir| <= 1), so
// every later computed distance exceeds 0.001: the reference marches to its 128-step limit
// without a hit (renderer.cpp:30-40).  The march stops there and reports exactly that.
__device__ __forceinline__ void march_eval_block(const KParams& P, uint32_t b, float px, float py, float pz,
                                                 float& dist, uint32_t& best_k)
{
    const uint32_t k0 = b * kDistBlock, k1 = min(k0 + kDistBlock, P.ntris);
    for (uint32_t k = k0; k < k1; k++)
    {
        const float4 *r = P.tri_dist + 6 * size_t(k);
        const float d = rtd::dist_point_tri(px, py, pz, r[0], r[1], r[2], r[3], r[4], r[5]);
        if (d < dist)
        {
            dist = d;
            best_k = k;
        }
    }
}

// true when block b can still lower some active lane's minimum
__device__ __forceinline__ bool march_block_needed(const KParams& P, uint32_t b, float px, float py, float pz,
                                                   float margin, float dist)
{
    const float4 mn = P.dist_blk[2 * b], mx = P.dist_blk[2 * b + 1];
    const float ex = fmaxf(fmaxf(mn.x - px, px - mx.x), 0.0f);
    const float ey = fmaxf(fmaxf(mn.y - py, py - mx.y), 0.0f);
    const float ez = fmaxf(fmaxf(mn.z - pz, pz - mx.z), 0.0f);
    const float lb = __builtin_sqrtf(ex * ex + ey * ey + ez * ez) - margin;
    return __any(!(lb > dist));
}

template <bool STATS, bool EXHAUSTIVE>
__device__ __forceinline__ bool ray_march(const KParams& P, float ox, float oy, float oz, float dx, float dy,
                                          float dz, float& t, uint32_t& steps, uint32_t& tests)
{
    t = 0.0f;
    uint32_t best_k = 0;                 // sorted index of the previous step's nearest triangle
    for (uint32_t s = 0; s < kMarchSteps; s++)
    {
        const float px = ox + t * dx, py = oy + t * dy, pz = oz + t * dz;
        float dist = rtd::kFltMax;
        if (EXHAUSTIVE)
        {
            for (uint32_t i = 0; i < P.ntris; i++)
            {
                const float4 *r = P.tri_dist + 6 * size_t(i);
                const float d = rtd::dist_point_tri(px, py, pz, r[0], r[1], r[2], r[3], r[4], r[5]);
                dist = (d < dist) ? d : dist;                        // std::min(dist, d)
            }
            if (STATS) tests += P.ntris;
        }
        else
        {
            const float margin = 1e-5f * (fmaxf(fmaxf(fabsf(px), fabsf(py)), fabsf(pz)) + P.scene_scale);
            {
                const float wx = px - fminf(fmaxf(px, P.smin[0]), P.smax[0]);
                const float wy = py - fminf(fmaxf(py, P.smin[1]), P.smax[1]);
                const float wz = pz - fminf(fmaxf(pz, P.smin[2]), P.smax[2]);
                const float db = __builtin_sqrtf(wx * wx + wy * wy + wz * wz);
                const float rate = dx * wx + dy * wy + dz * wz;
                if (db > 1.00001f * (margin + 0.001f) && rate >= 2e-5f * db)
                {
                    if (STATS) steps = kMarchSteps;
                    return false;
                }
            }
            {
                const float4 *r = P.tri_dist + 6 * size_t(best_k);
                dist = rtd::dist_point_tri(px, py, pz, r[0], r[1], r[2], r[3], r[4], r[5]);
            }
            uint32_t evals = 1;
            const uint32_t start = __builtin_amdgcn_readfirstlane(best_k / kDistBlock);
            for (uint32_t b = start; b < P.ndist_blk; b++)
            {
                if (!march_block_needed(P, b, px, py, pz, margin, dist)) continue;
                march_eval_block(P, b, px, py, pz, dist, best_k);
                evals += min(b * kDistBlock + kDistBlock, P.ntris) - b * kDistBlock;
            }
            for (uint32_t b = start; b-- > 0;)
            {
                if (!march_block_needed(P, b, px, py, pz, margin, dist)) continue;
                march_eval_block(P, b, px, py, pz, dist, best_k);
                evals += min(b * kDistBlock + kDistBlock, P.ntris) - b * kDistBlock;
            }
            if (STATS) tests += evals;
        }
        t += dist;
        if (STATS) steps = s + 1;
        if (dist < 0.001f) return true;
    }
    return false;
}

// What a product walk leaves for rt_render_records_device: hit, t, u, v, the CSR reference of the hit
// and the walk's end cell (raw: a box-run miss's cell still in its box-word copy).
struct SampleOut { bool hit; float t, u, v; uint32_t voxel, csr; };

// renderer.cpp:88-122: one sample -> its colour contribution; hit_tri = the hit triangle
// (Grid::Intersect's tri_idx, renderer.cpp:105) or kNoTri
template <bool STATS, int TRI, int VAR>
__device__ __forceinline__ void trace_sample(const KParams& P, uint32_t px, uint32_t py, uint32_t s, float& cr,
                                             float& cg, float& cb, uint32_t& hit_tri, rt_sample_rec *rec,
                                             uint32_t off = 0u, SampleOut *so = nullptr)
{
    float dx, dy, dz;
    rtd::dir_from_xy(P.m, P.ndcx[px * P.spp + s], P.ndcy[py * P.spp + s], dx, dy, dz);    // camera.h:8-47
    float t = 0.0f, u = 0.0f, v = 0.0f;
    uint32_t tri = rtd::kNoTri, voxel = rtd::kNoTri, steps = 0, tests = 0;
    bool hit;
    if constexpr ((VAR & kVarMarch) != 0)
        hit = ray_march<STATS, (VAR & kVarExhaustive) != 0>(P, P.org[0], P.org[1], P.org[2], dx, dy, dz, t, steps,
                                                             tests);
    else if constexpr ((VAR & kVarBrute) != 0)
        hit = brute_intersect<STATS>(P, P.org[0], P.org[1], P.org[2], dx, dy, dz, t, u, v, tri, tests);
    else
        hit = grid_intersect<STATS, TRI, VAR>(P, P.org[0], P.org[1], P.org[2], dx, dy, dz, t, u, v, tri, voxel,
                                              steps, tests);
    const KParams& Q = late_params(P, off);
    constexpr bool CSR_TRI = (VAR & (kVarMarch | kVarBrute)) == 0 && (VAR & kVarOriginPre) && TRI == RT_TRI_MOLLER_TRUMBORE;
    if (so)                     // the walk's outcome for a record (process_item stores it)
    {
        so->hit = hit;
        so->t = t;
        so->u = u;
        so->v = v;
        so->voxel = voxel;
        so->csr = CSR_TRI ? tri : rtd::kNoTri;
    }
    if constexpr (CSR_TRI)
        if (hit) tri = __float_as_uint(Q.refs[3 * size_t(tri) + 2].y);     // CSR reference -> triangle id
    if constexpr ((VAR & kVarMarch) != 0)
    {
        // The reference's RayMarch leaves u, v, tri_idx unset (renderer.cpp:103), so the
        // march is shaded by depth: the reference's own alternative at renderer.cpp:118.
        if (hit) cr = cg = cb = t / 3.0f;
        else cr = cg = cb = float(py) / float(Q.H);
    }
    else if (hit)
    {
        const float4 a = Q.shade[3 * tri + 0], b = Q.shade[3 * tri + 1], c = Q.shade[3 * tri + 2];
        rtd::shade_hit(u, v, a, b, c, cr, cg, cb);
    }
    else
    {
        const float m = float(py) / float(Q.H);                  // renderer.cpp:121
        cr = cg = cb = m;
    }
    hit_tri = hit ? tri : rtd::kNoTri;
    if (STATS)
    {
        rec->hit = hit;
        rec->tri = hit ? tri : rtd::kNoTri;
        rec->voxel = voxel;
        rec->steps = steps;
        rec->tests = tests;
        rec->t = hit ? t : 0.0f;
        rec->u = hit ? u : 0.0f;
        rec->v = hit ? v : 0.0f;
        rec->r = cr; rec->g = cg; rec->b = cb;
        rec->pad = 0;
    }
}

// Tile bookkeeping: block -> (local tile k, sub-block)
struct TileCoord { uint32_t k, sub, tx0, ty0; };

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

__device__ __forceinline__ TileCoord tile_of_block(const KParams& P)
{
    TileCoord c;
    c.k = blockIdx.x / P.wg_per_tile;
    c.sub = blockIdx.x - c.k * P.wg_per_tile;
    uint32_t tx, ty;
    shard_tile_xy(c.k, P.rank, P.nranks, P.tiles_x, tx, ty);
    c.tx0 = P.rx0 + tx * kTile;
    c.ty0 = P.ry0 + ty * kTile;
    return c;
}

__device__ __forceinline__ void store_pixel(const KParams& P, const TileCoord& c, uint32_t p, uint32_t x,
                                            uint32_t y, uint32_t word)
{
    if (P.shard_mode == 2u)
    {
        // the Framebuffer's tile buffers back to back in tile order c + r * fb_tx: tile (c, r) starts
        // at y0 * W + th_r * x0 (the tiles above it, then the row's tiles left of it, all th_r tall),
        // pixel (x, y) at buf[(x - x0) + (y - y0) * tw_c] (renderer.cpp:133).  x, y < 2^16 and the
        // tile sizes < 2^16, so the mul_hi quotients are exact.
        const uint32_t c = P.fb_tw ? min(__umulhi(x, P.fb_mtw), P.fb_tx - 1u) : P.fb_tx - 1u;
        const uint32_t r = P.fb_th ? min(__umulhi(y, P.fb_mth), P.fb_ty - 1u) : P.fb_ty - 1u;
        const uint32_t x0 = c * P.fb_tw, y0 = r * P.fb_th;
        const uint32_t tw = c == P.fb_tx - 1u ? P.W - x0 : P.fb_tw;
        const uint32_t th = r == P.fb_ty - 1u ? P.H - y0 : P.fb_th;
        P.out[size_t(y0) * P.W + size_t(th) * x0 + (y - y0) * tw + (x - x0)] = word;
    }
    else if (P.shard_mode)
        P.out[size_t(c.k) * kTilePix + compact_bits(p >> 1) * kTile + compact_bits(p)] = word;
    else
        P.out[size_t(y - P.ry0) * P.pitch + (x - P.rx0)] = word;     // renderer.cpp:133
}

// renderer.cpp:124 col / float(spp); exact as a multiply when spp is a power of two
__device__ __forceinline__ float average(const KParams& P, float sum)
{
    return P.inv_spp != 0.0f ? sum * P.inv_spp : sum / float(P.spp);
}

struct ItemCoord { TileCoord c; uint32_t p, s, x, y; bool valid; };

// Sample slot `slot` (pixel-major, Morton pixel order) of local tile k.
__device__ __forceinline__ ItemCoord tile_slot_coord(const KParams& P, uint32_t k, uint32_t slot)
{
    ItemCoord ic;
    ic.c.k = k;
    uint32_t tx, ty;
    shard_tile_xy(k, P.rank, P.nranks, P.tiles_x, tx, ty);
    ic.c.tx0 = P.rx0 + tx * kTile;
    ic.c.ty0 = P.ry0 + ty * kTile;
    ic.p = slot >> P.spp_shift;                               // pixel index in the tile (Morton)
    ic.s = slot & (P.spp - 1u);
    ic.x = ic.c.tx0 + compact_bits(ic.p);
    ic.y = ic.c.ty0 + compact_bits(ic.p >> 1);
    ic.valid = ic.x < P.rx0 + P.rw && ic.y < P.ry0 + P.rh;
    return ic;
}

// Pixel/sample of this lane in work item `item` (wave-uniform).  Called before AND after the
// traversal so none of it is live (in VGPRs) across the DDA walk.
__device__ __forceinline__ ItemCoord item_coord(const KParams& P, uint32_t item, uint32_t lane)
{
    const uint32_t items_per_tile = P.wg_per_tile * kWavesPerWG;
    const uint32_t kseq = item / items_per_tile;              // position in the launch's tile order
    const uint32_t slot = (item - kseq * items_per_tile) * 64u + lane;
    return tile_slot_coord(P, P.tile_order ? P.tile_order[kseq] : kseq, slot);   // local tile k
}

// The record of one sample of AUTO's walk (rt_render_records_device), raw (store_record): a box-run
// miss's end cell is still in its box-word copy.
template <int VAR>
__device__ __forceinline__ void process_record(const KParams& Q, const ItemCoord& ic, const SampleOut& so, float cr,
                                               float cg, float cb)
{
    constexpr uint32_t box = (RT_BOX_RUN && (VAR & kVarSkipRun) && (VAR & kVarPackedRem)) ? kRecRawBox : 0u;
    store_record(Q, ic.x, ic.y, ic.s, so.hit, so.csr, so.voxel, so.t, so.u, so.v,
                 (so.csr != rtd::kNoTri ? kRecRawCsr : 0u) | (so.voxel < kVoxelUnknown ? box : 0u));
    store_record_colour(Q, ic.x, ic.y, ic.s, cr, cg, cb);
}

// One wave-sized work item = 64 consecutive sample slots of a 16x16 tile in Morton order
// (a 2^k x 2^k pixel block x spp samples).  Traces the lane's sample, sums the pixel's
// samples across its adjacent lanes in sample order (renderer.cpp:87-122, hazard H10) and
// stores the packed pixel (renderer.cpp:124-133).
template <int TRI, int VAR>
__device__ __forceinline__ void process_item(const KParams& P, uint32_t item, uint32_t off = 0u)
{
    item = __builtin_amdgcn_readfirstlane(item);
    const uint32_t lane = threadIdx.x & 63u;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    uint32_t hit_tri = rtd::kNoTri;
    SampleOut so{false, 0.0f, 0.0f, 0.0f, rtd::kNoTri, rtd::kNoTri};
    {
        const ItemCoord ic = item_coord(P, item, lane);
        if (ic.valid)
            trace_sample<false, TRI, VAR>(P, ic.x, ic.y, ic.s, cr, cg, cb, hit_tri, nullptr, off, &so);
    }
    const KParams& Q = late_params(P, off);
    const ItemCoord ic = item_coord(Q, item, lane);
    // rt_render_hits_device only: the sample's hit triangle, after the walk (a scalar test of a
    // kernel parameter; the walk above is the same code whatever the pointer holds)
    if (Q.hits && ic.valid) Q.hits[(size_t(ic.y) * Q.W + ic.x) * Q.spp + ic.s] = hit_tri;
    // rt_render_records_device only, likewise: the sample's record (process_record)
    if (Q.recs && ic.valid) process_record<VAR>(Q, ic, so, cr, cg, cb);
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    if (Q.spp == 4u)
    {
        // the bench's 4 spp: a pixel's samples are one quad of lanes, so each sample's colour is
        // a quad broadcast (DPP, one VALU) instead of an LDS permute; same values, same order.
        // renderer.cpp:87-122 starts the sum at 0.0f; 0.0f + x == x for every colour (>= +0:
        // (n + 1) * 0.5 of a normalised component, py / H, t / 3 -- never -0), so the sum
        // starts at the first sample
        sr = quad_bcast<0>(cr) + quad_bcast<1>(cr) + quad_bcast<2>(cr) + quad_bcast<3>(cr);
        sg = quad_bcast<0>(cg) + quad_bcast<1>(cg) + quad_bcast<2>(cg) + quad_bcast<3>(cg);
        sb = quad_bcast<0>(cb) + quad_bcast<1>(cb) + quad_bcast<2>(cb) + quad_bcast<3>(cb);
        // ... and the quad's lanes 0, 1, 2 resolve one channel each (b, g, r: the byte at their
        // position in pack_bgra8's word; lane 3 contributes the zero alpha byte), so the correctly
        // rounded square root and the packing run once per wave instead of three times; the
        // bytes meet in the pixel's lane by quad broadcasts (same per-channel arithmetic)
#if RT_QUAD_RESOLVE
        const uint32_t j = lane & 3u;
        const float c = j == 0u ? sb : (j == 1u ? sg : sr);
        uint32_t v = rtd::pack_channel(rtd::gamma_half(c * 0.25f)) << (8u * j);   // renderer.cpp:124, exact
        v = j == 3u ? 0u : v;
        const uint32_t word = quad_bcast_u<0>(v) | quad_bcast_u<1>(v) | quad_bcast_u<2>(v);
        if (ic.valid && ic.s == 0) store_pixel(Q, ic.c, ic.p, ic.x, ic.y, word);
        return;
#endif
    }
    else
    {
        const uint32_t base = lane & ~(Q.spp - 1u);
        for (uint32_t k = 0; k < Q.spp; k++)
        {
            sr += __shfl(cr, int(base + k), 64);
            sg += __shfl(cg, int(base + k), 64);
            sb += __shfl(cb, int(base + k), 64);
        }
    }
    if (ic.valid && ic.s == 0)
    {
        const uint32_t word = rtd::pack_bgra8(rtd::gamma_half(average(Q, sr)), rtd::gamma_half(average(Q, sg)),
                                              rtd::gamma_half(average(Q, sb)));
        store_pixel(Q, ic.c, ic.p, ic.x, ic.y, word);
    }
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
constexpr uint32_t kHfFrontMax = 1024;      // blocks (4 waves each): half the chip's wave slots
constexpr uint32_t kWhMax = 4096;           // kVarWideHeavy: work items the wide section can list
constexpr uint32_t kHfShift = 2;            // heavy: cost > last max >> kHfShift; very heavy: >> 1
constexpr uint32_t kHfPeriod = 16;          // a plan from every kHfPeriod-th frame of a launch shape
// A plan lists blocks only when the slowest block is a real tail: its cost (one wave's
// duration) above kHfTail / 16 of the estimated frame span, sum of wave costs / resident waves
constexpr uint32_t kHfTail = 6;
constexpr uint32_t kHfSlots = 256u * 4u * 8u;   // resident waves: 256 CUs x 4 SIMDs x 8
constexpr int kHfCtxs = 16;                 // launch shapes remembered per scene (a process driving
                                            // the 8 ranks of two scenes' shards keeps all of them)

__device__ __forceinline__ uint32_t xcd_band_block(uint32_t b, uint32_t nb, uint32_t chunk)
{
    if (chunk == 0u)
    {
        const uint32_t q = nb / kXcds, r = nb % kXcds;
        const uint32_t x = b % kXcds, i = b / kXcds;
        return x < r ? x * (q + 1u) + i : r * (q + 1u) + (x - r) * q + i;
    }
    const uint32_t full = nb / (kXcds * chunk) * (kXcds * chunk);
    if (b >= full) return b;
    const uint32_t x = b % kXcds, i = b / kXcds;
    const uint32_t row = (i / chunk) * kXcds + x;
    return row * chunk + i % chunk;
}

// Heavy-first planning, after a measured frame's render kernel on its stream: per block the cost
// of its slowest wave; blocks above max(hf_floor, last max >> kHfShift) are listed for the next
// frames -- above last max >> 1 at the front of the front section, the rest from its back -- and
// marked so the natural order skips them.  Nothing is listed when the last measurement showed no
// tail (its slowest block well under the frame's estimated span).  Each thread takes kHfPlanPer
// blocks (kWG apart, so the cost loads stay coalesced); each workgroup reduces its maximum and sum
// and reserves its list slots with ONE atomic per level (the render waves themselves touch no
// atomics: thousands of same-address atomics from waves cost milliseconds, measured).  The plan's
// time is those same-address atomics: one block per thread (1,013 workgroups for the batched
// bench pair) took 26.6 us per plan, which a moving camera pays every frame.
constexpr uint32_t kHfPlanPer = 8;
__global__ void __launch_bounds__(kWG) k_hf_plan(KParams P, uint32_t nblocks)
{
    __shared__ uint32_t s_max, s_hi, s_lo, s_w, s_w4, s_bhi, s_blo, s_bw, s_bw4, s_last;
    __shared__ unsigned long long s_sum;
    if (threadIdx.x == 0u)
    {
        s_max = s_hi = s_lo = s_w = s_w4 = 0u;
        s_sum = 0ull;
    }
    __syncthreads();
    const HfPlan last = *P.hf_plan_in;
    const bool tail = uint64_t(last.maxc) * kHfSlots * 16u > uint64_t(kHfTail) * (last.sum << 4);
    const uint32_t thr = max(P.hf_floor, last.maxc >> kHfShift);
    const uint32_t b0 = blockIdx.x * (kWG * kHfPlanPer) + threadIdx.x;
    uint32_t tmax = 0u, wmasks = 0u, wmasks4 = 0u, heavy = 0u, hi = 0u;
    unsigned long long tsum = 0ull;
    uint32_t rank[kHfPlanPer], wrank[kHfPlanPer], wrank4[kHfPlanPer];
#pragma unroll
    for (uint32_t j = 0; j < kHfPlanPer; j++)
    {
        const uint32_t b = b0 + j * kWG;
        uint32_t cost = 0u, sum = 0u, wmask = 0u, wmask4 = 0u;
        if (b < nblocks)
        {
            const uint4 c = reinterpret_cast<const uint4 *>(P.hf_cost)[b];      // kWavesPerWG == 4
            sum = (c.x >> 4) + (c.y >> 4) + (c.z >> 4) + (c.w >> 4);          // in 16-cycle units
            if (P.wh_on && !P.wh_wgs && last.sum_full)
            {
                // wide section: items above a fraction of the frame span estimated from the last
                // measurement of every item one lane per sample (sum of wave costs over the resident
                // waves).  New items are listed only from such frames (the first ones of a shape, the
                // refresh frames): with the section running, the lane waves' costs shrink as items
                // leave them, which pulled the span estimate down and listed ever more items
                // (killeroo's rank of 4: 298 -> 587 items over 100 frames, measured).
                const uint64_t span = (last.sum_full << 4) / kHfSlots;
                const uint32_t wt = max(P.wh_floor, uint32_t(min<uint64_t>(span * P.wh_alpha16 / 16u, 0xFFFFFFFFull)));
                wmask = uint32_t(c.x > wt) | (uint32_t(c.y > wt) << 1) | (uint32_t(c.z > wt) << 2) |
                        (uint32_t(c.w > wt) << 3);
                // second tier (4 lanes per sample): items between the beta and the alpha thresholds
                const uint32_t wt4 = P.wh_beta16 ? max(P.wh_floor, uint32_t(min<uint64_t>(span * P.wh_beta16 / 16u,
                                                                                            0xFFFFFFFFull)))
                                                 : 0xFFFFFFFFu;
                wmask4 = (uint32_t(c.x > wt4) | (uint32_t(c.y > wt4) << 1) | (uint32_t(c.z > wt4) << 2) |
                          (uint32_t(c.w > wt4) << 3)) & ~wmask;
            }
            if (P.wh_on && !P.wh_refresh && P.hf_ver)
            {
                // sticky: the current plan's items stay listed in their tier (mark = the plan version,
                // bit 31 = the second tier)
                const uint4 m = reinterpret_cast<const uint4 *>(P.wh_mark_in)[b];
                const uint32_t in = uint32_t((m.x & 0x7FFFFFFFu) == P.hf_ver) | (uint32_t((m.y & 0x7FFFFFFFu) == P.hf_ver) << 1) |
                                    (uint32_t((m.z & 0x7FFFFFFFu) == P.hf_ver) << 2) |
                                    (uint32_t((m.w & 0x7FFFFFFFu) == P.hf_ver) << 3);
                const uint32_t t4 = (m.x >> 31) | ((m.y >> 31) << 1) | ((m.z >> 31) << 2) | ((m.w >> 31) << 3);
                wmask |= in & ~t4;
                wmask4 = (wmask4 | (in & t4)) & ~wmask;
            }
            // the heavy-first order ranks a block by its slowest wave left in the lane section
            const uint32_t wm = wmask | wmask4;
            cost = max(max((wm & 1u) ? 0u : c.x, (wm & 2u) ? 0u : c.y), max((wm & 4u) ? 0u : c.z, (wm & 8u) ? 0u : c.w));
        }
        const bool hv = P.hf_front && tail && cost > thr;
        const bool h1 = hv && cost > (last.maxc >> 1);
        tmax = max(tmax, cost);
        tsum += sum;
        rank[j] = hv ? atomicAdd(h1 ? &s_hi : &s_lo, 1u) : 0u;
        wrank[j] = wmask ? atomicAdd(&s_w, uint32_t(__popc(wmask))) : 0u;
        wrank4[j] = wmask4 ? atomicAdd(&s_w4, uint32_t(__popc(wmask4))) : 0u;
        heavy |= uint32_t(hv) << j;
        hi |= uint32_t(h1) << j;
        wmasks |= wmask << (4u * j);
        wmasks4 |= wmask4 << (4u * j);
    }
    if (tmax) atomicMax(&s_max, tmax);
    if (tsum) atomicAdd(&s_sum, tsum);
    __syncthreads();
    if (threadIdx.x == 0u)
    {
        if (s_max) atomicMax(&P.hf_plan_out->maxc, s_max);
        if (s_sum) atomicAdd(&P.hf_plan_out->sum, s_sum);
        if (P.wh_on)
        {
            if (!P.wh_wgs)
            {
                if (s_sum) atomicAdd(&P.hf_plan_out->sum_full, s_sum);
            }
            else if (blockIdx.x == 0u)
                P.hf_plan_out->sum_full = last.sum_full;      // carried
        }
        s_bhi = s_hi ? atomicAdd(&P.hf_plan_out->cnt_hi, s_hi) : 0u;
        s_blo = s_lo ? atomicAdd(&P.hf_plan_out->cnt_lo, s_lo) : 0u;
        s_bw = s_w ? atomicAdd(&P.hf_plan_out->cnt_w, s_w) : 0u;
        s_bw4 = s_w4 ? atomicAdd(&P.hf_plan_out->cnt_w4, s_w4) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kHfPlanPer; j++)
    {
        const uint32_t b = b0 + j * kWG;
        if ((heavy >> j) & 1u)
        {
            // very heavy blocks fill the front section from its start, the others from its end; a
            // level that runs into the other is cut (those blocks stay in the natural order)
            const bool h1 = (hi >> j) & 1u;
            const uint32_t r = (h1 ? s_bhi : s_blo) + rank[j];
            if (r < P.hf_front)
            {
                const uint32_t slot = h1 ? r : P.hf_front - 1u - r;
                P.hf_list_out[slot] = b;           // may be overwritten by the other level: see below
            }
        }
        // wide items: listed and marked for the next plan's frames (beyond kWhMax they stay in the
        // lane section)
        const uint32_t wmask = (wmasks >> (4u * j)) & 15u, wmask4 = (wmasks4 >> (4u * j)) & 15u;
        uint32_t wr = wrank[j], wr4 = wrank4[j];
        for (uint32_t k = 0; k < kWavesPerWG; k++)
            if (wmask & (1u << k))
            {
                const uint32_t item = b * kWavesPerWG + k;
                const uint32_t r = s_bw + wr++;
                if (r < kWhMax)
                {
                    P.wh_list_out[r] = item;
                    P.wh_mark_out[item] = P.hf_ver + 1u;
                }
            }
            else if (wmask4 & (1u << k))
            {
                const uint32_t item = b * kWavesPerWG + k;
                const uint32_t r = s_bw4 + wr4++;
                if (r < kWhMax)
                {
                    P.wh_list_out[kWhMax + r] = item;
                    P.wh_mark_out[item] = (P.hf_ver + 1u) | 0x80000000u;
                }
            }
    }
    // The block marks are written by a second pass over the final list, so a slot claimed by
    // both levels marks only the block whose entry survived.  That pass runs in the workgroup
    // that finishes last (a ticket after a release fence), not in a second launch: a kernel
    // launch costs ~4 us, as much as the whole plan at a rank of 8.
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0u) s_last = atomicAdd(P.hf_ticket, 1u) == gridDim.x - 1u;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    const volatile HfPlan *vp = P.hf_plan_out;
    const uint32_t ch = vp->cnt_hi, cl = vp->cnt_lo;
    const uint32_t nhi = min(ch, P.hf_front);
    const uint32_t nlo = min(cl, P.hf_front - nhi);
    const volatile uint32_t *vl = P.hf_list_out;
    for (uint32_t j = threadIdx.x; j < P.hf_front; j += kWG)
        if (j < nhi || j >= P.hf_front - nlo) P.hf_mark_out[vl[j]] = P.hf_ver + 1u;
    if (threadIdx.x == 0u)
    {
        // hands the wide section's item count to the host (it sizes the section of later
        // launches) and re-arms the ticket
        if (P.wh_host_cnt)
            *(volatile uint32_t *)P.wh_host_cnt = P.wh_g * min(vp->cnt_w, kWhMax) + (P.wh_g == 16u ? 4u * min(vp->cnt_w4, kWhMax) : 0u);
        *P.hf_ticket = 0u;
    }
}

// The launch's block -> block-of-work map.  With the heavy-first order on, blocks [0, hf_front)
// take the blocks listed by the previous frame (in the order their heavy waves finished) and the
// rest walk the natural (XCD-banded) order, skipping the listed blocks.  Returns false when this
// block has nothing to do.  The marks read here are never written by this launch (the next
// frame's marks live in the other buffer), so every wave of a block decides alike.
// lead: the first lane of launch block 0's first wave (the one that clears the next plan).
template <int VAR>
__device__ __forceinline__ bool block_of_launch(const KParams& P, uint32_t& b, uint32_t bid, uint32_t nblk,
                                                bool lead)
{
    if ((VAR & kVarWideHeavy) && P.hf_measure && lead)
        *P.hf_plan_out = HfPlan{};                            // k_hf_plan runs after this kernel
    if (P.hf_front)
    {
        if (P.hf_measure && lead)
            *P.hf_plan_out = HfPlan{};                        // k_hf_plan runs after this kernel
        const uint32_t front = P.hf_front;
        if (bid < front)
        {
            const uint32_t hi = min(P.hf_plan_in->cnt_hi, front);
            const uint32_t lo = min(P.hf_plan_in->cnt_lo, front - hi);
            if (bid >= hi && bid < front - lo) return false;
            b = P.hf_list_in[bid];
            return true;
        }
        const uint32_t q = bid - front;
        const uint32_t nb = nblk - front;
        b = (VAR & kVarXcdBands) ? xcd_band_block(q, nb, P.xcd_chunk) : q;
        return P.hf_ver == 0u || P.hf_mark_in[b] != P.hf_ver;
    }
    b = (VAR & kVarXcdBands) ? xcd_band_block(bid, nblk, P.xcd_chunk) : bid;
    return true;
}

// The wide section's per-sample trace (AUTO's record layout, spp a power of two <= 64 / G): G
// lanes per sample.  The heaviest waves of a frame (killeroo's body, scene 5's cat) run ~1000
// triangle tests per lane in a serial chain -- ~1M cycles per wave, the launch's critical path
// once a rank renders 1/8 of the frame.  Here the G lanes of a group walk the same ray (identical
// state, so identical control flow) and split each cell's list: sublane j tests references
// kb + j, kb + j + G, ... with strict '<' in ascending order, and a butterfly over the group takes
// the lexicographic minimum of (t, k) -- the first minimum in list order, exactly what
// grid.cpp:258-266 keeps.  The chain per lane shrinks by G; the DDA walk is repeated G times.
// Returns the sample's colour in every lane of the group (and stores its hit triangle for
// rt_render_hits_device).
// (G: a wave-uniform value -- 16, or 4 -- so both tiers of the wide section share one code path and
// one register allocation; the butterfly's trip count follows it.)
template <int VAR>
__device__ __forceinline__ void wide_trace(const KParams& P, uint32_t k, uint32_t slot, uint32_t sub, uint32_t G,
                                           float& cr, float& cg, float& cb, uint32_t& hit_tri)
{
    static_assert((VAR & kVarOriginPre) && (VAR & kVarDistSkip) && (VAR & kVarPackedRem), "AUTO layout");
    const float ox = P.org[0], oy = P.org[1], oz = P.org[2];
    cr = cg = cb = 0.0f;
    {
        const ItemCoord ic = tile_slot_coord(P, k, slot);
        if (ic.valid)
        {
            float dx, dy, dz;
            rtd::dir_from_xy(P.m, P.ndcx[ic.x * P.spp + ic.s], P.ndcy[ic.y * P.spp + ic.s], dx, dy, dz);
            float nct0, nct1, nct2, dt0, dt1, dt2;
            int rem0, rem1, rem2, cs0, cs1, cs2, cell;
            bool hit = false;
            float t = 0.0f, u = 0.0f, v = 0.0f;
            uint32_t tri = 0u;
            if (dda_setup(P, ox, oy, oz, dx, dy, dz, nct0, nct1, nct2, dt0, dt1, dt2, rem0, rem1, rem2, cs0, cs1,
                          cs2, cell))
            {
#if RT_WIDE_BOX
                // AUTO's box-run walk (grid_intersect) with per-lane runs: the G lanes of a sample
                // walk identically, and the samples of a wave share no list loop (each lane tests
                // its own share of its sample's cell), so every group jumps through its empty
                // boxes on its own (box_exit_bound's add chains, then the exit step)
                int remp = rem0 | (rem1 << 11) | (rem2 << 22);
                int boxw = kRemGuards;
                cell += box_offset(P, dx, dy, dz);
                for (;;)
                {
                    uint32_t kb = 0u, ke = 0u;
                    float nct_ax;
                    bool more;
                    if ((boxw & kRemGuards) != 0)
                    {
                        const uint32_t w = P.cellwb[uint32_t(cell)];
                        const uint32_t ne = uint32_t(int(w) >> 31);
                        kb = (w >> 11) & 0xFFFFFu;
                        ke = kb + (w & ne & 2047u);
                        boxw = int(w & ~ne);
                    }
                    RT_DDA_ADVANCE_BOX(nct_ax, more);
                    if ((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u)
                    {
                        const uint32_t b0 = uint32_t(boxw);
                        const int f0 = boxw & 1023, f1 = (boxw >> 11) & 1023, f2 = int(uint32_t(boxw) >> 22);
                        const float tl = __builtin_fminf(__builtin_fminf(box_exit_bound(nct0, dt0, f0),
                                                                         box_exit_bound(nct1, dt1, f1)),
                                                         box_exit_bound(nct2, dt2, f2));
                        int c0 = 0, c1 = 0, c2 = 0;
                        while (nct0 < tl && c0 < f0) { nct0 += dt0; c0++; }
                        while (nct1 < tl && c1 < f1) { nct1 += dt1; c1++; }
                        while (nct2 < tl && c2 < f2) { nct2 += dt2; c2++; }
                        boxw -= c0 + (c1 << 11) + (c2 << 22);
                        do
                            RT_DDA_BOX_BARE_STEP();
                        while ((uint32_t(boxw) & uint32_t(kRemGuards)) == 0u);
                        const uint32_t d = b0 - uint32_t(boxw);
                        remp = int(uint32_t(remp) - d);
                        cell += int(d & 2047u) * cs0 + int((d >> 11) & 2047u) * cs1 + int(d >> 22) * cs2;
                        more = (remp & kRemGuards) == 0;
                    }
#else
                int skip = 0;
                int remp = rem0 | (rem1 << 11) | (rem2 << 22);
                cell += oct_offset(P, dx, dy, dz);
                for (;;)
                {
                    uint32_t kb = 0u, ke = 0u;
                    float nct_ax;
                    bool more;
                    if (skip == 0)
                    {
                        const uint32_t w = P.cellwo[uint32_t(cell)];
                        const uint32_t cnt = w & 2047u;
                        kb = w >> 11;
                        ke = kb + cnt;
                        skip = cnt ? 0 : int(kb) - 1;
                    }
                    else
                        skip--;
                    RT_DDA_ADVANCE_PACKED(nct_ax, more);
#endif
                    if (kb < ke)
                    {
                        // tb starts at the cell's exit time (test_cell's bound); a lane that takes
                        // nothing keeps (nct_ax, ~0), which every taken (t < nct_ax, k) beats
                        float bt = __builtin_fminf(rtd::kFltMax, nct_ax), bu = 0.0f, bv = 0.0f;
                        uint32_t bk = 0xFFFFFFFFu;
                        const rtd::f2v ra = {dx, dy}, rc = {dy, dz};
                        for (uint32_t k = kb + sub; k < ke; k += G)
                        {
                            const float4 *rp = P.frefs + size_t(k) * 4u;
                            const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2], r3 = rp[3];
                            float inv, cu;
                            const bool ok1 = rtd::mt_rec_first<(VAR & kVarFastRcp) != 0>(
                                ra, rc, rtd::f2v{r0.x, r0.y}, rtd::f2v{r0.z, r0.w}, rtd::f2v{r1.x, r1.y},
                                rtd::f2v{r1.z, r1.w}, rtd::f2v{r2.x, r2.y}, inv, cu);
                            if (__any(ok1))
                            {
                                float cv, ct;
                                const bool h = ok1 & rtd::mt_rec_second(ra, rc, rtd::f2v{r2.z, r2.w}, r3.x, r3.y, inv, cu,
                                                                        cv, ct);
                                const bool take = h & (ct < bt);
                                bt = take ? ct : bt;
                                bu = take ? cu : bu;
                                bv = take ? cv : bv;
                                bk = take ? k : bk;
                            }
                        }
                        for (int m = 1; m < int(G); m <<= 1)
                        {
                            const float ot = __shfl_xor(bt, m, 64), ou = __shfl_xor(bu, m, 64),
                                        ov = __shfl_xor(bv, m, 64);
                            const uint32_t ok = uint32_t(__shfl_xor(int(bk), m, 64));
                            const bool better = (ot < bt) | ((ot == bt) & (ok < bk));
                            bt = better ? ot : bt;
                            bu = better ? ou : bu;
                            bv = better ? ov : bv;
                            bk = better ? ok : bk;
                        }
                        if (bk != 0xFFFFFFFFu)
                        {
                            u = bu;
                            v = bv;
                            tri = bk;
                            hit = true;
                            t = bt;
                            break;
                        }
                    }
                    if (!more)
                    {
                        // records of a miss: the exit step is the last one taken (the lowest
                        // borrowed guard)
                        // rt_render_records_device only: a miss's raw record where the walk ends
                        // (the walk state it needs stays live no further; the pixel again from k and
                        // slot); the colour words after the resolve
                        if (P.recs && sub == 0u)
                        {
                            const ItemCoord rc = tile_slot_coord(P, k, slot);
                            store_record(P, rc.x, rc.y, rc.s, false, 0u, exit_voxel(remp, cell, cs0, cs1, cs2), 0.0f,
                                         0.0f, 0.0f, RT_WIDE_BOX ? kRecRawBox : kRecRawOct);
                        }
                        break;
                    }
                }
            }
            else if (P.recs && sub == 0u)      // records of a ray that misses the grid
            {
                const ItemCoord rc = tile_slot_coord(P, k, slot);
                store_record(P, rc.x, rc.y, rc.s, false, 0u, rtd::kNoTri, 0.0f, 0.0f, 0.0f, 0u);
            }
            const KParams& Q = P;
            if (hit && Q.recs && sub == 0u)               // a hit's raw record (records only)
            {
                const ItemCoord rc = tile_slot_coord(Q, k, slot);
                store_record(Q, rc.x, rc.y, rc.s, true, tri, 0u, t, u, v, kRecRawCsr);
            }
            if (hit)
            {
                tri = __float_as_uint(Q.refs[3 * size_t(tri) + 2].y);     // CSR reference -> triangle id
                const float4 a = Q.shade[3 * tri + 0], bb = Q.shade[3 * tri + 1], c = Q.shade[3 * tri + 2];
                rtd::shade_hit(u, v, a, bb, c, cr, cg, cb);
            }
            else
                cr = cg = cb = float(ic.y) / float(Q.H);                   // renderer.cpp:121
            hit_tri = hit ? tri : rtd::kNoTri;
        }
    }
}

// One wave of the wide mode: the 64 / G consecutive sample slots slot0 .. of local tile k.
template <int VAR>
__device__ __forceinline__ void wide_samples(const KParams& P, uint32_t k, uint32_t slot0, uint32_t G)
{
    const uint32_t lane = threadIdx.x & 63u, sub = lane & (G - 1u), grp = lane >> (31u - __builtin_clz(G));
    const uint32_t slot = slot0 + grp;
    float cr, cg, cb;
    uint32_t hit_tri = rtd::kNoTri;
    wide_trace<VAR>(P, k, slot, sub, G, cr, cg, cb, hit_tri);
    // the pixel's samples are the groups grp0 .. grp0 + spp - 1 of this wave: sum in sample order
    const ItemCoord ic = tile_slot_coord(P, k, slot);
    // rt_render_hits_device / rt_render_records_device only (scalar tests of kernel parameters)
    if (P.hits && sub == 0u && ic.valid) P.hits[(size_t(ic.y) * P.W + ic.x) * P.spp + ic.s] = hit_tri;
    if (P.recs && sub == 0u && ic.valid) store_record_colour(P, ic.x, ic.y, ic.s, cr, cg, cb);
    const uint32_t grp0 = grp & ~(P.spp - 1u);
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    for (uint32_t j = 0; j < P.spp; j++)
    {
        const int src = int((grp0 + j) * G);
        sr += __shfl(cr, src, 64);
        sg += __shfl(cg, src, 64);
        sb += __shfl(cb, src, 64);
    }
    if (ic.valid && ic.s == 0 && sub == 0)
    {
        const uint32_t word = rtd::pack_bgra8(rtd::gamma_half(average(P, sr)), rtd::gamma_half(average(P, sg)),
                                              rtd::gamma_half(average(P, sb)));
        store_pixel(P, ic.c, ic.p, ic.x, ic.y, word);
    }
}

// kVarWaveClock: the four words of one wave's record (rt_debug_wave_clocks): s_memtime at its start and
// end (per clock domain: durations), and the XCD it ran on (bits 32-35 of word 2) with the low 28 bits
// of the device-wide 100 MHz s_memrealtime at its start (word 2, bits 36-63) and end (word 3, bits
// 32-59): launch timelines use the real-time clock.  c0 / c1: the words' low 32 bits.
__device__ __forceinline__ void store_wave_clock(uint64_t *clk, uint32_t idx, uint64_t t0, uint64_t t1, uint64_t r0,
                                                 uint64_t r1, uint32_t c0, uint32_t c1)
{
    clk[4 * size_t(idx)] = t0;
    clk[4 * size_t(idx) + 1] = t1;
    clk[4 * size_t(idx) + 2] = c0 | (uint64_t(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u) << 32) |
                               ((r0 & 0xFFFFFFFull) << 36);
    clk[4 * size_t(idx) + 3] = c1 | ((r1 & 0xFFFFFFFull) << 32);
}

// kVarWideHeavy: the launch's wide section.  Its waves take the current plan's heavy work items
// in list order, wh_g waves per item (each 64 / wh_g of the item's sample slots, wh_g lanes per
// sample): persistent over the list, so a section smaller than the list (the host sizes it from
// an older plan's count) still renders every listed item.  They record no cost: an item's cost
// word keeps its lane-mode measurement until a refresh frame renders it one lane per sample again.
// In a batch (KBatch, BATCH = true) P is p[0] (the batch's list, launch-wide item indices) and each
// item is rendered with its own frame's parameters.
// w: this wave's index in the section (4 per 256-lane workgroup, or one per one-wave workgroup).
template <bool BATCH, uint32_t G, bool CLK = false>
__device__ __forceinline__ void wide_section(const KParams& P, uint32_t w)
{
    const uint32_t n = P.hf_ver ? min(P.hf_plan_in->cnt_w, kWhMax) : 0u;
    // the second tier (G = 16 only): 4 lanes per sample, 4 waves per item, after the first tier's
    const uint32_t n4 = (G == 16u && P.hf_ver) ? min(P.hf_plan_in->cnt_w4, kWhMax) : 0u;
    const uint32_t nw = P.wh_wgs * kWavesPerWG;
    const uint32_t ipt = P.wg_per_tile * kWavesPerWG;              // items per tile
    for (uint32_t e = w; e < n * G + n4 * 4u; e += nw)
    {
        const bool t4 = e >= n * G;                                 // wave-uniform
        const uint32_t e4 = e - n * G;
        const uint32_t li = t4 ? kWhMax + e4 / 4u : e / G;          // list entry
        uint32_t item = __builtin_amdgcn_readfirstlane(P.wh_list_in[li]);
        uint32_t off = 0u;
        if constexpr (BATCH)
        {
            const KBatch& B = late_batch();
            const uint32_t f = batch_frame(B, item / kWavesPerWG);
            item -= B.base[f] * kWavesPerWG;                      // the frame's own item index
            off = uint32_t(offsetof(KBatch, p)) + f * uint32_t(sizeof(KParams));
        }
        const uint32_t kseq = item / ipt;
        const uint32_t slot0 = (item - kseq * ipt) * 64u + (t4 ? (e4 % 4u) * 16u : (e % G) * (64u / G));
        // the parameters re-read per item (late_params): hoisted out of the loop they held ~30
        // more SGPRs across it and spilled
        const KParams& Q = late_params(P, off);
        const uint32_t k = Q.tile_order ? Q.tile_order[kseq] : kseq;
        uint64_t r0 = 0, t0 = 0;
        if constexpr (CLK && BATCH)
        {
            r0 = __builtin_amdgcn_s_memrealtime();
            t0 = __builtin_amdgcn_s_memtime();
        }
        wide_samples<kVarWide>(Q, k, slot0, __builtin_amdgcn_readfirstlane(t4 ? 4u : G));
        if constexpr (CLK && BATCH)
        {
            // kVarWaveClock: one record per (listed item, wave) of the section, after the batch's lane
            // items: word 2's low bits = 0x80000000 | 0x40000000 for the second tier | list entry,
            // word 3's = the launch-wide item
            const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            const KBatch& B = late_batch();
            const KParams& Q0 = late_params(P, uint32_t(offsetof(KBatch, p)));
            if ((threadIdx.x & 63u) == 0u)
                store_wave_clock(Q0.wave_clk, B.base[B.nframes] * kWavesPerWG + e, t0, t1, r0, r1,
                                 0x80000000u | (t4 ? 0x40000000u : 0u) | li,
                                 __builtin_amdgcn_readfirstlane(Q0.wh_list_in[li]));
        }
    }
}

// Wave `wib` (0-3) of launch block bid of nblk: its work item after the heavy-first / XCD-band map.
template <int TRI, int VAR>
__device__ __forceinline__ void lanes_block_wave(const KParams& P, uint32_t bid, uint32_t nblk, uint32_t wib,
                                                 volatile uint32_t *t0v)
{
    uint32_t b;
    if (!block_of_launch<VAR>(P, b, bid, nblk, bid == 0u && wib == 0u && (threadIdx.x & 63u) == 0u)) return;
    const uint32_t item = b * kWavesPerWG + wib;
    if constexpr ((VAR & kVarWideHeavy) != 0)
        if (P.wh_wgs && P.hf_ver && (P.wh_mark_in[item] & 0x7FFFFFFFu) == P.hf_ver) return;   // the wide section's
    if constexpr ((VAR & kVarWaveClock) != 0)
    {
        // debug arm (RT_KERNEL_FLAG_WAVE_CLOCK): s_memtime at the item's start and end, and how
        // many records the item tested in wave-uniform loops vs lane-loop iterations
        if ((threadIdx.x & 63u) == 0u)
        {
            wave_counters()[0] = 0u;
            wave_counters()[1] = 0u;
        }
        wave_lds_sync();
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        process_item<TRI, VAR>(P, item);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
        wave_lds_sync();
        if ((threadIdx.x & 63u) == 0u)
            store_wave_clock(P.wave_clk, item, t0, t1, r0, r1, wave_counters()[0], wave_counters()[1]);
    }
    else
    {
        const bool hf = P.hf_measure != 0u;
        if (hf && (threadIdx.x & 63u) == 0u) t0v[threadIdx.x >> 6] = uint32_t(__builtin_amdgcn_s_memtime());
        process_item<TRI, VAR>(P, item);
        const KParams& Q = late_params(P);
        if (Q.hf_measure)
        {
            const uint32_t t1 = uint32_t(__builtin_amdgcn_s_memtime());
            const uint32_t t0 = __builtin_amdgcn_readfirstlane(t0v[threadIdx.x >> 6]);
            if ((threadIdx.x & 63u) == 0u) Q.hf_cost[__builtin_amdgcn_readfirstlane(item)] = t1 - t0;
        }
    }
}

// RT_KERNEL_LANES / AUTO: one lane per sample (spp = 2^spp_shift <= 64), one work item per
// wave.  Heavy-first order: see block_of_launch and k_hf_plan; wide section: wide_section.
template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) k_render_lanes(KParams P)
{
    __shared__ uint32_t t0s[kWavesPerWG];
    volatile uint32_t *t0v = t0s;                 // a wave's start time waits in LDS across the walk
    lanes_block_wave<TRI, VAR>(P, blockIdx.x, gridDim.x, threadIdx.x >> 6, t0v);
}

// The same launch blocks as one-wave workgroups (AUTO's whole-frame launches of >= wg64_min_blocks
// blocks; rt_scene::wg64).  A wave slot that frees up takes the next workgroup by itself instead of
// waiting until three more slots of its CU are free for a 256-lane workgroup: with waves of very
// different lengths (killeroo 1080p x 4: median 13 us, p99 100 us, max 450 us) the dispatched
// 256-lane grid held only ~75 % of the 8,192 wave slots mid-frame (profiles/r03q_waves_*.json).
// Workgroup w runs wave r % 4 of launch block (r / 4) * 8 + w % 8, r = w / 8, so every block keeps
// the XCD its 256-lane workgroup had (workgroups w and w + 8 share one under the dispatcher's
// round-robin deal: the XCD bands of xcd_band_block hold) and the launch keeps its block order
// (the heavy-first front first).  Grid: 4 x vblocks rounded up to 8; pixels and per-sample
// arithmetic are unchanged (process_item per work item, as in k_render_lanes).  Measured in-process
// (tools/launch_ab.py, profiles/r03w_w64_all.json, 1080p x 4 steady): killeroo 0.390 -> 0.369 ms,
// head 0.258 -> 0.251, the 10 scenes 2.99 -> 2.95 ms; resident waves on per-XCD work queues
// (one returning atomic per item) lost 10-60 % to the dequeues (profiles/r03u_launch_ab_pq_w64.json, r03v_persist_*.json).
template <int TRI, int VAR>
__global__ void __launch_bounds__(64) k_render_lanes_w64(KParams P)
{
    __shared__ uint32_t t0s[1];
    const uint32_t w = blockIdx.x, r = w / kXcds;
    const uint32_t vbid = (r >> 2) * kXcds + w % kXcds;
    const KParams& Q = late_params(P);
    if (vbid >= Q.vblocks) return;
    lanes_block_wave<TRI, VAR>(P, vbid, Q.vblocks, r & 3u, t0s);
}

// kVarWideHeavy: the wide section, launched on the scene's side stream beside the lane kernel
// (its own register allocation: folded into the lane kernel it cost 106 SGPRs and spills)
template <uint32_t G>
__global__ void __launch_bounds__(kWG) k_render_wh(KParams P)
{
    wide_section<false, G>(P, blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
}

// The multi-frame launch (KBatch): the launch's blocks are the frames' blocks, frame-major; the
// heavy-first order (p[0]'s state) ranks them all, and every wave renders its item with its own
// frame's parameters (KParams re-read from the kernarg segment at the frame's offset).
// (The fused variant holds 83 SGPRs: 7 waves / SIMD.  Forced to 8 it spills a VGPR and measured
// slower: rank of 4 / 8 0.256 / 0.139 ms vs 0.241 / 0.136, profiles/r03g_ab_wide_fused_*.json.)
// Wave `wib` of launch block bid of nblk's lane blocks (after the fused wide section's workgroups).
template <int TRI, int VAR>
__device__ __forceinline__ void batch_block_wave(const KBatch& B, uint32_t bid, uint32_t nblk, uint32_t wib,
                                                 volatile uint32_t *t0v)
{
    uint32_t b;
    if (!block_of_launch<VAR>(B.p[0], b, bid, nblk, bid == 0u && wib == 0u && (threadIdx.x & 63u) == 0u)) return;
    const uint32_t gitem = b * kWavesPerWG + wib;                    // launch-wide item
    if constexpr ((VAR & kVarWideHeavy) != 0)
        if (B.p[0].wh_wgs && B.p[0].hf_ver && (B.p[0].wh_mark_in[gitem] & 0x7FFFFFFFu) == B.p[0].hf_ver) return;
    const uint32_t f = batch_frame(B, b);
    const uint32_t off = uint32_t(offsetof(KBatch, p)) + f * uint32_t(sizeof(KParams));
    const uint32_t item = gitem - B.base[f] * kWavesPerWG;
    if constexpr ((VAR & kVarWaveClock) != 0)
    {
        // debug arm: the wave's clocks at its launch-wide item index (rt_debug_wave_clocks; the
        // batch's heavy-first / wide-section machinery runs as in the product launch), with the
        // frame (bits 0-3) and the records it tested in wave-uniform loops (bits 4-31), and its
        // per-lane list iterations
        if ((threadIdx.x & 63u) == 0u)
        {
            wave_counters()[0] = 0u;
            wave_counters()[1] = 0u;
        }
        wave_lds_sync();
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
        process_item<TRI, VAR>(late_params(B.p[0], off), item, off);
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        wave_lds_sync();
        const KParams& Q = late_params(B.p[0], uint32_t(offsetof(KBatch, p)));
        if ((threadIdx.x & 63u) == 0u)
        {
            store_wave_clock(Q.wave_clk, gitem, t0, t1, r0, r1, f | (min(wave_counters()[0], 0x0FFFFFFFu) << 4),
                             wave_counters()[1]);
            if (Q.hf_measure) Q.hf_cost[gitem] = uint32_t(t1 - t0);
        }
        return;
    }
    const bool hf = B.p[0].hf_measure != 0u;
    if (hf && (threadIdx.x & 63u) == 0u) t0v[threadIdx.x >> 6] = uint32_t(__builtin_amdgcn_s_memtime());
    process_item<TRI, VAR>(late_params(B.p[0], off), item, off);
    const KParams& Q = late_params(B.p[0], uint32_t(offsetof(KBatch, p)));
    if (Q.hf_measure)
    {
        const uint32_t t1 = uint32_t(__builtin_amdgcn_s_memtime());
        const uint32_t t0 = __builtin_amdgcn_readfirstlane(t0v[threadIdx.x >> 6]);
        if ((threadIdx.x & 63u) == 0u) Q.hf_cost[__builtin_amdgcn_readfirstlane(gitem)] = t1 - t0;
    }
}

// The multi-frame launch (KBatch): the launch's blocks are the frames' blocks, frame-major; the
// heavy-first order (p[0]'s state) ranks them all, and every wave renders its item with its own
// frame's parameters (KParams re-read from the kernarg segment at the frame's offset).
// (The fused variant holds 83 SGPRs: 7 waves / SIMD.  Forced to 8 it spills a VGPR and measured
// slower: rank of 4 / 8 0.256 / 0.139 ms vs 0.241 / 0.136, profiles/r03g_ab_wide_fused_*.json.)
template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) k_render_batch(KBatch B)
{
    __shared__ uint32_t t0s[kWavesPerWG];
    volatile uint32_t *t0v = t0s;                 // a wave's start time waits in LDS across the walk
    // kVarWideFused: the wide section's wh_wgs workgroups lead the grid (dispatched first, no
    // side stream and no fork / join between the two), the lane blocks follow
    uint32_t bid = blockIdx.x, nblk = gridDim.x;
    if constexpr ((VAR & kVarWideFused) != 0)
    {
        const uint32_t nw = B.p[0].wh_wgs;
        if (bid < nw)
        {
            wide_section<true, (VAR & kVarWideG4) ? 4u : 16u, (VAR & kVarWaveClock) != 0>(
                B.p[0], bid * kWavesPerWG + (threadIdx.x >> 6));
            return;
        }
        bid -= nw;
        nblk -= nw;
    }
    batch_block_wave<TRI, VAR>(B, bid, nblk, threadIdx.x >> 6, t0v);
}

// k_render_batch as one-wave workgroups (k_render_lanes_w64's map): the fused wide section's
// 4 x wh_wgs waves first, then wave r % 4 of lane block (r / 4) * 8 + w % 8, r = w / 8, of the
// p[0].vblocks lane blocks.
template <int TRI, int VAR>
__global__ void __launch_bounds__(64) k_render_batch_w64(KBatch B)
{
    __shared__ uint32_t t0s[1];
    uint32_t w = blockIdx.x;
    if constexpr ((VAR & kVarWideFused) != 0)
    {
        const uint32_t nw = B.p[0].wh_wgs * kWavesPerWG;
        if (w < nw)
        {
            wide_section<true, (VAR & kVarWideG4) ? 4u : 16u, (VAR & kVarWaveClock) != 0>(B.p[0], w);
            return;
        }
        w -= nw;
    }
    const uint32_t r = w / kXcds;
    const uint32_t vbid = (r >> 2) * kXcds + w % kXcds;
    const uint32_t nv = late_params(B.p[0], uint32_t(offsetof(KBatch, p))).vblocks;
    if (vbid >= nv) return;
    batch_block_wave<TRI, VAR>(B, vbid, nv, r & 3u, t0s);
}

template <uint32_t G>
__global__ void __launch_bounds__(kWG) k_render_wh_batch(KBatch B)
{
    wide_section<true, G>(B.p[0], blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
}

// k_render_wh_batch as one-wave workgroups (beside a one-wave lane grid, rt_scene::wg64_wide)
template <uint32_t G>
__global__ void __launch_bounds__(64) k_render_wh_batch_w64(KBatch B)
{
    wide_section<true, G>(B.p[0], blockIdx.x);
}

// RT_KERNEL_COMPACT (grid intersector, spp a power of two <= 64): wavefront active-ray
// compaction.  In the LANES kernel a wave lives until its slowest ray ends, so lanes whose ray
// already hit (or left the grid) idle through the rest of the walk (~23 % of lane-cycles on
// the bench frames).  Here persistent waves keep 64 rays in flight: each iteration walks the
// active lanes cell by cell until `refill` of them have finished, stores the finished samples'
// colours in LDS, and hands the idle lanes fresh samples from the wave's work items with a
// ballot + prefix count (mbcnt) -- the lanes of one refill take consecutive samples, so new
// rays stay spatially coherent.  Items (64 sample slots, as in LANES) are dealt to the waves
// round-robin; a wave holds up to kCompactSlots items whose per-sample colours wait in LDS until
// all 64 are stored, then the pixel sums run over LDS in sample order from 0.0f (hazard H10),
// bit-identical to the shuffle sums of process_item.
constexpr uint32_t kCompactSlots = 4;            // work items in flight per wave
constexpr uint32_t kCompactRefill = 48;          // default: refill when this many lanes idle

struct CompactLds
{
    float col[kWavesPerWG][kCompactSlots][3][64];  // per-sample colours until the item resolves
    uint32_t left[kWavesPerWG][kCompactSlots];     // samples of the slot's item not yet stored
    uint32_t item[kWavesPerWG][kCompactSlots];     // work item held by the slot
};

template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_render_compact(KParams P, uint32_t n_items, uint32_t refill)
{
    __shared__ CompactLds L;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const float ox = P.org[0], oy = P.org[1], oz = P.org[2];
    if (lane < kCompactSlots) L.left[wv][lane] = 0u;
    // wave-uniform bookkeeping
    uint32_t busy = 0u;                          // slots holding an item
    uint32_t feed_slot = 0u, feed_next = 64u;    // next sample slot to hand out (64: none)
    bool drained = false;                        // the global item counter ran out
    // Items are dealt statically, wave w taking w, w + nwaves, ...: neighbouring items cost
    // alike, so the interleave balances, and a global atomic counter measured 2-4x slower
    // (one device-scope atomic per item serialises at the memory side).
    const uint32_t nwaves = gridDim.x * kWavesPerWG;
    uint32_t next_item = blockIdx.x * kWavesPerWG + wv;
    const uint32_t walk_min = 64u - refill;
    // lane state: 0 idle, 1 walking, 2 finished (colour not yet stored)
    uint32_t state = 0u, tag = 0u;
    float dx = 0.0f, dy = 0.0f, dz = 0.0f, t = 0.0f, u = 0.0f, v = 0.0f;
    uint32_t tri = 0u;
    bool hit = false;
    float nct0 = 0.0f, nct1 = 0.0f, nct2 = 0.0f, dt0 = 0.0f, dt1 = 0.0f, dt2 = 0.0f;
    int rem0 = 0, rem1 = 0, rem2 = 0, cs0 = 0, cs1 = 0, cs2 = 0, cell = 0, skip = 0;
    // AUTO's box-run walk (kVarSkipRun + kVarPackedRem: box words present): packed remaining-cell
    // counts and the lane's box counts; a lane inside its empty box steps without a lookup
    constexpr bool BOX = RT_BOX_RUN && (VAR & kVarSkipRun) && (VAR & kVarPackedRem);
    int remp = 0, boxw = 0;
    for (;;)
    {
        // (1) store the colours of finished samples (renderer.cpp:107-121)
        if (state == 2u)
        {
            const uint32_t slot = tag >> 6, j = tag & 63u;
            const ItemCoord ic = item_coord(P, L.item[wv][slot], j);
            float cr = 0.0f, cg = 0.0f, cb = 0.0f;
            if (ic.valid)
            {
                if (hit)
                {
                    if ((VAR & kVarOriginPre) && TRI == RT_TRI_MOLLER_TRUMBORE)
                        tri = __float_as_uint(P.refs[3 * size_t(tri) + 2].y);   // CSR ref -> triangle id
                    const float4 a = P.shade[3 * tri + 0], b = P.shade[3 * tri + 1], c = P.shade[3 * tri + 2];
                    rtd::shade_hit(u, v, a, b, c, cr, cg, cb);
                }
                else
                    cr = cg = cb = float(ic.y) / float(P.H);                    // renderer.cpp:121
                if (P.hits) P.hits[(size_t(ic.y) * P.W + ic.x) * P.spp + ic.s] = hit ? tri : rtd::kNoTri;
            }
            L.col[wv][slot][0][j] = cr;
            L.col[wv][slot][1][j] = cg;
            L.col[wv][slot][2][j] = cb;
            __hip_atomic_fetch_sub(&L.left[wv][slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            state = 0u;
        }
        wave_lds_sync();
        // (2) resolve items whose 64 samples are all stored (renderer.cpp:124-133)
        uint64_t ready = __ballot(lane < kCompactSlots && ((busy >> lane) & 1u) &&
                                  __hip_atomic_load(&L.left[wv][lane < kCompactSlots ? lane : 0u], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP) == 0u);
        while (ready)
        {
            const uint32_t r = uint32_t(__builtin_ctzll(ready));
            ready &= ready - 1u;
            busy &= ~(1u << r);
            const uint32_t item = __builtin_amdgcn_readfirstlane(L.item[wv][r]);
            const ItemCoord ic = item_coord(P, item, lane);
            const uint32_t base = lane & ~(P.spp - 1u);
            float sr = 0.0f, sg = 0.0f, sb = 0.0f;
            for (uint32_t k = 0; k < P.spp; k++)
            {
                sr += L.col[wv][r][0][base + k];
                sg += L.col[wv][r][1][base + k];
                sb += L.col[wv][r][2][base + k];
            }
            if (ic.valid && ic.s == 0)
            {
                const uint32_t word = rtd::pack_bgra8(rtd::gamma_half(average(P, sr)),
                                                      rtd::gamma_half(average(P, sg)),
                                                      rtd::gamma_half(average(P, sb)));
                store_pixel(P, ic.c, ic.p, ic.x, ic.y, word);
            }
        }
        // (3) refill: idle lanes take the next sample slots in lane order (ballot + mbcnt)
        const uint64_t idle = __ballot(state == 0u);
        const uint32_t n_idle = uint32_t(__popcll(idle));
        if (!drained && n_idle >= refill)
        {
            const uint32_t rank = uint32_t(__builtin_amdgcn_mbcnt_hi(uint32_t(idle >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo(uint32_t(idle), 0u)));
            const uint32_t avail = 64u - feed_next;
            uint32_t new_slot = kCompactSlots;
            if (n_idle > avail && busy != (1u << kCompactSlots) - 1u)
            {
                const uint32_t item = next_item;
                next_item += nwaves;
                if (item >= n_items)
                    drained = true;
                else
                {
                    new_slot = uint32_t(__builtin_ctz(~busy));
                    busy |= 1u << new_slot;
                    if (lane == 0u)
                    {
                        L.item[wv][new_slot] = item;
                        L.left[wv][new_slot] = 64u;
                    }
                }
            }
            wave_lds_sync();
            if (state == 0u)
            {
                bool take = false;
                uint32_t slot = 0u, j = 0u;
                if (rank < avail)
                {
                    take = true;
                    slot = feed_slot;
                    j = feed_next + rank;
                }
                else if (new_slot < kCompactSlots)
                {
                    take = true;
                    slot = new_slot;
                    j = rank - avail;
                }
                if (take)
                {
                    tag = (slot << 6) | j;
                    state = 2u;
                    hit = false;
                    const ItemCoord ic = item_coord(P, L.item[wv][slot], j);
                    if (ic.valid)
                    {
                        rtd::dir_from_xy(P.m, P.ndcx[ic.x * P.spp + ic.s], P.ndcy[ic.y * P.spp + ic.s], dx, dy,
                                         dz);
                        if (dda_setup(P, ox, oy, oz, dx, dy, dz, nct0, nct1, nct2, dt0, dt1, dt2, rem0, rem1, rem2,
                                      cs0, cs1, cs2, cell))
                        {
                            state = 1u;
                            t = rtd::kFltMax;
                            skip = 0;
                            if constexpr (BOX)
                            {
                                remp = rem0 | (rem1 << 11) | (rem2 << 22);
                                boxw = kRemGuards;              // look the first cell up
                                cell += box_offset(P, dx, dy, dz);
                            }
                        }
                    }
                }
            }
            if (new_slot < kCompactSlots)
            {
                feed_slot = new_slot;
                feed_next = n_idle - avail;
            }
            else
                feed_next += avail < n_idle ? avail : n_idle;
        }
        // Nothing in flight: after a refill attempt this means the counter is drained and every
        // held item has been resolved (an item is resolved in the iteration its last sample is
        // stored), so the wave is done.
        if (__ballot(state != 0u) == 0u) break;
        // (4) walk the active lanes until `refill` of them have finished (all, once drained)
        const uint32_t wmin = drained ? 0u : walk_min;
        do
        {
            if (BOX && state == 1u)
            {
                // one DDA iteration of the box-run walk (grid_intersect's, per lane: the lanes of a
                // refilled wave are at different points of their walks, so no wave-uniform runs)
                uint32_t kb = 0u, ke = 0u;
                if ((boxw & kRemGuards) != 0)
                {
                    const uint32_t w = P.cellwb[uint32_t(cell)];
                    const uint32_t ne = uint32_t(int(w) >> 31);
                    kb = (w >> 11) & 0xFFFFFu;
                    ke = kb + (w & ne & 2047u);
                    boxw = int(w & ~ne);
                }
                float nct_ax;
                bool more;
                RT_DDA_ADVANCE_BOX(nct_ax, more);
                uint32_t tests = 0u;
                if (kb < ke &&
                    test_cell<false, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests))
                {
                    state = 2u;
                    hit = true;
                }
                else if (!more)                   // terminates: see grid_intersect
                    state = 2u;
            }
            else if (state == 1u)
            {
                uint32_t kb = 0u, ke = 0u;
                if ((VAR & kVarDistSkip) && P.cellw)
                {
                    if (skip == 0)
                    {
                        const uint32_t cw = P.cellw[uint32_t(cell)];
                        const uint32_t cnt = cw & 2047u;
                        kb = cw >> 11;
                        ke = kb + cnt;
                        skip = cnt ? 0 : int(kb) - 1;
                    }
                    else
                        skip--;
                }
                else
                    cell_range(P, uint32_t(cell), kb, ke);
                float nct_ax;
                bool more;
                RT_DDA_ADVANCE_ADD(nct_ax, more);
                uint32_t tests = 0u;
                if (kb < ke &&
                    test_cell<false, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests))
                {
                    state = 2u;
                    hit = true;
                }
                else if (!more)                   // terminates: see grid_intersect
                    state = 2u;
            }
        } while (uint32_t(__popcll(__ballot(state == 1u))) > wmin);
    }
}

// RT_KERNEL_PIXEL_LOOP: one lane per pixel, samples looped in order (any spp)
template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) k_render_pixel_loop(KParams P)
{
    const TileCoord c = tile_of_block(P);
    const uint32_t p = threadIdx.x;
    const uint32_t x = c.tx0 + compact_bits(p), y = c.ty0 + compact_bits(p >> 1);
    if (!(x < P.rx0 + P.rw && y < P.ry0 + P.rh)) return;
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    for (uint32_t s = 0; s < P.spp; s++)
    {
        float cr, cg, cb;
        uint32_t hit_tri;
        trace_sample<false, TRI, VAR>(P, x, y, s, cr, cg, cb, hit_tri, nullptr);
        if (P.hits) P.hits[(size_t(y) * P.W + x) * P.spp + s] = hit_tri;
        sr += cr; sg += cg; sb += cb;
    }
    store_pixel(P, c, p, x, y, rtd::pack_bgra8(rtd::gamma_half(average(P, sr)), rtd::gamma_half(average(P, sg)),
                                               rtd::gamma_half(average(P, sb))));
}

// Debug records: one thread per sample of the rectangle, order (y, x, s)
__global__ void __launch_bounds__(kWG) k_trace_records(KParams P, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = i % P.spp, pix = i / P.spp;
    const uint32_t x = P.rec_x0 + pix % P.rec_w, y = P.rec_y0 + pix / P.rec_w;
    float cr, cg, cb;
    uint32_t ht;
    // Records walk the distance-skipping traversal with the wave-gated test, so the per-sample
    // parity tests (hit, tri, voxel, steps, tests) cover the walk the frames take.
    if (P.isect == RT_ISECT_RAY_MARCH)
        trace_sample<true, RT_TRI_MOLLER_TRUMBORE, kVarMarch>(P, x, y, s, cr, cg, cb, ht, &P.recs[i]);
    else if (P.isect == RT_ISECT_RAY_MARCH + 0x100)   // exhaustive arm (RT_KERNEL_FLAG_EXHAUSTIVE)
        trace_sample<true, RT_TRI_MOLLER_TRUMBORE, kVarMarch | kVarExhaustive>(P, x, y, s, cr, cg, cb, ht, &P.recs[i]);
    else if (P.isect == RT_ISECT_BRUTE_FORCE)
        trace_sample<true, RT_TRI_MOLLER_TRUMBORE, kVarBrute>(P, x, y, s, cr, cg, cb, ht, &P.recs[i]);
    else if (P.tri_test == RT_TRI_BARYCENTRIC)
        trace_sample<true, RT_TRI_BARYCENTRIC, kVarDistSkip>(P, x, y, s, cr, cg, cb, ht, &P.recs[i]);
    else
        trace_sample<true, RT_TRI_MOLLER_TRUMBORE, kVarWaveGate | kVarDistSkip>(P, x, y, s, cr, cg, cb, ht, &P.recs[i]);
}

// rt_render_records_device: the raw records (store_record) of the rectangle made final -- a hit's CSR
// reference becomes Grid::Intersect's tri_idx (the reference's triangle) and the cell whose list holds it
// (the cell the hit was accepted in, grid.cpp:258-271); a miss's end cell leaves its copy of the cell
// words (the ray's direction again, camera.h:8-47, picks the copy).  Records no launch wrote are left.
__global__ void __launch_bounds__(kWG) k_record_fixup(KParams P, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t *o = reinterpret_cast<uint32_t *>(P.recs + i);
    const uint32_t fl = o[11];
    if ((fl & 0xFFFF0000u) != kRecMagic) return;
    if (fl & kRecRawCsr)
    {
        const uint32_t k = o[1];
        o[1] = __float_as_uint(P.refs[3 * size_t(k) + 2].y);
        o[2] = cell_of_ref(P, k);
    }
    else if (fl & (kRecRawBox | kRecRawOct))
    {
        const uint32_t s = i % P.spp, pix = i / P.spp;
        const uint32_t x = P.rec_x0 + pix % P.rec_w, y = P.rec_y0 + pix / P.rec_w;
        float dx, dy, dz;
        rtd::dir_from_xy(P.m, P.ndcx[x * P.spp + s], P.ndcy[y * P.spp + s], dx, dy, dz);
        o[2] -= uint32_t((fl & kRecRawBox) ? box_offset(P, dx, dy, dz) : oct_offset(P, dx, dy, dz));
    }
    o[11] = 0u;
}

// K3: gathered shards [rank][local tile][256] -> frame
__global__ void __launch_bounds__(kWG) k_unshard(const uint32_t *g, uint32_t *out, uint32_t W, uint32_t H,
                                                 uint32_t tiles_x, uint32_t nranks, uint64_t shard_elems)
{
    const uint32_t x = blockIdx.x * 64 + (threadIdx.x & 63u);
    const uint32_t y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    // the inverse of shard_tile_xy's deal
    const uint32_t ty = y / kTile, rot = nranks > 1u ? (kShardRot * ty) % tiles_x : 0u;
    const uint32_t tr = x / kTile + rot;
    const uint32_t t = ty * tiles_x + (tr >= tiles_x ? tr - tiles_x : tr);
    const uint32_t r = t % nranks, k = t / nranks;
    out[size_t(y) * W + x] = g[r * shard_elems + size_t(k) * kTilePix + (y % kTile) * kTile + (x % kTile)];
}

// Per-camera-origin records (kVarOriginPre): for CSR reference k, tvec = o - v0,
// qvec = tvec x e1 and DOT(e2, qvec) exactly as triangle.h:82, 90, 98 compute them, in the
// packed-pair layout of rtd::make_frec (64 B per reference).
__global__ void __launch_bounds__(kWG) k_origin_pre(const float4 *refs, float4 *frefs, uint32_t n, float ox,
                                                    float oy, float oz)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float4 r0 = refs[3 * size_t(k)], r1 = refs[3 * size_t(k) + 1], r2 = refs[3 * size_t(k) + 2];
    const rtd::FRec f = rtd::make_frec(ox, oy, oz, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x);
    frefs[4 * size_t(k) + 0] = f.r0;
    frefs[4 * size_t(k) + 1] = f.r1;
    frefs[4 * size_t(k) + 2] = f.r2;
    frefs[4 * size_t(k) + 3] = f.r3;
}

// Device KATs (rt_debug_primitives)
// Exhaustive check of rtd::rcp_nr against the correctly rounded 1.0f / x over every finite
// nonzero float: mismatches counted per biased exponent (bad[256]).
__global__ void __launch_bounds__(kWG) k_rcp_check(unsigned long long *bad)
{
    const uint64_t n = 1ull << 32;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    {
        const uint32_t b = uint32_t(i);
        const uint32_t ex = (b >> 23) & 255u;
        if (ex == 255u || (b & 0x7FFFFFFFu) == 0u) continue;
        const float x = __uint_as_float(b);
        if (__float_as_uint(rtd::rcp_nr(x)) != __float_as_uint(1.0f / x)) atomicAdd(&bad[ex], 1ull);
    }
}

// Exhaustive check of the packed gamma bytes: every non-negative float (bits 0 .. 0x7F800000,
// +inf included), pack_channel of the hardware sqrt vs of the correctly rounded one.
__global__ void __launch_bounds__(kWG) k_gamma_check(unsigned long long *bad)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b <= 0x7F800000u; b += gridDim.x * blockDim.x)
    {
        const float x = __uint_as_float(b);
        if (rtd::pack_channel(rtd::gamma_fast(x)) != rtd::pack_channel(rtd::gamma_half(x))) atomicAdd(bad, 1ull);
        if (b == 0x7F800000u) break;
    }
}

__global__ void __launch_bounds__(kWG) k_primitives(int kind, const float *in, uint32_t n, float *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (kind == 0)
    {
        const float *a = in + 18 * i;
        float *o = out + 8 * i;
        const float e1x = a[9] - a[6], e1y = a[10] - a[7], e1z = a[11] - a[8];
        const float e2x = a[12] - a[6], e2y = a[13] - a[7], e2z = a[14] - a[8];
        float t = __builtin_nanf(""), u = t, v = t;
        const bool h = rtd::ray_tri_mt(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
                                       e1x, e1y, e1z, e2x, e2y, e2z, t, u, v);
        o[0] = __uint_as_float(h); o[1] = t; o[2] = u; o[3] = v;
        float bt = __builtin_nanf(""), bu = bt, bv = bt;
        const bool hb = rtd::ray_tri_bary(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
                                          e1x, e1y, e1z, e2x, e2y, e2z, a[15], a[16], a[17], bt, bu, bv);
        o[4] = __uint_as_float(hb); o[5] = bt; o[6] = bu; o[7] = bv;
    }
    else if (kind == 6)   // the wave-gated forms (64 records per wave, so the exits really fire):
    {                     // gated MT, and the per-camera-record form with the Newton 1/det
        const float *a = in + 18 * i;
        float *o = out + 8 * i;
        const float e1x = a[9] - a[6], e1y = a[10] - a[7], e1z = a[11] - a[8];
        const float e2x = a[12] - a[6], e2y = a[13] - a[7], e2z = a[14] - a[8];
        float t = 0, u = 0, v = 0, pt = 0, pu = 0, pv = 0;
        const bool hg = rtd::ray_tri_mt_gated(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
                                              e1x, e1y, e1z, e2x, e2y, e2z, t, u, v);
        const rtd::FRec fr = rtd::make_frec(a[0], a[1], a[2], a[6], a[7], a[8], e1x, e1y, e1z, e2x, e2y, e2z);
        const bool hp = rtd::ray_tri_frec_gated<true>(rtd::f2v{a[3], a[4]}, rtd::f2v{a[4], a[5]}, fr, pt, pu, pv);
        o[0] = __uint_as_float(hg); o[1] = t; o[2] = u; o[3] = v;
        o[4] = __uint_as_float(hp); o[5] = pt; o[6] = pu; o[7] = pv;
    }
    else if (kind == 5)   // branch-free traversal variants: hit flag + t,u,v (hits only)
    {
        const float *a = in + 18 * i;
        float *o = out + 8 * i;
        const float e1x = a[9] - a[6], e1y = a[10] - a[7], e1z = a[11] - a[8];
        const float e2x = a[12] - a[6], e2y = a[13] - a[7], e2z = a[14] - a[8];
        float t, u, v, bt, bu, bv;
        const bool h = rtd::ray_tri_mt_pred(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
                                            e1x, e1y, e1z, e2x, e2y, e2z, t, u, v);
        const bool hb = rtd::ray_tri_bary_pred(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8],
                                               e1x, e1y, e1z, e2x, e2y, e2z, a[15], a[16], a[17], bt, bu, bv);
        o[0] = __uint_as_float(h); o[1] = t; o[2] = u; o[3] = v;
        o[4] = __uint_as_float(hb); o[5] = bt; o[6] = bu; o[7] = bv;
    }
    else if (kind == 7)   // DistancePointTri over the scene's distance record
    {
        const float4 *a = reinterpret_cast<const float4 *>(in + 28 * size_t(i));
        out[i] = rtd::dist_point_tri(a[0].x, a[0].y, a[0].z, a[1], a[2], a[3], a[4], a[5], a[6]);
    }
    else if (kind == 1)
    {
        const float *a = in + 12 * i;
        float *o = out + 4 * i;
        float t0 = __builtin_nanf(""), t1 = t0;
        const bool h = rtd::ray_aabb(a[0], a[1], a[2], a[3], a[4], a[5], a + 6, a + 9, t0, t1);
        o[0] = __uint_as_float(h); o[1] = t0; o[2] = t1;
        o[3] = __uint_as_float(rtd::point_in_aabb(a[0], a[1], a[2], a + 6, a + 9));
    }
    else if (kind == 2)
    {
        // camera inputs: cam[16], px, py, W, H (u32 bits), sx, sy, fov; constants as the host does
        const float *a = in + 23 * i;
        float *o = out + 6 * i;
        const float m[9] = { a[0], a[1], a[2], a[4], a[5], a[6], a[8], a[9], a[10] };
        const uint32_t W = __float_as_uint(a[18]), H = __float_as_uint(a[19]);
        const float fov_xs = a[22];          // replaced on the host by (float)tan(double) (H5)
        const float aspect = float(W) / float(H);
        float dx, dy, dz;
        rtd::gen_dir(m, fov_xs, aspect, __float_as_uint(a[16]), __float_as_uint(a[17]), W, H, a[20], a[21],
                     dx, dy, dz);
        o[0] = 0.0f * a[0] + 0.0f * a[4] + 0.0f * a[8] + a[12];
        o[1] = 0.0f * a[1] + 0.0f * a[5] + 0.0f * a[9] + a[13];
        o[2] = 0.0f * a[2] + 0.0f * a[6] + 0.0f * a[10] + a[14];
        o[3] = dx; o[4] = dy; o[5] = dz;
    }
    else if (kind == 3)
    {
        const float *a = in + 3 * i;
        float *o = out + 4 * i;
        const float r = rtd::gamma_half(a[0]), g = rtd::gamma_half(a[1]), b = rtd::gamma_half(a[2]);   // the resolve's
        o[0] = r; o[1] = g; o[2] = b; o[3] = __uint_as_float(rtd::pack_bgra8(r, g, b));
    }
    else if (kind == 4)
    {
        const float *a = in + 11 * i;
        float *o = out + 3 * i;
        const float4 A = make_float4(a[2], a[3], a[4], a[5]);
        const float4 B = make_float4(a[6], a[7], a[8], a[9]);
        const float4 C = make_float4(a[10], 0.0f, 0.0f, 0.0f);
        rtd::shade_hit(a[0], a[1], A, B, C, o[0], o[1], o[2]);
    }
}

// ------------------------------------------------------------------------ host side
// sampling.h:113-120, sampling.cpp:194-210 (base 2), renderer.cpp:52-55
void hammersley(uint32_t spp, std::vector<float>& xy)
{
    xy.resize(size_t(spp) * 2);
    for (uint32_t s = 0; s < spp; s++)
    {
        double val = 0.0, inv_i = 0.5;
        for (uint32_t n = s; n > 0; n /= 2)
        {
            val += (n % 2) * inv_i;
            inv_i *= 0.5;
        }
        xy[2 * s + 0] = float(double(s) / double(spp) - 0.5f);
        xy[2 * s + 1] = float(val - 0.5f);
    }
}

bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }

uint32_t log2u(uint32_t x)
{
    uint32_t r = 0;
    while ((1u << r) < x) r++;
    return r;
}

// Dot (lin_alg.h:138-144), accumulating from T() = 0
float dot_ref(const float *a, const float *b)
{
    float r = 0.0f;
    r += a[0] * b[0];
    r += a[1] * b[1];
    r += a[2] * b[2];
    return r;
}

// Distance record of one triangle (layout: rtd::dist_point_tri); the position-independent
// terms of ComputeBarycentric / LineSegMinDistSq (triangle.h:140-150, 166-167)
void dist_record(const float *p0, const float *p1, const float *p2, float4 *r)
{
    const float e0[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };
    const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };
    const float e12[3] = { p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2] };
    const float d00 = dot_ref(e0, e0), d01 = dot_ref(e0, e1), d11 = dot_ref(e1, e1);
    const float inv_denom = 1 / (d00 * d11 - d01 * d01);
    r[0] = make_float4(p0[0], p0[1], p0[2], p1[0]);
    r[1] = make_float4(p1[1], p1[2], p2[0], p2[1]);
    r[2] = make_float4(p2[2], e0[0], e0[1], e0[2]);
    r[3] = make_float4(e1[0], e1[1], e1[2], e12[0]);
    r[4] = make_float4(e12[1], e12[2], d00, d01);
    r[5] = make_float4(d11, inv_denom, dot_ref(e12, e12), 0.0f);
}

// Heavy-first state of one launch shape (device arrays; see KParams::hf_*)
struct HfCtx
{
    uint64_t key[5] = { 0, 0, 0, 0, 0 };   // launch shape: blocks, spp, region, shard, variant, batch
    uint32_t nblocks = 0, front = 0;
    uint32_t cap_blocks = 0;            // allocated marks per buffer
    uint32_t *marks = nullptr;          // [2][cap_blocks]
    uint32_t *cost = nullptr;           // [cap_blocks * kWavesPerWG] wave cycles of the last frame
    uint32_t *lists = nullptr;          // [2][kHfFrontMax], by plan version parity
    HfPlan *plans = nullptr;            // [2], by plan version parity
    uint32_t *ticket = nullptr;         // k_hf_plan's workgroup ticket
    uint32_t *wh_marks = nullptr;       // [2][cap_blocks * kWavesPerWG] wide items, by version parity
    uint32_t *wh_lists = nullptr;       // [2][kWhMax]
    uint32_t *wh_cnt = nullptr;         // host-mapped: the newest plan's wide item count
    uint32_t frames = 0;                // frames rendered with this shape
    uint32_t ver = 0;                   // version of the newest plan launched
    uint64_t used = 0;                  // LRU stamp
    uint64_t cam = 0;                   // camera signature of the last frame (cam_signature)
};

} // namespace

constexpr uint32_t kTimeRing = 64;  // rt_kernel_times: launches kept
constexpr uint32_t kTimeEvery = 8;  // default: every 8th launch gets the timed event pair
constexpr uint32_t kMaxBands = 64;   // rt_render_frame_host: row bands per frame
constexpr uint32_t kTileBands = 8;   // rt_render_tiles: D2H bands overlapped with the scatter

struct rt_scene
{
    int device = 0;
    std::mutex mtx;
    uint32_t dims[3] = { 0, 0, 0 };
    float bmin[3], bmax[3], cw = 0, icw = 0;
    uint32_t ncells = 0, nrefs = 0, ntris = 0, max_cell_refs = 0;
    uint32_t *d_off = nullptr, *d_cellw = nullptr, *d_cellwo = nullptr, oct_stride = 0;
    uint32_t *d_cellwb = nullptr, box_stride = 0;  // box-run words: 24 copies (octant x major axis)
    float4 *d_refs = nullptr, *d_shade = nullptr, *d_facen = nullptr, *d_frefs = nullptr;
    float4 *d_trimt = nullptr, *d_tridist = nullptr, *d_distblk = nullptr;
    uint32_t ndist_blk = 0;
    float scene_scale = 0.0f;
    float vmin[3] = { 0, 0, 0 }, vmax[3] = { 0, 0, 0 };
    uint64_t device_bytes = 0;
    uint32_t compact_wgs = 2048;    // RT_KERNEL_COMPACT grid: 8 x 256-lane workgroups per CU
    bool rcp_safe = false;          // every |det| of the ray/tri test is far below 2^126 (FAST_RCP)
    bool pack_ok = false;           // dims <= 512: the remaining-cell counts pack into one word
    // frefs hold the per-reference terms of this camera origin (bit patterns; valid once computed)
    bool fref_valid = false;
    uint32_t fref_org[3] = { 0, 0, 0 };
    uint64_t *d_clk = nullptr;      // RT_KERNEL_FLAG_WAVE_CLOCK records of the last such launch
    size_t clk_cap = 0;
    uint32_t clk_items = 0;
    // AUTO heavy-first order: per launch shape, which blocks the previous frame found heavy
    HfCtx hf[kHfCtxs];
    uint64_t hf_clock = 0;
    uint64_t hf_evictions = 0;      // launch shapes that displaced another's state (rt_scene_info)
    uint64_t batch_launches = 0;    // rt_render_batch_device chunks led by this scene: one launch ...
    uint64_t batch_fallbacks = 0;   // ... or one launch per frame (frames that cannot share a launch)
    // scheduling tunables, read ONCE from the environment at rt_scene_create (A/B sweeps): the
    // launch path never calls getenv
    uint32_t hf_floor = 100000;     // RT_HF_FLOOR: heavy-first threshold floor, shader cycles
    uint32_t hf_min_blocks = 4096;  // RT_HF_MIN_BLOCKS: smallest whole launch taking the heavy-first order
    uint32_t wh_floor = 100000;     // RT_WH_FLOOR: wide-section threshold floor, shader cycles
    uint32_t wh_alpha16 = 32;       // RT_WH_ALPHA16: wide threshold, sixteenths of the estimated span
    uint32_t wh_alpha16_n2 = 16;    // RT_WH_ALPHA16_N2: the same for a rank of 2 of a batched step
    uint32_t wh_alpha16_n4 = 28;    // RT_WH_ALPHA16_N4: the same for a rank of 3-7 of a batched step
    uint32_t wh_beta16 = 0;         // RT_WH_BETA16: the second tier's threshold (4 lanes per sample),
    uint32_t wh_beta16_n2 = 0;      // sixteenths of the span estimate, for a rank of >= 8 / of 2
    uint32_t wh_beta16_n4 = 0;      // (RT_WH_BETA16_N2) / of 3-7 (RT_WH_BETA16_N4); 0: one tier
                                    // (measured, profiles/r03o_alpha_n2_sweep.json)
    uint32_t wh_auto_refs = 128;    // RT_WH_AUTO_REFS: AUTO takes the wide section for >= 2-rank
                                    // shards of scenes with a cell list this long
    uint32_t wh_fused = 1;          // RT_WH_FUSED: a batch's wide section leads the batch kernel's grid
                                    // (0: its own kernel on the side stream, fork / join)
    uint32_t wg64 = 1;              // RT_WG64: AUTO launches of >= wg64_min_blocks 256-lane blocks run
    uint32_t wg64_min_blocks = 8192; // as one-wave workgroups (k_render_lanes_w64; RT_WG64_MIN_BLOCKS)
    uint32_t wg64_batch_min_blocks = 0;  // the same for batched launches (RT_WG64_BATCH_MIN_BLOCKS)
    uint32_t wg64_wide = 0xA;       // RT_WG64_WIDE: bit log2(N) (3: N >= 8): one-wave workgroups also
                                    // for a rank of N's batch with a wide section
    uint32_t wh_fused_min_ranks = 2; // RT_WH_FUSED_MIN_RANKS: smallest rank count of a fused section
    uint32_t hf_follow = 1;         // RT_HF_FOLLOW: re-plan the heavy-first order on every frame whose
                                    // camera moved (0: every kHfPeriod-th frame only)
    bool octant_words = false;      // 8 ray-octant copies of the empty-run words (else one L-inf word)
    bool box_words = false;         // 24 box-run word copies: AUTO's empty runs (kVarSkipRun)
    // camera-space x / y tables of the current frame shape (prepare_ndc)
    float *d_ndc = nullptr;
    size_t ndc_cap = 0;
    std::vector<float> ndc_key;
    uint32_t ndc_w = 0, ndc_spp = 0;
    // the frame description the tables above were built for (prepare_samples' fast check: width,
    // height, spp, fov bits and the caller's sample table; no table rebuild per launch)
    uint32_t fp_w = 0, fp_h = 0, fp_spp = 0, fp_fov = 0;
    bool fp_valid = false, fp_custom = false;
    std::vector<float> fp_tbl;
    // sample table cache
    float2 *d_smp = nullptr;
    uint32_t smp_cap = 0;
    std::vector<float> smp_host;
    float *h_smp_pinned = nullptr;
    // internal stream + timing events
    hipStream_t stream = nullptr;
    hipEvent_t ev1 = nullptr;       // after each launch's last kernel (ordering only, no timestamp)
    bool ev_recorded = false;
    // render-kernel-only timing: event pair around the render kernel(s) of each launch (not the
    // heavy-first planning kernels), a ring of the last kTimeRing launches (rt_kernel_times)
    hipEvent_t kt0[kTimeRing] = {}, kt1[kTimeRing] = {};
    uint32_t kt_next = 0, kt_count = 0;
    uint32_t kt_last = kTimeRing;   // ring slot of the last timed launch (kTimeRing: none)
    uint32_t time_every = kTimeEvery; // rt_scene_set_timing: time every n-th launch (0: none)
    uint64_t launches = 0;
    hipStream_t last_stream = nullptr;  // stream of the last launch (cross-stream ordering)
    // RT_KERNEL_FLAG_WIDE_HEAVY: side stream of the wide section, fork / join events
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // staging for rt_render_tiles / records
    uint32_t *d_frame = nullptr;
    size_t frame_cap = 0;
    uint32_t *h_frame = nullptr;
    size_t hframe_cap = 0;
    // D2H row bands: rt_render_frame_host's (band_ev/band_y1, read by rt_frame_host_wait) and
    // rt_render_tiles' own (tile_ev), each event recorded after its band's copy
    hipEvent_t band_ev[kMaxBands] = {};
    uint32_t band_y1[kMaxBands] = {};
    uint32_t nbands = 0;
    hipEvent_t tile_ev[kTileBands] = {};
    // rt_render_frame_host_tiled: the second launch stream of its row-band launches and the fork
    // event (the frame's per-origin records ready) / join event (the other stream's work done)
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_t_fork = nullptr, ev_t_join = nullptr;
};

namespace {

// AUTO's packed counts + empty-run loop: dims <= 512 and (box-run build) the box words exist
bool auto_runs(const rt_scene *s)
{
    return s->pack_ok && (RT_BOX_RUN == 0 || s->box_words);
}

int ensure_device(const rt_scene *s)
{
    int cur = -1;
    RT_HIP(hipGetDevice(&cur));
    if (cur != s->device) RT_HIP(hipSetDevice(s->device));
    return RT_OK;
}

// Uploads the frame's sample table if it differs from the cached one.
// The scene's per-frame constants that live in device memory are rewritten only after its last
// launch has finished with them (launches are asynchronous; the copies are not stream-ordered).
int wait_scene_idle(rt_scene *s)
{
    if (s->ev_recorded) RT_HIP(hipEventSynchronize(s->ev1));
    return RT_OK;
}

// camera.h:41-42 fov_xs = (float)tan(double(DegToRad(fov) / 2)) (H5), computed on the host
float fov_xs_of(const rt_frame *f)
{
    const float hfov = f->fov * float(0.0174532925);           // lin_alg.h:232 DegToRad
    return float(::tan(double(hfov / 2.0f)));
}

// Camera-space x per (column, sample) and y per (row, sample) of GenerateRay (camera.h:20-21,
// 40-42): the only parts of a ray's direction that depend on the pixel and the sample offsets
// alone, computed here with the kernels' own operations (rtd::cam_x / cam_y: IEEE float on the
// host too, no contraction) and uploaded when the frame shape changes.  tbl = the sample table.
std::vector<float> ndc_key(const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    std::vector<float> key = { float(f->width), float(f->height), float(spp), fov_xs_of(f),
                               float(f->width) / float(f->height) };
    key.insert(key.end(), tbl.begin(), tbl.end());
    return key;
}

// the sample table of a frame (rt_frame.sample_offsets, or the Hammersley table)
std::vector<float> sample_table(const rt_frame *f, uint32_t spp)
{
    std::vector<float> tbl;
    if (f->sample_offsets)
        tbl.assign(f->sample_offsets, f->sample_offsets + 2 * size_t(spp));
    else
        hammersley(spp, tbl);
    return tbl;
}

int prepare_ndc(rt_scene *s, const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    const float fx = fov_xs_of(f), aspect = float(f->width) / float(f->height);
    std::vector<float> key = ndc_key(f, spp, tbl);
    if (key == s->ndc_key) return RT_OK;
    const size_t n = (size_t(f->width) + f->height) * spp;
    std::vector<float> h(n);
    for (uint32_t x = 0; x < f->width; x++)
        for (uint32_t k = 0; k < spp; k++) h[size_t(x) * spp + k] = rtd::cam_x(x, tbl[2 * k], f->width, fx);
    float *hy = h.data() + size_t(f->width) * spp;
    for (uint32_t y = 0; y < f->height; y++)
        for (uint32_t k = 0; k < spp; k++) hy[size_t(y) * spp + k] = rtd::cam_y(y, tbl[2 * k + 1], f->height, fx, aspect);
    if (int rc = wait_scene_idle(s)) return rc;
    if (n > s->ndc_cap)
    {
        if (s->d_ndc) RT_HIP(hipFree(s->d_ndc));
        s->d_ndc = nullptr;
        s->ndc_cap = 0;
        RT_HIP(hipMalloc(&s->d_ndc, n * sizeof(float)));
        s->ndc_cap = n;
    }
    RT_HIP(hipMemcpy(s->d_ndc, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    s->ndc_key = key;
    s->ndc_w = f->width;
    s->ndc_spp = spp;
    return RT_OK;
}

int remember_tables(rt_scene *s, const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    s->fp_w = f->width;
    s->fp_h = f->height;
    s->fp_spp = spp;
    std::memcpy(&s->fp_fov, &f->fov, 4);
    s->fp_custom = f->sample_offsets != nullptr;
    s->fp_tbl = tbl;
    s->fp_valid = true;
    return RT_OK;
}

// true when the scene's camera-space and sample tables are those of this frame (no host work)
bool tables_match(const rt_scene *s, const rt_frame *f, uint32_t spp)
{
    uint32_t fov;
    std::memcpy(&fov, &f->fov, 4);
    if (!s->fp_valid || s->fp_w != f->width || s->fp_h != f->height || s->fp_spp != spp || s->fp_fov != fov ||
        s->fp_custom != (f->sample_offsets != nullptr))
        return false;
    return !f->sample_offsets || std::memcmp(s->fp_tbl.data(), f->sample_offsets, sizeof(float) * 2 * spp) == 0;
}

int prepare_samples(rt_scene *s, const rt_frame *f, uint32_t spp)
{
    if (tables_match(s, f, spp)) return RT_OK;
    s->fp_valid = false;
    const std::vector<float> tbl = sample_table(f, spp);
    if (int rc = prepare_ndc(s, f, spp, tbl)) return rc;
    if (tbl == s->smp_host) return remember_tables(s, f, spp, tbl);
    if (int rc = wait_scene_idle(s)) return rc;
    if (spp > s->smp_cap)
    {
        if (s->d_smp) RT_HIP(hipFree(s->d_smp));
        if (s->h_smp_pinned) RT_HIP(hipHostFree(s->h_smp_pinned));
        s->d_smp = nullptr;
        s->h_smp_pinned = nullptr;
        const uint32_t cap = std::max<uint32_t>(64, spp);
        RT_HIP(hipMalloc(&s->d_smp, sizeof(float2) * cap));
        RT_HIP(hipHostMalloc(&s->h_smp_pinned, sizeof(float2) * cap));
        s->smp_cap = cap;
    }
    std::memcpy(s->h_smp_pinned, tbl.data(), tbl.size() * sizeof(float));
    RT_HIP(hipMemcpy(s->d_smp, s->h_smp_pinned, tbl.size() * sizeof(float), hipMemcpyHostToDevice));
    s->smp_host = tbl;
    return remember_tables(s, f, spp, tbl);
}

constexpr uint32_t kKernelFlags = RT_KERNEL_FLAG_WIDE_HEAVY | RT_KERNEL_FLAG_EXHAUSTIVE |
                                  RT_KERNEL_FLAG_WAVE_CLOCK | RT_KERNEL_BUDGET_MASK;

int validate_frame(const rt_frame *f)
{
    if (!f) return fail(RT_E_INVALID, "frame is NULL");
    if (f->width == 0 || f->height == 0 || f->width > 65536 || f->height > 65536)
        return fail(RT_E_INVALID, "frame width/height must be in [1, 65536]");
    if (f->tri_test > RT_TRI_BARYCENTRIC) return fail(RT_E_INVALID, "unknown tri_test");
    if (f->intersector > RT_ISECT_RAY_MARCH) return fail(RT_E_INVALID, "unknown intersector");
    if (f->intersector == RT_ISECT_BRUTE_FORCE && f->tri_test != RT_TRI_MOLLER_TRUMBORE)
        return fail(RT_E_INVALID, "IntersectBruteForce uses IntersectRayTri only (renderer.cpp:176)");
    const uint32_t kind = f->kernel & RT_KERNEL_KIND_MASK;
    if (kind > RT_KERNEL_COMPACT || (f->kernel & ~(RT_KERNEL_KIND_MASK | kKernelFlags)))
        return fail(RT_E_INVALID, "unknown or removed kernel kind / flag");
    const uint32_t spp = std::max(1u, f->spp);
    if (spp > 4096) return fail(RT_E_INVALID, "spp must be <= 4096");
    if (kind == RT_KERNEL_COMPACT && ((f->kernel & RT_KERNEL_BUDGET_MASK) >> RT_KERNEL_BUDGET_SHIFT) > 64u)
        return fail(RT_E_INVALID, "compaction refill threshold must be <= 64 lanes");
    if ((kind == RT_KERNEL_LANES || kind == RT_KERNEL_COMPACT) && !(is_pow2(spp) && spp <= 64))
        return fail(RT_E_INVALID, "RT_KERNEL_LANES needs spp to be a power of two <= 64");
    return RT_OK;
}

// Fills the per-frame parameters (camera constants exactly as camera.h computes them).
void frame_params(const rt_scene *s, const rt_frame *f, KParams& P)
{
    std::memset(&P, 0, sizeof(P));
    const float (*c)[4] = reinterpret_cast<const float (*)[4]>(f->cam);
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++) P.m[3 * r + k] = c[r][k];
    P.fov_xs = fov_xs_of(f);                                    // camera.h:42, double tan (H5)
    P.aspect = float(f->width) / float(f->height);
    P.ndcx = s->d_ndc;                                          // prepare_ndc (this frame's shape)
    P.ndcy = s->d_ndc + size_t(s->ndc_w) * s->ndc_spp;
    for (int k = 0; k < 3; k++)                                 // lin_alg.h:518-535
        P.org[k] = 0.0f * c[0][k] + 0.0f * c[1][k] + 0.0f * c[2][k] + c[3][k];
    P.W = f->width;
    P.H = f->height;
    P.spp = std::max(1u, f->spp);
    P.spp_shift = is_pow2(P.spp) ? log2u(P.spp) : 0;
    P.inv_spp = is_pow2(P.spp) ? 1.0f / float(P.spp) : 0.0f;
    P.smp = s->d_smp;
    for (int a = 0; a < 3; a++)
    {
        P.bmin[a] = s->bmin[a];
        P.bmax[a] = s->bmax[a];
        P.dim[a] = int(s->dims[a]);
    }
    P.cw = s->cw;
    P.icw = s->icw;
    P.dxdz = int(s->dims[0] * s->dims[2]);
    P.max_steps = s->dims[0] + s->dims[1] + s->dims[2] + 3;
    P.off = s->d_off;
    P.cellw = s->d_cellw;
    P.cellwo = s->d_cellwo ? s->d_cellwo : s->d_cellw;
    P.oct_stride = s->d_cellwo ? s->oct_stride : 0u;
    P.cellwb = s->d_cellwb;
    P.box_stride = s->box_stride;
    P.refs = s->d_refs;
    P.frefs = s->d_frefs;
    P.shade = s->d_shade;
    P.face_n = s->d_facen;
    P.tri_mt = s->d_trimt;
    P.tri_dist = s->d_tridist;
    P.dist_blk = s->d_distblk;
    P.ndist_blk = s->ndist_blk;
    P.scene_scale = s->scene_scale;
    for (int a = 0; a < 3; a++)
    {
        P.smin[a] = s->vmin[a];
        P.smax[a] = s->vmax[a];
    }
    P.ntris = s->ntris;
    P.tri_test = f->tri_test;
    P.isect = f->intersector;
}

bool use_lanes(const rt_frame *f, uint32_t spp)
{
    if ((f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_PIXEL_LOOP) return false;
    return is_pow2(spp) && spp <= 64;
}

// The per-reference origin terms for this frame's camera origin: computed when the origin
// differs from the one the records hold (a moving camera pays one small launch per frame).
int ensure_origin_terms(rt_scene *s, const KParams& P, hipStream_t st)
{
    uint32_t ob[3];
    std::memcpy(ob, P.org, sizeof(ob));
    if (s->fref_valid && std::memcmp(ob, s->fref_org, sizeof(ob)) == 0) return RT_OK;
    if (s->nrefs)
        hipLaunchKernelGGL(k_origin_pre, dim3((s->nrefs + kWG - 1) / kWG), dim3(kWG), 0, st, s->d_refs, s->d_frefs,
                           s->nrefs, P.org[0], P.org[1], P.org[2]);
    RT_HIP(hipGetLastError());
    std::memcpy(s->fref_org, ob, sizeof(ob));
    s->fref_valid = true;
    return RT_OK;
}

constexpr uint32_t kWhRefresh = 128;        // frames between refresh frames (a multiple of kHfPeriod)

// One tunable from the environment (rt_scene_create only).
uint32_t env_tunable(const char *name, uint32_t dflt)
{
    const char *e = std::getenv(name);
    return e && *e ? uint32_t(std::strtoul(e, nullptr, 0)) : dflt;
}

// The camera of a frame as one 64-bit signature (FNV-1a over the bits of the rotation, the origin
// and the field of view): heavy-first plans are re-measured when it changes between frames.
uint64_t cam_signature(const KParams& P, uint64_t h = 0xcbf29ce484222325ull)
{
    float v[13];
    std::memcpy(v, P.m, sizeof(P.m));
    std::memcpy(v + 9, P.org, sizeof(P.org));
    v[12] = P.fov_xs;
    const unsigned char *b = reinterpret_cast<const unsigned char *>(v);
    for (size_t i = 0; i < sizeof(v); i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

// Heavy-first state for this launch shape (AUTO): fills P.hf_*.  A new shape takes the least
// recently used context and clears it on the launch stream (no host synchronisation).
// batch: 0 for a single-frame launch, else an identity of the batch (its scenes and frame count).
int hf_prepare(rt_scene *s, KParams& P, uint64_t blocks, int var, bool front, hipStream_t st, uint64_t batch = 0,
               uint64_t cam_sig = 0)
{
    if (!batch) cam_sig = cam_signature(P);
    const uint64_t key[5] = { (blocks << 16) | (uint64_t(P.spp) << 1) | 1u,
                              (uint64_t(P.rx0) << 32) | P.ry0, (uint64_t(P.rw) << 32) | P.rh,
                              (uint64_t(P.rank) << 40) | (uint64_t(P.nranks) << 20) | uint64_t(uint32_t(var) >> 12),
                              batch };
    HfCtx *c = nullptr;
    for (HfCtx& h : s->hf)
        if (std::memcmp(h.key, key, sizeof(key)) == 0) c = &h;
    if (!c)
    {
        c = &s->hf[0];
        for (HfCtx& h : s->hf)
            if (h.used < c->used) c = &h;
        if (c->used) s->hf_evictions++;
        // invalidated first: if an allocation below fails, no later launch may match the old
        // shape and read freed (null) state arrays
        std::memset(c->key, 0, sizeof(c->key));
        c->frames = 0;
        c->ver = 0;
        if (blocks > c->cap_blocks || !c->lists)
        {
            c->cap_blocks = 0;
            if (c->marks) RT_HIP(hipFree(c->marks));
            if (c->cost) RT_HIP(hipFree(c->cost));
            if (c->wh_marks) RT_HIP(hipFree(c->wh_marks));
            c->marks = c->cost = c->wh_marks = nullptr;
            RT_HIP(hipMalloc(&c->marks, sizeof(uint32_t) * 2 * blocks));
            RT_HIP(hipMalloc(&c->cost, sizeof(uint32_t) * kWavesPerWG * blocks));
            RT_HIP(hipMalloc(&c->wh_marks, sizeof(uint32_t) * 2 * kWavesPerWG * blocks));
            if (!c->lists)
            {
                RT_HIP(hipMalloc(&c->plans, sizeof(HfPlan) * 2));
                RT_HIP(hipMalloc(&c->ticket, sizeof(uint32_t)));
                RT_HIP(hipMalloc(&c->wh_lists, sizeof(uint32_t) * 2 * 2 * kWhMax));   // [version][tier][kWhMax]
                RT_HIP(hipHostMalloc(&c->wh_cnt, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
                RT_HIP(hipMalloc(&c->lists, sizeof(uint32_t) * 2 * kHfFrontMax));   // last: marks completion
            }
            c->cap_blocks = uint32_t(blocks);
        }
        RT_HIP(hipMemsetAsync(c->marks, 0, sizeof(uint32_t) * 2 * c->cap_blocks, st));
        RT_HIP(hipMemsetAsync(c->wh_marks, 0, sizeof(uint32_t) * 2 * kWavesPerWG * c->cap_blocks, st));
        RT_HIP(hipMemsetAsync(c->plans, 0, sizeof(HfPlan) * 2, st));
        RT_HIP(hipMemsetAsync(c->ticket, 0, sizeof(uint32_t), st));
        *(volatile uint32_t *)c->wh_cnt = 0u;
        c->nblocks = uint32_t(blocks);
        // front: an eighth of the blocks, capped, a multiple of the XCD count so the natural
        // section keeps its block -> XCD assignment
        c->front = front ? std::min<uint32_t>(kHfFrontMax, uint32_t(blocks / 8u) & ~(kXcds - 1u)) : 0u;
        std::memcpy(c->key, key, sizeof(key));          // valid only now
    }
    c->used = ++s->hf_clock;
    const uint32_t v = c->ver;
    P.hf_front = c->front;
    P.hf_ver = v;
    // measured: the first two frames (the first plan has no earlier maximum to test a tail
    // against, so it lists nothing) and then every kHfPeriod-th
    // ... and every frame whose camera differs from the previous frame's: a moving camera's heavy
    // blocks move with the view, so the plan comes from the newest view (one frame old) instead of
    // one up to kHfPeriod frames old
    P.hf_measure = c->frames < 2u || c->frames % kHfPeriod == 0u || (s->hf_follow && cam_sig != c->cam);
    c->cam = cam_sig;
    c->frames++;
    P.hf_floor = s->hf_floor;
    P.hf_ticket = c->ticket;
    P.hf_mark_in = c->marks + size_t(v & 1u) * c->cap_blocks;
    P.hf_mark_out = c->marks + size_t((v + 1u) & 1u) * c->cap_blocks;
    P.hf_list_in = c->lists + size_t(v & 1u) * kHfFrontMax;
    P.hf_list_out = c->lists + size_t((v + 1u) & 1u) * kHfFrontMax;
    P.hf_plan_in = c->plans + (v & 1u);
    P.hf_plan_out = c->plans + ((v + 1u) & 1u);
    P.hf_cost = c->cost;
    if (var & kVarWideHeavy)
    {
        // spp <= 4: 16 lanes per sample; spp 8-16: a pixel's samples fill a wave at 4 lanes each.
        // The section holds wh_g waves per listed item of the newest plan the host has seen (a
        // plan or two old: the count is read without waiting); at least one workgroup, since
        // the device-side list may already be longer (the section is persistent over it).
        // Refresh: every kWhRefresh-th frame renders every item one lane per sample, so the next
        // plan re-ranks all items on lane-mode costs (the wide set is otherwise sticky).
        P.wh_g = P.spp <= 4u ? 16u : 4u;
        const uint32_t units = *(volatile uint32_t *)c->wh_cnt;         // waves: k_hf_plan counts them
        P.wh_on = 1u;
        P.wh_refresh = (c->frames - 1u) % kWhRefresh == 0u;       // frames counts this one
        P.wh_wgs = P.wh_refresh ? 0u : (units + kWavesPerWG - 1u) / kWavesPerWG;
        P.wh_floor = s->wh_floor;
        // a rank of 2 of a batched step lists more (its span estimate includes the other frames'
        // work); one scene's own rank-of-2 launch measured 25 % slower with it
        // (profiles/r03o_shard_scaling_bench.json), so it keeps the default
        // and a rank of 4-7 of a batched step one notch lower than the default (rank of 4, measured
        // in profiles/r03ad_alpha_n4_n8.json: 0.182 ms at 28/16 vs 0.191 at 32/16, 0.219 at 36/16;
        // a rank of 8 keeps 32/16: 0.117 vs 0.119 at 28/16)
        P.wh_alpha16 = (P.nranks == 2u && batch != 0u)                  ? s->wh_alpha16_n2
                       : (P.nranks >= 3u && P.nranks < 8u && batch != 0u) ? s->wh_alpha16_n4
                                                                          : s->wh_alpha16;
        // the second tier (4 lanes per sample, spp <= 4)
        P.wh_beta16 = P.wh_g != 16u ? 0u
                      : (P.nranks == 2u && batch != 0u)                  ? s->wh_beta16_n2
                      : (P.nranks >= 3u && P.nranks < 8u && batch != 0u) ? s->wh_beta16_n4
                                                                         : s->wh_beta16;
        if (P.wh_beta16 >= P.wh_alpha16) P.wh_beta16 = 0u;
        P.wh_mark_in = c->wh_marks + size_t(v & 1u) * kWavesPerWG * c->cap_blocks;
        P.wh_mark_out = c->wh_marks + size_t((v + 1u) & 1u) * kWavesPerWG * c->cap_blocks;
        P.wh_list_in = c->wh_lists + size_t(v & 1u) * 2u * kWhMax;
        P.wh_list_out = c->wh_lists + size_t((v + 1u) & 1u) * 2u * kWhMax;
        void *dev = nullptr;
        RT_HIP(hipHostGetDevicePointer(&dev, c->wh_cnt, 0));
        P.wh_host_cnt = static_cast<uint32_t *>(dev);
    }
    if (P.hf_measure) c->ver = v + 1u;                  // the plan launched after this frame
    return RT_OK;
}

typedef void (*kfn_t)(KParams);

// k_render_lanes instantiation of a variant (nullptr: not built)
kfn_t lanes_kernel(int tri, int var)
{
    if (tri == RT_TRI_BARYCENTRIC) return var == 0 ? k_render_lanes<RT_TRI_BARYCENTRIC, 0> : nullptr;
    switch (var)
    {
    case 0: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, 0>;
    case kVarMarch: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarMarch>;
    case kVarMarch | kVarExhaustive: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarMarch | kVarExhaustive>;
    case kVarBrute: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarBrute>;
    case kVarAuto: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAuto>;
    case kVarAutoCore | kVarPackedRem | kVarSkipRun:
        return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAutoCore | kVarPackedRem | kVarSkipRun>;
    case kVarAutoCore | kVarFastRcp: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAutoCore | kVarFastRcp>;
    case kVarAutoCore: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAutoCore>;
    case kVarAuto | kVarWideHeavy: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAuto | kVarWideHeavy>;
    case kVarAuto | kVarWaveClock: return k_render_lanes<RT_TRI_MOLLER_TRUMBORE, kVarAuto | kVarWaveClock>;
    default: return nullptr;
    }
}

// Launches the render kernel over region/shard described by P (tiles_x, rank, ...).
int launch_render(rt_scene *s, const rt_frame *f, KParams& P, uint32_t n_local_tiles, hipStream_t st,
                  bool order_streams = true)
{
    if (n_local_tiles == 0) return RT_OK;
    const bool lanes = use_lanes(f, P.spp);
    P.wg_per_tile = lanes ? (kTilePix * P.spp) / kWG : 1;
    if (P.wg_per_tile == 0) P.wg_per_tile = 1;
    const uint64_t blocks = uint64_t(n_local_tiles) * P.wg_per_tile;
    if (blocks > 0x3FFFFFFFull) return fail(RT_E_INVALID, "frame too large for one launch");
    const uint32_t kind = f->kernel & RT_KERNEL_KIND_MASK;
    const bool bary = P.tri_test == RT_TRI_BARYCENTRIC;
    const bool grid_mt = P.isect == RT_ISECT_GRID && !bary;
    // The per-camera records (frefs) are scene state: a launch on another stream than the last
    // one waits for it, so frames of one scene never overlap on the device.
    // (order_streams false: the caller orders its streams itself, rt_render_frame_host_tiled)
    if (order_streams && s->ev_recorded && st != s->last_stream) RT_HIP(hipStreamWaitEvent(st, s->ev1, 0));
    s->last_stream = st;
    // kVarXcdBands turn size: one row of this launch's tiles (ceil(tiles_x / nranks) local tiles
    // span a full frame row in shard mode).  Measured best of 1/4 .. 4 rows and 1..16 tiles:
    // whole rows interleave over the XCDs, so each L2 sees compact rows AND the frame's cost
    // spreads evenly (half rows put every left half on the even XCDs).
    P.xcd_chunk = ((P.tiles_x + P.nranks - 1u) / P.nranks) * P.wg_per_tile;
    // AUTO (and the COMPACT arm built on its per-ray code): the feature set of kVarAuto that this
    // scene allows -- the Newton reciprocal needs rcp_safe, the packed counts and the empty-run
    // loop need pack_ok.  DESIGN.md §4.1 has the measured progression.
    const bool auto_path = lanes && grid_mt && (kind == RT_KERNEL_AUTO || kind == RT_KERNEL_COMPACT);
    int var = 0;
    if (auto_path)
    {
        var = kVarAutoCore | (s->rcp_safe ? kVarFastRcp : 0) | (auto_runs(s) ? kVarPackedRem | kVarSkipRun : 0) |
              ((f->kernel & RT_KERNEL_FLAG_WAVE_CLOCK) ? kVarWaveClock : 0);
        if (int rc = ensure_origin_terms(s, P, st)) return rc;
    }
    else if (lanes && P.isect == RT_ISECT_RAY_MARCH)
        var = kVarMarch | ((f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE) ? kVarExhaustive : 0);
    else if (lanes && P.isect == RT_ISECT_BRUTE_FORCE)
        var = kVarBrute;
    // kernel-time events only outside stream capture (a captured record has no time to read)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    // A timed event pair costs ~10 us of device time per launch (measured: bench step 0.755 ->
    // 0.736 ms without), so only every time_every-th launch is timed (rt_scene_set_timing)
    const bool timed = cap == hipStreamCaptureStatusNone && s->time_every && s->launches % s->time_every == 0u;
    s->launches++;
    const uint32_t kslot = s->kt_next;
    hipEvent_t kt0 = nullptr, kt1 = nullptr;        // null stand for "not timed"
    if (timed && !s->kt0[kslot])
    {
        RT_HIP(hipEventCreate(&s->kt0[kslot]));
        RT_HIP(hipEventCreate(&s->kt1[kslot]));
    }
    if (timed)
    {
        kt0 = s->kt0[kslot];
        kt1 = s->kt1[kslot];
    }
    auto mark = [&](hipEvent_t e) { return e ? hipEventRecord(e, st) : hipSuccess; };
    if (var & kVarWaveClock)
    {
        const size_t need = size_t(blocks) * kWavesPerWG * 4u;
        if (need > s->clk_cap)
        {
            if (s->d_clk) RT_HIP(hipFree(s->d_clk));
            s->d_clk = nullptr;
            RT_HIP(hipMalloc(&s->d_clk, need * sizeof(uint64_t)));
            s->clk_cap = need;
        }
        s->clk_items = uint32_t(need / 4u);
        P.wave_clk = s->d_clk;
    }
    const dim3 wg(kWG);
    const uint32_t budget = (f->kernel & RT_KERNEL_BUDGET_MASK) >> RT_KERNEL_BUDGET_SHIFT;
    // AUTO takes the wide section (kVarWideHeavy: AUTO's full record/count layout, spp <= 16) for
    // a shard of >= 2 ranks of a scene with dense cells: there a rank's launch is bound by its few
    // ~1000-test waves, which the section splits 16 ways (4 for spp 8-16) beside the lane kernel
    // (measured, tools/wh_probe.py, killeroo rank of 2 / 4 / 8: 0.36 / 0.33 / 0.25 ms with the
    // two-phase arm it replaced -> 0.35 / 0.20 / 0.15).  On a whole frame the
    // lanes are busy with other items anyway and the section's repeated walks cost more than they
    // save (+1-3 %).
    const bool wide_ok = auto_path && var == kVarAuto && P.spp <= 16u;
    const bool wide_heavy = wide_ok && kind == RT_KERNEL_AUTO &&
                            ((f->kernel & RT_KERNEL_FLAG_WIDE_HEAVY) ||
                             (P.nranks >= 2u && s->max_cell_refs >= s->wh_auto_refs));
    if (lanes && kind == RT_KERNEL_COMPACT && P.isect == RT_ISECT_GRID)
    {
        const uint32_t n_items = uint32_t(blocks * kWavesPerWG);
        const uint32_t refill = budget ? budget : kCompactRefill;
        const dim3 grid(std::max(1u, std::min(s->compact_wgs, (n_items + 3u) / 4u)));
        RT_HIP(mark(kt0));
        if (bary)
            hipLaunchKernelGGL((k_render_compact<RT_TRI_BARYCENTRIC, kVarDistSkip>), grid, wg, 0, st, P, n_items,
                               refill);
        else if (auto_runs(s) && s->rcp_safe)
            // AUTO's walk and record test: box runs, packed counts, the Newton 1/det (the wave-uniform
            // scalar list loop left out: its SGPRs made the persistent kernel spill to scratch)
            hipLaunchKernelGGL((k_render_compact<RT_TRI_MOLLER_TRUMBORE, kVarCompactBox>), grid, wg, 0, st, P,
                               n_items, refill);
        else
            hipLaunchKernelGGL((k_render_compact<RT_TRI_MOLLER_TRUMBORE, kVarWaveGate | kVarDistSkip | kVarOriginPre>),
                               grid, wg, 0, st, P, n_items, refill);
        RT_HIP(mark(kt1));
    }
    else if (lanes)
    {
        // AUTO, LANES, and COMPACT where its layout does not apply
        const int kvar = ((kind == RT_KERNEL_AUTO || P.isect != RT_ISECT_GRID) ? var : 0) |
                         (wide_heavy ? kVarWideHeavy : 0);
        const kfn_t fn = lanes_kernel(bary ? RT_TRI_BARYCENTRIC : RT_TRI_MOLLER_TRUMBORE, kvar);
        if (!fn) return fail(RT_E_INVALID, "kernel variant not built: " + std::to_string(kvar));
        uint32_t grid = uint32_t(blocks);
        // heavy-first order: AUTO grid frames large enough that blocks start in several rounds
        // (and every wide-section launch of >= 64 blocks: its lane kernel's heaviest items)
        const bool front = kind == RT_KERNEL_AUTO && P.isect == RT_ISECT_GRID && !(kvar & kVarWaveClock) &&
                           (blocks >= s->hf_min_blocks || (wide_heavy && blocks >= 64u));
        if (front || wide_heavy)
        {
            if (int rc = hf_prepare(s, P, blocks, kvar, front, st)) return rc;
            grid += P.hf_front;
        }
        // one-wave workgroups (k_render_lanes_w64): the same blocks, each wave dispatched by itself
        kfn_t lfn = fn;
        uint32_t lgrid = grid, lwg = kWG;
        if (s->wg64 && kvar == kVarAuto && grid >= s->wg64_min_blocks)
        {
            lfn = k_render_lanes_w64<RT_TRI_MOLLER_TRUMBORE, kVarAuto>;
            P.vblocks = grid;
            lgrid = kWavesPerWG * ((grid + kXcds - 1u) / kXcds * kXcds);
            lwg = 64u;
        }
        RT_HIP(mark(kt0));
        if (P.wh_wgs)
        {
            // the wide section runs on the side stream beside the lane kernel (fork / join by
            // events, so the pair also captures into a hipGraph); submitted first so its waves
            // -- the frame's longest -- start first
            if (!s->side)
            {
                RT_HIP(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
                RT_HIP(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
                RT_HIP(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
            }
            RT_HIP(hipEventRecord(s->ev_fork, st));
            RT_HIP(hipStreamWaitEvent(s->side, s->ev_fork, 0));
            if (P.wh_g == 4u) hipLaunchKernelGGL(k_render_wh<4>, dim3(P.wh_wgs), wg, 0, s->side, P);
            else hipLaunchKernelGGL(k_render_wh<16>, dim3(P.wh_wgs), wg, 0, s->side, P);
        }
        hipLaunchKernelGGL(lfn, dim3(lgrid), dim3(lwg), 0, st, P);
        if (P.wh_wgs)
        {
            RT_HIP(hipEventRecord(s->ev_join, s->side));
            RT_HIP(hipStreamWaitEvent(st, s->ev_join, 0));
        }
        RT_HIP(mark(kt1));
        if ((P.hf_front || P.wh_on) && P.hf_measure)
        {
            hipLaunchKernelGGL(k_hf_plan, dim3(uint32_t((blocks + kWG * kHfPlanPer - 1) / (kWG * kHfPlanPer))), wg, 0, st, P,
                               uint32_t(blocks));
        }
    }
    else
    {
        RT_HIP(mark(kt0));
        if (P.isect == RT_ISECT_RAY_MARCH && (f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE))
            hipLaunchKernelGGL((k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarMarch | kVarExhaustive>),
                               dim3(uint32_t(blocks)), wg, 0, st, P);
        else if (P.isect == RT_ISECT_RAY_MARCH)
            hipLaunchKernelGGL((k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarMarch>), dim3(uint32_t(blocks)), wg, 0, st, P);
        else if (P.isect == RT_ISECT_BRUTE_FORCE)
            hipLaunchKernelGGL((k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarBrute>), dim3(uint32_t(blocks)), wg, 0, st, P);
        else if (bary)
            hipLaunchKernelGGL((k_render_pixel_loop<RT_TRI_BARYCENTRIC, 0>), dim3(uint32_t(blocks)), wg, 0, st, P);
        else
            hipLaunchKernelGGL((k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, 0>), dim3(uint32_t(blocks)), wg, 0, st, P);
        RT_HIP(mark(kt1));
    }
    RT_HIP(hipGetLastError());
    RT_HIP(hipEventRecord(s->ev1, st));
    s->ev_recorded = true;
    if (timed)
    {
        s->kt_last = kslot;
        s->kt_next = (kslot + 1u) % kTimeRing;
        s->kt_count = std::min(s->kt_count + 1u, kTimeRing);
    }
    return RT_OK;
}


// k_render_batch instantiation of a variant (nullptr: the frames take one launch each)
typedef void (*kbfn_t)(KBatch);
template <int VAR>
kbfn_t batch_kernel_of(bool w64)
{
    return w64 ? k_render_batch_w64<RT_TRI_MOLLER_TRUMBORE, VAR> : k_render_batch<RT_TRI_MOLLER_TRUMBORE, VAR>;
}
kbfn_t batch_kernel(int var, bool w64)
{
    if (var == kVarAuto) return batch_kernel_of<kVarAuto>(w64);
    if (var == (kVarAuto | kVarWideHeavy)) return batch_kernel_of<kVarAuto | kVarWideHeavy>(w64);
    if (var == (kVarAuto | kVarWideHeavy | kVarWideFused))
        return batch_kernel_of<kVarAuto | kVarWideHeavy | kVarWideFused>(w64);
    if (var == (kVarAuto | kVarWideHeavy | kVarWideFused | kVarWideG4))
        return batch_kernel_of<kVarAuto | kVarWideHeavy | kVarWideFused | kVarWideG4>(w64);
    // RT_KERNEL_FLAG_WAVE_CLOCK (debug timelines, tools/batch_waves.py): the bench pair's batched step
    // at one rank and with the fused wide section
    if (var == (kVarAuto | kVarWaveClock)) return batch_kernel_of<kVarAuto | kVarWaveClock>(w64);
    if (var == (kVarAuto | kVarWideHeavy | kVarWideFused | kVarWaveClock))
        return batch_kernel_of<kVarAuto | kVarWideHeavy | kVarWideFused | kVarWaveClock>(w64);
    return nullptr;
}

static_assert(sizeof(KBatch) <= 4096, "kernel arguments are limited to 4 KiB");

// n frames (2 <= n <= kMaxBatch, scenes on one device, mutexes held by the caller) in ONE launch
// of k_render_batch.  P[i] holds frame i's parameters (frame_params + region + shard + outputs).
// Returns RT_E_INVALID with *batched == false, doing nothing, when the frames cannot share a
// launch (the caller then renders them one launch each).
int launch_batch(rt_scene *const *S, const rt_frame *F, uint32_t n, KParams *P, uint32_t n_local_tiles,
                 hipStream_t st, bool *batched)
{
    *batched = false;
    if (n < 2 || n > kMaxBatch || n_local_tiles == 0) return RT_E_INVALID;
    const uint32_t spp = P[0].spp;
    if (!use_lanes(&F[0], spp) || spp > 16u) return RT_E_INVALID;
    int var = -1;
    bool wide_heavy = false;
    for (uint32_t i = 0; i < n; i++)
    {
        const uint32_t kind = F[i].kernel & RT_KERNEL_KIND_MASK;
        if (kind != RT_KERNEL_AUTO ||
            (F[i].kernel & ~uint32_t(RT_KERNEL_FLAG_WIDE_HEAVY | RT_KERNEL_FLAG_WAVE_CLOCK)) != 0u ||
            (F[i].kernel & RT_KERNEL_FLAG_WAVE_CLOCK) != (F[0].kernel & RT_KERNEL_FLAG_WAVE_CLOCK))
            return RT_E_INVALID;
        if (P[i].isect != RT_ISECT_GRID || P[i].tri_test != RT_TRI_MOLLER_TRUMBORE) return RT_E_INVALID;
        if (P[i].W != P[0].W || P[i].H != P[0].H || P[i].spp != spp || S[i]->device != S[0]->device)
            return RT_E_INVALID;
        const int v = kVarAutoCore | (S[i]->rcp_safe ? kVarFastRcp : 0) |
                      (auto_runs(S[i]) ? kVarPackedRem | kVarSkipRun : 0);
        if (var >= 0 && v != var) return RT_E_INVALID;
        var = v;
        wide_heavy = wide_heavy || (F[i].kernel & RT_KERNEL_FLAG_WIDE_HEAVY) ||
                     (P[i].nranks >= 2u && S[i]->max_cell_refs >= S[0]->wh_auto_refs);
    }
    if (var != kVarAuto) return RT_E_INVALID;
    // fused (measured, profiles/r03f_ab_wide_fused.json): 18 % faster at a rank of 8, 9 % at 4,
    // 4 % slower at 2 on the build of that A/B; re-measured on the current one, a rank of 2 takes
    // 0.321 ms fused vs 0.338 (profiles/r03aa_wg64_wide_fused2_sweep.json): fused from 2 ranks
    const bool fused = wide_heavy && S[0]->wh_fused && P[0].nranks >= S[0]->wh_fused_min_ranks;
    const bool clk = (F[0].kernel & RT_KERNEL_FLAG_WAVE_CLOCK) != 0u;
    const int kvar = var | (wide_heavy ? kVarWideHeavy : 0) | (fused ? kVarWideFused : 0) |
                     (fused && spp > 4u ? kVarWideG4 : 0) | (clk ? kVarWaveClock : 0);
    if (!batch_kernel(kvar, false)) return RT_E_INVALID;
    *batched = true;
    KBatch KB;
    std::memset(&KB, 0, sizeof(KB));
    const uint32_t wgpt = (kTilePix * spp) / kWG;
    const uint64_t fblocks = uint64_t(n_local_tiles) * wgpt;
    const uint64_t blocks = fblocks * n;
    if (blocks > 0x3FFFFFFFull) return fail(RT_E_INVALID, "batch too large for one launch");
    KB.nframes = n;
    for (uint32_t i = 0; i <= n; i++) KB.base[i] = uint32_t(fblocks * i);
    for (uint32_t i = n + 1; i <= kMaxBatch; i++) KB.base[i] = uint32_t(blocks);
    // per-origin records of every scene, and the cross-stream order of every scene's state
    for (uint32_t i = 0; i < n; i++)
    {
        P[i].wg_per_tile = wgpt;
        P[i].xcd_chunk = ((P[i].tiles_x + P[i].nranks - 1u) / P[i].nranks) * wgpt;
        rt_scene *s = S[i];
        bool first = true;
        for (uint32_t j = 0; j < i; j++) first = first && S[j] != s;
        if (!first) continue;
        if (s->ev_recorded && st != s->last_stream) RT_HIP(hipStreamWaitEvent(st, s->ev1, 0));
        s->last_stream = st;
        if (int rc = ensure_origin_terms(s, P[i], st)) return rc;
    }
    // the batch's heavy-first / wide-section state lives in scene 0's table, keyed by the batch
    uint64_t ident = n;
    for (uint32_t i = 0; i < n; i++) ident = ident * 0x9E3779B97F4A7C15ull + uint64_t(uintptr_t(S[i]));
    rt_scene *s0 = S[0];
    const bool front = blocks >= s0->hf_min_blocks || (wide_heavy && blocks >= 64u);
    uint64_t cams = 0xcbf29ce484222325ull;
    for (uint32_t i = 0; i < n; i++) cams = cam_signature(P[i], cams);
    if (front || wide_heavy)
        if (int rc = hf_prepare(s0, P[0], blocks, kvar, front, st, ident | 1u, cams)) return rc;
    // fused: the wide section's workgroups lead the grid, a multiple of the XCD count so the lane
    // blocks keep their block -> XCD assignment
    if (fused && P[0].wh_wgs) P[0].wh_wgs = (P[0].wh_wgs + kXcds - 1u) & ~(kXcds - 1u);
    uint32_t grid = uint32_t(blocks) + P[0].hf_front + (fused ? P[0].wh_wgs : 0u);
    // one-wave workgroups (k_render_batch_w64, as k_render_lanes_w64): the same blocks and order.
    // Without a wide section (N = 1) the bench pair took 0.569 vs 0.598 ms with 256-lane
    // workgroups (profiles/r03y_wg64_batch_sweep.json).  Beside one, per rank count (wg64_wide, bit
    // log2 N, 3 for N >= 8): with the section fused from 2 ranks and one-wave workgroups on both
    // (profiles/r03aa_wg64_wide_*.json) a rank of 2 took 0.306 ms (0.321 with 256-lane ones, 0.338
    // unfused), of 8 0.117 (0.121); a rank of 4 0.206 vs 0.193, so 4 keeps 256-lane workgroups
    const uint32_t lg_ranks = P[0].nranks >= 8u ? 3u : (P[0].nranks >= 4u ? 2u : (P[0].nranks >= 2u ? 1u : 0u));
    const bool w64 = s0->wg64 != 0u && (!wide_heavy || ((s0->wg64_wide >> lg_ranks) & 1u) != 0u) &&
                     uint32_t(blocks) + P[0].hf_front >= s0->wg64_batch_min_blocks;
    uint32_t bwg = kWG;
    if (w64)
    {
        P[0].vblocks = uint32_t(blocks) + P[0].hf_front;
        grid = kWavesPerWG * ((fused ? P[0].wh_wgs : 0u) + (P[0].vblocks + kXcds - 1u) / kXcds * kXcds);
        bwg = 64u;
    }
    const kbfn_t fn = batch_kernel(kvar, w64);
    if (clk)
    {
        // one record per lane item and per (listed item, wave) of the wide section
        const size_t need = (size_t(blocks) * kWavesPerWG + size_t(kWhMax) * 20u) * 4u;
        if (need > s0->clk_cap)
        {
            if (s0->d_clk) RT_HIP(hipFree(s0->d_clk));
            s0->d_clk = nullptr;
            RT_HIP(hipMalloc(&s0->d_clk, need * sizeof(uint64_t)));
            s0->clk_cap = need;
        }
        RT_HIP(hipMemsetAsync(s0->d_clk, 0, need * sizeof(uint64_t), st));
        s0->clk_items = uint32_t(need / 4u);
        P[0].wave_clk = s0->d_clk;
    }
    for (uint32_t i = 0; i < n; i++) KB.p[i] = P[i];
    // timing: scene 0's ring (one timed launch for the whole batch)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    const bool timed = cap == hipStreamCaptureStatusNone && s0->time_every && s0->launches % s0->time_every == 0u;
    s0->launches++;
    const uint32_t kslot = s0->kt_next;
    if (timed && !s0->kt0[kslot])
    {
        RT_HIP(hipEventCreate(&s0->kt0[kslot]));
        RT_HIP(hipEventCreate(&s0->kt1[kslot]));
    }
    if (timed) RT_HIP(hipEventRecord(s0->kt0[kslot], st));
    const dim3 wg(kWG);
    if (P[0].wh_wgs && !fused)
    {
        if (!s0->side)
        {
            RT_HIP(hipStreamCreateWithFlags(&s0->side, hipStreamNonBlocking));
            RT_HIP(hipEventCreateWithFlags(&s0->ev_fork, hipEventDisableTiming));
            RT_HIP(hipEventCreateWithFlags(&s0->ev_join, hipEventDisableTiming));
        }
        RT_HIP(hipEventRecord(s0->ev_fork, st));
        RT_HIP(hipStreamWaitEvent(s0->side, s0->ev_fork, 0));
        if (w64 && P[0].wh_g == 4u)
            hipLaunchKernelGGL(k_render_wh_batch_w64<4>, dim3(kWavesPerWG * P[0].wh_wgs), dim3(64), 0, s0->side, KB);
        else if (w64)
            hipLaunchKernelGGL(k_render_wh_batch_w64<16>, dim3(kWavesPerWG * P[0].wh_wgs), dim3(64), 0, s0->side, KB);
        else if (P[0].wh_g == 4u) hipLaunchKernelGGL(k_render_wh_batch<4>, dim3(P[0].wh_wgs), wg, 0, s0->side, KB);
        else hipLaunchKernelGGL(k_render_wh_batch<16>, dim3(P[0].wh_wgs), wg, 0, s0->side, KB);
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(bwg), 0, st, KB);
    if (P[0].wh_wgs && !fused)
    {
        RT_HIP(hipEventRecord(s0->ev_join, s0->side));
        RT_HIP(hipStreamWaitEvent(st, s0->ev_join, 0));
    }
    if (timed) RT_HIP(hipEventRecord(s0->kt1[kslot], st));
    if ((P[0].hf_front || P[0].wh_on) && P[0].hf_measure)
        hipLaunchKernelGGL(k_hf_plan, dim3(uint32_t((blocks + kWG * kHfPlanPer - 1) / (kWG * kHfPlanPer))), wg, 0, st,
                           KB.p[0], uint32_t(blocks));
    RT_HIP(hipGetLastError());
    for (uint32_t i = 0; i < n; i++)
    {
        RT_HIP(hipEventRecord(S[i]->ev1, st));
        S[i]->ev_recorded = true;
    }
    if (timed)
    {
        s0->kt_last = kslot;
        s0->kt_next = (kslot + 1u) % kTimeRing;
        s0->kt_count = std::min(s0->kt_count + 1u, kTimeRing);
    }
    return RT_OK;
}

} // namespace

namespace {
// Device staging frame (and, for rt_render_tiles, the scene's pinned host frame) of >= words.
int ensure_frame(rt_scene *s, size_t words, bool host)
{
    if (words > s->frame_cap)
    {
        if (s->d_frame) RT_HIP(hipFree(s->d_frame));
        s->d_frame = nullptr;
        RT_HIP(hipMalloc(&s->d_frame, words * 4));
        s->frame_cap = words;
    }
    if (host && words > s->hframe_cap)
    {
        if (s->h_frame) RT_HIP(hipHostFree(s->h_frame));
        s->h_frame = nullptr;
        RT_HIP(hipHostMalloc(&s->h_frame, words * 4));
        s->hframe_cap = words;
    }
    return RT_OK;
}
} // namespace

int rt_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

int rt_internal_use_device(int device, int *num_cus)
{
    int ndev = 0;
    RT_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(RT_E_NODEVICE, "device index out of range / no GPU");
    hipDeviceProp_t prop;
    RT_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RT_E_NODEVICE, std::string("librt_tracer is built for gfx950, device is ") + prop.gcnArchName);
    RT_HIP(hipSetDevice(device));
    if (num_cus) *num_cus = prop.multiProcessorCount;
    return RT_OK;
}

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_last_error(char *buf, size_t len)
{
    if (!buf || len == 0) return RT_E_INVALID;
    std::snprintf(buf, len, "%s", g_err.c_str());
    return RT_OK;
}

int rt_get_device_count(int *count)
{
    if (!count) return fail(RT_E_INVALID, "count is NULL");
    *count = 0;
    RT_HIP(hipGetDeviceCount(count));
    return RT_OK;
}

#ifndef RT_SRC_HASH
#define RT_SRC_HASH "unknown"
#endif

int rt_build_hash(char *buf, size_t len)
{
    if (!buf || len == 0) return fail(RT_E_INVALID, "bad arguments");
    std::snprintf(buf, len, "%s", RT_SRC_HASH);
    return RT_OK;
}

int rt_scene_info_get(rt_scene *s, rt_scene_info *out)
{
    if (!s || !out) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    std::memset(out, 0, sizeof(*out));
    out->octant_words = s->octant_words;
    out->box_words = s->box_words;
    out->packed_cells = s->d_cellw != nullptr;
    out->rcp_safe = s->rcp_safe;
    out->pack_ok = s->pack_ok;
    out->max_cell_refs = s->max_cell_refs;
    out->hf_floor = s->hf_floor;
    out->hf_min_blocks = s->hf_min_blocks;
    out->wh_floor = s->wh_floor;
    out->wh_alpha16 = s->wh_alpha16;
    out->wh_alpha16_n2 = s->wh_alpha16_n2;
    out->wh_auto_refs = s->wh_auto_refs;
    out->wh_fused = s->wh_fused;
    out->hf_contexts = kHfCtxs;
    out->hf_evictions = s->hf_evictions;
    out->batch_launches = s->batch_launches;
    out->batch_fallbacks = s->batch_fallbacks;
    out->device_bytes = s->device_bytes;
    return RT_OK;
}

int rt_sample_table(uint32_t spp, float *out_xy)
{
    if (!out_xy || spp == 0) return fail(RT_E_INVALID, "bad arguments");
    std::vector<float> t;
    hammersley(spp, t);
    std::memcpy(out_xy, t.data(), t.size() * sizeof(float));
    return RT_OK;
}

// Cap on the 8 octant copies of the cell words (device and host): 64 M cells at most.
constexpr uint64_t kOctWordsMaxBytes = 256ull << 20;
// ... and on the 24 box-run copies
constexpr uint64_t kBoxWordsMaxBytes = 384ull << 20;

int rt_scene_create(const rt_scene_desc *d, int device, rt_scene **out)
{
    if (!d || !out) return fail(RT_E_INVALID, "desc/out is NULL");
    *out = nullptr;
    const rt_grid_desc& g = d->grid;
    if (d->num_triangles == 0 || d->num_vertices == 0 || !d->vertices || !d->triangles)
        return fail(RT_E_INVALID, "empty mesh");
    if (!g.cell_offsets || g.dims[0] == 0 || g.dims[1] == 0 || g.dims[2] == 0)
        return fail(RT_E_INVALID, "empty grid");
    const uint64_t nc64 = uint64_t(g.dims[0]) * g.dims[1] * g.dims[2];
    if (nc64 >= 0x7FFFFFFFull) return fail(RT_E_INVALID, "grid too large");
    const uint32_t nc = uint32_t(nc64);
    if (g.cell_offsets[0] != 0) return fail(RT_E_INVALID, "cell_offsets[0] != 0");
    for (uint32_t c = 0; c < nc; c++)
        if (g.cell_offsets[c + 1] < g.cell_offsets[c]) return fail(RT_E_INVALID, "cell_offsets not monotonic");
    const uint32_t nr = g.cell_offsets[nc];
    if (nr && !g.cell_tris) return fail(RT_E_INVALID, "cell_tris is NULL");
    for (uint32_t k = 0; k < nr; k++)
        if (g.cell_tris[k] >= d->num_triangles) return fail(RT_E_INVALID, "cell_tris index out of range");
    for (uint32_t i = 0; i < d->num_triangles; i++)
    {
        const rt_triangle& t = d->triangles[i];
        if (t.v0 >= d->num_vertices || t.v1 >= d->num_vertices || t.v2 >= d->num_vertices)
            return fail(RT_E_INVALID, "triangle vertex index out of range");
    }
    int ncus = 0;
    if (int rc = rt_internal_use_device(device, &ncus)) return rc;

    std::unique_ptr<rt_scene> s(new rt_scene());
    s->device = device;
    s->compact_wgs = 8u * uint32_t(std::max(1, ncus));
    // scheduling tunables: read once here, never per launch (A/B sweeps set them per scene)
    s->hf_floor = env_tunable("RT_HF_FLOOR", s->hf_floor);
    s->hf_min_blocks = env_tunable("RT_HF_MIN_BLOCKS", s->hf_min_blocks);
    s->wg64 = env_tunable("RT_WG64", s->wg64);
    s->wg64_min_blocks = env_tunable("RT_WG64_MIN_BLOCKS", s->wg64_min_blocks);
    s->wg64_batch_min_blocks = env_tunable("RT_WG64_BATCH_MIN_BLOCKS", s->wg64_batch_min_blocks);
    s->wh_floor = env_tunable("RT_WH_FLOOR", s->wh_floor);
    s->wh_alpha16 = env_tunable("RT_WH_ALPHA16", s->wh_alpha16);
    s->wh_alpha16_n2 = env_tunable("RT_WH_ALPHA16_N2", s->wh_alpha16_n2);
    s->wh_alpha16_n4 = env_tunable("RT_WH_ALPHA16_N4", s->wh_alpha16_n4);
    s->wh_beta16 = env_tunable("RT_WH_BETA16", s->wh_beta16);
    s->wh_beta16_n2 = env_tunable("RT_WH_BETA16_N2", s->wh_beta16 ? s->wh_beta16 : s->wh_beta16_n2);
    s->wh_beta16_n4 = env_tunable("RT_WH_BETA16_N4", s->wh_beta16 ? s->wh_beta16 : s->wh_beta16_n4);
    s->wh_auto_refs = env_tunable("RT_WH_AUTO_REFS", s->wh_auto_refs);
    s->wh_fused = env_tunable("RT_WH_FUSED", s->wh_fused);
    s->wg64_wide = env_tunable("RT_WG64_WIDE", s->wg64_wide);
    s->wh_fused_min_ranks = env_tunable("RT_WH_FUSED_MIN_RANKS", s->wh_fused_min_ranks);
    s->hf_follow = env_tunable("RT_HF_FOLLOW", s->hf_follow);
    for (int a = 0; a < 3; a++)
    {
        s->dims[a] = g.dims[a];
        s->bmin[a] = g.aabb_min[a];
        s->bmax[a] = g.aabb_max[a];
    }
    s->cw = g.cell_wdh;
    s->icw = g.inv_cell_wdh;
    s->ncells = nc;
    s->nrefs = nr;
    s->ntris = d->num_triangles;

    // Per-reference triangle records in CSR order (see file header)
    std::vector<float4> refs(size_t(std::max(nr, 1u)) * 3);
    double det_bound = 0.0;
    for (uint32_t k = 0; k < nr; k++)
    {
        const uint32_t ti = g.cell_tris[k];
        const rt_triangle& t = d->triangles[ti];
        const float *p0 = d->vertices[t.v0].p, *p1 = d->vertices[t.v1].p, *p2 = d->vertices[t.v2].p;
        const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };  // triangle.h:41
        const float e2[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };  // triangle.h:42
        float idf;
        std::memcpy(&idf, &ti, 4);
        refs[3 * size_t(k) + 0] = make_float4(p0[0], p0[1], p0[2], e1[0]);
        refs[3 * size_t(k) + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
        refs[3 * size_t(k) + 2] = make_float4(e2[2], idf, 0.0f, 0.0f);
        // |det| = |e1 . (d x e2)| <= |e1|_1 |e2|_1 for |d| ~ 1 (FAST_RCP range, rcp_nr)
        const double b = (std::fabs(double(e1[0])) + std::fabs(double(e1[1])) + std::fabs(double(e1[2]))) *
                         (std::fabs(double(e2[0])) + std::fabs(double(e2[1])) + std::fabs(double(e2[2])));
        det_bound = (b > det_bound || b != b) ? b : det_bound;
    }
    s->rcp_safe = det_bound == det_bound && det_bound < 0x1p120;
    s->pack_ok = g.dims[0] <= 512 && g.dims[1] <= 512 && g.dims[2] <= 512;
    std::vector<float4> shade(size_t(d->num_triangles) * 3), facen(d->num_triangles);
    std::vector<float4> trimt(size_t(d->num_triangles) * 3), tridist(size_t(d->num_triangles) * 6);
    for (uint32_t i = 0; i < d->num_triangles; i++)
    {
        const rt_triangle& t = d->triangles[i];
        const float *p0 = d->vertices[t.v0].p, *p1 = d->vertices[t.v1].p, *p2 = d->vertices[t.v2].p;
        {
            // brute force: {v0, e1 = v1 - v0, e2 = v2 - v0} (triangle.h:41-42) in triangle order
            const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };
            const float e2[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };
            trimt[3 * size_t(i) + 0] = make_float4(p0[0], p0[1], p0[2], e1[0]);
            trimt[3 * size_t(i) + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
            trimt[3 * size_t(i) + 2] = make_float4(e2[2], 0.0f, 0.0f, 0.0f);
        }
        const float *n0 = d->vertices[t.v0].n, *n1 = d->vertices[t.v1].n, *n2 = d->vertices[t.v2].n;
        shade[3 * size_t(i) + 0] = make_float4(n0[0], n0[1], n0[2], n1[0]);
        shade[3 * size_t(i) + 1] = make_float4(n1[1], n1[2], n2[0], n2[1]);
        shade[3 * size_t(i) + 2] = make_float4(n2[2], 0.0f, 0.0f, 0.0f);
        facen[i] = make_float4(t.n[0], t.n[1], t.n[2], 0.0f);
    }
    // Packed cell ranges: start < 2^21 and count < 2^11 for every cell -> one load per DDA step
    std::vector<uint32_t> cellw, cellwo, cellwb;
    bool packable = nr < (1u << 21);
    for (uint32_t c = 0; c < nc && packable; c++) packable = g.cell_offsets[c + 1] - g.cell_offsets[c] < 2048u;
    if (packable)
    {
        // Empty cells carry their Chebyshev (L-inf) distance to the nearest non-empty cell in
        // the start field: a DDA step moves to a face neighbour, so the next dist-1 cells of
        // any walk leaving this cell are empty and need no lookup.  BFS over 26-neighbours
        // from all non-empty cells gives exactly the L-inf distance.
        const uint32_t dxs = g.dims[0], dys = g.dims[1], dzs = g.dims[2];
        std::vector<uint32_t> dist(nc, 0xFFFFFFFFu), frontier, next;
        for (uint32_t c = 0; c < nc; c++)
            if (g.cell_offsets[c + 1] != g.cell_offsets[c]) { dist[c] = 0; frontier.push_back(c); }
        for (uint32_t d = 1; !frontier.empty(); d++)
        {
            next.clear();
            for (uint32_t c : frontier)
            {
                const uint32_t x = c % dxs, z = (c / dxs) % dzs, y = c / (dxs * dzs);   // grid.h:41-42
                for (int oy = -1; oy <= 1; oy++)
                    for (int oz = -1; oz <= 1; oz++)
                        for (int ox = -1; ox <= 1; ox++)
                        {
                            const int nx = int(x) + ox, ny = int(y) + oy, nz = int(z) + oz;
                            if (nx < 0 || ny < 0 || nz < 0 || nx >= int(dxs) || ny >= int(dys) || nz >= int(dzs))
                                continue;
                            const uint32_t n = uint32_t(nx) + uint32_t(nz) * dxs + uint32_t(ny) * dxs * dzs;
                            if (dist[n] == 0xFFFFFFFFu) { dist[n] = d; next.push_back(n); }
                        }
            }
            frontier.swap(next);
        }
        cellw.resize(nc);
        for (uint32_t c = 0; c < nc; c++)
        {
            const uint32_t cnt = g.cell_offsets[c + 1] - g.cell_offsets[c];
            cellw[c] = cnt ? ((g.cell_offsets[c] << 11) | cnt)
                           : (std::min<uint32_t>(dist[c] == 0xFFFFFFFFu ? 0x1FFFFFu : dist[c], 0x1FFFFFu) << 11);
        }
        // Per ray octant (sign of dx, dy, dz) a directional bound: D(c) = the side of the largest
        // empty cube with corner c that extends along the octant's signs (cells outside the grid
        // count as empty).  j steps of a walk in that octant move each coordinate by 0..j in the
        // octant's direction, so the next D-1 cells are empty -- the same contract as the L-inf
        // word, and D >= the L-inf distance.  D(c) = 1 + min of D over the 7 forward neighbours
        // (the 3-D largest-square recurrence).  RT_OCT_DIST=0 keeps the L-inf words (A/B arm),
        // and so does a grid whose 8 copies would pass kOctWordsMaxBytes (they measured ~2 %).
        if (env_tunable("RT_OCT_DIST", 1u) != 0u && uint64_t(nc) * 8u * 4u <= kOctWordsMaxBytes)
        {
            s->octant_words = true;
            constexpr uint32_t kInf = 0x1FFFFFu;
            cellwo.resize(size_t(8) * nc);
            std::vector<uint32_t> D(nc);
            for (uint32_t o = 0; o < 8; o++)
            {
                const int sx = (o & 1) ? -1 : 1, sy = (o & 2) ? -1 : 1, sz = (o & 4) ? -1 : 1;
                auto at = [&](int x, int y, int z) -> uint32_t {
                    if (x < 0 || y < 0 || z < 0 || x >= int(dxs) || y >= int(dys) || z >= int(dzs)) return kInf;
                    return D[uint32_t(x) + uint32_t(z) * dxs + uint32_t(y) * dxs * dzs];
                };
                for (int iy = 0; iy < int(dys); iy++)
                    for (int iz = 0; iz < int(dzs); iz++)
                        for (int ix = 0; ix < int(dxs); ix++)
                        {
                            // visit forward neighbours first: against the octant's direction
                            const int x = sx > 0 ? int(dxs) - 1 - ix : ix;
                            const int y = sy > 0 ? int(dys) - 1 - iy : iy;
                            const int z = sz > 0 ? int(dzs) - 1 - iz : iz;
                            const uint32_t c = uint32_t(x) + uint32_t(z) * dxs + uint32_t(y) * dxs * dzs;
                            if (g.cell_offsets[c + 1] != g.cell_offsets[c]) { D[c] = 0; continue; }
                            uint32_t m = kInf;
                            for (int n = 1; n < 8; n++)
                                m = std::min(m, at(x + ((n & 1) ? sx : 0), y + ((n & 2) ? sy : 0), z + ((n & 4) ? sz : 0)));
                            D[c] = std::min(kInf, m + 1);
                        }
                for (uint32_t c = 0; c < nc; c++)
                    cellwo[size_t(o) * nc + c] = (cellw[c] & 2047u) ? cellw[c] : (D[c] << 11);
            }
        }
        // AUTO's box-run words (build_box_words): the non-empty words keep start < 2^20
        if (RT_BOX_RUN && nr < (1u << 20) && uint64_t(nc) * 24u * 4u <= kBoxWordsMaxBytes)
        {
            s->box_words = rtbox::build_box_words(g.cell_offsets, g.dims, cellwb);
            if (!s->box_words) cellwb.clear();          // out of host memory: AUTO walks without them
        }
    }
    for (uint32_t c = 0; c < nc; c++)
        s->max_cell_refs = std::max(s->max_cell_refs, g.cell_offsets[c + 1] - g.cell_offsets[c]);

    const size_t nfrefs = size_t(std::max(nr, 1u)) * 4;
    RT_HIP(hipMalloc(&s->d_off, sizeof(uint32_t) * (nc + 1)));
    RT_HIP(hipMalloc(&s->d_refs, sizeof(float4) * refs.size()));
    RT_HIP(hipMalloc(&s->d_frefs, sizeof(float4) * nfrefs));
    RT_HIP(hipMalloc(&s->d_shade, sizeof(float4) * shade.size()));
    RT_HIP(hipMalloc(&s->d_facen, sizeof(float4) * facen.size()));
    RT_HIP(hipMemcpy(s->d_off, g.cell_offsets, sizeof(uint32_t) * (nc + 1), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_refs, refs.data(), sizeof(float4) * refs.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_shade, shade.data(), sizeof(float4) * shade.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_facen, facen.data(), sizeof(float4) * facen.size(), hipMemcpyHostToDevice));
    // Distance records in Morton order of the triangle centroids, blocks of kDistBlock with their
    // exact float AABB (the ray march's block cull, see ray_march)
    std::vector<float4> distblk;
    {
        const uint32_t nt = d->num_triangles;
        float mn[3] = { rtd::kFltMax, rtd::kFltMax, rtd::kFltMax }, mx[3] = { -rtd::kFltMax, -rtd::kFltMax, -rtd::kFltMax };
        float scale = 0.0f;
        for (uint32_t i = 0; i < d->num_vertices; i++)
            for (int a = 0; a < 3; a++)
            {
                mn[a] = std::min(mn[a], d->vertices[i].p[a]);
                mx[a] = std::max(mx[a], d->vertices[i].p[a]);
                scale = std::max(scale, std::fabs(d->vertices[i].p[a]));
            }
        std::vector<std::pair<uint64_t, uint32_t>> order(nt);
        for (uint32_t i = 0; i < nt; i++)
        {
            const rt_triangle& t = d->triangles[i];
            uint64_t code = 0;
            uint32_t q[3];
            for (int a = 0; a < 3; a++)
            {
                const double c = (double(d->vertices[t.v0].p[a]) + d->vertices[t.v1].p[a] + d->vertices[t.v2].p[a]) / 3.0;
                const double ext = double(mx[a]) - double(mn[a]);
                const double f = ext > 0.0 ? (c - mn[a]) / ext : 0.0;
                q[a] = uint32_t(std::min(1023.0, std::max(0.0, f * 1024.0)));
            }
            for (int bit = 9; bit >= 0; bit--)
                for (int a = 0; a < 3; a++) code = (code << 1) | ((q[a] >> bit) & 1u);
            order[i] = { code, i };
        }
        std::sort(order.begin(), order.end());
        s->ndist_blk = (nt + kDistBlock - 1) / kDistBlock;
        distblk.resize(size_t(s->ndist_blk) * 2);
        for (uint32_t b = 0; b < s->ndist_blk; b++)
        {
            float bmn[3] = { rtd::kFltMax, rtd::kFltMax, rtd::kFltMax }, bmx[3] = { -rtd::kFltMax, -rtd::kFltMax, -rtd::kFltMax };
            for (uint32_t k = b * kDistBlock; k < std::min(nt, (b + 1) * kDistBlock); k++)
            {
                const rt_triangle& t = d->triangles[order[k].second];
                const float *p[3] = { d->vertices[t.v0].p, d->vertices[t.v1].p, d->vertices[t.v2].p };
                dist_record(p[0], p[1], p[2], &tridist[6 * size_t(k)]);
                for (int v = 0; v < 3; v++)
                    for (int a = 0; a < 3; a++)
                    {
                        bmn[a] = std::min(bmn[a], p[v][a]);
                        bmx[a] = std::max(bmx[a], p[v][a]);
                    }
            }
            distblk[2 * b] = make_float4(bmn[0], bmn[1], bmn[2], 0.0f);
            distblk[2 * b + 1] = make_float4(bmx[0], bmx[1], bmx[2], 0.0f);
        }
        s->scene_scale = scale;
        for (int a = 0; a < 3; a++)
        {
            s->vmin[a] = mn[a];
            s->vmax[a] = mx[a];
        }
    }
    RT_HIP(hipMalloc(&s->d_distblk, sizeof(float4) * std::max<size_t>(1, distblk.size())));
    RT_HIP(hipMemcpy(s->d_distblk, distblk.data(), sizeof(float4) * distblk.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMalloc(&s->d_trimt, sizeof(float4) * trimt.size()));
    RT_HIP(hipMalloc(&s->d_tridist, sizeof(float4) * tridist.size()));
    RT_HIP(hipMemcpy(s->d_trimt, trimt.data(), sizeof(float4) * trimt.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_tridist, tridist.data(), sizeof(float4) * tridist.size(), hipMemcpyHostToDevice));
    if (packable)
    {
        RT_HIP(hipMalloc(&s->d_cellw, sizeof(uint32_t) * nc));
        RT_HIP(hipMemcpy(s->d_cellw, cellw.data(), sizeof(uint32_t) * nc, hipMemcpyHostToDevice));
        if (!cellwo.empty())
        {
            RT_HIP(hipMalloc(&s->d_cellwo, sizeof(uint32_t) * cellwo.size()));
            RT_HIP(hipMemcpy(s->d_cellwo, cellwo.data(), sizeof(uint32_t) * cellwo.size(), hipMemcpyHostToDevice));
            s->oct_stride = nc;
        }
        if (!cellwb.empty())
        {
            RT_HIP(hipMalloc(&s->d_cellwb, sizeof(uint32_t) * cellwb.size()));
            RT_HIP(hipMemcpy(s->d_cellwb, cellwb.data(), sizeof(uint32_t) * cellwb.size(), hipMemcpyHostToDevice));
            s->box_stride = nc;
        }
    }
    s->device_bytes = sizeof(uint32_t) * (nc + 1) +
                      sizeof(float4) * (refs.size() + nfrefs + shade.size() + facen.size() + trimt.size() +
                                        tridist.size() + distblk.size()) +
                      sizeof(uint32_t) * (cellw.size() + cellwo.size() + cellwb.size());
    RT_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    RT_HIP(hipEventCreateWithFlags(&s->ev1, hipEventDisableTiming));

    *out = s.release();
    return RT_OK;
}

int rt_scene_destroy(rt_scene *s)
{
    if (!s) return RT_OK;
    {
        std::lock_guard<std::mutex> lk(s->mtx);
        (void)hipSetDevice(s->device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->last_stream && s->ev_recorded) (void)hipEventSynchronize(s->ev1);
        (void)hipFree(s->d_off);
        (void)hipFree(s->d_refs);
        (void)hipFree(s->d_frefs);
        (void)hipFree(s->d_shade);
        (void)hipFree(s->d_facen);
        (void)hipFree(s->d_cellw);
        (void)hipFree(s->d_cellwo);
        (void)hipFree(s->d_cellwb);
        (void)hipFree(s->d_trimt);
        (void)hipFree(s->d_tridist);
        (void)hipFree(s->d_distblk);
        (void)hipFree(s->d_clk);
        for (HfCtx& h : s->hf)
        {
            (void)hipFree(h.marks);
            (void)hipFree(h.cost);
            (void)hipFree(h.lists);
            (void)hipFree(h.plans);
            (void)hipFree(h.ticket);
            (void)hipFree(h.wh_marks);
            (void)hipFree(h.wh_lists);
            if (h.wh_cnt) (void)hipHostFree(h.wh_cnt);
        }
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
        if (s->ev_join) (void)hipEventDestroy(s->ev_join);
        (void)hipFree(s->d_smp);
        (void)hipFree(s->d_ndc);
        (void)hipFree(s->d_frame);
        if (s->h_smp_pinned) (void)hipHostFree(s->h_smp_pinned);
        if (s->h_frame) (void)hipHostFree(s->h_frame);
        if (s->ev1) (void)hipEventDestroy(s->ev1);
        for (hipEvent_t e : s->band_ev) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : s->kt0) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : s->kt1) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : s->tile_ev) if (e) (void)hipEventDestroy(e);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        if (s->stream2) (void)hipStreamDestroy(s->stream2);
        if (s->ev_t_fork) (void)hipEventDestroy(s->ev_t_fork);
        if (s->ev_t_join) (void)hipEventDestroy(s->ev_t_join);

    }
    delete s;
    return RT_OK;
}

int rt_scene_device_bytes(const rt_scene *s, uint64_t *bytes)
{
    if (!s || !bytes) return fail(RT_E_INVALID, "NULL argument");
    *bytes = s->device_bytes;
    return RT_OK;
}

} // extern "C"

namespace {
// Per-sample records requested from the product kernels (rt_render_records_device): the
// rectangle's samples land in d[((y - y0) * w + (x - x0)) * spp + s].
struct RecOut { rt_sample_rec *d; uint32_t x0, y0, w, h; };

void set_records(KParams& P, const RecOut& r)
{
    P.recs = r.d;
    P.rec_x0 = r.x0;
    P.rec_y0 = r.y0;
    P.rec_w = r.w;
    P.rec_h = r.h;
}

// Frame parameters of a device-resident render (see render_device); returns the local tile count.
uint32_t device_params(const rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, bool shard,
                       uint32_t *d_out, uint32_t *d_hits, KParams& P)
{
    frame_params(s, f, P);
    P.rx0 = 0; P.ry0 = 0; P.rw = f->width; P.rh = f->height;
    P.tiles_x = (f->width + kTile - 1) / kTile;
    const uint32_t ntiles = P.tiles_x * ((f->height + kTile - 1) / kTile);
    P.rank = rank; P.nranks = nranks;
    P.out = d_out;
    P.hits = d_hits;
    P.pitch = shard ? 0u : f->width;
    P.shard_mode = shard ? 1u : 0u;
    return ntiles > rank ? (ntiles - rank + nranks - 1) / nranks : 0;
}

// The device-resident render of a whole frame (shard false: d_out[y*W + x]) or of one rank's
// interleaved 16x16 tiles (shard true: d_out = the compact shard, also for nranks == 1),
// optionally with per-sample hit IDs.
int render_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, bool shard, uint32_t *d_out,
                  uint32_t *d_hits, void *hip_stream, const RecOut *recs = nullptr)
{
    if (!s || !d_out || nranks == 0 || rank >= nranks) return fail(RT_E_INVALID, "bad arguments");
    int rc = validate_frame(f);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    KParams P;
    const uint32_t local = device_params(s, f, rank, nranks, shard, d_out, d_hits, P);
    if (recs) set_records(P, *recs);
    return launch_render(s, f, P, local, static_cast<hipStream_t>(hip_stream));
}

// rt_render_batch_device's frames [0, n): one k_render_batch launch when they can share it.  The
// cheap checks (one device) come before anything touches a scene's device state; a scene listed
// twice with another frame shape or sample table than its last frame's would read the last one's
// tables, so such batches take one launch per frame (counted in rt_scene_info.batch_fallbacks).
int render_batch_chunk(rt_scene *const *S, const rt_frame *F, uint32_t n, uint32_t rank, uint32_t nranks,
                       uint32_t *const *outs, uint32_t *const *hits, const RecOut *recs, void *hip_stream)
{
    bool batched = false;
    bool one_device = true;
    for (uint32_t i = 1; i < n; i++) one_device = one_device && S[i]->device == S[0]->device;
    if (n >= 2 && one_device)
    {
        std::vector<rt_scene *> uniq(S, S + n);
        std::sort(uniq.begin(), uniq.end());
        uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
        std::vector<std::unique_lock<std::mutex>> locks;
        for (rt_scene *s : uniq) locks.emplace_back(s->mtx);
        int rc = ensure_device(S[0]);
        if (rc) return rc;
        KParams P[kMaxBatch];
        uint32_t local = 0;
        for (uint32_t i = 0; i < n; i++)
        {
            if ((rc = prepare_samples(S[i], &F[i], std::max(1u, F[i].spp)))) return rc;
            local = device_params(S[i], &F[i], rank, nranks, nranks > 1, outs[i], hits ? hits[i] : nullptr, P[i]);
            if (recs) set_records(P[i], recs[i]);
        }
        bool tables_ok = true;
        for (uint32_t i = 0; i < n; i++) tables_ok = tables_ok && tables_match(S[i], &F[i], std::max(1u, F[i].spp));
        if (tables_ok) rc = launch_batch(S, F, n, P, local, static_cast<hipStream_t>(hip_stream), &batched);
        if (batched)
        {
            S[0]->batch_launches++;
            return rc;
        }
    }
    if (n >= 2)
    {
        std::lock_guard<std::mutex> lk(S[0]->mtx);
        S[0]->batch_fallbacks++;
    }
    for (uint32_t i = 0; i < n; i++)
        if (int rc = render_device(S[i], &F[i], rank, nranks, nranks > 1, outs[i], hits ? hits[i] : nullptr, hip_stream,
                                   recs ? &recs[i] : nullptr))
            return rc;
    return RT_OK;
}
} // namespace

extern "C" {

int rt_render_frame_device(rt_scene *s, const rt_frame *f, uint32_t *d_bgra, void *hip_stream)
{
    return render_device(s, f, 0, 1, false, d_bgra, nullptr, hip_stream);
}

int rt_shard_elems(uint32_t width, uint32_t height, uint32_t nranks, uint64_t *elems)
{
    if (!elems || nranks == 0 || width == 0 || height == 0) return fail(RT_E_INVALID, "bad arguments");
    const uint64_t ntiles = uint64_t((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
    *elems = ((ntiles + nranks - 1) / nranks) * kTilePix;
    return RT_OK;
}

int rt_render_shard_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, uint32_t *d_shard,
                           void *hip_stream)
{
    return render_device(s, f, rank, nranks, true, d_shard, nullptr, hip_stream);
}

int rt_render_batch_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                           uint32_t nranks, uint32_t *const *d_outs, uint32_t *const *d_hits, void *hip_stream)
{
    if (!scenes || !frames || !d_outs || nranks == 0 || rank >= nranks) return fail(RT_E_INVALID, "bad arguments");
    for (uint32_t i = 0; i < n; i++)
    {
        if (!scenes[i] || !d_outs[i]) return fail(RT_E_INVALID, "NULL scene or output");
        if (int rc = validate_frame(&frames[i])) return rc;
    }
    for (uint32_t i = 0; i < n;)
    {
        const uint32_t c = batch_chunk_len(n, i);
        if (int rc = render_batch_chunk(scenes + i, frames + i, c, rank, nranks, d_outs + i,
                                        d_hits ? d_hits + i : nullptr, nullptr, hip_stream))
            return rc;
        i += c;
    }
    return RT_OK;
}

int rt_render_records_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                             uint32_t nranks, uint32_t *const *d_outs, const rt_tile *rects,
                             rt_sample_rec *const *d_recs, void *hip_stream)
{
    if (!scenes || !frames || !d_outs || !rects || !d_recs || n == 0 || nranks == 0 || rank >= nranks)
        return fail(RT_E_INVALID, "bad arguments");
    std::vector<RecOut> ro(n);
    for (uint32_t i = 0; i < n; i++)
    {
        if (!scenes[i] || !d_outs[i] || !d_recs[i]) return fail(RT_E_INVALID, "NULL scene, output or record array");
        if (int rc = validate_frame(&frames[i])) return rc;
        if ((frames[i].kernel & RT_KERNEL_KIND_MASK) != RT_KERNEL_AUTO || frames[i].intersector != RT_ISECT_GRID ||
            frames[i].tri_test != RT_TRI_MOLLER_TRUMBORE)
            return fail(RT_E_INVALID, "records come from AUTO's grid / IntersectRayTri path only");
        const rt_tile& r = rects[i];
        if (r.x1 <= r.x0 || r.y1 <= r.y0 || r.x1 > frames[i].width || r.y1 > frames[i].height)
            return fail(RT_E_INVALID, "record rectangle outside the frame or empty");
        ro[i] = RecOut{ d_recs[i], r.x0, r.y0, r.x1 - r.x0, r.y1 - r.y0 };
    }
    if (n == 1)
    {
        if (int rc = render_device(scenes[0], &frames[0], rank, nranks, nranks > 1, d_outs[0], nullptr, hip_stream,
                                   &ro[0]))
            return rc;
    }
    else
        for (uint32_t i = 0; i < n;)
        {
            const uint32_t c = batch_chunk_len(n, i);
            if (int rc = render_batch_chunk(scenes + i, frames + i, c, rank, nranks, d_outs + i, nullptr,
                                            ro.data() + i, hip_stream))
                return rc;
            i += c;
        }
    // the raw records made final (k_record_fixup), per frame on the launch stream
    for (uint32_t i = 0; i < n; i++)
    {
        rt_scene *s = scenes[i];
        std::lock_guard<std::mutex> lk(s->mtx);
        if (int rc = ensure_device(s)) return rc;
        if (int rc = prepare_samples(s, &frames[i], std::max(1u, frames[i].spp))) return rc;
        KParams P;
        frame_params(s, &frames[i], P);
        set_records(P, ro[i]);
        const uint64_t nrec = uint64_t(ro[i].w) * ro[i].h * P.spp;
        if (nrec > 0xFFFFFFFFull) return fail(RT_E_INVALID, "record rectangle too large");
        hipLaunchKernelGGL(k_record_fixup, dim3(uint32_t((nrec + kWG - 1) / kWG)), dim3(kWG), 0,
                           static_cast<hipStream_t>(hip_stream), P, uint32_t(nrec));
        RT_HIP(hipGetLastError());
    }
    return RT_OK;
}

int rt_render_hits_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, uint32_t *d_out,
                          uint32_t *d_hits, void *hip_stream)
{
    if (!d_hits) return fail(RT_E_INVALID, "d_hits is NULL");
    return render_device(s, f, rank, nranks, nranks > 1, d_out, d_hits, hip_stream);
}

int rt_unshard_device(uint32_t width, uint32_t height, uint32_t nranks, const uint32_t *d_gathered,
                      uint32_t *d_bgra, void *hip_stream)
{
    if (!d_gathered || !d_bgra || nranks == 0) return fail(RT_E_INVALID, "bad arguments");
    uint64_t elems = 0;
    int rc = rt_shard_elems(width, height, nranks, &elems);
    if (rc) return rc;
    const uint32_t tiles_x = (width + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_unshard, dim3((width + 63) / 64, (height + 3) / 4), dim3(kWG), 0,
                       static_cast<hipStream_t>(hip_stream), d_gathered, d_bgra, width, height, tiles_x, nranks,
                       elems);
    RT_HIP(hipGetLastError());
    return RT_OK;
}

int rt_last_kernel_ms(rt_scene *s, float *ms)
{
    if (!s || !ms) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    if (s->kt_last >= kTimeRing) return fail(RT_E_INVALID, "no timed kernel recorded yet");
    RT_HIP(hipEventSynchronize(s->kt1[s->kt_last]));
    RT_HIP(hipEventElapsedTime(ms, s->kt0[s->kt_last], s->kt1[s->kt_last]));
    return RT_OK;
}

int rt_scene_set_timing(rt_scene *s, uint32_t every)
{
    if (!s) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    s->time_every = every;
    s->launches = 0;
    return RT_OK;
}

int rt_kernel_times(rt_scene *s, float *ms, uint32_t max_n, uint32_t *n)
{
    if (!s || !n || (max_n && !ms)) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    const uint32_t cnt = std::min(max_n, s->kt_count);
    const uint32_t next = s->kt_next;
    s->kt_count = 0;                      // consumed whatever happens below
    uint32_t got = 0;
    for (uint32_t i = 0; i < cnt; i++)
    {
        // a pair that cannot be read (a launch that failed between its two records) is skipped
        const uint32_t slot = (next + kTimeRing - cnt + i) % kTimeRing;
        float v = 0.0f;
        if (hipEventSynchronize(s->kt1[slot]) == hipSuccess &&
            hipEventElapsedTime(&v, s->kt0[slot], s->kt1[slot]) == hipSuccess && v >= 0.0f)
            ms[got++] = v;
        else
            (void)hipGetLastError();
    }
    *n = got;
    return RT_OK;
}

int rt_render_tiles(rt_scene *s, const rt_frame *f, const rt_tile *tiles, uint32_t n, uint32_t *const *bufs)
{
    if (!s || (n && (!tiles || !bufs))) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    uint32_t bx0 = 0xFFFFFFFFu, by0 = 0xFFFFFFFFu, bx1 = 0, by1 = 0;
    for (uint32_t i = 0; i < n; i++)
    {
        const rt_tile& t = tiles[i];
        if (!bufs[i] || t.x1 <= t.x0 || t.y1 <= t.y0 || t.x1 > f->width || t.y1 > f->height)
            return fail(RT_E_INVALID, "tile outside the frame or empty");
        bx0 = std::min(bx0, t.x0); by0 = std::min(by0, t.y0);
        bx1 = std::max(bx1, t.x1); by1 = std::max(by1, t.y1);
    }
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint32_t rw = bx1 - bx0, rh = by1 - by0;
    const size_t words = size_t(rw) * rh;
    if ((rc = ensure_frame(s, words, true))) return rc;
    KParams P;
    frame_params(s, f, P);
    P.rx0 = bx0; P.ry0 = by0; P.rw = rw; P.rh = rh;
    P.tiles_x = (rw + kTile - 1) / kTile;
    P.rank = 0; P.nranks = 1;
    P.out = s->d_frame; P.pitch = rw; P.shard_mode = 0;
    if ((rc = launch_render(s, f, P, P.tiles_x * ((rh + kTile - 1) / kTile), s->stream))) return rc;
    // D2H in row bands; band k's rows are scattered into the tiles while band k+1 is in flight
    const uint32_t nb = std::min(kTileBands, rh), bh = (rh + nb - 1) / nb;
    for (uint32_t b = 0; b < nb; b++)
    {
        const uint32_t ya = b * bh, yb = std::min(rh, ya + bh);
        if (ya >= yb) break;
        if (!s->tile_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->tile_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(s->h_frame + size_t(ya) * rw, s->d_frame + size_t(ya) * rw,
                              size_t(yb - ya) * rw * 4, hipMemcpyDeviceToHost, s->stream));
        RT_HIP(hipEventRecord(s->tile_ev[b], s->stream));
    }
    for (uint32_t b = 0; b < nb; b++)
    {
        const uint32_t ya = by0 + b * bh, yb = std::min(by1, ya + bh);
        if (ya >= yb) break;
        RT_HIP(hipEventSynchronize(s->tile_ev[b]));
        for (uint32_t i = 0; i < n; i++)                         // framebuffer.h:41-45 layout
        {
            const rt_tile& t = tiles[i];
            const uint32_t tw = t.x1 - t.x0;
            for (uint32_t y = std::max(t.y0, ya); y < std::min(t.y1, yb); y++)
                std::memcpy(bufs[i] + size_t(y - t.y0) * tw, s->h_frame + size_t(y - by0) * rw + (t.x0 - bx0),
                            size_t(tw) * 4);
        }
    }
    return RT_OK;
}

int rt_host_alloc(size_t bytes, void **out)
{
    if (!out || bytes == 0) return fail(RT_E_INVALID, "bad arguments");
    *out = nullptr;
    RT_HIP(hipHostMalloc(out, bytes));
    return RT_OK;
}

int rt_host_free(void *p)
{
    if (p) RT_HIP(hipHostFree(p));
    return RT_OK;
}

int rt_render_frame_host(rt_scene *s, const rt_frame *f, uint32_t *h_bgra, const uint32_t *band_y1,
                         uint32_t nbands)
{
    if (!s || !h_bgra || (nbands && !band_y1)) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (nbands > kMaxBands) return fail(RT_E_INVALID, "more than 64 row bands");
    for (uint32_t b = 0; b < nbands; b++)
        if (band_y1[b] == 0 || band_y1[b] > f->height || (b && band_y1[b] <= band_y1[b - 1]) ||
            (b + 1 == nbands && band_y1[b] != f->height))
            return fail(RT_E_INVALID, "band ends must increase strictly and end at the frame height");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint32_t W = f->width, H = f->height;
    if ((rc = ensure_frame(s, size_t(W) * H, false))) return rc;
    KParams P;
    frame_params(s, f, P);
    P.rx0 = 0; P.ry0 = 0; P.rw = W; P.rh = H;
    P.tiles_x = (W + kTile - 1) / kTile;
    P.rank = 0; P.nranks = 1;
    P.out = s->d_frame; P.pitch = W; P.shard_mode = 0;
    s->nbands = 0;
    if ((rc = launch_render(s, f, P, P.tiles_x * ((H + kTile - 1) / kTile), s->stream))) return rc;
    const uint32_t nb = nbands ? nbands : 1;
    for (uint32_t b = 0, ya = 0; b < nb; b++)
    {
        const uint32_t yb = nbands ? band_y1[b] : H;
        if (!s->band_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->band_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(h_bgra + size_t(ya) * W, s->d_frame + size_t(ya) * W, size_t(yb - ya) * W * 4,
                              hipMemcpyDeviceToHost, s->stream));
        RT_HIP(hipEventRecord(s->band_ev[b], s->stream));
        s->band_y1[b] = yb;
        ya = yb;
    }
    s->nbands = nb;
    return RT_OK;
}

int rt_render_frame_host_tiled(rt_scene *s, const rt_frame *f, uint32_t *h_tiles, uint32_t tiles_x, uint32_t tiles_y,
                               uint32_t nlaunch)
{
    if (!s || !h_tiles || tiles_x == 0 || tiles_y == 0 || nlaunch == 0) return fail(RT_E_INVALID, "bad arguments");
    int rc = validate_frame(f);
    if (rc) return rc;
    const uint32_t W = f->width, H = f->height;
    if (tiles_y > kMaxBands) return fail(RT_E_INVALID, "more than 64 tile rows");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    if ((rc = ensure_frame(s, size_t(W) * H, false))) return rc;
    if (!s->stream2)
    {
        RT_HIP(hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking));
        RT_HIP(hipEventCreateWithFlags(&s->ev_t_fork, hipEventDisableTiming));
        RT_HIP(hipEventCreateWithFlags(&s->ev_t_join, hipEventDisableTiming));
    }
    // Framebuffer::Resize's tile rows (framebuffer.cpp:106-117): row r spans [r * th, (r + 1) * th),
    // the last one to H; launch j renders tile rows [j * R / n, (j + 1) * R / n)
    const uint32_t tw = W / tiles_x, th = H / tiles_y;
    const uint32_t nl = std::min(nlaunch, tiles_y);
    auto row_y = [&](uint32_t r) { return r >= tiles_y ? H : r * th; };
    hipStream_t st[2] = { s->stream, s->stream2 };
    // both streams after everything earlier on this scene (the scene's tables and records are shared)
    if (s->ev_recorded) RT_HIP(hipStreamWaitEvent(st[0], s->ev1, 0));
    KParams P0;
    frame_params(s, f, P0);
    if (use_lanes(f, spp) && P0.isect == RT_ISECT_GRID && P0.tri_test == RT_TRI_MOLLER_TRUMBORE &&
        ((f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_AUTO || (f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_COMPACT))
        if ((rc = ensure_origin_terms(s, P0, st[0]))) return rc;
    RT_HIP(hipEventRecord(s->ev_t_fork, st[0]));
    RT_HIP(hipStreamWaitEvent(st[1], s->ev_t_fork, 0));
    s->nbands = 0;
    for (uint32_t j = 0; j < nl; j++)
    {
        const uint32_t r0 = j * tiles_y / nl, r1 = (j + 1) * tiles_y / nl;
        const uint32_t ya = row_y(r0), yb = row_y(r1);
        if (ya >= yb) continue;
        KParams P = P0;
        P.rx0 = 0; P.ry0 = ya; P.rw = W; P.rh = yb - ya;
        P.tiles_x = (W + kTile - 1) / kTile;
        P.rank = 0; P.nranks = 1;
        P.out = s->d_frame; P.pitch = W; P.shard_mode = 2;
        P.fb_tw = tw; P.fb_th = th; P.fb_tx = tiles_x; P.fb_ty = tiles_y;
        P.fb_mtw = tw ? uint32_t(((1ull << 32) + tw - 1) / tw) : 0u;
        P.fb_mth = th ? uint32_t(((1ull << 32) + th - 1) / th) : 0u;
        // launches alternate between the two streams, so one launch's tail overlaps the next one's
        // start and its tile rows' copy-back overlaps the next launch's render
        hipStream_t sj = st[j & 1u];
        if ((rc = launch_render(s, f, P, P.tiles_x * ((P.rh + kTile - 1) / kTile), sj, false))) return rc;
        // the launch's tile rows are words [ya * W, yb * W) of the tile layout: ONE contiguous copy
        // (a copy per tile row cost ~14 us of launch overhead each, measured: 9 copies of a whole
        // frame 0.50 ms vs one 0.37, profiles/r04l_e2e_breakdown.json)
        const uint32_t b = s->nbands;
        if (!s->band_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->band_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(h_tiles + size_t(ya) * W, s->d_frame + size_t(ya) * W, size_t(yb - ya) * W * 4,
                              hipMemcpyDeviceToHost, sj));
        RT_HIP(hipEventRecord(s->band_ev[b], sj));
        s->band_y1[b] = yb;
        s->nbands = b + 1;
    }
    // the frame is done when both streams are: join on the first one, whose event ev1 marks it
    RT_HIP(hipEventRecord(s->ev_t_join, st[1]));
    RT_HIP(hipStreamWaitEvent(st[0], s->ev_t_join, 0));
    RT_HIP(hipEventRecord(s->ev1, st[0]));
    s->ev_recorded = true;
    s->last_stream = st[0];
    // bands land per tile row but not in row order across the two streams: rt_frame_host_wait(y1)
    // needs every row below y1, so a band's wait covers the bands before it (events in row order)
    return RT_OK;
}

int rt_frame_host_wait(rt_scene *s, uint32_t y1)
{
    if (!s) return fail(RT_E_INVALID, "NULL argument");
    hipEvent_t ev[kMaxBands];
    uint32_t n = 0;
    {
        std::lock_guard<std::mutex> lk(s->mtx);
        if (s->nbands == 0) return fail(RT_E_INVALID, "no rt_render_frame_host in flight");
        // every band below y1 (rt_render_frame_host_tiled's bands land from two streams, so a later
        // band may be done before an earlier one); a finished event costs nothing to wait on
        while (n < s->nbands && (n == 0 || s->band_y1[n - 1] < y1)) { ev[n] = s->band_ev[n]; n++; }
    }
    for (uint32_t b = 0; b < n; b++)
        RT_HIP(hipEventSynchronize(ev[b]));     // events are only re-recorded by a later frame
    return RT_OK;
}

int rt_trace_samples(rt_scene *s, const rt_frame *f, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                     rt_sample_rec *out)
{
    if (!s || !out) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (w == 0 || h == 0 || x0 + w > f->width || y0 + h > f->height)
        return fail(RT_E_INVALID, "rectangle outside the frame");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint64_t n64 = uint64_t(w) * h * spp;
    if (n64 > (1ull << 28)) return fail(RT_E_INVALID, "too many samples for one record call");
    const uint32_t n = uint32_t(n64);
    rt_sample_rec *d_rec = nullptr;
    RT_HIP(hipMalloc(&d_rec, sizeof(rt_sample_rec) * n));
    KParams P;
    frame_params(s, f, P);
    P.recs = d_rec;
    P.rec_x0 = x0; P.rec_y0 = y0; P.rec_w = w; P.rec_h = h;
    if (P.isect == RT_ISECT_RAY_MARCH && (f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE)) P.isect += 0x100;
    hipLaunchKernelGGL(k_trace_records, dim3((n + kWG - 1) / kWG), dim3(kWG), 0, s->stream, P, n);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_rec, sizeof(rt_sample_rec) * n, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d_rec);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_trace_samples: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_wave_clocks(rt_scene *s, uint64_t *out, uint32_t max_items, uint32_t *n_items)
{
    if (!s || !n_items) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    int rc;
    if ((rc = ensure_device(s))) return rc;
    *n_items = s->clk_items;
    if (!out || !s->d_clk) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out, s->d_clk, sizeof(uint64_t) * 4 * std::min(max_items, s->clk_items), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_heavy_first(rt_scene *s, uint32_t *front, uint32_t *listed, uint32_t *epoch)
{
    if (!s || !front || !listed || !epoch) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    int rc;
    if ((rc = ensure_device(s))) return rc;
    *front = *listed = *epoch = 0;
    const HfCtx *c = nullptr;
    for (const HfCtx& h : s->hf)
        if (h.frames && (!c || h.used > c->used)) c = &h;
    if (!c) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    HfPlan pl;
    RT_HIP(hipMemcpy(&pl, c->plans + (c->ver & 1u), sizeof(pl), hipMemcpyDeviceToHost));
    *front = c->front;
    *listed = c->ver ? std::min(pl.cnt_hi + pl.cnt_lo, c->front) : 0u;
    *epoch = c->frames;
    return RT_OK;
}

int rt_debug_wide_items(rt_scene *s, uint32_t *count)
{
    if (!s || !count) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    const HfCtx *c = nullptr;
    for (const HfCtx& h : s->hf)
        if (h.wh_cnt && (!c || h.used > c->used)) c = &h;
    if (c) RT_HIP(hipDeviceSynchronize());
    *count = c ? *(volatile uint32_t *)c->wh_cnt : 0u;
    return RT_OK;
}

int rt_debug_rcp_check(uint64_t *bad_by_exponent, int device)
{
    if (!bad_by_exponent) return fail(RT_E_INVALID, "NULL argument");
    RT_HIP(hipSetDevice(device));
    unsigned long long *d_bad = nullptr;
    RT_HIP(hipMalloc(&d_bad, 256 * sizeof(unsigned long long)));
    hipError_t e = hipMemset(d_bad, 0, 256 * sizeof(unsigned long long));
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(k_rcp_check, dim3(8192), dim3(kWG), 0, nullptr, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(bad_by_exponent, d_bad, 256 * sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_rcp_check: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_gamma_check(uint64_t *mismatches, int device)
{
    if (!mismatches) return fail(RT_E_INVALID, "NULL argument");
    RT_HIP(hipSetDevice(device));
    unsigned long long *d_bad = nullptr;
    RT_HIP(hipMalloc(&d_bad, sizeof(unsigned long long)));
    hipError_t e = hipMemset(d_bad, 0, sizeof(unsigned long long));
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(k_gamma_check, dim3(8192), dim3(kWG), 0, nullptr, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(mismatches, d_bad, sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_gamma_check: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_primitives(int kind, const float *in, uint32_t n, float *out, int device)
{
    // kind 7 (DistancePointTri) reaches the device as pos + pad + the 24-float scene record
    static const uint32_t in_w[8] = { 18, 12, 23, 3, 11, 18, 18, 28 }, out_w[8] = { 8, 4, 6, 4, 3, 8, 8, 1 };
    if (kind < 0 || kind > 7 || !in || !out) return fail(RT_E_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    RT_HIP(hipSetDevice(device));
    std::vector<float> host_in;
    if (kind == 7)
    {
        host_in.resize(size_t(28) * n);
        for (uint32_t i = 0; i < n; i++)
        {
            const float *a = in + 12 * size_t(i);
            float *o = &host_in[28 * size_t(i)];
            o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = 0.0f;
            dist_record(a + 3, a + 6, a + 9, reinterpret_cast<float4 *>(o + 4));
        }
    }
    else
        host_in.assign(in, in + size_t(in_w[kind]) * n);
    if (kind == 2)   // camera.h:41-42 fov_xs is a host-side constant (double ::tan, hazard H5)
        for (uint32_t i = 0; i < n; i++)
        {
            const float hfov = host_in[23 * size_t(i) + 22] * float(0.0174532925);
            host_in[23 * size_t(i) + 22] = float(::tan(double(hfov / 2.0f)));
        }
    in = host_in.data();
    float *d_in = nullptr, *d_out = nullptr;
    RT_HIP(hipMalloc(&d_in, sizeof(float) * in_w[kind] * n));
    RT_HIP(hipMalloc(&d_out, sizeof(float) * out_w[kind] * n));
    hipError_t e = hipMemcpy(d_in, in, sizeof(float) * in_w[kind] * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(k_primitives, dim3((n + kWG - 1) / kWG), dim3(kWG), 0, nullptr, kind, d_in, n, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(float) * out_w[kind] * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_primitives: ") + hipGetErrorString(e));
    return RT_OK;
}

} // extern "C"
