// rt_scene.h -- the library's scene object (struct rt_scene, opaque in the C ABI) and the host
// functions rt_tracer.hip and rt_plan.hip share.  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rt_tracer.h"
#include "rt_internal.h"
#include "rt_kparams.h"

// HIP call -> RT_E_HIP with the call's text and the runtime's message (rt_last_error)
#define RT_HIP(expr)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return rt_internal_fail(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace rtk {

// A HIP event shared by the scenes whose last launch it marks: a batched launch's stop event is every
// batched scene's "last launch" (rt_scene::ev_last), so it lives while any of them refers to it.
struct EvHolder
{
    hipEvent_t ev = nullptr;
    EvHolder() = default;
    EvHolder(const EvHolder&) = delete;
    EvHolder& operator=(const EvHolder&) = delete;
    ~EvHolder()
    {
        if (ev) (void)hipEventDestroy(ev);
    }
};
using EvRef = std::shared_ptr<EvHolder>;

// Heavy-first state of one launch shape (device arrays; see KParams::hf_*)
struct HfCtx
{
    uint64_t key[5] = { 0, 0, 0, 0, 0 };   // launch shape: blocks, spp, region, shard, variant, batch
    uint32_t nblocks = 0, front = 0;
    uint32_t cap_blocks = 0;            // allocated marks per buffer
    void *mem = nullptr;                // one allocation holding the arrays below (hf_prepare)
    size_t cleared_bytes = 0;           // its head that a new shape clears
    uint32_t *marks = nullptr;          // [2][cap_blocks]
    uint32_t *cost = nullptr;           // [cap_blocks * kWavesPerWG] wave cycles of the last frame
    uint32_t *lists = nullptr;          // [2][kHfFrontMax], by plan version parity
    HfPlan *plans = nullptr;            // [2], by plan version parity
    uint32_t *ticket = nullptr;         // k_hf_plan's workgroup ticket
    uint32_t *wh_marks = nullptr;       // [2][cap_blocks * kWavesPerWG] wide items, by version parity
    uint32_t *wh_lists = nullptr;       // [2][kWhMax]
    volatile uint32_t *wh_cnt = nullptr;  // host-mapped [2]: the newest plan's G-lane waves, LDS items (rt_scene::h_wh_cnt)
    uint32_t *wh_cnt_dev = nullptr;     // its device address
    uint32_t frames = 0;                // frames rendered with this shape
    uint32_t ver = 0;                   // version of the plan the frames use
    // a plan launched on the scene's plan stream after a measured frame (launch_plans): version pend
    // (0: none), adopted -- the launch stream waits for pend_ev -- by the second frame after it, or
    // by the next frame that measures
    uint32_t pend = 0, pend_age = 0;
    hipEvent_t pend_ev = nullptr;
    // an adopted plan still running: EVERY later frame of the shape waits for it (fence_ev), not only
    // the adopting one -- an overlapped frame on the other stream orders only after the launch two
    // back, and read the plan's buffers while k_hf_plan wrote them (blocks left unrendered,
    // tools/overlap_stress.py --prebatch)
    bool fence = false;
    hipEvent_t fence_ev = nullptr;
    hipStream_t fence_st = nullptr;     // the adopting frame's stream (already ordered after it)
    uint64_t used = 0;                  // LRU stamp
    uint64_t cam = 0;                   // camera signature of the last frame (cam_signature)
};

} // namespace rtk

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
    float4 *d_refs = nullptr, *d_shade = nullptr, *d_facen = nullptr;
    float4 *d_trimt = nullptr, *d_tridist = nullptr, *d_distblk = nullptr;
    uint32_t ndist_blk = 0;
    float scene_scale = 0.0f;
    float vmin[3] = { 0, 0, 0 }, vmax[3] = { 0, 0, 0 };
    uint64_t device_bytes = 0;
    uint32_t compact_wgs = 2048;    // RT_KERNEL_COMPACT grid: 8 x 256-lane workgroups per CU
    bool rcp_safe = false;          // every |det| of the ray/tri test is far below 2^126 (FAST_RCP)
    bool pack_ok = false;           // dims <= 512: the remaining-cell counts pack into one word
    // Per-camera-origin records (k_origin_pre), TWO buffers: a frame whose origin is in neither computes
    // its records into the one the scene's last launch does not read, so consecutive frames of a moving
    // camera may still overlap (RT_KERNEL_FLAG_OVERLAP): the launch before the last -- the only other one
    // in flight -- is waited for first (order_overlap).  fref_org: each buffer's origin (bit patterns),
    // fref_ok: computed; fref_last: bit b = the last launch reads buffer b.
    float4 *d_frefs[2] = { nullptr, nullptr };
    bool fref_ok[2] = { false, false };
    uint32_t fref_org[2][3] = { { 0, 0, 0 }, { 0, 0, 0 } };
    uint32_t fref_last = 0;
    uint64_t *d_clk = nullptr;      // RT_KERNEL_FLAG_WAVE_CLOCK records of the last such launch
    size_t clk_cap = 0;
    uint32_t clk_items = 0;
    // AUTO heavy-first order: per launch shape, which blocks the previous frame found heavy
    rtk::HfCtx hf[rtk::kHfCtxs];
    uint32_t *h_wh_cnt = nullptr;       // [kHfCtxs][2] host-mapped counters of the contexts (one allocation)
    uint32_t *d_wh_cnt = nullptr;
    uint64_t hf_clock = 0;
    uint64_t hf_evictions = 0;      // launch shapes that displaced another's state (rt_scene_info)
    uint64_t batch_launches = 0;    // rt_render_batch_device chunks led by this scene: one launch ...
    uint64_t batch_fallbacks = 0;   // ... or one launch per frame (frames that cannot share a launch)
    // scheduling tunables, read ONCE from the environment at rt_scene_create (A/B sweeps): the
    // launch path never calls getenv
    uint32_t hf_floor = 100000;     // RT_HF_FLOOR: heavy-first threshold floor, shader cycles
    uint32_t hf_min_blocks = 4096;  // RT_HF_MIN_BLOCKS: smallest whole launch taking the heavy-first order
    uint32_t hf_front_div = 8;      // the front section holds 1 / this of a launch's blocks ...
    uint32_t hf_front_max = 1024;   // ... at most this many, or 1 / 128 of the blocks if more
                                    // (<= kHfFrontMax: config 5's one launch of 324,000 blocks ran 2.731 / 2.734
                                    // ms at 2048 / 4096 against 2.741 at 1024, profiles/r05q_batch10_partition_front.json)
    uint32_t hf_shift = 2;          // RT_HF_SHIFT: heavy = cost > last max >> hf_shift (very heavy: >> 1)
    uint32_t hf_pos16 = 16;         // RT_HF_POS16: position-aware threshold (k_hf_plan) of single-frame
                                    // launches, sixteenths of the span left; 0: max >> hf_shift
    uint32_t wh_floor = 100000;     // RT_WH_FLOOR: wide-section threshold floor, shader cycles
    uint32_t wh_alpha16 = 32;       // RT_WH_ALPHA16: wide threshold of single-frame launches, sixteenths of the estimated span
    uint32_t wh_alpha16_n2 = 16;    // RT_WH_ALPHA16_N2: the same for a rank of 2 of a batched step
    uint32_t wh_alpha16_n4 = 28;    // RT_WH_ALPHA16_N4: the same for a rank of 3-7 of a batched step
    uint32_t wh_alpha16_n8 = 40;    // RT_WH_ALPHA16_N8: the same for a rank of >= 8 of a batched step
    uint32_t wh_auto_refs = 128;    // RT_WH_AUTO_REFS: AUTO takes the wide section for >= 2-rank
                                    // shards of scenes with a cell list this long
    uint32_t wg64 = 1;              // RT_WG64: AUTO launches of >= wg64_min_blocks 256-lane blocks run
    uint32_t wg64_min_blocks = 8192; // as one-wave workgroups (k_render_lanes_w64)
    uint32_t wg64_batch_min_blocks = 0;  // the same for batched launches
    uint32_t wg64_max_refs = 1024;  // RT_WG64_MAX_REFS: single-frame launches of scenes with a cell of this many
                                    // references keep 256-lane workgroups
    uint32_t wh_lds = 0x8;          // RT_WH_LDS: bit log2(N) (3: N >= 8): a rank of N's wide section has the LDS
                                    // tier (kVarLdsSplit: one 256-lane workgroup per item, its cell lists split
                                    // between the four waves) for its next heaviest items,
                                    // in launches without RT_KERNEL_FLAG_OVERLAP
    uint32_t wh_beta16 = 24;        // RT_WH_BETA16: the LDS tier's threshold, sixteenths of the span estimate
                                    // (items above it and at most wh_alpha16 / 16)
    uint32_t wg64_o8 = 0x2;         // RT_WG64_O8: bit log2(N) (3: N >= 8): a rank of N's fused one-wave
                                    // batch kernel held to 8 waves / SIMD
    uint32_t wg64_wide = 0xA;       // RT_WG64_WIDE: bit log2(N) (3: N >= 8): one-wave workgroups also
                                    // for a rank of N's batch with a wide section
    uint32_t plan_delay = 0;        // rt_debug_set_plan_delay: k_hf_plan idles this many 100 MHz ticks first (tests)
    uint32_t hf_follow = 1;         // RT_HF_FOLLOW: re-plan the heavy-first order on every frame whose
                                    // camera moved (0: every kHfPeriod-th frame only)
    bool octant_words = false;      // 8 ray-octant copies of the empty-run words (else one L-inf word)
    bool box_words = false;         // 24 box-run word copies: AUTO's empty runs (kVarSkipRun)
    // camera-space x / y tables of the current frame shape (prepare_ndc)
    float *d_ndc = nullptr;
    size_t ndc_cap = 0;
    std::vector<float> ndc_key;
    rtk::TabParams tab = {};            // the tables' parameters while tab_dirty (flush_tables)
    bool tab_dirty = false;
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
    // Ordering of the scene's launches across streams and against host rewrites of its state: ev_last
    // completes when the scene's last launch has.  The product launches carry it as the dispatch's own
    // stop event (hipExtLaunchKernelGGL: a free one of ev_done[], or the timed launch's kt1), so no marker packet sits
    // between two frames on a stream -- a marker after each launch cost 2 % of the bench step and of
    // config 5's (profiles/r05u_marker_ab.json); the other launch paths record ev_own after theirs.
    rtk::EvRef ev_own, ev_last;
    rtk::EvRef ev_done[4];              // stop events, each re-recorded only when no scene refers to it
    rtk::EvRef ev_prev;                 // RT_KERNEL_FLAG_OVERLAP: the launch ev_last's launch overlaps (else null)
    hipStream_t prev_stream = nullptr;  // ... and its stream
    bool ev_recorded = false;
    // render-kernel-only timing: event pair around the render kernel(s) of each launch (not the
    // heavy-first planning kernels), a ring of the last kTimeRing launches (rt_kernel_times)
    rtk::HfCtx *hf_last = nullptr;       // the context of the last hf_prepare (launch_plans)
    hipStream_t plan_st = nullptr;       // k_hf_plan after a measured frame, beside the next frame
    hipEvent_t kt0[kTimeRing] = {};
    rtk::EvRef kt1[kTimeRing];          // a timed launch's stop event (also its ev_last)
    // The library's own events order device work (a scene's frames on different streams; the side-stream
    // fork / join) or time kernels (kt0 / kt1); none of them hands memory to the host.  A default event
    // record ends in a system-scope release (L2 write-back and invalidate), which the next frame pays in
    // refetches; device scope is enough for these.  The host-visible band / tile events keep the default.
    unsigned ev_time_flags = hipEventDisableSystemFence;                         // kt0 / kt1
    unsigned ev_order_flags = hipEventDisableTiming | hipEventReleaseToDevice;   // ev_own, ev_fork, ev_join
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

namespace rtk {

// rt_plan.hip: one context's device state sized for `blocks` (frees the old)
int hf_alloc(HfCtx *c, uint64_t blocks);
// the first context's capacity at rt_scene_create: a 1080p x 4 frame's 32,640 blocks
constexpr uint64_t kHfPreBlocks = 32768;
// rt_plan.hip: the heavy-first / wide-section state of this launch shape (fills P.hf_*, P.wh_*)
// batch: 0 for a single-frame launch, else an identity of the batch (its scenes and frame count)
int hf_prepare(rt_scene *s, KParams& P, uint64_t blocks, int var, bool front, hipStream_t st, uint64_t batch = 0,
               uint64_t cam_sig = 0);
// What hf_prepare would find for this launch, without side effects: whether the shape's context exists
// (no allocation, no eviction) and whether this frame would be measured (RT_KERNEL_FLAG_OVERLAP)
// measure_ok: a measured frame of this shape may still overlap (its plan runs after every frame in
// flight, launch_plans; a measured frame adopts a pending plan first): not the shape's first two frames
struct HfPeek { bool found, measure, measure_ok; };
HfPeek hf_peek(const rt_scene *s, const KParams& P, uint64_t blocks, int var, uint64_t batch, uint64_t cam_sig);
// The plan kernel(s) after a measured frame on its stream (k_hf_plan; two passes after a shape's first
// measured frame, see launch_plans)
int launch_plans(rt_scene *s, const KParams& P, uint64_t blocks, hipStream_t st, bool pipelined);
// The camera of a frame as one 64-bit signature (FNV-1a over the rotation, origin and fov bits)
uint64_t cam_signature(const KParams& P, uint64_t h = 0xcbf29ce484222325ull);

} // namespace rtk
