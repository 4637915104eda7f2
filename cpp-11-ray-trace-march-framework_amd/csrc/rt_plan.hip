// rt_plan.hip -- the heavy-first order and the wide section's item list:
// k_hf_plan, which turns a measured frame's per-wave costs into the next frames' plan, and the host
// side that keeps one plan context per launch shape (hf_prepare).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>
#include <cstring>

#include "rt_scene.h"
#include "rt_walk.h"

namespace rtk {
namespace {

// Heavy-first planning, after a measured frame's render kernel on its stream: per block the cost
// of its slowest wave; blocks above max(hf_floor, last max >> hf_shift (RT_HF_SHIFT)) are listed for the next
// frames -- above last max >> 1 at the front of the front section, the rest from its back -- and
// marked so the natural order skips them.  Nothing is listed when the last measurement showed no
// tail (its slowest block well under the frame's estimated span).  Each thread takes kHfPlanPer
// blocks (kWG apart, so the cost loads stay coalesced); each workgroup reduces its maximum and sum
// and reserves its list slots with ONE atomic per level (the render waves themselves touch no
// atomics: thousands of same-address atomics from waves cost milliseconds, measured).  The plan's
// time is those same-address atomics: one block per thread (1,013 workgroups for the batched
// bench pair) took 26.6 us per plan, which a moving camera pays every frame.
// pos16 (RT_HF_POS16, 0: off): a block is heavy when its cost exceeds pos16 / 16 of the span left
// after its natural start (b / nblocks of the estimated span, sum of wave costs / kHfSlots) -- a
// late block needs less to make the tail than an early one -- and last max >> kHfPosShift.
constexpr uint32_t kHfPosShift = 4;
// delay (rt_debug_set_plan_delay, tests only; 0 in the product): the kernel first idles that many
// 100 MHz ticks, so a frame that may read the plan's buffers while it runs always finds it mid-write
// (tests/test_gpu_overlap.py, the HfCtx::fence ordering).
__global__ void __launch_bounds__(kWG) k_hf_plan(KParams P, uint32_t nblocks, uint32_t shift, uint32_t pos16,
                                                 uint32_t delay)
{
    if (delay)
    {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < delay) __builtin_amdgcn_s_sleep(64);
    }
    __shared__ uint32_t s_max, s_hi, s_lo, s_w, s_l, s_bhi, s_blo, s_bw, s_bl, s_last;
    __shared__ unsigned long long s_sum;
    if (threadIdx.x == 0u)
    {
        s_max = s_hi = s_lo = s_w = s_l = 0u;
        s_sum = 0ull;
    }
    __syncthreads();
    const HfPlan last = *P.hf_plan_in;
    const bool tail = uint64_t(last.maxc) * kHfSlots * 16u > uint64_t(kHfTail) * (last.sum << 4);
    const uint32_t thr = max(P.hf_floor, last.maxc >> (pos16 ? kHfPosShift : shift));
    const uint64_t span = (last.sum << 4) / kHfSlots;
    const uint32_t b0 = blockIdx.x * (kWG * kHfPlanPer) + threadIdx.x;
    uint32_t tmax = 0u, wmasks = 0u, lmasks = 0u, heavy = 0u, hi = 0u;
    unsigned long long tsum = 0ull;
    uint32_t rank[kHfPlanPer], wrank[kHfPlanPer], lrank[kHfPlanPer];
#pragma unroll
    for (uint32_t j = 0; j < kHfPlanPer; j++)
    {
        const uint32_t b = b0 + j * kWG;
        uint32_t cost = 0u, sum = 0u, wmask = 0u, lmask = 0u;
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
                // the LDS tier (kVarLdsSplit): the next heaviest items, one workgroup each
                if (P.wh_lds)
                {
                    const uint32_t lt = max(P.wh_floor, uint32_t(min<uint64_t>(span * P.wh_beta16 / 16u, 0xFFFFFFFFull)));
                    lmask = (uint32_t(c.x > lt) | (uint32_t(c.y > lt) << 1) | (uint32_t(c.z > lt) << 2) |
                             (uint32_t(c.w > lt) << 3)) & ~wmask;
                }
            }
            if (P.wh_on && !P.wh_refresh && P.hf_ver)
            {
                // sticky: the current plan's items stay listed in their tier (mark = the plan version,
                // bit 31: the LDS tier)
                const uint4 m = reinterpret_cast<const uint4 *>(P.wh_mark_in)[b];
                const uint32_t v = P.hf_ver, vl = P.hf_ver | 0x80000000u;
                wmask |= uint32_t(m.x == v) | (uint32_t(m.y == v) << 1) | (uint32_t(m.z == v) << 2) | (uint32_t(m.w == v) << 3);
                lmask |= uint32_t(m.x == vl) | (uint32_t(m.y == vl) << 1) | (uint32_t(m.z == vl) << 2) |
                         (uint32_t(m.w == vl) << 3);
                wmask &= ~lmask;
            }
            // the heavy-first order ranks a block by its slowest wave left in the lane section
            const uint32_t wm = wmask | lmask;
            cost = max(max((wm & 1u) ? 0u : c.x, (wm & 2u) ? 0u : c.y), max((wm & 4u) ? 0u : c.z, (wm & 8u) ? 0u : c.w));
        }
        uint32_t tb = thr;
        if (pos16 && b < nblocks)
            tb = max(tb, uint32_t(min<uint64_t>(span * pos16 / 16u * (nblocks - b) / nblocks, 0xFFFFFFFFull)));
        const bool hv = P.hf_front && tail && cost > tb;
        const bool h1 = hv && cost > (last.maxc >> 1);
        tmax = max(tmax, cost);
        tsum += sum;
        rank[j] = hv ? atomicAdd(h1 ? &s_hi : &s_lo, 1u) : 0u;
        wrank[j] = wmask ? atomicAdd(&s_w, uint32_t(__popc(wmask))) : 0u;
        lrank[j] = lmask ? atomicAdd(&s_l, uint32_t(__popc(lmask))) : 0u;
        heavy |= uint32_t(hv) << j;
        hi |= uint32_t(h1) << j;
        wmasks |= wmask << (4u * j);
        lmasks |= lmask << (4u * j);
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
        s_bl = s_l ? atomicAdd(&P.hf_plan_out->cnt_l, s_l) : 0u;
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
        const uint32_t wmask = (wmasks >> (4u * j)) & 15u, lmask = (lmasks >> (4u * j)) & 15u;
        uint32_t wr = wrank[j], lr = lrank[j];
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
            else if (lmask & (1u << k))
            {
                const uint32_t item = b * kWavesPerWG + k;
                const uint32_t r = s_bl + lr++;
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
        {
            P.wh_host_cnt[0] = P.wh_g * min(vp->cnt_w, kWhMax);     // the G-lane tier's waves
            P.wh_host_cnt[1] = min(vp->cnt_l, kWhMax);              // the LDS tier's items (workgroups)
        }
        *P.hf_ticket = 0u;
    }
}

} // namespace

// k_hf_plan after a measured frame.  A plan lists a block only against the PREVIOUS measurement (its
// maximum and span decide the thresholds), so the first measured frame of a launch shape listed
// nothing and its second frame ran in the natural order too (killeroo 1080p x 4: 0.62 ms against 0.36
// in steady state, BENCH_r04 first_frame_ms).  After that frame a second pass ranks the same wave
// costs against the first pass's maximum and span: the second frame already runs heavy-first.  The
// passes alternate the plan / list / mark buffers by version parity, as consecutive frames do
// (hf_prepare bumps the version by 2).
// Later plans (a current version exists) run on the scene's plan stream, forked after the measured
// frame: the next frame keeps the current plan and does not wait for this one (on the launch stream
// the plan took ~20 us per scene after every 16th frame: the 16-step spikes of a frame series,
// profiles/r05k_frame_series*.json).  hf_prepare adopts it (a stream wait on its event) at the second
// frame after, or at the next measured frame (which reuses the plan's buffers).  Inside a stream
// capture every plan stays on the launch stream.
int launch_plans(rt_scene *s, const KParams& P, uint64_t blocks, hipStream_t st, bool pipelined)
{
    const dim3 grid(uint32_t((blocks + kWG * kHfPlanPer - 1) / (kWG * kHfPlanPer))), wg(kWG);
    HfCtx *c = s->hf_last;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    // two passes after a shape's first measurement (version 0): the second pass ranks against the first's
    const bool twice = P.hf_ver == 0u;
    // the position-aware threshold for single-frame launches; a batched launch keeps max >> shift
    // (the bench pair's batched step: 0.5396 vs 0.5318 ms with it, scenes 4 / 5 in their own launches
    // 0.2486 / 0.4518 vs 0.252 / 0.46: profiles/r05ar_hf_pos_sweep.json), and so does a pipelined one
    // (RT_KERNEL_FLAG_OVERLAP: a late block's tail runs under the next launch; the bench pair as
    // overlapped frames 0.5074 vs 0.5121 ms per step, profiles/r06_pipelined_plan_ab.json)
    const uint32_t pos16 = ((c && c->key[4] != 0u) || pipelined) ? 0u : s->hf_pos16;
    // the second pass: the first pass's outputs are its inputs, written into the buffers of the version
    // before (the two passes alternate them by parity, as consecutive frames do)
    KParams Q = P;
    if (twice)
    {
        Q.hf_ver = P.hf_ver + 1u;
        Q.hf_plan_in = P.hf_plan_out;
        Q.hf_plan_out = const_cast<HfPlan *>(P.hf_plan_in);
        Q.hf_list_in = P.hf_list_out;
        Q.hf_list_out = const_cast<uint32_t *>(P.hf_list_in);
        Q.hf_mark_in = P.hf_mark_out;
        Q.hf_mark_out = const_cast<uint32_t *>(P.hf_mark_in);
        if (P.wh_on)
        {
            Q.wh_list_in = P.wh_list_out;
            Q.wh_list_out = const_cast<uint32_t *>(P.wh_list_in);
            Q.wh_mark_in = P.wh_mark_out;
            Q.wh_mark_out = const_cast<uint32_t *>(P.wh_mark_in);
        }
    }
    if (c && cap == hipStreamCaptureStatusNone)
    {
        if (!s->plan_st)
        {
            RT_HIP(hipStreamCreateWithFlags(&s->plan_st, hipStreamNonBlocking));
        }
        if (!c->pend_ev) RT_HIP(hipEventCreateWithFlags(&c->pend_ev, s->ev_order_flags));
        // forked after the measured launch's own completion event (ev_last, the dispatch's stop
        // event): a marker packet on the launch stream here put ~13 us between that launch and the
        // next one (rocprofv3 kernel trace of a frame series, profiles/r05t_series_kernel_trace.csv)
        RT_HIP(hipStreamWaitEvent(s->plan_st, s->ev_last->ev, 0));
        // a measured frame that overlapped its predecessor (RT_KERNEL_FLAG_OVERLAP): the plan rewrites
        // the buffers of the version before this frame's, which that predecessor may read
        if (s->ev_prev) RT_HIP(hipStreamWaitEvent(s->plan_st, s->ev_prev->ev, 0));
        RT_HIP(hipMemsetAsync(P.hf_plan_out, 0, sizeof(HfPlan), s->plan_st));
        hipLaunchKernelGGL(k_hf_plan, grid, wg, 0, s->plan_st, P, uint32_t(blocks), s->hf_shift, pos16, s->plan_delay);
        // (a shape's first plans too: the first frame's time to the frame no longer includes them; its
        // second frame, measured, adopts them)
        if (twice)
        {
            RT_HIP(hipMemsetAsync(Q.hf_plan_out, 0, sizeof(HfPlan), s->plan_st));
            hipLaunchKernelGGL(k_hf_plan, grid, wg, 0, s->plan_st, Q, uint32_t(blocks), s->hf_shift, pos16, s->plan_delay);
        }
        RT_HIP(hipEventRecord(c->pend_ev, s->plan_st));
        c->pend = P.hf_ver + (twice ? 2u : 1u);
        c->pend_age = 0;
        RT_HIP(hipGetLastError());
        return RT_OK;
    }
    // inside a stream capture (no wait on an outside event): on the launch stream
    RT_HIP(hipMemsetAsync(P.hf_plan_out, 0, sizeof(HfPlan), st));
    hipLaunchKernelGGL(k_hf_plan, grid, wg, 0, st, P, uint32_t(blocks), s->hf_shift, pos16, s->plan_delay);
    if (twice)
    {
        RT_HIP(hipMemsetAsync(Q.hf_plan_out, 0, sizeof(HfPlan), st));
        hipLaunchKernelGGL(k_hf_plan, grid, wg, 0, st, Q, uint32_t(blocks), s->hf_shift, pos16, s->plan_delay);
    }
    if (c) c->ver = P.hf_ver + (twice ? 2u : 1u);
    RT_HIP(hipGetLastError());
    // plans on the launch stream are part of the scene's last launch: a launch on another stream orders
    // after them, not only after the render (ev_last was the render's own stop event).  Plans run here
    // only inside a stream capture, where nothing overlaps (launch_render / launch_batch), so no ev_prev
    // refers to ev_own here.
    RT_HIP(hipEventRecord(s->ev_own->ev, st));
    s->ev_last = s->ev_own;
    return RT_OK;
}

constexpr uint32_t kWhRefresh = 128;        // frames between refresh frames (a multiple of kHfPeriod)


// The camera of a frame as one 64-bit signature (FNV-1a over the bits of the rotation, the origin
// and the field of view): heavy-first plans are re-measured when it changes between frames.
uint64_t cam_signature(const KParams& P, uint64_t h)
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
// The key of a launch shape's heavy-first context
void hf_key(const KParams& P, uint64_t blocks, int var, uint64_t batch, uint64_t key[5])
{
    key[0] = (blocks << 16) | (uint64_t(P.spp) << 1) | 1u;
    key[1] = (uint64_t(P.rx0) << 32) | P.ry0;
    key[2] = (uint64_t(P.rw) << 32) | P.rh;
    key[3] = (uint64_t(P.rank) << 40) | (uint64_t(P.nranks) << 20) | uint64_t(uint32_t(var) >> 12);
    key[4] = batch;
}

// Whether a frame of this context is measured.  pend: the plan pending after this frame's adoption (see
// hf_prepare).  A moved camera re-plans (RT_HF_FOLLOW) only when no plan is pending: a measured frame
// must wait for the pending plan, which reads the cost words it would write, so measuring every moved
// frame put each frame after the previous frame's plan -- no two frames of a moving camera overlapped,
// and every step paid the plan's latency.  A moving camera is measured every other frame instead, and
// frame i + 2 adopts frame i's plan.
bool measures(const rt_scene *s, const HfCtx& c, uint64_t cam_sig, uint32_t pend)
{
    return c.frames < 2u || c.frames % kHfPeriod == 0u || (s->hf_follow && cam_sig != c.cam && pend == 0u);
}

// The plan still pending after a frame's adoption step (hf_prepare: the second frame after a plan adopts
// it; a measured frame does too, but only a frame with no plan pending is measured for a moved camera)
uint32_t pend_after_adoption(const HfCtx& c)
{
    return (c.pend && c.pend_age >= 1u) ? 0u : c.pend;
}

HfPeek hf_peek(const rt_scene *s, const KParams& P, uint64_t blocks, int var, uint64_t batch, uint64_t cam_sig)
{
    uint64_t key[5];
    hf_key(P, blocks, var, batch, key);
    for (const HfCtx& h : s->hf)
        if (std::memcmp(h.key, key, sizeof(key)) == 0)
            // a measured frame adopts any pending plan first (waiting for it on its stream; later frames
            // wait for it as the fence), so it may overlap once the shape's first two frames (whose plans
            // run on the launch stream) have passed
            return HfPeek{ true, measures(s, h, cam_sig, pend_after_adoption(h)), h.frames >= 2u };
    return HfPeek{ false, true, false };
}

// ONE device allocation per context (a new launch shape's first frame waits for the host's
// allocation calls: seven of them took ~0.1 ms, profiles/r05i_first_frame_probe.json), the cleared
// arrays first so one memset clears them: plans [2], ticket (+ pad to 16 B), marks [2][cap],
// wh_marks [2][4 cap]; then cost [4 cap], lists [2][kHfFrontMax], wh_lists [2][2][kWhMax] ([version][tier]).  rt_scene_create sizes the first context for kHfPreBlocks, so a first frame up
// to that shape allocates nothing.
int hf_alloc(HfCtx *c, uint64_t blocks)
{
    c->cap_blocks = 0;
    if (c->mem) RT_HIP(hipFree(c->mem));
    c->mem = nullptr;
    const size_t head = sizeof(HfPlan) * 2 + 16u;
    const size_t cleared = head + sizeof(uint32_t) * (2u + 2u * kWavesPerWG) * blocks;
    const size_t bytes = cleared + sizeof(uint32_t) * (kWavesPerWG * blocks + 2u * kHfFrontMax + 4u * kWhMax);
    RT_HIP(hipMalloc(&c->mem, bytes));
    char *m = static_cast<char *>(c->mem);
    c->plans = reinterpret_cast<HfPlan *>(m);
    c->ticket = reinterpret_cast<uint32_t *>(m + sizeof(HfPlan) * 2);
    c->marks = reinterpret_cast<uint32_t *>(m + head);
    c->wh_marks = c->marks + 2u * blocks;
    c->cost = c->wh_marks + 2u * kWavesPerWG * blocks;
    c->lists = c->cost + kWavesPerWG * blocks;
    c->wh_lists = c->lists + 2u * kHfFrontMax;
    c->cleared_bytes = cleared;
    c->cap_blocks = uint32_t(blocks);
    return RT_OK;
}

int hf_prepare(rt_scene *s, KParams& P, uint64_t blocks, int var, bool front, hipStream_t st, uint64_t batch,
               uint64_t cam_sig)
{
    if (!batch) cam_sig = cam_signature(P);
    uint64_t key[5];
    hf_key(P, blocks, var, batch, key);
    HfCtx *c = nullptr;
    for (HfCtx& h : s->hf)
        if (std::memcmp(h.key, key, sizeof(h.key)) == 0) c = &h;
    if (!c)
    {
        c = &s->hf[0];
        for (HfCtx& h : s->hf)
            if (h.used < c->used) c = &h;
        if (c->used) s->hf_evictions++;
        if (c->pend)
        {
            RT_HIP(hipEventSynchronize(c->pend_ev));      // its plan still writes these buffers
            c->pend = 0u;
        }
        if (c->fence)
        {
            RT_HIP(hipEventSynchronize(c->fence_ev));
            c->fence = false;
        }
        // invalidated first: if an allocation below fails, no later launch may match the old
        // shape and read freed (null) state arrays
        std::memset(c->key, 0, sizeof(c->key));
        c->frames = 0;
        c->ver = 0;
        if (blocks > c->cap_blocks || !c->mem)
            if (int rc = hf_alloc(c, blocks)) return rc;
        RT_HIP(hipMemsetAsync(c->mem, 0, c->cleared_bytes, st));
        c->wh_cnt = s->h_wh_cnt + 2 * (c - s->hf);     // the scene's mapped counters (rt_scene_create)
        c->wh_cnt_dev = s->d_wh_cnt + 2 * (c - s->hf);
        c->wh_cnt[0] = c->wh_cnt[1] = 0u;
        c->nblocks = uint32_t(blocks);
        // front: 1 / hf_front_div of the blocks (an eighth), capped at hf_front_max (1024) -- or 1 / 128 of
        // a larger launch's blocks -- at most kHfFrontMax, a multiple of the XCD count so the natural
        // section keeps its block -> XCD assignment
        const uint32_t fr = std::max(std::min(s->hf_front_max, uint32_t(blocks / std::max(s->hf_front_div, 1u))),
                                     uint32_t(blocks / 128u));
        c->front = front ? std::min(fr, kHfFrontMax) & ~(kXcds - 1u) : 0u;
        std::memcpy(c->key, key, sizeof(c->key));       // valid only now
    }
    c->used = ++s->hf_clock;
    s->hf_last = c;
    // measured: the first two frames (the first plan has no earlier maximum to test a tail
    // against, so it lists nothing) and then every kHfPeriod-th
    // ... and a frame whose camera differs from the previous frame's, when no plan is pending after its
    // adoption step: a moving camera's heavy blocks move with the view, so the plan comes from a view
    // two frames old instead of one up to kHfPeriod frames old (measures)
    P.hf_measure = measures(s, *c, cam_sig, pend_after_adoption(*c)) ? 1u : 0u;
    if (c->fence || c->pend)
    {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        RT_HIP(hipStreamIsCapturing(st, &cap));
        // the adopted plan's fence (see HfCtx::fence); a capture cannot wait on an outside event, so
        // the host waits for it there
        if (c->fence)
        {
            if (hipEventQuery(c->fence_ev) == hipSuccess)
                c->fence = false;
            else if (cap != hipStreamCaptureStatusNone)
            {
                RT_HIP(hipEventSynchronize(c->fence_ev));
                c->fence = false;
            }
            else if (st != c->fence_st)
                RT_HIP(hipStreamWaitEvent(st, c->fence_ev, 0));
        }
        // a plan on the plan stream (launch_plans): adopted by the second frame after it and by a
        // measured frame; inside a stream capture (no wait on an outside event) the current plan
        // stays and nothing is measured
        if (!c->pend)
            ;
        else if (cap != hipStreamCaptureStatusNone)
            P.hf_measure = 0u;
        else if (P.hf_measure || c->pend_age >= 1u)
        {
            // (a plan that has finished needs no wait packet: a stream wait costs the launch stream a
            // few us of idle chip even on a completed event).  One still running becomes the fence
            // of the frames after this one, which may run on another stream beside it.
            if (hipEventQuery(c->pend_ev) != hipSuccess)
            {
                RT_HIP(hipStreamWaitEvent(st, c->pend_ev, 0));
                std::swap(c->pend_ev, c->fence_ev);     // launch_plans records the next plan elsewhere
#ifndef RT_DEBUG_NO_PLAN_FENCE   // (tools/build_variant.sh: the race of DESIGN.md §4.21 made visible)
                c->fence = true;
                c->fence_st = st;
#endif
            }
            c->ver = c->pend;
            c->pend = 0u;
        }
        else
            c->pend_age++;
    }
    const uint32_t v = c->ver;
    P.hf_front = c->front;
    P.hf_ver = v;
    c->cam = cam_sig;
    c->frames++;
    // with the LDS tier the lone heavy waves have left the lane section, and its tail is the lane waves
    // of 40-100 us that the natural order starts late: the front takes them from half the floor (a
    // rank of 8's one-stream step 0.110 -> 0.096 ms at 50 k cycles, profiles/r06_lds_tier_ab.json)
    P.hf_floor = (var & kVarLdsSplit) ? s->hf_floor / 2u : s->hf_floor;
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
        // plan or two old: the count is read without waiting; the section is persistent over the
        // device-side list, which may already be longer).  wh_wgs == 0 (no list seen yet, or a
        // refresh frame): no section, and the lane kernel renders every item itself.
        // Refresh: every kWhRefresh-th frame renders every item one lane per sample, so the next
        // plan re-ranks all items on lane-mode costs (the wide set is otherwise sticky).
        // The LDS tier (kVarLdsSplit): its items one 256-lane workgroup each (k_hf_plan counts its waves).
        P.wh_g = P.spp <= 4u ? 16u : 4u;
        P.wh_lds = (var & kVarLdsSplit) ? 1u : 0u;
        P.wh_beta16 = s->wh_beta16;
        // (k_hf_plan writes the counts: the G-lane tier's waves, the LDS tier's items)
        const uint32_t units = c->wh_cnt[0], litems = P.wh_lds ? c->wh_cnt[1] : 0u;
        P.wh_on = 1u;
        P.wh_refresh = (c->frames - 1u) % kWhRefresh == 0u;       // frames counts this one
        // each tier gets workgroups of its own, at least one once anything is listed (a tier's list may
        // have grown since the counts the host saw: its loop is persistent): the G-lane tier the first
        // wh_wgs_g, the LDS tier the rest, one item per workgroup at a time, both from the launch's start
        P.wh_wgs = P.wh_wgs_g = 0u;
        if (!P.wh_refresh && (units || litems))
        {
            P.wh_wgs_g = std::max(1u, (units + kWavesPerWG - 1u) / kWavesPerWG);
            P.wh_wgs = P.wh_wgs_g + (P.wh_lds ? std::max(1u, litems) : 0u);
        }
        P.wh_floor = s->wh_floor;
        // a rank of 2 of a batched step lists more (its span estimate includes the other frames'
        // work); one scene's own rank-of-2 launch measured 25 % slower with it
        // (profiles/r03o_shard_scaling_bench.json), so one scene's own launches keep wh_alpha16 (32/16),
        // and a rank of 4-7 of a batched step one notch lower (rank of 4, measured in
        // profiles/r03ad_alpha_n4_n8.json: 0.182 ms at 28/16 vs 0.191 at 32/16, 0.219 at 36/16).  A
        // batched rank of >= 8 lists less since round 6 (wh_alpha16_n8 40/16: the bench pair's
        // overlapped step 0.0818-0.0839 vs 0.0855-0.0868 ms at 32/16, one stream 0.096 vs 0.099; 48-64
        // unstable; killeroo's own rank of 8 mixed, so it keeps 32: profiles/r06_lds_tier_ab.json r06l, r06m)
        P.wh_alpha16 = batch == 0u      ? s->wh_alpha16
                       : P.nranks == 2u ? s->wh_alpha16_n2
                       : P.nranks < 8u  ? s->wh_alpha16_n4
                                        : s->wh_alpha16_n8;
        P.wh_mark_in = c->wh_marks + size_t(v & 1u) * kWavesPerWG * c->cap_blocks;
        P.wh_mark_out = c->wh_marks + size_t((v + 1u) & 1u) * kWavesPerWG * c->cap_blocks;
        P.wh_list_in = c->wh_lists + size_t(v & 1u) * 2u * kWhMax;
        P.wh_list_out = c->wh_lists + size_t((v + 1u) & 1u) * 2u * kWhMax;
        P.wh_host_cnt = c->wh_cnt_dev;
    }
    return RT_OK;
}

} // namespace rtk
