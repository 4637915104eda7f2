// rt_kernels.hip -- the render kernels of librt_tracer.so for gfx950 (MI355X).
//
// One launch renders a whole frame (or one rank's shard): a workgroup of 256 lanes owns
// 256/spp pixels of a 16x16 pixel tile in Morton order, one lane per sample, so a pixel's
// samples sit in adjacent lanes and a wave covers a compact 2^k x 2^k pixel block (coherent
// DDA walks).  Each lane runs the reference's per-sample path (GenerateRay -> Grid::Intersect
// -> IntersectRayTri -> shading, renderer.cpp:88-122); the pixel's samples are then summed IN
// SAMPLE ORDER across lanes (renderer.cpp:87-122, hazard H10), averaged, gamma'd and packed
// (renderer.cpp:124-133).
//
// The per-sample code lives in rt_walk.h; the heavy-first planner kernel in rt_plan.hip; the
// host side (scene tables, launches, the C ABI) in rt_tracer.hip.
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

#include <cstddef>
#include <cstdint>

#include "rt_walk.h"

namespace rtk {
namespace {

// XCD-aware block order (kVarXcdBands).  The dispatcher deals workgroups round-robin to the 8
// XCDs (block b runs on XCD b % 8), so consecutive blocks -- the 4 workgroups of one tile and
// the tiles of one row -- land on 8 different L2s, and every XCD's L2 caches the whole visible
// scene.  Remapped, XCD x takes turns of `chunk` consecutive blocks (one tile row): rows x,
// x + 8, x + 16, ... -- compact rows for its L2, and the frame's cost still spread over all
// XCDs.  chunk 0: one contiguous band per XCD (measured: load imbalance, up to 58 % slower).
// A bijection on [0, nblocks) for any grid size (the tail past whole 8-turn rounds keeps its
// order); on a device with another XCD count only the locality changes.
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

// The launch's block -> block-of-work map.  With the heavy-first order on, blocks [0, hf_front)
// take the blocks listed by the previous frame (in the order their heavy waves finished) and the
// rest walk the natural (XCD-banded) order, skipping the listed blocks.  Returns false when this
// block has nothing to do.  The marks read here are never written by this launch (the next
// frame's marks live in the other buffer), so every wave of a block decides alike.
// lead: the first lane of launch block 0's first wave (unused since round 5: launch_plans clears the next plan).
template <int VAR>
__device__ __forceinline__ bool block_of_launch(const KParams& P, uint32_t& b, uint32_t bid, uint32_t nblk,
                                                bool lead)
{
    // (the next plan's counters are cleared by launch_plans right before k_hf_plan, not here: a
    // measured frame may run beside a frame that still reads the buffer it would clear)
    (void)lead;
    if (P.hf_front)
    {
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
                                         0.0f, 0.0f, kRecRawBox);
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
// One wave's share of one listed item (wide_section): list entry li, the e-th wave of the section
// (its clock record), the item's wave q.
template <bool BATCH, uint32_t G, bool CLK>
__device__ __forceinline__ void wide_item(const KParams& P, uint32_t li, uint32_t q, uint32_t e)
{
    const uint32_t ipt = P.wg_per_tile * kWavesPerWG;              // items per tile
    uint32_t item = __builtin_amdgcn_readfirstlane(P.wh_list_in[li]);
    uint32_t off = 0u;
    if constexpr (BATCH)
    {
        const KBatch& B = late_batch();
        const uint32_t f = batch_frame(B, item / kWavesPerWG);
        item -= B.base[f] * kWavesPerWG;                          // the frame's own item index
        off = uint32_t(offsetof(KBatch, p)) + f * uint32_t(sizeof(KParams));
    }
    const uint32_t kseq = item / ipt;
    const uint32_t slot0 = (item - kseq * ipt) * 64u + q * (64u / G);
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
    wide_samples<kVarWide>(Q, k, slot0, G);
    if constexpr (CLK && BATCH)
    {
        // kVarWaveClock: one record per (listed item, wave) of the section, after the batch's lane
        // items: word 2's low bits = 0x80000000 | list entry, word 3's = the launch-wide item
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const KBatch& B = late_batch();
        const KParams& Q0 = late_params(P, uint32_t(offsetof(KBatch, p)));
        if ((threadIdx.x & 63u) == 0u)
            store_wave_clock(Q0.wave_clk, B.base[B.nframes] * kWavesPerWG + e, t0, t1, r0, r1, 0x80000000u | li,
                             __builtin_amdgcn_readfirstlane(Q0.wh_list_in[li]));
    }
}

// w: this wave's index in the section (4 per 256-lane workgroup, or one per one-wave workgroup).
template <bool BATCH, uint32_t G, bool CLK = false>
__device__ __forceinline__ void wide_section(const KParams& P, uint32_t w)
{
    const uint32_t n = P.hf_ver ? min(P.hf_plan_in->cnt_w, kWhMax) : 0u;
    const uint32_t nw = P.wh_wgs * kWavesPerWG;
    for (uint32_t e = w; e < n * G; e += nw) wide_item<BATCH, G, CLK>(P, e / G, e % G, e);
}

// The wide section's LDS tier (kVarLdsSplit): ONE listed item per 256-lane workgroup.
// Its four waves each hold the item's 64 sample slots one lane per sample -- the lane kernel's own
// process_item, same walk (approach, lock-step, box runs, wave-uniform scalar lists) -- so their walk
// states are identical, and every cell list the walk tests is split between them: wave w tests
// records kb + w, kb + w + 4, ... (test_cell), and the four local first minima are reduced through
// LDS to the lexicographic minimum (t, list position), the reference's first minimum
// (grid.cpp:243-267, H8), which every wave then holds: the walks stay identical.  A lone heavy wave's
// ~1,000-record chain becomes four chains of ~250 on four SIMDs; the walk is
// repeated four times (against 16 in the G-lane tier).  Wave 0 stores the pixels.
// li: the item's entry in the LDS tier's list (the list's second half, wh_list_in + kWhMax)
template <bool BATCH, bool CLK = false>
__device__ __forceinline__ void wide_item_lds(const KParams& P, uint32_t li)
{
    uint32_t item = __builtin_amdgcn_readfirstlane(P.wh_list_in[kWhMax + li]);
    uint32_t off = 0u;
    if constexpr (BATCH)
    {
        const KBatch& B = late_batch();
        const uint32_t f = batch_frame(B, item / kWavesPerWG);
        item -= B.base[f] * kWavesPerWG;                          // the frame's own item index
        off = uint32_t(offsetof(KBatch, p)) + f * uint32_t(sizeof(KParams));
    }
    uint64_t r0 = 0, t0 = 0;
    if constexpr (CLK && BATCH)
    {
        r0 = __builtin_amdgcn_s_memrealtime();
        t0 = __builtin_amdgcn_s_memtime();
    }
    process_item<RT_TRI_MOLLER_TRUMBORE, kVarAuto | kVarLdsSplit>(late_params(P, off), item, off);
    // every wave has read the last reduction before any wave starts the next item's first
    lds_barrier();
    if constexpr (CLK && BATCH)
    {
        // one record per listed item (wave 0's clocks), after the batch's lane items, as wide_item's
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const KBatch& B = late_batch();
        const KParams& Q0 = late_params(P, uint32_t(offsetof(KBatch, p)));
        if (threadIdx.x == 0u)
            store_wave_clock(Q0.wave_clk, B.base[B.nframes] * kWavesPerWG + kWhMax * 16u + li, t0, t1, r0, r1,
                             0x80000000u | (kWhMax + li), __builtin_amdgcn_readfirstlane(Q0.wh_list_in[kWhMax + li]));
    }
}

// A section with both tiers (kVarLdsSplit; 256-lane workgroups): its first wh_wgs_g workgroups take the
// G-lane tier's items (the heaviest) wave by wave, the others the LDS tier's, workgroup by workgroup, so
// both start with the launch (each loop persistent over its list).  wg: this workgroup's index in the
// section.
template <bool BATCH, uint32_t G, bool CLK = false>
__device__ __forceinline__ void wide_section_lds(const KParams& P, uint32_t wg)
{
    const uint32_t ng = P.wh_wgs_g;
    if (wg < ng)
    {
        const uint32_t n = P.hf_ver ? min(P.hf_plan_in->cnt_w, kWhMax) : 0u;
        const uint32_t nw = ng * kWavesPerWG;
        for (uint32_t e = wg * kWavesPerWG + (threadIdx.x >> 6); e < n * G; e += nw) wide_item<BATCH, G, CLK>(P, e / G, e % G, e);
        return;
    }
    const uint32_t n = P.hf_ver ? min(P.hf_plan_in->cnt_l, kWhMax) : 0u;
    const uint32_t nwg = P.wh_wgs - ng;
    for (uint32_t li = wg - ng; li < n; li += nwg) wide_item_lds<BATCH, CLK>(P, li);
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

// the same section with the LDS tier after it (kVarLdsSplit: one listed item per workgroup), held to 7
// waves / SIMD (the split walk: 80 VGPRs unbounded)
template <uint32_t G>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(7, 8))) k_render_wh_lds(KParams P)
{
    wide_section_lds<false, G>(P, blockIdx.x);
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
__device__ __forceinline__ void batch_body(const KBatch& B)
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
            if constexpr ((VAR & kVarLdsSplit) != 0)
                wide_section_lds<true, (VAR & kVarWideG4) ? 4u : 16u, (VAR & kVarWaveClock) != 0>(B.p[0], bid);
            else
                wide_section<true, (VAR & kVarWideG4) ? 4u : 16u, (VAR & kVarWaveClock) != 0>(
                    B.p[0], bid * kWavesPerWG + (threadIdx.x >> 6));
            return;
        }
        bid -= nw;
        nblk -= nw;
    }
    // (the lane blocks: one work item per wave, no split)
    batch_block_wave<TRI, VAR & ~kVarLdsSplit>(B, bid, nblk, threadIdx.x >> 6, t0v);
}

template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) k_render_batch(KBatch B)
{
    batch_body<TRI, VAR>(B);
}

// The batch kernel with the wide section's LDS tier (kVarLdsSplit), held to 7 waves / SIMD: the split
// walk needs 80 VGPRs unbounded (6 waves for the whole grid, lane blocks included), 72 at 7 waves with
// no spill (8 spills 36 B / lane)
template <int TRI, int VAR>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(7, 8))) k_render_batch_lds(KBatch B)
{
    batch_body<TRI, VAR>(B);
}

// k_render_batch as one-wave workgroups (k_render_lanes_w64's map): the fused wide section's
// 4 x wh_wgs waves first, then wave r % 4 of lane block (r / 4) * 8 + w % 8, r = w / 8, of the
// p[0].vblocks lane blocks.
template <int TRI, int VAR>
__device__ __forceinline__ void batch_w64_body(const KBatch& B)
{
    __shared__ uint32_t t0s[1];
    uint32_t w = blockIdx.x;
    if constexpr ((VAR & kVarWideFused) != 0)
    {
        const uint32_t nw = B.p[0].wh_wgs * kWavesPerWG;
        if (w < nw)
        {
            static_assert((VAR & kVarLdsSplit) == 0, "the LDS tier needs 256-lane workgroups");
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

template <int TRI, int VAR>
__global__ void __launch_bounds__(64) k_render_batch_w64(KBatch B)
{
    batch_w64_body<TRI, VAR>(B);
}

// The same, held to 8 waves per SIMD.  The hardware admits ⌊800 / (⌈sgpr/16⌉·16 + 16)⌋ waves per SIMD
// (MI355X_MICROARCH.md, residency): <= 80 SGPRs -> 8, 82-96 -> 7, while the compiler's occupancy
// estimate says 8 up to 96.  The fused wide section's kernel held 83 SGPRs, so a rank of N >= 2 ran
// its lane blocks at 7 waves / SIMD (measured: ~5,000-5,800 resident waves at a rank of 8 vs
// ~6,500-7,000 for the same blocks without the section, profiles/r05e_*); with the attribute the
// compiler fits it in 80.
template <int TRI, int VAR>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) k_render_batch_w64_o8(KBatch B)
{
    batch_w64_body<TRI, VAR>(B);
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
    constexpr bool BOX = (VAR & kVarSkipRun) && (VAR & kVarPackedRem);
    uint32_t no_par = 0u;                        // (test_cell's LDS-tier parity: unused here)
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
                    test_cell<false, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests, no_par))
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
                    test_cell<false, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests, no_par))
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

// A frame shape's tables (TabParams): ndc[x * spp + k] = cam_x(x, smp_k.x), then
// ndc[W * spp + y * spp + k] = cam_y(y, smp_k.y) (camera.h:20-21 with the host's fov_xs and aspect),
// and smp[k] = the sample table -- the same values the host path computes and copies.
__global__ void __launch_bounds__(kWG) k_frame_tables(float *ndc, float2 *smp, TabParams T)
{
    const uint32_t i = blockIdx.x * kWG + threadIdx.x;
    const uint32_t nx = T.W * T.spp, n = (T.W + T.H) * T.spp;
    if (i < T.spp) smp[i] = make_float2(T.smp[2 * i], T.smp[2 * i + 1]);
    if (i >= n) return;
    if (i < nx)
    {
        const uint32_t x = i / T.spp, k = i - x * T.spp;
        ndc[i] = rtd::cam_x(x, T.smp[2 * k], T.W, T.fx);
    }
    else
    {
        const uint32_t j = i - nx, y = j / T.spp, k = j - y * T.spp;
        ndc[i] = rtd::cam_y(y, T.smp[2 * k + 1], T.H, T.fx, T.aspect);
    }
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

} // namespace

// ------------------------------------------------------------------------ the kernel table

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

kfn_t lanes_w64_kernel(int var)
{
    return var == kVarAuto ? k_render_lanes_w64<RT_TRI_MOLLER_TRUMBORE, kVarAuto> : nullptr;
}

kfn_t wide_kernel(uint32_t g, bool lds)
{
    if (lds) return g == 4u ? k_render_wh_lds<4> : (g == 16u ? k_render_wh_lds<16> : nullptr);
    return g == 4u ? k_render_wh<4> : (g == 16u ? k_render_wh<16> : nullptr);
}

kfn_t pixel_loop_kernel(int tri, int var)
{
    if (tri == RT_TRI_BARYCENTRIC) return var == 0 ? k_render_pixel_loop<RT_TRI_BARYCENTRIC, 0> : nullptr;
    switch (var)
    {
    case 0: return k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, 0>;
    case kVarMarch: return k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarMarch>;
    case kVarMarch | kVarExhaustive: return k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarMarch | kVarExhaustive>;
    case kVarBrute: return k_render_pixel_loop<RT_TRI_MOLLER_TRUMBORE, kVarBrute>;
    default: return nullptr;
    }
}

kcfn_t compact_kernel(int tri, int var)
{
    if (tri == RT_TRI_BARYCENTRIC) return var == kVarDistSkip ? k_render_compact<RT_TRI_BARYCENTRIC, kVarDistSkip> : nullptr;
    switch (var)
    {
    // AUTO's walk and record test: box runs, packed counts, the Newton 1/det (the wave-uniform
    // scalar list loop left out: its SGPRs made the persistent kernel spill to scratch)
    case kVarCompactBox: return k_render_compact<RT_TRI_MOLLER_TRUMBORE, kVarCompactBox>;
    case kVarWaveGate | kVarDistSkip | kVarOriginPre:
        return k_render_compact<RT_TRI_MOLLER_TRUMBORE, kVarWaveGate | kVarDistSkip | kVarOriginPre>;
    default: return nullptr;
    }
}

namespace {
// o8: the 8-wave instantiation, built for the fused product kernels only (the wave-clock arm spills to
// scratch when held to 8; it keeps its 6-7 waves).  The LDS tier runs in 256-lane workgroups only.
template <int VAR>
kbfn_t batch_kernel_of(bool w64, bool o8)
{
    if constexpr ((VAR & kVarLdsSplit) != 0)
    {
        // (the wave-clock arm spills at 7 waves: unbounded, 6)
        if constexpr ((VAR & kVarWaveClock) != 0)
            return w64 ? nullptr : k_render_batch<RT_TRI_MOLLER_TRUMBORE, VAR>;
        else
            return w64 ? nullptr : k_render_batch_lds<RT_TRI_MOLLER_TRUMBORE, VAR>;
    }
    else
    {
        constexpr bool kO8 = (VAR & kVarWideFused) != 0 && (VAR & kVarWaveClock) == 0;
        if constexpr (kO8)
            if (w64 && o8) return k_render_batch_w64_o8<RT_TRI_MOLLER_TRUMBORE, VAR>;
        return w64 ? k_render_batch_w64<RT_TRI_MOLLER_TRUMBORE, VAR> : k_render_batch<RT_TRI_MOLLER_TRUMBORE, VAR>;
    }
}
} // namespace

kbfn_t batch_kernel(int var, bool w64, bool o8)
{
    constexpr int kFused = kVarAuto | kVarWideHeavy | kVarWideFused;
    if (var == kVarAuto) return batch_kernel_of<kVarAuto>(w64, o8);
    if (var == kFused) return batch_kernel_of<kFused>(w64, o8);
    if (var == (kFused | kVarWideG4)) return batch_kernel_of<kFused | kVarWideG4>(w64, o8);
    if (var == (kFused | kVarLdsSplit)) return batch_kernel_of<kFused | kVarLdsSplit>(w64, o8);
    if (var == (kFused | kVarWideG4 | kVarLdsSplit)) return batch_kernel_of<kFused | kVarWideG4 | kVarLdsSplit>(w64, o8);
    // RT_KERNEL_FLAG_WAVE_CLOCK (debug timelines, tools/batch_waves.py): the bench pair's batched step
    // at one rank and with the fused wide section (either tier)
    if (var == (kVarAuto | kVarWaveClock)) return batch_kernel_of<kVarAuto | kVarWaveClock>(w64, o8);
    if (var == (kFused | kVarWaveClock)) return batch_kernel_of<kFused | kVarWaveClock>(w64, o8);
    if (var == (kFused | kVarLdsSplit | kVarWaveClock)) return batch_kernel_of<kFused | kVarLdsSplit | kVarWaveClock>(w64, o8);
    return nullptr;
}

knfn_t trace_records_kernel() { return k_trace_records; }
knfn_t record_fixup_kernel() { return k_record_fixup; }
origin_pre_fn origin_pre_kernel() { return k_origin_pre; }
tables_fn frame_tables_kernel() { return k_frame_tables; }
unshard_fn unshard_kernel() { return k_unshard; }
check_fn rcp_check_kernel() { return k_rcp_check; }
check_fn gamma_check_kernel() { return k_gamma_check; }
primitives_fn primitives_kernel() { return k_primitives; }

} // namespace rtk
