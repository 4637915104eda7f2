// rt_walk.h -- the per-sample device code of the render kernels (rt_kernels.hip only): the
// reference's GenerateRay -> Grid::Intersect (3D-DDA over the packed cell words, box runs, the
// per-camera-record ray/triangle tests) -> shading -> resolve path, one wave-sized work item at a
// time (process_item), and the alternate intersectors.  See DESIGN.md §4.1-4.13.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "rt_device.h"
#include "rt_kparams.h"

namespace rtk {
namespace {

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

// Workgroup barrier for the LDS tier's reductions (kVarLdsSplit): this wave's LDS (and scalar)
// operations complete, then s_barrier.  The memory clobber keeps the compiler from moving LDS accesses
// across it (the s_barrier builtin alone is not a memory operation).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// kVarLdsSplit: the per-lane (t, list position) and (u, v) of every wave of the workgroup,
// double-buffered by reduction parity: [parity][wave][lane] each
__device__ __forceinline__ float2 *lds_red_tk()
{
    __shared__ float2 r[2 * kWavesPerWG * 64];
    return r;
}
__device__ __forceinline__ float2 *lds_red_uv()
{
    __shared__ float2 r[2 * kWavesPerWG * 64];
    return r;
}

// kVarLdsSplit: cell lists shorter than this (in every lane) are tested whole by every wave, with no
// reduction; longer ones are split between the workgroup's waves
#ifndef RT_LDS_SPLIT_MIN       // (tools/build_variant.sh -DRT_LDS_SPLIT_MIN=n: the A/B arms)
#define RT_LDS_SPLIT_MIN 8
#endif
constexpr uint32_t kLdsSplitMin = RT_LDS_SPLIT_MIN;

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

// The per-lane list loop of the per-camera-record test: this lane's list [kb, ke) in order
// (grid.cpp:243-267), lowering tb on every accepted hit.  The first-half terms (r0..r2) per
// iteration, the second-half terms (r3) only when the gate passes.  Measured against a one-ahead
// prefetch in VGPRs (+12, 6 waves/SIMD) and by LDS-DMA into a per-wave slot
// (global_load_lds_dwordx4; no VGPRs, but four DMA issues per record): both slower on the frame
// and no shorter on the lone heavy waves (profiles/r02e_ab_lane_prefetch.json).
// (kVarLdsSplit: this wave's share kb + first, kb + first + step, ... of the list)
template <bool STATS, int VAR>
__device__ __forceinline__ void lane_list(const KParams& P, rtd::f2v ra, rtd::f2v rc, uint32_t kb, uint32_t ke,
                                          float& tb, float& u, float& v, uint32_t& tri, uint32_t& tests,
                                          uint32_t first = 0u, uint32_t step = 1u)
{
    constexpr bool F = (VAR & kVarFastRcp) != 0;
    constexpr bool SPLIT = (VAR & kVarLdsSplit) != 0;
    for (uint32_t k = kb + (SPLIT ? first : 0u); k < ke; k += (SPLIT ? step : 1u))
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
//
// kVarLdsSplit (the wide section's LDS tier, wide_item_lds): the workgroup's waves hold the same rays in
// the same walk state, so they reach every call with the same lanes and lists.  When some lane's list
// has kLdsSplitMin references or more (a vote, so alike in every wave), wave w tests only positions
// kb + w, kb + w + 4, ...; each lane's local first minimum (t, position) is written to LDS, and after a
// workgroup barrier every wave takes the lexicographic minimum over the four (smaller t, then the lower
// list position: the reference's first minimum, H8) with its u, v.  The buffers alternate by parity
// (lpar), so one barrier per reduction suffices: a wave can only overwrite a buffer after every wave
// has passed the next barrier, i.e. finished reading it.
template <bool STATS, int TRI, int VAR>
__device__ __forceinline__ bool test_cell(const KParams& P, float ox, float oy, float oz, float dx, float dy,
                                          float dz, uint32_t kb, uint32_t ke, float nct_ax, float& t,
                                          float& u, float& v, uint32_t& tri, uint32_t& tests, uint32_t& lpar)
{
    constexpr bool PRE = (VAR & kVarOriginPre) != 0 && TRI == RT_TRI_MOLLER_TRUMBORE;
    constexpr bool F = (VAR & kVarFastRcp) != 0;
    constexpr bool SPLIT = (VAR & kVarLdsSplit) != 0;
    static_assert(!SPLIT || (PRE && !STATS), "the LDS tier runs AUTO's record test");
    (void)lpar;
    // wave-uniform, and the same in every wave of the workgroup (their lanes and lists are the same)
    bool split = false;
    if constexpr (SPLIT) split = __any(ke - kb >= kLdsSplitMin);
    const uint32_t first = split ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u, step = split ? kWavesPerWG : 1u;
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
            const uint32_t kfirst = kb0 + (SPLIT ? first : 0u), kstep = SPLIT ? step : 1u;
            if (!SPLIT || kfirst < ke0)
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
                cvf4 *np = crefs + size_t(kfirst) * 4u;
                vf4 a0 = np[0], a1 = np[1], a2 = np[2], a3 = np[3];
                for (uint32_t k = kfirst;; k += 2u * kstep)
                {
                    vf4 b0, b1, b2, b3;
                    const bool more1 = k + kstep < ke0;
                    if (more1)
                    {
                        np = crefs + size_t(k + kstep) * 4u;
                        b0 = np[0];
                        b1 = np[1];
                        b2 = np[2];
                        b3 = np[3];
                    }
                    test_rec(a0, a1, a2, a3, k);
                    if (!more1) break;
                    const bool more2 = k + 2u * kstep < ke0;
                    if (more2)
                    {
                        np = crefs + size_t(k + 2u * kstep) * 4u;
                        a0 = np[0];
                        a1 = np[1];
                        a2 = np[2];
                        a3 = np[3];
                    }
                    test_rec(b0, b1, b2, b3, k + kstep);
                    if (!more2) break;
                }
            }
            uniform_done = true;
        }
    }
    if constexpr (PRE)
    {
        if (!uniform_done) lane_list<STATS, VAR>(P, ra, rc, kb, ke, tb, u, v, tri, tests, first, step);
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
    if constexpr (SPLIT)
    {
        if (split)
        {
            // the four waves' first minima of this cell -> the list's (kLdsSplit: see above)
            const uint32_t base = lpar * (kWavesPerWG * 64u), lane = threadIdx.x & 63u;
            float2 *tk = lds_red_tk() + base, *uv = lds_red_uv() + base;
            tk[threadIdx.x] = make_float2(tb, __uint_as_float(tb < tb0 ? tri : 0xFFFFFFFFu));
            uv[threadIdx.x] = make_float2(u, v);
            lds_barrier();
            float bt = tb0;
            uint32_t bk = 0xFFFFFFFFu, bj = 0u;
#pragma unroll
            for (uint32_t j = 0; j < kWavesPerWG; j++)
            {
                const float2 o = tk[j * 64u + lane];
                const uint32_t ok = __float_as_uint(o.y);
                const bool better = (o.x < bt) | ((o.x == bt) & (ok < bk));
                bt = better ? o.x : bt;
                bk = better ? ok : bk;
                bj = better ? j : bj;
            }
            lpar ^= 1u;
            if (bk != 0xFFFFFFFFu)
            {
                const float2 w = uv[bj * 64u + lane];
                tb = bt;
                u = w.x;
                v = w.y;
                tri = bk;
            }
        }
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
                                          int& rem0, int& rem1, int& rem2, int& cs0, int& cs1, int& cs2, int& cell,
                                          float *enter_out = nullptr)
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
    if (enter_out) *enter_out = enter_t;
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
    uint32_t lpar = 0u;                 // kVarLdsSplit: the reduction buffers' parity (test_cell)

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
        // Two phases (profiles/r04g_ab_box_run_modes.json): the APPROACH, through
        // the empty space before the wave's first contact, runs per lane (each lane jumps to just
        // before its own box exit by per-axis add chains, then waits at its first non-empty cell);
        // from the moment every active lane is at its own non-empty cell the wave walks in
        // LOCK-STEP, with wave-uniform bare steps while every lane is inside its box, so rays of a
        // wave that cross the same cells test them together (wave-uniform lists).
        static_assert(!STATS, "the records kernel walks the distance words, not the box runs");
        int remp = rem0 | (rem1 << 11) | (rem2 << 22);
        int boxw = kRemGuards;                              // no box yet: look the first cell up
        const int coff = box_offset(P, dx, dy, dz);
        cell += coff;
        bool sync = false;                                  // wave-uniform: the lock-step phase
        for (;;)
        {
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
            if (!sync)
            {
                // Approach: a lane at its first non-empty cell waits there (no step, no test; the
                // cell is looked up again) until every active lane of the wave is at its own.
                // Waiting changes no lane's walk, only when it is taken.
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
            if (kb < ke) hit = test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests, lpar);
            const bool inside = (uint32_t(boxw) & uint32_t(kRemGuards)) == 0u;
            if (!sync && inside)
            {
                // Per-lane box run.  Inside a box the three crossing-time sequences are independent
                // add chains x_a(k+1) = fl(x_a(k) + dt_a), and the box is left at the first of the
                // (f_a + 1)-th crossings E_a = x_a(f_a) (f_a = the box field).  tl is a lower bound
                // of every E_a: f dt + x fused (one rounding) is within 2^-24 |.| of it, the chain
                // within f 2^-24 max|x_k| <= f 2^-24 (|x| + |E|) of it, so
                // E_a >= e_a - (f_a + 2) 2^-23 (|e_a| + |x_a|) with room for the bound's own
                // roundings.  Each axis then takes its crossings below tl (at most f_a of them):
                // every taken crossing is < tl <= every untaken one, so these are exactly the
                // walk's next sum c_a steps, in some order, all inside the box (empty cells, no
                // test, no exit).  Bare steps then run to the box's exit (normally one) -- the
                // same cells, crossing times and exits as one step per cell.
                const uint32_t b0 = uint32_t(boxw);
                const int f0 = boxw & 1023, f1 = (boxw >> 11) & 1023, f2 = int(uint32_t(boxw) >> 22);
                const float tl = __builtin_fminf(__builtin_fminf(box_exit_bound(nct0, dt0, f0), box_exit_bound(nct1, dt1, f1)),
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
                remp = int(uint32_t(remp) - d);           // wrapping (d may reach 2^31)
                cell += int(d & 2047u) * cs0 + int((d >> 11) & 2047u) * cs1 + int(d >> 22) * cs2;
                more = (remp & kRemGuards) == 0;
            }
            else if (sync && wave_all(inside))
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
            if (hit | !more) break;
        }
        // records only: the exit cell in the ray's box-word copy (trace_sample removes the copy's
        // offset, so nothing extra is live across the walk)
        voxel = exit_voxel(remp, cell, cs0, cs1, cs2);
        return t != rtd::kFltMax;                            // t is only set by a hit
    }

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
            if (kb < ke) hit = test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests, lpar);
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
        if (kb < ke && test_cell<STATS, TRI, VAR>(P, ox, oy, oz, dx, dy, dz, kb, ke, nct_ax, t, u, v, tri, tests, lpar))
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
    constexpr uint32_t box = ((VAR & kVarSkipRun) && (VAR & kVarPackedRem)) ? kRecRawBox : 0u;
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
    // kVarLdsSplit: the workgroup's four waves traced the same samples; wave 0 stores them
    const bool owner = (VAR & kVarLdsSplit) == 0 || threadIdx.x < 64u;
    // rt_render_hits_device only: the sample's hit triangle, after the walk (a scalar test of a
    // kernel parameter; the walk above is the same code whatever the pointer holds)
    if (Q.hits && ic.valid && owner) Q.hits[(size_t(ic.y) * Q.W + ic.x) * Q.spp + ic.s] = hit_tri;
    // rt_render_records_device only, likewise: the sample's record (process_record)
    if (Q.recs && ic.valid && owner) process_record<VAR>(Q, ic, so, cr, cg, cb);
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
        const uint32_t j = lane & 3u;
        const float c = j == 0u ? sb : (j == 1u ? sg : sr);
        uint32_t v = rtd::pack_channel(rtd::gamma_half(c * 0.25f)) << (8u * j);   // renderer.cpp:124, exact
        v = j == 3u ? 0u : v;
        const uint32_t word = quad_bcast_u<0>(v) | quad_bcast_u<1>(v) | quad_bcast_u<2>(v);
        if (ic.valid && ic.s == 0 && owner) store_pixel(Q, ic.c, ic.p, ic.x, ic.y, word);
        return;
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
    if (ic.valid && ic.s == 0 && owner)
    {
        const uint32_t word = rtd::pack_bgra8(rtd::gamma_half(average(Q, sr)), rtd::gamma_half(average(Q, sg)),
                                              rtd::gamma_half(average(Q, sb)));
        store_pixel(Q, ic.c, ic.p, ic.x, ic.y, word);
    }
}

} // namespace
} // namespace rtk
