// rt_box_words.h -- host-side construction of AUTO's box-run words (plain C++11, no HIP): included
// by rt_tracer.hip (rt_scene_create) and by the CPU checks (tests/test_box_words.py, tools/box_sim.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

namespace rtbox {

// Box-run words (AUTO's empty runs, grid_intersect): 24 copies of the cell words, one per ray
// octant o (signs of dx, dy, dz) and major axis m (the largest |d| component), in GridIdx order.
//   non-empty cell: 0x80000000 | start << 11 | count        (start < 2^20, count < 2^11)
//   empty cell:     (E0 - 1) | (E1 - 1) << 11 | (E2 - 1) << 22
// where E0 x E1 x E2 cells (x, y, z) is an empty box with its corner at the cell, extending along
// the octant's signs (cells outside the grid count as empty while the shape is chosen; the
// stored box is clipped to the grid).  A walk in octant o starting in the
// cell stays in that box while it has taken fewer than E_a steps along every axis a, whatever its
// direction inside the octant -- so the counts are decremented with the packed remaining-cell
// counts' own axis unit, and the walk needs the next cell word only when one borrows (DESIGN.md
// §4.10).  Any box is exact; the shape only decides how long runs are.  Rays of major axis m
// advance fastest along m, so the box is a square cross-section e x e (bounded by S_m, the largest
// empty square in the cross plane) stretched along m: among the (e, L) a walk along m offers, the
// one maximising min(L, kBoxRatio * e) -- the m-steps a ray of cross slopes <= 1 / kBoxRatio stays
// inside -- and then (kBoxExtend) run on along m as long as that cross-section stays empty.
// Measured on the oracle's walks (tools/box_sim.cpp, 1080p x 4, lookup iterations per wave64 /
// word loads per lane): Cornell 11.9 / 8.5 with the octant cube words -> 4.5 / 3.2 (the exact
// bound, every empty cell skipped: 3.7 / 2.8), killeroo 14.1 / 11.4 -> 5.9 / 4.7 (4.0 / 3.5).
#ifndef RT_BOX_RATIO
#define RT_BOX_RATIO 2
#endif
#ifndef RT_BOX_EXTEND
#define RT_BOX_EXTEND 1
#endif
constexpr uint32_t kBoxRatio = RT_BOX_RATIO;
constexpr uint32_t kBoxSquareCap = 64;      // cross-section sides searched
constexpr uint32_t kBoxLenCap = 128;        // box length along m searched
constexpr bool kBoxExtend = RT_BOX_EXTEND != 0;   // the chosen cross-section's box runs on along m while it stays empty
#ifndef RT_BOX_GROW
#define RT_BOX_GROW 1
#endif
constexpr bool kBoxGrow = RT_BOX_GROW != 0;       // then grows each cross side (and m again) while the box stays empty

// Returns false (out emptied) when a host allocation fails.
inline bool build_box_words(const uint32_t *off, const uint32_t dims[3], std::vector<uint32_t>& out,
                            uint32_t ratio = kBoxRatio, bool extend = kBoxExtend, bool grow = kBoxGrow)
{
    const int dimv[3] = { int(dims[0]), int(dims[1]), int(dims[2]) };
    const uint32_t nc = dims[0] * dims[1] * dims[2];
    const uint32_t field_max[3] = { 1023u, 1023u, 511u };      // E_a - 1 fits bits 0-9 / 11-20 / 22-30
    auto idx = [&](int x, int y, int z) {                      // grid.h:41-42 GridIdx
        return uint32_t(x) + uint32_t(z) * dims[0] + uint32_t(y) * dims[0] * dims[2];
    };
    try
    {
        out.assign(size_t(24) * nc, 0u);
    }
    catch (const std::bad_alloc&)
    {
        out.clear();
        return false;
    }
    // occupancy prefix sums over [0, x) x [0, y) x [0, z) (grow: O(1) box-emptiness queries)
    const size_t px = size_t(dimv[0]) + 1, py = size_t(dimv[1]) + 1, pz = size_t(dimv[2]) + 1;
    std::vector<uint32_t> PS;
    auto pidx = [&](int x, int y, int z) { return (size_t(x) * py + size_t(y)) * pz + size_t(z); };
    if (grow)
    {
        try
        {
            PS.assign(px * py * pz, 0u);
        }
        catch (const std::bad_alloc&)
        {
            out.clear();
            return false;
        }
        for (int x = 1; x <= dimv[0]; x++)
            for (int y = 1; y <= dimv[1]; y++)
                for (int z = 1; z <= dimv[2]; z++)
                {
                    const uint32_t c = idx(x - 1, y - 1, z - 1);
                    PS[pidx(x, y, z)] = (off[c + 1] != off[c] ? 1u : 0u) + PS[pidx(x - 1, y, z)] + PS[pidx(x, y - 1, z)] +
                                        PS[pidx(x, y, z - 1)] - PS[pidx(x - 1, y - 1, z)] - PS[pidx(x - 1, y, z - 1)] -
                                        PS[pidx(x, y - 1, z - 1)] + PS[pidx(x - 1, y - 1, z - 1)];
                }
    }
    // no non-empty cell in the cells [lo, hi) (clipped to the grid by the caller)
    auto empty_box = [&](const int lo[3], const int hi[3]) {
        const int64_t v = int64_t(PS[pidx(hi[0], hi[1], hi[2])]) - PS[pidx(lo[0], hi[1], hi[2])] - PS[pidx(hi[0], lo[1], hi[2])] -
                          PS[pidx(hi[0], hi[1], lo[2])] + PS[pidx(lo[0], lo[1], hi[2])] + PS[pidx(lo[0], hi[1], lo[2])] +
                          PS[pidx(hi[0], lo[1], lo[2])] - PS[pidx(lo[0], lo[1], lo[2])];
        return v == 0;
    };
    // one copy (octant o, major axis m) per task; the copies are independent
    auto copy = [&](uint32_t o, int m, std::vector<uint16_t>& S) {
        const int sg[3] = { (o & 1) ? -1 : 1, (o & 2) ? -1 : 1, (o & 4) ? -1 : 1 };
        {
            const int a = (m + 1) % 3, b = (m + 2) % 3;        // the cross axes
            // S(c): side of the largest empty square in the (a, b) plane with its corner at c,
            // extending along the octant's signs of a and b (2-D largest-square recurrence)
            int p[3];
            for (int im = 0; im < dimv[m]; im++)
                for (int ib = 0; ib < dimv[b]; ib++)
                    for (int ia = 0; ia < dimv[a]; ia++)
                    {
                        p[m] = im;
                        p[a] = sg[a] > 0 ? dimv[a] - 1 - ia : ia;
                        p[b] = sg[b] > 0 ? dimv[b] - 1 - ib : ib;
                        const uint32_t c = idx(p[0], p[1], p[2]);
                        if (off[c + 1] != off[c]) { S[c] = 0; continue; }
                        auto at = [&](int da, int db) -> uint32_t {
                            int q[3] = { p[0], p[1], p[2] };
                            q[a] += da * sg[a];
                            q[b] += db * sg[b];
                            if (q[a] < 0 || q[a] >= dimv[a] || q[b] < 0 || q[b] >= dimv[b]) return kBoxSquareCap;
                            return S[idx(q[0], q[1], q[2])];
                        };
                        S[c] = uint16_t(std::min<uint32_t>(kBoxSquareCap, 1u + std::min(at(1, 0), std::min(at(0, 1), at(1, 1)))));
                    }
            uint32_t *w = out.data() + size_t(o * 3u + uint32_t(m)) * nc;
            for (int y = 0; y < dimv[1]; y++)
                for (int z = 0; z < dimv[2]; z++)
                    for (int x = 0; x < dimv[0]; x++)
                    {
                        const uint32_t c = idx(x, y, z);
                        if (off[c + 1] != off[c])
                        {
                            w[c] = 0x80000000u | (off[c] << 11) | (off[c + 1] - off[c]);
                            continue;
                        }
                        // walk along m with the running minimum of S: a box e x e x L is empty
                        // while every cross-section on the way has S >= e
                        int q[3] = { x, y, z };
                        uint32_t mins = kBoxSquareCap, L = 0, be = 1, bl = 1, best = 0;
                        const uint32_t lcap = std::min(field_max[m] + 1u, kBoxLenCap);
                        for (;;)
                        {
                            const uint32_t sv = (q[m] < 0 || q[m] >= dimv[m]) ? kBoxSquareCap : S[idx(q[0], q[1], q[2])];
                            mins = std::min(mins, sv);
                            if (mins == 0u) break;
                            L++;
                            const uint32_t sc = std::min(L, ratio * mins);
                            if (sc > best) { best = sc; be = mins; bl = L; }
                            else if (extend && mins >= be) bl = L;      // same cross-section, longer box
                            // mins never grows, so no longer box scores higher
                            if ((!extend && L >= ratio * mins) || mins < be || L >= lcap) break;
                            q[m] += sg[m];
                        }
                        uint32_t E[3];
                        E[m] = bl;
                        E[a] = be;
                        E[b] = be;
                        // clipped to the grid: a field never exceeds the walk's remaining-cell
                        // count along its axis (the cells left before the grid's far face), so a
                        // box run's borrow also catches the walk leaving the grid
                        const int pos[3] = { x, y, z };
                        for (int k = 0; k < 3; k++)
                        {
                            const uint32_t rem = uint32_t(sg[k] > 0 ? dimv[k] - 1 - pos[k] : pos[k]);
                            E[k] = std::min(std::min(E[k] - 1u, field_max[k]), rem);
                        }
                        if (grow)
                        {
                            // E[k] now counts cells beyond the corner; grow one side at a time by one
                            // cell while the box stays empty and inside the grid and the field
                            auto fits = [&](const uint32_t *e) {
                                int lo[3], hi[3];
                                for (int k = 0; k < 3; k++)
                                {
                                    const int far = pos[k] + sg[k] * int(e[k]);
                                    lo[k] = std::min(pos[k], far);
                                    hi[k] = std::max(pos[k], far) + 1;
                                    if (lo[k] < 0 || hi[k] > dimv[k]) return false;
                                }
                                return empty_box(lo, hi);
                            };
                            const int order[3] = { a, b, m };
                            for (int k : order)
                                while (E[k] < field_max[k] && E[k] < (k == m ? kBoxLenCap : kBoxSquareCap))
                                {
                                    uint32_t e2[3] = { E[0], E[1], E[2] };
                                    e2[k]++;
                                    if (!fits(e2)) break;
                                    E[k]++;
                                }
                        }
                        w[c] = E[0] | (E[1] << 11) | (E[2] << 22);
                    }
        }
    };
    const uint32_t nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    std::atomic<bool> failed(false);
    auto task = [&](uint32_t t) {
        try
        {
            std::vector<uint16_t> S(nc);
            for (uint32_t k = t; k < 24u; k += nth) copy(k / 3u, int(k % 3u), S);
        }
        catch (const std::bad_alloc&)
        {
            failed = true;
        }
    };
    try
    {
        for (uint32_t t = 1; t < nth; t++) pool.emplace_back(task, t);
    }
    catch (const std::exception&)       // no threads: the remaining tasks run here
    {
    }
    for (uint32_t t = uint32_t(pool.size()) + 1u; t < nth; t++) task(t);
    task(0);
    for (std::thread& th : pool) th.join();
    if (failed)
    {
        out.clear();
        return false;
    }
    return true;
}

}  // namespace rtbox
