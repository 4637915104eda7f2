// box_sim.cpp -- analysis only (links the oracle restatement; never part of the product): how many
// cell-word lookups AUTO's empty-run policies leave per lane and how many lookup iterations
// ("outer") vs bare steps ("inner") a wave64 takes in lock-step, for
//   policy 0: the octant cube words (D - 1 bare steps after an empty cell),
//   policy 1: the exact bound (every empty cell skipped: the floor any per-cell bound can reach),
//   policy 2: the box-run words of csrc/rt_box_words.h (the kernel's).
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tools/box_sim.cpp -o /tmp/box_sim
//   /tmp/box_sim data/scenes/scene8.rtscene 1920 1080 4 2
// A wave = 64 consecutive sample slots of a 16x16 tile in Morton pixel order (AUTO's work item).
// Its lanes advance one DDA cell per iteration in lock-step (the kernel's outer loop and its
// empty-run loop both step every active lane once), so at step j lane l sits in its j-th cell.
// Per step, the lanes whose cell has a list either all share one cell (the wave-uniform scalar
// loop: L iterations) or not (the per-lane loop: max L iterations, sum L useful lane-tests).
// A cooperative pair loop would need ceil(sum L / 64) iterations instead.
#include "../oracle/cpu_tracer.cpp"
#include "../cpp-11-ray-trace-march-framework_amd/csrc/rt_box_words.h"

#include <algorithm>
#include <atomic>
#include <cstdio>

namespace {

struct Walk { std::vector<uint32_t> cell, len; uint32_t oct = 0, maj = 0; float slope = 0; };   // per DDA step: cell, list length

// The octant empty-run words of rt_scene_create: per octant o and empty cell, D = the side of the
// largest empty cube with its corner there extending along the octant's signs (out-of-grid counts
// as empty); 0 for non-empty cells.
std::vector<uint32_t> octant_dist(const Scene& s)
{
    const uint32_t dxs = s.dim[0], dys = s.dim[1], dzs = s.dim[2], nc = dxs * dys * dzs;
    constexpr uint32_t kInf = 0x1FFFFFu;
    std::vector<uint32_t> out(size_t(8) * nc), D(nc);
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
                    const int x = sx > 0 ? int(dxs) - 1 - ix : ix;
                    const int y = sy > 0 ? int(dys) - 1 - iy : iy;
                    const int z = sz > 0 ? int(dzs) - 1 - iz : iz;
                    const uint32_t c = uint32_t(x) + uint32_t(z) * dxs + uint32_t(y) * dxs * dzs;
                    if (s.off[c + 1] != s.off[c]) { D[c] = 0; continue; }
                    uint32_t m = kInf;
                    for (int n = 1; n < 8; n++)
                        m = std::min(m, at(x + ((n & 1) ? sx : 0), y + ((n & 2) ? sy : 0), z + ((n & 4) ? sz : 0)));
                    D[c] = std::min(kInf, m + 1);
                }
        for (uint32_t c = 0; c < nc; c++) out[size_t(o) * nc + c] = D[c];
    }
    return out;
}

void walk(const Scene& s, const V3 o, const V3 d, Walk& w)
{
    w.cell.clear(); w.len.clear();
    w.oct = uint32_t(d.x < 0.0f) | (uint32_t(d.y < 0.0f) << 1) | (uint32_t(d.z < 0.0f) << 2);
    {   // box_offset's major axis
        const float ax = std::fabs(d.x), ay = std::fabs(d.y), az = std::fabs(d.z);
        w.maj = (ax >= ay && ax >= az) ? 0u : (ay >= az ? 1u : 2u);
        const float mx = std::max(ax, std::max(ay, az)), sm = ax + ay + az - mx - std::min(ax, std::min(ay, az));
        w.slope = sm / mx;
    }
    float enter_t, leave_t;
    V3 g;
    if (PointAABB(o, s.aabb_min, s.aabb_max)) { enter_t = 0.0f; g = o; }
    else if (RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t))
        g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
    else return;
    float nct[3], dt[3] = {0, 0, 0};
    int step[3] = {0, 0, 0}, out[3] = {0, 0, 0}, pos[3];
    for (int ax = 0; ax < 3; ax++)
    {
        pos[ax] = s.ToVoxel(g, ax);
        const float da = comp(d, ax);
        if (da == 0.0f) nct[ax] = std::numeric_limits<float>::max();
        else if (da > 0.0f)
        {
            nct[ax] = enter_t + (s.ToPos(pos[ax] + 1, ax) - comp(g, ax)) / da;
            dt[ax] = s.cell_wdh / da; step[ax] = 1; out[ax] = int(s.dim[ax]);
        }
        else
        {
            nct[ax] = enter_t + (s.ToPos(pos[ax], ax) - comp(g, ax)) / da;
            dt[ax] = -s.cell_wdh / da; step[ax] = -1; out[ax] = -1;
        }
    }
    float t = std::numeric_limits<float>::max();
    while (true)
    {
        const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
        const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
        const uint32_t k0 = s.off[cell], k1 = s.off[cell + 1];
        w.cell.push_back(cell);
        w.len.push_back(k1 - k0);
        for (uint32_t k = k0; k < k1; k++)
        {
            const Triangle& tr = s.tris[s.refs[k]];
            float ct, cu, cv;
            if (RayTri(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p, ct, cu, cv) && ct < t && ct < nct[ax])
                t = ct;
        }
        if (t != std::numeric_limits<float>::max()) break;
        pos[ax] += step[ax];
        if (pos[ax] == out[ax]) break;
        nct[ax] += dt[ax];
    }
}

uint32_t compact_bits(uint32_t v)
{
    v &= 0x55u; v = (v | (v >> 1)) & 0x33u; v = (v | (v >> 2)) & 0x0Fu; return v;
}

int axis_of(const Scene& s, uint32_t c0, uint32_t c1)     // the DDA step's axis from GridIdx
{
    const int d = int(c1) - int(c0);
    if (d == 1 || d == -1) return 0;
    if (d == int(s.dim[0]) || d == -int(s.dim[0])) return 2;
    return 1;
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 6) { std::fprintf(stderr, "usage: box_sim scene.rtscene W H spp policy\n"); return 2; }
    Scene s;
    if (!ReadScene(argv[1], s)) return 1;
    BuildGrid(s, 64);
    const std::vector<uint32_t> octD = octant_dist(s);
    std::vector<uint32_t> boxw;
    rtbox::build_box_words(s.off.data(), s.dim, boxw, argc > 6 ? uint32_t(std::atoi(argv[6])) : rtbox::kBoxRatio,
                           argc > 8 ? std::atoi(argv[8]) != 0 : rtbox::kBoxExtend, argc > 9 ? std::atoi(argv[9]) != 0 : rtbox::kBoxGrow);
    const uint32_t ncells = s.dim[0] * s.dim[1] * s.dim[2];
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]);
    const int policy = std::atoi(argv[5]);
    std::vector<uint32_t> boxw2;       // policy 3: a second set for shallow rays (cross slope <= 1 / r2)
    const uint32_t r2 = argc > 7 ? uint32_t(std::atoi(argv[7])) : 4u;
    if (policy == 3) rtbox::build_box_words(s.off.data(), s.dim, boxw2, r2);
    const std::vector<float> smp = Hammersley(spp);
    const uint32_t tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16, items_per_tile = 256 * spp / 64;
    const uint32_t nitems = tiles_x * tiles_y * items_per_tile;
    const uint32_t nth = std::max(1u, std::thread::hardware_concurrency());
    std::atomic<uint32_t> next(0);
    std::atomic<uint64_t> outer(0), inner(0), loads(0), waves(0), steps(0);
    std::atomic<uint64_t> uni_recs(0), lane_iters(0), lane_useful(0), test_iters(0), chain_axis(0), chain_tot(0);
    std::vector<std::thread> pool;
    for (uint32_t th = 0; th < nth; th++)
        pool.emplace_back([&]() {
            std::vector<Walk> lanes(64);
            uint64_t o_ = 0, i_ = 0, l_ = 0, w_ = 0, s_ = 0;
            for (;;)
            {
                const uint32_t item = next.fetch_add(1);
                if (item >= nitems) break;
                const uint32_t t = item / items_per_tile, sub = item % items_per_tile;
                const uint32_t tx0 = (t % tiles_x) * 16, ty0 = (t / tiles_x) * 16;
                uint32_t maxlen = 0;
                for (uint32_t l = 0; l < 64; l++)
                {
                    const uint32_t slot = sub * 64 + l, p = slot / spp, si = slot % spp;
                    const uint32_t x = tx0 + compact_bits(p), y = ty0 + compact_bits(p >> 1);
                    lanes[l].cell.clear(); lanes[l].len.clear();
                    if (x >= W || y >= H) continue;
                    V3 o, d;
                    GenRay(s.cam, x, y, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
                    walk(s, o, d, lanes[l]);
                    maxlen = std::max<uint32_t>(maxlen, uint32_t(lanes[l].cell.size()));
                    s_ += lanes[l].cell.size();
                }
                w_++;
                // test-step uniformity: per outer iteration, the lanes looking up a non-empty cell
                auto tally = [&](const std::vector<std::pair<uint32_t, uint32_t>>& tl, uint64_t& ur, uint64_t& li,
                                 uint64_t& lu, uint64_t& ti) {
                    if (tl.empty()) return;
                    ti++;
                    bool uni = true; uint32_t mx = 0, sum = 0;
                    for (auto& p : tl) { if (p.first != tl[0].first) uni = false; mx = std::max(mx, p.second); sum += p.second; }
                    if (uni) ur += mx; else { li += mx; lu += sum; }
                };
                uint64_t ur_ = 0, li_ = 0, lu_ = 0, ti_ = 0;
                if (policy == 4)
                {
                    // per-lane runs: each outer iteration every active lane looks its cell up
                    // (testing it when non-empty) and, when empty, jumps to its box's exit cell
                    std::vector<uint32_t> pos(64, 0);
                    for (;;)
                    {
                        std::vector<std::pair<uint32_t, uint32_t>> tl;
                        uint32_t act = 0, mx_ax[3] = {0, 0, 0}, mx_tot = 0;
                        for (uint32_t l = 0; l < 64; l++)
                        {
                            const Walk& wk = lanes[l];
                            if (pos[l] >= wk.cell.size()) continue;
                            act++;
                            l_++;
                            const uint32_t j = pos[l], c = wk.cell[j];
                            if (wk.len[j]) { tl.push_back({c, wk.len[j]}); pos[l] = j + 1; continue; }
                            const uint32_t w = boxw[size_t(wk.oct * 3u + wk.maj) * ncells + c];
                            int bcnt[3] = { int(w & 1023u), int((w >> 11) & 1023u), int((w >> 22) & 511u) };
                            uint32_t k = j, nax[3] = {0, 0, 0};
                            while (k + 1 < wk.cell.size())
                            {
                                const int ax = axis_of(s, wk.cell[k], wk.cell[k + 1]);
                                k++;
                                nax[ax]++;
                                if (--bcnt[ax] < 0) break;
                            }
                            for (int q = 0; q < 3; q++) mx_ax[q] = std::max(mx_ax[q], nax[q]);
                            mx_tot = std::max(mx_tot, nax[0] + nax[1] + nax[2]);
                            if (k + 1 >= wk.cell.size() && bcnt[0] >= 0 && bcnt[1] >= 0 && bcnt[2] >= 0) k = uint32_t(wk.cell.size());
                            pos[l] = k;
                        }
                        if (!act) break;
                        o_++;
                        tally(tl, ur_, li_, lu_, ti_);
                        chain_axis += mx_ax[0] + mx_ax[1] + mx_ax[2];
                        chain_tot += mx_tot;
                    }
                    uni_recs += ur_; lane_iters += li_; lane_useful += lu_; test_iters += ti_;
                    continue;
                }
                if (policy == 5)
                {
                    // hybrid: one step per lane per outer iteration (lookups as policy 2), and when
                    // after it every active lane is inside its box, each lane jumps to its own
                    // box's exit (per-lane add chains), instead of wave-uniform bare steps
                    std::vector<uint32_t> pos(64, 0);
                    int inbox[64] = {}, bcn[64][3] = {};
                    for (;;)
                    {
                        std::vector<std::pair<uint32_t, uint32_t>> tl;
                        uint32_t act = 0;
                        for (uint32_t l = 0; l < 64; l++)
                        {
                            const Walk& wk = lanes[l];
                            if (pos[l] >= wk.cell.size()) continue;
                            act++;
                            const uint32_t j = pos[l], c = wk.cell[j];
                            if (!inbox[l])
                            {
                                l_++;
                                if (wk.len[j]) tl.push_back({c, wk.len[j]});
                                else
                                {
                                    const uint32_t w = boxw[size_t(wk.oct * 3u + wk.maj) * ncells + c];
                                    bcn[l][0] = int(w & 1023u); bcn[l][1] = int((w >> 11) & 1023u); bcn[l][2] = int((w >> 22) & 511u);
                                    inbox[l] = 1;
                                }
                            }
                            if (j + 1 < wk.cell.size() && inbox[l])
                                if (--bcn[l][axis_of(s, wk.cell[j], wk.cell[j + 1])] < 0) inbox[l] = 0;
                            pos[l] = j + 1;
                        }
                        if (!act) break;
                        o_++;
                        tally(tl, ur_, li_, lu_, ti_);
                        bool all = true; uint32_t n = 0;
                        for (uint32_t l = 0; l < 64; l++)
                            if (pos[l] < lanes[l].cell.size()) { n++; if (!inbox[l]) all = false; }
                        if (!n || !all) continue;
                        uint32_t mx_ax[3] = {0, 0, 0};
                        for (uint32_t l = 0; l < 64; l++)
                        {
                            const Walk& wk = lanes[l];
                            if (pos[l] >= wk.cell.size()) continue;
                            uint32_t k = pos[l], nax[3] = {0, 0, 0};
                            while (k + 1 < wk.cell.size())
                            {
                                const int ax = axis_of(s, wk.cell[k], wk.cell[k + 1]);
                                k++;
                                if (--bcn[l][ax] < 0) { inbox[l] = 0; break; }
                                nax[ax]++;
                            }
                            if (k + 1 >= wk.cell.size() && inbox[l]) k = uint32_t(wk.cell.size());
                            for (int q = 0; q < 3; q++) mx_ax[q] = std::max(mx_ax[q], nax[q]);
                            pos[l] = k;
                        }
                        i_++;
                        chain_axis += mx_ax[0] + mx_ax[1] + mx_ax[2];
                    }
                    uni_recs += ur_; lane_iters += li_; lane_useful += lu_; test_iters += ti_;
                    continue;
                }
                // known[l] > 0: the lane's current cell is proven empty (no lookup); bc: box counts
                int known[64] = {}, bc[64][3] = {};
                auto advance = [&](uint32_t l, uint32_t j) {      // the step from cell j to j + 1
                    known[l]--;
                    if (policy >= 2 && known[l] > 0 && j + 1 < lanes[l].cell.size())
                        if (--bc[l][axis_of(s, lanes[l].cell[j], lanes[l].cell[j + 1])] < 0) known[l] = 0;
                };
                uint32_t j = 0;
                while (j < maxlen)
                {
                    uint32_t act = 0;
                    std::vector<std::pair<uint32_t, uint32_t>> tl;
                    for (uint32_t l = 0; l < 64; l++)
                    {
                        if (j >= lanes[l].cell.size()) continue;
                        act++;
                        if (known[l] == 0 && lanes[l].len[j]) tl.push_back({lanes[l].cell[j], lanes[l].len[j]});
                        if (known[l] == 0)
                        {
                            l_++;
                            const uint32_t c = lanes[l].cell[j];
                            if (lanes[l].len[j]) known[l] = 0;
                            else if (policy == 0) known[l] = int(octD[size_t(lanes[l].oct) * ncells + c]);
                            else if (policy == 1)
                            {
                                uint32_t k = j + 1;
                                while (k < lanes[l].cell.size() && lanes[l].len[k] == 0) k++;
                                known[l] = int(k - j);
                            }
                            else
                            {
                                const std::vector<uint32_t>& bw = (policy == 3 && lanes[l].slope * float(r2) <= 1.0f) ? boxw2 : boxw;
                                const uint32_t w = bw[size_t(lanes[l].oct * 3u + lanes[l].maj) * ncells + c];
                                bc[l][0] = int(w & 1023u); bc[l][1] = int((w >> 11) & 1023u); bc[l][2] = int((w >> 22) & 511u);
                                known[l] = 1 << 30;
                            }
                            if (known[l]) advance(l, j);
                        }
                        else advance(l, j);
                    }
                    if (!act) break;
                    o_++;
                    tally(tl, ur_, li_, lu_, ti_);
                    j++;
                    for (;;)        // wave-uniform bare steps while every active lane's cell is known empty
                    {
                        bool all = true; uint32_t n = 0;
                        for (uint32_t l = 0; l < 64; l++)
                            if (j < lanes[l].cell.size()) { n++; if (known[l] <= 0) all = false; }
                        if (!n || !all) break;
                        for (uint32_t l = 0; l < 64; l++)
                            if (j < lanes[l].cell.size()) advance(l, j);
                        i_++;
                        j++;
                    }
                }
                uni_recs += ur_; lane_iters += li_; lane_useful += lu_; test_iters += ti_;
            }
            outer += o_; inner += i_; loads += l_; waves += w_; steps += s_;
        });
    // (policy 2's tallies are added per item below)
    for (auto& t : pool) t.join();
    std::printf("{\"policy\": %d, \"outer_per_wave\": %.2f, \"inner_per_wave\": %.2f, \"loads_per_lane\": %.2f, "
                "\"steps_per_lane\": %.2f, \"uniform_records_per_wave\": %.2f, \"lane_iterations_per_wave\": %.2f, "
                "\"lane_util\": %.3f, \"test_iterations_per_wave\": %.2f, \"chain_axis_max_per_wave\": %.2f, \"chain_total_max_per_wave\": %.2f}\n", policy, double(outer) / waves,
                double(inner) / waves, double(loads) / (64.0 * waves), double(steps) / (64.0 * waves),
                double(uni_recs) / waves, double(lane_iters) / waves, double(lane_useful) / (64.0 * std::max<uint64_t>(1, lane_iters)),
                double(test_iters) / waves, double(chain_axis) / waves, double(chain_tot) / waves);
}
