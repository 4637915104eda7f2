// segment_sim.cpp -- analysis only (links the oracle restatement; never part of the product): a
// ray's walk split into J segments of the t axis, each walked by its own lane (DESIGN.md §7, next
// steps 0).  Checks the exact-state rule and measures the critical chain it would leave.
//
// Rule: for a boundary value c, S(c) = "every axis crossing x_a(k) < c taken".  The reference's
// DDA (grid.cpp:218-281) always steps the axis of a smallest next crossing, so S(c) is one of its
// states: the one it holds when its smallest next crossing first reaches >= c.  Per axis, S(c)
// needs only that axis's own chain x_a(k + 1) = fl(x_a(k) + dt_a) (the reference's nct[a] += dt[a])
// counted up to c: k_a crossings, position start_a + step_a * k_a, next crossing x_a(k_a).  A
// segment lane for [T_j, T_j+1) starts from S(T_j), tests the current cell with the reference's own
// exit bound and steps until its smallest next crossing is >= T_j+1 (that cell is the next lane's).
//
// For every sample of a frame: the reference walk to its first accepted hit (or out of the grid),
// its DDA state before every cell; then for J segments with T_j equal splits of [enter_t,
// leave_t]: S(T_j) from the per-axis chains against the walk's own state (mismatches are printed
// and counted; an S(T_j) past the walk's end must have left the grid or lie past the hit), and
// the costs: serial = cells + tests of the walk; segmented = max over the segments up to the
// hit's of (cells + tests + chain adds / 8) -- the lanes after the hit's segment are cut.
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tools/segment_sim.cpp -o /tmp/segment_sim
//   /tmp/segment_sim data/scenes/scene8.rtscene 1920 1080 4 [J=16] [G=1 list lanes] [cell weight=1]
#include "../oracle/cpu_tracer.cpp"

#include <algorithm>
#include <atomic>
#include <cstdio>

namespace {

struct CellState { int pos[3]; float nct[3]; uint32_t tests; };

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5) return 2;
    Scene s;
    if (!ReadScene(argv[1], s)) return 1;
    BuildGrid(s, 64);
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]);
    const int J = argc > 5 ? std::atoi(argv[5]) : 16;
    // lanes splitting each cell's list (the wide section's G): a cell costs 1 + ceil(tests / G)
    const uint32_t G = argc > 6 ? uint32_t(std::atoi(argv[6])) : 1u;
    // a cell's own cost in test units (its word, list range and first record are dependent memory
    // round trips: on the GPU a cell iteration costs a few tests' latency)
    const float Wc = argc > 7 ? float(std::atof(argv[7])) : 1.0f;
    const std::vector<float> smp = Hammersley(spp);
    std::atomic<uint32_t> next(0);
    std::atomic<uint64_t> mismatches(0), checks(0), rays(0);
    const size_t nth = std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::vector<std::pair<float, float>>> costs(nth);   // (serial, segmented) per ray
    std::vector<std::vector<float>> split(nth);                     // list split only, per ray
    std::vector<std::thread> pool;
    for (size_t th = 0; th < nth; th++)
        pool.emplace_back([&, th]() {
            std::vector<CellState> walk;
            uint64_t mm = 0, ck = 0, rr = 0;
            for (;;)
            {
                const uint32_t y = next.fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; x++)
                    for (uint32_t si = 0; si < spp; si++)
                    {
                        V3 o, d;
                        GenRay(s.cam, x, y, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
                        rr++;
                        float enter_t, leave_t;
                        V3 g;
                        const bool inside = PointAABB(o, s.aabb_min, s.aabb_max);
                        if (!RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t)) continue;
                        if (inside) { enter_t = 0.0f; g = o; }
                        else g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
                        float nct0[3], dt[3] = {0, 0, 0};
                        int step[3] = {0, 0, 0}, out[3] = {0, 0, 0}, pos0[3];
                        for (int ax = 0; ax < 3; ax++)
                        {
                            pos0[ax] = s.ToVoxel(g, ax);
                            const float da = comp(d, ax);
                            if (da == 0.0f) nct0[ax] = std::numeric_limits<float>::max();
                            else if (da > 0.0f)
                            {
                                nct0[ax] = enter_t + (s.ToPos(pos0[ax] + 1, ax) - comp(g, ax)) / da;
                                dt[ax] = s.cell_wdh / da; step[ax] = 1; out[ax] = int(s.dim[ax]);
                            }
                            else
                            {
                                nct0[ax] = enter_t + (s.ToPos(pos0[ax], ax) - comp(g, ax)) / da;
                                dt[ax] = -s.cell_wdh / da; step[ax] = -1; out[ax] = -1;
                            }
                        }
                        // the reference walk (grid.cpp:218-281, as oracle IntersectT), state per cell
                        walk.clear();
                        int pos[3] = {pos0[0], pos0[1], pos0[2]};
                        float nct[3] = {nct0[0], nct0[1], nct0[2]};
                        bool hit = false;
                        for (;;)
                        {
                            const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
                            const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
                            const uint32_t k0 = s.off[cell], k1 = s.off[cell + 1];
                            CellState cs;
                            std::memcpy(cs.pos, pos, sizeof(pos));
                            std::memcpy(cs.nct, nct, sizeof(nct));
                            cs.tests = k1 - k0;
                            walk.push_back(cs);
                            float t = std::numeric_limits<float>::max();
                            for (uint32_t k = k0; k < k1; k++)
                            {
                                const Triangle& tr = s.tris[s.refs[k]];
                                float ct, cu, cv;
                                if (RayTri(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p, ct, cu, cv) &&
                                    ct < t && ct < nct[ax])
                                    t = ct;
                            }
                            if (t != std::numeric_limits<float>::max()) { hit = true; break; }
                            pos[ax] += step[ax];
                            if (pos[ax] == out[ax]) break;
                            nct[ax] += dt[ax];
                        }
                        // segments
                        float serial = 0.0f;
                        for (const CellState& c : walk) serial += Wc + float(c.tests);
                        float listsplit = 0.0f;                            // one segment, G lanes
                        for (const CellState& c : walk) listsplit += Wc + float((c.tests + G - 1u) / G);
                        std::vector<size_t> first(J + 1, walk.size());   // first walk cell of segment j
                        std::vector<float> adds(J + 1, 0.0f);
                        first[0] = 0;
                        for (int j = 1; j < J; j++)
                        {
                            const float T = enter_t + (leave_t - enter_t) * float(j) / float(J);
                            // S(T) from the per-axis chains, capped at the grid's exit on each axis
                            int sp[3];
                            float sn[3];
                            bool left = false;
                            for (int a = 0; a < 3; a++)
                            {
                                float xv = nct0[a];
                                int k = 0;
                                const int rem = step[a] > 0 ? out[a] - pos0[a] : (step[a] < 0 ? pos0[a] - out[a] : 0);
                                while (xv < T && k < rem && step[a] != 0)
                                {
                                    xv += dt[a];
                                    k++;
                                }
                                sp[a] = pos0[a] + step[a] * k;
                                sn[a] = xv;
                                adds[j] += float(k);
                                left = left || (step[a] != 0 && sp[a] == out[a]);
                            }
                            // the walk's state when its smallest next crossing first reaches >= T
                            size_t i = 0;
                            while (i < walk.size() &&
                                   std::min(walk[i].nct[0], std::min(walk[i].nct[1], walk[i].nct[2])) < T)
                                i++;
                            first[j] = i;
                            ck++;
                            if (i < walk.size())
                            {
                                const CellState& c = walk[i];
                                const bool same = c.pos[0] == sp[0] && c.pos[1] == sp[1] && c.pos[2] == sp[2] &&
                                                  fbits(c.nct[0]) == fbits(sn[0]) && fbits(c.nct[1]) == fbits(sn[1]) &&
                                                  fbits(c.nct[2]) == fbits(sn[2]);
                                if (!same && !left)
                                {
                                    if (mm < 5)
                                        std::fprintf(stderr, "mismatch px %u %u s %u seg %d: walk (%d %d %d) state (%d %d %d)\n",
                                                     x, y, si, j, c.pos[0], c.pos[1], c.pos[2], sp[0], sp[1], sp[2]);
                                    mm++;
                                }
                            }
                            else if (!hit && !left)
                            {
                                // the walk left the grid before T: S(T) must be out of the grid too
                                if (mm < 5)
                                    std::fprintf(stderr, "exit mismatch px %u %u s %u seg %d\n", x, y, si, j);
                                mm++;
                            }
                        }
                        // latency: the segments up to the hit's (all of them without a hit)
                        float lat = 0.0f;
                        for (int j = 0; j < J; j++)
                        {
                            const size_t a = first[j], b = std::max(first[j], first[j + 1]);
                            if (a >= walk.size()) break;
                            float c = adds[j] / 8.0f;
                            for (size_t i = a; i < std::min(b, walk.size()); i++)
                                c += Wc + float((walk[i].tests + G - 1u) / G);
                            lat = std::max(lat, c);
                        }
                        costs[th].push_back(std::make_pair(serial, lat));
                        split[th].push_back(listsplit);
                    }
            }
            mismatches += mm;
            checks += ck;
            rays += rr;
        });
    for (auto& t : pool) t.join();
    std::vector<std::pair<float, float>> all;
    std::vector<float> lsp;
    for (auto& v : costs) all.insert(all.end(), v.begin(), v.end());
    for (auto& v : split) lsp.insert(lsp.end(), v.begin(), v.end());
    std::vector<size_t> idx(all.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return all[a].first > all[b].first; });
    double l1 = 0.0, l01 = 0.0;
    auto summary = [&](double frac, double& ser, double& seg, double& ls) {
        const size_t n = std::max<size_t>(1, size_t(double(all.size()) * frac));
        ser = seg = ls = 0.0;
        for (size_t i = 0; i < n && i < idx.size(); i++)
        {
            ser += all[idx[i]].first;
            seg += all[idx[i]].second;
            ls += lsp[idx[i]];
        }
        ser /= double(n);
        seg /= double(n);
        ls /= double(n);
    };
    double s1, g1, s01, g01, sa, ga, la;
    summary(0.01, s1, g1, l1);
    summary(0.001, s01, g01, l01);
    summary(1.0, sa, ga, la);
    std::printf("{\"scene\": \"%s\", \"segments\": %d, \"list_lanes\": %u, \"top1pct_list_split_only\": %.1f, "
                "\"top0.1pct_list_split_only\": %.1f, \"rays\": %llu, \"state_checks\": %llu, \"mismatches\": %llu, "
                "\"mean_serial\": %.1f, \"mean_segmented\": %.1f, \"top1pct_serial\": %.1f, \"top1pct_segmented\": %.1f, "
                "\"top0.1pct_serial\": %.1f, \"top0.1pct_segmented\": %.1f, \"max_serial\": %.1f}\n",
                argv[1], J, G, l1, l01, (unsigned long long)rays.load(), (unsigned long long)checks.load(),
                (unsigned long long)mismatches.load(), sa, ga, s1, g1, s01, g01, all.empty() ? 0.0 : all[0].first);
}
