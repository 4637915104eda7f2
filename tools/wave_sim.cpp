// wave_sim.cpp -- analysis only (links the oracle restatement; never part of the product): how
// AUTO's wave64 lock-step spends its triangle-list work, to size a wave-cooperative (ray, record)
// pair path before building it.
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tools/wave_sim.cpp -o /tmp/wave_sim
//   /tmp/wave_sim data/scenes/scene8.rtscene 1920 1080 4
// A wave = 64 consecutive sample slots of a 16x16 tile in Morton pixel order (AUTO's work item).
// Its lanes advance one DDA cell per iteration in lock-step (the kernel's outer loop and its
// empty-run loop both step every active lane once), so at step j lane l sits in its j-th cell.
// Per step, the lanes whose cell has a list either all share one cell (the wave-uniform scalar
// loop: L iterations) or not (the per-lane loop: max L iterations, sum L useful lane-tests).
// A cooperative pair loop would need ceil(sum L / 64) iterations instead.
#include "../oracle/cpu_tracer.cpp"

#include <algorithm>
#include <atomic>
#include <cstdio>

namespace {

struct Walk { std::vector<uint32_t> cell, len; uint32_t oct = 0; };   // per DDA step: cell, list length

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

struct Acc
{
    uint64_t waves = 0, steps = 0, uni_steps = 0, uni_recs = 0, lane_steps = 0, lane_iters = 0, lane_useful = 0;
    uint64_t coop_iters = 0, distinct_sum = 0, dist_iters = 0;
    uint64_t outer = 0, inner = 0, outer_lanes = 0, inner_lanes = 0, loads = 0, empty_lane_steps = 0;
    uint64_t hist_util[11] = {};            // per-lane steps by useful / (64 * iterations), deciles
    uint64_t hist_util_w[11] = {};          // ... weighted by iterations
    void add(const Acc& o)
    {
        waves += o.waves; steps += o.steps; uni_steps += o.uni_steps; uni_recs += o.uni_recs;
        lane_steps += o.lane_steps; lane_iters += o.lane_iters; lane_useful += o.lane_useful;
        coop_iters += o.coop_iters; distinct_sum += o.distinct_sum; dist_iters += o.dist_iters;
        outer += o.outer; inner += o.inner; outer_lanes += o.outer_lanes; inner_lanes += o.inner_lanes;
        loads += o.loads; empty_lane_steps += o.empty_lane_steps;
        for (int i = 0; i < 11; i++) { hist_util[i] += o.hist_util[i]; hist_util_w[i] += o.hist_util_w[i]; }
    }
};

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5) { std::fprintf(stderr, "usage: wave_sim scene.rtscene W H spp\n"); return 2; }
    Scene s;
    if (!ReadScene(argv[1], s)) { std::fprintf(stderr, "cannot read %s\n", argv[1]); return 1; }
    BuildGrid(s, 64);
    const std::vector<uint32_t> octD = octant_dist(s);
    const uint32_t ncells = s.dim[0] * s.dim[1] * s.dim[2];
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]);
    const std::vector<float> smp = Hammersley(spp);
    const uint32_t tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16, items_per_tile = 256 * spp / 64;
    const uint32_t nitems = tiles_x * tiles_y * items_per_tile;
    const uint32_t nth = std::max(1u, std::thread::hardware_concurrency());
    std::vector<Acc> acc(nth);
    std::atomic<uint32_t> next(0);
    std::vector<double> item_cost(nitems, 0.0);     // modelled VALU of each work item (shard balance)
    std::vector<std::thread> pool;
    for (uint32_t th = 0; th < nth; th++)
        pool.emplace_back([&, th]() {
            std::vector<Walk> lanes(64);
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
                }
                Acc& a = acc[th];
                const Acc a0 = a;
                a.waves++;
                a.steps += maxlen;
                // AUTO's two loops (grid_intersect): an outer iteration processes cell j of every
                // active lane (its word loaded when skip == 0, else skip--), then, while EVERY
                // active lane is inside a proven-empty run (skip > 0), inner iterations take bare
                // steps.  A lane leaves after its last cell (hit or grid exit).
                {
                    int skip[64] = {};
                    uint32_t j = 0;
                    while (j < maxlen)
                    {
                        uint32_t act = 0;
                        for (uint32_t l = 0; l < 64; l++)
                        {
                            if (j >= lanes[l].cell.size()) continue;
                            act++;
                            a.empty_lane_steps += lanes[l].len[j] == 0;
                            if (skip[l] == 0)
                            {
                                a.loads++;
                                const uint32_t c = lanes[l].cell[j];
                                skip[l] = lanes[l].len[j] ? 0 : int(octD[size_t(lanes[l].oct) * ncells + c]) - 1;
                            }
                            else skip[l]--;
                        }
                        if (!act) break;
                        a.outer++; a.outer_lanes += act;
                        j++;
                        for (;;)
                        {
                            bool all = true; uint32_t n = 0;
                            for (uint32_t l = 0; l < 64; l++)
                                if (j < lanes[l].cell.size()) { n++; if (skip[l] <= 0) all = false; }
                                else if (j - 1 < lanes[l].cell.size() && false) {}
                            if (!n || !all) break;
                            for (uint32_t l = 0; l < 64; l++)
                                if (j < lanes[l].cell.size()) { skip[l]--; a.empty_lane_steps++; }
                            a.inner++; a.inner_lanes += n;
                            j++;
                        }
                    }
                }
                for (uint32_t j = 0; j < maxlen; j++)
                {
                    uint32_t mx = 0, sum = 0, ntest = 0, c0 = 0xFFFFFFFFu;
                    bool uni = true;
                    std::vector<std::pair<uint32_t, uint32_t>> cells;
                    for (uint32_t l = 0; l < 64; l++)
                    {
                        if (j >= lanes[l].cell.size() || lanes[l].len[j] == 0) continue;
                        const uint32_t L = lanes[l].len[j], c = lanes[l].cell[j];
                        ntest++;
                        if (c0 == 0xFFFFFFFFu) c0 = c; else if (c != c0) uni = false;
                        mx = std::max(mx, L); sum += L;
                        cells.push_back({c, L});
                    }
                    if (!ntest) continue;
                    if (uni) { a.uni_steps++; a.uni_recs += mx; continue; }
                    a.lane_steps++; a.lane_iters += mx; a.lane_useful += sum;
                    a.coop_iters += (sum + 63) / 64;
                    std::sort(cells.begin(), cells.end());
                    cells.erase(std::unique(cells.begin(), cells.end()), cells.end());
                    a.distinct_sum += cells.size();
                    uint32_t di = 0;
                    for (auto& c : cells) di += c.second;
                    a.dist_iters += di;
                    const int b = int(10.0 * sum / (64.0 * mx));
                    a.hist_util[b]++; a.hist_util_w[b] += mx;
                }
                // VALU model of the item (per wave instruction counts of AUTO's loops):
                // outer DDA iteration ~35, bare empty-run step ~22, uniform record ~25, per-lane
                // list iteration ~35, ray setup + resolve ~150
                item_cost[item] = 150.0 + 35.0 * double(a.outer - a0.outer) + 22.0 * double(a.inner - a0.inner) +
                                  25.0 * double(a.uni_recs - a0.uni_recs) + 35.0 * double(a.lane_iters - a0.lane_iters);
            }
        });
    for (auto& t : pool) t.join();
    Acc a;
    for (auto& x : acc) a.add(x);
    std::printf("{\"waves\": %llu, \"wave_steps\": %llu, \"uniform_steps\": %llu, \"uniform_records\": %llu,\n",
                (unsigned long long)a.waves, (unsigned long long)a.steps, (unsigned long long)a.uni_steps,
                (unsigned long long)a.uni_recs);
    std::printf(" \"lane_steps\": %llu, \"lane_iterations\": %llu, \"lane_useful_tests\": %llu, \"lane_util\": %.4f,\n",
                (unsigned long long)a.lane_steps, (unsigned long long)a.lane_iters, (unsigned long long)a.lane_useful,
                double(a.lane_useful) / (64.0 * a.lane_iters));
    std::printf(" \"coop_iterations\": %llu, \"distinct_cells_per_lane_step\": %.2f, \"distinct_cell_iterations\": %llu,\n",
                (unsigned long long)a.coop_iters, double(a.distinct_sum) / a.lane_steps, (unsigned long long)a.dist_iters);
    std::printf(" \"outer_iterations\": %llu, \"inner_iterations\": %llu, \"outer_lane_util\": %.3f, \"inner_lane_util\": %.3f, \"word_loads_per_wave\": %.2f, \"empty_lane_steps_frac\": %.3f,\n",
                (unsigned long long)a.outer, (unsigned long long)a.inner, a.outer_lanes / (64.0 * a.outer),
                a.inner_lanes / (64.0 * a.inner), double(a.loads) / a.waves,
                double(a.empty_lane_steps) / (a.outer_lanes + a.inner_lanes));
    std::printf(" \"lane_steps_by_util_decile\": [");
    for (int i = 0; i < 11; i++) std::printf("%s%llu", i ? ", " : "", (unsigned long long)a.hist_util[i]);
    std::printf("],\n \"lane_iterations_by_util_decile\": [");
    for (int i = 0; i < 11; i++) std::printf("%s%llu", i ? ", " : "", (unsigned long long)a.hist_util_w[i]);
    std::printf("],\n \"shard_balance\": {");
    // per-rank modelled cost of tile-shard mappings: owner(tx, ty) = (ty * tiles_x + (tx + s * ty) mod
    // tiles_x) mod N, i.e. every tile row rotated by s columns per row before the t mod N deal
    // (s = 0: the plain t mod N), as max over ranks / mean
    std::vector<double> tile_cost(tiles_x * tiles_y, 0.0);
    for (uint32_t i = 0; i < nitems; i++) tile_cost[i / items_per_tile] += item_cost[i];
    const char *sep = "";
    for (uint32_t N : {2u, 4u, 8u})
    {
        std::printf("%s\"%u\": {", sep, N); sep = ", ";
        for (uint32_t sh = 0; sh < 8; sh++)
        {
            std::vector<double> r(N, 0.0);
            for (uint32_t ty = 0; ty < tiles_y; ty++)
                for (uint32_t tx = 0; tx < tiles_x; tx++)
                    r[(ty * tiles_x + (tx + sh * ty) % tiles_x) % N] += tile_cost[ty * tiles_x + tx];
            double mx = 0, sum = 0;
            for (double v : r) { mx = std::max(mx, v); sum += v; }
            std::printf("%s\"s%u\": %.4f", sh ? ", " : "", sh, mx / (sum / N));
        }
        std::printf("}");
    }
    std::printf("}}\n");
    return 0;
}
