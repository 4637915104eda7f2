// walk_stats.cpp -- analysis only (links the oracle restatement; never part of the product):
// where a scene's ray/triangle tests go at a given frame size, to decide what a faster exact
// treatment of the heavy samples could save.
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tools/walk_stats.cpp -o /tmp/walk_stats
//   /tmp/walk_stats data/scenes/scene8.rtscene 1920 1080 4
// Per sample it re-walks Grid::Intersect (grid.cpp:159-281, as oracle IntersectT) and reports:
//   tests by the length of the cell list they come from; tests of a triangle already tested
//   earlier in the same walk (what mailboxing would skip) and how many of those were misses;
//   first-half passes (det outside +-1e-8 and u in [0,1], triangle.h:41-70); the share of the
//   tests done by the samples above a per-sample test budget.
#include "../oracle/cpu_tracer.cpp"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <unordered_map>

namespace {

struct Acc
{
    uint64_t samples = 0, tests = 0, dup = 0, dup_miss = 0, first_pass = 0, hits = 0;
    uint64_t by_len[6] = {0, 0, 0, 0, 0, 0};        // list length <16, <64, <128, <256, <512, >=512
    uint64_t heavy_samples[4] = {0, 0, 0, 0};        // > 64, 128, 256, 512 tests
    uint64_t heavy_tests[4] = {0, 0, 0, 0};
    uint64_t heavy_cells = 0;                        // cells with list >= 128 visited by samples > 128 tests
    uint64_t steps = 0;
    void add(const Acc& o)
    {
        samples += o.samples; tests += o.tests; dup += o.dup; dup_miss += o.dup_miss;
        first_pass += o.first_pass; hits += o.hits; steps += o.steps; heavy_cells += o.heavy_cells;
        for (int i = 0; i < 6; i++) by_len[i] += o.by_len[i];
        for (int i = 0; i < 4; i++) { heavy_samples[i] += o.heavy_samples[i]; heavy_tests[i] += o.heavy_tests[i]; }
    }
};

bool first_half(const V3& o, const V3& d, const V3& v0, const V3& v1, const V3& v2)
{
    const V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const V3 pv = mk(d.y * e2.z - d.z * e2.y, d.z * e2.x - d.x * e2.z, d.x * e2.y - d.y * e2.x);
    const float det = e1.x * pv.x + e1.y * pv.y + e1.z * pv.z;
    if (det > -0.00000001f && det < 0.00000001f) return false;
    const float inv_det = 1.0f / det;
    const V3 tv = sub(o, v0);
    const float u = (tv.x * pv.x + tv.y * pv.y + tv.z * pv.z) * inv_det;
    return !(u < 0.0f || u > 1.0f);
}

void walk(const Scene& s, const V3 o, const V3 d, Acc& a)
{
    float enter_t, leave_t;
    V3 g;
    if (PointAABB(o, s.aabb_min, s.aabb_max)) { enter_t = 0.0f; g = o; }
    else if (RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t))
        g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
    else { a.samples++; return; }
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
    std::unordered_map<uint32_t, bool> seen;       // triangle -> hit (any) when first tested
    float t = std::numeric_limits<float>::max();
    uint32_t tests = 0, heavy_cells = 0;
    Acc loc;
    while (true)
    {
        const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
        const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
        loc.steps++;
        const uint32_t k0 = s.off[cell], k1 = s.off[cell + 1], len = k1 - k0;
        const int bin = len < 16 ? 0 : len < 64 ? 1 : len < 128 ? 2 : len < 256 ? 3 : len < 512 ? 4 : 5;
        if (len >= 128) heavy_cells++;
        for (uint32_t k = k0; k < k1; k++)
        {
            const uint32_t ci = s.refs[k];
            const Triangle& tr = s.tris[ci];
            float ct, cu, cv;
            tests++;
            loc.by_len[bin]++;
            const bool hit = RayTri(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p, ct, cu, cv);
            if (first_half(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p)) loc.first_pass++;
            auto it = seen.find(ci);
            if (it != seen.end()) { loc.dup++; if (!it->second) loc.dup_miss++; }
            else seen[ci] = hit;
            if (hit && ct < t && ct < nct[ax]) t = ct;
        }
        if (t != std::numeric_limits<float>::max()) { loc.hits++; break; }
        pos[ax] += step[ax];
        if (pos[ax] == out[ax]) break;
        nct[ax] += dt[ax];
    }
    loc.samples = 1;
    loc.tests = tests;
    const uint32_t lim[4] = {64, 128, 256, 512};
    for (int i = 0; i < 4; i++)
        if (tests > lim[i]) { loc.heavy_samples[i] = 1; loc.heavy_tests[i] = tests; }
    if (tests > 128) loc.heavy_cells = heavy_cells;
    a.add(loc);
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5) { std::fprintf(stderr, "usage: walk_stats scene.rtscene W H spp [stride]\n"); return 2; }
    Scene s;
    if (!ReadScene(argv[1], s)) { std::fprintf(stderr, "cannot read %s\n", argv[1]); return 1; }
    BuildGrid(s, 64);                                        // as orc_scene_load
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]);
    const uint32_t stride = argc > 5 ? std::atoi(argv[5]) : 1;   // every stride-th row
    const std::vector<float> smp = Hammersley(spp);
    const uint32_t nth = std::max(1u, std::thread::hardware_concurrency());
    std::vector<Acc> acc(nth);
    std::atomic<uint32_t> next(0);
    std::vector<std::thread> pool;
    for (uint32_t i = 0; i < nth; i++)
        pool.emplace_back([&, i]() {
            for (;;)
            {
                const uint32_t y = stride * next.fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; x++)
                    for (uint32_t si = 0; si < spp; si++)
                    {
                        V3 o, d;
                        GenRay(s.cam, x, y, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
                        walk(s, o, d, acc[i]);
                    }
            }
        });
    for (auto& th : pool) th.join();
    Acc a;
    for (const auto& x : acc) a.add(x);
    const double T = double(a.tests);
    std::printf("{\"samples\": %llu, \"tests_per_sample\": %.3f, \"steps_per_sample\": %.3f,\n",
                (unsigned long long)a.samples, T / a.samples, double(a.steps) / a.samples);
    std::printf(" \"dup_frac\": %.4f, \"dup_miss_frac\": %.4f, \"first_half_pass_frac\": %.4f,\n",
                a.dup / T, a.dup_miss / T, a.first_pass / T);
    std::printf(" \"tests_by_list_len\": {\"<16\": %.4f, \"<64\": %.4f, \"<128\": %.4f, \"<256\": %.4f, \"<512\": %.4f, \">=512\": %.4f},\n",
                a.by_len[0] / T, a.by_len[1] / T, a.by_len[2] / T, a.by_len[3] / T, a.by_len[4] / T, a.by_len[5] / T);
    std::printf(" \"heavy\": {");
    const uint32_t lim[4] = {64, 128, 256, 512};
    for (int i = 0; i < 4; i++)
        std::printf("%s\">%u\": {\"sample_frac\": %.4f, \"test_frac\": %.4f}", i ? ", " : "", lim[i],
                    double(a.heavy_samples[i]) / a.samples, a.heavy_tests[i] / T);
    std::printf("},\n \"heavy128_cells_ge128_per_sample\": %.2f}\n",
                a.heavy_samples[1] ? double(a.heavy_cells) / a.heavy_samples[1] : 0.0);
    return 0;
}
