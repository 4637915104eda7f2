// lane_run_check.cpp -- analysis only (links the oracle restatement; never part of the product):
// the per-lane box-run jump of grid_intersect (RT_LANE_RUNS, csrc/rt_tracer.hip) replayed on the CPU
// in the kernel's own f32 arithmetic, for every sample of a frame, against the reference's cell by
// cell walk (grid.cpp:218-281 as the oracle restates it).  Hits are ignored on both sides, so every
// walk runs to the grid's exit: the (cell, crossing t) of every non-empty cell a walk tests and the
// last cell must agree exactly.  Also counts the jump's work (crossings taken by the add chains,
// bare steps after them) per walk.
// A second mode walks random rays: origins inside and around the grid, directions with zeroed,
// tiny (1e-30) and near-axis components.  tests/test_lane_runs.py runs both.
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tests/lane_run_check.cpp -o /tmp/lane_run_check
//   /tmp/lane_run_check data/scenes/scene8.rtscene 1920 1080 4
//   /tmp/lane_run_check data/scenes/scene8.rtscene random 2000000 7
// A fifth argument 'shrink' replaces each jump's bound by a random value between the lane's next
// crossing and the bound (a wave's lower bound: RT_LANE_RUNS 2 and 4).
#include "../oracle/cpu_tracer.cpp"
#include "../cpp-11-ray-trace-march-framework_amd/csrc/rt_box_words.h"

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace {

struct Ev { uint32_t cell; float t; };

constexpr uint32_t kGuards = (1u << 10) | (1u << 21) | (1u << 31);

// per-axis DDA setup as walk() in tools/box_sim.cpp (grid.cpp:174-216)
bool setup(const Scene& s, const V3 o, const V3 d, float nct[3], float dt[3], int pos[3], int step[3], int out[3])
{
    float enter_t, leave_t;
    V3 g;
    if (PointAABB(o, s.aabb_min, s.aabb_max)) { enter_t = 0.0f; g = o; }
    else if (RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t))
        g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
    else return false;
    for (int ax = 0; ax < 3; ax++)
    {
        pos[ax] = s.ToVoxel(g, ax);
        dt[ax] = 0.0f; step[ax] = 0; out[ax] = 0;
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
    return true;
}

// the reference's walk, every non-empty cell tested, to the grid's exit
void ref_walk(const Scene& s, const V3 o, const V3 d, std::vector<Ev>& ev, uint32_t& last)
{
    ev.clear(); last = ~0u;
    float nct[3], dt[3]; int pos[3], step[3], out[3];
    if (!setup(s, o, d, nct, dt, pos, step, out)) return;
    for (;;)
    {
        const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
        const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
        if (s.off[cell + 1] != s.off[cell]) ev.push_back({cell, nct[ax]});
        last = cell;
        pos[ax] += step[ax];
        if (pos[ax] == out[ax]) break;
        nct[ax] += dt[ax];
    }
}

// AUTO's box-run walk with the per-lane jump, as grid_intersect writes it
void lane_walk(const Scene& s, const std::vector<uint32_t>& boxw_all, const V3 o, const V3 d, std::vector<Ev>& ev,
               uint32_t& last, uint64_t& taken, uint64_t& bare, uint64_t& runs, bool shrink, uint64_t& rng)
{
    ev.clear(); last = ~0u;
    float nct[3], dt[3]; int pos[3], step[3], out[3];
    if (!setup(s, o, d, nct, dt, pos, step, out)) return;
    const uint32_t nc = s.dim[0] * s.dim[1] * s.dim[2];
    const int dxdz = int(s.dim[0] * s.dim[2]);
    int rem[3], cs[3];
    const int stride[3] = {1, dxdz, int(s.dim[0])};
    for (int a = 0; a < 3; a++)
    {
        rem[a] = step[a] > 0 ? int(s.dim[a]) - 1 - pos[a] : (step[a] < 0 ? pos[a] : 0);
        cs[a] = step[a] > 0 ? stride[a] : (step[a] < 0 ? -stride[a] : 0);
    }
    int cell = int(s.GridIdx(pos[0], pos[1], pos[2]));
    const uint32_t oct = uint32_t(d.x < 0.0f) | (uint32_t(d.y < 0.0f) << 1) | (uint32_t(d.z < 0.0f) << 2);
    const float ax_ = std::fabs(d.x), ay_ = std::fabs(d.y), az_ = std::fabs(d.z);
    const uint32_t maj = (ax_ >= ay_ && ax_ >= az_) ? 0u : (ay_ >= az_ ? 1u : 2u);
    const uint32_t *bw = boxw_all.data() + size_t(oct * 3u + maj) * nc;
    uint32_t remp = uint32_t(rem[0] | (rem[1] << 11) | (rem[2] << 22));
    uint32_t boxw = kGuards;
    auto step_box = [&](float& nct_ax, bool with_cell) {
        const float m = std::fmin(std::fmin(nct[0], nct[1]), nct[2]);
        const bool a2 = nct[2] == m, a1 = !a2 && nct[1] == m, a0 = !a2 && !a1;
        nct_ax = m;
        const uint32_t u = a2 ? (1u << 22) : (a1 ? (1u << 11) : 1u);
        boxw -= u;
        if (with_cell) { remp -= u; cell += a2 ? cs[2] : (a1 ? cs[1] : cs[0]); }
        nct[0] += a0 ? dt[0] : 0.0f;
        nct[1] += a1 ? dt[1] : 0.0f;
        nct[2] += a2 ? dt[2] : 0.0f;
    };
    for (int guard = 0; guard < 1 << 20; guard++)
    {
        uint32_t kb = 0, ke = 0;
        if (boxw & kGuards)
        {
            const uint32_t w = bw[uint32_t(cell)];
            const uint32_t ne = uint32_t(int32_t(w) >> 31);
            kb = (w >> 11) & 0xFFFFFu;
            ke = kb + (w & ne & 2047u);
            boxw = w & ~ne;
        }
        const uint32_t cur = uint32_t(cell);
        float nct_ax;
        step_box(nct_ax, true);
        bool more = (remp & kGuards) == 0;
        if (kb < ke) ev.push_back({cur, nct_ax});
        if ((boxw & kGuards) == 0u)
        {
            runs++;
            const uint32_t b0 = boxw;
            const int f[3] = {int(boxw & 1023u), int((boxw >> 11) & 1023u), int(boxw >> 22)};
            float lo[3];
            for (int a = 0; a < 3; a++)
            {
                const float e = std::fma(float(f[a]), dt[a], nct[a]), k = float(f[a] + 2) * 1.1920928955078125e-7f;
                lo[a] = e - std::fma(std::fabs(nct[a]), k, std::fabs(e) * k);
            }
            float tl = std::fmin(std::fmin(lo[0], lo[1]), lo[2]);
            if (shrink)
            {
                // a wave's lower bound (time-synchronised runs) is any T <= tl: pull tl down
                // towards the lane's next crossing by a pseudo-random fraction
                rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                const float fr = float(rng >> 40) * (1.0f / 16777216.0f);
                const float m = std::fmin(std::fmin(nct[0], nct[1]), nct[2]);
                if (tl > m) tl = tl - fr * (tl - m);
            }
            int c[3] = {0, 0, 0};
            for (int a = 0; a < 3; a++)
                while (nct[a] < tl && c[a] < f[a]) { nct[a] += dt[a]; c[a]++; }
            taken += uint64_t(c[0] + c[1] + c[2]);
            boxw -= uint32_t(c[0]) + (uint32_t(c[1]) << 11) + (uint32_t(c[2]) << 22);
            do { float x; step_box(x, false); bare++; } while ((boxw & kGuards) == 0u);
            const uint32_t dd = b0 - boxw;
            remp -= dd;
            cell += int(dd & 2047u) * cs[0] + int((dd >> 11) & 2047u) * cs[1] + int(dd >> 22) * cs[2];
            more = (remp & kGuards) == 0;
        }
        if (!more) break;
    }
    // exit_voxel: the exit step borrowed into the lowest set guard; cell includes that step
    const uint32_t g = remp & kGuards;
    last = uint32_t(cell - ((g & (1u << 10)) ? cs[0] : ((g & (1u << 21)) ? cs[1] : cs[2])));
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5) { std::fprintf(stderr, "usage: lane_run_check scene.rtscene (W H spp | random N seed) [shrink]\n"); return 2; }
    Scene s;
    if (!ReadScene(argv[1], s)) return 1;
    BuildGrid(s, 64);
    std::vector<uint32_t> boxw;
    rtbox::build_box_words(s.off.data(), s.dim, boxw, rtbox::kBoxRatio, rtbox::kBoxExtend, rtbox::kBoxGrow);
    const bool rnd = std::strcmp(argv[2], "random") == 0;
    const bool shrink = argc > 5 && std::strcmp(argv[5], "shrink") == 0;   // T = any bound <= tl
    const uint32_t W = rnd ? 1024u : uint32_t(std::atoi(argv[2])), spp = rnd ? 1u : uint32_t(std::atoi(argv[4]));
    const uint32_t H = rnd ? uint32_t((std::strtoull(argv[3], nullptr, 10) + 1023) / 1024) : uint32_t(std::atoi(argv[3]));
    const uint64_t seed = rnd ? std::strtoull(argv[4], nullptr, 10) : 0;
    // random rays: row y, column x -> a splitmix64 stream
    auto rnd_ray = [&](uint32_t x, uint32_t y, V3& o, V3& d) {
        uint64_t st = seed * 0x9E3779B97F4A7C15ull + (uint64_t(y) << 20) + x;
        auto next = [&]() {
            uint64_t z = (st += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            return z ^ (z >> 31);
        };
        auto uni = [&]() { return float(next() >> 40) * (1.0f / 16777216.0f); };
        float p[3], v[3];
        const float lo[3] = {s.aabb_min.x, s.aabb_min.y, s.aabb_min.z}, hi[3] = {s.aabb_max.x, s.aabb_max.y, s.aabb_max.z};
        const bool inside = (next() & 1) != 0;
        for (int a = 0; a < 3; a++)
        {
            const float ext = hi[a] - lo[a];
            p[a] = inside ? lo[a] + uni() * ext : lo[a] - ext + uni() * 3.0f * ext;
            v[a] = uni() * 2.0f - 1.0f;
        }
        const uint64_t k = next();
        const int a = int(k % 3u);
        switch ((k >> 8) & 7u)
        {
        case 0: v[a] = 0.0f; break;                                   // still axis
        case 1: v[a] = 0.0f; v[(a + 1) % 3] = 0.0f; break;            // axis-aligned
        case 2: v[a] = (k & 0x10000u) ? 1e-30f : -1e-30f; break;      // tiny component
        case 3: v[a] *= 1e-4f; v[(a + 1) % 3] *= 1e-4f; break;        // near an axis
        default: break;
        }
        if (v[0] == 0.0f && v[1] == 0.0f && v[2] == 0.0f) v[0] = 1.0f;
        o = mk(p[0], p[1], p[2]);
        const float n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        d = mk(v[0] / n, v[1] / n, v[2] / n);
    };
    const std::vector<float> smp = Hammersley(spp);
    const uint32_t nth = std::max(1u, std::thread::hardware_concurrency());
    std::atomic<uint32_t> next(0);
    std::atomic<uint64_t> bad(0), rays(0), events(0), taken(0), bare(0), runs(0);
    std::vector<std::thread> pool;
    for (uint32_t th = 0; th < nth; th++)
        pool.emplace_back([&]() {
            std::vector<Ev> a, b;
            uint64_t tk = 0, br = 0, rn = 0, nr = 0, ne = 0, nb = 0, rng = 0x243F6A8885A308D3ull;
            for (;;)
            {
                const uint32_t y = next.fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; x++)
                    for (uint32_t si = 0; si < spp; si++)
                    {
                        V3 o, d;
                        if (rnd) rnd_ray(x, y, o, d);
                        else GenRay(s.cam, x, y, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
                        uint32_t la, lb;
                        ref_walk(s, o, d, a, la);
                        lane_walk(s, boxw, o, d, b, lb, tk, br, rn, shrink, rng);
                        nr++;
                        ne += a.size();
                        bool ok = a.size() == b.size();
                        for (size_t i = 0; ok && i < a.size(); i++)
                            ok = a[i].cell == b[i].cell && std::memcmp(&a[i].t, &b[i].t, 4) == 0;
                        if (ok && lb != la) ok = false;
                        if (!ok && nb++ < 5)
                            std::fprintf(stderr, "mismatch x=%u y=%u s=%u: %zu vs %zu events, last %u vs %u\n", x, y, si,
                                         a.size(), b.size(), la, lb);
                    }
            }
            bad += nb; rays += nr; events += ne; taken += tk; bare += br; runs += rn;
        });
    for (auto& t : pool) t.join();
    std::printf("{\"scene\": \"%s\", \"rays\": %llu, \"tested_cells\": %llu, \"mismatches\": %llu, \"runs_per_ray\": %.3f, "
                "\"chain_steps_per_ray\": %.3f, \"bare_steps_per_run\": %.4f}\n", argv[1],
                (unsigned long long)rays.load(), (unsigned long long)events.load(), (unsigned long long)bad.load(),
                double(runs) / rays, double(taken) / rays, double(bare) / std::max<uint64_t>(1, runs));
    return bad ? 1 : 0;
}
