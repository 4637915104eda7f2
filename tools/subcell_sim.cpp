// subcell_sim.cpp -- analysis only (links the oracle restatement; never part of the product): how
// many of a walk's record tests a conservative per-cell subdivision could skip.  Each cell with a
// list of >= Lmin references is split into S x S x S subcells; a reference "touches" a subcell when
// its triangle's bounding box overlaps the subcell box grown by a margin.  For every tested cell of
// the reference walk (grid.cpp:218-281, to its first hit) the ray segment [t_in - m, t_out] (t_out =
// the step's crossing, the reference's acceptance bound) is clipped against the subcells; only the
// references touching a crossed subcell would be tested.
//   g++ -O2 -std=c++11 -pthread -ffp-contract=off -I oracle tools/subcell_sim.cpp -o /tmp/subcell_sim
//   /tmp/subcell_sim data/scenes/scene8.rtscene 1920 1080 4 [S=4] [Lmin=16] [margin_cells=0.05]
#include "../oracle/cpu_tracer.cpp"

#include <algorithm>
#include <atomic>
#include <cstdio>

namespace {

struct SubMasks { uint32_t first = 0; };   // index into masks: S^3 * words per dense cell

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5) return 2;
    Scene s;
    if (!ReadScene(argv[1], s)) return 1;
    BuildGrid(s, 64);
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]);
    const int S = argc > 5 ? std::atoi(argv[5]) : 4;
    const uint32_t Lmin = argc > 6 ? std::atoi(argv[6]) : 16;
    const float mcell = argc > 7 ? float(std::atof(argv[7])) : 0.05f;
    const uint32_t nc = s.dim[0] * s.dim[1] * s.dim[2];
    const int S3 = S * S * S;
    // per dense cell: S^3 bit rows of ceil(len / 64) words
    std::vector<int64_t> base(nc, -1);
    std::vector<uint64_t> masks;
    const float cw = s.cell_wdh, sw = cw / float(S), gm = mcell * cw;
    for (uint32_t x = 0; x < s.dim[0]; x++)
        for (uint32_t y = 0; y < s.dim[1]; y++)
            for (uint32_t z = 0; z < s.dim[2]; z++)
            {
                const uint32_t c = s.GridIdx(x, y, z);
                const uint32_t len = s.off[c + 1] - s.off[c];
                if (len < Lmin) continue;
                const uint32_t nw = (len + 63) / 64;
                base[c] = int64_t(masks.size());
                masks.resize(masks.size() + size_t(S3) * nw, 0ull);
                const float cx = s.ToPos(int(x), 0), cy = s.ToPos(int(y), 1), cz = s.ToPos(int(z), 2);
                for (uint32_t i = 0; i < len; i++)
                {
                    const Triangle& t = s.tris[s.refs[s.off[c] + i]];
                    const V3 &a = s.verts[t.v0].p, &b = s.verts[t.v1].p, &d = s.verts[t.v2].p;
                    const float mn[3] = {std::min(a.x, std::min(b.x, d.x)), std::min(a.y, std::min(b.y, d.y)),
                                         std::min(a.z, std::min(b.z, d.z))};
                    const float mx[3] = {std::max(a.x, std::max(b.x, d.x)), std::max(a.y, std::max(b.y, d.y)),
                                         std::max(a.z, std::max(b.z, d.z))};
                    const float org[3] = {cx, cy, cz};
                    for (int q = 0; q < S3; q++)
                    {
                        const int sx = q % S, sy = (q / S) % S, sz = q / (S * S);
                        const int si[3] = {sx, sy, sz};
                        bool ov = true;
                        for (int k = 0; k < 3 && ov; k++)
                        {
                            const float lo = org[k] + float(si[k]) * sw - gm, hi = org[k] + float(si[k] + 1) * sw + gm;
                            ov = mx[k] >= lo && mn[k] <= hi;
                        }
                        if (ov) masks[size_t(base[c]) + size_t(q) * nw + i / 64] |= 1ull << (i % 64);
                    }
                }
            }
    const std::vector<float> smp = Hammersley(spp);
    std::atomic<uint32_t> next(0);
    std::atomic<uint64_t> t_full(0), t_cull(0), t_dense_full(0), rays(0);
    std::vector<std::vector<uint32_t>> per_ray_full(std::max(1u, std::thread::hardware_concurrency())),
        per_ray_cull(per_ray_full.size());
    std::vector<std::thread> pool;
    for (uint32_t th = 0; th < per_ray_full.size(); th++)
        pool.emplace_back([&, th]() {
            uint64_t f_ = 0, c_ = 0, d_ = 0, r_ = 0;
            std::vector<uint64_t> acc;
            for (;;)
            {
                const uint32_t y = next.fetch_add(1);
                if (y >= H) break;
                for (uint32_t x = 0; x < W; x++)
                    for (uint32_t si = 0; si < spp; si++)
                    {
                        V3 o, d;
                        GenRay(s.cam, x, y, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
                        r_++;
                        float enter_t, leave_t;
                        V3 g;
                        if (PointAABB(o, s.aabb_min, s.aabb_max)) { enter_t = 0.0f; g = o; }
                        else if (RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t))
                            g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
                        else { per_ray_full[th].push_back(0); per_ray_cull[th].push_back(0); continue; }
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
                        float t = std::numeric_limits<float>::max(), t_in = enter_t;
                        uint32_t rf = 0, rc = 0;
                        for (;;)
                        {
                            const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
                            const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
                            const uint32_t k0 = s.off[cell], k1 = s.off[cell + 1], len = k1 - k0;
                            rf += len;
                            if (base[cell] < 0) rc += len;
                            else
                            {
                                d_ += len;
                                // subcells crossed by [t_in - m, t_out] (slab test per subcell)
                                const uint32_t nw = (len + 63) / 64;
                                acc.assign(nw, 0ull);
                                const float ta = std::max(0.0f, t_in - gm), tb = nct[ax];
                                const float org[3] = {s.ToPos(pos[0], 0), s.ToPos(pos[1], 1), s.ToPos(pos[2], 2)};
                                const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
                                for (int q = 0; q < S3; q++)
                                {
                                    const int sidx[3] = {q % S, (q / S) % S, q / (S * S)};
                                    float lo = ta, hi = tb;
                                    for (int k = 0; k < 3 && lo <= hi; k++)
                                    {
                                        const float bl = org[k] + float(sidx[k]) * sw - gm, bh = org[k] + float(sidx[k] + 1) * sw + gm;
                                        if (dd[k] == 0.0f) { if (oo[k] < bl || oo[k] > bh) hi = -1.0f; continue; }
                                        float t0 = (bl - oo[k]) / dd[k], t1 = (bh - oo[k]) / dd[k];
                                        if (t0 > t1) std::swap(t0, t1);
                                        lo = std::max(lo, t0);
                                        hi = std::min(hi, t1);
                                    }
                                    if (lo <= hi)
                                        for (uint32_t w = 0; w < nw; w++) acc[w] |= masks[size_t(base[cell]) + size_t(q) * nw + w];
                                }
                                for (uint32_t w = 0; w < nw; w++) rc += uint32_t(__builtin_popcountll(acc[w]));
                            }
                            for (uint32_t k = k0; k < k1; k++)
                            {
                                const Triangle& tr = s.tris[s.refs[k]];
                                float ct, cu, cv;
                                if (RayTri(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p, ct, cu, cv) && ct < t &&
                                    ct < nct[ax])
                                    t = ct;
                            }
                            if (t != std::numeric_limits<float>::max()) break;
                            pos[ax] += step[ax];
                            if (pos[ax] == out[ax]) break;
                            t_in = nct[ax];
                            nct[ax] += dt[ax];
                        }
                        f_ += rf;
                        c_ += rc;
                        per_ray_full[th].push_back(rf);
                        per_ray_cull[th].push_back(rc);
                    }
            }
            t_full += f_; t_cull += c_; t_dense_full += d_; rays += r_;
        });
    for (auto& t : pool) t.join();
    std::vector<uint32_t> F, C;
    for (size_t i = 0; i < per_ray_full.size(); i++)
    {
        F.insert(F.end(), per_ray_full[i].begin(), per_ray_full[i].end());
        C.insert(C.end(), per_ray_cull[i].begin(), per_ray_cull[i].end());
    }
    std::vector<size_t> idx(F.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return F[a] > F[b]; });
    uint64_t tf = 0, tc = 0;
    const size_t top = idx.size() / 100;
    for (size_t i = 0; i < top; i++) { tf += F[idx[i]]; tc += C[idx[i]]; }
    std::printf("{\"scene\": \"%s\", \"S\": %d, \"Lmin\": %u, \"margin_cells\": %.3f, \"mask_MB\": %.1f, "
                "\"tests_per_ray\": %.2f, \"culled_per_ray\": %.2f, \"dense_share\": %.3f, \"top1pct_tests\": %.1f, "
                "\"top1pct_culled\": %.1f}\n",
                argv[1], S, Lmin, mcell, masks.size() * 8.0 / 1e6, double(t_full) / rays, double(t_cull) / rays,
                double(t_dense_full) / std::max<uint64_t>(1, t_full), double(tf) / top, double(tc) / top);
}
