// box_words_check.cpp -- CPU check of AUTO's box-run words (csrc/rt_box_words.h), test
// infrastructure only: the scene's grid comes from the oracle's Grid::Grid restatement (pinned to
// the reference's CSR by tests/test_oracle_golden.py).  For every one of the 24 copies (ray octant
// x major axis) and every cell:
//   * a non-empty cell's word is 0x80000000 | start << 11 | count of its CSR range;
//   * an empty cell's word has bit 31 and the guard bits 10 / 21 clear, and its box -- E0 x E1 x E2
//     cells with the corner at the cell, extending along the octant's signs -- lies inside the grid
//     (the kernel's box runs rely on it to see the grid exit) and holds no non-empty cell (3-D
//     prefix sums of the occupancy).
// Prints "cells <checked> empty <empty cells> mean_box_volume <cells>" and exits 1 on the first
// violation.
//   g++ -O2 -std=c++11 -pthread -I oracle tests/box_words_check.cpp -o box_words_check
//   ./box_words_check data/scenes/scene8.rtscene
#include "../oracle/cpu_tracer.cpp"
#include "../cpp-11-ray-trace-march-framework_amd/csrc/rt_box_words.h"

#include <cstdio>

int main(int argc, char **argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: box_words_check scene.rtscene\n"); return 2; }
    Scene s;
    if (!ReadScene(argv[1], s)) { std::fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }
    BuildGrid(s, 64);
    const int D[3] = { int(s.dim[0]), int(s.dim[1]), int(s.dim[2]) };
    const uint32_t nc = s.dim[0] * s.dim[1] * s.dim[2];
    std::vector<uint32_t> w;
    if (!rtbox::build_box_words(s.off.data(), s.dim, w)) { std::fprintf(stderr, "build failed\n"); return 1; }
    if (w.size() != size_t(24) * nc) { std::fprintf(stderr, "size %zu\n", w.size()); return 1; }
    // occupancy prefix sums P[x][y][z] over [0, x) x [0, y) x [0, z)
    auto pidx = [&](int x, int y, int z) { return (size_t(x) * (D[1] + 1) + y) * (D[2] + 1) + z; };
    std::vector<uint32_t> P(size_t(D[0] + 1) * (D[1] + 1) * (D[2] + 1), 0u);
    for (int x = 1; x <= D[0]; x++)
        for (int y = 1; y <= D[1]; y++)
            for (int z = 1; z <= D[2]; z++)
            {
                const uint32_t c = s.GridIdx(uint32_t(x - 1), uint32_t(y - 1), uint32_t(z - 1));
                const uint32_t occ = s.off[c + 1] != s.off[c] ? 1u : 0u;
                P[pidx(x, y, z)] = occ + P[pidx(x - 1, y, z)] + P[pidx(x, y - 1, z)] + P[pidx(x, y, z - 1)] -
                                   P[pidx(x - 1, y - 1, z)] - P[pidx(x - 1, y, z - 1)] - P[pidx(x, y - 1, z - 1)] +
                                   P[pidx(x - 1, y - 1, z - 1)];
            }
    auto occupied = [&](const int lo[3], const int hi[3]) {       // cells in [lo, hi) (inclusive-exclusive)
        const int64_t v = int64_t(P[pidx(hi[0], hi[1], hi[2])]) - P[pidx(lo[0], hi[1], hi[2])] - P[pidx(hi[0], lo[1], hi[2])] -
                          P[pidx(hi[0], hi[1], lo[2])] + P[pidx(lo[0], lo[1], hi[2])] + P[pidx(lo[0], hi[1], lo[2])] +
                          P[pidx(hi[0], lo[1], lo[2])] - P[pidx(lo[0], lo[1], lo[2])];
        return v;
    };
    uint64_t checked = 0, vol = 0, empties = 0;
    for (uint32_t o = 0; o < 8; o++)
        for (uint32_t m = 0; m < 3; m++)
        {
            const uint32_t *cw = w.data() + size_t(o * 3u + m) * nc;
            const int sg[3] = { (o & 1) ? -1 : 1, (o & 2) ? -1 : 1, (o & 4) ? -1 : 1 };
            for (int y = 0; y < D[1]; y++)
                for (int z = 0; z < D[2]; z++)
                    for (int x = 0; x < D[0]; x++)
                    {
                        const uint32_t c = s.GridIdx(uint32_t(x), uint32_t(y), uint32_t(z));
                        const uint32_t word = cw[c];
                        checked++;
                        if (s.off[c + 1] != s.off[c])
                        {
                            const uint32_t want = 0x80000000u | (s.off[c] << 11) | (s.off[c + 1] - s.off[c]);
                            if (word != want)
                            {
                                std::fprintf(stderr, "copy %u cell %u: word %08x, want %08x\n", o * 3 + m, c, word, want);
                                return 1;
                            }
                            continue;
                        }
                        if (word & 0x80200400u)
                        {
                            std::fprintf(stderr, "copy %u empty cell %u: word %08x has flag/guard bits\n", o * 3 + m, c, word);
                            return 1;
                        }
                        const int E[3] = { int(word & 1023u) + 1, int((word >> 11) & 1023u) + 1, int((word >> 22) & 511u) + 1 };
                        const int p[3] = { x, y, z };
                        int lo[3], hi[3];
                        for (int a = 0; a < 3; a++)
                        {
                            const int far = p[a] + sg[a] * (E[a] - 1);
                            if (far < 0 || far >= D[a])
                            {
                                std::fprintf(stderr, "copy %u cell (%d,%d,%d): box leaves the grid along axis %d\n",
                                             o * 3 + m, x, y, z, a);
                                return 1;
                            }
                            lo[a] = std::max(0, std::min(p[a], far));
                            hi[a] = std::min(D[a], std::max(p[a], far) + 1);
                        }
                        if (occupied(lo, hi) != 0)
                        {
                            std::fprintf(stderr, "copy %u cell (%d,%d,%d): box %dx%dx%d holds a non-empty cell\n", o * 3 + m,
                                         x, y, z, E[0], E[1], E[2]);
                            return 1;
                        }
                        empties++;
                        vol += uint64_t(E[0]) * E[1] * E[2];
                    }
        }
    std::printf("cells %llu empty %llu mean_box_volume %.2f\n", (unsigned long long)checked,
                (unsigned long long)empties, empties ? double(vol) / empties : 0.0);
    return 0;
}
