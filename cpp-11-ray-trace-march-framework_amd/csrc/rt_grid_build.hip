// rt_grid_build.hip -- GPU restatement of Grid::Grid (grid.cpp:12-154) for gfx950.
//
// The reference voxelizes sequentially: for every triangle in index order, every cell of the
// triangle's AABB cell range (grid.cpp:77-92) gets an exact double-precision tri/box SAT test
// (aabb.h:15-32 -> aabb_tri_internal.h:112-186) and a push_back of the triangle index, so every
// cell's list ends up in ascending triangle order.  Here, on one stream:
//   K1 k_tri_ranges   one lane per triangle: cell range (same float arithmetic) -> candidates
//   exclusive scan (64-bit out) -> each triangle's first candidate
//   K2 k_candidates   one lane per (triangle, candidate cell): cell bounds in float, SAT in
//                     double; an overlap appends key = cell << tb | triangle (atomic counter,
//                     any order: the keys are distinct)
//   LSD radix sort of the keys over tb + cb bits, 8 bits a pass: (cell, triangle) order IS the
//                     reference's per-cell push_back order
//   K3 k_offsets      one lane per cell: CSR offset = lower_bound(keys, cell << tb); one lane
//                     per reference: triangle = key & (2^tb - 1)
// The scan and the sort are this file's own (k_scan_*, k_rs_*): a few hundred lines instead of
// rocPRIM's template instantiations (round 6: 2.8 MB of the library's object code).
// The grid AABB / cell size / dims (grid.cpp:18-41, mesh.cpp:112-134) are O(triangles) and are
// computed on the host exactly as the reference does (float::min() seed, hazard H11).
// Bit-exactness vs the reference's CSR: tests/test_gpu_grid.py.
#include <cstring>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <string>
#include <vector>

#include "../../include/rt_tracer.h"
#include "rt_internal.h"

namespace {

struct GridParams
{
    float bmin[3];
    float cw;
    uint32_t dims[3];
    uint32_t nt;
    uint32_t tb;              // bits of the triangle field of a key
};

// std::min / std::max argument order of the reference (triangle.h:116-131)
__device__ __forceinline__ float min_ref(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float max_ref(float a, float b) { return (a < b) ? b : a; }

// K1: TriangleAABB (seeded with float max / float::min()) relative to the grid, grid.cpp:77-92
__global__ void __launch_bounds__(256) k_tri_ranges(GridParams G, const rt_vertex *__restrict__ verts,
                                                     const rt_triangle *__restrict__ tris, uint4 *range_lo,
                                                     uint4 *range_hi, uint32_t *count)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= G.nt) return;
    const rt_triangle tr = tris[t];
    const float *p0 = verts[tr.v0].p, *p1 = verts[tr.v1].p, *p2 = verts[tr.v2].p;
    uint32_t st[3], en[3];
#pragma unroll
    for (int a = 0; a < 3; a++)
    {
        const float mn = min_ref(min_ref(min_ref(3.402823466e+38f, p0[a]), p1[a]), p2[a]) - G.bmin[a];
        const float mx = max_ref(max_ref(max_ref(1.175494351e-38f, p0[a]), p1[a]), p2[a]) - G.bmin[a];
        st[a] = uint32_t((long long)(mn / G.cw));          // uint(float), grid.cpp:81-92
        en[a] = uint32_t((long long)(mx / G.cw));
    }
    range_lo[t] = make_uint4(st[0], st[1], st[2], 0);
    range_hi[t] = make_uint4(en[0], en[1], en[2], 0);
    count[t] = (en[0] - st[0] + 1) * (en[1] - st[1] + 1) * (en[2] - st[2] + 1);
}

// aabb_tri_internal.h:42-63 planeBoxOverlap
__device__ __forceinline__ bool plane_box(const double n[3], double d, const double h[3])
{
    double vmin[3], vmax[3];
#pragma unroll
    for (int q = 0; q < 3; q++)
    {
        if (n[q] > 0.0f) { vmin[q] = -h[q]; vmax[q] = h[q]; }
        else             { vmin[q] = h[q];  vmax[q] = -h[q]; }
    }
    if (n[0] * vmin[0] + n[1] * vmin[1] + n[2] * vmin[2] + d > 0.0f) return false;
    return n[0] * vmax[0] + n[1] * vmax[1] + n[2] * vmax[2] + d >= 0.0f;
}

// One separating-axis test of the AXISTEST_* macros (aabb_tri_internal.h:67-110); the Z12
// form orders with (p2 < p1), the others with (p0 < p2): identical except for NaN.
__device__ __forceinline__ bool separated(double pa, double pb, double rad, bool z12)
{
    double mn, mx;
    if (z12) { if (pb < pa) { mn = pb; mx = pa; } else { mn = pa; mx = pb; } }
    else     { if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; } }
    return mn > rad || mx < -rad;
}

// aabb_tri_internal.h:112-186 triBoxOverlap in double, the reference's operation order
__device__ bool tri_box_overlap(const double c[3], const double h[3], const float *p0, const float *p1,
                                const float *p2)
{
    double v0[3], v1[3], v2[3], e0[3], e1[3], e2[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
    {
        v0[i] = double(p0[i]) - c[i];
        v1[i] = double(p1[i]) - c[i];
        v2[i] = double(p2[i]) - c[i];
    }
#pragma unroll
    for (int i = 0; i < 3; i++)
    {
        e0[i] = v1[i] - v0[i];
        e1[i] = v2[i] - v1[i];
        e2[i] = v0[i] - v2[i];
    }
    double fx = fabs(e0[0]), fy = fabs(e0[1]), fz = fabs(e0[2]);
    if (separated(e0[2] * v0[1] - e0[1] * v0[2], e0[2] * v2[1] - e0[1] * v2[2], fz * h[1] + fy * h[2], false)) return false;
    if (separated(-e0[2] * v0[0] + e0[0] * v0[2], -e0[2] * v2[0] + e0[0] * v2[2], fz * h[0] + fx * h[2], false)) return false;
    if (separated(e0[1] * v1[0] - e0[0] * v1[1], e0[1] * v2[0] - e0[0] * v2[1], fy * h[0] + fx * h[1], true)) return false;
    fx = fabs(e1[0]); fy = fabs(e1[1]); fz = fabs(e1[2]);
    if (separated(e1[2] * v0[1] - e1[1] * v0[2], e1[2] * v2[1] - e1[1] * v2[2], fz * h[1] + fy * h[2], false)) return false;
    if (separated(-e1[2] * v0[0] + e1[0] * v0[2], -e1[2] * v2[0] + e1[0] * v2[2], fz * h[0] + fx * h[2], false)) return false;
    if (separated(e1[1] * v0[0] - e1[0] * v0[1], e1[1] * v1[0] - e1[0] * v1[1], fy * h[0] + fx * h[1], false)) return false;
    fx = fabs(e2[0]); fy = fabs(e2[1]); fz = fabs(e2[2]);
    if (separated(e2[2] * v0[1] - e2[1] * v0[2], e2[2] * v1[1] - e2[1] * v1[2], fz * h[1] + fy * h[2], false)) return false;
    if (separated(-e2[2] * v0[0] + e2[0] * v0[2], -e2[2] * v1[0] + e2[0] * v1[2], fz * h[0] + fx * h[2], false)) return false;
    if (separated(e2[1] * v1[0] - e2[0] * v1[1], e2[1] * v2[0] - e2[0] * v2[1], fy * h[0] + fx * h[1], true)) return false;
#pragma unroll
    for (int a = 0; a < 3; a++)                      // FINDMINMAX, aabb_tri_internal.h:166-176
    {
        double mn = v0[a], mx = v0[a];
        if (v1[a] < mn) mn = v1[a];
        if (v1[a] > mx) mx = v1[a];
        if (v2[a] < mn) mn = v2[a];
        if (v2[a] > mx) mx = v2[a];
        if (mn > h[a] || mx < -h[a]) return false;
    }
    double n[3];                                     // CROSS(normal, e0, e1), :180
    n[0] = e0[1] * e1[2] - e0[2] * e1[1];
    n[1] = e0[2] * e1[0] - e0[0] * e1[2];
    n[2] = e0[0] * e1[1] - e0[1] * e1[0];
    const double d = -(n[0] * v0[0] + n[1] * v0[1] + n[2] * v0[2]);
    return plane_box(n, d, h);
}

// K2: one lane per (triangle, candidate cell).  err bit 0: overlap outside the grid.
__global__ void __launch_bounds__(256) k_candidates(GridParams G, const rt_vertex *__restrict__ verts,
                                                    const rt_triangle *__restrict__ tris,
                                                    const uint4 *__restrict__ range_lo,
                                                    const uint4 *__restrict__ range_hi,
                                                    const unsigned long long *__restrict__ first, uint64_t n_cand,
                                                    unsigned long long *keys, uint32_t *n_keys, uint32_t *tri_hit,
                                                    uint32_t *err)
{
    const uint64_t pidx = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (pidx >= n_cand) return;
    uint32_t lo = 0, hi = G.nt;                      // owner: last t with first[t] <= pidx
    while (hi - lo > 1)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] <= pidx) lo = mid; else hi = mid;
    }
    const uint32_t t = lo;
    const uint4 a = range_lo[t], b = range_hi[t];
    const uint32_t ny = b.y - a.y + 1, nz = b.z - a.z + 1;
    uint32_t j = uint32_t(pidx - first[t]);          // x outer, y, z inner: grid.cpp:81-92
    const uint32_t z = a.z + j % nz;
    j /= nz;
    const uint32_t y = a.y + j % ny;
    const uint32_t x = a.x + j / ny;
    // grid.cpp:101-108 cell bounds in float; aabb.h:19-26 centre / half size (float -> double)
    const float cmin[3] = { G.bmin[0] + float(x) * G.cw, G.bmin[1] + float(y) * G.cw, G.bmin[2] + float(z) * G.cw };
    const float cmax[3] = { G.bmin[0] + float(x + 1) * G.cw, G.bmin[1] + float(y + 1) * G.cw,
                            G.bmin[2] + float(z + 1) * G.cw };
    const double ctr[3] = { (cmin[0] + cmax[0]) * 0.5f, (cmin[1] + cmax[1]) * 0.5f, (cmin[2] + cmax[2]) * 0.5f };
    const double half[3] = { (cmax[0] - cmin[0]) * 0.5f, (cmax[1] - cmin[1]) * 0.5f, (cmax[2] - cmin[2]) * 0.5f };
    const rt_triangle tr = tris[t];
    const bool hit = tri_box_overlap(ctr, half, verts[tr.v0].p, verts[tr.v1].p, verts[tr.v2].p);
    if (hit)
    {
        // GridIdx (grid.h:41-42); the reference only asserts cell_idx < #cells (grid.cpp:119)
        const uint32_t cell = x + z * G.dims[0] + y * G.dims[0] * G.dims[2];
        if (cell < G.dims[0] * G.dims[1] * G.dims[2])
        {
            keys[atomicAdd(n_keys, 1u)] = (unsigned long long)cell << G.tb | t;   // any order: the sort
            tri_hit[t] = 1u;                                                     // orders the keys fully
        }
        else
            atomicOr(err, 1u);
    }
}

// K3: CSR offsets by lower_bound in the sorted keys; triangle ids from the low bits.
// err bit 1: a triangle overlaps no cell (grid.cpp:125 assert).
__global__ void __launch_bounds__(256) k_offsets(const unsigned long long *__restrict__ keys, uint32_t n_keys,
                                                 uint32_t n_cells, uint32_t tb, const uint32_t *__restrict__ tri_hit,
                                                 uint32_t nt, uint32_t *offsets, uint32_t *refs, uint32_t *err)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_keys) refs[i] = uint32_t(keys[i] & ((1ull << tb) - 1));
    if (i < nt && !tri_hit[i]) atomicOr(err, 2u);
    if (i > n_cells) return;
    const unsigned long long target = (unsigned long long)i << tb;
    uint32_t lo = 0, hi = n_keys;
    while (lo < hi)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    offsets[i] = lo;
}

// ---- exclusive scan: 1024 elements per 256-lane block, block sums scanned recursively ----
constexpr uint32_t kScanBlock = 256, kScanPer = 4, kScanTile = kScanBlock * kScanPer;

// Exclusive prefix of v over the block (wave64 shuffles, then the four wave totals through LDS);
// *total = the block's sum.
template <class T> __device__ __forceinline__ T block_exclusive(T v, T *total)
{
    __shared__ T wsum[kScanBlock / 64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1)
    {
        const T o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63u) wsum[w] = inc;
    __syncthreads();
    T base = 0, all = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanBlock / 64; i++)
    {
        if (i < w) base += wsum[i];
        all += wsum[i];
    }
    __syncthreads();                                 // wsum reusable by the next call
    *total = all;
    return base + inc - v;
}

template <class Tin, class Tout>
__global__ void __launch_bounds__(kScanBlock) k_scan_tiles(const Tin *__restrict__ in, Tout *out, Tout *sums, uint32_t n)
{
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    Tout v[kScanPer], run = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++)
    {
        v[k] = (i0 + k < n) ? Tout(in[i0 + k]) : Tout(0);
        run += v[k];
    }
    Tout total;
    Tout pre = block_exclusive(run, &total);
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++)
    {
        if (i0 + k < n) out[i0 + k] = pre;
        pre += v[k];
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

template <class T> __global__ void __launch_bounds__(kScanBlock) k_scan_add(T *out, const T *__restrict__ sums, uint32_t n)
{
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    const T add = sums[blockIdx.x];
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++)
        if (i0 + k < n) out[i0 + k] += add;
}

// ---- LSD radix sort of 64-bit keys, 8 bits a pass; 1024 keys per 256-lane block ----
constexpr uint32_t kRsBlock = 256, kRsRounds = 4, kRsTile = kRsBlock * kRsRounds;

// Per block the histogram of its tile's digits, digit-major: counts[digit * nblocks + block], so the
// exclusive scan of counts is each (digit, block)'s first output position.
__global__ void __launch_bounds__(kRsBlock) k_rs_count(const unsigned long long *__restrict__ keys, uint32_t n,
                                                       uint32_t shift, uint32_t *counts)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t base = blockIdx.x * kRsTile;
#pragma unroll
    for (uint32_t r = 0; r < kRsRounds; r++)
    {
        const uint32_t i = base + r * kRsBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[uint32_t(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    counts[threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter: the tile's keys in index order, 256 a round; within a wave a key's rank among the
// wave's keys of the same digit comes from eight ballots (the lanes sharing all eight bits), across
// waves and rounds from LDS counts -- so equal digits keep their input order.
__global__ void __launch_bounds__(kRsBlock) k_rs_scatter(const unsigned long long *__restrict__ keys, uint32_t n,
                                                         uint32_t shift, const uint32_t *__restrict__ offs,
                                                         unsigned long long *out)
{
    __shared__ uint32_t run[256];                    // keys of each digit in earlier rounds
    __shared__ uint32_t wcnt[kRsBlock / 64][256];    // keys of each digit per wave, this round
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    run[threadIdx.x] = offs[threadIdx.x * gridDim.x + blockIdx.x];
    const uint32_t base = blockIdx.x * kRsTile;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (uint32_t r = 0; r < kRsRounds; r++)
    {
#pragma unroll
        for (uint32_t q = 0; q < kRsBlock / 64; q++) wcnt[q][threadIdx.x] = 0u;
        __syncthreads();
        const uint32_t i = base + r * kRsBlock + threadIdx.x;
        const bool valid = i < n;
        const unsigned long long key = valid ? keys[i] : 0ull;
        const uint32_t d = uint32_t(key >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (uint32_t b = 0; b < 8; b++)
        {
            const unsigned long long set = __ballot(valid && ((d >> b) & 1u));
            peers &= ((d >> b) & 1u) ? set : ~set;
        }
        const uint32_t rank = uint32_t(__popcll(peers & below));
        if (valid && rank == 0u) wcnt[w][d] = uint32_t(__popcll(peers));
        __syncthreads();
        if (valid)
        {
            uint32_t pos = run[d] + rank;
            for (uint32_t q = 0; q < w; q++) pos += wcnt[q][d];
            out[pos] = key;
        }
        __syncthreads();
        uint32_t add = 0u;
#pragma unroll
        for (uint32_t q = 0; q < kRsBlock / 64; q++) add += wcnt[q][threadIdx.x];
        run[threadIdx.x] += add;
    }
}

uint32_t bits_for(uint64_t v)            // smallest b with v < 2^b
{
    uint32_t b = 0;
    while (b < 64 && (v >> b) != 0) b++;
    return b;
}

// grid.cpp:18-41 + mesh.cpp:112-134 on the host (float::min() max seed, hazard H11)
bool grid_meta(const rt_vertex *v, const rt_triangle *t, uint32_t nt, uint32_t res, rt_grid_desc& g)
{
    const float fmax = std::numeric_limits<float>::max(), fmin = std::numeric_limits<float>::min();
    float mn[3] = { fmax, fmax, fmax }, mx[3] = { fmin, fmin, fmin };
    for (uint32_t i = 0; i < nt; i++)
        for (uint32_t vi : { t[i].v0, t[i].v1, t[i].v2 })
            for (int a = 0; a < 3; a++)
            {
                mn[a] = std::min(mn[a], v[vi].p[a]);
                mx[a] = std::max(mx[a], v[vi].p[a]);
            }
    float ext[3];
    for (int a = 0; a < 3; a++)
    {
        g.aabb_min[a] = mn[a] - 0.0001f;
        g.aabb_max[a] = mx[a] + 0.0001f;
        ext[a] = g.aabb_max[a] - g.aabb_min[a];
    }
    const float largest = std::max(std::max(ext[0], ext[1]), ext[2]);
    g.cell_wdh = largest / float(res);
    g.inv_cell_wdh = 1.0f / g.cell_wdh;
    for (int a = 0; a < 3; a++) g.dims[a] = uint32_t(std::ceil(ext[a] / g.cell_wdh));
    const uint64_t nc = uint64_t(g.dims[0]) * g.dims[1] * g.dims[2];
    return nc > 0 && nc < 0x7FFFFFFFull;
}

// Device buffers of one build, released on every exit path.
struct BuildBuffers
{
    std::vector<void *> ptrs;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    template <class T> hipError_t alloc(T **p, size_t n)
    {
        *p = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
    ~BuildBuffers()
    {
        if (st) (void)hipStreamSynchronize(st);
        for (void *p : ptrs) (void)hipFree(p);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (st) (void)hipStreamDestroy(st);
    }
};

#define RG_HIP(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return rt_internal_fail(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

// Block-sum buffers of the scan levels, allocated once per build and reused by every scan.
struct ScanLevels
{
    std::vector<unsigned long long *> buf;
    std::vector<uint32_t> cap;
};

// Exclusive scan of n elements on B.st; the block sums are scanned the same way, in place.
template <class Tin, class Tout>
int exclusive_scan(BuildBuffers& B, ScanLevels& L, const Tin *in, Tout *out, uint32_t n, uint32_t level = 0)
{
    const uint32_t nb = (n + kScanTile - 1) / kScanTile;
    if (L.buf.size() <= level)
    {
        L.buf.push_back(nullptr);
        L.cap.push_back(0u);
    }
    if (L.cap[level] < nb)
    {
        RG_HIP(B.alloc(&L.buf[level], nb));          // 8 bytes an entry: either element type fits
        L.cap[level] = nb;
    }
    Tout *sums = reinterpret_cast<Tout *>(L.buf[level]);
    hipLaunchKernelGGL((k_scan_tiles<Tin, Tout>), dim3(nb), dim3(kScanBlock), 0, B.st, in, out, sums, n);
    RG_HIP(hipGetLastError());
    if (nb == 1u) return RT_OK;
    if (int rc = exclusive_scan<Tout, Tout>(B, L, sums, sums, nb, level + 1)) return rc;
    hipLaunchKernelGGL((k_scan_add<Tout>), dim3(nb), dim3(kScanBlock), 0, B.st, out, sums, n);
    RG_HIP(hipGetLastError());
    return RT_OK;
}

// Sorts n keys by their low `bits` bits; *sorted = the buffer (a or b) that holds the result.
int radix_sort(BuildBuffers& B, ScanLevels& L, unsigned long long *a, unsigned long long *b, uint32_t n,
               uint32_t bits, unsigned long long **sorted)
{
    const uint32_t nb = (n + kRsTile - 1) / kRsTile;
    uint32_t *counts, *offs;
    RG_HIP(B.alloc(&counts, size_t(256) * nb));
    RG_HIP(B.alloc(&offs, size_t(256) * nb));
    for (uint32_t shift = 0; shift < bits; shift += 8)
    {
        hipLaunchKernelGGL(k_rs_count, dim3(nb), dim3(kRsBlock), 0, B.st, a, n, shift, counts);
        RG_HIP(hipGetLastError());
        if (int rc = exclusive_scan<uint32_t, uint32_t>(B, L, counts, offs, 256u * nb)) return rc;
        hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(kRsBlock), 0, B.st, a, n, shift, offs, b);
        RG_HIP(hipGetLastError());
        std::swap(a, b);
    }
    *sorted = a;
    return RT_OK;
}

int build(const rt_vertex *v, uint32_t nv, const rt_triangle *t, uint32_t nt, uint32_t res, int device,
          rt_grid_desc *out, float *device_ms)
{
    if (!v || !t || !out || nv == 0 || nt == 0) return rt_internal_fail(RT_E_INVALID, "empty mesh (grid.cpp:15)");
    if (res == 0) return rt_internal_fail(RT_E_INVALID, "grid_res must be > 0 (grid.cpp:16)");
    if (nt >= 0x7FFFFFFFu) return rt_internal_fail(RT_E_INVALID, "too many triangles");
    for (uint32_t i = 0; i < nt; i++)
        if (t[i].v0 >= nv || t[i].v1 >= nv || t[i].v2 >= nv)
            return rt_internal_fail(RT_E_INVALID, "triangle vertex index out of range");
    rt_grid_desc g;
    std::memset(&g, 0, sizeof(g));
    if (!grid_meta(v, t, nt, res, g)) return rt_internal_fail(RT_E_INVALID, "degenerate grid");
    if (int rc = rt_internal_use_device(device, nullptr)) return rc;
    const uint32_t nc = g.dims[0] * g.dims[1] * g.dims[2];
    GridParams G;
    for (int a = 0; a < 3; a++) { G.bmin[a] = g.aabb_min[a]; G.dims[a] = g.dims[a]; }
    G.cw = g.cell_wdh;
    G.nt = nt;
    G.tb = std::max(1u, bits_for(nt - 1));
    const uint32_t cb = bits_for(nc);                // 2^cb > nc: every cell field, and nc << tb for K3
    if (G.tb + cb > 64) return rt_internal_fail(RT_E_INVALID, "grid too large for 64-bit keys");

    BuildBuffers B;
    RG_HIP(hipStreamCreateWithFlags(&B.st, hipStreamNonBlocking));
    RG_HIP(hipEventCreate(&B.e0));
    RG_HIP(hipEventCreate(&B.e1));
    rt_vertex *d_v;
    rt_triangle *d_t;
    uint4 *d_lo, *d_hi;
    uint32_t *d_cnt, *d_hit, *d_err, *d_off, *d_refs;
    unsigned long long *d_first, *d_keys, *d_sorted;
    RG_HIP(B.alloc(&d_v, nv));
    RG_HIP(B.alloc(&d_t, nt));
    RG_HIP(B.alloc(&d_lo, nt));
    RG_HIP(B.alloc(&d_hi, nt));
    RG_HIP(B.alloc(&d_cnt, nt));
    RG_HIP(B.alloc(&d_hit, nt));
    RG_HIP(B.alloc(&d_err, 1));
    RG_HIP(B.alloc(&d_first, nt));
    RG_HIP(hipMemcpyAsync(d_v, v, sizeof(rt_vertex) * nv, hipMemcpyHostToDevice, B.st));
    RG_HIP(hipMemcpyAsync(d_t, t, sizeof(rt_triangle) * nt, hipMemcpyHostToDevice, B.st));
    RG_HIP(hipMemsetAsync(d_hit, 0, sizeof(uint32_t) * nt, B.st));
    RG_HIP(hipMemsetAsync(d_err, 0, sizeof(uint32_t), B.st));

    RG_HIP(hipEventRecord(B.e0, B.st));
    hipLaunchKernelGGL(k_tri_ranges, dim3((nt + 255) / 256), dim3(256), 0, B.st, G, d_v, d_t, d_lo, d_hi, d_cnt);
    RG_HIP(hipGetLastError());
    ScanLevels L;
    if (int rc = exclusive_scan<uint32_t, unsigned long long>(B, L, d_cnt, d_first, nt)) return rc;
    unsigned long long last_first = 0;
    uint32_t last_cnt = 0;
    RG_HIP(hipMemcpyAsync(&last_first, d_first + nt - 1, sizeof(last_first), hipMemcpyDeviceToHost, B.st));
    RG_HIP(hipMemcpyAsync(&last_cnt, d_cnt + nt - 1, sizeof(last_cnt), hipMemcpyDeviceToHost, B.st));
    RG_HIP(hipStreamSynchronize(B.st));
    const uint64_t n_cand = last_first + last_cnt;
    if (n_cand >= 0x7FFFFFFFull) return rt_internal_fail(RT_E_INVALID, "too many candidate cells");
    uint32_t *d_nkeys;
    RG_HIP(B.alloc(&d_keys, n_cand));
    RG_HIP(B.alloc(&d_nkeys, 1));
    RG_HIP(hipMemsetAsync(d_nkeys, 0, sizeof(uint32_t), B.st));
    hipLaunchKernelGGL(k_candidates, dim3(uint32_t((n_cand + 255) / 256)), dim3(256), 0, B.st, G, d_v, d_t, d_lo,
                       d_hi, d_first, n_cand, d_keys, d_nkeys, d_hit, d_err);
    RG_HIP(hipGetLastError());
    uint32_t n_keys = 0;                             // the overlapping (cell, triangle) pairs: the sort's size
    RG_HIP(hipMemcpyAsync(&n_keys, d_nkeys, sizeof(n_keys), hipMemcpyDeviceToHost, B.st));
    RG_HIP(hipStreamSynchronize(B.st));
    RG_HIP(B.alloc(&d_sorted, n_keys));
    if (n_keys)
        if (int rc = radix_sort(B, L, d_keys, d_sorted, n_keys, G.tb + cb, &d_sorted)) return rc;
    RG_HIP(B.alloc(&d_off, size_t(nc) + 1));
    RG_HIP(B.alloc(&d_refs, n_keys));
    const uint64_t k3 = std::max<uint64_t>(std::max<uint64_t>(n_keys, uint64_t(nc) + 1), nt);
    hipLaunchKernelGGL(k_offsets, dim3(uint32_t((k3 + 255) / 256)), dim3(256), 0, B.st, d_sorted, n_keys,
                       nc, G.tb, d_hit, nt, d_off, d_refs, d_err);
    RG_HIP(hipGetLastError());
    RG_HIP(hipEventRecord(B.e1, B.st));
    uint32_t *h_off = static_cast<uint32_t *>(std::malloc(sizeof(uint32_t) * (size_t(nc) + 1)));
    if (!h_off) return rt_internal_fail(RT_E_INVALID, "out of host memory");
    uint32_t err = 0;
    hipError_t e = hipMemcpyAsync(h_off, d_off, sizeof(uint32_t) * (size_t(nc) + 1), hipMemcpyDeviceToHost, B.st);
    if (e == hipSuccess) e = hipMemcpyAsync(&err, d_err, sizeof(err), hipMemcpyDeviceToHost, B.st);
    if (e == hipSuccess) e = hipStreamSynchronize(B.st);
    if (e != hipSuccess)
    {
        std::free(h_off);
        return rt_internal_fail(RT_E_HIP, std::string("grid build: ") + hipGetErrorString(e));
    }
    if (err)
    {
        std::free(h_off);
        return rt_internal_fail(RT_E_INVALID, (err & 1) ? "a triangle overlaps a cell outside the grid"
                                                        : "a triangle touches no cell (grid.cpp:121-125)");
    }
    const uint32_t nr = h_off[nc];                   // lower_bound(nc << tb) = n_keys
    uint32_t *h_refs = static_cast<uint32_t *>(std::malloc(sizeof(uint32_t) * std::max(nr, 1u)));
    if (!h_refs)
    {
        std::free(h_off);
        return rt_internal_fail(RT_E_INVALID, "out of host memory");
    }
    e = nr ? hipMemcpy(h_refs, d_refs, sizeof(uint32_t) * nr, hipMemcpyDeviceToHost) : hipSuccess;
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, B.e0, B.e1);
    if (e != hipSuccess)
    {
        std::free(h_off);
        std::free(h_refs);
        return rt_internal_fail(RT_E_HIP, std::string("grid build: ") + hipGetErrorString(e));
    }
    if (device_ms) *device_ms = ms;
    g.cell_offsets = h_off;
    g.cell_tris = h_refs;
    *out = g;
    return RT_OK;
}

} // namespace

extern "C" {

int rt_grid_build(const rt_vertex *vertices, uint32_t num_vertices, const rt_triangle *triangles,
                  uint32_t num_triangles, uint32_t grid_res, int device, rt_grid_desc *out, float *device_ms)
{
    if (out) std::memset(out, 0, sizeof(*out));
    return build(vertices, num_vertices, triangles, num_triangles, grid_res, device, out, device_ms);
}

int rt_grid_free(rt_grid_desc *grid)
{
    if (!grid) return rt_internal_fail(RT_E_INVALID, "grid is NULL");
    std::free(const_cast<uint32_t *>(grid->cell_offsets));
    std::free(const_cast<uint32_t *>(grid->cell_tris));
    grid->cell_offsets = nullptr;
    grid->cell_tris = nullptr;
    return RT_OK;
}

int rt_scene_create_from_mesh(const rt_vertex *vertices, uint32_t num_vertices, const rt_triangle *triangles,
                              uint32_t num_triangles, uint32_t grid_res, int device, rt_scene **out)
{
    if (!out) return rt_internal_fail(RT_E_INVALID, "out is NULL");
    *out = nullptr;
    rt_scene_desc d;
    std::memset(&d, 0, sizeof(d));
    if (int rc = build(vertices, num_vertices, triangles, num_triangles, grid_res, device, &d.grid, nullptr))
        return rc;
    d.num_vertices = num_vertices;
    d.num_triangles = num_triangles;
    d.vertices = vertices;
    d.triangles = triangles;
    const int rc = rt_scene_create(&d, device, out);
    rt_grid_free(&d.grid);
    return rc;
}

} // extern "C"
