// oracle/cpu_tracer.cpp -- TEST INFRASTRUCTURE ONLY (see cpu_tracer.h).
//
// Scalar C++11 restatement of the reference's per-sample tile path.  Every function cites
// the reference file:line it follows; evaluation order of every float expression is kept
// (built with -ffp-contract=off, no -march, like the reference Makefile:9-11) so the
// results are bit-identical to oracle/_ref/refdriver.  Pinned by tests/golden/.

#include "cpu_tracer.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace {

struct V3 { float x, y, z; };
inline V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
inline float comp(const V3& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
inline V3 sub(const V3& a, const V3& b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
// lin_alg.h:138-144: T result = T(); result += a[i]*b[i] for i = 0..2
inline float dot0(const V3& a, const V3& b)
{
    float r = 0.0f;
    r += a.x * b.x;
    r += a.y * b.y;
    r += a.z * b.z;
    return r;
}
// lin_alg.h:151-156: length = 1 / sqrt(Dot); vec * length
inline V3 normalize(const V3& v)
{
    const float len = 1.0f / std::sqrt(dot0(v, v));
    return mk(v.x * len, v.y * len, v.z * len);
}
// x86 cvttss2si semantics (what the reference's (int)/(uchar) casts compile to):
// out-of-range and NaN give INT_MIN.
inline int cvt_i32(float x)
{
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return std::numeric_limits<int>::min();
    return int(x);
}

struct Vertex { V3 p, n; };
struct Triangle { uint32_t v0, v1, v2; V3 n; };

struct Scene
{
    uint32_t id = 0;
    float fov = 45.0f;
    float cam[4][4];
    std::vector<Vertex> verts;
    std::vector<Triangle> tris;
    // Grid (grid.h:26-39)
    uint32_t dim[3];
    float cell_wdh, inv_cell_wdh;
    V3 aabb_min, aabb_max;
    std::vector<uint32_t> off, refs;      // CSR of m_cells, GridIdx order
    double build_s = 0.0;

    uint32_t GridIdx(uint32_t x, uint32_t y, uint32_t z) const   // grid.h:41-42
        { return x + z * dim[0] + y * dim[0] * dim[2]; }
    int ToVoxel(const V3& pos, int axis) const                   // grid.h:44-48
    {
        const int v = cvt_i32((comp(pos, axis) - comp(aabb_min, axis)) * inv_cell_wdh);
        const int hi = int(dim[axis]) - 1;
        return v < 0 ? 0 : (v > hi ? hi : v);
    }
    float ToPos(int vox, int axis) const                         // grid.h:50-51
        { return comp(aabb_min, axis) + float(vox) * cell_wdh; }
};

// ------------------------------------------------------------- tri/box overlap (double)
// aabb_tri_internal.h:42-63 planeBoxOverlap
int PlaneBoxOverlap(const double n[3], double d, const double maxbox[3])
{
    double vmin[3], vmax[3];
    for (int q=0; q<3; q++)
    {
        if (n[q] > 0.0f) { vmin[q] = -maxbox[q]; vmax[q] = maxbox[q]; }
        else             { vmin[q] = maxbox[q];  vmax[q] = -maxbox[q]; }
    }
    if (n[0] * vmin[0] + n[1] * vmin[1] + n[2] * vmin[2] + d > 0.0f) return 0;
    if (n[0] * vmax[0] + n[1] * vmax[1] + n[2] * vmax[2] + d >= 0.0f) return 1;
    return 0;
}

// one separating-axis test of aabb_tri_internal.h:67-110: project two vertices, compare to rad
inline bool AxisSeparates(double pa, double pb, double rad)
{
    double mn, mx;
    if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
    return mn > rad || mx < -rad;
}

// aabb_tri_internal.h:112-186 triBoxOverlap (Akenine-Moller SAT), operand order preserved
int TriBoxOverlap(const double c[3], const double h[3], const double tv[3][3])
{
    double v0[3], v1[3], v2[3], e0[3], e1[3], e2[3];
    for (int i=0; i<3; i++) { v0[i] = tv[0][i] - c[i]; v1[i] = tv[1][i] - c[i]; v2[i] = tv[2][i] - c[i]; }
    for (int i=0; i<3; i++) { e0[i] = v1[i] - v0[i]; e1[i] = v2[i] - v1[i]; e2[i] = v0[i] - v2[i]; }
    const int X = 0, Y = 1, Z = 2;
    double fex, fey, fez;
    // edge 0: X01, Y02, Z12
    fex = std::fabs(e0[X]); fey = std::fabs(e0[Y]); fez = std::fabs(e0[Z]);
    if (AxisSeparates(e0[Z]*v0[Y] - e0[Y]*v0[Z], e0[Z]*v2[Y] - e0[Y]*v2[Z], fez*h[Y] + fey*h[Z])) return 0;
    if (AxisSeparates(-e0[Z]*v0[X] + e0[X]*v0[Z], -e0[Z]*v2[X] + e0[X]*v2[Z], fez*h[X] + fex*h[Z])) return 0;
    {   // AXISTEST_Z12 orders its min/max with p2 first (aabb_tri_internal.h:101)
        const double p1 = e0[Y]*v1[X] - e0[X]*v1[Y], p2 = e0[Y]*v2[X] - e0[X]*v2[Y];
        double mn, mx;
        if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }
        const double rad = fey*h[X] + fex*h[Y];
        if (mn > rad || mx < -rad) return 0;
    }
    // edge 1: X01, Y02, Z0
    fex = std::fabs(e1[X]); fey = std::fabs(e1[Y]); fez = std::fabs(e1[Z]);
    if (AxisSeparates(e1[Z]*v0[Y] - e1[Y]*v0[Z], e1[Z]*v2[Y] - e1[Y]*v2[Z], fez*h[Y] + fey*h[Z])) return 0;
    if (AxisSeparates(-e1[Z]*v0[X] + e1[X]*v0[Z], -e1[Z]*v2[X] + e1[X]*v2[Z], fez*h[X] + fex*h[Z])) return 0;
    if (AxisSeparates(e1[Y]*v0[X] - e1[X]*v0[Y], e1[Y]*v1[X] - e1[X]*v1[Y], fey*h[X] + fex*h[Y])) return 0;
    // edge 2: X2, Y1, Z12
    fex = std::fabs(e2[X]); fey = std::fabs(e2[Y]); fez = std::fabs(e2[Z]);
    if (AxisSeparates(e2[Z]*v0[Y] - e2[Y]*v0[Z], e2[Z]*v1[Y] - e2[Y]*v1[Z], fez*h[Y] + fey*h[Z])) return 0;
    if (AxisSeparates(-e2[Z]*v0[X] + e2[X]*v0[Z], -e2[Z]*v1[X] + e2[X]*v1[Z], fez*h[X] + fex*h[Z])) return 0;
    {
        const double p1 = e2[Y]*v1[X] - e2[X]*v1[Y], p2 = e2[Y]*v2[X] - e2[X]*v2[Y];
        double mn, mx;
        if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }
        const double rad = fey*h[X] + fex*h[Y];
        if (mn > rad || mx < -rad) return 0;
    }
    // bullet 1: FINDMINMAX per axis (aabb_tri_internal.h:35-40, 166-176)
    for (int a=0; a<3; a++)
    {
        double mn = v0[a], mx = v0[a];
        if (v1[a] < mn) mn = v1[a];
        if (v1[a] > mx) mx = v1[a];
        if (v2[a] < mn) mn = v2[a];
        if (v2[a] > mx) mx = v2[a];
        if (mn > h[a] || mx < -h[a]) return 0;
    }
    // bullet 2: plane (aabb_tri_internal.h:181-183)
    double n[3];
    n[0] = e0[1]*e1[2] - e0[2]*e1[1];
    n[1] = e0[2]*e1[0] - e0[0]*e1[2];
    n[2] = e0[0]*e1[1] - e0[1]*e1[0];
    const double d = -(n[0]*v0[0] + n[1]*v0[1] + n[2]*v0[2]);
    if (!PlaneBoxOverlap(n, d, h)) return 0;
    return 1;
}

// aabb.h:15-32 IntersectTriAABB: centre/half in float, widened to double
bool TriAABB(const V3& a, const V3& b, const V3& c, const V3& bmin, const V3& bmax)
{
    const double ctr[3] = { (bmin.x + bmax.x) * 0.5f, (bmin.y + bmax.y) * 0.5f, (bmin.z + bmax.z) * 0.5f };
    const double half[3] = { (bmax.x - bmin.x) * 0.5f, (bmax.y - bmin.y) * 0.5f, (bmax.z - bmin.z) * 0.5f };
    const double tv[3][3] = { { a.x, a.y, a.z }, { b.x, b.y, b.z }, { c.x, c.y, c.z } };
    return TriBoxOverlap(ctr, half, tv) == 1;
}

// -------------------------------------------------------------------- grid build
// grid.cpp:12-154 (Grid::Grid) with resolution 64 (scene.cpp:7)
void BuildGrid(Scene& s, uint32_t grid_res)
{
    const auto t0 = std::chrono::steady_clock::now();
    // mesh.cpp:112-134 ComputeAABB, with the numeric_limits<float>::min() max-seed quirk
    V3 mn = mk(std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max());
    V3 mx = mk(std::numeric_limits<float>::min(), std::numeric_limits<float>::min(), std::numeric_limits<float>::min());
    for (const auto& t : s.tris)
    {
        const uint32_t ids[3] = { t.v0, t.v1, t.v2 };
        for (int k=0; k<3; k++)
        {
            const V3& p = s.verts[ids[k]].p;
            mn = mk(std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z));
            mx = mk(std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z));
        }
    }
    // grid.cpp:29-38
    s.aabb_min = sub(mn, mk(0.0001f, 0.0001f, 0.0001f));
    s.aabb_max = mk(mx.x + 0.0001f, mx.y + 0.0001f, mx.z + 0.0001f);
    const V3 ext = sub(s.aabb_max, s.aabb_min);
    const float largest = std::max(std::max(ext.x, ext.y), ext.z);
    s.cell_wdh = largest / float(grid_res);
    s.inv_cell_wdh = 1.0f / s.cell_wdh;
    for (int a=0; a<3; a++)
        s.dim[a] = uint32_t(std::ceil(comp(ext, a) / s.cell_wdh));
    const uint32_t ncells = s.dim[0] * s.dim[1] * s.dim[2];
    std::vector<std::vector<uint32_t>> cells(ncells);

    // grid.cpp:65-129, triangles in index order -> each cell list ascending
    for (uint32_t ti=0; ti<uint32_t(s.tris.size()); ti++)
    {
        const Triangle& t = s.tris[ti];
        const V3 &p0 = s.verts[t.v0].p, &p1 = s.verts[t.v1].p, &p2 = s.verts[t.v2].p;
        // triangle.h:116-131 TriangleAABB (same float::min() seed)
        V3 tmn = mk(std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max());
        V3 tmx = mk(std::numeric_limits<float>::min(), std::numeric_limits<float>::min(), std::numeric_limits<float>::min());
        const V3 *pp[3] = { &p0, &p1, &p2 };
        for (int k=0; k<3; k++)
        {
            tmn = mk(std::min(tmn.x, pp[k]->x), std::min(tmn.y, pp[k]->y), std::min(tmn.z, pp[k]->z));
            tmx = mk(std::max(tmx.x, pp[k]->x), std::max(tmx.y, pp[k]->y), std::max(tmx.z, pp[k]->z));
        }
        tmn = sub(tmn, s.aabb_min);
        tmx = sub(tmx, s.aabb_min);
        uint32_t st[3], en[3];
        for (int a=0; a<3; a++)
        {
            st[a] = uint32_t(int64_t(comp(tmn, a) / s.cell_wdh));   // grid.cpp:81-92 uint(float)
            en[a] = uint32_t(int64_t(comp(tmx, a) / s.cell_wdh));
        }
        for (uint32_t x=st[0]; x<=en[0]; x++)
            for (uint32_t y=st[1]; y<=en[1]; y++)
                for (uint32_t z=st[2]; z<=en[2]; z++)
                {
                    const V3 cmn = mk(s.aabb_min.x + float(x) * s.cell_wdh,
                                      s.aabb_min.y + float(y) * s.cell_wdh,
                                      s.aabb_min.z + float(z) * s.cell_wdh);
                    const V3 cmx = mk(s.aabb_min.x + float(x + 1) * s.cell_wdh,
                                      s.aabb_min.y + float(y + 1) * s.cell_wdh,
                                      s.aabb_min.z + float(z + 1) * s.cell_wdh);
                    if (TriAABB(p0, p1, p2, cmn, cmx))
                        cells[s.GridIdx(x, y, z)].push_back(ti);
                }
    }
    s.off.assign(ncells + 1, 0);
    for (uint32_t c=0; c<ncells; c++) s.off[c + 1] = s.off[c] + uint32_t(cells[c].size());
    s.refs.resize(s.off[ncells]);
    for (uint32_t c=0; c<ncells; c++)
        std::copy(cells[c].begin(), cells[c].end(), s.refs.begin() + s.off[c]);
    s.build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// ------------------------------------------------------------------ primitives
// triangle.h:15-107 IntersectRayTri, non-culling branch
inline bool RayTri(const V3& o, const V3& d, const V3& v0, const V3& v1, const V3& v2,
                   float& t, float& u, float& v)
{
    const V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    const V3 pv = mk(d.y * e2.z - d.z * e2.y, d.z * e2.x - d.x * e2.z, d.x * e2.y - d.y * e2.x);
    const float det = e1.x * pv.x + e1.y * pv.y + e1.z * pv.z;
    if (det > -0.00000001f && det < 0.00000001f) return false;
    const float inv_det = 1.0f / det;
    const V3 tv = sub(o, v0);
    u = (tv.x * pv.x + tv.y * pv.y + tv.z * pv.z) * inv_det;
    if (u < 0.0f || u > 1.0f) return false;
    const V3 qv = mk(tv.y * e1.z - tv.z * e1.y, tv.z * e1.x - tv.x * e1.z, tv.x * e1.y - tv.y * e1.x);
    v = (d.x * qv.x + d.y * qv.y + d.z * qv.z) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = (e2.x * qv.x + e2.y * qv.y + e2.z * qv.z) * inv_det;
    return t >= 0.0f;
}

// triangle.h:200-226 IntersectRayPlane + ComputeBarycentric (:133-156)
inline bool RayTriBary(const V3& o, const V3& d, const V3& v0, const V3& v1, const V3& v2,
                       const V3& n, float& t, float& u, float& v)
{
    const float denom = dot0(n, d);
    if (std::fabs(denom) < 0.00000001f) return false;
    const float dd = dot0(n, v0);
    t = (dd - dot0(n, o)) / denom;
    if (!(double(t) >= 0.0)) return false;
    const V3 pos = mk(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
    const V3 e0 = sub(v2, v0), e1 = sub(v1, v0), e2 = sub(pos, v0);
    const float d00 = dot0(e0, e0), d01 = dot0(e0, e1), d02 = dot0(e0, e2);
    const float d11 = dot0(e1, e1), d12 = dot0(e1, e2);
    const float inv_denom = 1.0f / (d00 * d11 - d01 * d01);
    u = (d00 * d12 - d01 * d02) * inv_denom;
    v = (d11 * d02 - d01 * d12) * inv_denom;
    return (u >= 0) && (v >= 0) && (u + v < 1);
}

// aabb.h:9-13
inline bool PointAABB(const V3& p, const V3& mn, const V3& mx)
{
    return p.x >= mn.x && p.y >= mn.y && p.z >= mn.z && p.x <= mx.x && p.y <= mx.y && p.z <= mx.z;
}

// aabb.h:34-83 (Williams et al. slab test; no tmax < 0 rejection)
inline bool RayAABB(const V3& o, const V3& d, const V3& mn, const V3& mx, float& tmin, float& tmax)
{
    const V3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const V3 box[2] = { mn, mx };
    const int sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
    tmin = (box[sx].x - o.x) * inv.x;
    tmax = (box[1 - sx].x - o.x) * inv.x;
    const float tymin = (box[sy].y - o.y) * inv.y;
    const float tymax = (box[1 - sy].y - o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = (box[sz].z - o.z) * inv.z;
    const float tzmax = (box[1 - sz].z - o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return true;
}

// camera.h:8-47, perspective branch; fov_xs uses double ::tan like camera.h:42 under libstdc++
inline void GenRay(const float m[4][4], uint32_t px, uint32_t py, uint32_t W, uint32_t H,
                   float sx, float sy, float fov, V3& o, V3& d)
{
    const float ndc_x = (float(px) + sx) / float(W) * 2.0f - 1.0f;
    const float ndc_y = (float(py) + sy) / float(H) * 2.0f - 1.0f;
    const float aspect = float(W) / float(H);
    const float hfov = fov * float(0.0174532925);                 // lin_alg.h:232
    const float fov_xs = float(::tan(double(hfov / 2.0f)));
    o = mk(0.0f * m[0][0] + 0.0f * m[1][0] + 0.0f * m[2][0] + m[3][0],   // lin_alg.h:518-535
           0.0f * m[0][1] + 0.0f * m[1][1] + 0.0f * m[2][1] + m[3][1],
           0.0f * m[0][2] + 0.0f * m[1][2] + 0.0f * m[2][2] + m[3][2]);
    const V3 p = normalize(mk(ndc_x * fov_xs, ndc_y * fov_xs / aspect, -1.0f));
    d = mk(p.x * m[0][0] + p.y * m[1][0] + p.z * m[2][0],                // lin_alg.h:495-509
           p.x * m[0][1] + p.y * m[1][1] + p.z * m[2][1],
           p.x * m[0][2] + p.y * m[1][2] + p.z * m[2][2]);
}

// triangle.h:158-161 BarycentricInterpolate + Normalize + renderer.cpp:117 (n+1)*0.5
inline V3 ShadeHit(float u, float v, const V3& n0, const V3& n1, const V3& n2)
{
    const float w = 1.0f - u - v;
    const V3 b = mk(n1.x * u + n2.x * v + n0.x * w,
                    n1.y * u + n2.y * v + n0.y * w,
                    n1.z * u + n2.z * v + n0.z * w);
    const V3 n = normalize(b);
    return mk((n.x + 1.0f) * 0.5f, (n.y + 1.0f) * 0.5f, (n.z + 1.0f) * 0.5f);
}

// lin_alg.h:125-132 ToBGRA8 with the x86 float->int truncation of the (uchar) cast
inline uint32_t Pack(float r, float g, float b)
{
    const uint32_t rc = r > 1.0f ? 255u : uint32_t(cvt_i32(r * 255.0f)) & 255u;
    const uint32_t gc = g > 1.0f ? 255u : uint32_t(cvt_i32(g * 255.0f)) & 255u;
    const uint32_t bc = b > 1.0f ? 255u : uint32_t(cvt_i32(b * 255.0f)) & 255u;
    return rc << 16 | gc << 8 | bc;
}

// sampling.h:113-120 + sampling.cpp:194-210 (base 2) + renderer.cpp:52-55
std::vector<float> Hammersley(uint32_t spp)
{
    std::vector<float> xy(size_t(spp) * 2);
    for (uint32_t s=0; s<spp; s++)
    {
        double val = 0.0, inv_i = 0.5;
        for (uint32_t n=s; n>0; n/=2)
        {
            val += (n % 2) * inv_i;
            inv_i *= 0.5;
        }
        xy[2 * s + 0] = float(double(s) / double(spp) - 0.5f);
        xy[2 * s + 1] = float(val - 0.5f);
    }
    return xy;
}

// -------------------------------------------------------------- grid traversal
// grid.cpp:159-281 Grid::Intersect (NEW_GRID_TRAVERSAL), instrumented with counters.  Like the
// reference (origin/dir by value, grid.cpp:160-161) the walk runs on locals: results and counters
// are stored once at the end, so no store inside the loop can alias the ray or the scene arrays.
template <int TRI_TEST>
bool IntersectT(const Scene& s, const V3 o, const V3 d, float& t_out, float& u_out, float& v_out,
                uint32_t& tri_out, uint32_t& voxel_out, uint32_t& steps_out, uint32_t& tests_out)
{
    uint32_t steps = 0, tests = 0, voxel = 0xFFFFFFFFu;
    float enter_t, leave_t;
    V3 g;
    bool found = false;
    float t = std::numeric_limits<float>::max(), u = 0.0f, v = 0.0f;
    uint32_t tri_idx = tri_out;
    if (PointAABB(o, s.aabb_min, s.aabb_max)) { enter_t = 0.0f; g = o; }
    else if (RayAABB(o, d, s.aabb_min, s.aabb_max, enter_t, leave_t))
        g = mk(o.x + d.x * enter_t, o.y + d.y * enter_t, o.z + d.z * enter_t);
    else
    {
        steps_out = tests_out = 0;
        voxel_out = voxel;
        return false;
    }

    float nct[3], dt[3] = { 0, 0, 0 };
    int step[3] = { 0, 0, 0 }, out[3] = { 0, 0, 0 }, pos[3];
    for (int a=0; a<3; a++)
    {
        pos[a] = s.ToVoxel(g, a);
        const float da = comp(d, a);
        if (da == 0.0f)
            nct[a] = std::numeric_limits<float>::max();
        else if (da > 0.0f)
        {
            nct[a] = enter_t + (s.ToPos(pos[a] + 1, a) - comp(g, a)) / da;
            dt[a] = s.cell_wdh / da;
            step[a] = 1;
            out[a] = int(s.dim[a]);
        }
        else
        {
            nct[a] = enter_t + (s.ToPos(pos[a], a) - comp(g, a)) / da;
            dt[a] = -s.cell_wdh / da;
            step[a] = -1;
            out[a] = -1;
        }
    }
    const uint32_t *off = s.off.data(), *refs = s.refs.data();
    const Triangle *tris = s.tris.data();
    const Vertex *verts = s.verts.data();
    while (true)
    {
        const int ax = (nct[0] < nct[1]) ? ((nct[0] < nct[2]) ? 0 : 2) : ((nct[1] < nct[2]) ? 1 : 2);
        const uint32_t cell = s.GridIdx(pos[0], pos[1], pos[2]);
        voxel = cell;
        steps++;
        const uint32_t k1 = off[cell + 1];
        for (uint32_t k=off[cell]; k<k1; k++)
        {
            const uint32_t ci = refs[k];
            const Triangle& tr = tris[ci];
            float ct, cu, cv;
            tests++;
            const bool hit = TRI_TEST == 1
                ? RayTriBary(o, d, verts[tr.v0].p, verts[tr.v1].p, verts[tr.v2].p, tr.n, ct, cu, cv)
                : RayTri(o, d, verts[tr.v0].p, verts[tr.v1].p, verts[tr.v2].p, ct, cu, cv);
            if (hit && ct < t && ct < nct[ax])
            {
                t = ct; u = cu; v = cv; tri_idx = ci;
            }
        }
        if (t != std::numeric_limits<float>::max()) { found = true; break; }
        pos[ax] += step[ax];
        if (pos[ax] == out[ax]) break;
        nct[ax] += dt[ax];
    }
    t_out = t;
    if (found) { u_out = u; v_out = v; tri_out = tri_idx; }
    voxel_out = voxel; steps_out = steps; tests_out = tests;
    return found;
}

inline bool Intersect(const Scene& s, const V3& o, const V3& d, int tri_test, float& t, float& u, float& v,
                      uint32_t& tri_idx, uint32_t& voxel, uint32_t& steps, uint32_t& tests)
{
    return tri_test == 1 ? IntersectT<1>(s, o, d, t, u, v, tri_idx, voxel, steps, tests)
                         : IntersectT<0>(s, o, d, t, u, v, tri_idx, voxel, steps, tests);
}

// renderer.cpp:157-197 Renderer::IntersectBruteForce: all triangles in index order, closest
// accepted IntersectRayTri hit, strict '<' keeps the lower index on ties
bool IntersectBruteForce(const Scene& s, const V3& o, const V3& d, float& t, float& u, float& v,
                         uint32_t& tri_idx, uint32_t& tests)
{
    t = std::numeric_limits<float>::max();
    for (uint32_t i=0; i<uint32_t(s.tris.size()); i++)
    {
        const Triangle& tr = s.tris[i];
        float ct, cu, cv;
        const bool hit = RayTri(o, d, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p, ct, cu, cv);
        if (hit && ct < t)
        {
            t = ct; u = cu; v = cv; tri_idx = i;
        }
    }
    tests = uint32_t(s.tris.size());
    return t != std::numeric_limits<float>::max();
}

// triangle.h:163-172 LineSegMinDistSq; Clamp = lin_alg.h:205-212
inline float LineSegMinDistSq(const V3& a, const V3& b, const V3& p)
{
    const V3 ab = sub(b, a);
    const float len_sq = dot0(ab, ab);
    float t = dot0(sub(p, a), ab) / len_sq;
    if (t < 0.0f) t = 0.0f;
    else if (t > 1.0f) t = 1.0f;
    const V3 proj = mk(a.x + t * ab.x, a.y + t * ab.y, a.z + t * ab.z);
    return dot0(sub(p, proj), sub(p, proj));
}

// triangle.h:174-198 DistancePointTri with ComputeBarycentric (:133-156) and
// BarycentricInterpolate (:158-161); std::min(a, b) = (b < a) ? b : a
inline float DistancePointTri(const V3& pos, const V3& v0, const V3& v1, const V3& v2)
{
    const V3 e0 = sub(v2, v0), e1 = sub(v1, v0), e2 = sub(pos, v0);
    const float dot00 = dot0(e0, e0), dot01 = dot0(e0, e1), dot02 = dot0(e0, e2);
    const float dot11 = dot0(e1, e1), dot12 = dot0(e1, e2);
    const float inv_denom = 1 / (dot00 * dot11 - dot01 * dot01);
    const float u = (dot00 * dot12 - dot01 * dot02) * inv_denom;
    const float v = (dot11 * dot02 - dot01 * dot12) * inv_denom;
    if ((u >= 0) && (v >= 0) && (u + v < 1))
    {
        const float w = 1 - u - v;
        const V3 q = mk(v1.x * u + v2.x * v + v0.x * w, v1.y * u + v2.y * v + v0.y * w,
                        v1.z * u + v2.z * v + v0.z * w);
        return std::sqrt(dot0(sub(pos, q), sub(pos, q)));
    }
    const float a = LineSegMinDistSq(v0, v1, pos), b = LineSegMinDistSq(v0, v2, pos),
                c = LineSegMinDistSq(v1, v2, pos);
    const float bc = (c < b) ? c : b;
    return std::sqrt((bc < a) ? bc : a);
}

// renderer.cpp:24-41 Renderer::RayMarch over DistanceBruteForce (:138-155)
bool RayMarch(const Scene& s, const V3& o, const V3& d, float& t, uint32_t& steps, uint32_t& tests)
{
    const uint32_t max_steps = 128;
    const float min_dist = 0.001f;
    t = 0.0f;
    steps = tests = 0;
    for (uint32_t i=0; i<max_steps; i++)
    {
        const V3 pos = mk(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
        float dist = std::numeric_limits<float>::max();
        for (const auto& tr : s.tris)
        {
            const float di = DistancePointTri(pos, s.verts[tr.v0].p, s.verts[tr.v1].p, s.verts[tr.v2].p);
            dist = (di < dist) ? di : dist;
        }
        t += dist;
        steps = i + 1;
        tests += uint32_t(s.tris.size());
        if (dist < min_dist) return true;
    }
    return false;
}

// renderer.cpp:90-121: one sample.  mode = tri_test | intersector << 8 (rt_intersector)
inline V3 TraceSample(const Scene& s, const float* smp, uint32_t px, uint32_t py, uint32_t W, uint32_t H,
                      uint32_t si, int mode, orc_rec *rec)
{
    const int tri_test = mode & 0xFF, isect = mode >> 8;
    V3 o, d;
    GenRay(s.cam, px, py, W, H, smp[2 * si], smp[2 * si + 1], s.fov, o, d);
    float t = 0, u = 0, v = 0;
    uint32_t tri = 0xFFFFFFFFu, voxel = 0xFFFFFFFFu, steps = 0, tests = 0;
    bool hit;
    if (isect == 2) hit = RayMarch(s, o, d, t, steps, tests);
    else if (isect == 1) hit = IntersectBruteForce(s, o, d, t, u, v, tri, tests);
    else hit = Intersect(s, o, d, tri_test, t, u, v, tri, voxel, steps, tests);
    V3 c;
    if (hit && isect == 2)
    {
        c = mk(t / 3, t / 3, t / 3);                               // renderer.cpp:118 (depth)
        u = v = 0.0f;
        tri = 0xFFFFFFFFu;
    }
    else if (hit)
    {
        const Triangle& tr = s.tris[tri];
        c = ShadeHit(u, v, s.verts[tr.v0].n, s.verts[tr.v1].n, s.verts[tr.v2].n);
    }
    else
    {
        const float m = float(py) / float(H);
        c = mk(m, m, m);
        t = u = v = 0.0f;
        tri = 0xFFFFFFFFu;
    }
    if (rec)
    {
        rec->hit = hit; rec->tri = tri; rec->voxel = voxel; rec->steps = steps; rec->tests = tests;
        rec->t = t; rec->u = u; rec->v = v; rec->r = c.x; rec->g = c.y; rec->b = c.z; rec->pad = 0;
    }
    return c;
}

// renderer.cpp:43-136 Renderer::RenderTile
void RenderTile(const Scene& s, uint32_t W, uint32_t H, uint32_t spp, int tri_test,
                uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t *buf, uint32_t *hit_ids)
{
    const std::vector<float> smp = Hammersley(spp);
    const uint32_t tw = x1 - x0;
    orc_rec rec;
    for (uint32_t y=y0; y<y1; y++)
        for (uint32_t x=x0; x<x1; x++)
        {
            float cr = 0.0f, cg = 0.0f, cb = 0.0f;
            for (uint32_t si=0; si<spp; si++)
            {
                const V3 c = TraceSample(s, &smp[0], x, y, W, H, si, tri_test, hit_ids ? &rec : nullptr);
                cr += c.x; cg += c.y; cb += c.z;
                if (hit_ids) hit_ids[(size_t(y) * W + x) * spp + si] = rec.tri;
            }
            float fr = cr / float(spp), fg = cg / float(spp), fb = cb / float(spp);
            const float gamma = 1.0f / 2.0f;
            fr = std::pow(fr, gamma);
            fg = std::pow(fg, gamma);
            fb = std::pow(fb, gamma);
            buf[(x - x0) + (y - y0) * tw] = Pack(fr, fg, fb);
        }
}

bool ReadScene(const char *path, Scene& s)
{
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[8];
    uint32_t nv = 0, nt = 0;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "RTSCENE1", 8) == 0 &&
              std::fread(&s.id, 4, 1, f) == 1 && std::fread(&s.fov, 4, 1, f) == 1 &&
              std::fread(&s.cam[0][0], 4, 16, f) == 16 && std::fread(&nv, 4, 1, f) == 1 &&
              std::fread(&nt, 4, 1, f) == 1;
    if (ok)
    {
        s.verts.resize(nv);
        s.tris.resize(nt);
        for (auto& v : s.verts)
        {
            float b[6];
            ok = ok && std::fread(b, 4, 6, f) == 6;
            v.p = mk(b[0], b[1], b[2]); v.n = mk(b[3], b[4], b[5]);
        }
        for (auto& t : s.tris)
        {
            uint32_t b[6];
            ok = ok && std::fread(b, 4, 6, f) == 6;
            t.v0 = b[0]; t.v1 = b[1]; t.v2 = b[2];
            float n[3];
            std::memcpy(n, b + 3, 12);
            t.n = mk(n[0], n[1], n[2]);
        }
        for (const auto& t : s.tris)
            ok = ok && t.v0 < nv && t.v1 < nv && t.v2 < nv;
    }
    std::fclose(f);
    return ok && nt > 0;
}

inline float bitsf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

} // namespace

struct orc_scene { Scene s; };

extern "C" {

orc_scene *orc_scene_load(const char *path)
{
    std::unique_ptr<orc_scene> h(new orc_scene());
    if (!ReadScene(path, h->s)) return nullptr;
    BuildGrid(h->s, 64);
    return h.release();
}

void orc_scene_free(orc_scene *s) { delete s; }

int orc_scene_info(const orc_scene *h, orc_info *o)
{
    if (!h || !o) return 1;
    const Scene& s = h->s;
    o->scene_id = s.id;
    o->num_vertices = uint32_t(s.verts.size());
    o->num_triangles = uint32_t(s.tris.size());
    o->fov = s.fov;
    std::memcpy(o->cam, &s.cam[0][0], 64);
    for (int a=0; a<3; a++)
    {
        o->dims[a] = s.dim[a];
        o->aabb_min[a] = comp(s.aabb_min, a);
        o->aabb_max[a] = comp(s.aabb_max, a);
    }
    o->cell_wdh = s.cell_wdh;
    o->inv_cell_wdh = s.inv_cell_wdh;
    o->num_cells = uint32_t(s.off.size() - 1);
    o->num_refs = uint32_t(s.refs.size());
    uint32_t mx = 0;
    for (size_t c=0; c + 1<s.off.size(); c++) mx = std::max(mx, s.off[c + 1] - s.off[c]);
    o->max_refs_per_cell = mx;
    o->grid_build_s = s.build_s;
    return 0;
}

int orc_scene_csr(const orc_scene *h, uint32_t *offsets, uint32_t *refs)
{
    if (!h) return 1;
    std::copy(h->s.off.begin(), h->s.off.end(), offsets);
    std::copy(h->s.refs.begin(), h->s.refs.end(), refs);
    return 0;
}

int orc_scene_mesh(const orc_scene *h, float *vertices, uint32_t *triangles)
{
    if (!h) return 1;
    for (size_t i=0; i<h->s.verts.size(); i++)
    {
        const Vertex& v = h->s.verts[i];
        const float b[6] = { v.p.x, v.p.y, v.p.z, v.n.x, v.n.y, v.n.z };
        std::memcpy(vertices + 6 * i, b, 24);
    }
    for (size_t i=0; i<h->s.tris.size(); i++)
    {
        const Triangle& t = h->s.tris[i];
        const uint32_t b[6] = { t.v0, t.v1, t.v2, fbits(t.n.x), fbits(t.n.y), fbits(t.n.z) };
        std::memcpy(triangles + 6 * i, b, 24);
    }
    return 0;
}

int orc_render(const orc_scene *h, uint32_t W, uint32_t H, uint32_t spp, uint32_t tri_test,
               uint32_t nthreads, uint32_t *out, uint32_t *hit_ids, double *seconds)
{
    if (!h || !out || W == 0 || H == 0) return 1;
    spp = std::max(1u, spp);                                     // renderer.cpp:21
    if (nthreads == 0) nthreads = std::max(1u, std::thread::hardware_concurrency());
    // framebuffer.cpp:94-122: 12 x 9 tiles, edge tiles absorb the remainder
    const uint32_t TX = 12, TY = 9, tw = W / TX, th = H / TY;
    struct Tile { uint32_t x0, y0, x1, y1; std::vector<uint32_t> buf; };
    std::vector<Tile> tiles(TX * TY);
    for (uint32_t y=0; y<TY; y++)
        for (uint32_t x=0; x<TX; x++)
        {
            Tile& t = tiles[x + y * TX];
            t.x0 = x * tw; t.y0 = y * th;
            t.x1 = (x == TX - 1) ? W : (x + 1) * tw;
            t.y1 = (y == TY - 1) ? H : (y + 1) * th;
            t.buf.assign(size_t(t.x1 - t.x0) * (t.y1 - t.y0), 0);
        }
    // framebuffer.cpp:136-147 shuffled LIFO queue; framebuffer.cpp:43-92 workers
    std::vector<uint32_t> queue;
    for (uint32_t i=0; i<TX * TY; i++) queue.push_back(i);
    std::random_shuffle(queue.begin(), queue.end());
    std::mutex qm;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (uint32_t i=0; i<nthreads; i++)
        pool.emplace_back([&]() {
            while (true)
            {
                uint32_t idx;
                {
                    std::lock_guard<std::mutex> g(qm);
                    if (queue.empty()) break;
                    idx = queue.back();
                    queue.pop_back();
                }
                Tile& t = tiles[idx];
                RenderTile(h->s, W, H, spp, int(tri_test), t.x0, t.y0, t.x1, t.y1, &t.buf[0], hit_ids);
            }
        });
    for (auto& th : pool) th.join();
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (const auto& t : tiles)                                   // framebuffer.cpp:195-221 copy-out
        for (uint32_t y=t.y0; y<t.y1; y++)
            std::memcpy(out + size_t(y) * W + t.x0, &t.buf[size_t(y - t.y0) * (t.x1 - t.x0)],
                        size_t(t.x1 - t.x0) * 4);
    return 0;
}

int orc_trace_samples(const orc_scene *h, uint32_t W, uint32_t H, uint32_t spp, uint32_t tri_test,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t hh, orc_rec *out)
{
    if (!h || !out) return 1;
    spp = std::max(1u, spp);
    const std::vector<float> smp = Hammersley(spp);
    size_t i = 0;
    for (uint32_t y=y0; y<y0 + hh; y++)
        for (uint32_t x=x0; x<x0 + w; x++)
            for (uint32_t s=0; s<spp; s++)
                TraceSample(h->s, &smp[0], x, y, W, H, s, int(tri_test), &out[i++]);
    return 0;
}

void orc_hammersley(uint32_t spp, float *out)
{
    const std::vector<float> t = Hammersley(spp);
    std::copy(t.begin(), t.end(), out);
}

void orc_kat_ray_tri(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++, in += 18, out += 8)
    {
        const V3 o = mk(in[0], in[1], in[2]), d = mk(in[3], in[4], in[5]);
        const V3 a = mk(in[6], in[7], in[8]), b = mk(in[9], in[10], in[11]), c = mk(in[12], in[13], in[14]);
        const V3 nn = mk(in[15], in[16], in[17]);
        float t = NAN, u = NAN, v = NAN, bt = NAN, bu = NAN, bv = NAN;
        const bool h1 = RayTri(o, d, a, b, c, t, u, v);
        const bool h2 = RayTriBary(o, d, a, b, c, nn, bt, bu, bv);
        out[0] = bitsf(h1); out[1] = t; out[2] = u; out[3] = v;
        out[4] = bitsf(h2); out[5] = bt; out[6] = bu; out[7] = bv;
    }
}

void orc_kat_dist(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++)
    {
        const float *a = in + 12 * size_t(i);
        out[i] = DistancePointTri(mk(a[0], a[1], a[2]), mk(a[3], a[4], a[5]), mk(a[6], a[7], a[8]),
                                  mk(a[9], a[10], a[11]));
    }
}

void orc_kat_ray_aabb(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++, in += 12, out += 4)
    {
        const V3 o = mk(in[0], in[1], in[2]), d = mk(in[3], in[4], in[5]);
        const V3 mn = mk(in[6], in[7], in[8]), mx = mk(in[9], in[10], in[11]);
        float t0 = NAN, t1 = NAN;
        const bool h = RayAABB(o, d, mn, mx, t0, t1);
        out[0] = bitsf(h); out[1] = t0; out[2] = t1; out[3] = bitsf(PointAABB(o, mn, mx));
    }
}

void orc_kat_genray(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++, in += 23, out += 6)
    {
        float m[4][4];
        std::memcpy(&m[0][0], in, 64);
        V3 o, d;
        GenRay(m, fbits(in[16]), fbits(in[17]), fbits(in[18]), fbits(in[19]), in[20], in[21], in[22], o, d);
        out[0] = o.x; out[1] = o.y; out[2] = o.z; out[3] = d.x; out[4] = d.y; out[5] = d.z;
    }
}

void orc_kat_bgra8(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++, in += 3, out += 4)
    {
        const float gamma = 1.0f / 2.0f;
        const float r = std::pow(in[0], gamma), g = std::pow(in[1], gamma), b = std::pow(in[2], gamma);
        out[0] = r; out[1] = g; out[2] = b; out[3] = bitsf(Pack(r, g, b));
    }
}

void orc_kat_shade(const float *in, uint32_t n, float *out)
{
    for (uint32_t i=0; i<n; i++, in += 11, out += 3)
    {
        const V3 c = ShadeHit(in[0], in[1], mk(in[2], in[3], in[4]), mk(in[5], in[6], in[7]),
                              mk(in[8], in[9], in[10]));
        out[0] = c.x; out[1] = c.y; out[2] = c.z;
    }
}

// orc_render with another camera (Scene::GetCameraParameters' matrix and fov replaced): the same
// restated tile pool over a copy of the scene (test infrastructure: custom-view parity of the
// product walk -- cameras inside the grid, axis-aligned views)
int orc_render_cam(const orc_scene *h, uint32_t W, uint32_t H, uint32_t spp, const float *cam16, float fov,
                   uint32_t *out, uint32_t *hit_ids)
{
    if (!h || !cam16) return 1;
    orc_scene c = *h;
    std::memcpy(&c.s.cam[0][0], cam16, 64);
    c.s.fov = fov;
    double sec = 0.0;
    return orc_render(&c, W, H, spp, 0, 0, out, hit_ids, &sec);
}

} // extern "C"
