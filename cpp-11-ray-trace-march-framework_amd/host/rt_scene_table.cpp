// rt_scene_table.cpp -- mesh ingestion and the built-in scene table on the host (C++11).
//
// the reference builds every scene on the host from ASCII .dat meshes
// (Mesh::Read, mesh.cpp:138-391), normalises and transforms them (mesh.cpp:96-136), merges
// them (AddMesh / AddQuad / CornellBox, mesh.cpp:16-70) and places a look-at camera
// (Application::InitializeScene, application.cpp:304-517).  This file restates that data path
// so a .dat scene reaches rth_scene_from_mesh -> rt_scene_create without the reference, with
// every float operation in the reference's order (lin_alg.h is header-only float math; no
// contraction: the library is built with -ffp-contract=off like the reference's -std=c++11
// build).  Parity: tests/test_scene_table.py compares all 10 scenes bit for bit against the
// .rtscene dumps the reference's own code produced (oracle/ref_driver.cpp dump-scenes).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt_host.h"

int rth_internal_fail(int code, const std::string& msg);   // rt_host.cpp

namespace {

// ---- lin_alg.h vector / matrix restatement (float) ---------------------------------------

struct V3
{
    float x, y, z;
};

inline V3 v3(float a, float b, float c) { V3 r = { a, b, c }; return r; }
inline V3 operator-(const V3& a, const V3& b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator+(const V3& a, const V3& b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 scale(const V3& a, float s) { return v3(a.x * s, a.y * s, a.z * s); }       // lin_alg.h:85
inline V3 divide(const V3& a, float s) { return v3(a.x / s, a.y / s, a.z / s); }      // lin_alg.h:86

// lin_alg.h:136-142 Dot: accumulates from T() in component order
inline float dot(const V3& a, const V3& b)
{
    float r = 0.0f;
    r += a.x * b.x;
    r += a.y * b.y;
    r += a.z * b.z;
    return r;
}

// lin_alg.h:107-111 operator ^ (cross product)
inline V3 cross(const V3& a, const V3& b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// lin_alg.h:150-155 Normalize: reciprocal of the length, then a scale (NaN for a zero vector,
// exactly as the reference)
inline V3 normalize(const V3& a) { return scale(a, 1.0f / std::sqrt(dot(a, a))); }

inline V3 vmin(const V3& a, const V3& b) { return v3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)); }
inline V3 vmax(const V3& a, const V3& b) { return v3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)); }

// triangle.h:109-114 TriangleNormal
inline V3 tri_normal(const V3& p0, const V3& p1, const V3& p2) { return normalize(cross(p1 - p0, p2 - p0)); }

inline float deg_to_rad(float d) { return d * float(0.0174532925); }                // lin_alg.h:232

// Matrix44_t<float>: m[r][c] with the translation in row 3 (row-vector convention).  Set()
// (lin_alg.h:271-280) stores its k-th argument row-major TRANSPOSED: m[c][r] = f_rc.
struct M44
{
    float m[4][4];

    static M44 identity()
    {
        M44 a;
        std::memset(a.m, 0, sizeof(a.m));
        a.m[0][0] = a.m[1][1] = a.m[2][2] = a.m[3][3] = 1.0f;
        return a;
    }
    // Set(f11 .. f44) in reading order: f[r][c] lands in m[c][r]
    static M44 set(const float f[4][4])
    {
        M44 a;
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) a.m[c][r] = f[r][c];
        return a;
    }
    static M44 translation(float x, float y, float z)                                // lin_alg.h:317-327
    {
        const float f[4][4] = { { 1, 0, 0, x }, { 0, 1, 0, y }, { 0, 0, 1, z }, { 0, 0, 0, 1 } };
        return set(f);
    }
    static M44 scaling(float s)                                                      // lin_alg.h:469-475
    {
        const float f[4][4] = { { s, 0, 0, 0 }, { 0, s, 0, 0 }, { 0, 0, s, 0 }, { 0, 0, 0, 1 } };
        return set(f);
    }
    static M44 rotation_x(float deg)                                                 // lin_alg.h:330-343
    {
        const float r = deg_to_rad(deg), c = std::cos(r), s = std::sin(r);
        const float f[4][4] = { { 1, 0, 0, 0 }, { 0, c, -s, 0 }, { 0, s, c, 0 }, { 0, 0, 0, 1 } };
        return set(f);
    }
    static M44 rotation_y(float deg)                                                 // lin_alg.h:345-358
    {
        const float r = deg_to_rad(deg), c = std::cos(r), s = std::sin(r);
        const float f[4][4] = { { c, 0, -s, 0 }, { 0, 1, 0, 0 }, { s, 0, c, 0 }, { 0, 0, 0, 1 } };
        return set(f);
    }

    // lin_alg.h:477-493 Multiply: four products summed left to right
    M44 operator*(const M44& b) const
    {
        M44 r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++)
                r.m[i][j] = m[i][0] * b.m[0][j] + m[i][1] * b.m[1][j] + m[i][2] * b.m[2][j] + m[i][3] * b.m[3][j];
        return r;
    }

    M44 transposed() const                                                           // lin_alg.h:584-608
    {
        M44 r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) r.m[i][j] = m[j][i];
        return r;
    }

    V3 transf3x3(const V3& p) const                                                  // lin_alg.h:495-509
    {
        return v3(p.x * m[0][0] + p.y * m[1][0] + p.z * m[2][0],
                  p.x * m[0][1] + p.y * m[1][1] + p.z * m[2][1],
                  p.x * m[0][2] + p.y * m[1][2] + p.z * m[2][2]);
    }
    V3 transf4x4(const V3& p) const                                                  // lin_alg.h:518-535
    {
        return v3(p.x * m[0][0] + p.y * m[1][0] + p.z * m[2][0] + m[3][0],
                  p.x * m[0][1] + p.y * m[1][1] + p.z * m[2][1] + m[3][1],
                  p.x * m[0][2] + p.y * m[1][2] + p.z * m[2][2] + m[3][2]);
    }

    bool invert();
};

// Cofactor expansion of lin_alg.h:635-688 Invert (MESA GLU's __gluInvertMatrix) over the
// flattened matrix e[16]: out[k] = sum over six signed triple products e[a]*e[b]*e[c], each
// product evaluated (e[a] * e[b]) * e[c] and the six accumulated left to right in this order.
// Sign +1/-1, then the three element indices.
const signed char kCofactor[16][6][4] = {
    { { 1, 5, 10, 15 }, { -1, 5, 11, 14 }, { -1, 9, 6, 15 }, { 1, 9, 7, 14 }, { 1, 13, 6, 11 }, { -1, 13, 7, 10 } },
    { { -1, 1, 10, 15 }, { 1, 1, 11, 14 }, { 1, 9, 2, 15 }, { -1, 9, 3, 14 }, { -1, 13, 2, 11 }, { 1, 13, 3, 10 } },
    { { 1, 1, 6, 15 }, { -1, 1, 7, 14 }, { -1, 5, 2, 15 }, { 1, 5, 3, 14 }, { 1, 13, 2, 7 }, { -1, 13, 3, 6 } },
    { { -1, 1, 6, 11 }, { 1, 1, 7, 10 }, { 1, 5, 2, 11 }, { -1, 5, 3, 10 }, { -1, 9, 2, 7 }, { 1, 9, 3, 6 } },
    { { -1, 4, 10, 15 }, { 1, 4, 11, 14 }, { 1, 8, 6, 15 }, { -1, 8, 7, 14 }, { -1, 12, 6, 11 }, { 1, 12, 7, 10 } },
    { { 1, 0, 10, 15 }, { -1, 0, 11, 14 }, { -1, 8, 2, 15 }, { 1, 8, 3, 14 }, { 1, 12, 2, 11 }, { -1, 12, 3, 10 } },
    { { -1, 0, 6, 15 }, { 1, 0, 7, 14 }, { 1, 4, 2, 15 }, { -1, 4, 3, 14 }, { -1, 12, 2, 7 }, { 1, 12, 3, 6 } },
    { { 1, 0, 6, 11 }, { -1, 0, 7, 10 }, { -1, 4, 2, 11 }, { 1, 4, 3, 10 }, { 1, 8, 2, 7 }, { -1, 8, 3, 6 } },
    { { 1, 4, 9, 15 }, { -1, 4, 11, 13 }, { -1, 8, 5, 15 }, { 1, 8, 7, 13 }, { 1, 12, 5, 11 }, { -1, 12, 7, 9 } },
    { { -1, 0, 9, 15 }, { 1, 0, 11, 13 }, { 1, 8, 1, 15 }, { -1, 8, 3, 13 }, { -1, 12, 1, 11 }, { 1, 12, 3, 9 } },
    { { 1, 0, 5, 15 }, { -1, 0, 7, 13 }, { -1, 4, 1, 15 }, { 1, 4, 3, 13 }, { 1, 12, 1, 7 }, { -1, 12, 3, 5 } },
    { { -1, 0, 5, 11 }, { 1, 0, 7, 9 }, { 1, 4, 1, 11 }, { -1, 4, 3, 9 }, { -1, 8, 1, 7 }, { 1, 8, 3, 5 } },
    { { -1, 4, 9, 14 }, { 1, 4, 10, 13 }, { 1, 8, 5, 14 }, { -1, 8, 6, 13 }, { -1, 12, 5, 10 }, { 1, 12, 6, 9 } },
    { { 1, 0, 9, 14 }, { -1, 0, 10, 13 }, { -1, 8, 1, 14 }, { 1, 8, 2, 13 }, { 1, 12, 1, 10 }, { -1, 12, 2, 9 } },
    { { -1, 0, 5, 14 }, { 1, 0, 6, 13 }, { 1, 4, 1, 14 }, { -1, 4, 2, 13 }, { -1, 12, 1, 6 }, { 1, 12, 2, 5 } },
    { { 1, 0, 5, 10 }, { -1, 0, 6, 9 }, { -1, 4, 1, 10 }, { 1, 4, 2, 9 }, { 1, 8, 1, 6 }, { -1, 8, 2, 5 } },
};

bool M44::invert()
{
    const float *e = &m[0][0];
    float inv[16];
    for (int k = 0; k < 16; k++)
    {
        float acc = 0.0f;
        for (int t = 0; t < 6; t++)
        {
            const signed char *c = kCofactor[k][t];
            const float p = (e[c[1]] * e[c[2]]) * e[c[3]];
            // the first term starts the sum ((-a) * b * c == -(a * b * c) exactly)
            acc = t == 0 ? (c[0] > 0 ? p : -p) : (c[0] > 0 ? acc + p : acc - p);
        }
        inv[k] = acc;
    }
    float det = e[0] * inv[0] + e[1] * inv[4] + e[2] * inv[8] + e[3] * inv[12];
    if (det == 0.0f) return false;
    det = 1.0f / det;
    for (int i = 0; i < 16; i++) (&m[0][0])[i] = inv[i] * det;
    return true;
}

// lin_alg.h:431-467 BuildLookAtMatrix (up = +Y)
M44 look_at(const V3& eye, const V3& at)
{
    const V3 up = v3(0.0f, 1.0f, 0.0f);
    const V3 z = normalize(eye - at);
    const V3 x = normalize(cross(up, z));
    const V3 y = normalize(cross(z, x));
    M44 rot = M44::identity();
    rot.m[0][0] = x.x; rot.m[0][1] = x.y; rot.m[0][2] = x.z;
    rot.m[1][0] = y.x; rot.m[1][1] = y.y; rot.m[1][2] = y.z;
    rot.m[2][0] = z.x; rot.m[2][1] = z.y; rot.m[2][2] = z.z;
    return M44::translation(dot(x, eye), dot(y, eye), dot(z, eye)) * rot;
}

// ---- Mesh (mesh.h) ------------------------------------------------------------------------

struct Mesh
{
    std::vector<rt_vertex> vtx;
    std::vector<rt_triangle> tri;

    static V3 pos(const rt_vertex& v) { return v3(v.p[0], v.p[1], v.p[2]); }
    static V3 nrm(const rt_vertex& v) { return v3(v.n[0], v.n[1], v.n[2]); }
    static void put(float *d, const V3& a) { d[0] = a.x; d[1] = a.y; d[2] = a.z; }

    // mesh.cpp:27-53 AddQuad: 4 vertices sharing the face normal of (q0, q1, q2), split 012 / 023
    void add_quad(const float *q)
    {
        const V3 n = tri_normal(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), v3(q[6], q[7], q[8]));
        const uint32_t base = uint32_t(vtx.size());
        for (int i = 0; i < 4; i++)
        {
            rt_vertex v;
            put(v.p, v3(q[3 * i], q[3 * i + 1], q[3 * i + 2]));
            put(v.n, n);
            vtx.push_back(v);
        }
        rt_triangle t;
        put(t.n, n);
        t.v0 = base; t.v1 = base + 1; t.v2 = base + 2;
        tri.push_back(t);
        t.v0 = base; t.v1 = base + 2; t.v2 = base + 3;
        tri.push_back(t);
    }

    // mesh.cpp:55-70 AddMesh
    void add_mesh(const Mesh& o)
    {
        const uint32_t off = uint32_t(vtx.size());
        vtx.insert(vtx.end(), o.vtx.begin(), o.vtx.end());
        for (rt_triangle t : o.tri)
        {
            t.v0 += off; t.v1 += off; t.v2 += off;
            tri.push_back(t);
        }
    }

    // mesh.cpp:72-94 ComputeAABB over the vertices referenced by triangles (float::min() seed)
    void aabb(V3& mn, V3& mx) const
    {
        if (tri.empty())
        {
            mn = mx = v3(0.0f, 0.0f, 0.0f);
            return;
        }
        const float hi = std::numeric_limits<float>::max(), lo = std::numeric_limits<float>::min();
        mn = v3(hi, hi, hi);
        mx = v3(lo, lo, lo);
        for (const rt_triangle& t : tri)
            for (uint32_t i : { t.v0, t.v1, t.v2 })
            {
                mn = vmin(mn, pos(vtx[i]));
                mx = vmax(mx, pos(vtx[i]));
            }
    }

    // mesh.cpp:96-119 Transform: normals by the inverse transpose, renormalised
    bool transform(const M44& mat)
    {
        M44 it = mat;
        if (!it.invert()) return false;
        it = it.transposed();
        for (rt_triangle& t : tri) put(t.n, normalize(it.transf3x3(v3(t.n[0], t.n[1], t.n[2]))));
        for (rt_vertex& v : vtx)
        {
            put(v.p, mat.transf4x4(pos(v)));
            put(v.n, normalize(it.transf3x3(nrm(v))));
        }
        return true;
    }

    // mesh.cpp:121-136 NormalizeDimensions: centre, then scale the longest extent to 1
    bool normalize_dimensions()
    {
        V3 mn, mx;
        aabb(mn, mx);
        const V3 c = divide(mn + mx, 2.0f);
        const V3 ext = mx - mn;
        return transform(M44::translation(-c.x, -c.y, -c.z) *
                         M44::scaling(1.0f / std::max(std::max(ext.x, ext.y), ext.z)));
    }

    bool read(const std::string& path, bool flip_winding, std::string& err);
};

// mesh.cpp:138-391 Mesh::Read: ASCII .dat, indexed ("<nv>\n\n<vertices>\n<ni>\n\n<indices>")
// or a flat vertex list, vertices "x y z [nx ny nz [u v | r g b]]".  Same stdio calls and
// format strings as the reference, so every float is parsed by the same strtof.
bool Mesh::read(const std::string& path, bool flip_winding, std::string& err)
{
    vtx.clear();
    tri.clear();
    std::unique_ptr<std::FILE, int (*)(std::FILE *)> fh(std::fopen(path.c_str(), "r"), std::fclose);
    std::FILE *f = fh.get();
    if (!f)
    {
        err = "can't open " + path;
        return false;
    }
    char line[1024];
    if (!std::fgets(line, sizeof(line), f)) { err = "can't read 1st line"; return false; }
    const bool indexed = std::strchr(line, ' ') == nullptr;   // a bare count line
    std::rewind(f);

    unsigned nv_decl = 0;
    if (indexed)
    {
        if (std::fscanf(f, "%i\n\n", reinterpret_cast<int *>(&nv_decl)) != 1) { err = "no vertex count"; return false; }
        if (nv_decl < 3) { err = "invalid vertex count"; return false; }
    }
    const long first = std::ftell(f);
    if (!std::fgets(line, sizeof(line), f)) { err = "can't read 1st vertex"; return false; }
    std::fseek(f, first, SEEK_SET);

    float scratch[9];
    const int fields = std::sscanf(line, "%f %f %f %f %f %f %f %f %f", &scratch[0], &scratch[1], &scratch[2],
                                   &scratch[3], &scratch[4], &scratch[5], &scratch[6], &scratch[7], &scratch[8]);
    if (fields != 3 && fields != 6 && fields != 8 && fields != 9) { err = "invalid vertex spec"; return false; }
    const bool has_normal = fields >= 6;

    unsigned nv = 0;
    while (std::feof(f) == 0)
    {
        rt_vertex v;
        v.n[0] = v.n[1] = v.n[2] = 0.0f;
        if (std::fscanf(f, "%f %f %f ", &v.p[0], &v.p[1], &v.p[2]) != 3) { err = "can't read position"; return false; }
        if (has_normal)
        {
            if (std::fscanf(f, "%f %f %f ", &v.n[0], &v.n[1], &v.n[2]) != 3) { err = "can't read normal"; return false; }
            if (fields == 8 && std::fscanf(f, "%f %f ", &scratch[0], &scratch[1]) != 2) { err = "can't read UV"; return false; }
            if (fields == 9 && std::fscanf(f, "%f %f %f ", &scratch[0], &scratch[1], &scratch[2]) != 3)
            {
                err = "can't read RGB";
                return false;
            }
        }
        vtx.push_back(v);
        nv++;
        if (indexed && nv >= nv_decl) break;
    }
    if (nv == 0 || (indexed && nv != nv_decl)) { err = "can't read all vertices"; return false; }
    if (!indexed && nv % 3 != 0) { err = "invalid vertex count"; return false; }

    unsigned nt;
    if (indexed)
    {
        unsigned ni = 0;
        if (std::fscanf(f, "%i\n\n", reinterpret_cast<int *>(&ni)) != 1) { err = "no index count"; return false; }
        if (ni < 3 || ni % 3 != 0) { err = "invalid index count"; return false; }
        nt = ni / 3;
    }
    else
        nt = nv / 3;
    tri.resize(nt);
    for (unsigned i = 0; i < nt; i++)
    {
        rt_triangle& t = tri[i];
        if (indexed)
        {
            if (std::fscanf(f, "%i %i %i ", reinterpret_cast<int *>(&t.v0), reinterpret_cast<int *>(&t.v1),
                            reinterpret_cast<int *>(&t.v2)) != 3)
            {
                err = "can't read triangle indices";
                return false;
            }
            if (t.v0 >= nv || t.v1 >= nv || t.v2 >= nv) { err = "vertex index out of bounds"; return false; }
        }
        else
        {
            t.v0 = 3 * i;
            t.v1 = 3 * i + 1;
            t.v2 = 3 * i + 2;
        }
        if (flip_winding) std::swap(t.v0, t.v1);
        put(t.n, tri_normal(pos(vtx[t.v0]), pos(vtx[t.v1]), pos(vtx[t.v2])));
    }
    // position-only meshes take the face normals as vertex normals, later triangles winning
    if (!has_normal)
        for (const rt_triangle& t : tri)
            for (uint32_t k : { t.v0, t.v1, t.v2 }) std::memcpy(vtx[k].n, t.n, sizeof(t.n));
    return true;
}

// data/meshes/cornell_box_quads.txt: the reference's g_cornell_quads (cornell_box.cpp), dumped
// by oracle/_ref/refdriver cornell-quads -- geometry data, 16 quads x 4 vertices
bool cornell_box(Mesh& m, const std::string& data_dir, std::string& err)
{
    const std::string path = data_dir + "/cornell_box_quads.txt";
    std::unique_ptr<std::FILE, int (*)(std::FILE *)> fh(std::fopen(path.c_str(), "r"), std::fclose);
    if (!fh) { err = "can't open " + path; return false; }
    unsigned nq = 0;
    if (std::fscanf(fh.get(), "%u", &nq) != 1 || nq == 0 || nq > 1024) { err = "bad quad count"; return false; }
    std::vector<float> q(size_t(nq) * 12);
    for (float& x : q)
        if (std::fscanf(fh.get(), "%f", &x) != 1) { err = "bad quad data"; return false; }
    m.vtx.clear();
    m.tri.clear();
    for (unsigned i = 0; i < nq; i++) m.add_quad(&q[12 * size_t(i)]);        // mesh.cpp:16-25
    return true;
}

struct Built
{
    Mesh mesh;
    M44 cam;
    float fov;
};

// Application::InitializeScene (application.cpp:304-517), scenes 0-9
bool build_scene(uint32_t id, const std::string& md, const std::string& data_dir, Built& b, std::string& err)
{
    Mesh& m = b.mesh;
    b.fov = 45.0f;
    auto rd = [&](Mesh& into, const char *name, bool flip) {
        return into.read(md + "/" + name, flip, err) && into.normalize_dimensions();
    };
    auto quad = [&](Mesh& into, float x0, float x1, float y, float z0, float z1) {
        const float q[12] = { x0, y, z1, x1, y, z1, x1, y, z0, x0, y, z0 };
        into.add_quad(q);
    };
    switch (id)
    {
    case 0:
        if (!rd(m, "torusknot_column_teapot_plane.dat", false)) return false;
        b.cam = look_at(v3(-1.00001f, 1.0f, 1.0f), v3(0.0f, -0.2f, 0.0f));
        b.fov = 51.0f;
        return true;
    case 1:
    {
        if (!cornell_box(m, data_dir, err) || !m.normalize_dimensions()) return false;
        Mesh cube;
        if (!rd(cube, "cube.dat", false)) return false;
        if (!cube.transform(M44::scaling(0.25f) * M44::rotation_x(45.0f) * M44::rotation_y(45.0f) *
                            M44::translation(0.0f, 0.3f, 0.0f)))
            return false;
        m.add_mesh(cube);
        b.cam = look_at(v3(0.0f, 0.0f, -2.0f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 51.0f;
        return true;
    }
    case 2:
        if (!rd(m, "room_table_chair_tv.dat", false)) return false;
        b.cam = look_at(v3(-0.47f, 0.15f, -0.3f), v3(1.0f, -0.7f, 0.9f));
        b.fov = 90.0f;
        return true;
    case 3:
        if (!rd(m, "table_chair.dat", true)) return false;
        quad(m, -1.2f, 1.2f, -0.219097f, -1.2f, 1.2f);
        b.cam = look_at(v3(1.001f, 1.002f, -1.0f), v3(0.0f, 0.0f, -0.3f));
        b.fov = 45.0f;
        return true;
    case 4:
        if (!rd(m, "head.dat", false) || !m.transform(M44::rotation_y(30.0f))) return false;
        b.cam = look_at(v3(0.0f, 0.0f, -1.0f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 75.0f;
        return true;
    case 5:
    {
        Mesh cat;
        if (!rd(m, "room_three_windows_two_columns.dat", false) || !rd(cat, "cat.dat", false)) return false;
        if (!cat.transform(M44::scaling(0.25f) * M44::rotation_y(30.0f) * M44::translation(-0.065f, -0.1f, 0.05f)))
            return false;
        m.add_mesh(cat);
        b.cam = look_at(v3(-0.2f, 0.0f, -0.33f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 90.0f;
        return true;
    }
    case 6:
    {
        Mesh knot;
        if (!rd(m, "water_surface.dat", false) || !rd(knot, "torus_knot.dat", false)) return false;
        if (!knot.transform(M44::scaling(0.25f) * M44::translation(-0.0f, 0.2f, 0.0f))) return false;
        m.add_mesh(knot);
        b.cam = look_at(v3(-1.0f, 2.0f, -1.0f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 30.0f;
        return true;
    }
    case 7:
    {
        Mesh pot;
        if (!rd(m, "griebel.dat", false) || !rd(pot, "teapot.dat", false)) return false;
        if (!pot.transform(M44::scaling(0.3f) * M44::rotation_y(90.0f) * M44::translation(0.0f, 0.1f, 0.0f)))
            return false;
        m.add_mesh(pot);
        b.cam = look_at(v3(float(0.5), float(0.5), 0.0f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 75.0f;
        return true;
    }
    case 8:
        if (!rd(m, "killeroo.dat", false)) return false;
        quad(m, -0.75f, 0.75f, -0.229267f, -0.75f, 0.75f);
        b.cam = look_at(v3(-1.6f, 1.2f, -1.0f), v3(0.0f, 0.0f, float(-0.1)));
        b.fov = 30.0f;
        return true;
    case 9:
    {
        Mesh dwarf, hand, blob;
        if (!rd(dwarf, "d3d_dwarf.dat", false) || !dwarf.transform(M44::translation(0.0f, 0.500100f, 0.0f)))
            return false;
        m.add_mesh(dwarf);
        if (!rd(hand, "hand.dat", false) ||
            !hand.transform(M44::rotation_x(90.0f) * M44::rotation_y(90.0f) * M44::translation(0.7f, 0.490801f, 0.0f)))
            return false;
        m.add_mesh(hand);
        if (!rd(blob, "blob.dat", false) ||
            !blob.transform(M44::scaling(0.6f) * M44::translation(-0.8f, 0.278176f, 0.0f)))
            return false;
        m.add_mesh(blob);
        quad(m, -1.5f, 1.5f, 0.0f, -1.0f, 1.0f);
        b.cam = look_at(v3(0.0f, 1.5f, -2.0f), v3(0.0f, 0.0f, 0.0f));
        b.fov = 60.0f;
        return true;
    }
    default:
        err = "scene id must be 0..9";
        return false;
    }
}

} // namespace

struct rth_mesh
{
    Mesh mesh;
};

extern "C" {

int rth_mesh_read(const char *path, int flip_winding, rth_mesh **out)
{
    if (!path || !out) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    std::unique_ptr<rth_mesh> m(new rth_mesh);
    std::string err;
    if (!m->mesh.read(path, flip_winding != 0, err)) return rth_internal_fail(RT_E_INVALID, "Mesh::Read: " + err);
    *out = m.release();
    return RT_OK;
}

int rth_mesh_normalize_dimensions(rth_mesh *m)
{
    if (!m) return rth_internal_fail(RT_E_INVALID, "NULL mesh");
    if (!m->mesh.normalize_dimensions()) return rth_internal_fail(RT_E_INVALID, "singular normalisation matrix");
    return RT_OK;
}

int rth_mesh_transform(rth_mesh *m, const float mat[16])
{
    if (!m || !mat) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    M44 a;
    std::memcpy(a.m, mat, sizeof(a.m));
    if (!m->mesh.transform(a)) return rth_internal_fail(RT_E_INVALID, "Transform: matrix not invertible");
    return RT_OK;
}

int rth_mesh_add_quad(rth_mesh *m, const float quad[12])
{
    if (!m || !quad) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    m->mesh.add_quad(quad);
    return RT_OK;
}

int rth_mesh_add_mesh(rth_mesh *m, const rth_mesh *other)
{
    if (!m || !other) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    m->mesh.add_mesh(other->mesh);
    return RT_OK;
}

int rth_mesh_data(const rth_mesh *m, const rt_vertex **vertices, uint32_t *num_vertices,
                  const rt_triangle **triangles, uint32_t *num_triangles)
{
    if (!m || !vertices || !num_vertices || !triangles || !num_triangles)
        return rth_internal_fail(RT_E_INVALID, "NULL argument");
    *vertices = m->mesh.vtx.data();
    *num_vertices = uint32_t(m->mesh.vtx.size());
    *triangles = m->mesh.tri.data();
    *num_triangles = uint32_t(m->mesh.tri.size());
    return RT_OK;
}

void rth_mesh_free(rth_mesh *m) { delete m; }

int rth_look_at(const float eye[3], const float at[3], float cam[16])
{
    if (!eye || !at || !cam) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    const M44 c = look_at(v3(eye[0], eye[1], eye[2]), v3(at[0], at[1], at[2]));
    std::memcpy(cam, c.m, sizeof(c.m));
    return RT_OK;
}

int rth_scene_table(uint32_t scene_id, const char *mesh_dir, const char *data_dir, uint32_t nthreads,
                    rth_scene **out)
{
    if (!mesh_dir || !data_dir || !out) return rth_internal_fail(RT_E_INVALID, "NULL argument");
    Built b;
    std::string err;
    if (!build_scene(scene_id, mesh_dir, data_dir, b, err))
        return rth_internal_fail(RT_E_INVALID, "scene " + std::to_string(scene_id) + ": " + (err.empty() ? "transform failed" : err));
    // Scene::Scene builds Grid(mesh, 64) (scene.cpp:6-7)
    const int rc = rth_scene_from_mesh(b.mesh.vtx.data(), uint32_t(b.mesh.vtx.size()), b.mesh.tri.data(),
                                       uint32_t(b.mesh.tri.size()), b.fov, &b.cam.m[0][0], 64, nthreads, out);
    if (rc == RT_OK) rth_scene_set_id(*out, scene_id);
    return rc;
}

} // extern "C"
