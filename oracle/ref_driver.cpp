// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A headless driver around the reference's OWN translation units, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/refdriver.  It is the parity
// anchor ("the real reference run here") for everything under tests/golden/.
//
// What is the reference's own code here:
//   Mesh::Read / Transform / NormalizeDimensions / AddQuad / AddMesh / CornellBox  (mesh.cpp)
//   Grid::Grid (voxelizer) and Grid::Intersect (3D-DDA)                         (grid.cpp)
//   GenerateRay (camera.h), IntersectRayTri / IntersectRayTriBarycentric /
//   BarycentricInterpolate (triangle.h), IntersectRayAABB / IntersectPointAABB (aabb.h),
//   Normalize / ToBGRA8 / Matrix44 ops (lin_alg.h), SAMP::HammersleySequence (sampling.*)
// What is restated here (because renderer.cpp / framebuffer.cpp / application.cpp
// include <OpenGL/gl.h> or GLUT, which this image lacks -- unbuildable):
//   * the scene table of Application::InitializeScene        (application.cpp:304-517)
//   * the per-pixel/per-sample loop body of Renderer::RenderTile (renderer.cpp:43-136)
//   * the 12x9 std::thread tile pool of Framebuffer           (framebuffer.cpp:10-130)
//   * the loops of Renderer::IntersectBruteForce / DistanceBruteForce / RayMarch
//     (renderer.cpp:24-41, 138-197) around the reference's IntersectRayTri / DistancePointTri
// The restated glue only sequences calls into the reference's functions above.
//
// Subcommands (all output little-endian binary files or one "RESULT {json}" line):
//   dump-scenes <meshdir> <outdir>           post-setup meshes + cameras -> <outdir>/scene<i>.rtscene
//   grid   <scene.rtscene> <out.bin>         grid meta + CSR export of Grid::Grid's cells
//   render <scene.rtscene> W H spp [--threads N] [--reps R] [--out f] [--hits f] [--bmp f]
//                                            --bmp: the reference's WriteBitmap of the gathered frame
//   samples <scene.rtscene> W H spp x0 y0 w h <out.bin>    per-sample records; refdriver_instr
//                                            (grid.cpp + ref_instr.h) appends voxel, steps, tests
//   alt-samples <scene.rtscene> W H spp x0 y0 w h brute|march <out.bin>
//                                            records of Renderer::IntersectBruteForce / RayMarch
//   render ... [--isect grid|brute|march]   the frame with another intersector (renderer.cpp:103-105)
//   kat <outdir>                             primitive known-answer vectors
//   kat-dist <out.f32>                       DistancePointTri known answers

#include <memory>
#include <vector>
#include <array>
#include <cstdio>
#include <thread>
#include <mutex>
#include <atomic>
#include <random>
#include <algorithm>
#include <cassert>
#include <cstdlib>
#include <cstring>
#include <string>
#include <limits>

#include "types.h"
#include "lin_alg.h"
#include "mesh.h"
#include "cornell_box.h"
#include "grid.h"
#include "sampling.h"
#include "camera.h"
#include "triangle.h"
#include "aabb.h"
#include "timer.h"
#include "bmp_writer.h"

#ifdef RT_REF_INSTR
#define RT_REF_INSTR_NO_HOOKS
#include "ref_instr.h"
thread_local RtRefWalk g_rt_ref_walk;   // written by the instrumented grid.cpp (ref_instr.h)
#endif

namespace {

// ---------------------------------------------------------------- scene files
// .rtscene: "RTSCENE1" | u32 scene_id | f32 fov | f32 cam[16] (m_mat[4][4] row-major)
//           | u32 nv | u32 nt | nv x {f32 p[3], f32 n[3]} | nt x {u32 v0,v1,v2, f32 n[3]}
struct SceneFile
{
    uint32 id = 0;
    float fov = 45.0f;
    Matrix44f cam;
    std::unique_ptr<Mesh> mesh;
};

bool WriteScene(const char *path, uint32 id, float fov, const Matrix44f& cam, const Mesh& m)
{
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    std::fwrite("RTSCENE1", 1, 8, f);
    std::fwrite(&id, 4, 1, f);
    std::fwrite(&fov, 4, 1, f);
    std::fwrite(&cam.m_mat[0][0], 4, 16, f);
    const uint32 nv = uint32(m.m_vertices.size()), nt = uint32(m.m_triangles.size());
    std::fwrite(&nv, 4, 1, f);
    std::fwrite(&nt, 4, 1, f);
    for (const auto& v : m.m_vertices)
    {
        std::fwrite(&v.p.m_vec[0], 4, 3, f);
        std::fwrite(&v.n.m_vec[0], 4, 3, f);
    }
    for (const auto& t : m.m_triangles)
    {
        const uint32 idx[3] = { t.v0, t.v1, t.v2 };
        std::fwrite(idx, 4, 3, f);
        std::fwrite(&t.n.m_vec[0], 4, 3, f);
    }
    std::fclose(f);
    return true;
}

bool ReadScene(const char *path, SceneFile& s)
{
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[8];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "RTSCENE1", 8) == 0;
    uint32 nv = 0, nt = 0;
    ok = ok && std::fread(&s.id, 4, 1, f) == 1 && std::fread(&s.fov, 4, 1, f) == 1 &&
         std::fread(&s.cam.m_mat[0][0], 4, 16, f) == 16 &&
         std::fread(&nv, 4, 1, f) == 1 && std::fread(&nt, 4, 1, f) == 1;
    s.mesh.reset(new Mesh());
    if (ok)
    {
        s.mesh->m_vertices.resize(nv);
        s.mesh->m_triangles.resize(nt);
        for (auto& v : s.mesh->m_vertices)
            ok = ok && std::fread(&v.p.m_vec[0], 4, 3, f) == 3 && std::fread(&v.n.m_vec[0], 4, 3, f) == 3;
        for (auto& t : s.mesh->m_triangles)
        {
            uint32 idx[3];
            ok = ok && std::fread(idx, 4, 3, f) == 3 && std::fread(&t.n.m_vec[0], 4, 3, f) == 3;
            t.v0 = idx[0]; t.v1 = idx[1]; t.v2 = idx[2];
        }
    }
    std::fclose(f);
    return ok;
}

// ------------------------------------------------- scene table (application.cpp:304-517)
// Restated call-for-call; every numeric literal and the order of Mesh operations follow
// the cited lines so the post-setup mesh is the one the reference renders.
bool BuildScene(uint id, const std::string& dir, Mesh& mesh, Matrix44f& cam_mat, float& fov)
{
    auto P = [&](const char *n) { return dir + "/" + n; };
    fov = 45.0f;
    switch (id)
    {
    case 0: // application.cpp:312-317
        if (!mesh.Read(P("torusknot_column_teapot_plane.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        cam_mat.BuildLookAtMatrix(Vec3f(-1.00001f, 1.0f, 1.0f), Vec3f(0.0f, -0.2f, 0.0f));
        fov = 51.0f;
        return true;
    case 1: // application.cpp:319-341
    {
        mesh.CornellBox();
        mesh.NormalizeDimensions();
        Mesh cube;
        if (!cube.Read(P("cube.dat").c_str())) return false;
        cube.NormalizeDimensions();
        Matrix44f scale, roty, rotx, trans;
        scale.Scaling(0.25f);
        rotx.RotationX(45.0f);
        roty.RotationY(45.0f);
        trans.Translation(0.0f, 0.3f, 0.0f);
        cube.Transform(scale * rotx * roty * trans);
        mesh.AddMesh(cube);
        cam_mat.BuildLookAtMatrix(Vec3f(0.0f, 0.0f, -2.0f), Vec3f(0.0f));
        fov = 51.0f;
        return true;
    }
    case 2: // application.cpp:343-348
        if (!mesh.Read(P("room_table_chair_tv.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        cam_mat.BuildLookAtMatrix(Vec3f(-0.47f, 0.15f, -0.3f), Vec3f(1.0f, -0.7f, 0.9f));
        fov = 90.0f;
        return true;
    case 3: // application.cpp:350-366
    {
        if (!mesh.Read(P("table_chair.dat").c_str(), true)) return false;
        mesh.NormalizeDimensions();
        const float quad[4][3] { { -1.2f, -0.219097f,  1.2f }, {  1.2f, -0.219097f,  1.2f },
                                 {  1.2f, -0.219097f, -1.2f }, { -1.2f, -0.219097f, -1.2f } };
        mesh.AddQuad(&quad[0][0]);
        cam_mat.BuildLookAtMatrix(Vec3f(1.001f, 1.002f, -1.0f), Vec3f(0.0f, 0.0f, -0.3f));
        fov = 45.0f;
        return true;
    }
    case 4: // application.cpp:368-378
    {
        if (!mesh.Read(P("head.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        Matrix44f roty;
        roty.RotationY(30.0f);
        mesh.Transform(roty);
        cam_mat.BuildLookAtMatrix(Vec3f(0.0f, 0.0f, -1.0f), Vec3f(0.0f));
        fov = 75.0f;
        return true;
    }
    case 5: // application.cpp:380-399
    {
        if (!mesh.Read(P("room_three_windows_two_columns.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        Mesh extra;
        if (!extra.Read(P("cat.dat").c_str())) return false;
        extra.NormalizeDimensions();
        Matrix44f scale, roty, trans;
        scale.Scaling(0.25f);
        roty.RotationY(30.0f);
        trans.Translation(-0.065f, -0.1f, 0.05f);
        extra.Transform(scale * roty * trans);
        mesh.AddMesh(extra);
        cam_mat.BuildLookAtMatrix(Vec3f(-0.2f, 0.0f, -0.33f), Vec3f(0.0f, 0.0f, 0.0f));
        fov = 90.0f;
        return true;
    }
    case 6: // application.cpp:401-419
    {
        if (!mesh.Read(P("water_surface.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        Mesh extra;
        if (!extra.Read(P("torus_knot.dat").c_str())) return false;
        extra.NormalizeDimensions();
        Matrix44f scale, trans;
        scale.Scaling(0.25f);
        trans.Translation(-0.0f, 0.2f, 0.0f);
        extra.Transform(scale * trans);
        mesh.AddMesh(extra);
        cam_mat.BuildLookAtMatrix(Vec3f(-1.0f, 2.0f, -1.0f), Vec3f(0.0f, 0.0f, 0.0f));
        fov = 30.0f;
        return true;
    }
    case 7: // application.cpp:421-440
    {
        if (!mesh.Read(P("griebel.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        Mesh extra;
        if (!extra.Read(P("teapot.dat").c_str())) return false;
        extra.NormalizeDimensions();
        Matrix44f scale, roty, trans;
        scale.Scaling(0.3f);
        roty.RotationY(90.0f);
        trans.Translation(0.0f, 0.1f, 0.0f);
        extra.Transform(scale * roty * trans);
        mesh.AddMesh(extra);
        cam_mat.BuildLookAtMatrix(Vec3f(0.5, 0.5, 0.0f), Vec3f(0.0f, 0.0f, 0.0f));
        fov = 75.0f;
        return true;
    }
    case 8: // application.cpp:442-458
    {
        if (!mesh.Read(P("killeroo.dat").c_str())) return false;
        mesh.NormalizeDimensions();
        const float quad[4][3] { { -0.75f, -0.229267f,  0.75f }, {  0.75f, -0.229267f,  0.75f },
                                 {  0.75f, -0.229267f, -0.75f }, { -0.75f, -0.229267f, -0.75f } };
        mesh.AddQuad(&quad[0][0]);
        cam_mat.BuildLookAtMatrix(Vec3f(-1.6f, 1.2f, -1.0f), Vec3f(0.0f, 0.0f, -0.1));
        fov = 30.0f;
        return true;
    }
    case 9: // application.cpp:460-500
    {
        Matrix44f mat_trans, mat_scale, mat_rotx, mat_roty;
        Mesh dwarf;
        if (!dwarf.Read(P("d3d_dwarf.dat").c_str())) return false;
        dwarf.NormalizeDimensions();
        mat_trans.Translation(0.0f, 0.500100f, 0.0f);
        dwarf.Transform(mat_trans);
        mesh.AddMesh(dwarf);
        Mesh hand;
        if (!hand.Read(P("hand.dat").c_str())) return false;
        hand.NormalizeDimensions();
        mat_rotx.RotationX(90.0f);
        mat_roty.RotationY(90.0f);
        mat_trans.Translation(0.7f, 0.490801f, 0.0f);
        hand.Transform(mat_rotx * mat_roty * mat_trans);
        mesh.AddMesh(hand);
        Mesh blob;
        if (!blob.Read(P("blob.dat").c_str())) return false;
        blob.NormalizeDimensions();
        mat_trans.Translation(-0.8f, 0.278176f, 0.0f);
        mat_scale.Scaling(0.6f);
        blob.Transform(mat_scale * mat_trans);
        mesh.AddMesh(blob);
        const float quad[4][3] { { -1.5f, 0.0f,  1.0f }, {  1.5f, 0.0f,  1.0f },
                                 {  1.5f, 0.0f, -1.0f }, { -1.5f, 0.0f, -1.0f } };
        mesh.AddQuad(&quad[0][0]);
        cam_mat.BuildLookAtMatrix(Vec3f(0.0f, 1.5f, -2.0f), Vec3f(0.0f, 0.0f, 0.0f));
        fov = 60.0f;
        return true;
    }
    default:
        return false;
    }
}

// Grid subclass: the reference keeps the cells protected (grid.h:25-39); this only reads them.
struct GridExport : public Grid
{
    GridExport(std::unique_ptr<Mesh> mesh, uint res) : Grid(std::move(mesh), res) { }
    void Export(std::FILE *f) const
    {
        // u32 dims[3] | f32 aabb_min[3] | f32 aabb_max[3] | f32 cell_wdh | f32 inv_cell_wdh
        // | u32 ncells | u32 nrefs | u32 offsets[ncells+1] | u32 refs[nrefs]
        std::fwrite(m_grid_dim, 4, 3, f);
        std::fwrite(&m_aabb_min.m_vec[0], 4, 3, f);
        std::fwrite(&m_aabb_max.m_vec[0], 4, 3, f);
        std::fwrite(&m_cell_wdh, 4, 1, f);
        std::fwrite(&m_inv_cell_wdh, 4, 1, f);
        const uint32 nc = uint32(m_cells.size());
        uint32 nr = 0;
        for (const auto& c : m_cells) nr += uint32(c.m_isect_tri_idx.size());
        std::fwrite(&nc, 4, 1, f);
        std::fwrite(&nr, 4, 1, f);
        uint32 off = 0;
        for (const auto& c : m_cells) { std::fwrite(&off, 4, 1, f); off += uint32(c.m_isect_tri_idx.size()); }
        std::fwrite(&off, 4, 1, f);
        for (const auto& c : m_cells)
            if (!c.m_isect_tri_idx.empty())
                std::fwrite(&c.m_isect_tri_idx[0], 4, c.m_isect_tri_idx.size(), f);
    }
};

// ----------------------------------------- per-sample loop (renderer.cpp:74-135, glue only)
struct Frame
{
    const Grid *grid;
    const Mesh *mesh;
    Matrix44f cam;
    float fov;
    uint width, height, spp;
    int isect = 0;                  // 0 Grid::Intersect, 1 IntersectBruteForce, 2 RayMarch
};

// renderer.cpp:157-197 (loop glue; IntersectRayTri is the reference's, triangle.h:15-107)
bool IntersectBruteForceRef(const Mesh *mesh, Vec3f origin, Vec3f dir, float& t, float& u, float& v,
                            uint32& tri_idx)
{
    t = std::numeric_limits<float>::max();
    const uint32 n = uint32(mesh->m_triangles.size());
    for (uint32 i=0; i<n; i++)
    {
        const Mesh::Triangle& tri = mesh->m_triangles[i];
        float ct, cu, cv;
        const bool hit = IntersectRayTri(origin, dir, mesh->m_vertices[tri.v0].p, mesh->m_vertices[tri.v1].p,
                                         mesh->m_vertices[tri.v2].p, ct, cu, cv);
        if (hit && ct < t) { t = ct; u = cu; v = cv; tri_idx = i; }
    }
    return t != std::numeric_limits<float>::max();
}

// renderer.cpp:138-155 (loop glue; DistancePointTri is the reference's, triangle.h:174-198)
float DistanceBruteForceRef(const Mesh *mesh, Vec3f pos)
{
    float dist = std::numeric_limits<float>::max();
    for (const auto& tri : mesh->m_triangles)
        dist = std::min(dist, DistancePointTri(pos, mesh->m_vertices[tri.v0].p, mesh->m_vertices[tri.v1].p,
                                               mesh->m_vertices[tri.v2].p));
    return dist;
}

// renderer.cpp:24-41; steps_out counts the march steps taken (instrumentation only)
bool RayMarchRef(const Mesh *mesh, Vec3f origin, Vec3f dir, float& t, uint& steps_out)
{
    const uint max_steps = 128;
    const float min_dist = 0.001f;
    t = 0.0f;
    for (uint steps=0; steps<max_steps; steps++)
    {
        const Vec3f pos = origin + t * dir;
        const float dist = DistanceBruteForceRef(mesh, pos);
        t += dist;
        steps_out = steps + 1;
        if (dist < min_dist) return true;
    }
    return false;
}

std::vector<Vec2f> SampleTable(uint spp)
{
    // renderer.cpp:49-60
    std::vector<Vec2f> smp_loc(spp);
    for (uint smp=0; smp<spp; smp++)
    {
        smp_loc[smp].x = SAMP::HammersleySequence<SAMP::ScrambleNone>(smp, 0, spp) - 0.5f;
        smp_loc[smp].y = SAMP::HammersleySequence<SAMP::ScrambleNone>(smp, 1, spp) - 0.5f;
    }
    return smp_loc;
}

// u32 hit, tri | f32 t, u, v, r, g, b [| u32 voxel, steps, tests in the instrumented build]
struct SampleRec
{
    uint32 hit, tri;
    float t, u, v, r, g, b;
#ifdef RT_REF_INSTR
    uint32 voxel, steps, tests;
#endif
};

// One tile, exactly the reference's arithmetic order; optionally records per-sample hits.
void RenderTileRef(const Frame& fr, uint x0, uint y0, uint x1, uint y1, uint32 *buf,
                   uint32 *hit_ids /* full frame, (y*W + x)*spp + s, may be null */)
{
    const std::vector<Vec2f> smp_loc = SampleTable(fr.spp);
    const uint tw = x1 - x0, th = y1 - y0;
    for (uint y=0; y<th; y++)
    {
        for (uint x=0; x<tw; x++)
        {
            Vec2ui pixel(x0 + x, y0 + y);
            Vec3f col(0.0f);
            for (uint smp=0; smp<fr.spp; smp++)
            {
                Vec3f origin, dir;
                GenerateRay(fr.cam, pixel, fr.width, fr.height, smp_loc[smp], false, fr.fov, origin, dir);
                float t, u, v;
                uint32 tri_idx;
                uint steps = 0;
                bool hit;
                if (fr.isect == 2) hit = RayMarchRef(fr.mesh, origin, dir, t, steps);
                else if (fr.isect == 1) hit = IntersectBruteForceRef(fr.mesh, origin, dir, t, u, v, tri_idx);
                else hit = fr.grid->Intersect(origin, dir, t, u, v, tri_idx);
                if (hit && fr.isect == 2)
                {
                    col += Vec3f(t / 3);                              // renderer.cpp:118
                    tri_idx = 0xFFFFFFFFu;
                }
                else if (hit)
                {
                    const Mesh::Triangle& tri = fr.mesh->m_triangles[tri_idx];
                    const Vec3f n = Normalize(BarycentricInterpolate(
                        u, v,
                        fr.mesh->m_vertices[tri.v0].n,
                        fr.mesh->m_vertices[tri.v1].n,
                        fr.mesh->m_vertices[tri.v2].n));
                    col += Vec3f((n + 1.0f) * 0.5f);
                }
                else
                    col += Vec3f(float(pixel.y) / float(fr.height));
                if (hit_ids)
                    hit_ids[(size_t(pixel.y) * fr.width + pixel.x) * fr.spp + smp] = hit ? tri_idx : 0xFFFFFFFFu;
            }
            Vec3f final_col = col / float(fr.spp);
            const float gamma = 1.0f / 2.0f;
            final_col.x = std::pow(final_col.x, gamma);
            final_col.y = std::pow(final_col.y, gamma);
            final_col.z = std::pow(final_col.z, gamma);
            buf[x + y * tw] = ToBGRA8(final_col);
        }
    }
}

// -------------------------------------------------- tile pool (framebuffer.cpp restated)
struct TilePool
{
    static const uint tiles_x = 12, tiles_y = 9;               // framebuffer.h:87-88
    struct T { uint x0, y0, x1, y1; std::vector<uint32> bgra; };
    std::array<T, tiles_x * tiles_y> tiles;
    uint width = 0, height = 0;

    void Resize(uint w, uint h)                                  // framebuffer.cpp:94-122
    {
        width = w; height = h;
        const uint tw = w / tiles_x, th = h / tiles_y;
        for (uint y=0; y<tiles_y; y++)
            for (uint x=0; x<tiles_x; x++)
            {
                T& t = tiles[x + y * tiles_x];
                t.x0 = x * tw; t.y0 = y * th;
                t.x1 = (x == tiles_x - 1) ? w : (x + 1) * tw;
                t.y1 = (y == tiles_y - 1) ? h : (y + 1) * th;
                t.bgra.assign(size_t(t.x1 - t.x0) * (t.y1 - t.y0), 0);
            }
    }

    // Returns seconds from pool start to the last tile finishing (framebuffer.cpp:21, 81-88)
    double Render(const Frame& fr, uint nthreads, uint32 *hit_ids)
    {
        std::vector<uint> queue;
        for (uint i=0; i<tiles_x * tiles_y; i++) queue.push_back(i);
        std::random_shuffle(queue.begin(), queue.end());       // framebuffer.cpp:146
        std::mutex qmtx;
        const double t0 = TimerGetTick();
        std::vector<std::thread> threads;
        for (uint i=0; i<nthreads; i++)
            threads.push_back(std::thread([&]() {
                while (true)
                {
                    uint idx;
                    {
                        std::lock_guard<std::mutex> g(qmtx);
                        if (queue.empty()) break;
                        idx = queue.back();
                        queue.pop_back();
                    }
                    T& t = tiles[idx];
                    RenderTileRef(fr, t.x0, t.y0, t.x1, t.y1, &t.bgra[0], hit_ids);
                }
            }));
        for (auto& th : threads) th.join();
        return TimerGetTick() - t0;
    }

    void Gather(std::vector<uint32>& img) const                 // framebuffer.cpp:197-216
    {
        img.assign(size_t(width) * height, 0);
        for (const auto& t : tiles)
            for (uint y=0; y<t.y1 - t.y0; y++)
                for (uint x=0; x<t.x1 - t.x0; x++)
                    img[size_t(t.y0 + y) * width + t.x0 + x] = t.bgra[x + y * (t.x1 - t.x0)];
    }
};

bool WriteFile(const char *path, const void *data, size_t bytes)
{
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(data, 1, bytes, f) == bytes;
    std::fclose(f);
    return ok;
}

int Usage()
{
    std::fprintf(stderr, "usage: refdriver dump-scenes|grid|render|samples|kat ...\n");
    return 2;
}

// ----------------------------------------------------------------------------- KATs
float RandF(std::mt19937& g, float lo, float hi)
{
    return std::uniform_real_distribution<float>(lo, hi)(g);
}

Vec3f RandV(std::mt19937& g, float lo, float hi)
{
    return Vec3f(RandF(g, lo, hi), RandF(g, lo, hi), RandF(g, lo, hi));
}

// DistancePointTri (triangle.h:174-198) known answers: in pos, v0, v1, v2 (12 f32), out dist
int CmdKatDist(const char *path)
{
    std::mt19937 g(20261016u);
    std::vector<float> rec;
    const int N = 6000;
    for (int i=0; i<N; i++)
    {
        Vec3f v0 = RandV(g, -1, 1), v1 = RandV(g, -1, 1), v2 = RandV(g, -1, 1), pos = RandV(g, -2, 2);
        const int kind = i % 8;
        if (kind == 1)          // on the plane, inside or just outside (barycentric edge cases)
        {
            const float a = RandF(g, -0.1f, 1.1f), b = RandF(g, -0.1f, 1.1f);
            pos = v0 + (v1 - v0) * a + (v2 - v0) * b;
        }
        else if (kind == 2)     // at a vertex or an edge midpoint
            pos = (i & 8) ? v2 : (v1 + v2) * 0.5f;
        else if (kind == 3)     // repeated vertex (zero area -> inf/NaN barycentrics)
            v2 = v0;
        else if (kind == 4)     // collinear
            v2 = v0 + (v1 - v0) * RandF(g, -1.0f, 2.0f);
        else if (kind == 5)     // all three vertices equal (zero-length edges -> 0/0 clamps)
            v1 = v2 = v0;
        else if (kind == 6)     // tiny triangle far away
        {
            v1 = v0 + RandV(g, -1e-4f, 1e-4f);
            v2 = v0 + RandV(g, -1e-4f, 1e-4f);
            pos = pos * 50.0f;
        }
        const float d = DistancePointTri(pos, v0, v1, v2);
        const Vec3f in[4] = { pos, v0, v1, v2 };
        for (const auto& x : in) { rec.push_back(x.x); rec.push_back(x.y); rec.push_back(x.z); }
        rec.push_back(d);
    }
    if (!WriteFile(path, &rec[0], rec.size() * 4)) return 1;
    std::printf("RESULT {\"kat_dist\": %d}\n", N);
    return 0;
}

int CmdKat(const char *outdir)
{
    std::mt19937 g(20261015u);
    const std::string dir(outdir);
    const float nan = std::numeric_limits<float>::quiet_NaN();

    // ---- IntersectRayTri / IntersectRayTriBarycentric: in 18 floats, out hit,t,u,v (x2)
    {
        std::vector<float> rec;
        const int N = 6000;
        for (int i=0; i<N; i++)
        {
            Vec3f v0 = RandV(g, -1, 1), v1 = RandV(g, -1, 1), v2 = RandV(g, -1, 1);
            Vec3f o = RandV(g, -2, 2), d;
            const int kind = i % 8;
            if (kind == 0)       // aim at a vertex exactly
                d = Normalize((i & 8 ? v1 : v0) - o);
            else if (kind == 1)  // aim at an edge midpoint
                d = Normalize((v0 + v1) * 0.5f - o);
            else if (kind == 2)  // axis aligned with signed zeros
            {
                const int ax = (i / 8) % 3;
                d = Vec3f((i & 16) ? -0.0f : 0.0f, (i & 32) ? -0.0f : 0.0f, (i & 64) ? -0.0f : 0.0f);
                d[ax] = (i & 128) ? -1.0f : 1.0f;
            }
            else if (kind == 3)  // (near) parallel to the triangle plane -> det ~ 0
            {
                d = Normalize(v1 - v0 + (v2 - v0) * RandF(g, 0.0f, 1e-6f));
            }
            else if (kind == 4)  // tiny triangle, det around +-1e-8
            {
                v1 = v0 + RandV(g, -2e-4f, 2e-4f);
                v2 = v0 + RandV(g, -2e-4f, 2e-4f);
                d = Normalize((v0 + v1 + v2) * (1.0f / 3.0f) - o);
            }
            else                 // aimed roughly at the triangle
            {
                const float a = RandF(g, -0.2f, 1.2f), b = RandF(g, -0.2f, 1.2f);
                d = Normalize(v0 + (v1 - v0) * a + (v2 - v0) * b * (1.0f - a) - o);
            }
            const Vec3f n = TriangleNormal(v0, v1, v2);
            float t = nan, u = nan, v = nan;
            const bool hit = IntersectRayTri(o, d, v0, v1, v2, t, u, v);
            float bt = nan, bu = nan, bv = nan;
            const bool bhit = IntersectRayTriBarycentric(o, d, v0, v1, v2, n, bt, bu, bv);
            const Vec3f in[6] = { o, d, v0, v1, v2, n };
            for (const auto& x : in) { rec.push_back(x.x); rec.push_back(x.y); rec.push_back(x.z); }
            uint32 h = hit, bh = bhit;
            float fh, fbh;
            std::memcpy(&fh, &h, 4);
            std::memcpy(&fbh, &bh, 4);
            rec.push_back(fh); rec.push_back(t); rec.push_back(u); rec.push_back(v);
            rec.push_back(fbh); rec.push_back(bt); rec.push_back(bu); rec.push_back(bv);
        }
        WriteFile((dir + "/kat_ray_tri.f32").c_str(), &rec[0], rec.size() * 4);
    }

    // ---- IntersectRayAABB + IntersectPointAABB: in o,d,bmin,bmax (12), out hit,tmin,tmax,inside
    {
        std::vector<float> rec;
        const int N = 6000;
        for (int i=0; i<N; i++)
        {
            Vec3f a = RandV(g, -1, 1), b = RandV(g, -1, 1);
            Vec3f bmin = ComponentMin(a, b), bmax = ComponentMax(a, b);
            Vec3f o = RandV(g, -3, 3), d = Normalize(RandV(g, -1, 1));
            const int kind = i % 6;
            if (kind == 1)       // origin on a slab face
            {
                const int ax = (i / 6) % 3;
                o[ax] = (i & 64) ? bmin[ax] : bmax[ax];
            }
            else if (kind == 2)  // signed zero direction components
            {
                const int ax = (i / 6) % 3;
                d[ax] = (i & 128) ? -0.0f : 0.0f;
            }
            else if (kind == 3)  // zero component AND origin on that slab (0 * inf = NaN)
            {
                const int ax = (i / 6) % 3;
                d[ax] = (i & 128) ? -0.0f : 0.0f;
                o[ax] = (i & 64) ? bmin[ax] : bmax[ax];
            }
            else if (kind == 4)  // box entirely behind the origin
            {
                d = Normalize(o - (bmin + bmax) * 0.5f);
            }
            float tmin = nan, tmax = nan;
            const bool hit = IntersectRayAABB(o, d, bmin, bmax, tmin, tmax);
            const bool inside = IntersectPointAABB(o, bmin, bmax);
            const Vec3f in[4] = { o, d, bmin, bmax };
            for (const auto& x : in) { rec.push_back(x.x); rec.push_back(x.y); rec.push_back(x.z); }
            uint32 h = hit, ins = inside;
            float fh, fi;
            std::memcpy(&fh, &h, 4);
            std::memcpy(&fi, &ins, 4);
            rec.push_back(fh); rec.push_back(tmin); rec.push_back(tmax); rec.push_back(fi);
        }
        WriteFile((dir + "/kat_ray_aabb.f32").c_str(), &rec[0], rec.size() * 4);
    }

    // ---- GenerateRay (perspective): in cam[16], px, py (u32 bits), W, H (u32 bits), sx, sy, fov
    //      out origin[3], dir[3]
    {
        std::vector<float> rec;
        const int N = 2000;
        for (int i=0; i<N; i++)
        {
            Matrix44f cam;
            cam.BuildLookAtMatrix(RandV(g, -3, 3), RandV(g, -0.5f, 0.5f));
            const uint W = 1 + (g() % 4096), H = 1 + (g() % 4096);
            const uint px = g() % W, py = g() % H;
            const Vec2f so(RandF(g, -0.5f, 0.5f), RandF(g, -0.5f, 0.5f));
            const float fov = RandF(g, 10.0f, 120.0f);
            Vec3f o, d;
            GenerateRay(cam, Vec2ui(px, py), W, H, so, false, fov, o, d);
            for (int k=0; k<16; k++) rec.push_back((&cam.m_mat[0][0])[k]);
            const uint32 ints[4] = { px, py, W, H };
            for (int k=0; k<4; k++) { float f; std::memcpy(&f, &ints[k], 4); rec.push_back(f); }
            rec.push_back(so.x); rec.push_back(so.y); rec.push_back(fov);
            rec.push_back(o.x); rec.push_back(o.y); rec.push_back(o.z);
            rec.push_back(d.x); rec.push_back(d.y); rec.push_back(d.z);
        }
        WriteFile((dir + "/kat_genray.f32").c_str(), &rec[0], rec.size() * 4);
    }

    // ---- ToBGRA8 + gamma: in col[3] (pre-gamma average), out gamma'd rgb[3], packed u32
    {
        std::vector<float> rec;
        const int N = 8000;
        for (int i=0; i<N; i++)
        {
            Vec3f c = RandV(g, -0.01f, 1.01f);
            if (i % 5 == 0) c = Vec3f(float(g() % 256) / 255.0f);
            if (i % 7 == 0) c.x = (i & 8) ? -0.0f : 0.0f;
            Vec3f fc = c;
            const float gamma = 1.0f / 2.0f;
            fc.x = std::pow(fc.x, gamma);
            fc.y = std::pow(fc.y, gamma);
            fc.z = std::pow(fc.z, gamma);
            const uint32 p = ToBGRA8(fc);
            float fp;
            std::memcpy(&fp, &p, 4);
            rec.push_back(c.x); rec.push_back(c.y); rec.push_back(c.z);
            rec.push_back(fc.x); rec.push_back(fc.y); rec.push_back(fc.z); rec.push_back(fp);
        }
        WriteFile((dir + "/kat_bgra8.f32").c_str(), &rec[0], rec.size() * 4);
    }

    // ---- Hammersley sample tables (renderer.cpp:49-60) for spp 1..64 and 128, 256
    {
        std::vector<float> rec;
        std::vector<uint> spps;
        for (uint s=1; s<=64; s++) spps.push_back(s);
        spps.push_back(128); spps.push_back(256);
        for (uint spp : spps)
        {
            const std::vector<Vec2f> t = SampleTable(spp);
            for (const auto& p : t) { rec.push_back(p.x); rec.push_back(p.y); }
        }
        WriteFile((dir + "/kat_hammersley.f32").c_str(), &rec[0], rec.size() * 4);
    }

    // ---- shading: BarycentricInterpolate + Normalize + (n+1)*0.5 ; in u,v,n0,n1,n2 out col
    {
        std::vector<float> rec;
        const int N = 5000;
        for (int i=0; i<N; i++)
        {
            const float u = RandF(g, 0, 1), v = RandF(g, 0, 1 - u);
            const Vec3f n0 = Normalize(RandV(g, -1, 1)), n1 = Normalize(RandV(g, -1, 1)),
                        n2 = Normalize(RandV(g, -1, 1));
            const Vec3f n = Normalize(BarycentricInterpolate(u, v, n0, n1, n2));
            const Vec3f c = Vec3f((n + 1.0f) * 0.5f);
            rec.push_back(u); rec.push_back(v);
            const Vec3f in[3] = { n0, n1, n2 };
            for (const auto& x : in) { rec.push_back(x.x); rec.push_back(x.y); rec.push_back(x.z); }
            rec.push_back(c.x); rec.push_back(c.y); rec.push_back(c.z);
        }
        WriteFile((dir + "/kat_shade.f32").c_str(), &rec[0], rec.size() * 4);
    }
    std::printf("RESULT {\"kat\": \"ok\"}\n");
    return 0;
}

} // namespace

int main(int argc, char **argv)
{
    if (argc < 2) return Usage();
    const std::string cmd = argv[1];

    if (cmd == "dump-scenes" && argc == 4)
    {
        for (uint id=0; id<10; id++)
        {
            Mesh mesh;
            Matrix44f cam;
            float fov;
            if (!BuildScene(id, argv[2], mesh, cam, fov))
            {
                std::fprintf(stderr, "scene %u failed\n", id);
                return 1;
            }
            const std::string path = std::string(argv[3]) + "/scene" + std::to_string(id) + ".rtscene";
            if (!WriteScene(path.c_str(), id, fov, cam, mesh)) return 1;
        }
        std::printf("RESULT {\"dump\": \"ok\"}\n");
        return 0;
    }

    if (cmd == "mesh-read" && argc == 5)
    {
        // Mesh::Read(path, flip) [+ NormalizeDimensions when argv[3] has bit 1] -> raw dump:
        // u32 ok | u32 nv | u32 nt | nv x Vertex | nt x Triangle (mesh.h layouts)
        const int mode = std::atoi(argv[3]);
        Mesh m;
        uint32 ok = m.Read(argv[2], (mode & 1) != 0) ? 1u : 0u;
        if (ok && (mode & 2)) m.NormalizeDimensions();
        const uint32 nv = uint32(m.m_vertices.size()), nt = uint32(m.m_triangles.size());
        std::FILE *f = std::fopen(argv[4], "wb");
        if (!f) return 1;
        std::fwrite(&ok, 4, 1, f);
        std::fwrite(&nv, 4, 1, f);
        std::fwrite(&nt, 4, 1, f);
        if (nv) std::fwrite(&m.m_vertices[0], sizeof(Mesh::Vertex), nv, f);
        if (nt) std::fwrite(&m.m_triangles[0], sizeof(Mesh::Triangle), nt, f);
        std::fclose(f);
        return 0;
    }

    if (cmd == "cornell-quads" && argc == 3)
    {
        // the reference's Cornell box geometry table (cornell_box.cpp), one vertex per line
        // with 9 significant digits (round-trips every float): data for the host scene table
        std::FILE *f = std::fopen(argv[2], "w");
        if (!f) return 1;
        std::fprintf(f, "%u\n", g_cornell_num_quads);
        for (uint i = 0; i < g_cornell_num_quads * 4; i++)
            std::fprintf(f, "%.9g %.9g %.9g\n", g_cornell_quads[i][0], g_cornell_quads[i][1], g_cornell_quads[i][2]);
        std::fclose(f);
        return 0;
    }

    if (cmd == "look-at" && argc == 9)
    {
        // Matrix44f::BuildLookAtMatrix (lin_alg.h:431-467), the reference's own, with the default up
        // vector: eye (3 floats) and target (3 floats) read as %a / decimal, 16 floats written raw
        Matrix44f m;
        m.BuildLookAtMatrix(Vec3f(std::strtof(argv[2], nullptr), std::strtof(argv[3], nullptr), std::strtof(argv[4], nullptr)),
                            Vec3f(std::strtof(argv[5], nullptr), std::strtof(argv[6], nullptr), std::strtof(argv[7], nullptr)));
        return WriteFile(argv[8], &m.m_mat[0][0], 16 * sizeof(float)) ? 0 : 1;
    }

    if (cmd == "kat" && argc == 3)
        return CmdKat(argv[2]);
    if (cmd == "kat-dist" && argc == 3)
        return CmdKatDist(argv[2]);

    if ((cmd == "grid" && argc == 4) || (cmd == "render" && argc >= 6) || (cmd == "samples" && argc >= 11) ||
        (cmd == "alt-samples" && argc == 12))
    {
        SceneFile sf;
        if (!ReadScene(argv[2], sf)) { std::fprintf(stderr, "bad scene file\n"); return 1; }
        const Mesh *mesh_ptr = sf.mesh.get();
        const double tb0 = TimerGetTick();
        GridExport grid(std::move(sf.mesh), 64);                  // scene.cpp:6-7
        const double build_s = TimerGetTick() - tb0;

        if (cmd == "grid")
        {
            std::FILE *f = std::fopen(argv[3], "wb");
            if (!f) return 1;
            grid.Export(f);
            std::fclose(f);
            std::printf("RESULT {\"grid_build_s\": %.6f}\n", build_s);
            return 0;
        }

        Frame fr;
        fr.grid = &grid;
        fr.mesh = mesh_ptr;
        fr.cam = sf.cam;
        fr.fov = sf.fov;
        fr.width = uint(std::atoi(argv[3]));
        fr.height = uint(std::atoi(argv[4]));
        fr.spp = std::max(1u, uint(std::atoi(argv[5])));   // Renderer::SetSampleCount
        // --view <file>: another camera (f32 Matrix44f m_mat[16] + f32 fov, raw) in place of the scene's
        // (Scene::GetCameraParameters, scene.h:17-19): any view through the same GenerateRay and walk
        for (int i = (cmd == "samples" ? 11 : 6); i + 1 < argc; i++)
            if (std::string(argv[i]) == "--view")
            {
                std::FILE *vf = std::fopen(argv[i + 1], "rb");
                const bool vok = vf && std::fread(&fr.cam.m_mat[0][0], 4, 16, vf) == 16 && std::fread(&fr.fov, 4, 1, vf) == 1;
                if (vf) std::fclose(vf);
                if (!vok) { std::fprintf(stderr, "bad view file\n"); return 1; }
            }

        if (cmd == "samples")
        {
            const uint x0 = std::atoi(argv[6]), y0 = std::atoi(argv[7]);
            const uint w = std::atoi(argv[8]), h = std::atoi(argv[9]);
            const std::vector<Vec2f> smp_loc = SampleTable(fr.spp);
            std::vector<SampleRec> recs;
            for (uint y=y0; y<y0 + h; y++)
                for (uint x=x0; x<x0 + w; x++)
                    for (uint s=0; s<fr.spp; s++)
                    {
                        Vec3f origin, dir;
                        GenerateRay(fr.cam, Vec2ui(x, y), fr.width, fr.height, smp_loc[s], false, fr.fov, origin, dir);
                        SampleRec r;
                        float t = 0, u = 0, v = 0;
                        uint32 tri = 0xFFFFFFFFu;
#ifdef RT_REF_INSTR
                        g_rt_ref_walk = RtRefWalk{0xFFFFFFFFu, 0u, 0u};
#endif
                        const bool hit = grid.Intersect(origin, dir, t, u, v, tri);
                        Vec3f c;
                        if (hit)
                        {
                            const Mesh::Triangle& tr = mesh_ptr->m_triangles[tri];
                            const Vec3f n = Normalize(BarycentricInterpolate(u, v,
                                mesh_ptr->m_vertices[tr.v0].n, mesh_ptr->m_vertices[tr.v1].n,
                                mesh_ptr->m_vertices[tr.v2].n));
                            c = Vec3f((n + 1.0f) * 0.5f);
                        }
                        else
                        {
                            c = Vec3f(float(y) / float(fr.height));
                            t = u = v = 0.0f;
                            tri = 0xFFFFFFFFu;
                        }
                        r.hit = hit; r.tri = tri; r.t = t; r.u = u; r.v = v;
                        r.r = c.x; r.g = c.y; r.b = c.z;
#ifdef RT_REF_INSTR
                        r.voxel = g_rt_ref_walk.cell; r.steps = g_rt_ref_walk.steps;
                        r.tests = g_rt_ref_walk.tests;
#endif
                        recs.push_back(r);
                    }
            if (!WriteFile(argv[10], &recs[0], recs.size() * sizeof(SampleRec))) return 1;
            std::printf("RESULT {\"samples\": %zu}\n", recs.size());
            return 0;
        }

        if (cmd == "alt-samples")
        {
            // u32 hit, tri, steps | f32 t, u, v, r, g, b   (t, u, v = 0 and tri = ~0 on a miss)
            struct AltRec { uint32 hit, tri, steps; float t, u, v, r, g, b; };
            const uint x0 = std::atoi(argv[6]), y0 = std::atoi(argv[7]);
            const uint w = std::atoi(argv[8]), h = std::atoi(argv[9]);
            const std::string mode = argv[10];
            if (mode != "brute" && mode != "march") return Usage();
            const std::vector<Vec2f> smp_loc = SampleTable(fr.spp);
            std::vector<AltRec> recs;
            for (uint y=y0; y<y0 + h; y++)
                for (uint x=x0; x<x0 + w; x++)
                    for (uint s=0; s<fr.spp; s++)
                    {
                        Vec3f origin, dir;
                        GenerateRay(fr.cam, Vec2ui(x, y), fr.width, fr.height, smp_loc[s], false, fr.fov, origin, dir);
                        AltRec r;
                        float t = 0, u = 0, v = 0;
                        uint32 tri = 0xFFFFFFFFu;
                        uint steps = 0;
                        Vec3f c;
                        bool hit;
                        if (mode == "march")
                        {
                            hit = RayMarchRef(mesh_ptr, origin, dir, t, steps);
                            if (hit) c = Vec3f(t / 3);
                        }
                        else
                        {
                            hit = IntersectBruteForceRef(mesh_ptr, origin, dir, t, u, v, tri);
                            if (hit)
                            {
                                const Mesh::Triangle& tr = mesh_ptr->m_triangles[tri];
                                const Vec3f n = Normalize(BarycentricInterpolate(u, v,
                                    mesh_ptr->m_vertices[tr.v0].n, mesh_ptr->m_vertices[tr.v1].n,
                                    mesh_ptr->m_vertices[tr.v2].n));
                                c = Vec3f((n + 1.0f) * 0.5f);
                            }
                        }
                        if (!hit)
                        {
                            c = Vec3f(float(y) / float(fr.height));
                            t = u = v = 0.0f;
                            tri = 0xFFFFFFFFu;
                        }
                        r.hit = hit; r.tri = tri; r.steps = steps; r.t = t; r.u = u; r.v = v;
                        r.r = c.x; r.g = c.y; r.b = c.z;
                        recs.push_back(r);
                    }
            if (!WriteFile(argv[11], &recs[0], recs.size() * sizeof(AltRec))) return 1;
            std::printf("RESULT {\"samples\": %zu}\n", recs.size());
            return 0;
        }

        // render
        uint nthreads = std::max(1u, std::thread::hardware_concurrency());   // framebuffer.cpp:11
        uint reps = 1;
        const char *out = nullptr, *hits = nullptr, *bmp = nullptr;
        for (int i=6; i<argc; i++)
        {
            const std::string a = argv[i];
            if (a == "--threads" && i + 1 < argc) nthreads = std::atoi(argv[++i]);
            else if (a == "--reps" && i + 1 < argc) reps = std::atoi(argv[++i]);
            else if (a == "--out" && i + 1 < argc) out = argv[++i];
            else if (a == "--hits" && i + 1 < argc) hits = argv[++i];
            else if (a == "--bmp" && i + 1 < argc) bmp = argv[++i];
            else if (a == "--isect" && i + 1 < argc)
            {
                const std::string m = argv[++i];
                fr.isect = m == "brute" ? 1 : (m == "march" ? 2 : 0);
            }
        }
        TilePool pool;
        pool.Resize(fr.width, fr.height);
        std::vector<uint32> hit_ids;
        if (hits) hit_ids.assign(size_t(fr.width) * fr.height * fr.spp, 0xFFFFFFFEu);
        std::vector<double> times;
        for (uint r=0; r<reps; r++)
            times.push_back(pool.Render(fr, nthreads, hits ? &hit_ids[0] : nullptr));
        std::vector<double> sorted = times;
        std::sort(sorted.begin(), sorted.end());
        const double med = sorted[sorted.size() / 2];
        std::vector<uint32> img;
        pool.Gather(img);
        if (out && !WriteFile(out, &img[0], img.size() * 4)) return 1;
        if (hits && !WriteFile(hits, &hit_ids[0], hit_ids.size() * 4)) return 1;
        if (bmp) WriteBitmap(bmp, fr.width, fr.height, &img[0]);   // bmp_writer.cpp:27-57 (SaveToBMP's call)
        std::printf("RESULT {\"threads\": %u, \"reps\": %u, \"median_s\": %.6f, \"first_s\": %.6f, "
                    "\"samples\": %llu, \"msamples_per_s\": %.3f, \"grid_build_s\": %.6f}\n",
                    nthreads, reps, med, times[0],
                    (unsigned long long)fr.width * fr.height * fr.spp,
                    double(fr.width) * fr.height * fr.spp / med / 1e6, build_s);
        return 0;
    }
    return Usage();
}
