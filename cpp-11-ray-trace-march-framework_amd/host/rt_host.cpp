// rt_host.cpp -- C++11 host side above the GPU boundary (include/rt_host.h).
//
//  * Scene loading (.rtscene) and the uniform-grid build of Grid::Grid (grid.cpp:12-154),
//    emitted directly as CSR in GridIdx order.  The build is bit-identical to the
//    reference (tests/test_host_grid.py checks every scene's CSR hash against the fixture
//    produced by the reference's own Grid::Grid); it runs the per-triangle tri/box tests in
//    parallel and keeps each cell's list in ascending triangle order with a stable
//    counting sort, which is what the reference's sequential push_back order produces.
//  * A headless Framebuffer (framebuffer.h / framebuffer.cpp) whose RenderTile override is
//    served by librt_tracer: one batched GPU launch per frame, then each worker thread
//    copies its own tile under its tile mutex.
//
// Built with -ffp-contract=off and no -march (reference Makefile:9-11): the float
// arithmetic of the grid build must round exactly as the reference's does.

#include "../../include/rt_host.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& m)
{
    g_err = m;
    return code;
}

// ------------------------------------------------------------------ tri/box overlap
// Akenine-Moller separating-axis test in double (aabb_tri_internal.h:112-186), as called
// by IntersectTriAABB (aabb.h:15-32).  The nine edge-axis tests are table driven here:
// for edge e and world axis a the test projects onto e x a, i.e. uses components (b, c) =
// the other two axes, with p = e[c]*v[b] - e[b]*v[c] (sign conventions of the X/Y/Z macros).
struct AxisTest { int e; int b; int c; int va; int vb; bool p2_first; bool neg; };

inline int plane_box(const double n[3], double d, const double h[3])
{
    double vmin[3], vmax[3];
    for (int q = 0; q < 3; q++)
    {
        if (n[q] > 0.0f) { vmin[q] = -h[q]; vmax[q] = h[q]; }
        else             { vmin[q] = h[q];  vmax[q] = -h[q]; }
    }
    if (n[0] * vmin[0] + n[1] * vmin[1] + n[2] * vmin[2] + d > 0.0f) return 0;
    if (n[0] * vmax[0] + n[1] * vmax[1] + n[2] * vmax[2] + d >= 0.0f) return 1;
    return 0;
}

bool tri_box(const double ctr[3], const double h[3], const float* p0, const float* p1, const float* p2)
{
    double v[3][3], e[3][3];
    for (int i = 0; i < 3; i++)
    {
        v[0][i] = double(p0[i]) - ctr[i];
        v[1][i] = double(p1[i]) - ctr[i];
        v[2][i] = double(p2[i]) - ctr[i];
    }
    for (int i = 0; i < 3; i++)
    {
        e[0][i] = v[1][i] - v[0][i];
        e[1][i] = v[2][i] - v[1][i];
        e[2][i] = v[0][i] - v[2][i];
    }
    // Which two vertices each macro projects (aabb_tri_internal.h:142-158):
    //   edge0: X01(v0,v2) Y02(v0,v2) Z12(v1,v2)   edge1: X01(v0,v2) Y02(v0,v2) Z0(v0,v1)
    //   edge2: X2(v0,v1)  Y1(v0,v1)  Z12(v1,v2)
    static const int verts[3][3][2] = { { { 0, 2 }, { 0, 2 }, { 1, 2 } },
                                        { { 0, 2 }, { 0, 2 }, { 0, 1 } },
                                        { { 0, 1 }, { 0, 1 }, { 1, 2 } } };
    for (int ei = 0; ei < 3; ei++)
    {
        const double* E = e[ei];
        const double fa[3] = { std::fabs(E[0]), std::fabs(E[1]), std::fabs(E[2]) };
        for (int ax = 0; ax < 3; ax++)
        {
            const int a = verts[ei][ax][0], b = verts[ei][ax][1];
            double pa, pb, rad;
            if (ax == 0)      // X tests: p = E.z*v.y - E.y*v.z ; rad = |E.z|*h.y + |E.y|*h.z
            {
                pa = E[2] * v[a][1] - E[1] * v[a][2];
                pb = E[2] * v[b][1] - E[1] * v[b][2];
                rad = fa[2] * h[1] + fa[1] * h[2];
            }
            else if (ax == 1) // Y tests: p = -E.z*v.x + E.x*v.z ; rad = |E.z|*h.x + |E.x|*h.z
            {
                pa = -E[2] * v[a][0] + E[0] * v[a][2];
                pb = -E[2] * v[b][0] + E[0] * v[b][2];
                rad = fa[2] * h[0] + fa[0] * h[2];
            }
            else              // Z tests: p = E.y*v.x - E.x*v.y ; rad = |E.y|*h.x + |E.x|*h.y
            {
                pa = E[1] * v[a][0] - E[0] * v[a][1];
                pb = E[1] * v[b][0] - E[0] * v[b][1];
                rad = fa[1] * h[0] + fa[0] * h[1];
            }
            // Z12 orders with '(p2 < p1)', the others with '(pa < pb)'; min/max coincide
            // except for NaN, where the chosen branch decides -- keep each macro's form.
            double mn, mx;
            const bool z12 = (ax == 2) && !(ei == 1);
            if (z12) { if (pb < pa) { mn = pb; mx = pa; } else { mn = pa; mx = pb; } }
            else     { if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; } }
            if (mn > rad || mx < -rad) return false;
        }
    }
    for (int a = 0; a < 3; a++)      // FINDMINMAX per axis
    {
        double mn = v[0][a], mx = v[0][a];
        if (v[1][a] < mn) mn = v[1][a];
        if (v[1][a] > mx) mx = v[1][a];
        if (v[2][a] < mn) mn = v[2][a];
        if (v[2][a] > mx) mx = v[2][a];
        if (mn > h[a] || mx < -h[a]) return false;
    }
    double n[3];
    n[0] = e[0][1] * e[1][2] - e[0][2] * e[1][1];
    n[1] = e[0][2] * e[1][0] - e[0][0] * e[1][2];
    n[2] = e[0][0] * e[1][1] - e[0][1] * e[1][0];
    const double d = -(n[0] * v[0][0] + n[1] * v[0][1] + n[2] * v[0][2]);
    return plane_box(n, d, h) == 1;
}

} // namespace

struct rth_scene
{
    uint32_t id = 0xFFFFFFFFu;
    float fov = 45.0f;
    float cam[16];
    std::vector<rt_vertex> verts;
    std::vector<rt_triangle> tris;
    uint32_t dims[3] = { 0, 0, 0 };
    float bmin[3], bmax[3], cw = 0, icw = 0;
    std::vector<uint32_t> off, refs;
    double build_s = 0.0;
};

namespace {

// grid.cpp:12-129 Grid::Grid -> CSR
int build_grid(rth_scene& s, uint32_t res, uint32_t nthreads)
{
    if (s.tris.empty() || s.verts.empty()) return fail(RT_E_INVALID, "empty mesh (grid.cpp:15)");
    if (res == 0) return fail(RT_E_INVALID, "grid_res must be > 0 (grid.cpp:16)");
    const auto t0 = std::chrono::steady_clock::now();
    const float fmax = std::numeric_limits<float>::max(), fmin = std::numeric_limits<float>::min();
    // mesh.cpp:112-134 ComputeAABB (max seeded with float::min(), hazard H11)
    float mn[3] = { fmax, fmax, fmax }, mx[3] = { fmin, fmin, fmin };
    for (const auto& t : s.tris)
        for (uint32_t vi : { t.v0, t.v1, t.v2 })
            for (int a = 0; a < 3; a++)
            {
                mn[a] = std::min(mn[a], s.verts[vi].p[a]);
                mx[a] = std::max(mx[a], s.verts[vi].p[a]);
            }
    // grid.cpp:29-38
    float ext[3];
    for (int a = 0; a < 3; a++)
    {
        s.bmin[a] = mn[a] - 0.0001f;
        s.bmax[a] = mx[a] + 0.0001f;
        ext[a] = s.bmax[a] - s.bmin[a];
    }
    const float largest = std::max(std::max(ext[0], ext[1]), ext[2]);
    s.cw = largest / float(res);
    s.icw = 1.0f / s.cw;
    for (int a = 0; a < 3; a++) s.dims[a] = uint32_t(std::ceil(ext[a] / s.cw));
    const uint64_t nc64 = uint64_t(s.dims[0]) * s.dims[1] * s.dims[2];
    if (nc64 == 0 || nc64 > (1ull << 31)) return fail(RT_E_INVALID, "degenerate grid");
    const uint32_t nc = uint32_t(nc64), dx = s.dims[0], dxdz = s.dims[0] * s.dims[2];
    const float cw = s.cw;

    // Per triangle (in parallel, contiguous ranges): the overlapped cells (grid.cpp:65-129)
    const uint32_t nt = uint32_t(s.tris.size());
    if (nthreads == 0) nthreads = std::max(1u, std::thread::hardware_concurrency());
    nthreads = std::min(nthreads, std::max(1u, nt / 64));
    std::vector<std::vector<uint32_t>> pairs(nthreads);      // (cell, tri) flattened
    std::atomic<bool> bad(false);
    auto work = [&](uint32_t w) {
        const uint32_t lo = uint32_t(uint64_t(nt) * w / nthreads), hi = uint32_t(uint64_t(nt) * (w + 1) / nthreads);
        std::vector<uint32_t>& out = pairs[w];
        for (uint32_t ti = lo; ti < hi; ti++)
        {
            const rt_triangle& t = s.tris[ti];
            const float *p0 = s.verts[t.v0].p, *p1 = s.verts[t.v1].p, *p2 = s.verts[t.v2].p;
            uint32_t st[3], en[3];
            for (int a = 0; a < 3; a++)
            {
                // triangle.h:116-131 TriangleAABB (same float::min() seed), relative to the grid
                const float tmn = std::min(std::min(std::min(fmax, p0[a]), p1[a]), p2[a]) - s.bmin[a];
                const float tmx = std::max(std::max(std::max(fmin, p0[a]), p1[a]), p2[a]) - s.bmin[a];
                st[a] = uint32_t(int64_t(tmn / cw));          // grid.cpp:81-92 uint(float)
                en[a] = uint32_t(int64_t(tmx / cw));
            }
            uint32_t hits = 0;
            for (uint32_t x = st[0]; x <= en[0]; x++)
                for (uint32_t y = st[1]; y <= en[1]; y++)
                    for (uint32_t z = st[2]; z <= en[2]; z++)
                    {
                        // grid.cpp:101-108 cell bounds in float, aabb.h:19-26 centre/half
                        const float cmin[3] = { s.bmin[0] + float(x) * cw, s.bmin[1] + float(y) * cw,
                                                s.bmin[2] + float(z) * cw };
                        const float cmax[3] = { s.bmin[0] + float(x + 1) * cw, s.bmin[1] + float(y + 1) * cw,
                                                s.bmin[2] + float(z + 1) * cw };
                        const double ctr[3] = { (cmin[0] + cmax[0]) * 0.5f, (cmin[1] + cmax[1]) * 0.5f,
                                                (cmin[2] + cmax[2]) * 0.5f };
                        const double half[3] = { (cmax[0] - cmin[0]) * 0.5f, (cmax[1] - cmin[1]) * 0.5f,
                                                 (cmax[2] - cmin[2]) * 0.5f };
                        if (tri_box(ctr, half, p0, p1, p2))
                        {
                            const uint32_t cell = x + z * dx + y * dxdz;   // grid.h:41-42
                            if (cell >= nc) { bad = true; continue; }
                            out.push_back(cell);
                            out.push_back(ti);
                            hits++;
                        }
                    }
            if (hits == 0) bad = true;                        // grid.cpp:125 assert
        }
    };
    std::vector<std::thread> pool;
    for (uint32_t w = 1; w < nthreads; w++) pool.emplace_back(work, w);
    work(0);
    for (auto& th : pool) th.join();
    if (bad) return fail(RT_E_INVALID, "a triangle touches no cell or lies outside the grid (grid.cpp:121-125)");

    // Stable counting sort by cell: thread ranges are in triangle order, so every cell's
    // list comes out ascending -- the push_back order of grid.cpp:122.
    s.off.assign(size_t(nc) + 1, 0);
    for (const auto& pv : pairs)
        for (size_t i = 0; i < pv.size(); i += 2) s.off[pv[i] + 1]++;
    for (uint32_t c = 0; c < nc; c++) s.off[c + 1] += s.off[c];
    s.refs.resize(s.off[nc]);
    std::vector<uint32_t> cursor(s.off.begin(), s.off.end() - 1);
    for (const auto& pv : pairs)
        for (size_t i = 0; i < pv.size(); i += 2) s.refs[cursor[pv[i]]++] = pv[i + 1];
    s.build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

int read_scene(const char* path, rth_scene& s)
{
    std::FILE* f = std::fopen(path, "rb");
    if (!f) return fail(RT_E_INVALID, std::string("cannot open ") + path);
    char magic[8];
    uint32_t nv = 0, nt = 0;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "RTSCENE1", 8) == 0 &&
              std::fread(&s.id, 4, 1, f) == 1 && std::fread(&s.fov, 4, 1, f) == 1 &&
              std::fread(s.cam, 4, 16, f) == 16 && std::fread(&nv, 4, 1, f) == 1 && std::fread(&nt, 4, 1, f) == 1 &&
              nv > 0 && nt > 0 && nv < (1u << 28) && nt < (1u << 28);
    if (ok)
    {
        s.verts.resize(nv);
        s.tris.resize(nt);
        ok = std::fread(s.verts.data(), sizeof(rt_vertex), nv, f) == nv &&
             std::fread(s.tris.data(), sizeof(rt_triangle), nt, f) == nt;
    }
    std::fclose(f);
    if (!ok) return fail(RT_E_INVALID, std::string("malformed .rtscene: ") + path);
    for (const auto& t : s.tris)
        if (t.v0 >= nv || t.v1 >= nv || t.v2 >= nv) return fail(RT_E_INVALID, "vertex index out of bounds");
    return RT_OK;
}

static_assert(sizeof(rt_vertex) == 24 && sizeof(rt_triangle) == 24, "Mesh::Vertex/Triangle layouts (mesh.h)");

} // namespace

int rth_internal_fail(int code, const std::string& m) { return fail(code, m); }

// ================================================================= Framebuffer (host)
// framebuffer.h:16-101 / framebuffer.cpp restated without OpenGL: 12x9 tiles, a
// hardware_concurrency() worker pool, shuffled LIFO queue, per-tile mutex held across
// RenderTile, stop flag polled between tiles.  Two changes that nothing outside can observe:
// the workers are created once and parked between frames (the reference spawns and joins a
// std::thread per worker per frame, framebuffer.cpp:16-41), and StartRendering's tile clear
// (framebuffer.cpp:127-131) is deferred: a tile RenderTile overwrites whole is never cleared,
// and the tiles a stopped frame left unrendered are cleared when the frame is finished.
namespace {

class Framebuffer
{
public:
    explicit Framebuffer(uint32_t nthreads)
        : m_num_cpus(nthreads ? nthreads : std::max(1u, std::thread::hardware_concurrency())) { }
    virtual ~Framebuffer() { Shutdown(); }

    void Resize(uint32_t width, uint32_t height)               // framebuffer.cpp:94-122
    {
        KillAllWorkerThreads();
        m_width = width;
        m_height = height;
        const uint32_t tw = width / kTilesX, th = height / kTilesY;
        for (uint32_t y = 0; y < kTilesY; y++)
            for (uint32_t x = 0; x < kTilesX; x++)
                m_tiles[x + y * kTilesX].SetPosition(x * tw, y * th, (x == kTilesX - 1) ? width : (x + 1) * tw,
                                                     (y == kTilesY - 1) ? height : (y + 1) * th);
        CreateWorkerThreads();
    }

    // framebuffer.cpp:124-134.  The synchronous form (rth_framebuffer_start_rendering) is followed by
    // Wait(); StartRenderingAsync is the reference's own threading: it returns at once, and the frame's
    // tiles are delivered in the background -- by the worker pool, or (an inline frame) by the
    // delivery thread -- each under its mutex with its dirty flag set, for Draw to pick up.
    void StartRendering() { Start(false); }
    void StartRenderingAsync() { Start(true); }

    // Blocks until every worker has finished the current frame (the reference's join).
    void Wait()
    {
        if (m_inline_pending)
        {
            // a frame completed by the waiting thread itself (CompletesInline): its tiles, in tile-row
            // order, each under its mutex as a worker would mark it
            m_inline_pending = false;
            FinishInline(false);
            m_last_frame_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - m_start).count();
        }
        // spin briefly first: a GPU frame ends within a millisecond, and a condition-variable wake-up
        // costs tens of microseconds of it (the frame's last worker sets m_done_gen).  The spin is
        // bounded by time (2 ms), so a long frame -- CPU-bound or multi-GPU -- blocks instead.
        const uint64_t gen = m_generation_seen.load(std::memory_order_acquire);
        if (m_done_gen.load(std::memory_order_acquire) < gen)
        {
            const auto spin_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
            for (uint32_t i = 1; m_done_gen.load(std::memory_order_acquire) < gen; i++)
            {
                std::this_thread::yield();
                if ((i & 63u) == 0u && std::chrono::steady_clock::now() > spin_end) break;
            }
        }
        std::unique_lock<std::mutex> lk(m_pool_mtx);
        m_pool_cv.wait(lk, [&] { return m_threads_done == m_running; });
        lk.unlock();
        bool unreached = false;
        for (const auto& t : m_tiles) unreached = unreached || t.clear_pending;
        if (unreached) DrainIssued();                           // no copy-back lands in them after the clear
        for (auto& t : m_tiles)                                 // tiles the frame did not reach
            if (t.clear_pending)
            {
                std::lock_guard<std::mutex> g(t.mtx);
                t.Clear();
                t.clear_pending = false;
            }
    }

    double LastFrameSeconds() const { return m_last_frame_s; }
    uint32_t Width() const { return m_width; }
    uint32_t Height() const { return m_height; }

    // framebuffer.cpp:149-193 Draw, with the tiles' GL textures replaced by `display` (width x height
    // words, row-major; NULL: count only).  A tile whose mutex is free (try_lock, as Draw) and whose
    // buffer changed since its last upload (dirty) is copied into its rectangle and its dirty flag
    // reset (Tile::UpdateTexture); a tile StartRendering cleared shows cleared until then.  Returns the
    // tiles uploaded; *done = the current frame's tiles delivered so far (of kTilesX * kTilesY).
    uint32_t Draw(uint32_t* display, uint32_t* done)
    {
        uint32_t updated = 0, ndone = 0;
        for (auto& t : m_tiles)
        {
            if (!t.mtx.try_lock()) continue;
            ndone += t.delivered ? 1u : 0u;
            if (display && (t.dirty || t.texture_clear))
            {
                for (uint32_t y = 0; y < t.GetHeight(); y++)
                {
                    uint32_t* row = display + size_t(t.y0 + y) * m_width + t.x0;
                    if (t.dirty) std::memcpy(row, t.GetBuffer() + size_t(y) * t.GetWidth(), size_t(t.GetWidth()) * 4);
                    else std::fill(row, row + t.GetWidth(), 0u);
                }
                updated += t.dirty ? 1u : 0u;
                t.dirty = false;
                t.texture_clear = false;
            }
            t.mtx.unlock();
        }
        if (done) *done = ndone;
        return updated;
    }

    // framebuffer.cpp:195-221 SaveToBMP's assembly step; bitmap row 0 = pixel row 0
    void Assemble(uint32_t* bitmap) const
    {
        for (const auto& t : m_tiles)
            for (uint32_t y = 0; y < t.GetHeight(); y++)
                std::memcpy(bitmap + size_t(t.y0 + y) * m_width + t.x0, t.GetBuffer() + size_t(y) * t.GetWidth(),
                            size_t(t.GetWidth()) * 4);
    }

protected:
    struct Tile                                                 // framebuffer.h:34-70
    {
        void GetPosition(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) const { a = x0; b = y0; c = x1; d = y1; }
        uint32_t GetWidth() const { return x1 - x0; }
        uint32_t GetHeight() const { return y1 - y0; }
        // the tile's buffer: its own, or (a renderer's zero-copy frame) its view into that frame,
        // laid out the same way (row-major at the tile's width)
        uint32_t* GetBuffer() { return view ? view : &bgra[0]; }
        const uint32_t* GetBuffer() const { return view ? view : &bgra[0]; }
        void SetPosition(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
        {
            x0 = a; y0 = b; x1 = c; y1 = d;
            view = nullptr;
            bgra.assign(std::max<size_t>(1, size_t(GetWidth()) * GetHeight()), 0);
            clear_pending = false;
            dirty = delivered = false;
            texture_clear = true;
        }
        // a worker (or the delivery) finished the tile: under its mutex
        void MarkDelivered() { clear_pending = false; dirty = delivered = true; }
        void Clear() { std::fill(GetBuffer(), GetBuffer() + size_t(GetWidth()) * GetHeight(), 0u); }
        std::mutex mtx;
        std::vector<uint32_t> bgra = std::vector<uint32_t>(1, 0);
        uint32_t* view = nullptr;
        uint32_t x0 = 0, y0 = 0, x1 = 1, y1 = 1;
        bool clear_pending = false;                             // StartRendering's clear, deferred
        bool dirty = false;                                     // framebuffer.h:54-65 m_dirty
        bool delivered = false;                                 // done in the current frame
        bool texture_clear = true;                              // Draw shows the tile cleared
    };

    // true = the whole tile buffer was written (renderer.cpp:74-135 writes every pixel), false =
    // it returned early (stop flag, renderer.cpp:76-77) and the tile keeps its cleared state.
    virtual bool RenderTile(Tile& tile) = 0;
    virtual void BeginFrame() { }
    // true: BeginFrame produces the whole frame by itself (a GPU frame issued from the starting
    // thread), so no worker is woken: Wait() runs FinishInline, which delivers every tile in the
    // calling thread.  The pool's wake-ups and hand-offs cost 0.1-0.4 ms of a 0.2-0.4 ms frame.
    virtual bool CompletesInline() const { return false; }
    // async: run by the delivery thread (StartRenderingAsync), which stops between tiles when asked
    virtual void FinishInline(bool async) { (void)async; }
    // waits out a frame's copy-back still in flight (a stopped frame's tiles are cleared after it)
    virtual void DrainIssued() { }

    void KillAllWorkerThreads()                                 // framebuffer.cpp:30-41
    {
        m_threads_stop = true;
        Wait();
        m_threads_stop = false;
    }

    // Stops and joins the parked workers (derived destructors call it first: the workers call
    // the derived RenderTile).
    void Shutdown()
    {
        KillAllWorkerThreads();
        {
            std::lock_guard<std::mutex> lk(m_pool_mtx);
            m_shutdown = true;
        }
        m_pool_cv.notify_all();
        for (auto& th : m_threads)
            if (th.joinable()) th.join();
        m_threads.clear();
        if (m_delivery.joinable()) m_delivery.join();
    }

    uint32_t m_width = 1, m_height = 1;
    std::atomic<bool> m_threads_stop{ false };                  // volatile bool in the reference
    static const uint32_t kTilesX = 12, kTilesY = 9;           // framebuffer.h:87-88
    std::array<Tile, kTilesX * kTilesY> m_tiles;

private:
    void Start(bool async)
    {
        KillAllWorkerThreads();
        for (auto& t : m_tiles)                                 // Tile::Clear + UpdateTexture, deferred
        {
            std::lock_guard<std::mutex> g(t.mtx);
            t.clear_pending = true;
            t.dirty = t.delivered = false;
            t.texture_clear = true;
        }
        m_async = async;
        CreateWorkerThreads();
    }

    void CreateWorkerThreads()                                  // framebuffer.cpp:16-28
    {
        if (CompletesInline() && !m_threads_stop)
        {
            {
                std::lock_guard<std::mutex> lk(m_pool_mtx);
                m_start = std::chrono::steady_clock::now();
                BeginFrame();
                m_generation++;
                m_generation_seen.store(m_generation, std::memory_order_release);
                if (!m_async)
                {
                    m_threads_done = m_running = 0;
                    m_done_gen.store(m_generation, std::memory_order_release);
                    m_inline_pending = true;
                    return;
                }
                // asynchronous: the delivery thread takes the frame's tiles as they land
                if (!m_delivery.joinable()) m_delivery = std::thread(&Framebuffer::DeliveryThread, this);
                m_threads_done = 0;
                m_running = 1;
                m_deliver_gen++;
            }
            m_pool_cv.notify_all();
            return;
        }
        BeginFrame();
        m_work_queue.clear();
        for (uint32_t i = 0; i < kTilesX * kTilesY; i++) m_work_queue.push_back(i);
        std::shuffle(m_work_queue.begin(), m_work_queue.end(), std::mt19937(m_frame_seed++));
        while (m_threads.size() < m_num_cpus)
            m_threads.emplace_back(&Framebuffer::PoolThread, this, uint32_t(m_threads.size()));
        {
            std::lock_guard<std::mutex> lk(m_pool_mtx);
            m_threads_done = 0;
            m_running = m_num_cpus;
            m_start = std::chrono::steady_clock::now();
            m_generation++;
            m_generation_seen.store(m_generation, std::memory_order_release);
        }
        m_pool_cv.notify_all();
    }

    Tile* GetNextTileFromQueue()                                // framebuffer.cpp:43-57
    {
        std::lock_guard<std::mutex> g(m_queue_mtx);
        if (m_work_queue.empty()) return nullptr;
        Tile* t = &m_tiles[m_work_queue.back()];
        m_work_queue.pop_back();
        return t;
    }

    // The asynchronous inline frame's delivery: one parked thread (a frame's wake-up costs one
    // thread, not the pool's), which runs FinishInline and then reports the frame done as the pool's
    // last worker would.
    void DeliveryThread()
    {
        uint64_t seen = 0;
        for (;;)
        {
            {
                std::unique_lock<std::mutex> lk(m_pool_mtx);
                m_pool_cv.wait(lk, [&] { return m_shutdown || m_deliver_gen != seen; });
                if (m_shutdown) return;
                seen = m_deliver_gen;
            }
            FinishInline(true);
            std::lock_guard<std::mutex> lk(m_pool_mtx);
            if (++m_threads_done == m_running)
            {
                if (!m_threads_stop)
                    m_last_frame_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - m_start).count();
                m_done_gen.store(m_generation, std::memory_order_release);
                m_pool_cv.notify_all();
            }
        }
    }

    void PoolThread(uint32_t)
    {
        uint64_t seen = 0;
        for (;;)
        {
            {
                std::unique_lock<std::mutex> lk(m_pool_mtx);
                m_pool_cv.wait(lk, [&] { return m_shutdown || m_generation != seen; });
                if (m_shutdown) return;
                seen = m_generation;
            }
            WorkerThread();
        }
    }

    void WorkerThread()                                         // framebuffer.cpp:59-92
    {
        while (!m_threads_stop)
        {
            Tile* tile = GetNextTileFromQueue();
            if (!tile) break;
            std::lock_guard<std::mutex> g(tile->mtx);
            if (RenderTile(*tile)) tile->MarkDelivered();       // framebuffer.cpp:72-77 SetDirty(true)
        }
        std::lock_guard<std::mutex> lk(m_pool_mtx);
        if (++m_threads_done == m_running)
        {
            if (!m_threads_stop)
                m_last_frame_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - m_start).count();
            m_done_gen.store(m_generation, std::memory_order_release);
            m_pool_cv.notify_all();
        }
    }

    const uint32_t m_num_cpus;
    std::vector<uint32_t> m_work_queue;
    std::mutex m_queue_mtx;
    std::vector<std::thread> m_threads;
    std::thread m_delivery;                                     // StartRenderingAsync's inline frames
    uint64_t m_deliver_gen = 0;
    bool m_async = false;                                       // the current frame was started async
    std::mutex m_pool_mtx;                                      // generation / done counters
    std::condition_variable m_pool_cv;
    uint64_t m_generation = 0;
    std::atomic<uint64_t> m_generation_seen{ 0 }, m_done_gen{ 0 };   // Wait's spin phase
    uint32_t m_threads_done = 0, m_running = 0;
    bool m_shutdown = false;
    bool m_inline_pending = false;                              // CompletesInline: Wait delivers the frame
    std::chrono::steady_clock::time_point m_start;
    double m_last_frame_s = 0.0;
    uint32_t m_frame_seed = 1;
};

// Renderer (renderer.h) with the tile callback served by GPU frames: the first worker of a frame
// issues the whole frame (Issue: one launch per device) whose copy-back lands, tile row by tile
// row, in this renderer's page-locked frame; every worker then waits only for its own tile row
// (WaitRows) and copies its tile straight out of that frame while holding the tile's mutex (the
// reference's locking contract, framebuffer.cpp:71-74).  One DMA pass and one tile copy per pixel.
class FrameRenderer : public Framebuffer
{
public:
    explicit FrameRenderer(uint32_t nthreads) : Framebuffer(nthreads) { }

    void SetSampleCount(uint32_t cnt) { m_spp = std::max(1u, cnt); }   // renderer.cpp:18-22
    void SetOptions(uint32_t tri_test, uint32_t kernel) { m_tri_test = tri_test; m_kernel = kernel; }
    void SetIntersector(uint32_t isect) { m_isect = isect; }             // renderer.cpp:103-105
    int LastStatus() const { return m_status; }
    const std::string& LastError() const { return m_err; }

    // The last frame, whole, when every tile of it was delivered (else nullptr): what
    // SaveToBMP's assembly (framebuffer.cpp:197-216) would rebuild from the tiles.  (A tiled frame
    // holds the tile buffers themselves: the assembly runs.)
    const uint32_t* CompleteFrame() const
    {
        return (!Tiled() && m_status == RT_OK && m_issued && m_tiles_done.load() == kTilesX * kTilesY) ? m_frame
                                                                                                      : nullptr;
    }

protected:
    // One frame into the page-locked frame: band b holds rows [ends[b-1], ends[b]).  Asynchronous;
    // WaitRows(y1) returns once rows [0, y1) have landed.  On failure: an RT_E* code, message in
    // m_err.
    virtual int Issue(const rt_frame& f, uint32_t* host_frame, const uint32_t* ends, uint32_t nb) = 0;
    virtual int WaitRows(uint32_t y1) = 0;
    // true: Issue delivers the frame as the tiles' own buffers (rt_render_frame_host_tiled's layout):
    // the tiles are views into the page-locked frame and RenderTile copies nothing
    virtual bool Tiled() const { return false; }
    virtual int AllocHost(size_t bytes, void** p) = 0;
    virtual void FreeHost(void* p) = 0;

    // derived destructors: Shutdown(), then this (workers call the derived WaitRows)
    void ReleaseFrame()
    {
        DrainFrame();
        if (m_frame) FreeHost(m_frame);
        m_frame = nullptr;
        m_frame_cap = 0;
    }

    // The frame is issued here, by the thread that starts it (Resize / StartRendering), before the
    // workers are woken: the GPU starts at once instead of after a worker's wake-up, and the workers'
    // wake-up overlaps the render.  (A stopped frame issues nothing: RenderTile's check.)
    void BeginFrame() override
    {
        std::lock_guard<std::mutex> g(m_frame_mtx);
        m_frame_ready = false;
        m_status = RT_OK;
        m_tiles_done = 0;
        m_rows_ready = 0;
        if (!m_threads_stop && m_issue_early)
        {
            m_frame_ready = true;
            IssueFrame();
        }
    }

    // The inline delivery (RTH_POOL=0, the default): the starting thread issued the frame in
    // BeginFrame; the waiting thread takes its tiles row by row -- one wait per tile row, then each
    // tile of the row under its mutex, as RenderTile would (a copy only for the row-major frame).
    bool CompletesInline() const override { return m_inline && m_issue_early; }
    void FinishInline(bool async) override
    {
        for (auto& t : m_tiles)
        {
            if (async && m_threads_stop)
            {
                // stopped (the next StartRendering / Resize): the frame's copy-back still lands in the
                // tiles' buffers, so it is waited out before Wait clears the tiles not reached
                DrainFrame();
                return;
            }
            if (t.y1 > m_rows_ready.load())
            {
                {
                    std::lock_guard<std::mutex> g(m_frame_mtx);
                    if (!m_frame_ready || m_status != RT_OK) return;
                }
                const int rc = WaitRows(t.y1);
                if (rc != RT_OK)
                {
                    std::lock_guard<std::mutex> g(m_frame_mtx);
                    m_status = rc;
                    return;
                }
                m_rows_ready.store(t.y1);
            }
            std::lock_guard<std::mutex> g(t.mtx);
            if (RenderTile(t)) t.MarkDelivered();
        }
    }

    void DrainIssued() override { DrainFrame(); }

    bool RenderTile(Tile& tile) override
    {
        {
            std::lock_guard<std::mutex> g(m_frame_mtx);
            if (!m_frame_ready)
            {
                if (m_threads_stop) return false;                 // renderer.cpp:76-77
                m_frame_ready = true;
                IssueFrame();
            }
            if (m_status != RT_OK) return false;
        }
        uint32_t x0, y0, x1, y1;
        tile.GetPosition(x0, y0, x1, y1);
        const int rc = y1 <= m_rows_ready.load() ? RT_OK : WaitRows(y1);
        if (rc != RT_OK)
        {
            std::lock_guard<std::mutex> g(m_frame_mtx);
            m_status = rc;
            return false;
        }
        if (!Tiled())
        {
            uint32_t* buf = tile.GetBuffer();
            for (uint32_t y = 0; y < tile.GetHeight(); y++)    // renderer.cpp:133 layout
                std::memcpy(buf + size_t(y) * tile.GetWidth(), m_frame + size_t(y0 + y) * m_width + x0,
                            size_t(tile.GetWidth()) * 4);
        }
        m_tiles_done.fetch_add(1);
        return true;
    }

    std::string m_err;
    bool m_issue_early = true;          // the starting thread issues the frame (round 4: before the workers wake)
    bool m_inline = true;               // RTH_POOL=1: the worker pool delivers the tiles (A/B)

private:
    // A frame's copy-back may still be landing in m_frame (workers stopped early): wait it out
    // before the frame memory is reused or freed.
    void DrainFrame()
    {
        if (m_issued && m_issued_h) (void)WaitRows(m_issued_h);
        m_issued = false;
    }

    void IssueFrame()                                           // under m_frame_mtx
    {
        const size_t words = size_t(m_width) * m_height;
        if (words > m_frame_cap)
        {
            DrainFrame();
            if (m_frame) FreeHost(m_frame);
            m_frame = nullptr;
            m_frame_cap = 0;
            void* p = nullptr;
            const int rc = AllocHost(words * 4, &p);
            if (rc != RT_OK) { m_status = rc; return; }
            m_frame = static_cast<uint32_t*>(p);
            m_frame_cap = words;
        }
        if (Tiled())
        {
            // the tiles' buffers are views of the frame's tile layout: tile (c, r) at word
            // y0 * W + th_r * x0 (rt_render_frame_host_tiled), row-major at its own width
            for (auto& t : m_tiles) t.view = m_frame + size_t(t.y0) * m_width + size_t(t.GetHeight()) * t.x0;
        }
        rt_frame f;
        std::memset(&f, 0, sizeof(f));
        std::memcpy(f.cam, m_host_cam, sizeof(f.cam));          // Scene::GetCameraParameters
        f.fov = m_host_fov;
        f.width = m_width;
        f.height = m_height;
        f.spp = m_spp;
        f.tri_test = m_tri_test;
        f.kernel = m_kernel;
        f.intersector = m_isect;
        // one copy-back band per tile row (framebuffer.cpp:106-117: rows of height/9, the last
        // row absorbs the remainder)
        uint32_t ends[kTilesY];
        uint32_t nb = 0;
        for (uint32_t j = 0; j < kTilesY; j++)
        {
            const uint32_t e = (j == kTilesY - 1) ? m_height : (j + 1) * (m_height / kTilesY);
            if (e > (nb ? ends[nb - 1] : 0u)) ends[nb++] = e;
        }
        const int rc = Issue(f, m_frame, ends, nb);
        if (rc != RT_OK) { m_status = rc; return; }
        m_issued = true;
        m_issued_h = m_height;
    }

protected:
    float m_host_cam[16] = {};
    float m_host_fov = 45.0f;

private:
    uint32_t m_spp = 16;                                        // renderer.h:34
    uint32_t m_tri_test = RT_TRI_MOLLER_TRUMBORE, m_kernel = RT_KERNEL_AUTO, m_isect = RT_ISECT_GRID;
    std::mutex m_frame_mtx;
    bool m_frame_ready = false;
    uint32_t* m_frame = nullptr;                                // page-locked, m_width x m_height
    size_t m_frame_cap = 0;
    bool m_issued = false;
    uint32_t m_issued_h = 0;
    std::atomic<uint32_t> m_tiles_done{ 0 };
    std::atomic<uint32_t> m_rows_ready{ 0 };                    // rows [0, m_rows_ready) known landed
    int m_status = RT_OK;
};

// One device: librt_tracer renders the frame in one launch and copies it back in row bands
// (rt_render_frame_host / rt_frame_host_wait).
class GpuRenderer : public FrameRenderer
{
public:
    GpuRenderer(rt_scene* gpu, const rth_scene* host, uint32_t nthreads) : FrameRenderer(nthreads), m_gpu(gpu)
    {
        std::memcpy(m_host_cam, host->cam, sizeof(m_host_cam));
        m_host_fov = host->fov;
        const char* e = std::getenv("RTH_TILED");
        m_tiled = !(e && *e == '0');
        const char* l = std::getenv("RTH_LAUNCHES");
        m_launches = l && *l ? std::max(1, std::atoi(l)) : 1;
        const char* po = std::getenv("RTH_POOL");
        m_inline = !(po && *po == '1');
    }
    ~GpuRenderer() override
    {
        Shutdown();
        ReleaseFrame();
    }

protected:
    // The zero-copy drop-in: the tile buffers are views of the page-locked frame, which the kernels
    // write in the tiles' layout and which comes back one tile row per D2H copy, rendered in
    // m_launches row-band launches on two streams (copies overlap the next band's render).
    // RTH_TILED=0 keeps the row-major frame + per-tile copy (A/B arm).
    int Issue(const rt_frame& f, uint32_t* host_frame, const uint32_t* ends, uint32_t nb) override
    {
        if (m_tiled)
            return Check(rt_render_frame_host_tiled(m_gpu, &f, host_frame, kTilesX, kTilesY, m_launches));
        return Check(rt_render_frame_host(m_gpu, &f, host_frame, ends, nb));
    }
    int WaitRows(uint32_t y1) override { return Check(rt_frame_host_wait(m_gpu, y1)); }
    bool Tiled() const override { return m_tiled; }
    int AllocHost(size_t bytes, void** p) override { return Check(rt_host_alloc(bytes, p)); }
    void FreeHost(void* p) override { (void)rt_host_free(p); }

private:
    int Check(int rc)
    {
        if (rc != RT_OK)
        {
            char msg[512];
            rt_last_error(msg, sizeof(msg));
            m_err = msg;
        }
        return rc;
    }
    rt_scene* m_gpu;
    bool m_tiled = true;
    uint32_t m_launches = 1;    // row-band launches per frame (RTH_LAUNCHES)
};

// ================================================================= multi-GPU frame source
// RCCL (librccl.so.1), loaded on the first multi-device framebuffer: single-device users never
// map it, and in a process that already holds one (torch) the loader returns that one.
struct RcclApi
{
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*ErrorString)(ncclResult_t) = nullptr;
};

const RcclApi* rccl_api(std::string& err)
{
    static std::mutex mtx;
    static RcclApi api;
    static bool tried = false, ok = false;
    static std::string why;
    std::lock_guard<std::mutex> g(mtx);
    if (!tried)
    {
        tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h)
            why = std::string("cannot load librccl.so.1: ") + dlerror();
        else
        {
            ok = true;
            auto sym = [&](const char* name) {
                void* f = dlsym(h, name);
                if (!f) { ok = false; why = std::string("librccl.so.1 lacks ") + name; }
                return f;
            };
            api.CommInitAll = reinterpret_cast<decltype(api.CommInitAll)>(sym("ncclCommInitAll"));
            api.CommDestroy = reinterpret_cast<decltype(api.CommDestroy)>(sym("ncclCommDestroy"));
            api.Send = reinterpret_cast<decltype(api.Send)>(sym("ncclSend"));
            api.Recv = reinterpret_cast<decltype(api.Recv)>(sym("ncclRecv"));
            api.GroupStart = reinterpret_cast<decltype(api.GroupStart)>(sym("ncclGroupStart"));
            api.GroupEnd = reinterpret_cast<decltype(api.GroupEnd)>(sym("ncclGroupEnd"));
            api.ErrorString = reinterpret_cast<decltype(api.ErrorString)>(sym("ncclGetErrorString"));
        }
    }
    err = why;
    return ok ? &api : nullptr;
}

constexpr uint32_t kMaxRanks = 64;

// The Framebuffer's RenderTile served by N GPUs of this node (the drop-in for the
// CPU pool of framebuffer.cpp:16-28, 59-92): the scene is replicated on every device (one
// rt_scene each), device i renders rank i's interleaved 16x16 tiles compactly
// (rt_render_shard_device), ONE gather collects the shards on devices[0], K3 un-permutes them
// (rt_unshard_device) and the frame comes back in tile-row bands.  The gather is RCCL when every
// device is listed once (ncclCommInitAll in this process, then one group of ncclSend on every
// rank -- rank 0 to itself -- and ncclRecv of every rank's slice on rank 0: each peer's slice on
// its own xGMI link, not an all-gather ring).  A device listed more than once holds several
// logical ranks (a rehearsal of N ranks on fewer GPUs); RCCL takes each device once, so those
// shards move by device copies instead.
class MultiGpuRenderer : public FrameRenderer
{
public:
    MultiGpuRenderer(const rth_scene* host, uint32_t nthreads) : FrameRenderer(nthreads)
    {
        std::memcpy(m_host_cam, host->cam, sizeof(m_host_cam));
        m_host_fov = host->fov;
    }

    ~MultiGpuRenderer() override
    {
        Shutdown();
        ReleaseFrame();
        for (uint32_t i = 0; i < m_n; i++)
        {
            (void)hipSetDevice(m_dev[i]);
            if (m_stream[i]) (void)hipStreamSynchronize(m_stream[i]);
        }
        for (uint32_t i = 0; i < m_n; i++)
        {
            (void)hipSetDevice(m_dev[i]);
            if (m_comm[i] && m_rccl) (void)m_rccl->CommDestroy(m_comm[i]);
            if (m_shard[i]) (void)hipFree(m_shard[i]);
            if (m_done[i]) (void)hipEventDestroy(m_done[i]);
            if (m_stream[i]) (void)hipStreamDestroy(m_stream[i]);
            if (m_scene[i]) (void)rt_scene_destroy(m_scene[i]);
        }
        if (m_n)
        {
            (void)hipSetDevice(m_dev[0]);
            if (m_gathered) (void)hipFree(m_gathered);
            if (m_dframe) (void)hipFree(m_dframe);
            for (hipEvent_t e : m_band_ev) if (e) (void)hipEventDestroy(e);
        }
    }

    int Init(const rth_scene* host, const int* devices, uint32_t n)
    {
        m_n = n;
        rt_scene_desc d;
        std::memset(&d, 0, sizeof(d));
        fill_desc(*host, d);
        bool distinct = true;
        for (uint32_t i = 0; i < n; i++)
        {
            m_dev[i] = devices[i];
            for (uint32_t j = 0; j < i; j++) distinct = distinct && devices[j] != devices[i];
            // one scene per rank (its own heavy-first state, as one process per GPU would have)
            int rc = rt_scene_create(&d, devices[i], &m_scene[i]);
            if (rc) return TracerError(rc);
            if ((rc = Hip(hipSetDevice(devices[i]), "hipSetDevice"))) return rc;
            if ((rc = Hip(hipStreamCreateWithFlags(&m_stream[i], hipStreamNonBlocking), "hipStreamCreate"))) return rc;
            if ((rc = Hip(hipEventCreateWithFlags(&m_done[i], hipEventDisableTiming), "hipEventCreate"))) return rc;
        }
        m_transport = distinct ? RTH_TRANSPORT_RCCL : RTH_TRANSPORT_DEVICE_COPY;
        if (distinct)
        {
            std::string why;
            m_rccl = rccl_api(why);
            if (!m_rccl) { m_err = why; return RT_E_RCCL; }
            if (int rc = Nccl(m_rccl->CommInitAll(m_comm, int(n), devices), "ncclCommInitAll")) return rc;
        }
        return RT_OK;
    }

    const std::string& InitError() const { return m_err; }
    uint32_t Transport() const { return m_transport; }
    uint32_t Ranks() const { return m_n; }

protected:
    int AllocHost(size_t bytes, void** p) override
    {
        if (int rc = Hip(hipSetDevice(m_dev[0]), "hipSetDevice")) return rc;
        return Hip(hipHostMalloc(p, bytes), "hipHostMalloc");
    }
    void FreeHost(void* p) override { (void)hipHostFree(p); }

    int Issue(const rt_frame& f, uint32_t* host_frame, const uint32_t* ends, uint32_t nb) override
    {
        uint64_t elems = 0;
        int rc = rt_shard_elems(f.width, f.height, m_n, &elems);
        if (rc) return TracerError(rc);
        if ((rc = Buffers(elems, size_t(f.width) * f.height))) return rc;
        // (1) every rank renders its tiles on its own device and stream
        for (uint32_t i = 0; i < m_n; i++)
            if ((rc = rt_render_shard_device(m_scene[i], &f, i, m_n, m_shard[i], m_stream[i]))) return TracerError(rc);
        // (2) one gather to rank 0
        if (m_transport == RTH_TRANSPORT_RCCL)
        {
            if ((rc = Nccl(m_rccl->GroupStart(), "ncclGroupStart"))) return rc;
            for (uint32_t i = 0; i < m_n && !rc; i++)
                rc = Nccl(m_rccl->Send(m_shard[i], elems, ncclUint32, 0, m_comm[i], m_stream[i]), "ncclSend");
            for (uint32_t i = 0; i < m_n && !rc; i++)
                rc = Nccl(m_rccl->Recv(m_gathered + i * elems, elems, ncclUint32, int(i), m_comm[0], m_stream[0]),
                          "ncclRecv");
            const int rc2 = Nccl(m_rccl->GroupEnd(), "ncclGroupEnd");
            if (rc || rc2) return rc ? rc : rc2;
        }
        else
            for (uint32_t i = 0; i < m_n; i++)
            {
                if ((rc = Hip(hipSetDevice(m_dev[i]), "hipSetDevice")) ||
                    (rc = Hip(hipEventRecord(m_done[i], m_stream[i]), "hipEventRecord")) ||
                    (rc = Hip(hipSetDevice(m_dev[0]), "hipSetDevice")) ||
                    (rc = Hip(hipStreamWaitEvent(m_stream[0], m_done[i], 0), "hipStreamWaitEvent")) ||
                    (rc = Hip(hipMemcpyPeerAsync(m_gathered + i * elems, m_dev[0], m_shard[i], m_dev[i], elems * 4,
                                                 m_stream[0]), "hipMemcpyPeerAsync")))
                    return rc;
            }
        // (3) K3 un-permute on rank 0, (4) copy-back in tile-row bands
        if ((rc = Hip(hipSetDevice(m_dev[0]), "hipSetDevice"))) return rc;
        if ((rc = rt_unshard_device(f.width, f.height, m_n, m_gathered, m_dframe, m_stream[0]))) return TracerError(rc);
        m_nbands = 0;
        for (uint32_t b = 0, ya = 0; b < nb; b++)
        {
            const uint32_t yb = ends[b];
            if (!m_band_ev[b] && (rc = Hip(hipEventCreateWithFlags(&m_band_ev[b], hipEventDisableTiming), "hipEventCreate")))
                return rc;
            if ((rc = Hip(hipMemcpyAsync(host_frame + size_t(ya) * f.width, m_dframe + size_t(ya) * f.width,
                                         size_t(yb - ya) * f.width * 4, hipMemcpyDeviceToHost, m_stream[0]),
                          "hipMemcpyAsync")) ||
                (rc = Hip(hipEventRecord(m_band_ev[b], m_stream[0]), "hipEventRecord")))
                return rc;
            m_band_y1[b] = yb;
            m_nbands = b + 1;
            ya = yb;
        }
        return RT_OK;
    }

    int WaitRows(uint32_t y1) override
    {
        if (!m_nbands) return RT_OK;
        uint32_t b = 0;
        while (b + 1 < m_nbands && m_band_y1[b] < y1) b++;
        return Hip(hipEventSynchronize(m_band_ev[b]), "hipEventSynchronize");
    }

private:
    static void fill_desc(const rth_scene& s, rt_scene_desc& d)        // as rth_scene_desc
    {
        d.num_vertices = uint32_t(s.verts.size());
        d.num_triangles = uint32_t(s.tris.size());
        d.vertices = s.verts.data();
        d.triangles = s.tris.data();
        for (int a = 0; a < 3; a++)
        {
            d.grid.dims[a] = s.dims[a];
            d.grid.aabb_min[a] = s.bmin[a];
            d.grid.aabb_max[a] = s.bmax[a];
        }
        d.grid.cell_wdh = s.cw;
        d.grid.inv_cell_wdh = s.icw;
        d.grid.cell_offsets = s.off.data();
        d.grid.cell_tris = s.refs.data();
    }

    int Buffers(uint64_t elems, size_t frame_words)
    {
        int rc;
        if (elems > m_elems_cap)
        {
            for (uint32_t i = 0; i < m_n; i++)
            {
                if ((rc = Hip(hipSetDevice(m_dev[i]), "hipSetDevice"))) return rc;
                if (m_shard[i]) (void)hipFree(m_shard[i]);
                m_shard[i] = nullptr;
                if ((rc = Hip(hipMalloc(&m_shard[i], elems * 4), "hipMalloc"))) return rc;
            }
            if ((rc = Hip(hipSetDevice(m_dev[0]), "hipSetDevice"))) return rc;
            if (m_gathered) (void)hipFree(m_gathered);
            m_gathered = nullptr;
            if ((rc = Hip(hipMalloc(&m_gathered, elems * 4 * m_n), "hipMalloc"))) return rc;
            m_elems_cap = elems;
        }
        if (frame_words > m_frame_cap)
        {
            if ((rc = Hip(hipSetDevice(m_dev[0]), "hipSetDevice"))) return rc;
            if (m_dframe) (void)hipFree(m_dframe);
            m_dframe = nullptr;
            if ((rc = Hip(hipMalloc(&m_dframe, frame_words * 4), "hipMalloc"))) return rc;
            m_frame_cap = frame_words;
        }
        return RT_OK;
    }

    int Hip(hipError_t e, const char* what)
    {
        if (e == hipSuccess) return RT_OK;
        m_err = std::string(what) + ": " + hipGetErrorString(e);
        return RT_E_HIP;
    }
    int Nccl(ncclResult_t r, const char* what)
    {
        if (r == ncclSuccess) return RT_OK;
        m_err = std::string(what) + ": " + (m_rccl ? m_rccl->ErrorString(r) : "RCCL not loaded");
        return RT_E_RCCL;
    }
    int TracerError(int rc)
    {
        char msg[512];
        rt_last_error(msg, sizeof(msg));
        m_err = msg;
        return rc;
    }

    uint32_t m_n = 0;
    uint32_t m_transport = RTH_TRANSPORT_NONE;
    const RcclApi* m_rccl = nullptr;
    int m_dev[kMaxRanks] = {};
    rt_scene* m_scene[kMaxRanks] = {};
    hipStream_t m_stream[kMaxRanks] = {};
    hipEvent_t m_done[kMaxRanks] = {};
    ncclComm_t m_comm[kMaxRanks] = {};
    uint32_t* m_shard[kMaxRanks] = {};
    uint64_t m_elems_cap = 0;
    uint32_t* m_gathered = nullptr;                             // devices[0]: [rank][shard]
    uint32_t* m_dframe = nullptr;                               // devices[0]: the frame
    size_t m_frame_cap = 0;
    hipEvent_t m_band_ev[16] = {};
    uint32_t m_band_y1[16] = {};
    uint32_t m_nbands = 0;
};

} // namespace

struct rth_framebuffer
{
    std::unique_ptr<FrameRenderer> r;
    const MultiGpuRenderer* multi = nullptr;      // rth_framebuffer_create_multi only
};

extern "C" {

int rth_last_error(char* buf, size_t len)
{
    if (!buf || !len) return RT_E_INVALID;
    std::snprintf(buf, len, "%s", g_err.c_str());
    return RT_OK;
}

int rth_scene_load(const char* path, uint32_t nthreads, rth_scene** out)
{
    if (!path || !out) return fail(RT_E_INVALID, "NULL argument");
    *out = nullptr;
    std::unique_ptr<rth_scene> s(new rth_scene());
    int rc = read_scene(path, *s);
    if (rc) return rc;
    if ((rc = build_grid(*s, 64, nthreads))) return rc;       // scene.cpp:7
    *out = s.release();
    return RT_OK;
}

int rth_scene_from_mesh(const rt_vertex* v, uint32_t nv, const rt_triangle* t, uint32_t nt, float fov,
                        const float cam[16], uint32_t res, uint32_t nthreads, rth_scene** out)
{
    if (!v || !t || !cam || !out || nv == 0 || nt == 0) return fail(RT_E_INVALID, "bad arguments");
    *out = nullptr;
    std::unique_ptr<rth_scene> s(new rth_scene());
    s->verts.assign(v, v + nv);
    s->tris.assign(t, t + nt);
    for (const auto& tr : s->tris)
        if (tr.v0 >= nv || tr.v1 >= nv || tr.v2 >= nv) return fail(RT_E_INVALID, "vertex index out of bounds");
    s->fov = fov;
    std::memcpy(s->cam, cam, sizeof(s->cam));
    int rc = build_grid(*s, res, nthreads);
    if (rc) return rc;
    *out = s.release();
    return RT_OK;
}

void rth_scene_free(rth_scene* s) { delete s; }

int rth_scene_set_id(rth_scene* s, uint32_t id)
{
    if (!s) return fail(RT_E_INVALID, "NULL scene");
    s->id = id;
    return RT_OK;
}

// The .rtscene cache: what rth_scene_load reads back, bit for bit.
int rth_scene_save(const rth_scene* s, const char* path)
{
    if (!s || !path) return fail(RT_E_INVALID, "NULL argument");
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_E_INVALID, std::string("cannot create ") + path);
    const uint32_t nv = uint32_t(s->verts.size()), nt = uint32_t(s->tris.size());
    bool ok = std::fwrite("RTSCENE1", 1, 8, f) == 8 && std::fwrite(&s->id, 4, 1, f) == 1 &&
              std::fwrite(&s->fov, 4, 1, f) == 1 && std::fwrite(s->cam, 4, 16, f) == 16 &&
              std::fwrite(&nv, 4, 1, f) == 1 && std::fwrite(&nt, 4, 1, f) == 1 &&
              std::fwrite(s->verts.data(), sizeof(rt_vertex), nv, f) == nv &&
              std::fwrite(s->tris.data(), sizeof(rt_triangle), nt, f) == nt;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_OK : fail(RT_E_INVALID, std::string("write failed: ") + path);
}

int rth_scene_desc(const rth_scene* s, rt_scene_desc* d)
{
    if (!s || !d) return fail(RT_E_INVALID, "NULL argument");
    std::memset(d, 0, sizeof(*d));
    d->num_vertices = uint32_t(s->verts.size());
    d->num_triangles = uint32_t(s->tris.size());
    d->vertices = s->verts.data();
    d->triangles = s->tris.data();
    for (int a = 0; a < 3; a++)
    {
        d->grid.dims[a] = s->dims[a];
        d->grid.aabb_min[a] = s->bmin[a];
        d->grid.aabb_max[a] = s->bmax[a];
    }
    d->grid.cell_wdh = s->cw;
    d->grid.inv_cell_wdh = s->icw;
    d->grid.cell_offsets = s->off.data();
    d->grid.cell_tris = s->refs.data();
    return RT_OK;
}

int rth_scene_camera(const rth_scene* s, float* fov, float cam[16])
{
    if (!s || !fov || !cam) return fail(RT_E_INVALID, "NULL argument");
    *fov = s->fov;
    std::memcpy(cam, s->cam, sizeof(s->cam));
    return RT_OK;
}

int rth_scene_stats_get(const rth_scene* s, rth_scene_stats* o)
{
    if (!s || !o) return fail(RT_E_INVALID, "NULL argument");
    o->scene_id = s->id;
    o->num_vertices = uint32_t(s->verts.size());
    o->num_triangles = uint32_t(s->tris.size());
    o->num_cells = uint32_t(s->off.size() - 1);
    o->num_refs = uint32_t(s->refs.size());
    o->max_refs_per_cell = 0;
    o->empty_cells = 0;
    for (size_t c = 0; c + 1 < s->off.size(); c++)
    {
        const uint32_t n = s->off[c + 1] - s->off[c];
        o->max_refs_per_cell = std::max(o->max_refs_per_cell, n);
        o->empty_cells += n == 0;
    }
    o->grid_build_s = s->build_s;
    return RT_OK;
}

int rth_framebuffer_create(rt_scene* gpu, const rth_scene* host, uint32_t nthreads, rth_framebuffer** out)
{
    if (!gpu || !host || !out) return fail(RT_E_INVALID, "NULL argument");
    std::unique_ptr<rth_framebuffer> fb(new rth_framebuffer());
    fb->r.reset(new GpuRenderer(gpu, host, nthreads));
    *out = fb.release();
    return RT_OK;
}

int rth_framebuffer_create_multi(const rth_scene* host, const int* devices, uint32_t ndevices, uint32_t nthreads,
                                 rth_framebuffer** out)
{
    if (!host || !devices || !out || ndevices == 0 || ndevices > kMaxRanks)
        return fail(RT_E_INVALID, "bad arguments (1 <= ndevices <= 64)");
    *out = nullptr;
    std::unique_ptr<MultiGpuRenderer> m(new MultiGpuRenderer(host, nthreads));
    const int rc = m->Init(host, devices, ndevices);
    if (rc) return fail(rc, m->InitError());
    std::unique_ptr<rth_framebuffer> fb(new rth_framebuffer());
    fb->multi = m.get();
    fb->r.reset(m.release());
    *out = fb.release();
    return RT_OK;
}

int rth_framebuffer_transport(const rth_framebuffer* fb, uint32_t* transport, uint32_t* nranks)
{
    if (!fb || !transport || !nranks) return fail(RT_E_INVALID, "NULL argument");
    *transport = fb->multi ? fb->multi->Transport() : RTH_TRANSPORT_NONE;
    *nranks = fb->multi ? fb->multi->Ranks() : 1u;
    return RT_OK;
}

void rth_framebuffer_free(rth_framebuffer* fb) { delete fb; }

int rth_framebuffer_set_sample_count(rth_framebuffer* fb, uint32_t spp)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    fb->r->SetSampleCount(spp);
    return RT_OK;
}

int rth_framebuffer_set_options(rth_framebuffer* fb, uint32_t tri_test, uint32_t kernel)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    fb->r->SetOptions(tri_test, kernel);
    return RT_OK;
}

int rth_framebuffer_set_intersector(rth_framebuffer* fb, uint32_t intersector)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    if (intersector > RT_ISECT_RAY_MARCH) return fail(RT_E_INVALID, "unknown intersector");
    fb->r->SetIntersector(intersector);
    return RT_OK;
}

static int finish_frame(rth_framebuffer* fb, double* seconds)
{
    fb->r->Wait();
    if (seconds) *seconds = fb->r->LastFrameSeconds();
    if (fb->r->LastStatus() != RT_OK) return fail(fb->r->LastStatus(), fb->r->LastError());
    return RT_OK;
}

int rth_framebuffer_resize(rth_framebuffer* fb, uint32_t w, uint32_t h, double* seconds)
{
    if (!fb || w == 0 || h == 0) return fail(RT_E_INVALID, "bad arguments");
    fb->r->Resize(w, h);
    return finish_frame(fb, seconds);
}

int rth_framebuffer_start_rendering(rth_framebuffer* fb, double* seconds)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    fb->r->StartRendering();
    return finish_frame(fb, seconds);
}

int rth_framebuffer_start_rendering_async(rth_framebuffer* fb)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    fb->r->StartRenderingAsync();
    return fb->r->LastStatus() != RT_OK ? fail(fb->r->LastStatus(), fb->r->LastError()) : RT_OK;
}

int rth_framebuffer_draw(rth_framebuffer* fb, uint32_t* display, uint32_t* tiles_updated, uint32_t* tiles_done)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    const uint32_t u = fb->r->Draw(display, tiles_done);
    if (tiles_updated) *tiles_updated = u;
    return RT_OK;
}

int rth_framebuffer_wait(rth_framebuffer* fb, double* seconds)
{
    if (!fb) return fail(RT_E_INVALID, "NULL argument");
    return finish_frame(fb, seconds);
}

int rth_framebuffer_read(const rth_framebuffer* fb, uint32_t* out)
{
    if (!fb || !out) return fail(RT_E_INVALID, "NULL argument");
    if (const uint32_t* whole = fb->r->CompleteFrame())
        std::memcpy(out, whole, size_t(fb->r->Width()) * fb->r->Height() * 4);
    else
        fb->r->Assemble(out);
    return RT_OK;
}

// bmp_writer.cpp:7-57: packed 54-byte header, 32 bpp, positive height (bottom-up rows)
int rth_framebuffer_save_bmp(const rth_framebuffer* fb, const char* path)
{
    if (!fb || !path) return fail(RT_E_INVALID, "NULL argument");
    const uint32_t w = fb->r->Width(), h = fb->r->Height();
    // a complete frame is written straight from the page-locked frame; otherwise the tiles are
    // assembled as SaveToBMP does (tiles never rendered stay as they are)
    std::vector<uint32_t> img;
    const uint32_t* src = fb->r->CompleteFrame();
    if (!src)
    {
        img.resize(size_t(w) * h);
        fb->r->Assemble(img.data());
        src = img.data();
    }
    unsigned char hdr[54];
    std::memset(hdr, 0, sizeof(hdr));
    auto put16 = [&](int o, uint32_t v) { hdr[o] = v & 255; hdr[o + 1] = (v >> 8) & 255; };
    auto put32 = [&](int o, uint32_t v) { put16(o, v & 0xFFFF); put16(o + 2, v >> 16); };
    hdr[0] = 'B';
    hdr[1] = 'M';
    put32(2, 54 + w * h * 4);   // size_file
    put32(10, 54);              // offs_bits
    put32(14, 40);              // bmih_size
    put32(18, w);
    put32(22, h);
    put16(26, 1);               // planes
    put16(28, 32);              // bitcount
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_E_INVALID, std::string("cannot write ") + path);
    const size_t n = size_t(w) * h;
    const bool ok = std::fwrite(hdr, 1, 54, f) == 54 && std::fwrite(src, 4, n, f) == n;
    std::fclose(f);
    return ok ? RT_OK : fail(RT_E_INVALID, "short write");
}

} // extern "C"
