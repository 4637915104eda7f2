// rt_tracer.hip -- the host side of librt_tracer.so (C ABI, include/rt_tracer.h): scene upload
// (rt_scene_create), per-frame tables, the render launches (single frames, shards, batched steps,
// records) and the copy-back entry points of the drop-in.  The kernels are in rt_kernels.hip (per-
// sample code in rt_walk.h), the heavy-first planner in rt_plan.hip; rt_kparams.h is what they share.
//
// Scene layout in HBM (built once by rt_scene_create):
//   cellw     u32[C]              packed cell word in GridIdx order (grid.h:41-42): non-empty
//                                 start << 11 | count, empty: L-inf distance to geometry << 11
//   cellwo    u32[8][C]           the same per ray octant: an empty cell holds the side of the
//                                 largest empty cube extending along the octant
//   cellwb    u32[24][C]          box-run words per octant x major axis (rt_box_words.h)
//   cell_off  u32[C+1]            CSR offsets (scenes whose lists do not fit the packed word)
//   refs      float4[3*R]         one 48-B record per CSR reference, in CSR order:
//                                 {v0.xyz, e1.x} {e1.yz, e2.xy} {e2.z, tri_idx bits, 0, 0}
//   frefs     float4[4*R]         per camera origin (k_origin_pre), one 64-B record per CSR
//                                 reference: the origin-only terms of triangle.h:82-98
//   shade     float4[3*T]         per triangle the 3 vertex normals (shading of a hit)
//   face_n    float4[T]           face normal (IntersectRayTriBarycentric only)

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rt_tracer.h"
#include "rt_device.h"
#include "rt_internal.h"
#include "rt_box_words.h"
#include "rt_scene.h"

using namespace rtk;

namespace {
// RT_HOST_TRACE=1: the host time of a render call's phases, printed to stderr per call (a new frame
// shape's first call waits for the host; this names what it waits for)
struct HostTrace
{
    bool on = std::getenv("RT_HOST_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0;
    char buf[512];
    int len = 0;
    void start() { if (on) { t0 = std::chrono::steady_clock::now(); len = 0; } }
    void mark(const char *what)
    {
        if (!on || len > 400) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        len += std::snprintf(buf + len, sizeof(buf) - size_t(len), " %s %.1f", what, us);
    }
    void end() { if (on) std::fprintf(stderr, "rt_host_trace:%s\n", buf); }
};
HostTrace g_ht;

// a new shared event (rt_scene::ev_last and its sources)
int new_event(rtk::EvRef& r, unsigned flags)
{
    rtk::EvRef n = std::make_shared<rtk::EvHolder>();
    RT_HIP(hipEventCreateWithFlags(&n->ev, flags));
    r = std::move(n);
    return RT_OK;
}

// A stop event for the scene's next untimed launch: one of ev_done[] that no scene still holds as its
// ev_last / ev_prev (re-recording a held one would make that scene wait for this launch instead of
// its own), else a new one in a slot
int free_done_event(rt_scene *s, rtk::EvRef& out)
{
    for (rtk::EvRef& e : s->ev_done)
        if (e && e.use_count() == 1)
        {
            out = e;
            return RT_OK;
        }
    rtk::EvRef& slot = s->ev_done[0];
    if (int rc = new_event(slot, s->ev_time_flags)) return rc;
    out = slot;
    return RT_OK;
}


thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

// sampling.h:113-120, sampling.cpp:194-210 (base 2), renderer.cpp:52-55
void hammersley(uint32_t spp, std::vector<float>& xy)
{
    xy.resize(size_t(spp) * 2);
    for (uint32_t s = 0; s < spp; s++)
    {
        double val = 0.0, inv_i = 0.5;
        for (uint32_t n = s; n > 0; n /= 2)
        {
            val += (n % 2) * inv_i;
            inv_i *= 0.5;
        }
        xy[2 * s + 0] = float(double(s) / double(spp) - 0.5f);
        xy[2 * s + 1] = float(val - 0.5f);
    }
}

bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }

uint32_t log2u(uint32_t x)
{
    uint32_t r = 0;
    while ((1u << r) < x) r++;
    return r;
}

// Dot (lin_alg.h:138-144), accumulating from T() = 0
float dot_ref(const float *a, const float *b)
{
    float r = 0.0f;
    r += a[0] * b[0];
    r += a[1] * b[1];
    r += a[2] * b[2];
    return r;
}

// Distance record of one triangle (layout: rtd::dist_point_tri); the position-independent
// terms of ComputeBarycentric / LineSegMinDistSq (triangle.h:140-150, 166-167)
void dist_record(const float *p0, const float *p1, const float *p2, float4 *r)
{
    const float e0[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };
    const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };
    const float e12[3] = { p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2] };
    const float d00 = dot_ref(e0, e0), d01 = dot_ref(e0, e1), d11 = dot_ref(e1, e1);
    const float inv_denom = 1 / (d00 * d11 - d01 * d01);
    r[0] = make_float4(p0[0], p0[1], p0[2], p1[0]);
    r[1] = make_float4(p1[1], p1[2], p2[0], p2[1]);
    r[2] = make_float4(p2[2], e0[0], e0[1], e0[2]);
    r[3] = make_float4(e1[0], e1[1], e1[2], e12[0]);
    r[4] = make_float4(e12[1], e12[2], d00, d01);
    r[5] = make_float4(d11, inv_denom, dot_ref(e12, e12), 0.0f);
}

// AUTO's packed counts + empty-run loop: dims <= 512 and (box-run build) the box words exist
bool auto_runs(const rt_scene *s)
{
    return s->pack_ok && s->box_words;
}

int ensure_device(const rt_scene *s)
{
    int cur = -1;
    RT_HIP(hipGetDevice(&cur));
    if (cur != s->device) RT_HIP(hipSetDevice(s->device));
    return RT_OK;
}

// Uploads the frame's sample table if it differs from the cached one.
// The scene's per-frame constants that live in device memory are rewritten only after its last
// launch has finished with them (launches are asynchronous; the copies are not stream-ordered).
int wait_scene_idle(rt_scene *s)
{
    if (s->ev_recorded) RT_HIP(hipEventSynchronize(s->ev_last->ev));
    if (s->ev_prev) RT_HIP(hipEventSynchronize(s->ev_prev->ev));
    s->ev_prev.reset();
    return RT_OK;
}

// st waits for e -- unless e has already completed (a stream wait enqueues a packet that idles the
// chip for a few us even then)
hipError_t wait_unless_done(hipStream_t st, hipEvent_t e)
{
    return hipEventQuery(e) == hipSuccess ? hipSuccess : hipStreamWaitEvent(st, e, 0);
}

// Orders stream st after every launch of scene s that may still run: the last one (ev_last, implicit
// on its own stream) and, when that one overlapped its predecessor (RT_KERNEL_FLAG_OVERLAP), the
// predecessor (ev_prev).  The caller's next launch on st then follows them all.
// The last launch becomes the "launch two back" of the next one: an overlapped launch after this one
// on a third stream is ordered by nothing else.
int order_all(rt_scene *s, hipStream_t st)
{
    if (!s->ev_recorded) return RT_OK;
    if (st != s->last_stream) RT_HIP(wait_unless_done(st, s->ev_last->ev));
    if (s->ev_prev && s->prev_stream != st) RT_HIP(wait_unless_done(st, s->ev_prev->ev));
    s->ev_prev = s->ev_last;
    s->prev_stream = s->last_stream;
    return RT_OK;
}

// An overlapped launch on st (RT_KERNEL_FLAG_OVERLAP): it may run beside the scene's last launch, but
// after the one before that (at most two in flight)
int order_overlap(rt_scene *s, hipStream_t st)
{
    if (s->ev_prev && s->prev_stream != st) RT_HIP(wait_unless_done(st, s->ev_prev->ev));
    s->ev_prev = s->ev_last;
    s->prev_stream = s->last_stream;
    return RT_OK;
}

// camera.h:41-42 fov_xs = (float)tan(double(DegToRad(fov) / 2)) (H5), computed on the host
float fov_xs_of(const rt_frame *f)
{
    const float hfov = f->fov * float(0.0174532925);           // lin_alg.h:232 DegToRad
    return float(::tan(double(hfov / 2.0f)));
}

// Camera-space x per (column, sample) and y per (row, sample) of GenerateRay (camera.h:20-21,
// 40-42): the only parts of a ray's direction that depend on the pixel and the sample offsets
// alone, computed here with the kernels' own operations (rtd::cam_x / cam_y: IEEE float on the
// host too, no contraction) and uploaded when the frame shape changes.  tbl = the sample table.
std::vector<float> ndc_key(const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    std::vector<float> key = { float(f->width), float(f->height), float(spp), fov_xs_of(f),
                               float(f->width) / float(f->height) };
    key.insert(key.end(), tbl.begin(), tbl.end());
    return key;
}

// the sample table of a frame (rt_frame.sample_offsets, or the Hammersley table)
std::vector<float> sample_table(const rt_frame *f, uint32_t spp)
{
    std::vector<float> tbl;
    if (f->sample_offsets)
        tbl.assign(f->sample_offsets, f->sample_offsets + 2 * size_t(spp));
    else
        hammersley(spp, tbl);
    return tbl;
}

// The frame tables of prepare_samples' device path, written on stream st after every launch that
// may still read the old ones (st's own, and the scene's last launch on another stream: ev1).
int flush_tables(rt_scene *s, hipStream_t st)
{
    if (!s->tab_dirty) return RT_OK;
    if (int rc = order_all(s, st)) return rc;
    const uint32_t n = (s->tab.W + s->tab.H) * s->tab.spp;
    hipLaunchKernelGGL(frame_tables_kernel(), dim3((n + kWG - 1) / kWG), dim3(kWG), 0, st, s->d_ndc, s->d_smp, s->tab);
    RT_HIP(hipGetLastError());
    s->tab_dirty = false;
    return RT_OK;
}

int prepare_ndc(rt_scene *s, const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    const float fx = fov_xs_of(f), aspect = float(f->width) / float(f->height);
    std::vector<float> key = ndc_key(f, spp, tbl);
    if (key == s->ndc_key) return RT_OK;
    const size_t n = (size_t(f->width) + f->height) * spp;
    std::vector<float> h(n);
    for (uint32_t x = 0; x < f->width; x++)
        for (uint32_t k = 0; k < spp; k++) h[size_t(x) * spp + k] = rtd::cam_x(x, tbl[2 * k], f->width, fx);
    float *hy = h.data() + size_t(f->width) * spp;
    for (uint32_t y = 0; y < f->height; y++)
        for (uint32_t k = 0; k < spp; k++) hy[size_t(y) * spp + k] = rtd::cam_y(y, tbl[2 * k + 1], f->height, fx, aspect);
    if (int rc = wait_scene_idle(s)) return rc;
    if (n > s->ndc_cap)
    {
        if (s->d_ndc) RT_HIP(hipFree(s->d_ndc));
        s->d_ndc = nullptr;
        s->ndc_cap = 0;
        RT_HIP(hipMalloc(&s->d_ndc, n * sizeof(float)));
        s->ndc_cap = n;
    }
    RT_HIP(hipMemcpy(s->d_ndc, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    s->ndc_key = key;
    s->ndc_w = f->width;
    s->ndc_spp = spp;
    return RT_OK;
}

int remember_tables(rt_scene *s, const rt_frame *f, uint32_t spp, const std::vector<float>& tbl)
{
    s->fp_w = f->width;
    s->fp_h = f->height;
    s->fp_spp = spp;
    std::memcpy(&s->fp_fov, &f->fov, 4);
    s->fp_custom = f->sample_offsets != nullptr;
    s->fp_tbl = tbl;
    s->fp_valid = true;
    return RT_OK;
}

// true when the scene's camera-space and sample tables are those of this frame (no host work)
bool tables_match(const rt_scene *s, const rt_frame *f, uint32_t spp)
{
    uint32_t fov;
    std::memcpy(&fov, &f->fov, 4);
    if (!s->fp_valid || s->fp_w != f->width || s->fp_h != f->height || s->fp_spp != spp || s->fp_fov != fov ||
        s->fp_custom != (f->sample_offsets != nullptr))
        return false;
    return !f->sample_offsets || std::memcmp(s->fp_tbl.data(), f->sample_offsets, sizeof(float) * 2 * spp) == 0;
}

int prepare_samples(rt_scene *s, const rt_frame *f, uint32_t spp)
{
    if (tables_match(s, f, spp)) return RT_OK;
    s->fp_valid = false;
    const std::vector<float> tbl = sample_table(f, spp);
    const size_t n = (size_t(f->width) + f->height) * spp;
    if (spp <= kTabMaxSpp && n <= s->ndc_cap)
    {
        // the tables are written on the device, in stream order before the frame's launch
        // (flush_tables): a new frame shape costs no host wait and no synchronous copy
        std::vector<float> key = ndc_key(f, spp, tbl);
        if (key != s->ndc_key || tbl != s->smp_host)
        {
            s->tab.fx = fov_xs_of(f);
            s->tab.aspect = float(f->width) / float(f->height);
            s->tab.W = f->width;
            s->tab.H = f->height;
            s->tab.spp = spp;
            std::memcpy(s->tab.smp, tbl.data(), tbl.size() * sizeof(float));
            s->tab_dirty = true;
            s->ndc_key = key;
            s->ndc_w = f->width;
            s->ndc_spp = spp;
            s->smp_host = tbl;
        }
        return remember_tables(s, f, spp, tbl);
    }
    s->tab_dirty = false;           // a pending device write is superseded (its key differs: spp)
    if (int rc = prepare_ndc(s, f, spp, tbl)) return rc;
    if (tbl == s->smp_host) return remember_tables(s, f, spp, tbl);
    if (int rc = wait_scene_idle(s)) return rc;
    if (spp > s->smp_cap)
    {
        if (s->d_smp) RT_HIP(hipFree(s->d_smp));
        if (s->h_smp_pinned) RT_HIP(hipHostFree(s->h_smp_pinned));
        s->d_smp = nullptr;
        s->h_smp_pinned = nullptr;
        const uint32_t cap = std::max<uint32_t>(64, spp);
        RT_HIP(hipMalloc(&s->d_smp, sizeof(float2) * cap));
        RT_HIP(hipHostMalloc(&s->h_smp_pinned, sizeof(float2) * cap));
        s->smp_cap = cap;
    }
    std::memcpy(s->h_smp_pinned, tbl.data(), tbl.size() * sizeof(float));
    RT_HIP(hipMemcpy(s->d_smp, s->h_smp_pinned, tbl.size() * sizeof(float), hipMemcpyHostToDevice));
    s->smp_host = tbl;
    return remember_tables(s, f, spp, tbl);
}

constexpr uint32_t kKernelFlags = RT_KERNEL_FLAG_WIDE_HEAVY | RT_KERNEL_FLAG_EXHAUSTIVE |
                                  RT_KERNEL_FLAG_WAVE_CLOCK | RT_KERNEL_FLAG_OVERLAP | RT_KERNEL_BUDGET_MASK;

int validate_frame(const rt_frame *f)
{
    if (!f) return fail(RT_E_INVALID, "frame is NULL");
    if (f->width == 0 || f->height == 0 || f->width > 65536 || f->height > 65536)
        return fail(RT_E_INVALID, "frame width/height must be in [1, 65536]");
    if (f->tri_test > RT_TRI_BARYCENTRIC) return fail(RT_E_INVALID, "unknown tri_test");
    if (f->intersector > RT_ISECT_RAY_MARCH) return fail(RT_E_INVALID, "unknown intersector");
    if (f->intersector == RT_ISECT_BRUTE_FORCE && f->tri_test != RT_TRI_MOLLER_TRUMBORE)
        return fail(RT_E_INVALID, "IntersectBruteForce uses IntersectRayTri only (renderer.cpp:176)");
    const uint32_t kind = f->kernel & RT_KERNEL_KIND_MASK;
    if (kind > RT_KERNEL_COMPACT || (f->kernel & ~(RT_KERNEL_KIND_MASK | kKernelFlags)))
        return fail(RT_E_INVALID, "unknown or removed kernel kind / flag");
    const uint32_t spp = std::max(1u, f->spp);
    if (spp > 4096) return fail(RT_E_INVALID, "spp must be <= 4096");
    if (kind == RT_KERNEL_COMPACT && ((f->kernel & RT_KERNEL_BUDGET_MASK) >> RT_KERNEL_BUDGET_SHIFT) > 64u)
        return fail(RT_E_INVALID, "compaction refill threshold must be <= 64 lanes");
    if ((kind == RT_KERNEL_LANES || kind == RT_KERNEL_COMPACT) && !(is_pow2(spp) && spp <= 64))
        return fail(RT_E_INVALID, "RT_KERNEL_LANES needs spp to be a power of two <= 64");
    return RT_OK;
}

// Fills the per-frame parameters (camera constants exactly as camera.h computes them).
void frame_params(const rt_scene *s, const rt_frame *f, KParams& P)
{
    std::memset(&P, 0, sizeof(P));
    const float (*c)[4] = reinterpret_cast<const float (*)[4]>(f->cam);
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++) P.m[3 * r + k] = c[r][k];
    P.fov_xs = fov_xs_of(f);                                    // camera.h:42, double tan (H5)
    P.aspect = float(f->width) / float(f->height);
    P.ndcx = s->d_ndc;                                          // prepare_ndc (this frame's shape)
    P.ndcy = s->d_ndc + size_t(s->ndc_w) * s->ndc_spp;
    for (int k = 0; k < 3; k++)                                 // lin_alg.h:518-535
        P.org[k] = 0.0f * c[0][k] + 0.0f * c[1][k] + 0.0f * c[2][k] + c[3][k];
    P.W = f->width;
    P.H = f->height;
    P.spp = std::max(1u, f->spp);
    P.spp_shift = is_pow2(P.spp) ? log2u(P.spp) : 0;
    P.inv_spp = is_pow2(P.spp) ? 1.0f / float(P.spp) : 0.0f;
    P.smp = s->d_smp;
    for (int a = 0; a < 3; a++)
    {
        P.bmin[a] = s->bmin[a];
        P.bmax[a] = s->bmax[a];
        P.dim[a] = int(s->dims[a]);
    }
    P.cw = s->cw;
    P.icw = s->icw;
    P.dxdz = int(s->dims[0] * s->dims[2]);
    P.max_steps = s->dims[0] + s->dims[1] + s->dims[2] + 3;
    P.off = s->d_off;
    P.cellw = s->d_cellw;
    P.cellwo = s->d_cellwo ? s->d_cellwo : s->d_cellw;
    P.oct_stride = s->d_cellwo ? s->oct_stride : 0u;
    P.cellwb = s->d_cellwb;
    P.box_stride = s->box_stride;
    P.refs = s->d_refs;
    P.frefs = s->d_frefs[0];                                    // ensure_origin_terms picks the buffer
    P.shade = s->d_shade;
    P.face_n = s->d_facen;
    P.tri_mt = s->d_trimt;
    P.tri_dist = s->d_tridist;
    P.dist_blk = s->d_distblk;
    P.ndist_blk = s->ndist_blk;
    P.scene_scale = s->scene_scale;
    for (int a = 0; a < 3; a++)
    {
        P.smin[a] = s->vmin[a];
        P.smax[a] = s->vmax[a];
    }
    P.ntris = s->ntris;
    P.tri_test = f->tri_test;
    P.isect = f->intersector;
}

bool use_lanes(const rt_frame *f, uint32_t spp)
{
    if ((f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_PIXEL_LOOP) return false;
    return is_pow2(spp) && spp <= 64;
}

// The per-reference origin terms for this frame's camera origin: computed when the origin
// differs from the one the records hold (a moving camera pays one small launch per frame).
// One tunable from the environment (rt_scene_create only).
uint32_t env_tunable(const char *name, uint32_t dflt)
{
    const char *e = std::getenv(name);
    return e && *e ? uint32_t(std::strtoul(e, nullptr, 0)) : dflt;
}

// The per-origin record buffer a frame of origin `org` reads (rt_scene::d_frefs): the one holding that
// origin, else the one to compute it into -- never one the scene's last launch reads (mask `busy`, bit b:
// buffer b), preferring an empty one.  -1: both are busy (a batch that read two origins of the scene).
int fref_slot(const rt_scene *s, const float org[3], uint32_t busy, bool *compute)
{
    uint32_t ob[3];
    std::memcpy(ob, org, sizeof(ob));
    for (int b = 0; b < 2; b++)
        if (s->fref_ok[b] && std::memcmp(ob, s->fref_org[b], sizeof(ob)) == 0)
        {
            *compute = false;
            return b;
        }
    *compute = true;
    for (int b = 0; b < 2; b++)
        if (!(busy & (1u << b)) && !s->fref_ok[b]) return b;
    for (int b = 0; b < 2; b++)
        if (!(busy & (1u << b))) return b;
    return -1;
}

// A frame of this origin may overlap the scene's last launch (RT_KERNEL_FLAG_OVERLAP) as far as the
// per-origin records go: its origin is computed, or the buffer it would be computed into is one the last
// launch does not read.
bool fref_overlap_ok(const rt_scene *s, const float org[3])
{
    bool compute;
    return fref_slot(s, org, s->fref_last, &compute) >= 0;
}

// The per-reference origin terms for this frame's camera origin in a buffer of their own (fref_slot),
// computed when neither buffer holds them (a moving camera pays one small launch per frame), ordered after
// every launch that may still read that buffer (the caller has ordered st after the launch before the
// last one, which is the only other one in flight; busy: buffers that launches of this call read already).
// Sets P.frefs and marks the buffer in *used.
int ensure_origin_terms(rt_scene *s, KParams& P, hipStream_t st, uint32_t busy, uint32_t *used)
{
    bool compute = false;
    const int b = fref_slot(s, P.org, s->fref_last | busy, &compute);
    if (b < 0) return fail(RT_E_INVALID, "internal: no free per-origin record buffer");
    if (compute)
    {
        if (s->nrefs)
            hipLaunchKernelGGL(origin_pre_kernel(), dim3((s->nrefs + kWG - 1) / kWG), dim3(kWG), 0, st, s->d_refs,
                               s->d_frefs[b], s->nrefs, P.org[0], P.org[1], P.org[2]);
        RT_HIP(hipGetLastError());
        std::memcpy(s->fref_org[b], P.org, sizeof(s->fref_org[b]));
        s->fref_ok[b] = true;
    }
    P.frefs = s->d_frefs[b];
    *used |= 1u << b;
    return RT_OK;
}

// AUTO's own choice of the wide section for a single-frame launch: a shard of >= 2 ranks of a scene
// with dense cells
bool auto_wide(const rt_scene *s, const KParams& P)
{
    return P.nranks >= 2u && s->max_cell_refs >= s->wh_auto_refs;
}

// Launches the render kernel over region/shard described by P (tiles_x, rank, ...).
int launch_render(rt_scene *s, const rt_frame *f, KParams& P, uint32_t n_local_tiles, hipStream_t st,
                  bool order_streams = true)
{
    if (n_local_tiles == 0) return RT_OK;
    const bool lanes = use_lanes(f, P.spp);
    P.wg_per_tile = lanes ? (kTilePix * P.spp) / kWG : 1;
    if (P.wg_per_tile == 0) P.wg_per_tile = 1;
    const uint64_t blocks = uint64_t(n_local_tiles) * P.wg_per_tile;
    if (blocks > 0x3FFFFFFFull) return fail(RT_E_INVALID, "frame too large for one launch");
    const uint32_t kind = f->kernel & RT_KERNEL_KIND_MASK;
    const bool bary = P.tri_test == RT_TRI_BARYCENTRIC;
    const bool grid_mt = P.isect == RT_ISECT_GRID && !bary;
    // The per-camera records (frefs) are scene state: a launch on another stream than the last
    // one waits for it -- unless the caller allows overlap (RT_KERNEL_FLAG_OVERLAP) and nothing the
    // two launches share changes between them (as launch_batch): AUTO's lane kernel (not the wide
    // section's side-stream pair, not the wave clocks), the same tables and camera origin, and an
    // existing launch shape whose frame is not measured.
    // (order_streams false: the caller orders its streams itself, rt_render_frame_host_tiled)
    // No overlap inside a stream capture: plans there run on the launch stream (launch_plans).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    bool overlap = false;
    if (order_streams && cap == hipStreamCaptureStatusNone && (f->kernel & RT_KERNEL_FLAG_OVERLAP) && s->ev_recorded &&
        st != s->last_stream &&
        kind == RT_KERNEL_AUTO && lanes && grid_mt && !(f->kernel & (RT_KERNEL_FLAG_WAVE_CLOCK | RT_KERNEL_FLAG_WIDE_HEAVY)) &&
        !auto_wide(s, P) && P.spp <= 64u && !s->tab_dirty)
    {
        overlap = fref_overlap_ok(s, P.org);
        const int v = kVarAutoCore | (s->rcp_safe ? kVarFastRcp : 0) | (auto_runs(s) ? kVarPackedRem | kVarSkipRun : 0);
        if (overlap && blocks >= s->hf_min_blocks)
        {
            const HfPeek pk = hf_peek(s, P, blocks, v, 0u, cam_signature(P));
            overlap = pk.found && (!pk.measure || pk.measure_ok);
        }
    }
    if (overlap)
    {
        if (int rc = order_overlap(s, st)) return rc;
    }
    else if (order_streams)
        if (int rc = order_all(s, st)) return rc;
    if (int rc = flush_tables(s, st)) return rc;
    g_ht.mark("tables");
    s->last_stream = st;
    // kVarXcdBands turn size: one row of this launch's tiles (ceil(tiles_x / nranks) local tiles
    // span a full frame row in shard mode).  Measured best of 1/4 .. 4 rows and 1..16 tiles:
    // whole rows interleave over the XCDs, so each L2 sees compact rows AND the frame's cost
    // spreads evenly (half rows put every left half on the even XCDs).
    P.xcd_chunk = ((P.tiles_x + P.nranks - 1u) / P.nranks) * P.wg_per_tile;
    // AUTO (and the COMPACT arm built on its per-ray code): the feature set of kVarAuto that this
    // scene allows -- the Newton reciprocal needs rcp_safe, the packed counts and the empty-run
    // loop need pack_ok.  DESIGN.md §4.1 has the measured progression.
    const bool auto_path = lanes && grid_mt && (kind == RT_KERNEL_AUTO || kind == RT_KERNEL_COMPACT);
    int var = 0;
    if (auto_path)
    {
        var = kVarAutoCore | (s->rcp_safe ? kVarFastRcp : 0) | (auto_runs(s) ? kVarPackedRem | kVarSkipRun : 0) |
              ((f->kernel & RT_KERNEL_FLAG_WAVE_CLOCK) ? kVarWaveClock : 0);
        uint32_t used = 0;
        if (int rc = ensure_origin_terms(s, P, st, 0u, &used)) return rc;
        s->fref_last = used;
        g_ht.mark("origin");
    }
    else
        s->fref_last = 0u;                      // (this launch reads no per-origin records)
    if (auto_path)
        ;
    else if (lanes && P.isect == RT_ISECT_RAY_MARCH)
        var = kVarMarch | ((f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE) ? kVarExhaustive : 0);
    else if (lanes && P.isect == RT_ISECT_BRUTE_FORCE)
        var = kVarBrute;
    // kernel-time events only outside stream capture (a captured record has no time to read)
    // A timed event pair costs ~10 us of device time per launch (measured: bench step 0.755 ->
    // 0.736 ms without), so only every time_every-th launch is timed (rt_scene_set_timing)
    const bool timed = cap == hipStreamCaptureStatusNone && s->time_every && s->launches % s->time_every == 0u;
    s->launches++;
    const uint32_t kslot = s->kt_next;
    hipEvent_t kt0 = nullptr, kt1 = nullptr;        // null stand for "not timed"
    if (timed && !s->kt0[kslot]) RT_HIP(hipEventCreateWithFlags(&s->kt0[kslot], s->ev_time_flags));
    // a ring slot's stop event still marking another scene's last launch is left to it
    if (timed && (!s->kt1[kslot] || s->kt1[kslot].use_count() > 1))
        if (int rc = new_event(s->kt1[kslot], s->ev_time_flags)) return rc;
    if (timed)
    {
        kt0 = s->kt0[kslot];
        kt1 = s->kt1[kslot]->ev;
    }
    bool stop_done = false;             // the launch carried its own stop event (ev_last set)
    auto mark = [&](hipEvent_t e) { return e ? hipEventRecord(e, st) : hipSuccess; };
    if (var & kVarWaveClock)
    {
        const size_t need = size_t(blocks) * kWavesPerWG * 4u;
        if (need > s->clk_cap)
        {
            if (s->d_clk) RT_HIP(hipFree(s->d_clk));
            s->d_clk = nullptr;
            RT_HIP(hipMalloc(&s->d_clk, need * sizeof(uint64_t)));
            s->clk_cap = need;
        }
        s->clk_items = uint32_t(need / 4u);
        P.wave_clk = s->d_clk;
    }
    const dim3 wg(kWG);
    const uint32_t budget = (f->kernel & RT_KERNEL_BUDGET_MASK) >> RT_KERNEL_BUDGET_SHIFT;
    // AUTO takes the wide section (kVarWideHeavy: AUTO's full record/count layout, spp <= 16) for
    // a shard of >= 2 ranks of a scene with dense cells: there a rank's launch is bound by its few
    // ~1000-test waves, which the section splits 16 ways (4 for spp 8-16) beside the lane kernel
    // (measured, tools/wh_probe.py, killeroo rank of 2 / 4 / 8: 0.36 / 0.33 / 0.25 ms with the
    // two-phase arm it replaced -> 0.35 / 0.20 / 0.15).  On a whole frame the
    // lanes are busy with other items anyway and the section's repeated walks cost more than they
    // save (+1-3 %).
    const bool wide_ok = auto_path && var == kVarAuto && P.spp <= 16u;
    const bool wide_heavy = wide_ok && kind == RT_KERNEL_AUTO &&
                            ((f->kernel & RT_KERNEL_FLAG_WIDE_HEAVY) || auto_wide(s, P));
    if (lanes && kind == RT_KERNEL_COMPACT && P.isect == RT_ISECT_GRID)
    {
        const uint32_t n_items = uint32_t(blocks * kWavesPerWG);
        const uint32_t refill = budget ? budget : kCompactRefill;
        const dim3 grid(std::max(1u, std::min(s->compact_wgs, (n_items + 3u) / 4u)));
        RT_HIP(mark(kt0));
        // bary: the plain distance-skip walk; AUTO's box-run walk where the scene allows it
        const kcfn_t cfn = bary ? compact_kernel(RT_TRI_BARYCENTRIC, kVarDistSkip)
                           : (auto_runs(s) && s->rcp_safe)
                               ? compact_kernel(RT_TRI_MOLLER_TRUMBORE, kVarCompactBox)
                               : compact_kernel(RT_TRI_MOLLER_TRUMBORE, kVarWaveGate | kVarDistSkip | kVarOriginPre);
        hipLaunchKernelGGL(cfn, grid, wg, 0, st, P, n_items, refill);
        RT_HIP(mark(kt1));
    }
    else if (lanes)
    {
        // AUTO, LANES, and COMPACT where its layout does not apply
        const int kvar = ((kind == RT_KERNEL_AUTO || P.isect != RT_ISECT_GRID) ? var : 0) |
                         (wide_heavy ? kVarWideHeavy : 0);
        const kfn_t fn = lanes_kernel(bary ? RT_TRI_BARYCENTRIC : RT_TRI_MOLLER_TRUMBORE, kvar);
        if (!fn) return fail(RT_E_INVALID, "kernel variant not built: " + std::to_string(kvar));
        uint32_t grid = uint32_t(blocks);
        // heavy-first order: AUTO grid frames large enough that blocks start in several rounds
        // (and every wide-section launch of >= 64 blocks: its lane kernel's heaviest items)
        const bool front = kind == RT_KERNEL_AUTO && P.isect == RT_ISECT_GRID && !(kvar & kVarWaveClock) &&
                           (blocks >= s->hf_min_blocks || (wide_heavy && blocks >= 64u));
        // the wide section's LDS tier (kVarLdsSplit) per rank count (wh_lds, bit log2 N), without
        // RT_KERNEL_FLAG_OVERLAP (as launch_batch)
        const uint32_t lg_ranks = P.nranks >= 8u ? 3u : (P.nranks >= 4u ? 2u : (P.nranks >= 2u ? 1u : 0u));
        const bool lds = wide_heavy && ((s->wh_lds >> lg_ranks) & 1u) != 0u && !(f->kernel & RT_KERNEL_FLAG_OVERLAP);
        if (front || wide_heavy)
        {
            if (int rc = hf_prepare(s, P, blocks, kvar | (lds ? kVarLdsSplit : 0), front, st)) return rc;
            g_ht.mark("hf_prepare");
            grid += P.hf_front;
        }
        // one-wave workgroups (k_render_lanes_w64): the same blocks, each wave dispatched by itself
        kfn_t lfn = fn;
        uint32_t lgrid = grid, lwg = kWG;
        // (not for a scene with very dense cells: scene 5, a cell of 1,226 references, runs its whole
        // frame 3 % faster in 256-lane workgroups, while killeroo (426) and scene 4 (132) run 4-6 %
        // slower that way: profiles/r05av_wg64_dense.json -- unless the launch may overlap the one before
        // it, whose work fills the tail: config 5 as overlapped frames 2.575 vs 2.607 ms per step,
        // profiles/r06_pipelined_plan_ab.json)
        const bool pipelined = (f->kernel & RT_KERNEL_FLAG_OVERLAP) != 0u;
        if (s->wg64 && kvar == kVarAuto && grid >= s->wg64_min_blocks &&
            (s->max_cell_refs < s->wg64_max_refs || pipelined))
        {
            lfn = lanes_w64_kernel(kVarAuto);
            P.vblocks = grid;
            lgrid = kWavesPerWG * ((grid + kXcds - 1u) / kXcds * kXcds);
            lwg = 64u;
        }
        if (P.wh_wgs)
        {
            RT_HIP(mark(kt0));
            // the wide section runs on the side stream beside the lane kernel (fork / join by
            // events, so the pair also captures into a hipGraph); submitted first so its waves
            // -- the frame's longest -- start first
            if (!s->side)
            {
                RT_HIP(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
                RT_HIP(hipEventCreateWithFlags(&s->ev_fork, s->ev_order_flags));
                RT_HIP(hipEventCreateWithFlags(&s->ev_join, s->ev_order_flags));
            }
            RT_HIP(hipEventRecord(s->ev_fork, st));
            RT_HIP(hipStreamWaitEvent(s->side, s->ev_fork, 0));
            hipLaunchKernelGGL(wide_kernel(P.wh_g, lds), dim3(P.wh_wgs), wg, 0, s->side, P);
        }
        if (P.wh_wgs)
        {
            hipLaunchKernelGGL(lfn, dim3(lgrid), dim3(lwg), 0, st, P);
            RT_HIP(hipEventRecord(s->ev_join, s->side));
            RT_HIP(hipStreamWaitEvent(st, s->ev_join, 0));
            RT_HIP(mark(kt1));
            RT_HIP(hipEventRecord(s->ev_own->ev, st));     // (launch_plans forks after ev_last)
            s->ev_last = s->ev_own;
            stop_done = true;
            s->ev_recorded = true;
        }
        else
        {
            // the dispatch carries its own events (no marker packets): the timed launch's pair, or
            // the scene's completion event alone
            if (timed)
                s->ev_last = s->kt1[kslot];
            else if (int rc = free_done_event(s, s->ev_last))
                return rc;
            hipExtLaunchKernelGGL(lfn, dim3(lgrid), dim3(lwg), 0, st, kt0, s->ev_last->ev, 0u, P);
            stop_done = true;
            s->ev_recorded = true;
        }
        if ((P.hf_front || P.wh_on) && P.hf_measure)
            if (int rc = launch_plans(s, P, blocks, st, pipelined)) return rc;
    }
    else
    {
        RT_HIP(mark(kt0));
        const int pvar = P.isect == RT_ISECT_RAY_MARCH
                             ? kVarMarch | ((f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE) ? kVarExhaustive : 0)
                             : (P.isect == RT_ISECT_BRUTE_FORCE ? kVarBrute : 0);
        hipLaunchKernelGGL(pixel_loop_kernel(bary ? RT_TRI_BARYCENTRIC : RT_TRI_MOLLER_TRUMBORE, pvar),
                           dim3(uint32_t(blocks)), wg, 0, st, P);
        RT_HIP(mark(kt1));
    }
    RT_HIP(hipGetLastError());
    g_ht.mark("launched");
    if (!stop_done)
    {
        RT_HIP(hipEventRecord(s->ev_own->ev, st));
        s->ev_last = s->ev_own;
        s->ev_recorded = true;
    }
    if (timed)
    {
        s->kt_last = kslot;
        s->kt_next = (kslot + 1u) % kTimeRing;
        s->kt_count = std::min(s->kt_count + 1u, kTimeRing);
    }
    return RT_OK;
}


// n frames (2 <= n <= kMaxBatch, scenes on one device, mutexes held by the caller) in ONE launch
// of k_render_batch.  P[i] holds frame i's parameters (frame_params + region + shard + outputs).
// Returns RT_E_INVALID with *batched == false, doing nothing, when the frames cannot share a
// launch (the caller then renders them one launch each).
int launch_batch(rt_scene *const *S, const rt_frame *F, uint32_t n, KParams *P, uint32_t n_local_tiles,
                 hipStream_t st, bool *batched)
{
    *batched = false;
    if (n < 2 || n > kMaxBatch || n_local_tiles == 0) return RT_E_INVALID;
    const uint32_t spp = P[0].spp;
    if (!use_lanes(&F[0], spp) || spp > 16u) return RT_E_INVALID;
    int var = -1;
    bool wide_heavy = false;
    for (uint32_t i = 0; i < n; i++)
    {
        const uint32_t kind = F[i].kernel & RT_KERNEL_KIND_MASK;
        if (kind != RT_KERNEL_AUTO ||
            (F[i].kernel & ~uint32_t(RT_KERNEL_FLAG_WIDE_HEAVY | RT_KERNEL_FLAG_WAVE_CLOCK | RT_KERNEL_FLAG_OVERLAP)) != 0u ||
            (F[i].kernel & RT_KERNEL_FLAG_WAVE_CLOCK) != (F[0].kernel & RT_KERNEL_FLAG_WAVE_CLOCK))
            return RT_E_INVALID;
        if (P[i].isect != RT_ISECT_GRID || P[i].tri_test != RT_TRI_MOLLER_TRUMBORE) return RT_E_INVALID;
        if (P[i].W != P[0].W || P[i].H != P[0].H || P[i].spp != spp || S[i]->device != S[0]->device)
            return RT_E_INVALID;
        const int v = kVarAutoCore | (S[i]->rcp_safe ? kVarFastRcp : 0) |
                      (auto_runs(S[i]) ? kVarPackedRem | kVarSkipRun : 0);
        if (var >= 0 && v != var) return RT_E_INVALID;
        var = v;
        wide_heavy = wide_heavy || (F[i].kernel & RT_KERNEL_FLAG_WIDE_HEAVY) ||
                     (P[i].nranks >= 2u && S[i]->max_cell_refs >= S[0]->wh_auto_refs);
    }
    if (var != kVarAuto) return RT_E_INVALID;
    // the wide section always leads the batch kernel's own grid (measured against its own kernel on a
    // side stream, profiles/r03f_ab_wide_fused.json: 18 % faster at a rank of 8, 9 % at 4; a rank of
    // 2 0.321 ms fused vs 0.338, profiles/r03aa_wg64_wide_fused2_sweep.json; the side-stream arm was
    // removed in round 5)
    const bool fused = wide_heavy;
    const bool clk = (F[0].kernel & RT_KERNEL_FLAG_WAVE_CLOCK) != 0u;
    const uint32_t lg_ranks = P[0].nranks >= 8u ? 3u : (P[0].nranks >= 4u ? 2u : (P[0].nranks >= 2u ? 1u : 0u));
    // the section's LDS tier (kVarLdsSplit) per rank count (wh_lds, bit log2 N), for
    // launches that do not ask to overlap the previous one (RT_KERNEL_FLAG_OVERLAP): there the launch's
    // tail is exposed and the tier shortens it (a rank of 8's step 0.106 -> 0.096 ms), while an
    // overlapped launch's tail is filled by the next one and the tier's 256-lane grid costs more
    // (0.0875 -> 0.090 ms, profiles/r06_lds_tier_ab.json)
    const bool lds = fused && ((S[0]->wh_lds >> lg_ranks) & 1u) != 0u && !(F[0].kernel & RT_KERNEL_FLAG_OVERLAP);
    const int kvar = var | (wide_heavy ? kVarWideHeavy : 0) | (fused ? kVarWideFused : 0) |
                     (fused && spp > 4u ? kVarWideG4 : 0) | (lds ? kVarLdsSplit : 0) |
                     (clk ? kVarWaveClock : 0);
    if (!batch_kernel(kvar, false)) return RT_E_INVALID;
    const uint32_t wgpt = (kTilePix * spp) / kWG;
    const uint64_t fblocks = uint64_t(n_local_tiles) * wgpt;
    const uint64_t blocks = fblocks * n;
    if (blocks > 0x3FFFFFFFull) return RT_E_INVALID;        // one launch per frame (each checks its own size)
    *batched = true;
    KBatch KB;
    std::memset(&KB, 0, sizeof(KB));
    KB.nframes = n;
    for (uint32_t i = 0; i <= n; i++) KB.base[i] = uint32_t(fblocks * i);
    for (uint32_t i = n + 1; i <= kMaxBatch; i++) KB.base[i] = uint32_t(blocks);
    // the batch's heavy-first / wide-section state lives in scene 0's table, keyed by the batch
    uint64_t ident = n;
    for (uint32_t i = 0; i < n; i++) ident = ident * 0x9E3779B97F4A7C15ull + uint64_t(uintptr_t(S[i]));
    rt_scene *s0 = S[0];
    const bool front = blocks >= s0->hf_min_blocks || (wide_heavy && blocks >= 64u);
    uint64_t cams = 0xcbf29ce484222325ull;
    for (uint32_t i = 0; i < n; i++) cams = cam_signature(P[i], cams);
    for (uint32_t i = 0; i < n; i++)
    {
        P[i].wg_per_tile = wgpt;
        P[i].xcd_chunk = ((P[i].tiles_x + P[i].nranks - 1u) / P[i].nranks) * wgpt;
    }
    // RT_KERNEL_FLAG_OVERLAP (every frame of the batch): this launch may run beside the scenes' last
    // launch on another stream -- its tail under this launch's start -- when no scene state changes
    // between them: the frame tables and the per-origin records stay, the batch's heavy-first
    // context exists and this frame is not measured (a measured frame clears and rewrites plan
    // buffers that an older version's frames read), no wave clocks or segmented-tier scratch
    // (per-scene buffers), no stream capture (its plans run on the launch stream).  At most two
    // launches of a scene are in flight: an overlapped launch waits for the one before the launch it
    // overlaps (ev_prev).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    bool overlap = !clk && cap == hipStreamCaptureStatusNone;
    for (uint32_t i = 0; i < n; i++)
    {
        overlap = overlap && (F[i].kernel & RT_KERNEL_FLAG_OVERLAP) && !S[i]->tab_dirty && fref_overlap_ok(S[i], P[i].org);
        // a scene twice in the batch at another origin: both record buffers are this launch's, so it
        // orders after every launch of the scene; more than two origins of one scene: no batch
        uint32_t org_i[3], org_j[3];
        std::memcpy(org_i, P[i].org, sizeof(org_i));
        int others = 0;
        for (uint32_t j = 0; j < i; j++)
        {
            std::memcpy(org_j, P[j].org, sizeof(org_j));
            if (S[j] == S[i] && std::memcmp(org_i, org_j, sizeof(org_i)) != 0) others++;
        }
        if (others) overlap = false;
        if (others > 1) return RT_E_INVALID;
    }
    if (overlap && (front || wide_heavy))
    {
        const HfPeek pk = hf_peek(s0, P[0], blocks, kvar, ident | 1u, cams);
        overlap = pk.found && (!pk.measure || pk.measure_ok);
    }
    // per-origin records of every frame, and the cross-stream order of every scene's state
    uint32_t used[kMaxBatch] = {};             // per frame: its scene's record buffers this launch reads
    for (uint32_t i = 0; i < n; i++)
    {
        rt_scene *s = S[i];
        int first = -1;
        for (uint32_t j = 0; j < i && first < 0; j++)
            if (S[j] == s) first = int(j);
        if (first < 0)
        {
            if (overlap && s->ev_recorded && st != s->last_stream)
            {
                if (int rc = order_overlap(s, st)) return rc;
            }
            else if (int rc = order_all(s, st))
                return rc;
            if (int rc = flush_tables(s, st)) return rc;
            s->last_stream = st;
            if (int rc = ensure_origin_terms(s, P[i], st, 0u, &used[i])) return rc;
        }
        else
        {
            uint32_t u = used[first];
            if (int rc = ensure_origin_terms(s, P[i], st, u, &u)) return rc;
            used[first] = u;
        }
    }
    for (uint32_t i = 0; i < n; i++)
    {
        bool first = true;
        for (uint32_t j = 0; j < i; j++) first = first && S[j] != S[i];
        if (first) S[i]->fref_last = used[i];
    }
    if (front || wide_heavy)
        if (int rc = hf_prepare(s0, P[0], blocks, kvar, front, st, ident | 1u, cams)) return rc;
    // fused: the wide section's workgroups lead the grid, a multiple of the XCD count so the lane
    // blocks keep their block -> XCD assignment
    // (the rounding's extra workgroups join the LDS tier, or without one the G-lane tier)
    if (fused && P[0].wh_wgs)
    {
        P[0].wh_wgs = (P[0].wh_wgs + kXcds - 1u) & ~(kXcds - 1u);
        if (!P[0].wh_lds) P[0].wh_wgs_g = P[0].wh_wgs;
    }
    uint32_t grid = uint32_t(blocks) + P[0].hf_front + (fused ? P[0].wh_wgs : 0u);
    // one-wave workgroups (k_render_batch_w64, as k_render_lanes_w64): the same blocks and order.
    // Without a wide section (N = 1) the bench pair took 0.569 vs 0.598 ms with 256-lane
    // workgroups (profiles/r03y_wg64_batch_sweep.json).  Beside one, per rank count (wg64_wide, bit
    // log2 N, 3 for N >= 8): with the section fused from 2 ranks and one-wave workgroups on both
    // (profiles/r03aa_wg64_wide_*.json) a rank of 2 took 0.306 ms (0.321 with 256-lane ones, 0.338
    // unfused), of 8 0.117 (0.121); a rank of 4 0.206 vs 0.193, so 4 keeps 256-lane workgroups
    const bool w64 = s0->wg64 != 0u && !lds && (!wide_heavy || ((s0->wg64_wide >> lg_ranks) & 1u) != 0u) &&
                     uint32_t(blocks) + P[0].hf_front >= s0->wg64_batch_min_blocks;
    uint32_t bwg = kWG;
    if (w64)
    {
        P[0].vblocks = uint32_t(blocks) + P[0].hf_front;
        grid = kWavesPerWG * ((fused ? P[0].wh_wgs : 0u) + (P[0].vblocks + kXcds - 1u) / kXcds * kXcds);
        bwg = 64u;
    }
    // the fused one-wave kernel held to 8 waves / SIMD (76 SGPRs; the plain build's 83 admit 7), per
    // rank count (wg64_o8, bit log2 N): a rank of 2 0.2925 vs 0.3025 ms, of 8 0.1171-0.1182 vs
    // 0.1139-0.1151 (profiles/r05f_ab_o8.json), so 2 only
    const bool o8 = ((s0->wg64_o8 >> lg_ranks) & 1u) != 0u && (kvar & kVarWideFused) != 0;
    const kbfn_t fn = batch_kernel(kvar, w64, o8);
    if (clk)
    {
        // one record per lane item and per (listed item, wave) of the wide section
        const size_t need = (size_t(blocks) * kWavesPerWG + size_t(kWhMax) * 17u) * 4u;
        if (need > s0->clk_cap)
        {
            if (s0->d_clk) RT_HIP(hipFree(s0->d_clk));
            s0->d_clk = nullptr;
            RT_HIP(hipMalloc(&s0->d_clk, need * sizeof(uint64_t)));
            s0->clk_cap = need;
        }
        RT_HIP(hipMemsetAsync(s0->d_clk, 0, need * sizeof(uint64_t), st));
        s0->clk_items = uint32_t(need / 4u);
        P[0].wave_clk = s0->d_clk;
    }
    for (uint32_t i = 0; i < n; i++) KB.p[i] = P[i];
    // timing: scene 0's ring (one timed launch for the whole batch)
    const bool timed = cap == hipStreamCaptureStatusNone && s0->time_every && s0->launches % s0->time_every == 0u;
    s0->launches++;
    const uint32_t kslot = s0->kt_next;
    if (timed && !s0->kt0[kslot]) RT_HIP(hipEventCreateWithFlags(&s0->kt0[kslot], s0->ev_time_flags));
    if (timed && (!s0->kt1[kslot] || s0->kt1[kslot].use_count() > 1))
        if (int rc = new_event(s0->kt1[kslot], s0->ev_time_flags)) return rc;
    // the dispatch's stop event marks every batched scene's last launch (no marker per scene: ten of
    // them cost config 5's step 50 us, profiles/r05u_marker_ab.json)
    rtk::EvRef stop = timed ? s0->kt1[kslot] : nullptr;
    if (!timed)
        if (int rc = free_done_event(s0, stop)) return rc;
    // a timed launch carries its start / stop events in the dispatch itself: separate event records
    // around it cost a measured 3-4 % of that frame (profiles/r05j_frame_series_*.json, steps 8, 24, ...)
    hipExtLaunchKernelGGL(fn, dim3(grid), dim3(bwg), 0, st, timed ? s0->kt0[kslot] : nullptr, stop->ev, 0u, KB);
    for (uint32_t i = 0; i < n; i++)
    {
        S[i]->ev_last = stop;
        S[i]->ev_recorded = true;
    }
    if ((P[0].hf_front || P[0].wh_on) && P[0].hf_measure)
        if (int rc = launch_plans(s0, KB.p[0], blocks, st, false)) return rc;
    RT_HIP(hipGetLastError());
    if (timed)
    {
        s0->kt_last = kslot;
        s0->kt_next = (kslot + 1u) % kTimeRing;
        s0->kt_count = std::min(s0->kt_count + 1u, kTimeRing);
    }
    return RT_OK;
}

} // namespace

namespace {
// Device staging frame (and, for rt_render_tiles, the scene's pinned host frame) of >= words.
int ensure_frame(rt_scene *s, size_t words, bool host)
{
    if (words > s->frame_cap)
    {
        if (s->d_frame) RT_HIP(hipFree(s->d_frame));
        s->d_frame = nullptr;
        RT_HIP(hipMalloc(&s->d_frame, words * 4));
        s->frame_cap = words;
    }
    if (host && words > s->hframe_cap)
    {
        if (s->h_frame) RT_HIP(hipHostFree(s->h_frame));
        s->h_frame = nullptr;
        RT_HIP(hipHostMalloc(&s->h_frame, words * 4));
        s->hframe_cap = words;
    }
    return RT_OK;
}
} // namespace

int rt_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

int rt_internal_use_device(int device, int *num_cus)
{
    int ndev = 0;
    RT_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(RT_E_NODEVICE, "device index out of range / no GPU");
    hipDeviceProp_t prop;
    RT_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RT_E_NODEVICE, std::string("librt_tracer is built for gfx950, device is ") + prop.gcnArchName);
    RT_HIP(hipSetDevice(device));
    if (num_cus) *num_cus = prop.multiProcessorCount;
    return RT_OK;
}

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_last_error(char *buf, size_t len)
{
    if (!buf || len == 0) return RT_E_INVALID;
    std::snprintf(buf, len, "%s", g_err.c_str());
    return RT_OK;
}

int rt_get_device_count(int *count)
{
    if (!count) return fail(RT_E_INVALID, "count is NULL");
    *count = 0;
    RT_HIP(hipGetDeviceCount(count));
    return RT_OK;
}

#ifndef RT_SRC_HASH
#define RT_SRC_HASH "unknown"
#endif

int rt_build_hash(char *buf, size_t len)
{
    if (!buf || len == 0) return fail(RT_E_INVALID, "bad arguments");
    std::snprintf(buf, len, "%s", RT_SRC_HASH);
    return RT_OK;
}

int rt_scene_info_get(rt_scene *s, rt_scene_info *out)
{
    if (!s || !out) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    std::memset(out, 0, sizeof(*out));
    out->octant_words = s->octant_words;
    out->box_words = s->box_words;
    out->packed_cells = s->d_cellw != nullptr;
    out->rcp_safe = s->rcp_safe;
    out->pack_ok = s->pack_ok;
    out->max_cell_refs = s->max_cell_refs;
    out->hf_floor = s->hf_floor;
    out->hf_min_blocks = s->hf_min_blocks;
    out->wh_floor = s->wh_floor;
    out->wh_alpha16 = s->wh_alpha16;
    out->wh_alpha16_n2 = s->wh_alpha16_n2;
    out->wh_lds = s->wh_lds;
    out->wh_auto_refs = s->wh_auto_refs;
    out->wh_fused = 1;
    out->hf_contexts = kHfCtxs;
    out->hf_evictions = s->hf_evictions;
    out->batch_launches = s->batch_launches;
    out->batch_fallbacks = s->batch_fallbacks;
    out->device_bytes = s->device_bytes;
    return RT_OK;
}

int rt_sample_table(uint32_t spp, float *out_xy)
{
    if (!out_xy || spp == 0) return fail(RT_E_INVALID, "bad arguments");
    std::vector<float> t;
    hammersley(spp, t);
    std::memcpy(out_xy, t.data(), t.size() * sizeof(float));
    return RT_OK;
}

// Cap on the 8 octant copies of the cell words (device and host): 64 M cells at most.
constexpr uint64_t kOctWordsMaxBytes = 256ull << 20;
// ... and on the 24 box-run copies
constexpr uint64_t kBoxWordsMaxBytes = 384ull << 20;

int rt_scene_create(const rt_scene_desc *d, int device, rt_scene **out)
{
    if (!d || !out) return fail(RT_E_INVALID, "desc/out is NULL");
    *out = nullptr;
    const rt_grid_desc& g = d->grid;
    if (d->num_triangles == 0 || d->num_vertices == 0 || !d->vertices || !d->triangles)
        return fail(RT_E_INVALID, "empty mesh");
    if (!g.cell_offsets || g.dims[0] == 0 || g.dims[1] == 0 || g.dims[2] == 0)
        return fail(RT_E_INVALID, "empty grid");
    const uint64_t nc64 = uint64_t(g.dims[0]) * g.dims[1] * g.dims[2];
    if (nc64 >= 0x7FFFFFFFull) return fail(RT_E_INVALID, "grid too large");
    const uint32_t nc = uint32_t(nc64);
    if (g.cell_offsets[0] != 0) return fail(RT_E_INVALID, "cell_offsets[0] != 0");
    for (uint32_t c = 0; c < nc; c++)
        if (g.cell_offsets[c + 1] < g.cell_offsets[c]) return fail(RT_E_INVALID, "cell_offsets not monotonic");
    const uint32_t nr = g.cell_offsets[nc];
    if (nr && !g.cell_tris) return fail(RT_E_INVALID, "cell_tris is NULL");
    for (uint32_t k = 0; k < nr; k++)
        if (g.cell_tris[k] >= d->num_triangles) return fail(RT_E_INVALID, "cell_tris index out of range");
    for (uint32_t i = 0; i < d->num_triangles; i++)
    {
        const rt_triangle& t = d->triangles[i];
        if (t.v0 >= d->num_vertices || t.v1 >= d->num_vertices || t.v2 >= d->num_vertices)
            return fail(RT_E_INVALID, "triangle vertex index out of range");
    }
    int ncus = 0;
    if (int rc = rt_internal_use_device(device, &ncus)) return rc;

    std::unique_ptr<rt_scene> s(new rt_scene());
    s->device = device;
    s->compact_wgs = 8u * uint32_t(std::max(1, ncus));
    // scheduling tunables: read once here, never per launch (A/B sweeps set them per scene)
    s->hf_floor = env_tunable("RT_HF_FLOOR", s->hf_floor);
    s->hf_min_blocks = env_tunable("RT_HF_MIN_BLOCKS", s->hf_min_blocks);
    s->hf_shift = std::min(env_tunable("RT_HF_SHIFT", s->hf_shift), 8u);
    s->hf_pos16 = std::min(env_tunable("RT_HF_POS16", s->hf_pos16), 64u);
    s->wg64 = env_tunable("RT_WG64", s->wg64);
    s->wh_floor = env_tunable("RT_WH_FLOOR", s->wh_floor);
    s->wh_alpha16 = env_tunable("RT_WH_ALPHA16", s->wh_alpha16);
    s->wh_alpha16_n2 = env_tunable("RT_WH_ALPHA16_N2", s->wh_alpha16_n2);
    s->wh_alpha16_n4 = env_tunable("RT_WH_ALPHA16_N4", s->wh_alpha16_n4);
    s->wh_alpha16_n8 = env_tunable("RT_WH_ALPHA16_N8", s->wh_alpha16_n8);
    s->wh_auto_refs = env_tunable("RT_WH_AUTO_REFS", s->wh_auto_refs);
    s->wg64_max_refs = env_tunable("RT_WG64_MAX_REFS", s->wg64_max_refs);
    s->wg64_wide = env_tunable("RT_WG64_WIDE", s->wg64_wide);
    s->wg64_o8 = env_tunable("RT_WG64_O8", s->wg64_o8);
    s->wh_lds = env_tunable("RT_WH_LDS", s->wh_lds);
    s->wh_beta16 = env_tunable("RT_WH_BETA16", s->wh_beta16);
    s->hf_follow = env_tunable("RT_HF_FOLLOW", s->hf_follow);
    for (int a = 0; a < 3; a++)
    {
        s->dims[a] = g.dims[a];
        s->bmin[a] = g.aabb_min[a];
        s->bmax[a] = g.aabb_max[a];
    }
    s->cw = g.cell_wdh;
    s->icw = g.inv_cell_wdh;
    s->ncells = nc;
    s->nrefs = nr;
    s->ntris = d->num_triangles;

    // Per-reference triangle records in CSR order (see file header)
    std::vector<float4> refs(size_t(std::max(nr, 1u)) * 3);
    double det_bound = 0.0;
    for (uint32_t k = 0; k < nr; k++)
    {
        const uint32_t ti = g.cell_tris[k];
        const rt_triangle& t = d->triangles[ti];
        const float *p0 = d->vertices[t.v0].p, *p1 = d->vertices[t.v1].p, *p2 = d->vertices[t.v2].p;
        const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };  // triangle.h:41
        const float e2[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };  // triangle.h:42
        float idf;
        std::memcpy(&idf, &ti, 4);
        refs[3 * size_t(k) + 0] = make_float4(p0[0], p0[1], p0[2], e1[0]);
        refs[3 * size_t(k) + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
        refs[3 * size_t(k) + 2] = make_float4(e2[2], idf, 0.0f, 0.0f);
        // |det| = |e1 . (d x e2)| <= |e1|_1 |e2|_1 for |d| ~ 1 (FAST_RCP range, rcp_nr)
        const double b = (std::fabs(double(e1[0])) + std::fabs(double(e1[1])) + std::fabs(double(e1[2]))) *
                         (std::fabs(double(e2[0])) + std::fabs(double(e2[1])) + std::fabs(double(e2[2])));
        det_bound = (b > det_bound || b != b) ? b : det_bound;
    }
    s->rcp_safe = det_bound == det_bound && det_bound < 0x1p120;
    s->pack_ok = g.dims[0] <= 512 && g.dims[1] <= 512 && g.dims[2] <= 512;
    std::vector<float4> shade(size_t(d->num_triangles) * 3), facen(d->num_triangles);
    std::vector<float4> trimt(size_t(d->num_triangles) * 3), tridist(size_t(d->num_triangles) * 6);
    for (uint32_t i = 0; i < d->num_triangles; i++)
    {
        const rt_triangle& t = d->triangles[i];
        const float *p0 = d->vertices[t.v0].p, *p1 = d->vertices[t.v1].p, *p2 = d->vertices[t.v2].p;
        {
            // brute force: {v0, e1 = v1 - v0, e2 = v2 - v0} (triangle.h:41-42) in triangle order
            const float e1[3] = { p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2] };
            const float e2[3] = { p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2] };
            trimt[3 * size_t(i) + 0] = make_float4(p0[0], p0[1], p0[2], e1[0]);
            trimt[3 * size_t(i) + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
            trimt[3 * size_t(i) + 2] = make_float4(e2[2], 0.0f, 0.0f, 0.0f);
        }
        const float *n0 = d->vertices[t.v0].n, *n1 = d->vertices[t.v1].n, *n2 = d->vertices[t.v2].n;
        shade[3 * size_t(i) + 0] = make_float4(n0[0], n0[1], n0[2], n1[0]);
        shade[3 * size_t(i) + 1] = make_float4(n1[1], n1[2], n2[0], n2[1]);
        shade[3 * size_t(i) + 2] = make_float4(n2[2], 0.0f, 0.0f, 0.0f);
        facen[i] = make_float4(t.n[0], t.n[1], t.n[2], 0.0f);
    }
    // Packed cell ranges: start < 2^21 and count < 2^11 for every cell -> one load per DDA step
    std::vector<uint32_t> cellw, cellwo, cellwb;
    bool packable = nr < (1u << 21);
    for (uint32_t c = 0; c < nc && packable; c++) packable = g.cell_offsets[c + 1] - g.cell_offsets[c] < 2048u;
    if (packable)
    {
        // Empty cells carry their Chebyshev (L-inf) distance to the nearest non-empty cell in
        // the start field: a DDA step moves to a face neighbour, so the next dist-1 cells of
        // any walk leaving this cell are empty and need no lookup.  BFS over 26-neighbours
        // from all non-empty cells gives exactly the L-inf distance.
        const uint32_t dxs = g.dims[0], dys = g.dims[1], dzs = g.dims[2];
        std::vector<uint32_t> dist(nc, 0xFFFFFFFFu), frontier, next;
        for (uint32_t c = 0; c < nc; c++)
            if (g.cell_offsets[c + 1] != g.cell_offsets[c]) { dist[c] = 0; frontier.push_back(c); }
        for (uint32_t d = 1; !frontier.empty(); d++)
        {
            next.clear();
            for (uint32_t c : frontier)
            {
                const uint32_t x = c % dxs, z = (c / dxs) % dzs, y = c / (dxs * dzs);   // grid.h:41-42
                for (int oy = -1; oy <= 1; oy++)
                    for (int oz = -1; oz <= 1; oz++)
                        for (int ox = -1; ox <= 1; ox++)
                        {
                            const int nx = int(x) + ox, ny = int(y) + oy, nz = int(z) + oz;
                            if (nx < 0 || ny < 0 || nz < 0 || nx >= int(dxs) || ny >= int(dys) || nz >= int(dzs))
                                continue;
                            const uint32_t n = uint32_t(nx) + uint32_t(nz) * dxs + uint32_t(ny) * dxs * dzs;
                            if (dist[n] == 0xFFFFFFFFu) { dist[n] = d; next.push_back(n); }
                        }
            }
            frontier.swap(next);
        }
        cellw.resize(nc);
        for (uint32_t c = 0; c < nc; c++)
        {
            const uint32_t cnt = g.cell_offsets[c + 1] - g.cell_offsets[c];
            cellw[c] = cnt ? ((g.cell_offsets[c] << 11) | cnt)
                           : (std::min<uint32_t>(dist[c] == 0xFFFFFFFFu ? 0x1FFFFFu : dist[c], 0x1FFFFFu) << 11);
        }
        // Per ray octant (sign of dx, dy, dz) a directional bound: D(c) = the side of the largest
        // empty cube with corner c that extends along the octant's signs (cells outside the grid
        // count as empty).  j steps of a walk in that octant move each coordinate by 0..j in the
        // octant's direction, so the next D-1 cells are empty -- the same contract as the L-inf
        // word, and D >= the L-inf distance.  D(c) = 1 + min of D over the 7 forward neighbours
        // (the 3-D largest-square recurrence).  A grid whose 8 copies would pass kOctWordsMaxBytes keeps
        // the L-inf words (they measured ~2 % slower, profiles/r02x_ab_octant_dist.json).
        if (uint64_t(nc) * 8u * 4u <= kOctWordsMaxBytes)
        {
            s->octant_words = true;
            constexpr uint32_t kInf = 0x1FFFFFu;
            cellwo.resize(size_t(8) * nc);
            std::vector<uint32_t> D(nc);
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
                            // visit forward neighbours first: against the octant's direction
                            const int x = sx > 0 ? int(dxs) - 1 - ix : ix;
                            const int y = sy > 0 ? int(dys) - 1 - iy : iy;
                            const int z = sz > 0 ? int(dzs) - 1 - iz : iz;
                            const uint32_t c = uint32_t(x) + uint32_t(z) * dxs + uint32_t(y) * dxs * dzs;
                            if (g.cell_offsets[c + 1] != g.cell_offsets[c]) { D[c] = 0; continue; }
                            uint32_t m = kInf;
                            for (int n = 1; n < 8; n++)
                                m = std::min(m, at(x + ((n & 1) ? sx : 0), y + ((n & 2) ? sy : 0), z + ((n & 4) ? sz : 0)));
                            D[c] = std::min(kInf, m + 1);
                        }
                for (uint32_t c = 0; c < nc; c++)
                    cellwo[size_t(o) * nc + c] = (cellw[c] & 2047u) ? cellw[c] : (D[c] << 11);
            }
        }
        // AUTO's box-run words (build_box_words): the non-empty words keep start < 2^20
        if (nr < (1u << 20) && uint64_t(nc) * 24u * 4u <= kBoxWordsMaxBytes)
        {
            s->box_words = rtbox::build_box_words(g.cell_offsets, g.dims, cellwb);
            if (!s->box_words) cellwb.clear();          // out of host memory: AUTO walks without them
        }
    }
    for (uint32_t c = 0; c < nc; c++)
        s->max_cell_refs = std::max(s->max_cell_refs, g.cell_offsets[c + 1] - g.cell_offsets[c]);

    const size_t nfrefs = size_t(std::max(nr, 1u)) * 4;
    RT_HIP(hipMalloc(&s->d_off, sizeof(uint32_t) * (nc + 1)));
    RT_HIP(hipMalloc(&s->d_refs, sizeof(float4) * refs.size()));
    RT_HIP(hipMalloc(&s->d_frefs[0], sizeof(float4) * nfrefs));
    RT_HIP(hipMalloc(&s->d_frefs[1], sizeof(float4) * nfrefs));
    RT_HIP(hipMalloc(&s->d_shade, sizeof(float4) * shade.size()));
    RT_HIP(hipMalloc(&s->d_facen, sizeof(float4) * facen.size()));
    RT_HIP(hipMemcpy(s->d_off, g.cell_offsets, sizeof(uint32_t) * (nc + 1), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_refs, refs.data(), sizeof(float4) * refs.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_shade, shade.data(), sizeof(float4) * shade.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_facen, facen.data(), sizeof(float4) * facen.size(), hipMemcpyHostToDevice));
    // Distance records in Morton order of the triangle centroids, blocks of kDistBlock with their
    // exact float AABB (the ray march's block cull, see ray_march)
    std::vector<float4> distblk;
    {
        const uint32_t nt = d->num_triangles;
        float mn[3] = { rtd::kFltMax, rtd::kFltMax, rtd::kFltMax }, mx[3] = { -rtd::kFltMax, -rtd::kFltMax, -rtd::kFltMax };
        float scale = 0.0f;
        for (uint32_t i = 0; i < d->num_vertices; i++)
            for (int a = 0; a < 3; a++)
            {
                mn[a] = std::min(mn[a], d->vertices[i].p[a]);
                mx[a] = std::max(mx[a], d->vertices[i].p[a]);
                scale = std::max(scale, std::fabs(d->vertices[i].p[a]));
            }
        std::vector<std::pair<uint64_t, uint32_t>> order(nt);
        for (uint32_t i = 0; i < nt; i++)
        {
            const rt_triangle& t = d->triangles[i];
            uint64_t code = 0;
            uint32_t q[3];
            for (int a = 0; a < 3; a++)
            {
                const double c = (double(d->vertices[t.v0].p[a]) + d->vertices[t.v1].p[a] + d->vertices[t.v2].p[a]) / 3.0;
                const double ext = double(mx[a]) - double(mn[a]);
                const double f = ext > 0.0 ? (c - mn[a]) / ext : 0.0;
                q[a] = uint32_t(std::min(1023.0, std::max(0.0, f * 1024.0)));
            }
            for (int bit = 9; bit >= 0; bit--)
                for (int a = 0; a < 3; a++) code = (code << 1) | ((q[a] >> bit) & 1u);
            order[i] = { code, i };
        }
        std::sort(order.begin(), order.end());
        s->ndist_blk = (nt + kDistBlock - 1) / kDistBlock;
        distblk.resize(size_t(s->ndist_blk) * 2);
        for (uint32_t b = 0; b < s->ndist_blk; b++)
        {
            float bmn[3] = { rtd::kFltMax, rtd::kFltMax, rtd::kFltMax }, bmx[3] = { -rtd::kFltMax, -rtd::kFltMax, -rtd::kFltMax };
            for (uint32_t k = b * kDistBlock; k < std::min(nt, (b + 1) * kDistBlock); k++)
            {
                const rt_triangle& t = d->triangles[order[k].second];
                const float *p[3] = { d->vertices[t.v0].p, d->vertices[t.v1].p, d->vertices[t.v2].p };
                dist_record(p[0], p[1], p[2], &tridist[6 * size_t(k)]);
                for (int v = 0; v < 3; v++)
                    for (int a = 0; a < 3; a++)
                    {
                        bmn[a] = std::min(bmn[a], p[v][a]);
                        bmx[a] = std::max(bmx[a], p[v][a]);
                    }
            }
            distblk[2 * b] = make_float4(bmn[0], bmn[1], bmn[2], 0.0f);
            distblk[2 * b + 1] = make_float4(bmx[0], bmx[1], bmx[2], 0.0f);
        }
        s->scene_scale = scale;
        for (int a = 0; a < 3; a++)
        {
            s->vmin[a] = mn[a];
            s->vmax[a] = mx[a];
        }
    }
    RT_HIP(hipMalloc(&s->d_distblk, sizeof(float4) * std::max<size_t>(1, distblk.size())));
    RT_HIP(hipMemcpy(s->d_distblk, distblk.data(), sizeof(float4) * distblk.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMalloc(&s->d_trimt, sizeof(float4) * trimt.size()));
    RT_HIP(hipMalloc(&s->d_tridist, sizeof(float4) * tridist.size()));
    RT_HIP(hipMemcpy(s->d_trimt, trimt.data(), sizeof(float4) * trimt.size(), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(s->d_tridist, tridist.data(), sizeof(float4) * tridist.size(), hipMemcpyHostToDevice));
    if (packable)
    {
        RT_HIP(hipMalloc(&s->d_cellw, sizeof(uint32_t) * nc));
        RT_HIP(hipMemcpy(s->d_cellw, cellw.data(), sizeof(uint32_t) * nc, hipMemcpyHostToDevice));
        if (!cellwo.empty())
        {
            RT_HIP(hipMalloc(&s->d_cellwo, sizeof(uint32_t) * cellwo.size()));
            RT_HIP(hipMemcpy(s->d_cellwo, cellwo.data(), sizeof(uint32_t) * cellwo.size(), hipMemcpyHostToDevice));
            s->oct_stride = nc;
        }
        if (!cellwb.empty())
        {
            RT_HIP(hipMalloc(&s->d_cellwb, sizeof(uint32_t) * cellwb.size()));
            RT_HIP(hipMemcpy(s->d_cellwb, cellwb.data(), sizeof(uint32_t) * cellwb.size(), hipMemcpyHostToDevice));
            s->box_stride = nc;
        }
    }
    s->device_bytes = sizeof(uint32_t) * (nc + 1) +
                      sizeof(float4) * (refs.size() + 2 * nfrefs + shade.size() + facen.size() + trimt.size() +
                                        tridist.size() + distblk.size()) +
                      sizeof(uint32_t) * (cellw.size() + cellwo.size() + cellwb.size());
    RT_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    if (int rc = new_event(s->ev_own, s->ev_order_flags)) return rc;
    for (rtk::EvRef& e : s->ev_done)                                    // dispatches' stop events
        if (int rc = new_event(e, s->ev_time_flags)) return rc;
    s->ev_last = s->ev_own;
    // the plan stream (launch_plans) and the first timed launch's events: created here, not by a
    // frame (a stream's creation took ~0.33 ms of the second frame's call, profiles/r05p_host_trace.log)
    RT_HIP(hipStreamCreateWithFlags(&s->plan_st, hipStreamNonBlocking));
    RT_HIP(hipEventCreateWithFlags(&s->kt0[0], s->ev_time_flags));
    if (int rc = new_event(s->kt1[0], s->ev_time_flags)) return rc;
    // the heavy-first contexts' host-mapped counters, and the frame tables at a 4K x 16 spp capacity:
    // allocated here so a new launch shape's first frame waits for no allocation call
    RT_HIP(hipHostMalloc(&s->h_wh_cnt, sizeof(uint32_t) * 2 * kHfCtxs, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(s->h_wh_cnt, 0, sizeof(uint32_t) * 2 * kHfCtxs);
    {
        void *dev = nullptr;
        RT_HIP(hipHostGetDevicePointer(&dev, s->h_wh_cnt, 0));
        s->d_wh_cnt = static_cast<uint32_t *>(dev);
    }
    s->ndc_cap = size_t(4096 + 4096) * 16u;
    RT_HIP(hipMalloc(&s->d_ndc, s->ndc_cap * sizeof(float)));
    s->smp_cap = 64u;
    RT_HIP(hipMalloc(&s->d_smp, sizeof(float2) * s->smp_cap));
    RT_HIP(hipHostMalloc(&s->h_smp_pinned, sizeof(float2) * s->smp_cap));
    // and the first heavy-first context's state (a new shape's first frame took ~25 us of host time
    // in hf_prepare's hipMalloc: RT_HOST_TRACE, profiles/r05at_host_trace.log)
    if (int rc = hf_alloc(&s->hf[0], kHfPreBlocks)) return rc;

    *out = s.release();
    return RT_OK;
}

int rt_scene_destroy(rt_scene *s)
{
    if (!s) return RT_OK;
    {
        std::lock_guard<std::mutex> lk(s->mtx);
        (void)hipSetDevice(s->device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->last_stream && s->ev_recorded) (void)hipEventSynchronize(s->ev_last->ev);
        if (s->ev_prev) (void)hipEventSynchronize(s->ev_prev->ev);
        if (s->plan_st) (void)hipStreamSynchronize(s->plan_st);
        if (s->side) (void)hipStreamSynchronize(s->side);
        (void)hipFree(s->d_off);
        (void)hipFree(s->d_refs);
        (void)hipFree(s->d_frefs[0]);
        (void)hipFree(s->d_frefs[1]);
        (void)hipFree(s->d_shade);
        (void)hipFree(s->d_facen);
        (void)hipFree(s->d_cellw);
        (void)hipFree(s->d_cellwo);
        (void)hipFree(s->d_cellwb);
        (void)hipFree(s->d_trimt);
        (void)hipFree(s->d_tridist);
        (void)hipFree(s->d_distblk);
        (void)hipFree(s->d_clk);
        for (HfCtx& h : s->hf)
        {
            (void)hipFree(h.mem);
            if (h.pend_ev) (void)hipEventDestroy(h.pend_ev);
            if (h.fence_ev) (void)hipEventDestroy(h.fence_ev);
        }
        if (s->h_wh_cnt) (void)hipHostFree(s->h_wh_cnt);
        if (s->side) (void)hipStreamDestroy(s->side);
        if (s->plan_st) (void)hipStreamDestroy(s->plan_st);
        if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
        if (s->ev_join) (void)hipEventDestroy(s->ev_join);
        (void)hipFree(s->d_smp);
        (void)hipFree(s->d_ndc);
        (void)hipFree(s->d_frame);
        if (s->h_smp_pinned) (void)hipHostFree(s->h_smp_pinned);
        if (s->h_frame) (void)hipHostFree(s->h_frame);
        s->ev_own.reset();             // shared events: destroyed with their last reference
        for (rtk::EvRef& e : s->ev_done) e.reset();
        s->ev_last.reset();
        s->ev_prev.reset();
        for (hipEvent_t e : s->band_ev) if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : s->kt0) if (e) (void)hipEventDestroy(e);
        for (rtk::EvRef& e : s->kt1) e.reset();
        for (hipEvent_t e : s->tile_ev) if (e) (void)hipEventDestroy(e);
        if (s->stream) (void)hipStreamDestroy(s->stream);
        if (s->stream2) (void)hipStreamDestroy(s->stream2);
        if (s->ev_t_fork) (void)hipEventDestroy(s->ev_t_fork);
        if (s->ev_t_join) (void)hipEventDestroy(s->ev_t_join);

    }
    delete s;
    return RT_OK;
}

int rt_scene_device_bytes(const rt_scene *s, uint64_t *bytes)
{
    if (!s || !bytes) return fail(RT_E_INVALID, "NULL argument");
    *bytes = s->device_bytes;
    return RT_OK;
}

} // extern "C"

namespace {
// Per-sample records requested from the product kernels (rt_render_records_device): the
// rectangle's samples land in d[((y - y0) * w + (x - x0)) * spp + s].
struct RecOut { rt_sample_rec *d; uint32_t x0, y0, w, h; };

void set_records(KParams& P, const RecOut& r)
{
    P.recs = r.d;
    P.rec_x0 = r.x0;
    P.rec_y0 = r.y0;
    P.rec_w = r.w;
    P.rec_h = r.h;
}

// Frame parameters of a device-resident render (see render_device); returns the local tile count.
uint32_t device_params(const rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, bool shard,
                       uint32_t *d_out, uint32_t *d_hits, KParams& P)
{
    frame_params(s, f, P);
    P.rx0 = 0; P.ry0 = 0; P.rw = f->width; P.rh = f->height;
    P.tiles_x = (f->width + kTile - 1) / kTile;
    const uint32_t ntiles = P.tiles_x * ((f->height + kTile - 1) / kTile);
    P.rank = rank; P.nranks = nranks;
    P.out = d_out;
    P.hits = d_hits;
    P.pitch = shard ? 0u : f->width;
    P.shard_mode = shard ? 1u : 0u;
    return ntiles > rank ? (ntiles - rank + nranks - 1) / nranks : 0;
}

// The device-resident render of a whole frame (shard false: d_out[y*W + x]) or of one rank's
// interleaved 16x16 tiles (shard true: d_out = the compact shard, also for nranks == 1),
// optionally with per-sample hit IDs.
int render_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, bool shard, uint32_t *d_out,
                  uint32_t *d_hits, void *hip_stream, const RecOut *recs = nullptr)
{
    if (!s || !d_out || nranks == 0 || rank >= nranks) return fail(RT_E_INVALID, "bad arguments");
    int rc = validate_frame(f);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(s->mtx);
    g_ht.start();
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    g_ht.mark("samples");
    KParams P;
    const uint32_t local = device_params(s, f, rank, nranks, shard, d_out, d_hits, P);
    if (recs) set_records(P, *recs);
    rc = launch_render(s, f, P, local, static_cast<hipStream_t>(hip_stream));
    g_ht.mark("done");
    g_ht.end();
    return rc;
}

// rt_render_batch_device's frames [0, n): one k_render_batch launch when they can share it.  The
// cheap checks (one device) come before anything touches a scene's device state; a scene listed
// twice with another frame shape or sample table than its last frame's would read the last one's
// tables, so such batches take one launch per frame (counted in rt_scene_info.batch_fallbacks).
int render_batch_chunk(rt_scene *const *S, const rt_frame *F, uint32_t n, uint32_t rank, uint32_t nranks,
                       uint32_t *const *outs, uint32_t *const *hits, const RecOut *recs, void *hip_stream)
{
    bool batched = false;
    bool one_device = true;
    for (uint32_t i = 1; i < n; i++) one_device = one_device && S[i]->device == S[0]->device;
    if (n >= 2 && one_device)
    {
        std::vector<rt_scene *> uniq(S, S + n);
        std::sort(uniq.begin(), uniq.end());
        uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
        std::vector<std::unique_lock<std::mutex>> locks;
        for (rt_scene *s : uniq) locks.emplace_back(s->mtx);
        int rc = ensure_device(S[0]);
        if (rc) return rc;
        KParams P[kMaxBatch];
        uint32_t local = 0;
        for (uint32_t i = 0; i < n; i++)
        {
            if ((rc = prepare_samples(S[i], &F[i], std::max(1u, F[i].spp)))) return rc;
            local = device_params(S[i], &F[i], rank, nranks, nranks > 1, outs[i], hits ? hits[i] : nullptr, P[i]);
            if (recs) set_records(P[i], recs[i]);
        }
        bool tables_ok = true;
        for (uint32_t i = 0; i < n; i++) tables_ok = tables_ok && tables_match(S[i], &F[i], std::max(1u, F[i].spp));
        if (tables_ok) rc = launch_batch(S, F, n, P, local, static_cast<hipStream_t>(hip_stream), &batched);
        if (batched)
        {
            if (rc == RT_OK) S[0]->batch_launches++;      // bench.py trusts this count (VALU roofline)
            return rc;
        }
    }
    if (n >= 2)
    {
        std::lock_guard<std::mutex> lk(S[0]->mtx);
        S[0]->batch_fallbacks++;
    }
    for (uint32_t i = 0; i < n; i++)
        if (int rc = render_device(S[i], &F[i], rank, nranks, nranks > 1, outs[i], hits ? hits[i] : nullptr, hip_stream,
                                   recs ? &recs[i] : nullptr))
            return rc;
    return RT_OK;
}
} // namespace

extern "C" {

int rt_render_frame_device(rt_scene *s, const rt_frame *f, uint32_t *d_bgra, void *hip_stream)
{
    return render_device(s, f, 0, 1, false, d_bgra, nullptr, hip_stream);
}

int rt_shard_elems(uint32_t width, uint32_t height, uint32_t nranks, uint64_t *elems)
{
    if (!elems || nranks == 0 || width == 0 || height == 0) return fail(RT_E_INVALID, "bad arguments");
    const uint64_t ntiles = uint64_t((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
    *elems = ((ntiles + nranks - 1) / nranks) * kTilePix;
    return RT_OK;
}

int rt_render_shard_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, uint32_t *d_shard,
                           void *hip_stream)
{
    return render_device(s, f, rank, nranks, true, d_shard, nullptr, hip_stream);
}

int rt_render_batch_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                           uint32_t nranks, uint32_t *const *d_outs, uint32_t *const *d_hits, void *hip_stream)
{
    if (!scenes || !frames || !d_outs || nranks == 0 || rank >= nranks) return fail(RT_E_INVALID, "bad arguments");
    for (uint32_t i = 0; i < n; i++)
    {
        if (!scenes[i] || !d_outs[i]) return fail(RT_E_INVALID, "NULL scene or output");
        if (int rc = validate_frame(&frames[i])) return rc;
    }
    for (uint32_t i = 0; i < n;)
    {
        const uint32_t c = batch_chunk_len(n, i);
        if (int rc = render_batch_chunk(scenes + i, frames + i, c, rank, nranks, d_outs + i,
                                        d_hits ? d_hits + i : nullptr, nullptr, hip_stream))
            return rc;
        i += c;
    }
    return RT_OK;
}

int rt_render_records_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                             uint32_t nranks, uint32_t *const *d_outs, const rt_tile *rects,
                             rt_sample_rec *const *d_recs, void *hip_stream)
{
    if (!scenes || !frames || !d_outs || !rects || !d_recs || n == 0 || nranks == 0 || rank >= nranks)
        return fail(RT_E_INVALID, "bad arguments");
    std::vector<RecOut> ro(n);
    // A records call never overlaps the scene's previous launch (RT_KERNEL_FLAG_OVERLAP is dropped): its
    // fixup below reads the scene's tables after the render and marks the call's end with its own event.
    std::vector<rt_frame> fr(frames, frames + n);
    for (rt_frame& f : fr) f.kernel &= ~uint32_t(RT_KERNEL_FLAG_OVERLAP);
    frames = fr.data();
    for (uint32_t i = 0; i < n; i++)
    {
        if (!scenes[i] || !d_outs[i] || !d_recs[i]) return fail(RT_E_INVALID, "NULL scene, output or record array");
        if (int rc = validate_frame(&frames[i])) return rc;
        if ((frames[i].kernel & RT_KERNEL_KIND_MASK) != RT_KERNEL_AUTO || frames[i].intersector != RT_ISECT_GRID ||
            frames[i].tri_test != RT_TRI_MOLLER_TRUMBORE)
            return fail(RT_E_INVALID, "records come from AUTO's grid / IntersectRayTri path only");
        const rt_tile& r = rects[i];
        if (r.x1 <= r.x0 || r.y1 <= r.y0 || r.x1 > frames[i].width || r.y1 > frames[i].height)
            return fail(RT_E_INVALID, "record rectangle outside the frame or empty");
        ro[i] = RecOut{ d_recs[i], r.x0, r.y0, r.x1 - r.x0, r.y1 - r.y0 };
    }
    if (n == 1)
    {
        if (int rc = render_device(scenes[0], &frames[0], rank, nranks, nranks > 1, d_outs[0], nullptr, hip_stream,
                                   &ro[0]))
            return rc;
    }
    else
        for (uint32_t i = 0; i < n;)
        {
            const uint32_t c = batch_chunk_len(n, i);
            if (int rc = render_batch_chunk(scenes + i, frames + i, c, rank, nranks, d_outs + i, nullptr,
                                            ro.data() + i, hip_stream))
                return rc;
            i += c;
        }
    // the raw records made final (k_record_fixup), per frame on the launch stream
    for (uint32_t i = 0; i < n; i++)
    {
        rt_scene *s = scenes[i];
        std::lock_guard<std::mutex> lk(s->mtx);
        if (int rc = ensure_device(s)) return rc;
        if (int rc = prepare_samples(s, &frames[i], std::max(1u, frames[i].spp))) return rc;
        KParams P;
        frame_params(s, &frames[i], P);
        set_records(P, ro[i]);
        const uint64_t nrec = uint64_t(ro[i].w) * ro[i].h * P.spp;
        if (nrec > 0xFFFFFFFFull) return fail(RT_E_INVALID, "record rectangle too large");
        hipLaunchKernelGGL(record_fixup_kernel(), dim3(uint32_t((nrec + kWG - 1) / kWG)), dim3(kWG), 0,
                           static_cast<hipStream_t>(hip_stream), P, uint32_t(nrec));
        RT_HIP(hipGetLastError());
        // the fixup reads the scene's tables (camera-space x / y, CSR offsets): a later call that
        // rewrites them (prepare_samples -> wait_scene_idle) must wait for it, as for a render launch.
        // Its own completion event (a free one: re-recording an event that the scene still holds as
        // ev_prev would move that mark past the launch it stands for)
        rtk::EvRef done;
        if (int rc = free_done_event(s, done)) return rc;
        RT_HIP(hipEventRecord(done->ev, static_cast<hipStream_t>(hip_stream)));
        s->ev_last = done;
        s->ev_recorded = true;
        s->last_stream = static_cast<hipStream_t>(hip_stream);
    }
    return RT_OK;
}

int rt_render_hits_device(rt_scene *s, const rt_frame *f, uint32_t rank, uint32_t nranks, uint32_t *d_out,
                          uint32_t *d_hits, void *hip_stream)
{
    if (!d_hits) return fail(RT_E_INVALID, "d_hits is NULL");
    return render_device(s, f, rank, nranks, nranks > 1, d_out, d_hits, hip_stream);
}

int rt_unshard_device(uint32_t width, uint32_t height, uint32_t nranks, const uint32_t *d_gathered,
                      uint32_t *d_bgra, void *hip_stream)
{
    if (!d_gathered || !d_bgra || nranks == 0) return fail(RT_E_INVALID, "bad arguments");
    uint64_t elems = 0;
    int rc = rt_shard_elems(width, height, nranks, &elems);
    if (rc) return rc;
    const uint32_t tiles_x = (width + kTile - 1) / kTile;
    hipLaunchKernelGGL(unshard_kernel(), dim3((width + 63) / 64, (height + 3) / 4), dim3(kWG), 0,
                       static_cast<hipStream_t>(hip_stream), d_gathered, d_bgra, width, height, tiles_x, nranks,
                       elems);
    RT_HIP(hipGetLastError());
    return RT_OK;
}

int rt_last_kernel_ms(rt_scene *s, float *ms)
{
    if (!s || !ms) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    if (s->kt_last >= kTimeRing) return fail(RT_E_INVALID, "no timed kernel recorded yet");
    RT_HIP(hipEventSynchronize(s->kt1[s->kt_last]->ev));
    RT_HIP(hipEventElapsedTime(ms, s->kt0[s->kt_last], s->kt1[s->kt_last]->ev));
    return RT_OK;
}

int rt_scene_set_timing(rt_scene *s, uint32_t every)
{
    if (!s) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    s->time_every = every;
    s->launches = 0;
    return RT_OK;
}

int rt_kernel_times(rt_scene *s, float *ms, uint32_t max_n, uint32_t *n)
{
    if (!s || !n || (max_n && !ms)) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    const uint32_t cnt = std::min(max_n, s->kt_count);
    const uint32_t next = s->kt_next;
    s->kt_count = 0;                      // consumed whatever happens below
    uint32_t got = 0;
    for (uint32_t i = 0; i < cnt; i++)
    {
        // a pair that cannot be read (a launch that failed between its two records) is skipped
        const uint32_t slot = (next + kTimeRing - cnt + i) % kTimeRing;
        float v = 0.0f;
        if (hipEventSynchronize(s->kt1[slot]->ev) == hipSuccess &&
            hipEventElapsedTime(&v, s->kt0[slot], s->kt1[slot]->ev) == hipSuccess && v >= 0.0f)
            ms[got++] = v;
        else
            (void)hipGetLastError();
    }
    *n = got;
    return RT_OK;
}

int rt_render_tiles(rt_scene *s, const rt_frame *f, const rt_tile *tiles, uint32_t n, uint32_t *const *bufs)
{
    if (!s || (n && (!tiles || !bufs))) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    uint32_t bx0 = 0xFFFFFFFFu, by0 = 0xFFFFFFFFu, bx1 = 0, by1 = 0;
    for (uint32_t i = 0; i < n; i++)
    {
        const rt_tile& t = tiles[i];
        if (!bufs[i] || t.x1 <= t.x0 || t.y1 <= t.y0 || t.x1 > f->width || t.y1 > f->height)
            return fail(RT_E_INVALID, "tile outside the frame or empty");
        bx0 = std::min(bx0, t.x0); by0 = std::min(by0, t.y0);
        bx1 = std::max(bx1, t.x1); by1 = std::max(by1, t.y1);
    }
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint32_t rw = bx1 - bx0, rh = by1 - by0;
    const size_t words = size_t(rw) * rh;
    if ((rc = ensure_frame(s, words, true))) return rc;
    KParams P;
    frame_params(s, f, P);
    P.rx0 = bx0; P.ry0 = by0; P.rw = rw; P.rh = rh;
    P.tiles_x = (rw + kTile - 1) / kTile;
    P.rank = 0; P.nranks = 1;
    P.out = s->d_frame; P.pitch = rw; P.shard_mode = 0;
    if ((rc = launch_render(s, f, P, P.tiles_x * ((rh + kTile - 1) / kTile), s->stream))) return rc;
    // D2H in row bands; band k's rows are scattered into the tiles while band k+1 is in flight
    const uint32_t nb = std::min(kTileBands, rh), bh = (rh + nb - 1) / nb;
    for (uint32_t b = 0; b < nb; b++)
    {
        const uint32_t ya = b * bh, yb = std::min(rh, ya + bh);
        if (ya >= yb) break;
        if (!s->tile_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->tile_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(s->h_frame + size_t(ya) * rw, s->d_frame + size_t(ya) * rw,
                              size_t(yb - ya) * rw * 4, hipMemcpyDeviceToHost, s->stream));
        RT_HIP(hipEventRecord(s->tile_ev[b], s->stream));
    }
    for (uint32_t b = 0; b < nb; b++)
    {
        const uint32_t ya = by0 + b * bh, yb = std::min(by1, ya + bh);
        if (ya >= yb) break;
        RT_HIP(hipEventSynchronize(s->tile_ev[b]));
        for (uint32_t i = 0; i < n; i++)                         // framebuffer.h:41-45 layout
        {
            const rt_tile& t = tiles[i];
            const uint32_t tw = t.x1 - t.x0;
            for (uint32_t y = std::max(t.y0, ya); y < std::min(t.y1, yb); y++)
                std::memcpy(bufs[i] + size_t(y - t.y0) * tw, s->h_frame + size_t(y - by0) * rw + (t.x0 - bx0),
                            size_t(tw) * 4);
        }
    }
    return RT_OK;
}

int rt_host_alloc(size_t bytes, void **out)
{
    if (!out || bytes == 0) return fail(RT_E_INVALID, "bad arguments");
    *out = nullptr;
    RT_HIP(hipHostMalloc(out, bytes));
    return RT_OK;
}

int rt_host_free(void *p)
{
    if (p) RT_HIP(hipHostFree(p));
    return RT_OK;
}

int rt_render_frame_host(rt_scene *s, const rt_frame *f, uint32_t *h_bgra, const uint32_t *band_y1,
                         uint32_t nbands)
{
    if (!s || !h_bgra || (nbands && !band_y1)) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (nbands > kMaxBands) return fail(RT_E_INVALID, "more than 64 row bands");
    for (uint32_t b = 0; b < nbands; b++)
        if (band_y1[b] == 0 || band_y1[b] > f->height || (b && band_y1[b] <= band_y1[b - 1]) ||
            (b + 1 == nbands && band_y1[b] != f->height))
            return fail(RT_E_INVALID, "band ends must increase strictly and end at the frame height");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint32_t W = f->width, H = f->height;
    if ((rc = ensure_frame(s, size_t(W) * H, false))) return rc;
    KParams P;
    frame_params(s, f, P);
    P.rx0 = 0; P.ry0 = 0; P.rw = W; P.rh = H;
    P.tiles_x = (W + kTile - 1) / kTile;
    P.rank = 0; P.nranks = 1;
    P.out = s->d_frame; P.pitch = W; P.shard_mode = 0;
    s->nbands = 0;
    if ((rc = launch_render(s, f, P, P.tiles_x * ((H + kTile - 1) / kTile), s->stream))) return rc;
    const uint32_t nb = nbands ? nbands : 1;
    for (uint32_t b = 0, ya = 0; b < nb; b++)
    {
        const uint32_t yb = nbands ? band_y1[b] : H;
        if (!s->band_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->band_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(h_bgra + size_t(ya) * W, s->d_frame + size_t(ya) * W, size_t(yb - ya) * W * 4,
                              hipMemcpyDeviceToHost, s->stream));
        RT_HIP(hipEventRecord(s->band_ev[b], s->stream));
        s->band_y1[b] = yb;
        ya = yb;
    }
    s->nbands = nb;
    return RT_OK;
}

int rt_render_frame_host_tiled(rt_scene *s, const rt_frame *f, uint32_t *h_tiles, uint32_t tiles_x, uint32_t tiles_y,
                               uint32_t nlaunch)
{
    if (!s || !h_tiles || tiles_x == 0 || tiles_y == 0 || nlaunch == 0) return fail(RT_E_INVALID, "bad arguments");
    int rc = validate_frame(f);
    if (rc) return rc;
    const uint32_t W = f->width, H = f->height;
    if (tiles_y > kMaxBands) return fail(RT_E_INVALID, "more than 64 tile rows");
    // row-band launches of one scene overlap on two streams and share its scene-wide debug and
    // wide-section buffers (wave clocks from index 0, the side stream's fork / join): one launch only
    if (nlaunch > 1u && (f->kernel & (RT_KERNEL_FLAG_WAVE_CLOCK | RT_KERNEL_FLAG_WIDE_HEAVY)))
        return fail(RT_E_INVALID, "row-band launches (nlaunch > 1) take neither WAVE_CLOCK nor WIDE_HEAVY");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    if ((rc = ensure_frame(s, size_t(W) * H, false))) return rc;
    if (!s->stream2)
    {
        RT_HIP(hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking));
        RT_HIP(hipEventCreateWithFlags(&s->ev_t_fork, hipEventDisableTiming));
        RT_HIP(hipEventCreateWithFlags(&s->ev_t_join, hipEventDisableTiming));
    }
    // Framebuffer::Resize's tile rows (framebuffer.cpp:106-117): row r spans [r * th, (r + 1) * th),
    // the last one to H; launch j renders tile rows [j * R / n, (j + 1) * R / n)
    const uint32_t tw = W / tiles_x, th = H / tiles_y;
    const uint32_t nl = std::min(nlaunch, tiles_y);
    auto row_y = [&](uint32_t r) { return r >= tiles_y ? H : r * th; };
    hipStream_t st[2] = { s->stream, s->stream2 };
    // both streams after everything earlier on this scene (the scene's tables and records are shared)
    if (s->ev_recorded)
    {
        RT_HIP(hipStreamWaitEvent(st[0], s->ev_last->ev, 0));
        if (s->ev_prev) RT_HIP(hipStreamWaitEvent(st[0], s->ev_prev->ev, 0));
        s->ev_prev.reset();
    }
    KParams P0;
    frame_params(s, f, P0);
    if (use_lanes(f, spp) && P0.isect == RT_ISECT_GRID && P0.tri_test == RT_TRI_MOLLER_TRUMBORE &&
        ((f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_AUTO || (f->kernel & RT_KERNEL_KIND_MASK) == RT_KERNEL_COMPACT))
    {
        uint32_t used = 0;                      // (every launch before this one is waited for above)
        if ((rc = ensure_origin_terms(s, P0, st[0], 0u, &used))) return rc;
        s->fref_last = used;
    }
    if ((rc = flush_tables(s, st[0]))) return rc;      // before the fork: both streams read them
    RT_HIP(hipEventRecord(s->ev_t_fork, st[0]));
    RT_HIP(hipStreamWaitEvent(st[1], s->ev_t_fork, 0));
    s->nbands = 0;
    for (uint32_t j = 0; j < nl; j++)
    {
        const uint32_t r0 = j * tiles_y / nl, r1 = (j + 1) * tiles_y / nl;
        const uint32_t ya = row_y(r0), yb = row_y(r1);
        if (ya >= yb) continue;
        KParams P = P0;
        P.rx0 = 0; P.ry0 = ya; P.rw = W; P.rh = yb - ya;
        P.tiles_x = (W + kTile - 1) / kTile;
        P.rank = 0; P.nranks = 1;
        P.out = s->d_frame; P.pitch = W; P.shard_mode = 2;
        P.fb_tw = tw; P.fb_th = th; P.fb_tx = tiles_x; P.fb_ty = tiles_y;
        P.fb_mtw = tw ? uint32_t(((1ull << 32) + tw - 1) / tw) : 0u;
        P.fb_mth = th ? uint32_t(((1ull << 32) + th - 1) / th) : 0u;
        // launches alternate between the two streams, so one launch's tail overlaps the next one's
        // start and its tile rows' copy-back overlaps the next launch's render
        hipStream_t sj = st[j & 1u];
        if ((rc = launch_render(s, f, P, P.tiles_x * ((P.rh + kTile - 1) / kTile), sj, false))) return rc;
        // the launch's tile rows are words [ya * W, yb * W) of the tile layout: ONE contiguous copy
        // (a copy per tile row cost ~14 us of launch overhead each, measured: 9 copies of a whole
        // frame 0.50 ms vs one 0.37, profiles/r04l_e2e_breakdown.json)
        const uint32_t b = s->nbands;
        if (!s->band_ev[b]) RT_HIP(hipEventCreateWithFlags(&s->band_ev[b], hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(h_tiles + size_t(ya) * W, s->d_frame + size_t(ya) * W, size_t(yb - ya) * W * 4,
                              hipMemcpyDeviceToHost, sj));
        RT_HIP(hipEventRecord(s->band_ev[b], sj));
        s->band_y1[b] = yb;
        s->nbands = b + 1;
    }
    // the frame is done when both streams are: join on the first one, whose event ev1 marks it
    RT_HIP(hipEventRecord(s->ev_t_join, st[1]));
    RT_HIP(hipStreamWaitEvent(st[0], s->ev_t_join, 0));
    RT_HIP(hipEventRecord(s->ev_own->ev, st[0]));
    s->ev_last = s->ev_own;
    s->ev_recorded = true;
    s->last_stream = st[0];
    // bands land per tile row but not in row order across the two streams: rt_frame_host_wait(y1)
    // needs every row below y1, so a band's wait covers the bands before it (events in row order)
    return RT_OK;
}

int rt_frame_host_wait(rt_scene *s, uint32_t y1)
{
    if (!s) return fail(RT_E_INVALID, "NULL argument");
    hipEvent_t ev[kMaxBands];
    uint32_t n = 0;
    {
        std::lock_guard<std::mutex> lk(s->mtx);
        if (s->nbands == 0) return fail(RT_E_INVALID, "no rt_render_frame_host in flight");
        // every band below y1 (rt_render_frame_host_tiled's bands land from two streams, so a later
        // band may be done before an earlier one); a finished event costs nothing to wait on
        while (n < s->nbands && (n == 0 || s->band_y1[n - 1] < y1)) { ev[n] = s->band_ev[n]; n++; }
    }
    for (uint32_t b = 0; b < n; b++)
        RT_HIP(hipEventSynchronize(ev[b]));     // events are only re-recorded by a later frame
    return RT_OK;
}

int rt_trace_samples(rt_scene *s, const rt_frame *f, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                     rt_sample_rec *out)
{
    if (!s || !out) return fail(RT_E_INVALID, "NULL argument");
    int rc = validate_frame(f);
    if (rc) return rc;
    if (w == 0 || h == 0 || x0 + w > f->width || y0 + h > f->height)
        return fail(RT_E_INVALID, "rectangle outside the frame");
    std::lock_guard<std::mutex> lk(s->mtx);
    if ((rc = ensure_device(s))) return rc;
    const uint32_t spp = std::max(1u, f->spp);
    if ((rc = prepare_samples(s, f, spp))) return rc;
    const uint64_t n64 = uint64_t(w) * h * spp;
    if (n64 > (1ull << 28)) return fail(RT_E_INVALID, "too many samples for one record call");
    const uint32_t n = uint32_t(n64);
    rt_sample_rec *d_rec = nullptr;
    RT_HIP(hipMalloc(&d_rec, sizeof(rt_sample_rec) * n));
    KParams P;
    frame_params(s, f, P);
    P.recs = d_rec;
    P.rec_x0 = x0; P.rec_y0 = y0; P.rec_w = w; P.rec_h = h;
    if (P.isect == RT_ISECT_RAY_MARCH && (f->kernel & RT_KERNEL_FLAG_EXHAUSTIVE)) P.isect += 0x100;
    if ((rc = flush_tables(s, s->stream)))
    {
        (void)hipFree(d_rec);
        return rc;
    }
    hipLaunchKernelGGL(trace_records_kernel(), dim3((n + kWG - 1) / kWG), dim3(kWG), 0, s->stream, P, n);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_rec, sizeof(rt_sample_rec) * n, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d_rec);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_trace_samples: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_wave_clocks(rt_scene *s, uint64_t *out, uint32_t max_items, uint32_t *n_items)
{
    if (!s || !n_items) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    int rc;
    if ((rc = ensure_device(s))) return rc;
    *n_items = s->clk_items;
    if (!out || !s->d_clk) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out, s->d_clk, sizeof(uint64_t) * 4 * std::min(max_items, s->clk_items), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_heavy_first(rt_scene *s, uint32_t *front, uint32_t *listed, uint32_t *epoch)
{
    if (!s || !front || !listed || !epoch) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    int rc;
    if ((rc = ensure_device(s))) return rc;
    *front = *listed = *epoch = 0;
    const HfCtx *c = nullptr;
    for (const HfCtx& h : s->hf)
        if (h.frames && (!c || h.used > c->used)) c = &h;
    if (!c) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    HfPlan pl;
    const uint32_t nv = c->pend ? c->pend : c->ver;        // the newest plan launched
    RT_HIP(hipMemcpy(&pl, c->plans + (nv & 1u), sizeof(pl), hipMemcpyDeviceToHost));
    *front = c->front;
    *listed = nv ? std::min(pl.cnt_hi + pl.cnt_lo, c->front) : 0u;
    *epoch = c->frames;
    return RT_OK;
}

int rt_debug_set_plan_delay(rt_scene *s, uint32_t us)
{
    if (!s) return fail(RT_E_INVALID, "NULL scene");
    if (us > 100000u) return fail(RT_E_INVALID, "plan delay must be <= 100000 us");
    std::lock_guard<std::mutex> lk(s->mtx);
    s->plan_delay = us * 100u;          // s_memrealtime ticks (100 MHz)
    return RT_OK;
}

int rt_debug_wide_items(rt_scene *s, uint32_t *count)
{
    if (!s || !count) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    const HfCtx *c = nullptr;
    for (const HfCtx& h : s->hf)
        if (h.wh_cnt && (!c || h.used > c->used)) c = &h;
    if (c) RT_HIP(hipDeviceSynchronize());
    *count = c ? c->wh_cnt[0] + kWavesPerWG * c->wh_cnt[1] : 0u;
    return RT_OK;
}

int rt_debug_wide_tiers(rt_scene *s, uint32_t *listed, uint32_t *lds)
{
    if (!s || !listed || !lds) return fail(RT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(s->mtx);
    int rc;
    if ((rc = ensure_device(s))) return rc;
    *listed = *lds = 0u;
    const HfCtx *c = nullptr;
    for (const HfCtx& h : s->hf)
        if (h.wh_cnt && (!c || h.used > c->used)) c = &h;
    const uint32_t nv = c ? (c->pend ? c->pend : c->ver) : 0u;     // the newest plan launched
    if (!nv) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    HfPlan pl;
    RT_HIP(hipMemcpy(&pl, c->plans + (nv & 1u), sizeof(pl), hipMemcpyDeviceToHost));
    *listed = std::min(pl.cnt_w, kWhMax);
    *lds = std::min(pl.cnt_l, kWhMax);
    return RT_OK;
}

int rt_debug_rcp_check(uint64_t *bad_by_exponent, int device)
{
    if (!bad_by_exponent) return fail(RT_E_INVALID, "NULL argument");
    RT_HIP(hipSetDevice(device));
    unsigned long long *d_bad = nullptr;
    RT_HIP(hipMalloc(&d_bad, 256 * sizeof(unsigned long long)));
    hipError_t e = hipMemset(d_bad, 0, 256 * sizeof(unsigned long long));
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(rcp_check_kernel(), dim3(8192), dim3(kWG), 0, nullptr, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(bad_by_exponent, d_bad, 256 * sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_rcp_check: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_gamma_check(uint64_t *mismatches, int device)
{
    if (!mismatches) return fail(RT_E_INVALID, "NULL argument");
    RT_HIP(hipSetDevice(device));
    unsigned long long *d_bad = nullptr;
    RT_HIP(hipMalloc(&d_bad, sizeof(unsigned long long)));
    hipError_t e = hipMemset(d_bad, 0, sizeof(unsigned long long));
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(gamma_check_kernel(), dim3(8192), dim3(kWG), 0, nullptr, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(mismatches, d_bad, sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_gamma_check: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_debug_primitives(int kind, const float *in, uint32_t n, float *out, int device)
{
    // kind 7 (DistancePointTri) reaches the device as pos + pad + the 24-float scene record
    static const uint32_t in_w[8] = { 18, 12, 23, 3, 11, 18, 18, 28 }, out_w[8] = { 8, 4, 6, 4, 3, 8, 8, 1 };
    if (kind < 0 || kind > 7 || !in || !out) return fail(RT_E_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    RT_HIP(hipSetDevice(device));
    std::vector<float> host_in;
    if (kind == 7)
    {
        host_in.resize(size_t(28) * n);
        for (uint32_t i = 0; i < n; i++)
        {
            const float *a = in + 12 * size_t(i);
            float *o = &host_in[28 * size_t(i)];
            o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = 0.0f;
            dist_record(a + 3, a + 6, a + 9, reinterpret_cast<float4 *>(o + 4));
        }
    }
    else
        host_in.assign(in, in + size_t(in_w[kind]) * n);
    if (kind == 2)   // camera.h:41-42 fov_xs is a host-side constant (double ::tan, hazard H5)
        for (uint32_t i = 0; i < n; i++)
        {
            const float hfov = host_in[23 * size_t(i) + 22] * float(0.0174532925);
            host_in[23 * size_t(i) + 22] = float(::tan(double(hfov / 2.0f)));
        }
    in = host_in.data();
    float *d_in = nullptr, *d_out = nullptr;
    RT_HIP(hipMalloc(&d_in, sizeof(float) * in_w[kind] * n));
    RT_HIP(hipMalloc(&d_out, sizeof(float) * out_w[kind] * n));
    hipError_t e = hipMemcpy(d_in, in, sizeof(float) * in_w[kind] * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
    {
        hipLaunchKernelGGL(primitives_kernel(), dim3((n + kWG - 1) / kWG), dim3(kWG), 0, nullptr, kind, d_in, n, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(float) * out_w[kind] * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_debug_primitives: ") + hipGetErrorString(e));
    return RT_OK;
}

} // extern "C"
