/*
 * rt_tracer.h -- C ABI of librt_tracer.so, the MI355X (gfx950) primary-ray tile tracer.
 *
 * This is the drop-in boundary for the reference's Renderer tile callback
 * (blitzcode/cpp-11-ray-trace-march-framework):
 *
 *   reference interface                                   replaced by
 *   ----------------------------------------------------  ---------------------------------
 *   Renderer::RenderTile(Tile&)      renderer.cpp:43-136   rt_render_frame_host + rt_frame_host_wait
 *                                                          (the Framebuffer's tiles, framebuffer.cpp:
 *                                                          59-92), rt_render_tiles, rt_render_frame_device
 *     per-pixel / per-sample loops   renderer.cpp:74-135   (one batched HIP launch per frame)
 *   GenerateRay (perspective)        camera.h:8-47         in-kernel, from rt_frame
 *   Grid::Intersect (3D-DDA)         grid.cpp:159-281      in-kernel, CSR cells from rt_grid_desc
 *   IntersectRayTri                  triangle.h:15-107     RT_TRI_MOLLER_TRUMBORE (default)
 *   IntersectRayTriBarycentric       triangle.h:210-226    RT_TRI_BARYCENTRIC
 *   shading, average, gamma, ToBGRA8 renderer.cpp:107-133, in-kernel resolve
 *                                    lin_alg.h:125-132
 *   Scene / Grid / Mesh data         scene.h:17-26,        rt_scene_create (uploaded once)
 *                                    grid.h:26-39, mesh.h:12-27
 *
 * Plain pointers and sizes only; every function returns 0 on success or a nonzero
 * RT_E* code, with a message retrievable through rt_last_error (thread-local).  No
 * exceptions cross the ABI.  The library owns device copies of the scene; it never
 * retains caller pointers past a call.  Calls on one rt_scene from several threads are
 * serialised internally (the reference's worker threads call RenderTile concurrently,
 * framebuffer.cpp:59-92).
 */
#ifndef RT_TRACER_H
#define RT_TRACER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 8   /* 8: rt_render_records_device, rt_scene_info batch counters; 7: rt_scene_info.box_words (box-run empty runs); 6: row-rotated shard deal */

enum rt_status {
    RT_OK = 0,
    RT_E_INVALID = 1,   /* bad argument / malformed scene */
    RT_E_HIP = 2,       /* HIP runtime error (message has the hipError_t string) */
    RT_E_NODEVICE = 3,  /* no gfx950 device visible */
    RT_E_RCCL = 4,
};

/* Mesh::Vertex (mesh.h:20-24) and Mesh::Triangle (mesh.h:12-18), same 24-byte layouts, so
 * a caller can pass &mesh->m_vertices[0] / &mesh->m_triangles[0] directly. */
typedef struct rt_vertex   { float p[3]; float n[3]; } rt_vertex;
typedef struct rt_triangle { uint32_t v0, v1, v2; float n[3]; } rt_triangle;

/* Grid state (grid.h:28-39).  Cells are CSR in GridIdx order (grid.h:41-42:
 * x + z*dims[0] + y*dims[0]*dims[2]); each cell's list keeps the reference's push order
 * (ascending triangle index, grid.cpp:65-122) -- the kernel's tie-break depends on it. */
typedef struct rt_grid_desc {
    uint32_t dims[3];
    float    aabb_min[3];
    float    aabb_max[3];
    float    cell_wdh;
    float    inv_cell_wdh;
    const uint32_t *cell_offsets;   /* dims[0]*dims[1]*dims[2] + 1 entries */
    const uint32_t *cell_tris;      /* cell_offsets[num_cells] entries */
} rt_grid_desc;

typedef struct rt_scene_desc {
    uint32_t           num_vertices;
    uint32_t           num_triangles;
    const rt_vertex   *vertices;
    const rt_triangle *triangles;
    rt_grid_desc       grid;
} rt_scene_desc;

enum rt_tri_test { RT_TRI_MOLLER_TRUMBORE = 0, RT_TRI_BARYCENTRIC = 1 };

/* The per-sample intersector of Renderer::RenderTile (renderer.cpp:103-105). */
enum rt_intersector {
    RT_ISECT_GRID = 0,         /* Grid::Intersect 3D-DDA (grid.cpp:159-281), the default */
    RT_ISECT_BRUTE_FORCE = 1,  /* Renderer::IntersectBruteForce (renderer.cpp:157-197); MT only */
    RT_ISECT_RAY_MARCH = 2,    /* Renderer::RayMarch over DistanceBruteForce (renderer.cpp:24-41,
                                  138-155).  Shaded by depth, t/3 (renderer.cpp:118): the live
                                  reference line would read the unset tri_idx/u/v */
};

enum rt_kernel {
    RT_KERNEL_AUTO = 0,        /* the fastest measured path for the frame: one lane per
                                  sample, distance-skipping 3D-DDA, per-camera-origin triangle records,
                                  wave-uniform cell lists on scalar loads, XCD-aware tile rows, and the
                                  heavy-first block order; for >= 2-rank shards of dense scenes at
                                  spp <= 16 the wide section (RT_KERNEL_FLAG_WIDE_HEAVY) */
    RT_KERNEL_LANES = 1,       /* the plain per-lane kernel: one lane per sample, the reference's walk
                                  and ray/triangle test cell by cell (A/B baseline) */
    RT_KERNEL_PIXEL_LOOP = 2,  /* one lane per pixel looping over its samples (any spp) */
    RT_KERNEL_COMPACT = 3,     /* AUTO's per-ray code in persistent waves with wavefront active-ray
                                  compaction: finished lanes are refilled with new samples by
                                  ballot + prefix count (grid intersector; else = LANES) */
    /* 4 was the persistent LDS-bitmap arm and 5 the all-wide kernel (both removed after losing
       their A/Bs; a frame naming them is rejected) */
    RT_KERNEL_KIND_MASK = 0x07,       /* the kernel kind above; the bits above it are flags */
    /* 0x80 was RT_KERNEL_FLAG_LDS_CELLS (long uniform lists staged through LDS; removed in round 4
       after losing on every scene; a frame naming it is rejected) */
    RT_KERNEL_FLAG_WIDE_HEAVY = 0x200, /* OR-able (AUTO, spp <= 16; AUTO's own choice for >= 2-rank
                                          shards of dense scenes): work items that earlier frames of
                                          the same launch shape measured as heavy are traced wide (16
                                          lanes per sample, 4 for spp 8-16) by a kernel on the scene's
                                          side stream, beside the one-lane-per-sample kernel (fork /
                                          join) */
    RT_KERNEL_FLAG_EXHAUSTIVE = 0x8000, /* OR-able, ray march: evaluate every triangle per step
                                           (no block culling; A/B arm, identical results) */
    RT_KERNEL_FLAG_WAVE_CLOCK = 0x400000, /* OR-able (AUTO), debug: record s_memtime {start, end} of
                                             every 64-sample work item (rt_debug_wave_clocks) */
    RT_KERNEL_FLAG_OVERLAP = 0x800000, /* OR-able (AUTO; in a batch: every frame of it): the caller
                                          lets this launch run beside the scene's previous launch when
                                          that one is on another stream (it writes other output
                                          buffers), so the previous frame's tail overlaps this one's
                                          start.  The library still orders the two when scene state
                                          changes between them (frame tables, camera origin, a new launch
                                          shape and its first two frames, a pending plan, a single frame's
                                          wide-section pair, wave clocks); at most two launches of a
                                          scene run at once. */
    RT_KERNEL_BUDGET_SHIFT = 24,      /* bits 24-30: RT_KERNEL_COMPACT: lanes that must be idle before
                                         a wave refills (1..64; 0 = default 48) */
    RT_KERNEL_BUDGET_MASK = 0x7F000000,
    RT_KERNEL_COMPACT_REFILL_SHIFT = RT_KERNEL_BUDGET_SHIFT,
    RT_KERNEL_COMPACT_REFILL_MASK = RT_KERNEL_BUDGET_MASK,
};
/* Removed A/B flags (they lost; a frame that sets one is rejected): 0x10 centre-out
   row order, 0x20 static block order, 0x40 16-lane wide kernel, 0x100 one-phase shards, bit 31
   the two-phase arm (replaced by RT_KERNEL_FLAG_WIDE_HEAVY in round 2), 0x1000 the wave-cooperative
   (ray, record) pair pass (round 3; it lost inside the batched step at every rank count).  The scheduling tunables
   are read once per scene from the environment at rt_scene_create (rt_scene_info). */

/* Per-frame parameters: what Renderer::RenderTile reads from the Scene and itself. */
typedef struct rt_frame {
    float        cam[16];         /* Matrix44f::m_mat row-major [4][4] (lin_alg.h:689), from
                                     Scene::GetCameraParameters (scene.h:17-18) */
    float        fov;             /* horizontal FOV in degrees (camera.h:39-45) */
    uint32_t     width, height;   /* Framebuffer m_width / m_height (framebuffer.h:29-30) */
    uint32_t     spp;             /* Renderer::m_sample_count (renderer.h:34); 0 -> 1 */
    const float *sample_offsets;  /* [spp][2] offsets in [-.5,.5], or NULL for the
                                     Hammersley table of renderer.cpp:49-60 */
    uint32_t     tri_test;        /* enum rt_tri_test */
    uint32_t     kernel;          /* enum rt_kernel */
    uint32_t     intersector;     /* enum rt_intersector (ABI version 2) */
} rt_frame;

/* Tile::GetPosition (framebuffer.h:41-42); buffer row stride = x1 - x0. */
typedef struct rt_tile { uint32_t x0, y0, x1, y1; } rt_tile;

/* Debug per-sample record (parity tests). */
typedef struct rt_sample_rec {
    uint32_t hit;     /* 1 = hit */
    uint32_t tri;     /* hit triangle (Grid::Intersect tri_idx), 0xFFFFFFFF on miss */
    uint32_t voxel;   /* GridIdx of the cell the hit was accepted in (last cell walked on a
                         miss), 0xFFFFFFFF when the ray misses the grid AABB and for the
                         brute-force and ray-march intersectors */
    uint32_t steps;   /* DDA iterations (cells visited); ray march: march steps */
    uint32_t tests;   /* ray/triangle tests executed; ray march: point/triangle distances */
    float    t, u, v; /* 0 on miss */
    float    r, g, b; /* this sample's colour contribution before averaging */
    uint32_t pad;
} rt_sample_rec;

typedef struct rt_scene rt_scene;

/* ---- lifetime ---------------------------------------------------------------------- */
int  rt_get_device_count(int *count);
int  rt_scene_create(const rt_scene_desc *desc, int device, rt_scene **out);
int  rt_scene_destroy(rt_scene *scene);
/* device bytes held by the scene (all arrays) */
int  rt_scene_device_bytes(const rt_scene *scene, uint64_t *bytes);

/* ---- grid build on the GPU (Grid::Grid, grid.cpp:12-154; grid.h:15) ----------------------
 * Voxelizes the mesh into the reference's uniform grid on `device`: the same AABB, cell size
 * and dims (grid.cpp:18-41), the same exact double tri/box test per candidate cell
 * (aabb.h:15-32), every cell's list in ascending triangle order (grid.cpp:119-122).  `out`
 * receives host arrays (cell_offsets, cell_tris) owned by the caller until rt_grid_free.
 * device_ms (optional): device time of the build kernels (HIP events). */
int  rt_grid_build(const rt_vertex *vertices, uint32_t num_vertices, const rt_triangle *triangles,
                   uint32_t num_triangles, uint32_t grid_res, int device, rt_grid_desc *out,
                   float *device_ms);
int  rt_grid_free(rt_grid_desc *grid);
/* Scene::Scene's mesh + Grid(mesh, grid_res) in one call: rt_grid_build + rt_scene_create. */
int  rt_scene_create_from_mesh(const rt_vertex *vertices, uint32_t num_vertices,
                               const rt_triangle *triangles, uint32_t num_triangles,
                               uint32_t grid_res, int device, rt_scene **out);

/* ---- rendering --------------------------------------------------------------------- */
/* Renders every listed tile in ONE batched launch (over the tiles' bounding box), copies
 * back and scatters into the caller's host buffers: tile_bufs[i][(x-x0) + (y-y0)*(x1-x0)]
 * = 0x00RRGGBB, exactly the words renderer.cpp:133 stores.  The copy-back runs in 8 row bands,
 * each band scattered while the next is in flight.  Synchronous. */
int  rt_render_tiles(rt_scene *scene, const rt_frame *frame, const rt_tile *tiles,
                     uint32_t n_tiles, uint32_t *const *tile_bufs);

/* Whole frame to host memory, asynchronously: one launch, then the D2H copy in row bands
 * [0, band_y1[0]), [band_y1[0], band_y1[1]), ... (strictly increasing, last = height; nbands <= 64,
 * 0 = one band).  h_bgra[y*width + x] = 0x00RRGGBB; page-locked memory from rt_host_alloc makes
 * the copy a DMA.  rt_frame_host_wait(scene, y1) blocks until rows [0, y1) have landed, so the
 * reference's tile workers (framebuffer.cpp:59-92) each copy their tile out of h_bgra as soon as
 * its tile row is there -- the drop-in for RenderTile's per-tile buffer writes, renderer.cpp:133.
 * Call the wait (for y1 = height at least once) before reusing h_bgra or the scene. */
int  rt_render_frame_host(rt_scene *scene, const rt_frame *frame, uint32_t *h_bgra,
                          const uint32_t *band_y1, uint32_t nbands);
int  rt_frame_host_wait(rt_scene *scene, uint32_t y1);
/* The drop-in's zero-copy form: the frame lands in h_tiles laid out as the tile buffers of the
 * reference's Framebuffer (framebuffer.cpp:94-122, framebuffer.h:41-45): a tiles_x x tiles_y grid,
 * tile (c, r) = pixels [c*tw, c < tiles_x-1 ? (c+1)*tw : width) x [r*th, r < tiles_y-1 ? (r+1)*th :
 * height) with tw = width / tiles_x, th = height / tiles_y; the tiles' buffers back to back in tile
 * order c + r*tiles_x, each row-major at its own width (so buffer (c, r) starts at word
 * r*th*width + th_r*c*tw, th_r = that row's height).  A Framebuffer whose tile buffers are those
 * views needs no copy at all: the kernels write this layout (renderer.cpp:133's buf[x + y*tileW]),
 * and consecutive tile rows are contiguous.  The frame is rendered in `nlaunch` launches of
 * consecutive tile rows alternating over two streams, each followed by ONE D2H copy of its rows,
 * so one launch's copy overlaps the next launch's render (the drop-in uses 1: a whole-frame launch
 * keeps the heavy-first order).  Asynchronous; rt_frame_host_wait(scene, y1) as above (a launch's
 * rows are one band).  h_tiles: width*height words of page-locked memory (rt_host_alloc). */
int  rt_render_frame_host_tiled(rt_scene *scene, const rt_frame *frame, uint32_t *h_tiles, uint32_t tiles_x,
                                uint32_t tiles_y, uint32_t nlaunch);
/* Page-locked host memory (hipHostMalloc) for rt_render_frame_host. */
int  rt_host_alloc(size_t bytes, void **out);
int  rt_host_free(void *p);

/* Device-resident frame: d_bgra[y*width + x] on the caller's HIP stream (NULL = default
 * stream).  Asynchronous: never waits on the host.  Allocates only for the first frame of a
 * launch shape (AUTO's heavy-first state) or a changed sample table, so a hipGraph captured after
 * one warm-up frame replays without allocations; a replay keeps the heavy-first order of the frame
 * before the capture (the pixels never depend on the order). */
int  rt_render_frame_device(rt_scene *scene, const rt_frame *frame, uint32_t *d_bgra,
                            void *hip_stream);

/* Multi-GPU sharding: the frame is cut into 16x16 pixel tiles; tile (tx, ty) gets the
 * row-rotated number t' = ty*tiles_x + (tx + 3*ty) % tiles_x (tiles_x = ceil(width/16); no
 * rotation when nranks == 1) and is owned by rank t' % nranks as its local tile t' / nranks.  The
 * rotation spreads a compact heavy region over every rank (plain t % nranks deals whole tile
 * columns to a rank when nranks divides tiles_x).  A rank renders its tiles compactly into d_shard
 * (rt_shard_elems words, tile-local row-major, 256 words per tile); after an all-gather of
 * the equal-sized shards, rt_unshard_device rebuilds the frame. */
int  rt_shard_elems(uint32_t width, uint32_t height, uint32_t nranks, uint64_t *elems);
int  rt_render_shard_device(rt_scene *scene, const rt_frame *frame, uint32_t rank,
                            uint32_t nranks, uint32_t *d_shard, void *hip_stream);
int  rt_unshard_device(uint32_t width, uint32_t height, uint32_t nranks,
                       const uint32_t *d_gathered, uint32_t *d_bgra, void *hip_stream);

/* rt_render_frame_device (nranks == 1, d_out = the W*H frame) or rt_render_shard_device
 * (nranks > 1, d_out = the rank's shard) that ALSO stores every traced sample's hit triangle --
 * Grid::Intersect's tri_idx (grid.cpp:258-266, renderer.cpp:105), 0xFFFFFFFF on a miss -- into
 * d_hits[(y*width + x)*spp + s] (frame-absolute, so the shards of all ranks fill one array).  Same
 * launch path, same heavy-first / wide-section state and the same kernel binaries as the frame and
 * shard entry points: the store sits after the walk behind a null test of the pointer, which is
 * NULL in the plain calls (the parity tests pin the benchmarked kernel's hit IDs through here). */
int  rt_render_hits_device(rt_scene *scene, const rt_frame *frame, uint32_t rank, uint32_t nranks,
                           uint32_t *d_out, uint32_t *d_hits, void *hip_stream);

/* Several frames -- of one or more scenes on one device -- in ONE launch (at most 6 per launch;
 * longer lists take ceil(n / 6) launches of near-equal size, 10 frames as 5 + 5): frame i renders into d_outs[i] exactly as
 * rt_render_frame_device (nranks == 1) or rt_render_shard_device (nranks > 1: rank's shard) would,
 * and, when d_hits and d_hits[i] are non-NULL, stores per-sample hit IDs as rt_render_hits_device.
 * The frames' blocks share one grid, so one frame's tail overlaps the others' work and AUTO's
 * heavy-first order (and, for dense shards, the wide section) ranks the blocks of all of them; the
 * batch keeps its own heavy-first state.  Frames that cannot share a launch (another kernel kind
 * or flag, different size / spp, scenes on different devices or outside AUTO's full traversal
 * variant) take one launch each.  Asynchronous on hip_stream; each launch's kernel time lands in
 * the rt_kernel_times ring of its first frame's scene. */
int  rt_render_batch_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                            uint32_t nranks, uint32_t *const *d_outs, uint32_t *const *d_hits,
                            void *hip_stream);

/* The benchmarked launch path with per-sample records (the parity pin of the product kernels'
 * walk): as rt_render_frame_device / rt_render_shard_device (n == 1) or rt_render_batch_device
 * (n >= 2; one batched launch where the frames can share it), and in addition every traced sample
 * of frame i inside rects[i] (frame pixels [x0, x1) x [y0, y1)) stores its record
 * d_recs[i][((y - y0) * (x1 - x0) + (x - x0)) * spp + s]: hit, Grid::Intersect's tri_idx, the GridIdx
 * of the accepted cell (of the last cell walked on a miss; 0xFFFFFFFF when the ray misses the grid;
 * grid.cpp:243-271), t, u, v (grid.cpp:258-266) and the sample's colour (renderer.cpp:107-121).
 * steps / tests are 0xFFFFFFFF: the product walks skip proven-empty cells and do not count
 * (rt_trace_samples reports them).  Same kernels and the same walk code as the plain entry points:
 * the stores sit after the walk behind a null test of the record pointer.  AUTO frames only (grid
 * intersector, IntersectRayTri). */
int  rt_render_records_device(rt_scene *const *scenes, const rt_frame *frames, uint32_t n, uint32_t rank,
                              uint32_t nranks, uint32_t *const *d_outs, const rt_tile *rects,
                              rt_sample_rec *const *d_recs, void *hip_stream);

/* Render-kernel time of the last timed rendering call on this scene (ms): the HIP events on the
 * launch stream immediately around its render kernel(s), as rt_kernel_times.  Waits for them. */
int  rt_last_kernel_ms(rt_scene *scene, float *ms);
/* Render-kernel durations (ms, HIP events recorded on the launch stream immediately around the
 * render kernel(s) of a launch -- not the heavy-first planning kernels), for the timed launches
 * since the previous call, oldest first, at most max_n and at most the last 64.  Waits for them.
 * A launch is timed when it is the n-th, 2n-th, ... of the scene (rt_scene_set_timing, default
 * n = 8): a timed event pair costs ~10 us of device time per launch. */
int  rt_kernel_times(rt_scene *scene, float *ms, uint32_t max_n, uint32_t *n);
/* Times every `every`-th launch from the next one on (1: every launch, 0: none). */
int  rt_scene_set_timing(rt_scene *scene, uint32_t every);

/* ---- parity / debug ---------------------------------------------------------------- */
/* Per-sample records for pixels [x0,x0+w) x [y0,y0+h), order (y, x, sample).  Synchronous. */
int  rt_trace_samples(rt_scene *scene, const rt_frame *frame, uint32_t x0, uint32_t y0,
                      uint32_t w, uint32_t h, rt_sample_rec *out);

/* Device evaluation of the primitives for known-answer tests (input layouts as the
 * tests/golden/kat_*.f32 records):  0 ray/tri (18 in, 8 out), 1 ray/aabb (12 in, 4 out),
 * 2 generate ray (23 in, 6 out), 3 gamma+pack (3 in, 4 out), 4 shade (11 in, 3 out),
 * 5 the branch-free ray/tri forms the traversal uses (18 in, 8 out; t,u,v valid on hits),
 * 6 the wave-gated forms: pre-gated MT, gated MT (18 in, 8 out; t,u,v valid on hits),
 * 7 DistancePointTri through the ray-march kernel's per-triangle record (12 in: pos, v0, v1,
 * v2; 1 out). */
int  rt_debug_primitives(int kind, const float *in, uint32_t n, float *out, int device);
/* Exhaustive check of the kernels' Newton-refined reciprocal (rt_device.h rcp_nr) against the
   correctly rounded 1.0f / x for all 2^32 - 2^24 finite nonzero floats; bad_by_exponent[256]
   receives the mismatch count per biased exponent. */
int  rt_debug_rcp_check(uint64_t *bad_by_exponent, int device);
/* Exhaustive check of the resolve's gamma: for every non-negative float x (+inf included) the
   packed byte of the hardware square root (rtd::gamma_fast) against that of the correctly rounded
   sqrtf; *mismatches receives the count (0 would let the kernels use the hardware form; MI355X
   reports 80, so the resolve keeps sqrtf). */
int  rt_debug_gamma_check(uint64_t *mismatches, int device);
/* Per 64-sample work item of the last RT_KERNEL_FLAG_WAVE_CLOCK launch on this scene, in launch
   item order, four words: {start, end} shader clock (s_memtime: per clock domain, for
   durations), records tested in wave-uniform list loops (bits 0-31; bits 32-35: the wave's XCD;
   bits 36-63: low 28 bits of the 100 MHz s_memrealtime at its start), iterations of the
   per-lane list loop (bits 0-31; bits 32-59: s_memrealtime at its end).  out holds 4 x max_items words; *n_items = how many
   items the launch wrote. */
int  rt_debug_wave_clocks(rt_scene *s, uint64_t *out, uint32_t max_items, uint32_t *n_items);

/* AUTO's heavy-first order for the most recent launch shape on this scene: *front = blocks the
   front section holds, *listed = blocks the last frame listed for the next one (heavy waves found),
   *epoch = frames rendered with this shape.  Synchronises the device. */
int rt_debug_heavy_first(rt_scene *s, uint32_t *front, uint32_t *listed, uint32_t *epoch);
/* RT_KERNEL_FLAG_WIDE_HEAVY: the wide section's waves for the items the newest plan of the most
   recent wide-section launch shape lists (16 or 4 per item of the lane-split tier, 4 per item -- one
   256-lane workgroup -- of the LDS tier).  Synchronises the device. */
int rt_debug_wide_items(rt_scene *s, uint32_t *count);
/* Tests only: every later heavy-first plan kernel (k_hf_plan) of this scene first idles `us`
   microseconds (<= 100000; 0: off, the default), so a frame that could read a plan's buffers while
   the plan writes them -- the ordering HfCtx::fence exists for -- always
   overlaps it.  Frames stay exact: the library orders every reader after the plan. */
int rt_debug_set_plan_delay(rt_scene *s, uint32_t us);
/* The same plan's items: *listed = all of them, *lds = those the LDS tier renders (the launch shape's
   section runs it: all of them, else 0; kVarLdsSplit, RT_WH_LDS).  Synchronises the device. */
int rt_debug_wide_tiers(rt_scene *s, uint32_t *listed, uint32_t *lds);

/* What rt_scene_create chose for a scene, and the scheduling tunables it read once from the
   environment (RT_HF_FLOOR, RT_HF_MIN_BLOCKS, RT_WH_FLOOR, RT_WH_ALPHA16, RT_WH_ALPHA16_N2,
   RT_WH_AUTO_REFS, RT_WH_LDS, ...): never re-read per launch. */
typedef struct rt_scene_info {
    uint32_t octant_words;      /* 1: 8 ray-octant copies of the cell words (AUTO's empty runs);
                                   0: one L-inf word per cell (above the size cap) */
    uint32_t packed_cells;      /* cell ranges packed into one word per cell */
    uint32_t rcp_safe, pack_ok; /* Newton 1/det and packed remaining-cell counts in range */
    uint32_t max_cell_refs;
    uint32_t hf_floor, hf_min_blocks, wh_floor, wh_alpha16, wh_auto_refs;
    uint32_t wh_fused;          /* batched shards of >= 4 ranks: the wide section leads the batch
                                   kernel's grid (else its own kernel on a side stream) */
    uint32_t hf_contexts;       /* heavy-first launch shapes remembered per scene */
    uint64_t hf_evictions;      /* launch shapes evicted (each restarts its heavy-first state) */
    uint64_t device_bytes;
    uint32_t box_words;         /* 1: AUTO's empty runs use the 24 box-run word copies (octant x major
                                   axis); 0: none (references >= 2^20 or above the size cap: AUTO then
                                   walks without the packed counts and empty runs) */
    uint32_t wh_alpha16_n2;     /* RT_WH_ALPHA16_N2: the wide threshold at a rank of 2 of a batched step */
    uint32_t wh_lds;            /* RT_WH_LDS: bit log2 N (3: N >= 8) -- a rank of N's wide section runs the LDS tier */
    uint64_t batch_launches;    /* rt_render_batch_device chunks led by this scene (frames[0]) that ran as
                                   ONE launch ... */
    uint64_t batch_fallbacks;   /* ... and that fell back to one launch per frame (frames that cannot
                                   share a launch): the batch's kernel time then covers only frame 0 */
} rt_scene_info;
int  rt_scene_info_get(rt_scene *scene, rt_scene_info *out);

/* SHA-256 prefix (16 hex digits) of the kernel sources this library was compiled from, baked in
   at build time (csrc/Makefile): counter files are matched against the LOADED library. */
int  rt_build_hash(char *buf, size_t len);

/* Hammersley table the library uses when rt_frame.sample_offsets is NULL. */
int  rt_sample_table(uint32_t spp, float *out_xy);

int  rt_last_error(char *buf, size_t len);
int  rt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_TRACER_H */
