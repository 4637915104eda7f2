/*
 * rt_host.h -- C ABI of librt_host.so, the C++11 host side above the GPU boundary.
 *
 * The reference keeps scene setup and grid construction on the host (scene.cpp:6-7,
 * grid.cpp:12-154) and so does this build: librt_host builds the uniform grid exactly as
 * Grid::Grid does (same AABB padding, 64 cells on the longest axis, Akenine-Moller tri/box
 * test in double, per-cell lists in ascending triangle order) but emits it directly as the
 * CSR arrays rt_scene_create (rt_tracer.h) uploads.  It also hosts the Framebuffer tile pool
 * (framebuffer.h) with a GPU RenderTile override -- see rth_framebuffer_*.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "rt_tracer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene rth_scene;

typedef struct rth_scene_stats {
    uint32_t scene_id;          /* from the .rtscene header (0xFFFFFFFF for in-memory meshes) */
    uint32_t num_vertices, num_triangles;
    uint32_t num_cells, num_refs, max_refs_per_cell, empty_cells;
    double   grid_build_s;
} rth_scene_stats;

/* Loads a post-setup scene (.rtscene written by the scene table; format in DESIGN.md) and
 * builds its grid (resolution 64, scene.cpp:7).  nthreads 0 = hardware_concurrency. */
int  rth_scene_load(const char *path, uint32_t nthreads, rth_scene **out);
/* Builds a scene from an in-memory Mesh (mesh.h layouts) and camera (scene.h:17-26). */
int  rth_scene_from_mesh(const rt_vertex *vertices, uint32_t num_vertices,
                         const rt_triangle *triangles, uint32_t num_triangles,
                         float fov, const float cam[16], uint32_t grid_res, uint32_t nthreads,
                         rth_scene **out);
void rth_scene_free(rth_scene *s);
int  rth_scene_set_id(rth_scene *s, uint32_t scene_id);
/* Writes the scene (mesh + camera) as .rtscene -- the binary scene cache rth_scene_load reads. */
int  rth_scene_save(const rth_scene *s, const char *path);

/* ---- Mesh ingestion and the built-in scene table --------------- */
typedef struct rth_mesh rth_mesh;
/* Mesh::Read (mesh.cpp:138-391): ASCII .dat, indexed or flat, "x y z [n [uv|rgb]]" vertices;
 * flip_winding swaps v0/v1 of every triangle.  Face normals = TriangleNormal; position-only
 * meshes copy them to the vertices. */
int  rth_mesh_read(const char *path, int flip_winding, rth_mesh **out);
int  rth_mesh_normalize_dimensions(rth_mesh *m);                  /* mesh.cpp:121-136 */
/* Mesh::Transform (mesh.cpp:96-119); mat = Matrix44f::m_mat row-major (translation in row 3) */
int  rth_mesh_transform(rth_mesh *m, const float mat[16]);
int  rth_mesh_add_quad(rth_mesh *m, const float quad[12]);          /* mesh.cpp:27-53 */
int  rth_mesh_add_mesh(rth_mesh *m, const rth_mesh *other);         /* mesh.cpp:55-70 */
/* Pointers into the mesh's own arrays (mesh.h layouts); valid while the mesh lives. */
int  rth_mesh_data(const rth_mesh *m, const rt_vertex **vertices, uint32_t *num_vertices,
                   const rt_triangle **triangles, uint32_t *num_triangles);
void rth_mesh_free(rth_mesh *m);
/* Matrix44f::BuildLookAtMatrix(eye, at, up = +Y) (lin_alg.h:431-467) -> cam[16] */
int  rth_look_at(const float eye[3], const float at[3], float cam[16]);
/* Application::InitializeScene (application.cpp:304-517): builds built-in scene 0..9 from the
 * reference's .dat meshes in mesh_dir (data_dir holds cornell_box_quads.txt, the Cornell box
 * geometry table) and its grid (resolution 64).  Bit-identical to the reference's own setup. */
int  rth_scene_table(uint32_t scene_id, const char *mesh_dir, const char *data_dir, uint32_t nthreads,
                     rth_scene **out);
/* Pointers into the scene's own host arrays; valid while the scene lives. */
int  rth_scene_desc(const rth_scene *s, rt_scene_desc *out);
int  rth_scene_camera(const rth_scene *s, float *fov, float cam[16]);
int  rth_scene_stats_get(const rth_scene *s, rth_scene_stats *out);

/* ---- Framebuffer (framebuffer.h:16-101) with the GPU RenderTile --------------------- */
typedef struct rth_framebuffer rth_framebuffer;
/* A headless Framebuffer whose RenderTile is served by librt_tracer: the first worker to
 * reach a frame renders ALL tiles in one batched launch (rt_render_tiles), every worker then
 * copies its own tile.  nthreads 0 = hardware_concurrency (framebuffer.cpp:11). */
int  rth_framebuffer_create(rt_scene *gpu_scene, const rth_scene *host_scene, uint32_t nthreads,
                            rth_framebuffer **out);
/* The same Framebuffer with its RenderTile served by several GPUs of this node -- the native
 * multi-GPU drop-in for the CPU pool of framebuffer.cpp:16-28, 59-92.  The scene is
 * replicated on every device (one rt_scene per entry of devices[], created here); per frame,
 * device i renders rank i's interleaved 16x16 tiles (rt_render_shard_device), ONE gather brings
 * every shard to devices[0], rt_unshard_device rebuilds the frame there and it is copied back in
 * tile-row bands to the tiles, as in rth_framebuffer_create.  When every device is listed once
 * the gather is RCCL: ncclCommInitAll over devices[] in this process, then one group of ncclSend
 * (every rank, rank 0 to itself) and ncclRecv (rank 0, one slice per rank) -- each peer's slice on
 * its own xGMI link.  A device listed more than once holds several logical ranks (a rehearsal of
 * N ranks on fewer GPUs): RCCL takes each device once, so those shards move by device copies.
 * RCCL (librccl.so.1) is loaded on first use; RCCL failures return RT_E_RCCL. */
int  rth_framebuffer_create_multi(const rth_scene *host_scene, const int *devices, uint32_t ndevices,
                                  uint32_t nthreads, rth_framebuffer **out);
enum rth_transport { RTH_TRANSPORT_NONE = 0, RTH_TRANSPORT_RCCL = 1, RTH_TRANSPORT_DEVICE_COPY = 2 };
/* How a framebuffer gathers its shards (enum rth_transport; NONE = one device) and its rank count. */
int  rth_framebuffer_transport(const rth_framebuffer *fb, uint32_t *transport, uint32_t *nranks);
void rth_framebuffer_free(rth_framebuffer *fb);
int  rth_framebuffer_set_sample_count(rth_framebuffer *fb, uint32_t spp);   /* renderer.cpp:18-22 */
int  rth_framebuffer_set_options(rth_framebuffer *fb, uint32_t tri_test, uint32_t kernel);
/* Which of Renderer::RenderTile's intersectors runs (renderer.cpp:103-105; enum rt_intersector). */
int  rth_framebuffer_set_intersector(rth_framebuffer *fb, uint32_t intersector);
/* Framebuffer::Resize (framebuffer.cpp:94-122): re-tiles 12x9 and renders; blocks until
 * the frame is complete.  seconds = pool start -> last tile (framebuffer.cpp:21, 86). */
int  rth_framebuffer_resize(rth_framebuffer *fb, uint32_t width, uint32_t height, double *seconds);
int  rth_framebuffer_start_rendering(rth_framebuffer *fb, double *seconds);  /* 'r' key */
/* The reference's own threading (framebuffer.cpp:124-134, 149-193): start_rendering_async returns
 * at once; the frame's tiles are delivered in the background (one delivery thread, or the worker
 * pool with RTH_POOL=1), each under its tile mutex with its dirty flag set (framebuffer.cpp:72-77).
 * draw is Framebuffer::Draw with the GL textures replaced by `display` (width*height words,
 * row-major; NULL: only count): every tile whose mutex is free (try_lock) and whose dirty flag is
 * set is copied into its rectangle and the flag reset; tiles_done = the frame's tiles delivered so
 * far (of 108).  wait joins the frame (what the next start / resize does first); seconds = start ->
 * last tile delivered. */
int  rth_framebuffer_start_rendering_async(rth_framebuffer *fb);
int  rth_framebuffer_draw(rth_framebuffer *fb, uint32_t *display, uint32_t *tiles_updated, uint32_t *tiles_done);
int  rth_framebuffer_wait(rth_framebuffer *fb, double *seconds);
/* Assembled frame (row 0 = bottom row, like SaveToBMP), width*height words. */
int  rth_framebuffer_read(const rth_framebuffer *fb, uint32_t *out_bgra);
/* Framebuffer::SaveToBMP -> WriteBitmap (bmp_writer.cpp:27-57): 32-bpp bottom-up BMP. */
int  rth_framebuffer_save_bmp(const rth_framebuffer *fb, const char *path);

int  rth_last_error(char *buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
