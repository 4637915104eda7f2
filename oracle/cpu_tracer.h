/* oracle/cpu_tracer.h -- TEST INFRASTRUCTURE ONLY.
 *
 * C-ABI of liboracle_tracer.so: a plain C++11 CPU restatement ("port") of the reference's
 * per-sample tile path, used as
 *   (1) the parity checker for the HIP path in tests/ and __graft_entry__.smoke(), and
 *   (2) bench.py's cpu_baseline leg (kind "port") on the GPU box, where the reference
 *       itself (/root/reference) does not exist.
 * It is pinned against oracle/_ref/refdriver (the reference's own code) by the fixtures
 * under tests/golden/ (see tests/test_oracle_golden.py).  The product never links it.
 */
#ifndef ORACLE_CPU_TRACER_H
#define ORACLE_CPU_TRACER_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

typedef struct orc_info {
    uint32_t scene_id, num_vertices, num_triangles;
    float    fov;
    float    cam[16];
    uint32_t dims[3];
    float    aabb_min[3], aabb_max[3];
    float    cell_wdh, inv_cell_wdh;
    uint32_t num_cells, num_refs, max_refs_per_cell;
    double   grid_build_s;
} orc_info;

/* Per-sample record; identical layout to rt_sample_rec in include/rt_tracer.h. */
typedef struct orc_rec {
    uint32_t hit;     /* 1 = hit */
    uint32_t tri;     /* hit triangle index, 0xFFFFFFFF on miss */
    uint32_t voxel;   /* GridIdx of the cell the hit was accepted in / last cell walked, 0xFFFFFFFF if the grid was missed */
    uint32_t steps;   /* DDA loop iterations (cells visited) */
    uint32_t tests;   /* ray/triangle tests executed */
    float    t, u, v; /* 0 on miss */
    float    r, g, b; /* this sample's pre-average colour contribution */
    uint32_t pad;
} orc_rec;

orc_scene *orc_scene_load(const char *path);          /* NULL on error */
void       orc_scene_free(orc_scene *s);
int        orc_scene_info(const orc_scene *s, orc_info *out);
/* offsets: num_cells+1 u32, refs: num_refs u32 (GridIdx order, ascending tri per cell) */
int        orc_scene_csr(const orc_scene *s, uint32_t *offsets, uint32_t *refs);
/* mesh arrays as in the file: vertices [nv][6] f32, triangles [nt][6] (3 u32 + 3 f32) */
int        orc_scene_mesh(const orc_scene *s, float *vertices, uint32_t *triangles);

/* tri_test: 0 = IntersectRayTri (Moller-Trumbore, default), 1 = IntersectRayTriBarycentric,
 * OR'ed with (intersector << 8): 0 = Grid::Intersect, 1 = Renderer::IntersectBruteForce
 * (renderer.cpp:157-197), 2 = Renderer::RayMarch (renderer.cpp:24-41, shaded by depth t/3). */
/* Full frame through the restated 12x9 std::thread tile pool; out_bgra W*H row-major.
 * hit_ids (optional, W*H*spp): tri index per sample or 0xFFFFFFFF.  seconds = pool span. */
int orc_render(const orc_scene *s, uint32_t W, uint32_t H, uint32_t spp, uint32_t tri_test,
               uint32_t nthreads, uint32_t *out_bgra, uint32_t *hit_ids, double *seconds);
/* orc_render (Grid::Intersect, Moller-Trumbore) from another camera: cam16 = the view matrix as
 * Scene::GetCameraParameters returns it, fov in degrees. */
int orc_render_cam(const orc_scene *s, uint32_t W, uint32_t H, uint32_t spp, const float *cam16, float fov,
                   uint32_t *out_bgra, uint32_t *hit_ids);
/* Per-sample records for the pixel rectangle [x0,x0+w) x [y0,y0+h), order (y, x, s). */
int orc_trace_samples(const orc_scene *s, uint32_t W, uint32_t H, uint32_t spp, uint32_t tri_test,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, orc_rec *out);

/* Primitive restatements, vectorised over n records (layouts = tests/golden/kat_*.f32). */
void orc_hammersley(uint32_t spp, float *out_xy);
void orc_kat_ray_tri(const float *in18, uint32_t n, float *out8);
void orc_kat_ray_aabb(const float *in12, uint32_t n, float *out4);
void orc_kat_genray(const float *in23, uint32_t n, float *out6);
void orc_kat_bgra8(const float *in3, uint32_t n, float *out4);
void orc_kat_shade(const float *in11, uint32_t n, float *out3);
void orc_kat_dist(const float *in12, uint32_t n, float *out1);   /* triangle.h:174-198 */

#ifdef __cplusplus
}
#endif
#endif
