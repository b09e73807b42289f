/*
 * oracle/oracle_render.h — TEST INFRASTRUCTURE (oracle). Not part of the product.
 * CPU restatement of go-pbrt's hot path; see oracle_render.c.
 */
#ifndef ORACLE_RENDER_H
#define ORACLE_RENDER_H

#include "oracle_core.h"

#define ORACLE_FLAG_MIS_RAY 1   /* trace EstimateDirect's (no-op) BSDF-sampled ray */
#define ORACLE_FLAG_RANDOM_SAMPLER 2   /* sampler.RandomSampler (random.go) with spp = sampler_x * sampler_y */

typedef struct { uint64_t state, inc; } orc_pcg;
uint32_t orc_pcg_next(orc_pcg* r);
void orc_pcg_set_sequence(orc_pcg* r, uint64_t seed);
uint32_t orc_pcg_bounded(orc_pcg* r, uint32_t b);
double orc_pcg_float(orc_pcg* r);

typedef struct {
    const pbrt_scene_desc* scene;
    const pbrt_render_desc* rd;
    int flags;
    pbrt_distribution_desc dist;
    panic_ctx pc;
    int64_t cur_tile, cur_px, cur_py;
    int32_t cur_sample, cur_bounce;
    int unsupported;
    uint64_t paths, camera_samples, closest_rays, shadow_rays;
    const struct orc_mesh* mesh;   /* triangle meshes of the scene (extension), or NULL */
    int64_t* pixel_draws;          /* orc_tile_draws: PCG32 draws per pixel of the tile, or NULL */
} orc_ctx;

typedef struct {
    uint64_t tiles, paths, camera_samples, closest_rays, shadow_rays;
    uint64_t flops;   /* fp64 add/sub/mul/div/sqrt executed (liboracle_flops.so only) */
    int32_t panic_kind;
    int64_t panic_tile, panic_px, panic_py, panic_sample, panic_bounce;
    uint64_t flops_light;   /* the part of flops spent in UniformSampleOneLight + L += beta*Ld */
} orc_stats;

void orc_light_distribution(const pbrt_scene_desc* sc, const pbrt_render_desc* rd,
                            pbrt_distribution_desc* d);
int64_t orc_num_tiles(const pbrt_scene_desc* sc, const pbrt_render_desc* rd);
void orc_tile_bounds(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int64_t tile,
                     int64_t* x0, int64_t* y0, int64_t* x1, int64_t* y1);
void orc_film_tile_bounds(const pbrt_scene_desc* sc, int64_t x0, int64_t y0, int64_t x1, int64_t y1,
                          int64_t* px0, int64_t* py0, int64_t* px1, int64_t* py1);
int orc_render(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int n_threads, int flags,
               double* film_xyz, orc_stats* stats);
int orc_tile_draws(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int64_t tile, int64_t* out);
int orc_intersect(const pbrt_scene_desc* sc, const double* rays, size_t n, int closest, double* out);

#endif
