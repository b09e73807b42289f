/*
 * pbrt_scene.h — host-side scene construction with go-pbrt semantics.
 *
 * The Go side of the integration computes transforms, shapes, lights and the
 * BVH with its own code and hands the result over as a pbrt_scene_desc
 * (include/pbrt_gpu.h). Where no Go toolchain exists (this repository's tests
 * and bench) these C-ABI functions restate the reference constructors with
 * identical arithmetic (Go math: pure-Go Cephes trig, Nextafter, Max/Min), so
 * the descriptor is bit-identical to what go-pbrt would build:
 *
 *   pbrt_translate/scale/rotate_{x,y,z}  <- pkg/pbrt/transform.go:347-424
 *   pbrt_transform_mul                   <- transform.go:179-184 (+ Matrix4x4.Mul :62-70)
 *   pbrt_matrix_inverse                  <- transform.go:72-142 (Gauss-Jordan)
 *   pbrt_look_at                         <- transform.go:453-486
 *   pbrt_perspective                     <- transform.go:492-502
 *   pbrt_make_sphere                     <- pkg/pbrt/sphere.go:19-36
 *   pbrt_make_disk                       <- pkg/shapes/disk.go:22-35
 *   pbrt_make_point_light                <- pkg/lights/point.go:19-30
 *   pbrt_make_distant_light              <- pkg/lights/distant.go:19-26 (+Preprocess :36-38 at build)
 *   pbrt_make_diffuse_area_light         <- pkg/lights/diffuse.go:17-25
 *   pbrt_sb_set_film                     <- pkg/pbrt/film.go:42-76
 *   pbrt_sb_set_perspective_camera       <- camera.go:106-165
 *   pbrt_sb_build                        <- accelerator.NewBVH (bvh.go:223-265, 272-411,
 *                                           632-651), pbrt.NewScene (scene.go:16-36),
 *                                           CreateLightSampleDistribution (lightdistribution.go)
 *   pbrt_scene_readme                    <- internal/render/server.go:29-164
 */
#ifndef PBRT_SCENE_H
#define PBRT_SCENE_H

#include "pbrt_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

void pbrt_translate(double x, double y, double z, pbrt_transform* out);
void pbrt_scale(double x, double y, double z, pbrt_transform* out);
void pbrt_rotate_x(double degrees, pbrt_transform* out);
void pbrt_rotate_y(double degrees, pbrt_transform* out);
void pbrt_rotate_z(double degrees, pbrt_transform* out);
void pbrt_transform_mul(const pbrt_transform* a, const pbrt_transform* b, pbrt_transform* out);
void pbrt_transform_inverse(const pbrt_transform* t, pbrt_transform* out);
/* Matrix4x4.Inverse; returns PBRT_E_INVALID for a singular matrix */
int pbrt_matrix_inverse(const pbrt_matrix4x4* m, pbrt_matrix4x4* out);
/* NewTransform(m): Matrix = m, MatrixInverse = Inverse(m) */
int pbrt_new_transform(const pbrt_matrix4x4* m, pbrt_transform* out);
int pbrt_look_at(const double pos[3], const double look[3], const double up[3], pbrt_transform* out);
void pbrt_perspective(double fov, double n, double f, pbrt_transform* out);
/* Transform.TransformPoint / TransformRay (for tests of the Go arithmetic) */
void pbrt_transform_point(const pbrt_transform* t, const double p[3], const double perr[3],
                          double out_p[3], double out_err[3]);
void pbrt_transform_ray(const pbrt_transform* t, const double o[3], const double d[3],
                        double out_o[3], double out_d[3]);

void pbrt_make_sphere(const pbrt_transform* o2w, int reverse_orientation, double radius,
                      double z_min, double z_max, double phi_max, pbrt_shape_desc* out);
void pbrt_make_disk(const pbrt_transform* o2w, double height, double radius,
                    double inner_radius, double phi_max, pbrt_shape_desc* out);
void pbrt_make_matte_constant(double r, double g, double b, double sigma, pbrt_material_desc* out);
void pbrt_make_matte_checkerboard(const double vs[3], const double vt[3], double ds, double dt,
                                  const double tex1[3], const double tex2[3], double sigma,
                                  pbrt_material_desc* out);
/* sampler.NewRandomSampler(ns, seed) (pkg/sampler/random.go:12-57): sets the
 * sampler fields of rd (sampler_x = ns, sampler_y = 1, n_dims = 0, jitter = 0),
 * under which the Stratified path consumes exactly the RandomSampler's stream */
void pbrt_random_sampler(int32_t samples_per_pixel, pbrt_render_desc* rd);
/* pkg/materials/mirror.go:9-32 (NewMirror's Kr is 0.9) */
void pbrt_make_mirror(const double kr[3], pbrt_material_desc* out);
/* pkg/materials/glass.go:15-75 with constant textures (see pbrt_material_desc) */
void pbrt_make_glass(const double kr[3], const double kt[3], double u_roughness, double v_roughness,
                     double eta, pbrt_material_desc* out);
void pbrt_make_point_light(const pbrt_transform* l2w, const double I[3], pbrt_light_desc* out);
void pbrt_make_distant_light(const pbrt_transform* l2w, const double L[3], const double w[3],
                             pbrt_light_desc* out);
void pbrt_make_diffuse_area_light(const double Lemit[3], int shape_index, int two_sided,
                                  pbrt_light_desc* out);

/* Scene builder: owns the arrays a pbrt_scene_desc points to. */
typedef struct pbrt_scene_builder pbrt_scene_builder;
pbrt_scene_builder* pbrt_sb_create(void);
void pbrt_sb_destroy(pbrt_scene_builder* b);
int pbrt_sb_add_shape(pbrt_scene_builder* b, const pbrt_shape_desc* s);        /* -> index */
int pbrt_sb_add_material(pbrt_scene_builder* b, const pbrt_material_desc* m);  /* -> index */
int pbrt_sb_add_primitive(pbrt_scene_builder* b, const pbrt_primitive_desc* p);/* -> index */
int pbrt_sb_add_light(pbrt_scene_builder* b, const pbrt_light_desc* l);        /* -> index */
/* Extension (configs D/E): a triangle mesh, copied; p = n_vertices*3 float32
 * world-space positions, indices = n_triangles*3. Returns the mesh index. */
int pbrt_sb_add_mesh(pbrt_scene_builder* b, int32_t n_vertices, const float* p, int32_t n_triangles,
                     const int32_t* indices, int32_t material, int32_t reverse_orientation);
/* film.go:42-76 with a BoxFilter of the given radius */
int pbrt_sb_set_film(pbrt_scene_builder* b, int64_t res_x, int64_t res_y, const double crop[4],
                     double filter_rx, double filter_ry, double max_sample_luminance);
/* NewPerspectiveCamera(cam2world (non-animated), screenWindow{minx,miny,maxx,maxy}, ...);
 * must be called after pbrt_sb_set_film */
int pbrt_sb_set_perspective_camera(pbrt_scene_builder* b, const pbrt_transform* cam2world,
                                   const double screen_window[4], double shutter_open,
                                   double shutter_close, double lens_radius,
                                   double focal_distance, double fov);
/* NewBVH(prims, maxPrimsInNode, SplitSAH) + NewScene (light Preprocess).
 * The descriptor stays valid until the builder is destroyed. */
int pbrt_sb_build(pbrt_scene_builder* b, int max_prims_in_node, const pbrt_scene_desc** out);
/* BVHPrimitiveInfo order -> scene primitive index of BVH slot i (orderedPrims) */
int pbrt_sb_prim_order(const pbrt_scene_builder* b, int32_t* out, int n);
/* The light-sample distribution for a Path integrator strategy */
int pbrt_scene_light_distribution(const pbrt_scene_desc* s, int strategy,
                                  pbrt_distribution_desc* out);

/* Fixtures. */
/* internal/render/server.go:29-164, resolution w x h */
int pbrt_scene_readme(int64_t w, int64_t h, pbrt_scene_builder** out);
/* Cornell-style 6 disks + 2 spheres, built only from reference types */
int pbrt_scene_cornell(int64_t w, int64_t h, pbrt_scene_builder** out);

/* SURVEY §8(d) configs D/E (extension): a height field of quads x quads
 * cells (2 triangles each) over x, z in [-100, 200], height
 * y = 2 sin(.3x) cos(.2z) + 3 valuenoise(x, z; seed) (Go-math trig, vertices
 * rounded to float32), checkerboard Matte as the README floor, with the README
 * lights and camera (server.go:112-164). flags & PBRT_HF_README_SPHERES adds
 * the README's 21 spheres (a mixed analytic + mesh scene).
 * D: quads = 707 (999 698 triangles); E: quads = 2236 (9 999 392). */
#define PBRT_HF_README_SPHERES 1
int pbrt_scene_heightfield(int64_t w, int64_t h, int32_t quads, uint64_t seed, int32_t flags,
                           pbrt_scene_builder** out);

#ifdef __cplusplus
}
#endif
#endif /* PBRT_SCENE_H */
