/*
 * oracle/oracle_scene.h — TEST INFRASTRUCTURE (oracle). Not part of the product.
 * Independent restatement of go-pbrt's host-side scene construction.
 */
#ifndef ORACLE_SCENE_H
#define ORACLE_SCENE_H

#include "oracle_core.h"

#define ORC_MAX 64
typedef struct {
    int n_shapes, n_materials, n_prims_in, n_nodes, n_lights;
    pbrt_shape_desc shapes[ORC_MAX];
    pbrt_material_desc materials[ORC_MAX];
    pbrt_primitive_desc prims_in[ORC_MAX];   /* construction order      */
    pbrt_primitive_desc prims[ORC_MAX];      /* BVH order (orderedPrims) */
    int order[ORC_MAX];
    pbrt_bvh_node nodes[2 * ORC_MAX];
    pbrt_light_desc lights[ORC_MAX];
    pbrt_camera_desc camera;
    pbrt_film_desc film;
    double world_min[3], world_max[3];
    int n_meshes;                 /* extension: the height field (0 or 1) */
    pbrt_mesh_desc mesh;
    float* mesh_p;
    int32_t* mesh_idx;
} orc_scene;

pbrt_matrix4x4 orc_m_mul(const pbrt_matrix4x4* m, const pbrt_matrix4x4* o);
int orc_m_inverse(const pbrt_matrix4x4* m, pbrt_matrix4x4* out);
pbrt_transform orc_translate(double x, double y, double z);
pbrt_transform orc_scale(double x, double y, double z);
pbrt_transform orc_rotate(int axis, double degrees);
pbrt_transform orc_xf_mul(const pbrt_transform* a, const pbrt_transform* b);
int orc_look_at(v3 pos, v3 look, v3 up, pbrt_transform* out);
pbrt_transform orc_perspective(double fov, double n, double f);
pbrt_shape_desc orc_sphere(pbrt_transform o2w, int rev, double radius, double zmin, double zmax, double phimax);
pbrt_shape_desc orc_disk(pbrt_transform o2w, double height, double radius, double inner, double phimax);
int orc_add_shape(orc_scene* sc, pbrt_shape_desc s);
int orc_add_material(orc_scene* sc, pbrt_material_desc m);
int orc_scene_finalize(orc_scene* sc, int max_prims);
orc_scene* orc_scene_readme(int64_t w, int64_t h);
orc_scene* orc_scene_cornell(int64_t w, int64_t h);
orc_scene* orc_scene_heightfield(int64_t w, int64_t h, int quads, uint64_t seed);
orc_scene* orc_scene_readme_glass(int64_t w, int64_t h, int special, int mirror);
void orc_scene_desc(orc_scene* sc, pbrt_scene_desc* d);
void orc_scene_free(orc_scene* sc);

#endif
