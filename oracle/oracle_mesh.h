/*
 * oracle/oracle_mesh.h — TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * CPU restatement of the triangle-mesh extension of include/pbrt_gpu.h
 * (BASELINE configs D/E; go-pbrt itself has no triangle shape):
 *  - the triangle test is pbrt-v3's Triangle::Intersect (watertight ray /
 *    triangle test of Woop, Benthin and Wald; pbrt-v3 shapes/triangle.cpp,
 *    "Physically Based Rendering" 3rd ed. §3.6.2-3.6.3) in float64 after exact
 *    widening of the float32 vertices, error bounds with epsilon = 2^-53;
 *  - its own acceleration structure (a median-split BVH built here), which
 *    shares nothing with the device's LBVH: the closest hit is defined as the
 *    smallest (t, global triangle index) over every triangle the ray hits
 *    with t below TMax, so any correct traversal returns the same triangle.
 * Parity of this extension is "unpinned": there is no reference arithmetic to
 * pin it to; the device is checked against this file.
 */
#ifndef ORACLE_MESH_H
#define ORACLE_MESH_H

#include "oracle_core.h"

typedef struct orc_mesh orc_mesh;

typedef struct {
    double t, b0, b1, b2;
    int32_t gid;        /* global triangle index (meshes concatenated)        */
    int32_t material;
    int32_t reverse;
    v3 p0, p1, p2;
} orc_tri_hit;

/* The scene's meshes with their BVH, built on first use and cached per
 * descriptor contents (NULL: the scene has no triangle). Thread-safe. */
const orc_mesh* orc_mesh_get(const pbrt_scene_desc* sc);

/* Closest triangle with t < tmax, or t == tmax and a smaller index than
 * best_gid (pass -1 when an analytic primitive already holds tmax: it wins
 * ties). Returns 1 and fills h on a hit. */
int orc_mesh_closest(const orc_mesh* m, const ray_t* r, double tmax, int32_t best_gid, orc_tri_hit* h);
/* Any triangle with 0 < t < r->tmax. */
int orc_mesh_any(const orc_mesh* m, const ray_t* r);

/* the triangle test alone (for tests): 1 = hit, t and barycentrics out */
int orc_triangle_hit(const double v[9], const ray_t* r, double* t, double* b0, double* b1, double* b2);

#endif
