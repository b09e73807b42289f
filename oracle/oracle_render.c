/*
 * oracle/oracle_render.c — TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * Scalar C restatement of go-pbrt's render loop, integrators, BVH traversal,
 * shapes, lights, material/BSDF, sampler and film, following the reference
 * line by line (file:line cited per function). It consumes the same
 * pbrt_scene_desc the device path does and is used ONLY as the parity checker
 * (tests/, __graft_entry__.smoke) and as bench.py's cpu_baseline ("port").
 *
 * Deliberate deviations (none changes a film value), both undone by the
 * render flag PBRT_FLAG_PANIC_FIDELITY (or ORACLE_FLAG_MIS_RAY for the first):
 *  - EstimateDirect's BSDF-sampling (MIS) branch for the area light is
 *    skipped: in every scene the reference can build, no primitive carries an
 *    area light (primitive.go:33), so the branch always adds 0
 *    (integrator.go:132-192). It costs Sphere.PdfWi and one closest-hit ray,
 *    either of which can panic in EFloat.Check.
 *  - the closest-hit ray at bounces == maxDepth is not traced: path.go:66
 *    breaks there whether or not it hit (its traversal can panic too).
 *  - tile films are merged in tile-index order (the reference merges in
 *    goroutine completion order under a mutex, film.go:115-132).
 */
#include "oracle_render.h"
#include "oracle_mesh.h"

#ifdef ORACLE_COUNT_FLOPS
__thread uint64_t orc_flops;
static __thread uint64_t orc_flops_saved;
static __thread uint64_t orc_flops_light;
/* bracket reference computations whose results never reach an output (the
 * device path does not execute them) */
#define FL_OFF_BEGIN (orc_flops_saved = orc_flops)
#define FL_OFF_END (orc_flops = orc_flops_saved)
#else
#define FL_OFF_BEGIN ((void)0)
#define FL_OFF_END ((void)0)
#endif

#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ================================================================= sampler */
/* pkg/pbrt/rng.go:5-57 (PCG32 with the (rot+1)&31 output rotate, #1) */
#define PCG32_DEFAULT_STATE 0x853c49e6748fea9bULL
#define PCG32_MULT 0x5851f42d4c957f2dULL

/* PCG32 draws made by this thread (orc_tile_draws: per-pixel draw counts) */
static __thread uint64_t orc_draws;

uint32_t orc_pcg_next(orc_pcg* r) {
    orc_draws++;
    uint64_t old = r->state;
    r->state = old * PCG32_MULT + r->inc;
    uint32_t xorshifted = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xorshifted >> rot) | (xorshifted << ((rot + 1u) & 31u));
}
void orc_pcg_set_sequence(orc_pcg* r, uint64_t seed) {
    r->state = 0;
    r->inc = (seed << 1) | 1;
    orc_pcg_next(r);
    r->state += PCG32_DEFAULT_STATE;
    orc_pcg_next(r);
}
uint32_t orc_pcg_bounded(orc_pcg* r, uint32_t b) {
    uint32_t threshold = (~b + 1u) % b;
    for (;;) {
        uint32_t v = orc_pcg_next(r);
        if (v >= threshold) return v % b;
    }
}
double orc_pcg_float(orc_pcg* r) {
    FL(1);
    return go_min(GO_ONE_MINUS_EPSILON, (double)orc_pcg_next(r) * 2.3283064365386963e-10);
}

/* Stratified / PixelSampler (pkg/sampler/stratified.go, pixel.go, sampler.go) */
typedef struct {
    orc_pcg rng;
    int32_t xs, ys, spp, ndims, jitter;
    int32_t sample_index, cur1d, cur2d;
    double* s1d;   /* ndims * spp */
    int random;    /* RandomSampler (pkg/sampler/random.go:12-57) */
} sampler_t;

/* stratified.go:21-48 + sampling.go:101-145 */
static void sampler_start_pixel(sampler_t* s) {
    int32_t n = s->spp;
    if (s->random) {   /* random.go:41-55: no sample arrays are requested, so no draws */
        s->sample_index = 0;
        s->cur1d = s->cur2d = 0;
        return;
    }
    for (int d = 0; d < s->ndims; d++) {
        double* samp = s->s1d + (size_t)d * n;
        double inv = 1.0 / (double)n;
        FL(1 + 2 * n);
        for (int32_t i = 0; i < n; i++) {
            double delta = 0.5;
            if (s->jitter) delta = orc_pcg_float(&s->rng);
            samp[i] = go_min(((double)i + delta) * inv, GO_ONE_MINUS_EPSILON);
        }
        for (int32_t i = 0; i < n; i++) {
            int32_t other = i + (int32_t)orc_pcg_bounded(&s->rng, (uint32_t)(n - i));
            double t = samp[i]; samp[i] = samp[other]; samp[other] = t;
        }
    }
    for (int d = 0; d < s->ndims; d++) {
        /* StratifiedSample2D writes into a copy (sampling.go:122-124, #3): only
         * the jitter draws survive; every 2D value stays (0,0). */
        if (s->jitter)
            for (int32_t y = 0; y < s->ys; y++)
                for (int32_t x = 0; x < s->xs; x++) { orc_pcg_float(&s->rng); orc_pcg_float(&s->rng); }
        for (int32_t i = 0; i < n; i++) orc_pcg_bounded(&s->rng, (uint32_t)(n - i));
    }
    s->sample_index = 0;
    s->cur1d = s->cur2d = 0;
}
/* sampler.go:29-34 (pre-increment: sample 0 is never traced, #2) */
static int sampler_next_sample(sampler_t* s) {
    s->cur1d = s->cur2d = 0;
    s->sample_index += 1;
    return s->sample_index < s->spp;
}
/* pixel.go:60-69 */
static double sampler_get1d(sampler_t* s) {
    if (s->random) return orc_pcg_float(&s->rng);   /* random.go:21-23 */
    if (s->cur1d < s->ndims) {
        double v = s->s1d[(size_t)s->cur1d * s->spp + s->sample_index];
        s->cur1d++;
        return v;
    }
    return orc_pcg_float(&s->rng);
}
/* pixel.go:71-80 */
static v2 sampler_get2d(sampler_t* s) {
    v2 v;
    if (s->random) {   /* random.go:25-27: X then Y */
        v.x = orc_pcg_float(&s->rng);
        v.y = orc_pcg_float(&s->rng);
        return v;
    }
    if (s->cur2d < s->ndims) {
        s->cur2d++;
        v.x = 0.0; v.y = 0.0;
        return v;
    }
    v.x = orc_pcg_float(&s->rng);
    v.y = orc_pcg_float(&s->rng);
    return v;
}

/* ===================================================== surface interaction */
/* SurfaceInteraction with the reference's pointer sharing made explicit:
 * p/perr/n/wo/time live in the shared *interaction, sn..sdndv in the shared
 * *Shading (interaction.go:124-148); dpdu..dndv are SurfaceInteraction's own. */
typedef struct {
    v3 p, perr, n, wo;
    double time;
    double u, v;
    v3 dpdu, dpdv, dndu, dndv;
    v3 sn, sdpdu, sdpdv, sdndu, sdndv;
    int prim;
} si_t;

/* interaction.go:176-207 */
static si_t si_new_with(v3 p, v3 perr, double u, double v, v3 wo, v3 dpdu, v3 dpdv, v3 dndu,
                        v3 dndv, double time, int rev, int swaps) {
    si_t si;
    v3 n = v_normalized(v_cross(dpdu, dpdv));
    if (rev != swaps) n = v_muls(n, -1);
    si.p = p; si.perr = perr; si.time = time; si.wo = wo; si.n = n;
    si.u = u; si.v = v;
    si.dpdu = dpdu; si.dpdv = dpdv; si.dndu = dndu; si.dndv = dndv;
    si.sn = n; si.sdpdu = dpdu; si.sdpdv = dpdv; si.sdndu = dndu; si.sdndv = dndv;
    si.prim = -1;
    return si;
}

/* transform.go:302-334 TransformSurfaceInteraction. `full` = the caller
 * assigns the returned copy (`*si = *t.TransformSurfaceInteraction(si)`,
 * sphere.go:185, disk.go:110); otherwise only the shared interaction and
 * Shading objects change (primitive.go:104-106 discards the copy, #20). */
static void si_transform(const pbrt_transform* t, si_t* si, int full) {
    v3 perr2;
    v3 p2 = xf_point(t, si->p, si->perr, &perr2);
    si->p = p2; si->perr = perr2;
    si->n = v_normalized(xf_normal(t, si->n));
    si->wo = v_normalized(xf_vector(t, si->wo));
    if (full) {
        si->dpdu = xf_vector(t, si->dpdu);
        si->dpdv = xf_vector(t, si->dpdv);
        si->dndu = xf_normal(t, si->dndu);
        si->dndv = xf_normal(t, si->dndv);
    }
    si->sn = xf_normal(t, si->sn);
    si->sdpdu = xf_vector(t, si->sdpdu);
    si->sdpdv = xf_vector(t, si->sdpdv);
    si->sdndu = xf_normal(t, si->sdndu);
    si->sdndv = xf_normal(t, si->sdndv);
    si->sn = face_forward(si->sn, si->n);
}

/* =================================================================== shapes */
/* sphere.go:64-268: returns 0 miss, 1 hit. si may be NULL (IntersectP). */
static int sphere_intersect(panic_ctx* pc, const pbrt_shape_desc* s, const ray_t* r, si_t* si,
                            double* t_hit) {
    pbrt_transform w2o = xf_inverse(&s->object_to_world);
    v3 oerr, derr;
    ray_t ray = xf_ray(&w2o, r, &oerr, &derr);
    ef_t ox = ef_new(pc, ray.o.x, oerr.x);
    ef_t oy = ef_new(pc, ray.o.y, oerr.y);
    ef_t oz = ef_new(pc, ray.o.z, oerr.z);
    ef_t dx = ef_new(pc, ray.d.x, derr.x);
    ef_t dy = ef_new(pc, ray.d.y, derr.y);
    ef_t dz = ef_new(pc, ray.d.z, derr.z);
    ef_t a = ef_add(pc, ef_add(pc, ef_mul(pc, dx, dx), ef_mul(pc, dy, dy)), ef_mul(pc, dz, dz));
    ef_t b = ef_muls(pc, ef_add(pc, ef_add(pc, ef_mul(pc, dx, ox), ef_mul(pc, dy, oy)), ef_mul(pc, dz, oz)), 2.0);
    ef_t cc0 = ef_add(pc, ef_add(pc, ef_mul(pc, ox, ox), ef_mul(pc, oy, oy)), ef_mul(pc, oz, oz));
    ef_t c = ef_sub(pc, cc0, ef_muls(pc, ef_new(pc, s->radius, 0), s->radius));
    ef_t t0, t1;
    if (!ef_quadratic(pc, a, b, c, &t0, &t1)) return 0;
    if (t0.hi > ray.tmax || t1.lo <= 0) return 0;
    ef_t ts = t0;
    int used_t1 = 0;
    if (ts.lo <= 0) {
        ts = t1; used_t1 = 1;
        if (ts.hi > ray.tmax) return 0;
    }
    v3 ph = v_add(ray.o, v_muls(ray.d, ts.v));
    ph = v_muls(ph, s->radius / v_dist(ph, V3(0, 0, 0)));
    FL(1);
    if (ph.x == 0.0 && ph.y == 0.0) { ph.x = 1e-5 * s->radius; FL(1); }
    double phi = go_atan2(ph.y, ph.x);
    if (phi < 0.0) { phi += 2 * go_Pi; FL(2); }
    if ((s->z_min > -s->radius && ph.z < s->z_min) || (s->z_max < s->radius && ph.z > s->z_max) ||
        phi > s->phi_max) {
        if (used_t1) return 0;
        if (t1.hi > ray.tmax) return 0;
        ts = t1;
        ph = v_add(ray.o, v_muls(ray.d, ts.v));
        ph = v_muls(ph, s->radius / v_dist(ph, V3(0, 0, 0)));
        FL(1);
        if (ph.x == 0.0 && ph.y == 0.0) { ph.x = 1e-5 * s->radius; FL(1); }
        /* sphere.go:127 declares a NEW phi (`phi :=`): the outer phi is kept */
        double phi2 = go_atan2(ph.y, ph.x);
        if (phi2 < 0.0) { phi2 += 2 * go_Pi; FL(2); }
        if ((s->z_min > -s->radius && ph.z < s->z_min) || (s->z_max < s->radius && ph.z > s->z_max) ||
            phi2 > s->phi_max)
            return 0;
    }
    if (!si) {
        *t_hit = ts.v;
        return 1;
    }
    /* live part: reaches SurfaceInteraction fields the path reads */
    double theta = go_acos(go_clamp(ph.z / s->radius, -1, 1));
    double zr = sqrt(ph.x * ph.x + ph.y * ph.y);
    double izr = 1.0 / zr;
    double cos_phi = ph.x * izr, sin_phi = ph.y * izr;
    v3 dpdu = V3(-s->phi_max * ph.y, s->phi_max * ph.x, 0);
    double dth = s->theta_max - s->theta_min;
    v3 dpdv = v_muls(V3(ph.z * cos_phi, ph.z * sin_phi, -s->radius * go_sin(theta)), dth);
    FL(1 + 4 + 1 + 2 + 2 + 1 + 3);   /* ph.z/r, zr, 1/zr, cos/sin phi, dpdu, dth, dpdv comps */
    /* dead part: uv and dndu/dndv never reach an output (not executed on the device) */
    FL_OFF_BEGIN;
    double u = phi / s->phi_max;
    double v = (theta - s->theta_min) / (s->theta_max - s->theta_min);
    v3 d2uu = v_muls(V3(ph.x, ph.y, 0.0), -s->phi_max * s->phi_max);
    v3 d2uv = v_muls(V3(-sin_phi, cos_phi, 0.0), dth * ph.z * s->phi_max);
    v3 d2vv = v_muls(ph, -dth * dth);
    double E = v_dot(dpdu, dpdu), F = v_dot(dpdu, dpdv), G = v_dot(dpdv, dpdv);
    v3 N = v_normalized(v_cross(dpdu, dpdv));
    double e = v_dot(N, d2uu), f = v_dot(N, d2uv), g = v_dot(N, d2vv);
    double inv = 1.0 / (E * G - F * F);
    v3 dndu = v_add(v_muls(dpdu, (f * F - e * G) * inv), v_muls(dpdv, (e * F - f * E) * inv));
    v3 dndv = v_add(v_muls(dpdu, (g * F - f * G) * inv), v_muls(dpdv, (f * F - g * E) * inv));
    FL_OFF_END;
    v3 perr = v_muls(v_abs(ph), go_gamma(5));
    *si = si_new_with(ph, perr, u, v, v_muls(ray.d, -1), dpdu, dpdv, dndu, dndv, ray.time,
                      s->reverse_orientation, s->transform_swaps_handedness);
    si_transform(&s->object_to_world, si, 1);
    *t_hit = ts.v;
    return 1;
}

/* disk.go:64-159 */
static int disk_intersect(const pbrt_shape_desc* s, const ray_t* r, si_t* si, double* t_hit) {
    pbrt_transform w2o = xf_inverse(&s->object_to_world);
    ray_t ray = xf_ray(&w2o, r, NULL, NULL);
    if (ray.d.z == 0) return 0;
    double ts = (s->height - ray.o.z) / ray.d.z;
    FL(2);
    if (ts <= 0 || ts >= ray.tmax) return 0;
    v3 ph = v_add(ray.o, v_muls(ray.d, ts));
    double dist2 = ph.x * ph.x + ph.y * ph.y;
    FL(5);
    if (dist2 > s->radius * s->radius || dist2 < s->inner_radius * s->inner_radius) return 0;
    double phi = go_atan2(ph.y, ph.x);
    if (phi < 0) { phi += 2 * go_Pi; FL(2); }
    if (phi > s->phi_max) return 0;
    if (!si) {
        *t_hit = ts;
        return 1;
    }
    double rhit = sqrt(dist2);
    FL(1 + 2 + 2);   /* sqrt, dpdu comps, (r - inner)/rhit */
    FL_OFF_BEGIN;   /* uv: never reaches an output */
    double u = phi / s->phi_max;
    double omv = (rhit - s->inner_radius) / (s->radius - s->inner_radius);
    double v = 1 - omv;
    FL_OFF_END;
    v3 dpdu = V3(-s->phi_max * ph.y, s->phi_max * ph.x, 0);
    v3 dpdv = v_muls(V3(ph.x, ph.y, 0), (s->radius - s->inner_radius) / rhit);
    ph.z = s->height;
    *si = si_new_with(ph, V3(0, 0, 0), u, v, v_muls(ray.d, -1), dpdu, dpdv, V3(0, 0, 0), V3(0, 0, 0),
                      ray.time, s->reverse_orientation, s->transform_swaps_handedness);
    si_transform(&s->object_to_world, si, 1);
    *t_hit = ts;
    return 1;
}

static int shape_intersect(panic_ctx* pc, const pbrt_shape_desc* s, const ray_t* r, si_t* si,
                           double* t_hit) {
    if (s->type == PBRT_SHAPE_SPHERE) return sphere_intersect(pc, s, r, si, t_hit);
    return disk_intersect(s, r, si, t_hit);
}

/* ============================================================== primitives */
/* primitive.go:46-61 GeometricPrimitive.Intersect; :94-115 TransformedPrimitive */
static int prim_intersect(panic_ctx* pc, const pbrt_scene_desc* sc, int pi, ray_t* r, si_t* si) {
    const pbrt_primitive_desc* p = &sc->prims[pi];
    const pbrt_shape_desc* shape = &sc->shapes[p->shape];
    double t_hit;
    if (p->kind == PBRT_PRIM_TRANSFORMED) {
        pbrt_transform inv = xf_inverse(&p->prim_to_world);
        ray_t ray = xf_ray(&inv, r, NULL, NULL);
        if (!shape_intersect(pc, shape, &ray, si, &t_hit)) return 0;
        ray.tmax = t_hit;                 /* GeometricPrimitive.Intersect      */
        si->prim = pi;
        r->tmax = ray.tmax;
        if (!xf_is_identity(&p->prim_to_world)) si_transform(&p->prim_to_world, si, 0);
        return 1;
    }
    if (!shape_intersect(pc, shape, r, si, &t_hit)) return 0;
    r->tmax = t_hit;
    si->prim = pi;
    return 1;
}
static int prim_intersect_p(panic_ctx* pc, const pbrt_scene_desc* sc, int pi, const ray_t* r) {
    const pbrt_primitive_desc* p = &sc->prims[pi];
    const pbrt_shape_desc* shape = &sc->shapes[p->shape];
    double t_hit;
    if (p->kind == PBRT_PRIM_TRANSFORMED) {
        pbrt_transform inv = xf_inverse(&p->prim_to_world);
        ray_t ray = xf_ray(&inv, r, NULL, NULL);
        return shape_intersect(pc, shape, &ray, NULL, &t_hit);
    }
    return shape_intersect(pc, shape, r, NULL, &t_hit);
}

/* ===================================================================== BVH */
/* bounds.go:149-185 */
static int bounds_intersect_p(const pbrt_bvh_node* nd, const ray_t* r, v3 inv, const int neg[3]) {
    const double* bx[2] = {nd->bmin, nd->bmax};
    double tmin = (bx[neg[0]][0] - r->o.x) * inv.x;
    double tmax = (bx[1 - neg[0]][0] - r->o.x) * inv.x;
    double tymin = (bx[neg[1]][1] - r->o.y) * inv.y;
    double tymax = (bx[1 - neg[1]][1] - r->o.y) * inv.y;
    double robust = 1 + 2 * go_gamma(3);
    tmax *= robust;
    tymax *= robust;
    FL(8 + 2 + 2);
    if (tmin > tymax || tymin > tmax) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    double tzmin = (bx[neg[2]][2] - r->o.z) * inv.z;
    double tzmax = (bx[1 - neg[2]][2] - r->o.z) * inv.z;
    tzmax *= robust;
    FL(4 + 2 + 1);
    if (tmin > tzmax || tzmin > tmax) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return tmin < r->tmax && tmax > 0;
}

static void tri_si(const orc_tri_hit* h, const ray_t* r, si_t* si);

/* bvh.go:659-712, then the triangle meshes (extension, oracle_mesh.h) */
static int orc_bvh_intersect(orc_ctx* oc, ray_t* ray, si_t* si) {
    panic_ctx* pc = &oc->pc;
    const pbrt_scene_desc* sc = oc->scene;
    int hit = 0;
    if (sc->n_nodes == 0) goto meshes;
    v3 inv = V3(1 / ray->d.x, 1 / ray->d.y, 1 / ray->d.z);
    FL(3);
    int neg[3] = {inv.x < 0, inv.y < 0, inv.z < 0};
    uint64_t to_visit = 0, cur = 0;
    uint64_t stack[64];
    for (;;) {
        const pbrt_bvh_node* nd = &sc->nodes[cur];
        if (bounds_intersect_p(nd, ray, inv, neg)) {
            if (nd->n_prims > 0) {
                for (uint32_t i = 0; i < nd->n_prims; i++)
                    if (prim_intersect(pc, sc, (int)(nd->offset + i), ray, si)) hit = 1;
                if (to_visit == 0) break;
                cur = stack[--to_visit];
            } else {
                if (to_visit >= 64) { pc->kind = PBRT_PANIC_BVH_STACK; longjmp(pc->jb, 1); }
                if (neg[nd->axis]) {
                    stack[to_visit++] = cur + 1;
                    cur = nd->offset;
                } else {
                    stack[to_visit++] = nd->offset;
                    cur = cur + 1;
                }
            }
        } else {
            if (to_visit == 0) break;
            cur = stack[--to_visit];
        }
    }
meshes:
    if (oc->mesh) {
        orc_tri_hit h;
        /* a triangle at exactly TMax never wins: TMax is exclusive, and an
           analytic primitive that set it is tested first */
        if (orc_mesh_closest(oc->mesh, ray, ray->tmax, -1, &h)) {
            ray->tmax = h.t;
            tri_si(&h, ray, si);
            si->prim = sc->n_prims + h.gid;
            hit = 1;
        }
    }
    return hit;
}
/* bvh.go:713-765 */
static int orc_bvh_intersect_p_analytic(panic_ctx* pc, const pbrt_scene_desc* sc, const ray_t* ray) {
    if (sc->n_nodes == 0) return 0;
    v3 inv = V3(1 / ray->d.x, 1 / ray->d.y, 1 / ray->d.z);
    FL(3);
    int neg[3] = {inv.x < 0, inv.y < 0, inv.z < 0};
    uint64_t to_visit = 0, cur = 0;
    uint64_t stack[64];
    for (;;) {
        const pbrt_bvh_node* nd = &sc->nodes[cur];
        if (bounds_intersect_p(nd, ray, inv, neg)) {
            if (nd->n_prims > 0) {
                for (uint32_t i = 0; i < nd->n_prims; i++)
                    if (prim_intersect_p(pc, sc, (int)(nd->offset + i), ray)) return 1;
                if (to_visit == 0) return 0;
                cur = stack[--to_visit];
            } else {
                if (to_visit >= 64) { pc->kind = PBRT_PANIC_BVH_STACK; longjmp(pc->jb, 1); }
                if (neg[nd->axis]) {
                    stack[to_visit++] = cur + 1;
                    cur = nd->offset;
                } else {
                    stack[to_visit++] = nd->offset;
                    cur++;
                }
            }
        } else {
            if (to_visit == 0) return 0;
            cur = stack[--to_visit];
        }
    }
}

static int orc_bvh_intersect_p(orc_ctx* oc, const ray_t* ray) {
    if (orc_bvh_intersect_p_analytic(&oc->pc, oc->scene, ray)) return 1;
    return oc->mesh ? orc_mesh_any(oc->mesh, ray) : 0;
}

/* pbrt-v3 Triangle::Intersect, interaction part (default uv (0,0), (1,0),
 * (1,1); no shading normals), float64: the extension's SurfaceInteraction.
 * With those uv, dpdu = dp12 - dp02 and dpdv = -dp12 (the uv determinant is
 * exactly 1). wo is normalized as every go-pbrt interaction's (the shapes'
 * TransformSurfaceInteraction, transform.go:302-334). */
static void tri_si(const orc_tri_hit* h, const ray_t* r, si_t* si) {
    const double eps = 1.1102230246251565e-16;
    const double g7 = (7 * eps) / (1 - 7 * eps);
    FL(4);
    v3 dp02 = v_sub(h->p0, h->p2), dp12 = v_sub(h->p1, h->p2);
    v3 dpdu = v_sub(dp12, dp02);
    v3 dpdv = V3(-dp12.x, -dp12.y, -dp12.z);
    if (v_len2(v_cross(dpdu, dpdv)) == 0) {
        v3 ng = v_cross(v_sub(h->p2, h->p0), v_sub(h->p1, h->p0));
        v3 nn = v_normalized(ng), a, b;
        coordinate_system(nn, &a, &b);
        dpdu = a;
        dpdv = b;
    }
    v3 p = V3(h->b0 * h->p0.x + h->b1 * h->p1.x + h->b2 * h->p2.x,
              h->b0 * h->p0.y + h->b1 * h->p1.y + h->b2 * h->p2.y,
              h->b0 * h->p0.z + h->b1 * h->p1.z + h->b2 * h->p2.z);
    v3 err = V3(gm_abs(h->b0 * h->p0.x) + gm_abs(h->b1 * h->p1.x) + gm_abs(h->b2 * h->p2.x),
                gm_abs(h->b0 * h->p0.y) + gm_abs(h->b1 * h->p1.y) + gm_abs(h->b2 * h->p2.y),
                gm_abs(h->b0 * h->p0.z) + gm_abs(h->b1 * h->p1.z) + gm_abs(h->b2 * h->p2.z));
    FL(15 + 15);
    v3 n = v_normalized(v_cross(dp02, dp12));
    if (h->reverse) n = V3(-n.x, -n.y, -n.z);
    memset(si, 0, sizeof(*si));
    si->p = p;
    si->perr = v_muls(err, g7);
    si->n = n;
    si->wo = v_normalized(V3(-r->d.x, -r->d.y, -r->d.z));
    si->time = r->time;
    si->dpdu = dpdu; si->dpdv = dpdv;
    si->sn = n; si->sdpdu = dpdu; si->sdpdv = dpdv;
    si->prim = -1;
}

/* material of primitive index `prim`: scene prims, then the meshes' triangles */
static int prim_material(const pbrt_scene_desc* sc, int prim) {
    if (prim < sc->n_prims) return sc->prims[prim].material;
    int64_t g = prim - sc->n_prims;
    for (int mi = 0; mi < sc->n_meshes; mi++) {
        if (g < sc->meshes[mi].n_triangles) return sc->meshes[mi].material;
        g -= sc->meshes[mi].n_triangles;
    }
    return 0;
}

/* ========================================== BSDF (Matte, Mirror, Glass) */
/* kind of the BSDF's BxDFs: LambertianReflection (matte.go), SpecularReflection
 * with FresnelNoOp (mirror.go), FresnelSpecular (smooth glass with multiple
 * lobes allowed, glass.go:45-46 -- Path.Li passes allowMultipleLobes true),
 * rough glass's microfacet pair, OrenNayar, or SPEC_PAIR: smooth glass without
 * multiple lobes (DirectLighting.Li passes false, directlighting.go:76), i.e.
 * SpecularReflection(R, FresnelDielectric(1, eta)) if R is not black, then
 * SpecularTransmission(T, 1, eta, Radiance) if T is not black (glass.go:58-72);
 * mf_r / mf_t say which of the two exist, in that order. */
enum { BXDF_KIND_LAMBERT = 0, BXDF_KIND_SPEC_REFL = 1, BXDF_KIND_FRESNEL_SPEC = 2, BXDF_KIND_MICROFACET = 3,
       BXDF_KIND_OREN_NAYAR = 4, BXDF_KIND_SPEC_PAIR = 5 };
typedef struct {
    v3 ns, ng, ss, ts;
    int n_bxdfs;        /* 0 or 1; 0-2 for MICROFACET (mf_r + mf_t)           */
    int kind;           /* BXDF_KIND_*                                        */
    int mf_r, mf_t;     /* rough glass: MicrofacetReflection / -Transmission  */
    double ax, ay;      /* TrowbridgeReitz alphas (remapRoughness false)      */
    double on_a, on_b;  /* OrenNayar A, B (reflection.go:616-625)             */
    spec r, t;          /* Lambert/mirror R; glass R and T                    */
    double eta;         /* NewBSDF(si, eta): 1 for matte/mirror, index for glass */
} bsdf_t;

#define BXDF_REFLECTION 1
#define BXDF_TRANSMISSION 2
#define BXDF_DIFFUSE 4
#define BXDF_GLOSSY 8
#define BXDF_SPECULAR 16
#define BXDF_ALL 31
#define LAMBERT_TYPE (BXDF_REFLECTION | BXDF_DIFFUSE)
/* reflection.go:538-544: SpecularReflection is typed Reflection|Diffuse (not
 * Specular), so it counts as a non-specular component and its sampled type is 0 */
#define SPEC_REFL_TYPE (BXDF_REFLECTION | BXDF_DIFFUSE)
#define FRESNEL_SPEC_TYPE (BXDF_REFLECTION | BXDF_TRANSMISSION | BXDF_SPECULAR)   /* reflection.go:465-474 */
#define MF_REFL_TYPE (BXDF_REFLECTION | BXDF_GLOSSY)     /* reflection.go:670-677 */
#define MF_TRANS_TYPE (BXDF_TRANSMISSION | BXDF_GLOSSY)  /* reflection.go:738-747 */
#define SPEC_TRANS_TYPE (BXDF_TRANSMISSION | BXDF_SPECULAR)   /* reflection.go:405-415 */

static double inv_pi(void) { FL(1); return 1.0 / go_Pi; }   /* pkg/math InvPi = 1.0 / Pi */
static int matches_flags(int t, int flags) { return (t & flags) == t; }

/* matte.go:21-37 + reflection.go:128-140 + checkerboard.go:30-40; multi_lobes
 * is ComputeScatteringFunctions' allowMultipleLobes (interaction.go:217-223):
 * true for Path.Li (path.go:74), false for DirectLighting.Li (directlighting.go:76) */
static int material_bsdf(const pbrt_scene_desc* sc, const si_t* si, bsdf_t* b, int multi_lobes) {
    const pbrt_material_desc* m = &sc->materials[prim_material(sc, si->prim)];
    b->ns = si->sn;
    b->ng = si->n;
    b->ss = v_normalized(si->sdpdu);
    b->ts = v_cross(b->ns, b->ss);
    b->n_bxdfs = 0;
    b->kind = BXDF_KIND_LAMBERT;
    b->mf_r = b->mf_t = 0;
    b->eta = 1.0;
    if (m->type == PBRT_MAT_MIRROR) {   /* mirror.go:21-32 */
        spec r = S3(m->kr[0], m->kr[1], m->kr[2]);
        for (int i = 0; i < 3; i++) r.c[i] = go_clamp(r.c[i], 0, INFINITY);
        if (!s_is_black(r)) {
            b->n_bxdfs = 1;
            b->kind = BXDF_KIND_SPEC_REFL;
            b->r = r;
        }
        return 0;
    }
    if (m->type == PBRT_MAT_GLASS) {    /* glass.go:28-75 */
        spec R = S3(m->kr[0], m->kr[1], m->kr[2]), T = S3(m->kt[0], m->kt[1], m->kt[2]);
        for (int i = 0; i < 3; i++) {
            R.c[i] = go_clamp(R.c[i], 0, 1);
            T.c[i] = go_clamp(T.c[i], 0, 1);
        }
        b->eta = m->eta;
        if (s_is_black(R) && s_is_black(T)) return 0;
        if (!(m->u_roughness == 0 && m->v_roughness == 0)) {   /* glass.go:49-73 */
            b->kind = BXDF_KIND_MICROFACET;
            b->ax = m->u_roughness;
            b->ay = m->v_roughness;
            b->mf_r = !s_is_black(R);
            b->mf_t = !s_is_black(T);
            b->n_bxdfs = b->mf_r + b->mf_t;
            b->r = R;
            b->t = T;
            return 0;
        }
        b->r = R;
        b->t = T;
        if (!multi_lobes) {   /* glass.go:58-72 with isSpecular */
            b->kind = BXDF_KIND_SPEC_PAIR;
            b->mf_r = !s_is_black(R);
            b->mf_t = !s_is_black(T);
            b->n_bxdfs = b->mf_r + b->mf_t;
            return 0;
        }
        b->n_bxdfs = 1;
        b->kind = BXDF_KIND_FRESNEL_SPEC;
        return 0;
    }
    spec r;
    if (m->kd_type == PBRT_TEX_CHECKERBOARD2D) {
        double s = m->ds + v_dot(si->p, V3(m->vs[0], m->vs[1], m->vs[2]));
        double t = m->dt + v_dot(si->p, V3(m->vt[0], m->vt[1], m->vt[2]));
        int64_t k = go_f2i(floor(s) + floor(t));
        FL(3);
        if (k % 2 == 0) r = S3(m->tex1[0], m->tex1[1], m->tex1[2]);
        else r = S3(m->tex2[0], m->tex2[1], m->tex2[2]);
    } else {
        r = S3(m->kd[0], m->kd[1], m->kd[2]);
    }
    for (int i = 0; i < 3; i++) r.c[i] = go_clamp(r.c[i], 0, INFINITY);
    double sig = go_clamp(m->sigma, 0, 90);
    if (!s_is_black(r)) {
        b->n_bxdfs = 1;
        b->r = r;
        if (sig != 0) {   /* NewOrenNayar (reflection.go:616-625): B's sigma2 * 0.09 kept */
            double s = go_radians(sig);
            double s2 = s * s;
            b->kind = BXDF_KIND_OREN_NAYAR;
            b->on_a = 1.0 - (s2 / (2.0 * (s2 + 0.33)));
            b->on_b = 0.45 * s2 / (s2 * 0.09);
        }
    }
    return 0;
}
static v3 bsdf_w2l(const bsdf_t* b, v3 v) { return V3(v_dot(v, b->ss), v_dot(v, b->ts), v_dot(v, b->ns)); }

/* reflection.go:21-42 FrDielectric */
static double fr_dielectric(double cos_i, double eta_i, double eta_t) {
    cos_i = go_clamp(cos_i, -1, 1);
    if (!(cos_i > 0)) {
        double tmp = eta_i; eta_i = eta_t; eta_t = tmp;
        cos_i = gm_abs(cos_i);
    }
    double sin_i = sqrt(go_max(0, 1 - cos_i * cos_i));
    double sin_t = eta_i / eta_t * sin_i;
    if (sin_t >= 1) return 1;
    double cos_t = sqrt(go_max(0, 1 - sin_t * sin_t));
    double rparl = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    double rperp = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (rparl * rparl + rperp * rperp) / 2;
}
/* TrowbridgeReitz (microfacet.go:36-84, 117-124; sampleVisibleArea true) and the
 * trig helpers (reflection.go:48-100); D's e keeps the reference's
 * alphaX*alphaY under Cos2Phi */
static double cos2_theta(v3 w) { return w.z * w.z; }
static double sin2_theta(v3 w) { return go_max(0, 1 - cos2_theta(w)); }
static double sin_theta(v3 w) { return sqrt(sin2_theta(w)); }
static double tan_theta(v3 w) { return sin_theta(w) / w.z; }
static double tan2_theta(v3 w) { return sin2_theta(w) / cos2_theta(w); }
static double cos_phi(v3 w) { double st = sin_theta(w); return st == 0 ? 1 : go_clamp(w.x / st, -1, 1); }
static double sin_phi(v3 w) { double st = sin_theta(w); return st == 0 ? 0 : go_clamp(w.y / st, -1, 1); }
static double cos2_phi(v3 w) { return cos_phi(w) * cos_phi(w); }
static double sin2_phi(v3 w) { return sin_phi(w) * sin_phi(w); }
static double tr_d(const bsdf_t* b, v3 wh) {
    double t2 = tan2_theta(wh);
    if (isinf(t2)) return 0;
    double c4 = cos2_theta(wh) * cos2_theta(wh);
    double e = (cos2_phi(wh) / (b->ax * b->ay) + sin2_phi(wh) / (b->ay * b->ay)) * t2;
    return 1 / (go_Pi * b->ax * b->ay * c4 * (1 + e) * (1 + e));
}
static double tr_lambda(const bsdf_t* b, v3 w) {
    double at = gm_abs(tan_theta(w));
    if (isinf(at)) return 0;
    double alpha = sqrt(cos2_phi(w) * b->ax * b->ax + sin2_phi(w) * b->ay * b->ay);
    double a2t2 = (alpha * at) * (alpha * at);
    return (-1 + sqrt(1.0 + a2t2)) / 2;
}
static double tr_g1(const bsdf_t* b, v3 w) { return 1 / (1 + tr_lambda(b, w)); }
static double tr_g(const bsdf_t* b, v3 wo, v3 wi) { return 1 / (1 + tr_lambda(b, wo) + tr_lambda(b, wi)); }
static double tr_pdf(const bsdf_t* b, v3 wo, v3 wh) {   /* microfacet.go:26-32 */
    return tr_d(b, wh) * tr_g1(b, wo) * v_absdot(wo, wh) / gm_abs(wo.z);
}
/* MicrofacetReflection.F / .Pdf (reflection.go:690-704, 730-736), FresnelDielectric(1, eta) */
static spec mf_refl_f(const bsdf_t* b, v3 wo, v3 wi) {
    double c0 = gm_abs(wo.z), c1 = gm_abs(wi.z);
    v3 wh = v_add(wi, wo);
    if (c1 == 0 || c0 == 0) return S3(0, 0, 0);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return S3(0, 0, 0);
    wh = v_normalized(wh);
    double F = fr_dielectric(v_dot(wi, wh), 1.0, b->eta);
    return s_muls(s_mul(b->r, S3(F, F, F)), tr_d(b, wh) * tr_g(b, wo, wi) / (4 * c1 * c0));
}
static double mf_refl_pdf(const bsdf_t* b, v3 wo, v3 wi) {
    if (!(wo.z * wi.z > 0)) return 0;
    v3 wh = v_normalized(v_add(wo, wi));
    return tr_pdf(b, wo, wh) / (4 * v_dot(wo, wh));
}
/* MicrofacetTransmission.F / .Pdf (reflection.go:758-790, 820-835): F is 0 unless
 * wo and wi share a hemisphere (the reference's inverted test), wh is not
 * normalized, and NewMicrofacetTransmission leaves mode at its zero value (not
 * Radiance, material.go:10), so factor stays 1 */
static spec mf_trans_f(const bsdf_t* b, v3 wo, v3 wi) {
    if (!(wo.z * wi.z > 0)) return S3(0, 0, 0);
    double co = wo.z, ci = wi.z;
    if (ci == 0 || co == 0) return S3(0, 0, 0);
    double eta = wo.z > 0 ? 1.0 / b->eta : b->eta / 1.0;
    v3 wh = v_add(wo, v_muls(wi, eta));
    if (wh.z < 0) wh = v_muls(wh, -1);
    double F = fr_dielectric(v_dot(wo, wh), 1.0, b->eta);
    double sd = v_dot(wo, wh) * eta * v_dot(wi, wh);
    double factor = 1.0;
    spec a = s_mul(S3(1 - F, 1 - F, 1 - F), b->t);
    return s_muls(a, gm_abs(tr_d(b, wh) * tr_g(b, wo, wi) * eta * eta * v_absdot(wi, wh) * v_absdot(wo, wh) *
                            factor * factor / (ci * co * sd * sd)));
}
static double mf_trans_pdf(const bsdf_t* b, v3 wo, v3 wi) {
    if (wo.z * wi.z > 0) return 0;
    double eta = wo.z > 0 ? 1.0 / b->eta : b->eta / 1.0;
    v3 wh = v_add(wo, v_muls(wi, eta));
    double sd = v_dot(wo, wh) + eta * v_dot(wi, wh);
    double dwh = gm_abs((eta * eta * v_dot(wi, wh)) / (sd * sd));
    return tr_pdf(b, wo, wh) * dwh;
}
/* OrenNayar.F (reflection.go:627-652); the else branch's tanBeta keeps sinThetaO */
static spec oren_nayar_f(const bsdf_t* b, v3 wo, v3 wi) {
    double sin_i = sin_theta(wi), sin_o = sin_theta(wo);
    double max_cos = 0.0;
    if (sin_i > 1e-4 && sin_o > 1e-4) {
        double sp_i = sin_phi(wi), cp_i = cos_phi(wi), sp_o = sin_phi(wo), cp_o = cos_phi(wo);
        double d_cos = cp_i * cp_o + sp_i * sp_o;
        max_cos = go_max(0.0, d_cos);
    }
    double sin_alpha, tan_beta;
    if (gm_abs(wi.z) > gm_abs(wo.z)) {
        sin_alpha = sin_o;
        tan_beta = sin_o / gm_abs(wo.z);
    } else {
        sin_alpha = sin_i;
        tan_beta = sin_o / gm_abs(wo.z);
    }
    return s_muls(b->r, inv_pi() * (b->on_a + b->on_b * max_cos * sin_alpha * tan_beta));
}
/* reflection.go:169-186 */
static spec bsdf_f(const bsdf_t* b, v3 woW, v3 wiW, int flags) {
    FL_OFF_BEGIN;
    v3 wi = bsdf_w2l(b, wiW);   /* dead for Lambertian */
    FL_OFF_END;
    v3 wo = bsdf_w2l(b, woW);
    (void)wi;
    if (wo.z == 0.0) return S3(0, 0, 0);
    int reflect = v_dot(wiW, b->ng) * v_dot(woW, b->ng) > 0;
    FL(1);
    spec f = S3(0, 0, 0);
    if (b->kind == BXDF_KIND_MICROFACET) {
        if (b->mf_r && matches_flags(MF_REFL_TYPE, flags) && reflect) f = s_add(f, mf_refl_f(b, wo, wi));
        if (b->mf_t && matches_flags(MF_TRANS_TYPE, flags) && !reflect) f = s_add(f, mf_trans_f(b, wo, wi));
        return f;
    }
    if (b->kind == BXDF_KIND_SPEC_PAIR) {   /* both F are 0 (reflection.go:424-426, 553-555) */
        if (b->mf_r && matches_flags(SPEC_REFL_TYPE, flags) && reflect) f = s_add(f, S3(0, 0, 0));
        if (b->mf_t && matches_flags(SPEC_TRANS_TYPE, flags) && !reflect) f = s_add(f, S3(0, 0, 0));
        return f;
    }
    if (b->n_bxdfs && b->kind == BXDF_KIND_LAMBERT && matches_flags(LAMBERT_TYPE, flags) && reflect)
        f = s_add(f, s_muls(b->r, inv_pi()));
    else if (b->n_bxdfs && b->kind == BXDF_KIND_OREN_NAYAR && matches_flags(LAMBERT_TYPE, flags) && reflect)
        f = s_add(f, oren_nayar_f(b, wo, bsdf_w2l(b, wiW)));
    else if (b->n_bxdfs && b->kind != BXDF_KIND_LAMBERT)
        f = s_add(f, S3(0, 0, 0));   /* reflection.go:486-488, 553-555: F is 0 */
    return f;
}
/* reflection.go:343-348 */
static double lambert_pdf(v3 wo, v3 wi) {
    FL(1);
    if (wo.z * wi.z > 0) { FL(1); return gm_abs(wi.z) * inv_pi(); }
    return 0;
}
/* reflection.go:255-278 */
static double bsdf_pdf(const bsdf_t* b, v3 woW, v3 wiW, int flags) {
    if (b->n_bxdfs == 0) return 0;
    v3 wo = bsdf_w2l(b, woW);
    v3 wi = bsdf_w2l(b, wiW);
    if (wo.z == 0) return 0;
    double pdf = 0;
    int matching = 0;
    if (b->kind == BXDF_KIND_LAMBERT || b->kind == BXDF_KIND_OREN_NAYAR) {   /* both use pdf() :343-348 */
        if (matches_flags(LAMBERT_TYPE, flags)) { matching++; pdf += lambert_pdf(wo, wi); FL(1); }
    } else if (b->kind == BXDF_KIND_MICROFACET) {
        if (b->mf_r && matches_flags(MF_REFL_TYPE, flags)) { matching++; pdf += mf_refl_pdf(b, wo, wi); }
        if (b->mf_t && matches_flags(MF_TRANS_TYPE, flags)) { matching++; pdf += mf_trans_pdf(b, wo, wi); }
    } else if (b->kind == BXDF_KIND_SPEC_PAIR) {   /* both Pdf are 0 (reflection.go:461-463, 572-574) */
        if (b->mf_r && matches_flags(SPEC_REFL_TYPE, flags)) { matching++; pdf += 0.0; }
        if (b->mf_t && matches_flags(SPEC_TRANS_TYPE, flags)) { matching++; pdf += 0.0; }
    } else {   /* reflection.go:534-536, 572-574: Pdf is 0 */
        int ty = b->kind == BXDF_KIND_SPEC_REFL ? SPEC_REFL_TYPE : FRESNEL_SPEC_TYPE;
        if (matches_flags(ty, flags)) { matching++; pdf += 0.0; }
    }
    if (matching <= 0) return 0;
    FL(1);
    return pdf / (double)matching;
}
/* sampling.go:173-198 */
static v2 concentric_sample_disk(v2 u) {
    v2 uo = {u.x * 2.0 - 1, u.y * 2.0 - 1};
    FL(4);
    v2 z = {0, 0};
    if (uo.x == 0 && uo.y == 0) return z;
    double theta, r;
    if (gm_abs(uo.x) > gm_abs(uo.y)) {
        r = uo.x;
        theta = (go_Pi / 4.0) * (uo.y / uo.x);
        FL(3);
    } else {
        r = uo.y;
        theta = (go_Pi / 2.0) - (go_Pi / 4.0) * (uo.x / uo.y);
        FL(5);
    }
    v2 p = {go_cos(theta) * r, go_sin(theta) * r};
    FL(2);
    return p;
}
static v3 cosine_sample_hemisphere(v2 u) {
    v2 d = concentric_sample_disk(u);
    double z = sqrt(go_max(0.0, 1.0 - d.x * d.x - d.y * d.y));
    FL(5);
    return V3(d.x, d.y, z);
}
double oracle_fr_dielectric(double cos_i, double eta_i, double eta_t) { return fr_dielectric(cos_i, eta_i, eta_t); }
/* FresnelSpecular.SampleF (reflection.go:489-524), incl. its (etaT / etaT)
 * radiance scale; FaceForward (geometry.go:111-116) + Refract (:106-118) */
static spec fresnel_specular_sample(const bsdf_t* b, v3 wo, v2 u, v3* wi, double* pdf, int* type) {
    double F = fr_dielectric(wo.z, 1.0, b->eta);
    if (u.x < F) {
        *wi = V3(-wo.x, -wo.y, wo.z);
        *pdf = F;
        *type = BXDF_SPECULAR | BXDF_REFLECTION;
        return s_divs(s_muls(b->r, F), gm_abs(wi->z));
    }
    double eta_i, eta_t;
    if (wo.z > 0) { eta_i = 1.0; eta_t = b->eta; } else { eta_i = b->eta; eta_t = 1.0; }
    v3 n = V3(0, 0, 1);
    if (v_dot(n, wo) < 0.0) n = v_muls(n, -1);
    double eta = eta_i / eta_t;
    double cos_i = v_dot(n, wo);
    double sin2_i = go_max(0, 1 - cos_i * cos_i);
    double sin2_t = eta * eta * sin2_i;
    if (sin2_t >= 1) { *pdf = 0; *type = 0; return S3(0, 0, 0); }
    double cos_t = sqrt(1 - sin2_t);
    *wi = v_add(v_muls(wo, -eta), v_muls(n, eta * cos_i - cos_t));
    spec ft = s_muls(b->t, 1 - F);
    ft = s_muls(ft, (eta_i * eta_i) / (eta_t / eta_t));   /* mode == Radiance */
    *pdf = 1 - F;
    *type = BXDF_SPECULAR | BXDF_TRANSMISSION;
    return s_divs(ft, gm_abs(wi->z));
}
/* reflection.go:188-253; returns the LOCAL-frame wi (#7) and the sampled type;
 * type -1: the reference panics (rough glass, PBRT_PANIC_NIL_DEREF) */
static spec bsdf_sample_f_t(const bsdf_t* b, v3 woW, v2 u, int t, v3* wi_out, double* pdf_out, int* type_out) {
    const int ty = (b->kind == BXDF_KIND_LAMBERT || b->kind == BXDF_KIND_OREN_NAYAR) ? LAMBERT_TYPE
                 : b->kind == BXDF_KIND_SPEC_REFL ? SPEC_REFL_TYPE : FRESNEL_SPEC_TYPE;
    int matching = (b->n_bxdfs && matches_flags(ty, t)) ? 1 : 0;
    if (b->kind == BXDF_KIND_MICROFACET)
        matching = (b->mf_r && matches_flags(MF_REFL_TYPE, t)) + (b->mf_t && matches_flags(MF_TRANS_TYPE, t));
    if (b->kind == BXDF_KIND_SPEC_PAIR)
        matching = (b->mf_r && matches_flags(SPEC_REFL_TYPE, t)) + (b->mf_t && matches_flags(SPEC_TRANS_TYPE, t));
    *wi_out = V3(0, 0, 0);
    *pdf_out = 0;
    *type_out = 0;
    if (matching == 0) return S3(0, 0, 0);
    double comp = go_min(floor(u.x * (double)matching), (double)matching - 1);
    v2 ur = {go_min(u.x * (double)matching - comp, GO_ONE_MINUS_EPSILON), u.y};
    FL(4);
    v3 wo = bsdf_w2l(b, woW);
    if (wo.z == 0.0) return S3(0, 0, 0);
    if (b->kind == BXDF_KIND_MICROFACET) {   /* SampleWH's nil wh reaches Reflect/Refract */
        *type_out = -1;
        return S3(0, 0, 0);
    }
    if (b->kind == BXDF_KIND_SPEC_REFL) {   /* reflection.go:557-562 (FresnelNoOp) */
        v3 wi = V3(-wo.x, -wo.y, wo.z);
        spec f = s_divs(s_mul(S3(1, 1, 1), b->r), gm_abs(wi.z));
        *wi_out = wi;
        *pdf_out = 1.0;
        return f;
    }
    if (b->kind == BXDF_KIND_SPEC_PAIR) {
        /* the comp-th matching BxDF, in BSDF order (reflection.go:194-206) */
        const int refl_ok = b->mf_r && matches_flags(SPEC_REFL_TYPE, t);
        const int pick_refl = refl_ok && comp == 0.0;
        v3 wi;
        spec f;
        if (pick_refl) {   /* SpecularReflection.SampleF with FresnelDielectric(1, eta) (reflection.go:557-562) */
            wi = V3(-wo.x, -wo.y, wo.z);
            double F = fr_dielectric(wi.z, 1.0, b->eta);
            f = s_divs(s_mul(S3(F, F, F), b->r), gm_abs(wi.z));
        } else {           /* SpecularTransmission.SampleF (reflection.go:428-451) */
            double eta_i, eta_t;
            if (wo.z > 0) { eta_i = 1.0; eta_t = b->eta; } else { eta_i = b->eta; eta_t = 1.0; }
            v3 n = V3(0, 0, 1);
            if (v_dot(n, wo) < 0.0) n = v_muls(n, -1);   /* FaceForward (geometry.go:111-116) */
            double eta = eta_i / eta_t;                   /* Refract (reflection.go:106-118) */
            double cos_i = v_dot(n, wo);
            double sin2_i = go_max(0, 1 - cos_i * cos_i);
            double sin2_t = eta * eta * sin2_i;
            if (sin2_t >= 1) return S3(0, 0, 0);          /* pdf 0 (reflection.go:440-442, 226-228) */
            double cos_t = sqrt(1 - sin2_t);
            wi = v_add(v_muls(wo, -eta), v_muls(n, eta * cos_i - cos_t));
            double F = fr_dielectric(wi.z, 1.0, b->eta);  /* t.fresnel = FresnelDielectric(etaA, etaB) */
            spec ft = s_mul(b->t, S3(1 - F, 1 - F, 1 - F));
            ft = s_muls(ft, (eta_i * eta_i) / (eta_t * eta_t));   /* mode == Radiance (directlighting.go:76) */
            f = s_divs(ft, gm_abs(wi.z));
        }
        double pdf = 1.0;   /* both SampleF return pdf 1 and sampled type 0 */
        if (matching > 1) {
            /* reflection.go:233-250: a non-specular pick (SpecularReflection is typed
             * Reflection|Diffuse) adds the other's Pdf (0) and re-evaluates f as the
             * sum of the matching F (all 0); either pick divides pdf by matching */
            if (pick_refl) pdf += 0.0;
            pdf /= (double)matching;
            if (pick_refl) f = S3(0, 0, 0);
        }
        *wi_out = wi;
        *pdf_out = pdf;
        *type_out = 0;
        return f;
    }
    if (b->kind == BXDF_KIND_FRESNEL_SPEC) {
        v3 wi; double pdf; int st;
        spec f = fresnel_specular_sample(b, wo, ur, &wi, &pdf, &st);
        if (pdf == 0.0) return S3(0, 0, 0);
        *wi_out = wi;
        *pdf_out = pdf;
        *type_out = st;
        return f;
    }
    /* reflection.go:305-314 sampleF */
    v3 wi = cosine_sample_hemisphere(ur);
    if (wo.z < 0) { wi.z *= -1; FL(1); }
    double pdf = lambert_pdf(wo, wi);
    spec f = b->kind == BXDF_KIND_OREN_NAYAR ? oren_nayar_f(b, wo, wi) : s_muls(b->r, inv_pi());
    if (pdf == 0.0) return S3(0, 0, 0);
    *wi_out = wi;
    *pdf_out = pdf;
    return f;
}
static spec bsdf_sample_f(const bsdf_t* b, v3 woW, v2 u, int t, v3* wi_out, double* pdf_out) {
    int ty;
    return bsdf_sample_f_t(b, woW, u, t, wi_out, pdf_out, &ty);
}

/* ================================================================== lights */
typedef struct { v3 p, perr, n; double time; } intr_t;

/* sphere.go:270-285 */
static intr_t sphere_sample(const pbrt_shape_desc* s, v2 u, double* pdf) {
    /* sampling.go:158-163 UniformSampleSphere */
    double z = 1.0 - 2.0 * u.x;
    double rr = sqrt(go_max(0, 1 - z * z));
    double phi = 2 * go_Pi * u.y;
    FL(2 + 3 + 2 + 2 + 1);   /* z, rr, phi, rr*cos/sin, radius/dist */
    v3 pobj = v_muls(V3(rr * go_cos(phi), rr * go_sin(phi), z), s->radius);
    intr_t it;
    it.n = v_normalized(xf_normal(&s->object_to_world, pobj));
    if (s->reverse_orientation) it.n = v_muls(it.n, -1);
    pobj = v_muls(pobj, s->radius / v_dist(pobj, V3(0, 0, 0)));
    v3 pobj_err = v_muls(v_abs(pobj), go_gamma(5));
    it.p = xf_point(&s->object_to_world, pobj, pobj_err, &it.perr);
    it.time = 0;
    double area = s->phi_max * s->radius * (s->z_max - s->z_min);
    *pdf = 1.0 / area;
    FL(4);
    return it;
}
/* sphere.go:287-344 */
static intr_t sphere_sample_at(const pbrt_shape_desc* s, const si_t* ref, v2 u, double* pdf) {
    v3 pc = xf_point(&s->object_to_world, V3(0, 0, 0), V3(0, 0, 0), NULL);
    v3 po = offset_ray_origin(ref->p, ref->perr, ref->n, v_sub(pc, ref->p));
    if (v_dist2(po, pc) <= s->radius * s->radius) {
        intr_t it = sphere_sample(s, u, pdf);
        v3 wi = v_sub(it.p, ref->p);
        if (v_len2(wi) == 0) {
            *pdf = 0;
        } else {
            /* Normalize() in place (xyz.go:587-594) */
            double n2 = v_len2(wi);
            if (n2 > 0) { double invn = 1.0 / sqrt(n2); wi.x *= invn; wi.y *= invn; wi.z *= invn; FL(5); }
            *pdf *= v_dist2(ref->p, it.p) / v_absdot(it.n, v_muls(wi, -1));
            FL(2);
        }
        if (gm_isinf(*pdf, 0)) *pdf = 0.0;
        return it;
    }
    v3 wc = v_normalized(v_sub(pc, ref->p));
    v3 wcx, wcy;
    coordinate_system(wc, &wcx, &wcy);
    double r2 = s->radius * s->radius;
    double sin2max = r2 / v_dist2(ref->p, pc);
    double cosmax = sqrt(go_max(0, 1.0 - sin2max));
    double cost = (1.0 - u.x) + u.x * cosmax;
    double sint = sqrt(go_max(0, 1 - cost * cost));
    double phi = u.y * 2 * go_Pi;
    double dc = v_dist(ref->p, pc);
    double ds = dc * cost - sqrt(go_max(0, r2 - (dc * dc) * (sint * sint)));
    double cosa = (dc * dc + r2 - ds * ds) / (2.0 * dc * s->radius);
    double sina = sqrt(go_max(0, 1.0 - cosa * cosa));
    FL(1 + 1 + 2 + 3 + 3 + 2 + 6 + 7 + 3 + 2);
    /* geometry.go:66-70 SphericalDirectionXYZ */
    v3 x = v_muls(wcx, -1), y = v_muls(wcy, -1), zz = v_muls(wc, -1);
    v3 nw = v_add(v_add(v_muls(x, sina * go_cos(phi)), v_muls(y, sina * go_sin(phi))), v_muls(zz, cosa));
    v3 pw = v_add(pc, v_muls(nw, s->radius));
    intr_t it;
    it.p = pw;
    it.perr = v_muls(v_abs(pw), go_gamma(5.0));
    it.n = nw;
    if (s->reverse_orientation) it.n = v_muls(it.n, -1);
    it.time = 0;
    *pdf = 1.0 / (2.0 * go_Pi * (1.0 - cosmax));
    FL(4);
    return it;
}

/* sphere.go:350-363 Sphere.PdfWi: the cone pdf from outside; from inside the
 * generic shape.go:29-47 PdfWi (SpawnRay + Sphere.Intersect, may panic) */
static double sphere_pdf_wi(orc_ctx* oc, const pbrt_shape_desc* s, const si_t* ref, v3 wi) {
    v3 pc = xf_point(&s->object_to_world, V3(0, 0, 0), V3(0, 0, 0), NULL);
    v3 po = offset_ray_origin(ref->p, ref->perr, ref->n, v_sub(ref->p, pc));
    if (v_dist2(po, pc) <= s->radius * s->radius) {
        ray_t r;
        r.o = offset_ray_origin(ref->p, ref->perr, ref->n, wi);
        r.d = wi; r.tmax = INFINITY; r.time = ref->time;
        si_t hs;
        double t;
        if (!sphere_intersect(&oc->pc, s, &r, &hs, &t)) return 0;
        double area = s->phi_max * s->radius * (s->z_max - s->z_min);
        double pdf = v_dist2(ref->p, hs.p) / v_absdot(hs.n, v_muls(v_muls(wi, -1), area));
        return gm_isinf(pdf, 0) ? 0 : pdf;
    }
    double sin2max = s->radius * s->radius / v_dist2(ref->p, pc);
    double cosmax = sqrt(go_max(0, 1.0 - sin2max));
    return 1.0 / (2.0 * go_Pi * (1.0 - cosmax));
}
static int panic_fidelity(const orc_ctx* oc) {
    return (oc->flags & ORACLE_FLAG_MIS_RAY) || (oc->rd->flags & PBRT_FLAG_PANIC_FIDELITY);
}

/* interaction.go:91-102 SpawnRayToInteraction: Origin is the UN-offset point (#14) */
static ray_t spawn_ray_to(const si_t* from, v3 to_p, v3 to_perr, v3 to_n) {
    v3 origin = offset_ray_origin(from->p, from->perr, from->n, v_sub(to_p, from->p));
    v3 target = offset_ray_origin(to_p, to_perr, to_n, v_sub(origin, to_p));
    ray_t r;
    r.o = from->p;
    r.d = v_sub(target, origin);
    r.tmax = 1 - 0.0001;
    r.time = from->time;
    FL(1);
    return r;
}

/* integrator.go:79-195 EstimateDirect (light-sampling half; see header) */
static spec estimate_direct(orc_ctx* oc, const si_t* si, const bsdf_t* b, v2 u_scat, int li, v2 u_light) {
    const pbrt_scene_desc* sc = oc->scene;
    const pbrt_light_desc* L = &sc->lights[li];
    int flags = BXDF_ALL & ~BXDF_SPECULAR;
    spec Ld = S3(0, 0, 0);
    spec Li;
    v3 wi;
    double light_pdf;
    v3 tp, tperr, tn;
    int is_delta = L->type != PBRT_LIGHT_DIFFUSE_AREA;
    if (L->type == PBRT_LIGHT_POINT) {
        /* point.go:44-49 */
        v3 pl = V3(L->p_light[0], L->p_light[1], L->p_light[2]);
        wi = v_normalized(v_sub(pl, si->p));
        light_pdf = 1.0;
        Li = s_divs(S3(L->spectrum[0], L->spectrum[1], L->spectrum[2]), v_dist2(pl, si->p));
        tp = pl; tperr = V3(0, 0, 0); tn = V3(0, 0, 0);
    } else if (L->type == PBRT_LIGHT_DISTANT) {
        /* distant.go:40-44: pOutside = wLight * 2R, not ref + wLight*2R (#15) */
        v3 w = V3(L->w_light[0], L->w_light[1], L->w_light[2]);
        tp = v_muls(w, 2 * L->world_radius);
        tperr = V3(0, 0, 0); tn = V3(0, 0, 0);
        Li = S3(L->spectrum[0], L->spectrum[1], L->spectrum[2]);
        wi = w;
        light_pdf = 1;
    } else {
        /* diffuse.go:47-59: unnormalized wi (#12) */
        const pbrt_shape_desc* shp = &sc->shapes[L->shape];
        double pdf;
        intr_t ps = sphere_sample_at(shp, si, u_light, &pdf);
        if (pdf == 0 || v_len2(v_sub(ps.p, si->p)) == 0) {
            Li = S3(0, 0, 0); wi = V3(0, 0, 0); light_pdf = 0;
            tp = tperr = tn = V3(0, 0, 0);
        } else {
            wi = v_sub(ps.p, si->p);
            light_pdf = pdf;
            tp = ps.p; tperr = ps.perr; tn = ps.n;
            if (L->two_sided || v_dot(ps.n, v_muls(wi, -1)) > 0)
                Li = S3(L->spectrum[0], L->spectrum[1], L->spectrum[2]);
            else
                Li = S3(0, 0, 0);
        }
    }
    if (light_pdf > 0 && !s_is_black(Li)) {
        spec f = bsdf_f(b, si->wo, wi, flags);
        double wdn = v_absdot(wi, si->sn);
        f = s_muls(f, wdn);
        double scat_pdf = bsdf_pdf(b, si->wo, wi, flags);
        if (!s_is_black(f)) {
            ray_t sr = spawn_ray_to(si, tp, tperr, tn);
            oc->shadow_rays++;
            if (orc_bvh_intersect_p(oc, &sr)) Li = S3(0, 0, 0);
            if (!s_is_black(Li)) {
                if (is_delta) {
                    Ld = s_add(Ld, s_divs(s_mul(f, Li), light_pdf));
                } else {
                    double fp = 1.0 * light_pdf, gp = 1.0 * scat_pdf;
                    double weight = (fp * fp) / (fp * fp + gp * gp);
                    FL(7);
                    Ld = s_add(Ld, s_divs(s_muls(s_mul(f, Li), weight), light_pdf));
                }
            }
        }
    }
    if (!is_delta && b->kind == BXDF_KIND_MICROFACET && b->n_bxdfs > 0 && bsdf_w2l(b, si->wo).z != 0) {
        /* integrator.go:134-139: BSDF.SampleF runs for every area light */
        oc->pc.kind = PBRT_PANIC_NIL_DEREF;
        longjmp(oc->pc.jb, 1);
    }
    if (!is_delta && panic_fidelity(oc)) {
        /* integrator.go:132-192: BSDF-sampled ray toward the area light. No
         * primitive has an area light, so Li is always 0 here; PdfLi and the
         * ray are evaluated only for fidelity (panics). */
        v3 wi2; double spdf;
        FL_OFF_BEGIN;
        spec f2 = bsdf_sample_f(b, si->wo, u_scat, flags, &wi2, &spdf);
        double lpdf = (!s_is_black(f2) && spdf > 0.0) ? sphere_pdf_wi(oc, &sc->shapes[L->shape], si, wi2) : 0;
        FL_OFF_END;
        if (!s_is_black(f2) && spdf > 0.0 && lpdf != 0) {
            ray_t r2;
            r2.o = offset_ray_origin(si->p, si->perr, si->n, wi2);
            r2.d = wi2; r2.tmax = INFINITY; r2.time = si->time;
            si_t tmp;   /* not counted in closest_rays (its result is always 0) */
            orc_bvh_intersect(oc, &r2, &tmp);
        }
    }
    return Ld;
}

/* sampling.go:42-55 + pkg/math FindInterval (math.go:64-80) */
static int sample_discrete(const pbrt_distribution_desc* d, double u, double* pdf) {
    int size = d->count + 1;
    int first = 0, len = size;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (d->cdf[middle] <= u) { first = middle + 1; len -= half + 1; }
        else len = half;
    }
    int off = (int)go_clamp((double)(first - 1), 0, (double)(size - 2));
    *pdf = 0;
    if (d->func_int > 0) { *pdf = d->func[off] / (d->func_int / (double)d->count); FL(2); }
    return off;
}

/* integrator.go:48-77 UniformSampleOneLight */
static spec uniform_sample_one_light(orc_ctx* oc, sampler_t* smp, const si_t* si, const bsdf_t* b,
                                     const pbrt_distribution_desc* dist) {
    int n = oc->scene->n_lights;
    if (n == 0) return S3(0, 0, 0);
    int ln;
    double lpdf;
    if (dist) {
        ln = sample_discrete(dist, sampler_get1d(smp), &lpdf);
        if (lpdf == 0.0) return S3(0, 0, 0);
    } else {
        ln = (int)go_f2i(go_min(sampler_get1d(smp) * (double)n, (double)(n - 1)));
        lpdf = 1.0 / (double)n;
        FL(2);
    }
    v2 ul = sampler_get2d(smp);
    v2 us = sampler_get2d(smp);
    spec s = estimate_direct(oc, si, b, us, ln, ul);
    /* spectrum.DivScalar(lightPdf) result discarded (#10) */
    if (s_max_component(s) > 10) {
        oc->pc.kind = PBRT_PANIC_LD_GT_10;
        longjmp(oc->pc.jb, 1);
    }
    return s;
}

/* ============================================================== integrators */
/* pkg/integrator/path.go:32-157 */
static spec path_li(orc_ctx* oc, sampler_t* smp, ray_t ray) {
    const pbrt_scene_desc* sc = oc->scene;
    const pbrt_render_desc* rd = oc->rd;
    spec L = S3(0, 0, 0), beta = S3(1, 1, 1);
    int32_t bounces = 0;
    double eta_scale = 1.0;
    for (;;) {
        bounces++;
        oc->cur_bounce = bounces;
        if (bounces >= rd->max_depth) {          /* path.go:66 (hit or miss)  */
            oc->closest_rays++;                  /* traced by path.go:45 first */
            if (panic_fidelity(oc)) {
                si_t tmp;
                orc_bvh_intersect(oc, &ray, &tmp);
            }
            break;
        }
        si_t isect;
        oc->closest_rays++;
        if (!orc_bvh_intersect(oc, &ray, &isect)) break;
        bsdf_t b;
        if (material_bsdf(sc, &isect, &b, 1) < 0) { oc->unsupported = 1; break; }
        if (b.n_bxdfs > 0 && b.kind != BXDF_KIND_FRESNEL_SPEC) {   /* NumComponents(BSDFAll &^ BSDFSpecular) > 0 */
#ifdef ORACLE_COUNT_FLOPS
            const uint64_t f0 = orc_flops;
#endif
            spec ld = uniform_sample_one_light(oc, smp, &isect, &b, &oc->dist);
            L = s_add(L, s_mul(beta, ld));
#ifdef ORACLE_COUNT_FLOPS
            orc_flops_light += orc_flops - f0;
#endif
        }
        v3 wo = ray.d;                           /* path.go:91 (#8)           */
        v2 u = sampler_get2d(smp);
        v3 wi; double pdf; int flags;
        spec f = bsdf_sample_f_t(&b, wo, u, BXDF_ALL, &wi, &pdf, &flags);
        if (flags == -1) {
            oc->pc.kind = PBRT_PANIC_NIL_DEREF;
            longjmp(oc->pc.jb, 1);
        }
        if (s_is_black(f) || pdf == 0.0) break;
        double wabs = v_absdot(wi, isect.sn);
        double wp = wabs / pdf;
        FL(1);
        spec fm = s_muls(f, wp);
        beta = s_mul(beta, fm);
        if ((flags & BXDF_SPECULAR) && (flags & BXDF_TRANSMISSION)) {   /* path.go:106-117 */
            double eta = b.eta;
            if (v_dot(wo, isect.n) > 0) eta_scale *= eta * eta;
            else eta_scale *= 1 / (eta * eta);
        }
        /* interaction.go:68-77 SpawnRay */
        ray.o = offset_ray_origin(isect.p, isect.perr, isect.n, wi);
        ray.d = wi;
        ray.tmax = INFINITY;
        ray.time = isect.time;
        spec rr = s_muls(beta, eta_scale);
        if (s_max_component(rr) < rd->rr_threshold && bounces > 3) {
            double q = go_max(0.05, 1 - s_max_component(rr));
            FL(1);
            if (sampler_get1d(smp) < q) break;
            beta = s_divs(beta, 1 - q);
            FL(1);
        }
    }
    return L;
}

/* pkg/integrator/directlighting.go:62-104 DirectLighting.Li at `depth`
 * (renderWorker calls it with 0). A smooth glass carries SpecularTransmission
 * (allowMultipleLobes false, directlighting.go:76), so SpecularTransmit
 * recurses here. */
static spec direct_li_d(orc_ctx* oc, sampler_t* smp, ray_t ray, int depth);

/* SamplerIntegratorSpecularReflect / -Transmit (integrator.go:352-422) with
 * BSDF.SampleF flags t = Reflection|Specular or Transmission|Specular. The
 * Get2D is drawn first (an argument of SampleF); wi is the LOCAL-frame
 * direction SampleF returns (#7), used for |wi.ns|, SpawnRay and the recursion;
 * Li runs at depth + 1 where `depth` already is the caller's depth + 1 (#23). */
static spec specular_bounce(orc_ctx* oc, sampler_t* smp, const si_t* si, const bsdf_t* b, int depth, int t) {
    v2 u = sampler_get2d(smp);
    v3 wi; double pdf; int ty;
    spec f = bsdf_sample_f_t(b, si->wo, u, t, &wi, &pdf, &ty);
    if (ty == -1) {   /* not reachable: no BxDF of rough glass matches a specular flag set */
        oc->pc.kind = PBRT_PANIC_NIL_DEREF;
        longjmp(oc->pc.jb, 1);
    }
    double adn = v_absdot(wi, si->sn);
    if (pdf > 0 && !s_is_black(f) && adn != 0.0) {
        /* interaction.go:68-77 SpawnRay; the differentials never reach an output (#27) */
        ray_t rd;
        rd.o = offset_ray_origin(si->p, si->perr, si->n, wi);
        rd.d = wi;
        rd.tmax = INFINITY;
        rd.time = si->time;
        spec li = direct_li_d(oc, smp, rd, depth + 1);
        return s_muls(s_mul(f, li), adn / pdf);
    }
    return S3(0, 0, 0);
}

static spec direct_li_d(orc_ctx* oc, sampler_t* smp, ray_t ray, int depth) {
    const pbrt_scene_desc* sc = oc->scene;
    const pbrt_render_desc* rd = oc->rd;
    spec L = S3(0, 0, 0);
    si_t si;
    oc->cur_bounce = depth + 1;   /* panic report: 1 + the recursion depth */
    oc->closest_rays++;
    if (!orc_bvh_intersect(oc, &ray, &si)) {
        for (int i = 0; i < sc->n_lights; i++) L = s_add(L, S3(0, 0, 0));   /* Light.Le: 0 */
        return L;
    }
    bsdf_t b;
    if (material_bsdf(sc, &si, &b, 0) < 0) { oc->unsupported = 1; return L; }
    L = s_add(L, S3(0, 0, 0));       /* si.Le(si.Wo): no area-light prims  */
    if (sc->n_lights > 0) {
        if (rd->dl_strategy == PBRT_DL_UNIFORM_SAMPLE_ALL) {
            /* integrator.go:23-46; clones carry no sample arrays (#23) */
            spec acc = S3(0, 0, 0);
            for (int j = 0; j < sc->n_lights; j++) {
                v2 ul = sampler_get2d(smp);
                v2 us = sampler_get2d(smp);
                acc = s_add(acc, estimate_direct(oc, &si, &b, us, j, ul));
            }
            L = s_add(L, acc);
        } else {
            L = s_add(L, uniform_sample_one_light(oc, smp, &si, &b, NULL));
        }
    }
    if (depth + 1 < rd->max_depth) {
        /* directlighting.go:97-101. No supported BxDF is Reflection|Specular
         * (SpecularReflection is typed Reflection|Diffuse, reflection.go:538-544),
         * so SpecularReflect only draws its Get2D; SpecularTransmit follows a
         * smooth glass's SpecularTransmission. */
        L = s_add(L, specular_bounce(oc, smp, &si, &b, depth + 1, BXDF_REFLECTION | BXDF_SPECULAR));
        L = s_add(L, specular_bounce(oc, smp, &si, &b, depth + 1, BXDF_TRANSMISSION | BXDF_SPECULAR));
    }
    return L;
}
static spec direct_li(orc_ctx* oc, sampler_t* smp, ray_t ray) { return direct_li_d(oc, smp, ray, 0); }

/* =================================================================== camera */
/* camera.go:192-242 GenerateRayDifferential (differentials have no effect, #27) */
static ray_t camera_ray(const pbrt_camera_desc* cam, double fx, double fy, double time_u, v2 plens) {
    v3 pcam = xf_point(&cam->raster_to_camera, V3(fx, fy, 0), V3(0, 0, 0), NULL);
    ray_t r;
    r.o = V3(0, 0, 0);
    r.d = v_normalized(pcam);
    r.tmax = INFINITY;
    r.time = 0;
    if (cam->lens_radius > 0) {
        v2 pl = concentric_sample_disk(plens);
        pl.x *= cam->lens_radius; pl.y *= cam->lens_radius;
        double ft = cam->focal_distance / r.d.z;
        FL(3);
        v3 pf = v_add(v_muls(r.d, ft), r.o);
        r.o = V3(pl.x, pl.y, 0);
        r.d = v_normalized(v_sub(pf, r.o));
    }
    ray_t w = xf_ray(&cam->camera_to_world, &r, NULL, NULL);
    w.time = go_lerp(time_u, cam->shutter_open, cam->shutter_close);
    return w;
}

/* ================================================================ tiles */
void orc_tile_bounds(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int64_t tile,
                     int64_t* x0, int64_t* y0, int64_t* x1, int64_t* y1) {
    const pbrt_film_desc* fm = &sc->film;
    int64_t ts = rd->tile_size;
    int64_t ntx = (fm->crop_max_x - fm->crop_min_x + ts - 1) / ts;
    int64_t tx = tile % ntx, ty = tile / ntx;
    *x0 = fm->crop_min_x + tx * ts;
    *x1 = go_f2i(go_min((double)(*x0 + ts), (double)fm->crop_max_x));
    *y0 = fm->crop_min_y + ty * ts;
    *y1 = go_f2i(go_min((double)(*y0 + ts), (double)fm->crop_max_y));
}
int64_t orc_num_tiles(const pbrt_scene_desc* sc, const pbrt_render_desc* rd) {
    const pbrt_film_desc* fm = &sc->film;
    int64_t ts = rd->tile_size;
    int64_t ntx = (fm->crop_max_x - fm->crop_min_x + ts - 1) / ts;
    int64_t nty = (fm->crop_max_y - fm->crop_min_y + ts - 1) / ts;
    return ntx * nty;
}
/* film.go:106-113 GetFilmTile pixel bounds */
void orc_film_tile_bounds(const pbrt_scene_desc* sc, int64_t x0, int64_t y0, int64_t x1, int64_t y1,
                          int64_t* px0, int64_t* py0, int64_t* px1, int64_t* py1) {
    const pbrt_film_desc* fm = &sc->film;
    double rx = fm->filter_radius_x, ry = fm->filter_radius_y;
    int64_t p0x = go_f2i(ceil(((double)x0 - 0.5) - rx));
    int64_t p0y = go_f2i(ceil(((double)y0 - 0.5) - ry));
    int64_t p1x = go_f2i(floor(((double)x1 - 0.5) + rx)) + 1;
    int64_t p1y = go_f2i(floor(((double)y1 - 0.5) + ry)) + 1;
    /* bounds.go:93-98 Intersect (through float64 Max/Min) */
    *px0 = go_f2i(go_max((double)fm->crop_min_x, (double)p0x));
    *py0 = go_f2i(go_max((double)fm->crop_min_y, (double)p0y));
    *px1 = go_f2i(go_min((double)fm->crop_max_x, (double)p1x));
    *py1 = go_f2i(go_min((double)fm->crop_max_y, (double)p1y));
}

typedef struct {
    int64_t px0, py0, px1, py1;
    double* contrib;    /* (px1-px0)*(py1-py0)*3 */
} film_tile_t;

/* film.go:211-248 AddSample */
static void film_tile_add(const pbrt_film_desc* fm, film_tile_t* ft, double pfx, double pfy, spec L,
                          double w) {
    if (0.0 > fm->max_sample_luminance) L = s_muls(L, fm->max_sample_luminance / 0.0); /* L.Y() == 0 (#5) */
    double dx = pfx - 0.5, dy = pfy - 0.5;
    FL(2);
    double p0fx = ceil(dx - fm->filter_radius_x), p0fy = ceil(dy - fm->filter_radius_y);
    double p1fx = floor(dx + fm->filter_radius_x) + 1, p1fy = floor(dy + fm->filter_radius_y) + 1;
    int64_t p0x = go_f2i(go_max(p0fx, (double)ft->px0)), p0y = go_f2i(go_max(p0fy, (double)ft->py0));
    int64_t p1x = go_f2i(go_min(p1fx, (double)ft->px1)), p1y = go_f2i(go_min(p1fy, (double)ft->py1));
    double ifr_x = 1.0 / fm->filter_radius_x, ifr_y = 1.0 / fm->filter_radius_y;
    int ifx[64], ify[64];
    for (int64_t x = p0x; x < p1x; x++) {
        double f = gm_abs(((double)x - dx) * ifr_x * 16.0);
        ifx[x - p0x] = (int)go_f2i(go_min(floor(f), 16.0 - 1));
    }
    for (int64_t y = p0y; y < p1y; y++) {
        double f = gm_abs(((double)y - dy) * ifr_y * 16.0);
        ify[y - p0y] = (int)go_f2i(go_min(floor(f), 16.0 - 1));
    }
    int64_t tw = ft->px1 - ft->px0;
    for (int64_t y = p0y; y < p1y; y++)
        for (int64_t x = p0x; x < p1x; x++) {
            double fw = fm->filter_table[ify[y - p0y] * 16 + ifx[x - p0x]];
            double* px = ft->contrib + ((x - ft->px0) + (y - ft->py0) * tw) * 3;
            spec add = s_muls(L, w * fw);
            px[0] += add.c[0]; px[1] += add.c[1]; px[2] += add.c[2];
            FL(4);
        }
}

/* THROUGHPUT mode ("Mode B"); NOT in the reference. The
 * build's own definition, stated identically in csrc/pbrt_path.h mb_state:
 * stream s of pixel pi (row-major in its tile) of tile t starts at PCG32
 * state mb_state(t, pi, s) with the tile's increment; s = 0 feeds StartPixel,
 * s = k >= 1 feeds sample k. Everything else is the EXACT arithmetic. */
static uint64_t mb_mix(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static uint64_t mb_state(uint64_t tile, uint64_t pi, uint64_t s) { return mb_mix(mb_mix(mb_mix(tile) ^ pi) ^ s); }

/* integrator.go:228-289 renderWorker body for one tile */
static int render_tile(orc_ctx* oc, int64_t tile, film_tile_t* ft, double* s1d_buf) {
    const pbrt_scene_desc* sc = oc->scene;
    const pbrt_render_desc* rd = oc->rd;
    int64_t x0, y0, x1, y1;
    orc_tile_bounds(sc, rd, tile, &x0, &y0, &x1, &y1);
    orc_film_tile_bounds(sc, x0, y0, x1, y1, &ft->px0, &ft->py0, &ft->px1, &ft->py1);
    size_t npx = (size_t)((ft->px1 - ft->px0) * (ft->py1 - ft->py0));
    memset(ft->contrib, 0, npx * 3 * sizeof(double));

    sampler_t smp;
    memset(&smp, 0, sizeof(smp));
    smp.xs = rd->sampler_x; smp.ys = rd->sampler_y; smp.spp = rd->sampler_x * rd->sampler_y;
    smp.ndims = rd->n_dims; smp.jitter = rd->jitter; smp.s1d = s1d_buf;
    smp.random = (oc->flags & ORACLE_FLAG_RANDOM_SAMPLER) != 0;
    if (smp.random) smp.ndims = 0;
    /* integrator.go:318,328; RandomSampler.Clone = NewRNGWithSeed + SetSequence
     * (random.go:33-37), which resets the state: the same stream */
    orc_pcg_set_sequence(&smp.rng, (uint64_t)tile);

    const int mb = rd->mode == PBRT_MODE_THROUGHPUT;
    oc->pc.kind = 0;
    oc->cur_tile = tile;
    if (setjmp(oc->pc.jb)) return -1;
    for (int64_t py = y0; py < y1; py++) {
        for (int64_t px = x0; px < x1; px++) {
            oc->cur_px = px; oc->cur_py = py;
            const uint64_t pi = (uint64_t)((py - y0) * (x1 - x0) + (px - x0));
            const uint64_t draws0 = orc_draws;
            if (mb) smp.rng.state = mb_state((uint64_t)tile, pi, 0);
            sampler_start_pixel(&smp);
            while (sampler_next_sample(&smp)) {
                oc->cur_sample = smp.sample_index;
                if (mb) smp.rng.state = mb_state((uint64_t)tile, pi, (uint64_t)smp.sample_index);
                /* sampler.go:75-80: pFilm = pixel + Get2D, pLens = Get2D, time = Get1D */
                v2 u0 = sampler_get2d(&smp);
                double fx = (double)px + u0.x, fy = (double)py + u0.y;
                v2 plens = sampler_get2d(&smp);
                double tu = sampler_get1d(&smp);
                ray_t ray = camera_ray(&sc->camera, fx, fy, tu, plens);
                spec L;
                oc->camera_samples++;
                oc->paths++;
                if (rd->integrator == PBRT_INTEGRATOR_PATH) L = path_li(oc, &smp, ray);
                else L = direct_li(oc, &smp, ray);
                if (oc->unsupported) return -2;
                if (s_has_nans(L)) L = S3(0.1, 0.1, 0.1);    /* integrator.go:256-262 */
                film_tile_add(&sc->film, ft, fx, fy, L, 1.0);
            }
            if (oc->pixel_draws) oc->pixel_draws[pi] = (int64_t)(orc_draws - draws0);
        }
    }
    return 0;
}

/* PCG32 draws each pixel of `tile` consumes (StartPixel + its samples), row-major
 * in the tile; out holds tile_size^2 entries. Returns 0, or the render_tile status. */
int orc_tile_draws(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int64_t tile, int64_t* out) {
    orc_ctx oc;
    memset(&oc, 0, sizeof(oc));
    oc.scene = sc; oc.rd = rd;
    oc.mesh = orc_mesh_get(sc);
    oc.pixel_draws = out;
    orc_light_distribution(sc, rd, &oc.dist);
    const int spp = rd->sampler_x * rd->sampler_y;
    double* s1d = (double*)malloc(sizeof(double) * (size_t)spp * (size_t)(rd->n_dims > 0 ? rd->n_dims : 1));
    int64_t maxw = rd->tile_size + 2 * (int64_t)(sc->film.filter_radius_x + 2);
    int64_t maxh = rd->tile_size + 2 * (int64_t)(sc->film.filter_radius_y + 2);
    film_tile_t ft;
    ft.contrib = (double*)malloc(sizeof(double) * (size_t)(maxw * maxh * 3));
    int rc = render_tile(&oc, tile, &ft, s1d);
    free(ft.contrib);
    free(s1d);
    return rc;
}

/* ================================================================ driver */
typedef struct {
    const pbrt_scene_desc* sc;
    const pbrt_render_desc* rd;
    const int64_t* tiles;
    int64_t n_tiles;
    atomic_long next;
    film_tile_t* films;
    int* status;
    int* panic_kind;
    int64_t* panic_info;    /* 4 per tile: px, py, sample, bounce */
    int flags;
    atomic_ullong paths, samples, closest, shadow, flops, flops_light;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    orc_ctx oc;
    memset(&oc, 0, sizeof(oc));
    oc.scene = j->sc; oc.rd = j->rd; oc.flags = j->flags;
    oc.mesh = orc_mesh_get(j->sc);
#ifdef ORACLE_COUNT_FLOPS
    orc_flops = 0;
    orc_flops_light = 0;
#endif
    orc_light_distribution(j->sc, j->rd, &oc.dist);
    int spp = j->rd->sampler_x * j->rd->sampler_y;
    double* s1d = (double*)malloc(sizeof(double) * (size_t)spp * (size_t)(j->rd->n_dims > 0 ? j->rd->n_dims : 1));
    for (;;) {
        long i = atomic_fetch_add(&j->next, 1);
        if (i >= j->n_tiles) break;
        int st = render_tile(&oc, j->tiles[i], &j->films[i], s1d);
        j->status[i] = st;
        j->panic_kind[i] = oc.pc.kind;
        if (st == -1) {
            j->panic_info[4 * i + 0] = oc.cur_px;
            j->panic_info[4 * i + 1] = oc.cur_py;
            j->panic_info[4 * i + 2] = oc.cur_sample;
            j->panic_info[4 * i + 3] = oc.cur_bounce;
        }
        oc.unsupported = 0;
    }
    atomic_fetch_add(&j->paths, oc.paths);
    atomic_fetch_add(&j->samples, oc.camera_samples);
    atomic_fetch_add(&j->closest, oc.closest_rays);
    atomic_fetch_add(&j->shadow, oc.shadow_rays);
#ifdef ORACLE_COUNT_FLOPS
    atomic_fetch_add(&j->flops, orc_flops);
    atomic_fetch_add(&j->flops_light, orc_flops_light);
#endif
    free(s1d);
    return NULL;
}

/* Distribution1D for the Path integrator's LightSampleStrategy
 * (lightdistribution.go:11-68, sampling.go:10-36). Power builds a 2n array
 * (make n + append n) of Y() == 0 values (#28). */
void orc_light_distribution(const pbrt_scene_desc* sc, const pbrt_render_desc* rd,
                            pbrt_distribution_desc* d) {
    memset(d, 0, sizeof(*d));
    int n = sc->n_lights;
    int cnt = (rd->light_strategy == PBRT_LIGHT_STRATEGY_POWER) ? 2 * n : n;
    if (cnt > PBRT_MAX_DIST) cnt = PBRT_MAX_DIST;
    for (int i = 0; i < cnt; i++)
        d->func[i] = (rd->light_strategy == PBRT_LIGHT_STRATEGY_POWER) ? 0.0 : 1.0;
    d->count = cnt;
    d->cdf[0] = 0;
    for (int i = 1; i < cnt + 1; i++) d->cdf[i] = d->cdf[i - 1] + d->func[i - 1] / (double)cnt;
    d->func_int = d->cdf[cnt];
    if (d->func_int == 0.0) {
        for (int i = 1; i < cnt + 1; i++) d->cdf[i] = (double)i / (double)cnt;
    } else {
        for (int i = 1; i < cnt + 1; i++) d->cdf[i] /= d->func_int;
    }
}

int orc_render(const pbrt_scene_desc* sc, const pbrt_render_desc* rd, int n_threads, int flags,
               double* film_xyz, orc_stats* stats) {
    if (!sc || !rd || rd->tile_size <= 0 || rd->sampler_x <= 0 || rd->sampler_y <= 0) return PBRT_E_INVALID;
    int64_t total = orc_num_tiles(sc, rd);
    int64_t begin = rd->tile_begin, end = rd->tile_end > 0 ? rd->tile_end : total;
    int64_t stride = rd->tile_stride > 0 ? rd->tile_stride : 1;
    if (end > total) end = total;
    int64_t n = 0;
    for (int64_t t = begin; t < end; t += stride) n++;
    int64_t* tiles = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    n = 0;
    for (int64_t t = begin; t < end; t += stride) tiles[n++] = t;

    int64_t maxw = rd->tile_size + 2 * (int64_t)(sc->film.filter_radius_x + 2);
    int64_t maxh = rd->tile_size + 2 * (int64_t)(sc->film.filter_radius_y + 2);
    job_t j;
    memset(&j, 0, sizeof(j));
    j.sc = sc; j.rd = rd; j.tiles = tiles; j.n_tiles = n; j.flags = flags;
    atomic_init(&j.next, 0);
    j.films = (film_tile_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(film_tile_t));
    j.status = (int*)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    j.panic_kind = (int*)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    j.panic_info = (int64_t*)calloc((size_t)(n > 0 ? n : 1) * 4, sizeof(int64_t));
    double* pool = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1) * (size_t)(maxw * maxh * 3));
    for (int64_t i = 0; i < n; i++) j.films[i].contrib = pool + (size_t)i * (size_t)(maxw * maxh * 3);

    if (n_threads < 1) n_threads = 1;
    pthread_t th[256];
    if (n_threads > 256) n_threads = 256;
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);

    int rc = PBRT_OK;
    if (stats) memset(stats, 0, sizeof(*stats));
    for (int64_t i = 0; i < n; i++) {
        if (j.status[i] == -2) { rc = PBRT_E_UNSUPPORTED; break; }
        if (j.status[i] == -1) {
            rc = PBRT_E_REF_PANIC;
            if (stats) {
                stats->panic_kind = j.panic_kind[i];
                stats->panic_tile = tiles[i];
                stats->panic_px = j.panic_info[4 * i + 0];
                stats->panic_py = j.panic_info[4 * i + 1];
                stats->panic_sample = j.panic_info[4 * i + 2];
                stats->panic_bounce = j.panic_info[4 * i + 3];
            }
            break;
        }
    }
    if (film_xyz) {
        const pbrt_film_desc* fm = &sc->film;
        int64_t W = fm->crop_max_x - fm->crop_min_x, H = fm->crop_max_y - fm->crop_min_y;
        memset(film_xyz, 0, sizeof(double) * (size_t)(W * H * 3));
        /* film.go:115-132 MergeFilmTile, in tile-index order */
        for (int64_t i = 0; i < n && rc == PBRT_OK; i++) {
            film_tile_t* ft = &j.films[i];
            int64_t tw = ft->px1 - ft->px0;
            for (int64_t y = ft->py0; y < ft->py1; y++)
                for (int64_t x = ft->px0; x < ft->px1; x++) {
                    const double* c = ft->contrib + ((x - ft->px0) + (y - ft->py0) * tw) * 3;
                    double X = 0.412453 * c[0] + 0.357580 * c[1] + 0.180423 * c[2];
                    double Y = 0.212671 * c[0] + 0.715160 * c[1] + 0.072169 * c[2];
                    double Z = 0.019334 * c[0] + 0.119193 * c[1] + 0.950227 * c[2];
                    double* f = film_xyz + ((x - fm->crop_min_x) + (y - fm->crop_min_y) * W) * 3;
                    f[0] += X; f[1] += Y; f[2] += Z;
                }
        }
    }
    if (stats) {
        stats->tiles = (uint64_t)n;
        stats->paths = atomic_load(&j.paths);
        stats->camera_samples = atomic_load(&j.samples);
        stats->closest_rays = atomic_load(&j.closest);
        stats->shadow_rays = atomic_load(&j.shadow);
        stats->flops = atomic_load(&j.flops);
        stats->flops_light = atomic_load(&j.flops_light);
    }
    free(pool); free(j.films); free(j.status); free(j.panic_kind); free(j.panic_info); free(tiles);
    return rc;
}

/* ------------------------------------------------------- batch intersect */
static void intersect_one(orc_ctx* oc, const double* q, int closest, double* o) {
    ray_t r;
    r.o = V3(q[0], q[1], q[2]); r.d = V3(q[3], q[4], q[5]); r.tmax = q[6]; r.time = 0;
    if (setjmp(oc->pc.jb)) {
        if (closest) { for (int k = 0; k < 9; k++) o[k] = NAN; }
        else o[0] = NAN;
        return;
    }
    if (closest) {
        si_t si;
        memset(&si, 0, sizeof(si));
        si.prim = -1;
        int h = orc_bvh_intersect(oc, &r, &si);
        o[0] = h; o[1] = r.tmax; o[2] = h ? si.prim : -1;
        o[3] = si.p.x; o[4] = si.p.y; o[5] = si.p.z;
        o[6] = si.n.x; o[7] = si.n.y; o[8] = si.n.z;
    } else {
        o[0] = orc_bvh_intersect_p(oc, &r);
    }
}

/* rays: n x 7 (o, d, tmax); out (closest): n x 9 (hit, tmax, prim, p, n);
 * out (any-hit): n x 1. A reference panic yields NaNs for that ray. */
int orc_intersect(const pbrt_scene_desc* sc, const double* rays, size_t n, int closest, double* out) {
    orc_ctx oc;
    memset(&oc, 0, sizeof(oc));
    oc.scene = sc;
    oc.mesh = orc_mesh_get(sc);
    for (size_t i = 0; i < n; i++)
        intersect_one(&oc, rays + 7 * i, closest, closest ? out + 9 * i : out + i);
    return 0;
}
