/*
 * oracle/oracle_scene.c — TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * Independent C restatement of go-pbrt's host-side scene construction:
 * Matrix4x4/Transform arithmetic (pkg/pbrt/transform.go), shapes
 * (sphere.go:19-55, shapes/disk.go:22-57), lights (pkg/lights), camera
 * (camera.go:106-165), film (film.go:42-76), BVH build (accelerator/bvh.go:
 * 223-411, 632-651) and the README scene of internal/render/server.go:29-164.
 * tests/ compare its descriptor with the product's host builder bit for bit.
 */
#include "oracle_scene.h"

#include <stdlib.h>
#include <string.h>

/* ============================================================== matrices */
static pbrt_matrix4x4 m_ident(void) {
    pbrt_matrix4x4 r;
    memset(&r, 0, sizeof(r));
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0;
    return r;
}
/* transform.go:62-70 (last term uses m[3][j], #18) */
pbrt_matrix4x4 orc_m_mul(const pbrt_matrix4x4* m, const pbrt_matrix4x4* o) {
    pbrt_matrix4x4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = m->m[i][0] * o->m[0][j] + m->m[i][1] * o->m[1][j] + m->m[i][2] * o->m[2][j] +
                        m->m[i][3] * m->m[3][j];
    return r;
}
static pbrt_matrix4x4 m_transpose(const pbrt_matrix4x4* m) {
    pbrt_matrix4x4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.m[i][j] = m->m[j][i];
    return r;
}
/* transform.go:72-142 Gauss-Jordan with full pivoting */
int orc_m_inverse(const pbrt_matrix4x4* m, pbrt_matrix4x4* out) {
    int indxc[4] = {0}, indxr[4] = {0}, ipiv[4] = {0};
    pbrt_matrix4x4 minv = *m;
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        double big = 0.0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (gm_abs(minv.m[j][k]) >= big) {
                            big = gm_abs(minv.m[j][k]);
                            irow = j;
                            icol = k;
                        }
                    } else if (ipiv[k] > 1) {
                        return -1;
                    }
                }
            }
        }
        ipiv[icol]++;
        if (irow != icol)
            for (int k = 0; k < 4; k++) {
                double t = minv.m[irow][k]; minv.m[irow][k] = minv.m[icol][k]; minv.m[icol][k] = t;
            }
        indxr[i] = irow;
        indxc[i] = icol;
        if (minv.m[icol][icol] == 0.0) return -1;
        double pivinv = 1.0 / minv.m[icol][icol];
        minv.m[icol][icol] = 1.0;
        for (int j = 0; j < 4; j++) minv.m[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                double save = minv.m[j][icol];
                minv.m[j][icol] = 0.0;
                for (int k = 0; k < 4; k++) minv.m[j][k] -= minv.m[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) {
                double t = minv.m[k][indxr[j]];
                minv.m[k][indxr[j]] = minv.m[k][indxc[j]];
                minv.m[k][indxc[j]] = t;
            }
    }
    *out = minv;
    return 0;
}

/* ============================================================ transforms */
pbrt_transform orc_translate(double x, double y, double z) {
    pbrt_transform t;
    t.m = m_ident(); t.m_inv = m_ident();
    t.m.m[0][3] = x; t.m.m[1][3] = y; t.m.m[2][3] = z;
    t.m_inv.m[0][3] = -x; t.m_inv.m[1][3] = -y; t.m_inv.m[2][3] = -z;
    return t;
}
pbrt_transform orc_scale(double x, double y, double z) {
    pbrt_transform t;
    t.m = m_ident(); t.m_inv = m_ident();
    t.m.m[0][0] = x; t.m.m[1][1] = y; t.m.m[2][2] = z;
    t.m_inv.m[0][0] = 1.0 / x; t.m_inv.m[1][1] = 1.0 / y; t.m_inv.m[2][2] = 1.0 / z;
    return t;
}
/* transform.go:381-424 */
pbrt_transform orc_rotate(int axis, double degrees) {
    double s = go_sin(go_radians(degrees));
    double c = go_cos(go_radians(degrees));
    pbrt_transform t;
    t.m = m_ident();
    if (axis == 0) {
        t.m.m[1][1] = c; t.m.m[1][2] = -s; t.m.m[2][1] = s; t.m.m[2][2] = c;
    } else if (axis == 1) {
        t.m.m[0][0] = c; t.m.m[0][2] = s; t.m.m[2][0] = -s; t.m.m[2][2] = c;
    } else {
        t.m.m[0][0] = c; t.m.m[0][1] = -s; t.m.m[1][0] = s; t.m.m[1][1] = c;
    }
    t.m_inv = m_transpose(&t.m);
    return t;
}
/* transform.go:179-184 (inverses composed in the wrong order, #18) */
pbrt_transform orc_xf_mul(const pbrt_transform* a, const pbrt_transform* b) {
    pbrt_transform r;
    r.m = orc_m_mul(&a->m, &b->m);
    r.m_inv = orc_m_mul(&a->m_inv, &b->m_inv);
    return r;
}
static pbrt_transform new_transform(const pbrt_matrix4x4* m) {
    pbrt_transform t;
    t.m = *m;
    orc_m_inverse(m, &t.m_inv);
    return t;
}
/* transform.go:453-486 */
int orc_look_at(v3 pos, v3 look, v3 up, pbrt_transform* out) {
    pbrt_matrix4x4 m;
    memset(&m, 0, sizeof(m));
    m.m[0][3] = pos.x; m.m[1][3] = pos.y; m.m[2][3] = pos.z; m.m[3][3] = 1;
    v3 dir = v_normalized(v_sub(look, pos));
    if (v_len(v_cross(v_normalized(up), dir)) == 0) return -1;
    v3 right = v_normalized(v_cross(v_normalized(up), dir));
    v3 nup = v_cross(dir, right);
    m.m[0][0] = right.x; m.m[1][0] = right.y; m.m[2][0] = right.z; m.m[3][0] = 0.;
    m.m[0][1] = nup.x; m.m[1][1] = nup.y; m.m[2][1] = nup.z; m.m[3][1] = 0.;
    m.m[0][2] = dir.x; m.m[1][2] = dir.y; m.m[2][2] = dir.z; m.m[3][2] = 0.;
    out->m = m;
    return orc_m_inverse(&m, &out->m_inv);
}
/* transform.go:492-502 */
pbrt_transform orc_perspective(double fov, double n, double f) {
    pbrt_matrix4x4 p;
    memset(&p, 0, sizeof(p));
    p.m[0][0] = 1; p.m[1][1] = 1;
    p.m[2][2] = f / (f - n); p.m[2][3] = -f * n / (f - n);
    p.m[3][2] = 1;
    double inv_tan = 1.0 / go_tan(go_radians(fov) / 2);
    pbrt_transform s = orc_scale(inv_tan, inv_tan, 1);
    pbrt_transform pt = new_transform(&p);
    return orc_xf_mul(&s, &pt);
}

/* ================================================================ bounds */
typedef struct { v3 mn, mx; int has_min, has_max; } bounds3;

static v3 min_point(v3 a, v3 b) { return V3(go_min(a.x, b.x), go_min(a.y, b.y), go_min(a.z, b.z)); }
static v3 max_point(v3 a, v3 b) { return V3(go_max(a.x, b.x), go_max(a.y, b.y), go_max(a.z, b.z)); }
/* bounds.go:209-238 (nil-pointer semantics of the zero Bounds3) */
static void b_union_point(bounds3* b, v3 p) {
    if (!b->has_min) { b->mn = p; b->has_min = 1; }
    if (!b->has_max) { b->mx = p; b->has_max = 1; }
    b->mn = min_point(b->mn, p);
    b->mx = max_point(b->mx, p);
}
static void b_union(bounds3* b, const bounds3* b2) {
    if (!b->has_min) { b->mn = b2->mn; b->has_min = b2->has_min; }
    if (!b->has_max) { b->mx = b2->mx; b->has_max = b2->has_max; }
    if (!b2->has_min || !b2->has_max) return;
    b->mn = min_point(b->mn, b2->mn);
    b->mx = max_point(b->mx, b2->mx);
}
static double b_surface_area(const bounds3* b) {
    v3 d = v_sub(b->mx, b->mn);
    return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
}
static int b_max_extent(const bounds3* b) {
    v3 d = v_sub(b->mx, b->mn);
    if (d.x > d.y && d.x > d.z) return 0;
    if (d.y > d.z) return 1;
    return 2;
}
static v3 b_offset(const bounds3* b, v3 p) {
    v3 o = v_sub(p, b->mn);
    if (b->mx.x > b->mn.x) o.x /= b->mx.x - b->mn.x;
    if (b->mx.y > b->mn.y) o.y /= b->mx.y - b->mn.y;
    if (b->mx.z > b->mn.z) o.z /= b->mx.z - b->mn.z;
    return o;
}
/* transform.go:336-345 */
static bounds3 xf_bounds(const pbrt_transform* t, v3 mn, v3 mx) {
    bounds3 r;
    v3 c = xf_point(t, mn, V3(0, 0, 0), NULL);
    r.mn = c; r.mx = c; r.has_min = r.has_max = 1;
    for (int i = 1; i < 8; i++) {
        v3 corner = V3((i & 1) ? mx.x : mn.x, ((i & 2) / 2) ? mx.y : mn.y, ((i & 4) / 4) ? mx.z : mn.z);
        c = xf_point(t, corner, V3(0, 0, 0), NULL);
        b_union_point(&r, c);
    }
    return r;
}

/* ================================================================ shapes */
pbrt_shape_desc orc_sphere(pbrt_transform o2w, int rev, double radius, double zmin, double zmax, double phimax) {
    pbrt_shape_desc s;
    memset(&s, 0, sizeof(s));
    s.type = PBRT_SHAPE_SPHERE;
    s.reverse_orientation = rev;
    s.object_to_world = o2w;
    s.radius = radius;
    s.z_min = go_clamp(go_min(zmin, zmax), -radius, radius);
    s.z_max = go_clamp(go_max(zmin, zmax), -radius, radius);
    s.theta_min = go_acos(go_clamp(go_min(zmin, zmax) / radius, -1, 1));
    s.theta_max = go_acos(go_clamp(go_max(zmin, zmax) / radius, -1, 1));
    s.phi_max = go_radians(go_clamp(phimax, 0, 360));
    return s;
}
pbrt_shape_desc orc_disk(pbrt_transform o2w, double height, double radius, double inner, double phimax) {
    pbrt_shape_desc s;
    memset(&s, 0, sizeof(s));
    s.type = PBRT_SHAPE_DISK;
    s.object_to_world = o2w;
    s.height = height;
    s.radius = radius;
    s.inner_radius = inner;
    s.phi_max = go_radians(go_clamp(phimax, 0, 360));
    return s;
}
static bounds3 shape_world_bound(const pbrt_shape_desc* s) {
    if (s->type == PBRT_SHAPE_SPHERE)
        return xf_bounds(&s->object_to_world, V3(-s->radius, -s->radius, s->z_min),
                         V3(s->radius, s->radius, s->z_max));
    return xf_bounds(&s->object_to_world, V3(-s->radius, -s->radius, s->height),
                     V3(s->radius, s->radius, s->height));
}
static bounds3 prim_world_bound(const orc_scene* sc, const pbrt_primitive_desc* p) {
    bounds3 b = shape_world_bound(&sc->shapes[p->shape]);
    if (p->kind == PBRT_PRIM_TRANSFORMED) return xf_bounds(&p->prim_to_world, b.mn, b.mx);
    return b;
}

/* =================================================================== BVH */
typedef struct { int prim; bounds3 b; v3 c; } prim_info;
typedef struct build_node {
    bounds3 b;
    struct build_node* ch[2];
    int axis;
    int64_t first, n;
} build_node;

typedef struct {
    const orc_scene* sc;
    int max_prims;
    prim_info* info;
    int* ordered;
    int n_ordered;
    build_node* pool;
    int n_nodes;
    int failed;
} bvh_build;

static build_node* new_node(bvh_build* bb) {
    build_node* n = &bb->pool[bb->n_nodes++];
    memset(n, 0, sizeof(*n));
    return n;
}
static void init_leaf(bvh_build* bb, build_node* node, int64_t start, int64_t end, bounds3 b) {
    node->first = bb->n_ordered;
    for (int64_t i = start; i < end; i++) bb->ordered[bb->n_ordered++] = bb->info[i].prim;
    node->n = end - start;
    node->b = b;
}
static int sah_bucket(const bounds3* cb, v3 c, int dim) {
    int b = 12 * (int)go_f2i(v_idx(b_offset(cb, c), dim));
    if (b == 12) b = 11;
    return b;
}
/* bvh.go:163-175: pivot moved to `end`, Lomuto pass over [start,end), pivot
 * swapped to the returned position */
static int64_t partition_at(prim_info* in, int64_t start, int64_t end, int64_t pivot, int mode,
                            int dim, const bounds3* cb, int split_bucket) {
    prim_info pv = in[pivot];
    prim_info t = in[pivot]; in[pivot] = in[end]; in[end] = t;
    for (int64_t i = start; i < end; i++) {
        int take;
        if (mode == 0) take = v_idx(in[i].c, dim) < v_idx(pv.c, dim);
        else take = sah_bucket(cb, in[i].c, dim) <= split_bucket;
        if (take) { t = in[start]; in[start] = in[i]; in[i] = t; start++; }
    }
    t = in[end]; in[end] = in[start]; in[start] = t;
    return start;
}
/* bvh.go:272-411 RecursiveBuild, SplitSAH */
static build_node* recursive_build(bvh_build* bb, int64_t start, int64_t end) {
    build_node* node = new_node(bb);
    bounds3 bounds;
    memset(&bounds, 0, sizeof(bounds));
    for (int64_t i = start; i < end; i++) b_union(&bounds, &bb->info[i].b);
    int64_t np = end - start;
    if (np == 1) { init_leaf(bb, node, start, end, bounds); return node; }
    bounds3 cb;
    memset(&cb, 0, sizeof(cb));
    for (int64_t i = start; i < end; i++) b_union_point(&cb, bb->info[i].c);
    if (np == 0 || !cb.has_min) { bb->failed = 1; return node; }  /* nil deref in Go */
    int dim = b_max_extent(&cb);
    int64_t mid = (start + end) / 2;
    if (v_idx(cb.mx, dim) == v_idx(cb.mn, dim)) { init_leaf(bb, node, start, end, bounds); return node; }
    if (np <= 2) {
        partition_at(bb->info, start, end - 1, mid, 0, dim, &cb, 0);
    } else {
        bounds3 bk[12];
        int cnt[12] = {0};
        memset(bk, 0, sizeof(bk));
        for (int64_t i = start; i < end; i++) {
            int b = sah_bucket(&cb, bb->info[i].c, dim);
            cnt[b]++;
            b_union(&bk[b], &bb->info[i].b);
        }
        double cost[11];
        for (int i = 0; i < 11; i++) {
            bounds3 b0, b1;
            memset(&b0, 0, sizeof(b0)); memset(&b1, 0, sizeof(b1));
            int c0 = 0, c1 = 0;
            for (int j = 0; j <= i; j++) { b_union(&b0, &bk[j]); c0 += cnt[j]; }
            for (int j = i + 1; j < 12; j++) { b_union(&b1, &bk[j]); c1 += cnt[j]; }
            cost[i] = 1.0 + ((double)c0 * b_surface_area(&b0) + (double)c1 * b_surface_area(&b1)) /
                                b_surface_area(&bounds);
        }
        double min_cost = cost[0];
        int min_b = 0;
        for (int i = 1; i < 11; i++)
            if (cost[i] < min_cost) { min_cost = cost[i]; min_b = i; }
        double leaf_cost = (double)np;
        if (np > bb->max_prims || min_cost < leaf_cost) {
            mid = partition_at(bb->info, start, end - 1, end - 1, 1, dim, &cb, min_b);
        } else {
            init_leaf(bb, node, start, end, bounds);
            return node;
        }
    }
    node->axis = dim;
    node->n = 0;
    node->ch[0] = recursive_build(bb, start, mid);
    node->ch[1] = recursive_build(bb, mid, end);
    node->b = node->ch[0]->b;
    b_union(&node->b, &node->ch[1]->b);
    return node;
}
/* bvh.go:632-651 */
static uint32_t flatten(orc_scene* sc, build_node* node, uint32_t* offset) {
    pbrt_bvh_node* ln = &sc->nodes[*offset];
    memset(ln, 0, sizeof(*ln));
    ln->bmin[0] = node->b.mn.x; ln->bmin[1] = node->b.mn.y; ln->bmin[2] = node->b.mn.z;
    ln->bmax[0] = node->b.mx.x; ln->bmax[1] = node->b.mx.y; ln->bmax[2] = node->b.mx.z;
    uint32_t my = (*offset)++;
    if (node->n > 0) {
        ln->offset = (uint32_t)node->first;
        ln->n_prims = (uint16_t)node->n;
    } else {
        ln->axis = (uint8_t)node->axis;
        ln->n_prims = 0;
        flatten(sc, node->ch[0], offset);
        ln->offset = flatten(sc, node->ch[1], offset);
    }
    return my;
}

/* ================================================================= scene */
int orc_scene_finalize(orc_scene* sc, int max_prims) {
    int n = sc->n_prims_in;
    bvh_build bb;
    memset(&bb, 0, sizeof(bb));
    bb.sc = sc;
    bb.max_prims = (int)go_min(255, (double)max_prims);
    bb.info = (prim_info*)calloc((size_t)n, sizeof(prim_info));
    bb.ordered = (int*)calloc((size_t)n, sizeof(int));
    bb.pool = (build_node*)calloc((size_t)(2 * n + 1), sizeof(build_node));
    for (int i = 0; i < n; i++) {
        bb.info[i].prim = i;
        bb.info[i].b = prim_world_bound(sc, &sc->prims_in[i]);
        bb.info[i].c = v_add(v_muls(bb.info[i].b.mn, 0.5), v_muls(bb.info[i].b.mx, 0.5));
    }
    if (n == 0) { free(bb.info); free(bb.ordered); free(bb.pool); sc->n_nodes = 0; return 0; }
    build_node* root = recursive_build(&bb, 0, n);
    if (bb.failed) { free(bb.info); free(bb.ordered); free(bb.pool); return -1; }
    sc->n_nodes = bb.n_nodes;
    uint32_t off = 0;
    flatten(sc, root, &off);
    for (int i = 0; i < n; i++) {
        sc->prims[i] = sc->prims_in[bb.ordered[i]];
        sc->order[i] = bb.ordered[i];
    }
    free(bb.info); free(bb.ordered); free(bb.pool);

    /* scene.go:16-36: worldBound = BVH root; Distant.Preprocess (distant.go:36-38) */
    for (int k = 0; k < 3; k++) { sc->world_min[k] = sc->nodes[0].bmin[k]; sc->world_max[k] = sc->nodes[0].bmax[k]; }
    v3 mn = V3(sc->world_min[0], sc->world_min[1], sc->world_min[2]);
    v3 mx = V3(sc->world_max[0], sc->world_max[1], sc->world_max[2]);
    v3 center = v_divs(v_add(mn, mx), 2.0);
    double radius = 0;
    if (center.x >= mn.x && center.x <= mx.x && center.y >= mn.y && center.y <= mx.y && center.z >= mn.z &&
        center.z <= mx.z)
        radius = v_dist(center, mx);
    for (int i = 0; i < sc->n_lights; i++)
        if (sc->lights[i].type == PBRT_LIGHT_DISTANT) sc->lights[i].world_radius = radius;
    return 0;
}

static void set_film_camera(orc_scene* sc, int64_t w, int64_t h, pbrt_transform cam2world, double fov,
                            double lens, double focal) {
    pbrt_film_desc* f = &sc->film;
    memset(f, 0, sizeof(*f));
    f->res_x = w; f->res_y = h;
    /* film.go:43-46 with crop [0,1]^2 */
    f->crop_min_x = go_f2i(ceil((double)w * 0)); f->crop_min_y = go_f2i(ceil((double)h * 0));
    f->crop_max_x = go_f2i(ceil((double)w * 1)); f->crop_max_y = go_f2i(ceil((double)h * 1));
    f->filter_radius_x = 1; f->filter_radius_y = 1;
    f->max_sample_luminance = 1.0;
    for (int i = 0; i < 256; i++) f->filter_table[i] = 1.0;   /* BoxFilter.Evaluate */
    /* camera.go:106-124 with screenWindow = crop [0,1]^2 (server.go:159) */
    pbrt_transform cs = orc_perspective(fov, 1e-2, 1000.0);
    pbrt_transform s2r = orc_scale((double)w, (double)h, 1.0);
    pbrt_transform t1 = orc_scale(1.0 / (1.0 - 0.0), 1.0 / (0.0 - 1.0), 1.0);
    s2r = orc_xf_mul(&s2r, &t1);
    pbrt_transform t2 = orc_translate(-0.0, -1.0, 0);
    s2r = orc_xf_mul(&s2r, &t2);
    pbrt_transform r2s = xf_inverse(&s2r);
    pbrt_transform csi = xf_inverse(&cs);
    sc->camera.raster_to_camera = orc_xf_mul(&csi, &r2s);
    sc->camera.camera_to_world = cam2world;
    sc->camera.lens_radius = lens;
    sc->camera.focal_distance = focal;
    sc->camera.shutter_open = 0.0;
    sc->camera.shutter_close = 0.0;   /* camera.go:116 passes shutterOpen twice (#19) */
}

int orc_add_shape(orc_scene* sc, pbrt_shape_desc s) { sc->shapes[sc->n_shapes] = s; return sc->n_shapes++; }
int orc_add_material(orc_scene* sc, pbrt_material_desc m) { sc->materials[sc->n_materials] = m; return sc->n_materials++; }
static pbrt_material_desc matte_const(double r, double g, double b) {
    pbrt_material_desc m;
    memset(&m, 0, sizeof(m));
    m.kd_type = PBRT_TEX_CONSTANT;
    m.kd[0] = r; m.kd[1] = g; m.kd[2] = b;
    return m;
}

/* server.go:94-104: the floor's Checkerboard2D (1, 0.18), planar mapping vs (.2, 0, 0), vt (0, 0, .2) */
static pbrt_material_desc readme_checker(void) {
    pbrt_material_desc chk;
    memset(&chk, 0, sizeof(chk));
    chk.kd_type = PBRT_TEX_CHECKERBOARD2D;
    chk.vs[0] = .2; chk.vt[2] = .2; chk.ds = 0; chk.dt = 0;
    chk.tex1[0] = chk.tex1[1] = chk.tex1[2] = 1.0;
    chk.tex2[0] = chk.tex2[1] = chk.tex2[2] = 0.18;
    return chk;
}

/* server.go:106-159: the four lights, the film and the camera */
static void readme_lights_camera(orc_scene* sc, int64_t w, int64_t h) {
    /* lights, server.go:106-130 */
    pbrt_light_desc l;
    memset(&l, 0, sizeof(l));
    {
        pbrt_transform l2w = orc_translate(-100, 100, 100);
        v3 wl = v_normalized(xf_vector(&l2w, V3(-1, 1, 1)));
        l.type = PBRT_LIGHT_DISTANT;
        l.spectrum[0] = l.spectrum[1] = l.spectrum[2] = 0.05;
        l.w_light[0] = wl.x; l.w_light[1] = wl.y; l.w_light[2] = wl.z;
        sc->lights[sc->n_lights++] = l;
    }
    {
        double pos[2][3] = {{50, 20, 50}, {-50, 30, -50}};
        double I[2] = {100, 50};
        for (int k = 0; k < 2; k++) {
            memset(&l, 0, sizeof(l));
            pbrt_transform l2w = orc_translate(pos[k][0], pos[k][1], pos[k][2]);
            v3 pl = xf_point(&l2w, V3(0, 0, 0), V3(0, 0, 0), NULL);
            l.type = PBRT_LIGHT_POINT;
            l.spectrum[0] = l.spectrum[1] = l.spectrum[2] = I[k];
            l.p_light[0] = pl.x; l.p_light[1] = pl.y; l.p_light[2] = pl.z;
            sc->lights[sc->n_lights++] = l;
        }
    }
    {
        memset(&l, 0, sizeof(l));
        int ls = orc_add_shape(sc, orc_sphere(orc_translate(-10, 5, 20), 0, 5.0, -5.0, 5.0, 360.0));
        l.type = PBRT_LIGHT_DIFFUSE_AREA;
        l.shape = ls;
        l.two_sided = 0;
        l.spectrum[0] = l.spectrum[1] = l.spectrum[2] = 0.2;
        sc->lights[sc->n_lights++] = l;
    }
    /* camera, server.go:152-159 */
    pbrt_transform cam;
    orc_look_at(V3(150, 150, 150), V3(0, 0, 0), V3(0, 1, 0), &cam);
    pbrt_transform ry = orc_rotate(1, -30), rxx = orc_rotate(0, -30);
    cam = orc_xf_mul(&cam, &ry);
    cam = orc_xf_mul(&cam, &rxx);
    set_film_camera(sc, w, h, cam, 100, 0, 20);
}

/* internal/render/server.go:29-164, up to (not including) the BVH build */
static orc_scene* readme_unbuilt(int64_t w, int64_t h) {
    orc_scene* sc = (orc_scene*)calloc(1, sizeof(orc_scene));
    int n = 8;
    for (int k = 1; k < n; k++) {
        for (int i = 0; i < 3; i++) {
            double x = 0, y = 0, z = 0, cr = 0, cg = 0, cb = 0;
            if (i == 0) { x = (double)k / (double)n * 100; cr = 1; }
            if (i == 1) { y = (double)k / (double)n * 100; cg = 1; }
            if (i == 2) { z = (double)k / (double)n * 100; cb = 1; }
            double radius = 2.0;
            y = go_max(y, radius / 2);
            pbrt_transform o2w = orc_translate(0, 0, 0);
            int s = orc_add_shape(sc, orc_sphere(o2w, 1, radius, -radius, radius, 360.0));
            int m = orc_add_material(sc, matte_const(cr, cg, cb));
            pbrt_primitive_desc p;
            memset(&p, 0, sizeof(p));
            p.kind = PBRT_PRIM_TRANSFORMED; p.shape = s; p.material = m;
            p.prim_to_world = orc_translate(x, y, z);
            sc->prims_in[sc->n_prims_in++] = p;
        }
    }
    int mchk = orc_add_material(sc, readme_checker());
    pbrt_transform t0 = orc_translate(0, 0, 0);
    pbrt_transform rx = orc_rotate(0, 90);
    pbrt_transform dx1 = orc_xf_mul(&t0, &rx);
    int d1 = orc_add_shape(sc, orc_disk(dx1, 0.01, 10000, 0, 360));
    int d2 = orc_add_shape(sc, orc_disk(orc_translate(-50, 0, -50), 0.01, 10000, 0, 360));
    pbrt_primitive_desc p;
    memset(&p, 0, sizeof(p));
    p.kind = PBRT_PRIM_GEOMETRIC; p.shape = d1; p.material = mchk;
    sc->prims_in[sc->n_prims_in++] = p;
    p.shape = d2;
    sc->prims_in[sc->n_prims_in++] = p;

    readme_lights_camera(sc, w, h);
    return sc;
}

orc_scene* orc_scene_readme(int64_t w, int64_t h) {
    orc_scene* sc = readme_unbuilt(w, h);
    orc_scene_finalize(sc, 2);   /* server.go:162: NewBVH(primitives, 2, ...) */
    return sc;
}

/* The README scene plus internal/render/server.go:67-91's commented-out sphere:
 * radius 5 at (50, 2.5, 50) under a Translate, material NewGlass with Kr = Kt
 * = 0.5, index 1.5 and no roughness (glass.go:15-26); special = 0 makes it a
 * black Matte instead. mirror = 1 adds a NewMirror (Kr 0.9, mirror.go:9-14)
 * sphere of radius 5 at (35, 5, 45). The primitives follow the README's in
 * construction order (glass, then mirror), then the BVH is built with 2
 * primitives per node as server.go:162 does. Restated here from that
 * description, independently of the product's scene builder, so a
 * construction error on either side shows up as a parity failure. */
orc_scene* orc_scene_readme_glass(int64_t w, int64_t h, int special, int mirror) {
    orc_scene* sc = readme_unbuilt(w, h);
    pbrt_material_desc g;
    memset(&g, 0, sizeof(g));
    if (special) {
        g.type = PBRT_MAT_GLASS;
        for (int i = 0; i < 3; i++) { g.kr[i] = 0.5; g.kt[i] = 0.5; }
        g.u_roughness = 0.0;
        g.v_roughness = 0.0;
        g.eta = 1.5;
    } else {
        g = matte_const(0.0, 0.0, 0.0);
    }
    double pos[2][3] = {{50, 2.5, 50}, {35, 5.0, 45}};
    for (int k = 0; k < (mirror ? 2 : 1); k++) {
        pbrt_material_desc m;
        if (k == 0) {
            m = g;
        } else {
            memset(&m, 0, sizeof(m));
            m.type = PBRT_MAT_MIRROR;
            m.kr[0] = m.kr[1] = m.kr[2] = 0.9;
        }
        int mi = orc_add_material(sc, m);
        int s = orc_add_shape(sc, orc_sphere(orc_translate(0, 0, 0), 0, 5.0, -5.0, 5.0, 360.0));
        pbrt_primitive_desc p;
        memset(&p, 0, sizeof(p));
        p.kind = PBRT_PRIM_TRANSFORMED; p.shape = s; p.material = mi;
        p.prim_to_world = orc_translate(pos[k][0], pos[k][1], pos[k][2]);
        sc->prims_in[sc->n_prims_in++] = p;
    }
    orc_scene_finalize(sc, 2);
    return sc;
}

/* Extension (BASELINE configs D/E; no reference arithmetic, parity unpinned
 * against Go): the procedural height field of DESIGN.md §1, restated here
 * from its description so the oracle's side of the mesh fixtures does not
 * come from the product's builder. quads x quads cells over [-100, 200]^2
 * (x, z), two triangles per cell, counter-clockwise from +y; vertex height
 * y = 2 Sin(.3x) Cos(.2z) + 3 noise(x, z) in float64 (Go's Sin / Cos), stored
 * as float32; noise = value noise on the lattice (x, z) / 10: lattice values
 * in [-1, 1) from a splitmix64 finalizer of seed * phi ^ i * c1 ^ j * c2,
 * blended with smoothstep weights. The README's checker material, lights,
 * film and camera; no analytic primitive. The world bound is the union of the
 * triangles' vertices (the aggregate holds the mesh). */
static double hf_lattice(uint64_t seed, int64_t i, int64_t j) {
    uint64_t z = (seed * 0x9e3779b97f4a7c15ULL) ^ ((uint64_t)i * 0xbf58476d1ce4e5b9ULL) ^
                 ((uint64_t)j * 0x94d049bb133111ebULL);
    z += 0x9e3779b97f4a7c15ULL;   /* splitmix64 */
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return (double)(z >> 11) / 9007199254740992.0 * 2.0 - 1.0;
}
static double hf_height(uint64_t seed, double x, double z) {
    double gx = x / 10.0, gz = z / 10.0, fx = floor(gx), fz = floor(gz);
    int64_t i = (int64_t)fx, j = (int64_t)fz;
    double tx = gx - fx, tz = gz - fz;
    double sx = tx * tx * (3.0 - 2.0 * tx), sz = tz * tz * (3.0 - 2.0 * tz);
    double v00 = hf_lattice(seed, i, j), v10 = hf_lattice(seed, i + 1, j);
    double v01 = hf_lattice(seed, i, j + 1), v11 = hf_lattice(seed, i + 1, j + 1);
    double near = v00 + (v10 - v00) * sx, far = v01 + (v11 - v01) * sx;
    double noise = near + (far - near) * sz;
    return 2.0 * go_sin(0.3 * x) * go_cos(0.2 * z) + 3.0 * noise;
}
orc_scene* orc_scene_heightfield(int64_t w, int64_t h, int quads, uint64_t seed) {
    if (quads < 1 || quads > 46340) return NULL;
    orc_scene* sc = (orc_scene*)calloc(1, sizeof(orc_scene));
    int mchk = orc_add_material(sc, readme_checker());
    int64_t nv = (int64_t)(quads + 1) * (quads + 1), nt = 2 * (int64_t)quads * quads;
    sc->mesh_p = (float*)malloc(sizeof(float) * 3 * (size_t)nv);
    sc->mesh_idx = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)nt);
    for (int64_t j = 0; j <= quads; j++)
        for (int64_t i = 0; i <= quads; i++) {
            double x = -100.0 + 300.0 * (double)i / (double)quads, z = -100.0 + 300.0 * (double)j / (double)quads;
            float* v = sc->mesh_p + 3 * (j * (quads + 1) + i);
            v[0] = (float)x;
            v[1] = (float)hf_height(seed, x, z);
            v[2] = (float)z;
        }
    int32_t* t = sc->mesh_idx;
    for (int64_t j = 0; j < quads; j++)
        for (int64_t i = 0; i < quads; i++) {
            int32_t a = (int32_t)(j * (quads + 1) + i), b = a + 1, c = a + (quads + 1), d = c + 1;
            *t++ = a; *t++ = c; *t++ = b;   /* (i, j), (i, j+1), (i+1, j) */
            *t++ = b; *t++ = c; *t++ = d;   /* (i+1, j), (i, j+1), (i+1, j+1) */
        }
    memset(&sc->mesh, 0, sizeof(sc->mesh));
    sc->mesh.n_vertices = (int32_t)nv;
    sc->mesh.n_triangles = (int32_t)nt;
    sc->mesh.material = mchk;
    sc->mesh.reverse_orientation = 0;
    sc->mesh.p = sc->mesh_p;
    sc->mesh.indices = sc->mesh_idx;
    sc->n_meshes = 1;
    readme_lights_camera(sc, w, h);
    orc_scene_finalize(sc, 2);   /* no analytic primitive: no nodes */
    /* world bound: the union of the triangles' vertices (bounds.go:54-66 Union) */
    for (int64_t k = 0; k < 3 * nt; k++) {
        const float* v = sc->mesh_p + 3 * (int64_t)sc->mesh_idx[k];
        for (int a = 0; a < 3; a++) {
            double x = (double)v[a];
            sc->world_min[a] = k == 0 ? x : go_min(sc->world_min[a], x);
            sc->world_max[a] = k == 0 ? x : go_max(sc->world_max[a], x);
        }
    }
    v3 mn = V3(sc->world_min[0], sc->world_min[1], sc->world_min[2]);
    v3 mx = V3(sc->world_max[0], sc->world_max[1], sc->world_max[2]);
    v3 center = v_divs(v_add(mn, mx), 2.0);   /* bounds.go:105-112 BoundingSphere */
    double radius = 0;
    if (center.x >= mn.x && center.x <= mx.x && center.y >= mn.y && center.y <= mx.y && center.z >= mn.z &&
        center.z <= mx.z)
        radius = v_dist(center, mx);
    for (int i = 0; i < sc->n_lights; i++)
        if (sc->lights[i].type == PBRT_LIGHT_DISTANT) sc->lights[i].world_radius = radius;
    return sc;
}

/* Cornell-style box from reference types only */
orc_scene* orc_scene_cornell(int64_t w, int64_t h) {
    orc_scene* sc = (orc_scene*)calloc(1, sizeof(orc_scene));
    int white = orc_add_material(sc, matte_const(0.73, 0.73, 0.73));
    int red = orc_add_material(sc, matte_const(0.63, 0.065, 0.05));
    int green = orc_add_material(sc, matte_const(0.14, 0.45, 0.091));
    /* walls: Disk(h=0, r=20) placed by Translate * Rotate */
    struct { double t[3]; int axis; double deg; int mat; } walls[6] = {
        {{5, 0, 5}, 0, 90, 0},  {{5, 10, 5}, 0, 90, 0}, {{0, 5, 5}, 1, 90, 1},
        {{10, 5, 5}, 1, 90, 2}, {{5, 5, 0}, -1, 0, 0},  {{5, 5, 10}, -1, 0, 0}};
    for (int i = 0; i < 6; i++) {
        pbrt_transform t = orc_translate(walls[i].t[0], walls[i].t[1], walls[i].t[2]);
        if (walls[i].axis >= 0) {
            pbrt_transform r = orc_rotate(walls[i].axis, walls[i].deg);
            t = orc_xf_mul(&t, &r);
        }
        int s = orc_add_shape(sc, orc_disk(t, 0, 20, 0, 360));
        pbrt_primitive_desc p;
        memset(&p, 0, sizeof(p));
        p.kind = PBRT_PRIM_GEOMETRIC; p.shape = s;
        p.material = walls[i].mat == 0 ? white : (walls[i].mat == 1 ? red : green);
        sc->prims_in[sc->n_prims_in++] = p;
    }
    double sp[2][4] = {{3, 1.5, 6, 1.5}, {7, 2, 4, 2}};
    for (int i = 0; i < 2; i++) {
        int s = orc_add_shape(sc, orc_sphere(orc_translate(0, 0, 0), 0, sp[i][3], -sp[i][3], sp[i][3], 360.0));
        pbrt_primitive_desc p;
        memset(&p, 0, sizeof(p));
        p.kind = PBRT_PRIM_TRANSFORMED; p.shape = s; p.material = white;
        p.prim_to_world = orc_translate(sp[i][0], sp[i][1], sp[i][2]);
        sc->prims_in[sc->n_prims_in++] = p;
    }
    pbrt_light_desc l;
    memset(&l, 0, sizeof(l));
    pbrt_transform l2w = orc_translate(5, 9.5, 5);
    v3 pl = xf_point(&l2w, V3(0, 0, 0), V3(0, 0, 0), NULL);
    l.type = PBRT_LIGHT_POINT;
    l.spectrum[0] = l.spectrum[1] = l.spectrum[2] = 10;
    l.p_light[0] = pl.x; l.p_light[1] = pl.y; l.p_light[2] = pl.z;
    sc->lights[sc->n_lights++] = l;
    memset(&l, 0, sizeof(l));
    int ls = orc_add_shape(sc, orc_sphere(orc_translate(5, 9, 5), 0, 0.5, -0.5, 0.5, 360.0));
    l.type = PBRT_LIGHT_DIFFUSE_AREA; l.shape = ls;
    l.spectrum[0] = l.spectrum[1] = l.spectrum[2] = 5;
    sc->lights[sc->n_lights++] = l;
    pbrt_transform cam;
    orc_look_at(V3(5, 5, 0.5), V3(5, 5, 10), V3(0, 1, 0), &cam);
    set_film_camera(sc, w, h, cam, 90, 0, 20);
    orc_scene_finalize(sc, 2);
    return sc;
}

void orc_scene_desc(orc_scene* sc, pbrt_scene_desc* d) {
    memset(d, 0, sizeof(*d));
    d->n_shapes = sc->n_shapes; d->n_materials = sc->n_materials; d->n_prims = sc->n_prims_in;
    d->n_nodes = sc->n_nodes; d->n_lights = sc->n_lights;
    d->shapes = sc->shapes; d->materials = sc->materials; d->prims = sc->prims;
    d->nodes = sc->nodes; d->lights = sc->lights;
    d->camera = sc->camera; d->film = sc->film;
    for (int k = 0; k < 3; k++) { d->world_min[k] = sc->world_min[k]; d->world_max[k] = sc->world_max[k]; }
    if (sc->n_meshes) {
        d->n_meshes = 1;
        d->meshes = &sc->mesh;
    }
}
void orc_scene_free(orc_scene* sc) {
    if (!sc) return;
    free(sc->mesh_p);
    free(sc->mesh_idx);
    free(sc);
}

/* bvh.go:163-175 PartitionPrimitiveInfoAt with bvh_test.go's centroid-x
 * predicate (mode 0, dim 0) on (prim, cx) records; for tests/ */
int64_t orc_partition_at_x(int32_t* prim, double* cx, int64_t n, int64_t start, int64_t end, int64_t pivot) {
    if (n <= 0 || start < 0 || end >= n || pivot < start || pivot > end || start > end) return -1;
    prim_info* in = (prim_info*)calloc((size_t)n, sizeof(prim_info));
    for (int64_t i = 0; i < n; i++) { in[i].prim = prim[i]; in[i].c = V3(cx[i], 0, 0); }
    int64_t m = partition_at(in, start, end, pivot, 0, 0, NULL, 0);
    for (int64_t i = 0; i < n; i++) { prim[i] = in[i].prim; cx[i] = in[i].c.x; }
    free(in);
    return m;
}
