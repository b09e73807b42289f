// scene_builder.cpp — host-side scene construction with go-pbrt semantics
// (implements include/pbrt_scene.h).
//
// The Go side of an integration builds its scene with go-pbrt itself and only
// flattens it into a pbrt_scene_desc. Without a Go toolchain this file plays
// that role: every constructor restates the reference's arithmetic so the
// descriptor (matrices, shapes, BVH order and bounds, Distant light radius) is
// bit-identical to what go-pbrt computes. Citations per function.
#pragma clang fp contract(off)

#include <cstring>
#include <memory>
#include <vector>

#include "../../include/pbrt_diag.h"
#include "../../include/pbrt_scene.h"
#include "pbrt_core.h"

using namespace pbrt;
namespace gm = gomath;

namespace {

pbrt_matrix4x4 identity4() {
    pbrt_matrix4x4 r;
    std::memset(&r, 0, sizeof(r));
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0;
    return r;
}
// transform.go:62-70 — the last term reads the LEFT matrix's row 3 (#18)
pbrt_matrix4x4 matmul(const pbrt_matrix4x4& a, const pbrt_matrix4x4& b) {
    pbrt_matrix4x4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] + a.m[i][3] * a.m[3][j];
    return r;
}
pbrt_matrix4x4 transpose(const pbrt_matrix4x4& a) {
    pbrt_matrix4x4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.m[i][j] = a.m[j][i];
    return r;
}

// pkg/pbrt/bounds.go Bounds3 with the nil-pointer semantics of its zero value
struct Bounds {
    V3 mn{0, 0, 0}, mx{0, 0, 0};
    bool has_min = false, has_max = false;
};
V3 min_pt(V3 a, V3 b) { return V3{gm::min(a.x, b.x), gm::min(a.y, b.y), gm::min(a.z, b.z)}; }
V3 max_pt(V3 a, V3 b) { return V3{gm::max(a.x, b.x), gm::max(a.y, b.y), gm::max(a.z, b.z)}; }
void union_point(Bounds& b, V3 p) {  // bounds.go:209-219
    if (!b.has_min) { b.mn = p; b.has_min = true; }
    if (!b.has_max) { b.mx = p; b.has_max = true; }
    b.mn = min_pt(b.mn, p);
    b.mx = max_pt(b.mx, p);
}
void union_bounds(Bounds& b, const Bounds& o) {  // bounds.go:221-238
    if (!b.has_min) { b.mn = o.mn; b.has_min = o.has_min; }
    if (!b.has_max) { b.mx = o.mx; b.has_max = o.has_max; }
    if (!o.has_min || !o.has_max) return;
    b.mn = min_pt(b.mn, o.mn);
    b.mx = max_pt(b.mx, o.mx);
}
double surface_area(const Bounds& b) {
    V3 d = b.mx - b.mn;
    return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
}
int maximum_extent(const Bounds& b) {
    V3 d = b.mx - b.mn;
    if (d.x > d.y && d.x > d.z) return 0;
    if (d.y > d.z) return 1;
    return 2;
}
V3 offset_in(const Bounds& b, V3 p) {  // bounds.go:195-207
    V3 o = p - b.mn;
    if (b.mx.x > b.mn.x) o.x /= b.mx.x - b.mn.x;
    if (b.mx.y > b.mn.y) o.y /= b.mx.y - b.mn.y;
    if (b.mx.z > b.mn.z) o.z /= b.mx.z - b.mn.z;
    return o;
}
// transform.go:336-345 TransformBounds (corner order of bounds.go:114-120)
Bounds transform_bounds(const pbrt_transform& t, V3 mn, V3 mx) {
    Bounds r;
    V3 c = xf_point(t.m, mn, V3{0, 0, 0}, nullptr);
    r.mn = c; r.mx = c; r.has_min = r.has_max = true;
    for (int i = 1; i < 8; i++) {
        V3 corner{(i & 1) ? mx.x : mn.x, ((i & 2) / 2) ? mx.y : mn.y, ((i & 4) / 4) ? mx.z : mn.z};
        union_point(r, xf_point(t.m, corner, V3{0, 0, 0}, nullptr));
    }
    return r;
}

// -------------------------------------------------------------------- BVH
struct PrimInfo {
    int prim;
    Bounds bounds;
    V3 centroid;
};
struct BuildNode {
    Bounds bounds;
    int child[2] = {-1, -1};
    int axis = 0;
    int64_t first = 0, n = 0;
};

struct BVHBuilder {
    std::vector<PrimInfo> info;
    std::vector<BuildNode> nodes;
    std::vector<int> ordered;
    int max_prims = 2;
    bool failed = false;

    void leaf(BuildNode& nd, int64_t start, int64_t end, const Bounds& b) {  // bvh.go:45-52
        nd.first = (int64_t)ordered.size();
        for (int64_t i = start; i < end; i++) ordered.push_back(info[i].prim);
        nd.n = end - start;
        nd.bounds = b;
    }
    static int bucket(const Bounds& cb, V3 c, int dim) {  // bvh.go:349-352 (truncated index)
        int b = 12 * (int)gm::to_int(idx(offset_in(cb, c), dim));
        return b == 12 ? 11 : b;
    }
    // bvh.go:163-175: Lomuto partition around in[pivot] swapped to `end`
    template <class F>
    int64_t partition_at(int64_t start, int64_t end, int64_t pivot, F f) {
        PrimInfo pv = info[pivot];
        std::swap(info[pivot], info[end]);
        for (int64_t i = start; i < end; i++)
            if (f(info[i], pv)) { std::swap(info[start], info[i]); start++; }
        std::swap(info[end], info[start]);
        return start;
    }
    // bvh.go:272-411 (SplitSAH)
    int build(int64_t start, int64_t end) {
        int me = (int)nodes.size();
        nodes.emplace_back();
        Bounds bounds;
        for (int64_t i = start; i < end; i++) union_bounds(bounds, info[i].bounds);
        int64_t np = end - start;
        if (np == 1) { leaf(nodes[me], start, end, bounds); return me; }
        Bounds cb;
        for (int64_t i = start; i < end; i++) union_point(cb, info[i].centroid);
        if (np == 0 || !cb.has_min) { failed = true; return me; }  // Go: nil dereference panic
        int dim = maximum_extent(cb);
        int64_t mid = (start + end) / 2;
        if (idx(cb.mx, dim) == idx(cb.mn, dim)) { leaf(nodes[me], start, end, bounds); return me; }
        if (np <= 2) {
            partition_at(start, end - 1, mid,
                         [&](const PrimInfo& a, const PrimInfo& b) { return idx(a.centroid, dim) < idx(b.centroid, dim); });
        } else {
            Bounds bk[12];
            int cnt[12] = {0};
            for (int64_t i = start; i < end; i++) {
                int b = bucket(cb, info[i].centroid, dim);
                cnt[b]++;
                union_bounds(bk[b], info[i].bounds);
            }
            double cost[11];
            for (int i = 0; i < 11; i++) {
                Bounds b0, b1;
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= i; j++) { union_bounds(b0, bk[j]); c0 += cnt[j]; }
                for (int j = i + 1; j < 12; j++) { union_bounds(b1, bk[j]); c1 += cnt[j]; }
                cost[i] = 1.0 + ((double)c0 * surface_area(b0) + (double)c1 * surface_area(b1)) / surface_area(bounds);
            }
            double min_cost = cost[0];
            int min_bucket = 0;
            for (int i = 1; i < 11; i++)
                if (cost[i] < min_cost) { min_cost = cost[i]; min_bucket = i; }
            if (np > max_prims || min_cost < (double)np) {
                mid = partition_at(start, end - 1, end - 1, [&](const PrimInfo& a, const PrimInfo&) {
                    return bucket(cb, a.centroid, dim) <= min_bucket;
                });
            } else {
                leaf(nodes[me], start, end, bounds);
                return me;
            }
        }
        int c0 = build(start, mid);
        int c1 = build(mid, end);
        BuildNode& nd = nodes[me];
        nd.child[0] = c0; nd.child[1] = c1;
        nd.axis = dim;
        nd.n = 0;
        nd.bounds = nodes[c0].bounds;   // bvh.go:54-66 InitInterior
        union_bounds(nd.bounds, nodes[c1].bounds);
        return me;
    }
    // bvh.go:632-651 depth-first flattening
    uint32_t flatten(int node, std::vector<pbrt_bvh_node>& out) {
        const BuildNode& nd = nodes[node];
        uint32_t my = (uint32_t)out.size();
        out.emplace_back();
        pbrt_bvh_node ln;
        std::memset(&ln, 0, sizeof(ln));
        ln.bmin[0] = nd.bounds.mn.x; ln.bmin[1] = nd.bounds.mn.y; ln.bmin[2] = nd.bounds.mn.z;
        ln.bmax[0] = nd.bounds.mx.x; ln.bmax[1] = nd.bounds.mx.y; ln.bmax[2] = nd.bounds.mx.z;
        if (nd.n > 0) {
            ln.offset = (uint32_t)nd.first;
            ln.n_prims = (uint16_t)nd.n;
        } else {
            ln.axis = (uint8_t)nd.axis;
            flatten(nd.child[0], out);
            ln.offset = flatten(nd.child[1], out);
        }
        out[my] = ln;
        return my;
    }
};

}  // namespace

struct pbrt_scene_builder {
    std::vector<pbrt_shape_desc> shapes;
    std::vector<pbrt_material_desc> materials;
    std::vector<pbrt_primitive_desc> prims_in, prims;
    std::vector<int32_t> order;
    std::vector<pbrt_bvh_node> nodes;
    std::vector<pbrt_light_desc> lights;
    pbrt_camera_desc camera;
    pbrt_film_desc film;
    bool has_film = false, has_camera = false;
    // triangle meshes (extension): owned copies of the vertex / index arrays
    std::vector<std::vector<float>> mesh_p;
    std::vector<std::vector<int32_t>> mesh_idx;
    std::vector<pbrt_mesh_desc> meshes;
    pbrt_scene_desc desc;
};

extern "C" {

void pbrt_translate(double x, double y, double z, pbrt_transform* out) {  // transform.go:347-362
    out->m = identity4();
    out->m_inv = identity4();
    out->m.m[0][3] = x; out->m.m[1][3] = y; out->m.m[2][3] = z;
    out->m_inv.m[0][3] = -x; out->m_inv.m[1][3] = -y; out->m_inv.m[2][3] = -z;
}
void pbrt_scale(double x, double y, double z, pbrt_transform* out) {  // transform.go:364-379
    out->m = identity4();
    out->m_inv = identity4();
    out->m.m[0][0] = x; out->m.m[1][1] = y; out->m.m[2][2] = z;
    out->m_inv.m[0][0] = 1.0 / x; out->m_inv.m[1][1] = 1.0 / y; out->m_inv.m[2][2] = 1.0 / z;
}
static void rotate_axis(int axis, double degrees, pbrt_transform* out) {  // transform.go:381-424
    double s = gm::sin(gm::radians(degrees));
    double c = gm::cos(gm::radians(degrees));
    out->m = identity4();
    double(*m)[4] = out->m.m;
    if (axis == 0) { m[1][1] = c; m[1][2] = -s; m[2][1] = s; m[2][2] = c; }
    else if (axis == 1) { m[0][0] = c; m[0][2] = s; m[2][0] = -s; m[2][2] = c; }
    else { m[0][0] = c; m[0][1] = -s; m[1][0] = s; m[1][1] = c; }
    out->m_inv = transpose(out->m);
}
void pbrt_rotate_x(double d, pbrt_transform* out) { rotate_axis(0, d, out); }
void pbrt_rotate_y(double d, pbrt_transform* out) { rotate_axis(1, d, out); }
void pbrt_rotate_z(double d, pbrt_transform* out) { rotate_axis(2, d, out); }
void pbrt_transform_mul(const pbrt_transform* a, const pbrt_transform* b, pbrt_transform* out) {
    pbrt_transform r;   // transform.go:179-184: inverses composed in the same order (#18)
    r.m = matmul(a->m, b->m);
    r.m_inv = matmul(a->m_inv, b->m_inv);
    *out = r;
}
void pbrt_transform_inverse(const pbrt_transform* t, pbrt_transform* out) {
    pbrt_transform r;
    r.m = t->m_inv;
    r.m_inv = t->m;
    *out = r;
}
int pbrt_matrix_inverse(const pbrt_matrix4x4* m, pbrt_matrix4x4* out) {  // transform.go:72-142
    int indxc[4] = {0}, indxr[4] = {0}, ipiv[4] = {0};
    pbrt_matrix4x4 minv = *m;
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        double big = 0.0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] == 1) continue;
            for (int k = 0; k < 4; k++) {
                if (ipiv[k] == 0) {
                    if (gm::abs(minv.m[j][k]) >= big) {
                        big = gm::abs(minv.m[j][k]);
                        irow = j;
                        icol = k;
                    }
                } else if (ipiv[k] > 1) {
                    return PBRT_E_INVALID;
                }
            }
        }
        ipiv[icol]++;
        if (irow != icol)
            for (int k = 0; k < 4; k++) std::swap(minv.m[irow][k], minv.m[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (minv.m[icol][icol] == 0.0) return PBRT_E_INVALID;
        double pivinv = 1.0 / minv.m[icol][icol];
        minv.m[icol][icol] = 1.0;
        for (int j = 0; j < 4; j++) minv.m[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j == icol) continue;
            double save = minv.m[j][icol];
            minv.m[j][icol] = 0.0;
            for (int k = 0; k < 4; k++) minv.m[j][k] -= minv.m[icol][k] * save;
        }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(minv.m[k][indxr[j]], minv.m[k][indxc[j]]);
    *out = minv;
    return PBRT_OK;
}
int pbrt_new_transform(const pbrt_matrix4x4* m, pbrt_transform* out) {  // transform.go:148-157
    out->m = *m;
    return pbrt_matrix_inverse(m, &out->m_inv);
}
int pbrt_look_at(const double pos[3], const double look[3], const double up[3], pbrt_transform* out) {
    // transform.go:453-486
    pbrt_matrix4x4 m;
    std::memset(&m, 0, sizeof(m));
    m.m[0][3] = pos[0]; m.m[1][3] = pos[1]; m.m[2][3] = pos[2]; m.m[3][3] = 1;
    V3 dir = normalized(load3(look) - load3(pos));
    V3 upn = normalized(load3(up));
    if (length(cross(upn, dir)) == 0) return PBRT_E_INVALID;
    V3 right = normalized(cross(upn, dir));
    V3 nup = cross(dir, right);
    m.m[0][0] = right.x; m.m[1][0] = right.y; m.m[2][0] = right.z; m.m[3][0] = 0.;
    m.m[0][1] = nup.x; m.m[1][1] = nup.y; m.m[2][1] = nup.z; m.m[3][1] = 0.;
    m.m[0][2] = dir.x; m.m[1][2] = dir.y; m.m[2][2] = dir.z; m.m[3][2] = 0.;
    out->m = m;
    return pbrt_matrix_inverse(&m, &out->m_inv);
}
void pbrt_perspective(double fov, double n, double f, pbrt_transform* out) {  // transform.go:492-502
    pbrt_matrix4x4 p;
    std::memset(&p, 0, sizeof(p));
    p.m[0][0] = 1; p.m[1][1] = 1;
    p.m[2][2] = f / (f - n); p.m[2][3] = -f * n / (f - n);
    p.m[3][2] = 1;
    double inv_tan = 1.0 / gm::tan(gm::radians(fov) / 2);
    pbrt_transform s, pt;
    pbrt_scale(inv_tan, inv_tan, 1, &s);
    pbrt_new_transform(&p, &pt);
    pbrt_transform_mul(&s, &pt, out);
}
void pbrt_transform_point(const pbrt_transform* t, const double p[3], const double perr[3], double out_p[3],
                          double out_err[3]) {
    V3 e;
    V3 r = xf_point(t->m, load3(p), load3(perr), &e);
    out_p[0] = r.x; out_p[1] = r.y; out_p[2] = r.z;
    out_err[0] = e.x; out_err[1] = e.y; out_err[2] = e.z;
}
void pbrt_transform_ray(const pbrt_transform* t, const double o[3], const double d[3], double out_o[3],
                        double out_d[3]) {
    Ray r{load3(o), load3(d), kInf, 0};
    Ray w = xf_ray(t->m, r, nullptr, nullptr);
    out_o[0] = w.o.x; out_o[1] = w.o.y; out_o[2] = w.o.z;
    out_d[0] = w.d.x; out_d[1] = w.d.y; out_d[2] = w.d.z;
}

void pbrt_make_sphere(const pbrt_transform* o2w, int rev, double radius, double z_min, double z_max, double phi_max,
                      pbrt_shape_desc* out) {  // sphere.go:19-32
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_SHAPE_SPHERE;
    out->reverse_orientation = rev;
    out->object_to_world = *o2w;
    out->radius = radius;
    out->z_min = gm::clamp(gm::min(z_min, z_max), -radius, radius);
    out->z_max = gm::clamp(gm::max(z_min, z_max), -radius, radius);
    out->theta_min = gm::acos(gm::clamp(gm::min(z_min, z_max) / radius, -1, 1));
    out->theta_max = gm::acos(gm::clamp(gm::max(z_min, z_max) / radius, -1, 1));
    out->phi_max = gm::radians(gm::clamp(phi_max, 0, 360));
}
void pbrt_make_disk(const pbrt_transform* o2w, double height, double radius, double inner, double phi_max,
                    pbrt_shape_desc* out) {  // disk.go:22-35
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_SHAPE_DISK;
    out->object_to_world = *o2w;
    out->height = height;
    out->radius = radius;
    out->inner_radius = inner;
    out->phi_max = gm::radians(gm::clamp(phi_max, 0, 360));
}
void pbrt_make_matte_constant(double r, double g, double b, double sigma, pbrt_material_desc* out) {
    std::memset(out, 0, sizeof(*out));
    out->kd_type = PBRT_TEX_CONSTANT;
    out->kd[0] = r; out->kd[1] = g; out->kd[2] = b;
    out->sigma = sigma;
}
void pbrt_make_matte_checkerboard(const double vs[3], const double vt[3], double ds, double dt, const double tex1[3],
                                  const double tex2[3], double sigma, pbrt_material_desc* out) {
    std::memset(out, 0, sizeof(*out));
    out->kd_type = PBRT_TEX_CHECKERBOARD2D;
    for (int i = 0; i < 3; i++) {
        out->vs[i] = vs[i]; out->vt[i] = vt[i]; out->tex1[i] = tex1[i]; out->tex2[i] = tex2[i];
    }
    out->ds = ds; out->dt = dt;
    out->sigma = sigma;
}
void pbrt_random_sampler(int32_t samples_per_pixel, pbrt_render_desc* rd) {
    // sampler.NewRandomSampler (random.go:12-57) == Stratified(ns, 1) with no sampled
    // dimensions: StartPixel draws nothing, Get1D/Get2D fall through to the same
    // PCG32 stream, Clone seeds it the same way (tests/test_materials.py pins this
    // against the oracle's own RandomSampler restatement)
    rd->sampler_x = samples_per_pixel;
    rd->sampler_y = 1;
    rd->n_dims = 0;
    rd->jitter = 0;
}
void pbrt_make_mirror(const double kr[3], pbrt_material_desc* out) {   // mirror.go:9-14 (NewMirror: Kr 0.9)
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_MAT_MIRROR;
    for (int i = 0; i < 3; i++) out->kr[i] = kr[i];
}
void pbrt_make_glass(const double kr[3], const double kt[3], double u_roughness, double v_roughness, double eta,
                     pbrt_material_desc* out) {   // glass.go:15-26 (remapRoughness false)
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_MAT_GLASS;
    for (int i = 0; i < 3; i++) {
        out->kr[i] = kr[i];
        out->kt[i] = kt[i];
    }
    out->u_roughness = u_roughness;
    out->v_roughness = v_roughness;
    out->eta = eta;
}
void pbrt_make_point_light(const pbrt_transform* l2w, const double I[3], pbrt_light_desc* out) {  // point.go:19-30
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_LIGHT_POINT;
    V3 p = xf_point(l2w->m, V3{0, 0, 0}, V3{0, 0, 0}, nullptr);
    out->p_light[0] = p.x; out->p_light[1] = p.y; out->p_light[2] = p.z;
    for (int i = 0; i < 3; i++) out->spectrum[i] = I[i];
}
void pbrt_make_distant_light(const pbrt_transform* l2w, const double L[3], const double w[3],
                             pbrt_light_desc* out) {  // distant.go:19-26
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_LIGHT_DISTANT;
    V3 wl = normalized(xf_vector(l2w->m, load3(w)));
    out->w_light[0] = wl.x; out->w_light[1] = wl.y; out->w_light[2] = wl.z;
    for (int i = 0; i < 3; i++) out->spectrum[i] = L[i];
}
void pbrt_make_diffuse_area_light(const double Lemit[3], int shape_index, int two_sided, pbrt_light_desc* out) {
    std::memset(out, 0, sizeof(*out));
    out->type = PBRT_LIGHT_DIFFUSE_AREA;
    out->shape = shape_index;
    out->two_sided = two_sided;
    for (int i = 0; i < 3; i++) out->spectrum[i] = Lemit[i];
}

pbrt_scene_builder* pbrt_sb_create(void) { return new pbrt_scene_builder(); }
void pbrt_sb_destroy(pbrt_scene_builder* b) { delete b; }
int pbrt_sb_add_shape(pbrt_scene_builder* b, const pbrt_shape_desc* s) {
    b->shapes.push_back(*s);
    return (int)b->shapes.size() - 1;
}
int pbrt_sb_add_material(pbrt_scene_builder* b, const pbrt_material_desc* m) {
    b->materials.push_back(*m);
    return (int)b->materials.size() - 1;
}
int pbrt_sb_add_primitive(pbrt_scene_builder* b, const pbrt_primitive_desc* p) {
    b->prims_in.push_back(*p);
    return (int)b->prims_in.size() - 1;
}
int pbrt_sb_add_light(pbrt_scene_builder* b, const pbrt_light_desc* l) {
    b->lights.push_back(*l);
    return (int)b->lights.size() - 1;
}
int pbrt_sb_add_mesh(pbrt_scene_builder* b, int32_t n_vertices, const float* p, int32_t n_triangles,
                     const int32_t* indices, int32_t material, int32_t reverse_orientation) {
    if (n_vertices <= 0 || n_triangles <= 0 || !p || !indices) return -PBRT_E_INVALID;
    for (int64_t i = 0; i < 3 * (int64_t)n_triangles; i++)
        if (indices[i] < 0 || indices[i] >= n_vertices) return -PBRT_E_INVALID;
    b->mesh_p.emplace_back(p, p + 3 * (size_t)n_vertices);
    b->mesh_idx.emplace_back(indices, indices + 3 * (size_t)n_triangles);
    pbrt_mesh_desc m;
    std::memset(&m, 0, sizeof(m));
    m.n_vertices = n_vertices;
    m.n_triangles = n_triangles;
    m.material = material;
    m.reverse_orientation = reverse_orientation;
    b->meshes.push_back(m);
    return (int)b->meshes.size() - 1;
}
int pbrt_sb_set_film(pbrt_scene_builder* b, int64_t res_x, int64_t res_y, const double crop[4], double frx,
                     double fry, double max_lum) {  // film.go:42-76 (BoxFilter)
    pbrt_film_desc& f = b->film;
    std::memset(&f, 0, sizeof(f));
    f.res_x = res_x; f.res_y = res_y;
    f.crop_min_x = gm::to_int(gm::ceil((double)res_x * crop[0]));
    f.crop_min_y = gm::to_int(gm::ceil((double)res_y * crop[1]));
    f.crop_max_x = gm::to_int(gm::ceil((double)res_x * crop[2]));
    f.crop_max_y = gm::to_int(gm::ceil((double)res_y * crop[3]));
    f.filter_radius_x = frx; f.filter_radius_y = fry;
    f.max_sample_luminance = max_lum;
    for (int i = 0; i < 256; i++) f.filter_table[i] = 1.0;   // BoxFilter.Evaluate (filter.go:28-32)
    b->has_film = true;
    return (f.crop_max_x > f.crop_min_x && f.crop_max_y > f.crop_min_y) ? PBRT_OK : PBRT_E_INVALID;
}
int pbrt_sb_set_perspective_camera(pbrt_scene_builder* b, const pbrt_transform* cam2world, const double sw[4],
                                   double shutter_open, double shutter_close, double lens_radius,
                                   double focal_distance, double fov) {
    (void)shutter_close;   // camera.go:116 passes shutterOpen as shutterClose (#19)
    if (!b->has_film) return PBRT_E_INVALID;
    // camera.go:106-124 NewProjectiveCamera with cameraToScreen = Perspective(fov, 1e-2, 1000)
    pbrt_transform cs, s2r, t;
    pbrt_perspective(fov, 1e-2, 1000.0, &cs);
    pbrt_scale((double)b->film.res_x, (double)b->film.res_y, 1.0, &s2r);
    pbrt_scale(1.0 / (sw[2] - sw[0]), 1.0 / (sw[1] - sw[3]), 1.0, &t);
    pbrt_transform_mul(&s2r, &t, &s2r);
    pbrt_translate(-sw[0], -sw[3], 0, &t);
    pbrt_transform_mul(&s2r, &t, &s2r);
    pbrt_transform r2s, csi;
    pbrt_transform_inverse(&s2r, &r2s);
    pbrt_transform_inverse(&cs, &csi);
    pbrt_transform_mul(&csi, &r2s, &b->camera.raster_to_camera);
    b->camera.camera_to_world = *cam2world;
    b->camera.lens_radius = lens_radius;
    b->camera.focal_distance = focal_distance;
    b->camera.shutter_open = shutter_open;
    b->camera.shutter_close = shutter_open;
    b->has_camera = true;
    return PBRT_OK;
}

int pbrt_sb_build(pbrt_scene_builder* b, int max_prims_in_node, const pbrt_scene_desc** out) {
    if (!b->has_film || !b->has_camera) return PBRT_E_INVALID;
    for (const auto& p : b->prims_in)
        if (p.shape < 0 || p.shape >= (int)b->shapes.size() || p.material < 0 ||
            p.material >= (int)b->materials.size())
            return PBRT_E_INVALID;
    // accelerator.NewBVH (bvh.go:223-265)
    BVHBuilder bb;
    bb.max_prims = (int)gm::min(255, (double)max_prims_in_node);
    int n = (int)b->prims_in.size();
    for (int i = 0; i < n; i++) {
        const pbrt_primitive_desc& p = b->prims_in[i];
        const pbrt_shape_desc& s = b->shapes[p.shape];
        Bounds wb = (s.type == PBRT_SHAPE_SPHERE)
                        ? transform_bounds(s.object_to_world, V3{-s.radius, -s.radius, s.z_min},
                                           V3{s.radius, s.radius, s.z_max})
                        : transform_bounds(s.object_to_world, V3{-s.radius, -s.radius, s.height},
                                           V3{s.radius, s.radius, s.height});
        if (p.kind == PBRT_PRIM_TRANSFORMED) wb = transform_bounds(p.prim_to_world, wb.mn, wb.mx);
        // bvh.go:29-35 centroid = .5*Min + .5*Max
        bb.info.push_back(PrimInfo{i, wb, muls(wb.mn, 0.5) + muls(wb.mx, 0.5)});
    }
    b->nodes.clear();
    b->prims.clear();
    b->order.clear();
    if (n > 0) {
        int root = bb.build(0, n);
        if (bb.failed) return PBRT_E_REF_PANIC;
        bb.flatten(root, b->nodes);
        for (int i = 0; i < n; i++) {
            b->prims.push_back(b->prims_in[bb.ordered[i]]);
            b->order.push_back(bb.ordered[i]);
        }
    }
    for (const auto& m : b->meshes)
        if (m.material < 0 || m.material >= (int)b->materials.size()) return PBRT_E_INVALID;
    pbrt_scene_desc& d = b->desc;
    std::memset(&d, 0, sizeof(d));
    // scene.go:16-36: WorldBound = BVH root bounds; Distant.Preprocess (distant.go:36-38)
    if (!b->nodes.empty())
        for (int k = 0; k < 3; k++) { d.world_min[k] = b->nodes[0].bmin[k]; d.world_max[k] = b->nodes[0].bmax[k]; }
    // extension: the aggregate also holds the meshes, so the world bound is the
    // union with their vertex bounds (Bounds3.Union, bounds.go:54-66)
    bool have = !b->nodes.empty();
    for (size_t mi = 0; mi < b->meshes.size(); mi++) {
        const std::vector<float>& P = b->mesh_p[mi];
        for (int32_t v : b->mesh_idx[mi]) {
            for (int k = 0; k < 3; k++) {
                const double x = (double)P[3 * (size_t)v + k];
                d.world_min[k] = have ? gm::min(d.world_min[k], x) : x;
                d.world_max[k] = have ? gm::max(d.world_max[k], x) : x;
            }
            have = true;
        }
    }
    V3 mn = load3(d.world_min), mx = load3(d.world_max);
    V3 center = divs(mn + mx, 2.0);   // bounds.go:105-112 BoundingSphere
    double radius = 0;
    if (center.x >= mn.x && center.x <= mx.x && center.y >= mn.y && center.y <= mx.y && center.z >= mn.z &&
        center.z <= mx.z)
        radius = dist(center, mx);
    for (auto& l : b->lights)
        if (l.type == PBRT_LIGHT_DISTANT) l.world_radius = radius;
    d.n_shapes = (int)b->shapes.size();
    d.n_materials = (int)b->materials.size();
    d.n_prims = (int)b->prims.size();
    d.n_nodes = (int)b->nodes.size();
    d.n_lights = (int)b->lights.size();
    d.shapes = b->shapes.data();
    d.materials = b->materials.data();
    d.prims = b->prims.data();
    d.nodes = b->nodes.data();
    d.lights = b->lights.data();
    d.camera = b->camera;
    d.film = b->film;
    for (size_t mi = 0; mi < b->meshes.size(); mi++) {
        b->meshes[mi].p = b->mesh_p[mi].data();
        b->meshes[mi].indices = b->mesh_idx[mi].data();
    }
    d.n_meshes = (int)b->meshes.size();
    d.meshes = b->meshes.empty() ? nullptr : b->meshes.data();
    if (out) *out = &d;
    return PBRT_OK;
}
int pbrt_sb_prim_order(const pbrt_scene_builder* b, int32_t* out, int n) {
    int m = (int)b->order.size();
    for (int i = 0; i < n && i < m; i++) out[i] = b->order[i];
    return m;
}

// lightdistribution.go:11-68 + sampling.go:10-36 (Power: a 2n array of Y()==0, #28)
int pbrt_scene_light_distribution(const pbrt_scene_desc* s, int strategy, pbrt_distribution_desc* d) {
    std::memset(d, 0, sizeof(*d));
    int n = s->n_lights;
    if (strategy != PBRT_LIGHT_STRATEGY_UNIFORM && strategy != PBRT_LIGHT_STRATEGY_POWER) return PBRT_E_UNSUPPORTED;
    int cnt = (strategy == PBRT_LIGHT_STRATEGY_POWER) ? 2 * n : n;
    if (cnt > PBRT_MAX_DIST) return PBRT_E_UNSUPPORTED;
    for (int i = 0; i < cnt; i++) d->func[i] = (strategy == PBRT_LIGHT_STRATEGY_POWER) ? 0.0 : 1.0;
    d->count = cnt;
    d->cdf[0] = 0;
    for (int i = 1; i < cnt + 1; i++) d->cdf[i] = d->cdf[i - 1] + d->func[i - 1] / (double)cnt;
    d->func_int = d->cdf[cnt];
    if (d->func_int == 0.0)
        for (int i = 1; i < cnt + 1; i++) d->cdf[i] = (double)i / (double)cnt;
    else
        for (int i = 1; i < cnt + 1; i++) d->cdf[i] /= d->func_int;
    return PBRT_OK;
}

// internal/render/server.go:44-69: the 21 reverse-oriented spheres
static void readme_spheres(pbrt_scene_builder* b) {
    const int n = 8;
    for (int k = 1; k < n; k++) {
        for (int i = 0; i < 3; i++) {
            double x = 0, y = 0, z = 0, rgb[3] = {0, 0, 0};
            if (i == 0) { x = (double)k / (double)n * 100; rgb[0] = 1; }
            if (i == 1) { y = (double)k / (double)n * 100; rgb[1] = 1; }
            if (i == 2) { z = (double)k / (double)n * 100; rgb[2] = 1; }
            double radius = 2.0;
            y = gm::max(y, radius / 2);
            pbrt_transform o2w, xf;
            pbrt_translate(0, 0, 0, &o2w);
            pbrt_shape_desc s;
            pbrt_make_sphere(&o2w, 1, radius, -radius, radius, 360.0, &s);   // NewSphereShape(.., true, r)
            pbrt_material_desc m;
            pbrt_make_matte_constant(rgb[0], rgb[1], rgb[2], 0.0, &m);
            pbrt_translate(x, y, z, &xf);
            pbrt_primitive_desc p;
            std::memset(&p, 0, sizeof(p));
            p.kind = PBRT_PRIM_TRANSFORMED;
            p.shape = pbrt_sb_add_shape(b, &s);
            p.material = pbrt_sb_add_material(b, &m);
            p.prim_to_world = xf;
            pbrt_sb_add_primitive(b, &p);
        }
    }
}
// server.go:71-81: the floor's checkerboard Matte
static int readme_checker(pbrt_scene_builder* b) {
    const double vs[3] = {.2, 0, 0}, vt[3] = {0, 0, .2}, one[3] = {1, 1, 1}, dark[3] = {0.18, 0.18, 0.18};
    pbrt_material_desc chk;
    pbrt_make_matte_checkerboard(vs, vt, 0, 0, one, dark, 0.0, &chk);
    return pbrt_sb_add_material(b, &chk);
}
// server.go:112-164: the four lights, the film and the camera
static void readme_lights_camera(pbrt_scene_builder* b, int64_t w, int64_t h) {
    pbrt_light_desc l;
    pbrt_transform l2w;
    const double Ld[3] = {0.05, 0.05, 0.05}, wd[3] = {-1, 1, 1};
    pbrt_translate(-100, 100, 100, &l2w);
    pbrt_make_distant_light(&l2w, Ld, wd, &l);
    pbrt_sb_add_light(b, &l);
    const double I1[3] = {100, 100, 100}, I2[3] = {50, 50, 50};
    pbrt_translate(50, 20, 50, &l2w);
    pbrt_make_point_light(&l2w, I1, &l);
    pbrt_sb_add_light(b, &l);
    pbrt_translate(-50, 30, -50, &l2w);
    pbrt_make_point_light(&l2w, I2, &l);
    pbrt_sb_add_light(b, &l);
    pbrt_shape_desc ls;
    pbrt_translate(-10, 5, 20, &l2w);
    pbrt_make_sphere(&l2w, 0, 5.0, -5.0, 5.0, 360.0, &ls);
    const double Le[3] = {0.2, 0.2, 0.2};
    pbrt_make_diffuse_area_light(Le, pbrt_sb_add_shape(b, &ls), 0, &l);
    pbrt_sb_add_light(b, &l);

    const double crop[4] = {0, 0, 1, 1};
    pbrt_sb_set_film(b, w, h, crop, 1, 1, 1.0);
    const double pos[3] = {150, 150, 150}, look[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    pbrt_transform cam, r;
    pbrt_look_at(pos, look, up, &cam);
    pbrt_rotate_y(-30, &r);
    pbrt_transform_mul(&cam, &r, &cam);
    pbrt_rotate_x(-30, &r);
    pbrt_transform_mul(&cam, &r, &cam);
    pbrt_sb_set_perspective_camera(b, &cam, crop, 0.0, 1.0, 0, 20, 100);
}

// internal/render/server.go:29-164
int pbrt_scene_readme(int64_t w, int64_t h, pbrt_scene_builder** out) {
    pbrt_scene_builder* b = pbrt_sb_create();
    readme_spheres(b);
    int mchk = readme_checker(b);
    pbrt_transform t0, rx, dx;
    pbrt_translate(0, 0, 0, &t0);
    pbrt_rotate_x(90, &rx);
    pbrt_transform_mul(&t0, &rx, &dx);
    pbrt_shape_desc d1, d2;
    pbrt_make_disk(&dx, 0.01, 10000, 0, 360, &d1);
    pbrt_translate(-50, 0, -50, &dx);
    pbrt_make_disk(&dx, 0.01, 10000, 0, 360, &d2);
    pbrt_primitive_desc p;
    std::memset(&p, 0, sizeof(p));
    p.kind = PBRT_PRIM_GEOMETRIC;
    p.material = mchk;
    p.shape = pbrt_sb_add_shape(b, &d1);
    pbrt_sb_add_primitive(b, &p);
    p.shape = pbrt_sb_add_shape(b, &d2);
    pbrt_sb_add_primitive(b, &p);
    readme_lights_camera(b, w, h);
    int rc = pbrt_sb_build(b, 2, nullptr);
    if (rc != PBRT_OK) { pbrt_sb_destroy(b); return rc; }
    *out = b;
    return PBRT_OK;
}

// Value noise of the height field: lattice values in [-1, 1) at integer
// points of (x, z) / 10, from a splitmix64 hash of (seed, i, j), blended with
// the smoothstep weights.
static double hf_lattice(uint64_t seed, int64_t i, int64_t j) {
    uint64_t z = seed * 0x9e3779b97f4a7c15ULL ^ (uint64_t)i * 0xbf58476d1ce4e5b9ULL ^ (uint64_t)j * 0x94d049bb133111ebULL;
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}
static double hf_noise(uint64_t seed, double x, double z) {
    const double gx = x / 10.0, gz = z / 10.0;
    const double fx = gm::floor(gx), fz = gm::floor(gz);
    const int64_t i = (int64_t)fx, j = (int64_t)fz;
    const double tx = gx - fx, tz = gz - fz;
    const double sx = tx * tx * (3.0 - 2.0 * tx), sz = tz * tz * (3.0 - 2.0 * tz);
    const double a = hf_lattice(seed, i, j), bb = hf_lattice(seed, i + 1, j);
    const double c = hf_lattice(seed, i, j + 1), d = hf_lattice(seed, i + 1, j + 1);
    const double top = a + (bb - a) * sx, bot = c + (d - c) * sx;
    return top + (bot - top) * sz;
}

int pbrt_scene_heightfield(int64_t w, int64_t h, int32_t quads, uint64_t seed, int32_t flags,
                           pbrt_scene_builder** out) {
    if (quads < 1 || quads > 46340) return PBRT_E_INVALID;
    pbrt_scene_builder* b = pbrt_sb_create();
    if (flags & PBRT_HF_README_SPHERES) readme_spheres(b);
    const int mchk = readme_checker(b);
    const int64_t nv = (int64_t)(quads + 1) * (quads + 1);
    std::vector<float> P((size_t)(3 * nv));
    const double lo = -100.0, span = 300.0;
    for (int64_t j = 0; j <= quads; j++) {
        for (int64_t i = 0; i <= quads; i++) {
            const double x = lo + span * (double)i / (double)quads;
            const double z = lo + span * (double)j / (double)quads;
            const double y = 2.0 * gm::sin(0.3 * x) * gm::cos(0.2 * z) + 3.0 * hf_noise(seed, x, z);
            const size_t v = (size_t)(j * (quads + 1) + i);
            P[3 * v + 0] = (float)x;
            P[3 * v + 1] = (float)y;
            P[3 * v + 2] = (float)z;
        }
    }
    std::vector<int32_t> I((size_t)6 * quads * quads);
    size_t k = 0;
    for (int64_t j = 0; j < quads; j++) {
        for (int64_t i = 0; i < quads; i++) {
            const int32_t v00 = (int32_t)(j * (quads + 1) + i), v10 = v00 + 1;
            const int32_t v01 = v00 + (quads + 1), v11 = v01 + 1;
            // counter-clockwise seen from +y: the geometric normal points up
            I[k++] = v00; I[k++] = v01; I[k++] = v10;
            I[k++] = v10; I[k++] = v01; I[k++] = v11;
        }
    }
    int mi = pbrt_sb_add_mesh(b, (int32_t)nv, P.data(), (int32_t)(2 * (int64_t)quads * quads), I.data(), mchk, 0);
    if (mi < 0) { pbrt_sb_destroy(b); return -mi; }
    readme_lights_camera(b, w, h);
    int rc = pbrt_sb_build(b, 2, nullptr);
    if (rc != PBRT_OK) { pbrt_sb_destroy(b); return rc; }
    *out = b;
    return PBRT_OK;
}

// Cornell-style box (6 Disk walls r=20, 2 spheres,
// Point + DiffuseArea lights, camera inside), reference types only.
int pbrt_scene_cornell(int64_t w, int64_t h, pbrt_scene_builder** out) {
    pbrt_scene_builder* b = pbrt_sb_create();
    pbrt_material_desc m;
    pbrt_make_matte_constant(0.73, 0.73, 0.73, 0, &m);
    int white = pbrt_sb_add_material(b, &m);
    pbrt_make_matte_constant(0.63, 0.065, 0.05, 0, &m);
    int red = pbrt_sb_add_material(b, &m);
    pbrt_make_matte_constant(0.14, 0.45, 0.091, 0, &m);
    int green = pbrt_sb_add_material(b, &m);
    struct Wall { double t[3]; int axis; double deg; int mat; };
    const Wall walls[6] = {{{5, 0, 5}, 0, 90, white},  {{5, 10, 5}, 0, 90, white}, {{0, 5, 5}, 1, 90, red},
                           {{10, 5, 5}, 1, 90, green}, {{5, 5, 0}, -1, 0, white},  {{5, 5, 10}, -1, 0, white}};
    for (const Wall& wl : walls) {
        pbrt_transform t, r;
        pbrt_translate(wl.t[0], wl.t[1], wl.t[2], &t);
        if (wl.axis == 0) { pbrt_rotate_x(wl.deg, &r); pbrt_transform_mul(&t, &r, &t); }
        if (wl.axis == 1) { pbrt_rotate_y(wl.deg, &r); pbrt_transform_mul(&t, &r, &t); }
        pbrt_shape_desc s;
        pbrt_make_disk(&t, 0, 20, 0, 360, &s);
        pbrt_primitive_desc p;
        std::memset(&p, 0, sizeof(p));
        p.kind = PBRT_PRIM_GEOMETRIC;
        p.shape = pbrt_sb_add_shape(b, &s);
        p.material = wl.mat;
        pbrt_sb_add_primitive(b, &p);
    }
    const double sp[2][4] = {{3, 1.5, 6, 1.5}, {7, 2, 4, 2}};
    for (int i = 0; i < 2; i++) {
        pbrt_transform o2w;
        pbrt_translate(0, 0, 0, &o2w);
        pbrt_shape_desc s;
        pbrt_make_sphere(&o2w, 0, sp[i][3], -sp[i][3], sp[i][3], 360.0, &s);
        pbrt_primitive_desc p;
        std::memset(&p, 0, sizeof(p));
        p.kind = PBRT_PRIM_TRANSFORMED;
        p.shape = pbrt_sb_add_shape(b, &s);
        p.material = white;
        pbrt_translate(sp[i][0], sp[i][1], sp[i][2], &p.prim_to_world);
        pbrt_sb_add_primitive(b, &p);
    }
    pbrt_light_desc l;
    pbrt_transform l2w;
    const double I[3] = {10, 10, 10}, Le[3] = {5, 5, 5};
    pbrt_translate(5, 9.5, 5, &l2w);
    pbrt_make_point_light(&l2w, I, &l);
    pbrt_sb_add_light(b, &l);
    pbrt_shape_desc ls;
    pbrt_translate(5, 9, 5, &l2w);
    pbrt_make_sphere(&l2w, 0, 0.5, -0.5, 0.5, 360.0, &ls);
    pbrt_make_diffuse_area_light(Le, pbrt_sb_add_shape(b, &ls), 0, &l);
    pbrt_sb_add_light(b, &l);
    const double crop[4] = {0, 0, 1, 1};
    pbrt_sb_set_film(b, w, h, crop, 1, 1, 1.0);
    const double pos[3] = {5, 5, 0.5}, look[3] = {5, 5, 10}, up[3] = {0, 1, 0};
    pbrt_transform cam;
    pbrt_look_at(pos, look, up, &cam);
    pbrt_sb_set_perspective_camera(b, &cam, crop, 0.0, 1.0, 0, 20, 90);
    int rc = pbrt_sb_build(b, 2, nullptr);
    if (rc != PBRT_OK) { pbrt_sb_destroy(b); return rc; }
    *out = b;
    return PBRT_OK;
}


// ------------------------------------------------------------- diagnostics
int pbrt_diag_vec_op(int op, const double* a, const double* b, double s, double* out) {
    const V3 x = load3(a), y = b ? load3(b) : V3{0, 0, 0};
    const Spec p = spec3(a), q = b ? spec3(b) : spec(0);
    V3 r{0, 0, 0};
    Spec t = spec(0);
    bool vec = true, sp = false;
    double sc = 0;
    switch (op) {
        case PBRT_VOP_ABS: r = vabs(x); break;
        case PBRT_VOP_ABSDOT: sc = absdot(x, y); vec = false; break;
        case PBRT_VOP_ADD: r = x + y; break;
        case PBRT_VOP_CROSS: r = cross(x, y); break;
        case PBRT_VOP_DISTANCE: sc = dist(x, y); vec = false; break;
        case PBRT_VOP_DISTANCE_SQUARED: sc = dist2(x, y); vec = false; break;
        case PBRT_VOP_DIV: r = divv(x, y); break;
        case PBRT_VOP_DIV_SCALAR: r = divs(x, s); break;
        case PBRT_VOP_DOT: sc = dot(x, y); vec = false; break;
        case PBRT_VOP_LENGTH: sc = length(x); vec = false; break;
        case PBRT_VOP_LENGTH_SQUARED: sc = len2(x); vec = false; break;
        case PBRT_VOP_MUL: r = mul(x, y); break;
        case PBRT_VOP_MUL_SCALAR: r = muls(x, s); break;
        case PBRT_VOP_NORMALIZED: r = normalized(x); break;
        case PBRT_VOP_SUB: r = x - y; break;
        case PBRT_SOP_ADD: t = p + q; sp = true; break;
        case PBRT_SOP_MUL: t = smul(p, q); sp = true; break;
        case PBRT_SOP_DIV_SCALAR: t = sdivs(p, s); sp = true; break;
        case PBRT_SOP_MUL_SCALAR: t = smuls(p, s); sp = true; break;
        case PBRT_SOP_IS_BLACK: sc = is_black(p) ? 1.0 : 0.0; vec = false; break;
        default: return PBRT_E_INVALID;
    }
    if (sp) { out[0] = t.r; out[1] = t.g; out[2] = t.b; }
    else if (vec) { out[0] = r.x; out[1] = r.y; out[2] = r.z; }
    else { out[0] = sc; out[1] = out[2] = 0; }
    return PBRT_OK;
}

int64_t pbrt_diag_partition_at(int32_t* prim, double* cx, int64_t n, int64_t start, int64_t end, int64_t pivot) {
    if (!prim || !cx || n <= 0 || start < 0 || end >= n || pivot < start || pivot > end || start > end) return -1;
    BVHBuilder bb;
    for (int64_t i = 0; i < n; i++) bb.info.push_back(PrimInfo{prim[i], Bounds{}, V3{cx[i], 0, 0}});
    const int64_t m = bb.partition_at(start, end, pivot, [](const PrimInfo& x, const PrimInfo& y) {
        return x.centroid.x < y.centroid.x;
    });
    for (int64_t i = 0; i < n; i++) { prim[i] = bb.info[(size_t)i].prim; cx[i] = bb.info[(size_t)i].centroid.x; }
    return m;
}

}  // extern "C"
