/*
 * oracle/oracle_mesh.c — TEST INFRASTRUCTURE (oracle). Not part of the product.
 * See oracle_mesh.h for what this restates and why it has its own BVH.
 */
#include "oracle_mesh.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* pbrt-v3 gamma(n) with MachineEpsilon = 2^-53 (core/pbrt.h) */
#define MESH_EPS 1.1102230246251565e-16
static inline double tg(double n) { FL(4); return (n * MESH_EPS) / (1 - n * MESH_EPS); }
static inline double mx2(double a, double b) { return a > b ? a : b; }
static inline double mn2(double a, double b) { return a < b ? a : b; }

/* pbrt-v3 Triangle::Intersect, hit part (shapes/triangle.cpp), float64 */
int orc_triangle_hit(const double v[9], const ray_t* r, double* t_out, double* b0o, double* b1o, double* b2o) {
    double p0t[3] = {v[0] - r->o.x, v[1] - r->o.y, v[2] - r->o.z};
    double p1t[3] = {v[3] - r->o.x, v[4] - r->o.y, v[5] - r->o.z};
    double p2t[3] = {v[6] - r->o.x, v[7] - r->o.y, v[8] - r->o.z};
    FL(9);
    const double rd[3] = {r->d.x, r->d.y, r->d.z};
    const double ax = gm_abs(rd[0]), ay = gm_abs(rd[1]), az = gm_abs(rd[2]);
    const int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);   /* MaxDimension */
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    const double dx = rd[kx], dy = rd[ky], dz = rd[kz];
    double q0x = p0t[kx], q0y = p0t[ky], q0z = p0t[kz];
    double q1x = p1t[kx], q1y = p1t[ky], q1z = p1t[kz];
    double q2x = p2t[kx], q2y = p2t[ky], q2z = p2t[kz];
    const double Sx = -dx / dz, Sy = -dy / dz, Sz = 1.0 / dz;
    q0x += Sx * q0z; q0y += Sy * q0z;
    q1x += Sx * q1z; q1y += Sy * q1z;
    q2x += Sx * q2z; q2y += Sy * q2z;
    FL(3 + 12);
    const double e0 = q1x * q2y - q1y * q2x;
    const double e1 = q2x * q0y - q2y * q0x;
    const double e2 = q0x * q1y - q0y * q1x;
    FL(9);
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return 0;
    const double det = e0 + e1 + e2;
    FL(2);
    if (det == 0) return 0;
    q0z *= Sz; q1z *= Sz; q2z *= Sz;
    const double ts = e0 * q0z + e1 * q1z + e2 * q2z;
    FL(3 + 5);
    if (det < 0 && ts >= 0) return 0;
    if (det > 0 && ts <= 0) return 0;
    const double inv = 1 / det;
    const double b0 = e0 * inv, b1 = e1 * inv, b2 = e2 * inv;
    const double t = ts * inv;
    FL(5);
    /* conservative t > 0 */
    const double maxZt = mx2(gm_abs(q0z), mx2(gm_abs(q1z), gm_abs(q2z)));
    const double deltaZ = tg(3) * maxZt;
    const double maxXt = mx2(gm_abs(q0x), mx2(gm_abs(q1x), gm_abs(q2x)));
    const double maxYt = mx2(gm_abs(q0y), mx2(gm_abs(q1y), gm_abs(q2y)));
    const double deltaX = tg(5) * (maxXt + maxZt);
    const double deltaY = tg(5) * (maxYt + maxZt);
    const double deltaE = 2 * (tg(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    const double maxE = mx2(gm_abs(e0), mx2(gm_abs(e1), gm_abs(e2)));
    const double deltaT = 3 * (tg(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * gm_abs(inv);
    FL(1 + 4 + 9 + 9);
    if (t <= deltaT) return 0;
    *t_out = t;
    *b0o = b0; *b1o = b1; *b2o = b2;
    return 1;
}

/* ------------------------------------------------------------------- BVH */
typedef struct {
    double bmin[3], bmax[3];
    int32_t left, right;    /* interior: children; leaf: left = -1          */
    int32_t first, count;   /* leaf: triangles perm[first .. first+count)  */
} mnode;

struct orc_mesh {
    int32_t n_tris;
    double* v;          /* [gid][9] */
    int32_t* mat;       /* [gid]    */
    int8_t* rev;        /* [gid]    */
    double* cen;        /* [gid][3] */
    int32_t* perm;      /* leaf order -> gid (degenerate triangles left out) */
    int32_t n_perm;
    mnode* nodes;
    int32_t n_nodes, cap;
};

/* per-triangle box rounded out by one float32 ulp, as the device does */
static void tri_box(const orc_mesh* m, int32_t g, double* lo, double* hi) {
    for (int k = 0; k < 3; k++) {
        float a = (float)m->v[9 * g + k], b = (float)m->v[9 * g + 3 + k], c = (float)m->v[9 * g + 6 + k];
        float l = a < b ? a : b, h = a > b ? a : b;
        l = l < c ? l : c;
        h = h > c ? h : c;
        lo[k] = (double)nextafterf(l, -INFINITY);
        hi[k] = (double)nextafterf(h, INFINITY);
    }
}

static int g_axis;
static const double* g_cen;
static int cmp_cen(const void* a, const void* b) {
    const int32_t i = *(const int32_t*)a, j = *(const int32_t*)b;
    const double x = g_cen[3 * i + g_axis], y = g_cen[3 * j + g_axis];
    if (x < y) return -1;
    if (x > y) return 1;
    return (i > j) - (i < j);
}

static int32_t build(orc_mesh* m, int32_t first, int32_t count) {
    if (m->n_nodes == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 1024;
        m->nodes = (mnode*)realloc(m->nodes, sizeof(mnode) * (size_t)m->cap);
    }
    const int32_t id = m->n_nodes++;
    mnode nd;
    double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 3; k++) { nd.bmin[k] = INFINITY; nd.bmax[k] = -INFINITY; }
    for (int32_t i = first; i < first + count; i++) {
        double lo[3], hi[3];
        tri_box(m, m->perm[i], lo, hi);
        for (int k = 0; k < 3; k++) {
            nd.bmin[k] = mn2(nd.bmin[k], lo[k]);
            nd.bmax[k] = mx2(nd.bmax[k], hi[k]);
            clo[k] = mn2(clo[k], m->cen[3 * m->perm[i] + k]);
            chi[k] = mx2(chi[k], m->cen[3 * m->perm[i] + k]);
        }
    }
    if (count <= 4) {
        nd.left = nd.right = -1;
        nd.first = first;
        nd.count = count;
        m->nodes[id] = nd;
        return id;
    }
    int axis = 0;
    for (int k = 1; k < 3; k++)
        if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
    g_axis = axis;
    g_cen = m->cen;
    qsort(m->perm + first, (size_t)count, sizeof(int32_t), cmp_cen);
    const int32_t half = count / 2;
    nd.first = first;
    nd.count = count;
    const int32_t l = build(m, first, half);
    const int32_t r = build(m, first + half, count - half);
    nd.left = l;
    nd.right = r;
    m->nodes[id] = nd;
    return id;
}

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static orc_mesh* g_mesh;
static uint64_t g_key;

static uint64_t mesh_key(const pbrt_scene_desc* sc) {
    uint64_t h = 1469598103934665603ull;
#define MIX(x) (h = (h ^ (uint64_t)(x)) * 1099511628211ull)
    MIX(sc->n_meshes);
    for (int mi = 0; mi < sc->n_meshes; mi++) {
        const pbrt_mesh_desc* d = &sc->meshes[mi];
        MIX(d->n_vertices); MIX(d->n_triangles); MIX(d->material); MIX(d->reverse_orientation);
        MIX((uintptr_t)d->p); MIX((uintptr_t)d->indices);
        for (int32_t i = 0; i < 3 * d->n_vertices; i += 1 + 3 * d->n_vertices / 64) {
            uint32_t b;
            memcpy(&b, &d->p[i], 4);
            MIX(b);
        }
    }
#undef MIX
    return h;
}

static void mesh_free(orc_mesh* m) {
    if (!m) return;
    free(m->v); free(m->mat); free(m->rev); free(m->cen); free(m->perm); free(m->nodes);
    free(m);
}

const orc_mesh* orc_mesh_get(const pbrt_scene_desc* sc) {
    if (!sc || sc->n_meshes <= 0 || !sc->meshes) return NULL;
    const uint64_t key = mesh_key(sc);
    pthread_mutex_lock(&g_lock);
    if (g_mesh && g_key == key) {
        pthread_mutex_unlock(&g_lock);
        return g_mesh;
    }
    mesh_free(g_mesh);
    orc_mesh* m = (orc_mesh*)calloc(1, sizeof(orc_mesh));
    int64_t nt = 0;
    for (int mi = 0; mi < sc->n_meshes; mi++) nt += sc->meshes[mi].n_triangles;
    m->n_tris = (int32_t)nt;
    m->v = (double*)malloc(sizeof(double) * 9 * (size_t)(nt ? nt : 1));
    m->mat = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nt ? nt : 1));
    m->rev = (int8_t*)malloc((size_t)(nt ? nt : 1));
    m->cen = (double*)malloc(sizeof(double) * 3 * (size_t)(nt ? nt : 1));
    m->perm = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nt ? nt : 1));
    int32_t g = 0;
    for (int mi = 0; mi < sc->n_meshes; mi++) {
        const pbrt_mesh_desc* d = &sc->meshes[mi];
        for (int32_t i = 0; i < d->n_triangles; i++, g++) {
            for (int c = 0; c < 3; c++)
                for (int k = 0; k < 3; k++) m->v[9 * g + 3 * c + k] = (double)d->p[3 * d->indices[3 * i + c] + k];
            m->mat[g] = d->material;
            m->rev[g] = (int8_t)(d->reverse_orientation != 0);
            const double* q = &m->v[9 * g];
            v3 e1 = V3(q[3] - q[0], q[4] - q[1], q[5] - q[2]), e2 = V3(q[6] - q[0], q[7] - q[1], q[8] - q[2]);
            for (int k = 0; k < 3; k++) m->cen[3 * g + k] = (q[k] + q[3 + k] + q[6 + k]) / 3.0;
            /* zero-area triangles are never hit (left out of the BVH, as on the device) */
            if (v_len2(v_cross(e1, e2)) > 0) m->perm[m->n_perm++] = g;
        }
    }
    if (m->n_perm > 0) build(m, 0, m->n_perm);
    g_mesh = m;
    g_key = key;
    pthread_mutex_unlock(&g_lock);
    return m;
}

/* slab test against a box rounded out in float32, inclusive of tmax */
static int box_hit(const mnode* nd, const ray_t* r, v3 inv, double tmax) {
    const double o[3] = {r->o.x, r->o.y, r->o.z}, iv[3] = {inv.x, inv.y, inv.z};
    double t0 = 0, t1 = INFINITY;
    for (int k = 0; k < 3; k++) {
        double n, f;
        if (iv[k] == INFINITY || iv[k] == -INFINITY) {   /* d[k] == 0: inside the slab or never */
            const int in = nd->bmin[k] <= o[k] && o[k] <= nd->bmax[k];
            n = in ? -INFINITY : INFINITY;
            f = in ? INFINITY : -INFINITY;
        } else {
            const double a = (nd->bmin[k] - o[k]) * iv[k], b = (nd->bmax[k] - o[k]) * iv[k];
            n = a < b ? a : b;
            f = a < b ? b : a;
            f *= 1 + 2 * tg(3);
        }
        t0 = n > t0 ? n : t0;
        t1 = f < t1 ? f : t1;
    }
    return t0 <= t1 && t0 <= tmax;
}

int orc_mesh_closest(const orc_mesh* m, const ray_t* r, double tmax, int32_t best_gid, orc_tri_hit* h) {
    if (!m || m->n_perm == 0) return 0;
    const v3 inv = V3(1 / r->d.x, 1 / r->d.y, 1 / r->d.z);
    int32_t stack[128], sp = 0, cur = 0, found = 0;
    double bt = tmax, tb0 = 0, tb1 = 0, tb2 = 0;
    int32_t bg = best_gid;
    for (;;) {
        const mnode* nd = &m->nodes[cur];
        if (box_hit(nd, r, inv, bt)) {
            if (nd->left < 0) {
                for (int32_t i = nd->first; i < nd->first + nd->count; i++) {
                    const int32_t g = m->perm[i];
                    double t, b0, b1, b2;
                    if (!orc_triangle_hit(&m->v[9 * g], r, &t, &b0, &b1, &b2)) continue;
                    if (t < bt || (t == bt && g < bg)) {
                        bt = t; bg = g; tb0 = b0; tb1 = b1; tb2 = b2;
                        found = 1;
                    }
                }
            } else {
                stack[sp++] = nd->right;
                cur = nd->left;
                continue;
            }
        }
        if (sp == 0) break;
        cur = stack[--sp];
    }
    if (!found) return 0;
    h->t = bt; h->gid = bg; h->b0 = tb0; h->b1 = tb1; h->b2 = tb2;
    h->material = m->mat[bg];
    h->reverse = m->rev[bg];
    const double* q = &m->v[9 * bg];
    h->p0 = V3(q[0], q[1], q[2]); h->p1 = V3(q[3], q[4], q[5]); h->p2 = V3(q[6], q[7], q[8]);
    return 1;
}

int orc_mesh_any(const orc_mesh* m, const ray_t* r) {
    if (!m || m->n_perm == 0) return 0;
    const v3 inv = V3(1 / r->d.x, 1 / r->d.y, 1 / r->d.z);
    int32_t stack[128], sp = 0, cur = 0;
    for (;;) {
        const mnode* nd = &m->nodes[cur];
        if (box_hit(nd, r, inv, r->tmax)) {
            if (nd->left < 0) {
                for (int32_t i = nd->first; i < nd->first + nd->count; i++) {
                    double t, b0, b1, b2;
                    if (orc_triangle_hit(&m->v[9 * m->perm[i]], r, &t, &b0, &b1, &b2) && t < r->tmax) return 1;
                }
            } else {
                stack[sp++] = nd->right;
                cur = nd->left;
                continue;
            }
        }
        if (sp == 0) return 0;
        cur = stack[--sp];
    }
}
