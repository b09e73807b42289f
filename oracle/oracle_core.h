/*
 * oracle/oracle_core.h — TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * Scalar C restatement of go-pbrt's geometry, transform and interval
 * arithmetic, line by line, with Go evaluation order (left-to-right, no FMA
 * contraction, float64 everywhere). Used only as the parity checker and as
 * bench.py's cpu_baseline ("port").
 */
#ifndef ORACLE_CORE_H
#define ORACLE_CORE_H

#include <setjmp.h>
#include "go_math.h"
#include "../include/pbrt_gpu.h"

/* ------------------------------------------------------------------ vectors */
/* pkg/geometry/xyz.go:424-614 (XYZFloat64) */
typedef struct { double x, y, z; } v3;

static inline v3 V3(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 v_add(v3 a, v3 b) { FL(3); return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v_sub(v3 a, v3 b) { FL(3); return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v_mul(v3 a, v3 b) { FL(3); return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 v_muls(v3 a, double s) { FL(3); return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 v_divs(v3 a, double s) { FL(3); return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 v_divv(v3 a, v3 b) { FL(3); return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline double v_dot(v3 a, v3 b) { FL(5); return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double v_absdot(v3 a, v3 b) { return gm_abs(v_dot(a, b)); }
static inline v3 v_cross(v3 a, v3 b) {
    FL(9);
    return V3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
static inline double v_len2(v3 a) { FL(5); return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline double v_len(v3 a) { FL(1); return sqrt(v_len2(a)); }
static inline v3 v_abs(v3 a) { return V3(gm_abs(a.x), gm_abs(a.y), gm_abs(a.z)); }
/* xyz.go:596-606 Normalized: multiply by 1/sqrt, only when nor2 > 0 */
static inline v3 v_normalized(v3 a) {
    double n2 = v_len2(a);
    if (n2 > 0) {
        double inv = 1.0 / sqrt(n2);
        a.x *= inv; a.y *= inv; a.z *= inv;
        FL(5);
    }
    return a;
}
/* xyz.go:570-576: a.DistanceSquared(b) = (b - a).LengthSquared() */
static inline double v_dist2(v3 a, v3 b) { return v_len2(v_sub(b, a)); }
static inline double v_dist(v3 a, v3 b) { FL(1); return sqrt(v_dist2(a, b)); }
static inline double v_idx(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void v_set_idx(v3* a, int i, double v) {
    if (i == 0) a->x = v; else if (i == 1) a->y = v; else a->z = v;
}
static inline int v_is_zero_all(v3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }

typedef struct { double x, y; } v2;

/* ------------------------------------------------------------------ spectra */
/* pkg/pbrt/spectrum.go (RGB Spectrum, 3 x float64) */
typedef struct { double c[3]; } spec;
static inline spec S3(double r, double g, double b) { spec s = {{r, g, b}}; return s; }
static inline spec s_add(spec a, spec b) { FL(3); return S3(a.c[0] + b.c[0], a.c[1] + b.c[1], a.c[2] + b.c[2]); }
static inline spec s_mul(spec a, spec b) { FL(3); return S3(a.c[0] * b.c[0], a.c[1] * b.c[1], a.c[2] * b.c[2]); }
static inline spec s_muls(spec a, double s) { FL(3); return S3(a.c[0] * s, a.c[1] * s, a.c[2] * s); }
static inline spec s_divs(spec a, double s) { FL(3); return S3(a.c[0] / s, a.c[1] / s, a.c[2] / s); }
static inline int s_is_black(spec a) { return a.c[0] == 0.0 && a.c[1] == 0.0 && a.c[2] == 0.0; }
static inline int s_has_nans(spec a) { return gm_isnan(a.c[0]) || gm_isnan(a.c[1]) || gm_isnan(a.c[2]); }
/* spectrum.go:185-191 */
static inline double s_max_component(spec a) { return go_max(go_max(a.c[0], a.c[1]), a.c[2]); }

/* ---------------------------------------------------------------- transform */
static inline double g3(void) { return go_gamma(3.0); }

/* transform.go:227-247 TransformPoint, including the abs-error quirks (#17) */
static inline v3 xf_point(const pbrt_transform* t, v3 p, v3 pe, v3* err) {
    const double (*m)[4] = t->m.m;
    double xp = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
    double yp = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
    double zp = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
    double wp = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
    FL(24);
    if (err) {
        FL(3 * 15);
        double g = go_gamma(3.0);
        err->x = (go_gamma(3.0) + 1.0) * (gm_abs(m[0][0]) * pe.x + gm_abs(m[0][1]) * pe.y + gm_abs(m[0][2]) * pe.z) +
                 (g * (gm_abs(m[0][0] * p.x) + gm_abs(m[0][1]) * p.y + gm_abs(m[0][2] * p.z + gm_abs(m[0][3]))));
        err->y = (go_gamma(3.0) + 1.0) * (gm_abs(m[1][0]) * pe.x + gm_abs(m[1][1]) * pe.y + gm_abs(m[1][2]) * pe.z) +
                 (g * (gm_abs(m[1][0] * p.x) + gm_abs(m[1][1]) * p.y + gm_abs(m[1][2] * p.z + gm_abs(m[1][3]))));
        err->z = (go_gamma(3.0) + 1.0) * (gm_abs(m[2][0]) * pe.x + gm_abs(m[2][1]) * pe.y + gm_abs(m[2][2]) * pe.z) +
                 (g * (gm_abs(m[2][0] * p.x) + gm_abs(m[2][1]) * p.y + gm_abs(m[2][2] * p.z + gm_abs(m[2][3]))));
    }
    v3 np = V3(xp, yp, zp);
    if (wp == 1.0) return np;
    return v_divs(np, wp);
}
/* transform.go:249-255 */
static inline v3 xf_vector(const pbrt_transform* t, v3 v) {
    const double (*m)[4] = t->m.m;
    FL(15);
    return V3(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z,
              m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
              m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z);
}
/* transform.go:257-269 */
static inline v3 xf_vector_err(const pbrt_transform* t, v3 v, v3* err) {
    const double (*m)[4] = t->m.m;
    double g = go_gamma(3.0);
    FL(18);
    err->x = g * (gm_abs(m[0][0] * v.x) + gm_abs(m[0][1] * v.y) + gm_abs(m[0][2] * v.z));
    err->y = g * (gm_abs(m[1][0] * v.x) + gm_abs(m[1][1] * v.y) + gm_abs(m[1][2] * v.z));
    err->z = g * (gm_abs(m[2][0] * v.x) + gm_abs(m[2][1] * v.y) + gm_abs(m[2][2] * v.z));
    return xf_vector(t, v);
}
/* transform.go:271-277 (uses MatrixInverse transposed) */
static inline v3 xf_normal(const pbrt_transform* t, v3 n) {
    const double (*mi)[4] = t->m_inv.m;
    FL(15);
    return V3(mi[0][0] * n.x + mi[1][0] * n.y + mi[2][0] * n.z,
              mi[0][1] * n.x + mi[1][1] * n.y + mi[2][1] * n.z,
              mi[0][2] * n.x + mi[1][2] * n.y + mi[2][2] * n.z);
}
static inline pbrt_transform xf_inverse(const pbrt_transform* t) {
    pbrt_transform r; r.m = t->m_inv; r.m_inv = t->m; return r;
}
/* transform.go:167-173 */
static inline int xf_is_identity(const pbrt_transform* t) {
    const double (*m)[4] = t->m.m;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            if (m[i][j] != (i == j ? 1.0 : 0.0)) return 0;
    return 1;
}

/* -------------------------------------------------------------------- rays */
typedef struct { v3 o, d; double tmax, time; } ray_t;

/* transform.go:279-300 TransformRay (origin pushed by dt along the direction) */
static inline ray_t xf_ray(const pbrt_transform* t, const ray_t* r, v3* oerr, v3* derr) {
    v3 oe, de;
    ray_t out;
    out.o = xf_point(t, r->o, V3(0, 0, 0), &oe);
    out.d = xf_vector_err(t, r->d, &de);
    double l2 = v_len2(out.d);
    if (l2 > 0) {
        double dt = v_dot(v_abs(out.d), oe) / l2;
        v3 add = v_muls(out.d, dt);
        out.o.x += add.x; out.o.y += add.y; out.o.z += add.z;
        FL(4);
    }
    out.tmax = r->tmax;
    out.time = r->time;
    if (oerr) *oerr = oe;
    if (derr) *derr = de;
    return out;
}

/* ray.go:57-74 OffsetRayOrigin (x1024 and Nextafter per nonzero component) */
static inline v3 offset_ray_origin(v3 p, v3 perr, v3 n, v3 w) {
    double d = v_dot(v_abs(n), perr) * 1024.0;
    FL(1);
    v3 off = v_muls(n, d);
    if (v_dot(w, n) < 0) off = v_muls(off, -1);
    v3 po = v_add(p, off);
    for (int i = 0; i < 3; i++) {
        double oi = v_idx(off, i);
        if (oi > 0) v_set_idx(&po, i, go_next_float_up(v_idx(po, i)));
        else if (oi < 0) v_set_idx(&po, i, go_next_float_down(v_idx(po, i)));
    }
    return po;
}

/* geometry.go:111-116 */
static inline v3 face_forward(v3 n1, v3 n2) {
    if (v_dot(n1, n2) < 0.0) return v_muls(n1, -1);
    return n1;
}
/* geometry.go:47-60 (divides by the squared length, not its sqrt) */
static inline void coordinate_system(v3 v1, v3* v2, v3* v3o) {
    if (gm_abs(v1.x) > gm_abs(v1.y)) {
        double v = v1.x * v1.x + v1.z * v1.z;
        FL(3);
        *v2 = v_divv(V3(-v1.z, 0, v1.x), V3(v, v, v));
    } else {
        double v = v1.y * v1.y + v1.z * v1.z;
        FL(3);
        *v2 = v_divv(V3(0, v1.z, -v1.y), V3(v, v, v));
    }
    *v3o = v_cross(v1, *v2);
}

/* ------------------------------------------------------------------- panics */
typedef struct {
    jmp_buf jb;
    int kind;
} panic_ctx;

/* ------------------------------------------------------------------ EFloat */
/* pkg/efloat/efloat.go */
typedef struct { double v, lo, hi; } ef_t;

static inline void ef_check(panic_ctx* pc, ef_t f) {
    if (gm_isinf(f.lo, 0) || gm_isnan(f.lo) || gm_isinf(f.hi, 0) || gm_isnan(f.hi) || f.lo > f.hi) {
        pc->kind = PBRT_PANIC_EFLOAT;
        longjmp(pc->jb, 1);
    }
}
static inline ef_t ef_new(panic_ctx* pc, double v, double err) {
    ef_t f = {v, v, v};
    if (err != 0) {
        FL(2);
        f.lo = go_next_float_down(v - err);
        f.hi = go_next_float_up(v + err);
    }
    ef_check(pc, f);
    return f;
}
static inline ef_t ef_add(panic_ctx* pc, ef_t a, ef_t b) {
    ef_t r;
    FL(3);
    r.v = a.v + b.v;
    r.lo = go_next_float_down(a.lo + b.lo);
    r.hi = go_next_float_up(a.hi + b.hi);
    ef_check(pc, r);
    return r;
}
static inline ef_t ef_sub(panic_ctx* pc, ef_t a, ef_t b) {
    ef_t r;
    FL(3);
    r.v = a.v - b.v;
    r.lo = go_next_float_down(a.lo - b.hi);
    r.hi = go_next_float_up(a.hi - b.lo);
    ef_check(pc, r);
    return r;
}
static inline ef_t ef_mul(panic_ctx* pc, ef_t a, ef_t b) {
    double p0 = a.lo * b.lo, p1 = a.hi * b.lo, p2 = a.lo * b.hi, p3 = a.hi * b.hi;
    ef_t r;
    FL(5);
    r.v = a.v * b.v;
    r.lo = go_next_float_down(go_min(go_min(p0, p1), go_min(p2, p3)));
    r.hi = go_next_float_up(go_max(go_max(p0, p1), go_max(p2, p3)));
    ef_check(pc, r);
    return r;
}
static inline ef_t ef_muls(panic_ctx* pc, ef_t a, double s) { return ef_mul(pc, a, ef_new(pc, s, 0.0)); }
static inline ef_t ef_div(panic_ctx* pc, ef_t a, ef_t b) {
    ef_t r;
    FL(1);
    r.v = a.v / b.v;
    if (b.lo < 0 && b.hi > 0) {
        r.lo = -INFINITY;
        r.hi = INFINITY;
    } else {
        double d0 = a.lo / b.lo, d1 = a.hi / b.lo, d2 = a.lo / b.hi, d3 = a.hi / b.hi;
        FL(4);
        r.lo = go_next_float_down(go_min(go_min(d0, d1), go_min(d2, d3)));
        r.hi = go_next_float_up(go_max(go_max(d0, d1), go_max(d2, d3)));
    }
    ef_check(pc, r);
    return r;
}
/* pkg/efloat/math.go:35-59 */
static inline int ef_quadratic(panic_ctx* pc, ef_t a, ef_t b, ef_t c, ef_t* t0, ef_t* t1) {
    double disc = b.v * b.v - 4. * a.v * c.v;
    FL(4);
    if (disc < 0) return 0;
    double rd = sqrt(disc);
    FL(2);
    ef_t frd = ef_new(pc, rd, GO_MACHINE_EPSILON * rd);
    ef_t q;
    if (b.v < 0) q = ef_muls(pc, ef_sub(pc, b, frd), -0.5);
    else q = ef_muls(pc, ef_add(pc, b, frd), -0.5);
    ef_t r0 = ef_div(pc, q, a);
    ef_t r1 = ef_div(pc, c, q);
    if (r0.v > r1.v) { ef_t tmp = r0; r0 = r1; r1 = tmp; }
    *t0 = r0; *t1 = r1;
    return 1;
}

#endif
