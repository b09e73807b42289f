// pbrt_core.h — float64 geometry, transforms and EFloat with go-pbrt semantics,
// usable from host (scene builder) and device (kernels).
//
// Reference: pkg/geometry/xyz.go:424-614 (vector ops; Normalized multiplies by
// 1/sqrt), pkg/pbrt/transform.go:227-334 (TransformPoint/Vector/Normal/Ray/
// SurfaceInteraction, with the abs-error quirks of parity ledger #17),
// pkg/pbrt/ray.go:57-74 (OffsetRayOrigin), pkg/efloat (running-error
// intervals; Check() panics become a sticky flag the kernel reports as
// PBRT_E_REF_PANIC).
#pragma once
#pragma clang fp contract(off)

#include "../../include/pbrt_gpu.h"
#include "gomath.h"

namespace pbrt {

using gomath::kInf;

struct V3 {
    double x, y, z;
};
GO_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
GO_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
GO_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
GO_HD V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
GO_HD V3 muls(V3 a, double s) { return V3{a.x * s, a.y * s, a.z * s}; }
GO_HD V3 divs(V3 a, double s) { return V3{a.x / s, a.y / s, a.z / s}; }
GO_HD V3 divv(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
GO_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GO_HD double absdot(V3 a, V3 b) { return gomath::abs(dot(a, b)); }
GO_HD V3 cross(V3 a, V3 b) {
    return V3{(a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)};
}
GO_HD double len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
GO_HD double length(V3 a) { return gomath::sqrt(len2(a)); }
GO_HD V3 vabs(V3 a) { return V3{gomath::abs(a.x), gomath::abs(a.y), gomath::abs(a.z)}; }
GO_HD V3 normalized(V3 a) {
    double n2 = len2(a);
    if (n2 > 0) {
        double inv = 1.0 / gomath::sqrt(n2);
        a.x *= inv; a.y *= inv; a.z *= inv;
    }
    return a;
}
// a.DistanceSquared(b) = (b - a).LengthSquared()  (xyz.go:570-576)
GO_HD double dist2(V3 a, V3 b) { return len2(b - a); }
GO_HD double dist(V3 a, V3 b) { return gomath::sqrt(dist2(a, b)); }
GO_HD double idx(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
GO_HD V3 load3(const double* p) { return V3{p[0], p[1], p[2]}; }

struct Spec {
    double r, g, b;
};
GO_HD Spec spec(double v) { return Spec{v, v, v}; }
GO_HD Spec spec3(const double* p) { return Spec{p[0], p[1], p[2]}; }
GO_HD Spec operator+(Spec a, Spec b) { return Spec{a.r + b.r, a.g + b.g, a.b + b.b}; }
GO_HD Spec smul(Spec a, Spec b) { return Spec{a.r * b.r, a.g * b.g, a.b * b.b}; }
GO_HD Spec smuls(Spec a, double s) { return Spec{a.r * s, a.g * s, a.b * s}; }
GO_HD Spec sdivs(Spec a, double s) { return Spec{a.r / s, a.g / s, a.b / s}; }
GO_HD bool is_black(Spec a) { return a.r == 0.0 && a.g == 0.0 && a.b == 0.0; }
GO_HD bool has_nans(Spec a) { return gomath::is_nan(a.r) || gomath::is_nan(a.g) || gomath::is_nan(a.b); }
GO_HD double max_component(Spec a) { return gomath::max(gomath::max(a.r, a.g), a.b); }

struct Ray {
    V3 o, d;
    double tmax, time;
};

// ------------------------------------------------------------- transforms
// TransformPoint (transform.go:227-247); err may be null
GO_HD V3 xf_point(const pbrt_matrix4x4& M, V3 p, V3 pe, V3* err) {
    const double(*m)[4] = M.m;
    double xp = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
    double yp = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
    double zp = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
    double wp = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
    if (err) {
        double g = gomath::gamma(3.0), g1 = gomath::gamma(3.0) + 1.0;
        err->x = g1 * (gomath::abs(m[0][0]) * pe.x + gomath::abs(m[0][1]) * pe.y + gomath::abs(m[0][2]) * pe.z) +
                 (g * (gomath::abs(m[0][0] * p.x) + gomath::abs(m[0][1]) * p.y +
                       gomath::abs(m[0][2] * p.z + gomath::abs(m[0][3]))));
        err->y = g1 * (gomath::abs(m[1][0]) * pe.x + gomath::abs(m[1][1]) * pe.y + gomath::abs(m[1][2]) * pe.z) +
                 (g * (gomath::abs(m[1][0] * p.x) + gomath::abs(m[1][1]) * p.y +
                       gomath::abs(m[1][2] * p.z + gomath::abs(m[1][3]))));
        err->z = g1 * (gomath::abs(m[2][0]) * pe.x + gomath::abs(m[2][1]) * pe.y + gomath::abs(m[2][2]) * pe.z) +
                 (g * (gomath::abs(m[2][0] * p.x) + gomath::abs(m[2][1]) * p.y +
                       gomath::abs(m[2][2] * p.z + gomath::abs(m[2][3]))));
    }
    V3 np{xp, yp, zp};
    if (wp == 1.0) return np;
    return divs(np, wp);
}
GO_HD V3 xf_vector(const pbrt_matrix4x4& M, V3 v) {
    const double(*m)[4] = M.m;
    return V3{m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z, m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
              m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z};
}
// TransformVectorWithAbsError (transform.go:257-269)
GO_HD V3 xf_vector_err(const pbrt_matrix4x4& M, V3 v, V3* err) {
    const double(*m)[4] = M.m;
    double g = gomath::gamma(3.0);
    err->x = g * (gomath::abs(m[0][0] * v.x) + gomath::abs(m[0][1] * v.y) + gomath::abs(m[0][2] * v.z));
    err->y = g * (gomath::abs(m[1][0] * v.x) + gomath::abs(m[1][1] * v.y) + gomath::abs(m[1][2] * v.z));
    err->z = g * (gomath::abs(m[2][0] * v.x) + gomath::abs(m[2][1] * v.y) + gomath::abs(m[2][2] * v.z));
    return xf_vector(M, v);
}
// TransformNormal uses MatrixInverse transposed (transform.go:271-277)
GO_HD V3 xf_normal(const pbrt_matrix4x4& Mi, V3 n) {
    const double(*mi)[4] = Mi.m;
    return V3{mi[0][0] * n.x + mi[1][0] * n.y + mi[2][0] * n.z, mi[0][1] * n.x + mi[1][1] * n.y + mi[2][1] * n.z,
              mi[0][2] * n.x + mi[1][2] * n.y + mi[2][2] * n.z};
}
GO_HD bool is_identity(const pbrt_matrix4x4& M) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            if (M.m[i][j] != (i == j ? 1.0 : 0.0)) return false;
    return true;
}
// TransformRay (transform.go:279-300): the origin is pushed along d by dt
GO_HD Ray xf_ray(const pbrt_matrix4x4& M, const Ray& r, V3* oerr, V3* derr) {
    V3 oe, de;
    Ray out;
    out.o = xf_point(M, r.o, V3{0, 0, 0}, &oe);
    out.d = xf_vector_err(M, r.d, &de);
    double l2 = len2(out.d);
    if (l2 > 0) {
        double dt = dot(vabs(out.d), oe) / l2;
        V3 add = muls(out.d, dt);
        out.o.x += add.x; out.o.y += add.y; out.o.z += add.z;
    }
    out.tmax = r.tmax;
    out.time = r.time;
    if (oerr) *oerr = oe;
    if (derr) *derr = de;
    return out;
}

// Value-only TransformRay (transform.go:279-300) for a hit test.
// TransformRay pushes the transformed origin along d by
// dt = (|d'| . oError) / |d'|^2; oError = gamma(3) * (...) and gamma(3) is
// 3 * MachineEpsilon, a denormal. With every |m_ij| <= 1e10,
// |p_i|, |d'_i| <= 1e50 and |d'|^2 >= 1e-20, |oError_i| <= 6e-263 and each
// component of the push is <= 2e-142, below a quarter ulp of any |o'_i| >=
// 1e-100: o' + push rounds back to o'. So where these hold the origin is
// M*p, the direction M*d, and both error vectors are below 1e-150 with
// oError's sign irrelevant (|o'| >= 1e-100) -- all sphere_roots_filter needs
// (DESIGN.md 3.6). Classes (xf_fast_kind, host):
//   kXfIdentity:    M = I; M*p = p, M*d = d when no component is 0
//                   (the matrix product adds signed zeros, which only matter
//                   for zero components -- those take the exact path);
//   kXfTranslation: M*p = p + t (the three 1*p_i and 0*p_j products are
//                   exact; t_i + p_i is the one rounding), M*d = d;
//   kXfAffine:      last row (0,0,0,1), |m_ij| <= 1e10: the product as
//                   xf_point / xf_vector compute it, without the errors;
//   kXfSlow:        anything else: always the exact path.
constexpr int kXfIdentity = 0, kXfTranslation = 1, kXfAffine = 2, kXfSlow = 3;
GO_HD bool xf_fast(int kind, const pbrt_matrix4x4& M, V3& o, V3& d) {
    if (kind == kXfSlow) return false;
    const double big = 1e50;
    bool ok = gomath::abs(o.x) <= big && gomath::abs(o.y) <= big && gomath::abs(o.z) <= big;
    if (kind == kXfAffine) {
        const double(*m)[4] = M.m;
        const V3 p = o, v = d;
        o = V3{m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3],
               m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3],
               m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3]};
        d = xf_vector(M, v);
    } else {
        // no zero direction component (signed-zero sums), and d' = d
        ok = ok && d.x != 0 && d.y != 0 && d.z != 0;
        if (kind == kXfTranslation) o = V3{o.x + M.m[0][3], o.y + M.m[1][3], o.z + M.m[2][3]};
    }
    const double l2 = len2(d), small = 1e-100;
    return ok && gomath::abs(d.x) <= big && gomath::abs(d.y) <= big && gomath::abs(d.z) <= big && l2 >= 1e-20 &&
           gomath::abs(o.x) >= small && gomath::abs(o.y) >= small && gomath::abs(o.z) >= small;
}
// Host: the xf_fast class of a world->object matrix.
inline int xf_fast_kind(const pbrt_matrix4x4& M) {
    const double(*m)[4] = M.m;
    if (m[3][0] != 0 || m[3][1] != 0 || m[3][2] != 0 || m[3][3] != 1) return kXfSlow;
    bool lin_identity = true, small = true;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 4; j++) {
            const double v = m[i][j];
            if (!(v >= -1e10 && v <= 1e10)) small = false;
            if (j < 3 && __builtin_bit_cast(uint64_t, v) != __builtin_bit_cast(uint64_t, i == j ? 1.0 : 0.0))
                lin_identity = false;
        }
    if (!small) return kXfSlow;
    if (lin_identity) {
        // the identity test of the translation column is on values: +-0 both give p + 0 = p for p != 0
        if (m[0][3] == 0 && m[1][3] == 0 && m[2][3] == 0) return kXfIdentity;
        return kXfTranslation;
    }
    return kXfAffine;
}

// ray.go:57-74
GO_HD V3 offset_ray_origin(V3 p, V3 perr, V3 n, V3 w) {
    double d = dot(vabs(n), perr) * 1024.0;
    V3 off = muls(n, d);
    if (dot(w, n) < 0) off = muls(off, -1);
    V3 po = p + off;
    if (off.x > 0) po.x = gomath::next_up(po.x); else if (off.x < 0) po.x = gomath::next_down(po.x);
    if (off.y > 0) po.y = gomath::next_up(po.y); else if (off.y < 0) po.y = gomath::next_down(po.y);
    if (off.z > 0) po.z = gomath::next_up(po.z); else if (off.z < 0) po.z = gomath::next_down(po.z);
    return po;
}
// geometry.go:111-116
GO_HD V3 face_forward(V3 n1, V3 n2) { return dot(n1, n2) < 0.0 ? muls(n1, -1) : n1; }
// geometry.go:47-60 (divides by the squared length)
GO_HD void coordinate_system(V3 v1, V3& v2, V3& v3o) {
    if (gomath::abs(v1.x) > gomath::abs(v1.y)) {
        double v = v1.x * v1.x + v1.z * v1.z;
        v2 = divv(V3{-v1.z, 0, v1.x}, V3{v, v, v});
    } else {
        double v = v1.y * v1.y + v1.z * v1.z;
        v2 = divv(V3{0, v1.z, -v1.y}, V3{v, v, v});
    }
    v3o = cross(v1, v2);
}

// ----------------------------------------------------------------- EFloat
struct EF {
    double v, lo, hi;
};
// efloat.go:102-111 Check(): Inf/NaN bounds or Low > High panics in Go
GO_HD void ef_check(const EF& f, int& panic) {
    // !(|lo| < Inf) is true for ±Inf and NaN
    const bool bad = (int)!(gomath::abs(f.lo) < kInf) | (int)!(gomath::abs(f.hi) < kInf) | (int)(f.lo > f.hi);
    panic = bad ? (int)PBRT_PANIC_EFLOAT : panic;
}
GO_HD EF ef_new(double v, double err, int& panic) {
    EF f{v, v, v};
    if (err != 0) {
        f.lo = gomath::next_down(v - err);
        f.hi = gomath::next_up(v + err);
    }
    ef_check(f, panic);
    return f;
}
GO_HD EF ef_add(EF a, EF b, int& panic) {
    EF r{a.v + b.v, gomath::next_down(a.lo + b.lo), gomath::next_up(a.hi + b.hi)};
    ef_check(r, panic);
    return r;
}
GO_HD EF ef_sub(EF a, EF b, int& panic) {
    EF r{a.v - b.v, gomath::next_down(a.lo - b.hi), gomath::next_up(a.hi - b.lo)};
    ef_check(r, panic);
    return r;
}
// efloat.go Mul. Operands that passed Check are finite, so the four bound
// products are never NaN and Go's Min/Max reduce to IEEE min/max (-0 < +0).
// An operand that failed Check has already set the sticky panic: the caller
// discards everything computed after it.
GO_HD EF ef_mul(EF a, EF b, int& panic) {
    double p0 = a.lo * b.lo, p1 = a.hi * b.lo, p2 = a.lo * b.hi, p3 = a.hi * b.hi;
    EF r{a.v * b.v,
         gomath::next_down(gomath::min_nonan(gomath::min_nonan(p0, p1), gomath::min_nonan(p2, p3))),
         gomath::next_up(gomath::max_nonan(gomath::max_nonan(p0, p1), gomath::max_nonan(p2, p3)))};
    ef_check(r, panic);
    return r;
}
// MulScalar(s) = Mul(New(s, 0)) (efloat.go:86-88)
GO_HD EF ef_muls(EF a, double s, int& panic) { return ef_mul(a, ef_new(s, 0.0, panic), panic); }
// efloat.go Div. When b's interval excludes 0 the extreme quotients are known
// from the signs alone: correctly rounded division is monotone in each operand,
// so min/max over the four rounded quotients are the rounded quotients of the
// analytic extremes (ties and the sign of a zero vanish in NextFloatDown/Up).
// Two divisions instead of four; an interval with a zero end keeps the
// four-quotient form (its Inf/NaN reaches Check as in Go), and so does any
// operand with a non-finite bound (Go's Min/Max see NaN quotients there).
GO_HD EF ef_div(EF a, EF b, int& panic) {
    EF r;
    r.v = a.v / b.v;
    const bool finite = gomath::abs(a.lo) < kInf && gomath::abs(a.hi) < kInf && gomath::abs(b.lo) < kInf &&
                        gomath::abs(b.hi) < kInf;
    if (b.lo < 0 && b.hi > 0) {
        r.lo = -kInf;
        r.hi = kInf;
    } else if (finite && b.lo > 0) {
        r.lo = gomath::next_down(a.lo / (a.lo >= 0 ? b.hi : b.lo));
        r.hi = gomath::next_up(a.hi / (a.hi >= 0 ? b.lo : b.hi));
    } else if (finite && b.hi < 0) {
        r.lo = gomath::next_down(a.hi / (a.hi >= 0 ? b.hi : b.lo));
        r.hi = gomath::next_up(a.lo / (a.lo >= 0 ? b.lo : b.hi));
    } else {
        double d0 = a.lo / b.lo, d1 = a.hi / b.lo, d2 = a.lo / b.hi, d3 = a.hi / b.hi;
        r.lo = gomath::next_down(gomath::min(gomath::min(d0, d1), gomath::min(d2, d3)));
        r.hi = gomath::next_up(gomath::max(gomath::max(d0, d1), gomath::max(d2, d3)));
    }
    ef_check(r, panic);
    return r;
}
// efloat/math.go:35-59
GO_HD bool ef_quadratic(EF a, EF b, EF c, EF& t0, EF& t1, int& panic) {
    double disc = b.v * b.v - 4. * a.v * c.v;
    if (disc < 0) return false;
    double rd = gomath::sqrt(disc);
    EF frd = ef_new(rd, gomath::kMachineEpsilon * rd, panic);
    EF q = (b.v < 0) ? ef_muls(ef_sub(b, frd, panic), -0.5, panic) : ef_muls(ef_add(b, frd, panic), -0.5, panic);
    EF r0 = ef_div(q, a, panic);
    EF r1 = ef_div(c, q, panic);
    if (r0.v > r1.v) {
        EF t = r0; r0 = r1; r1 = t;
    }
    t0 = r0;
    t1 = r1;
    return true;
}

}  // namespace pbrt
