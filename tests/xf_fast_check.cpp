// tests/xf_fast_check.cpp — host check of the product's value-only TransformRay
// (xf_fast, go-pbrt_amd/csrc/pbrt_core.h) against the exact one (xf_ray, the
// restatement of transform.go:279-300 that the GPU parity tests pin to the
// oracle). Wherever xf_fast accepts a ray, the object-space origin and
// direction must be bit-identical to xf_ray's and the error vectors must pass
// the sphere filter's guard the same way zeros do (|err| <= 1e-150; a negative
// origin error only where |o_i| >= 1e-100). Compiled and run by
// tests/test_sphere_filter.py; prints "cases=.. fast=.. bad=.." per family.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../go-pbrt_amd/csrc/pbrt_core.h"

using namespace pbrt;

static uint64_t rs = 0x2545F4914F6CDD1Dull;
static uint64_t nextu() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static double unif() { return (double)(nextu() >> 11) * (1.0 / 9007199254740992.0); }
static double sym(double s) { return (2 * unif() - 1) * s; }

static pbrt_matrix4x4 ident() {
    pbrt_matrix4x4 m;
    std::memset(&m, 0, sizeof m);
    for (int i = 0; i < 4; i++) m.m[i][i] = 1;
    return m;
}
static pbrt_matrix4x4 mul(const pbrt_matrix4x4& a, const pbrt_matrix4x4& b) {
    pbrt_matrix4x4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += a.m[i][k] * b.m[k][j];
            r.m[i][j] = s;
        }
    return r;
}
static double pick_coord(double scale) {
    switch (nextu() % 10) {
    case 0: return 0.0;
    case 1: return -0.0;
    case 2: return 4.9406564584124654e-324 * (double)(nextu() % 5);
    case 3: return std::ldexp(sym(1), -(int)(nextu() % 1100));
    default: return sym(scale);
    }
}
static bool same(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

static pbrt_matrix4x4 random_matrix(int kind) {
    pbrt_matrix4x4 m = ident();
    if (kind == 0) {   // identity, maybe with -0 translation (Go's Translate(0).Inverse())
        if (nextu() & 1) m.m[0][3] = m.m[1][3] = m.m[2][3] = -0.0;
    } else if (kind == 1) {   // translation
        for (int i = 0; i < 3; i++) m.m[i][3] = (nextu() % 4 == 0) ? -0.0 : sym(100);
    } else if (kind == 2) {   // rotation (Go trig) x translation, as the host builds
        const double a = gomath::radians(sym(180));
        const double c = gomath::cos(a), s = gomath::sin(a);
        pbrt_matrix4x4 r = ident();
        const int ax = (int)(nextu() % 3), u = (ax + 1) % 3, v = (ax + 2) % 3;
        r.m[u][u] = c; r.m[u][v] = -s; r.m[v][u] = s; r.m[v][v] = c;
        pbrt_matrix4x4 t = ident();
        for (int i = 0; i < 3; i++) t.m[i][3] = sym(60);
        m = mul(t, r);
    } else if (kind == 3) {   // general affine, incl. scales
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 4; j++) m.m[i][j] = (nextu() % 5 == 0) ? 0.0 : sym(j == 3 ? 100 : 3);
    } else {                  // projective or huge entries: always the exact path
        m.m[3][2] = (nextu() & 1) ? 1.0 : 0.0;
        m.m[0][0] = (nextu() & 1) ? 1e12 : 1.0;
    }
    return m;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 200000;
    int rc = 0;
    const char* names[] = {"identity", "translation", "rotation", "affine", "slow"};
    for (int kind = 0; kind < 5; kind++) {
        long fast = 0, bad = 0;
        for (long k = 0; k < n; k++) {
            const pbrt_matrix4x4 M = random_matrix(kind);
            const int fk = xf_fast_kind(M);
            Ray r;
            r.o = V3{pick_coord(100), pick_coord(100), pick_coord(100)};
            r.d = V3{pick_coord(1), pick_coord(1), pick_coord(1)};
            if (nextu() % 3 == 0) r.d = normalized(r.d);
            r.tmax = 1e30;
            r.time = 0;
            V3 o = r.o, d = r.d;
            if (!xf_fast(fk, M, o, d)) continue;
            fast++;
            V3 oe, de;
            const Ray x = xf_ray(M, r, &oe, &de);
            bool ok = same(o.x, x.o.x) && same(o.y, x.o.y) && same(o.z, x.o.z) && same(d.x, x.d.x) &&
                      same(d.y, x.d.y) && same(d.z, x.d.z);
            const double E = 1e-150, V = 1e-100;
            const double ov[3] = {x.o.x, x.o.y, x.o.z}, oev[3] = {oe.x, oe.y, oe.z}, dev[3] = {de.x, de.y, de.z};
            for (int i = 0; i < 3; i++) {
                ok = ok && std::fabs(oev[i]) <= E && (oev[i] >= 0 || std::fabs(ov[i]) >= V);
                ok = ok && dev[i] >= 0 && dev[i] <= E;
            }
            if (!ok) {
                if (bad < 5)
                    std::fprintf(stderr, "%s: o=(%a,%a,%a) d=(%a,%a,%a) fast o=(%a,%a,%a) exact o=(%a,%a,%a)\n",
                                 names[kind], r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, o.x, o.y, o.z, x.o.x, x.o.y,
                                 x.o.z);
                bad++;
            }
        }
        std::printf("%s cases=%ld fast=%ld bad=%ld\n", names[kind], n, fast, bad);
        if (bad) rc = 1;
    }
    return rc;
}
