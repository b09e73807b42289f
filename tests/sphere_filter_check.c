/* tests/sphere_filter_check.c — CPU check of the product's value-first sphere
 * filter (go-pbrt_amd/csrc/sphere_filter.h) against the oracle's EFloat
 * restatement of Sphere.Intersect's quadratic (oracle/oracle_core.h, which
 * follows pkg/pbrt/sphere.go:64-92 and pkg/efloat).
 *
 * Test infrastructure: compiled and run by tests/test_sphere_filter.py.
 * For every case the filter's verdict must agree with the intervals:
 *   0  -> the reference returns false and no Check() panics;
 *   1  -> no Check() panics, the bound tests pass, and t0/t1 values and the
 *         t0.Low <= 0 / t1.High > TMax decisions are identical;
 *  -1  -> undecided (counted, not checked).
 * Prints one line "cases=.. decided0=.. decided1=.. undecided=.. bad=.." per
 * family and exits non-zero on any disagreement.
 */
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../oracle/oracle_core.h"
#include "../go-pbrt_amd/csrc/sphere_filter.h"

static uint64_t rng_s = 0x9E3779B97F4A7C15ull;
static uint64_t nextu(void) {
    rng_s ^= rng_s << 13;
    rng_s ^= rng_s >> 7;
    rng_s ^= rng_s << 17;
    return rng_s;
}
static double unif(void) { return (double)(nextu() >> 11) * (1.0 / 9007199254740992.0); }
static double sym(double s) { return (2 * unif() - 1) * s; }

typedef struct {
    double o[3], d[3], oe[3], de[3], r, tmax;
} Case;

/* oracle verdict: 0 miss (no panic), 1 roots (fills), 2 panic */
static int oracle_verdict(const Case* c, sf_roots* out) {
    panic_ctx pc;
    pc.kind = 0;
    if (setjmp(pc.jb)) return 2;
    ef_t ox = ef_new(&pc, c->o[0], c->oe[0]), oy = ef_new(&pc, c->o[1], c->oe[1]), oz = ef_new(&pc, c->o[2], c->oe[2]);
    ef_t dx = ef_new(&pc, c->d[0], c->de[0]), dy = ef_new(&pc, c->d[1], c->de[1]), dz = ef_new(&pc, c->d[2], c->de[2]);
    ef_t a = ef_add(&pc, ef_add(&pc, ef_mul(&pc, dx, dx), ef_mul(&pc, dy, dy)), ef_mul(&pc, dz, dz));
    ef_t b = ef_muls(&pc, ef_add(&pc, ef_add(&pc, ef_mul(&pc, dx, ox), ef_mul(&pc, dy, oy)), ef_mul(&pc, dz, oz)), 2.0);
    ef_t cc = ef_sub(&pc, ef_add(&pc, ef_add(&pc, ef_mul(&pc, ox, ox), ef_mul(&pc, oy, oy)), ef_mul(&pc, oz, oz)),
                     ef_muls(&pc, ef_new(&pc, c->r, 0), c->r));
    ef_t t0, t1;
    if (!ef_quadratic(&pc, a, b, cc, &t0, &t1)) return 0;
    if (t0.hi > c->tmax || t1.lo <= 0) return 0;
    out->t0v = t0.v;
    out->t1v = t1.v;
    out->t0lo_le0 = t0.lo <= 0;
    out->t1hi_gt = t1.hi > c->tmax;
    return 1;
}

static void norm3(double* d) {
    double l = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    d[0] /= l; d[1] /= l; d[2] /= l;
}

/* TransformRay-like error vectors: gamma(3) (denormal) times magnitudes */
static void small_errors(Case* c) {
    const double g3 = (3 * 4.9406564584124654e-324) / (1 - 3 * 4.9406564584124654e-324);
    for (int i = 0; i < 3; i++) {
        c->oe[i] = g3 * (fabs(c->o[i]) * 3 + 1);
        c->de[i] = g3 * (fabs(c->d[i]) * 3);
    }
}

static int family(const char* name, int kind, long n) {
    long cnt[3] = {0, 0, 0}, bad = 0, panics = 0;
    for (long k = 0; k < n; k++) {
        Case c;
        memset(&c, 0, sizeof c);
        double s = 1.0;
        if (kind == 5) s = pow(10.0, sym(60));  /* extreme scales */
        c.r = (0.05 + unif() * 10) * s;
        for (int i = 0; i < 3; i++) c.o[i] = sym(30) * s, c.d[i] = sym(1);
        norm3(c.d);
        if (kind == 1) {        /* rays aimed at the sphere, tangent-ish */
            double t[3] = {-c.o[0], -c.o[1], -c.o[2]};
            norm3(t);
            double p[3] = {sym(1), sym(1), sym(1)};
            for (int i = 0; i < 3; i++) c.d[i] = t[i] + p[i] * (c.r / (30 * s)) * unif() * 2;
            norm3(c.d);
        } else if (kind == 2) { /* origin on the surface (c ~ 0): secondary rays */
            double u[3] = {sym(1), sym(1), sym(1)};
            norm3(u);
            for (int i = 0; i < 3; i++) c.o[i] = u[i] * c.r * (1 + sym(1e-15));
            if (nextu() & 1) { /* tangent direction too (b ~ 0) */
                double w[3] = {sym(1), sym(1), sym(1)};
                double dd = w[0] * u[0] + w[1] * u[1] + w[2] * u[2];
                for (int i = 0; i < 3; i++) c.d[i] = w[i] - dd * u[i] + sym(1e-14);
                norm3(c.d);
            }
        } else if (kind == 4) { /* large input errors: the guard must refuse */
            for (int i = 0; i < 3; i++) c.o[i] = sym(30);
        }
        small_errors(&c);
        if (kind == 4)
            for (int i = 0; i < 3; i++) c.oe[i] = fabs(c.o[i]) * pow(10.0, -16 + 10 * unif()), c.de[i] = 1e-140 * unif();
        if (kind == 6) { /* unnormalised / tiny / huge directions */
            double m = pow(10.0, sym(40));
            for (int i = 0; i < 3; i++) c.d[i] *= m;
            small_errors(&c);
        }
        if (kind == 7) { /* negative origin errors (TransformPoint's signed p.Y term) and zero/denormal origins */
            for (int i = 0; i < 3; i++) {
                c.oe[i] = -(double)(nextu() % 6) * 4.9406564584124654e-324;
                int z = (int)(nextu() % 4);
                if (z == 0) c.o[i] = 0.0;
                else if (z == 1) c.o[i] = (double)(nextu() % 4) * 4.9406564584124654e-324;
            }
        }
        c.tmax = INFINITY;
        /* TMax near the roots' values: exact ties and a few ulps either side */
        sf_roots pre;
        int fv = sphere_roots_filter(c.o[0], c.o[1], c.o[2], c.d[0], c.d[1], c.d[2], c.oe[0], c.oe[1], c.oe[2], c.de[0],
                                     c.de[1], c.de[2], c.r, c.tmax, &pre);
        if (fv == 1 || kind == 3) {
            int pick = (int)(nextu() % 6);
            double base = pick < 3 ? pre.t0v : pre.t1v;
            if (fv != 1) base = 1.0;
            int steps = (int)(nextu() % 41) - 20;
            double t = base;
            for (int j = 0; j < (steps < 0 ? -steps : steps); j++) t = nextafter(t, steps < 0 ? -INFINITY : INFINITY);
            c.tmax = (pick % 3 == 2) ? INFINITY : t;
            if (nextu() % 8 == 0) c.tmax = 0.9999;   /* a shadow ray's TMax */
        }
        sf_roots fr, orr;
        int f = sphere_roots_filter(c.o[0], c.o[1], c.o[2], c.d[0], c.d[1], c.d[2], c.oe[0], c.oe[1], c.oe[2], c.de[0],
                                    c.de[1], c.de[2], c.r, c.tmax, &fr);
        int o = oracle_verdict(&c, &orr);
        if (o == 2) panics++;
        if (f < 0) { cnt[2]++; continue; }
        cnt[f]++;
        int ok;
        if (f == 0) ok = (o == 0);
        else ok = (o == 1) && memcmp(&fr.t0v, &orr.t0v, 8) == 0 && memcmp(&fr.t1v, &orr.t1v, 8) == 0 &&
                  fr.t0lo_le0 == orr.t0lo_le0 && fr.t1hi_gt == orr.t1hi_gt;
        if (!ok) {
            if (bad < 5)
                fprintf(stderr, "%s: filter %d oracle %d o=(%a,%a,%a) d=(%a,%a,%a) r=%a tmax=%a\n", name, f, o, c.o[0],
                        c.o[1], c.o[2], c.d[0], c.d[1], c.d[2], c.r, c.tmax);
            bad++;
        }
    }
    printf("%s cases=%ld decided0=%ld decided1=%ld undecided=%ld oracle_panics=%ld bad=%ld\n", name, n, cnt[0], cnt[1],
           cnt[2], panics, bad);
    return bad != 0;
}

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 200000;
    int rc = 0;
    rc |= family("random", 0, n);
    rc |= family("aimed", 1, n);
    rc |= family("on_surface", 2, n);
    rc |= family("tmax_any", 3, n);
    rc |= family("big_errors", 4, n / 4);
    rc |= family("extreme_scale", 5, n / 4);
    rc |= family("odd_direction", 6, n / 4);
    rc |= family("negative_origin_error", 7, n / 4);
    return rc;
}
