/*
 * oracle/go_math.h — TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * Plain-C restatement of the Go (amd64, Go <= 1.11 era) standard-library
 * `math` routines and the reference's pkg/math helpers that go-pbrt's hot path
 * depends on. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may use this file.
 *
 * Provenance: the Go standard library is a third-party dependency absent from
 * /root/reference (no Go toolchain or Go source in this image). The algorithms
 * below restate Go's published pure-Go implementations (src/math/sin.go,
 * tan.go, atan.go, atan2.go, asin.go, nextafter.go, dim.go), which are
 * Cephes-derived. Pinned by the reference's own test
 *   pkg/pbrt/transform_test.go:77-81  Cos(Pi/180*90) == 6.123233995736757e-17
 * (libm gives ...766e-17) and by the widely observed Go value
 *   Sin(Pi) == 1.2246467991473515e-16 (libm ...532e-16).
 * Everything else about these routines is parity-unpinned beyond those anchors.
 *
 * Must be compiled with -ffp-contract=off and without -ffast-math.
 */
#ifndef ORACLE_GO_MATH_H
#define ORACLE_GO_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

/* Algorithmic-FLOP accounting (bench.py roofline): one fp64 add, sub, mul, div
 * or sqrt = 1; comparisons, Max/Min, abs, negation and Nextafter's bit steps = 0.
 * Compiled in only for _build/liboracle_flops.so (-DORACLE_COUNT_FLOPS). */
#ifdef ORACLE_COUNT_FLOPS
extern __thread uint64_t orc_flops;
#define FL(n) (orc_flops += (uint64_t)(n))
#else
#define FL(n) ((void)0)
#endif

static inline uint64_t gm_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double gm_from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static inline int gm_isnan(double x) { return x != x; }
/* math.NaN() = Float64frombits(0x7FF8000000000001) (src/math/bits.go) */
static inline double go_nan(void) {
    union { uint64_t u; double d; } v = {0x7FF8000000000001ULL};
    return v.d;
}
static inline int gm_isinf(double x, int sign) {
    if (sign > 0) return x == INFINITY;
    if (sign < 0) return x == -INFINITY;
    return x == INFINITY || x == -INFINITY;
}
static inline int gm_signbit(double x) { return (int)(gm_bits(x) >> 63); }
static inline double gm_copysign(double x, double s) {
    return gm_from_bits((gm_bits(x) & ~(1ULL << 63)) | (gm_bits(s) & (1ULL << 63)));
}
static inline double gm_abs(double x) { return gm_from_bits(gm_bits(x) & ~(1ULL << 63)); }

/* math.Max / math.Min (src/math/dim.go; amd64 asm has the same special cases) */
static inline double go_max(double x, double y) {
    if (gm_isinf(x, 1) || gm_isinf(y, 1)) return INFINITY;
    if (gm_isnan(x) || gm_isnan(y)) return go_nan();
    if (x == 0 && x == y) return gm_signbit(x) ? y : x;
    return x > y ? x : y;
}
static inline double go_min(double x, double y) {
    if (gm_isinf(x, -1) || gm_isinf(y, -1)) return -INFINITY;
    if (gm_isnan(x) || gm_isnan(y)) return go_nan();
    if (x == 0 && x == y) return gm_signbit(x) ? x : y;
    return x < y ? x : y;
}

/* math.Nextafter (src/math/nextafter.go) */
static inline double go_nextafter(double x, double y) {
    if (gm_isnan(x) || gm_isnan(y)) return go_nan();
    if (x == y) return x;
    if (x == 0) return gm_copysign(gm_from_bits(1), y);
    if ((y > x) == (x > 0)) return gm_from_bits(gm_bits(x) + 1);
    return gm_from_bits(gm_bits(x) - 1);
}

/* pkg/math/math.go:122-128 */
static inline double go_next_float_up(double v) { FL(1); return go_nextafter(v, v + 1); }
static inline double go_next_float_down(double v) { FL(1); return go_nextafter(v, v - 1); }

/* pkg/math/math.go:17-19: MachineEpsilon = NextFloatUp(0) (smallest denormal) */
#define GO_MACHINE_EPSILON 4.9406564584124654e-324
/* OneMinusEpsilon = NextFloatDown(1) */
#define GO_ONE_MINUS_EPSILON 0.99999999999999988898
/* pkg/math/math.go:82-84 */
static inline double go_gamma(double n) {
    FL(4);
    return (n * GO_MACHINE_EPSILON) / (1 - n * GO_MACHINE_EPSILON);
}
/* pkg/math/math.go:42-51 */
static inline double go_clamp(double v, double lo, double hi) {
    if (v < lo) return lo;
    if (v > hi) return hi;
    return v;
}
static inline double go_lerp(double t, double v1, double v2) { FL(4); return (1.0 - t) * v1 + t * v2; }

/* int(float64) / int64(float64) on amd64: CVTTSD2SQ, NaN / out of range -> INT64_MIN */
static inline int64_t go_f2i(double x) {
    if (gm_isnan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0)
        return INT64_MIN;
    return (int64_t)x;
}

/* pkg/math Pi family (package vars, float64 runtime arithmetic) */
#define GO_PI 3.14159265358979323846264338327950288
static const double go_Pi = GO_PI;

/* ---------------------------------------------------------- sin / cos / tan */
static const double gm_PI4A = 7.85398125648498535156e-1;
static const double gm_PI4B = 3.77489470793079817668e-8;
static const double gm_PI4C = 2.69515142907905952645e-15;
static const double gm_4_over_pi = 1.27323954473516268615;   /* const 4/Pi rounded */
static const double gm_sin[6] = {
    1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
    -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1};
static const double gm_cos[6] = {
    -1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
    2.48015872888517045348e-5, -1.38888888888730564116e-3, 4.16666666666665929218e-2};

static inline void gm_trig_reduce(double x, uint64_t* jo, double* zo) {
    /* arguments on the hot path are far below reduceThreshold (1<<29) */
    uint64_t j = (uint64_t)(x * gm_4_over_pi);
    double y = (double)j;
    FL(7);
    if (j & 1) { j++; y++; FL(1); }
    j &= 7;
    *zo = ((x - y * gm_PI4A) - y * gm_PI4B) - y * gm_PI4C;
    *jo = j;
}
static inline double gm_sin_poly(double z, double zz) {
    FL(14);
    return z + z * zz * ((((((gm_sin[0] * zz) + gm_sin[1]) * zz + gm_sin[2]) * zz + gm_sin[3]) * zz + gm_sin[4]) * zz + gm_sin[5]);
}
static inline double gm_cos_poly(double zz) {
    FL(16);
    return 1.0 - 0.5 * zz + zz * zz * ((((((gm_cos[0] * zz) + gm_cos[1]) * zz + gm_cos[2]) * zz + gm_cos[3]) * zz + gm_cos[4]) * zz + gm_cos[5]);
}

/* src/math/sin.go cos() */
static inline double go_cos(double x) {
    if (gm_isnan(x) || gm_isinf(x, 0)) return go_nan();
    int sign = 0;
    x = gm_abs(x);
    uint64_t j; double z;
    gm_trig_reduce(x, &j, &z);
    if (j > 3) { j -= 4; sign = !sign; }
    if (j > 1) sign = !sign;
    double zz = z * z, y;
    FL(1);
    if (j == 1 || j == 2) y = gm_sin_poly(z, zz);
    else y = gm_cos_poly(zz);
    return sign ? -y : y;
}
/* src/math/sin.go sin() */
static inline double go_sin(double x) {
    if (x == 0 || gm_isnan(x)) return x;
    if (gm_isinf(x, 0)) return go_nan();
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j; double z;
    gm_trig_reduce(x, &j, &z);
    if (j > 3) { sign = !sign; j -= 4; }
    double zz = z * z, y;
    FL(1);
    if (j == 1 || j == 2) y = gm_cos_poly(zz);
    else y = gm_sin_poly(z, zz);
    return sign ? -y : y;
}
/* src/math/tan.go tan() (host-side setup only: Perspective) */
static inline double go_tan(double x) {
    static const double P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
    /* _tanQ[1..4]; _tanQ[0] = 1.0 is implicit in the leading zz term */
    static const double Q1 = 1.36812963470692954678e4, Q2 = -1.32089234440210967447e6,
                        Q3 = 2.50083801823357915839e7, Q4 = -5.38695755929454629881e7;
    if (x == 0 || gm_isnan(x)) return x;
    if (gm_isinf(x, 0)) return go_nan();
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j; double z;
    gm_trig_reduce(x, &j, &z);   /* tan.go does not mask j&7; j&2 is unaffected */
    double zz = z * z, y;
    FL(1);
    if (zz > 1e-14) FL(15);
    if (zz > 1e-14)
        y = z + z * (zz * (((P[0] * zz) + P[1]) * zz + P[2]) / ((((zz + Q1) * zz + Q2) * zz + Q3) * zz + Q4));
    else
        y = z;
    if (j & 2) { y = -1 / y; FL(1); }
    return sign ? -y : y;
}

/* ------------------------------------------------------ atan / asin / acos */
static inline double gm_xatan(double x) {
    const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
                 P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
                 P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
                 Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
                 Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
    FL(22);
    double z = x * x;
    z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
    z = x * z + x;
    return z;
}
static inline double gm_satan(double x) {
    const double Morebits = 6.123233995736765886130e-17;
    const double Tan3pio8 = 2.41421356237309504880;
    if (x <= 0.66) return gm_xatan(x);
    if (x > Tan3pio8) { FL(3); return GO_PI / 2 - gm_xatan(1 / x) + Morebits; }
    FL(5);
    return GO_PI / 4 + gm_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
/* src/math/atan.go */
static inline double go_atan(double x) {
    if (x == 0) return x;
    if (x > 0) return gm_satan(x);
    return -gm_satan(-x);
}
/* src/math/atan2.go */
static inline double go_atan2(double y, double x) {
    if (gm_isnan(y) || gm_isnan(x)) return go_nan();
    if (y == 0) {
        if (x >= 0 && !gm_signbit(x)) return gm_copysign(0, y);
        return gm_copysign(GO_PI, y);
    }
    if (x == 0) return gm_copysign(GO_PI / 2, y);
    if (gm_isinf(x, 0)) {
        if (gm_isinf(x, 1)) {
            if (gm_isinf(y, 0)) return gm_copysign(GO_PI / 4, y);
            return gm_copysign(0, y);
        }
        if (gm_isinf(y, 0)) return gm_copysign(2.35619449019234492884698253745962716, y); /* const 3*Pi/4 */
        return gm_copysign(GO_PI, y);
    }
    if (gm_isinf(y, 0)) return gm_copysign(GO_PI / 2, y);
    double q = go_atan(y / x);
    FL(1);
    if (x < 0) {
        FL(1);
        if (q <= 0) return q + GO_PI;
        return q - GO_PI;
    }
    return q;
}
/* src/math/asin.go */
static inline double go_asin(double x) {
    if (x == 0) return x;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    if (x > 1) return go_nan();
    double temp = sqrt(1 - x * x);
    FL(3);
    if (x > 0.7) { temp = GO_PI / 2 - gm_satan(temp / x); FL(2); }
    else { temp = gm_satan(x / temp); FL(1); }
    return sign ? -temp : temp;
}
static inline double go_acos(double x) { FL(1); return GO_PI / 2 - go_asin(x); }

/* pkg/math/math.go:113-115: Radians(deg) = Pi / 180.0 * deg (float64 vars) */
static inline double go_radians(double deg) { FL(2); return go_Pi / 180.0 * deg; }

#endif
