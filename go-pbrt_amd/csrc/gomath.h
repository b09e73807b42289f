// gomath.h — Go (amd64) float64 semantics for host and device code.
//
// go-pbrt's arithmetic is float64 with Go's standard-library `math`
// (pure-Go Cephes trig, Nextafter, NaN/±0-aware Max/Min) and pkg/math
// helpers (pkg/math/math.go). Every routine here is evaluated with no FMA
// contraction (the translation units are built with -ffp-contract=off) so
// device results are bit-identical to the Go reference:
//   Cos(Pi/180*90) == 6.123233995736757e-17   (pkg/pbrt/transform_test.go:80)
// fp64 denormals must be preserved: MachineEpsilon is the smallest denormal
// (pkg/math/math.go:17) and every error bound in the hot path is denormal-scale.
#pragma once
#pragma clang fp contract(off)

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GO_HD __host__ __device__ __forceinline__
#else
// plain C++ (host-only checks of the product headers, tests/xf_fast_check.cpp)
#define GO_HD inline
#endif
// Go's trig routines are long polynomial sequences; GO_TRIG lets a build keep
// one out-of-line copy of each instead of inlining them at every call site.
#ifndef GO_TRIG
#define GO_TRIG GO_HD
#endif

namespace gomath {

constexpr double kPi = 3.14159265358979323846264338327950288;   // float64(math.Pi)
constexpr double kMachineEpsilon = 4.9406564584124654e-324;     // NextFloatUp(0)
constexpr double kOneMinusEpsilon = 0.99999999999999988898;     // NextFloatDown(1)
constexpr double kInf = __builtin_huge_val();

GO_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
GO_HD double from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }
GO_HD bool is_nan(double x) { return x != x; }
GO_HD bool is_inf(double x) { return x == kInf || x == -kInf; }
GO_HD bool signbit(double x) { return (bits(x) >> 63) != 0; }
GO_HD double abs(double x) { return from_bits(bits(x) & ~(1ULL << 63)); }
GO_HD double copysign(double x, double s) {
    return from_bits((bits(x) & ~(1ULL << 63)) | (bits(s) & (1ULL << 63)));
}
GO_HD double nan() { return from_bits(0x7FF8000000000001ULL); }

// src/math/dim.go Max/Min (+Inf / -Inf win over NaN; +0 > -0). Written as
// selects (no early returns) so 64-lane waves do not branch on them; the
// results are bit-identical to the Go code path by path:
//   x == y (incl. +0 vs -0): Max -> bits(x) & bits(y)  (+0 unless both -0)
//                            Min -> bits(x) | bits(y)  (-0 unless both +0)
GO_HD double max(double x, double y) {
    double r = x > y ? x : y;
    r = x == y ? from_bits(bits(x) & bits(y)) : r;
    r = (is_nan(x) || is_nan(y)) ? nan() : r;
    return (x == kInf || y == kInf) ? kInf : r;
}
GO_HD double min(double x, double y) {
    double r = x < y ? x : y;
    r = x == y ? from_bits(bits(x) | bits(y)) : r;
    r = (is_nan(x) || is_nan(y)) ? nan() : r;
    return (x == -kInf || y == -kInf) ? -kInf : r;
}

// Go's Max/Min restricted to non-NaN operands, where they order -0 < +0 like
// IEEE maximum/minimum; on the device this is one v_max_f64 / v_min_f64
// (the ±0 ordering is checked against the oracle by the device probes).
GO_HD double max_nonan(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmax(x, y);
#else
    return max(x, y);
#endif
}
GO_HD double min_nonan(double x, double y) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmin(x, y);
#else
    return min(x, y);
#endif
}

// src/math/nextafter.go
GO_HD double nextafter(double x, double y) {
    if (is_nan(x) || is_nan(y)) return nan();
    if (x == y) return x;
    if (x == 0) return copysign(from_bits(1), y);
    if ((y > x) == (x > 0)) return from_bits(bits(x) + 1);
    return from_bits(bits(x) - 1);
}
// pkg/math/math.go:122-128: Nextafter(v, v+1) / Nextafter(v, v-1); no-op for
// |v| >= 2^53 (v == v±1, parity ledger #24). Branch-free forms of the above.
GO_HD double next_up(double v) {
    const uint64_t u = bits(v);
    uint64_t r = v > 0 ? u + 1 : u - 1;
    r = v == 0 ? 1ULL : r;
    double d = from_bits(r);
    d = v == v + 1 ? v : d;
    return is_nan(v) ? nan() : d;
}
GO_HD double next_down(double v) {
    const uint64_t u = bits(v);
    uint64_t r = v > 0 ? u - 1 : u + 1;
    r = v == 0 ? 0x8000000000000001ULL : r;
    double d = from_bits(r);
    d = v == v - 1 ? v : d;
    return is_nan(v) ? nan() : d;
}

// pkg/math/math.go:82-84: Gamma(n) = n*eps/(1-n*eps) with eps a denormal
GO_HD double gamma(double n) { return (n * kMachineEpsilon) / (1 - n * kMachineEpsilon); }
GO_HD double clamp(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }
GO_HD double lerp(double t, double a, double b) { return (1.0 - t) * a + t * b; }
GO_HD double radians(double deg) { return kPi / 180.0 * deg; }

// Go int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> math.MinInt64
GO_HD int64_t to_int(double x) {
    if (is_nan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0)
        return (int64_t)0x8000000000000000ULL;
    return (int64_t)x;
}

// -------------------------------------------------------- sin / cos / tan
namespace detail {
constexpr double PI4A = 7.85398125648498535156e-1;
constexpr double PI4B = 3.77489470793079817668e-8;
constexpr double PI4C = 2.69515142907905952645e-15;
constexpr double FOUR_OVER_PI = 1.27323954473516268615;   // const 4/Pi, rounded once

GO_HD double sin_poly(double z, double zz) {
    return z + z * zz * ((((((1.58962301576546568060e-10 * zz) + -2.50507477628578072866e-8) * zz +
                            2.75573136213857245213e-6) * zz + -1.98412698295895385996e-4) * zz +
                          8.33333333332211858878e-3) * zz + -1.66666666666666307295e-1);
}
GO_HD double cos_poly(double zz) {
    return 1.0 - 0.5 * zz +
           zz * zz * ((((((-1.13585365213876817300e-11 * zz) + 2.08757008419747316778e-9) * zz +
                         -2.75573141792967388112e-7) * zz + 2.48015872888517045348e-5) * zz +
                       -1.38888888888730564116e-3) * zz + 4.16666666666665929218e-2);
}
// Cody-Waite reduction of sin.go; hot-path arguments are < reduceThreshold
GO_HD double reduce(double x, uint64_t& j) {
    j = (uint64_t)(x * FOUR_OVER_PI);
    double y = (double)j;
    if (j & 1) { j++; y++; }
    j &= 7;
    return ((x - y * PI4A) - y * PI4B) - y * PI4C;
}
}  // namespace detail

GO_TRIG double cos(double x) {
    if (is_nan(x) || is_inf(x)) return nan();
    bool sign = false;
    x = abs(x);
    uint64_t j;
    double z = detail::reduce(x, j);
    if (j > 3) { j -= 4; sign = !sign; }
    if (j > 1) sign = !sign;
    double zz = z * z;
    double y = (j == 1 || j == 2) ? detail::sin_poly(z, zz) : detail::cos_poly(zz);
    return sign ? -y : y;
}
GO_TRIG double sin(double x) {
    if (x == 0 || is_nan(x)) return x;
    if (is_inf(x)) return nan();
    bool sign = false;
    if (x < 0) { x = -x; sign = true; }
    uint64_t j;
    double z = detail::reduce(x, j);
    if (j > 3) { sign = !sign; j -= 4; }
    double zz = z * z;
    double y = (j == 1 || j == 2) ? detail::cos_poly(zz) : detail::sin_poly(z, zz);
    return sign ? -y : y;
}
// src/math/tan.go (host-side camera setup)
GO_TRIG double tan(double x) {
    if (x == 0 || is_nan(x)) return x;
    if (is_inf(x)) return nan();
    bool sign = false;
    if (x < 0) { x = -x; sign = true; }
    uint64_t j;
    double z = detail::reduce(x, j);
    double zz = z * z;
    double y = z;
    if (zz > 1e-14)
        y = z + z * (zz * (((-1.30936939181383777646e4 * zz) + 1.15351664838587416140e6) * zz +
                           -1.79565251976484877988e7) /
                     ((((zz + 1.36812963470692954678e4) * zz + -1.32089234440210967447e6) * zz +
                       2.50083801823357915839e7) * zz + -5.38695755929454629881e7));
    if (j & 2) y = -1 / y;
    return sign ? -y : y;
}

// ------------------------------------------------------------ atan family
namespace detail {
GO_HD double xatan(double x) {
    double z = x * x;
    z = z * ((((-8.750608600031904122785e-01 * z + -1.615753718733365076637e+01) * z +
               -7.500855792314704667340e+01) * z + -1.228866684490136173410e+02) * z +
             -6.485021904942025371773e+01) /
        (((((z + 2.485846490142306297962e+01) * z + 1.650270098316988542046e+02) * z +
           4.328810604912902668951e+02) * z + 4.853903996359136964868e+02) * z +
         1.945506571482613964425e+02);
    return x * z + x;
}
GO_HD double satan(double x) {
    constexpr double Morebits = 6.123233995736765886130e-17;
    if (x <= 0.66) return xatan(x);
    if (x > 2.41421356237309504880) return kPi / 2 - xatan(1 / x) + Morebits;
    return kPi / 4 + xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
}  // namespace detail

GO_HD double atan(double x) {
    if (x == 0) return x;
    return x > 0 ? detail::satan(x) : -detail::satan(-x);
}
// src/math/atan2.go
GO_TRIG double atan2(double y, double x) {
    if (is_nan(y) || is_nan(x)) return nan();
    if (y == 0) return (x >= 0 && !signbit(x)) ? copysign(0, y) : copysign(kPi, y);
    if (x == 0) return copysign(kPi / 2, y);
    if (is_inf(x)) {
        if (x == kInf) return is_inf(y) ? copysign(kPi / 4, y) : copysign(0, y);
        return is_inf(y) ? copysign(2.35619449019234492884698253745962716, y) : copysign(kPi, y);
    }
    if (is_inf(y)) return copysign(kPi / 2, y);
    double q = atan(y / x);
    if (x < 0) return q <= 0 ? q + kPi : q - kPi;
    return q;
}
// src/math/asin.go
GO_TRIG double asin(double x) {
    if (x == 0) return x;
    bool sign = false;
    if (x < 0) { x = -x; sign = true; }
    if (x > 1) return nan();
    double t = __builtin_sqrt(1 - x * x);
    t = (x > 0.7) ? kPi / 2 - detail::satan(t / x) : detail::satan(x / t);
    return sign ? -t : t;
}
GO_TRIG double acos(double x) { return kPi / 2 - asin(x); }
GO_HD double sqrt(double x) { return __builtin_sqrt(x); }
GO_HD double floor(double x) { return __builtin_floor(x); }
GO_HD double ceil(double x) { return __builtin_ceil(x); }

}  // namespace gomath
