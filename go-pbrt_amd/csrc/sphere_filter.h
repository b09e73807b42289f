/* sphere_filter.h — value-first decisions for Sphere.Intersect's EFloat quadratic.
 *
 * Reference: pkg/pbrt/sphere.go:64-92 (the EFloat ray, a/b/c, Quadratic and the
 * two TMax comparisons), pkg/efloat/efloat.go:10-111 (New/Add/Sub/Mul/Div/Check),
 * pkg/efloat/math.go:35-59 (Quadratic).
 *
 * An EFloat's Value field is plain float64 arithmetic on the operands' values,
 * so t0.Value and t1.Value are computed here without any interval. The
 * reference's decisions read the bounds (t0.High > TMax, t1.Low <= 0,
 * t0.Low <= 0, t1.High > TMax), and every EFloat op may panic in Check().
 * This filter decides them from the values plus a runtime radius R with
 * [Low, High] inside [Value - R, Value + R], and only where it can prove that no
 * Check() on the way fails. Otherwise it returns -1 and the caller evaluates the
 * intervals exactly as the reference does. DESIGN.md §3.6 has the proof; in short:
 *   - every bound satisfies Low <= Value <= High (rounding is monotone, next_down
 *     / next_up move outward), so Value > TMax implies High > TMax and
 *     Value <= 0 implies Low <= 0: those rejects are exact;
 *   - with |o|,|d|,r <= 1e50, |errors| <= 1e-150 (direction errors >= 0, an
 *     origin error < 0 only where |o_i| >= 1e-100), r, a, |q| >= 1e-20 and
 *     |q| > 2 R_q, every bound is finite and a, q exclude zero, so no Check fails;
 *   - a running-error bound over the op sequence gives R_q <= 17.5 eps M_q,
 *     R(q/a) <= 31 eps M_q/a, R(c/q) <= (15 eps + 17.5 eps M_q/|q|) M_c/(|q| - R_q)
 *     (eps = 2^-52; M_* are magnitude sums); the constants below are twice these,
 *     which also covers the rounding of these formulas and of the comparisons.
 * Plain C (no Go-semantics helpers needed: no NaN reaches a comparison that
 * matters), so tests/sphere_filter_check.c checks it against the oracle's
 * EFloat restatement on the CPU.
 */
#ifndef PBRT_SPHERE_FILTER_H
#define PBRT_SPHERE_FILTER_H

#if defined(__HIPCC__)
#define SF_HD __host__ __device__ __forceinline__
#else
#define SF_HD static inline
#endif

typedef struct {
    double t0v, t1v; /* EFloat values of t0, t1 after Quadratic's swap */
    int t0lo_le0;    /* t0.Low <= 0 */
    int t1hi_gt;     /* t1.High > TMax */
} sf_roots;

#define SF_EPS 2.220446049250313080847e-16 /* 2^-52 */

SF_HD double sf_abs(double x) { return __builtin_fabs(x); }

/* o, d: the object-space ray (TransformRay's output), oe, de: its error
 * vectors. Returns 0 when the reference returns false without panicking, 1 when
 * *out holds the reference's decisions, -1 when undecided. */
SF_HD int sphere_roots_filter(double ox, double oy, double oz, double dx, double dy, double dz, double oex,
                              double oey, double oez, double dex, double dey, double dez, double radius,
                              double tmax, sf_roots* out) {
    /* the Values of a, b, c and the discriminant, in the reference's order */
    const double av = (dx * dx + dy * dy) + dz * dz;
    const double bv = ((dx * ox + dy * oy) + dz * oz) * 2.0;
    const double cv = ((ox * ox + oy * oy) + oz * oz) - radius * radius;
    const double disc = bv * bv - 4. * av * cv;
    const double V = 1e-100;
    /* New(v, err) keeps Low <= v <= High for err >= 0, and for err < 0 where
     * |err| is below half an ulp of v: the origin errors can be negative
     * (TransformPoint's signed |m[i][1]| * p.Y term); the
     * direction errors are sums of |.| products. (A NaN fails every test.) */
    const int sgn_ok = (oex >= 0 || sf_abs(ox) >= V) && (oey >= 0 || sf_abs(oy) >= V) &&
                       (oez >= 0 || sf_abs(oz) >= V) && dex >= 0 && dey >= 0 && dez >= 0;
    if (disc < 0) {
        /* efloat/math.go:38-40 returns false; with every operand finite and
         * below 1e100 (and errors of |.| <= 1e100 as above) no Check() before it
         * can panic */
        const double big = 1e100;
        const int moderate = sf_abs(ox) < big && sf_abs(oy) < big && sf_abs(oz) < big && sf_abs(dx) < big &&
                             sf_abs(dy) < big && sf_abs(dz) < big && sf_abs(oex) <= 1e-150 &&
                             sf_abs(oey) <= 1e-150 && sf_abs(oez) <= 1e-150 && dex < big && dey < big && dez < big &&
                             sf_abs(radius) < big;
        return moderate && sgn_ok ? 0 : -1;
    }
    const double B = 1e50, E = 1e-150, S = 1e-20;
    const int g1 = sgn_ok && sf_abs(ox) <= B && sf_abs(oy) <= B && sf_abs(oz) <= B && sf_abs(dx) <= B &&
                   sf_abs(dy) <= B && sf_abs(dz) <= B && sf_abs(oex) <= E && sf_abs(oey) <= E && sf_abs(oez) <= E &&
                   dex <= E && dey <= E && dez <= E && sf_abs(radius) <= B && sf_abs(radius) >= S;
    if (!g1) return -1;
    const double rd = __builtin_sqrt(disc);
    const double qv = (bv < 0 ? bv - rd : bv + rd) * -0.5;
    const double aq = sf_abs(qv);
    const double Mq = 0.5 * (2.0 * ((sf_abs(dx * ox) + sf_abs(dy * oy)) + sf_abs(dz * oz)) + rd);
    const double Rq = 36.0 * SF_EPS * Mq;   /* >= 2 x 17.5 eps */
    if (!(av >= S && aq >= S && aq > 2.0 * Rq)) return -1;
    const double Mc = ((ox * ox + oy * oy) + oz * oz) + radius * radius;
    const double r0v = qv / av, r1v = cv / qv;
    const double R0 = 64.0 * SF_EPS * Mq / av;
    const double R1 = (32.0 * SF_EPS + 36.0 * SF_EPS * (Mq / aq)) * (Mc / (aq - Rq));
    double t0v = r0v, t1v = r1v, e0 = R0, e1 = R1;
    if (r0v > r1v) {
        t0v = r1v; t1v = r0v; e0 = R1; e1 = R0;
    }
    /* sphere.go:84-86, exact on values */
    if (t0v > tmax || t1v <= 0) return 0;
    if (!(t0v + e0 <= tmax) || !(t1v - e1 > 0)) return -1;
    int t0lo, t1hi;
    if (t0v <= 0) t0lo = 1;
    else if (t0v - e0 > 0) t0lo = 0;
    else return -1;
    if (t1v > tmax) t1hi = 1;
    else if (t1v + e1 <= tmax) t1hi = 0;
    else return -1;
    out->t0v = t0v;
    out->t1v = t1v;
    out->t0lo_le0 = t0lo;
    out->t1hi_gt = t1hi;
    return 1;
}

#endif
