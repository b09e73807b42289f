// tests/mesh_box_check.cpp — host check of the mesh walk's float32 box test
// (mesh_box32_hit, go-pbrt_amd/csrc/pbrt_mesh.h, build option PBRT_MESH_F32)
// against the float64 slab test it replaces (mesh_box_hit): wherever the
// float64 test keeps a box, the float32 test must keep it too (it may keep a
// few more: those cost a node visit, never a result). Rays the float32 test
// does not apply to (a nonzero |d_i| outside [1e-30, 1e30]) must take the
// float64 test through mesh_box_test. Compiled and run by
// tests/test_mesh_box.py; prints "cases=.. kept64=.. extra32=.. bad=.." per family.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../go-pbrt_amd/csrc/pbrt_mesh.h"

using namespace pbrt;

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t nextu() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static double unif() { return (double)(nextu() >> 11) * (1.0 / 9007199254740992.0); }
static double sym(double s) { return (2 * unif() - 1) * s; }

struct Fam {
    const char* name;
    long cases = 0, kept64 = 0, extra32 = 0, bad = 0, f64path = 0;
};

static void box_around(float lo[3], float hi[3], double c, double size) {
    for (int a = 0; a < 3; a++) {
        float x = (float)(sym(c)), y = (float)(x + unif() * size);
        lo[a] = x < y ? x : y;
        hi[a] = x < y ? y : x;
    }
}

// one case: ray (o, d, tmax) against box [lo, hi]
static void check(Fam& f, const float lo[3], const float hi[3], V3 o, V3 d, double tmax) {
    Ray r{o, d, tmax, 0};
    const V3 inv{1 / d.x, 1 / d.y, 1 / d.z};
    const int zm = (d.x == 0 ? 1 : 0) | (d.y == 0 ? 2 : 0) | (d.z == 0 ? 4 : 0);
    const bool k64 = mesh_box_hit(lo, hi, r, inv, zm, tmax);
    const MeshRay32 q = mesh_ray32(r, zm, tmax);
    const bool k = mesh_box_test(lo, hi, r, inv, zm, tmax, q);
    f.cases++;
    f.kept64 += k64;
    f.f64path += !q.ok;
    if (k64 && !k) {
        if (f.bad < 5)
            std::printf("BAD %s o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) tmax=%.17g lo=(%.9g %.9g %.9g) "
                        "hi=(%.9g %.9g %.9g)\n", f.name, o.x, o.y, o.z, d.x, d.y, d.z, tmax, lo[0], lo[1], lo[2],
                        hi[0], hi[1], hi[2]);
        f.bad++;
    }
    if (k && !k64) f.extra32++;
}

static V3 unit_dir() {
    for (;;) {
        V3 d{sym(1), sym(1), sym(1)};
        const double l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
        if (l > 1e-3 && l <= 1) return V3{d.x / l, d.y / l, d.z / l};
    }
}

// the float64 entry distance of the box (tmax near it is the hard case)
static double entry64(const float lo[3], const float hi[3], V3 o, V3 d) {
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    double t0 = 0;
    for (int a = 0; a < 3; a++) {
        if (dd[a] == 0) continue;
        const double iv = 1 / dd[a], x = (lo[a] - oo[a]) * iv, y = (hi[a] - oo[a]) * iv;
        const double n = x < y ? x : y;
        t0 = n > t0 ? n : t0;
    }
    return t0;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 200000;
    Fam fams[] = {{"random"}, {"aimed"}, {"tmax_at_entry"}, {"grazing"}, {"axis_parallel"}, {"far_small"},
                  {"tiny_huge_dir"}, {"origin_on_face"}, {"origin_ulps_off_face"}};
    for (long i = 0; i < n; i++) {
        float lo[3], hi[3];
        // random: scene-scale boxes and rays
        box_around(lo, hi, 300, 50);
        check(fams[0], lo, hi, V3{sym(500), sym(500), sym(500)}, unit_dir(), unif() < 0.3 ? kInf : unif() * 1000);
        // aimed: rays through a random point of the box (kept by float64)
        {
            box_around(lo, hi, 300, 20);
            const V3 p{lo[0] + unif() * (hi[0] - lo[0]), lo[1] + unif() * (hi[1] - lo[1]),
                       lo[2] + unif() * (hi[2] - lo[2])};
            const V3 o{sym(500), sym(500), sym(500)};
            V3 d{p.x - o.x, p.y - o.y, p.z - o.z};
            const double l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
            d = V3{d.x / l, d.y / l, d.z / l};
            check(fams[1], lo, hi, o, d, unif() < 0.5 ? kInf : l * (0.5 + unif()));
            // TMax within a few ulps of the float64 entry distance
            const double t = entry64(lo, hi, o, d);
            double tm = t;
            const int steps = (int)(nextu() % 41) - 20;
            for (int s = 0; s < (steps < 0 ? -steps : steps); s++) tm = std::nextafter(tm, steps < 0 ? 0.0 : kInf);
            check(fams[2], lo, hi, o, d, tm);
        }
        // grazing: a direction component tiny, the origin on or near the slab plane
        {
            box_around(lo, hi, 300, 30);
            V3 d = unit_dir();
            const double tiny[] = {1e-8, 1e-15, 1e-25, 1e-30, 2e-30, 5e-31, 1e-300, 0.0};
            const int a = (int)(nextu() % 3);
            const double v = tiny[nextu() % 8] * (unif() < 0.5 ? -1 : 1);
            if (a == 0) d.x = v; else if (a == 1) d.y = v; else d.z = v;
            V3 o{sym(500), sym(500), sym(500)};
            const double plane = (unif() < 0.5 ? lo[a] : hi[a]) + (unif() < 0.3 ? 0.0 : sym(1e-6));
            if (a == 0) o.x = plane; else if (a == 1) o.y = plane; else o.z = plane;
            check(fams[3], lo, hi, o, d, unif() < 0.5 ? kInf : unif() * 2000);
        }
        // axis-parallel: two zero components
        {
            box_around(lo, hi, 100, 30);
            const int a = (int)(nextu() % 3);
            V3 d{0, 0, 0};
            const double s = unif() < 0.5 ? -1 : 1;
            if (a == 0) d.x = s; else if (a == 1) d.y = s; else d.z = s;
            const V3 o{lo[0] + unif() * (hi[0] - lo[0]) * 1.2 - 0.1 * (hi[0] - lo[0]),
                       lo[1] + unif() * (hi[1] - lo[1]) * 1.2 - 0.1 * (hi[1] - lo[1]),
                       lo[2] + unif() * (hi[2] - lo[2]) * 1.2 - 0.1 * (hi[2] - lo[2])};
            check(fams[4], lo, hi, o, d, unif() < 0.5 ? kInf : unif() * 500);
        }
        // far origins, tiny boxes (float32 rounding of the origin dominates)
        {
            const double c = 1e5 * unif();
            for (int a = 0; a < 3; a++) {
                const float x = (float)sym(c);
                lo[a] = x;
                hi[a] = std::nextafter(std::nextafter(x, 1e30f), 1e30f);
            }
            const V3 p{lo[0], lo[1], hi[2]};
            const V3 o{sym(1e6), sym(1e6), sym(1e6)};
            V3 d{p.x - o.x, p.y - o.y, p.z - o.z};
            const double l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
            d = V3{d.x / l, d.y / l, d.z / l};
            check(fams[5], lo, hi, o, d, unif() < 0.5 ? kInf : l * (1 + sym(1e-7)));
        }
        // directions beyond the float32 test's range: the float64 test runs
        {
            box_around(lo, hi, 300, 50);
            V3 d = unit_dir();
            const double e[] = {1e-31, 1e-40, 1e-200, 1e31, 1e100};
            const double v = e[nextu() % 5] * (unif() < 0.5 ? -1 : 1);
            d.y = v;
            check(fams[6], lo, hi, V3{sym(500), sym(500), sym(500)}, d, unif() < 0.5 ? kInf : unif() * 1000);
        }
        // origin exactly on a face or corner of the box
        {
            box_around(lo, hi, 300, 10);
            V3 o{unif() < 0.5 ? (double)lo[0] : (double)hi[0], lo[1] + unif() * (hi[1] - lo[1]),
                 unif() < 0.5 ? (double)lo[2] : (double)hi[2]};
            check(fams[7], lo, hi, o, unit_dir(), unif() < 0.5 ? kInf : unif() * 1e-3);
        }
        // origins a few float64 ulps off a face (not float32 values), TMax at the
        // float64 entry distance
        {
            box_around(lo, hi, 300, 10);
            const int a = (int)(nextu() % 3);
            double oa = unif() < 0.5 ? (double)lo[a] : (double)hi[a];
            const int steps = (int)(nextu() % 9) - 4;
            for (int s = 0; s < (steps < 0 ? -steps : steps); s++) oa = std::nextafter(oa, steps < 0 ? -kInf : kInf);
            V3 o{sym(400), sym(400), sym(400)};
            if (a == 0) o.x = oa; else if (a == 1) o.y = oa; else o.z = oa;
            const V3 d = unit_dir();
            const double t = entry64(lo, hi, o, d);
            check(fams[8], lo, hi, o, d, unif() < 0.5 ? kInf : t);
        }
    }
    int rc = 0;
    for (const Fam& f : fams) {
        std::printf("%s cases=%ld kept64=%ld extra32=%ld f64path=%ld bad=%ld\n", f.name, f.cases, f.kept64,
                    f.extra32, f.f64path, f.bad);
        rc |= f.bad != 0;
    }
    return rc;
}
