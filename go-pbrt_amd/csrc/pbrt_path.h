// pbrt_path.h — device implementation of go-pbrt's per-path inner loop.
//
// One call of path_li() is one Path.Li (pkg/integrator/path.go:32-157);
// direct_li() is DirectLighting.Li (pkg/integrator/directlighting.go:62-104).
// Everything below them — BVH traversal (pkg/accelerator/bvh.go:659-765),
// TransformedPrimitive/GeometricPrimitive (pkg/pbrt/primitive.go:42-115),
// Sphere (pkg/pbrt/sphere.go) and Disk (pkg/shapes/disk.go) intersection,
// Matte/Lambertian BSDF (pkg/materials/matte.go, pkg/pbrt/reflection.go),
// lights (pkg/lights), UniformSampleOneLight / EstimateDirect
// (pkg/pbrt/integrator.go:23-195) and the Stratified/PCG32 sampler
// (pkg/sampler, pkg/pbrt/rng.go) — is restated in float64 with the
// reference's evaluation order and every parity-ledger quirk.
//
// Reference panics (EFloat Check, Ld > 10, BVH stack overflow) set
// Thread::panic; the caller stops the tile and reports PBRT_E_REF_PANIC.
#pragma once
#pragma clang fp contract(off)

#include "pbrt_core.h"
#include "pbrt_mesh.h"
#include "sphere_filter.h"

namespace pbrt {

// Optional region timing of a trajectory step (built with -DPBRT_STEP_TIMING):
// the first active lane adds each region's wall time to g_step_cycles.
#ifdef PBRT_STEP_TIMING
__device__ unsigned long long g_step_cycles[8];
struct StepTimer {
    long long t;
    __device__ void start() { t = clock64(); }
    __device__ void mark(int i) {
        long long now = clock64();
        if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1)
            atomicAdd(&g_step_cycles[i], (unsigned long long)(now - t));
        t = now;
    }
};
#define STEP_T(x) x
#else
#define STEP_T(x)
#endif

// ----------------------------------------------------------------- scene view
struct DevScene {
    const pbrt_shape_desc* shapes;
    const pbrt_material_desc* materials;
    const pbrt_primitive_desc* prims;
    const struct DevNode* nodes;   // device copy of pbrt_bvh_node[], 64-byte records
    const uint32_t* order;         // [8 octants][n_nodes] preorder visit table (see bvh_walk)
    const struct DevPrim* fprims;  // primitive + its shape in one record (leaf tests)
    const pbrt_light_desc* lights;
    const pbrt_camera_desc* camera;
    const pbrt_film_desc* film;
    const pbrt_distribution_desc* dist;   // Path light distribution (may be null)
    int n_prims, n_nodes, n_lights;
    int use_lds_nodes;   // the kernel staged nodes[] in g_nodes_lds (uniform)
    int n_leaves;        // leaves of the BVH (order[8 * n_nodes + oct * n_nodes + j]: leaf preorder)
    DevMesh mesh;        // triangle meshes (extension, pbrt_mesh.h); mesh.n_nodes == 0: none
    // leaf culling groups of LDS-staged trees (see bvh_walk_analytic): [n_groups][6]
    // bounds, then per octant [n_groups + 1] leaf-position masks (the last: leaves
    // that are always tested); n_groups == 0: test every leaf
    const double* groups;
    const uint32_t* gmasks;
    int n_groups;
    // pbrt_gpu_cancel's flag for the render in flight (fine-grained host memory,
    // written by the host while kernels run), and its device-memory copy that
    // the first wave to read the host flag set publishes (cleared by the host
    // before every render); polled between units of work
    const int* cancel;
    int* cancel_seen;
    int dense_ok;   // k_chain_ci may use bvh_walk_dense (one primitive per leaf, groups, no meshes)
};
// Is the render cancelled? The device copy is an L2 read; poll_host (a rate
// the caller bounds: host-memory reads cross PCIe) also reads the host flag and
// publishes it. The value is the whole wave's (lane 0's).
__device__ __forceinline__ bool cancel_requested(const DevScene& sc, bool poll_host) {
    int v = __hip_atomic_load(sc.cancel_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!v && poll_host) {
        v = __hip_atomic_load(sc.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v) __hip_atomic_store(sc.cancel_seen, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return __builtin_amdgcn_readfirstlane(v) != 0;
}
// cancel_requested with the host flag read at most once a millisecond per
// caller (last_host: that caller's wall_clock64 of its last host read; the
// clock runs at 100 MHz): for loops whose iteration length varies by orders of
// magnitude (a pixel of Stratified(64,64) vs of (2,2)).
__device__ __forceinline__ bool cancel_polled(const DevScene& sc, uint64_t& last_host) {
    const uint64_t now = wall_clock64();
    const bool host = now - last_host >= 100000;
    if (host) last_host = now;
    return cancel_requested(sc, host);
}

// ---------------------------------------------------------------- PCG32 (rng.go)
struct Pcg {
    uint64_t state, inc;
};
__device__ __forceinline__ uint32_t pcg_next(Pcg& r) {
    uint64_t old = r.state;
    r.state = old * 0x5851f42d4c957f2dULL + r.inc;
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((rot + 1u) & 31u));   // (rot+1)&31, parity ledger #1
}
__device__ __forceinline__ void pcg_seed(Pcg& r, uint64_t seed) {   // rng.go:28-34
    r.state = 0;
    r.inc = (seed << 1) | 1;
    pcg_next(r);
    r.state += 0x853c49e6748fea9bULL;
    pcg_next(r);
}
// THROUGHPUT mode (SURVEY.md §8(a) "Mode B"; include/pbrt_gpu.h): the PCG32
// state that starts stream `s` of pixel `pi` (row-major index in its tile) of
// tile `tile`: s = 0 feeds Stratified.StartPixel, s = k >= 1 feeds sample k.
// The increment stays the tile's ((tile << 1) | 1, rng.go:28-34). splitmix64
// finalizer chain; the oracle states the same function (oracle_render.c).
__host__ __device__ __forceinline__ uint64_t mb_mix(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t mb_state(uint64_t tile, uint64_t pi, uint64_t s) {
    return mb_mix(mb_mix(mb_mix(tile) ^ pi) ^ s);
}
__device__ __forceinline__ uint32_t pcg_bounded(Pcg& r, uint32_t b) {   // rng.go:44-53
    uint32_t threshold = (~b + 1u) % b;
    for (;;) {
        uint32_t v = pcg_next(r);
        if (v >= threshold) return v % b;
    }
}
__device__ __forceinline__ double pcg_float(Pcg& r) {   // rng.go:55-57
    return gomath::min(gomath::kOneMinusEpsilon, (double)pcg_next(r) * 2.3283064365386963e-10);
}

// ------------------------------------------------------------ per-thread state
struct Thread {
    Pcg rng;
    int32_t spp, ndims, xs, ys, jitter;
    int32_t sample_index, cur1d, cur2d;
    double* s1d;              // ndims * spp shuffled stratified values (scratch)
    uint16_t* stack;          // BVH traversal stack column in LDS (stride kStackStride)
    int panic;                // PBRT_PANIC_* (sticky)
    int bounce;
    uint64_t closest_rays, shadow_rays;
};
constexpr int kStackStride = 64;   // one 64-lane wave per workgroup

// Stratified.StartPixel (stratified.go:21-48; sampling.go:101-145)
__device__ inline void start_pixel(Thread& t) {
    const int32_t n = t.spp;
    const double inv = 1.0 / (double)n;
    for (int d = 0; d < t.ndims; d++) {
        double* samp = t.s1d + (size_t)d * n;
        for (int32_t i = 0; i < n; i++) {
            double delta = t.jitter ? pcg_float(t.rng) : 0.5;
            samp[i] = gomath::min(((double)i + delta) * inv, gomath::kOneMinusEpsilon);
        }
        for (int32_t i = 0; i < n; i++) {
            int32_t other = i + (int32_t)pcg_bounded(t.rng, (uint32_t)(n - i));
            double a = samp[i];
            samp[i] = samp[other];
            samp[other] = a;
        }
    }
    // StratifiedSample2D writes into a copy (sampling.go:122-124, #3): the 2D
    // values stay (0,0); only the jitter and shuffle draws advance the stream.
    for (int d = 0; d < t.ndims; d++) {
        if (t.jitter)
            for (int32_t k = 0; k < n; k++) { pcg_next(t.rng); pcg_next(t.rng); }
        for (int32_t i = 0; i < n; i++) pcg_bounded(t.rng, (uint32_t)(n - i));
    }
    t.sample_index = 0;
    t.cur1d = t.cur2d = 0;
}
// sampler.go:29-34 — pre-increment, so sample 0 is never traced (#2)
__device__ __forceinline__ bool next_sample(Thread& t) {
    t.cur1d = t.cur2d = 0;
    t.sample_index += 1;
    return t.sample_index < t.spp;
}
__device__ __forceinline__ double get1d(Thread& t) {   // pixel.go:60-69
    if (t.cur1d < t.ndims) {
        double v = t.s1d[(size_t)t.cur1d * t.spp + t.sample_index];
        t.cur1d++;
        return v;
    }
    return pcg_float(t.rng);
}
struct V2 {
    double x, y;
};
__device__ __forceinline__ V2 get2d(Thread& t) {   // pixel.go:71-80
    if (t.cur2d < t.ndims) {
        t.cur2d++;
        return V2{0.0, 0.0};
    }
    double x = pcg_float(t.rng);
    double y = pcg_float(t.rng);
    return V2{x, y};
}

// ------------------------------------------------------- surface interaction
// The reference's SurfaceInteraction shares *interaction (p, perr, n, wo,
// time) and *Shading by pointer (interaction.go:124-148); dpdu..dndv are its
// own. Only fields that reach an output are kept.
struct SI {
    V3 p, perr, n, wo;
    double time;
    V3 sn, sdpdu;
    int prim;
};

// NewSurfaceInteractionWith (interaction.go:176-207) + the object-to-world
// TransformSurfaceInteraction assigned back (*si = *..., sphere.go:185 / disk.go:110)
__device__ inline void make_si(SI& si, const pbrt_matrix4x4& M, const pbrt_matrix4x4& Mi, V3 p, V3 perr, V3 wo,
                               V3 dpdu, V3 dpdv, double time, bool flip) {
    V3 n = normalized(cross(dpdu, dpdv));
    if (flip) n = muls(n, -1);
    // transform.go:302-334
    V3 perr2;
    si.p = xf_point(M, p, perr, &perr2);
    si.perr = perr2;
    si.n = normalized(xf_normal(Mi, n));
    si.wo = normalized(xf_vector(M, wo));
    si.time = time;
    V3 sn = xf_normal(Mi, n);
    si.sdpdu = xf_vector(M, dpdu);
    si.sn = face_forward(sn, si.n);
}
// TransformedPrimitive: only the shared interaction / Shading objects are
// mutated; the transformed copy itself is discarded (primitive.go:104-106, #20)
__device__ inline void transform_si_shared(SI& si, const pbrt_matrix4x4& M, const pbrt_matrix4x4& Mi) {
    V3 perr2;
    si.p = xf_point(M, si.p, si.perr, &perr2);
    si.perr = perr2;
    si.n = normalized(xf_normal(Mi, si.n));
    si.wo = normalized(xf_vector(M, si.wo));
    V3 sn = xf_normal(Mi, si.sn);
    si.sdpdu = xf_vector(M, si.sdpdu);
    si.sn = face_forward(sn, si.n);
}

// -------------------------------------------------------------------- shapes
// `phi > phiMax` of the partial-shape tests (sphere.go:115-131, disk.go:90-95)
// with phi = Atan2(y, x) (+2*Pi if negative). Go's Atan2 lies in [-Pi, Pi], so
// phi <= 2*Pi after rounding and the test is false whenever phiMax >= 2*Pi
// (every full sphere / disk): the Atan2 is skipped there, with the same result
// (a NaN phi compares false either way).
__device__ __forceinline__ bool phi_beyond(double y, double x, double phi_max) {
    const double two_pi = 2 * gomath::kPi;
    if (phi_max >= two_pi) return false;
    double phi = gomath::atan2(y, x);
    if (phi < 0.0) phi += two_pi;
    return phi > phi_max;
}

// Sphere.Intersect / IntersectP (sphere.go:64-268). world->object = the swap of
// object_to_world (Transform.Inverse, transform.go:175-177).
// Shapes are split into the hit test (t and the object-space hit point) and
// the SurfaceInteraction built from that point, so a closest-hit traversal
// runs the EFloat test once per candidate and builds one interaction at the
// end (see bvh_traverse).

// Sphere.Intersect / IntersectP, hit part (sphere.go:64-131). world->object
// = the swap of object_to_world (Transform.Inverse, transform.go:175-177).
// `ray` is already in object space (shape_hit), oerr/derr its transform errors.
// The EFloat path of Sphere.Intersect up to its bound comparisons
// (sphere.go:64-92): fills rt, or returns false where the reference does.
__device__ inline bool sphere_roots_exact(const pbrt_shape_desc& s, const Ray& ray, V3 oerr, V3 derr, sf_roots& rt,
                                          int& panic) {
    EF ox = ef_new(ray.o.x, oerr.x, panic), oy = ef_new(ray.o.y, oerr.y, panic), oz = ef_new(ray.o.z, oerr.z, panic);
    EF dx = ef_new(ray.d.x, derr.x, panic), dy = ef_new(ray.d.y, derr.y, panic), dz = ef_new(ray.d.z, derr.z, panic);
    EF a = ef_add(ef_add(ef_mul(dx, dx, panic), ef_mul(dy, dy, panic), panic), ef_mul(dz, dz, panic), panic);
    EF b = ef_muls(ef_add(ef_add(ef_mul(dx, ox, panic), ef_mul(dy, oy, panic), panic), ef_mul(dz, oz, panic), panic),
                   2.0, panic);
    EF c0 = ef_add(ef_add(ef_mul(ox, ox, panic), ef_mul(oy, oy, panic), panic), ef_mul(oz, oz, panic), panic);
    EF c = ef_sub(c0, ef_muls(ef_new(s.radius, 0, panic), s.radius, panic), panic);
    EF t0, t1;
    if (!ef_quadratic(a, b, c, t0, t1, panic)) return false;
    if (t0.hi > ray.tmax || t1.lo <= 0) return false;
    rt.t0v = t0.v;
    rt.t1v = t1.v;
    rt.t0lo_le0 = t0.lo <= 0;
    rt.t1hi_gt = t1.hi > ray.tmax;
    return true;
}
// sphere.go:87-131 on the decided comparisons: the root, the refined hit point
// and the partial-sphere clipping
__device__ inline bool sphere_accept(const pbrt_shape_desc& s, const Ray& ray, const sf_roots& rt, double& t_hit,
                                     V3& ph) {
    double tsv = rt.t0v;
    bool used_t1 = false;
    if (rt.t0lo_le0) {
        tsv = rt.t1v;
        used_t1 = true;
        if (rt.t1hi_gt) return false;
    }
    ph = ray.o + muls(ray.d, tsv);
    ph = muls(ph, s.radius / dist(ph, V3{0, 0, 0}));
    if (ph.x == 0.0 && ph.y == 0.0) ph.x = 1e-5 * s.radius;
    if ((s.z_min > -s.radius && ph.z < s.z_min) || (s.z_max < s.radius && ph.z > s.z_max) ||
        phi_beyond(ph.y, ph.x, s.phi_max)) {
        if (used_t1) return false;
        if (rt.t1hi_gt) return false;
        tsv = rt.t1v;
        ph = ray.o + muls(ray.d, tsv);
        ph = muls(ph, s.radius / dist(ph, V3{0, 0, 0}));
        if (ph.x == 0.0 && ph.y == 0.0) ph.x = 1e-5 * s.radius;
        // sphere.go:127 shadows phi (`:=`): the new phi is only tested here
        if ((s.z_min > -s.radius && ph.z < s.z_min) || (s.z_max < s.radius && ph.z > s.z_max) ||
            phi_beyond(ph.y, ph.x, s.phi_max))
            return false;
    }
    t_hit = tsv;
    return true;
}
// Sphere.Intersect / IntersectP, hit part (sphere.go:64-131). world->object
// = the swap of object_to_world (Transform.Inverse, transform.go:175-177).
// `ray` is already in object space (shape_hit), oerr/derr its transform errors.
// Value-first decisions (sphere_filter.h): the reference's
// bound comparisons decided from the EFloat values and a proven radius; the
// intervals are evaluated only when the filter cannot decide (a near-tie with
// TMax or 0, a near-zero divisor, extreme magnitudes).
__device__ inline bool sphere_hit(const pbrt_shape_desc& s, const Ray& ray, V3 oerr, V3 derr, double& t_hit, V3& ph,
                                  int& panic) {
    sf_roots rt;
    const int fr = sphere_roots_filter(ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z, oerr.x, oerr.y, oerr.z,
                                       derr.x, derr.y, derr.z, s.radius, ray.tmax, &rt);
    if (fr == 0) return false;
    if (fr < 0 && !sphere_roots_exact(s, ray, oerr, derr, rt, panic)) return false;
    return sphere_accept(s, ray, rt, t_hit, ph);
}
// Sphere.Intersect, interaction part (sphere.go:133-186); ray in object space.
// Only dpdu, dpdv of the parametric representation feed the outputs.
__device__ inline void sphere_si(const pbrt_shape_desc& s, const Ray& ray, V3 ph, SI& si) {
    double theta = gomath::acos(gomath::clamp(ph.z / s.radius, -1, 1));
    double zr = gomath::sqrt(ph.x * ph.x + ph.y * ph.y);
    double izr = 1.0 / zr;
    double cos_phi = ph.x * izr, sin_phi = ph.y * izr;
    V3 dpdu{-s.phi_max * ph.y, s.phi_max * ph.x, 0};
    double dth = s.theta_max - s.theta_min;
    V3 dpdv = muls(V3{ph.z * cos_phi, ph.z * sin_phi, -s.radius * gomath::sin(theta)}, dth);
    V3 perr = muls(vabs(ph), gomath::gamma(5));
    make_si(si, s.object_to_world.m, s.object_to_world.m_inv, ph, perr, muls(ray.d, -1), dpdu, dpdv, ray.time,
            s.reverse_orientation != s.transform_swaps_handedness);
}

// Disk.Intersect / IntersectP, hit part (disk.go:64-95); `ray` in object space
__device__ inline bool disk_hit(const pbrt_shape_desc& s, const Ray& ray, double& t_hit, V3& ph) {
    if (ray.d.z == 0) return false;
    double ts = (s.height - ray.o.z) / ray.d.z;
    if (ts <= 0 || ts >= ray.tmax) return false;
    ph = ray.o + muls(ray.d, ts);
    double d2 = ph.x * ph.x + ph.y * ph.y;
    if (d2 > s.radius * s.radius || d2 < s.inner_radius * s.inner_radius) return false;
    if (phi_beyond(ph.y, ph.x, s.phi_max)) return false;
    t_hit = ts;
    return true;
}
// Disk.Intersect, interaction part (disk.go:96-110); ray in object space
__device__ inline void disk_si(const pbrt_shape_desc& s, const Ray& ray, V3 ph, SI& si) {
    double d2 = ph.x * ph.x + ph.y * ph.y;
    double rhit = gomath::sqrt(d2);
    V3 dpdu{-s.phi_max * ph.y, s.phi_max * ph.x, 0};
    V3 dpdv = muls(V3{ph.x, ph.y, 0}, (s.radius - s.inner_radius) / rhit);
    ph.z = s.height;
    make_si(si, s.object_to_world.m, s.object_to_world.m_inv, ph, V3{0, 0, 0}, muls(ray.d, -1), dpdu, dpdv, ray.time,
            s.reverse_orientation != s.transform_swaps_handedness);
}

// Both shapes start with the same world->object TransformRay (sphere.go:66,
// disk.go:66), done once here so a wave whose lanes test different shape
// kinds runs it once.
__device__ inline bool shape_hit(const pbrt_shape_desc& s, const Ray& r, double& t_hit, V3& ph, int& panic) {
    V3 oerr, derr;
    const Ray ray = xf_ray(s.object_to_world.m_inv, r, &oerr, &derr);
    if (s.type == PBRT_SHAPE_SPHERE) return sphere_hit(s, ray, oerr, derr, t_hit, ph, panic);
    return disk_hit(s, ray, t_hit, ph);
}
// the interaction at an accepted hit point ph; r in the shape's parent space
// sphere_si / disk_si read only the object-space direction and the time, and
// TransformRay's direction is TransformVector's (transform.go:279-300: the
// origin push leaves it alone), so only the direction is transformed here.
__device__ inline void shape_si(const pbrt_shape_desc& s, const Ray& r, V3 ph, SI& si) {
    const Ray ray{V3{0, 0, 0}, xf_vector(s.object_to_world.m_inv, r.d), r.tmax, r.time};
    if (s.type == PBRT_SHAPE_SPHERE) sphere_si(s, ray, ph, si);
    else disk_si(s, ray, ph, si);
}

// A primitive with a copy of its shape: a leaf test reads one record (one
// dependent memory level) instead of primitive -> shape.
// fast: the value-only TransformRay class (xf_fast) of the primitive's
// world->primitive transform (bits 0-7) and of the shape's world->object
// transform (bits 8-15), set on the host by xf_fast_kind.
struct alignas(16) DevPrim {
    pbrt_shape_desc shape;
    pbrt_transform prim_to_world;   // TransformedPrimitive only
    int32_t kind, material, prim_identity, fast;
};

#if defined(PBRT_XF_FAST)
// The shape test on the exact TransformRay with its errors (the cold path of
// prim_hit_t). Out of line: inlined beside the value-only path it made every
// traversal loop too large to stay in registers (k_chain_ci spilled 320 B/lane).
__device__ __noinline__ bool prim_hit_exact(const DevScene& sc, int pi, const Ray& r, double& t_hit, V3& ph,
                                            int& panic) {
    const DevPrim& p = sc.fprims[pi];
    Ray ray = r;
    if (p.kind == PBRT_PRIM_TRANSFORMED) ray = xf_ray(p.prim_to_world.m_inv, r, nullptr, nullptr);
    return shape_hit(p.shape, ray, t_hit, ph, panic);
}
#endif

// Shape test without the SurfaceInteraction: the hit parameter and point.
// Default: the exact TransformRay with its errors, then the shape's test (the
// sphere's value-first filter, sphere_hit). Experiment builds (-DPBRT_XF_FAST)
// take the object-space ray from xf_fast where it applies: exact,
// but measured slower (the disk tests of rays leaving the floor fail its checks,
// so most waves ran both paths).
__device__ inline bool prim_hit_t(const DevScene& sc, int pi, const Ray& r, double& t_hit, V3& ph, int& panic) {
    const DevPrim& p = sc.fprims[pi];
    const bool xformed = p.kind == PBRT_PRIM_TRANSFORMED;
#ifdef PBRT_XF_FAST   // experiment builds (-DPBRT_XF_FAST): measured slower, DESIGN.md 3.6
    {
        Ray ro = r;
        bool fast = !xformed || xf_fast(p.fast & 0xff, p.prim_to_world.m_inv, ro.o, ro.d);
        fast = fast && xf_fast((p.fast >> 8) & 0xff, p.shape.object_to_world.m_inv, ro.o, ro.d);
        if (fast) {
            if (p.shape.type != PBRT_SHAPE_SPHERE) return disk_hit(p.shape, ro, t_hit, ph);
            sf_roots rt;
            const int fr = sphere_roots_filter(ro.o.x, ro.o.y, ro.o.z, ro.d.x, ro.d.y, ro.d.z, 0, 0, 0, 0, 0, 0,
                                               p.shape.radius, ro.tmax, &rt);
            if (fr == 0) return false;
            if (fr > 0) return sphere_accept(p.shape, ro, rt, t_hit, ph);
        }
    }
    return prim_hit_exact(sc, pi, r, t_hit, ph, panic);
#else
    Ray ray = r;
    if (xformed) ray = xf_ray(p.prim_to_world.m_inv, r, nullptr, nullptr);
    return shape_hit(p.shape, ray, t_hit, ph, panic);
#endif
}

// Mesh of global triangle index g (meshes are few: a linear scan)
__device__ __forceinline__ int tri_mesh(const DevScene& sc, int32_t g) {
    int m = 0;
    while (m + 1 < sc.mesh.n_meshes && sc.mesh.mesh_first[m + 1] <= g) m++;
    return m;
}
// The triangle of leaf slot `slot` hit by r (extension): pbrt-v3
// Triangle::Intersect's interaction part with the default uv (0,0), (1,0),
// (1,1) -- dpdu = dp12 - dp02, dpdv = -dp12 (uv determinant exactly 1) -- and
// go-pbrt's normalized wo; oracle/oracle_render.c tri_si states the same.
// The barycentrics come from re-running the (deterministic) hit test.
__device__ inline void mesh_si(const DevScene& sc, int32_t slot, const Ray& r, SI& si) {
    double v[9], t, b0 = 0, b1 = 0, b2 = 0;
    load_tri(sc.mesh.tris, (uint32_t)slot, v);
    (void)tri_hit(v, r, t, b0, b1, b2);
    const int32_t g = sc.mesh.gid[slot];
    const V3 p0{v[0], v[1], v[2]}, p1{v[3], v[4], v[5]}, p2{v[6], v[7], v[8]};
    const V3 dp02 = p0 - p2, dp12 = p1 - p2;
    V3 dpdu = dp12 - dp02;
    V3 dpdv{-dp12.x, -dp12.y, -dp12.z};
    if (len2(cross(dpdu, dpdv)) == 0) {
        const V3 nn = normalized(cross(p2 - p0, p1 - p0));
        coordinate_system(nn, dpdu, dpdv);
    }
    const V3 p{b0 * p0.x + b1 * p1.x + b2 * p2.x, b0 * p0.y + b1 * p1.y + b2 * p2.y,
               b0 * p0.z + b1 * p1.z + b2 * p2.z};
    const V3 err{gomath::abs(b0 * p0.x) + gomath::abs(b1 * p1.x) + gomath::abs(b2 * p2.x),
                 gomath::abs(b0 * p0.y) + gomath::abs(b1 * p1.y) + gomath::abs(b2 * p2.y),
                 gomath::abs(b0 * p0.z) + gomath::abs(b1 * p1.z) + gomath::abs(b2 * p2.z)};
    V3 n = normalized(cross(dp02, dp12));
    if (sc.mesh.mesh_rev[tri_mesh(sc, g)]) n = V3{-n.x, -n.y, -n.z};
    si.p = p;
    si.perr = muls(err, tri_gamma(7));
    si.n = n;
    si.wo = normalized(V3{-r.d.x, -r.d.y, -r.d.z});
    si.time = r.time;
    si.sn = n;
    si.sdpdu = dpdu;
    si.prim = sc.n_prims + g;
}

// GeometricPrimitive / TransformedPrimitive (primitive.go:42-115): the
// interaction of primitive pi at its accepted hit point ph (shape space).
// pi >= n_prims: leaf slot pi - n_prims of the meshes (mesh_si).
__device__ inline void prim_si(const DevScene& sc, int pi, const Ray& r, V3 ph, SI& si) {
    if (pi >= sc.n_prims) {
        mesh_si(sc, pi - sc.n_prims, r, si);
        return;
    }
    const DevPrim& p = sc.fprims[pi];
    const bool xformed = p.kind == PBRT_PRIM_TRANSFORMED;
    Ray ray = r;   // shape_si reads the direction and the time only
    if (xformed) ray.d = xf_vector(p.prim_to_world.m_inv, r.d);
    shape_si(p.shape, ray, ph, si);
    si.prim = pi;
    if (xformed && !p.prim_identity) transform_si_shared(si, p.prim_to_world.m, p.prim_to_world.m_inv);
}
__device__ inline bool prim_intersect_p(const DevScene& sc, int pi, const Ray& r, int& panic) {
    double t_hit;
    V3 ph;
    return prim_hit_t(sc, pi, r, t_hit, ph, panic);
}

// ------------------------------------------------------------------------ BVH
// BVH node as stored on the device: pbrt_bvh_node widened to 64 bytes so a
// node is fetched with four 16-byte loads issued together (the 56-byte ABI
// layout let the compiler sink each field load behind the previous test,
// one memory round trip per field).
struct alignas(16) DevNode {
    double bmin[3];
    double bmax[3];
    uint32_t offset;     // primitivesOffset (leaf) / secondChildOffset (interior)
    uint32_t nprims_axis;   // nPrimitives | axis << 16
    uint64_t pad;
};
static_assert(sizeof(DevNode) == 64, "DevNode is four 16-byte loads");
struct NodeView {
    double b[6];
    uint32_t offset, n_prims, axis;
};
// BVH nodes staged in LDS by kernels whose scene fits (README / Cornell:
// <= 45 nodes). A file-scope __shared__ array, so every access is a ds_read.
constexpr int kLdsNodes = 64;
__shared__ DevNode g_nodes_lds[kLdsNodes];

__device__ __forceinline__ NodeView load_node(const DevScene& sc, uint32_t i) {
    uint64_t w[7];
    if (sc.use_lds_nodes) {   // uniform
        const DevNode& n = g_nodes_lds[i];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            w[k] = __builtin_bit_cast(uint64_t, n.bmin[k]);
            w[3 + k] = __builtin_bit_cast(uint64_t, n.bmax[k]);
        }
        w[6] = (uint64_t)n.offset | ((uint64_t)n.nprims_axis << 32);
    } else {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(sc.nodes + i);
        const ulonglong2 a = q[0], b = q[1], c = q[2], d = q[3];
        w[0] = a.x; w[1] = a.y; w[2] = b.x; w[3] = b.y; w[4] = c.x; w[5] = c.y; w[6] = d.x;
    }
    NodeView v;
#pragma unroll
    for (int k = 0; k < 6; k++) v.b[k] = __builtin_bit_cast(double, w[k]);
    v.offset = (uint32_t)w[6];
    v.n_prims = (uint32_t)(w[6] >> 32) & 0xFFFFu;
    v.axis = (uint32_t)(w[6] >> 48) & 0xFFu;
    return v;
}
// Bounds3.IntersectP (bounds.go:149-185); (1 + 2*Gamma(3)) == 1 exactly.
// Branch-free: the same comparisons as the reference's early returns, folded
// into one flag (values computed after a failed test are ignored).
__device__ __forceinline__ bool node_hit(const NodeView& nd, const Ray& r, V3 inv, int nx, int ny, int nz) {
    const double robust = 1 + 2 * gomath::gamma(3);
    double tmin = ((nx ? nd.b[3] : nd.b[0]) - r.o.x) * inv.x;
    double tmax = ((nx ? nd.b[0] : nd.b[3]) - r.o.x) * inv.x;
    const double tymin = ((ny ? nd.b[4] : nd.b[1]) - r.o.y) * inv.y;
    double tymax = ((ny ? nd.b[1] : nd.b[4]) - r.o.y) * inv.y;
    tmax *= robust;
    tymax *= robust;
    int hit = (int)!(tmin > tymax) & (int)!(tymin > tmax);
    tmin = tymin > tmin ? tymin : tmin;
    tmax = tymax < tmax ? tymax : tmax;
    const double tzmin = ((nz ? nd.b[5] : nd.b[2]) - r.o.z) * inv.z;
    double tzmax = ((nz ? nd.b[2] : nd.b[5]) - r.o.z) * inv.z;
    tzmax *= robust;
    hit &= (int)!(tmin > tzmax) & (int)!(tzmin > tmax);
    tmin = tzmin > tmin ? tzmin : tmin;
    tmax = tzmax < tmax ? tzmax : tmax;
    return (hit & (int)(tmin < r.tmax) & (int)(tmax > 0)) != 0;
}

// Preorder visit table of the BVH, one per ray-direction octant (built on the
// host, dev_order in render.hip). The reference's traversal (bvh.go:659-765)
// is a depth-first walk whose child order at an interior node depends only on
// the sign of the ray direction along the node's split axis: for a given
// octant it visits nodes in one fixed preorder, skipping the subtree of every
// node whose box test fails. Entry i of an octant's table holds
//   bits  0-14  the node index (pbrt_bvh_node order)
//   bit   15    a hit at this interior node would push past the [64] stack
//               (bvh.go:670: the reference panics there)
//   bits 16-31  the table index that follows the node's subtree (its skip)
constexpr uint32_t kOrdNode = 0x7FFFu, kOrdOverflow = 0x8000u;
// Leaves only, per octant, in that preorder (LDS-staged trees).
__shared__ uint16_t g_leaf_lds[8 * kLdsNodes];
// Leaf culling groups (LDS-staged trees): boxes, and per octant the mask of
// leaf positions (in that octant's leaf preorder) each group covers, plus the
// mask of leaves tested unconditionally.
constexpr int kMaxCullGroups = 16;
__shared__ double g_grp_lds[kMaxCullGroups * 6];
__shared__ uint32_t g_gmask_lds[8 * (kMaxCullGroups + 1)];

// Shared leaf-primitive loop of both walks: tests the leaf's primitives in
// order; returns 1 when an any-hit query is answered, -1 on a panic.
template <bool kAny>
__device__ __forceinline__ int leaf_prims(const DevScene& sc, uint32_t first, uint32_t np, Ray& ray, int& panic,
                                          int& best, V3& best_ph) {
    for (uint32_t k = 0; k < np; k++) {
        double t_hit;
        V3 ph;
        const bool h = prim_hit_t(sc, (int)(first + k), ray, t_hit, ph, panic);
        if (panic) return -1;
        if (h) {
            if (kAny) return 1;
            ray.tmax = t_hit;
            best = (int)(first + k);
            best_ph = ph;
        }
    }
    return 0;
}

// BVH.Intersect (bvh.go:659-712) / IntersectP (:713-765).
//
// Closest hit: each accepted primitive only shrinks TMax; the interaction of
// the LAST accepted one is built once after the walk from its hit point. This
// equals the reference's per-hit SurfaceInteraction: every field is a function
// of that hit point and of the (unchanged) ray, and the shared-interaction
// aliasing of TransformedPrimitive (#20) only ever touches the last one.
// bvh_walk leaves the closest primitive in `best` (-1: none) and its hit point
// in `best_ph`.
//
// LDS-staged trees (<= 64 nodes: README, Cornell) walk only their leaves, in
// the octant's preorder (g_leaf_lds), each box tested with the current TMax.
// A leaf whose culling group's box (the union of its members' boxes, built on
// the host) the ray misses with its initial TMax is skipped: by the same
// monotonicity its own test would fail with any TMax <= the initial one. The
// groups only prune tests that fail; the leaves tested, their order and TMax
// at each test are the reference's.
// This tests exactly the primitives the reference tests, in its order, with
// its TMax. A child's box lies inside its parent's (bounds are unions,
// bvh.go:54-66) and the slab values are monotone in the bounds under
// rounding, so: if the reference rejects an interior node (with the TMax of
// its visit), every leaf below it fails its own test with the smaller or
// equal TMax of its turn; and a leaf that passes implies that all its
// ancestors passed when the reference visited them. Interior nodes therefore
// decide nothing, and a 64-node tree cannot overflow the [64] stack.
//
// Larger trees walk with the reference's [64] stack in LDS (one uint16 column
// per lane, kStride apart), structured "while-while" for 64-lane waves: loop
// A walks interior nodes until the lane reaches a leaf whose box it hits,
// loop B tests that leaf's primitives.
// Experiment builds may force the walk inline into its callers (-DPBRT_WALK_FORCE_INLINE).
#ifdef PBRT_WALK_FORCE_INLINE
#define PBRT_WALK_INLINE __forceinline__
#else
#define PBRT_WALK_INLINE inline
#endif
// kLB: leaf boxes tested per scan iteration (LDS-staged trees).
template <bool kAny, int kStride = kStackStride, int kLB = 4>
__device__ inline bool bvh_walk_analytic(const DevScene& sc, Ray& ray, uint16_t* stack, int& panic, int& best,
                                         V3& best_ph) {
    best = -1;
    const int n = sc.n_nodes;
    if (n == 0) return false;
    V3 inv{1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z};
    const int nx = inv.x < 0, ny = inv.y < 0, nz = inv.z < 0;
    STEP_T(StepTimer tt; tt.start();)
    if (sc.use_lds_nodes) {   // uniform: n <= kLdsNodes
        (void)stack;
        const int nl = sc.n_leaves;
        const int oct = nx | (ny << 1) | (nz << 2);
        const uint16_t* leaves = g_leaf_lds + oct * kLdsNodes;
        const int ng = sc.n_groups;
        if (ng > 0) {   // uniform; the host groups trees of <= 32 leaves only
            // candidate leaves: the unconditional ones, plus the members of
            // every group whose box the ray enters (initial TMax)
            const uint32_t* gm = g_gmask_lds + oct * (kMaxCullGroups + 1);
            uint32_t cand = gm[ng];
            for (int g = 0; g < ng; g++) {
                NodeView gv;
#pragma unroll
                for (int k = 0; k < 6; k++) gv.b[k] = g_grp_lds[g * 6 + k];
                if (node_hit(gv, ray, inv, nx, ny, nz)) cand |= gm[g];
            }
            for (;;) {
                // A: the next candidate in the octant's leaf preorder whose box the
                // ray enters; kLB per iteration (independent loads and slab tests;
                // a later result is used only if the earlier ones miss, same TMax)
                bool leaf = false;
                uint32_t first = 0, np = 0;
                while (cand) {
                    int js[kLB];
                    uint32_t rest[kLB];   // rest[q]: cand without its q + 1 lowest bits
                    uint32_t r = cand;
#pragma unroll
                    for (int q = 0; q < kLB; q++) {
                        js[q] = r ? __builtin_ctz(r) : js[0];
                        r = r & (r - 1);
                        rest[q] = r;
                    }
                    NodeView nv[kLB];
#pragma unroll
                    for (int q = 0; q < kLB; q++) nv[q] = load_node(sc, leaves[js[q]]);
                    int qh = -1;
#pragma unroll
                    for (int q = kLB - 1; q >= 0; q--)
                        if ((q == 0 || js[q] != js[0]) && node_hit(nv[q], ray, inv, nx, ny, nz)) qh = q;
                    if (qh >= 0) {
                        leaf = true;
#pragma unroll
                        for (int q = 0; q < kLB; q++)
                            if (q == qh) {
                                first = nv[q].offset;
                                np = nv[q].n_prims;
                                cand = rest[q];
                            }
                        break;
                    }
                    cand = rest[kLB - 1];
                }
                STEP_T(if (!kAny) tt.mark(5);)
                if (!leaf) break;
                // B: its primitives
                const int r = leaf_prims<kAny>(sc, first, np, ray, panic, best, best_ph);
                if (r < 0) return kAny ? false : best >= 0;
                if (kAny && r > 0) return true;
                STEP_T(if (!kAny) tt.mark(6);)
            }
            return best >= 0;
        }
        int j = 0;
        for (;;) {
            // A: the next leaf in the octant's preorder whose box the ray enters,
            // kLB leaves per iteration: independent loads and slab tests overlap;
            // a later result is used only if the earlier leaves miss (same TMax)
            bool leaf = false;
            uint32_t first = 0, np = 0;
            while (j < nl) {
                NodeView nv[kLB];
#pragma unroll
                for (int q = 0; q < kLB; q++) nv[q] = load_node(sc, leaves[j + q < nl ? j + q : j]);
                int qh = -1;
#pragma unroll
                for (int q = kLB - 1; q >= 0; q--)
                    if ((q == 0 || j + q < nl) && node_hit(nv[q], ray, inv, nx, ny, nz)) qh = q;
                if (qh >= 0) {
                    leaf = true;
#pragma unroll
                    for (int q = 0; q < kLB; q++)
                        if (q == qh) {
                            first = nv[q].offset;
                            np = nv[q].n_prims;
                        }
                    j += qh + 1;
                    break;
                }
                j += kLB;
            }
            STEP_T(if (!kAny) tt.mark(5);)
            if (!leaf) break;
            // B: its primitives
            const int r = leaf_prims<kAny>(sc, first, np, ray, panic, best, best_ph);
            if (r < 0) return kAny ? false : best >= 0;
            if (kAny && r > 0) return true;
            STEP_T(if (!kAny) tt.mark(6);)
        }
        return best >= 0;
    }
    const uint32_t negmask = (uint32_t)nx | ((uint32_t)ny << 1) | ((uint32_t)nz << 2);
    uint32_t to_visit = 0, cur = 0;
    for (;;) {
        // A: interior nodes
        bool done = false;
        for (;;) {
            const NodeView nd = load_node(sc, cur);
            if (node_hit(nd, ray, inv, nx, ny, nz)) {
                if (nd.n_prims > 0) break;
                if (to_visit >= 64) {
                    panic = PBRT_PANIC_BVH_STACK;
                    return kAny ? false : best >= 0;
                }
                uint32_t far_node, near_node;
                if ((negmask >> nd.axis) & 1u) { far_node = cur + 1; near_node = nd.offset; }
                else { far_node = nd.offset; near_node = cur + 1; }
                stack[(to_visit++) * kStride] = (uint16_t)far_node;
                cur = near_node;
            } else {
                if (to_visit == 0) {
                    done = true;
                    break;
                }
                cur = stack[(--to_visit) * kStride];
            }
        }
        STEP_T(if (!kAny) tt.mark(5);)
        if (done) break;
        // B: the leaf's primitives
        const NodeView nd = load_node(sc, cur);
        const int r = leaf_prims<kAny>(sc, nd.offset, nd.n_prims, ray, panic, best, best_ph);
        if (r < 0) return kAny ? false : best >= 0;
        if (kAny && r > 0) return true;
        STEP_T(if (!kAny) tt.mark(6);)
        if (to_visit == 0) break;
        cur = stack[(--to_visit) * kStride];
    }
    STEP_T(if (!kAny) tt.mark(6);)
    return best >= 0;
}

// The scene's aggregate: the reference BVH over the analytic primitives, then
// the triangle meshes (extension) with the TMax it left; a triangle wins only
// with a strictly smaller t, so an analytic primitive keeps a tie. A mesh hit
// is reported as best = n_prims + its leaf slot.
template <bool kAny, int kStride = kStackStride, int kLB = 4, bool kMeshOnly = false>
__device__ PBRT_WALK_INLINE bool bvh_walk(const DevScene& sc, Ray& ray, uint16_t* stack, int& panic, int& best, V3& best_ph) {
    // kMeshOnly: the scene has triangle meshes and no other primitive (host:
    // n_prims == 0), so the analytic walk -- whose sphere / disk code sets the
    // register peak of every traversal kernel -- is compiled out
    bool hit = false;
    if (kMeshOnly) best = -1;
    else hit = bvh_walk_analytic<kAny, kStride, kLB>(sc, ray, stack, panic, best, best_ph);
    if (sc.mesh.n_nodes == 0 || panic || (kAny && hit)) return hit;
    double tm = ray.tmax;
    int32_t slot = -1, gid = -1;
    // kernels over scenes with analytic primitives carry the lean wide walk, so
    // that it does not raise their register peak (k_paths_ci: 204 VGPRs; 230
    // and 252 B of scratch with the four-box walk)
    if (!(kMeshOnly ? mesh_walk<kAny>(sc.mesh, ray, tm, slot, gid) : mesh_walk_mixed<kAny>(sc.mesh, ray, tm, slot, gid)))
        return hit;
    if (kAny) return true;
    ray.tmax = tm;
    best = sc.n_prims + slot;
    return true;
}

template <bool kAny, int kLB = 4, bool kMeshOnly = false>
__device__ inline bool bvh_traverse(const DevScene& sc, Ray& ray, SI* si, uint16_t* stack, int& panic) {
    int best;
    V3 best_ph{0, 0, 0};
    const bool hit = bvh_walk<kAny, kStackStride, kLB, kMeshOnly>(sc, ray, stack, panic, best, best_ph);
    STEP_T(StepTimer tt; tt.start();)
    if (!kAny && best >= 0) prim_si(sc, best, ray, best_ph, *si);
    STEP_T(if (!kAny) tt.mark(7);)
    return hit;
}

// ------------------------------------------- dense closest hit (k_chain_ci)
// The closest-hit walk of an LDS-staged tree with culling groups and one
// primitive per leaf, for a whole wave at once. The per-lane walk
// (bvh_walk_analytic) runs a wave's leaf tests one per lane per iteration, so
// a wave pays for its lane with the most candidate leaves (the leaf tests are
// 89% of a closest-hit traversal, profiles/r03/phase_steptime_B.txt). Here:
//  1. each lane finds its candidate leaves: the culling groups' members whose
//     own box it enters with its initial TMax (a superset of what it will test);
//  2. the wave computes every (lane, candidate) primitive test, 64 pairs per
//     round, lane-dense: the part of Sphere/Disk.Intersect that does not read
//     TMax (EFloat quadratic, clipping of both roots, its panics);
//  3. each lane replays its own candidates in its octant's leaf preorder: the
//     leaf box with the current TMax (as the reference tests it), then the
//     TMax comparisons of Intersect (sphere.go:103-131, disk.go:72-95).
// Every test the reference runs is decided by the same values and comparisons
// in the same order; tests it never runs (a box that fails at the current TMax)
// only had their TMax-free part computed, and their panics are ignored. The
// result (best, TMax, hit point) is the per-lane walk's.
struct DensePair {
    double a, b, c, d, e, f;   // sphere: t0 lo/v/hi, t1 lo/v/hi; disk: a = t
    uint32_t flags;            // kDp*
    int32_t panic;
};
constexpr uint32_t kDpMiss = 1, kDpClip0 = 2, kDpClip1 = 4, kDpDisk = 8;
constexpr int kDenseScratch = 64 * (int)sizeof(DensePair) + 2 * 64 * 4;   // LDS bytes per wave
__device__ __forceinline__ void dense_wave_sync() {   // the wave's LDS writes are visible to the wave
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// the k-th set bit of m (k < popcount(m))
__device__ __forceinline__ int nth_bit(uint32_t m, int k) {
    for (int i = 0; i < k; i++) m &= m - 1;
    return __builtin_ctz(m);
}
__device__ __forceinline__ bool sphere_clipped(const pbrt_shape_desc& s, V3 ph) {
    return (s.z_min > -s.radius && ph.z < s.z_min) || (s.z_max < s.radius && ph.z > s.z_max) ||
           phi_beyond(ph.y, ph.x, s.phi_max);
}
__device__ __forceinline__ V3 sphere_point(const pbrt_shape_desc& s, const Ray& ray, double t) {   // sphere.go:111-114
    V3 ph = ray.o + muls(ray.d, t);
    ph = muls(ph, s.radius / dist(ph, V3{0, 0, 0}));
    if (ph.x == 0.0 && ph.y == 0.0) ph.x = 1e-5 * s.radius;
    return ph;
}
// the TMax-free part of prim pi's test against world ray r
__device__ inline void dense_pair(const DevScene& sc, int pi, const Ray& r, DensePair& o) {
    const DevPrim& p = sc.fprims[pi];
    Ray ray = r;
    if (p.kind == PBRT_PRIM_TRANSFORMED) ray = xf_ray(p.prim_to_world.m_inv, r, nullptr, nullptr);
    const pbrt_shape_desc& s = p.shape;
    V3 oerr, derr;
    const Ray ro = xf_ray(s.object_to_world.m_inv, ray, &oerr, &derr);
    o.flags = 0;
    o.panic = 0;
    o.a = o.b = o.c = o.d = o.e = o.f = 0;
    if (s.type != PBRT_SHAPE_SPHERE) {   // disk.go:72-95 without the TMax test
        o.flags = kDpDisk;
        if (ro.d.z == 0) {
            o.flags |= kDpMiss;
            return;
        }
        const double ts = (s.height - ro.o.z) / ro.d.z;
        o.a = ts;
        const V3 ph = ro.o + muls(ro.d, ts);
        const double d2 = ph.x * ph.x + ph.y * ph.y;
        if (d2 > s.radius * s.radius || d2 < s.inner_radius * s.inner_radius || phi_beyond(ph.y, ph.x, s.phi_max))
            o.flags |= kDpMiss;
        return;
    }
    // sphere_hit up to its first TMax comparison
    {
        const double av = (ro.d.x * ro.d.x + ro.d.y * ro.d.y) + ro.d.z * ro.d.z;
        const double bv = ((ro.d.x * ro.o.x + ro.d.y * ro.o.y) + ro.d.z * ro.o.z) * 2.0;
        const double cv = ((ro.o.x * ro.o.x + ro.o.y * ro.o.y) + ro.o.z * ro.o.z) - s.radius * s.radius;
        const double disc = bv * bv - 4. * av * cv;
        const double big = 1e100;
        const bool moderate =
            gomath::abs(ro.o.x) < big && gomath::abs(ro.o.y) < big && gomath::abs(ro.o.z) < big &&
            gomath::abs(ro.d.x) < big && gomath::abs(ro.d.y) < big && gomath::abs(ro.d.z) < big &&
            gomath::abs(oerr.x) < big && gomath::abs(oerr.y) < big && gomath::abs(oerr.z) < big &&
            gomath::abs(derr.x) < big && gomath::abs(derr.y) < big && gomath::abs(derr.z) < big &&
            gomath::abs(s.radius) < big;
#ifndef PBRT_NO_EARLY_MISS
        if (disc < 0 && moderate) {
            o.flags = kDpMiss;
            return;
        }
#endif
    }
    int panic = 0;
    EF ox = ef_new(ro.o.x, oerr.x, panic), oy = ef_new(ro.o.y, oerr.y, panic), oz = ef_new(ro.o.z, oerr.z, panic);
    EF dx = ef_new(ro.d.x, derr.x, panic), dy = ef_new(ro.d.y, derr.y, panic), dz = ef_new(ro.d.z, derr.z, panic);
    EF a = ef_add(ef_add(ef_mul(dx, dx, panic), ef_mul(dy, dy, panic), panic), ef_mul(dz, dz, panic), panic);
    EF b = ef_muls(ef_add(ef_add(ef_mul(dx, ox, panic), ef_mul(dy, oy, panic), panic), ef_mul(dz, oz, panic), panic),
                   2.0, panic);
    EF c0 = ef_add(ef_add(ef_mul(ox, ox, panic), ef_mul(oy, oy, panic), panic), ef_mul(oz, oz, panic), panic);
    EF c = ef_sub(c0, ef_muls(ef_new(s.radius, 0, panic), s.radius, panic), panic);
    EF t0, t1;
    const bool q = ef_quadratic(a, b, c, t0, t1, panic);
    o.panic = panic;
    if (panic) return;
    if (!q) {
        o.flags = kDpMiss;
        return;
    }
    o.a = t0.lo; o.b = t0.v; o.c = t0.hi;
    o.d = t1.lo; o.e = t1.v; o.f = t1.hi;
    if (s.z_min > -s.radius || s.z_max < s.radius || s.phi_max < 2 * gomath::kPi) {   // a partial sphere
        if (sphere_clipped(s, sphere_point(s, ro, t0.v))) o.flags |= kDpClip0;
        if (sphere_clipped(s, sphere_point(s, ro, t1.v))) o.flags |= kDpClip1;
    }
}
// sphere.go:103-131 / disk.go:72-74 given the TMax-free part: hit and its t
__device__ __forceinline__ bool dense_accept(const DensePair& r, double tmax, double& t) {
    if (r.flags & kDpMiss) return false;
    if (r.flags & kDpDisk) {
        if (r.a <= 0 || r.a >= tmax) return false;
        t = r.a;
        return true;
    }
    if (r.c > tmax || r.d <= 0) return false;   // t0.hi > tMax || t1.lo <= 0
    bool used_t1 = false;
    double lo = r.a, hi = r.c, v = r.b;
    if (lo <= 0) {
        used_t1 = true;
        lo = r.d; v = r.e; hi = r.f;
        if (hi > tmax) return false;
    }
    if (used_t1 ? (r.flags & kDpClip1) : (r.flags & kDpClip0)) {
        if (used_t1) return false;
        if (r.f > tmax) return false;
        if (r.flags & kDpClip1) return false;
        v = r.e;
    }
    (void)lo;
    t = v;
    return true;
}
// the object-space hit point of prim pi at t (what sphere_hit / disk_hit leave in ph)
__device__ inline V3 dense_hit_point(const DevScene& sc, int pi, const Ray& r, double t) {
    const DevPrim& p = sc.fprims[pi];
    Ray ray = r;
    if (p.kind == PBRT_PRIM_TRANSFORMED) ray = xf_ray(p.prim_to_world.m_inv, r, nullptr, nullptr);
    const Ray ro = xf_ray(p.shape.object_to_world.m_inv, ray, nullptr, nullptr);
    if (p.shape.type == PBRT_SHAPE_SPHERE) return sphere_point(p.shape, ro, t);
    return ro.o + muls(ro.d, t);
}
// Whole-wave closest hit (see above). Every lane of the wave calls it (active:
// the lane has a ray); scratch: kDenseScratch bytes of LDS for this wave.
// Preconditions (uniform, checked by the caller): LDS-staged nodes, culling
// groups, one primitive per leaf, no triangle meshes.
__device__ inline bool bvh_walk_dense(const DevScene& sc, Ray& ray, bool active, int& panic, int& best, V3& best_ph,
                                      unsigned char* scratch) {
    DensePair* res = (DensePair*)scratch;
    int* incl = (int*)(scratch + 64 * sizeof(DensePair));
    uint32_t* masks = (uint32_t*)(incl + 64);
    const int lane = threadIdx.x & 63;
    best = -1;
    const V3 inv{1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z};
    const int nx = inv.x < 0, ny = inv.y < 0, nz = inv.z < 0;
    const int oct = nx | (ny << 1) | (nz << 2);
    const uint16_t* leaves = g_leaf_lds + oct * kLdsNodes;
    const int ng = sc.n_groups;
    uint32_t m = 0;
    if (active) {
        const uint32_t* gm = g_gmask_lds + oct * (kMaxCullGroups + 1);
        uint32_t cand = gm[ng];
        for (int g = 0; g < ng; g++) {
            NodeView gv;
#pragma unroll
            for (int k = 0; k < 6; k++) gv.b[k] = g_grp_lds[g * 6 + k];
            if (node_hit(gv, ray, inv, nx, ny, nz)) cand |= gm[g];
        }
        while (cand) {   // each candidate leaf's own box with the initial TMax
            const int j = __builtin_ctz(cand);
            cand &= cand - 1;
            if (node_hit(load_node(sc, leaves[j]), ray, inv, nx, ny, nz)) m |= 1u << j;
        }
    }
    const int n = __builtin_popcount(m);
    int S = n;   // inclusive prefix sum of the lanes' pair counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(S, o);
        if (lane >= o) S += v;
    }
    const int T = __shfl(S, 63);
    const int S0 = S - n;
    incl[lane] = S;
    masks[lane] = m;
    dense_wave_sync();
    double tmax = ray.tmax;
    bool live = active;
    uint32_t rem = m;   // my candidates not replayed yet (positions in my leaf preorder)
    for (int base = 0; base < T; base += 64) {
        // 2. pair base + lane: its owner lane (the first whose inclusive sum exceeds it)
        const int p = base + lane;
        int own = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)   // own = #{l : incl[l] <= p} (incl is non-decreasing)
            if (incl[own + step - 1] <= p) own += step;
        const int ownc = own > 63 ? 63 : own;
        Ray r;
        r.o.x = __shfl(ray.o.x, ownc); r.o.y = __shfl(ray.o.y, ownc); r.o.z = __shfl(ray.o.z, ownc);
        r.d.x = __shfl(ray.d.x, ownc); r.d.y = __shfl(ray.d.y, ownc); r.d.z = __shfl(ray.d.z, ownc);
        r.tmax = kInf;
        r.time = 0;
        const int ooct = __shfl(oct, ownc);
        if (p < T) {
            const int k = p - (incl[ownc] - __builtin_popcount(masks[ownc]));
            const int j = nth_bit(masks[ownc], k);
            const int pi = (int)load_node(sc, g_leaf_lds[ooct * kLdsNodes + j]).offset;
            dense_pair(sc, pi, r, res[lane]);
        }
        dense_wave_sync();
        // 3. my pairs of this round, in my leaf preorder
        const int lo = S0 > base ? S0 : base, hi = S < base + 64 ? S : base + 64;
        for (int q = lo; live && q < hi; q++) {
            const int j = __builtin_ctz(rem);
            rem &= rem - 1;
            const NodeView nv = load_node(sc, leaves[j]);
            Ray rt = ray;
            rt.tmax = tmax;
            if (!node_hit(nv, rt, inv, nx, ny, nz)) continue;   // the reference does not test this leaf
            const DensePair& rr = res[q - base];
            if (rr.panic) {
                panic = rr.panic;
                live = false;
                break;
            }
            double t;
            if (dense_accept(rr, tmax, t)) {
                tmax = t;
                best = (int)nv.offset;
            }
        }
        dense_wave_sync();   // res is rewritten by the next round
    }
    ray.tmax = tmax;
    if (best >= 0) best_ph = dense_hit_point(sc, best, ray, tmax);
    return best >= 0;
}

// ----------------------------------------------------------------- material
constexpr int BXDF_REFLECTION = 1, BXDF_DIFFUSE = 4, BXDF_SPECULAR = 16, BXDF_ALL = 31;
constexpr int LAMBERT_TYPE = BXDF_REFLECTION | BXDF_DIFFUSE;

struct BSDF {
    V3 ns, ng, ss, ts;
    Spec r;
    int n_bxdfs;   // 0 or 1 (LambertianReflection)
};
__device__ __forceinline__ double inv_pi() { return 1.0 / gomath::kPi; }   // pkg/math InvPi

// MatteMaterial.ComputeScatteringFunctions (matte.go:21-37) + NewBSDF
// (reflection.go:128-140) + Checkerboard2D/PlanarMapping2D (checkerboard.go:30-40)
__device__ inline int compute_bsdf(const DevScene& sc, const SI& si, BSDF& b) {
    const pbrt_material_desc& m =
        sc.materials[si.prim < sc.n_prims ? sc.prims[si.prim].material
                                          : sc.mesh.mesh_mat[tri_mesh(sc, si.prim - sc.n_prims)]];
    b.ns = si.sn;
    b.ng = si.n;
    b.ss = normalized(si.sdpdu);
    b.ts = cross(b.ns, b.ss);
    b.n_bxdfs = 0;
    Spec r;
    if (m.kd_type == PBRT_TEX_CHECKERBOARD2D) {
        double s = m.ds + dot(si.p, load3(m.vs));
        double t = m.dt + dot(si.p, load3(m.vt));
        int64_t k = gomath::to_int(gomath::floor(s) + gomath::floor(t));
        r = (k % 2 == 0) ? spec3(m.tex1) : spec3(m.tex2);
    } else {
        r = spec3(m.kd);
    }
    r.r = gomath::clamp(r.r, 0, kInf);
    r.g = gomath::clamp(r.g, 0, kInf);
    r.b = gomath::clamp(r.b, 0, kInf);
    double sig = gomath::clamp(m.sigma, 0, 90);
    if (!is_black(r)) {
        if (sig != 0) return -1;   // OrenNayar: off the hot path (unsupported)
        b.n_bxdfs = 1;
        b.r = r;
    }
    return 0;
}
__device__ __forceinline__ V3 w2l(const BSDF& b, V3 v) { return V3{dot(v, b.ss), dot(v, b.ts), dot(v, b.ns)}; }
// BSDF.F (reflection.go:169-186)
__device__ inline Spec bsdf_f(const BSDF& b, V3 woW, V3 wiW) {
    V3 wo = w2l(b, woW);
    if (wo.z == 0.0) return spec(0);
    bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    Spec f = spec(0);
    if (b.n_bxdfs && reflect) f = f + smuls(b.r, inv_pi());
    return f;
}
__device__ __forceinline__ double lambert_pdf(V3 wo, V3 wi) {   // reflection.go:343-348
    return (wo.z * wi.z > 0) ? gomath::abs(wi.z) * inv_pi() : 0;
}
// BSDF.Pdf (reflection.go:255-278)
__device__ inline double bsdf_pdf(const BSDF& b, V3 woW, V3 wiW) {
    if (b.n_bxdfs == 0) return 0;
    V3 wo = w2l(b, woW);
    V3 wi = w2l(b, wiW);
    if (wo.z == 0) return 0;
    double pdf = 0 + lambert_pdf(wo, wi);
    return pdf / 1.0;
}
// sampling.go:173-198
__device__ inline V2 concentric_sample_disk(V2 u) {
    V2 uo{u.x * 2.0 - 1, u.y * 2.0 - 1};
    if (uo.x == 0 && uo.y == 0) return V2{0, 0};
    double theta, r;
    if (gomath::abs(uo.x) > gomath::abs(uo.y)) {
        r = uo.x;
        theta = (gomath::kPi / 4.0) * (uo.y / uo.x);
    } else {
        r = uo.y;
        theta = (gomath::kPi / 2.0) - (gomath::kPi / 4.0) * (uo.x / uo.y);
    }
    return V2{gomath::cos(theta) * r, gomath::sin(theta) * r};
}
// BSDF.SampleF (reflection.go:188-253) returning the LOCAL-frame wi (#7)
__device__ inline Spec bsdf_sample_f(const BSDF& b, V3 woW, V2 u, V3& wi, double& pdf) {
    wi = V3{0, 0, 0};
    pdf = 0;
    if (b.n_bxdfs == 0) return spec(0);
    double comp = gomath::min(gomath::floor(u.x * 1.0), 1.0 - 1);
    V2 ur{gomath::min(u.x * 1.0 - comp, gomath::kOneMinusEpsilon), u.y};
    V3 wo = w2l(b, woW);
    if (wo.z == 0.0) return spec(0);
    V2 d = concentric_sample_disk(ur);   // CosineSampleHemisphere (sampling.go:194-198)
    V3 w{d.x, d.y, gomath::sqrt(gomath::max(0.0, 1.0 - d.x * d.x - d.y * d.y))};
    if (wo.z < 0) w.z *= -1;
    double p = lambert_pdf(wo, w);
    Spec f = smuls(b.r, inv_pi());
    if (p == 0.0) return spec(0);
    wi = w;
    pdf = p;
    return f;
}

// --------------------------------------------- Mirror and smooth Glass (serial kernel)
// The BSDF of a Mirror (mirror.go:21-32) or Glass (glass.go:28-75) material. Its
// single BxDF has F = 0 and Pdf = 0 (reflection.go:486-488, 534-536, 553-555,
// 572-574), so light sampling sees it exactly as a BSDF without components: the
// shared estimate_direct/bsdf_f/bsdf_pdf run on `b` with n_bxdfs = 0. Only
// sampling (and the Path.Li bookkeeping) needs the kind.
constexpr int BXDF_TRANSMISSION = 2, BXDF_GLOSSY = 8;
constexpr int MF_REFL_TYPE = BXDF_REFLECTION | BXDF_GLOSSY, MF_TRANS_TYPE = BXDF_TRANSMISSION | BXDF_GLOSSY;
// SPEC_PAIR: smooth glass under DirectLighting (allowMultipleLobes false,
// directlighting.go:76): SpecularReflection(R, FresnelDielectric(1, eta)) if R
// is not black, then SpecularTransmission(T, 1, eta, Radiance) if T is not
// (glass.go:58-72); mf_r / mf_t say which exist. Both F and Pdf are 0.
enum { BXDF_KIND_LAMBERT = 0, BXDF_KIND_SPEC_REFL = 1, BXDF_KIND_FRESNEL_SPEC = 2, BXDF_KIND_MICROFACET = 3,
       BXDF_KIND_OREN_NAYAR = 4, BXDF_KIND_SPEC_PAIR = 5 };
struct BSDFX {
    int kind;       // BXDF_KIND_*; LAMBERT: `b` is the whole BSDF
    int n;          // number of BxDFs of that kind (MICROFACET: mf_r + mf_t)
    int mf_r, mf_t; // rough glass: MicrofacetReflection, MicrofacetTransmission
    Spec r, t;
    double eta;     // NewBSDF(si, eta)
    double ax, ay;  // TrowbridgeReitz alphas (remapRoughness false); OrenNayar A, B
};
// NumComponents(BSDFAll &^ BSDFSpecular) > 0: SpecularReflection is typed
// Reflection|Diffuse (reflection.go:538-544), FresnelSpecular is specular
__device__ __forceinline__ bool bsdfx_nonspecular(const BSDF& b, const BSDFX& x) {
    return x.kind == BXDF_KIND_LAMBERT ? b.n_bxdfs > 0 : (x.kind != BXDF_KIND_FRESNEL_SPEC && x.n > 0);
}
// multi_lobes: ComputeScatteringFunctions' allowMultipleLobes (interaction.go:217-223),
// true for Path.Li (path.go:74), false for DirectLighting.Li (directlighting.go:76)
__device__ inline int compute_bsdf_x(const DevScene& sc, const SI& si, BSDF& b, BSDFX& x, bool multi_lobes = true) {
    const pbrt_material_desc& m =
        sc.materials[si.prim < sc.n_prims ? sc.prims[si.prim].material
                                          : sc.mesh.mesh_mat[tri_mesh(sc, si.prim - sc.n_prims)]];
    x.kind = BXDF_KIND_LAMBERT;
    x.n = x.mf_r = x.mf_t = 0;
    x.eta = 1.0;
    if (m.type == PBRT_MAT_MATTE) {
        const double sig = gomath::clamp(m.sigma, 0, 90);
        if (sig == 0) return compute_bsdf(sc, si, b);
        // OrenNayar (matte.go:30-35, NewOrenNayar reflection.go:616-625; B's
        // sigma2 * 0.09 kept): sampled and weighted like a Lambertian, its F
        // differs, so it carries its own kind with b.r = Kd
        b.ns = si.sn;
        b.ng = si.n;
        b.ss = normalized(si.sdpdu);
        b.ts = cross(b.ns, b.ss);
        b.n_bxdfs = 0;
        Spec r;
        if (m.kd_type == PBRT_TEX_CHECKERBOARD2D) {
            double s = m.ds + dot(si.p, load3(m.vs));
            double t = m.dt + dot(si.p, load3(m.vt));
            int64_t k = gomath::to_int(gomath::floor(s) + gomath::floor(t));
            r = (k % 2 == 0) ? spec3(m.tex1) : spec3(m.tex2);
        } else {
            r = spec3(m.kd);
        }
        r.r = gomath::clamp(r.r, 0, kInf);
        r.g = gomath::clamp(r.g, 0, kInf);
        r.b = gomath::clamp(r.b, 0, kInf);
        x.kind = BXDF_KIND_OREN_NAYAR;
        x.r = r;
        x.n = is_black(r) ? 0 : 1;
        const double sr = gomath::radians(sig), s2 = sr * sr;
        x.ax = 1.0 - (s2 / (2.0 * (s2 + 0.33)));
        x.ay = 0.45 * s2 / (s2 * 0.09);
        return 0;
    }
    b.ns = si.sn;
    b.ng = si.n;
    b.ss = normalized(si.sdpdu);
    b.ts = cross(b.ns, b.ss);
    b.n_bxdfs = 0;
    if (m.type == PBRT_MAT_MIRROR) {
        Spec r = spec3(m.kr);
        r.r = gomath::clamp(r.r, 0, kInf);
        r.g = gomath::clamp(r.g, 0, kInf);
        r.b = gomath::clamp(r.b, 0, kInf);
        x.kind = BXDF_KIND_SPEC_REFL;
        x.n = is_black(r) ? 0 : 1;
        x.r = r;
        return 0;
    }
    Spec R = spec3(m.kr), T = spec3(m.kt);
    R.r = gomath::clamp(R.r, 0, 1); R.g = gomath::clamp(R.g, 0, 1); R.b = gomath::clamp(R.b, 0, 1);
    T.r = gomath::clamp(T.r, 0, 1); T.g = gomath::clamp(T.g, 0, 1); T.b = gomath::clamp(T.b, 0, 1);
    x.kind = BXDF_KIND_FRESNEL_SPEC;
    x.eta = m.eta;
    x.r = R;
    x.t = T;
    if (is_black(R) && is_black(T)) return 0;
    if (!(m.u_roughness == 0 && m.v_roughness == 0)) {   // glass.go:49-73
        x.kind = BXDF_KIND_MICROFACET;
        x.ax = m.u_roughness;
        x.ay = m.v_roughness;
        x.mf_r = is_black(R) ? 0 : 1;
        x.mf_t = is_black(T) ? 0 : 1;
        x.n = x.mf_r + x.mf_t;
        return 0;
    }
    if (!multi_lobes) {
        x.kind = BXDF_KIND_SPEC_PAIR;
        x.mf_r = is_black(R) ? 0 : 1;
        x.mf_t = is_black(T) ? 0 : 1;
        x.n = x.mf_r + x.mf_t;
        return 0;
    }
    x.n = 1;
    return 0;
}
// FrDielectric (reflection.go:21-42)
__device__ inline double fr_dielectric(double cos_i, double eta_i, double eta_t) {
    cos_i = gomath::clamp(cos_i, -1, 1);
    if (!(cos_i > 0)) {
        const double tmp = eta_i;
        eta_i = eta_t;
        eta_t = tmp;
        cos_i = gomath::abs(cos_i);
    }
    const double sin_i = gomath::sqrt(gomath::max(0.0, 1 - cos_i * cos_i));
    const double sin_t = eta_i / eta_t * sin_i;
    if (sin_t >= 1) return 1;
    const double cos_t = gomath::sqrt(gomath::max(0.0, 1 - sin_t * sin_t));
    const double rparl = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    const double rperp = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (rparl * rparl + rperp * rperp) / 2;
}
// TrowbridgeReitz (microfacet.go:36-84, 117-124; sampleVisibleArea true) and
// the trig helpers (reflection.go:48-100); D's e keeps the reference's
// alphaX*alphaY under Cos2Phi
__device__ inline double cos2_theta(V3 w) { return w.z * w.z; }
__device__ inline double sin2_theta(V3 w) { return gomath::max(0.0, 1 - cos2_theta(w)); }
__device__ inline double sin_theta(V3 w) { return gomath::sqrt(sin2_theta(w)); }
__device__ inline double cos_phi(V3 w) {
    const double st = sin_theta(w);
    return st == 0 ? 1 : gomath::clamp(w.x / st, -1, 1);
}
__device__ inline double sin_phi(V3 w) {
    const double st = sin_theta(w);
    return st == 0 ? 0 : gomath::clamp(w.y / st, -1, 1);
}
__device__ inline double tr_d(const BSDFX& x, V3 wh) {
    const double t2 = sin2_theta(wh) / cos2_theta(wh);
    if (gomath::is_inf(t2)) return 0;
    const double c4 = cos2_theta(wh) * cos2_theta(wh);
    const double cp = cos_phi(wh), sp = sin_phi(wh);
    const double e = (cp * cp / (x.ax * x.ay) + sp * sp / (x.ay * x.ay)) * t2;
    return 1 / (gomath::kPi * x.ax * x.ay * c4 * (1 + e) * (1 + e));
}
__device__ inline double tr_lambda(const BSDFX& x, V3 w) {
    const double at = gomath::abs(sin_theta(w) / w.z);
    if (gomath::is_inf(at)) return 0;
    const double cp = cos_phi(w), sp = sin_phi(w);
    const double alpha = gomath::sqrt(cp * cp * x.ax * x.ax + sp * sp * x.ay * x.ay);
    const double a2t2 = (alpha * at) * (alpha * at);
    return (-1 + gomath::sqrt(1.0 + a2t2)) / 2;
}
__device__ inline double tr_g(const BSDFX& x, V3 wo, V3 wi) { return 1 / (1 + tr_lambda(x, wo) + tr_lambda(x, wi)); }
__device__ inline double tr_pdf(const BSDFX& x, V3 wo, V3 wh) {   // microfacet.go:26-32
    return tr_d(x, wh) * (1 / (1 + tr_lambda(x, wo))) * absdot(wo, wh) / gomath::abs(wo.z);
}
// MicrofacetReflection.F / .Pdf (reflection.go:690-704, 730-736), FresnelDielectric(1, eta)
__device__ inline Spec mf_refl_f(const BSDFX& x, V3 wo, V3 wi) {
    const double c0 = gomath::abs(wo.z), c1 = gomath::abs(wi.z);
    V3 wh = wi + wo;
    if (c1 == 0 || c0 == 0) return spec(0);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return spec(0);
    wh = normalized(wh);
    const double F = fr_dielectric(dot(wi, wh), 1.0, x.eta);
    return smuls(smul(x.r, spec(F)), tr_d(x, wh) * tr_g(x, wo, wi) / (4 * c1 * c0));
}
__device__ inline double mf_refl_pdf(const BSDFX& x, V3 wo, V3 wi) {
    if (!(wo.z * wi.z > 0)) return 0;
    const V3 wh = normalized(wo + wi);
    return tr_pdf(x, wo, wh) / (4 * dot(wo, wh));
}
// MicrofacetTransmission.F / .Pdf (reflection.go:758-790, 820-835): F is 0 unless
// wo and wi share a hemisphere (the reference's inverted test), wh is not
// normalized, and the mode field is left at its zero value (not Radiance), so
// factor stays 1
__device__ inline Spec mf_trans_f(const BSDFX& x, V3 wo, V3 wi) {
    if (!(wo.z * wi.z > 0)) return spec(0);
    const double co = wo.z, ci = wi.z;
    if (ci == 0 || co == 0) return spec(0);
    const double eta = wo.z > 0 ? 1.0 / x.eta : x.eta / 1.0;
    V3 wh = wo + muls(wi, eta);
    if (wh.z < 0) wh = muls(wh, -1);
    const double F = fr_dielectric(dot(wo, wh), 1.0, x.eta);
    const double sd = dot(wo, wh) * eta * dot(wi, wh);
    const double factor = 1.0;
    return smuls(smul(spec(1 - F), x.t), gomath::abs(tr_d(x, wh) * tr_g(x, wo, wi) * eta * eta * absdot(wi, wh) *
                                                     absdot(wo, wh) * factor * factor / (ci * co * sd * sd)));
}
__device__ inline double mf_trans_pdf(const BSDFX& x, V3 wo, V3 wi) {
    if (wo.z * wi.z > 0) return 0;
    const double eta = wo.z > 0 ? 1.0 / x.eta : x.eta / 1.0;
    const V3 wh = wo + muls(wi, eta);
    const double sd = dot(wo, wh) + eta * dot(wi, wh);
    const double dwh = gomath::abs((eta * eta * dot(wi, wh)) / (sd * sd));
    return tr_pdf(x, wo, wh) * dwh;
}
// OrenNayar.F (reflection.go:627-652); the else branch's tanBeta keeps sinThetaO
__device__ inline Spec oren_nayar_f(const BSDFX& x, V3 wo, V3 wi) {
    const double sin_i = sin_theta(wi), sin_o = sin_theta(wo);
    double max_cos = 0.0;
    if (sin_i > 1e-4 && sin_o > 1e-4) {
        const double sp_i = sin_phi(wi), cp_i = cos_phi(wi), sp_o = sin_phi(wo), cp_o = cos_phi(wo);
        const double d_cos = cp_i * cp_o + sp_i * sp_o;
        max_cos = gomath::max(0.0, d_cos);
    }
    double sin_alpha, tan_beta;
    if (gomath::abs(wi.z) > gomath::abs(wo.z)) {
        sin_alpha = sin_o;
        tan_beta = sin_o / gomath::abs(wo.z);
    } else {
        sin_alpha = sin_i;
        tan_beta = sin_o / gomath::abs(wo.z);
    }
    return smuls(x.r, inv_pi() * (x.ax + x.ay * max_cos * sin_alpha * tan_beta));
}
// BSDF.F / BSDF.Pdf (reflection.go:169-186, 255-278) of a rough glass, flags
// BSDFAll &^ BSDFSpecular (both microfacet lobes match)
__device__ inline Spec mf_bsdf_f(const BSDF& b, const BSDFX& x, V3 woW, V3 wiW) {
    const V3 wi = w2l(b, wiW), wo = w2l(b, woW);
    if (wo.z == 0.0) return spec(0);
    const bool reflect = dot(wiW, b.ng) * dot(woW, b.ng) > 0;
    Spec f = spec(0);
    if (x.kind == BXDF_KIND_OREN_NAYAR) return (x.n && reflect) ? f + oren_nayar_f(x, wo, wi) : f;
    if (x.mf_r && reflect) f = f + mf_refl_f(x, wo, wi);
    if (x.mf_t && !reflect) f = f + mf_trans_f(x, wo, wi);
    return f;
}
__device__ inline double mf_bsdf_pdf(const BSDF& b, const BSDFX& x, V3 woW, V3 wiW) {
    if (x.n == 0) return 0;
    const V3 wo = w2l(b, woW), wi = w2l(b, wiW);
    if (wo.z == 0) return 0;
    if (x.kind == BXDF_KIND_OREN_NAYAR) return (0 + lambert_pdf(wo, wi)) / 1.0;
    double pdf = 0;
    if (x.mf_r) pdf += mf_refl_pdf(x, wo, wi);
    if (x.mf_t) pdf += mf_trans_pdf(x, wo, wi);
    return pdf / (double)x.n;
}
// BSDF.SampleF (reflection.go:188-253) over any BSDFX, flags BSDFAll (Path.Li),
// returning the LOCAL-frame wi (#7) and the sampled type; type -1: the
// reference panics (rough glass: SampleWH's nil wh reaches Reflect/Refract)
__device__ inline Spec bsdfx_sample_f(const BSDF& b, const BSDFX& x, V3 woW, V2 u, V3& wi, double& pdf, int& type) {
    type = 0;
    if (x.kind == BXDF_KIND_LAMBERT) return bsdf_sample_f(b, woW, u, wi, pdf);   // sampleF's type is 0
    wi = V3{0, 0, 0};
    pdf = 0;
    if (x.n == 0) return spec(0);
    const double comp = gomath::min(gomath::floor(u.x * 1.0), 1.0 - 1);
    const V2 ur{gomath::min(u.x * 1.0 - comp, gomath::kOneMinusEpsilon), u.y};
    const V3 wo = w2l(b, woW);
    if (wo.z == 0.0) return spec(0);
    if (x.kind == BXDF_KIND_OREN_NAYAR) {   // the default sampleF (reflection.go:305-314)
        const V2 d = concentric_sample_disk(ur);
        V3 w{d.x, d.y, gomath::sqrt(gomath::max(0.0, 1.0 - d.x * d.x - d.y * d.y))};
        if (wo.z < 0) w.z *= -1;
        const double p = lambert_pdf(wo, w);
        const Spec f = oren_nayar_f(x, wo, w);
        if (p == 0.0) return spec(0);
        wi = w;
        pdf = p;
        return f;
    }
    if (x.kind == BXDF_KIND_MICROFACET) {
        type = -1;
        return spec(0);
    }
    if (x.kind == BXDF_KIND_SPEC_REFL) {   // SpecularReflection.SampleF, FresnelNoOp (reflection.go:557-562)
        wi = V3{-wo.x, -wo.y, wo.z};
        pdf = 1.0;
        return sdivs(smul(spec(1.0), x.r), gomath::abs(wi.z));
    }
    // FresnelSpecular.SampleF (reflection.go:489-524), incl. its (etaT / etaT) radiance scale
    const double F = fr_dielectric(wo.z, 1.0, x.eta);
    if (ur.x < F) {
        wi = V3{-wo.x, -wo.y, wo.z};
        pdf = F;
        type = BXDF_SPECULAR | BXDF_REFLECTION;
        return sdivs(smuls(x.r, F), gomath::abs(wi.z));
    }
    double eta_i, eta_t;
    if (wo.z > 0) { eta_i = 1.0; eta_t = x.eta; } else { eta_i = x.eta; eta_t = 1.0; }
    V3 n{0, 0, 1};
    if (dot(n, wo) < 0.0) n = muls(n, -1);   // FaceForward (geometry.go:111-116)
    const double eta = eta_i / eta_t;        // Refract (reflection.go:106-118)
    const double cos_i = dot(n, wo);
    const double sin2_i = gomath::max(0.0, 1 - cos_i * cos_i);
    const double sin2_t = eta * eta * sin2_i;
    if (sin2_t >= 1) return spec(0);         // total internal reflection: pdf 0
    const double cos_t = gomath::sqrt(1 - sin2_t);
    const V3 w = muls(wo, -eta) + muls(n, eta * cos_i - cos_t);
    Spec ft = smuls(x.t, 1 - F);
    ft = smuls(ft, (eta_i * eta_i) / (eta_t / eta_t));   // mode == Radiance
    const double p = 1 - F;
    if (p == 0.0) return spec(0);
    wi = w;
    pdf = p;
    type = BXDF_SPECULAR | BXDF_TRANSMISSION;
    return sdivs(ft, gomath::abs(w.z));
}

// ------------------------------------------------------------------- lights
struct LightSample {
    Spec Li;
    V3 wi;
    double pdf;
    V3 tp, tperr, tn;   // VisibilityTester p1
};

// Sphere.SampleAtInteraction (sphere.go:287-344) incl. the inside-sphere branch
__device__ inline void sphere_sample_at(const pbrt_shape_desc& s, const SI& ref, V2 u, V3& p, V3& perr, V3& n,
                                        double& pdf) {
    const pbrt_matrix4x4& M = s.object_to_world.m;
    V3 pc = xf_point(M, V3{0, 0, 0}, V3{0, 0, 0}, nullptr);
    V3 po = offset_ray_origin(ref.p, ref.perr, ref.n, pc - ref.p);
    if (dist2(po, pc) <= s.radius * s.radius) {
        // Sphere.Sample (sphere.go:270-285) + UniformSampleSphere (sampling.go:158-163)
        double z = 1.0 - 2.0 * u.x;
        double rr = gomath::sqrt(gomath::max(0, 1 - z * z));
        double ph = 2 * gomath::kPi * u.y;
        V3 pobj = muls(V3{rr * gomath::cos(ph), rr * gomath::sin(ph), z}, s.radius);
        n = normalized(xf_normal(s.object_to_world.m_inv, pobj));
        if (s.reverse_orientation) n = muls(n, -1);
        pobj = muls(pobj, s.radius / dist(pobj, V3{0, 0, 0}));
        V3 pobj_err = muls(vabs(pobj), gomath::gamma(5));
        p = xf_point(M, pobj, pobj_err, &perr);
        pdf = 1.0 / (s.phi_max * s.radius * (s.z_max - s.z_min));
        V3 wi = p - ref.p;
        if (len2(wi) == 0) {
            pdf = 0;
        } else {
            wi = normalized(wi);
            pdf *= dist2(ref.p, p) / absdot(n, muls(wi, -1));
        }
        if (gomath::is_inf(pdf)) pdf = 0.0;
        return;
    }
    V3 wc = normalized(pc - ref.p);
    V3 wcx, wcy;
    coordinate_system(wc, wcx, wcy);
    double r2 = s.radius * s.radius;
    double sin2max = r2 / dist2(ref.p, pc);
    double cosmax = gomath::sqrt(gomath::max(0, 1.0 - sin2max));
    double cost = (1.0 - u.x) + u.x * cosmax;
    double sint = gomath::sqrt(gomath::max(0, 1 - cost * cost));
    double phi = u.y * 2 * gomath::kPi;
    double dc = dist(ref.p, pc);
    double ds = dc * cost - gomath::sqrt(gomath::max(0, r2 - (dc * dc) * (sint * sint)));
    double cosa = (dc * dc + r2 - ds * ds) / (2.0 * dc * s.radius);
    double sina = gomath::sqrt(gomath::max(0, 1.0 - cosa * cosa));
    // SphericalDirectionXYZ (geometry.go:66-70) with -wcX, -wcY, -wc
    V3 nw = (muls(muls(wcx, -1), sina * gomath::cos(phi)) + muls(muls(wcy, -1), sina * gomath::sin(phi))) +
            muls(muls(wc, -1), cosa);
    p = pc + muls(nw, s.radius);
    perr = muls(vabs(p), gomath::gamma(5.0));
    n = s.reverse_orientation ? muls(nw, -1) : nw;
    pdf = 1.0 / (2.0 * gomath::kPi * (1.0 - cosmax));   // UniformConePdf
}

// Light.SampleLi for Point (point.go:44-49), Distant (distant.go:40-44, #15)
// and DiffuseAreaLight (diffuse.go:47-59, unnormalized wi #12)
__device__ inline void sample_li(const DevScene& sc, const pbrt_light_desc& L, const SI& si, V2 u, LightSample& ls) {
    if (L.type == PBRT_LIGHT_POINT) {
        V3 pl = load3(L.p_light);
        ls.wi = normalized(pl - si.p);
        ls.pdf = 1.0;
        ls.Li = sdivs(spec3(L.spectrum), dist2(pl, si.p));
        ls.tp = pl; ls.tperr = V3{0, 0, 0}; ls.tn = V3{0, 0, 0};
    } else if (L.type == PBRT_LIGHT_DISTANT) {
        V3 w = load3(L.w_light);
        ls.tp = muls(w, 2 * L.world_radius);
        ls.tperr = V3{0, 0, 0}; ls.tn = V3{0, 0, 0};
        ls.Li = spec3(L.spectrum);
        ls.wi = w;
        ls.pdf = 1;
    } else {
        V3 p, perr, n;
        double pdf;
        sphere_sample_at(sc.shapes[L.shape], si, u, p, perr, n, pdf);
        if (pdf == 0 || len2(p - si.p) == 0) {
            ls.Li = spec(0); ls.wi = V3{0, 0, 0}; ls.pdf = 0;
            ls.tp = ls.tperr = ls.tn = V3{0, 0, 0};
            return;
        }
        ls.wi = p - si.p;
        ls.pdf = pdf;
        ls.tp = p; ls.tperr = perr; ls.tn = n;
        ls.Li = (L.two_sided || dot(n, muls(ls.wi, -1)) > 0) ? spec3(L.spectrum) : spec(0);
    }
}

// EstimateDirect, light-sampling half (integrator.go:79-130), up to its
// visibility test: the shadow ray (SpawnRayToInteraction) and the Ld the
// estimate returns if that ray is unoccluded. Returns false when no ray is
// traced (zero pdf, black Li or black f): Ld is then spec(0). The BSDF-sampled
// MIS half (:132-192) is not executed: no primitive carries an area light
// (primitive.go:33, GetAreaLight() == nil) so it always contributes 0.
__device__ inline bool estimate_direct_begin(const DevScene& sc, const SI& si, const BSDF& b, int li, V2 u_light,
                                             Ray& sr, Spec& ld_vis) {
    const pbrt_light_desc& L = sc.lights[li];
    const bool is_delta = L.type != PBRT_LIGHT_DIFFUSE_AREA;
    LightSample ls;
    sample_li(sc, L, si, u_light, ls);
    if (!(ls.pdf > 0 && !is_black(ls.Li))) return false;
    Spec f = bsdf_f(b, si.wo, ls.wi);
    double wdn = absdot(ls.wi, si.sn);
    f = smuls(f, wdn);
    double scat_pdf = bsdf_pdf(b, si.wo, ls.wi);
    if (is_black(f)) return false;
    // VisibilityTester.Unoccluded -> SpawnRayToInteraction (interaction.go:91-102, #14)
    V3 origin = offset_ray_origin(si.p, si.perr, si.n, ls.tp - si.p);
    V3 target = offset_ray_origin(ls.tp, ls.tperr, ls.tn, origin - ls.tp);
    sr = Ray{si.p, target - origin, 1 - 0.0001, si.time};
    Spec Ld = spec(0);
    if (is_delta) {
        Ld = Ld + sdivs(smul(f, ls.Li), ls.pdf);
    } else {
        double fp = 1.0 * ls.pdf, gp = 1.0 * scat_pdf;   // PowerHeuristic(1, lightPdf, 1, scatteringPdf)
        double w = (fp * fp) / (fp * fp + gp * gp);
        Ld = Ld + sdivs(smuls(smul(f, ls.Li), w), ls.pdf);
    }
    ld_vis = Ld;
    return true;
}
// estimate_direct_begin over a BSDFX (kX wave pipelines): OrenNayar evaluates
// its own F with the Lambertian Pdf; Lambert, Mirror (F = Pdf = 0: no shadow
// ray) and smooth glass take the shared begin on `b`.
__device__ inline bool estimate_direct_begin_x(const DevScene& sc, const SI& si, const BSDF& b, const BSDFX& x, int li,
                                               V2 u_light, Ray& sr, Spec& ld_vis) {
    if (x.kind != BXDF_KIND_OREN_NAYAR && x.kind != BXDF_KIND_MICROFACET)
        return estimate_direct_begin(sc, si, b, li, u_light, sr, ld_vis);
    const pbrt_light_desc& L = sc.lights[li];
    const bool is_delta = L.type != PBRT_LIGHT_DIFFUSE_AREA;
    LightSample ls;
    sample_li(sc, L, si, u_light, ls);
    if (!(ls.pdf > 0 && !is_black(ls.Li))) return false;
    const Spec f = smuls(mf_bsdf_f(b, x, si.wo, ls.wi), absdot(ls.wi, si.sn));
    const double scat_pdf = mf_bsdf_pdf(b, x, si.wo, ls.wi);
    if (is_black(f)) return false;
    const V3 origin = offset_ray_origin(si.p, si.perr, si.n, ls.tp - si.p);
    const V3 target = offset_ray_origin(ls.tp, ls.tperr, ls.tn, origin - ls.tp);
    sr = Ray{si.p, target - origin, 1 - 0.0001, si.time};
    Spec Ld = spec(0);
    if (is_delta) {
        Ld = Ld + sdivs(smul(f, ls.Li), ls.pdf);
    } else {
        const double fp = 1.0 * ls.pdf, gp = 1.0 * scat_pdf;
        const double w = (fp * fp) / (fp * fp + gp * gp);
        Ld = Ld + sdivs(smuls(smul(f, ls.Li), w), ls.pdf);
    }
    ld_vis = Ld;
    return true;
}
// EstimateDirect (integrator.go:79-195): an occluded shadow ray zeroes Li, so
// Ld stays spec(0).
// traced (optional): +1 when the visibility ray is traced (stats.rays_shadow).
__device__ inline Spec estimate_direct(const DevScene& sc, uint16_t* stack, int& panic, const SI& si, const BSDF& b,
                                       int li, V2 u_light, uint64_t* traced = nullptr) {
    Ray sr;
    Spec ld_vis;
    if (!estimate_direct_begin(sc, si, b, li, u_light, sr, ld_vis)) return spec(0);
    if (traced) ++*traced;
    if (bvh_traverse<true>(sc, sr, nullptr, stack, panic)) return spec(0);
    return ld_vis;
}

// EstimateDirect for the serial kernel's BSDFX: rough glass evaluates its
// microfacet F and Pdf, and for an area light the BSDF-sampled half's
// BSDF.SampleF panics (integrator.go:134-139 always runs it); every other BSDF
// is the shared estimate_direct.
// The microfacet / OrenNayar half of estimate_direct_x, out of line: the
// kernels that inline estimate_direct_x keep the common BSDFs' path small (an
// out-of-line estimate_direct_x made every light sample of k_paths_ci<kX> a call).
__device__ __forceinline__ Spec estimate_direct_rough(const DevScene& sc, uint16_t* stack, int& panic, const SI& si,
                                                   const BSDF& b, const BSDFX& x, int li, V2 u_light,
                                                   uint64_t* traced) {
    const pbrt_light_desc& L = sc.lights[li];
    const bool is_delta = L.type != PBRT_LIGHT_DIFFUSE_AREA;
    LightSample ls;
    sample_li(sc, L, si, u_light, ls);
    Spec Ld = spec(0);
    if (ls.pdf > 0 && !is_black(ls.Li)) {
        const Spec f = smuls(mf_bsdf_f(b, x, si.wo, ls.wi), absdot(ls.wi, si.sn));
        const double scat_pdf = mf_bsdf_pdf(b, x, si.wo, ls.wi);
        if (!is_black(f)) {
            const V3 origin = offset_ray_origin(si.p, si.perr, si.n, ls.tp - si.p);
            const V3 target = offset_ray_origin(ls.tp, ls.tperr, ls.tn, origin - ls.tp);
            Ray sr{si.p, target - origin, 1 - 0.0001, si.time};
            if (traced) ++*traced;
            const bool occluded = bvh_traverse<true>(sc, sr, nullptr, stack, panic);
            if (panic) return spec(0);
            if (!occluded) {
                if (is_delta) {
                    Ld = Ld + sdivs(smul(f, ls.Li), ls.pdf);
                } else {
                    const double fp = 1.0 * ls.pdf, gp = 1.0 * scat_pdf;
                    const double w = (fp * fp) / (fp * fp + gp * gp);
                    Ld = Ld + sdivs(smuls(smul(f, ls.Li), w), ls.pdf);
                }
            }
        }
    }
    if (x.kind == BXDF_KIND_MICROFACET && !is_delta && x.n > 0 && w2l(b, si.wo).z != 0) panic = PBRT_PANIC_NIL_DEREF;
    return Ld;
}
__device__ __forceinline__ Spec estimate_direct_x(const DevScene& sc, uint16_t* stack, int& panic, const SI& si,
                                                  const BSDF& b, const BSDFX& x, int li, V2 u_light,
                                                  uint64_t* traced = nullptr) {
    if (x.kind != BXDF_KIND_MICROFACET && x.kind != BXDF_KIND_OREN_NAYAR)
        return estimate_direct(sc, stack, panic, si, b, li, u_light, traced);
    return estimate_direct_rough(sc, stack, panic, si, b, x, li, u_light, traced);
}

// Sphere.PdfWi (sphere.go:350-363): the cone pdf from outside the sphere;
// from inside, the generic Shape PdfWi (shape.go:29-47): the spawned ray's
// Sphere.Intersect (EFloat: can panic), 0 on a miss or an infinite pdf.
__device__ inline double sphere_pdf_wi(const pbrt_shape_desc& s, const SI& ref, V3 wi, int& panic) {
    const V3 pc = xf_point(s.object_to_world.m, V3{0, 0, 0}, V3{0, 0, 0}, nullptr);
    const V3 po = offset_ray_origin(ref.p, ref.perr, ref.n, ref.p - pc);
    if (dist2(po, pc) <= s.radius * s.radius) {
        const Ray r{offset_ray_origin(ref.p, ref.perr, ref.n, wi), wi, kInf, ref.time};   // SpawnRay
        double t;
        V3 ph;
        if (!shape_hit(s, r, t, ph, panic) || panic) return 0.0;
        SI hs;
        shape_si(s, r, ph, hs);
        const double area = s.phi_max * s.radius * (s.z_max - s.z_min);
        const double pdf = dist2(ref.p, hs.p) / absdot(hs.n, muls(muls(wi, -1), area));
        return gomath::is_inf(pdf) ? 0.0 : pdf;
    }
    const double sin2max = s.radius * s.radius / dist2(ref.p, pc);
    const double cosmax = gomath::sqrt(gomath::max(0, 1.0 - sin2max));
    return 1.0 / (2.0 * gomath::kPi * (1.0 - cosmax));   // UniformConePdf
}

// PBRT_FLAG_PANIC_FIDELITY: EstimateDirect's BSDF-sampled half for an area
// light (integrator.go:132-192). Its radiance is always 0 (no primitive
// carries an area light, primitive.go:33), but Sphere.PdfWi and the spawned
// ray's closest hit run in the reference and can panic; only that is kept.
__device__ inline void estimate_direct_mis_ray(const DevScene& sc, uint16_t* stack, int& panic, const SI& si,
                                               const BSDF& b, int li, V2 u_scat) {
    const pbrt_light_desc& L = sc.lights[li];
    if (L.type != PBRT_LIGHT_DIFFUSE_AREA) return;   // IsDeltaLight
    V3 wi;
    double pdf;
    const Spec f = bsdf_sample_f(b, si.wo, u_scat, wi, pdf);   // local-frame wi (#7)
    if (is_black(f) || !(pdf > 0.0)) return;
    const double lpdf = sphere_pdf_wi(sc.shapes[L.shape], si, wi, panic);
    if (panic || lpdf == 0) return;
    Ray r{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf, si.time};
    SI tmp;
    (void)bvh_traverse<false>(sc, r, &tmp, stack, panic);
}

// Distribution1D.SampleDiscrete + FindInterval (sampling.go:42-55, math.go:64-80)
__device__ inline int sample_discrete(const pbrt_distribution_desc& d, double u, double& pdf) {
    int size = d.count + 1, first = 0, len = size;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (d.cdf[middle] <= u) { first = middle + 1; len -= half + 1; }
        else len = half;
    }
    int off = (int)gomath::clamp((double)(first - 1), 0, (double)(size - 2));
    pdf = 0;
    if (d.func_int > 0) pdf = d.func[off] / (d.func_int / (double)d.count);
    return off;
}

// UniformSampleOneLight (integrator.go:48-77): no /lightPdf, panic if > 10 (#10)
__device__ inline Spec uniform_sample_one_light(const DevScene& sc, Thread& t, const SI& si, const BSDF& b,
                                                const BSDFX& x, const pbrt_distribution_desc* dist,
                                                bool fidelity = false) {
    const int n = sc.n_lights;
    if (n == 0) return spec(0);
    int ln;
    if (dist) {
        double lpdf;
        ln = sample_discrete(*dist, get1d(t), lpdf);
        if (lpdf == 0.0) return spec(0);
    } else {
        ln = (int)gomath::to_int(gomath::min(get1d(t) * (double)n, (double)(n - 1)));
    }
    V2 ul = get2d(t);
    const V2 us = get2d(t);   // uScattering: only the MIS half reads it
    Spec s = estimate_direct_x(sc, t.stack, t.panic, si, b, x, ln, ul, &t.shadow_rays);
    if (fidelity && !t.panic) estimate_direct_mis_ray(sc, t.stack, t.panic, si, b, ln, us);
    if (!t.panic && max_component(s) > 10) t.panic = PBRT_PANIC_LD_GT_10;
    return s;
}

// -------------------------------------------------------------- integrators
// Path.Li (path.go:32-157). Out of line in the serial kernel: fully inlined
// into k_render_exact the compiler produced a kernel that faulted only after
// other kernels had run on the device (an uninitialized-register read).
// fidelity (PBRT_FLAG_PANIC_FIDELITY): also trace the rays whose results never
// reach the film but can panic in the reference -- the closest hit at
// bounces == maxDepth (path.go:44-45, 66) and the MIS half of EstimateDirect.
__device__ __noinline__ Spec path_li(const DevScene& sc, Thread& t, Ray ray, int max_depth, double rr_threshold,
                                     bool fidelity) {
    Spec L = spec(0), beta = spec(1);
    int32_t bounces = 0;
    double eta_scale = 1.0;
    for (;;) {
        bounces++;
        t.bounce = bounces;
        if (bounces >= max_depth) {   // path.go:66 breaks whether or not the ray hits
            t.closest_rays++;           // the reference traced it first (path.go:44-45)
            if (fidelity) {
                SI tmp;
                (void)bvh_traverse<false>(sc, ray, &tmp, t.stack, t.panic);
            }
            break;
        }
        SI isect;
        t.closest_rays++;
        if (!bvh_traverse<false>(sc, ray, &isect, t.stack, t.panic)) break;
        if (t.panic) break;
        BSDF b;
        BSDFX x;
        if (compute_bsdf_x(sc, isect, b, x) < 0) { t.panic = -1; break; }
        if (bsdfx_nonspecular(b, x)) {   // NumComponents(BSDFAll &^ BSDFSpecular) > 0
            Spec ld = uniform_sample_one_light(sc, t, isect, b, x, sc.dist, fidelity);
            if (t.panic) break;
            L = L + smul(beta, ld);
        }
        V3 wo = ray.d;   // path.go:91 (#8)
        V2 u = get2d(t);
        V3 wi;
        double pdf;
        int flags;
        Spec f = bsdfx_sample_f(b, x, wo, u, wi, pdf, flags);
        if (flags == -1) { t.panic = PBRT_PANIC_NIL_DEREF; break; }
        if (is_black(f) || pdf == 0.0) break;
        double wp = absdot(wi, isect.sn) / pdf;
        beta = smul(beta, smuls(f, wp));
        if ((flags & BXDF_SPECULAR) && (flags & BXDF_TRANSMISSION)) {   // path.go:106-117
            const double eta = x.eta;
            if (dot(wo, isect.n) > 0) eta_scale *= eta * eta;
            else eta_scale *= 1 / (eta * eta);
        }
        // SpawnRay (interaction.go:68-77)
        ray.o = offset_ray_origin(isect.p, isect.perr, isect.n, wi);
        ray.d = wi;
        ray.tmax = kInf;
        ray.time = isect.time;
        Spec rr = smuls(beta, eta_scale);
        if (max_component(rr) < rr_threshold && bounces > 3) {
            double q = gomath::max(0.05, 1 - max_component(rr));
            if (get1d(t) < q) break;
            beta = sdivs(beta, 1 - q);
        }
    }
    return L;
}

// SamplerIntegratorSpecularTransmit's BSDF.SampleF(wo, u, Transmission|Specular)
// (integrator.go:383-385, reflection.go:188-253) on a SPEC_PAIR BSDF: the one
// matching BxDF is SpecularTransmission (reflection.go:428-451); returns the
// LOCAL-frame wi (#7). pdf 0: no transmission (no such BxDF, wo.z == 0, or
// total internal reflection).
__device__ inline Spec spec_trans_sample(const BSDF& b, const BSDFX& x, V3 woW, V2 u, V3& wi, double& pdf) {
    wi = V3{0, 0, 0};
    pdf = 0;
    if (x.kind != BXDF_KIND_SPEC_PAIR || !x.mf_t) return spec(0);
    (void)u;   // one matching component: comp 0, u unused by SpecularTransmission
    const V3 wo = w2l(b, woW);
    if (wo.z == 0.0) return spec(0);
    double eta_i, eta_t;
    if (wo.z > 0) { eta_i = 1.0; eta_t = x.eta; } else { eta_i = x.eta; eta_t = 1.0; }
    V3 n{0, 0, 1};
    if (dot(n, wo) < 0.0) n = muls(n, -1);   // FaceForward (geometry.go:111-116)
    const double eta = eta_i / eta_t;        // Refract (reflection.go:106-118)
    const double cos_i = dot(n, wo);
    const double sin2_i = gomath::max(0.0, 1 - cos_i * cos_i);
    const double sin2_t = eta * eta * sin2_i;
    if (sin2_t >= 1) return spec(0);
    const double cos_t = gomath::sqrt(1 - sin2_t);
    const V3 w = muls(wo, -eta) + muls(n, eta * cos_i - cos_t);
    const double F = fr_dielectric(w.z, 1.0, x.eta);   // FresnelDielectric(etaA, etaB)
    Spec ft = smul(x.t, spec(1 - F));
    ft = smuls(ft, (eta_i * eta_i) / (eta_t * eta_t));  // mode == Radiance
    wi = w;
    pdf = 1;
    return sdivs(ft, gomath::abs(w.z));
}

// DirectLighting.Li (directlighting.go:62-104) from depth 0. SpecularReflect
// matches no supported BxDF (none is Reflection|Specular: SpecularReflection is
// typed Reflection|Diffuse, reflection.go:538-544) and only draws its Get2D;
// SpecularTransmit recurses into Li at depth + 2 (#23) through a smooth glass's
// SpecularTransmission. The recursion is linear, so it runs as a loop that
// keeps each level's own radiance, f and |wi.ns|/pdf, then folds them back
// innermost first as the reference's returns do: L_k = own_k + (f_k * L_k+1) * w_k.
constexpr int kDlMaxLevels = 32;   // maxDepth <= 64 (host check)
__device__ __noinline__ Spec direct_li(const DevScene& sc, Thread& t, Ray ray, int max_depth, int strategy,
                                       bool fidelity) {
    Spec own[kDlMaxLevels], fk[kDlMaxLevels];
    double wk[kDlMaxLevels];
    int levels = 0;
    Spec L;
    for (int depth = 0;; depth += 2) {
        L = spec(0);
        SI si;
        t.bounce = depth + 1;
        t.closest_rays++;
        if (!bvh_traverse<false>(sc, ray, &si, t.stack, t.panic)) {
            for (int i = 0; i < sc.n_lights; i++) L = L + spec(0);
            break;
        }
        if (t.panic) break;
        BSDF b;
        BSDFX x;   // Mirror: F and Pdf are 0 and SpecularReflect/Transmit match no lobe
        if (compute_bsdf_x(sc, si, b, x, false) < 0) { t.panic = -1; break; }
        L = L + spec(0);   // si.Le(si.Wo): no primitive carries an area light
        if (sc.n_lights > 0) {
            if (strategy == PBRT_DL_UNIFORM_SAMPLE_ALL) {
                // UniformSampleAllLights (integrator.go:23-46); clones carry no arrays (#23)
                Spec acc = spec(0);
                for (int j = 0; j < sc.n_lights; j++) {
                    V2 ul = get2d(t);
                    const V2 us = get2d(t);
                    acc = acc + estimate_direct_x(sc, t.stack, t.panic, si, b, x, j, ul, &t.shadow_rays);
                    if (fidelity && !t.panic) estimate_direct_mis_ray(sc, t.stack, t.panic, si, b, j, us);
                    if (t.panic) break;
                }
                if (t.panic) break;
                L = L + acc;
            } else {
                L = L + uniform_sample_one_light(sc, t, si, b, x, nullptr, fidelity);
                if (t.panic) break;
            }
        }
        if (!(depth + 1 < max_depth)) break;
        get2d(t);           // SpecularReflect (integrator.go:352-355): black
        L = L + spec(0);
        const V2 u = get2d(t);   // SpecularTransmit (integrator.go:383-385)
        V3 wi;
        double pdf;
        const Spec f = spec_trans_sample(b, x, si.wo, u, wi, pdf);
        const double adn = absdot(wi, si.sn);
        if (!(pdf > 0 && !is_black(f) && adn != 0.0) || levels == kDlMaxLevels) {
            L = L + spec(0);
            break;
        }
        own[levels] = L;
        fk[levels] = f;
        wk[levels] = adn / pdf;
        levels++;
        // SpawnRay (interaction.go:68-77) with the local-frame wi
        ray.o = offset_ray_origin(si.p, si.perr, si.n, wi);
        ray.d = wi;
        ray.tmax = kInf;
        ray.time = si.time;
    }
    for (int k = levels - 1; k >= 0; k--) L = own[k] + smuls(smul(fk[k], L), wk[k]);
    return L;
}

// PerspectiveCamera.GenerateRayDifferential (camera.go:192-242)
__device__ inline Ray camera_ray(const pbrt_camera_desc& cam, double fx, double fy, double time_u, V2 plens) {
    V3 pcam = xf_point(cam.raster_to_camera.m, V3{fx, fy, 0}, V3{0, 0, 0}, nullptr);
    Ray r{V3{0, 0, 0}, normalized(pcam), kInf, 0};
    if (cam.lens_radius > 0) {
        V2 pl = concentric_sample_disk(plens);
        pl.x *= cam.lens_radius;
        pl.y *= cam.lens_radius;
        double ft = cam.focal_distance / r.d.z;
        V3 pf = muls(r.d, ft) + r.o;
        r.o = V3{pl.x, pl.y, 0};
        r.d = normalized(pf - r.o);
    }
    Ray w = xf_ray(cam.camera_to_world.m, r, nullptr, nullptr);
    w.time = gomath::lerp(time_u, cam.shutter_open, cam.shutter_close);
    return w;
}

}  // namespace pbrt
