// pbrt_spec.h — pieces of the wave-parallel EXACT kernel (k_render_spec).
//
// The reference renders a tile with ONE sampler clone whose PCG32 stream is
// consumed path after path (integrator.go:311-340), so path k+1 starts at the
// RNG offset where path k stopped. Two facts make that chain parallel:
//
//  1. Within a pixel, with n_dims >= 3, the camera ray, the first hit, its
//     BSDF and the bounce-1 light sample are the same for every sample: the
//     2D stratified values are always (0,0) (sampling.go:122-124, ledger #3)
//     and ray time never reaches an output. Only the bounce-1 light INDEX
//     varies (stratified 1D dim 1), so bounce-1 NEE is cached per light.
//  2. The number of PCG draws D a path consumes depends only on its RNG
//     offset, never on the sample index k, as long as the stratified 1D
//     values it reads do not steer control flow (light selection is
//     Uniform, or Power with every light pdf > 0; a Russian-roulette draw
//     that lands on a stratified dim marks the lane k-dependent).
//
// So a wave evaluates path TRAJECTORIES (no NEE) at 64 candidate offsets
// (head + 2j) in parallel, follows the exact chain head -> head + D(head) ->
// ... through the evaluated offsets, and repeats from where the chain left
// the window. When all of a pixel's offsets are known, the pixel's samples
// run as full paths (with NEE) one per lane, and their radiance is added to
// the tile film in sample order. Lane 0 of every window evaluates the exact
// head, so every window makes progress. Results are bit-identical to the
// serial replay (k_render_exact) — only the schedule changes.
#pragma once
#pragma clang fp contract(off)

#include "pbrt_path.h"
#include <type_traits>

namespace pbrt {

// PCG32 jump-ahead: state after 2^i steps = a[i] * state + inc * b[i] (mod 2^64)
struct PcgJump {
    uint64_t a[64];
    uint64_t b[64];
};
__device__ __forceinline__ uint64_t pcg_advance(const PcgJump& J, uint64_t s, uint64_t inc, uint64_t n) {
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) s = J.a[i] * s + inc * J.b[i];
    return s;
}
__device__ __forceinline__ uint32_t pcg_output(uint64_t old) {   // rng.go:36-42 (#1)
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((rot + 1u) & 31u));
}

// Stratified sampler of one path (pixel.go:60-80) positioned at an RNG
// offset; k < 0 while the sample index is still unknown (speculation).
// Russian-roulette decisions of a speculative trajectory (k < 0) whose RR value
// is a stratified 1D value, i.e. depends on the sample index the chain has not
// reached yet (traj_scatter<kX>, k_chain_ci<kX>): the trajectory continues as
// if the path survived and records each such decision -- the draws so far, the
// dimension and the threshold q. At the chain head, with the sample index k
// known, the draw count is the first recorded draws whose s1d[dim][k] < q
// (the path ends there), else the trajectory's own.
constexpr int kRrBranches = 3;
struct RrBranches {
    double q[kRrBranches];
    uint32_t cd[kRrBranches];   // draws << 8 | dimension
    uint32_t n;
};
struct SpecSampler {
    const double* s1d;   // ndims x spp shuffled 1D values of the pixel (LDS)
    int spp, ndims;
    RrBranches* rrb;     // k_chain_ci<kX>: the group's RR decision records (by ring index), else null
};
struct Cursor {
    Pcg rng;
    uint32_t draws;
    int cur1d, cur2d;
    int k;
    int kdep;          // a stratified value was needed while k < 0
    int rri;           // k < 0 in k_chain_ci<kX>: ss.rrb[rri] takes the RR decisions (else -1)
    int rrn;           // decisions recorded in ss.rrb[rri] (its `n` is written with each record,
                       // so an issue writes nothing to the record)
};
__device__ __forceinline__ double c_get1d(Cursor& c, const SpecSampler& s) {
    if (c.cur1d < s.ndims) {
        const int d = c.cur1d++;
        if (c.k < 0) {
            c.kdep = 1;
            return 0.5;
        }
        return s.s1d[d * s.spp + c.k];
    }
    c.draws++;
    return pcg_float(c.rng);
}
// a 1D value whose only effect is on radiance (light index): consume it
__device__ __forceinline__ void c_skip1d(Cursor& c, const SpecSampler& s) {
    if (c.cur1d < s.ndims) {
        c.cur1d++;
        return;
    }
    c.draws++;
    pcg_next(c.rng);
}
__device__ __forceinline__ V2 c_get2d(Cursor& c, const SpecSampler& s) {
    if (c.cur2d < s.ndims) {
        c.cur2d++;
        return V2{0.0, 0.0};
    }
    c.draws += 2;
    double x = pcg_float(c.rng);
    double y = pcg_float(c.rng);
    return V2{x, y};
}

// a 2D value whose only effect is on radiance, or none at all: consume it
__device__ __forceinline__ void c_skip2d(Cursor& c, int ndims) {
    if (c.cur2d < ndims) {
        c.cur2d++;
        return;
    }
    c.draws += 2;
    pcg_next(c.rng);
    pcg_next(c.rng);
}
// A sample's CameraSample (sampler.go:75-80 GetCameraSample: pFilm = pixel +
// Get2D, pLens = Get2D, time = Get1D), from a fresh cursor: stratified while
// the dimension is below n_dims (pixel.go:60-80), PCG32 draws beyond. The wave
// pipeline runs only where the camera ray is the pixel's own (pFilm
// stratified: n_dims >= 1; pLens stratified or a pinhole), so only the draws
// count here: n_dims = 1 draws pLens (2), n_dims >= 2 draws nothing.
__device__ __forceinline__ void c_camera(Cursor& c, int ndims) {
    c.cur1d = c.cur2d = 0;
    c_skip2d(c, ndims);   // pFilm
    c_skip2d(c, ndims);   // pLens
    if (c.cur1d < ndims) {   // time
        c.cur1d++;
    } else {
        c.draws++;
        pcg_next(c.rng);
    }
}

// PCG32 draws of a CameraSample (c_camera): 2 for pFilm and for pLens, 1 for
// time, each beyond the sampled dims
__host__ __device__ __forceinline__ uint32_t camera_draws(int ndims) {
    return (ndims < 1 ? 2u : 0u) + (ndims < 2 ? 2u : 0u) + (ndims < 1 ? 1u : 0u);
}

constexpr int kMaxCachedLights = 16;
// a cached bounce-1 light estimate traced its visibility ray (ray counters;
// or-ed into the estimate's panic word, whose low 16 bits are the panic kind)
constexpr int kLdTraced = 0x10000;
// per-path ray counts (stats.rays_closest / rays_shadow): closest-hit queries
// in the low 16 bits, visibility rays in the high 16
constexpr uint32_t kRayClosest = 1u, kRayShadow = 1u << 16;

// Per-pixel bounce-1 state shared by all samples of the pixel (LDS).
struct PixelCache {
    SI si;
    BSDF b;
    BSDFX x;                          // kX pipelines: Mirror / smooth Glass / OrenNayar
    V3 wo;                            // camera ray direction (path.go:91, #8)
    Spec ld[kMaxCachedLights];        // EstimateDirect(light l, uLight = (0,0))
    int ld_panic[kMaxCachedLights];   // panic kind of that estimate (incl. Ld > 10) | kLdTraced
    int hit;                          // first hit exists and maxDepth > 1
    int first_panic;                  // panic of the camera-ray traversal
};

// Bounce-1 state without the per-light estimates (what trajectories need).
struct ChainCache {
    SI si;
    BSDF b;
    BSDFX x;   // kX pipelines
    V3 wo;
    int hit;
    int pad;
};

// One iteration of Path.Li's loop (path.go:32-157) from bounce 1 on, with
// bounce 1 taken from the pixel cache, for kernels that refill a lane with a
// new path as soon as its path ends (k_paths_ci) or run one bounce per launch
// (k_pw_*). The loop-carried state is PathState + the Cursor; `bounce`
// reports the bounce of a panic. Returns true when the path has ended
// (radiance in s.L). Arithmetic and draw order are the reference's.
#ifndef PBRT_PATHS_LB
#define PBRT_PATHS_LB 1   // leaf boxes per scan iteration in path_step's traversals (build option)
#endif
struct PathState {
    Spec L, beta;
    Ray ray;
    double eta_scale;   // Path.Li's etaScale (kX: specular transmission)
    int bounces;
    int first;
    uint32_t rays;   // kRayClosest / kRayShadow counts of the path
};
// k_paths_ci's variant: the radiance sum lives in the lane's LDS slot (it is
// only added to, never read, inside a bounce), freeing its registers for the
// traversals
struct PathStateLds {
    Spec* L;
    Spec* aux;   // [0] beta0 and [1] ld_vis of a deferred shadow ray, held across the BSDF sample
    uint32_t* rays;   // the path's ray counts (LDS slot)
    Spec beta;
    Ray ray;
    double eta_scale;
    int bounces;
    int first;
};
__device__ __forceinline__ void add_L(PathState& s, Spec v) { s.L = s.L + v; }
__device__ __forceinline__ void add_L(PathStateLds& s, Spec v) { *s.L = *s.L + v; }
__device__ __forceinline__ void add_rays(PathState& s, uint32_t v) { s.rays += v; }
__device__ __forceinline__ void add_rays(PathStateLds& s, uint32_t v) { *s.rays += v; }
// kWhich: 0 any iteration, 1 only the first (s.first == 1: bounce 1 from the
// pixel cache, no traversal), 2 only later ones (s.first == 0).
//
// A traced iteration defers its light sample's shadow ray to the end of the
// iteration: the light draws, the estimate up to its visibility test, the
// BSDF sample, the throughput and Russian roulette run first (in the
// reference's draw order), then the shadow ray is traced and L += beta * Ld
// with the throughput of the interaction. The interaction and its BSDF are
// dead by then, so the any-hit traversal runs with their registers free (no
// scratch spills). Every value and every draw is the reference's; a panic of
// the shadow ray or Ld > 10 ends the path at this bounce, as it would have.
//
// kX: scenes with Mirror, smooth Glass or OrenNayar materials (BSDFX,
// bsdfx_sample_f, Path.Li's etaScale; rough glass stays on the serial kernel).
// kX = false is the Matte-only code, unchanged.
template <int kWhich = 0, bool kX = false, class Cache, class State>
__device__ __forceinline__ bool path_step(const DevScene& sc, const Cache& pc, const SpecSampler& ss, Cursor& c,
                                 State& s, int max_depth, double rr_threshold, uint16_t* stack, int& panic,
                                 int& bounce) {
    const bool first = kWhich == 1 ? true : kWhich == 2 ? false : (s.first != 0);
    SI isect;
    BSDF b;
    BSDFX x;
    V3 wo;
    const int nl = sc.n_lights;
    if (!first) {
        s.bounces++;
        bounce = s.bounces;
        add_rays(s, kRayClosest);   // the reference's Intersect (path.go:44-45), also at maxDepth
        if (s.bounces >= max_depth) return true;
        const bool hit = bvh_traverse<false, PBRT_PATHS_LB>(sc, s.ray, &isect, stack, panic);
        if (!hit) return true;
        if (panic) return true;
        if ((kX ? compute_bsdf_x(sc, isect, b, x) : compute_bsdf(sc, isect, b)) < 0) {
            panic = -1;
            return true;
        }
        wo = s.ray.d;
    } else {
        isect = pc.si;
        b = pc.b;
        if constexpr (kX) x = pc.x;
        wo = pc.wo;
        add_rays(s, kRayClosest);   // the camera ray's closest hit
    }
    bool pending = false, shadow = false;   // a deferred L += beta0 * Ld (with a shadow ray)
    constexpr bool kLdsAux = std::is_same<State, PathStateLds>::value;
    Ray sr;
    Spec ld_vis = spec(0);
    Spec beta0 = s.beta;
    if constexpr (kLdsAux) s.aux[0] = beta0;
    // NumComponents(BSDFAll &^ BSDFSpecular) > 0: UniformSampleOneLight (integrator.go:48-77)
    if (kX ? bsdfx_nonspecular(b, x) : b.n_bxdfs > 0) {
        if (nl == 0) {
            add_L(s, smul(s.beta, spec(0)));
        } else {
            int ln;
            if (sc.dist) {
                double lpdf;   // > 0 for every light (launch precondition)
                ln = sample_discrete(*sc.dist, c_get1d(c, ss), lpdf);
            } else {
                ln = (int)gomath::to_int(gomath::min(c_get1d(c, ss) * (double)nl, (double)(nl - 1)));
            }
            // bounce 1's light sample is the pixel's cached estimate where uLight is
            // the stratified (0,0) (n_dims >= 3); with fewer sampled dims it is a
            // PCG32 draw per sample, estimated here like any later bounce's
            const bool ul_strat = c.cur2d < ss.ndims;
            V2 ul = c_get2d(c, ss);
            c_get2d(c, ss);
            if (first && ul_strat) {
                const Spec ld = pc.ld[ln];
                const int lp = pc.ld_panic[ln];
                if (lp & kLdTraced) add_rays(s, kRayShadow);
                if (lp & 0xFFFF) {
                    panic = lp & 0xFFFF;
                    return true;
                }
                add_L(s, smul(s.beta, ld));
            } else {
                pending = true;
                shadow = kX ? estimate_direct_begin_x(sc, isect, b, x, ln, ul, sr, ld_vis)
                            : estimate_direct_begin(sc, isect, b, ln, ul, sr, ld_vis);
                if constexpr (kLdsAux) s.aux[1] = ld_vis;
            }
        }
    }
    s.first = 0;
    bool done = false;
    {
        V2 u = c_get2d(c, ss);
        V3 wi;
        double pdf;
        int type = 0;
        Spec f = kX ? bsdfx_sample_f(b, x, wo, u, wi, pdf, type) : bsdf_sample_f(b, wo, u, wi, pdf);
        if (kX && type == -1) {   // rough glass: the reference's nil dereference (host keeps it off kX)
            panic = PBRT_PANIC_NIL_DEREF;
            return true;
        }
        if (is_black(f) || pdf == 0.0) {
            done = true;
        } else {
            double wp = absdot(wi, isect.sn) / pdf;
            s.beta = smul(s.beta, smuls(f, wp));
            if (kX && (type & BXDF_SPECULAR) && (type & BXDF_TRANSMISSION)) {   // path.go:106-117
                const double eta = x.eta;
                if (dot(wo, isect.n) > 0) s.eta_scale *= eta * eta;
                else s.eta_scale *= 1 / (eta * eta);
            }
            s.ray.o = offset_ray_origin(isect.p, isect.perr, isect.n, wi);
            s.ray.d = wi;
            s.ray.tmax = kInf;
            s.ray.time = isect.time;
            Spec rr = smuls(s.beta, kX ? s.eta_scale : 1.0);
            if (max_component(rr) < rr_threshold && s.bounces > 3) {
                double q = gomath::max(0.05, 1 - max_component(rr));
                double u1 = c_get1d(c, ss);
                if (c.kdep || u1 < q) done = true;
                else s.beta = sdivs(s.beta, 1 - q);
            }
        }
    }
    if (pending) {
        Spec ld = spec(0);
        if (shadow) {
            add_rays(s, kRayShadow);
            const bool occluded = bvh_traverse<true, PBRT_PATHS_LB>(sc, sr, nullptr, stack, panic);
            if (panic) return true;
            if (!occluded) {
                if constexpr (kLdsAux) ld = s.aux[1];
                else ld = ld_vis;
            }
        }
        if (max_component(ld) > 10) {
            panic = PBRT_PANIC_LD_GT_10;
            return true;
        }
        if constexpr (kLdsAux) beta0 = s.aux[0];
        add_L(s, smul(beta0, ld));
    }
    return done;
}

// The rest of one trajectory iteration (Path.Li without light sampling, whose
// draws are still consumed) once the interaction at bounce
// `bounces` and its BSDF are known (light draws consumed, BSDF sample,
// throughput, Russian roulette), then the next iteration's depth test; the
// chain kernel (k_chain_ci) and the cold-frame probe run one per bounce.
// Returns 0: trace `ray` next; 1: the trajectory ended (D = c.draws);
// 2: its draw count depends on the sample index (kBadD).
// kX (Mirror / smooth Glass / OrenNayar scenes): the BSDFX `x` and Path.Li's
// etaScale `eta_scale` (see path_step); a rough-glass sample (the reference
// panics) returns 2, so the offset is re-run at the chain head and the panic
// is found by the path stage.
template <bool kX = false>
__device__ inline int traj_scatter(const DevScene& sc, const SI& isect, const BSDF& b, const BSDFX& x, V3 wo,
                                   Cursor& c, const SpecSampler& ss, Spec& beta, double& eta_scale, int& bounces,
                                   Ray& ray, int max_depth, double rr_threshold) {
    if ((kX ? bsdfx_nonspecular(b, x) : b.n_bxdfs > 0) && sc.n_lights > 0) {   // UniformSampleOneLight's draws
        c_skip1d(c, ss);
        c_get2d(c, ss);
        c_get2d(c, ss);
    }
    V2 u = c_get2d(c, ss);
    V3 wi;
    double pdf;
    int type = 0;
    Spec f = kX ? bsdfx_sample_f(b, x, wo, u, wi, pdf, type) : bsdf_sample_f(b, wo, u, wi, pdf);
    if (kX && type == -1) return 2;
    if (is_black(f) || pdf == 0.0) return 1;
    double wp = absdot(wi, isect.sn) / pdf;
    beta = smul(beta, smuls(f, wp));
    if (kX && (type & BXDF_SPECULAR) && (type & BXDF_TRANSMISSION)) {   // path.go:106-117
        const double eta = x.eta;
        if (dot(wo, isect.n) > 0) eta_scale *= eta * eta;
        else eta_scale *= 1 / (eta * eta);
    }
    ray.o = offset_ray_origin(isect.p, isect.perr, isect.n, wi);
    ray.d = wi;
    ray.tmax = kInf;
    ray.time = isect.time;
    Spec rr = smuls(beta, kX ? eta_scale : 1.0);
    if (max_component(rr) < rr_threshold && bounces > 3) {
        double q = gomath::max(0.05, 1 - max_component(rr));
        if (kX && c.k < 0 && c.rri >= 0 && c.cur1d < ss.ndims) {
            // the RR value is s1d[cur1d][k] for a sample index not known yet
            // (specular bounces draw no light sample, so RR reaches the
            // stratified dims): record the decision, continue as a survivor
            RrBranches& rb = ss.rrb[c.rri];
            if (c.rrn == kRrBranches || c.draws >= (1u << 24)) return 2;
            rb.q[c.rrn] = q;
            rb.cd[c.rrn] = (c.draws << 8) | (uint32_t)c.cur1d;
            rb.n = (uint32_t)++c.rrn;
            c.cur1d++;
            beta = sdivs(beta, 1 - q);
        } else {
            double u1 = c_get1d(c, ss);
            if (c.kdep) return 2;
            if (u1 < q) return 1;
            beta = sdivs(beta, 1 - q);
        }
    }
    bounces++;
    return bounces >= max_depth ? 1 : 0;
}

}  // namespace pbrt
