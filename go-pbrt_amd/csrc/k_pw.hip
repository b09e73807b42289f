// k_pw.hip — the path wavefront: per-bounce queues, material sort, trace / shade / shadow
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

template <bool kX>
__global__ __launch_bounds__(kWave) void k_pw_cache(DevScene sc, WaveBufs wb, int64_t rec0, int64_t nrec,
                                                    Spec* __restrict__ ldc, int* __restrict__ ldp) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    stage_nodes(sc);
    const int nl = sc.n_lights;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec * nl) return;
    const int64_t r = i / nl;
    const int l = (int)(i - r * nl);
    const PixelRec& pr = wb.prec[rec0 + r];
    if (!(pr.hit && (kX ? bsdfx_nonspecular(pr.b, pr.x) : pr.b.n_bxdfs > 0))) return;
    int pl = 0;
    uint64_t traced = 0;
    const Spec ld = kX ? estimate_direct_x(sc, stack_lds + threadIdx.x, pl, pr.si, pr.b, pr.x, l, V2{0.0, 0.0}, &traced)
                       : estimate_direct(sc, stack_lds + threadIdx.x, pl, pr.si, pr.b, l, V2{0.0, 0.0}, &traced);
    if (!pl && max_component(ld) > 10) pl = PBRT_PANIC_LD_GT_10;
    ldc[i] = ld;
    ldp[i] = pl | (traced ? kLdTraced : 0);
}

template <bool kMB, bool kX>
__global__ __launch_bounds__(kWave) void k_pw_start(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                    int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc,
                                                    const int* __restrict__ ldp, PwPath* __restrict__ paths,
                                                    PwQueues qs, unsigned long long* __restrict__ pkey) {
    // bounce 1's shadow ray is traced here when its light sample is not the
    // pixel's cached one (n_dims < 3, path_step): trees beyond LDS need the stack
    __shared__ uint16_t stack_lds[64 * kStackStride];
    const int n = rp.spp;
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n < 2 || i >= nrec * (n - 1)) return;
    const int64_t r = i / (n - 1);
    const int k = 1 + (int)(i - r * (n - 1));
    const int64_t rec = rec0 + r, bs = rec / wb.ppt, pi = rec % wb.ppt;
    if (k == 1) pkey[rec] = ~0ULL;
    if (pi >= wb.tile_npx[bs]) return;
    const PixelRec& pr = wb.prec[rec];
    if (k >= pr.nvalid) return;
    PwPath p;
    p.rec = rec;
    p.k = k;
    p.L = spec(0);
    p.pnc = 0;
    p.bnc = 1;
    p.rays = kRayClosest;   // the camera ray's query
    if (!pr.hit) {   // no traced bounce: the sample's radiance is 0
        pw_finish(wb, n, p, pkey);
        return;
    }
    const uint64_t tile = (uint64_t)tile_of_slot(rp, slot_base + bs);
    Cursor c;
    c.rri = -1;
    c.rng.state = kMB ? mb_state(tile, (uint64_t)pi, (uint64_t)k) : wb.memb[rec * n + k];
    c.rng.inc = pcg_inc_of(tile);
    c.draws = 0;
    c_camera(c, rp.ndims);   // camera: Get2D pFilm, Get2D pLens, Get1D time
    c.k = k;
    c.kdep = 0;
    PathState s;
    s.L = spec(0);
    s.beta = spec(1);
    s.eta_scale = 1.0;
    s.bounces = 1;
    s.first = 1;
    s.rays = 0;
    const PwCache pc{pr.si, pr.b, pr.x, pr.wo, ldc + r * sc.n_lights, ldp + r * sc.n_lights};
    const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, rp.ndims};
    int pnc = 0, bnc = 1;
    bool done = path_step<1, kX>(sc, pc, ss, c, s, rp.max_depth, rp.rr_threshold, stack_lds + threadIdx.x, pnc, bnc);
    p.L = s.L;
    p.beta = s.beta;
    p.eta = s.eta_scale;
    p.ray = s.ray;
    p.bounces = s.bounces;
    p.rng = c.rng.state;
    p.cur1d = c.cur1d;
    p.cur2d = c.cur2d;
    p.kdep = c.kdep;
    p.pnc = pnc;
    p.bnc = bnc;
    p.rays = s.rays;   // path_step<1> counted the camera ray and its light sample
    if (!done) done = !pw_next_bounce(p, rp.max_depth);
    paths[i] = p;
    if (done)
        pw_finish(wb, n, p, pkey);
    else
        pw_push(&qs.cnt[0], qs.q[0], (uint32_t)i);
}

// in: trace queue `qin` (count cnt[cin]); out: hits (cnt[2], qs.q[2]) with
// their material key counted in cnt[3 + key]
// kMeshOnly: scenes of triangle meshes only (no analytic walk compiled in:
// 88 instead of 184 VGPRs, 5 waves per SIMD instead of 2)
template <bool kMeshOnly>
__global__ __launch_bounds__(kWave) void k_pw_trace(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths,
                                                    PwQueues qs, int cin, int n_keys,
                                                    unsigned long long* __restrict__ pkey) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const uint32_t* qin = qs.q[cin];
    const uint32_t nq = qs.cnt[cin];
    if (blockIdx.x == 0 && threadIdx.x == 0) qs.cnt[1] = 0;   // k_pw_shade's output, consumed after this pass's shadow step
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nq; t += gridDim.x * blockDim.x) {
        const uint32_t id = qin[t];
        PwPath& p = paths[id];
        Ray ray = p.ray;
        int panic = 0, best;
        V3 ph{0, 0, 0};
        const bool hit = bvh_walk<false, kStackStride, 4, kMeshOnly>(sc, ray, stack_lds + threadIdx.x, panic, best, ph);
        if (!hit || panic) {   // path_step: a miss or a traversal panic ends the path
            if (panic) p.pnc = panic;
            pw_finish(wb, rp.spp, p, pkey);
            continue;
        }
        p.ray.tmax = ray.tmax;
        p.best = best;
        p.ph = ph;
        int key = best < sc.n_prims ? sc.prims[best].material : sc.mesh.mesh_mat[tri_mesh(sc, best - sc.n_prims)];
        key = min(max(key, 0), n_keys - 1);
        p.flags = key;
        pw_push(&qs.cnt[2], qs.q[2], id);
        if (n_keys > 1) (void)pw_add_by_key(qs.cnt + 3, key);
    }
}

// exclusive scan of the key counts into offsets (one thread; n_keys <= 64)
__global__ void k_pw_scan(PwQueues qs, int n_keys) {
    uint32_t acc = 0;
    for (int k = 0; k < n_keys; k++) {
        qs.cnt[3 + kPwMaxKeys + k] = acc;
        acc += qs.cnt[3 + k];
    }
}

__global__ __launch_bounds__(256) void k_pw_scatter(const PwPath* __restrict__ paths, PwQueues qs) {
    const uint32_t nh = qs.cnt[2];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nh; t += gridDim.x * blockDim.x) {
        const uint32_t id = qs.q[2][t];
        qs.sorted[pw_add_by_key(qs.cnt + 3 + kPwMaxKeys, paths[id].flags)] = id;
    }
}

template <bool kX>
__global__ __launch_bounds__(kWave) void k_pw_shade(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                    PwPath* __restrict__ paths, PwQueues qs, int sorted,
                                                    unsigned long long* __restrict__ pkey) {
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    const uint32_t* qin = sorted ? qs.sorted : qs.q[2];
    const uint32_t nh = qs.cnt[2];
    const int n = rp.spp;
    if (blockIdx.x == 0 && threadIdx.x == 0) qs.cnt[0] = 0;   // k_pw_shadow's output (this pass's trace has read it)
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nh; t += gridDim.x * blockDim.x) {
        const uint32_t id = qin[t];
        PwPath& p = paths[id];
        SI isect;
        prim_si(sc, p.best, p.ray, p.ph, isect);
        BSDF b;
        BSDFX x;
        if ((kX ? compute_bsdf_x(sc, isect, b, x) : compute_bsdf(sc, isect, b)) < 0) {
            p.pnc = -1;
            pw_finish(wb, n, p, pkey);
            continue;
        }
        const V3 wo = p.ray.d;
        const int64_t bs = p.rec / wb.ppt;
        Cursor c;
        c.rri = -1;
        c.rng.state = p.rng;
        c.rng.inc = pcg_inc_of((uint64_t)tile_of_slot(rp, slot_base + bs));
        c.draws = 0;
        c.cur1d = p.cur1d;
        c.cur2d = p.cur2d;
        c.k = p.k;
        c.kdep = p.kdep;
        const SpecSampler ss{wb.s1d + p.rec * wb.s1d_stride, n, rp.ndims};
        // path_step<2> after its closest-hit traversal (pbrt_spec.h)
        int flags = 0;
        const Spec beta0 = p.beta;
        const int nl = sc.n_lights;
        if (kX ? bsdfx_nonspecular(b, x) : b.n_bxdfs > 0) {   // UniformSampleOneLight (integrator.go:48-77)
            if (nl == 0) {
                p.L = p.L + smul(p.beta, spec(0));
            } else {
                int ln;
                if (sc.dist) {
                    double lpdf;
                    ln = sample_discrete(*sc.dist, c_get1d(c, ss), lpdf);
                } else {
                    ln = (int)gomath::to_int(gomath::min(c_get1d(c, ss) * (double)nl, (double)(nl - 1)));
                }
                V2 ul = c_get2d(c, ss);
                c_get2d(c, ss);
                flags |= kPwPending;
                Ray sr;
                Spec ld_vis = spec(0);
                if (kX ? estimate_direct_begin_x(sc, isect, b, x, ln, ul, sr, ld_vis)
                       : estimate_direct_begin(sc, isect, b, ln, ul, sr, ld_vis))
                    flags |= kPwShadow;
                p.sr = sr;
                p.ld = ld_vis;
            }
        }
        {
            V2 u = c_get2d(c, ss);
            V3 wi;
            double pdf;
            int type = 0;
            Spec f = kX ? bsdfx_sample_f(b, x, wo, u, wi, pdf, type) : bsdf_sample_f(b, wo, u, wi, pdf);
            if (kX && type == -1) {   // rough glass: the reference's nil dereference (never routed here)
                p.pnc = PBRT_PANIC_NIL_DEREF;
                pw_finish(wb, n, p, pkey);
                continue;
            }
            if (is_black(f) || pdf == 0.0) {
                flags |= kPwDone;
            } else {
                double wp = absdot(wi, isect.sn) / pdf;
                p.beta = smul(p.beta, smuls(f, wp));
                if (kX && (type & BXDF_SPECULAR) && (type & BXDF_TRANSMISSION)) {   // path.go:106-117
                    const double eta = x.eta;
                    if (dot(wo, isect.n) > 0) p.eta *= eta * eta;
                    else p.eta *= 1 / (eta * eta);
                }
                p.ray.o = offset_ray_origin(isect.p, isect.perr, isect.n, wi);
                p.ray.d = wi;
                p.ray.tmax = kInf;
                p.ray.time = isect.time;
                Spec rr = smuls(p.beta, kX ? p.eta : 1.0);
                if (max_component(rr) < rp.rr_threshold && p.bounces > 3) {
                    double q = gomath::max(0.05, 1 - max_component(rr));
                    double u1 = c_get1d(c, ss);
                    if (c.kdep || u1 < q) flags |= kPwDone;
                    else p.beta = sdivs(p.beta, 1 - q);
                }
            }
        }
        p.beta0 = beta0;
        p.rng = c.rng.state;
        p.cur1d = c.cur1d;
        p.cur2d = c.cur2d;
        p.kdep = c.kdep;
        p.flags = flags;
        pw_push(&qs.cnt[1], qs.q[1], id);   // every shaded path passes the shadow step
    }
}

// in: the shaded paths (cnt[1], q[1]); out: the next trace queue (cnt[0], q[0])
template <bool kMeshOnly>
__global__ __launch_bounds__(kWave) void k_pw_shadow(DevScene sc, RenderParams rp, WaveBufs wb,
                                                     PwPath* __restrict__ paths, PwQueues qs,
                                                     unsigned long long* __restrict__ pkey) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const uint32_t ns = qs.cnt[1];
    if (blockIdx.x == 0)   // hits and key counts, for the next pass
        for (int i = threadIdx.x; i < 1 + kPwMaxKeys; i += blockDim.x) qs.cnt[2 + i] = 0;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ns; t += gridDim.x * blockDim.x) {
        const uint32_t id = qs.q[1][t];
        PwPath& p = paths[id];
        if (p.flags & kPwPending) {
            Spec ld = spec(0);
            if (p.flags & kPwShadow) {
                int panic = 0;
                Ray sr = p.sr;
                p.rays += kRayShadow;
                const bool occluded = bvh_traverse<true, 4, kMeshOnly>(sc, sr, nullptr, stack_lds + threadIdx.x, panic);
                if (panic) {
                    p.pnc = panic;
                    pw_finish(wb, rp.spp, p, pkey);
                    continue;
                }
                if (!occluded) ld = p.ld;
            }
            if (max_component(ld) > 10) {
                p.pnc = PBRT_PANIC_LD_GT_10;
                pw_finish(wb, rp.spp, p, pkey);
                continue;
            }
            p.L = p.L + smul(p.beta0, ld);
        }
        if ((p.flags & kPwDone) || !pw_next_bounce(p, rp.max_depth))
            pw_finish(wb, rp.spp, p, pkey);
        else
            pw_push(&qs.cnt[0], qs.q[0], id);
    }
}

// per pixel record: paths_group's epilogue (first panic in sample order, counters)
__global__ void k_pw_panics(RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec,
                            const unsigned long long* __restrict__ pkey, Counters* __restrict__ ctr) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const int64_t rec = rec0 + r, bs = rec / wb.ppt, pi = rec % wb.ppt;
    if (pi >= wb.tile_npx[bs]) return;
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile_of_slot(rp, slot_base + bs), x0, y0, x1, y1);
    PanicRec p{0, 0, 0, 0, x0 + pi % (x1 - x0), y0 + pi / (x1 - x0)};
    const PixelRec& pr = wb.prec[rec];
    const unsigned long long key = rp.spp >= 2 ? pkey[rec] : ~0ULL;
    if (pr.panic0) {
        p.kind = pr.panic0;
        p.sample = 1;
        p.bounce = 1;
    } else if (key != ~0ULL) {
        p.kind = (int)(key & 0xFF) - 1;
        p.bounce = (int)((key >> 8) & 0xFFFFFF);
        p.sample = (int)(key >> 32);
    }
    wb.ppanic[rec] = p;
    if (!p.kind && pr.nvalid > 1) {
        atomicAdd(&ctr->paths, (unsigned long long)(pr.nvalid - 1));
        atomicAdd(&ctr->camera_samples, (unsigned long long)(pr.nvalid - 1));
    }
}

template __global__ void k_pw_trace<false>(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, int cin, int n_keys, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_trace<true>(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, int cin, int n_keys, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_shadow<false>(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_shadow<true>(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_cache<false>(DevScene sc, WaveBufs wb, int64_t rec0, int64_t nrec, Spec* __restrict__ ldc, int* __restrict__ ldp);
template __global__ void k_pw_cache<true>(DevScene sc, WaveBufs wb, int64_t rec0, int64_t nrec, Spec* __restrict__ ldc, int* __restrict__ ldp);
template __global__ void k_pw_start<false, false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc, const int* __restrict__ ldp, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_start<false, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc, const int* __restrict__ ldp, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_start<true, false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc, const int* __restrict__ ldp, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_start<true, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc, const int* __restrict__ ldp, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_shade<false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, PwPath* __restrict__ paths, PwQueues qs, int sorted, unsigned long long* __restrict__ pkey);
template __global__ void k_pw_shade<true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, PwPath* __restrict__ paths, PwQueues qs, int sorted, unsigned long long* __restrict__ pkey);

}  // namespace pbrtk
