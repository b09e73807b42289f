// k_chain.h — k_chain_ci, the continuous-issue offset chain (EXACT mode); instantiated in k_chain_*.hip
// (Default template arguments live only in render_kernels.h, the declarations
// the host code sees; the definitions here repeat none, so the unity build works.)
#pragma once
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

//
// kW > 1: one tile per workgroup of kW waves (lanes_per_tile = 64 * kW). The
// tile's chain then advances kW times as many candidates per step, which cuts
// the slowest tile's latency, the frame's critical path when tiles are few
// per GPU (a multi-GPU shard). Idle lanes are ranked across the waves through
// LDS; StartPixel runs on the first wave.
// kDepth: traversal stack entries per lane. Trees of <= kLdsNodes (64) nodes
// are staged in LDS and walk their leaves only (no stack); larger trees walk
// with the reference's [64] stack (bvh.go:670).
// The ring entry's D of a trajectory with cursor c (kX: flagged when it
// recorded RR decisions; see kRrFlag)
template <bool kX>
__device__ __forceinline__ uint32_t ring_d(const Cursor& c, const SpecSampler& ss, uint32_t d) {
    if (!kX || c.rri < 0 || d == kBadExactD || c.rrn == 0) return d;
    return kRrFlag | (d == kBadSpecD ? kRrTailBad : d);
}

template <int kW, int kDepth, bool kX, int kEu, bool kSpWin>
// kDepth < 0 (kCiMeshOnly): scenes of triangle meshes only, no analytic walk
// compiled in (149 VGPRs), built for 3 waves per SIMD; Matte analytic scenes
// at PBRT_CI_EU_WAVES (3: 168 VGPRs, a few spills, faster than 2), kX at
// PBRT_CI_X_EU_WAVES (2). kEu > 0 sets the waves/SIMD the registers are
// budgeted for (the host picks <1, *, false, 2> where the workgroup's LDS
// allows fewer than 3 waves/SIMD anyway: then the 3-wave build only spills).
// kSpWin: the windowed wave StartPixel compiled in (rp.sp_window renders: large
// spp without jitter, config C).
__global__ __launch_bounds__(kWave * kW) __attribute__((amdgpu_waves_per_eu(kEu > 0 ? kEu : kDepth < 0 ? PBRT_CI_MESH_EU_WAVES : kX ? PBRT_CI_X_EU_WAVES : PBRT_CI_EU_WAVES, 8))) void k_chain_ci(
    DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
    int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr,
    const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint64_t t_begin = wall_clock64();
    // the frame's chain progress record (completion-driven path stage, render.hip;
    // null elsewhere; layout at kProgHead)
    if (prog && threadIdx.x == 0) __hip_atomic_fetch_add(&prog[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t cs = cstride == 1 ? 1u : 2u;   // candidate offsets head + cs * j
    constexpr int kT = kWave * kW;   // threads per workgroup (stack stride)
    // kDepth 0: an LDS-staged tree, walked without a stack (no stack array)
    __shared__ uint16_t stack_lds[kDepth > 0 ? kDepth * kT : 1];
#ifdef PBRT_CI_DENSE_WALK
    // bvh_walk_dense's per-wave scratch (LDS-staged trees only)
    __shared__ __attribute__((aligned(16))) unsigned char dense_lds[kDepth > 0 ? 16 : kW * kDenseScratch];
#endif
    __shared__ CiGroup gs[kCiMaxGroups];
    __shared__ uint64_t sh_state;
    __shared__ uint32_t sh_draws;   // StartPixel's draw count
    __shared__ int sh_act;          // next-pixel speculation started this step
    __shared__ int wcnt[kW];
#ifdef PBRT_CI_DIAG
    __shared__ uint32_t dh[64];   // on-chain D histogram of the block (diagnostics)
#endif
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    stage_nodes(sc);
    const int L = kW > 1 ? kT : lanes_per_tile, G = kW > 1 ? 1 : kWave / L;
    const int g = kW > 1 ? 0 : lane / L, gl = kW > 1 ? tid : lane - g * L;
    // workgroup -> tile slot: heaviest-first order from the previous frame
    // (one tile per workgroup only), else the identity
    const int64_t blk = order ? (int64_t)order[blockIdx.x] : (int64_t)blockIdx.x;
    const uint32_t R = (uint32_t)ring_size;   // a power of two (host: 256 / G or 256 * kW entries)
    const PcgJump& J = *jump;
    // StartPixel's values: staged in LDS, or (lay.s1d < 0: large spp, serial
    // StartPixel) written by it straight to the pixel's global record
    double* s1d = lay.s1d >= 0 ? (double*)(lds + lay.s1d) : nullptr;
    uint16_t* other = (uint16_t*)(lds + lay.other);
    uint32_t* vbuf = (uint32_t*)(lds + lay.vbuf);
    // Next-pixel speculation (multi-wave Matte tiles, rp.ci_nps): once the
    // current pixel's last sample has its offset, the lanes it leaves idle
    // trace trajectories of the NEXT pixel from every offset its first sample
    // can start at (a trajectory depends only on its offset's PCG32 state and
    // the pixel's bounce-1 record), so the next pixel's chain
    // starts on resolved entries instead of an empty pipeline. Each pixel
    // parity has its own ring (not aliased with the StartPixel staging) and
    // ChainCache; the next pixel's offset is only known after its StartPixel
    // (draw count sh_draws), and every entry is exact for the pixel it was
    // traced for, so the walk is unchanged.
    constexpr bool kNps = kW > 1 && !kX;
    const bool nps_on = kNps && rp.ci_nps != 0 && cstride == 1;
    // speculation on the next pixel starts rp.ci_nps samples before the current
    // pixel's end, once kNpsMinStats draw counts give the mean and spread
    constexpr uint32_t kNpsMinStats = 16;
    // the tile's on-chain draw-count statistics (Matte and mesh kernels): with
    // them the current pixel's candidates stop zcap sigmas above the expected
    // start of its last sample (next-pixel speculation: 3; PBRT_CI_SCAP otherwise).
    // Not in the one-wave Matte builds: there the statistics cost registers
    // (scratch 128 -> 140 B/lane) and idle lanes do not shorten a step of the
    // VALU-bound walk
    constexpr bool kStats = !kX && (kW > 1 || kDepth < 0);
    // (mesh scenes default to 1.5 sigma: config D chain 535 -> 479 ms, flat from 1 to 2,
    // profiles/r06/mesh_scap/)
    const float zcap = nps_on ? 3.0f : rp.ci_scap >= 0 ? 0.1f * (float)rp.ci_scap : kDepth < 0 ? 1.5f : 0.0f;
    // the ring of a pixel: per lane group, or (kNps) per pixel parity
    auto ring_of = [&](int64_t pix) -> RingEnt* {
        return (RingEnt*)(lds + lay.ring) + (size_t)(nps_on ? (int)(pix & 1) : g) * R;
    };
    auto rpar = [&](int64_t pix) -> int { return nps_on ? (int)(pix & 1) : 0; };
    // (rb0 / rb1 by select, not an indexed array or a reference to the group's
    // copy: either would put the copy in scratch)
    ChainCache* pcs = (ChainCache*)(lds + lay.pcs);   // [2 * group + pixel parity]
    uint16_t* stack = stack_lds + tid;
    const int n = rp.spp, ndims = rp.ndims;
#ifndef PBRT_CI_TAILCAP
#define PBRT_CI_TAILCAP 1
#endif
    // an upper bound of a path's draw count D: the CameraSample's PCG32 draws,
    // then per bounce at most 8 (UniformSampleOneLight's light choice + two 2D
    // samples, the BSDF's 2D sample, the RR draw); with `head` the chain's head
    // and kh its sample, no sample of the pixel starts beyond
    // head + (n - 1 - kh) * dmax, so candidates past that are never on the
    // chain (only a speed bound: the head is always issuable). Config B chain
    // 314.7 -> 310.1 ms, N=8 shard max 127.9 -> 124.8 ms; issuing only up to the
    // tile's largest D so far (+25%) measured the same (profiles/r05/tailcap/)
    const uint32_t dmax = (uint32_t)(camera_draws(ndims) + 8 * (rp.max_depth + 1) + 8);
    const pbrt_camera_desc& cam = *sc.camera;
    const unsigned long long gmask = L >= 64 ? ~0ULL : (((1ULL << (L & 63)) - 1ULL) << (g * L));
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int64_t bs = blk * G + g;
    const uint64_t inc = pcg_inc_of((uint64_t)tile_of_slot(rp, slot_base + (bs < nslots_batch ? bs : 0)));
#ifdef PBRT_CI_DIAG   // diagnostics build (make diag): steps, lane-0 phase clocks, on-chain D histogram
    unsigned long long steps = 0, busy = 0;
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long tprev = clock64();
    auto mark = [&](int k) {
        long long now = clock64();
        ph[k] += (unsigned long long)(now - tprev);
        tprev = now;
    };
    if (tid < 64) dh[tid] = 0;
#define CI_DIAG(x) x
#else
    auto mark = [](int) {};
#define CI_DIAG(x)
#endif
    if (tid < G) {
        const int64_t b = blk * G + tid;
        CiGroup& s = gs[tid];
        s.pi = 0;
        s.kh = 1;
        s.A = s.head = s.nxt = 0;
        s.rb0 = s.rb1 = 0;
        s.nb = s.nnx = 0;
        s.nps = 0;
        s.dcnt = 0;
        s.dsum = s.dsq = 0.0f;
        s.reissue = 0;
        if (b < nslots_batch) {
            int64_t x0, y0, x1, y1;
            tile_bounds(rp, tile_of_slot(rp, slot_base + b), x0, y0, x1, y1);
            Pcg seed;
            pcg_seed(seed, (uint64_t)tile_of_slot(rp, slot_base + b));   // Sampler.Clone(tile), integrator.go:318,328
            s.S = seed.state;
            s.npx = (x1 - x0) * (y1 - y0);
            s.phase = s.npx > 0 ? 0 : 2;
            wb.tile_npx[b] = 0;
        } else {
            s.S = 0;
            s.npx = 0;
            s.phase = 2;
        }
    }
    __syncthreads();

    uint32_t cancel_poll = 0;   // chain steps since the leader last read the cancel flag
    uint64_t last_host_poll = t_begin;   // when this workgroup last read the host flag
    // lane trajectory state
    uint32_t off = kNoOff;
    int opi = -1;   // the pixel the lane's candidate belongs to
    // kX: the trajectory's throughput, etaScale and start state live in LDS
    // (the BSDFX bounce needs their registers; 0 B of scratch)
#ifdef PBRT_CI_LDS_STATE   // experiment: the Matte chain too
    constexpr bool kLdsState = true;
#else
    constexpr bool kLdsState = kX;
#endif
    __shared__ Spec xs_beta[kLdsState ? kT : 1];
    __shared__ double xs_eta[kLdsState ? kT : 1];
    __shared__ uint64_t xs_st0[kLdsState ? kT : 1];
    uint64_t st0_r = 0;
    Spec beta_r = spec(1);
    double eta_r = 1.0;
    uint64_t& st0 = [&]() -> uint64_t& { if constexpr (kLdsState) return xs_st0[tid]; else return st0_r; }();
    Spec& beta = [&]() -> Spec& { if constexpr (kLdsState) return xs_beta[tid]; else return beta_r; }();
    double& eta_scale = [&]() -> double& { if constexpr (kLdsState) return xs_eta[tid]; else return eta_r; }();
    st0 = 0;
    beta = spec(1);
    eta_scale = 1.0;
    bool tracing = false;
    Cursor c;
    c.rri = -1;
    c.rrn = 0;
    c.rng.state = 0;
    c.rng.inc = inc;
    c.draws = 0;
    c.cur1d = c.cur2d = 0;
    c.k = -1;
    c.kdep = 0;
    int bounces = 1;
    Ray ray;
    ray.o = ray.d = V3{0, 0, 0};
    ray.tmax = kInf;
    ray.time = 0;

    for (;;) {
        // ---- (1) groups that need a pixel: StartPixel + bounce 1, one group at a time
        for (int q = 0; q < G; q++) {
            while (gs[q].phase == 0) {
                const int64_t bq = blk * G + q;
                const int64_t tile = tile_of_slot(rp, slot_base + bq);
                const uint64_t incq = pcg_inc_of((uint64_t)tile);
                const int64_t pi = gs[q].pi;
                const int64_t rec = bq * wb.ppt + pi;
                int64_t x0, y0, x1, y1;
                tile_bounds(rp, tile, x0, y0, x1, y1);
                const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
                double* gs1d = wb.s1d + rec * wb.s1d_stride;
                double* sp = s1d ? s1d : gs1d;
                const uint64_t S1 = start_pixel_wave<kSpWin>(rp, J, gs[q].S, incq, sp, other, vbuf, &sh_state, &sh_draws);
                if (s1d)
                    for (int idx = tid; idx < ndims * n; idx += kT) gs1d[idx] = s1d[idx];
                // the first traced sample's camera time value (read before the ring
                // clear: with one tile per workgroup the StartPixel staging aliases the ring)
                const double time_u = sp[1 < n ? 1 : 0];
                __syncthreads();
                // next-pixel speculation already filled this pixel's ring (kNps)
                const bool spec_ran = nps_on && gs[q].nps != 0;
                if (!spec_ran) {
                    RingEnt* rq = nps_on ? ring_of(pi) : (RingEnt*)(lds + lay.ring) + (size_t)q * R;
                    for (uint32_t i = (uint32_t)tid; i < R; i += kT) rq[i].tag = kNoOff;
                }
                // bounce 1 (camera ray, first hit, BSDF) was computed for every
                // pixel record by k_wf_primary; only the ray time needs StartPixel
                PixelRec& pr = wb.prec[rec];
                const int hit0 = pr.hit, panic0 = pr.panic0;
                if (tid == 0) {   // pbrt_gpu_cancel: every group of the workgroup ends
                    if (prog)   // the heartbeat k_gate tells running chains from undispatched ones by
                        __hip_atomic_fetch_add(&prog[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t now = wall_clock64();
                    const bool host = now - last_host_poll >= 100000;   // 1 ms at 100 MHz
                    if (host) last_host_poll = now;
                    if (cancel_requested(sc, host))
                        for (int q2 = 0; q2 < G; q2++) gs[q2].phase = 2;
                }
                if (tid == 0 && gs[q].phase == 0) {
                    if (hit0)   // the camera ray's time (Get1D after pFilm, pLens) of the pixel's first traced sample
                        pr.si.time = camera_ray(cam, (double)px, (double)py, time_u, V2{0.0, 0.0}).time;
                    ChainCache& pq = pcs[2 * q + rpar(pi)];
                    pq.si = pr.si;
                    pq.b = pr.b;
                    if constexpr (kX) pq.x = pr.x;
                    pq.wo = pr.wo;
                    pq.hit = hit0;
                    CiGroup& s = gs[q];
                    s.S = S1;
                    s.A += sh_draws;   // the first traced sample starts after StartPixel's draws
                    s.head = s.A;
                    // (a first sample below the speculation's base: dense issue from the head)
                    s.nxt = (spec_ran && s.A >= s.nb) ? max(s.nnx, s.A) : s.A;
                    if (!spec_ran) {
                        if (rpar(pi)) s.rb1 = s.A;
                        else s.rb0 = s.A;
                    }
                    s.nps = 0;
                    s.kh = 1;
                    s.reissue = 0;
                    wb.tile_npx[bq] = (int32_t)(pi + 1);
                    if (panic0) {   // the first traced sample panics at bounce 1: the tile ends here
                        s.phase = 2;
                    } else if (hit0) {
                        s.phase = 1;
                    } else {   // no traced bounce: every sample is black and draws only its
                        // CameraSample's PCG32 values (n_dims < 2: pLens; c_camera)
                        if (ndims < 2) {
                            s.S = pcg_advance(J, S1, incq, (uint64_t)(n - 1) * camera_draws(ndims));
                            s.A += (uint32_t)(n - 1) * camera_draws(ndims);
                        }
                        s.pi = pi + 1;
                        s.phase = s.pi < s.npx ? 0 : 2;
                    }
                }
                __syncthreads();
            }
        }
        mark(0);
        bool any_chain = false;
        for (int q = 0; q < G; q++) any_chain |= gs[q].phase == 1;
        if (!any_chain) break;
        CI_DIAG(steps++;)

        // ---- (2) idle lanes take the next offsets of their group
        const CiGroup sg = gs[g];
        const int64_t rec = bs * wb.ppt + sg.pi;
        const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, ndims,
                             kX && wb.rrb ? wb.rrb + bs * kCiMaxRing : nullptr};
        {
            const bool idle = sg.phase == 1 && off == kNoOff;
            const unsigned long long m = __ballot(idle) & gmask;
            int nidle = __popcll(m);
            int rank = __popcll(m & lt_mask);
            if (kW > 1) {   // rank the idle lanes across the tile's waves
                if (lane == 0) wcnt[wv] = nidle;
                __syncthreads();
                int before = 0, tot = 0;
                for (int w = 0; w < kW; w++) {
                    const int cw = wcnt[w];
                    before += w < wv ? cw : 0;
                    tot += cw;
                }
                rank += before;
                nidle = tot;
            }
            const int re = (sg.reissue && nidle > 0) ? 1 : 0;
            const uint32_t nx0 = sg.nxt;
            // offsets < head + R keep the ring collision-free
            const int avail = nx0 < sg.head + R ? (int)((sg.head + R - nx0 + cs - 1) / cs) : 0;
#if PBRT_CI_TAILCAP
            const uint32_t tail = sg.head + (uint32_t)(n - 1 - sg.kh) * dmax;
            const int capn = nx0 <= tail ? (int)((tail - nx0) / cs) + 1 : 0;
            int nspec = min(min(nidle - re, avail), capn);
            if (kStats && zcap > 0.0f && sg.dcnt >= kNpsMinStats) {
                // the current pixel's last sample starts near head + rem * mean: a cap
                // zcap sigmas above it (the lanes beyond go to the next pixel, or idle)
                const float rem = (float)(n - 1 - sg.kh);
                const float mu = sg.dsum / (float)sg.dcnt;
                const float sd = sqrtf(fmaxf(0.0f, sg.dsq / (float)sg.dcnt - mu * mu));
                const uint32_t scap = sg.head + (uint32_t)(rem * mu + zcap * sd * sqrtf(rem));
                nspec = min(nspec, nx0 <= scap ? (int)((scap - nx0) / cs) + 1 : 0);
            }
#else
            const int nspec = min(nidle - re, avail);
#endif
            // the lanes left: the next pixel's candidates (stride 1, within its ring's window)
            int nspec1 = 0;
            if (kNps && sg.phase == 1 && sg.nps) {
                const int avail1 = sg.nnx < sg.nb + R ? (int)(sg.nb + R - sg.nnx) : 0;
                nspec1 = max(0, min(nidle - re - max(nspec, 0), avail1));
            }
            uint32_t o = kNoOff;
            bool exact = false;
            int opix = (int)sg.pi;
            if (idle) {
                if (re && rank == 0) {
                    o = sg.head;
                    exact = true;
                } else {
                    rank -= re;
                    if (rank < nspec) {
                        o = nx0 + cs * (uint32_t)rank;
                    } else if (kNps && rank - nspec < nspec1) {
                        o = sg.nnx + (uint32_t)(rank - nspec);
                        opix = (int)sg.pi + 1;
                    }
                }
            }
            if (gl == 0 && sg.phase == 1) {
                gs[g].nxt = nx0 + cs * (uint32_t)max(nspec, 0);
                if (kNps) gs[g].nnx = sg.nnx + (uint32_t)nspec1;
                CI_DIAG(ph[5] += (unsigned long long)(max(nspec, 0) + nspec1 + re);)   // candidate trajectories issued
                CI_DIAG(ph[7] += (unsigned long long)nspec1;)   // of them next-pixel speculation
                if (re) gs[g].reissue = 0;
            }
            if (o != kNoOff) {
                off = o;
                opi = opix;
                st0 = pcg_advance(J, sg.S, inc, (uint64_t)(o - sg.A));
                c.rng.state = st0;
                c.draws = 0;
                c_camera(c, ndims);   // camera: Get2D pFilm, Get2D pLens, Get1D time
                c.k = exact ? sg.kh : -1;
                c.kdep = 0;
                if constexpr (kX) {   // speculative: RR decisions on stratified values are recorded
                    c.rri = (!exact && ss.rrb) ? (int)((off - sg.rb0) & (R - 1u)) : -1;
                    c.rrn = 0;
                }
                beta = spec(1);
                eta_scale = 1.0;
                bounces = 1;
                const ChainCache& pc = pcs[2 * g + rpar(opi)];
                const int r = traj_scatter<kX>(sc, pc.si, pc.b, pc.x, pc.wo, c, ss, beta, eta_scale, bounces, ray,
                                               rp.max_depth, rp.rr_threshold);
                tracing = r == 0;
                if (r != 0) {
                    RingEnt& e = ring_of(opi)[(off - (rpar(opi) ? sg.rb1 : sg.rb0)) & (R - 1u)];
                    e.st = st0;
                    e.d = ring_d<kX>(c, ss, r == 1 ? c.draws : (c.k >= 0 ? kBadExactD : kBadSpecD));
                    e.tag = off;
                    off = kNoOff;
                }
            }
        }
        mark(1);
        CI_DIAG(const unsigned long long tbusy = __ballot(tracing); if (lane == 0) busy += (unsigned long long)__popcll(tbusy);)
        // ---- (3) one bounce of every live trajectory
#ifdef PBRT_CI_DENSE_WALK   // experiment build: the whole wave walks together (dense leaf tests)
        const bool dense = kDepth == 0 && sc.dense_ok && sc.use_lds_nodes;
        int panic = 0, best = -1;
        V3 ph{0, 0, 0};
        if (dense) bvh_walk_dense(sc, ray, tracing, panic, best, ph, dense_lds + (size_t)wv * kDenseScratch);
        if (tracing) {
            if (!dense) bvh_walk<false, kT, PBRT_CHAIN_LB, (kDepth < 0)>(sc, ray, stack, panic, best, ph);
#else
        if (tracing) {
            int panic = 0, best;
            V3 ph;
            bvh_walk<false, kT, PBRT_CHAIN_LB, (kDepth < 0)>(sc, ray, stack, panic, best, ph);
#endif
            mark(2);
            uint32_t d = kNoOff;
            if (panic) {
                d = c.k >= 0 ? kBadExactD : kBadSpecD;
            } else if (best < 0) {
                d = c.draws;
            } else {
                SI si;
                prim_si(sc, best, ray, ph, si);
                BSDF b;
                BSDFX x;
                if ((kX ? compute_bsdf_x(sc, si, b, x) : compute_bsdf(sc, si, b)) < 0) {
                    d = c.k >= 0 ? kBadExactD : kBadSpecD;
                } else {
                    const int r = traj_scatter<kX>(sc, si, b, x, ray.d, c, ss, beta, eta_scale, bounces, ray,
                                                   rp.max_depth, rp.rr_threshold);
                    if (r == 1) d = c.draws;
                    else if (r == 2) d = c.k >= 0 ? kBadExactD : kBadSpecD;
                }
            }
            if (d != kNoOff) {
                RingEnt& e = ring_of(opi)[(off - (rpar(opi) ? sg.rb1 : sg.rb0)) & (R - 1u)];
                e.st = st0;
                e.d = ring_d<kX>(c, ss, d);
                e.tag = off;
                off = kNoOff;
                tracing = false;
            }
        }
        mark(3);
        __syncthreads();
        // ---- (4) each group leader walks its chain through the ring
        if (gl == 0 && sg.phase == 1) {
            CiGroup s = gs[g];
            if ((++cancel_poll & 127u) == 0) {   // long pixels (large spp)
                const uint64_t now = wall_clock64();
                const bool host = now - last_host_poll >= 100000;
                if (host) last_host_poll = now;
                if (cancel_requested(sc, host)) s.phase = 2;
            }
            RingEnt* rcur = ring_of(s.pi);
            const uint32_t rbase = rpar(s.pi) ? s.rb1 : s.rb0;
            for (; s.phase == 1;) {
                RingEnt& e = rcur[(s.head - rbase) & (R - 1u)];
                if (e.tag != s.head) break;
                uint32_t d = e.d;
                if (kX && d < kBadExactD && (d & kRrFlag)) {
                    // the trajectory survived RR decisions on stratified values of
                    // the then unknown sample index: with k = kh the first one whose
                    // value is below its q ends the path there
                    const RrBranches& b = ss.rrb[(s.head - rbase) & (R - 1u)];
                    d = (d & kRrTailBad) == kRrTailBad ? kBadSpecD : (d & kRrTailBad);
                    for (uint32_t i = 0; i < b.n; i++) {
                        const uint32_t cd = b.cd[i];
                        if (ss.s1d[(int)(cd & 0xFFu) * n + s.kh] < b.q[i]) {
                            d = cd >> 8;
                            break;
                        }
                    }
                }
                if (d == kBadSpecD) {   // re-run the head with its sample index known
                    e.tag = kNoOff;
                    s.reissue = 1;
                    break;
                }
                wb.memb[rec * n + s.kh] = e.st;
                if (d == kBadExactD) {   // the exact head's trajectory panics: the tile ends at this sample
                    wb.prec[rec].nvalid = s.kh + 1;
                    s.phase = 2;
                    break;
                }
                CI_DIAG(atomicAdd(&dh[min(d / 2u, 63u)], 1u);)
                // the tail cap's bound (dmax per sample): an on-chain D above it would
                // only slow the chain, never change a result; counted so tests can pin it
                CI_DIAG(if (d > dmax) ph[6]++;)
                CI_DIAG(if (d & 1u) atomicAdd(&ctr->odd_d, 1ull);)
                if (kStats) {   // the tile's draw-count statistics
                    s.dcnt++;
                    s.dsum += (float)d;
                    s.dsq += (float)d * (float)d;
                }
                s.kh++;
                s.head += d;
                if (s.kh >= n) {   // every sample of the pixel has its offset; the next StartPixel starts here
                    s.S = pcg_advance(J, s.S, inc, (uint64_t)(s.head - s.A));
                    s.A = s.head;
                    s.pi++;
                    s.phase = s.pi < s.npx ? 0 : 2;
                    break;
                }
            }
            if (s.nxt < s.head || (cs == 2u && ((s.nxt ^ s.head) & 1u))) s.nxt = s.head;
            // speculate on the next pixel: when the last sample has its offset (its
            // first traced sample then starts at least StartPixel's events past this
            // one), or, with the tile's draw-count statistics, from rp.ci_nps samples
            // before the end (base: 3 sigma below the expected end; a first sample
            // below it only wastes the speculation, the switch then issues from the head)
            int act = 0;
            const int left = n - s.kh;   // samples whose draw counts are still to come, the head's included
            const bool stats = s.dcnt >= kNpsMinStats;
            if (nps_on && s.phase == 1 && !s.nps && (left == 1 || (stats && left <= rp.ci_nps)) &&
                s.pi + 1 < s.npx) {
                const PixelRec& pn = wb.prec[rec + 1];
                if (pn.hit && !pn.panic0) {
                    float lo = 0.0f;
                    if (left > 1) {
                        const float mu = s.dsum / (float)s.dcnt;
                        const float sd = sqrtf(fmaxf(0.0f, s.dsq / (float)s.dcnt - mu * mu));
                        lo = fmaxf(0.0f, (float)left * mu - 3.0f * sd * sqrtf((float)left));
                    }
                    s.nps = 1;
                    s.nb = s.head + (uint32_t)lo + (uint32_t)rp.sp_events;
                    s.nnx = s.nb;
                    if (rpar(s.pi + 1)) s.rb1 = s.nb;
                    else s.rb0 = s.nb;
                    act = 1;
                }
            }
            if (kNps) sh_act = act;
            // write back what the walk changes (a whole-struct store kept the
            // untouched fields of the copy in scratch)
            CiGroup& gw = gs[g];
            gw.S = s.S;
            gw.A = s.A;
            gw.pi = s.pi;
            gw.head = s.head;
            gw.nxt = s.nxt;
            gw.kh = s.kh;
            gw.phase = s.phase;
            gw.reissue = s.reissue;
            if (kStats) {
                gw.dcnt = s.dcnt;
                gw.dsum = s.dsum;
                gw.dsq = s.dsq;
            }
            if (kNps) {
                gw.nps = s.nps;
                gw.nb = s.nb;
                gw.nnx = s.nnx;
                gw.rb0 = s.rb0;
                gw.rb1 = s.rb1;
            }
        }
        if (kNps && tid == 0 && !(gl == 0 && sg.phase == 1)) sh_act = 0;
        __syncthreads();
        if (kNps && sh_act) {   // the next pixel's ring (its parity's: the pixel before this one's) and ChainCache
            const CiGroup s3 = gs[g];
            RingEnt* rn = ring_of(s3.pi + 1);
            for (uint32_t i = (uint32_t)tid; i < R; i += kT) rn[i].tag = kNoOff;
            if (tid == 0) {
                const PixelRec& pn = wb.prec[rec + 1];
                ChainCache& pc = pcs[2 * g + rpar(s3.pi + 1)];
                pc.si = pn.si;
                pc.b = pn.b;
                pc.wo = pn.wo;
                pc.hit = pn.hit;
            }
        }
        // ---- (5) drop candidates the chain has left behind
        if (off != kNoOff) {
            const CiGroup s2 = gs[g];
            bool keep = false;
            if (opi == s2.pi && s2.phase == 1)   // the current pixel
                keep = !(off < s2.head || (cs == 2u && ((off ^ s2.head) & 1u)) ||
                         (PBRT_CI_TAILCAP && off > s2.head + (uint32_t)(n - 1 - s2.kh) * dmax));
            else if (kNps && opi == s2.pi && s2.phase == 0)   // speculated for the pixel whose StartPixel is next
                keep = s2.nps != 0;
            else if (kNps && opi == s2.pi + 1 && s2.phase == 1)   // the next pixel's speculation
                keep = s2.nps != 0;
            if (!keep) {
                off = kNoOff;
                tracing = false;
            }
        }
        mark(4);
    }
#ifdef PBRT_CI_DIAG
    __syncthreads();
    if (tid < 64 && dh[tid]) atomicAdd(&ctr->dhist[tid], (unsigned long long)dh[tid]);
    if (tid == 0) {
        atomicAdd(&ctr->windows, steps);
        for (int k = 0; k < 8; k++) atomicAdd(&ctr->phase[k], ph[k]);
        atomicAdd(&ctr->nps_issued, ph[7]);
    }
    if (lane == 0) atomicAdd(&ctr->busy, busy);
#endif
#undef CI_DIAG
    if (prog) {   // every thread's writes of this tile (records, sample states) reach L2 first
        __threadfence();
        __syncthreads();
    }
    if (tid == 0) {
        if (prog && G == 1 && bs < nslots_batch) {   // publish the tile for the path stage
            const uint32_t pos = __hip_atomic_fetch_add(&prog[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&prog[kProgHead + pos], (uint32_t)bs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (ticks && G == 1 && bs < nslots_batch) {
            const uint64_t t_end = wall_clock64();
            ticks[bs] = (uint32_t)min(t_end - t_begin, (uint64_t)0xFFFFFFFFu);
#ifdef PBRT_CI_DIAG   // start and end clocks (low 32 bits) for the occupancy timeline
            ticks[nslots_batch + bs] = (uint32_t)t_begin;
            ticks[2 * nslots_batch + bs] = (uint32_t)t_end;
#endif
        }
    }
}

}  // namespace pbrtk
