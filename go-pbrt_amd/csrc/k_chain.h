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
    // null elsewhere): [0] workgroups started, [1] completions, [2 + i] the slot of
    // the i-th completion
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
    RingEnt* ring = (RingEnt*)(lds + lay.ring) + (size_t)g * R;
    ChainCache* pcs = (ChainCache*)(lds + lay.pcs);
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
    unsigned long long steps = 0;
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
        s.head = s.nxt = 0;
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
                const uint64_t S1 = start_pixel_wave<kSpWin>(rp, J, gs[q].S, incq, sp, other, vbuf, &sh_state);
                if (s1d)
                    for (int idx = tid; idx < ndims * n; idx += kT) gs1d[idx] = s1d[idx];
                // the first traced sample's camera time value (read before the ring
                // clear: with one tile per workgroup the StartPixel staging aliases the ring)
                const double time_u = sp[1 < n ? 1 : 0];
                __syncthreads();
                RingEnt* rq = (RingEnt*)(lds + lay.ring) + (size_t)q * R;
                for (uint32_t i = (uint32_t)tid; i < R; i += kT) rq[i].tag = kNoOff;
                // bounce 1 (camera ray, first hit, BSDF) was computed for every
                // pixel record by k_wf_primary; only the ray time needs StartPixel
                PixelRec& pr = wb.prec[rec];
                const int hit0 = pr.hit, panic0 = pr.panic0;
                if (tid == 0) {   // pbrt_gpu_cancel: every group of the workgroup ends
                    const uint64_t now = wall_clock64();
                    const bool host = now - last_host_poll >= 100000;   // 1 ms at 100 MHz
                    if (host) last_host_poll = now;
                    if (cancel_requested(sc, host))
                        for (int q2 = 0; q2 < G; q2++) gs[q2].phase = 2;
                }
                if (tid == 0 && gs[q].phase == 0) {
                    if (hit0)   // the camera ray's time (Get1D after pFilm, pLens) of the pixel's first traced sample
                        pr.si.time = camera_ray(cam, (double)px, (double)py, time_u, V2{0.0, 0.0}).time;
                    pcs[q].si = pr.si;
                    pcs[q].b = pr.b;
                    if constexpr (kX) pcs[q].x = pr.x;
                    pcs[q].wo = pr.wo;
                    pcs[q].hit = hit0;
                    CiGroup& s = gs[q];
                    s.S = S1;
                    s.head = s.nxt = 0;
                    s.kh = 1;
                    s.reissue = 0;
                    wb.tile_npx[bq] = (int32_t)(pi + 1);
                    if (panic0) {   // the first traced sample panics at bounce 1: the tile ends here
                        s.phase = 2;
                    } else if (hit0) {
                        s.phase = 1;
                    } else {   // no traced bounce: every sample is black and draws only its
                        // CameraSample's PCG32 values (n_dims < 2: pLens; c_camera)
                        if (ndims < 2) s.S = pcg_advance(J, S1, incq, (uint64_t)(n - 1) * camera_draws(ndims));
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
            const int nspec = min(min(nidle - re, avail), capn);
#else
            const int nspec = min(nidle - re, avail);
#endif
            uint32_t o = kNoOff;
            bool exact = false;
            if (idle) {
                if (re && rank == 0) {
                    o = sg.head;
                    exact = true;
                } else {
                    rank -= re;
                    if (rank < nspec) o = nx0 + cs * (uint32_t)rank;
                }
            }
            if (gl == 0 && sg.phase == 1) {
                gs[g].nxt = nx0 + cs * (uint32_t)max(nspec, 0);
                CI_DIAG(ph[5] += (unsigned long long)(max(nspec, 0) + re);)   // candidate trajectories issued
                if (re) gs[g].reissue = 0;
            }
            if (o != kNoOff) {
                off = o;
                st0 = pcg_advance(J, sg.S, inc, (uint64_t)o);
                c.rng.state = st0;
                c.draws = 0;
                c_camera(c, ndims);   // camera: Get2D pFilm, Get2D pLens, Get1D time
                c.k = exact ? sg.kh : -1;
                c.kdep = 0;
                if constexpr (kX) {   // speculative: RR decisions on stratified values are recorded
                    c.rri = (!exact && ss.rrb) ? (int)(off & (R - 1u)) : -1;
                    c.rrn = 0;
                }
                beta = spec(1);
                eta_scale = 1.0;
                bounces = 1;
                const ChainCache& pc = pcs[g];
                const int r = traj_scatter<kX>(sc, pc.si, pc.b, pc.x, pc.wo, c, ss, beta, eta_scale, bounces, ray,
                                               rp.max_depth, rp.rr_threshold);
                tracing = r == 0;
                if (r != 0) {
                    RingEnt& e = ring[off & (R - 1u)];
                    e.st = st0;
                    e.d = ring_d<kX>(c, ss, r == 1 ? c.draws : (c.k >= 0 ? kBadExactD : kBadSpecD));
                    e.tag = off;
                    off = kNoOff;
                }
            }
        }
        mark(1);
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
                RingEnt& e = ring[off & (R - 1u)];
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
            for (; s.phase == 1;) {
                RingEnt& e = ring[s.head & (R - 1u)];
                if (e.tag != s.head) break;
                uint32_t d = e.d;
                if (kX && d < kBadExactD && (d & kRrFlag)) {
                    // the trajectory survived RR decisions on stratified values of
                    // the then unknown sample index: with k = kh the first one whose
                    // value is below its q ends the path there
                    const RrBranches& b = ss.rrb[s.head & (R - 1u)];
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
                s.kh++;
                s.head += d;
                if (s.kh >= n) {   // every sample of the pixel has its offset; the next StartPixel starts here
                    s.S = pcg_advance(J, s.S, inc, (uint64_t)s.head);
                    s.pi++;
                    s.phase = s.pi < s.npx ? 0 : 2;
                    break;
                }
            }
            if (s.nxt < s.head || (cs == 2u && ((s.nxt ^ s.head) & 1u))) s.nxt = s.head;
            gs[g] = s;
        }
        __syncthreads();
        // ---- (5) drop candidates the chain has left behind
        if (off != kNoOff) {
            const CiGroup s2 = gs[g];
            if (s2.phase != 1 || off < s2.head || (cs == 2u && ((off ^ s2.head) & 1u)) || s2.pi != sg.pi ||
                (PBRT_CI_TAILCAP && off > s2.head + (uint32_t)(n - 1 - s2.kh) * dmax)) {
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
    }
#endif
#undef CI_DIAG
    if (prog) {   // every thread's writes of this tile (records, sample states) reach L2 first
        __threadfence();
        __syncthreads();
    }
    if (tid == 0) {
        if (prog && G == 1 && bs < nslots_batch) {   // publish the tile for the path stage
            const uint32_t pos = __hip_atomic_fetch_add(&prog[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&prog[2 + pos], (uint32_t)bs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
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
