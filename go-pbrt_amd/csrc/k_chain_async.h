// k_chain_async.h — k_chain_async, the continuous-issue offset chain with
// asynchronous waves (EXACT mode, kW > 1 waves per tile); instantiated in k_chain_a.hip
//
// k_chain_ci steps all kW waves of a tile together: every step ends at a
// workgroup barrier, so a step lasts as long as the slowest wave's bounce, and
// at 8 waves per tile the heaviest tiles of a multi-GPU shard become barrier
// bound. Here each wave runs its own loop -- drop, issue, one bounce, ring
// write, walk -- and the waves meet only when the tile's chain reaches a new
// pixel (StartPixel is a workgroup operation):
//   - offsets are reserved from the shared next-offset counter with a
//     compare-and-swap (stride 1), below head + R so that a live offset owns its
//     ring slot;
//   - a ring entry is one 64-bit word ((offset + 1) << 32 | D), written with an
//     LDS atomic max: a lane the chain has already left behind (offset - R)
//     can never overwrite the entry of the live offset that shares its slot;
//   - the walk (the chain head through the resolved entries, as k_chain_ci's
//     leader does) is taken by whichever wave gets the walk lock; it tracks the
//     head's PCG32 state itself (advance by D), so entries carry no state;
//   - a speculative entry that could not resolve D (kBadSpecD) is cleared and
//     the head re-run with its sample index by the next wave with an idle lane.
// Results are those of k_chain_ci (the same offsets, draw counts and states
// reach wb.memb); only the schedule differs. Matte pipelines (kX = false).
#pragma once
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

__device__ __forceinline__ uint32_t lds_load32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int lds_load32(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store32(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store32(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int kW, int kDepth, bool kX>
__global__ __launch_bounds__(kWave * kW) __attribute__((amdgpu_waves_per_eu(kDepth < 0 ? PBRT_CI_MESH_EU_WAVES : PBRT_CI_EU_WAVES, 8))) void k_chain_async(
    DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
    int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr,
    const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride) {
    static_assert(kW > 1 && !kX, "k_chain_async: multi-wave Matte tiles");
    (void)lanes_per_tile;
    (void)ctr;
    (void)cstride;   // stride 1
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint64_t t_begin = wall_clock64();
    constexpr int kT = kWave * kW;
    __shared__ uint16_t stack_lds[kDepth > 0 ? kDepth * kT : 1];
    __shared__ CiGroup gs0;
    __shared__ uint64_t sh_state;
    __shared__ uint64_t st_head;   // PCG32 state at the head offset (the walker's)
    __shared__ uint32_t walk_lock;
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    stage_nodes(sc);
    const int64_t blk = order ? (int64_t)order[blockIdx.x] : (int64_t)blockIdx.x;
    const uint32_t R = (uint32_t)ring_size;   // a power of two
    const PcgJump& J = *jump;
    double* s1d = lay.s1d >= 0 ? (double*)(lds + lay.s1d) : nullptr;
    uint16_t* other = (uint16_t*)(lds + lay.other);
    uint32_t* vbuf = (uint32_t*)(lds + lay.vbuf);
    unsigned long long* ring = (unsigned long long*)(lds + lay.ring);   // (offset + 1) << 32 | D; 0 empty
    ChainCache* pcs = (ChainCache*)(lds + lay.pcs);
    uint16_t* stack = stack_lds + tid;
    const int n = rp.spp, ndims = rp.ndims;
    const pbrt_camera_desc& cam = *sc.camera;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int64_t bs = blk;
    const uint64_t inc = pcg_inc_of((uint64_t)tile_of_slot(rp, slot_base + (bs < nslots_batch ? bs : 0)));
    if (tid == 0) {
        CiGroup& s = gs0;
        s.pi = 0;
        s.kh = 1;
        s.head = s.nxt = 0;
        s.reissue = 0;
        walk_lock = 0;
        if (bs < nslots_batch) {
            int64_t x0, y0, x1, y1;
            tile_bounds(rp, tile_of_slot(rp, slot_base + bs), x0, y0, x1, y1);
            Pcg seed;
            pcg_seed(seed, (uint64_t)tile_of_slot(rp, slot_base + bs));   // Sampler.Clone(tile), integrator.go:318,328
            s.S = seed.state;
            s.npx = (x1 - x0) * (y1 - y0);
            s.phase = s.npx > 0 ? 0 : 2;
            wb.tile_npx[bs] = 0;
        } else {
            s.S = 0;
            s.npx = 0;
            s.phase = 2;
        }
    }
    __syncthreads();

    uint32_t walks = 0;                  // this wave's walks since its last cancel poll
    uint64_t last_host_poll = t_begin;   // when this wave last read the host flag
    uint32_t off = kNoOff;
    bool tracing = false;
    Cursor c;
    c.rri = -1;
    c.rng.state = 0;
    c.rng.inc = inc;
    c.draws = 0;
    c.cur1d = c.cur2d = 0;
    c.k = -1;
    c.kdep = 0;
    Spec beta = spec(1);
    double eta_scale = 1.0;
    int bounces = 1;
    Ray ray;
    ray.o = ray.d = V3{0, 0, 0};
    ray.tmax = kInf;
    ray.time = 0;

    for (;;) {
        const int phase = __builtin_amdgcn_readfirstlane(lds_load32(&gs0.phase));
        if (phase == 2) break;
        if (phase == 0) {
            // ---- a new pixel. Only the walker moves the phase off 1, and nothing
            // moves it off 0 before every wave is here: each wave meets this
            // barrier once its iteration ends (the StartPixel staging aliases the ring)
            __syncthreads();
            off = kNoOff;
            tracing = false;
            for (int again = 1; again;) {
                const int64_t tile = tile_of_slot(rp, slot_base + bs);
                const int64_t pi = gs0.pi;
                const int64_t rec = bs * wb.ppt + pi;
                int64_t x0, y0, x1, y1;
                tile_bounds(rp, tile, x0, y0, x1, y1);
                const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
                double* gs1d = wb.s1d + rec * wb.s1d_stride;
                double* sp = s1d ? s1d : gs1d;
                const uint64_t S1 = start_pixel_wave(rp, J, gs0.S, inc, sp, other, vbuf, &sh_state);
                if (s1d)
                    for (int idx = tid; idx < ndims * n; idx += kT) gs1d[idx] = s1d[idx];
                const double time_u = sp[1 < n ? 1 : 0];
                __syncthreads();
                for (uint32_t i = (uint32_t)tid; i < R; i += kT) ring[i] = 0ULL;
                PixelRec& pr = wb.prec[rec];
                const int hit0 = pr.hit, panic0 = pr.panic0;
                if (tid == 0) {   // pbrt_gpu_cancel
                    const uint64_t now = wall_clock64();
                    const bool host = now - last_host_poll >= 100000;   // 1 ms at 100 MHz
                    if (host) last_host_poll = now;
                    if (cancel_requested(sc, host)) gs0.phase = 2;
                }
                if (tid == 0 && gs0.phase == 0) {
                    if (hit0)   // the camera ray's time of the pixel's first traced sample
                        pr.si.time = camera_ray(cam, (double)px, (double)py, time_u, V2{0.0, 0.0}).time;
                    pcs[0].si = pr.si;
                    pcs[0].b = pr.b;
                    pcs[0].wo = pr.wo;
                    pcs[0].hit = hit0;
                    CiGroup& s = gs0;
                    s.S = S1;
                    st_head = S1;
                    s.head = s.nxt = 0;
                    s.kh = 1;
                    s.reissue = 0;
                    wb.tile_npx[bs] = (int32_t)(pi + 1);
                    if (panic0) {   // the first traced sample panics at bounce 1: the tile ends here
                        s.phase = 2;
                    } else if (hit0) {
                        s.phase = 1;
                    } else {   // no traced bounce: every sample is black and draws nothing
                        s.pi = pi + 1;
                        s.phase = s.pi < s.npx ? 0 : 2;
                    }
                }
                __syncthreads();
                again = gs0.phase == 0;
                __syncthreads();   // every wave has read the phase before any wave's walker can move it
            }
            continue;
        }

        // ---- phase 1: one iteration of this wave
        const int64_t rec = bs * wb.ppt + gs0.pi;   // the pixel changes only at the barrier above
        const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, ndims, nullptr};
        // (a) candidates the chain has left behind
        if (off != kNoOff && off < lds_load32(&gs0.head)) {
            off = kNoOff;
            tracing = false;
        }
        // (b) idle lanes take the next offsets (one reservation per wave)
        uint32_t d = kNoOff;   // D of a trajectory that ends in this iteration
        {
            const bool idle = off == kNoOff;
            const unsigned long long m = __ballot(idle);
            const int nidle = __popcll(m);
            if (nidle > 0) {
                int re = 0, kh = 0, k = 0;
                uint32_t base = 0, hre = 0;
                if (lane == 0) {
                    re = __hip_atomic_exchange(&gs0.reissue, 0, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (re) {   // the walker waits at the head until this exact run's entry lands
                        hre = lds_load32(&gs0.head);
                        kh = lds_load32(&gs0.kh);
                    }
                    uint32_t cur = lds_load32(&gs0.nxt);
                    for (;;) {
                        const uint32_t h = lds_load32(&gs0.head);
                        const uint32_t b0 = cur > h ? cur : h;
                        const int want = b0 < h + R ? min(nidle - re, (int)(h + R - b0)) : 0;
                        if (want <= 0) break;
                        uint32_t expect = cur;
                        if (__hip_atomic_compare_exchange_strong(&gs0.nxt, &expect, b0 + (uint32_t)want,
                                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
                            base = b0;
                            k = want;
                            break;
                        }
                        cur = expect;
                    }
                }
                re = __shfl(re, 0);
                kh = __shfl(kh, 0);
                k = __shfl(k, 0);
                base = (uint32_t)__shfl((int)base, 0);
                hre = (uint32_t)__shfl((int)hre, 0);
                int rank = __popcll(m & lt_mask);
                uint32_t o = kNoOff;
                bool exact = false;
                if (idle) {
                    if (re && rank == 0) {
                        o = hre;
                        exact = true;
                    } else {
                        rank -= re;
                        if (rank < k) o = base + (uint32_t)rank;
                    }
                }
                if (o != kNoOff) {
                    off = o;
                    c.rng.state = pcg_advance(J, gs0.S, inc, (uint64_t)o);
                    c.draws = 0;
                    c.cur1d = 1;   // camera: Get2D pFilm, Get2D pLens, Get1D time (stratified)
                    c.cur2d = 2;
                    c.k = exact ? kh : -1;
                    c.kdep = 0;
                    beta = spec(1);
                    eta_scale = 1.0;
                    bounces = 1;
                    const ChainCache& pc = pcs[0];
                    const int r = traj_scatter<kX>(sc, pc.si, pc.b, pc.x, pc.wo, c, ss, beta, eta_scale, bounces,
                                                   ray, rp.max_depth, rp.rr_threshold);
                    tracing = r == 0;
                    if (r != 0) d = r == 1 ? c.draws : (c.k >= 0 ? kBadExactD : kBadSpecD);
                }
            }
        }
        // (c) one bounce of every live trajectory of the wave
        if (tracing) {
            int panic = 0, best;
            V3 ph;
            bvh_walk<false, kT, PBRT_CHAIN_LB, (kDepth < 0)>(sc, ray, stack, panic, best, ph);
            if (panic) {
                d = c.k >= 0 ? kBadExactD : kBadSpecD;
            } else if (best < 0) {
                d = c.draws;
            } else {
                SI si;
                prim_si(sc, best, ray, ph, si);
                BSDF b;
                BSDFX x;
                if (compute_bsdf(sc, si, b) < 0) {
                    d = c.k >= 0 ? kBadExactD : kBadSpecD;
                } else {
                    const int r = traj_scatter<kX>(sc, si, b, x, ray.d, c, ss, beta, eta_scale, bounces, ray,
                                                   rp.max_depth, rp.rr_threshold);
                    if (r == 1) d = c.draws;
                    else if (r == 2) d = c.k >= 0 ? kBadExactD : kBadSpecD;
                }
            }
        }
        // (d) ring entries of the trajectories that ended (an older offset of the
        // same slot can never win the max against a live one)
        if (d != kNoOff) {
            if (off >= lds_load32(&gs0.head))
                __hip_atomic_fetch_max(&ring[off & (R - 1u)], ((unsigned long long)(off + 1u) << 32) | d,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            off = kNoOff;
            tracing = false;
        }
        // (e) the walk, by whichever wave holds the lock
        if (lane == 0) {
            uint32_t unlocked = 0;
            if (__hip_atomic_compare_exchange_strong(&walk_lock, &unlocked, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
                if (gs0.phase == 1) {
                    CiGroup s = gs0;
                    uint64_t st = st_head;
                    uint32_t head = lds_load32(&gs0.head);
                    int kh = lds_load32(&gs0.kh);
                    int ph = 1, set_re = 0;
                    if ((++walks & 127u) == 0) {   // long pixels (large spp)
                        const uint64_t now = wall_clock64();
                        const bool host = now - last_host_poll >= 100000;
                        if (host) last_host_poll = now;
                        if (cancel_requested(sc, host)) ph = 2;
                    }
                    for (; ph == 1;) {
                        unsigned long long* e = &ring[head & (R - 1u)];
                        const unsigned long long v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if ((uint32_t)(v >> 32) != head + 1u) break;
                        const uint32_t dv = (uint32_t)v;
                        if (dv == kBadSpecD) {   // re-run the head with its sample index known
                            __hip_atomic_store(e, 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            set_re = 1;   // published after the head it refers to
                            break;
                        }
                        wb.memb[rec * n + kh] = st;
                        if (dv == kBadExactD) {   // the exact head's trajectory panics: the tile ends at this sample
                            wb.prec[rec].nvalid = kh + 1;
                            ph = 2;
                            break;
                        }
                        kh++;
                        head += dv;
                        st = pcg_advance(J, st, inc, (uint64_t)dv);
                        if (kh >= n) {   // every sample of the pixel has its offset; the next StartPixel starts here
                            s.S = st;
                            s.pi++;
                            ph = s.pi < s.npx ? 0 : 2;
                            break;
                        }
                    }
                    st_head = st;
                    gs0.S = s.S;
                    gs0.pi = s.pi;
                    lds_store32(&gs0.kh, kh);
                    lds_store32(&gs0.head, head);
                    lds_store32(&gs0.phase, ph);
                    if (set_re) __hip_atomic_store(&gs0.reissue, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                __hip_atomic_store(&walk_lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (!__any(tracing)) {   // nothing in flight: let the tile's other waves issue
            __builtin_amdgcn_s_sleep(1);
            // watchdog: a tile whose chain has not ended after 60 s ends here (the
            // frame is then wrong, never hung)
            if (lane == 0 && wall_clock64() - t_begin > 6000000000ull) {
                int one = 1;
                __hip_atomic_compare_exchange_strong(&gs0.phase, &one, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    if (tid == 0 && ticks && bs < nslots_batch)
        ticks[bs] = (uint32_t)min(wall_clock64() - t_begin, (uint64_t)0xFFFFFFFFu);
}

}  // namespace pbrtk
