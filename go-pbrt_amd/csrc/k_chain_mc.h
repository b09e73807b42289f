// k_chain_mc.h — k_chain_mc: one tile's offset chain on several CUs (EXACT mode);
// instantiated in k_chain_a.hip
//
// A tile's chain is the frame's unit of latency: a multi-GPU shard ends when
// its heaviest tile's chain does, and one workgroup runs on one CU, so
// k_chain_ci / k_chain_async cannot give a tile more than a CU's 4 SIMDs
// (tile 5389 of config B: 282 / 118 / 92 ms at 1 / 4 / 8 waves). Here M
// workgroups of kW waves, on M CUs, share one tile's chain through global
// memory: the asynchronous-wave protocol of k_chain_async (k_chain_async.h)
// with its shared state -- next-offset counter, chain head, walk lock, offset
// ring -- in a McTile record and a ring in HBM, accessed with agent-scope
// atomics (L2). The workgroups meet at a pixel's end (a barrier on the
// record's counters): workgroup 0 runs StartPixel for the next pixel, writes
// its stratified values and the pixel record, and every workgroup then
// stages the pixel's bounce-1 cache in its own LDS.
//
// Forward progress: the host launches at most one workgroup per CU for this
// kernel (grid <= CUs), so every workgroup of a tile is resident together;
// every spin (barrier, ring-full issue) has a 60 s watchdog that ends the
// tile (a wrong frame, never a hung GPU).
// Results are k_chain_ci's: the same offsets, draw counts and states reach wb.memb.
#pragma once
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

__device__ __forceinline__ uint32_t g_load32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_load32(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store32(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store32(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_load64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint64_t kMcWatchdog = 6000000000ull;   // 60 s at 100 MHz

// The M workgroups of a tile meet (every thread of each calls it). Returns
// false if the watchdog fired (the tile is then ended).
__device__ bool mc_barrier(McTile* t, int M, uint64_t t_begin) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // this thread's global writes reach L2 first
    __syncthreads();
    __shared__ int ok_sh;
    if (threadIdx.x == 0) {
        int ok = 1;
        const uint32_t gen = __hip_atomic_load(&t->bar_gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t arrived = __hip_atomic_fetch_add(&t->bar_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == (uint32_t)M - 1u) {
            __hip_atomic_store(&t->bar_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&t->bar_gen, gen + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(&t->bar_gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t_begin > kMcWatchdog) {
                    ok = 0;
                    break;
                }
            }
        }
        ok_sh = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the other CUs' writes (L1 invalidate)
    return ok_sh != 0;
}

template <int kW, int kDepth, bool kX>
__global__ __launch_bounds__(kWave * kW) __attribute__((amdgpu_waves_per_eu(kDepth < 0 ? PBRT_CI_MESH_EU_WAVES : PBRT_CI_EU_WAVES, 8))) void k_chain_mc(
    DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
    int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M,
    const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks) {
    static_assert(!kX, "k_chain_mc: Matte pipelines");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint64_t t_begin = wall_clock64();
    constexpr int kT = kWave * kW;
    __shared__ uint16_t stack_lds[kDepth > 0 ? kDepth * kT : 1];
    __shared__ uint64_t sh_state;
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    stage_nodes(sc);
    const int ti = (int)(blockIdx.x / (unsigned)M), part = (int)(blockIdx.x % (unsigned)M);
    const int64_t bs = order ? (int64_t)order[ti] : (int64_t)ti;   // the tile slot
    McTile* t = tiles + ti;
    const uint32_t R = (uint32_t)ring_size;   // a power of two
    unsigned long long* ring = rings + (size_t)ti * R;   // (offset + 1) << 32 | D; 0 empty (host-zeroed)
    const PcgJump& J = *jump;
    double* s1d = lay.s1d >= 0 ? (double*)(lds + lay.s1d) : nullptr;
    uint16_t* other = (uint16_t*)(lds + lay.other);
    uint32_t* vbuf = (uint32_t*)(lds + lay.vbuf);
    ChainCache* pcs = (ChainCache*)(lds + lay.pcs);
    uint16_t* stack = stack_lds + tid;
    const int n = rp.spp, ndims = rp.ndims;
    const pbrt_camera_desc& cam = *sc.camera;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const uint64_t inc = pcg_inc_of((uint64_t)tile_of_slot(rp, slot_base + (bs < nslots_batch ? bs : 0)));
    // the record is zeroed by the host; workgroup 0 fills it before the first meeting
    if (part == 0 && tid == 0) {
        t->pi = 0;
        t->kh = 1;
        t->head = t->nxt = 0;
        t->reissue = 0;
        t->walk_lock = 0;
        if (bs < nslots_batch) {
            int64_t x0, y0, x1, y1;
            tile_bounds(rp, tile_of_slot(rp, slot_base + bs), x0, y0, x1, y1);
            Pcg seed;
            pcg_seed(seed, (uint64_t)tile_of_slot(rp, slot_base + bs));   // Sampler.Clone(tile), integrator.go:318,328
            t->S = seed.state;
            t->npx = (x1 - x0) * (y1 - y0);
            t->phase = t->npx > 0 ? 0 : 2;
            wb.tile_npx[bs] = 0;
        } else {
            t->S = 0;
            t->npx = 0;
            t->phase = 2;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    bool alive = mc_barrier(t, M, t_begin);

    uint32_t walks = 0;
    uint64_t last_host_poll = t_begin;
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
    uint64_t S = 0;        // the pixel's offset-0 state (fixed between meetings)
    int64_t rec = 0;       // the pixel's record

    while (alive) {
        const int phase = __builtin_amdgcn_readfirstlane(g_load32(&t->phase));
        if (phase == 2) break;
        if (phase == 0) {
            // ---- a new pixel: every wave of every workgroup meets here (only a
            // walker moves the phase off 1, and nothing moves it off 0 before the meeting)
            off = kNoOff;
            tracing = false;
            if (!mc_barrier(t, M, t_begin)) break;   // no ring writes or walks in flight past this point
            if (part == 0) {
                for (int again = 1; again;) {
                    const int64_t tile = tile_of_slot(rp, slot_base + bs);
                    const int64_t pi = t->pi;
                    const int64_t prec_i = bs * wb.ppt + pi;
                    int64_t x0, y0, x1, y1;
                    tile_bounds(rp, tile, x0, y0, x1, y1);
                    const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
                    double* gs1d = wb.s1d + prec_i * wb.s1d_stride;
                    double* sp = s1d ? s1d : gs1d;
                    const uint64_t S1 = start_pixel_wave(rp, J, t->S, inc, sp, other, vbuf, &sh_state);
                    if (s1d)
                        for (int idx = tid; idx < ndims * n; idx += kT) gs1d[idx] = s1d[idx];
                    const double time_u = sp[1 < n ? 1 : 0];
                    for (uint32_t i = (uint32_t)tid; i < R; i += kT) ring[i] = 0ULL;
                    PixelRec& pr = wb.prec[prec_i];
                    const int hit0 = pr.hit, panic0 = pr.panic0;
                    __syncthreads();
                    if (tid == 0) {
                        int ph = 0;
                        const uint64_t now = wall_clock64();
                        const bool host = now - last_host_poll >= 100000;   // 1 ms at 100 MHz
                        if (host) last_host_poll = now;
                        if (cancel_requested(sc, host)) {
                            ph = 2;
                        } else {
                            if (hit0)   // the camera ray's time of the pixel's first traced sample
                                pr.si.time = camera_ray(cam, (double)px, (double)py, time_u, V2{0.0, 0.0}).time;
                            t->S = S1;
                            t->st_head = S1;
                            t->head = t->nxt = 0;
                            t->kh = 1;
                            t->reissue = 0;
                            wb.tile_npx[bs] = (int32_t)(pi + 1);
                            if (panic0) {   // the first traced sample panics at bounce 1: the tile ends here
                                ph = 2;
                            } else if (hit0) {
                                ph = 1;
                            } else {   // no traced bounce: every sample is black and draws nothing
                                t->pi = pi + 1;
                                ph = t->pi < t->npx ? 0 : 2;
                            }
                        }
                        t->phase = ph;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    }
                    __syncthreads();
                    again = t->phase == 0;
                    __syncthreads();
                }
            }
            if (!mc_barrier(t, M, t_begin)) break;   // workgroup 0's pixel is published
            if (g_load32(&t->phase) == 1) {
                rec = bs * wb.ppt + t->pi;
                S = g_load64(&t->S);
                if (tid == 0) {
                    const PixelRec& pr = wb.prec[rec];
                    pcs[0].si = pr.si;
                    pcs[0].b = pr.b;
                    pcs[0].wo = pr.wo;
                    pcs[0].hit = pr.hit;
                }
            }
            // every wave has read the phase before any walker can move it again
            if (!mc_barrier(t, M, t_begin)) break;
            continue;
        }

        // ---- phase 1: one iteration of this wave
        const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, ndims, nullptr};
        if (off != kNoOff && off < g_load32(&t->head)) {   // left behind by the chain
            off = kNoOff;
            tracing = false;
        }
        uint32_t d = kNoOff;
        {
            const bool idle = off == kNoOff;
            const unsigned long long m = __ballot(idle);
            const int nidle = __popcll(m);
            if (nidle > 0) {
                int re = 0, kh = 0, k = 0;
                uint32_t base = 0, hre = 0;
                if (lane == 0) {
                    if (g_load32(&t->reissue))
                        re = __hip_atomic_exchange(&t->reissue, 0, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                    if (re) {   // the walkers wait at the head until this exact run's entry lands
                        hre = g_load32(&t->head);
                        kh = g_load32(&t->kh);
                    }
                    uint32_t cur = g_load32(&t->nxt);
                    for (;;) {
                        const uint32_t h = g_load32(&t->head);
                        const uint32_t b0 = cur > h ? cur : h;
                        const int want = b0 < h + R ? min(nidle - re, (int)(h + R - b0)) : 0;
                        if (want <= 0) break;
                        uint32_t expect = cur;
                        if (__hip_atomic_compare_exchange_strong(&t->nxt, &expect, b0 + (uint32_t)want, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
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
                    c.rng.state = pcg_advance(J, S, inc, (uint64_t)o);
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
        if (d != kNoOff) {   // an older offset of the same slot never wins the max against a live one
            if (off >= g_load32(&t->head))
                __hip_atomic_fetch_max(&ring[off & (R - 1u)], ((unsigned long long)(off + 1u) << 32) | d,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            off = kNoOff;
            tracing = false;
        }
        // the walk, by whichever wave of the tile holds the lock
        if (lane == 0) {
            uint32_t unlocked = 0;
            if (g_load32(&t->walk_lock) == 0 &&
                __hip_atomic_compare_exchange_strong(&t->walk_lock, &unlocked, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                if (g_load32(&t->phase) == 1) {
                    uint64_t st = g_load64(&t->st_head);
                    uint32_t head = g_load32(&t->head);
                    int kh = g_load32(&t->kh);
                    int ph = 1, set_re = 0;
                    int64_t pi = t->pi;
                    if ((++walks & 127u) == 0) {
                        const uint64_t now = wall_clock64();
                        const bool host = now - last_host_poll >= 100000;
                        if (host) last_host_poll = now;
                        if (cancel_requested(sc, host)) ph = 2;
                    }
                    if (wall_clock64() - t_begin > kMcWatchdog) ph = 2;
                    for (; ph == 1;) {
                        unsigned long long* e = &ring[head & (R - 1u)];
                        const unsigned long long v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((uint32_t)(v >> 32) != head + 1u) break;
                        const uint32_t dv = (uint32_t)v;
                        if (dv == kBadSpecD) {   // re-run the head with its sample index known
                            __hip_atomic_store(e, 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            set_re = 1;
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
                        if (kh >= n) {   // the pixel's offsets are complete; the next StartPixel starts here
                            g_store64(&t->S, st);
                            pi++;
                            ph = pi < t->npx ? 0 : 2;
                            break;
                        }
                    }
                    g_store64(&t->st_head, st);
                    t->pi = pi;
                    g_store32(&t->kh, kh);
                    g_store32(&t->head, head);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    g_store32(&t->phase, ph);
                    if (set_re) __hip_atomic_store(&t->reissue, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(&t->walk_lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!__any(tracing)) {
            __builtin_amdgcn_s_sleep(1);
            if (lane == 0 && wall_clock64() - t_begin > kMcWatchdog) {
                int one = 1;
                __hip_atomic_compare_exchange_strong(&t->phase, &one, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (part == 0 && tid == 0 && ticks && bs < nslots_batch)
        ticks[bs] = (uint32_t)min(wall_clock64() - t_begin, (uint64_t)0xFFFFFFFFu);
}

}  // namespace pbrtk
