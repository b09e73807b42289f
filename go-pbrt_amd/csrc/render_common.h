// render_common.h — types and device helpers shared by the kernel translation
// units (k_*.hip) and the host code of render.hip. Namespace pbrtk: the kernels
// are defined in their own translation units and launched from render.hip
// through the declarations of render_kernels.h.

#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/pbrt_gpu.h"
#include "../../include/pbrt_scene.h"
#include "mesh_bvh.h"
#include "pbrt_spec.h"

namespace pbrtk {

using namespace pbrt;


constexpr int kWave = 64;

struct RenderParams {
    int64_t film_min_x, film_min_y, film_w, film_h;   // CroppedPixelBounds
    int64_t tile_size, ntx, nty;
    int64_t tile_begin, tile_stride, n_slots;
    int64_t slot_w, slot_h;                            // max tile-film extent
    int32_t spp, xs, ys, ndims, jitter;
    int32_t integrator, max_depth, dl_strategy;
    double rr_threshold;
    int32_t lanes_per_wave;
    int32_t flags;   // pbrt_render_desc.flags
    int32_t sp_events, sp_draws, sp_serial;   // wave kernel StartPixel: events, raw draws buffered
    int32_t mode;                             // PBRT_MODE_EXACT / _THROUGHPUT
    int32_t sp_window;                        // sp_serial without jitter: the windowed wave StartPixel
    int32_t ci_nps;                           // k_chain_ci multi-wave tiles: next-pixel speculation
    int32_t ci_scap;                          // k_chain_ci statistical speculation cap, tenths of a sigma (0: off)
    int32_t pad1;
};

struct PanicRec {
    int32_t kind;
    int32_t sample;
    int32_t bounce;
    int32_t pad;
    int64_t px, py;
};

struct Counters {
    unsigned long long paths, camera_samples, closest_rays, shadow_rays;
    int32_t any_panic;
    int32_t gate_stall;   // a k_gate wait saw no chain progress for 1 s (serialised dispatch): the frame is rendered again
    // wave kernel diagnostics (pbrt_gpu_counters): speculation windows, and
    // lane-0 clock64 cycles in StartPixel / bounce 1 / chain / full paths / film add
    unsigned long long windows, phase[8];
    unsigned long long dhist[64];   // k_chain_ci diagnostics: on-chain draw counts D (bin D/2, last bin >= 126)
    unsigned long long busy;        // k_chain_ci diagnostics: lane-steps spent tracing (lane utilisation)
    unsigned long long nps_issued;  // k_chain_ci diagnostics: next-pixel speculation candidates issued
    unsigned long long odd_d;       // k_chain_ci diagnostics: on-chain draw counts that are odd (flip stride 2's parity)
};
constexpr int kNumCounters = 6 + 8 + 64 + 3;

__device__ __forceinline__ void tile_bounds(const RenderParams& rp, int64_t tile, int64_t& x0, int64_t& y0,
                                            int64_t& x1, int64_t& y1) {
    // integrator.go:316-325
    int64_t tx = tile % rp.ntx, ty = tile / rp.ntx;
    x0 = rp.film_min_x + tx * rp.tile_size;
    x1 = gomath::to_int(gomath::min((double)(x0 + rp.tile_size), (double)(rp.film_min_x + rp.film_w)));
    y0 = rp.film_min_y + ty * rp.tile_size;
    y1 = gomath::to_int(gomath::min((double)(y0 + rp.tile_size), (double)(rp.film_min_y + rp.film_h)));
}
// Film.GetFilmTile (film.go:106-113)
__device__ __host__ __forceinline__ void film_tile_bounds(const pbrt_film_desc& f, int64_t x0, int64_t y0, int64_t x1,
                                                          int64_t y1, int64_t& px0, int64_t& py0, int64_t& px1,
                                                          int64_t& py1) {
    int64_t p0x = gomath::to_int(gomath::ceil(((double)x0 - 0.5) - f.filter_radius_x));
    int64_t p0y = gomath::to_int(gomath::ceil(((double)y0 - 0.5) - f.filter_radius_y));
    int64_t p1x = gomath::to_int(gomath::floor(((double)x1 - 0.5) + f.filter_radius_x)) + 1;
    int64_t p1y = gomath::to_int(gomath::floor(((double)y1 - 0.5) + f.filter_radius_y)) + 1;
    px0 = gomath::to_int(gomath::max((double)f.crop_min_x, (double)p0x));
    py0 = gomath::to_int(gomath::max((double)f.crop_min_y, (double)p0y));
    px1 = gomath::to_int(gomath::min((double)f.crop_max_x, (double)p1x));
    py1 = gomath::to_int(gomath::min((double)f.crop_max_y, (double)p1y));
}

// Footprint of one sample on the tile film (film.go:211-248). pFilm is the
// pixel corner for every sample of a pixel (2D stratified dims are (0,0), #3),
// so the footprint and the filter weights are per pixel.
struct Footprint {
    int n;               // number of film pixels touched (<= 4 in the register path)
    int64_t off[4];      // offsets (in pixels) into the tile film slot
    double w[4];         // sampleWeight * filterWeight
};
__device__ inline int footprint(const pbrt_film_desc& f, double pfx, double pfy, int64_t px0, int64_t py0,
                                int64_t px1, int64_t py1, Footprint& fp, int64_t& p0x, int64_t& p0y, int64_t& p1x,
                                int64_t& p1y) {
    double dx = pfx - 0.5, dy = pfy - 0.5;
    double p0fx = gomath::ceil(dx - f.filter_radius_x), p0fy = gomath::ceil(dy - f.filter_radius_y);
    double p1fx = gomath::floor(dx + f.filter_radius_x) + 1, p1fy = gomath::floor(dy + f.filter_radius_y) + 1;
    p0x = gomath::to_int(gomath::max(p0fx, (double)px0));
    p0y = gomath::to_int(gomath::max(p0fy, (double)py0));
    p1x = gomath::to_int(gomath::min(p1fx, (double)px1));
    p1y = gomath::to_int(gomath::min(p1fy, (double)py1));
    int64_t nx = p1x - p0x, ny = p1y - p0y;
    if (nx <= 0 || ny <= 0) { fp.n = 0; return 0; }
    if (nx * ny > 4) return -1;
    const double ifx = 1.0 / f.filter_radius_x, ify = 1.0 / f.filter_radius_y;
    int64_t tw = px1 - px0;
    int k = 0;
    for (int64_t y = p0y; y < p1y; y++) {
        int iy = (int)gomath::to_int(gomath::min(gomath::floor(gomath::abs(((double)y - dy) * ify * 16.0)), 16.0 - 1));
        for (int64_t x = p0x; x < p1x; x++) {
            int ix =
                (int)gomath::to_int(gomath::min(gomath::floor(gomath::abs(((double)x - dx) * ifx * 16.0)), 16.0 - 1));
            fp.off[k] = (x - px0) + (y - py0) * tw;
            fp.w[k] = 1.0 * f.filter_table[iy * 16 + ix];
            k++;
        }
    }
    fp.n = k;
    return 0;
}

// ------------------------------------------------------ EXACT, wave-parallel
// The kernels that replace the serial tile replay (see pbrt_spec.h for why
// the results are the same bits):
//   k_chain_ci  per tile: StartPixel (lane-parallel, pcg_bounded rejections
//               resolved), then speculative trajectories at RNG offsets until
//               every sample's offset is known; writes the stratified values
//               and each sample's RNG state. The only serial dependency of the
//               reference (the per-tile PCG32 stream) lives here.
//   k_paths_ci  the samples as full paths (bounce-1 EstimateDirect per light
//               cached per pixel); writes L per sample and the pixel's first
//               panic. k_pw_*: the same as per-bounce compacted queues.
//   k_film      one thread per tile-film pixel: FilmTile.AddSample
//               contributions summed in the reference's order (pixels
//               row-major, samples in order), the serial replay's sums.
__device__ __forceinline__ void stage_nodes(DevScene& sc) {
    if (sc.n_nodes > kLdsNodes) return;
    for (int i = threadIdx.x; i < sc.n_nodes; i += blockDim.x) g_nodes_lds[i] = sc.nodes[i];
    for (int i = threadIdx.x; i < 8 * sc.n_nodes; i += blockDim.x) {
        const int oct = i / sc.n_nodes, j = i - oct * sc.n_nodes;
        if (j < sc.n_leaves) g_leaf_lds[oct * kLdsNodes + j] = (uint16_t)sc.order[8 * sc.n_nodes + i];
    }
    for (int i = threadIdx.x; i < sc.n_groups * 6; i += blockDim.x) g_grp_lds[i] = sc.groups[i];
    for (int i = threadIdx.x; i < 8 * (sc.n_groups + 1) && sc.n_groups > 0; i += blockDim.x) {
        const int oct = i / (sc.n_groups + 1), g = i - oct * (sc.n_groups + 1);
        g_gmask_lds[oct * (kMaxCullGroups + 1) + g] = sc.gmasks[i];
    }
    __syncthreads();
    sc.use_lds_nodes = 1;
}

struct PixelRec {
    SI si;
    BSDF b;
    BSDFX x;          // kX pipelines (Mirror / smooth Glass / OrenNayar scenes)
    V3 wo;
    int32_t hit;      // first hit exists and maxDepth > 1
    int32_t nvalid;   // samples 1 .. nvalid-1 have offsets (spp unless a panic cut the chain)
    int32_t panic0;   // the camera ray's traversal panics (kind), else 0
    int32_t dl_levels;   // DirectLighting: levels of the pixel's hit chain (k_wf_primary; see dl_chain_draws)
};
struct WaveBufs {
    PixelRec* prec;     // [slot][ppt]
    double* s1d;        // [slot][ppt][ndims * spp]
    uint64_t* memb;     // [slot][ppt][spp]   PCG32 state at sample k's offset
    double* L;          // [slot][ppt][spp][3]
    uint32_t* rays;     // [slot][ppt][spp]      the sample's reference ray counts (kRayClosest / kRayShadow)
    PanicRec* ppanic;   // [slot][ppt]        first panic of the pixel in sample order
    int32_t* tile_npx;  // [slot]             pixels with records (a panic ends the tile)
    RrBranches* rrb;    // [slot][kCiMaxRing] k_chain_ci<kX>: RR decisions of the speculative trajectory
                        //                    at each ring entry (null for Matte-only scenes)
    int64_t ppt;        // pixel records per tile slot (tile_size^2)
    int64_t s1d_stride; // ndims * spp
};
// Per-sample outputs (wb.L, wb.rays) are pixel-major: [slot][pixel][k]. A
// pixel's samples are one contiguous run (63 x 24 B of L at 64 spp), so the
// path stage's lanes, which hold samples of the same few pixels, write into a
// few KB that the L2 fills whole before write-back, and k_film stages a run of
// source pixels into LDS with contiguous loads.
__device__ __forceinline__ int64_t sample_index(const WaveBufs& wb, int64_t rec, int n, int k) {
    (void)wb;
    return rec * n + k;
}
constexpr int kFilmThreads = 256;           // k_film workgroup (one per tile slot)
constexpr int kFilmStageBytes = 24 * 1024;  // k_film: LDS staging of a run of source pixels' L
// k_film: source pixels per staged run (a row of a 16-px tile at 64 spp, one
// pixel at 1024), and its dynamic LDS: running sums [slot_w x slot_h][3],
// then the run [S][spp - 1][3]
__host__ __device__ inline int film_run_pixels(const RenderParams& rp) {
    const int64_t m = rp.spp - 1, npx = rp.tile_size * rp.tile_size;
    int64_t S = m > 0 ? kFilmStageBytes / (m * 24) : 1;
    if (S > npx) S = npx;
    if (S > kFilmThreads) S = kFilmThreads;
    return S < 1 ? 1 : (int)S;
}
__host__ __device__ inline int film_lds_bytes(const RenderParams& rp) {
    const int64_t nfp = rp.slot_w * rp.slot_h, m = rp.spp - 1;
    return (int)(((nfp * 3 + 1) & ~int64_t(1)) * 8 + (int64_t)film_run_pixels(rp) * (m > 0 ? m : 1) * 24);
}
struct ChainLayout {   // byte offsets into the chain / setup kernels' dynamic LDS block
    int s1d, other, sbuf, dbuf, vbuf, total;
    int ring;      // k_chain_ci: offset ring after the StartPixel staging (no sbuf / dbuf)
    int staging;   // k_chain_ci: bytes of the StartPixel staging (s1d, other, vbuf)
    int pcs;       // k_chain_ci: the lane groups' bounce-1 ChainCache records (ci_layout)
};
#ifndef PBRT_CI_RING_KB
#define PBRT_CI_RING_KB 4
#endif
constexpr int kCiRingBytes = PBRT_CI_RING_KB * 1024;   // k_chain_ci offset ring (all lane groups of a wave)
constexpr int kCiMaxGroups = 4;          // k_chain_ci lane groups (tiles) per wave
constexpr int kCiMaxRing = 4 * kCiRingBytes / 16;   // ring entries of a tile at the most waves of a kX tile (4)
// k_chain_ci ring entry D with recorded RR decisions (RrBranches at the entry):
// the low 30 bits are the survivor's D, or kRrTailBad when the survivor's own
// trajectory could not resolve D (then it is kBadSpecD unless a decision ends it)
constexpr uint32_t kRrFlag = 0x40000000u, kRrTailBad = 0x3FFFFFFFu;

__device__ __forceinline__ double pcg_float_of(uint32_t v) {
    return gomath::min(gomath::kOneMinusEpsilon, (double)v * 2.3283064365386963e-10);
}
__device__ __forceinline__ int64_t tile_of_slot(const RenderParams& rp, int64_t slot) {
    return rp.tile_begin + slot * rp.tile_stride;
}
__device__ __forceinline__ uint64_t pcg_inc_of(uint64_t seed) { return (seed << 1) | 1; }   // rng.go:28-34

// Stratified.StartPixel (stratified.go:21-48) for one pixel. Every thread of
// the workgroup calls it (it holds the block's barriers); the first wave does
// the work. The shuffled 1D values are left in s1d (LDS); returns the PCG32
// state after the pixel's draws.
__shared__ int g_sp_overflow;
constexpr int kSpRing = 256;   // windowed StartPixel: raw draws in flight (a power of two)
// Bytes of the StartPixel draw area (ChainLayout.vbuf): every raw draw (the wave
// StartPixel), or for the windowed one its uint16 permutations then the draw
// ring, or nothing (the serial StartPixel)
__host__ __device__ inline int64_t sp_vbuf_bytes(const RenderParams& rp) {
    if (rp.sp_window) return (((int64_t)rp.ndims * rp.spp * 2 + 15) & ~int64_t(15)) + kSpRing * 4;
    return rp.sp_serial ? 4 : (int64_t)rp.sp_draws * 4;
}
// kWin: the windowed version is compiled in (k_chain_ci instantiates it only
// where the host runs it: its code in the chain kernel raised the spills of the
// chain's main loop, config B 314 -> 340 ms)
template <bool kWin = true>
__device__ uint64_t start_pixel_wave(const RenderParams& rp, const PcgJump& J, uint64_t S, uint64_t inc, double* s1d,
                                     uint16_t* other, uint32_t* vbuf, uint64_t* sh_state, uint32_t* sh_draws = nullptr) {
    const int lane = threadIdx.x;
    const bool w0 = lane < kWave;
    const int n = rp.spp, ndims = rp.ndims;
    const double inv_n = 1.0 / (double)n;
    const int s1 = rp.jitter ? 2 * n : n, s2 = rp.jitter ? 3 * n : n;   // StartPixel draws per 1D / 2D dim
    // StartPixel (stratified.go:21-48). The pixel's draws form a fixed
    // list of E events (jitter floats and pcg_bounded picks,
    // sampling.go:101-145). A pick retries on v < 2^32 mod b, which
    // the reference's (rot+1)&31 output rotation makes common (v < 4
    // has probability ~1/64), so event e lands on draw e + R(e),
    // R(e) = rejections before it. Lanes fill the raw stream by
    // jump-ahead, then resolve R chunk by chunk: one ballot per
    // rejection shifts every later event by one draw.
    bool serial_sp = rp.sp_serial != 0;
    if (kWin && serial_sp && rp.sp_window && !(rp.flags & PBRT_FLAG_SERIAL_START_PIXEL)) {
        // Windowed wave StartPixel (large spp without jitter, where a buffer of
        // every raw draw would not fit LDS: config C's 256 spp). The same events
        // and rejection resolution as above, but the raw draws pass through a
        // ring of kSpRing entries, filled 64 at a time by jump-ahead as the
        // events advance. The 1D picks land in `other`; the Fisher-Yates swaps
        // (stratified.go:40-47, sampling.go:127-145) run on uint16 indices in
        // LDS (perm), and the values, min((i + 0.5) / n, OneMinusEpsilon) of
        // the index i a slot ends with (no jitter: a value is a function of its
        // index), are written once, coalesced, to s1d (the pixel's global
        // record). Replaces the lane-0 replay, whose swaps were dependent
        // global-memory round trips (18% of config C's chain cycles).
        uint16_t* perm = (uint16_t*)vbuf;
        uint32_t* ring = (uint32_t*)((unsigned char*)vbuf + (((size_t)ndims * n * 2 + 15) & ~(size_t)15));
        const int E = rp.sp_events;   // ndims * n 1D picks, then ndims * n 2D picks
        bool overflow = false;
        int R = 0;
        if (w0) {
            uint64_t st = pcg_advance(J, S, inc, (uint64_t)lane);
            int filled = 0;   // draws [0, filled) have been written to the ring
            auto fill64 = [&]() {
                ring[(filled + lane) & (kSpRing - 1)] = pcg_output(st);
                st = J.a[6] * st + inc * J.b[6];   // +64 draws
                filled += kWave;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            };
            for (int cb = 0; cb < E; cb += kWave) {
                while (filled < cb + R + 2 * kWave) fill64();   // the window covers the chunk and 64 rejections
                const int e = cb + lane;
                int kind = 0, slt = 0, i = 0;   // 2: 1D pick, 3: 2D pick
                if (e < E) {
                    if (e < ndims * n) { kind = 2; i = e % n; slt = e; }
                    else { kind = 3; i = (e - ndims * n) % n; }
                }
                const uint32_t b = (uint32_t)(n - i);
                const uint32_t thr = kind >= 2 ? (~b + 1u) % b : 0u;
                int local = 0;
                for (;;) {
                    const int t = e + R + local;
                    if (__any(kind != 0 && t >= filled)) {   // many rejections in one chunk
                        if (filled + kWave - (cb + R) > kSpRing) { overflow = true; break; }
                        fill64();
                        continue;
                    }
                    const bool bad = kind != 0 && ring[t & (kSpRing - 1)] < thr;
                    const unsigned long long m = __ballot(bad);
                    if (m == 0) break;
                    const int first = __ffsll((long long)m) - 1;
                    if (lane >= first) local++;
                }
                if (overflow) break;
                if (kind == 2) other[slt] = (uint16_t)(i + (int)(ring[(e + R + local) & (kSpRing - 1)] % b));
                R = __builtin_amdgcn_readfirstlane(R + __shfl(local, kWave - 1));   // wave-uniform
            }
            if (lane == 0) g_sp_overflow = overflow;
        }
        __syncthreads();
        if (!g_sp_overflow) {
            const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
            for (int idx = tid; idx < ndims * n; idx += nt) perm[idx] = (uint16_t)(idx % n);
            __syncthreads();
            if (tid < ndims) {
                uint16_t* pm = perm + tid * n;
                const uint16_t* oth = other + tid * n;
                for (int k = 0; k < n; k++) {
                    const int o = oth[k];
                    const uint16_t a = pm[k];
                    pm[k] = pm[o];
                    pm[o] = a;
                }
            }
            __syncthreads();
            for (int idx = tid; idx < ndims * n; idx += nt)
                s1d[idx] = gomath::min(((double)perm[idx] + 0.5) * inv_n, gomath::kOneMinusEpsilon);
            if (tid == 0) {
                *sh_state = pcg_advance(J, S, inc, (uint64_t)(E + R));
                if (sh_draws) *sh_draws = (uint32_t)(E + R);
            }
            __syncthreads();
            return *sh_state;
        }
        // (a window overflow, never seen: the lane-0 replay below)
    } else if (!serial_sp) {
        const int E = rp.sp_events, V = rp.sp_draws;
        if (w0) {
            uint64_t st = pcg_advance(J, S, inc, (uint64_t)lane);
            for (int t = lane; t < V; t += kWave) {
                vbuf[t] = pcg_output(st);
                st = J.a[6] * st + inc * J.b[6];   // +64 draws
            }
        }
        __syncthreads();
        int R = 0;
        bool overflow = false;
        for (int cb = 0; w0 && cb < E; cb += kWave) {
            const int e = cb + lane;
            int kind = 0, slt = 0, i = 0;   // 0 none, 1 1D float, 2 1D pick, 3 2D pick
            if (e < E) {
                if (e < ndims * s1) {
                    const int d = e / s1, qq = e - d * s1;
                    if (rp.jitter && qq < n) { kind = 1; slt = d * n + qq; }
                    else { kind = 2; i = qq - (rp.jitter ? n : 0); slt = d * n + i; }
                } else {
                    const int e2 = e - ndims * s1, d = e2 / s2, qq = e2 - d * s2;
                    if (!(rp.jitter && qq < 2 * n)) { kind = 3; i = qq - (rp.jitter ? 2 * n : 0); }
                }
            }
            const uint32_t b = (uint32_t)(n - i);
            const uint32_t thr = kind >= 2 ? (~b + 1u) % b : 0u;
            int local = 0;
            for (;;) {
                const int t = e + R + local;
                const bool out = kind != 0 && t >= V;
                const bool bad = !out && kind >= 2 && vbuf[t] < thr;
                if (__any(out)) { overflow = true; break; }
                const unsigned long long m = __ballot(bad);
                if (m == 0) break;
                const int first = __ffsll((long long)m) - 1;
                if (lane >= first) local++;
            }
            if (overflow) break;
            const uint32_t v = kind != 0 ? vbuf[e + R + local] : 0u;
            if (kind == 1)
                s1d[slt] = gomath::min(((double)(slt % n) + pcg_float_of(v)) * inv_n, gomath::kOneMinusEpsilon);
            else if (kind == 2)
                other[slt] = (uint16_t)(i + (int)(v % b));
            R += __shfl(local, kWave - 1);
        }
        if (lane == 0) g_sp_overflow = overflow;
        __syncthreads();
        serial_sp = g_sp_overflow != 0;
        if (!serial_sp) {
            if (!rp.jitter && w0)
                for (int idx = lane; idx < ndims * n; idx += kWave)
                    s1d[idx] = gomath::min(((double)(idx % n) + 0.5) * inv_n, gomath::kOneMinusEpsilon);
            __syncthreads();
            if (lane < ndims) {
                double* samp = s1d + lane * n;
                const uint16_t* oth = other + lane * n;
                for (int k = 0; k < n; k++) {
                    const int o = oth[k];
                    double a = samp[k];
                    samp[k] = samp[o];
                    samp[o] = a;
                }
            }
            if (lane == 0) {
                *sh_state = pcg_advance(J, S, inc, (uint64_t)(E + R));
                if (sh_draws) *sh_draws = (uint32_t)(E + R);
            }
        }
    }
    if (serial_sp || (rp.flags & PBRT_FLAG_SERIAL_START_PIXEL)) {
        if (lane == 0) {   // serial replay (huge sample counts, or forced)
            Thread t;
            t.rng.state = S;
            t.rng.inc = inc;
            t.spp = n; t.ndims = ndims; t.xs = rp.xs; t.ys = rp.ys; t.jitter = rp.jitter;
            t.s1d = s1d;
            start_pixel(t);
            *sh_state = t.rng.state;
            if (sh_draws) {   // its draw count: the events plus the rejections, found by stepping
                uint64_t st = pcg_advance(J, S, inc, (uint64_t)rp.sp_events);
                uint32_t k = (uint32_t)rp.sp_events;
                while (st != t.rng.state) {
                    st = st * 0x5851f42d4c957f2dULL + inc;
                    k++;
                }
                *sh_draws = k;
            }
        }
    }
    __syncthreads();
    return *sh_state;
}

#ifndef PBRT_PATHS_WAVES
#define PBRT_PATHS_WAVES 2
#endif
constexpr int kPathsWaves = PBRT_PATHS_WAVES;   // k_paths_ci waves/SIMD (build option)

// k_paths_ci: full paths with lane refill. One pixel's samples per wave would
// make a wave last as long as its longest path (~4x the mean). Here a wave
// owns P pixel records and treats their samples as one
// work list: a lane whose path ends writes its radiance and takes the next
// (pixel, sample) at once, so the wave only waits for its longest path at
// the end of the P pixels. Every path runs the same arithmetic as
// Path.Li (path_step), from the offset the chain found, so L per
// (pixel, sample) is bit-identical; k_film sums them in sample order as
// before. Requires LDS-staged nodes (no traversal stack) and P * n_lights <= 64.
//
// paths_group is the per-wave body, synchronised within the wave only (a
// fused variant that ran it inside k_chain_ci after each tile's chain was
// bit-exact but slower: 1000 vs 874 ms, the chain kernel spilled). Its LDS:
// PixelCache[P], then P panic keys, then the P pixels' stratified values.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
struct PMeta {   // per pixel of a paths_group: PCG increment, tile, nvalid, hit, first work index
    uint64_t inc, tile;
    int32_t nv, hit, cum, pad;
};
template <int P>
__host__ __device__ constexpr size_t paths_group_meta_off() {
    return (P * sizeof(PixelCache) + P * 8 + 15) & ~(size_t)15;
}
template <int P>
__host__ __device__ constexpr size_t paths_group_l_off() {   // per-lane radiance sums (PathStateLds)
    return paths_group_meta_off<P>() + (P + 1) * sizeof(PMeta);
}
template <int P>
__host__ __device__ constexpr int paths_group_lds(int per) {   // bytes, per wave
    return (int)(paths_group_l_off<P>() + 3 * kWave * sizeof(Spec) + kWave * 4 + (size_t)P * per * 8);
}
// kMB: THROUGHPUT mode, sample k of pixel pi starts from its own stream
// mb_state(tile, pi, k) instead of the chain's offset state.
// s1d_lds: the group's stratified values are staged in LDS (else read from
// their global records: large spp, e.g. config E's 1024).
template <int P, bool kMB = false, bool kX = false>
__device__ __forceinline__ void paths_group(const DevScene& sc, const RenderParams& rp, const WaveBufs& wb, int64_t slot_base,
                            int64_t rec0, int64_t rec_end, Counters* __restrict__ ctr, unsigned char* wlds,
                            int s1d_lds) {
    const int lane = threadIdx.x & (kWave - 1);
    const int n = rp.spp, ndims = rp.ndims, nl = sc.n_lights;
    const int per = ndims * n;
    PixelCache* pcs = (PixelCache*)wlds;
    unsigned long long* pkey = (unsigned long long*)(wlds + P * sizeof(PixelCache));
    // per-pixel metadata lives in LDS (not in per-lane register arrays)
    PMeta* meta = (PMeta*)(wlds + paths_group_meta_off<P>());
    Spec* Lslot = (Spec*)(wlds + paths_group_l_off<P>()) + lane;
    Spec* aux = (Spec*)(wlds + paths_group_l_off<P>()) + kWave + 2 * lane;
    uint32_t* rslot = (uint32_t*)(wlds + paths_group_l_off<P>() + 3 * kWave * sizeof(Spec)) + lane;
    double* s1d = (double*)(wlds + paths_group_l_off<P>() + 3 * kWave * sizeof(Spec) + kWave * 4);
    if (lane == 0) {
        int cum = 0;
        for (int j = 0; j < P; j++) {
            const int64_t rec = rec0 + j;
            PMeta m{0, 0, 0, 0, cum, 0};
            if (rec < rec_end) {
                const int64_t bslot = rec / wb.ppt, pi = rec % wb.ppt;
                if (pi < wb.tile_npx[bslot]) {
                    m.nv = wb.prec[rec].nvalid;
                    m.hit = wb.prec[rec].hit;
                    m.tile = (uint64_t)tile_of_slot(rp, slot_base + bslot);
                    m.inc = pcg_inc_of(m.tile);
                }
            }
            meta[j] = m;
            cum += m.nv > 1 ? m.nv - 1 : 0;
        }
        meta[P].cum = cum;
    }
    wave_sync();
    for (int idx = lane; s1d_lds && idx < P * per; idx += kWave) {
        const int j = idx / per;
        if (meta[j].nv > 0) s1d[idx] = wb.s1d[(rec0 + j) * wb.s1d_stride + (idx - j * per)];
    }
    if (lane < P) {
        pkey[lane] = ~0ULL;
        if (meta[lane].nv > 0) {
            const PixelRec& pr = wb.prec[rec0 + lane];
            pcs[lane].si = pr.si;
            pcs[lane].b = pr.b;
            if constexpr (kX) pcs[lane].x = pr.x;
            pcs[lane].wo = pr.wo;
            pcs[lane].hit = pr.hit;
        }
    }
    wave_sync();
    if (nl > 0 && lane < P * nl) {   // bounce-1 light samples, uLight = (0,0); lane = pixel * nl + light
        const int j = lane / nl, l = lane - j * nl;
        if (meta[j].nv > 0 && meta[j].hit && (kX ? bsdfx_nonspecular(pcs[j].b, pcs[j].x) : pcs[j].b.n_bxdfs > 0)) {
            int pl = 0;
            uint64_t traced = 0;
            Spec ld = kX ? estimate_direct_x(sc, nullptr, pl, pcs[j].si, pcs[j].b, pcs[j].x, l, V2{0.0, 0.0}, &traced)
                         : estimate_direct(sc, nullptr, pl, pcs[j].si, pcs[j].b, l, V2{0.0, 0.0}, &traced);
            if (!pl && max_component(ld) > 10) pl = PBRT_PANIC_LD_GT_10;
            pcs[j].ld[l] = ld;
            pcs[j].ld_panic[l] = pl | (traced ? kLdTraced : 0);
        }
    }
    wave_sync();
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int T = meta[P].cum;
    int base = 0;
    int w = -1, j = 0, k = 0;
    PathStateLds ps;
    ps.L = Lslot;
    ps.aux = aux;
    ps.rays = rslot;
    Cursor c;
    c.rri = -1;
    int pnc = 0, bnc = 1;
    for (;;) {
        const bool idle = w < 0;
        const unsigned long long m = __ballot(idle);
        if (idle) {
            const int t = base + __popcll(m & lt_mask);
            if (t < T) {
                j = 0;
#pragma unroll
                for (int q = 1; q < P; q++) j += t >= meta[q].cum ? 1 : 0;
                k = 1 + (t - meta[j].cum);
                const int64_t rec = rec0 + j;
                if (!meta[j].hit) {   // no traced bounce: the sample's radiance is 0
                    double* o = wb.L + sample_index(wb, rec, n, k) * 3;
                    o[0] = 0.0;
                    o[1] = 0.0;
                    o[2] = 0.0;
                    wb.rays[sample_index(wb, rec, n, k)] = kRayClosest;   // the camera ray's (missed or maxDepth 1) query
                } else {
                    w = t;
                    c.rng.state = kMB ? mb_state(meta[j].tile, (uint64_t)(rec % wb.ppt), (uint64_t)k)
                                      : wb.memb[rec * n + k];
                    c.rng.inc = meta[j].inc;
                    c.draws = 0;
                    c_camera(c, ndims);   // camera: Get2D pFilm, Get2D pLens, Get1D time
                    c.k = k;
                    c.kdep = 0;
                    *ps.L = spec(0);
                    *ps.rays = 0;
                    ps.beta = spec(1);
                    ps.eta_scale = 1.0;
                    ps.bounces = 1;
                    ps.first = 1;
                    pnc = 0;
                    bnc = 1;
                }
            }
        }
        base += __popcll(m);
        if (!__any(w >= 0)) {
            if (base >= T) break;
            continue;
        }
        if (w >= 0) {
            // a path taken this iteration runs its bounce 1 from the pixel cache
            // (no traversal) and then, with every other live path, one traced
            // bounce: the cheap first step does not cost the wave an iteration
            const SpecSampler ss{s1d_lds ? s1d + j * per : wb.s1d + (rec0 + j) * wb.s1d_stride, n, ndims};
            bool done = false;
            if (ps.first)
                done = path_step<1, kX>(sc, pcs[j], ss, c, ps, rp.max_depth, rp.rr_threshold, nullptr, pnc, bnc);
            if (!done)
                done = path_step<2, kX>(sc, pcs[j], ss, c, ps, rp.max_depth, rp.rr_threshold, nullptr, pnc, bnc);
            if (done) {
                const int64_t rec = rec0 + j;
                double* o = wb.L + sample_index(wb, rec, n, k) * 3;
                const Spec Lp = *ps.L;
                o[0] = Lp.r;
                o[1] = Lp.g;
                o[2] = Lp.b;
                wb.rays[sample_index(wb, rec, n, k)] = *ps.rays;
                if (pnc)
                    atomicMin(&pkey[j], ((unsigned long long)k << 32) | ((unsigned long long)(bnc & 0xFFFFFF) << 8) |
                                            (unsigned long long)((pnc + 1) & 0xFF));
                w = -1;
            }
        }
    }
    wave_sync();
    if (lane < P && meta[lane].nv > 0) {
        const int64_t rec = rec0 + lane;
        const int64_t bslot = rec / wb.ppt, pi = rec % wb.ppt;
        int64_t x0, y0, x1, y1;
        tile_bounds(rp, tile_of_slot(rp, slot_base + bslot), x0, y0, x1, y1);
        PanicRec p{0, 0, 0, 0, x0 + pi % (x1 - x0), y0 + pi / (x1 - x0)};
        const int panic0 = wb.prec[rec].panic0;
        if (panic0) {
            p.kind = panic0;
            p.sample = 1;
            p.bounce = 1;
        } else if (pkey[lane] != ~0ULL) {
            p.kind = (int)(pkey[lane] & 0xFF) - 1;
            p.bounce = (int)((pkey[lane] >> 8) & 0xFFFFFF);
            p.sample = (int)(pkey[lane] >> 32);
        }
        wb.ppanic[rec] = p;
        if (!p.kind && meta[lane].nv > 1) {
            atomicAdd(&ctr->paths, (unsigned long long)(meta[lane].nv - 1));
            atomicAdd(&ctr->camera_samples, (unsigned long long)(meta[lane].nv - 1));
        }
    }
    wave_sync();   // the LDS block is reused by the wave's next group
}

// ------------------------------------------------- path wavefront (k_pw_*)
// The full-path stage (k_paths_ci's work: every (pixel, sample) path from its
// RNG state, with light sampling) as per-bounce launches over queues of live
// paths, compacted every bounce and, between the closest-hit trace and the
// shading, counting-sorted by the hit's material (SURVEY §8 north_star: "rays
// compacted and sorted by material between bounces"):
//   k_pw_cache   bounce-1 EstimateDirect per (pixel, light), uLight = (0,0)
//   k_pw_start   per path: bounce 1 from the pixel record (path_step<1>),
//                then the next bounce's depth test -> trace queue or done
//   k_pw_trace   closest hit of every queued ray; a miss or a panic ends the
//                path, a hit goes to the hit queue with its material key
//   k_pw_count / k_pw_scan / k_pw_scatter   counting sort of the hit queue
//   k_pw_shade   interaction, BSDF, light-sample draws up to the shadow ray,
//                BSDF sample, throughput and Russian roulette
//   k_pw_shadow  the deferred shadow ray, L += beta0 * Ld, then the depth
//                test -> trace queue or done
//   k_pw_panics  per pixel record: its first panic (sample order) + counters
// Each step is path_step<2>'s code split at its two traversals, in its order,
// so L per (pixel, sample) is bit-identical to k_paths_ci's. Grid-stride
// kernels read the queue lengths on the device (no host round trip).
struct alignas(16) PwPath {
    Ray ray;         // next closest-hit ray (tmax: after the walk, for prim_si)
    Spec L, beta;
    Ray sr;          // deferred shadow ray
    Spec beta0, ld;  // its throughput and unoccluded Ld
    V3 ph;           // object-space hit point of the closest hit
    uint64_t rng;    // PCG32 state (the increment is the tile's)
    int64_t rec;     // pixel record in the batch
    int32_t k, cur1d, cur2d, kdep;
    int32_t bounces, best, flags, pnc;
    int32_t bnc;
    uint32_t rays;   // kRayClosest / kRayShadow counts of the path
    double eta;      // Path.Li's etaScale (kX)
};
constexpr int kPwPending = 1, kPwShadow = 2, kPwDone = 4;
constexpr int kPwMaxKeys = 64;   // material keys of the sort (more materials share the last)
struct PwQueues {
    uint32_t* q[3];          // trace queue (current / next) and the hit queue, path ids
    uint32_t* sorted;        // hit queue in material order
    uint32_t* cnt;           // [0] trace, [1] next trace, [2] hits, [3..3+kPwMaxKeys) key counts, then offsets
    int64_t cap;
};
__device__ __forceinline__ uint32_t pw_push(uint32_t* cnt, uint32_t* q, uint32_t v) {
    const unsigned long long m = __ballot(1);
    const int lead = __ffsll((long long)m) - 1, lane = threadIdx.x & (kWave - 1);
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, lead);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ULL << lane) - 1ULL));
    q[pos] = v;
    return pos;
}
// atomicAdd(&ctr[key], 1) for every active lane, aggregated per distinct key
// of the wave (few materials: a handful of atomics per wave instead of one per
// lane on the same few addresses); returns the lane's old-count position
__device__ __forceinline__ uint32_t pw_add_by_key(uint32_t* ctr, int key) {
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t pos = 0;
    unsigned long long todo = __ballot(1);
    for (;;) {
        const int lead = __ffsll((long long)todo) - 1;
        const int k0 = __shfl(key, lead);
        const unsigned long long m = __ballot(key == k0) & todo;
        uint32_t base = 0;
        if (lane == lead) base = atomicAdd(&ctr[k0], (uint32_t)__popcll(m));
        base = __shfl(base, lead);
        if (key == k0 && ((todo >> lane) & 1ULL)) pos = base + (uint32_t)__popcll(m & ((1ULL << lane) - 1ULL));
        todo &= ~m;
        if (!todo) break;
    }
    return pos;
}
// a finished path: its radiance, and its panic into the pixel's key
__device__ __forceinline__ void pw_finish(const WaveBufs& wb, int n, const PwPath& p, unsigned long long* pkey) {
    double* o = wb.L + sample_index(wb, p.rec, n, p.k) * 3;
    o[0] = p.L.r;
    o[1] = p.L.g;
    o[2] = p.L.b;
    wb.rays[sample_index(wb, p.rec, n, p.k)] = p.rays;
    if (p.pnc)
        atomicMin(&pkey[p.rec], ((unsigned long long)p.k << 32) | ((unsigned long long)(p.bnc & 0xFFFFFF) << 8) |
                                    (unsigned long long)((p.pnc + 1) & 0xFF));
}
// path_step's loop-top depth test; false: the path is done
__device__ __forceinline__ bool pw_next_bounce(PwPath& p, int max_depth) {
    p.bounces++;
    p.bnc = p.bounces;
    p.rays += kRayClosest;   // the reference's Intersect of this iteration (k_pw_trace, or the maxDepth break)
    return p.bounces < max_depth;
}
// the bounce-1 light estimates of the pixel record (global-memory PixelCache)
struct PwCache {
    SI si;
    BSDF b;
    BSDFX x;
    V3 wo;
    const Spec* ld;
    const int* ld_panic;
};

// ------------------------------------------- DirectLighting, wave-parallel
// DirectLighting.Li (directlighting.go:62-104) has no chain problem: with
// n_dims >= 1 (and n_dims >= 2 or a pinhole camera) every sample of a pixel
// traces the same camera ray, so hit or miss -- the only thing the number of
// PCG32 draws of a sample depends on -- is per pixel, and sample k of the
// pixel starts at the state after StartPixel advanced by (k - 1) * D.
// k_dl_setup replays the tile's pixels in order (StartPixel, then jump-ahead
// over the pixel's samples); k_dl_samples runs every (pixel, sample) at once.
//
// PCG32 draws of one DirectLighting sample whose recursion chain hits `levels`
// surfaces (directlighting.go:62-104 at depth 0, 2, 4, ...: the camera Get2D,
// Get2D, Get1D; per hit level the light samples -- UniformSampleAllLights' two
// Get2D per light (clones carry no sample arrays, #23) or UniformSampleOneLight's
// Get1D + 2 Get2D -- then, while depth + 1 < maxDepth, the Get2D of
// SpecularReflect and of SpecularTransmit (integrator.go:352-355, 383-385)),
// stratified dims first (pixel.go:60-80 counters), then 1 / 2 draws each.
// The chain is the same for every sample of a pixel: the camera ray is per
// pixel (2D stratified values are (0,0), #3) and SpecularTransmission's
// direction does not read its sample, so only the light samples differ.
__device__ __forceinline__ uint32_t dl_chain_draws(const RenderParams& rp, int levels, int n_lights) {
    int c1 = 0, c2 = 0;
    uint32_t d = 0;
    auto g1 = [&]() { if (c1 < rp.ndims) c1++; else d += 1; };
    auto g2 = [&]() { if (c2 < rp.ndims) c2++; else d += 2; };
    g2();
    g2();
    g1();
    for (int i = 0; i < levels; i++) {
        if (n_lights > 0) {
            if (rp.dl_strategy == PBRT_DL_UNIFORM_SAMPLE_ALL) {
                for (int j = 0; j < n_lights; j++) {
                    g2();
                    g2();
                }
            } else {
                g1();
                g2();
                g2();
            }
        }
        if (2 * i + 1 < rp.max_depth) {
            g2();
            g2();
        }
    }
    return d;
}
__device__ __forceinline__ uint32_t dl_draws(const RenderParams& rp, int hit, int n_lights) {
    return dl_chain_draws(rp, hit ? 1 : 0, n_lights);
}
// Cold-frame schedule of k_chain_ci. Workgroups start in launch order, so a
// heavy tile launched late stretches the frame; a context that has rendered
// this configuration before orders its tiles by their measured chain times
// (heaviest first). A fresh context (internal/render/server.go builds one per
// RPC) estimates them instead: one wave per tile slot runs kProbes trajectories
// per pixel from the pixel's bounce-1 record (k_wf_primary) at pseudo-random
// PCG32 states, exactly the work a chain candidate does (traj_scatter), and
// prices the slot as
//   cost = traced_spp * mean(D * bounces) summed over the hit pixels   (chain lane-bounces)
//        + kCostPixel * pixels                                         (StartPixel)
// Only the launch order depends on it, never a result. Writes the features
// (feat[4 * slot]: work, hit pixels, pixels, cost) and the sort key
// (~cost bits << 32 | slot: ascending = heaviest first).
constexpr int kProbes = 2;
constexpr double kCostPixel = 150.0;   // one StartPixel ~ this many trajectory bounces of one lane

// ------------------------------------------- continuous-issue offset chain
// k_chain_ci replaced round 1's fixed 64-candidate windows: a window lasts as
// long as its longest trajectory (~6.5 bounces for a 2.25-bounce mean), so
// most lanes idle through most of it. Here a lane that finishes a
// trajectory, or whose candidate the chain has jumped over, takes the next
// unissued offset at once: every bounce step keeps every lane busy, and
// candidates left behind by the chain are dropped mid-trajectory.
//
// Per lane group (L = 64 / G lanes = one tile): a ring of resolved offsets
// {offset, D, PCG state} in LDS; the group leader walks the exact chain
// head -> head + D(head) through it after every step. Offsets are relative
// to the pixel's first sample (the state after StartPixel). Candidates are
// issued at head + even offsets; when D is odd the parity of the chain flips
// and the group's in-flight candidates are dropped. A speculative result
// that is not usable at the head (a panic or a draw count that depends on
// the sample index) is re-run there with the sample index known; an exact
// panic ends the tile at that sample. Bit-identical to the
// serial replay: only the schedule changes.
#ifndef PBRT_CI_MESH_EU_WAVES
#define PBRT_CI_MESH_EU_WAVES 3   // k_chain_ci's mesh-only instantiations (kDepth < 0): waves/SIMD (build option)
#endif
#ifndef PBRT_CI_EU_WAVES
#define PBRT_CI_EU_WAVES 3   // k_chain_ci waves/SIMD, Matte analytic scenes (build option)
#endif
#ifndef PBRT_CI_X_EU_WAVES
#define PBRT_CI_X_EU_WAVES 2   // k_chain_ci waves/SIMD, Mirror / Glass / OrenNayar scenes (build option)
#endif
#ifndef PBRT_CHAIN_LB
#define PBRT_CHAIN_LB 1   // leaf boxes per scan iteration in k_chain_ci's traversal (build option)
#endif
constexpr uint32_t kNoOff = 0xFFFFFFFFu;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;   // an unwritten entry of k_chain_ci's completion list
// k_chain_ci's progress record: [0] workgroups started, [1] completions, [2] pixels
// started (a heartbeat), [kProgHead + i] the slot of the i-th completion
constexpr int kProgHead = 3;
constexpr uint32_t kBadSpecD = 0xFFFFFFFEu;   // speculative lane could not resolve D
constexpr uint32_t kBadExactD = 0xFFFFFFFDu;  // the exact head's trajectory panics
struct RingEnt {
    uint32_t tag;   // offset this entry resolves (kNoOff: empty)
    uint32_t d;     // its draw count D, or kBadSpecD / kBadExactD
    uint64_t st;    // PCG32 state at the offset
};
// Offsets are absolute: draws of the tile's PCG32 stream since the tile's
// first pixel's StartPixel began (< 2^31 for any supported frame).
struct CiGroup {
    uint64_t S;     // PCG32 state at absolute offset A
    int64_t pi;     // current pixel (row-major index in the tile)
    int64_t npx;    // pixels of the tile
    uint32_t A;     // absolute offset of S (the current pixel's first traced sample once it started)
    uint32_t head;  // offset of sample kh
    uint32_t nxt;   // next offset to issue (same parity as head)
    int kh;         // next sample without an offset
    int phase;      // 0 needs a pixel, 1 resolving offsets, 2 tile finished
    int reissue;    // the head must be re-run with its sample index known
    uint32_t rb0, rb1;   // ring base of the pixels of each parity: entry of offset o at (o - rb) & (R - 1)
    // next-pixel speculation (multi-wave Matte tiles): trajectories of pixel
    // pi + 1 from offsets nb, nb + 1, ... (nb: the lowest offset its first
    // traced sample can start at), issued to lanes the current pixel leaves idle
    uint32_t nb, nnx;   // its ring base and next offset to issue
    int nps;            // active (pixel pi + 1's ring and ChainCache are loaded)
    uint32_t dcnt;      // on-chain draw counts seen in the tile (kNps: their mean and spread set the
    float dsum, dsq;    // current pixel's speculation cap and when the next pixel's starts)
};

}  // namespace pbrtk
