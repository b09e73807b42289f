// render.hip — MI355X (gfx950) kernels and the C ABI of include/pbrt_gpu.h.
//
// Kernels
//   k_render_exact   EXACT mode: one lane per 16-px tile. The lane replays the
//                    tile's PCG32 stream exactly as pbrt.Render's worker does
//                    (integrator.go:228-289, 311-340): pixel loop, Stratified
//                    StartPixel, samples 1..spp-1, Path.Li / DirectLighting.Li,
//                    NaN guard, FilmTile.AddSample into the tile's film slot.
//   wave pipeline    k_wf_primary (bounce 1 per pixel), k_chain_ci (the
//                    tile's RNG-offset chain), k_paths_ci or the path
//                    wavefront k_pw_* (full paths), k_film (tile films);
//                    THROUGHPUT mode: k_mb_setup instead of the chain.
//   k_dl_*           DirectLighting: pixel-order StartPixel + jump-ahead, one
//                    lane per sample.
//   k_merge_film     Film.MergeFilmTile (film.go:115-132): per output pixel,
//                    RGBToXYZ of every covering tile film in tile-index order.
//   k_intersect[_p]  batch BVH closest-hit / any-hit (bvh.go:659-765).
//
// Everything is float64 with -ffp-contract=off (bit parity with the Go
// reference). The scene is a few KB and is read through the scalar/vector L1.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <functional>
#include <mutex>
#include <vector>

#include "../../include/pbrt_gpu.h"
#include "../../include/pbrt_scene.h"
#include "mesh_bvh.h"
#include "pbrt_spec.h"

using namespace pbrt;

namespace {

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
    int32_t pad;
    // wave kernel diagnostics (pbrt_gpu_counters): speculation windows, and
    // lane-0 clock64 cycles in StartPixel / bounce 1 / chain / full paths / film add
    unsigned long long windows, phase[8];
    unsigned long long dhist[64];   // k_chain_ci diagnostics: on-chain draw counts D (bin D/2, last bin >= 126)
};
constexpr int kNumCounters = 6 + 8 + 64;

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

// ----------------------------------------------------------- EXACT kernel
// One lane per tile; `lanes_per_wave` lanes of each 64-lane workgroup work
// (fewer busy lanes per wave = less divergence, more waves per SIMD).
template <int kMinWaves>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kMinWaves, 8))) void k_render_exact(DevScene sc, RenderParams rp, double* __restrict__ films,
                                                        double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics,
                                                        Counters* __restrict__ ctr) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    const int lane = threadIdx.x;
    if (lane >= rp.lanes_per_wave) return;
    const int64_t slot = (int64_t)blockIdx.x * rp.lanes_per_wave + lane;
    if (slot >= rp.n_slots) return;
    const int64_t tile = rp.tile_begin + slot * rp.tile_stride;
    const pbrt_film_desc& film = *sc.film;

    int64_t x0, y0, x1, y1, px0, py0, px1, py1;
    tile_bounds(rp, tile, x0, y0, x1, y1);
    film_tile_bounds(film, x0, y0, x1, y1, px0, py0, px1, py1);
    double* tf = films + slot * (rp.slot_w * rp.slot_h * 3);
    const int64_t npx = (px1 - px0) * (py1 - py0);
    for (int64_t i = 0; i < npx * 3; i++) tf[i] = 0.0;

    Thread t;
    t.spp = rp.spp; t.ndims = rp.ndims; t.xs = rp.xs; t.ys = rp.ys; t.jitter = rp.jitter;
    t.s1d = s1d_scratch + slot * (int64_t)(rp.ndims * rp.spp);
    t.stack = stack_lds + lane;
    t.panic = 0;
    t.bounce = 0;
    t.closest_rays = t.shadow_rays = 0;
    pcg_seed(t.rng, (uint64_t)tile);   // Sampler.Clone(seed = tile index), integrator.go:318,328
    unsigned long long paths = 0;
    const pbrt_camera_desc& cam = *sc.camera;

    const bool mb = rp.mode == PBRT_MODE_THROUGHPUT;
    uint64_t last_host_poll = wall_clock64();
    for (int64_t py = y0; py < y1; py++) {
        for (int64_t px = x0; px < x1; px++) {
            if (cancel_polled(sc, last_host_poll)) return;   // pbrt_gpu_cancel
            const uint64_t pi = (uint64_t)((py - y0) * (x1 - x0) + (px - x0));
            if (mb) t.rng.state = mb_state((uint64_t)tile, pi, 0);
            start_pixel(t);
            // camera sample: pFilm = pixel + Get2D() == pixel corner; pLens = Get2D() = (0,0)
            const double fx = (double)px + 0.0, fy = (double)py + 0.0;
            Footprint fp;
            int64_t p0x, p0y, p1x, p1y;
            // With n_dims >= 1 the camera's Get2D is stratified 2D dim 0 == (0,0) for every
            // sample, so pFilm is the pixel corner and the footprint is per pixel; with
            // n_dims == 0 it comes from the RNG and the footprint is per sample.
            const bool reg = rp.ndims >= 1 &&
                             footprint(film, fx, fy, px0, py0, px1, py1, fp, p0x, p0y, p1x, p1y) == 0;
            double acc[4][3];
            if (reg)
                for (int k = 0; k < fp.n; k++)
                    for (int c = 0; c < 3; c++) acc[k][c] = tf[fp.off[k] * 3 + c];
            while (next_sample(t)) {
                // (a pixel of large spp runs for milliseconds: poll inside it too)
                if ((t.sample_index & 15) == 0 && cancel_polled(sc, last_host_poll)) return;
                if (mb) t.rng.state = mb_state((uint64_t)tile, pi, (uint64_t)t.sample_index);
                V2 u0 = get2d(t);
                V2 plens = get2d(t);
                double tu = get1d(t);
                Ray ray = camera_ray(cam, (double)px + u0.x, (double)py + u0.y, tu, plens);
                const bool fid = (rp.flags & PBRT_FLAG_PANIC_FIDELITY) != 0;
                Spec L = (rp.integrator == PBRT_INTEGRATOR_PATH)
                             ? path_li(sc, t, ray, rp.max_depth, rp.rr_threshold, fid)
                             : direct_li(sc, t, ray, rp.max_depth, rp.dl_strategy, fid);
                paths++;
                if (t.panic) {
                    PanicRec pr;
                    pr.kind = t.panic;
                    pr.sample = t.sample_index;
                    pr.bounce = t.bounce;
                    pr.pad = 0;
                    pr.px = px;
                    pr.py = py;
                    panics[slot] = pr;
                    atomicExch(&ctr->any_panic, 1);
                    return;
                }
                if (has_nans(L)) L = spec(0.1);   // integrator.go:256-262
                if (0.0 > film.max_sample_luminance) L = smuls(L, film.max_sample_luminance / 0.0);   // L.Y() == 0
                if (reg) {
                    for (int k = 0; k < fp.n; k++) {
                        Spec a = smuls(L, fp.w[k]);
                        acc[k][0] += a.r; acc[k][1] += a.g; acc[k][2] += a.b;
                    }
                } else {
                    // general footprint: FilmTile.AddSample straight into the slot
                    const double sfx = (double)px + u0.x, sfy = (double)py + u0.y;
                    double dx = sfx - 0.5, dy = sfy - 0.5;
                    p0x = gomath::to_int(gomath::max(gomath::ceil(dx - film.filter_radius_x), (double)px0));
                    p0y = gomath::to_int(gomath::max(gomath::ceil(dy - film.filter_radius_y), (double)py0));
                    p1x = gomath::to_int(gomath::min(gomath::floor(dx + film.filter_radius_x) + 1, (double)px1));
                    p1y = gomath::to_int(gomath::min(gomath::floor(dy + film.filter_radius_y) + 1, (double)py1));
                    const double ifx = 1.0 / film.filter_radius_x, ify = 1.0 / film.filter_radius_y;
                    int64_t tw = px1 - px0;
                    for (int64_t y = p0y; y < p1y; y++) {
                        int iy = (int)gomath::to_int(
                            gomath::min(gomath::floor(gomath::abs(((double)y - dy) * ify * 16.0)), 16.0 - 1));
                        for (int64_t x = p0x; x < p1x; x++) {
                            int ix = (int)gomath::to_int(
                                gomath::min(gomath::floor(gomath::abs(((double)x - dx) * ifx * 16.0)), 16.0 - 1));
                            Spec a = smuls(L, 1.0 * film.filter_table[iy * 16 + ix]);
                            double* p = tf + ((x - px0) + (y - py0) * tw) * 3;
                            p[0] += a.r; p[1] += a.g; p[2] += a.b;
                        }
                    }
                }
            }
            if (reg)
                for (int k = 0; k < fp.n; k++)
                    for (int c = 0; c < 3; c++) tf[fp.off[k] * 3 + c] = acc[k][c];
        }
    }
    atomicAdd(&ctr->paths, paths);
    atomicAdd(&ctr->camera_samples, paths);
    atomicAdd(&ctr->closest_rays, (unsigned long long)t.closest_rays);
    atomicAdd(&ctr->shadow_rays, (unsigned long long)t.shadow_rays);
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
    int32_t pad;
};
struct WaveBufs {
    PixelRec* prec;     // [slot][ppt]
    double* s1d;        // [slot][ppt][ndims * spp]
    uint64_t* memb;     // [slot][ppt][spp]   PCG32 state at sample k's offset
    double* L;          // [slot][ppt][spp][3]
    uint32_t* rays;     // [slot][ppt][spp]      the sample's reference ray counts (kRayClosest / kRayShadow)
    PanicRec* ppanic;   // [slot][ppt]        first panic of the pixel in sample order
    int32_t* tile_npx;  // [slot]             pixels with records (a panic ends the tile)
    int64_t ppt;        // pixel records per tile slot (tile_size^2)
    int64_t s1d_stride; // ndims * spp
};
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
__device__ uint64_t start_pixel_wave(const RenderParams& rp, const PcgJump& J, uint64_t S, uint64_t inc, double* s1d,
                                     uint16_t* other, uint32_t* vbuf, uint64_t* sh_state) {
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
    if (!serial_sp) {
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
            if (lane == 0) *sh_state = pcg_advance(J, S, inc, (uint64_t)(E + R));
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
                    double* o = wb.L + (rec * n + k) * 3;
                    o[0] = 0.0;
                    o[1] = 0.0;
                    o[2] = 0.0;
                    wb.rays[rec * n + k] = kRayClosest;   // the camera ray's (missed or maxDepth 1) query
                } else {
                    w = t;
                    c.rng.state = kMB ? mb_state(meta[j].tile, (uint64_t)(rec % wb.ppt), (uint64_t)k)
                                      : wb.memb[rec * n + k];
                    c.rng.inc = meta[j].inc;
                    c.draws = 0;
                    c.cur1d = 1;   // camera: Get2D pFilm, Get2D pLens, Get1D time (stratified)
                    c.cur2d = 2;
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
                double* o = wb.L + (rec * n + k) * 3;
                const Spec Lp = *ps.L;
                o[0] = Lp.r;
                o[1] = Lp.g;
                o[2] = Lp.b;
                wb.rays[rec * n + k] = *ps.rays;
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

template <int P, bool kMB = false, bool kX = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kPathsWaves, 8))) void k_paths_ci(
    DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr,
    int s1d_lds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];   // paths_group_lds<P>
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;   // one wave per workgroup
    stage_nodes(sc);
    paths_group<P, kMB, kX>(sc, rp, wb, slot_base, (int64_t)blockIdx.x * P, nrec, ctr, lds, s1d_lds);
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
    double* o = wb.L + (p.rec * n + p.k) * 3;
    o[0] = p.L.r;
    o[1] = p.L.g;
    o[2] = p.L.b;
    wb.rays[p.rec * n + p.k] = p.rays;
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

template <bool kX = false>
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

template <bool kMB, bool kX = false>
__global__ __launch_bounds__(kWave) void k_pw_start(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                    int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc,
                                                    const int* __restrict__ ldp, PwPath* __restrict__ paths,
                                                    PwQueues qs, unsigned long long* __restrict__ pkey) {
    const int n = rp.spp;
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
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
    c.rng.state = kMB ? mb_state(tile, (uint64_t)pi, (uint64_t)k) : wb.memb[rec * n + k];
    c.rng.inc = pcg_inc_of(tile);
    c.draws = 0;
    c.cur1d = 1;   // camera: Get2D pFilm, Get2D pLens, Get1D time (stratified)
    c.cur2d = 2;
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
    bool done = path_step<1, kX>(sc, pc, ss, c, s, rp.max_depth, rp.rr_threshold, nullptr, pnc, bnc);
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
        const bool hit = bvh_walk<false>(sc, ray, stack_lds + threadIdx.x, panic, best, ph);
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

template <bool kX = false>
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
                const bool occluded = bvh_traverse<true>(sc, sr, nullptr, stack_lds + threadIdx.x, panic);
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

// THROUGHPUT mode setup for k_paths_ci<P, true>, one wave per pixel record:
// StartPixel on the pixel's own stream mb_state(tile, pi, 0) and bounce 1
// (camera ray, first hit, BSDF), written to the PixelRec / s1d buffers the
// EXACT pipeline fills with k_wf_primary + k_chain_ci. The same arithmetic as
// the serial kernel's pixel prologue.
template <bool kX = false>
__global__ __launch_bounds__(kWave) void k_mb_setup(DevScene sc, RenderParams rp, ChainLayout lay,
                                                    const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
                                                    int64_t nslots_batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint16_t stack_lds[64 * kStackStride];
    __shared__ uint64_t sh_state;
    const int lane = threadIdx.x;
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const int64_t bslot = blockIdx.x / wb.ppt, pi = blockIdx.x % wb.ppt, rec = blockIdx.x;
    if (bslot >= nslots_batch) return;
    const int64_t tile = tile_of_slot(rp, slot_base + bslot);
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile, x0, y0, x1, y1);
    if (pi == 0 && lane == 0) wb.tile_npx[bslot] = (int32_t)((x1 - x0) * (y1 - y0));
    if (pi >= (x1 - x0) * (y1 - y0)) return;
    const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
    const int n = rp.spp;
    double* s1d = (double*)(lds + lay.s1d);
    (void)start_pixel_wave(rp, *jump, mb_state((uint64_t)tile, (uint64_t)pi, 0), pcg_inc_of((uint64_t)tile), s1d,
                           (uint16_t*)(lds + lay.other), (uint32_t*)(lds + lay.vbuf), &sh_state);
    for (int idx = lane; idx < rp.ndims * n; idx += kWave) wb.s1d[rec * wb.s1d_stride + idx] = s1d[idx];
    int panic0 = 0, hit = 0;
    SI si0;
    BSDF b0;
    BSDFX bx0;
    b0.n_bxdfs = 0;
    bx0.kind = BXDF_KIND_LAMBERT;
    bx0.n = 0;
    Ray ray = camera_ray(*sc.camera, (double)px + 0.0, (double)py + 0.0, s1d[1 < n ? 1 : 0], V2{0.0, 0.0});
    if (n > 1 && 1 < rp.max_depth) {
        hit = bvh_traverse<false>(sc, ray, &si0, stack_lds + lane, panic0) ? 1 : 0;
        if (!panic0 && hit && (kX ? compute_bsdf_x(sc, si0, b0, bx0) : compute_bsdf(sc, si0, b0)) < 0) panic0 = -1;
    }
    if (panic0) hit = 0;
    if (lane == 0) {
        PixelRec& pr = wb.prec[rec];
        pr.si = si0;
        pr.b = b0;
        if constexpr (kX) pr.x = bx0;
        pr.wo = ray.d;
        pr.hit = hit;
        pr.nvalid = n;
        pr.panic0 = panic0;
    }
}

// One thread per tile-film pixel: the tile film of the serial replay.
__global__ __launch_bounds__(256) void k_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp,
                                              WaveBufs wb, int64_t slot_base, int64_t nslots_batch,
                                              double* __restrict__ films, const int* __restrict__ cancel_seen) {
    // a cancelled render's samples are incomplete: its film is not valid (pbrt_gpu_cancel)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(cancel_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
        return;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = rp.slot_w * rp.slot_h;
    if (gid >= nslots_batch * per) return;
    const int64_t bslot = gid / per, fi = gid % per;
    const int64_t slot = slot_base + bslot;
    const pbrt_film_desc& film = *film_desc;
    int64_t x0, y0, x1, y1, px0, py0, px1, py1;
    tile_bounds(rp, tile_of_slot(rp, slot), x0, y0, x1, y1);
    film_tile_bounds(film, x0, y0, x1, y1, px0, py0, px1, py1);
    const int64_t tw = px1 - px0;
    if (fi >= tw * (py1 - py0)) return;
    const int64_t fx = px0 + fi % tw, fy = py0 + fi / tw;
    const int n = rp.spp;
    const int64_t npx = wb.tile_npx[bslot];
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    // pixels whose footprint can reach (fx, fy): |p - f| < radius + 1, in row-major order
    for (int64_t py = fy - 2; py <= fy + 2; py++) {
        if (py < y0 || py >= y1) continue;
        for (int64_t px = fx - 2; px <= fx + 2; px++) {
            if (px < x0 || px >= x1) continue;
            const int64_t pi = (py - y0) * (x1 - x0) + (px - x0);
            if (pi >= npx) continue;
            Footprint fp;
            int64_t p0x, p0y, p1x, p1y;
            footprint(film, (double)px + 0.0, (double)py + 0.0, px0, py0, px1, py1, fp, p0x, p0y, p1x, p1y);
            const int64_t want = fi;
            int f = -1;
            for (int q = 0; q < fp.n; q++)
                if (fp.off[q] == want) f = q;
            if (f < 0) continue;
            const double w = fp.w[f];
            const int64_t rec = bslot * wb.ppt + pi;
            const int nv = wb.prec[rec].nvalid;
            const double* Lp = wb.L + rec * n * 3;
            for (int k = 1; k < nv; k++) {
                Spec Ls{Lp[k * 3 + 0], Lp[k * 3 + 1], Lp[k * 3 + 2]};
                if (has_nans(Ls)) Ls = spec(0.1);   // integrator.go:256-262
                if (0.0 > film.max_sample_luminance) Ls = smuls(Ls, film.max_sample_luminance / 0.0);
                a0 += Ls.r * w;
                a1 += Ls.g * w;
                a2 += Ls.b * w;
            }
        }
    }
    double* tf = films + slot * per * 3 + fi * 3;
    tf[0] = a0;
    tf[1] = a1;
    tf[2] = a2;
}

// First panic of each tile slot in pixel order -> panics[slot].
__global__ void k_panic_reduce(WaveBufs wb, int64_t slot_base, int64_t nslots_batch, PanicRec* __restrict__ panics,
                               Counters* __restrict__ ctr) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nslots_batch) return;
    const int npx = wb.tile_npx[b];
    for (int p = 0; p < npx; p++) {
        const PanicRec& r = wb.ppanic[b * wb.ppt + p];
        if (r.kind) {
            panics[slot_base + b] = r;
            atomicExch(&ctr->any_panic, 1);
            return;
        }
    }
}

// Bounce 1 of every pixel record of the batch: the camera ray through the
// pixel corner (pFilm and pLens are (0,0) for every sample), its closest hit
// and BSDF. The ray time is patched by the chain kernel once StartPixel gives it.
// stats.rays_closest / rays_shadow of a batch: every valid sample's counts
// (pixels with records, samples 1 .. nvalid-1), one atomic pair per wave
__global__ __launch_bounds__(256) void k_ray_count(WaveBufs wb, int64_t nb, int n, Counters* __restrict__ ctr,
                                                   const int* __restrict__ cancel_seen) {
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(cancel_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
        return;   // a cancelled render reports no counts
    unsigned long long cl = 0, sh = 0;
    const int64_t total = nb * wb.ppt * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rec = i / n, k = i - rec * n, bs = rec / wb.ppt, pi = rec % wb.ppt;
        if (k < 1 || pi >= wb.tile_npx[bs] || k >= wb.prec[rec].nvalid) continue;
        const uint32_t v = wb.rays[i];
        cl += v & 0xFFFFu;
        sh += v >> 16;
    }
    for (int off = kWave / 2; off > 0; off >>= 1) {
        cl += __shfl_down(cl, off);
        sh += __shfl_down(sh, off);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) {
        atomicAdd(&ctr->closest_rays, cl);
        atomicAdd(&ctr->shadow_rays, sh);
    }
}

template <bool kX = false>
__global__ __launch_bounds__(kWave) void k_wf_primary(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                      int64_t nb) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const int64_t rec = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rec >= nb * wb.ppt) return;
    const int64_t bs = rec / wb.ppt, pi = rec % wb.ppt;
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile_of_slot(rp, slot_base + bs), x0, y0, x1, y1);
    if (pi >= (x1 - x0) * (y1 - y0)) return;
    const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
    int panic0 = 0, hit0 = 0;
    SI si0;
    BSDF b0;
    BSDFX bx0;
    b0.n_bxdfs = 0;
    bx0.kind = BXDF_KIND_LAMBERT;
    bx0.n = 0;
    Ray ray = camera_ray(*sc.camera, (double)px + 0.0, (double)py + 0.0, 0.0, V2{0.0, 0.0});
    // Path.Li traces bounce 1 only below maxDepth (path.go:66); DirectLighting always
    if (rp.spp > 1 && (1 < rp.max_depth || rp.integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING)) {
        hit0 = bvh_traverse<false>(sc, ray, &si0, stack_lds + threadIdx.x, panic0) ? 1 : 0;
        if (!panic0 && hit0 && (kX ? compute_bsdf_x(sc, si0, b0, bx0) : compute_bsdf(sc, si0, b0)) < 0) panic0 = -1;
    }
    PixelRec& pr = wb.prec[rec];
    pr.si = si0;
    pr.b = b0;
    if constexpr (kX) pr.x = bx0;
    pr.wo = ray.d;
    pr.hit = panic0 ? 0 : hit0;
    pr.panic0 = panic0;
    pr.nvalid = rp.spp;
}

// ------------------------------------------- DirectLighting, wave-parallel
// DirectLighting.Li (directlighting.go:62-104) has no chain problem: with
// n_dims >= 1 (and n_dims >= 2 or a pinhole camera) every sample of a pixel
// traces the same camera ray, so hit or miss -- the only thing the number of
// PCG32 draws of a sample depends on -- is per pixel, and sample k of the
// pixel starts at the state after StartPixel advanced by (k - 1) * D.
// k_dl_setup replays the tile's pixels in order (StartPixel, then jump-ahead
// over the pixel's samples); k_dl_samples runs every (pixel, sample) at once.
//
// Draws of one DirectLighting sample (pixel.go:60-80 counters): the camera's
// Get2D pFilm, Get2D pLens, Get1D time (camera.go via integrator.go:240-255),
// then on a hit UniformSampleAllLights' two Get2D per light (clones carry no
// sample arrays, #23) or UniformSampleOneLight's Get1D + 2 Get2D, then the two
// Get2D of SpecularReflect / SpecularTransmit when maxDepth > 1.
__device__ __forceinline__ uint32_t dl_draws(const RenderParams& rp, int hit, int n_lights) {
    int c1 = 0, c2 = 0;
    uint32_t d = 0;
    auto g1 = [&]() { if (c1 < rp.ndims) c1++; else d += 1; };
    auto g2 = [&]() { if (c2 < rp.ndims) c2++; else d += 2; };
    g2();
    g2();
    g1();
    if (hit) {
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
        if (1 < rp.max_depth) {
            g2();
            g2();
        }
    }
    return d;
}

// One wave per tile slot: the tile's pixels in order. Leaves each pixel's
// stratified values in wb.s1d, the PCG32 state of each of its samples in
// wb.memb (slot 0 of a pixel: its panic key, reset here), and the pixels
// with records in wb.tile_npx (a camera-ray panic ends the tile, as in
// k_chain_ci). THROUGHPUT mode: each pixel and sample on its own stream.
__global__ __launch_bounds__(kWave) void k_dl_setup(DevScene sc, RenderParams rp, ChainLayout lay,
                                                    const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
                                                    int64_t nb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint64_t sh_state;
    const int64_t bs = blockIdx.x;
    const int lane = threadIdx.x;
    if (bs >= nb || cancel_requested(sc, (bs & 63) == 0)) return;
    const PcgJump& J = *jump;
    const int64_t tile = tile_of_slot(rp, slot_base + bs);
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile, x0, y0, x1, y1);
    const int64_t npx = (x1 - x0) * (y1 - y0);
    const uint64_t inc = pcg_inc_of((uint64_t)tile);
    const bool mb = rp.mode == PBRT_MODE_THROUGHPUT;
    const int n = rp.spp;
    double* s1d = lay.s1d >= 0 ? (double*)(lds + lay.s1d) : nullptr;
    uint16_t* other = (uint16_t*)(lds + lay.other);
    uint32_t* vbuf = (uint32_t*)(lds + lay.vbuf);
    Pcg seed;
    pcg_seed(seed, (uint64_t)tile);   // Sampler.Clone(tile), integrator.go:318,328
    uint64_t S = seed.state;
    int64_t used = npx;
    for (int64_t pi = 0; pi < npx; pi++) {
        if (cancel_requested(sc, (pi & 15) == 0)) {   // pbrt_gpu_cancel (large spp: a pixel's StartPixel is long)
            used = pi;
            break;
        }
        const int64_t rec = bs * wb.ppt + pi;
        double* gs1d = wb.s1d + rec * wb.s1d_stride;
        double* sp = s1d ? s1d : gs1d;
        const uint64_t S1 =
            start_pixel_wave(rp, J, mb ? mb_state((uint64_t)tile, (uint64_t)pi, 0) : S, inc, sp, other, vbuf, &sh_state);
        if (s1d)
            for (int idx = lane; idx < rp.ndims * n; idx += kWave) gs1d[idx] = s1d[idx];
        PixelRec& pr = wb.prec[rec];
        const int hit = pr.hit, panic0 = pr.panic0;
        const uint64_t D = dl_draws(rp, hit, sc.n_lights);
        uint64_t* mst = wb.memb + rec * n;
        for (int k = 1 + lane; k < n; k += kWave)
            mst[k] = mb ? mb_state((uint64_t)tile, (uint64_t)pi, (uint64_t)k) : pcg_advance(J, S1, inc, (uint64_t)(k - 1) * D);
        if (lane == 0) {
            mst[0] = ~0ULL;
            if (hit) {   // the camera ray's time (Get1D, dim 0) of the pixel's first traced sample
                const int64_t px = x0 + pi % (x1 - x0), py = y0 + pi / (x1 - x0);
                pr.si.time = camera_ray(*sc.camera, (double)px, (double)py, sp[1 < n ? 1 : 0], V2{0.0, 0.0}).time;
            }
            pr.nvalid = n;
        }
        __syncthreads();   // the StartPixel staging is reused by the next pixel
        if (panic0) {      // its first traced sample panics at bounce 1: the tile ends here
            used = pi + 1;
            break;
        }
        S = pcg_advance(J, S1, inc, (uint64_t)(n - 1) * D);
    }
    if (lane == 0) wb.tile_npx[bs] = (int32_t)used;
}

// One lane per (pixel record, traced sample): DirectLighting.Li at depth 0
// from the pixel's bounce-1 record, with the sample's own PCG32 state.
// Radiance to wb.L; a panic lowers the pixel's key (sample << 32 | kind + 1)
// in wb.memb[rec * spp + 0] (the first panic in sample order wins).
__global__ __launch_bounds__(kWave) void k_dl_samples(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                      int64_t nrec) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const int n = rp.spp;
    if (n < 2) return;
    // grid-stride over every (pixel record, sample): a bounded grid, so a cancel
    // (polled every 16 passes) ends the kernel quickly at any spp
    const int64_t total = nrec * (n - 1), stride = (int64_t)gridDim.x * blockDim.x;
    int pass = 0;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx - threadIdx.x < total; idx += stride) {
        if ((++pass & 15) == 0 && cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
        if (idx >= total) continue;
        const int64_t rec = idx / (n - 1);
        const int k = 1 + (int)(idx - rec * (n - 1));
        const int64_t bs = rec / wb.ppt, pi = rec % wb.ppt;
        if (pi >= wb.tile_npx[bs]) continue;
        const PixelRec& pr = wb.prec[rec];
        double* o = wb.L + (rec * n + k) * 3;
        Spec L = spec(0);
        int panic = pr.panic0;
        uint64_t shadow = 0;   // visibility rays traced (the camera ray's query is counted below)
        if (!panic && pr.hit) {
            Cursor c;
            c.rng.state = wb.memb[rec * n + k];
            c.rng.inc = pcg_inc_of((uint64_t)tile_of_slot(rp, slot_base + bs));
            c.draws = 0;
            c.cur1d = c.cur2d = 0;
            c.k = k;
            c.kdep = 0;
            const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, rp.ndims};
            c_get2d(c, ss);   // camera: pFilm, pLens, time
            c_get2d(c, ss);
            c_get1d(c, ss);
            L = L + spec(0);   // si.Le(si.Wo): no primitive carries an area light
            const int nl = sc.n_lights;
            if (nl > 0) {
                if (rp.dl_strategy == PBRT_DL_UNIFORM_SAMPLE_ALL) {   // integrator.go:23-46
                    Spec acc = spec(0);
                    for (int j = 0; j < nl && !panic; j++) {
                        const V2 ul = c_get2d(c, ss);
                        c_get2d(c, ss);
                        acc = acc + estimate_direct(sc, stack_lds + threadIdx.x, panic, pr.si, pr.b, j, ul, &shadow);
                    }
                    L = L + acc;
                } else {   // UniformSampleOneLight with no distribution (integrator.go:48-77)
                    const int ln = (int)gomath::to_int(gomath::min(c_get1d(c, ss) * (double)nl, (double)(nl - 1)));
                    const V2 ul = c_get2d(c, ss);
                    c_get2d(c, ss);
                    const Spec s = estimate_direct(sc, stack_lds + threadIdx.x, panic, pr.si, pr.b, ln, ul, &shadow);
                    if (!panic && max_component(s) > 10) panic = PBRT_PANIC_LD_GT_10;
                    L = L + s;
                }
            }
            // SpecularReflect / SpecularTransmit: black for a Lambertian-only BSDF
        }
        o[0] = L.r;
        o[1] = L.g;
        o[2] = L.b;
        wb.rays[rec * n + k] = kRayClosest + (uint32_t)shadow * kRayShadow;
        if (panic)
            atomicMin((unsigned long long*)&wb.memb[rec * n],
                      ((unsigned long long)k << 32) | (unsigned long long)((panic + 1) & 0xFF));

    }
}

// Per pixel record: its first panic (sample order) -> wb.ppanic, and the
// traced-path counters of pixels that finish (as paths_group counts them).
__global__ void k_dl_panics(RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr) {
    const int64_t rec = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rec >= nrec) return;
    const int64_t bs = rec / wb.ppt, pi = rec % wb.ppt;
    if (pi >= wb.tile_npx[bs]) return;
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile_of_slot(rp, slot_base + bs), x0, y0, x1, y1);
    PanicRec p{0, 0, 0, 0, x0 + pi % (x1 - x0), y0 + pi / (x1 - x0)};
    const uint64_t key = rp.spp >= 2 ? wb.memb[rec * rp.spp] : ~0ULL;
    if (wb.prec[rec].panic0) {
        p.kind = wb.prec[rec].panic0;
        p.sample = 1;
        p.bounce = 1;
    } else if (key != ~0ULL) {
        p.kind = (int)(key & 0xFF) - 1;
        p.sample = (int)(key >> 32);
        p.bounce = 1;
    }
    wb.ppanic[rec] = p;
    if (!p.kind && rp.spp > 1) {
        atomicAdd(&ctr->paths, (unsigned long long)(rp.spp - 1));
        atomicAdd(&ctr->camera_samples, (unsigned long long)(rp.spp - 1));
    }
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
template <bool kX = false>
__global__ __launch_bounds__(kWave) void k_tile_cost(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base,
                                                     int64_t nb, float* __restrict__ feat,
                                                     uint64_t* __restrict__ keys) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;
    stage_nodes(sc);
    const int64_t bs = blockIdx.x;
    const int lane = threadIdx.x;
    if (bs >= nb) return;
    const int64_t tile = tile_of_slot(rp, slot_base + bs);
    int64_t x0, y0, x1, y1;
    tile_bounds(rp, tile, x0, y0, x1, y1);
    const int64_t npx = (x1 - x0) * (y1 - y0);
    const uint64_t inc = pcg_inc_of((uint64_t)tile);
    const SpecSampler ss{nullptr, rp.spp, rp.ndims};   // k < 0: stratified values are never read
    double work = 0;
    int hits = 0;
    for (int64_t it = lane; it < npx * kProbes; it += kWave) {
        const int64_t pi = it / kProbes;
        const PixelRec& pr = wb.prec[bs * wb.ppt + pi];
        if (!pr.hit) continue;
        hits += (it % kProbes) == 0;
        Cursor c;
        c.rng.state = mb_state((uint64_t)tile, (uint64_t)pi, 0x70726f6265ULL + (uint64_t)(it % kProbes));
        c.rng.inc = inc;
        c.draws = 0;
        c.cur1d = 1;
        c.cur2d = 2;
        c.k = -1;
        c.kdep = 0;
        Spec beta = spec(1);
        double eta_scale = 1.0;
        int bounces = 1;
        Ray ray;
        int r = traj_scatter<kX>(sc, pr.si, pr.b, pr.x, pr.wo, c, ss, beta, eta_scale, bounces, ray, rp.max_depth,
                                 rp.rr_threshold);
        while (r == 0) {
            SI si;
            int panic = 0;
            if (!bvh_traverse<false>(sc, ray, &si, stack_lds + lane, panic) || panic) break;
            BSDF b;
            BSDFX x;
            if ((kX ? compute_bsdf_x(sc, si, b, x) : compute_bsdf(sc, si, b)) < 0) break;
            r = traj_scatter<kX>(sc, si, b, x, ray.d, c, ss, beta, eta_scale, bounces, ray, rp.max_depth,
                                 rp.rr_threshold);
        }
        work += (double)c.draws * (double)bounces;
    }
    for (int o = kWave / 2; o > 0; o >>= 1) {
        work += __shfl_xor(work, o);
        hits += __shfl_xor(hits, o);
    }
    if (lane == 0) {
        const double w = work / kProbes * (double)(rp.spp - 1);
        const float cost = (float)(w + kCostPixel * (double)npx);
        feat[4 * bs + 0] = (float)w;
        feat[4 * bs + 1] = (float)hits;
        feat[4 * bs + 2] = (float)npx;
        feat[4 * bs + 3] = cost;
        keys[bs] = ((uint64_t)~__float_as_uint(cost) << 32) | (uint64_t)bs;
    }
}
__global__ void k_order_of_keys(const uint64_t* __restrict__ keys, int64_t nb, uint32_t* __restrict__ order) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) order[i] = (uint32_t)keys[i];
}

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
#ifndef PBRT_CI_EU_WAVES
#define PBRT_CI_EU_WAVES 2   // k_chain_ci waves/SIMD (build option)
#endif
#ifndef PBRT_CHAIN_LB
#define PBRT_CHAIN_LB 1   // leaf boxes per scan iteration in k_chain_ci's traversal (build option)
#endif
constexpr uint32_t kNoOff = 0xFFFFFFFFu;
constexpr uint32_t kBadSpecD = 0xFFFFFFFEu;   // speculative lane could not resolve D
constexpr uint32_t kBadExactD = 0xFFFFFFFDu;  // the exact head's trajectory panics
struct RingEnt {
    uint32_t tag;   // offset this entry resolves (kNoOff: empty)
    uint32_t d;     // its draw count D, or kBadSpecD / kBadExactD
    uint64_t st;    // PCG32 state at the offset
};
struct CiGroup {
    uint64_t S;     // PCG32 state at the current pixel's first sample (offset 0)
    int64_t pi;     // current pixel (row-major index in the tile)
    int64_t npx;    // pixels of the tile
    uint32_t head;  // offset of sample kh
    uint32_t nxt;   // next offset to issue (same parity as head)
    int kh;         // next sample without an offset
    int phase;      // 0 needs a pixel, 1 resolving offsets, 2 tile finished
    int reissue;    // the head must be re-run with its sample index known
    int pad;
};

//
// kW > 1: one tile per workgroup of kW waves (lanes_per_tile = 64 * kW). The
// tile's chain then advances kW times as many candidates per step, which cuts
// the slowest tile's latency, the frame's critical path when tiles are few
// per GPU (a multi-GPU shard). Idle lanes are ranked across the waves through
// LDS; StartPixel runs on the first wave.
// kDepth: traversal stack entries per lane. Trees of <= kLdsNodes (64) nodes
// are staged in LDS and walk their leaves only (no stack); larger trees walk
// with the reference's [64] stack (bvh.go:670).
template <int kW, int kDepth = 0, bool kX = false>
__global__ __launch_bounds__(kWave * kW) __attribute__((amdgpu_waves_per_eu(PBRT_CI_EU_WAVES, 8))) void k_chain_ci(
    DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base,
    int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr,
    const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint64_t t_begin = wall_clock64();
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
    uint64_t st0 = 0;
    bool tracing = false;
    Cursor c;
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
                const uint64_t S1 = start_pixel_wave(rp, J, gs[q].S, incq, sp, other, vbuf, &sh_state);
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
                    } else {   // no traced bounce: every sample is black and draws nothing
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
        const SpecSampler ss{wb.s1d + rec * wb.s1d_stride, n, ndims};
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
            const int nspec = min(nidle - re, avail);
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
                c.cur1d = 1;   // camera: Get2D pFilm, Get2D pLens, Get1D time (stratified)
                c.cur2d = 2;
                c.k = exact ? sg.kh : -1;
                c.kdep = 0;
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
                    e.d = r == 1 ? c.draws : (c.k >= 0 ? kBadExactD : kBadSpecD);
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
            if (!dense) bvh_walk<false, kT, PBRT_CHAIN_LB>(sc, ray, stack, panic, best, ph);
#else
        if (tracing) {
            int panic = 0, best;
            V3 ph;
            bvh_walk<false, kT, PBRT_CHAIN_LB>(sc, ray, stack, panic, best, ph);
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
                e.d = d;
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
                const uint32_t d = e.d;
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
            if (s2.phase != 1 || off < s2.head || (cs == 2u && ((off ^ s2.head) & 1u)) || s2.pi != sg.pi) {
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
    if (tid == 0) {
        if (ticks && G == 1 && bs < nslots_batch) ticks[bs] = (uint32_t)min(wall_clock64() - t_begin, (uint64_t)0xFFFFFFFFu);
    }
}

// ---------------------------------------------------------- merge kernel
// Film.MergeFilmTile (film.go:115-132) in tile-index order. A film pixel is
// covered by at most the 3x3 tiles around its own (filter radius < tile size).
__global__ __launch_bounds__(256) void k_merge_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp,
                                                    const double* __restrict__ films, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rp.film_w * rp.film_h) return;
    const pbrt_film_desc& f = *film_desc;
    const int64_t x = rp.film_min_x + i % rp.film_w, y = rp.film_min_y + i / rp.film_w;
    const int64_t tx = (x - rp.film_min_x) / rp.tile_size, ty = (y - rp.film_min_y) / rp.tile_size;
    double v0 = 0, v1 = 0, v2 = 0;
    for (int64_t dy = -1; dy <= 1; dy++) {
        for (int64_t dx = -1; dx <= 1; dx++) {
            int64_t cx = tx + dx, cy = ty + dy;
            if (cx < 0 || cy < 0 || cx >= rp.ntx || cy >= rp.nty) continue;
            int64_t tile = cy * rp.ntx + cx;
            if (tile < rp.tile_begin || (tile - rp.tile_begin) % rp.tile_stride != 0) continue;
            int64_t slot = (tile - rp.tile_begin) / rp.tile_stride;
            if (slot >= rp.n_slots) continue;
            int64_t x0, y0, x1, y1, px0, py0, px1, py1;
            tile_bounds(rp, tile, x0, y0, x1, y1);
            film_tile_bounds(f, x0, y0, x1, y1, px0, py0, px1, py1);
            if (x < px0 || x >= px1 || y < py0 || y >= py1) continue;
            const double* c = films + slot * (rp.slot_w * rp.slot_h * 3) + ((x - px0) + (y - py0) * (px1 - px0)) * 3;
            // spectrum.go:35-41 RGBToXYZ
            v0 += 0.412453 * c[0] + 0.357580 * c[1] + 0.180423 * c[2];
            v1 += 0.212671 * c[0] + 0.715160 * c[1] + 0.072169 * c[2];
            v2 += 0.019334 * c[0] + 0.119193 * c[1] + 0.950227 * c[2];
        }
    }
    out[i * 3 + 0] = v0;
    out[i * 3 + 1] = v1;
    out[i * 3 + 2] = v2;
}

// ------------------------------------------------------- batch intersect
__global__ __launch_bounds__(kWave) void k_intersect(DevScene sc, int64_t n, const double* __restrict__ rays,
                                                     double* __restrict__ out, int any_hit) {
    __shared__ uint16_t stack_lds[64 * kStackStride];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* q = rays + 7 * i;
    Ray r{V3{q[0], q[1], q[2]}, V3{q[3], q[4], q[5]}, q[6], 0};
    int panic = 0;
    if (any_hit) {
        bool h = bvh_traverse<true>(sc, r, nullptr, stack_lds + threadIdx.x, panic);
        out[i] = panic ? gomath::nan() : (h ? 1.0 : 0.0);
        return;
    }
    SI si;
    si.p = si.n = V3{0, 0, 0};
    si.prim = -1;
    bool h = bvh_traverse<false>(sc, r, &si, stack_lds + threadIdx.x, panic);
    double* o = out + 9 * i;
    if (panic) {
        for (int k = 0; k < 9; k++) o[k] = gomath::nan();
        return;
    }
    o[0] = h ? 1.0 : 0.0;
    o[1] = r.tmax;
    o[2] = h ? (double)si.prim : -1.0;
    o[3] = si.p.x; o[4] = si.p.y; o[5] = si.p.z;
    o[6] = si.n.x; o[7] = si.n.y; o[8] = si.n.z;
}

}  // namespace

// =============================================================== C ABI
// Experiment knobs (environment), read ONCE when a context is created
// (pbrt_gpu_create), never per launch; defaults are the measured best.
struct Knobs {
    int ci_waves = 0;          // PBRT_CI_WAVES = 1, 2, 4, 8 (0: by tile count)
    int ci_stride = 0;         // PBRT_CI_STRIDE = 1, 2 (0: 2 at one wave per tile, else 1)
    int ci_heavy_waves = 4;    // PBRT_CI_HEAVY_WAVES = 4, 8
    int64_t ci_heavy = -1;     // PBRT_CI_HEAVY = K forces the heavy tile count (tests)
    bool ci_split = true;      // PBRT_CI_SPLIT=0
    bool ci_order = true;      // PBRT_CI_ORDER=0
    bool ci_probe = true;      // PBRT_CI_PROBE=0
    bool paths_s1d_lds = false;// PBRT_PATHS_S1D=lds
    int paths_ci = -1;         // PBRT_PATHS_CI = 0, 2, 4, 8 (-1: auto)
    int paths_wf = -1;         // PBRT_PATHS_WF = 0 / 1 (-1: mesh scenes)
    bool pw_sort = false;      // PBRT_PW_SORT=1
    double pw_gb = 24.0;       // PBRT_PW_GB
    double wave_buffer_gb = 0; // PBRT_WAVE_BUFFER_GB (0: min(96 GB, half the free HBM))
    int64_t ci_exclusive = 0;  // PBRT_CI_EXCLUSIVE = K: a shard's K heaviest tiles get a CU each (LDS pad)
    bool ci_dense = false;     // PBRT_CI_DENSE=1 (builds with -DPBRT_CI_DENSE_WALK): k_chain_ci's closest hit by
                               // bvh_walk_dense (bit-exact; slower on B)
    int cull_group = 4;        // PBRT_CULL_GROUP: leaves per culling group
    int cull_min = 2;          // PBRT_CULL_MIN
    bool cull_groups = true;   // PBRT_CULL_GROUPS=0
    static Knobs from_env() {
        Knobs k;
        auto ival = [](const char* n, int& out) { if (const char* e = getenv(n)) out = atoi(e); };
        if (const char* e = getenv("PBRT_CI_WAVES")) {
            const int v = atoi(e);
            if (v == 1 || v == 2 || v == 4 || v == 8) k.ci_waves = v;
        }
        if (const char* e = getenv("PBRT_CI_STRIDE")) {
            const int v = atoi(e);
            if (v == 1 || v == 2) k.ci_stride = v;
        }
        if (const char* e = getenv("PBRT_CI_HEAVY_WAVES")) k.ci_heavy_waves = atoi(e) == 8 ? 8 : 4;
        if (const char* e = getenv("PBRT_CI_HEAVY")) k.ci_heavy = (int64_t)atoll(e);
        if (const char* e = getenv("PBRT_CI_SPLIT")) k.ci_split = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_DENSE")) k.ci_dense = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_EXCLUSIVE")) k.ci_exclusive = std::max<int64_t>(0, (int64_t)atoll(e));
        if (const char* e = getenv("PBRT_CI_ORDER")) k.ci_order = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_PROBE")) k.ci_probe = atoi(e) != 0;
        if (const char* e = getenv("PBRT_PATHS_S1D")) k.paths_s1d_lds = std::strcmp(e, "lds") == 0;
        if (const char* e = getenv("PBRT_PATHS_CI")) {
            const int v = atoi(e);
            if (v == 0 || v == 2 || v == 4 || v == 8) k.paths_ci = v;
        }
        if (const char* e = getenv("PBRT_PATHS_WF")) k.paths_wf = atoi(e) == 1 ? 1 : 0;
        if (const char* e = getenv("PBRT_PW_SORT")) k.pw_sort = atoi(e) == 1;
        if (const char* e = getenv("PBRT_PW_GB")) k.pw_gb = atof(e) > 0 ? atof(e) : k.pw_gb;
        if (const char* e = getenv("PBRT_WAVE_BUFFER_GB")) k.wave_buffer_gb = atof(e) > 0 ? atof(e) : 0;
        if (const char* e = getenv("PBRT_CULL_GROUP")) k.cull_group = std::max(2, atoi(e));
        if (const char* e = getenv("PBRT_CULL_MIN")) k.cull_min = std::max(0, atoi(e));
        int cg = 1;
        ival("PBRT_CULL_GROUPS", cg);
        k.cull_groups = cg != 0;
        return k;
    }
};

struct pbrt_gpu_ctx {
    Knobs knobs;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // heavy/light split of k_chain_ci: the heaviest tiles with 4 waves each on
    // the main stream, the rest on stream2, concurrently
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_split = nullptr, ev_join = nullptr;
    MeshBuild mesh;                      // triangle meshes + their LBVH (extension)
    int64_t heavy_k = 0;                 // slots at the front of h_slot_order that get 4 waves
    int64_t last_heavy = 0;              // heavy slots of the last EXACT launch (0: no split)
    std::vector<uint32_t> h_last_ticks;  // per-slot chain ticks of the last EXACT frame
    std::vector<uint8_t> h_slot_kw;      // waves per tile each slot ran with in the last frame
    double* film_target = nullptr;   // caller buffer of the last render_async_into
    int lanes_per_wave = 64;
    bool lanes_per_wave_set = false;
    int min_waves = 1;      // amdgpu_waves_per_eu variant of k_render_exact
    int occ_req = 0;        // opts.occupancy as given (0 = each kernel's default)
    int kernel_req = PBRT_KERNEL_AUTO;
    int last_kernel = 0;    // PBRT_KERNEL_SERIAL / PBRT_KERNEL_WAVE
    PcgJump* d_jump = nullptr;
    pbrt_distribution_desc host_dist;
    // wave-parallel path (k_wf_primary, k_chain_ci, k_paths_ci / k_pw_*, k_film)
    ChainLayout lay{};
    bool use_spec = false;
    unsigned char* d_wave = nullptr;   // per-batch pixel records, stratified values, RNG states, L
    size_t wave_cap = 0;
    int64_t wave_batch = 0;            // tile slots per batch
    int tiles_per_wave = 1;            // k_chain_ci lane groups per wave (64 / lanes per tile)
    std::vector<hipEvent_t> bev;       // per batch: before the chain, after the chain, after the paths
    int n_batches = 0;
    int n_simd = 1024;                 // SIMDs of the device (4 per CU)
    size_t lds_per_block = 65536;      // the device's LDS limit per workgroup (sharedMemPerBlock)
    WaveBufs wb{};
    bool use_ci = false;   // the Path chain stage (k_chain_ci)
    bool use_dl = false;   // DirectLighting on k_dl_setup / k_dl_samples
    ChainLayout lay_ci{};
    // device scene
    pbrt_shape_desc* d_shapes = nullptr;
    pbrt_material_desc* d_materials = nullptr;
    pbrt_primitive_desc* d_prims = nullptr;
    DevNode* d_nodes = nullptr;
    uint32_t* d_order = nullptr;     // [8][n_nodes] preorder visit tables, then [8][n_nodes] leaf lists (dev_order)
    double* d_groups = nullptr;      // leaf culling groups (cull_groups)
    uint32_t* d_gmasks = nullptr;
    int n_groups = 0;
    std::vector<int> h_node_prims;   // nPrimitives per node (leaf count for DevScene)
    DevPrim* d_fprims = nullptr;
    pbrt_light_desc* d_lights = nullptr;
    pbrt_camera_desc* d_camera = nullptr;
    pbrt_film_desc* d_film = nullptr;
    pbrt_distribution_desc* d_dist = nullptr;
    pbrt_scene_desc host_scene;   // counts + film/camera (pointer fields are not kept)
    std::vector<pbrt_light_desc> host_lights;
    bool non_matte = false;       // Mirror, Glass or OrenNayar material: kX wave kernels or the serial kernel
    bool rough_glass = false;     // a Glass material with roughness: serial kernel only
    // per-render buffers (grown on demand)
    double* d_films = nullptr;
    size_t films_cap = 0;
    double* d_s1d = nullptr;
    size_t s1d_cap = 0;
    PanicRec* d_panics = nullptr;
    size_t panics_cap = 0;
    Counters* d_ctr = nullptr;
    // k_chain_ci heaviest-first schedule: per-slot chain time of the last
    // EXACT frame (wall_clock64 ticks) and the slot order derived from it
    uint32_t* d_ticks = nullptr;
    uint32_t* d_slot_order = nullptr;
    int64_t ticks_cap = 0;
    std::vector<uint32_t> h_slot_order;
    // path wavefront (k_pw_*, PBRT_PATHS_WF=1): path records, queues, counters,
    // bounce-1 light estimates, per-pixel panic keys (grown on demand)
    unsigned char* d_pw = nullptr;
    size_t pw_cap = 0;
    // cold-frame schedule (k_tile_cost): per-slot features and sort keys
    float* d_cost = nullptr;
    uint64_t* d_cost_keys = nullptr;
    int64_t cost_cap = 0, cost_n = 0;
    bool probed = false;               // the last EXACT frame ran the cost probe
    uint64_t order_key = 0, ticks_key = 0;
    int64_t ticks_n = 0;
    bool ticks_pending = false;
    double* d_out = nullptr;
    size_t out_cap = 0;
    // last render
    RenderParams rp{};
    bool rendered = false;
    // cancellation (pbrt_gpu_cancel): a flag in fine-grained host memory the
    // kernels poll; it belongs to the render in flight (render_async entry to
    // synchronize) and is cleared when that render ends, so a cancel never
    // outlives its render and never reaches the next one
    std::mutex cancel_mu;
    bool in_flight = false;
    bool cancel_req = false;
    int* h_cancel = nullptr;   // hipHostMalloc (coherent, mapped)
    int* d_cancel = nullptr;   // its device address
    int* d_cancel_seen = nullptr;   // device-memory copy the kernels publish (reset per render)
    std::string err;
    std::chrono::steady_clock::time_point t_start;
};

namespace {

int set_err(pbrt_gpu_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}
#define HIPCHK(ctx, call)                                                                            \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return set_err(ctx, PBRT_E_HIP, std::string(#call ": ") + hipGetErrorString(e_));      \
    } while (0)

template <class T>
int upload(pbrt_gpu_ctx* c, T** dst, const T* src, size_t n) {
    if (n == 0) n = 1;   // keep a valid pointer for empty arrays
    HIPCHK(c, hipMalloc((void**)dst, sizeof(T) * n));
    if (src) HIPCHK(c, hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice));
    return PBRT_OK;
}
template <class T>
int ensure(pbrt_gpu_ctx* c, T** buf, size_t* cap, size_t n) {
    if (*cap >= n && *buf) return PBRT_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    HIPCHK(c, hipMalloc((void**)buf, sizeof(T) * (n ? n : 1)));
    *cap = n;
    return PBRT_OK;
}

DevScene dev_scene(const pbrt_gpu_ctx* c, bool with_dist) {
    DevScene s;
    s.shapes = c->d_shapes;
    s.materials = c->d_materials;
    s.prims = c->d_prims;
    s.nodes = c->d_nodes;
    s.order = c->d_order;
    s.fprims = c->d_fprims;
    s.lights = c->d_lights;
    s.camera = c->d_camera;
    s.film = c->d_film;
    s.dist = with_dist ? c->d_dist : nullptr;
    s.n_prims = c->host_scene.n_prims;
    s.n_nodes = c->host_scene.n_nodes;
    s.n_lights = c->host_scene.n_lights;
    s.use_lds_nodes = 0;
    s.n_leaves = 0;
    for (int i = 0; i < c->host_scene.n_nodes; i++) s.n_leaves += c->h_node_prims[i] > 0;
    s.mesh = c->mesh.view();
    s.groups = c->d_groups;
    s.gmasks = c->d_gmasks;
    s.n_groups = c->n_groups;
    s.cancel = c->d_cancel;
    s.cancel_seen = c->d_cancel_seen;
    // bvh_walk_dense: culling groups over a tree of one primitive per leaf, no meshes
    s.dense_ok = c->knobs.ci_dense && s.n_groups > 0 && s.n_leaves == s.n_prims && s.mesh.n_nodes == 0 &&
                 s.n_nodes <= kLdsNodes;
    return s;
}

// The scene view a launch passes, tagged with its kernel's counter set for
// the mesh-traversal counting build (PBRT_MESH_COUNT; ignored otherwise):
// 1 k_wf_primary, 2 k_chain_ci, 3 k_paths_ci / k_pw_* EXACT, 4 k_mb_setup,
// 5 k_paths_ci / k_pw_* THROUGHPUT, 6 k_render_exact, 7 k_intersect.
DevScene with_slot(DevScene s, int slot) {
    s.mesh.count_slot = slot;
    return s;
}

std::vector<DevNode> dev_nodes(const pbrt_scene_desc* s) {
    std::vector<DevNode> v((size_t)(s->n_nodes > 0 ? s->n_nodes : 1));
    std::memset(v.data(), 0, v.size() * sizeof(DevNode));
    for (int i = 0; i < s->n_nodes; i++) {
        const pbrt_bvh_node& n = s->nodes[i];
        for (int k = 0; k < 3; k++) {
            v[i].bmin[k] = n.bmin[k];
            v[i].bmax[k] = n.bmax[k];
        }
        v[i].offset = n.offset;
        v[i].nprims_axis = (uint32_t)n.n_prims | ((uint32_t)n.axis << 16);
    }
    return v;
}

// Preorder visit tables of the BVH, one per ray-direction octant (bvh_walk,
// pbrt_path.h). Node i's children: i + 1 and nodes[i].offset; the reference
// visits offset first when the direction along nodes[i].axis is negative
// (bvh.go:693-703). depth = far children pending on the reference's stack.
// Returns false if the node array is not a tree in that depth-first layout.
bool dev_order(const pbrt_scene_desc* s, std::vector<uint32_t>& out) {
    const int n = s->n_nodes;
    out.assign((size_t)16 * (n > 0 ? n : 1), 0u);   // [8][n] preorder, then [8][n] leaves in preorder
    if (n == 0) return true;
    struct Item { uint32_t node, depth; int64_t slot; };   // slot: table index whose skip this item sets (-1: none)
    for (int oct = 0; oct < 8; oct++) {
        uint32_t* t = out.data() + (size_t)oct * n;
        std::vector<Item> st;
        std::vector<int64_t> open;   // table indices of interior nodes whose skip is still unknown
        int k = 0;
        st.push_back({0u, 0u, -1});
        while (!st.empty()) {
            Item it = st.back();
            st.pop_back();
            if (it.slot >= 0) {   // marker: the subtree of table entry `slot` ends here
                t[it.slot] |= (uint32_t)k << 16;
                continue;
            }
            if (k >= n || it.node >= (uint32_t)n) return false;
            const pbrt_bvh_node& nd = s->nodes[it.node];
            const int idx = k++;
            const bool interior = nd.n_prims == 0;
            t[idx] = it.node | ((interior && it.depth >= 64) ? kOrdOverflow : 0u);
            if (!interior) {
                t[idx] |= (uint32_t)(idx + 1) << 16;
                continue;
            }
            const bool neg = (oct >> nd.axis) & 1;
            const uint32_t near_node = neg ? nd.offset : it.node + 1, far_node = neg ? it.node + 1 : nd.offset;
            st.push_back({0u, 0u, (int64_t)idx});            // after both subtrees: set skip
            st.push_back({far_node, it.depth, -1});           // visited after the near subtree
            st.push_back({near_node, it.depth + 1, -1});      // far child pending on the stack
        }
        if (k != n) return false;
        int nl = 0;
        for (int i = 0; i < n; i++) {
            const uint32_t node = t[i] & kOrdNode;
            if (s->nodes[node].n_prims > 0) out[(size_t)8 * n + (size_t)oct * n + nl++] = node;
        }
    }
    return true;
}

// Leaf culling groups of an LDS-staged tree of <= 32 leaves (bvh_walk_analytic): leaves whose
// box diagonal exceeds half the root's (the README floor and wall disks) and
// singletons are tested unconditionally; the others are split recursively at
// the median of their box centres along the widest axis into groups of <= 8
// (the README's three rows of seven spheres become row segments). A group's
// box is the exact union of its members' boxes. Output: boxes [G][6], then per
// octant [G + 1] masks over the octant's leaf preorder positions (last: the
// unconditional leaves). G = 0 (no culling) when the tree is not LDS-staged
// or the grouping needs more than kMaxCullGroups groups.
int cull_groups(const Knobs& kn, const pbrt_scene_desc* s, const std::vector<uint32_t>& order, std::vector<double>& boxes,
                std::vector<uint32_t>& masks) {
    boxes.clear();
    masks.clear();
    const int n = s->n_nodes;
    if (n == 0 || n > kLdsNodes) return 0;
    std::vector<int> leaves;
    for (int i = 0; i < n; i++)
        if (s->nodes[i].n_prims > 0) leaves.push_back(i);
    if (leaves.size() > 32) return 0;
    auto diag2 = [&](int i) {
        double d = 0;
        for (int k = 0; k < 3; k++) d += (s->nodes[i].bmax[k] - s->nodes[i].bmin[k]) * (s->nodes[i].bmax[k] - s->nodes[i].bmin[k]);
        return d;
    };
    const double root = diag2(0);
    std::vector<int> rest;
    std::vector<int> group_of((size_t)n, -1);   // -1: unconditional
    for (int v : leaves)
        if (!(diag2(v) > 0.25 * root)) rest.push_back(v);
    std::vector<std::vector<int>> groups;
    // leaves per group at most: 4 measured best on config B (chain 420 -> 404 ms against 8;
    // 2: 450, 3: 403, 5: 418, 16: 492; profiles/r02/cull_group_ab.json). PBRT_CULL_GROUP overrides.
    const size_t gmax = (size_t)kn.cull_group;
    std::function<void(std::vector<int>)> split = [&](std::vector<int> g) {
        if (g.size() <= gmax) {
            if (g.size() > 1) groups.push_back(g);
            return;
        }
        double lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
        auto cen = [&](int v, int k) { return 0.5 * (s->nodes[v].bmin[k] + s->nodes[v].bmax[k]); };
        for (int v : g)
            for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], cen(v, k)); hi[k] = std::max(hi[k], cen(v, k)); }
        int a = 0;
        for (int k = 1; k < 3; k++)
            if (hi[k] - lo[k] > hi[a] - lo[a]) a = k;
        std::stable_sort(g.begin(), g.end(), [&](int x, int y) { return cen(x, a) < cen(y, a); });
        const size_t h = g.size() / 2;
        split(std::vector<int>(g.begin(), g.begin() + (long)h));
        split(std::vector<int>(g.begin() + (long)h, g.end()));
    };
    if (!rest.empty()) split(rest);
    const int G = (int)groups.size();
    // worth it only when the groups can skip a fair share of the leaf tests
    // (README: 21 of 23 leaves grouped; Cornell: 2 of 8, not grouped)
    const int min_frac2 = kn.cull_min;   // grouped leaves must be at least half of all (PBRT_CULL_MIN=0: any)
    if (G == 0 || G > kMaxCullGroups || min_frac2 * (int)rest.size() < (int)leaves.size()) return 0;
    boxes.assign((size_t)G * 6, 0.0);
    for (int gi = 0; gi < G; gi++) {
        for (int k = 0; k < 3; k++) {
            boxes[(size_t)gi * 6 + k] = kInf;
            boxes[(size_t)gi * 6 + 3 + k] = -kInf;
        }
        for (int v : groups[(size_t)gi]) {
            group_of[(size_t)v] = gi;
            for (int k = 0; k < 3; k++) {
                boxes[(size_t)gi * 6 + k] = std::min(boxes[(size_t)gi * 6 + k], s->nodes[v].bmin[k]);
                boxes[(size_t)gi * 6 + 3 + k] = std::max(boxes[(size_t)gi * 6 + 3 + k], s->nodes[v].bmax[k]);
            }
        }
    }
    masks.assign((size_t)8 * (G + 1), 0u);
    const int nl = (int)leaves.size();
    for (int oct = 0; oct < 8; oct++)
        for (int j = 0; j < nl; j++) {
            const uint32_t node = order[(size_t)8 * n + (size_t)oct * n + (size_t)j];
            const int gi = group_of[node];
            masks[(size_t)oct * (G + 1) + (size_t)(gi < 0 ? G : gi)] |= 1u << j;
        }
    return G;
}

std::vector<DevPrim> dev_prims(const pbrt_scene_desc* s) {
    std::vector<DevPrim> v((size_t)(s->n_prims > 0 ? s->n_prims : 1));
    std::memset(v.data(), 0, v.size() * sizeof(DevPrim));
    for (int i = 0; i < s->n_prims; i++) {
        const pbrt_primitive_desc& p = s->prims[i];
        v[i].shape = s->shapes[p.shape];
        v[i].prim_to_world = p.prim_to_world;
        v[i].kind = p.kind;
        v[i].material = p.material;
        v[i].prim_identity = is_identity(p.prim_to_world.m) ? 1 : 0;
    }
    return v;
}

int validate_scene(const pbrt_scene_desc* s) {
    if (!s) return PBRT_E_INVALID;
    if (s->n_prims < 0 || s->n_nodes < 0 || s->n_lights < 0 || s->n_shapes < 0 || s->n_materials < 0)
        return PBRT_E_INVALID;
    if (s->n_nodes > 32767) return PBRT_E_UNSUPPORTED;   // 15-bit node index in the preorder tables
    for (int i = 0; i < s->n_prims; i++) {
        const pbrt_primitive_desc& p = s->prims[i];
        if (p.shape < 0 || p.shape >= s->n_shapes || p.material < 0 || p.material >= s->n_materials)
            return PBRT_E_INVALID;
        if (p.kind != PBRT_PRIM_GEOMETRIC && p.kind != PBRT_PRIM_TRANSFORMED) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_shapes; i++)
        if (s->shapes[i].type != PBRT_SHAPE_SPHERE && s->shapes[i].type != PBRT_SHAPE_DISK) return PBRT_E_UNSUPPORTED;
    for (int i = 0; i < s->n_nodes; i++) {
        const pbrt_bvh_node& n = s->nodes[i];
        if (n.n_prims > 0 && (int64_t)n.offset + n.n_prims > s->n_prims) return PBRT_E_INVALID;
        if (n.n_prims == 0 && (n.offset >= (uint32_t)s->n_nodes || n.axis > 2)) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_materials; i++)
        if (s->materials[i].type < PBRT_MAT_MATTE || s->materials[i].type > PBRT_MAT_GLASS) return PBRT_E_UNSUPPORTED;
    if (s->n_meshes < 0 || (s->n_meshes > 0 && !s->meshes)) return PBRT_E_INVALID;
    for (int i = 0; i < s->n_meshes; i++) {
        const pbrt_mesh_desc& m = s->meshes[i];
        if (m.n_vertices < 0 || m.n_triangles < 0 || m.material < 0 || m.material >= s->n_materials ||
            (m.n_triangles > 0 && (!m.p || !m.indices)))
            return PBRT_E_INVALID;
        for (int64_t k = 0; k < 3 * (int64_t)m.n_triangles; k++)
            if (m.indices[k] < 0 || m.indices[k] >= m.n_vertices) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_lights; i++) {
        const pbrt_light_desc& l = s->lights[i];
        if (l.type < PBRT_LIGHT_POINT || l.type > PBRT_LIGHT_DIFFUSE_AREA) return PBRT_E_UNSUPPORTED;
        if (l.type == PBRT_LIGHT_DIFFUSE_AREA &&
            (l.shape < 0 || l.shape >= s->n_shapes || s->shapes[l.shape].type != PBRT_SHAPE_SPHERE))
            return PBRT_E_UNSUPPORTED;
    }
    const pbrt_film_desc& f = s->film;
    if (f.crop_max_x <= f.crop_min_x || f.crop_max_y <= f.crop_min_y) return PBRT_E_INVALID;
    return PBRT_OK;
}

const PcgJump& pcg_jump_table() {
    static PcgJump J = [] {
        PcgJump t;
        uint64_t a = 0x5851f42d4c957f2dULL, b = 1;   // one step: s' = a*s + inc*1
        for (int i = 0; i < 64; i++) {
            t.a[i] = a;
            t.b[i] = b;
            b = b * (a + 1);   // two applications of the 2^i jump
            a = a * a;
        }
        return t;
    }();
    return J;
}

int paths_ci_pixels(const pbrt_gpu_ctx* c, const RenderParams& rp);
bool paths_wf_enabled(const pbrt_gpu_ctx* c);
// Can the wave-parallel kernels replay this render exactly? (conditions: pbrt_spec.h)
bool wave_eligible(const pbrt_gpu_ctx* c, const pbrt_render_desc* rd, const RenderParams& rp, ChainLayout& L,
                   ChainLayout& Lci) {
    if (rd->flags & PBRT_FLAG_PANIC_FIDELITY) return false;   // the serial kernel traces the extra rays
    const bool dl = rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING;
    // Mirror, smooth Glass and OrenNayar: Path renders run the kX instantiations
    // of the wave pipeline (trajectories and paths over BSDFX, with etaScale):
    // k_chain_ci for LDS-staged trees, then k_paths_ci (P = 4, 8) or the path
    // wavefront (mesh scenes); DirectLighting's specular recursion, rough glass
    // (whose every BSDF sample panics) and larger trees stay on the serial kernel
    if (c->non_matte && (dl || c->rough_glass || c->host_scene.n_nodes > kLdsNodes ||
                         (!paths_wf_enabled(c) && paths_ci_pixels(c, rp) > 0 && paths_ci_pixels(c, rp) < 4)))
        return false;
    if (dl) {   // k_dl_*: the camera ray must be per pixel (pFilm stratified; pLens stratified or unused)
        if (rd->n_dims < 1 || (rd->n_dims < 2 && c->host_scene.camera.lens_radius > 0)) return false;
    } else if (rd->integrator != PBRT_INTEGRATOR_PATH || rd->n_dims < 3 || rd->max_depth > 2048) {
        return false;   // D < 2^32
    }
    const int nl = c->host_scene.n_lights;
    if (!dl && nl > kMaxCachedLights) return false;
    if (!dl && nl > 0) {
        const pbrt_distribution_desc& d = c->host_dist;
        if (!(d.func_int > 0)) return false;
        for (int i = 0; i < d.count; i++)
            if (!(d.func[i] > 0)) return false;   // a zero-pdf light changes the draw count
    }
    const pbrt_film_desc& f = c->host_scene.film;
    if (!(f.filter_radius_x < 1.5 && f.filter_radius_y < 1.5)) return false;   // <= 2x2 pixel footprint
    const int64_t n = rp.spp, nd = rp.ndims;
    if (n > 4096 || nd * n > 8192) return false;
    int64_t off = 0;
    auto put = [&](int64_t bytes) {
        int64_t o = off;
        off += (bytes + 15) & ~int64_t(15);
        return (int)o;
    };
    L.s1d = put(nd * n * 8);
    L.other = put(nd * n * 2);
    L.sbuf = put(kWave * 8);
    L.dbuf = put(kWave * 4);
    L.vbuf = put(rp.sp_serial ? 4 : (int64_t)rp.sp_draws * 4);
    L.total = (int)off;
    L.ring = 0;
    // k_chain_ci: the same staging without the window buffers, then the ring
    off = 0;
    // the pixel's stratified values are staged in LDS while the staging of one
    // 1-wave tile (aliased with the ring) stays <= 20 KB (5+ workgroups per CU;
    // config C's 256 spp needs 19.3 KB); above, StartPixel writes them straight
    // to the pixel's global record (always with the serial StartPixel, large spp)
    const int64_t al16 = 15;
    const int64_t lds_staging = ((nd * n * 8 + al16) & ~al16) + ((nd * n * 2 + al16) & ~al16) +
                                (((rp.sp_serial ? 4 : (int64_t)rp.sp_draws * 4) + al16) & ~al16);
    if (rp.sp_serial) {
        Lci.s1d = -1;
        Lci.other = put(16);
    } else if (lds_staging > 20 * 1024) {
        Lci.s1d = -1;
        Lci.other = put(nd * n * 2);
    } else {
        Lci.s1d = put(nd * n * 8);
        Lci.other = put(nd * n * 2);
    }
    Lci.sbuf = Lci.dbuf = 0;
    Lci.vbuf = put(rp.sp_serial ? 4 : (int64_t)rp.sp_draws * 4);
    Lci.staging = (int)off;
    Lci.ring = put(kCiRingBytes);
    Lci.total = (int)off;
    return L.total <= 48 * 1024;
}

// k_chain_ci's LDS layout for w waves per tile and G tiles per wave. With one
// tile per workgroup (G == 1) the StartPixel staging aliases the offset ring:
// a group starts a pixel only after its chain has dropped every candidate,
// so the two are never live together (config C, 256 spp: 19 KB of staging).
ChainLayout ci_layout(const ChainLayout& base, int w, int G, unsigned& lds_bytes) {
    ChainLayout l = base;
    if (G == 1) {
        l.ring = 0;
        lds_bytes = (unsigned)std::max(base.staging, w * kCiRingBytes);
    } else {
        lds_bytes = (unsigned)(base.total + (w - 1) * kCiRingBytes);
    }
    // then one ChainCache per lane group (only the groups in use: G, not kCiMaxGroups)
    l.pcs = (int)((lds_bytes + 15u) & ~15u);
    lds_bytes = (unsigned)l.pcs + (unsigned)(G * sizeof(ChainCache));
    l.total = (int)lds_bytes;
    return l;
}

// Waves per tile of k_chain_ci for a launch of nb tiles. The frame's EXACT
// time is bounded below by its slowest tile's chain, so when the tiles of a
// launch cannot keep every wave slot busy (2 waves/SIMD) a tile gets 2 or 4
// waves. PBRT_CI_WAVES (1, 2, 4) overrides.
int ci_waves(const pbrt_gpu_ctx* c, int64_t nb) {
    if (c->knobs.ci_waves) return c->non_matte ? std::min(c->knobs.ci_waves, 4) : c->knobs.ci_waves;
    if (c->tiles_per_wave > 1) return 1;
    // measured on config B shards (tools/shard_sim.py): 8160 tiles -> 1,
    // 4080 -> 2, 2040 and 1020 -> 4
    const int64_t slots = (int64_t)c->n_simd * 2;   // 2 waves/SIMD
    if (nb <= slots) return 4;
    if (nb <= 2 * slots) return 2;
    return 1;
}

// k_chain_ci schedule. An EXACT frame lasts at least as long as its slowest
// tile's chain, and workgroups start in launch order, so a heavy tile that
// starts late stretches the frame. Each EXACT frame records every tile's
// chain time; the next frame of the same configuration on this context
// launches its tiles heaviest first (LPT). Only the schedule changes, never
// a result. PBRT_CI_ORDER=0 disables it.
// Multi-GPU shards (launches that would run 2 or 4 waves per tile): the
// heaviest tiles of the previous frame get 4 waves in a launch of their own
// and the rest 1 wave each in a concurrent one (1/4- and 1/2-frame shards:
// 387 -> 305 ms and 524 -> 472 ms per rank). PBRT_CI_SPLIT=0 disables it;
// PBRT_CI_HEAVY=K forces the heavy count (tests).
bool ci_split_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_split; }
int64_t ci_heavy_override(const pbrt_gpu_ctx* c) { return c->knobs.ci_heavy; }
// k_chain_ci candidate stride: 2 issues candidates at the chain head's parity
// only (dropped when an odd draw count flips it), 1 at every offset (twice
// the candidates, none dropped). PBRT_CI_STRIDE = 1 / 2 overrides.
int ci_stride(const pbrt_gpu_ctx* c, int w) {
    if (c->knobs.ci_stride) return c->knobs.ci_stride;
    return w > 1 ? 1 : 2;
}
// PBRT_CI_HEAVY_WAVES = 4 (default) or 8: waves per heavy tile of the split
int ci_heavy_waves(const pbrt_gpu_ctx* c) { return c->non_matte ? 4 : c->knobs.ci_heavy_waves; }
bool ci_order_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_order; }
// PBRT_CI_PROBE=0: a fresh context's first frame runs in launch order (no k_tile_cost)
bool ci_probe_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_probe; }
uint64_t schedule_key(const RenderParams& rp, int kw) {
    const int64_t v[] = {rp.film_min_x, rp.film_min_y, rp.film_w,   rp.film_h,    rp.tile_size, rp.tile_begin,
                         rp.tile_stride, rp.n_slots,   rp.spp,      rp.ndims,     rp.jitter,    rp.max_depth,
                         rp.flags,       kw,           (int64_t)(rp.rr_threshold * 1e9)};
    uint64_t h = 1469598103934665603ull;
    for (int64_t x : v) h = (h ^ (uint64_t)x) * 1099511628211ull;
    return h;
}

// k_paths_ci (lane refill over kPathsPixels pixels per wave) where it fits:
// LDS-staged nodes, the pixels' stratified values in 16 KB of LDS and one
// lane per (pixel, light) for the bounce-1 estimates; 0: the path wavefront
// (k_pw_*) runs the paths. PBRT_PATHS_CI=0 forces that.
// Returns the pixels per wave (2, 4 or 8; PBRT_PATHS_CI overrides, 0 = off).
// k_paths_ci stages the stratified values of its P pixels in LDS when they take <= 16 KB
// Off by default: read from their global records (L2-resident; config B
// 111.0 -> 109.9 ms EXACT, 136.0 -> 134.8 ms THROUGHPUT against LDS staging).
// PBRT_PATHS_S1D=lds stages them where they fit (experiments).
bool paths_ci_s1d_lds(const pbrt_gpu_ctx* c, const RenderParams& rp, int P) {
    return c->knobs.paths_s1d_lds && (int64_t)P * rp.ndims * rp.spp * 8 <= 16 * 1024;
}
int paths_ci_pixels(const pbrt_gpu_ctx* c, const RenderParams& rp) {
    int pp = 4;
    bool forced = false;
    if (c->knobs.paths_ci == 0) return 0;
    if (c->knobs.paths_ci > 0) pp = c->knobs.paths_ci, forced = true;
    auto fits = [&](int p) {
        return c->host_scene.n_nodes <= kLdsNodes && p * c->host_scene.n_lights <= kWave;
    };
    if (forced) return fits(pp) ? pp : 0;
    // 8 pixels per wave where their lights fit one wave, else 4; stratified
    // values read from global memory (config B EXACT paths 109.9 -> 104.8 ms
    // for 8 against 4; config C at 256 spp 872 -> 869 ms, where 4 pixels with
    // global values already beat 2 with LDS values, 1150 ms)
    return fits(8) ? 8 : fits(4) ? 4 : 0;
}

// The full-path stage on the path wavefront (k_pw_*) instead of k_paths_ci:
// PBRT_PATHS_WF=1 / 0 forces it on / off; by default it runs for scenes with
// triangle meshes, where it measured faster (config D: 385 -> 343 ms EXACT,
// 420 -> 381 ms THROUGHPUT), and not for the analytic scenes, where the
// monolithic lane-refill kernel is twice as fast (config B: 118 vs 212-245 ms;
// profiles/r02/path_wavefront_ab.json). PBRT_PW_SORT=1 adds the material sort
// between trace and shade: a loss on every scene measured (B 212 -> 245 ms: a
// few matte materials leave no shading divergence to remove), so off by default.
bool paths_wf_enabled(const pbrt_gpu_ctx* c) {
    if (c->knobs.paths_wf >= 0) return c->knobs.paths_wf == 1;
    return c->mesh.n_nodes > 0;
}
int paths_wavefront(pbrt_gpu_ctx* c, const DevScene& sc, int64_t sb, int64_t nb) {
    const RenderParams& rp = c->rp;
    const int64_t nrec = nb * c->wb.ppt, per = rp.spp - 1;
    const int nl = sc.n_lights;
    const int sort = c->knobs.pw_sort ? 1 : 0;
    const int n_keys = std::max(1, std::min(c->host_scene.n_materials, kPwMaxKeys));
    const double gb = c->knobs.pw_gb;
    const int64_t per_path = (int64_t)sizeof(PwPath) + 4 * 4;   // record + 4 queue slots
    int64_t chunk = per > 0 ? std::max<int64_t>(1, (int64_t)(gb * 1073741824.0) / (per_path * per)) : nrec;
    chunk = std::min(chunk, nrec);
    if (per > 0) chunk = std::min<int64_t>(chunk, (int64_t)0xFFFFFFF0 / per);
    const int64_t cap = std::max<int64_t>(1, chunk * std::max<int64_t>(per, 1));
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    const int64_t ncnt = 3 + 2 * kPwMaxKeys;
    const size_t need = (size_t)(al(cap * (int64_t)sizeof(PwPath)) + 4 * al(cap * 4) + al(ncnt * 4) +
                                 al(chunk * std::max(nl, 1) * (int64_t)sizeof(Spec)) + al(chunk * std::max(nl, 1) * 4) +
                                 al(nrec * 8));
    if (c->pw_cap < need || !c->d_pw) {
        if (c->d_pw) (void)hipFree(c->d_pw);
        c->d_pw = nullptr;
        c->pw_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_pw, need));
        c->pw_cap = need;
    }
    unsigned char* p = c->d_pw;
    auto take = [&](int64_t bytes) {
        unsigned char* q = p;
        p += al(bytes);
        return q;
    };
    PwPath* paths = (PwPath*)take(cap * (int64_t)sizeof(PwPath));
    PwQueues qs;
    for (int i = 0; i < 3; i++) qs.q[i] = (uint32_t*)take(cap * 4);
    qs.sorted = (uint32_t*)take(cap * 4);
    qs.cnt = (uint32_t*)take(ncnt * 4);
    qs.cap = cap;
    Spec* ldc = (Spec*)take(chunk * std::max(nl, 1) * (int64_t)sizeof(Spec));
    int* ldp = (int*)take(chunk * std::max(nl, 1) * 4);
    unsigned long long* pkey = (unsigned long long*)take(nrec * 8);
    const unsigned G = (unsigned)std::max<int64_t>(64, (int64_t)c->n_simd * 8);   // grid-stride blocks
    HIPCHK(c, hipMemsetAsync(pkey, 0xFF, (size_t)nrec * 8, c->stream));
    const bool mb = rp.mode == PBRT_MODE_THROUGHPUT;
    const bool kx = c->non_matte;   // Mirror / smooth Glass / OrenNayar: the kX instantiations
    for (int64_t r0 = 0; r0 < nrec; r0 += chunk) {
        const int64_t nr = std::min(chunk, nrec - r0);
        if (per > 0) {
            HIPCHK(c, hipMemsetAsync(qs.cnt, 0, (size_t)ncnt * 4, c->stream));
            if (nl > 0)
                hipLaunchKernelGGL(kx ? k_pw_cache<true> : k_pw_cache<false>,
                                   dim3((unsigned)((nr * nl + kWave - 1) / kWave)), dim3(kWave), 0,
                                   c->stream, sc, c->wb, r0, nr, ldc, ldp);
            auto start = kx ? (mb ? k_pw_start<true, true> : k_pw_start<false, true>)
                            : (mb ? k_pw_start<true> : k_pw_start<false>);
            hipLaunchKernelGGL(start, dim3((unsigned)((nr * per + kWave - 1) / kWave)), dim3(kWave), 0, c->stream,
                               sc, rp, c->wb, sb, r0, nr, ldc, ldp, paths, qs, pkey);
            for (int pass = 0; pass + 1 < rp.max_depth; pass++) {
                hipLaunchKernelGGL(k_pw_trace, dim3(G), dim3(kWave), 0, c->stream, sc, rp, c->wb, paths, qs, 0,
                                   n_keys, pkey);
                if (sort && n_keys > 1) {
                    hipLaunchKernelGGL(k_pw_scan, dim3(1), dim3(1), 0, c->stream, qs, n_keys);
                    hipLaunchKernelGGL(k_pw_scatter, dim3(G / 4), dim3(256), 0, c->stream, paths, qs);
                }
                hipLaunchKernelGGL(kx ? k_pw_shade<true> : k_pw_shade<false>, dim3(G), dim3(kWave), 0, c->stream, sc,
                                   rp, c->wb, sb, paths, qs,
                                   sort && n_keys > 1 ? 1 : 0, pkey);
                hipLaunchKernelGGL(k_pw_shadow, dim3(G), dim3(kWave), 0, c->stream, sc, rp, c->wb, paths, qs, pkey);
            }
        }
        hipLaunchKernelGGL(k_pw_panics, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, c->stream, rp, c->wb, sb, r0,
                           nr, pkey, c->d_ctr);
    }
    HIPCHK(c, hipGetLastError());
    return PBRT_OK;
}

// Carve the per-batch buffers of the wave path. Budget: PBRT_WAVE_BUFFER_GB,
// default min(96 GB, half the free HBM) -- config C (1080p, 256 spp, ~34 GB)
// and one rank's 1/8 shard of config E (4K, 1024 spp, ~68 GB) are then one
// batch on a 288 GB MI355X, so the whole frame is one launch per kernel and
// gets the heaviest-first schedule.
int wave_buffers(pbrt_gpu_ctx* c) {
    const RenderParams& rp = c->rp;
    const int64_t ppt = rp.tile_size * rp.tile_size, n = rp.spp, nd = rp.ndims > 0 ? rp.ndims : 1;
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    const int64_t per_tile = al(ppt * (int64_t)sizeof(PixelRec)) + al(ppt * nd * n * 8) + al(ppt * n * 8) +
                             al(ppt * n * 24) + al(ppt * n * 4) + al(ppt * (int64_t)sizeof(PanicRec)) + al(4);
    double gb = 96.0;
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
            gb = std::min(gb, 0.5 * (double)(free_b + c->wave_cap) / 1073741824.0);
    }
    if (c->knobs.wave_buffer_gb > 0) gb = c->knobs.wave_buffer_gb;
    int64_t batch = (int64_t)(gb * 1073741824.0) / per_tile;
    if (batch < 1) batch = 1;
    if (batch > rp.n_slots) batch = rp.n_slots > 0 ? rp.n_slots : 1;
    const size_t need = (size_t)(batch * per_tile);
    if (c->wave_cap < need || !c->d_wave) {
        if (c->d_wave) (void)hipFree(c->d_wave);
        c->d_wave = nullptr;
        c->wave_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_wave, need));
        c->wave_cap = need;
    }
    WaveBufs& wb = c->wb;
    unsigned char* p = c->d_wave;
    auto take = [&](int64_t bytes_per_tile) {
        unsigned char* q = p;
        p += batch * al(bytes_per_tile);
        return q;
    };
    wb.prec = (PixelRec*)take(ppt * (int64_t)sizeof(PixelRec));
    wb.s1d = (double*)take(ppt * nd * n * 8);
    wb.memb = (uint64_t*)take(ppt * n * 8);
    wb.L = (double*)take(ppt * n * 24);
    wb.rays = (uint32_t*)take(ppt * n * 4);
    wb.ppanic = (PanicRec*)take(ppt * (int64_t)sizeof(PanicRec));
    wb.tile_npx = (int32_t*)take(4);
    wb.ppt = ppt;
    wb.s1d_stride = nd * n;
    c->wave_batch = batch;
    return PBRT_OK;
}

int prepare(pbrt_gpu_ctx* c, const pbrt_render_desc* rd) {
    if (!rd) return set_err(c, PBRT_E_INVALID, "null render desc");
    if (rd->tile_size <= 0 || rd->sampler_x <= 0 || rd->sampler_y <= 0 || rd->n_dims < 0 || rd->n_dims > 64)
        return set_err(c, PBRT_E_INVALID, "bad sampler / tile size");
    if ((int64_t)rd->sampler_x * rd->sampler_y > (1 << 20)) return set_err(c, PBRT_E_INVALID, "spp too large");
    if (rd->integrator != PBRT_INTEGRATOR_PATH && rd->integrator != PBRT_INTEGRATOR_DIRECT_LIGHTING)
        return set_err(c, PBRT_E_UNSUPPORTED, "unknown integrator");
    if (rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING && rd->dl_strategy != PBRT_DL_UNIFORM_SAMPLE_ALL &&
        rd->dl_strategy != PBRT_DL_UNIFORM_SAMPLE_ONE)
        return set_err(c, PBRT_E_UNSUPPORTED, "unknown DirectLighting strategy");
    if (rd->mode != PBRT_MODE_EXACT && rd->mode != PBRT_MODE_THROUGHPUT)
        return set_err(c, PBRT_E_INVALID, "unknown mode");
    const pbrt_film_desc& f = c->host_scene.film;
    if (f.filter_radius_x <= 0 || f.filter_radius_y <= 0 || f.filter_radius_x >= (double)rd->tile_size ||
        f.filter_radius_y >= (double)rd->tile_size)
        return set_err(c, PBRT_E_UNSUPPORTED, "filter radius must be in (0, tile_size)");
    if ((rd->flags & PBRT_FLAG_PANIC_FIDELITY) && c->non_matte)
        return set_err(c, PBRT_E_UNSUPPORTED, "panic fidelity covers Matte scenes only");
    if (rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING && c->non_matte && rd->max_depth > 2 * kDlMaxLevels)
        return set_err(c, PBRT_E_UNSUPPORTED, "DirectLighting through glass: maxDepth must be <= 64");
    RenderParams& rp = c->rp;
    std::memset(&rp, 0, sizeof(rp));
    rp.film_min_x = f.crop_min_x;
    rp.film_min_y = f.crop_min_y;
    rp.film_w = f.crop_max_x - f.crop_min_x;
    rp.film_h = f.crop_max_y - f.crop_min_y;
    rp.tile_size = rd->tile_size;
    rp.ntx = (rp.film_w + rd->tile_size - 1) / rd->tile_size;
    rp.nty = (rp.film_h + rd->tile_size - 1) / rd->tile_size;
    int64_t total = rp.ntx * rp.nty;
    int64_t begin = rd->tile_begin < 0 ? 0 : rd->tile_begin;
    int64_t end = rd->tile_end > 0 && rd->tile_end < total ? rd->tile_end : total;
    int64_t stride = rd->tile_stride > 0 ? rd->tile_stride : 1;
    rp.tile_begin = begin;
    rp.tile_stride = stride;
    rp.n_slots = begin < end ? (end - begin + stride - 1) / stride : 0;
    rp.slot_w = rd->tile_size + 2 * ((int64_t)f.filter_radius_x + 1);
    rp.slot_h = rd->tile_size + 2 * ((int64_t)f.filter_radius_y + 1);
    rp.xs = rd->sampler_x;
    rp.ys = rd->sampler_y;
    rp.spp = rd->sampler_x * rd->sampler_y;
    rp.ndims = rd->n_dims;
    rp.jitter = rd->jitter ? 1 : 0;
    rp.integrator = rd->integrator;
    rp.max_depth = rd->max_depth;
    rp.dl_strategy = rd->dl_strategy;
    rp.rr_threshold = rd->rr_threshold;
    rp.lanes_per_wave = c->lanes_per_wave;
    rp.flags = rd->flags;
    rp.mode = rd->mode;
    pbrt_distribution_desc& dist = c->host_dist;
    std::memset(&dist, 0, sizeof(dist));
    if (rd->integrator == PBRT_INTEGRATOR_PATH) {
        int rc = pbrt_scene_light_distribution(&c->host_scene, rd->light_strategy, &dist);
        if (rc != PBRT_OK) return set_err(c, rc, "unsupported light sample strategy");
        HIPCHK(c, hipMemcpyAsync(c->d_dist, &dist, sizeof(dist), hipMemcpyHostToDevice, c->stream));
    }
    {
        const int64_t n = rp.spp, s1 = rp.jitter ? 2 * n : n, s2 = rp.jitter ? 3 * n : n;
        const int64_t E = (int64_t)rp.ndims * (s1 + s2), V = E + 64 + E / 8;
        rp.sp_events = (int32_t)E;
        rp.sp_draws = (int32_t)V;
        rp.sp_serial = V * 4 <= 16 * 1024 ? 0 : 1;
    }
    c->use_spec = c->kernel_req != PBRT_KERNEL_SERIAL && wave_eligible(c, rd, rp, c->lay, c->lay_ci);
    if ((c->kernel_req == PBRT_KERNEL_WAVE || c->kernel_req == PBRT_KERNEL_WAVEFRONT ||
         c->kernel_req == PBRT_KERNEL_WAVE_CI) && !c->use_spec)
        return set_err(c, PBRT_E_UNSUPPORTED, "render not eligible for the wave-parallel kernels");
    c->use_dl = c->use_spec && rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING;
    if (c->use_dl && c->kernel_req != PBRT_KERNEL_AUTO && c->kernel_req != PBRT_KERNEL_WAVE_DL)
        return set_err(c, PBRT_E_UNSUPPORTED, "DirectLighting runs on the serial or the k_dl_* kernels");
    if (!c->use_dl && c->kernel_req == PBRT_KERNEL_WAVE_DL)
        return set_err(c, PBRT_E_UNSUPPORTED, "render not eligible for the DirectLighting wave kernels");
    // the chain stage of the wave pipeline is k_chain_ci (PBRT_KERNEL_WAVE and
    // _WAVEFRONT, whose window and wavefront chains it replaced, select it too)
    c->use_ci = c->use_spec && !c->use_dl;
    if (c->use_spec && rp.n_slots > 0) {
        int rcw = wave_buffers(c);
        if (rcw != PBRT_OK) return rcw;
        // tiles per k_chain_ci wave (opts.lanes_per_wave = 1, 2 or 4; default 1).
        // One tile per wave is fastest on MI355X: its 64 trajectories leave the
        // same bounce-1 point, so their traversals stay coherent; packing tiles
        // cuts speculation but a window lasts as long as its slowest lane, and
        // mixed-tile windows measured 2.5x slower per window.
        int G = 1;
        if (c->lanes_per_wave_set && c->lanes_per_wave >= 1 && c->lanes_per_wave <= kCiMaxGroups &&
            (c->lanes_per_wave & (c->lanes_per_wave - 1)) == 0)
            G = c->lanes_per_wave;
        c->tiles_per_wave = G;
    }
    size_t nslot = (size_t)(rp.n_slots > 0 ? rp.n_slots : 1);
    int rc;
    if ((rc = ensure(c, &c->d_films, &c->films_cap, nslot * (size_t)(rp.slot_w * rp.slot_h * 3)))) return rc;
    if ((rc = ensure(c, &c->d_s1d, &c->s1d_cap, nslot * (size_t)(rp.ndims > 0 ? rp.ndims : 1) * (size_t)rp.spp)))
        return rc;
    if ((rc = ensure(c, &c->d_panics, &c->panics_cap, nslot))) return rc;
    if ((rc = ensure(c, &c->d_out, &c->out_cap, (size_t)(rp.film_w * rp.film_h * 3)))) return rc;
    return PBRT_OK;
}

}  // namespace

extern "C" {

int pbrt_gpu_create(const pbrt_scene_desc* scene, const pbrt_gpu_opts* opts, pbrt_gpu_ctx** out) {
    if (!out) return PBRT_E_INVALID;
    *out = nullptr;
    int rc = validate_scene(scene);
    if (rc != PBRT_OK) return rc;
    auto* c = new pbrt_gpu_ctx();
    c->knobs = Knobs::from_env();
    c->device = (opts && opts->device >= 0) ? opts->device : -1;
    if (opts && opts->lanes_per_wave > 0 && opts->lanes_per_wave <= 64) {
        c->lanes_per_wave = opts->lanes_per_wave;
        c->lanes_per_wave_set = true;
    }
    if (opts && (opts->occupancy == 2 || opts->occupancy == 4 || opts->occupancy == 8)) c->min_waves = opts->occupancy;
    if (opts) c->occ_req = opts->occupancy;
    if (opts && (opts->kernel < PBRT_KERNEL_AUTO || opts->kernel > PBRT_KERNEL_WAVE_DL)) {
        delete c;
        return PBRT_E_INVALID;
    }
    if (opts) c->kernel_req = opts->kernel;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        delete c;
        return PBRT_E_HIP;
    }
    if (c->device >= 0) {
        if (hipSetDevice(c->device) != hipSuccess) { delete c; return PBRT_E_HIP; }
    } else {
        (void)hipGetDevice(&c->device);
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0) {
            c->n_simd = 4 * prop.multiProcessorCount;
            c->lds_per_block = prop.sharedMemPerBlock;
        }
    }
    std::vector<uint32_t> order;
    if (!dev_order(scene, order)) {
        delete c;
        return PBRT_E_INVALID;
    }
    c->host_scene = *scene;
    c->non_matte = false;
    for (int i = 0; i < scene->n_materials; i++)   // Mirror, Glass or OrenNayar (Matte with sigma != 0)
        c->non_matte |= scene->materials[i].type != PBRT_MAT_MATTE ||
                        !(std::min(std::max(scene->materials[i].sigma, 0.0), 90.0) == 0);
    c->rough_glass = false;
    for (int i = 0; i < scene->n_materials; i++)
        c->rough_glass |= scene->materials[i].type == PBRT_MAT_GLASS &&
                          !(scene->materials[i].u_roughness == 0 && scene->materials[i].v_roughness == 0);
    c->h_node_prims.resize((size_t)scene->n_nodes);
    for (int i = 0; i < scene->n_nodes; i++) c->h_node_prims[i] = scene->nodes[i].n_prims;
    c->host_scene.shapes = nullptr;
    c->host_scene.materials = nullptr;
    c->host_scene.prims = nullptr;
    c->host_scene.nodes = nullptr;
    c->host_lights.assign(scene->lights, scene->lights + scene->n_lights);
    c->host_scene.lights = c->host_lights.data();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_split, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        pbrt_gpu_destroy(c);
        return PBRT_E_HIP;
    }
    if (hipHostMalloc((void**)&c->h_cancel, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->d_cancel, c->h_cancel, 0) != hipSuccess) {
        pbrt_gpu_destroy(c);
        return PBRT_E_HIP;
    }
    __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    if ((rc = upload(c, &c->d_shapes, scene->shapes, scene->n_shapes)) ||
        (rc = upload(c, &c->d_materials, scene->materials, scene->n_materials)) ||
        (rc = upload(c, &c->d_prims, scene->prims, scene->n_prims)) ||
        (rc = upload(c, &c->d_nodes, dev_nodes(scene).data(), scene->n_nodes)) ||
        (rc = upload(c, &c->d_order, order.data(), order.size())) ||
        (rc = upload(c, &c->d_fprims, dev_prims(scene).data(), scene->n_prims)) ||
        (rc = upload(c, &c->d_lights, scene->lights, scene->n_lights)) ||
        (rc = upload(c, &c->d_camera, &scene->camera, 1)) || (rc = upload(c, &c->d_film, &scene->film, 1)) ||
        (rc = upload<pbrt_distribution_desc>(c, &c->d_dist, nullptr, 1)) ||
        (rc = upload<Counters>(c, &c->d_ctr, nullptr, 1)) || (rc = upload<int>(c, &c->d_cancel_seen, nullptr, 1)) ||
        (rc = upload<PcgJump>(c, &c->d_jump, &pcg_jump_table(), 1))) {
        pbrt_gpu_destroy(c);
        return rc;
    }
    {   // leaf culling groups of the LDS-staged walk
        std::vector<double> gb;
        std::vector<uint32_t> gm;
        c->n_groups = cull_groups(c->knobs, scene, order, gb, gm);
        if (!c->knobs.cull_groups) c->n_groups = 0;   // PBRT_CULL_GROUPS=0: test every leaf (A/B)
        if (c->n_groups > 0 && ((rc = upload(c, &c->d_groups, gb.data(), gb.size())) ||
                                (rc = upload(c, &c->d_gmasks, gm.data(), gm.size())))) {
            pbrt_gpu_destroy(c);
            return rc;
        }
    }
    if (scene->n_meshes > 0) {   // triangle meshes: LBVH built on the device (mesh_bvh.hip)
        std::string err;
        rc = mesh_bvh_build(scene, c->stream, c->mesh, err);
        if (rc != PBRT_OK) {
            pbrt_gpu_destroy(c);
            return rc;
        }
    }
    c->host_scene.meshes = nullptr;
    *out = c;
    return PBRT_OK;
}

int pbrt_gpu_render_async_into(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_device) {
    if (!c) return PBRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    c->t_start = std::chrono::steady_clock::now();
    int rc = prepare(c, rd);
    if (rc != PBRT_OK) return rc;
    {   // this render is the one pbrt_gpu_cancel now cancels
        std::lock_guard<std::mutex> lk(c->cancel_mu);
        c->in_flight = true;
        c->cancel_req = false;
        __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    const RenderParams& rp = c->rp;
    double* out = film_device ? film_device : c->d_out;
    c->film_target = out;
    c->last_heavy = 0;
    HIPCHK(c, hipMemsetAsync(c->d_ctr, 0, sizeof(Counters), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_cancel_seen, 0, sizeof(int), c->stream));
    if (rp.n_slots > 0) HIPCHK(c, hipMemsetAsync(c->d_panics, 0, sizeof(PanicRec) * (size_t)rp.n_slots, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if (rp.n_slots > 0) {
        DevScene sc = dev_scene(c, rd->integrator == PBRT_INTEGRATOR_PATH);
        if (c->use_spec) {
            c->last_kernel = c->use_dl ? PBRT_KERNEL_WAVE_DL
                             : rp.mode == PBRT_MODE_THROUGHPUT ? PBRT_KERNEL_WAVE : PBRT_KERNEL_WAVE_CI;
            const bool lds_nodes = c->host_scene.n_nodes <= kLdsNodes;
            const bool kx = c->non_matte;   // Mirror / smooth Glass / OrenNayar: the kX instantiations
            const int64_t per = rp.slot_w * rp.slot_h;
            c->n_batches = (int)((rp.n_slots + c->wave_batch - 1) / c->wave_batch);
            while ((int)c->bev.size() < 3 * c->n_batches) {
                hipEvent_t e;
                HIPCHK(c, hipEventCreate(&e));
                c->bev.push_back(e);
            }
            for (int64_t sb = 0, bi = 0; sb < rp.n_slots; sb += c->wave_batch, bi++) {
                const int64_t nb = std::min<int64_t>(c->wave_batch, rp.n_slots - sb);
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 0], c->stream));
                const int G = c->tiles_per_wave;
                if (c->use_dl) {
                    hipLaunchKernelGGL(k_wf_primary<false>, dim3((unsigned)((nb * c->wb.ppt + kWave - 1) / kWave)),
                                       dim3(kWave), 0, c->stream, with_slot(sc, 1), rp, c->wb, sb, nb);
                    unsigned lds = 0;
                    const ChainLayout lw = ci_layout(c->lay_ci, 1, 1, lds);
                    hipLaunchKernelGGL(k_dl_setup, dim3((unsigned)nb), dim3(kWave), lds, c->stream, sc, rp, lw,
                                       c->d_jump, c->wb, sb, nb);
                } else if (rp.mode == PBRT_MODE_THROUGHPUT) {
                    // no offset chain: every sample's stream is known up front
                } else {
                    hipLaunchKernelGGL(kx ? k_wf_primary<true> : k_wf_primary<false>,
                                       dim3((unsigned)((nb * c->wb.ppt + kWave - 1) / kWave)),
                                       dim3(kWave), 0, c->stream, with_slot(sc, 1), rp, c->wb, sb, nb);
                    const int kw = ci_waves(c, nb);
                    const uint32_t* order = nullptr;
                    bool learned = false;   // order from the last frame's measured chain times
                    uint32_t* ticks = nullptr;
                    if ((kw > 1 || G == 1) && c->n_batches == 1 && ci_order_enabled(c)) {
                        if (c->ticks_cap < nb) {
                            if (c->d_ticks) (void)hipFree(c->d_ticks);
                            if (c->d_slot_order) (void)hipFree(c->d_slot_order);
                            c->d_ticks = c->d_slot_order = nullptr;
                            c->ticks_cap = 0;
                            HIPCHK(c, hipMalloc((void**)&c->d_ticks, sizeof(uint32_t) * (size_t)nb));
                            HIPCHK(c, hipMalloc((void**)&c->d_slot_order, sizeof(uint32_t) * (size_t)nb));
                            c->ticks_cap = nb;
                        }
                        const uint64_t key = schedule_key(rp, kw);
                        if (c->order_key == key && (int64_t)c->h_slot_order.size() == nb) {
                            HIPCHK(c, hipMemcpyAsync(c->d_slot_order, c->h_slot_order.data(), sizeof(uint32_t) * (size_t)nb,
                                                     hipMemcpyHostToDevice, c->stream));
                            order = c->d_slot_order;
                            learned = true;
                        }
                        c->probed = false;
                        if (!order && ci_probe_enabled(c) && nb <= (int64_t)1 << 24) {
                            // no measured order for this configuration yet: estimate it
                            int64_t npad = 2048;
                            while (npad < nb) npad <<= 1;
                            if (c->cost_cap < npad) {
                                if (c->d_cost) (void)hipFree(c->d_cost);
                                if (c->d_cost_keys) (void)hipFree(c->d_cost_keys);
                                c->d_cost = nullptr;
                                c->d_cost_keys = nullptr;
                                c->cost_cap = 0;
                                HIPCHK(c, hipMalloc((void**)&c->d_cost, sizeof(float) * 4 * (size_t)npad));
                                HIPCHK(c, hipMalloc((void**)&c->d_cost_keys, sizeof(uint64_t) * (size_t)npad));
                                c->cost_cap = npad;
                            }
                            HIPCHK(c, hipMemsetAsync(c->d_cost_keys, 0xFF, sizeof(uint64_t) * (size_t)npad, c->stream));
                            hipLaunchKernelGGL(kx ? k_tile_cost<true> : k_tile_cost<false>, dim3((unsigned)nb),
                                               dim3(kWave), 0, c->stream, with_slot(sc, 0),
                                               rp, c->wb, sb, nb, c->d_cost, c->d_cost_keys);
                            bitonic_sort_u64(c->d_cost_keys, (uint32_t)npad, c->stream);
                            hipLaunchKernelGGL(k_order_of_keys, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
                                               c->stream, c->d_cost_keys, nb, c->d_slot_order);
                            order = c->d_slot_order;
                            c->probed = true;
                            c->cost_n = nb;
                        }
                        ticks = c->d_ticks;
                        c->ticks_pending = true;
                        c->ticks_key = key;
                        c->ticks_n = nb;
                    }
                    // one launch of n workgroups, workgroup b on slot ord[b] (identity if null)
                    // excl: pad the dynamic LDS so that no other chain workgroup fits
                    // beside one of these on a CU (a heavy tile's waves issue alone)
                    auto launch_ci = [&](int w, int64_t n, const uint32_t* ord, hipStream_t st, bool excl = false) {
                        if (w > 1) {   // one tile per workgroup of w waves; the ring grows with the lanes
                            const int ring = w * kCiRingBytes / (int)sizeof(RingEnt);
                            unsigned lds = 0;
                            const ChainLayout lw = ci_layout(c->lay_ci, w, 1, lds);
                            if (excl) {
                                // half the CU's LDS (160 KB on gfx950) plus a bit, within the per-workgroup limit
                                const size_t want = 84 * 1024;
                                if (c->lds_per_block >= want + 16 * 1024) lds = std::max<unsigned>(lds, (unsigned)want);
                            }
                            // kX: LDS-staged trees only, at most 4 waves per tile (wave_eligible, ci_waves)
                            auto kern = kx ? (w == 2 ? k_chain_ci<2, 0, true> : k_chain_ci<4, 0, true>)
                                           : (w == 2   ? (lds_nodes ? k_chain_ci<2> : k_chain_ci<2, 64>)
                                              : w == 4 ? (lds_nodes ? k_chain_ci<4> : k_chain_ci<4, 64>)
                                                       : (lds_nodes ? k_chain_ci<8> : k_chain_ci<8, 64>));
                            hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(kWave * w), lds, st, with_slot(sc, 2), rp, lw,
                                               c->d_jump, c->wb, sb, nb, kWave * w, ring, c->d_ctr, ord, ticks,
                                               ci_stride(c, w));
                        } else {
                            const int Gc = std::min(G, kCiMaxGroups);
                            const int ring = kCiRingBytes / (int)sizeof(RingEnt) / Gc;
                            unsigned lds = 0;
                            const ChainLayout lw = ci_layout(c->lay_ci, 1, Gc, lds);
                            auto kern1 = kx ? k_chain_ci<1, 0, true> : (lds_nodes ? k_chain_ci<1> : k_chain_ci<1, 64>);
                            hipLaunchKernelGGL(kern1, dim3((unsigned)((n + Gc - 1) / Gc)), dim3(kWave),
                                               lds, st, with_slot(sc, 2), rp, lw, c->d_jump, c->wb, sb,
                                               nb, kWave / Gc, ring, c->d_ctr, Gc == 1 ? ord : nullptr,
                                               Gc == 1 ? ticks : nullptr, ci_stride(c, 1));
                        }
                    };
                    // the heaviest tiles of the last frame get 4 waves each; they are
                    // launched first, on the main stream, and the rest concurrently on
                    // stream2 (same-stream launches would serialise)
                    // (multi-GPU shards, where kw > 1: the rest then run at 1 wave per
                    // tile, the most efficient per lane)
                    // measured wins at 1/2 and 1/4 shards (nb > n_simd); a loss at 1/8
                    // (1020 tiles: 294 -> 307 ms), so smaller launches never split
                    int64_t heavy = (learned && kw > 1 && G == 1 && nb > c->n_simd && ci_split_enabled(c))
                                        ? std::min<int64_t>(c->heavy_k, nb) : 0;
                    // PBRT_CI_EXCLUSIVE = K (experiment): the K heaviest tiles of a shard run first with
                    // a CU each; the rest at kw waves beside them on the second stream
                    int64_t excl = (learned && kw > 1 && G == 1 && c->knobs.ci_exclusive > 0)
                                       ? std::min<int64_t>({c->knobs.ci_exclusive, nb - 1, (int64_t)c->n_simd / 8})
                                       : 0;
                    if (excl > 0) heavy = 0;
                    if (ci_heavy_override(c) >= 0 && learned && G == 1)   // tests and experiments force the split
                        heavy = std::min<int64_t>(ci_heavy_override(c), nb);
                    if (heavy >= nb) heavy = 0;   // nothing left for the light launch: one launch at kw
                    c->last_heavy = heavy;
                    if (ticks) {   // label every slot with the waves it actually runs at
                        c->h_slot_kw.assign((size_t)nb, (uint8_t)(heavy > 0 ? 1 : kw));
                        for (int64_t i = 0; i < heavy; i++) c->h_slot_kw[c->h_slot_order[(size_t)i]] = (uint8_t)ci_heavy_waves(c);
                    }
                    if (excl > 0) {
                        HIPCHK(c, hipEventRecord(c->ev_split, c->stream));
                        launch_ci(kw, excl, order, c->stream, true);
                        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_split, 0));
                        launch_ci(kw, nb - excl, order + excl, c->stream2);
                        HIPCHK(c, hipEventRecord(c->ev_join, c->stream2));
                        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
                    } else if (heavy > 0) {
                        HIPCHK(c, hipEventRecord(c->ev_split, c->stream));
                        launch_ci(ci_heavy_waves(c), heavy, order, c->stream);
                        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_split, 0));
                        launch_ci(1, nb - heavy, order + heavy, c->stream2);
                        HIPCHK(c, hipEventRecord(c->ev_join, c->stream2));
                        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
                    } else {
                        launch_ci(kw, nb, order, c->stream);
                    }
                }
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 1], c->stream));
                if (c->use_dl) {
                    const int64_t nrec = nb * c->wb.ppt;
                    if (rp.spp > 1)
                        hipLaunchKernelGGL(k_dl_samples,
                                           dim3((unsigned)std::min<int64_t>((nrec * (rp.spp - 1) + kWave - 1) / kWave,
                                                                            (int64_t)c->n_simd * 64)),
                                           dim3(kWave), 0, c->stream, with_slot(sc, 3), rp, c->wb, sb, nrec);
                    hipLaunchKernelGGL(k_dl_panics, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, c->stream, rp,
                                       c->wb, sb, nrec, c->d_ctr);
                } else if (paths_wf_enabled(c) || paths_ci_pixels(c, rp) == 0) {
                    // the path wavefront: mesh scenes, and whatever k_paths_ci cannot
                    // take (a tree beyond LDS, more than 64 / P lights)
                    if (rp.mode == PBRT_MODE_THROUGHPUT)
                        hipLaunchKernelGGL(kx ? k_mb_setup<true> : k_mb_setup<false>, dim3((unsigned)(nb * c->wb.ppt)), dim3(kWave),
                                           (unsigned)c->lay.total, c->stream, with_slot(sc, 4), rp, c->lay, c->d_jump,
                                           c->wb, sb, nb);
                    const int rcp = paths_wavefront(c, with_slot(sc, rp.mode == PBRT_MODE_THROUGHPUT ? 5 : 3), sb, nb);
                    if (rcp != PBRT_OK) return rcp;
                } else if (rp.mode == PBRT_MODE_THROUGHPUT && paths_ci_pixels(c, rp) > 0) {
                    // setup (StartPixel + bounce 1 per pixel), then lane-refill paths
                    hipLaunchKernelGGL(kx ? k_mb_setup<true> : k_mb_setup<false>, dim3((unsigned)(nb * c->wb.ppt)),
                                       dim3(kWave), (unsigned)c->lay.total, c->stream, with_slot(sc, 4), rp, c->lay,
                                       c->d_jump, c->wb, sb, nb);
                    const int pp = paths_ci_pixels(c, rp);
                    const int per = rp.ndims * rp.spp;
                    auto kern = kx ? (pp == 8 ? k_paths_ci<8, true, true> : k_paths_ci<4, true, true>)
                                   : (pp == 8 ? k_paths_ci<8, true> : pp == 2 ? k_paths_ci<2, true> : k_paths_ci<4, true>);
                    const int sl = paths_ci_s1d_lds(c, rp, pp) ? 1 : 0;
                    const int lds = pp == 8 ? paths_group_lds<8>(sl * per) : pp == 2 ? paths_group_lds<2>(sl * per)
                                                                                     : paths_group_lds<4>(sl * per);
                    hipLaunchKernelGGL(kern, dim3((unsigned)((nb * c->wb.ppt + pp - 1) / pp)), dim3(kWave),
                                       (unsigned)lds, c->stream, with_slot(sc, 5), rp, c->wb, sb, nb * c->wb.ppt,
                                       c->d_ctr, sl);
                }
                else {
                    const int pp = paths_ci_pixels(c, rp);
                    const int per = rp.ndims * rp.spp;
                    auto kern = kx ? (pp == 8 ? k_paths_ci<8, false, true> : k_paths_ci<4, false, true>)
                                   : (pp == 8 ? k_paths_ci<8> : pp == 2 ? k_paths_ci<2> : k_paths_ci<4>);
                    const int sl = paths_ci_s1d_lds(c, rp, pp) ? 1 : 0;
                    const int lds = pp == 8 ? paths_group_lds<8>(sl * per) : pp == 2 ? paths_group_lds<2>(sl * per)
                                                                                     : paths_group_lds<4>(sl * per);
                    hipLaunchKernelGGL(kern, dim3((unsigned)((nb * c->wb.ppt + pp - 1) / pp)), dim3(kWave),
                                       (unsigned)lds, c->stream, with_slot(sc, 3), rp, c->wb, sb, nb * c->wb.ppt,
                                       c->d_ctr, sl);
                }
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 2], c->stream));
                hipLaunchKernelGGL(k_film, dim3((unsigned)((nb * per + 255) / 256)), dim3(256), 0, c->stream,
                                   c->d_film, rp, c->wb, sb, nb, c->d_films, c->d_cancel_seen);
                hipLaunchKernelGGL(k_panic_reduce, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, c->stream, c->wb,
                                   sb, nb, c->d_panics, c->d_ctr);
                if (rp.spp > 1)
                    hipLaunchKernelGGL(k_ray_count,
                                       dim3((unsigned)std::min<int64_t>((nb * c->wb.ppt * rp.spp + 255) / 256,
                                                                        (int64_t)c->n_simd * 16)),
                                       dim3(256), 0, c->stream, c->wb, nb, rp.spp, c->d_ctr, c->d_cancel_seen);
            }
        } else {
            c->last_kernel = PBRT_KERNEL_SERIAL;
            c->n_batches = 0;
            int64_t blocks = (rp.n_slots + rp.lanes_per_wave - 1) / rp.lanes_per_wave;
            auto kern = k_render_exact<1>;
            if (c->min_waves == 2) kern = k_render_exact<2>;
            else if (c->min_waves == 4) kern = k_render_exact<4>;
            else if (c->min_waves == 8) kern = k_render_exact<8>;
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kWave), 0, c->stream, with_slot(sc, 6), rp, c->d_films,
                               c->d_s1d, c->d_panics, c->d_ctr);
        }
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    int64_t npx = rp.film_w * rp.film_h;
    hipLaunchKernelGGL(k_merge_film, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, c->stream, c->d_film, rp,
                       c->d_films, out);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    c->rendered = true;
    return PBRT_OK;
}

int pbrt_gpu_render_async(pbrt_gpu_ctx* c, const pbrt_render_desc* rd) {
    return pbrt_gpu_render_async_into(c, rd, nullptr);
}

int pbrt_gpu_synchronize(pbrt_gpu_ctx* c, pbrt_gpu_stats* stats) {
    if (!c) return PBRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    const hipError_t se = hipStreamSynchronize(c->stream);
    bool cancelled = false;
    {   // the render has ended: its cancel flag dies with it
        std::lock_guard<std::mutex> lk(c->cancel_mu);
        cancelled = c->in_flight && c->cancel_req;
        c->in_flight = false;
        c->cancel_req = false;
        __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    HIPCHK(c, se);
    if (cancelled) {   // the kernels stopped early: the film and the schedule feedback are not valid
        c->ticks_pending = false;
        c->rendered = false;
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            stats->kernel = c->last_kernel;
            stats->total_ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->t_start).count();
        }
        return set_err(c, PBRT_E_CANCELLED, "cancelled by pbrt_gpu_cancel");
    }
    Counters ctr;
    HIPCHK(c, hipMemcpy(&ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost));
    float ms = 0, ms_merge = 0;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    (void)hipEventElapsedTime(&ms_merge, c->ev1, c->ev2);
    int rc = PBRT_OK;
    pbrt_gpu_stats st;
    std::memset(&st, 0, sizeof(st));
    st.tiles_rendered = (uint64_t)c->rp.n_slots;
    st.camera_samples = ctr.camera_samples;
    st.paths_traced = ctr.paths;
    st.kernel_ms = ms;
    st.merge_ms = ms_merge;
    st.kernel = c->last_kernel;
    st.batches = c->n_batches;
    st.rays_closest = ctr.closest_rays;
    st.rays_shadow = ctr.shadow_rays;
    for (int b = 0; b < c->n_batches; b++) {
        float a = 0, p = 0;
        (void)hipEventElapsedTime(&a, c->bev[3 * b + 0], c->bev[3 * b + 1]);
        (void)hipEventElapsedTime(&p, c->bev[3 * b + 1], c->bev[3 * b + 2]);
        st.chain_ms += a;
        st.paths_ms += p;
    }
    if (c->ticks_pending) {   // heaviest-first slot order for the next frame of this configuration
        c->ticks_pending = false;
        std::vector<uint32_t> t((size_t)c->ticks_n);
        HIPCHK(c, hipMemcpy(t.data(), c->d_ticks, sizeof(uint32_t) * t.size(), hipMemcpyDeviceToHost));
        c->h_last_ticks = t;   // pbrt_gpu_tile_ticks
        // cost at 1 wave per tile: 2 and 4 waves measured 1.3x / 1.8x faster per tile
        std::vector<double> cost(t.size());
        double sum = 0;
        for (size_t i = 0; i < t.size(); i++) {
            const int w = i < c->h_slot_kw.size() ? c->h_slot_kw[i] : 1;
            cost[i] = (double)t[i] * (w == 8 ? 2.3 : w == 4 ? 1.8 : w == 2 ? 1.3 : 1.0);
            sum += cost[i];
        }
        c->h_slot_order.resize(t.size());
        for (size_t i = 0; i < t.size(); i++) c->h_slot_order[i] = (uint32_t)i;
        std::stable_sort(c->h_slot_order.begin(), c->h_slot_order.end(),
                         [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
        // heavy: tiles whose 1-wave chain alone would take over 0.7x the
        // frame's throughput bound (summed cost over 2 waves/SIMD)
        const double thr = 0.7 * sum / (2.0 * (double)c->n_simd);
        int64_t k = 0;
        while (k < (int64_t)t.size() && cost[c->h_slot_order[(size_t)k]] > thr) k++;
        c->heavy_k = std::min<int64_t>(k, c->n_simd / 4);   // at most a quarter of the wave slots
        if (ci_heavy_override(c) >= 0) c->heavy_k = ci_heavy_override(c);
        c->order_key = c->ticks_key;
    }
    if (ctr.any_panic) {
        std::vector<PanicRec> pr((size_t)c->rp.n_slots);
        HIPCHK(c, hipMemcpy(pr.data(), c->d_panics, sizeof(PanicRec) * pr.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < pr.size(); i++) {
            if (pr[i].kind == 0) continue;
            st.panic_kind = pr[i].kind;
            st.panic_tile = (int32_t)(c->rp.tile_begin + (int64_t)i * c->rp.tile_stride);
            st.panic_pixel_x = pr[i].px;
            st.panic_pixel_y = pr[i].py;
            st.panic_sample = pr[i].sample;
            st.panic_bounce = pr[i].bounce;
            break;
        }
        if (st.panic_kind == -1) {
            rc = set_err(c, PBRT_E_UNSUPPORTED, "unsupported material");
            st.panic_kind = 0;
        } else {
            rc = set_err(c, PBRT_E_REF_PANIC, "the Go reference panics on this input");
        }
    }
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->t_start).count();
    if (stats) *stats = st;
    return rc;
}

int pbrt_gpu_render(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_xyz, pbrt_gpu_stats* stats) {
    if (!c) return PBRT_E_INVALID;
    int rc = pbrt_gpu_render_async(c, rd);
    if (rc != PBRT_OK) return rc;
    rc = pbrt_gpu_synchronize(c, stats);
    if (rc != PBRT_OK) return rc;
    if (film_xyz) return pbrt_gpu_film_download(c, film_xyz);
    return PBRT_OK;
}

double* pbrt_gpu_film_device(pbrt_gpu_ctx* c) { return c ? c->d_out : nullptr; }
void* pbrt_gpu_stream(pbrt_gpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

int pbrt_gpu_film_download(pbrt_gpu_ctx* c, double* film_xyz) {
    if (!c || !film_xyz || !c->rendered) return PBRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(film_xyz, c->film_target ? c->film_target : c->d_out,
                        sizeof(double) * (size_t)(c->rp.film_w * c->rp.film_h * 3),
                        hipMemcpyDeviceToHost));
    return PBRT_OK;
}

static int intersect_batch(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, int any, pbrt_hit_soa* hits,
                           uint8_t* occluded) {
    if (!c || !rays || (!hits && !occluded)) return PBRT_E_INVALID;
    if (n == 0) return PBRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<double> packed(n * 7);
    for (size_t i = 0; i < n; i++) {
        double* q = &packed[7 * i];
        q[0] = rays->ox[i]; q[1] = rays->oy[i]; q[2] = rays->oz[i];
        q[3] = rays->dx[i]; q[4] = rays->dy[i]; q[5] = rays->dz[i];
        q[6] = rays->tmax ? rays->tmax[i] : gomath::kInf;
    }
    size_t nout = any ? n : 9 * n;
    double *d_in = nullptr, *d_o = nullptr;
    HIPCHK(c, hipMalloc((void**)&d_in, sizeof(double) * packed.size()));
    if (hipMalloc((void**)&d_o, sizeof(double) * nout) != hipSuccess) {
        (void)hipFree(d_in);
        return set_err(c, PBRT_E_HIP, "hipMalloc");
    }
    std::vector<double> o(nout);
    hipError_t e = hipMemcpyAsync(d_in, packed.data(), sizeof(double) * packed.size(), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        DevScene sc = dev_scene(c, false);
        hipLaunchKernelGGL(k_intersect, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave), 0, c->stream,
                           with_slot(sc, 7),
                           (int64_t)n, d_in, d_o, any);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(o.data(), d_o, sizeof(double) * nout, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_in);
    (void)hipFree(d_o);
    if (e != hipSuccess) return set_err(c, PBRT_E_HIP, hipGetErrorString(e));
    int rc = PBRT_OK;
    for (size_t i = 0; i < n; i++) {
        if (any) {
            if (gomath::is_nan(o[i])) rc = PBRT_E_REF_PANIC;
            occluded[i] = o[i] == 1.0;
        } else {
            const double* r = &o[9 * i];
            if (gomath::is_nan(r[0])) { rc = PBRT_E_REF_PANIC; hits->hit[i] = 0; continue; }
            hits->hit[i] = r[0] == 1.0;
            if (hits->t_max) hits->t_max[i] = r[1];
            if (hits->prim) hits->prim[i] = (int32_t)r[2];
            if (hits->px) hits->px[i] = r[3];
            if (hits->py) hits->py[i] = r[4];
            if (hits->pz) hits->pz[i] = r[5];
            if (hits->nx) hits->nx[i] = r[6];
            if (hits->ny) hits->ny[i] = r[7];
            if (hits->nz) hits->nz[i] = r[8];
        }
    }
    if (rc != PBRT_OK) set_err(c, rc, "the Go reference panics on at least one ray");
    return rc;
}

int pbrt_gpu_intersect(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, pbrt_hit_soa* hits) {
    return intersect_batch(c, rays, n, 0, hits, nullptr);
}
int pbrt_gpu_intersect_p(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, uint8_t* occluded) {
    return intersect_batch(c, rays, n, 1, nullptr, occluded);
}

void pbrt_gpu_cancel(pbrt_gpu_ctx* c) {
    if (!c) return;
    std::lock_guard<std::mutex> lk(c->cancel_mu);
    if (!c->in_flight) return;   // nothing to cancel: no render is in flight
    c->cancel_req = true;
    __atomic_store_n(c->h_cancel, 1, __ATOMIC_SEQ_CST);
}
const char* pbrt_gpu_last_error(const pbrt_gpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

void pbrt_gpu_destroy(pbrt_gpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->d_shapes, c->d_materials, c->d_prims, c->d_nodes, c->d_order, c->d_lights, c->d_camera, c->d_film,
                    c->d_dist,   c->d_films,     c->d_s1d,   c->d_panics, c->d_ctr,   c->d_out,    c->d_jump,
                    c->d_wave,   c->d_fprims, c->d_ticks, c->d_slot_order, c->d_groups,
                    c->d_gmasks, c->d_cost,   c->d_cost_keys, c->d_pw, c->d_cancel_seen};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    mesh_bvh_free(c->mesh);
    for (hipEvent_t e : c->bev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->ev_split) (void)hipEventDestroy(c->ev_split);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->stream2) {
        (void)hipStreamSynchronize(c->stream2);
        (void)hipStreamDestroy(c->stream2);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->h_cancel) (void)hipHostFree(c->h_cancel);
    delete c;
}

// film.go:142-179 WriteImage pixel conversion
int pbrt_film_to_rgba8(const double* film, int64_t w, int64_t h, uint8_t* rgba) {
    if (!film || !rgba || w <= 0 || h <= 0) return PBRT_E_INVALID;
    for (int64_t i = 0; i < w * h; i++) {
        for (int c = 0; c < 3; c++)
            rgba[i * 4 + c] = (uint8_t)(gomath::to_int(gomath::clamp(film[i * 3 + c], 0, 1) * 255) & 0xFF);
        rgba[i * 4 + 3] = 255;
    }
    return PBRT_OK;
}

}  // extern "C"

// ============================================================ diagnostics
#include "../../include/pbrt_diag.h"

namespace {
__global__ void k_probe(int op, const double* __restrict__ in, int64_t n, int in_stride, double* __restrict__ out,
                        int out_stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* a = in + i * in_stride;
    double* o = out + i * out_stride;
    switch (op) {
        case PBRT_PROBE_SIN: o[0] = gomath::sin(a[0]); break;
        case PBRT_PROBE_COS: o[0] = gomath::cos(a[0]); break;
        case PBRT_PROBE_TAN: o[0] = gomath::tan(a[0]); break;
        case PBRT_PROBE_ATAN: o[0] = gomath::atan(a[0]); break;
        case PBRT_PROBE_ATAN2: o[0] = gomath::atan2(a[0], a[1]); break;
        case PBRT_PROBE_ASIN: o[0] = gomath::asin(a[0]); break;
        case PBRT_PROBE_ACOS: o[0] = gomath::acos(a[0]); break;
        case PBRT_PROBE_SQRT: o[0] = gomath::sqrt(a[0]); break;
        case PBRT_PROBE_DIV: o[0] = a[0] / a[1]; break;
        case PBRT_PROBE_NEXTAFTER: o[0] = gomath::nextafter(a[0], a[1]); break;
        case PBRT_PROBE_MAX: o[0] = gomath::max(a[0], a[1]); break;
        case PBRT_PROBE_MIN: o[0] = gomath::min(a[0], a[1]); break;
        case PBRT_PROBE_OFFSET_RAY_ORIGIN: {
            V3 r = offset_ray_origin(load3(a), load3(a + 3), load3(a + 6), load3(a + 9));
            o[0] = r.x; o[1] = r.y; o[2] = r.z;
            break;
        }
        case PBRT_PROBE_EFLOAT_ADD: {
            int panic = 0;
            EF r = ef_add(ef_new(a[0], a[1], panic), ef_new(a[2], a[3], panic), panic);
            o[0] = r.v; o[1] = r.lo; o[2] = r.hi; o[3] = panic;
            break;
        }
        case PBRT_PROBE_TRANSFORM_RAY: {
            pbrt_matrix4x4 m;
            for (int k = 0; k < 16; k++) m.m[k / 4][k % 4] = a[k];
            Ray r{load3(a + 16), load3(a + 19), gomath::kInf, 0};
            Ray w = xf_ray(m, r, nullptr, nullptr);
            o[0] = w.o.x; o[1] = w.o.y; o[2] = w.o.z; o[3] = w.d.x; o[4] = w.d.y; o[5] = w.d.z;
            break;
        }
        case PBRT_PROBE_SPAWN_RAY_TO: {
            V3 p0 = load3(a), e0 = load3(a + 3), n0 = load3(a + 6), p1 = load3(a + 9), e1 = load3(a + 12),
               n1 = load3(a + 15);
            V3 origin = offset_ray_origin(p0, e0, n0, p1 - p0);
            V3 target = offset_ray_origin(p1, e1, n1, origin - p1);
            V3 d = target - origin;
            o[0] = p0.x; o[1] = p0.y; o[2] = p0.z; o[3] = d.x; o[4] = d.y; o[5] = d.z; o[6] = 1 - 0.0001;
            break;
        }
        case PBRT_PROBE_PCG: {
            Pcg r;
            pcg_seed(r, (uint64_t)a[0]);
            for (int k = 0; k < out_stride; k++) o[k] = pcg_float(r);
            break;
        }
        case PBRT_PROBE_MIN_NONAN: o[0] = gomath::min_nonan(a[0], a[1]); break;
        case PBRT_PROBE_MAX_NONAN: o[0] = gomath::max_nonan(a[0], a[1]); break;
        case PBRT_PROBE_EFLOAT_MUL:
        case PBRT_PROBE_EFLOAT_DIV: {
            int panic = 0;
            EF x = ef_new(a[0], a[1], panic), y = ef_new(a[2], a[3], panic);
            EF r = op == PBRT_PROBE_EFLOAT_MUL ? ef_mul(x, y, panic) : ef_div(x, y, panic);
            o[0] = r.v; o[1] = r.lo; o[2] = r.hi; o[3] = panic;
            break;
        }
        case PBRT_PROBE_NEXT_FLOAT_UP: o[0] = gomath::next_up(a[0]); break;
        case PBRT_PROBE_NEXT_FLOAT_DOWN: o[0] = gomath::next_down(a[0]); break;
        default: o[0] = gomath::nan();
    }
}
}  // namespace

extern "C" int pbrt_gpu_probe(int device, int op, const double* in, size_t n, int in_stride, double* out,
                              int out_stride) {
    if (!in || !out || in_stride <= 0 || out_stride <= 0) return PBRT_E_INVALID;
    if (n == 0) return PBRT_OK;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return PBRT_E_HIP;
    double *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc((void**)&d_in, sizeof(double) * n * in_stride) != hipSuccess) return PBRT_E_HIP;
    if (hipMalloc((void**)&d_out, sizeof(double) * n * out_stride) != hipSuccess) {
        (void)hipFree(d_in);
        return PBRT_E_HIP;
    }
    hipError_t e = hipMemcpy(d_in, in, sizeof(double) * n * in_stride, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, d_in, (int64_t)n,
                           in_stride, d_out, out_stride);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(double) * n * out_stride, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return e == hipSuccess ? PBRT_OK : PBRT_E_HIP;
}

extern "C" int pbrt_gpu_counters(pbrt_gpu_ctx* c, uint64_t* out, int n) {
    if (!c || !out) return PBRT_E_INVALID;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) return PBRT_E_HIP;
    Counters ctr;
    if (hipMemcpy(&ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost) != hipSuccess) return PBRT_E_HIP;
    const uint64_t v[kNumCounters] = {ctr.paths,    ctr.camera_samples, ctr.closest_rays, ctr.shadow_rays,
                                      (uint64_t)ctr.any_panic, ctr.windows, ctr.phase[0], ctr.phase[1],
                                      ctr.phase[2], ctr.phase[3], ctr.phase[4], ctr.phase[5],
                                      ctr.phase[6], ctr.phase[7]};
    for (int i = 0; i < n && i < kNumCounters; i++) out[i] = i < 14 ? v[i] : (uint64_t)ctr.dhist[i - 14];
    return kNumCounters;
}

extern "C" int pbrt_gpu_mesh_info(pbrt_gpu_ctx* c, double* out, int n) {
    if (!c || !out) return -PBRT_E_INVALID;
    const double v[] = {(double)c->mesh.n_tris, (double)c->mesh.n_nodes, (double)c->mesh.depth, c->mesh.build_ms,
                        (double)c->mesh.n_meshes};
    const int m = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = v[i];
    return m;
}
extern "C" int pbrt_gpu_mesh_counters(uint64_t* out, int n, int reset) {
#ifdef PBRT_MESH_COUNT
    unsigned long long h[kMeshCountSlots * 6];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mesh_count), sizeof(h)) != hipSuccess) return -PBRT_E_HIP;
    for (int i = 0; i < n && i < kMeshCountSlots * 6; i++) out[i] = h[i];
    if (reset) {
        std::memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_mesh_count), h, sizeof(h)) != hipSuccess) return -PBRT_E_HIP;
    }
    return kMeshCountSlots * 6;
#else
    (void)out; (void)n; (void)reset;
    return 0;
#endif
}

extern "C" int pbrt_gpu_mesh_download(pbrt_gpu_ctx* c, void* nodes, int32_t* gid, float* tris) {
    if (!c) return PBRT_E_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) return PBRT_E_HIP;
    const size_t nn = (size_t)c->mesh.n_nodes * kMeshOrders, nt = (size_t)c->mesh.n_tris;
    if (nodes && nn && hipMemcpy(nodes, c->mesh.nodes, nn * sizeof(MeshNode), hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    if (gid && nt && hipMemcpy(gid, c->mesh.gid, nt * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    if (tris && nt && hipMemcpy(tris, c->mesh.tris, nt * 9 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    return PBRT_OK;
}

extern "C" int64_t pbrt_gpu_tile_ticks(pbrt_gpu_ctx* c, uint32_t* out, int64_t n, int64_t* heavy) {
    if (!c) return -PBRT_E_INVALID;
    if (heavy) *heavy = c->last_heavy;
    const int64_t m = (int64_t)c->h_last_ticks.size();
    for (int64_t i = 0; out && i < n && i < m; i++) out[i] = c->h_last_ticks[(size_t)i];
    return m;
}

extern "C" int64_t pbrt_gpu_tile_costs(pbrt_gpu_ctx* c, float* out, int64_t n) {
    if (!c) return -PBRT_E_INVALID;
    if (!c->probed || !c->d_cost) return 0;
    if (out && n > 0) {
        const int64_t m = std::min<int64_t>(n, c->cost_n);
        if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(out, c->d_cost, sizeof(float) * 4 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess)
            return -PBRT_E_HIP;
    }
    return c->cost_n;
}

// Region cycles of trajectory steps (PBRT_STEP_TIMING builds only; else zeros):
// [0] loop top / light-sample draws, [1] closest-hit traversal + interaction,
// [2] BSDF setup, [3] light sampling (full paths), [4] BSDF sample + spawn + RR.
extern "C" int pbrt_gpu_step_cycles(uint64_t* out, int n, int reset) {
#ifdef PBRT_STEP_TIMING
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_step_cycles), sizeof(h)) != hipSuccess) return PBRT_E_HIP;
    for (int i = 0; i < n && i < 8; i++) out[i] = h[i];
    if (reset) {
        std::memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_cycles), h, sizeof(h)) != hipSuccess) return PBRT_E_HIP;
    }
#else
    for (int i = 0; i < n && i < 8; i++) out[i] = 0;
    (void)reset;
#endif
    return 8;
}

extern "C" int pbrt_abi_sizes(size_t* out, int n) {
    const size_t s[] = {sizeof(pbrt_matrix4x4),   sizeof(pbrt_transform),    sizeof(pbrt_shape_desc),
                        sizeof(pbrt_material_desc), sizeof(pbrt_primitive_desc), sizeof(pbrt_bvh_node),
                        sizeof(pbrt_light_desc),  sizeof(pbrt_camera_desc),  sizeof(pbrt_film_desc),
                        sizeof(pbrt_distribution_desc), sizeof(pbrt_scene_desc), sizeof(pbrt_render_desc),
                        sizeof(pbrt_gpu_stats),   sizeof(pbrt_ray_soa),      sizeof(pbrt_hit_soa),
                        sizeof(pbrt_gpu_opts),    sizeof(pbrt_mesh_desc)};
    int m = (int)(sizeof(s) / sizeof(s[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = s[i];
    return m;
}
