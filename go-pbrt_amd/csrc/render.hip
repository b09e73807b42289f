// render.hip — MI355X (gfx950) kernels and the C ABI of include/pbrt_gpu.h.
//
// Kernels
//   k_render_exact   EXACT mode: one lane per 16-px tile. The lane replays the
//                    tile's PCG32 stream exactly as pbrt.Render's worker does
//                    (integrator.go:228-289, 311-340): pixel loop, Stratified
//                    StartPixel, samples 1..spp-1, Path.Li / DirectLighting.Li,
//                    NaN guard, FilmTile.AddSample into the tile's film slot.
//   k_render_decorr  THROUGHPUT mode: same arithmetic, one lane per
//                    (pixel, sample) path with its own PCG32 stream; paths of
//                    one pixel are summed in sample order in a second pass.
//   k_merge_film     Film.MergeFilmTile (film.go:115-132): per output pixel,
//                    RGBToXYZ of every covering tile film in tile-index order.
//   k_intersect[_p]  batch BVH closest-hit / any-hit (bvh.go:659-765).
//
// Everything is float64 with -ffp-contract=off (bit parity with the Go
// reference). The scene is a few KB and is read through the scalar/vector L1.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pbrt_gpu.h"
#include "../../include/pbrt_scene.h"
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
    int32_t sp_events, sp_draws, sp_serial, pad1;   // wave kernel StartPixel: events, raw draws buffered
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
};
constexpr int kNumCounters = 6 + 8;

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

    for (int64_t py = y0; py < y1; py++) {
        for (int64_t px = x0; px < x1; px++) {
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
                V2 u0 = get2d(t);
                V2 plens = get2d(t);
                double tu = get1d(t);
                Ray ray = camera_ray(cam, (double)px + u0.x, (double)py + u0.y, tu, plens);
                Spec L = (rp.integrator == PBRT_INTEGRATOR_PATH) ? path_li(sc, t, ray, rp.max_depth, rp.rr_threshold)
                                                                 : direct_li(sc, t, ray, rp.max_depth, rp.dl_strategy);
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
// One 64-lane wave per tile; see pbrt_spec.h for why this is the same
// computation as k_render_exact. Per pixel:
//   1. StartPixel: the ~ndims*2*spp draws are computed lane-parallel by PCG
//      jump-ahead (assuming pcg_bounded never rejects, checked; on a
//      rejection lane 0 replays StartPixel serially), then one lane per dim
//      runs the Fisher-Yates swaps.
//   2. Bounce 1: camera ray, first hit and BSDF (wave-uniform); lane l
//      computes EstimateDirect for light l with uLight = (0,0).
//   3. Chain: trajectories at offsets head + 2j (j = lane) give D per offset;
//      lane 0 walks head -> head + D -> ... to assign each sample its offset.
//   4. Samples 1..spp-1 run as full paths, one per lane (batches of 64), and
//      are added to the tile film (LDS) in sample order.
struct SpecLayout {   // byte offsets into the dynamic LDS block
    int film, s1d, other, memb, lbuf, sbuf, dbuf, pbuf, vbuf, total;
};
constexpr uint32_t kBadD = 0xFFFFFFFFu;

__device__ __forceinline__ double pcg_float_of(uint32_t v) {
    return gomath::min(gomath::kOneMinusEpsilon, (double)v * 2.3283064365386963e-10);
}

// Bounce 1 of a pixel (camera ray, first hit, BSDF; EstimateDirect per light
// with uLight = (0,0), lane l computing light l) into the LDS cache. Returns
// 1 = hit, 0 = no traced bounce, or kind - 1000 (< 0) when the first hit
// panics (kind = PBRT_PANIC_* or -1 for an unsupported material). Out of line:
// it runs once per pixel.
__device__ __noinline__ int pixel_setup(DevScene sc, const RenderParams& rp, const pbrt_camera_desc& cam, int64_t px,
                                        int64_t py, double time_u, PixelCache* pc, uint16_t* stack, int lane) {
    Ray ray = camera_ray(cam, (double)px + 0.0, (double)py + 0.0, time_u, V2{0.0, 0.0});
    int panic0 = 0;
    SI si0;
    BSDF b0;
    b0.n_bxdfs = 0;
    int hit0 = 0;
    if (1 < rp.max_depth) {
        hit0 = bvh_traverse<false>(sc, ray, &si0, stack, panic0) ? 1 : 0;
        if (!panic0 && hit0 && compute_bsdf(sc, si0, b0) < 0) panic0 = -1;
    }
    if (panic0) return panic0 - 1000;
    if (lane == 0) {
        pc->si = si0;
        pc->b = b0;
        pc->wo = ray.d;
        pc->hit = hit0;
    }
    if (hit0 && b0.n_bxdfs > 0 && lane < sc.n_lights) {
        int pl = 0;
        Spec ld = estimate_direct(sc, stack, pl, si0, b0, lane, V2{0.0, 0.0});
        if (!pl && max_component(ld) > 10) pl = PBRT_PANIC_LD_GT_10;
        pc->ld[lane] = ld;
        pc->ld_panic[lane] = pl;
    }
    return hit0;
}

template <int kWaves>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void k_render_spec(DevScene sc, RenderParams rp, SpecLayout lay,
                                                       const PcgJump* __restrict__ jump,
                                                       double* __restrict__ films, PanicRec* __restrict__ panics,
                                                       Counters* __restrict__ ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint16_t stack_lds[64 * kStackStride];
    __shared__ PixelCache pc;
    __shared__ uint64_t sh_state;
    __shared__ int sh_k, sh_flag, sh_trunc, sh_stop, sh_tkind, sh_tbounce;
    const int lane = threadIdx.x;
    const int64_t slot = blockIdx.x;
    const int64_t tile = rp.tile_begin + slot * rp.tile_stride;
    const pbrt_film_desc& film = *sc.film;
    const PcgJump& J = *jump;
    double* film_l = (double*)(lds + lay.film);
    double* s1d = (double*)(lds + lay.s1d);
    uint16_t* other = (uint16_t*)(lds + lay.other);
    uint64_t* memb = (uint64_t*)(lds + lay.memb);
    double* lbuf = (double*)(lds + lay.lbuf);
    uint64_t* sbuf = (uint64_t*)(lds + lay.sbuf);
    uint32_t* dbuf = (uint32_t*)(lds + lay.dbuf);
    int* pbuf = (int*)(lds + lay.pbuf);
    uint32_t* vbuf = (uint32_t*)(lds + lay.vbuf);
    uint16_t* stack = stack_lds + lane;

    int64_t x0, y0, x1, y1, px0, py0, px1, py1;
    tile_bounds(rp, tile, x0, y0, x1, y1);
    film_tile_bounds(film, x0, y0, x1, y1, px0, py0, px1, py1);
    const int64_t npx = (px1 - px0) * (py1 - py0);
    for (int64_t i = lane; i < npx * 3; i += kWave) film_l[i] = 0.0;

    const int n = rp.spp, ndims = rp.ndims, nl = sc.n_lights;
    const double inv_n = 1.0 / (double)n;
    const int s1 = rp.jitter ? 2 * n : n, s2 = rp.jitter ? 3 * n : n;   // StartPixel draws per 1D / 2D dim
    Pcg seed;
    pcg_seed(seed, (uint64_t)tile);   // Sampler.Clone(seed = tile index), integrator.go:318,328
    const uint64_t inc = seed.inc;
    uint64_t S = seed.state;
    const SpecSampler ss{s1d, n, ndims};
    const pbrt_camera_desc& cam = *sc.camera;
    unsigned long long paths = 0, windows = 0;
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long tprev = clock64();
    auto mark = [&](int i) {
        long long now = clock64();
        ph[i] += (unsigned long long)(now - tprev);
        tprev = now;
    };
    __syncthreads();

    for (int64_t py = y0; py < y1; py++) {
        for (int64_t px = x0; px < x1; px++) {
            // ---- 1. StartPixel (stratified.go:21-48)
            // The pixel's draws form a fixed list of E events (jitter floats and
            // pcg_bounded shuffle picks, sampling.go:101-145). A bounded pick
            // retries on v < 2^32 mod b, which the reference's (rot+1)&31 output
            // rotation makes common (v < 4 has probability ~1/64), so event e
            // lands on draw e + R(e), R(e) = rejections before it. Lanes fill
            // the raw stream by jump-ahead, then resolve R chunk by chunk: one
            // ballot per rejection shifts every later event by one draw.
            bool serial_sp = rp.sp_serial != 0;
            if (!serial_sp) {
                const int E = rp.sp_events, V = rp.sp_draws;
                uint64_t st = pcg_advance(J, S, inc, (uint64_t)lane);
                for (int t = lane; t < V; t += kWave) {
                    vbuf[t] = pcg_output(st);
                    st = J.a[6] * st + inc * J.b[6];   // +64 draws
                }
                __syncthreads();
                mark(5);
                int R = 0;
                bool overflow = false;
                for (int cb = 0; cb < E; cb += kWave) {
                    const int e = cb + lane;
                    int kind = 0, slot = 0, i = 0;   // kind 0 none, 1 1D float, 2 1D pick, 3 2D pick
                    if (e < E) {
                        if (e < ndims * s1) {
                            const int d = e / s1, q = e - d * s1;
                            if (rp.jitter && q < n) { kind = 1; slot = d * n + q; }
                            else { kind = 2; i = q - (rp.jitter ? n : 0); slot = d * n + i; }
                        } else {
                            const int e2 = e - ndims * s1, d = e2 / s2, q = e2 - d * s2;
                            if (!(rp.jitter && q < 2 * n)) { kind = 3; i = q - (rp.jitter ? 2 * n : 0); }
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
                        s1d[slot] = gomath::min(((double)(slot % n) + pcg_float_of(v)) * inv_n, gomath::kOneMinusEpsilon);
                    else if (kind == 2)
                        other[slot] = (uint16_t)(i + (int)(v % b));
                    R += __shfl(local, kWave - 1);
                }
                serial_sp = overflow;
                if (!serial_sp) {
                    if (!rp.jitter)
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
                    if (lane == 0) sh_state = pcg_advance(J, S, inc, (uint64_t)(E + R));
                }
            }
            if (serial_sp || (rp.flags & PBRT_FLAG_SERIAL_START_PIXEL)) {
                ph[7]++;
                if (lane == 0) {   // serial replay (huge sample counts, or forced)
                    Thread t;
                    t.rng.state = S;
                    t.rng.inc = inc;
                    t.spp = n; t.ndims = ndims; t.xs = rp.xs; t.ys = rp.ys; t.jitter = rp.jitter;
                    t.s1d = s1d;
                    start_pixel(t);
                    sh_state = t.rng.state;
                }
            }
            __syncthreads();
            S = sh_state;
            mark(0);
            if (n <= 1) continue;   // sample 0 is never traced (#2)

            // ---- 2. bounce 1, shared by every sample of the pixel
            const int hit0 = pixel_setup(sc, rp, cam, px, py, s1d[1 < n ? 1 : 0], &pc, stack, lane);
            if (hit0 < 0) {   // the first traced sample panics at bounce 1
                if (lane == 0) {
                    PanicRec pr{hit0 + 1000, 1, 1, 0, px, py};
                    panics[slot] = pr;
                    atomicExch(&ctr->any_panic, 1);
                }
                return;
            }
            if (lane == 0) {
                sh_trunc = 0;
                sh_stop = 0;
            }
            __syncthreads();
            mark(1);
            // ---- 3. offsets of samples 1..n-1 (chain through speculative trajectories)
            int kend = n;
            if (hit0) {
                uint64_t Sh = S;
                int kh = 1;
                while (kh < n) {
                    const uint64_t st = pcg_advance(J, Sh, inc, 2 * (uint64_t)lane);
                    Cursor c;
                    c.rng.state = st;
                    c.rng.inc = inc;
                    c.draws = 0;
                    c.cur1d = 1;   // camera: Get2D pFilm, Get2D pLens, Get1D time (stratified)
                    c.cur2d = 2;
                    c.k = lane == 0 ? kh : -1;
                    c.kdep = 0;
                    int pnc = 0, bnc = 0;
                    (void)spec_path(sc, pc, ss, c, rp.max_depth, rp.rr_threshold, stack, pnc, bnc, false);
                    windows++;
                    sbuf[lane] = st;
                    dbuf[lane] = (pnc || c.kdep) ? kBadD : c.draws;
                    __syncthreads();
                    mark(2);
                    if (lane == 0) {
                        uint64_t x = 0;
                        int k = kh;
                        while (k < n) {
                            if ((x & 1) || (x >> 1) >= (uint64_t)kWave) break;
                            const uint32_t d = dbuf[x >> 1];
                            if (d == kBadD) break;
                            memb[k++] = sbuf[x >> 1];
                            x += d;
                        }
                        if (k == kh) {   // the exact head itself panicked
                            memb[kh] = Sh;
                            sh_trunc = kh;
                            sh_tkind = pnc;
                            sh_tbounce = bnc;
                        }
                        sh_k = k;
                        sh_state = pcg_advance(J, Sh, inc, x);
                    }
                    __syncthreads();
                    kh = sh_k;
                    Sh = sh_state;
                    mark(6);
                    if (sh_trunc) break;
                }
                S = Sh;
                if (sh_trunc) kend = sh_trunc + 1;
            }

            mark(2);
            // ---- 4. full paths, one sample per lane, added in sample order
            const double fx = (double)px + 0.0, fy = (double)py + 0.0;
            Footprint fp;
            int64_t p0x, p0y, p1x, p1y;
            footprint(film, fx, fy, px0, py0, px1, py1, fp, p0x, p0y, p1x, p1y);
            for (int kb = 1; kb < kend; kb += kWave) {
                const int k = kb + lane;
                Spec L = spec(0);
                int pnc = 0, bnc = 0;
                if (k < kend && hit0) {
                    Cursor c;
                    c.rng.state = memb[k];
                    c.rng.inc = inc;
                    c.draws = 0;
                    c.cur1d = 1;
                    c.cur2d = 2;
                    c.k = k;
                    c.kdep = 0;
                    L = spec_path(sc, pc, ss, c, rp.max_depth, rp.rr_threshold, stack, pnc, bnc, true);
                }
                lbuf[lane * 3 + 0] = L.r;
                lbuf[lane * 3 + 1] = L.g;
                lbuf[lane * 3 + 2] = L.b;
                pbuf[lane * 2 + 0] = (k < kend) ? pnc : 0;
                pbuf[lane * 2 + 1] = bnc;
                __syncthreads();
                if (lane == 0) {
                    for (int m = 0; m < kWave && kb + m < kend; m++) {
                        if (pbuf[m * 2]) {
                            PanicRec pr{pbuf[m * 2], kb + m, pbuf[m * 2 + 1], 0, px, py};
                            panics[slot] = pr;
                            atomicExch(&ctr->any_panic, 1);
                            sh_stop = 1;
                            break;
                        }
                    }
                }
                __syncthreads();
                if (sh_stop) return;
                mark(3);
                const int kn = (kend - kb < kWave) ? kend - kb : kWave;
                if (lane < fp.n * 3) {
                    const int f = lane / 3, ch = lane - f * 3;
                    const double w = fp.w[f];
                    double acc = film_l[fp.off[f] * 3 + ch];
                    for (int m = 0; m < kn; m++) {
                        Spec Ls{lbuf[m * 3 + 0], lbuf[m * 3 + 1], lbuf[m * 3 + 2]};
                        if (has_nans(Ls)) Ls = spec(0.1);   // integrator.go:256-262
                        if (0.0 > film.max_sample_luminance) Ls = smuls(Ls, film.max_sample_luminance / 0.0);
                        const double v = ch == 0 ? Ls.r : (ch == 1 ? Ls.g : Ls.b);
                        acc += v * w;
                    }
                    film_l[fp.off[f] * 3 + ch] = acc;
                }
                __syncthreads();
                mark(4);
            }
            if (sh_trunc) {   // head panicked in the trajectory but no full path did: report it
                if (lane == 0) {
                    PanicRec pr{sh_tkind, sh_trunc, sh_tbounce, 0, px, py};
                    panics[slot] = pr;
                    atomicExch(&ctr->any_panic, 1);
                }
                return;
            }
            paths += (unsigned long long)(n - 1);
        }
    }
    double* tf = films + slot * (rp.slot_w * rp.slot_h * 3);
    for (int64_t i = lane; i < npx * 3; i += kWave) tf[i] = film_l[i];
    if (lane == 0) {
        atomicAdd(&ctr->paths, paths);
        atomicAdd(&ctr->camera_samples, paths);
        atomicAdd(&ctr->windows, windows);
        for (int i = 0; i < 8; i++) atomicAdd(&ctr->phase[i], ph[i]);
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
struct pbrt_gpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    double* film_target = nullptr;   // caller buffer of the last render_async_into
    int lanes_per_wave = 64;
    int min_waves = 1;      // amdgpu_waves_per_eu variant of k_render_exact
    int kernel_req = PBRT_KERNEL_AUTO;
    int last_kernel = 0;    // PBRT_KERNEL_SERIAL / PBRT_KERNEL_WAVE
    PcgJump* d_jump = nullptr;
    pbrt_distribution_desc host_dist;
    SpecLayout lay{};
    bool use_spec = false;
    // device scene
    pbrt_shape_desc* d_shapes = nullptr;
    pbrt_material_desc* d_materials = nullptr;
    pbrt_primitive_desc* d_prims = nullptr;
    pbrt_bvh_node* d_nodes = nullptr;
    pbrt_light_desc* d_lights = nullptr;
    pbrt_camera_desc* d_camera = nullptr;
    pbrt_film_desc* d_film = nullptr;
    pbrt_distribution_desc* d_dist = nullptr;
    pbrt_scene_desc host_scene;   // counts + film/camera (pointer fields are not kept)
    std::vector<pbrt_light_desc> host_lights;
    // per-render buffers (grown on demand)
    double* d_films = nullptr;
    size_t films_cap = 0;
    double* d_s1d = nullptr;
    size_t s1d_cap = 0;
    PanicRec* d_panics = nullptr;
    size_t panics_cap = 0;
    Counters* d_ctr = nullptr;
    double* d_out = nullptr;
    size_t out_cap = 0;
    // last render
    RenderParams rp{};
    bool rendered = false;
    std::atomic<int> cancel{0};
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
    s.lights = c->d_lights;
    s.camera = c->d_camera;
    s.film = c->d_film;
    s.dist = with_dist ? c->d_dist : nullptr;
    s.n_prims = c->host_scene.n_prims;
    s.n_nodes = c->host_scene.n_nodes;
    s.n_lights = c->host_scene.n_lights;
    s.pad = 0;
    return s;
}

int validate_scene(const pbrt_scene_desc* s) {
    if (!s) return PBRT_E_INVALID;
    if (s->n_prims < 0 || s->n_nodes < 0 || s->n_lights < 0 || s->n_shapes < 0 || s->n_materials < 0)
        return PBRT_E_INVALID;
    if (s->n_nodes > 65535) return PBRT_E_UNSUPPORTED;   // uint16 LDS stack entries
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

// Can k_render_spec replay this render exactly? (see pbrt_spec.h for the conditions)
bool spec_layout(const pbrt_gpu_ctx* c, const pbrt_render_desc* rd, const RenderParams& rp, SpecLayout& L) {
    if (rd->integrator != PBRT_INTEGRATOR_PATH || rd->n_dims < 3) return false;
    const int nl = c->host_scene.n_lights;
    if (nl > kMaxCachedLights) return false;
    if (nl > 0) {
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
    L.film = put(rp.slot_w * rp.slot_h * 3 * 8);
    L.s1d = put(nd * n * 8);
    L.other = put(nd * n * 2);
    L.memb = put(n * 8);
    L.lbuf = put(kWave * 3 * 8);
    L.sbuf = put(kWave * 8);
    L.dbuf = put(kWave * 4);
    L.pbuf = put(kWave * 2 * 4);
    const int64_t s1 = rd->jitter ? 2 * n : n, s2 = rd->jitter ? 3 * n : n;
    const int64_t E = nd * (s1 + s2), V = E + 64 + E / 8;
    const bool buffered = V * 4 <= 16 * 1024;
    L.vbuf = put(buffered ? V * 4 : 4);
    L.total = (int)off;
    return off <= 48 * 1024;
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
    if (rd->mode != PBRT_MODE_EXACT) return set_err(c, PBRT_E_UNSUPPORTED, "only EXACT mode is implemented");
    const pbrt_film_desc& f = c->host_scene.film;
    if (f.filter_radius_x <= 0 || f.filter_radius_y <= 0 || f.filter_radius_x >= (double)rd->tile_size ||
        f.filter_radius_y >= (double)rd->tile_size)
        return set_err(c, PBRT_E_UNSUPPORTED, "filter radius must be in (0, tile_size)");
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
    pbrt_distribution_desc& dist = c->host_dist;
    std::memset(&dist, 0, sizeof(dist));
    if (rd->integrator == PBRT_INTEGRATOR_PATH) {
        int rc = pbrt_scene_light_distribution(&c->host_scene, rd->light_strategy, &dist);
        if (rc != PBRT_OK) return set_err(c, rc, "unsupported light sample strategy");
        HIPCHK(c, hipMemcpyAsync(c->d_dist, &dist, sizeof(dist), hipMemcpyHostToDevice, c->stream));
    }
    c->use_spec = c->kernel_req != PBRT_KERNEL_SERIAL && spec_layout(c, rd, rp, c->lay);
    {
        const int64_t n = rp.spp, s1 = rp.jitter ? 2 * n : n, s2 = rp.jitter ? 3 * n : n;
        const int64_t E = (int64_t)rp.ndims * (s1 + s2), V = E + 64 + E / 8;
        rp.sp_events = (int32_t)E;
        rp.sp_draws = (int32_t)V;
        rp.sp_serial = V * 4 <= 16 * 1024 ? 0 : 1;
    }
    if (c->kernel_req == PBRT_KERNEL_WAVE && !c->use_spec)
        return set_err(c, PBRT_E_UNSUPPORTED, "render not eligible for the wave-parallel kernel");
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
    c->device = (opts && opts->device >= 0) ? opts->device : -1;
    if (opts && opts->lanes_per_wave > 0 && opts->lanes_per_wave <= 64) c->lanes_per_wave = opts->lanes_per_wave;
    if (opts && (opts->occupancy == 2 || opts->occupancy == 4 || opts->occupancy == 8)) c->min_waves = opts->occupancy;
    if (opts && (opts->kernel < PBRT_KERNEL_AUTO || opts->kernel > PBRT_KERNEL_WAVE)) {
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
    c->host_scene = *scene;
    c->host_scene.shapes = nullptr;
    c->host_scene.materials = nullptr;
    c->host_scene.prims = nullptr;
    c->host_scene.nodes = nullptr;
    c->host_lights.assign(scene->lights, scene->lights + scene->n_lights);
    c->host_scene.lights = c->host_lights.data();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess) {
        pbrt_gpu_destroy(c);
        return PBRT_E_HIP;
    }
    if ((rc = upload(c, &c->d_shapes, scene->shapes, scene->n_shapes)) ||
        (rc = upload(c, &c->d_materials, scene->materials, scene->n_materials)) ||
        (rc = upload(c, &c->d_prims, scene->prims, scene->n_prims)) ||
        (rc = upload(c, &c->d_nodes, scene->nodes, scene->n_nodes)) ||
        (rc = upload(c, &c->d_lights, scene->lights, scene->n_lights)) ||
        (rc = upload(c, &c->d_camera, &scene->camera, 1)) || (rc = upload(c, &c->d_film, &scene->film, 1)) ||
        (rc = upload<pbrt_distribution_desc>(c, &c->d_dist, nullptr, 1)) ||
        (rc = upload<Counters>(c, &c->d_ctr, nullptr, 1)) ||
        (rc = upload<PcgJump>(c, &c->d_jump, &pcg_jump_table(), 1))) {
        pbrt_gpu_destroy(c);
        return rc;
    }
    *out = c;
    return PBRT_OK;
}

int pbrt_gpu_render_async_into(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_device) {
    if (!c) return PBRT_E_INVALID;
    if (c->cancel.load()) return set_err(c, PBRT_E_CANCELLED, "cancelled");
    HIPCHK(c, hipSetDevice(c->device));
    c->t_start = std::chrono::steady_clock::now();
    int rc = prepare(c, rd);
    if (rc != PBRT_OK) return rc;
    const RenderParams& rp = c->rp;
    double* out = film_device ? film_device : c->d_out;
    c->film_target = out;
    HIPCHK(c, hipMemsetAsync(c->d_ctr, 0, sizeof(Counters), c->stream));
    if (rp.n_slots > 0) HIPCHK(c, hipMemsetAsync(c->d_panics, 0, sizeof(PanicRec) * (size_t)rp.n_slots, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if (rp.n_slots > 0) {
        DevScene sc = dev_scene(c, rd->integrator == PBRT_INTEGRATOR_PATH);
        if (c->use_spec) {
            c->last_kernel = PBRT_KERNEL_WAVE;
            auto kern = c->min_waves >= 2 ? k_render_spec<2> : k_render_spec<1>;
            hipLaunchKernelGGL(kern, dim3((unsigned)rp.n_slots), dim3(kWave), (unsigned)c->lay.total,
                               c->stream, sc, rp, c->lay, c->d_jump, c->d_films, c->d_panics, c->d_ctr);
        } else {
            c->last_kernel = PBRT_KERNEL_SERIAL;
            int64_t blocks = (rp.n_slots + rp.lanes_per_wave - 1) / rp.lanes_per_wave;
            auto kern = k_render_exact<1>;
            if (c->min_waves == 2) kern = k_render_exact<2>;
            else if (c->min_waves == 4) kern = k_render_exact<4>;
            else if (c->min_waves == 8) kern = k_render_exact<8>;
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kWave), 0, c->stream, sc, rp, c->d_films,
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
    HIPCHK(c, hipStreamSynchronize(c->stream));
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
            rc = set_err(c, PBRT_E_UNSUPPORTED, "material not on the hot path (OrenNayar)");
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
        hipLaunchKernelGGL(k_intersect, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave), 0, c->stream, sc,
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
    if (c) c->cancel.store(1);
}
const char* pbrt_gpu_last_error(const pbrt_gpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

void pbrt_gpu_destroy(pbrt_gpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->d_shapes, c->d_materials, c->d_prims, c->d_nodes, c->d_lights, c->d_camera, c->d_film,
                    c->d_dist,   c->d_films,     c->d_s1d,   c->d_panics, c->d_ctr,   c->d_out,    c->d_jump};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->stream) (void)hipStreamDestroy(c->stream);
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
    for (int i = 0; i < n && i < kNumCounters; i++) out[i] = v[i];
    return kNumCounters;
}

extern "C" int pbrt_abi_sizes(size_t* out, int n) {
    const size_t s[] = {sizeof(pbrt_matrix4x4),   sizeof(pbrt_transform),    sizeof(pbrt_shape_desc),
                        sizeof(pbrt_material_desc), sizeof(pbrt_primitive_desc), sizeof(pbrt_bvh_node),
                        sizeof(pbrt_light_desc),  sizeof(pbrt_camera_desc),  sizeof(pbrt_film_desc),
                        sizeof(pbrt_distribution_desc), sizeof(pbrt_scene_desc), sizeof(pbrt_render_desc),
                        sizeof(pbrt_gpu_stats),   sizeof(pbrt_ray_soa),      sizeof(pbrt_hit_soa),
                        sizeof(pbrt_gpu_opts)};
    int m = (int)(sizeof(s) / sizeof(s[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = s[i];
    return m;
}
