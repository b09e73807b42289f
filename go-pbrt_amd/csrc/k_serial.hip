// k_serial.hip — k_render_exact, the one-lane-per-tile EXACT kernel
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

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

template __global__ void k_render_exact<1>(DevScene sc, RenderParams rp, double* __restrict__ films, double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);
template __global__ void k_render_exact<2>(DevScene sc, RenderParams rp, double* __restrict__ films, double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);
template __global__ void k_render_exact<4>(DevScene sc, RenderParams rp, double* __restrict__ films, double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);
template __global__ void k_render_exact<8>(DevScene sc, RenderParams rp, double* __restrict__ films, double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);

}  // namespace pbrtk
