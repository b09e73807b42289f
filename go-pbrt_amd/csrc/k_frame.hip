// k_frame.hip — bounce-1 records, DirectLighting, tile cost probe, film kernels, batch intersect
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

// One workgroup per tile slot: the tile film of the serial replay
// (FilmTile.AddSample, film.go:211-248; integrator.go:256-262). Each film
// pixel's value is the sum, in the reference's order, of its source pixels
// (row-major) and of each source's samples (in order): one sequential chain
// per film pixel and channel, which no reassociation may shorten.
//
// The tile's source pixels stream through LDS in row-major runs of S pixels
// (S x (spp - 1) samples of L, S = the run that fits kFilmStageBytes: a whole
// 16-px row at 64 spp, one pixel at 1024 spp), each run read from HBM once,
// with contiguous loads (pixel-major L). A film pixel's thread adds the run's
// sources whose footprint holds it, in order; since every film pixel sees its
// sources in the global row-major order, every chain keeps the reference's
// order for any filter radius (< tile size; footprints of up to
// (2 floor(r + 0.5))^2 film pixels, the reference's BoxFilter of radius 1.5
// included). The footprint test and weight are film.go's own arithmetic
// (render_common.h footprint()). The running sums live in LDS, one per film
// pixel and channel. The workgroup also adds up its pixels' reference ray
// counts (pbrt_gpu_stats.rays_*).
__device__ __forceinline__ bool film_weight(const pbrt_film_desc& f, double ifx, double ify, int64_t sx, int64_t sy,
                                            int64_t fx, int64_t fy, double& w) {
    // film.go:216-246 with pFilm = the source pixel's corner (2D stratified values are (0,0), #3);
    // the tile-film clip [px0, px1) holds for every film pixel of the slot
    const double dx = (double)sx + 0.0 - 0.5, dy = (double)sy + 0.0 - 0.5;
    const double p0x = gomath::ceil(dx - f.filter_radius_x), p0y = gomath::ceil(dy - f.filter_radius_y);
    const double p1x = gomath::floor(dx + f.filter_radius_x) + 1, p1y = gomath::floor(dy + f.filter_radius_y) + 1;
    if (!((double)fx >= p0x && (double)fx < p1x && (double)fy >= p0y && (double)fy < p1y)) return false;
    const int iy = (int)gomath::to_int(gomath::min(gomath::floor(gomath::abs(((double)fy - dy) * ify * 16.0)), 16.0 - 1));
    const int ix = (int)gomath::to_int(gomath::min(gomath::floor(gomath::abs(((double)fx - dx) * ifx * 16.0)), 16.0 - 1));
    w = 1.0 * f.filter_table[iy * 16 + ix];
    return true;
}

constexpr int kFilmLoads = 12;   // k_film staging: loads in flight per thread

__global__ __launch_bounds__(kFilmThreads) void k_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp,
                                                       WaveBufs wb, int64_t slot_base, int64_t nslots_batch,
                                                       double* __restrict__ films, const int* __restrict__ cancel_seen,
                                                       Counters* __restrict__ ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int nvs[kFilmThreads];   // nvalid of the run's pixels (0: no record)
    // a cancelled render's samples are incomplete: its film is not valid (pbrt_gpu_cancel)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(cancel_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
        return;
    const int64_t bslot = blockIdx.x;
    if (bslot >= nslots_batch) return;
    const int tid = threadIdx.x;
    const pbrt_film_desc& film = *film_desc;
    const int64_t slot = slot_base + bslot;
    int64_t x0, y0, x1, y1, px0, py0, px1, py1;
    tile_bounds(rp, tile_of_slot(rp, slot), x0, y0, x1, y1);
    film_tile_bounds(film, x0, y0, x1, y1, px0, py0, px1, py1);
    const int tw = (int)(px1 - px0), nfp = (int)(tw * (py1 - py0));
    const int sw = (int)(x1 - x0);
    const int n = rp.spp, m = n - 1;   // traced samples 1 .. n-1
    const int npx = wb.tile_npx[bslot];
    const int S = film_run_pixels(rp);
    // a source pixel reaches film pixels within (int)r + 2 of it (footprint: |f - s| < r + 1.5)
    const double ifx = 1.0 / film.filter_radius_x, ify = 1.0 / film.filter_radius_y;   // film.go:231-232
    // a source pixel's footprint relative to it, [fa, fb) x [ga, gb) (film.go:216-219 with
    // pFilm = the pixel corner); the work items cover it widened by one, the exact test is film_weight
    const int fa = (int)gomath::ceil(-0.5 - film.filter_radius_x), fb = (int)gomath::floor(film.filter_radius_x - 0.5) + 1;
    const int ga = (int)gomath::ceil(-0.5 - film.filter_radius_y), gb = (int)gomath::floor(film.filter_radius_y - 0.5) + 1;
    // LDS: running sums [nfp][3], then the staged run [S][m][3]
    double* acc = (double*)lds;
    double* stg = acc + ((nfp * 3 + 1) & ~1);
    for (int i = tid; i < nfp * 3; i += kFilmThreads) acc[i] = 0.0;
    const int64_t rec0 = bslot * wb.ppt;
    unsigned long long cl = 0, sh = 0;
    for (int s0 = 0; s0 < npx && m > 0; s0 += S) {
        const int ns = min(S, npx - s0);
        __syncthreads();   // the previous run is consumed
        if (tid < ns) nvs[tid] = wb.prec[rec0 + s0 + tid].nvalid;
        __syncthreads();
        // stage the run's samples 1 .. nvalid-1: one contiguous stretch of L but
        // for each pixel's sample 0 (pixel-major); the ray counts on the way.
        // kFilmLoads loads per thread are in flight at once (a whole 16-px row
        // at 64 spp in one round): the HBM latency is paid once per run
        const double* Lrun = wb.L + (rec0 + s0) * (int64_t)n * 3;
        const int tot = ns * m * 3;
        for (int i0 = tid; i0 < tot; i0 += kFilmThreads * kFilmLoads) {
            double v[kFilmLoads];
#pragma unroll
            for (int u = 0; u < kFilmLoads; u++) {
                const int i = i0 + u * kFilmThreads;
                v[u] = 0.0;
                if (i < tot) {
                    const int s = i / (m * 3), j = i - s * (m * 3);
                    if (j / 3 < nvs[s] - 1) v[u] = Lrun[(int64_t)s * n * 3 + 3 + j];
                }
            }
#pragma unroll
            for (int u = 0; u < kFilmLoads; u++)
                if (i0 + u * kFilmThreads < tot) stg[i0 + u * kFilmThreads] = v[u];
        }
        for (int i0 = tid; i0 < ns * m; i0 += kFilmThreads * 4) {
            uint32_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * kFilmThreads, s = i / m, k = i - s * m;
                v[u] = (i < ns * m && k < nvs[s] - 1) ? wb.rays[(rec0 + s0 + s) * n + 1 + k] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                cl += v[u] & 0xFFFFu;
                sh += v[u] >> 16;
            }
        }
        __syncthreads();
        // NaN guard and luminance clamp per sample (integrator.go:256-262)
        for (int i = tid; i < ns * m; i += kFilmThreads) {
            const int s = i / m, k = i - s * m;
            if (k >= nvs[s] - 1) continue;
            double* d = stg + (int64_t)i * 3;
            Spec Ls{d[0], d[1], d[2]};
            const bool nan = has_nans(Ls);
            if (nan) Ls = spec(0.1);
            if (0.0 > film.max_sample_luminance) Ls = smuls(Ls, film.max_sample_luminance / 0.0);
            if (nan || 0.0 > film.max_sample_luminance) {
                d[0] = Ls.r;
                d[1] = Ls.g;
                d[2] = Ls.b;
            }
        }
        __syncthreads();
        // the film pixels the run can reach (a source pixel's footprint spans
        // [sx + fa, sx + fb), widened by one), one work item per (film pixel,
        // channel): each adds the run's sources that reach it, in order -- the
        // sources in the window its footprint allows, row-major, each checked
        // with film.go's own test (film_weight)
        const int sy0 = s0 / sw, sy1 = (s0 + ns - 1) / sw;   // the run's source rows (tile-relative)
        const int sxa = s0 - sy0 * sw, sxb = s0 + ns - 1 - sy1 * sw;   // first row from sxa, last row to sxb
        const int sxl = sy0 == sy1 ? sxa : 0, sxh = sy0 == sy1 ? sxb : sw - 1;
        const int fxl = max((int)x0 + sxl + fa - 1, (int)px0) - (int)px0;
        const int fxh = min((int)x0 + sxh + fb, (int)px1 - 1) - (int)px0;
        const int fyl = max((int)y0 + sy0 + ga - 1, (int)py0) - (int)py0;
        const int fyh = min((int)y0 + sy1 + gb, (int)py1 - 1) - (int)py0;
        const int nfx = fxh - fxl + 1, nit = nfx > 0 && fyh >= fyl ? nfx * (fyh - fyl + 1) * 3 : 0;
        for (int it = tid; it < nit; it += kFilmThreads) {
            const int f = it / 3, ch = it - f * 3;
            const int fr = f / nfx, fcol = fxl + (f - fr * nfx), frow = fyl + fr;
            const int fi = frow * tw + fcol;
            const int64_t fx = px0 + fcol, fy = py0 + frow;
            // candidate sources (tile-relative): rows (fy - gb, fy - ga], columns (fx - fb, fx - fa], widened by one
            const int ry0 = max(sy0, (int)(fy - y0) - gb), ry1 = min(sy1, (int)(fy - y0) - ga + 1);
            const int cx0 = (int)(fx - x0) - fb, cx1 = (int)(fx - x0) - fa + 1;
            double a = 0;
            bool any = false;
            for (int sy = ry0; sy <= ry1; sy++) {
                const int lo = max(cx0, sy == sy0 ? sxa : 0), hi = min(cx1, sy == sy1 ? sxb : sw - 1);
                for (int sx = lo; sx <= hi; sx++) {
                    double w;
                    if (!film_weight(film, ifx, ify, x0 + sx, y0 + sy, fx, fy, w)) continue;
                    const int s = sy * sw + sx - s0;
                    if (!any) {
                        a = acc[fi * 3 + ch];
                        any = true;
                    }
                    // the chain of adds is sequential; the LDS loads run 8 samples ahead
                    const int nk = nvs[s] - 1;
                    const double* d = stg + (int64_t)s * m * 3 + ch;
                    int k = 0;
                    for (; k + 8 <= nk; k += 8) {
                        double v[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) v[u] = d[(k + u) * 3];
#pragma unroll
                        for (int u = 0; u < 8; u++) a += v[u] * w;
                    }
                    for (; k < nk; k++) a += d[k * 3] * w;
                }
            }
            if (any) acc[fi * 3 + ch] = a;
        }
    }
    __syncthreads();
    double* tf = films + slot * rp.slot_w * rp.slot_h * 3;
    for (int i = tid; i < nfp * 3; i += kFilmThreads) tf[i] = acc[i];
    for (int off = kWave / 2; off > 0; off >>= 1) {
        cl += __shfl_down(cl, off);
        sh += __shfl_down(sh, off);
    }
    if ((tid & (kWave - 1)) == 0 && (cl | sh)) {
        atomicAdd(&ctr->closest_rays, cl);
        atomicAdd(&ctr->shadow_rays, sh);
    }
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


template <bool kX>
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
    const bool dl = rp.integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING;
    if (rp.spp > 1 && (1 < rp.max_depth || dl)) {
        hit0 = bvh_traverse<false>(sc, ray, &si0, stack_lds + threadIdx.x, panic0) ? 1 : 0;
        // DirectLighting asks for one lobe per BxDF (directlighting.go:76)
        if (!panic0 && hit0 && (kX ? compute_bsdf_x(sc, si0, b0, bx0, !dl) : compute_bsdf(sc, si0, b0)) < 0)
            panic0 = -1;
    }
    // DirectLighting's recursion chain (dl_chain_draws): SpecularTransmit's
    // direction reads no sample, so the levels it reaches are the pixel's
    int levels = (hit0 && !panic0) ? 1 : 0;
    if (kX && dl && levels) {
        SI si = si0;
        BSDF b = b0;
        BSDFX x = bx0;
        for (int depth = 0; depth + 1 < rp.max_depth && levels <= kDlMaxLevels; depth += 2) {
            V3 wi;
            double pdf;
            const Spec f = spec_trans_sample(b, x, si.wo, V2{0.0, 0.0}, wi, pdf);
            if (!(pdf > 0 && !is_black(f) && absdot(wi, si.sn) != 0.0)) break;
            Ray r{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf, si.time};   // local-frame wi (#7)
            int pn = 0;
            // a miss ends the chain; a panic ends the tile at that sample either way
            if (!bvh_traverse<false>(sc, r, &si, stack_lds + threadIdx.x, pn) || pn) break;
            if (compute_bsdf_x(sc, si, b, x, false) < 0) break;
            levels++;
        }
    }
    PixelRec& pr = wb.prec[rec];
    pr.dl_levels = levels;
    pr.si = si0;
    pr.b = b0;
    if constexpr (kX) pr.x = bx0;
    pr.wo = ray.d;
    pr.hit = panic0 ? 0 : hit0;
    pr.panic0 = panic0;
    pr.nvalid = rp.spp;
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
        const uint64_t D = dl_chain_draws(rp, hit ? pr.dl_levels : 0, sc.n_lights);
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
// kX (Mirror / smooth Glass / OrenNayar scenes): DirectLighting.Li's whole
// recursion per sample (directlighting.go:62-104, integrator.go:352-422), as the
// serial kernel's direct_li folds it: SpecularReflect matches no lobe of these
// materials, SpecularTransmit refracts through smooth glass (local-frame wi,
// #7) into Li at depth + 2 (#23). A panic's bounce is that level's depth + 1.
template <bool kX>
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
        double* o = wb.L + sample_index(wb, rec, n, k) * 3;
        Spec L = spec(0);
        int panic = pr.panic0;
        int bounce = 1;
        uint64_t shadow = 0;   // visibility rays traced (the camera ray's query is counted below)
        uint32_t closest = 1;
        if (kX && !panic && pr.hit) {
            Cursor c;
            c.rri = -1;
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
            Spec own[kDlMaxLevels], fk[kDlMaxLevels];
            double wk[kDlMaxLevels];
            int levels = 0;
            SI si = pr.si;
            BSDF b = pr.b;
            BSDFX x = pr.x;
            Ray ray;
            uint16_t* stack = stack_lds + threadIdx.x;
            for (int depth = 0;; depth += 2) {
                L = spec(0);
                bounce = depth + 1;
                if (depth > 0) {   // the refracted ray of the level above (level 0: the pixel record)
                    closest++;
                    if (!bvh_traverse<false>(sc, ray, &si, stack, panic)) {
                        for (int i = 0; i < sc.n_lights; i++) L = L + spec(0);
                        break;
                    }
                    if (panic) break;
                    if (compute_bsdf_x(sc, si, b, x, false) < 0) {
                        panic = -1;
                        break;
                    }
                }
                L = L + spec(0);   // si.Le(si.Wo): no primitive carries an area light
                const int nl = sc.n_lights;
                if (nl > 0) {
                    if (rp.dl_strategy == PBRT_DL_UNIFORM_SAMPLE_ALL) {   // integrator.go:23-46
                        Spec acc = spec(0);
                        for (int j = 0; j < nl && !panic; j++) {
                            const V2 ul = c_get2d(c, ss);
                            c_get2d(c, ss);
                            acc = acc + estimate_direct_x(sc, stack, panic, si, b, x, j, ul, &shadow);
                        }
                        if (panic) break;
                        L = L + acc;
                    } else {   // UniformSampleOneLight with no distribution (integrator.go:48-77)
                        const int ln = (int)gomath::to_int(gomath::min(c_get1d(c, ss) * (double)nl, (double)(nl - 1)));
                        const V2 ul = c_get2d(c, ss);
                        c_get2d(c, ss);
                        const Spec s1 = estimate_direct_x(sc, stack, panic, si, b, x, ln, ul, &shadow);
                        if (!panic && max_component(s1) > 10) panic = PBRT_PANIC_LD_GT_10;
                        if (panic) break;
                        L = L + s1;
                    }
                }
                if (!(depth + 1 < rp.max_depth)) break;
                c_get2d(c, ss);   // SpecularReflect (integrator.go:352-355): black
                L = L + spec(0);
                const V2 u = c_get2d(c, ss);   // SpecularTransmit (integrator.go:383-385)
                V3 wi;
                double pdf;
                const Spec f = spec_trans_sample(b, x, si.wo, u, wi, pdf);
                const double adn = absdot(wi, si.sn);
                if (!(pdf > 0 && !is_black(f) && adn != 0.0) || levels == kDlMaxLevels) {
                    L = L + spec(0);
                    break;
                }
                own[levels] = L;
                fk[levels] = f;
                wk[levels] = adn / pdf;
                levels++;
                ray.o = offset_ray_origin(si.p, si.perr, si.n, wi);   // SpawnRay with the local-frame wi
                ray.d = wi;
                ray.tmax = kInf;
                ray.time = si.time;
            }
            if (!panic)
                for (int q = levels - 1; q >= 0; q--) L = own[q] + smuls(smul(fk[q], L), wk[q]);
        } else if (!panic && pr.hit) {
            Cursor c;
            c.rri = -1;
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
        wb.rays[sample_index(wb, rec, n, k)] = closest * kRayClosest + (uint32_t)shadow * kRayShadow;
        if (panic)   // key: sample << 32 | bounce << 8 | kind + 1 (the first panic in sample order wins)
            atomicMin((unsigned long long*)&wb.memb[rec * n],
                      ((unsigned long long)k << 32) | ((unsigned long long)(bounce & 0xFFFFFF) << 8) |
                          (unsigned long long)((panic + 1) & 0xFF));

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
        p.bounce = (int)((key >> 8) & 0xFFFFFF);
    }
    wb.ppanic[rec] = p;
    if (!p.kind && rp.spp > 1) {
        atomicAdd(&ctr->paths, (unsigned long long)(rp.spp - 1));
        atomicAdd(&ctr->camera_samples, (unsigned long long)(rp.spp - 1));
    }
}

template <bool kX>
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
        c.rri = -1;
        c.rng.state = mb_state((uint64_t)tile, (uint64_t)pi, 0x70726f6265ULL + (uint64_t)(it % kProbes));
        c.rng.inc = inc;
        c.draws = 0;
        c_camera(c, rp.ndims);
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

// One wave that holds its stream's next launch back until the chain stage's
// progress record (k_chain_ci's `prog`, layout at kProgHead) allows it (the
// completion-driven path stage, render.hip):
//   b == e: until at least `b` chain workgroups have started (every one of them
//           has been dispatched);
//   b <  e: until the completion list's entries [b, e) are all written (those
//           tiles' chains have ended and their records are visible).
// Progress-driven, not timed: the chains waited for are queued before the gate
// and always run to their end (a cancelled chain ends early, but ends). The wait
// needs the chains to run beside it, which a dispatcher that serialises kernels
// across streams does not allow (rocprofv3 counter collection does: measured,
// DESIGN §3.3); there no chain starts a pixel and the record stands still. So
// 1 s in which no workgroup starts, no pixel starts and no listed tile ends
// ends the wait and flags the frame (Counters.gate_stall; every later gate of
// the frame then opens at once), and the host renders the frame again with the
// path stage after the chains (pbrt_gpu_synchronize). A running frame starts a
// pixel every few microseconds (config B: ~522k pixels in ~300 ms).
__global__ __launch_bounds__(kWave) void k_gate(const uint32_t* __restrict__ prog, uint32_t b, uint32_t e,
                                                Counters* __restrict__ ctr) {
    const int lane = threadIdx.x;
    uint32_t cur = b == e ? 0u : b;   // b < e: entries before cur are known written
    uint32_t seen = 0xFFFFFFFFu;
    uint64_t t_prog = wall_clock64();
    for (;;) {
        if (__hip_atomic_load(&ctr->gate_stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        const uint32_t started = __hip_atomic_load(&prog[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (b == e) {
            if (started >= b) return;
        } else {
            for (;;) {   // advance over written entries, 64 at a time
                const uint32_t i = cur + (uint32_t)lane;
                const bool ok = i >= e || __hip_atomic_load(&prog[kProgHead + i], __ATOMIC_ACQUIRE,
                                                            __HIP_MEMORY_SCOPE_AGENT) != kNoSlot;
                const unsigned long long bad = __ballot(!ok);
                if (bad) {
                    cur += (uint32_t)__builtin_ctzll(bad);
                    break;
                }
                cur += kWave;
                if (cur >= e) return;
            }
        }
        const uint32_t v = started + cur + __hip_atomic_load(&prog[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t now = wall_clock64();
        if (v != seen) {
            seen = v;
            t_prog = now;
        } else if (now - t_prog > 100000000ull) {   // 1 s at 100 MHz without progress
            if (lane == 0) atomicExch(&ctr->gate_stall, 1);
            return;
        }
        __builtin_amdgcn_s_sleep(32);
    }
}

__global__ void k_order_of_keys(const uint64_t* __restrict__ keys, int64_t nb, uint32_t* __restrict__ order) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) order[i] = (uint32_t)keys[i];
}

// ---------------------------------------------------------- merge kernel
// Film.MergeFilmTile (film.go:115-132) in tile-index order. A film pixel is
// covered by at most the 3x3 tiles around its own (filter radius < tile size).
__global__ __launch_bounds__(256) void k_merge_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp,
                                                    const double* __restrict__ films, double* __restrict__ out,
                                                    const int* __restrict__ cancel_seen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rp.film_w * rp.film_h) return;
    // a cancelled frame's tile films are partial (or the previous frame's):
    // leave the caller's buffer as it is (pbrt_gpu.h: undefined after a cancel)
    if (__atomic_load_n(cancel_seen, __ATOMIC_RELAXED)) return;
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

template __global__ void k_dl_samples<false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec);
template __global__ void k_dl_samples<true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec);
template __global__ void k_wf_primary<false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb);
template __global__ void k_wf_primary<true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb);
template __global__ void k_tile_cost<false>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb, float* __restrict__ feat, uint64_t* __restrict__ keys);
template __global__ void k_tile_cost<true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb, float* __restrict__ feat, uint64_t* __restrict__ keys);

}  // namespace pbrtk
