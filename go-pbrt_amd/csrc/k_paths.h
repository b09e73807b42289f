// k_paths.h — k_paths_ci (full paths with lane refill) and k_mb_setup (THROUGHPUT setup); instantiated in k_paths_*.hip
#pragma once
#pragma clang fp contract(off)

#include "render_common.h"

namespace pbrtk {

template <int P, bool kMB, bool kX>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kPathsWaves, 8))) void k_paths_ci(
    DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr,
    int s1d_lds, const uint32_t* __restrict__ order) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];   // paths_group_lds<P>
    if (cancel_requested(sc, (blockIdx.x & 63) == 0)) return;   // one wave per workgroup
    stage_nodes(sc);
    int64_t rec0 = (int64_t)blockIdx.x * P, rec_end = nrec;
    if (order) {   // the launch covers the slots order[0 .. nrec / ppt), ceil(ppt / P) workgroups per slot
        const int64_t gps = (wb.ppt + P - 1) / P;
        const uint32_t o = order[blockIdx.x / gps];
        if (o == kNoSlot) return;   // an unwritten completion entry (only after a k_gate stall)
        const int64_t slot = (int64_t)o;
        rec0 = slot * wb.ppt + (int64_t)(blockIdx.x % gps) * P;
        rec_end = (slot + 1) * wb.ppt;
    }
    paths_group<P, kMB, kX>(sc, rp, wb, slot_base, rec0, rec_end, ctr, lds, s1d_lds);
}

// THROUGHPUT mode setup for k_paths_ci<P, true>, one wave per pixel record:
// StartPixel on the pixel's own stream mb_state(tile, pi, 0) and bounce 1
// (camera ray, first hit, BSDF), written to the PixelRec / s1d buffers the
// EXACT pipeline fills with k_wf_primary + k_chain_ci. The same arithmetic as
// the serial kernel's pixel prologue.
template <bool kX>
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

}  // namespace pbrtk
