// render_kernels.h — declarations of the kernels, for the host code of render.hip.
// Each kernel is defined (and its template instantiations made) in its own
// translation unit; the launch goes through the host stub that unit emits.
#pragma once

#include "render_common.h"

namespace pbrtk {

template <int kMinWaves>
__global__ void k_render_exact(DevScene sc, RenderParams rp, double* __restrict__ films, double* __restrict__ s1d_scratch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);
template <int P, bool kMB = false, bool kX = false>
__global__ void k_paths_ci(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr, int s1d_lds, const uint32_t* __restrict__ order);
template <bool kX = false>
__global__ void k_pw_cache(DevScene sc, WaveBufs wb, int64_t rec0, int64_t nrec, Spec* __restrict__ ldc, int* __restrict__ ldp);
template <bool kMB, bool kX = false>
__global__ void k_pw_start(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const Spec* __restrict__ ldc, const int* __restrict__ ldp, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
template <bool kMeshOnly = false>
__global__ void k_pw_trace(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, int cin, int n_keys, unsigned long long* __restrict__ pkey);
__global__ void k_pw_scan(PwQueues qs, int n_keys);
__global__ void k_pw_scatter(const PwPath* __restrict__ paths, PwQueues qs);
template <bool kX = false>
__global__ void k_pw_shade(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, PwPath* __restrict__ paths, PwQueues qs, int sorted, unsigned long long* __restrict__ pkey);
template <bool kMeshOnly = false>
__global__ void k_pw_shadow(DevScene sc, RenderParams rp, WaveBufs wb, PwPath* __restrict__ paths, PwQueues qs, unsigned long long* __restrict__ pkey);
__global__ void k_pw_panics(RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t rec0, int64_t nrec, const unsigned long long* __restrict__ pkey, Counters* __restrict__ ctr);
template <bool kX = false>
__global__ void k_mb_setup(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch);
__global__ void k_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, double* __restrict__ films, const int* __restrict__ cancel_seen, Counters* __restrict__ ctr);
__global__ void k_panic_reduce(WaveBufs wb, int64_t slot_base, int64_t nslots_batch, PanicRec* __restrict__ panics, Counters* __restrict__ ctr);
template <bool kX = false>
__global__ void k_wf_primary(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb);
__global__ void k_dl_setup(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nb);
template <bool kX = false>
__global__ void k_dl_samples(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec);
__global__ void k_dl_panics(RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr);
template <bool kX = false>
__global__ void k_tile_cost(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nb, float* __restrict__ feat, uint64_t* __restrict__ keys);
__global__ void k_order_of_keys(const uint64_t* __restrict__ keys, int64_t nb, uint32_t* __restrict__ order);
__global__ void k_gate(const uint32_t* __restrict__ prog, uint32_t b, uint32_t e, Counters* __restrict__ ctr);
template <int kW, int kDepth = 0, bool kX = false, int kEu = 0, bool kSpWin = false>
__global__ void k_chain_ci(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
__global__ void k_merge_film(const pbrt_film_desc* __restrict__ film_desc, RenderParams rp, const double* __restrict__ films, double* __restrict__ out, const int* __restrict__ cancel_seen);
__global__ void k_intersect(DevScene sc, int64_t n, const double* __restrict__ rays, double* __restrict__ out, int any_hit);

}  // namespace pbrtk
