// k_chain_1.hip — k_chain_ci instantiations: one wave per tile (Matte)
#pragma clang fp contract(off)

#include "render_common.h"
#include "k_chain.h"

namespace pbrtk {

template __global__ void k_chain_ci<1, 0, false, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<1, 0, false, 2, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<1, 64, false, 2, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<1, 64, false, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);

// the windowed StartPixel (rp.sp_window: config C)
template __global__ void k_chain_ci<1, 0, false, 0, true>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<1, 0, false, 2, true>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);

template __global__ void k_chain_ci<1, -1, false, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);

}  // namespace pbrtk
