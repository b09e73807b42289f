// k_chain_x.hip — k_chain_ci instantiations over BSDFX (Mirror, Glass, OrenNayar)
#pragma clang fp contract(off)

#include "render_common.h"
#include "k_chain.h"

namespace pbrtk {

template __global__ void k_chain_ci<1, 0, true, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<2, 0, true, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);
template __global__ void k_chain_ci<4, 0, true, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride, uint32_t* __restrict__ prog);

}  // namespace pbrtk
