// k_chain_a.hip — k_chain_async and k_chain_mc instantiations (asynchronous waves; 2, 4, 8 waves per tile, Matte)
#pragma clang fp contract(off)

#include "render_common.h"
#include "k_chain_async.h"
#include "k_chain_mc.h"

namespace pbrtk {

template __global__ void k_chain_async<2, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<4, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<8, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<2, 64, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<4, 64, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<8, 64, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<2, -1, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<4, -1, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);
template __global__ void k_chain_async<8, -1, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, int lanes_per_tile, int ring_size, Counters* __restrict__ ctr, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks, int cstride);

template __global__ void k_chain_mc<4, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);
template __global__ void k_chain_mc<8, 0, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);
template __global__ void k_chain_mc<4, 64, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);
template __global__ void k_chain_mc<8, 64, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);
template __global__ void k_chain_mc<4, -1, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);
template __global__ void k_chain_mc<8, -1, false>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch, McTile* __restrict__ tiles, unsigned long long* __restrict__ rings, int ring_size, int M, const uint32_t* __restrict__ order, uint32_t* __restrict__ ticks);

}  // namespace pbrtk
