// k_paths_x.hip — k_paths_ci / k_mb_setup instantiations over BSDFX
#pragma clang fp contract(off)

#include "render_common.h"
#include "k_paths.h"

namespace pbrtk {

template __global__ void k_paths_ci<4, false, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr, int s1d_lds, const uint32_t* __restrict__ order);
template __global__ void k_paths_ci<8, false, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr, int s1d_lds, const uint32_t* __restrict__ order);
template __global__ void k_paths_ci<4, true, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr, int s1d_lds, const uint32_t* __restrict__ order);
template __global__ void k_paths_ci<8, true, true>(DevScene sc, RenderParams rp, WaveBufs wb, int64_t slot_base, int64_t nrec, Counters* __restrict__ ctr, int s1d_lds, const uint32_t* __restrict__ order);
template __global__ void k_mb_setup<true>(DevScene sc, RenderParams rp, ChainLayout lay, const PcgJump* __restrict__ jump, WaveBufs wb, int64_t slot_base, int64_t nslots_batch);

}  // namespace pbrtk
