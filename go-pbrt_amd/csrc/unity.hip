// unity.hip — every translation unit of the library as one, for the diagnostics
// and experiment builds (Makefile: steptime, meshcount, diag, variant), whose
// __device__ counters must exist once. The kernel definitions come before
// render.hip: their launch bounds must be on the first declaration a kernel
// sees (render_kernels.h's plain declarations first would leave every kernel
// at the default 1024-thread bound, i.e. 128 VGPRs, and spilling).
#include "mesh_bvh.hip"
#include "k_chain_1.hip"
#include "k_chain_n.hip"
#include "k_chain_x.hip"
#include "k_paths_m.hip"
#include "k_paths_x.hip"
#include "k_serial.hip"
#include "k_pw.hip"
#include "k_frame.hip"
#include "render.hip"
