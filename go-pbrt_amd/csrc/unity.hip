// unity.hip — every translation unit of the library as one, for the diagnostics
// and experiment builds (Makefile: steptime, meshcount, diag, variant), whose
// __device__ counters must exist once.
#include "render.hip"
#include "mesh_bvh.hip"
#include "k_chain_1.hip"
#include "k_chain_n.hip"
#include "k_chain_x.hip"
#include "k_paths_m.hip"
#include "k_paths_x.hip"
#include "k_serial.hip"
#include "k_pw.hip"
#include "k_frame.hip"
