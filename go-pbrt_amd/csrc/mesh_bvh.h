// mesh_bvh.h — device LBVH build for the triangle-mesh extension (pbrt_mesh.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "pbrt_mesh.h"

namespace pbrt {

struct MeshBuild {
    MeshNode* nodes = nullptr;        // [kMeshOrders][n_nodes]
    float* tris = nullptr;            // [n_tris][9], leaf order
    int32_t* gid = nullptr;           // [n_tris]
    int32_t* mesh_first = nullptr;    // [n_meshes + 1]
    int32_t* mesh_mat = nullptr;      // [n_meshes]
    int32_t* mesh_rev = nullptr;      // [n_meshes]
    int n_nodes = 0, n_tris = 0, n_meshes = 0;
    int depth = 0;                    // deepest leaf (diagnostics)
    double build_ms = 0;              // device time of the build kernels
    DevMesh view() const {
        return DevMesh{nodes, tris, gid, mesh_first, mesh_mat, mesh_rev, n_nodes, n_tris, n_meshes, 0};
    }
};

// Builds the meshes of `s` on the current device (stream `st`, synchronous).
// Returns PBRT_OK, or a pbrt_status with `err` set.
int mesh_bvh_build(const pbrt_scene_desc* s, hipStream_t st, MeshBuild& out, std::string& err);
void mesh_bvh_free(MeshBuild& b);

// Ascending bitonic sort of npad 64-bit keys on stream `st` (npad a power of
// two >= 2048; pad with ~0). Also orders k_chain_ci's cold-frame schedule.
void bitonic_sort_u64(uint64_t* keys, uint32_t npad, hipStream_t st);

}  // namespace pbrt
