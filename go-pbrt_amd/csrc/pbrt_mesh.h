// pbrt_mesh.h — triangle meshes on the device (extension: BASELINE configs D/E).
//
// go-pbrt has no triangle shape (pkg/shapes holds only disk.go) and its BVH
// builder is O(n^2) and chain-shaped (pkg/accelerator/bvh.go:272-411) with a
// fixed [64] traversal stack (bvh.go:670), so a million-triangle scene needs
// semantics and an accelerator of its own (include/pbrt_gpu.h, pbrt_mesh_desc):
//
//  * triangle test: pbrt-v3 Triangle::Intersect (watertight, Woop et al.), in
//    float64 after exact widening of the float32 world-space vertices, error
//    bounds with epsilon = 2^-53 (go-pbrt's own Gamma() is denormal, #16);
//  * accelerator: an LBVH built on the device (mesh_bvh.hip), stored as eight
//    stackless "threaded" node arrays, one per ray-direction octant: nodes in
//    depth-first order with, at every node, the child nearer along the node's
//    split axis for that octant first (pbrt's front-to-back rule), each node
//    holding the index that follows its subtree (its escape). A lane walks
//    i -> i + 1 on a box hit and i -> escape on a miss or after a leaf: no
//    stack, no LDS, one 32-byte node per step;
//  * closest hit = the smallest (t, global triangle index) over every
//    triangle hit with t < TMax. The traversal order and the tree shape then
//    cannot change a result, so the oracle (oracle/oracle_mesh.c) checks this
//    path with an accelerator of its own.
//
// HBM layout (per scene, built once in pbrt_gpu_create):
//   nodes  [8][n_nodes] MeshNode (32 B: float32 box rounded out by one ulp,
//          escape index, leaf word)
//   tris   [n_tris][9] float32 vertices in leaf order (36 B per triangle)
//   gid    [n_tris] global triangle index of each leaf slot (read on a hit)
#pragma once
#pragma clang fp contract(off)

#include "pbrt_core.h"

namespace pbrt {

struct alignas(16) MeshNode {
    float bmin[3];
    uint32_t escape;   // node index after this node's subtree (n_nodes: done)
    float bmax[3];
    uint32_t leaf;     // kMeshInterior, or (first leaf slot << 3) | count (1..7)
};
static_assert(sizeof(MeshNode) == 32, "MeshNode is two 16-byte loads");
constexpr uint32_t kMeshInterior = 0xFFFFFFFFu;
#ifndef PBRT_MESH_LEAF_MAX
#define PBRT_MESH_LEAF_MAX 1   // build option (1..7); 1 measured best on D (chain 667 / 699 / 746 / 802 / 898 ms at 1 / 2 / 3 / 4 / 6)
#endif
constexpr int kMeshLeafMax = PBRT_MESH_LEAF_MAX;   // triangles per leaf (subtrees this small are collapsed)
constexpr int kMeshOrders = 8;    // threaded orderings, one per ray-direction octant
constexpr int kMeshPad = 2;       // nodes allocated past the last ordering (mesh_walk's look-ahead loads)

struct DevMesh {
    const MeshNode* nodes;       // [kMeshOrders][n_nodes]
    const float* tris;           // [n_tris][9]
    const int32_t* gid;          // [n_tris]
    const int32_t* mesh_first;   // [n_meshes + 1] first global index of each mesh
    const int32_t* mesh_mat;     // [n_meshes]
    const int32_t* mesh_rev;     // [n_meshes]
    int n_nodes, n_tris, n_meshes;
    int count_slot;   // PBRT_MESH_COUNT builds: counter set of the launching kernel (0: off)
};

#ifdef PBRT_MESH_COUNT
// Diagnostics build (make meshcount): per kernel slot and query kind, the
// walks, nodes fetched and triangles tested -- the algorithmic bytes of the
// traversal (32 B per node, 36 B per triangle), read by tools/count_mesh_bytes.py.
constexpr int kMeshCountSlots = 8;
__device__ unsigned long long g_mesh_count[kMeshCountSlots][2][3];
#endif

// pbrt-v3 gamma(n), MachineEpsilon = 2^-53
GO_HD double tri_gamma(double n) {
    const double e = 1.1102230246251565e-16;
    return (n * e) / (1 - n * e);
}
GO_HD double tri_max(double a, double b) { return a > b ? a : b; }

// pbrt-v3 Triangle::Intersect, hit part (shapes/triangle.cpp), float64; the
// statement order is oracle/oracle_mesh.c's orc_triangle_hit.
GO_HD bool tri_hit(const double* v, const Ray& r, double& t_out, double& b0o, double& b1o, double& b2o) {
    double p0t[3] = {v[0] - r.o.x, v[1] - r.o.y, v[2] - r.o.z};
    double p1t[3] = {v[3] - r.o.x, v[4] - r.o.y, v[5] - r.o.z};
    double p2t[3] = {v[6] - r.o.x, v[7] - r.o.y, v[8] - r.o.z};
    const double ax = gomath::abs(r.d.x), ay = gomath::abs(r.d.y), az = gomath::abs(r.d.z);
    const int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);   // MaxDimension
    const int kx = kz == 2 ? 0 : kz + 1, ky = kx == 2 ? 0 : kx + 1;
    const double rd[3] = {r.d.x, r.d.y, r.d.z};
    const double dx = rd[kx], dy = rd[ky], dz = rd[kz];
    double q0x = p0t[kx], q0y = p0t[ky], q0z = p0t[kz];
    double q1x = p1t[kx], q1y = p1t[ky], q1z = p1t[kz];
    double q2x = p2t[kx], q2y = p2t[ky], q2z = p2t[kz];
    const double Sx = -dx / dz, Sy = -dy / dz, Sz = 1.0 / dz;
    q0x += Sx * q0z; q0y += Sy * q0z;
    q1x += Sx * q1z; q1y += Sy * q1z;
    q2x += Sx * q2z; q2y += Sy * q2z;
    const double e0 = q1x * q2y - q1y * q2x;
    const double e1 = q2x * q0y - q2y * q0x;
    const double e2 = q0x * q1y - q0y * q1x;
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    const double det = e0 + e1 + e2;
    if (det == 0) return false;
    q0z *= Sz; q1z *= Sz; q2z *= Sz;
    const double ts = e0 * q0z + e1 * q1z + e2 * q2z;
    if (det < 0 && ts >= 0) return false;
    if (det > 0 && ts <= 0) return false;
    const double inv = 1 / det;
    const double b0 = e0 * inv, b1 = e1 * inv, b2 = e2 * inv;
    const double t = ts * inv;
    const double maxZt = tri_max(gomath::abs(q0z), tri_max(gomath::abs(q1z), gomath::abs(q2z)));
    const double deltaZ = tri_gamma(3) * maxZt;
    const double maxXt = tri_max(gomath::abs(q0x), tri_max(gomath::abs(q1x), gomath::abs(q2x)));
    const double maxYt = tri_max(gomath::abs(q0y), tri_max(gomath::abs(q1y), gomath::abs(q2y)));
    const double deltaX = tri_gamma(5) * (maxXt + maxZt);
    const double deltaY = tri_gamma(5) * (maxYt + maxZt);
    const double deltaE = 2 * (tri_gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    const double maxE = tri_max(gomath::abs(e0), tri_max(gomath::abs(e1), gomath::abs(e2)));
    const double deltaT = 3 * (tri_gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * gomath::abs(inv);
    if (t <= deltaT) return false;
    t_out = t;
    b0o = b0; b1o = b1; b2o = b2;
    return true;
}

// Ordering of the threaded node arrays for a ray: its direction octant
#ifndef PBRT_MESH_ORDER_MASK
#define PBRT_MESH_ORDER_MASK 7   // experiment builds: octant bits that select an ordering (7: all three)
#endif
GO_HD int mesh_ordering(V3 d) {
    return ((d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0)) & PBRT_MESH_ORDER_MASK;
}

#ifdef __HIPCC__
__device__ __forceinline__ void load_tri(const float* __restrict__ tris, uint32_t slot, double v[9]) {
    const float* q = tris + (size_t)slot * 9;
#pragma unroll
    for (int k = 0; k < 9; k++) v[k] = (double)q[k];
}

// Slab test of a float32 box (rounded out), inclusive of tmax so a triangle at
// exactly the current TMax with a smaller index is never culled. An axis with
// d == 0 (inverse +-Inf) constrains only through the origin's position.
__device__ __forceinline__ bool mesh_box_hit(const float* bmin, const float* bmax, const Ray& r, V3 inv,
                                             int zero_mask, double tmax) {
    const double robust = 1 + 2 * tri_gamma(3);
    double t0 = 0, t1 = kInf;
    const double o[3] = {r.o.x, r.o.y, r.o.z}, iv[3] = {inv.x, inv.y, inv.z};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const double lo = (double)bmin[k], hi = (double)bmax[k];
        double n, f;
        if (zero_mask & (1 << k)) {
            const bool in = lo <= o[k] && o[k] <= hi;
            n = in ? -kInf : kInf;
            f = in ? kInf : -kInf;
        } else {
            const double a = (lo - o[k]) * iv[k], b = (hi - o[k]) * iv[k];
            n = a < b ? a : b;
            f = (a < b ? b : a) * robust;
        }
        t0 = n > t0 ? n : t0;
        t1 = f < t1 ? f : t1;
    }
    return t0 <= t1 && t0 <= tmax;
}

// Leaf tests batched across the wave (build option PBRT_MESH_BATCH, default on).
// With one-triangle leaves about one node visit in 17 is a leaf, so in a
// 64-lane wave nearly every step of a per-lane walk has some lane at a leaf,
// and the wave pays a triangle test (~5x a box test) on almost every step. A
// lane that reaches a leaf here waits with it while the others walk on; the
// wave tests its pending triangles together once half of its live lanes hold
// one, or no lane can walk further. A waiting lane makes no box test (none sees
// an older TMax than in the per-lane walk), and the closest hit is the smallest
// (t, index) whatever the order of the tests: the results are the same.
#ifndef PBRT_MESH_BATCH
#define PBRT_MESH_BATCH 1
#endif

// Closest (kAny = false) or any (kAny) triangle of the scene's meshes.
// Closest: a hit must have t < tmax, or t == tmax and a smaller global index
// than best_gid (-1: nothing of the meshes yet, TMax exclusive). On return
// tmax, best_slot and best_gid describe the winner; returns whether any
// triangle won. Any: returns true on the first triangle with t < tmax.
template <bool kAny>
__device__ inline bool mesh_walk(const DevMesh& m, const Ray& ray, double& tmax, int32_t& best_slot,
                                 int32_t& best_gid) {
    if (m.n_nodes == 0) return false;
    const MeshNode* __restrict__ N = m.nodes + (size_t)mesh_ordering(ray.d) * (size_t)m.n_nodes;
    const V3 inv{1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z};
    const int zero_mask = (ray.d.x == 0 ? 1 : 0) | (ray.d.y == 0 ? 2 : 0) | (ray.d.z == 0 ? 4 : 0);
    const uint32_t n = (uint32_t)m.n_nodes;
    bool found = false;
    uint32_t i = 0;
#ifdef PBRT_MESH_COUNT
    unsigned long long c_nodes = 0, c_tris = 0;
    struct Flush {
        int slot;
        unsigned long long &nn, &tt;
        __device__ ~Flush() {
            if (slot > 0 && slot < kMeshCountSlots) {
                atomicAdd(&g_mesh_count[slot][kAny ? 1 : 0][0], 1ull);
                atomicAdd(&g_mesh_count[slot][kAny ? 1 : 0][1], nn);
                atomicAdd(&g_mesh_count[slot][kAny ? 1 : 0][2], tt);
            }
        }
    } flush{m.count_slot, c_nodes, c_tris};
#define MESH_COUNT(x) x
#else
#define MESH_COUNT(x)
#endif
#ifdef PBRT_MESH_PREFETCH
    // (experiment build, a loss on D: chain 897 vs 798 ms, paths 272 vs 229)
    // node i in (a, b) and node i + 1 in (a2, b2): a hit interior node's first
    // child is the next node of the threaded order, so the walk down a hit
    // path moves to a node already loaded and fetches the one after it while
    // testing this one (the arrays carry kMeshPad nodes past their end)
    auto load_node = [&](uint32_t j, uint4& x, uint4& y) {
        const uint4* q = reinterpret_cast<const uint4*>(N + j);
        x = q[0];
        y = q[1];
    };
    uint4 a, b, a2, b2;
    load_node(0, a, b);
    load_node(1, a2, b2);
#endif
#if PBRT_MESH_BATCH && !defined(PBRT_MESH_PREFETCH)
    uint32_t pend = 0;   // a leaf word waiting for the wave's triangle batch (0: none)
    for (;;) {
        // nodes: until half the live lanes wait with a leaf, or none walks on
        for (;;) {
            const bool walking = i < n && pend == 0;
            const unsigned long long mw = __ballot(walking);
            if (mw == 0) break;
            const unsigned long long mp = __ballot(pend != 0), ml = mw | mp;
            if (2 * __popcll(mp) >= __popcll(ml)) break;
            if (walking) {
                MESH_COUNT(c_nodes++;)
                const uint4* q = reinterpret_cast<const uint4*>(N + i);
                const uint4 a = q[0], b = q[1];
                const float bmin[3] = {__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z)};
                const float bmax[3] = {__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)};
                if (!mesh_box_hit(bmin, bmax, ray, inv, zero_mask, tmax)) {
                    i = a.w;   // escape
                } else if (b.w == kMeshInterior) {
                    i++;
                } else {
                    pend = b.w;
                    i = a.w;
                }
            }
        }
        if (!__any(pend != 0)) break;
        if (pend != 0) {   // the batch: every waiting lane tests its leaf
            const uint32_t first = pend >> 3, cnt = pend & 7u;
            pend = 0;
            for (uint32_t k = 0; k < cnt; k++) {
                double v[9], t, b0, b1, b2;
                load_tri(m.tris, first + k, v);
                MESH_COUNT(c_tris++;)
                if (!tri_hit(v, ray, t, b0, b1, b2)) continue;
                if (kAny) {
                    if (t < tmax) {
                        found = true;
                        i = n;   // answered
                        break;
                    }
                    continue;
                }
                if (t < tmax || (t == tmax && m.gid[first + k] < best_gid)) {
                    tmax = t;
                    best_slot = (int32_t)(first + k);
                    best_gid = m.gid[first + k];
                    found = true;
                }
            }
        }
    }
    return found;
#endif
    while (i < n) {
        MESH_COUNT(c_nodes++;)
#ifndef PBRT_MESH_PREFETCH
        const uint4* q = reinterpret_cast<const uint4*>(N + i);
        const uint4 a = q[0], b = q[1];
#endif
        const float bmin[3] = {__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z)};
        const float bmax[3] = {__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)};
        const uint32_t escape = a.w, leaf = b.w;
        if (!mesh_box_hit(bmin, bmax, ray, inv, zero_mask, tmax)) {
            i = escape;
#ifdef PBRT_MESH_PREFETCH
            if (i < n) {
                load_node(i, a, b);
                load_node(i + 1, a2, b2);
            }
#endif
            continue;
        }
        if (leaf == kMeshInterior) {
            i++;
#ifdef PBRT_MESH_PREFETCH
            a = a2;
            b = b2;
            load_node(i + 1, a2, b2);
#endif
            continue;
        }
        const uint32_t first = leaf >> 3, cnt = leaf & 7u;
        for (uint32_t k = 0; k < cnt; k++) {
            double v[9], t, b0, b1, b2;
            load_tri(m.tris, first + k, v);
            MESH_COUNT(c_tris++;)
            if (!tri_hit(v, ray, t, b0, b1, b2)) continue;
            if (kAny) {
                if (t < tmax) return true;
                continue;
            }
            if (t < tmax || (t == tmax && m.gid[first + k] < best_gid)) {
                tmax = t;
                best_slot = (int32_t)(first + k);
                best_gid = m.gid[first + k];
                found = true;
            }
        }
        i = escape;
#ifdef PBRT_MESH_PREFETCH
        if (i < n) {
            load_node(i, a, b);
            load_node(i + 1, a2, b2);
        }
#endif
    }
    return found;
}
#undef MESH_COUNT
#endif

}  // namespace pbrt
