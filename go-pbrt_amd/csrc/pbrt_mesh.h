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

#include <cstring>

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

// Wide layout (build option PBRT_MESH_WIDE, default off: measured slower): a 4-ary tree
// collapsed from the same LBVH, one array for every ray. A node holds its up
// to four children's boxes (structure of arrays, so a visit is eight 16-byte
// loads and four independent slab tests), their child words, its parent and
// the axis along which the children are stored in ascending centre order.
// A ray visits the hit children front to back along that axis (ascending for
// a non-negative direction component) and keeps, per level, a 4-bit mask of
// the hit children still to visit (the trail: 32 levels in two 64-bit words);
// going back up reads the parent's last 32 bytes (child words, parent, axis).
// Triangles are child slots (one per slot: every triangle box is tested before
// its triangle). The builder guarantees <= kMeshWideLevels levels.
// Config D (float32 box tests, batched triangle tests): frame 1139 ms (chain
// 876) against the binary threaded walk's 723 ms (chain 547). A wide visit
// moves 128 B and tests four boxes; the binary walk's next node is mostly the
// next 32 bytes of the line it already holds (depth-first threading), and its
// 84 steps per closest walk cost less than the wide walk's ~25 visits + ~18
// steps back up (profiles/r05/mesh_wide/).
#ifndef PBRT_MESH_WIDE
#define PBRT_MESH_WIDE 0
#endif
struct alignas(16) MeshNode4 {
    float lo[3][4];        // [axis][child slot]
    float hi[3][4];
    uint32_t child[4];     // node index, kMeshTri | triangle slot, or kMeshEmpty
    uint32_t parent;       // kMeshEmpty at the root
    uint32_t axis;         // children stored in ascending centre order along it
    uint32_t count;        // children (slots count..3 are empty)
    uint32_t pad;
};
static_assert(sizeof(MeshNode4) == 128, "MeshNode4 is eight 16-byte loads");
constexpr uint32_t kMeshTri = 0x80000000u;
constexpr uint32_t kMeshEmpty = 0xFFFFFFFFu;
constexpr int kMeshWideLevels = 32;
// bytes of a scene's node array(s) of n_nodes nodes
constexpr size_t mesh_node_bytes(int n_nodes) {
    return PBRT_MESH_WIDE ? (size_t)n_nodes * sizeof(MeshNode4) : (size_t)n_nodes * kMeshOrders * sizeof(MeshNode);
}

struct DevMesh {
    const MeshNode* nodes;       // [kMeshOrders][n_nodes] (wide: MeshNode4 [n_nodes])
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

// Slab test of a float32 box (rounded out), inclusive of tmax so a triangle at
// exactly the current TMax with a smaller index is never culled. An axis with
// d == 0 (inverse +-Inf) constrains only through the origin's position.
GO_HD bool mesh_box_hit(const float* bmin, const float* bmax, const Ray& r, V3 inv, int zero_mask, double tmax) {
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

// Box tests in float32 (build option PBRT_MESH_F32, default on): an interval
// that contains the float64 test's [n, f * robust] above, so the float32 test
// culls no box the float64 test keeps (and the closest hit, the smallest (t,
// index) over the triangles whose boxes pass, is unchanged). Per slab, with
// o32 = fl32(o) and iv32 = fl32(iv), the float32 n32 = fl32(fl32(l - o32) iv32)
// differs from the float64 n64 = fl64(fl64(l - o) iv) by at most
// 3.01 * 2^-24 |n32| + 1.0001 * 2^-24 |o iv| (three float32 roundings, the
// origin's rounding, two float64 roundings); the test widens each bound by
// m = 2^-20 (|x| + |o32 iv32|) + 1e-35 (16x that, plus the rounding of the
// widening itself and of underflow), and compares with fl32 of TMax rounded
// up. A zero direction component keeps the origin-only test: rounding to
// nearest keeps o32 inside [l, h] whenever o is (l and h are float32).
// Rays with a nonzero |d_i| outside [1e-30, 1e30] take the float64 test.
#ifndef PBRT_MESH_F32
#define PBRT_MESH_F32 1
#endif
struct MeshRay32 {
    float o[3], iv[3], m0[3];   // fl32(o), fl32(1/d), 2^-20 |o32 iv32| + 1e-35
    float tmax_hi;              // fl32(TMax) rounded up
    int zero_mask;
    bool ok;                    // the float32 test applies
};
GO_HD float mesh_f32_up(double t) {
    const float f = (float)t;
    if (!((double)f < t)) return f;
    if (f == 0) return 0x1p-149f;   // the smallest positive float
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u = f > 0 ? u + 1 : u - 1;   // the next float up
    float g;
    std::memcpy(&g, &u, 4);
    return g;
}
GO_HD MeshRay32 mesh_ray32(const Ray& r, int zero_mask, double tmax) {
    MeshRay32 q;
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    q.ok = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double ad = d[a] < 0 ? -d[a] : d[a];
        q.ok = q.ok && (ad == 0 || (ad >= 1e-30 && ad <= 1e30));
        q.o[a] = (float)o[a];
        q.iv[a] = (float)(1 / d[a]);
        const float oi = q.o[a] * q.iv[a];
        q.m0[a] = (zero_mask >> a) & 1 ? 0.0f : 0x1p-20f * (oi < 0 ? -oi : oi) + 1e-35f;
    }
    q.tmax_hi = mesh_f32_up(tmax);
    q.zero_mask = zero_mask;
    return q;
}
GO_HD bool mesh_box32_hit(const float* bmin, const float* bmax, const MeshRay32& q) {
    float t0 = 0, t1 = __builtin_inff();
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float x = (bmin[a] - q.o[a]) * q.iv[a], y = (bmax[a] - q.o[a]) * q.iv[a];
        float n = x < y ? x : y, f = x < y ? y : x;
        n = n - (0x1p-20f * (n < 0 ? -n : n) + q.m0[a]);
        f = f + (0x1p-20f * (f < 0 ? -f : f) + q.m0[a]);
        const bool in = bmin[a] <= q.o[a] && q.o[a] <= bmax[a];
        const bool zero = (q.zero_mask >> a) & 1;
        n = zero ? (in ? -__builtin_inff() : __builtin_inff()) : n;
        f = zero ? (in ? __builtin_inff() : -__builtin_inff()) : f;
        t0 = n > t0 ? n : t0;
        t1 = f < t1 ? f : t1;
    }
    return t0 <= t1 && t0 <= q.tmax_hi;
}
// the box test a walk runs: float32 where it applies, else float64
GO_HD bool mesh_box_test(const float* bmin, const float* bmax, const Ray& r, V3 inv, int zero_mask, double tmax,
                         const MeshRay32& q) {
#if PBRT_MESH_F32
    if (q.ok) return mesh_box32_hit(bmin, bmax, q);
#endif
    return mesh_box_hit(bmin, bmax, r, inv, zero_mask, tmax);
}

#ifdef __HIPCC__
__device__ __forceinline__ void load_tri(const float* __restrict__ tris, uint32_t slot, double v[9]) {
    const float* q = tris + (size_t)slot * 9;
#pragma unroll
    for (int k = 0; k < 9; k++) v[k] = (double)q[k];
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
#ifndef PBRT_MESH_BATCH_Q8
#define PBRT_MESH_BATCH_Q8 2   // the batch runs once Q8/8 of the live lanes wait with a leaf (build option; D chain with float64 boxes 567 / 612 / 771 / 1201 ms at Q8 = 2 / 4 / 6 / 8, with float32 boxes 564 / 547 / 555 ms at Q8 = 1 / 2 / 3)
#endif
static_assert(PBRT_MESH_BATCH_Q8 >= 1, "a batch needs a waiting lane");

// Closest (kAny = false) or any (kAny) triangle of the scene's meshes.
// Closest: a hit must have t < tmax, or t == tmax and a smaller global index
// than best_gid (-1: nothing of the meshes yet, TMax exclusive). On return
// tmax, best_slot and best_gid describe the winner; returns whether any
// triangle won. Any: returns true on the first triangle with t < tmax.
#if PBRT_MESH_WIDE
__device__ __forceinline__ uint32_t u4_at(const uint4& v, int k) {
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}

// Slab test of child slot k of a wide node (the binary test's arithmetic);
// nf: the node as 32 floats (lo[a][k] at 4a + k, hi[a][k] at 12 + 4a + k).
__device__ __forceinline__ bool mesh_box4_hit(const float* __restrict__ nf, uint32_t k, const double* o,
                                              const double* iv, int zero_mask, double tmax) {
    const double robust = 1 + 2 * tri_gamma(3);
    double t0 = 0, t1 = kInf;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double l = (double)nf[4 * a + k], h = (double)nf[12 + 4 * a + k];
        double n, f;
        if (zero_mask & (1 << a)) {
            const bool in = l <= o[a] && o[a] <= h;
            n = in ? -kInf : kInf;
            f = in ? kInf : -kInf;
        } else {
            const double x = (l - o[a]) * iv[a], y = (h - o[a]) * iv[a];
            n = x < y ? x : y;
            f = (x < y ? y : x) * robust;
        }
        t0 = n > t0 ? n : t0;
        t1 = f < t1 ? f : t1;
    }
    return t0 <= t1 && t0 <= tmax;
}

// A whole wide-node visit: the node's eight 16-byte loads issued together, the
// four slab tests without branches (the same arithmetic as mesh_box4_hit; a
// zero direction component's axis selects the origin-only test), the hit
// slots (below `count`) and which of them are triangles.
__device__ __forceinline__ void mesh_visit4(const MeshNode4* __restrict__ node, const double* o, const double* iv,
                                            int zero_mask, double tmax, const MeshRay32& r32, uint4& ch, uint4& meta,
                                            uint32_t& hit, uint32_t& tri) {
    const uint4* q = reinterpret_cast<const uint4*>(node);
    const uint4 L[3] = {q[0], q[1], q[2]}, H[3] = {q[3], q[4], q[5]};
    ch = q[6];
    meta = q[7];
    const double robust = 1 + 2 * tri_gamma(3);
    hit = 0;
#if PBRT_MESH_F32
    if (r32.ok) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float bmin[3] = {__uint_as_float(u4_at(L[0], k)), __uint_as_float(u4_at(L[1], k)),
                                   __uint_as_float(u4_at(L[2], k))};
            const float bmax[3] = {__uint_as_float(u4_at(H[0], k)), __uint_as_float(u4_at(H[1], k)),
                                   __uint_as_float(u4_at(H[2], k))};
            hit |= mesh_box32_hit(bmin, bmax, r32) ? 1u << k : 0u;
        }
    } else
#endif
#pragma unroll
    for (int k = 0; k < 4; k++) {
        double t0 = 0, t1 = kInf;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const double l = (double)__uint_as_float(u4_at(L[a], k)), h = (double)__uint_as_float(u4_at(H[a], k));
            const double x = (l - o[a]) * iv[a], y = (h - o[a]) * iv[a];
            double n = x < y ? x : y, f = (x < y ? y : x) * robust;
            const bool in = l <= o[a] && o[a] <= h;
            const bool zero = (zero_mask >> a) & 1;
            n = zero ? (in ? -kInf : kInf) : n;
            f = zero ? (in ? kInf : -kInf) : f;
            t0 = n > t0 ? n : t0;
            t1 = f < t1 ? f : t1;
        }
        hit |= (t0 <= t1 && t0 <= tmax) ? 1u << k : 0u;
    }
    hit &= (1u << meta.z) - 1u;
    tri = hit & (((ch.x >> 31) << 0) | ((ch.y >> 31) << 1) | ((ch.z >> 31) << 2) | ((ch.w >> 31) << 3));
}

// kLean: one child's box at a time (the copy that kernels over analytic
// scenes carry for mixed scenes, where the four boxes' registers would raise
// the kernel's peak); else the four boxes' loads are issued together.
template <bool kAny, bool kLean = false>
__device__ inline bool mesh_walk(const DevMesh& m, const Ray& ray, double& tmax, int32_t& best_slot,
                                 int32_t& best_gid) {
    if (m.n_nodes == 0) return false;
    const MeshNode4* __restrict__ N = reinterpret_cast<const MeshNode4*>(m.nodes);
    const double o[3] = {ray.o.x, ray.o.y, ray.o.z};
    const double iv[3] = {1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z};
    const int zero_mask = (ray.d.x == 0 ? 1 : 0) | (ray.d.y == 0 ? 2 : 0) | (ray.d.z == 0 ? 4 : 0);
    const int neg = (ray.d.x < 0 ? 1 : 0) | (ray.d.y < 0 ? 2 : 0) | (ray.d.z < 0 ? 4 : 0);
    bool found = false;
    uint32_t cur = 0, par = kMeshEmpty;
    uint64_t tr0 = 0, tr1 = 0;   // the trail: 4-bit masks, the deepest level in tr0's low bits
    int depth = 0;
    MeshRay32 q32 = mesh_ray32(ray, zero_mask, tmax);
#ifdef PBRT_MESH_COUNT
    unsigned long long c_nodes = 0, c_tris = 0;   // c_nodes in 32-byte blocks
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
#if PBRT_MESH_BATCH
    if constexpr (!kLean) {
        // Triangle tests batched across the wave, as in the binary walk: a lane
        // whose visit hits triangle slots waits with them (pnode, ptri) and the
        // node's hit inner children (pin); the wave tests the waiting lanes'
        // triangles together once Q8/8 of its live lanes wait or no lane can
        // move. A move is one node visit or one level back up.
        bool up = false, done = false;
        uint32_t pnode = 0, ptri = 0, pin = 0;
        auto go_down = [&](uint32_t axis, const uint4& ch, uint32_t inner) {
            if (!inner) {
                up = true;
                return;
            }
            const int s = ((neg >> axis) & 1) ? 31 - __clz(inner) : __ffs(inner) - 1;
            tr1 = (tr1 << 4) | (tr0 >> 60);
            tr0 = (tr0 << 4) | (inner & ~(1u << s));
            depth++;
            cur = u4_at(ch, s);
        };
        for (;;) {
            for (;;) {
                const bool moving = !done && ptri == 0;
                const unsigned long long mw = __ballot(moving);
                if (mw == 0) break;
                const unsigned long long mp = __ballot(ptri != 0), ml = mw | mp;
                if (8 * __popcll(mp) >= PBRT_MESH_BATCH_Q8 * __popcll(ml)) break;
                if (!moving) continue;
                if (up) {
                    if (depth == 0) {
                        done = true;
                        continue;
                    }
                    const uint32_t rest = (uint32_t)tr0 & 15u;
                    const uint4* pq = reinterpret_cast<const uint4*>(N + par);
                    const uint4 pch = pq[6], pmeta = pq[7];
                    MESH_COUNT(c_nodes += 1;)
                    if (rest) {
                        const int s = ((neg >> pmeta.y) & 1) ? 31 - __clz(rest) : __ffs(rest) - 1;
                        tr0 &= ~(uint64_t)(1u << s);
                        cur = u4_at(pch, s);
                        up = false;
                    } else {
                        tr0 = (tr0 >> 4) | (tr1 << 60);
                        tr1 >>= 4;
                        depth--;
                        par = pmeta.x;
                    }
                    continue;
                }
                uint4 ch, meta;
                uint32_t hit, tri;
                mesh_visit4(N + cur, o, iv, zero_mask, tmax, q32, ch, meta, hit, tri);
                MESH_COUNT(c_nodes += 4;)
                par = meta.x;
                if (tri) {
                    pnode = cur;
                    ptri = tri;
                    pin = hit & ~tri;
                } else {
                    go_down(meta.y, ch, hit);
                }
            }
            if (!__any(ptri != 0)) break;
            if (ptri != 0) {   // the batch
                const uint4* q = reinterpret_cast<const uint4*>(N + pnode);
                const uint4 ch = q[6], meta = q[7];
                for (uint32_t h = ptri; h; h &= h - 1) {
                    const uint32_t slot = u4_at(ch, __ffs(h) - 1) & ~kMeshTri;
                    double v[9], t, b0, b1, b2;
                    load_tri(m.tris, slot, v);
                    MESH_COUNT(c_tris++;)
                    if (!tri_hit(v, ray, t, b0, b1, b2)) continue;
                    if (kAny) {
                        if (t < tmax) {
                            found = true;
                            done = true;
                            break;
                        }
                        continue;
                    }
                    if (t < tmax || (t == tmax && m.gid[slot] < best_gid)) {
                        tmax = t;
                        q32.tmax_hi = mesh_f32_up(t);
                        best_slot = (int32_t)slot;
                        best_gid = m.gid[slot];
                        found = true;
                    }
                }
                ptri = 0;
                if (!done) go_down(meta.y, ch, pin);
            }
        }
        return found;
    }
#endif
    for (;;) {
        // visit node cur: test its children's boxes, its triangles, then go
        // down to the nearest hit child node
        const float* __restrict__ nf = reinterpret_cast<const float*>(N + cur);
        const uint32_t* __restrict__ nu = reinterpret_cast<const uint32_t*>(N + cur);
        MESH_COUNT(c_nodes += 4;)
        par = nu[28];
        const uint32_t axis = nu[29], nch = nu[30];
        uint32_t hit = 0;
        if constexpr (kLean) {
#pragma unroll 1
            for (uint32_t k = 0; k < nch; k++)
                if (mesh_box4_hit(nf, k, o, iv, zero_mask, tmax)) hit |= 1u << k;
        } else {
            uint4 ch, meta;
            uint32_t tri;
            mesh_visit4(N + cur, o, iv, zero_mask, tmax, q32, ch, meta, hit, tri);
        }
        uint32_t inner = 0;
        for (uint32_t h = hit; h; h &= h - 1) {
            const uint32_t k = (uint32_t)__ffs(h) - 1, c = nu[24 + k];
            if (!(c & kMeshTri)) {
                inner |= 1u << k;
                continue;
            }
            const uint32_t slot = c & ~kMeshTri;
            double v[9], t, b0, b1, b2;
            load_tri(m.tris, slot, v);
            MESH_COUNT(c_tris++;)
            if (!tri_hit(v, ray, t, b0, b1, b2)) continue;
            if (kAny) {
                if (t < tmax) return true;
                continue;
            }
            if (t < tmax || (t == tmax && m.gid[slot] < best_gid)) {
                tmax = t;
                q32.tmax_hi = mesh_f32_up(t);
                best_slot = (int32_t)slot;
                best_gid = m.gid[slot];
                found = true;
            }
        }
        if (inner) {
            const int s = ((neg >> axis) & 1) ? 31 - __clz(inner) : __ffs(inner) - 1;
            tr1 = (tr1 << 4) | (tr0 >> 60);
            tr0 = (tr0 << 4) | (inner & ~(1u << s));
            depth++;
            cur = nu[24 + s];
            continue;
        }
        // back up: the deepest level with a hit child left
        for (;;) {
            if (depth == 0) return found;
            const uint32_t rest = (uint32_t)tr0 & 15u;
            const uint32_t* __restrict__ pu = reinterpret_cast<const uint32_t*>(N + par);
            MESH_COUNT(c_nodes += 1;)
            if (rest) {
                const int s = ((neg >> pu[29]) & 1) ? 31 - __clz(rest) : __ffs(rest) - 1;
                tr0 &= ~(uint64_t)(1u << s);
                cur = pu[24 + s];
                break;
            }
            tr0 = (tr0 >> 4) | (tr1 << 60);
            tr1 >>= 4;
            depth--;
            par = pu[28];
        }
    }
}
#else
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
    MeshRay32 q32 = mesh_ray32(ray, zero_mask, tmax);
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
            if (8 * __popcll(mp) >= PBRT_MESH_BATCH_Q8 * __popcll(ml)) break;
            if (walking) {
                MESH_COUNT(c_nodes++;)
                const uint4* q = reinterpret_cast<const uint4*>(N + i);
                const uint4 a = q[0], b = q[1];
                const float bmin[3] = {__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z)};
                const float bmax[3] = {__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z)};
                if (!mesh_box_test(bmin, bmax, ray, inv, zero_mask, tmax, q32)) {
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
                    q32.tmax_hi = mesh_f32_up(t);
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
        if (!mesh_box_test(bmin, bmax, ray, inv, zero_mask, tmax, q32)) {
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
                q32.tmax_hi = mesh_f32_up(t);
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
#endif   // PBRT_MESH_WIDE
#undef MESH_COUNT

// the walk as kernels over scenes with analytic primitives carry it
template <bool kAny>
__device__ __forceinline__ bool mesh_walk_mixed(const DevMesh& m, const Ray& ray, double& tmax, int32_t& best_slot,
                                                int32_t& best_gid) {
#if PBRT_MESH_WIDE
    return mesh_walk<kAny, true>(m, ray, tmax, best_slot, best_gid);
#else
    return mesh_walk<kAny>(m, ray, tmax, best_slot, best_gid);
#endif
}
#endif

}  // namespace pbrt
