// mesh_bvh.hip — LBVH build on the device for the triangle-mesh extension.
//
// The reference's builder (pkg/accelerator/bvh.go:272-411) is an O(n^2) SAH
// build whose truncated bucket index peels one primitive per level (a chain,
// SURVEY §9 #21): unusable at a million triangles. This is Karras' parallel
// LBVH ("Maximizing Parallelism in the Construction of BVHs, Octrees, and k-d
// Trees", HPG 2012), one pass per stage, every stage one thread per element:
//
//   1. centroids + their bounds            (k_centroids, uint-ordered atomics)
//   2. 30-bit Morton code << 32 | index    (k_morton: unique 64-bit keys)
//   3. bitonic sort of the keys            (k_bitonic_*: LDS for strides < 1024)
//   4. triangles gathered in key order     (k_gather: leaf order = sorted order)
//   5. radix-tree topology                 (k_karras: one thread per inner node)
//   6. boxes, triangle counts and collapsed subtree sizes bottom-up
//                                          (k_up: the second child to finish climbs)
//   7. eight threaded depth-first layouts  (k_flatten: each kept node finds its
//      position by walking to the root), one per ray-direction octant
//
// Subtrees of <= kMeshLeafMax triangles become one leaf (their triangles are a
// contiguous key range). Boxes are float32, each triangle's rounded out by one
// ulp, so every box contains its triangles under the float64 slab test.
// The tree only affects speed: a closest hit is the smallest (t, index).
#include "mesh_bvh.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

namespace pbrt {
namespace {

constexpr int kB = 256;

__device__ __forceinline__ uint32_t f2ord(float f) {   // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float ord2f(uint32_t u) {
    const uint32_t v = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}

__global__ __launch_bounds__(kB) void k_centroids(const float* __restrict__ tris, int n, float* __restrict__ cen,
                                                  uint32_t* __restrict__ bounds /* [6]: min xyz, max xyz (ord) */) {
    __shared__ uint32_t smin[3][kB], smax[3][kB];
    const int i = blockIdx.x * kB + threadIdx.x;
    uint32_t mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0, 0, 0};
    if (i < n) {
        const float* q = tris + (size_t)i * 9;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float c = (q[k] + q[3 + k] + q[6 + k]) * (1.0f / 3.0f);
            cen[(size_t)i * 3 + k] = c;
            mn[k] = mx[k] = f2ord(c);
        }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) { smin[k][threadIdx.x] = mn[k]; smax[k][threadIdx.x] = mx[k]; }
    __syncthreads();
    for (int s = kB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                smin[k][threadIdx.x] = min(smin[k][threadIdx.x], smin[k][threadIdx.x + s]);
                smax[k][threadIdx.x] = max(smax[k][threadIdx.x], smax[k][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int k = 0; k < 3; k++) {
            atomicMin(&bounds[k], smin[k][0]);
            atomicMax(&bounds[3 + k], smax[k][0]);
        }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {   // 10 bits -> every third bit
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ __launch_bounds__(kB) void k_morton(const float* __restrict__ cen, int n, int npad,
                                               const uint32_t* __restrict__ bounds, uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= npad) return;
    if (i >= n) {
        keys[i] = ~0ull;   // padding sorts last
        return;
    }
    // one scale for all axes (the largest extent): a flat scene (a height field
    // is 300 x 10 x 300) then spends its top Morton bits on its long axes
    // instead of splitting along the thin one first
    float ext = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) ext = fmaxf(ext, ord2f(bounds[3 + k]) - ord2f(bounds[k]));
    uint32_t code = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float lo = ord2f(bounds[k]);
        float u = ext > 0 ? (cen[(size_t)i * 3 + k] - lo) / ext : 0.5f;
        u = fminf(fmaxf(u, 0.0f), 1.0f);
        const uint32_t q = min((uint32_t)(u * 1024.0f), 1023u);
        code |= spread10(q) << (2 - k);
    }
    keys[i] = ((uint64_t)code << 32) | (uint32_t)i;
}

// Bitonic sort, ascending. Strides >= 2048: one global compare-exchange pass;
// strides <= 1024: every remaining pass of the stage in LDS (2048 keys a block).
__global__ __launch_bounds__(1024) void k_bitonic_global(uint64_t* __restrict__ keys, uint32_t k, uint32_t j) {
    const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t l = i ^ j;
    if (l <= i) return;
    const uint64_t a = keys[i], b = keys[l];
    const bool up = (i & k) == 0;
    if ((a > b) == up) {
        keys[i] = b;
        keys[l] = a;
    }
}
__global__ __launch_bounds__(1024) void k_bitonic_local(uint64_t* __restrict__ keys, uint32_t k_begin,
                                                        uint32_t k_end, uint32_t j_begin) {
    __shared__ uint64_t s[2048];
    const uint32_t base = blockIdx.x * 2048u;
    s[threadIdx.x] = keys[base + threadIdx.x];
    s[threadIdx.x + 1024] = keys[base + threadIdx.x + 1024];
    __syncthreads();
    for (uint32_t k = k_begin; k <= k_end; k <<= 1) {
        for (uint32_t j = (k == k_begin ? j_begin : k >> 1); j > 0; j >>= 1) {
            // thread t handles the pair (i, i ^ j) with i the lower index
            const uint32_t t = threadIdx.x;
            const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
            const uint32_t l = i | j;
            const uint64_t a = s[i], b = s[l];
            const bool up = ((base + i) & k) == 0;
            if ((a > b) == up) {
                s[i] = b;
                s[l] = a;
            }
            __syncthreads();
        }
    }
    keys[base + threadIdx.x] = s[threadIdx.x];
    keys[base + threadIdx.x + 1024] = s[threadIdx.x + 1024];
}

__global__ __launch_bounds__(kB) void k_gather(const uint64_t* __restrict__ keys, int n, const float* __restrict__ tris,
                                               const int32_t* __restrict__ gid, float* __restrict__ tris_s,
                                               int32_t* __restrict__ gid_s) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const uint32_t i = (uint32_t)keys[k];
#pragma unroll
    for (int c = 0; c < 9; c++) tris_s[(size_t)k * 9 + c] = tris[(size_t)i * 9 + c];
    gid_s[k] = gid[i];
}

__device__ __forceinline__ int delta(const uint64_t* __restrict__ keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    return __clzll((long long)(keys[i] ^ keys[j]));   // keys are unique (index in the low bits)
}

// Inner node i of n - 1 (Karras 2012, Fig. 4). Node ids: inner 0 .. n-2, leaf k = n - 1 + k.
__global__ __launch_bounds__(kB) void k_karras(const uint64_t* __restrict__ keys, int n, int32_t* __restrict__ cl,
                                               int32_t* __restrict__ cr, int32_t* __restrict__ parent,
                                               int32_t* __restrict__ rfirst) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    for (int div = 2;; div <<= 1) {
        const int t = (l + div - 1) / div;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int g = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    const int left = (lo == g) ? (n - 1 + g) : g;
    const int right = (hi == g + 1) ? (n - 1 + g + 1) : g + 1;
    cl[i] = left;
    cr[i] = right;
    parent[left] = i;
    parent[right] = i;
    rfirst[i] = lo;
}

struct Box6 {
    float v[6];
};

__device__ __forceinline__ float ld_coherent(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ int32_t ld_coherent(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bottom-up: boxes (float32, rounded out one ulp per triangle), triangle
// counts, and the size of each subtree after collapsing (<= kMeshLeafMax
// triangles -> one node). The second child to finish climbs to the parent.
__global__ __launch_bounds__(kB) void k_up(const float* __restrict__ tris_s, int n, const int32_t* __restrict__ cl,
                                           const int32_t* __restrict__ cr, const int32_t* __restrict__ parent,
                                           float* box, int32_t* tc, int32_t* sz, int32_t* ht,
                                           uint32_t* __restrict__ flag) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const int id = n - 1 + k;
    const float* q = tris_s + (size_t)k * 9;
    for (int c = 0; c < 3; c++) {
        const float lo = fminf(fminf(q[c], q[3 + c]), q[6 + c]);
        const float hi = fmaxf(fmaxf(q[c], q[3 + c]), q[6 + c]);
        box[(size_t)id * 6 + c] = nextafterf(lo, -INFINITY);
        box[(size_t)id * 6 + 3 + c] = nextafterf(hi, INFINITY);
    }
    tc[id] = 1;
    sz[id] = 1;
    ht[id] = 0;
    int p = parent[id];
    while (p >= 0) {
        __threadfence();
        if (atomicAdd(&flag[p], 1u) == 0) return;   // the sibling is not done yet
        __threadfence();
        const int l = cl[p], r = cr[p];
        for (int c = 0; c < 3; c++) {
            box[(size_t)p * 6 + c] = fminf(ld_coherent(&box[(size_t)l * 6 + c]), ld_coherent(&box[(size_t)r * 6 + c]));
            box[(size_t)p * 6 + 3 + c] =
                fmaxf(ld_coherent(&box[(size_t)l * 6 + 3 + c]), ld_coherent(&box[(size_t)r * 6 + 3 + c]));
        }
        const int t = ld_coherent(&tc[l]) + ld_coherent(&tc[r]);
        tc[p] = t;
        sz[p] = t <= kMeshLeafMax ? 1 : 1 + ld_coherent(&sz[l]) + ld_coherent(&sz[r]);
        ht[p] = 1 + max(ld_coherent(&ht[l]), ld_coherent(&ht[r]));
        p = parent[p];
    }
}

// Each kept node (the root, or a child of an uncollapsed node) walks to the
// root once and finds its depth-first position in all eight orderings (one
// per ray-direction octant): at each ancestor the child visited first is the
// nearer one along that ancestor's split axis (the axis where the children's
// box centres differ most) for the octant's sign on that axis -- pbrt's
// front-to-back rule (bvh.go:683-693 uses dirIsNeg[node.axis] the same way).
// A node whose nearer sibling is on the path comes after that sibling's subtree.
__global__ __launch_bounds__(kB) void k_flatten(int n, const int32_t* __restrict__ cl, const int32_t* __restrict__ cr,
                                                const int32_t* __restrict__ parent,
                                                const int32_t* __restrict__ rfirst, const float* __restrict__ box,
                                                const int32_t* __restrict__ tc, const int32_t* __restrict__ sz,
                                                int n_out, MeshNode* __restrict__ out, int* __restrict__ depth) {
    const int v = blockIdx.x * kB + threadIdx.x;
    if (v >= 2 * n - 1) return;
    const int pv = parent[v];
    if (pv >= 0 && tc[pv] <= kMeshLeafMax) return;   // inside a collapsed leaf
    uint32_t pos[kMeshOrders];
#pragma unroll
    for (int o = 0; o < kMeshOrders; o++) pos[o] = 0;
    int c = v, p = pv, dep = 0;
    while (p >= 0) {
        const int l = cl[p], r = cr[p];
        const int sib = (c == l) ? r : l;
        const uint32_t ssz = (uint32_t)sz[sib];
        float dl[3];
        int a = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            dl[k] = (box[(size_t)l * 6 + k] + box[(size_t)l * 6 + 3 + k]) -
                    (box[(size_t)r * 6 + k] + box[(size_t)r * 6 + 3 + k]);
        if (fabsf(dl[1]) > fabsf(dl[a])) a = 1;
        if (fabsf(dl[2]) > fabsf(dl[a])) a = 2;
#pragma unroll
        for (int o = 0; o < kMeshOrders; o++) {
            const bool neg = (o >> a) & 1;
            const bool left_first = neg ? (dl[a] >= 0) : (dl[a] <= 0);
            const int first = left_first ? l : r;
            pos[o] += 1u + (c == first ? 0u : ssz);
        }
        c = p;
        p = parent[p];
        dep++;
    }
    MeshNode nd;
    for (int k = 0; k < 3; k++) {
        nd.bmin[k] = box[(size_t)v * 6 + k];
        nd.bmax[k] = box[(size_t)v * 6 + 3 + k];
    }
    const int t = tc[v];
    if (t <= kMeshLeafMax) {
        const int first = v >= n - 1 ? v - (n - 1) : rfirst[v];
        nd.leaf = ((uint32_t)first << 3) | (uint32_t)t;
        atomicMax(depth, dep);
    } else {
        nd.leaf = kMeshInterior;
    }
    for (int o = 0; o < kMeshOrders; o++) {
        nd.escape = pos[o] + (uint32_t)sz[v];
        out[(size_t)o * n_out + pos[o]] = nd;
    }
}

// Wide layout (PBRT_MESH_WIDE): one level of the 4-ary tree per launch. Node
// i (binary node bin_of[i]) takes its binary children and opens the highest
// child subtree until it holds four slots, so that every slot is at least two
// binary levels below the node: with the Karras tree's <= 64 levels of inner
// nodes the wide tree has <= 32 levels (kMeshWideLevels). The slots are stored
// in ascending centre order along the axis of their centres' largest spread;
// the level's inner slots get consecutive indices after the level (atomic
// counter), so the tree is laid out level by level, siblings together.
__global__ __launch_bounds__(kB) void k_collapse(int n, const int32_t* __restrict__ cl, const int32_t* __restrict__ cr,
                                                 const float* __restrict__ box, const int32_t* __restrict__ tc,
                                                 const int32_t* __restrict__ ht, int32_t* __restrict__ bin_of,
                                                 uint32_t* __restrict__ par4, uint32_t lvl_begin, uint32_t lvl_end,
                                                 uint32_t* __restrict__ counter, MeshNode4* __restrict__ out) {
    const uint32_t i = lvl_begin + blockIdx.x * kB + threadIdx.x;
    if (i >= lvl_end) return;
    const int v = bin_of[i];
    int s[4] = {v, -1, -1, -1}, ns = 1;
    if (v < n - 1) {
        s[0] = cl[v];
        s[1] = cr[v];
        ns = 2;
    }
    while (ns < 4) {
        int best = -1;
        for (int j = 0; j < ns; j++) {
            if (s[j] >= n - 1) continue;   // a triangle
            if (best < 0 || ht[s[j]] > ht[s[best]] || (ht[s[j]] == ht[s[best]] && tc[s[j]] > tc[s[best]])) best = j;
        }
        if (best < 0) break;
        const int w = s[best];
        s[best] = cl[w];
        s[ns++] = cr[w];
    }
    float c[4][3];
    for (int j = 0; j < ns; j++)
        for (int a = 0; a < 3; a++) c[j][a] = box[(size_t)s[j] * 6 + a] + box[(size_t)s[j] * 6 + 3 + a];
    int axis = 0;
    float spread = -1;
    for (int a = 0; a < 3; a++) {
        float mn = c[0][a], mx = c[0][a];
        for (int j = 1; j < ns; j++) {
            mn = fminf(mn, c[j][a]);
            mx = fmaxf(mx, c[j][a]);
        }
        if (mx - mn > spread) {
            spread = mx - mn;
            axis = a;
        }
    }
    for (int j = 1; j < ns; j++)   // insertion sort by centre along the axis
        for (int k = j; k > 0 && c[k][axis] < c[k - 1][axis]; k--) {
            const int t = s[k];
            s[k] = s[k - 1];
            s[k - 1] = t;
            for (int a = 0; a < 3; a++) {
                const float f = c[k][a];
                c[k][a] = c[k - 1][a];
                c[k - 1][a] = f;
            }
        }
    int nin = 0;
    for (int j = 0; j < ns; j++) nin += s[j] < n - 1;
    uint32_t next = nin ? atomicAdd(counter, (uint32_t)nin) : 0u;
    MeshNode4 nd;
    for (int j = 0; j < 4; j++) {
        for (int a = 0; a < 3; a++) {
            nd.lo[a][j] = j < ns ? box[(size_t)s[j] * 6 + a] : 0.0f;
            nd.hi[a][j] = j < ns ? box[(size_t)s[j] * 6 + 3 + a] : 0.0f;
        }
        if (j >= ns) {
            nd.child[j] = kMeshEmpty;
        } else if (s[j] >= n - 1) {
            nd.child[j] = kMeshTri | (uint32_t)(s[j] - (n - 1));
        } else {
            bin_of[next] = s[j];
            par4[next] = i;
            nd.child[j] = next++;
        }
    }
    nd.parent = par4[i];
    nd.axis = (uint32_t)axis;
    nd.count = (uint32_t)ns;
    nd.pad = 0;
    out[i] = nd;
}

template <class T>
hipError_t dmalloc(T** p, size_t n) {
    return hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
}

}  // namespace

// stages k <= 2048 sort each 2048-key block in LDS (one launch); later
// stages: global passes for strides >= 2048, then the rest in LDS
void bitonic_sort_u64(uint64_t* keys, uint32_t npad, hipStream_t st) {
    hipLaunchKernelGGL(k_bitonic_local, dim3(npad / 2048), dim3(1024), 0, st, keys, 2u, 2048u, 1u);
    for (uint32_t k = 4096; k <= npad; k <<= 1) {
        for (uint32_t j = k >> 1; j >= 2048; j >>= 1)
            hipLaunchKernelGGL(k_bitonic_global, dim3(npad / 1024), dim3(1024), 0, st, keys, k, j);
        hipLaunchKernelGGL(k_bitonic_local, dim3(npad / 2048), dim3(1024), 0, st, keys, k, k, 1024u);
    }
}

void mesh_bvh_free(MeshBuild& b) {
    (void)hipFree(b.nodes);
    (void)hipFree(b.tris);
    (void)hipFree(b.gid);
    (void)hipFree(b.mesh_first);
    (void)hipFree(b.mesh_mat);
    (void)hipFree(b.mesh_rev);
    b = MeshBuild();
}

int mesh_bvh_build(const pbrt_scene_desc* s, hipStream_t st, MeshBuild& out, std::string& err) {
    out = MeshBuild();
    const int nm = s->n_meshes;
    std::vector<int32_t> first((size_t)nm + 1, 0), mat((size_t)nm), rev((size_t)nm);
    int64_t total = 0;
    for (int m = 0; m < nm; m++) {
        const pbrt_mesh_desc& d = s->meshes[m];
        first[(size_t)m] = (int32_t)total;
        mat[(size_t)m] = d.material;
        rev[(size_t)m] = d.reverse_orientation != 0;
        total += d.n_triangles;
    }
    first[(size_t)nm] = (int32_t)total;
    if (total >= (1LL << 29)) {
        err = "too many triangles (leaf slots are 29-bit)";
        return PBRT_E_UNSUPPORTED;
    }
    // gather the triangles (global index order); zero-area ones are never hit
    // (as in oracle/oracle_mesh.c) and stay out of the tree
    std::vector<float> V;
    std::vector<int32_t> G;
    V.reserve((size_t)total * 9);
    G.reserve((size_t)total);
    for (int m = 0; m < nm; m++) {
        const pbrt_mesh_desc& d = s->meshes[m];
        for (int32_t i = 0; i < d.n_triangles; i++) {
            float q[9];
            for (int c = 0; c < 3; c++)
                for (int k = 0; k < 3; k++) q[3 * c + k] = d.p[3 * (size_t)d.indices[3 * (size_t)i + c] + k];
            const V3 a{(double)q[3] - (double)q[0], (double)q[4] - (double)q[1], (double)q[5] - (double)q[2]};
            const V3 b{(double)q[6] - (double)q[0], (double)q[7] - (double)q[1], (double)q[8] - (double)q[2]};
            if (!(len2(cross(a, b)) > 0)) continue;
            V.insert(V.end(), q, q + 9);
            G.push_back(first[(size_t)m] + i);
        }
    }
    const int n = (int)G.size();
    out.n_meshes = nm;
    out.n_tris = n;
#define MB_CHK(x)                                            \
    do {                                                     \
        hipError_t e_ = (x);                                 \
        if (e_ != hipSuccess) {                              \
            err = std::string("mesh BVH: ") + hipGetErrorString(e_); \
            goto fail;                                       \
        }                                                    \
    } while (0)
    {
        float *tris = nullptr, *cen = nullptr, *box = nullptr;
        int32_t *gid = nullptr, *cl = nullptr, *cr = nullptr, *par = nullptr, *rfirst = nullptr, *tc = nullptr,
                *sz = nullptr, *ht = nullptr, *bin_of = nullptr;
        uint32_t *bounds = nullptr, *flag = nullptr, *par4 = nullptr, *counter = nullptr;
        uint64_t* keys = nullptr;
        int* depth = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        // the build's temporaries and events, released on every exit of this
        // scope (success, or an MB_CHK failure's goto fail)
        struct Temps {
            std::vector<void**> bufs;   // the local pointers (nullptr until allocated)
            hipEvent_t* ev[2];
            ~Temps() {
                for (void** b : bufs)
                    if (*b) (void)hipFree(*b);
                for (hipEvent_t* e : ev)
                    if (*e) (void)hipEventDestroy(*e);
            }
        } temps{{(void**)&tris, (void**)&gid, (void**)&cen, (void**)&bounds, (void**)&keys, (void**)&cl, (void**)&cr,
                 (void**)&par, (void**)&rfirst, (void**)&box, (void**)&tc, (void**)&sz, (void**)&flag, (void**)&depth,
                 (void**)&ht, (void**)&bin_of, (void**)&par4, (void**)&counter},
                {&e0, &e1}};
        int npad = 2048;
        while (npad < n) npad <<= 1;
        const unsigned gb = (unsigned)((n + kB - 1) / kB), gpad = (unsigned)(npad / kB);
        int n_out = 0;
        MB_CHK(dmalloc(&out.mesh_first, (size_t)nm + 1));
        MB_CHK(dmalloc(&out.mesh_mat, (size_t)nm));
        MB_CHK(dmalloc(&out.mesh_rev, (size_t)nm));
        MB_CHK(hipMemcpy(out.mesh_first, first.data(), sizeof(int32_t) * first.size(), hipMemcpyHostToDevice));
        if (nm) {
            MB_CHK(hipMemcpy(out.mesh_mat, mat.data(), sizeof(int32_t) * mat.size(), hipMemcpyHostToDevice));
            MB_CHK(hipMemcpy(out.mesh_rev, rev.data(), sizeof(int32_t) * rev.size(), hipMemcpyHostToDevice));
        }
        if (n == 0) return PBRT_OK;
        MB_CHK(hipEventCreate(&e0));
        MB_CHK(hipEventCreate(&e1));
        MB_CHK(dmalloc(&tris, (size_t)n * 9));
        MB_CHK(dmalloc(&gid, (size_t)n));
        MB_CHK(dmalloc(&cen, (size_t)n * 3));
        MB_CHK(dmalloc(&bounds, 6));
        MB_CHK(dmalloc(&keys, (size_t)npad));
        MB_CHK(dmalloc(&out.tris, (size_t)n * 9));
        MB_CHK(dmalloc(&out.gid, (size_t)n));
        MB_CHK(dmalloc(&cl, (size_t)n));
        MB_CHK(dmalloc(&cr, (size_t)n));
        MB_CHK(dmalloc(&par, (size_t)2 * n));
        MB_CHK(dmalloc(&rfirst, (size_t)n));
        MB_CHK(dmalloc(&box, (size_t)(2 * n) * 6));
        MB_CHK(dmalloc(&tc, (size_t)2 * n));
        MB_CHK(dmalloc(&sz, (size_t)2 * n));
        MB_CHK(dmalloc(&ht, (size_t)2 * n));
        MB_CHK(dmalloc(&flag, (size_t)n));
        MB_CHK(dmalloc(&depth, 1));
        MB_CHK(hipMemcpyAsync(tris, V.data(), sizeof(float) * V.size(), hipMemcpyHostToDevice, st));
        MB_CHK(hipMemcpyAsync(gid, G.data(), sizeof(int32_t) * G.size(), hipMemcpyHostToDevice, st));
        {
            const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0};
            MB_CHK(hipMemcpyAsync(bounds, init, sizeof(init), hipMemcpyHostToDevice, st));
        }
        MB_CHK(hipMemsetAsync(par, 0xFF, sizeof(int32_t) * 2 * (size_t)n, st));
        MB_CHK(hipMemsetAsync(flag, 0, sizeof(uint32_t) * (size_t)n, st));
        MB_CHK(hipMemsetAsync(depth, 0, sizeof(int), st));
        MB_CHK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(k_centroids, dim3(gb), dim3(kB), 0, st, tris, n, cen, bounds);
        hipLaunchKernelGGL(k_morton, dim3(gpad), dim3(kB), 0, st, cen, n, npad, bounds, keys);
        // stages k <= 2048 sort each 2048-key block in LDS (one launch); later
        // stages: global passes for strides >= 2048, then the rest in LDS
        bitonic_sort_u64(keys, (uint32_t)npad, st);
        hipLaunchKernelGGL(k_gather, dim3(gb), dim3(kB), 0, st, keys, n, tris, gid, out.tris, out.gid);
        if (n > 1)
            hipLaunchKernelGGL(k_karras, dim3((unsigned)((n - 1 + kB - 1) / kB)), dim3(kB), 0, st, keys, n, cl, cr,
                               par, rfirst);
        hipLaunchKernelGGL(k_up, dim3(gb), dim3(kB), 0, st, out.tris, n, cl, cr, par, box, tc, sz, ht, flag);
        MB_CHK(hipGetLastError());
#if PBRT_MESH_WIDE
        {
            const uint32_t cap = (uint32_t)std::max(n - 1, 1);   // one wide node per kept inner binary node
            const uint32_t one = 1, none = kMeshEmpty;
            MB_CHK(dmalloc(&bin_of, (size_t)cap));
            MB_CHK(dmalloc(&par4, (size_t)cap));
            MB_CHK(dmalloc(&counter, 1));
            MB_CHK(dmalloc(reinterpret_cast<MeshNode4**>(&out.nodes), (size_t)cap));
            MB_CHK(hipMemsetAsync(bin_of, 0, sizeof(int32_t), st));   // the root: binary node 0
            MB_CHK(hipMemcpyAsync(par4, &none, sizeof(uint32_t), hipMemcpyHostToDevice, st));
            MB_CHK(hipMemcpyAsync(counter, &one, sizeof(uint32_t), hipMemcpyHostToDevice, st));
            uint32_t b = 0, e = 1;
            int levels = 0;
            while (b < e) {
                if (++levels > kMeshWideLevels) {
                    err = "mesh BVH: wide tree deeper than 32 levels";
                    mesh_bvh_free(out);
                    return PBRT_E_UNSUPPORTED;
                }
                hipLaunchKernelGGL(k_collapse, dim3((e - b + kB - 1) / kB), dim3(kB), 0, st, n, cl, cr, box, tc, ht,
                                   bin_of, par4, b, e, counter, reinterpret_cast<MeshNode4*>(out.nodes));
                MB_CHK(hipGetLastError());
                uint32_t next = 0;
                MB_CHK(hipMemcpyAsync(&next, counter, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
                MB_CHK(hipStreamSynchronize(st));
                b = e;
                e = next;
            }
            n_out = (int)e;
            out.depth = levels;
        }
#else
        MB_CHK(hipMemcpyAsync(&n_out, sz, sizeof(int32_t), hipMemcpyDeviceToHost, st));   // root = node 0
        MB_CHK(hipStreamSynchronize(st));
        MB_CHK(dmalloc(&out.nodes, (size_t)kMeshOrders * n_out + kMeshPad));
        MB_CHK(hipMemsetAsync(out.nodes + (size_t)kMeshOrders * n_out, 0, sizeof(MeshNode) * kMeshPad, st));
        hipLaunchKernelGGL(k_flatten, dim3((unsigned)((2 * n - 1 + kB - 1) / kB)), dim3(kB), 0, st, n, cl, cr, par,
                           rfirst, box, tc, sz, n_out, out.nodes, depth);
#endif
        MB_CHK(hipEventRecord(e1, st));
        MB_CHK(hipGetLastError());
#if !PBRT_MESH_WIDE
        MB_CHK(hipMemcpyAsync(&out.depth, depth, sizeof(int), hipMemcpyDeviceToHost, st));
#endif
        MB_CHK(hipStreamSynchronize(st));
        {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            out.build_ms = ms;
        }
        out.n_nodes = n_out;
        return PBRT_OK;
    }
fail:
    mesh_bvh_free(out);
    return PBRT_E_HIP;
#undef MB_CHK
}

}  // namespace pbrt
