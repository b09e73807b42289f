// render.hip — host side of the MI355X (gfx950) library: scene upload, launch
// planning and the C ABI of include/pbrt_gpu.h.
//
// Kernels (each family in its own translation unit, k_*.hip; declarations in
// render_kernels.h, shared types and helpers in render_common.h)
//   k_render_exact   EXACT mode: one lane per 16-px tile. The lane replays the
//                    tile's PCG32 stream exactly as pbrt.Render's worker does
//                    (integrator.go:228-289, 311-340): pixel loop, Stratified
//                    StartPixel, samples 1..spp-1, Path.Li / DirectLighting.Li,
//                    NaN guard, FilmTile.AddSample into the tile's film slot.
//   wave pipeline    k_wf_primary (bounce 1 per pixel), k_chain_ci (the
//                    tile's RNG-offset chain), k_paths_ci or the path
//                    wavefront k_pw_* (full paths), k_film (tile films);
//                    THROUGHPUT mode: k_mb_setup instead of the chain.
//   k_dl_*           DirectLighting: pixel-order StartPixel + jump-ahead, one
//                    lane per sample.
//   k_merge_film     Film.MergeFilmTile (film.go:115-132): per output pixel,
//                    RGBToXYZ of every covering tile film in tile-index order.
//   k_intersect[_p]  batch BVH closest-hit / any-hit (bvh.go:659-765).
//
// Everything is float64 with -ffp-contract=off (bit parity with the Go
// reference). The scene is a few KB and is read through the scalar/vector L1.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <functional>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/pbrt_gpu.h"
#include "../../include/pbrt_diag.h"
#include "../../include/pbrt_scene.h"
#include "mesh_bvh.h"
#include "render_kernels.h"

using namespace pbrt;
using namespace pbrtk;


// =============================================================== C ABI
// per-slot chain clocks of the last EXACT frame: durations (the schedule's
// input), and in diagnostics builds start and end clocks (pbrt_gpu_tile_clocks)
#ifdef PBRT_CI_DIAG
constexpr int kTickPlanes = 3;   // durations, start clocks, end clocks
#else
constexpr int kTickPlanes = 1;
#endif

// Experiment knobs (environment), read ONCE when a context is created
// (pbrt_gpu_create), never per launch; defaults are the measured best.
struct Knobs {
    int ci_waves = 0;          // PBRT_CI_WAVES = 1, 2, 4, 8 (0: by tile count)
    int ci_stride = 0;         // PBRT_CI_STRIDE = 1, 2 (0: 2 at one wave per tile, else 1)
    int ci_heavy_waves = 4;    // PBRT_CI_HEAVY_WAVES = 4, 8
    bool ci_light_kw = false;  // PBRT_CI_LIGHT_KW=1: a multi-wave shard's split runs its light tiles at the
                               // shard's waves per tile (not 1), the heavy ones at PBRT_CI_HEAVY_WAVES
    int ci_split8 = 32;        // PBRT_CI_SPLIT8=K: a learned multi-wave Matte shard that fits the wave slots
                               // (no split otherwise: 1/8 of B) runs its K heaviest tiles (at most 1/16 of
                               // them) at 8 waves beside the rest at its waves per tile; 0: off
    int ci_eu = 0;             // PBRT_CI_EU = 2 / 3: the one-wave Matte chain's build (waves/SIMD its registers
                               // are budgeted for); 0: by the workgroup's LDS (ci_eu3_fits)
    int64_t ci_heavy = -1;     // PBRT_CI_HEAVY = K forces the heavy tile count (tests)
    bool ci_split = true;      // PBRT_CI_SPLIT=0
    bool ci_order = true;      // PBRT_CI_ORDER=0
    bool ci_probe = true;      // PBRT_CI_PROBE=0
    bool ci_order_cache = true;// PBRT_CI_ORDER_CACHE=0
    bool sp_window = true;     // PBRT_SP_WINDOW=0: the lane-0 StartPixel replay instead of the windowed one
    int ci_scap = -1;          // PBRT_CI_SCAP=Z: k_chain_ci's statistical speculation cap at Z/10 sigmas (0: off;
                               // -1: the kernel's default, 1.5 sigma for mesh scenes; multi-wave tiles with
                               // next-pixel speculation always use 3)
    int ci_nps = 8;            // PBRT_CI_NPS=K: next-pixel speculation in multi-wave k_chain_ci tiles from K
                               // samples before a pixel's end (0: off)
    int paths_overlap = 5;     // PBRT_PATHS_OVERLAP=K: a split frame's path stage runs in K chunks of the
                               // tiles in their chains' completion order, each released when its tiles'
                               // chains have ended (render_enqueue; 0: off, the path stage after the chains)
    bool paths_overlap_all = true;    // PBRT_PATHS_OVERLAP_ALL=0: the completion-driven path stage only for
                               // split frames (measured on: C 5056 -> 4603 ms, G 495 -> 472 ms, the
                               // N=8 shards' max 128.6 -> 119.7 ms)
    bool gate_hold = false;    // PBRT_GATE_HOLD=1 (tests): the light chain launch waits for the path stage,
                               // as a dispatcher that serialises kernels across streams may order them;
                               // k_gate's stall exit and the re-render recover the frame
    bool paths_s1d_lds = false;// PBRT_PATHS_S1D=lds
    int paths_ci = -1;         // PBRT_PATHS_CI = 0, 2, 4, 8 (-1: auto)
    int paths_wf = -1;         // PBRT_PATHS_WF = 0 / 1 (-1: mesh scenes)
    bool pw_sort = false;      // PBRT_PW_SORT=1
    double pw_gb = 24.0;       // PBRT_PW_GB
    double wave_buffer_gb = 0; // PBRT_WAVE_BUFFER_GB (0: min(96 GB, half the free HBM))
    bool ci_dense = false;     // PBRT_CI_DENSE=1 (builds with -DPBRT_CI_DENSE_WALK): k_chain_ci's closest hit by
                               // bvh_walk_dense (bit-exact; slower on B)
    int cull_group = 4;        // PBRT_CULL_GROUP: leaves per culling group
    int cull_min = 2;          // PBRT_CULL_MIN
    bool cull_groups = true;   // PBRT_CULL_GROUPS=0
    static Knobs from_env() {
        Knobs k;
        auto ival = [](const char* n, int& out) { if (const char* e = getenv(n)) out = atoi(e); };
        if (const char* e = getenv("PBRT_CI_WAVES")) {
            const int v = atoi(e);
            if (v == 1 || v == 2 || v == 4 || v == 8) k.ci_waves = v;
        }
        if (const char* e = getenv("PBRT_CI_STRIDE")) {
            const int v = atoi(e);
            if (v == 1 || v == 2) k.ci_stride = v;
        }
        if (const char* e = getenv("PBRT_CI_HEAVY_WAVES")) k.ci_heavy_waves = atoi(e) == 8 ? 8 : 4;
        if (const char* e = getenv("PBRT_CI_LIGHT_KW")) k.ci_light_kw = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_SPLIT8")) k.ci_split8 = std::max(0, atoi(e));
        if (const char* e = getenv("PBRT_CI_EU")) k.ci_eu = (atoi(e) == 2 || atoi(e) == 3) ? atoi(e) : 0;
        if (const char* e = getenv("PBRT_CI_HEAVY")) k.ci_heavy = (int64_t)atoll(e);
        if (const char* e = getenv("PBRT_CI_SPLIT")) k.ci_split = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_DENSE")) k.ci_dense = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_ORDER")) k.ci_order = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_PROBE")) k.ci_probe = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_ORDER_CACHE")) k.ci_order_cache = atoi(e) != 0;
        if (const char* e = getenv("PBRT_SP_WINDOW")) k.sp_window = atoi(e) != 0;
        if (const char* e = getenv("PBRT_CI_NPS")) k.ci_nps = std::max(0, atoi(e));
        if (const char* e = getenv("PBRT_CI_SCAP")) k.ci_scap = std::max(-1, atoi(e));
        if (const char* e = getenv("PBRT_PATHS_OVERLAP")) k.paths_overlap = std::min(std::max(0, atoi(e)), 16);
        if (const char* e = getenv("PBRT_PATHS_OVERLAP_ALL")) k.paths_overlap_all = atoi(e) != 0;
        if (const char* e = getenv("PBRT_GATE_HOLD")) k.gate_hold = atoi(e) != 0;
        if (const char* e = getenv("PBRT_PATHS_S1D")) k.paths_s1d_lds = std::strcmp(e, "lds") == 0;
        if (const char* e = getenv("PBRT_PATHS_CI")) {
            const int v = atoi(e);
            if (v == 0 || v == 2 || v == 4 || v == 8) k.paths_ci = v;
        }
        if (const char* e = getenv("PBRT_PATHS_WF")) k.paths_wf = atoi(e) == 1 ? 1 : 0;
        if (const char* e = getenv("PBRT_PW_SORT")) k.pw_sort = atoi(e) == 1;
        if (const char* e = getenv("PBRT_PW_GB")) k.pw_gb = atof(e) > 0 ? atof(e) : k.pw_gb;
        if (const char* e = getenv("PBRT_WAVE_BUFFER_GB")) k.wave_buffer_gb = atof(e) > 0 ? atof(e) : 0;
        if (const char* e = getenv("PBRT_CULL_GROUP")) k.cull_group = std::max(2, atoi(e));
        if (const char* e = getenv("PBRT_CULL_MIN")) k.cull_min = std::max(0, atoi(e));
        int cg = 1;
        ival("PBRT_CULL_GROUPS", cg);
        k.cull_groups = cg != 0;
        return k;
    }
};

struct pbrt_gpu_ctx {
    Knobs knobs;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // heavy/light split of k_chain_ci: the heaviest tiles with 4 waves each on
    // the main stream, the rest on stream2, concurrently
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_split = nullptr, ev_join = nullptr;
    // PBRT_PATHS_OVERLAP: a high-priority stream for the light chain launch, the
    // events of the completion-driven path stage, and k_chain_ci's progress record
    // (layout at kProgHead)
    hipStream_t stream3 = nullptr;
    hipEvent_t ev_l2 = nullptr, ev_p1 = nullptr;
    int64_t ov_done = 0;                 // slots whose path stage was launched beside the chains
    uint32_t* d_prog = nullptr;
    int64_t prog_cap = 0;
    // a frame whose k_gate saw the chains stand still (a dispatcher that serialises
    // kernels across streams) is rendered again without the overlap; two such
    // frames in a row turn the overlap off for the context
    pbrt_render_desc last_rd{};
    double* last_film_device = nullptr;
    int ov_stalls = 0;
    bool ov_retry = false;
    MeshBuild mesh;                      // triangle meshes + their LBVH (extension)
    int64_t heavy_k = 0;                 // slots at the front of h_slot_order that get 4 waves
    int ci_wps = 2;                      // waves/SIMD of the last one-wave k_chain_ci launch (3 or 2)
    int64_t last_heavy = 0;              // heavy slots of the last EXACT launch (0: no split)
    std::vector<uint32_t> h_last_ticks;  // per-slot chain ticks of the last EXACT frame
    std::vector<uint8_t> h_slot_kw;      // waves per tile each slot ran with in the last frame
    double* film_target = nullptr;   // caller buffer of the last render_async_into
    int lanes_per_wave = 64;
    bool lanes_per_wave_set = false;
    int min_waves = 1;      // amdgpu_waves_per_eu variant of k_render_exact
    int occ_req = 0;        // opts.occupancy as given (0 = each kernel's default)
    int kernel_req = PBRT_KERNEL_AUTO;
    int last_kernel = 0;    // PBRT_KERNEL_SERIAL / PBRT_KERNEL_WAVE
    PcgJump* d_jump = nullptr;
    pbrt_distribution_desc host_dist;
    // wave-parallel path (k_wf_primary, k_chain_ci, k_paths_ci / k_pw_*, k_film)
    ChainLayout lay{};
    bool use_spec = false;
    unsigned char* d_wave = nullptr;   // per-batch pixel records, stratified values, RNG states, L
    size_t wave_cap = 0;
    int64_t wave_batch = 0;            // tile slots per batch
    int tiles_per_wave = 1;            // k_chain_ci lane groups per wave (64 / lanes per tile)
    std::vector<hipEvent_t> bev;       // per batch: before the chain, after the chain, after the paths
    int n_batches = 0;
    int n_simd = 1024;                 // SIMDs of the device (4 per CU)
    size_t lds_per_block = 65536;      // the device's LDS limit per workgroup (sharedMemPerBlock)
    size_t lds_per_cu = 160 * 1024;    // LDS of a CU (maxSharedMemoryPerMultiProcessor)
    WaveBufs wb{};
    bool use_ci = false;   // the Path chain stage (k_chain_ci)
    bool use_dl = false;   // DirectLighting on k_dl_setup / k_dl_samples
    ChainLayout lay_ci{};
    // device scene
    pbrt_shape_desc* d_shapes = nullptr;
    pbrt_material_desc* d_materials = nullptr;
    pbrt_primitive_desc* d_prims = nullptr;
    DevNode* d_nodes = nullptr;
    uint32_t* d_order = nullptr;     // [8][n_nodes] preorder visit tables, then [8][n_nodes] leaf lists (dev_order)
    double* d_groups = nullptr;      // leaf culling groups (cull_groups)
    uint32_t* d_gmasks = nullptr;
    int n_groups = 0;
    std::vector<int> h_node_prims;   // nPrimitives per node (leaf count for DevScene)
    DevPrim* d_fprims = nullptr;
    pbrt_light_desc* d_lights = nullptr;
    pbrt_camera_desc* d_camera = nullptr;
    pbrt_film_desc* d_film = nullptr;
    pbrt_distribution_desc* d_dist = nullptr;
    pbrt_scene_desc host_scene;   // counts + film/camera (pointer fields are not kept)
    std::vector<pbrt_light_desc> host_lights;
    bool non_matte = false;       // Mirror, Glass or OrenNayar material: kX wave kernels or the serial kernel
    bool rough_glass = false;     // a Glass material with roughness: serial kernel only
    // per-render buffers (grown on demand)
    double* d_films = nullptr;
    size_t films_cap = 0;
    double* d_s1d = nullptr;
    size_t s1d_cap = 0;
    PanicRec* d_panics = nullptr;
    size_t panics_cap = 0;
    Counters* d_ctr = nullptr;
    // k_chain_ci heaviest-first schedule: per-slot chain time of the last
    // EXACT frame (wall_clock64 ticks) and the slot order derived from it
    uint32_t* d_ticks = nullptr;         // [kTickPlanes][slots]
    std::vector<uint32_t> h_tick_clocks; // diagnostics builds: [start | end] clocks of the last frame
    uint32_t* d_slot_order = nullptr;
    int64_t ticks_cap = 0;
    std::vector<uint32_t> h_slot_order;
    // path wavefront (k_pw_*, PBRT_PATHS_WF=1): path records, queues, counters,
    // bounce-1 light estimates, per-pixel panic keys (grown on demand)
    unsigned char* d_pw = nullptr;
    size_t pw_cap = 0;
    // cold-frame schedule (k_tile_cost): per-slot features and sort keys
    float* d_cost = nullptr;
    uint64_t* d_cost_keys = nullptr;
    int64_t cost_cap = 0, cost_n = 0;
    bool probed = false;               // the last EXACT frame ran the cost probe
    uint64_t order_key = 0, ticks_key = 0;
    uint64_t scene_hash = 0;           // content hash of the scene (process-wide schedule cache)
    int sched_src = 0;                 // schedule of the last EXACT frame: PBRT_SCHED_* (pbrt_diag.h)
    int64_t ticks_n = 0;
    bool ticks_pending = false;
    double* d_out = nullptr;
    size_t out_cap = 0;
    // last render
    RenderParams rp{};
    bool rendered = false;
    // cancellation (pbrt_gpu_cancel): a flag in fine-grained host memory the
    // kernels poll; it belongs to the render in flight (render_async entry to
    // synchronize) and is cleared when that render ends, so a cancel never
    // outlives its render and never reaches the next one
    std::mutex cancel_mu;
    bool in_flight = false;
    bool cancel_req = false;
    int* h_cancel = nullptr;   // hipHostMalloc (coherent, mapped)
    int* d_cancel = nullptr;   // its device address
    int* d_cancel_seen = nullptr;   // device-memory copy the kernels publish (reset per render)
    std::string err;
    std::chrono::steady_clock::time_point t_start;
};

namespace {

// Process-wide schedule cache. internal/render/server.go:29-164 builds a fresh
// scene, integrator and renderer for every request, so each request's context
// would otherwise start from the cold-frame probe. A context that measured a
// frame stores its heaviest-first slot order here, keyed by the scene's content
// hash and the frame's schedule key; a fresh context on the same scene and
// configuration starts from it. Only the schedule changes, never a result, so a
// hash collision could only cost speed.
struct SchedEntry {
    std::vector<uint32_t> order;   // slot order, heaviest first
    int64_t heavy_k = 0;           // slots at its front that run at 4 waves
};
std::mutex g_sched_mu;
std::unordered_map<uint64_t, SchedEntry> g_sched;
constexpr size_t kSchedCacheMax = 64;   // configurations kept (a full frame's order is 32 KB)

uint64_t fnv_bytes(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}
// Content hash of a scene descriptor: every analytic record, the camera and
// film, and per mesh its sizes plus up to 4096 evenly spread vertices and
// triangles (a mesh of 10M triangles is not hashed whole on every create).
uint64_t scene_content_hash(const pbrt_scene_desc* s) {
    uint64_t h = 1469598103934665603ull;
    const int32_t counts[] = {s->n_shapes, s->n_materials, s->n_prims, s->n_nodes, s->n_lights, s->n_meshes};
    h = fnv_bytes(h, counts, sizeof(counts));
    if (s->n_shapes > 0) h = fnv_bytes(h, s->shapes, sizeof(pbrt_shape_desc) * (size_t)s->n_shapes);
    if (s->n_materials > 0) h = fnv_bytes(h, s->materials, sizeof(pbrt_material_desc) * (size_t)s->n_materials);
    if (s->n_prims > 0) h = fnv_bytes(h, s->prims, sizeof(pbrt_primitive_desc) * (size_t)s->n_prims);
    if (s->n_nodes > 0) h = fnv_bytes(h, s->nodes, sizeof(pbrt_bvh_node) * (size_t)s->n_nodes);
    if (s->n_lights > 0) h = fnv_bytes(h, s->lights, sizeof(pbrt_light_desc) * (size_t)s->n_lights);
    h = fnv_bytes(h, &s->camera, sizeof(s->camera));
    h = fnv_bytes(h, &s->film, sizeof(s->film));
    for (int m = 0; m < s->n_meshes && s->meshes; m++) {
        const pbrt_mesh_desc& md = s->meshes[m];
        const int32_t mc[] = {md.n_vertices, md.n_triangles, md.material, md.reverse_orientation};
        h = fnv_bytes(h, mc, sizeof(mc));
        const int64_t nv = md.n_vertices, nt = md.n_triangles;
        for (int64_t i = 0, st = std::max<int64_t>(1, nv / 4096); md.p && i < nv; i += st)
            h = fnv_bytes(h, md.p + 3 * i, 3 * sizeof(float));
        for (int64_t i = 0, st = std::max<int64_t>(1, nt / 4096); md.indices && i < nt; i += st)
            h = fnv_bytes(h, md.indices + 3 * i, 3 * sizeof(int32_t));
    }
    return h;
}
uint64_t sched_cache_key(const pbrt_gpu_ctx* c, uint64_t skey) {
    uint64_t h = fnv_bytes(c->scene_hash, &skey, sizeof(skey));
    return fnv_bytes(h, &c->n_simd, sizeof(c->n_simd));   // the device's size shapes the split
}
bool sched_cache_get(const pbrt_gpu_ctx* c, uint64_t skey, int64_t nb, SchedEntry& out) {
    std::lock_guard<std::mutex> lk(g_sched_mu);
    auto it = g_sched.find(sched_cache_key(c, skey));
    if (it == g_sched.end() || (int64_t)it->second.order.size() != nb) return false;
    out = it->second;
    return true;
}
void sched_cache_put(const pbrt_gpu_ctx* c, uint64_t skey, const std::vector<uint32_t>& order, int64_t heavy_k) {
    std::lock_guard<std::mutex> lk(g_sched_mu);
    if (g_sched.size() >= kSchedCacheMax && !g_sched.count(sched_cache_key(c, skey))) g_sched.clear();
    SchedEntry& e = g_sched[sched_cache_key(c, skey)];
    e.order = order;
    e.heavy_k = heavy_k;
}

int set_err(pbrt_gpu_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}
#define HIPCHK(ctx, call)                                                                            \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return set_err(ctx, PBRT_E_HIP, std::string(#call ": ") + hipGetErrorString(e_));      \
    } while (0)

template <class T>
int upload(pbrt_gpu_ctx* c, T** dst, const T* src, size_t n) {
    if (n == 0) n = 1;   // keep a valid pointer for empty arrays
    HIPCHK(c, hipMalloc((void**)dst, sizeof(T) * n));
    if (src) HIPCHK(c, hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice));
    return PBRT_OK;
}
template <class T>
int ensure(pbrt_gpu_ctx* c, T** buf, size_t* cap, size_t n) {
    if (*cap >= n && *buf) return PBRT_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    HIPCHK(c, hipMalloc((void**)buf, sizeof(T) * (n ? n : 1)));
    *cap = n;
    return PBRT_OK;
}

DevScene dev_scene(const pbrt_gpu_ctx* c, bool with_dist) {
    DevScene s;
    s.shapes = c->d_shapes;
    s.materials = c->d_materials;
    s.prims = c->d_prims;
    s.nodes = c->d_nodes;
    s.order = c->d_order;
    s.fprims = c->d_fprims;
    s.lights = c->d_lights;
    s.camera = c->d_camera;
    s.film = c->d_film;
    s.dist = with_dist ? c->d_dist : nullptr;
    s.n_prims = c->host_scene.n_prims;
    s.n_nodes = c->host_scene.n_nodes;
    s.n_lights = c->host_scene.n_lights;
    s.use_lds_nodes = 0;
    s.n_leaves = 0;
    for (int i = 0; i < c->host_scene.n_nodes; i++) s.n_leaves += c->h_node_prims[i] > 0;
    s.mesh = c->mesh.view();
    s.groups = c->d_groups;
    s.gmasks = c->d_gmasks;
    s.n_groups = c->n_groups;
    s.cancel = c->d_cancel;
    s.cancel_seen = c->d_cancel_seen;
    // bvh_walk_dense: culling groups over a tree of one primitive per leaf, no meshes
    s.dense_ok = c->knobs.ci_dense && s.n_groups > 0 && s.n_leaves == s.n_prims && s.mesh.n_nodes == 0 &&
                 s.n_nodes <= kLdsNodes;
    return s;
}

// The scene view a launch passes, tagged with its kernel's counter set for
// the mesh-traversal counting build (PBRT_MESH_COUNT; ignored otherwise):
// 1 k_wf_primary, 2 k_chain_ci, 3 k_paths_ci / k_pw_* EXACT, 4 k_mb_setup,
// 5 k_paths_ci / k_pw_* THROUGHPUT, 6 k_render_exact, 7 k_intersect.
DevScene with_slot(DevScene s, int slot) {
    s.mesh.count_slot = slot;
    return s;
}

std::vector<DevNode> dev_nodes(const pbrt_scene_desc* s) {
    std::vector<DevNode> v((size_t)(s->n_nodes > 0 ? s->n_nodes : 1));
    std::memset(v.data(), 0, v.size() * sizeof(DevNode));
    for (int i = 0; i < s->n_nodes; i++) {
        const pbrt_bvh_node& n = s->nodes[i];
        for (int k = 0; k < 3; k++) {
            v[i].bmin[k] = n.bmin[k];
            v[i].bmax[k] = n.bmax[k];
        }
        v[i].offset = n.offset;
        v[i].nprims_axis = (uint32_t)n.n_prims | ((uint32_t)n.axis << 16);
    }
    return v;
}

// Preorder visit tables of the BVH, one per ray-direction octant (bvh_walk,
// pbrt_path.h). Node i's children: i + 1 and nodes[i].offset; the reference
// visits offset first when the direction along nodes[i].axis is negative
// (bvh.go:693-703). depth = far children pending on the reference's stack.
// Returns false if the node array is not a tree in that depth-first layout.
bool dev_order(const pbrt_scene_desc* s, std::vector<uint32_t>& out) {
    const int n = s->n_nodes;
    out.assign((size_t)16 * (n > 0 ? n : 1), 0u);   // [8][n] preorder, then [8][n] leaves in preorder
    if (n == 0) return true;
    struct Item { uint32_t node, depth; int64_t slot; };   // slot: table index whose skip this item sets (-1: none)
    for (int oct = 0; oct < 8; oct++) {
        uint32_t* t = out.data() + (size_t)oct * n;
        std::vector<Item> st;
        std::vector<int64_t> open;   // table indices of interior nodes whose skip is still unknown
        int k = 0;
        st.push_back({0u, 0u, -1});
        while (!st.empty()) {
            Item it = st.back();
            st.pop_back();
            if (it.slot >= 0) {   // marker: the subtree of table entry `slot` ends here
                t[it.slot] |= (uint32_t)k << 16;
                continue;
            }
            if (k >= n || it.node >= (uint32_t)n) return false;
            const pbrt_bvh_node& nd = s->nodes[it.node];
            const int idx = k++;
            const bool interior = nd.n_prims == 0;
            t[idx] = it.node | ((interior && it.depth >= 64) ? kOrdOverflow : 0u);
            if (!interior) {
                t[idx] |= (uint32_t)(idx + 1) << 16;
                continue;
            }
            const bool neg = (oct >> nd.axis) & 1;
            const uint32_t near_node = neg ? nd.offset : it.node + 1, far_node = neg ? it.node + 1 : nd.offset;
            st.push_back({0u, 0u, (int64_t)idx});            // after both subtrees: set skip
            st.push_back({far_node, it.depth, -1});           // visited after the near subtree
            st.push_back({near_node, it.depth + 1, -1});      // far child pending on the stack
        }
        if (k != n) return false;
        int nl = 0;
        for (int i = 0; i < n; i++) {
            const uint32_t node = t[i] & kOrdNode;
            if (s->nodes[node].n_prims > 0) out[(size_t)8 * n + (size_t)oct * n + nl++] = node;
        }
    }
    return true;
}

// Leaf culling groups of an LDS-staged tree of <= 32 leaves (bvh_walk_analytic): leaves whose
// box diagonal exceeds half the root's (the README floor and wall disks) and
// singletons are tested unconditionally; the others are split recursively at
// the median of their box centres along the widest axis into groups of <= 8
// (the README's three rows of seven spheres become row segments). A group's
// box is the exact union of its members' boxes. Output: boxes [G][6], then per
// octant [G + 1] masks over the octant's leaf preorder positions (last: the
// unconditional leaves). G = 0 (no culling) when the tree is not LDS-staged
// or the grouping needs more than kMaxCullGroups groups.
int cull_groups(const Knobs& kn, const pbrt_scene_desc* s, const std::vector<uint32_t>& order, std::vector<double>& boxes,
                std::vector<uint32_t>& masks) {
    boxes.clear();
    masks.clear();
    const int n = s->n_nodes;
    if (n == 0 || n > kLdsNodes) return 0;
    std::vector<int> leaves;
    for (int i = 0; i < n; i++)
        if (s->nodes[i].n_prims > 0) leaves.push_back(i);
    if (leaves.size() > 32) return 0;
    auto diag2 = [&](int i) {
        double d = 0;
        for (int k = 0; k < 3; k++) d += (s->nodes[i].bmax[k] - s->nodes[i].bmin[k]) * (s->nodes[i].bmax[k] - s->nodes[i].bmin[k]);
        return d;
    };
    const double root = diag2(0);
    std::vector<int> rest;
    std::vector<int> group_of((size_t)n, -1);   // -1: unconditional
    for (int v : leaves)
        if (!(diag2(v) > 0.25 * root)) rest.push_back(v);
    std::vector<std::vector<int>> groups;
    // leaves per group at most: 4 measured best on config B (chain 420 -> 404 ms against 8;
    // 2: 450, 3: 403, 5: 418, 16: 492; profiles/r02/cull_group_ab.json). PBRT_CULL_GROUP overrides.
    const size_t gmax = (size_t)kn.cull_group;
    std::function<void(std::vector<int>)> split = [&](std::vector<int> g) {
        if (g.size() <= gmax) {
            if (g.size() > 1) groups.push_back(g);
            return;
        }
        double lo[3] = {kInf, kInf, kInf}, hi[3] = {-kInf, -kInf, -kInf};
        auto cen = [&](int v, int k) { return 0.5 * (s->nodes[v].bmin[k] + s->nodes[v].bmax[k]); };
        for (int v : g)
            for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], cen(v, k)); hi[k] = std::max(hi[k], cen(v, k)); }
        int a = 0;
        for (int k = 1; k < 3; k++)
            if (hi[k] - lo[k] > hi[a] - lo[a]) a = k;
        std::stable_sort(g.begin(), g.end(), [&](int x, int y) { return cen(x, a) < cen(y, a); });
        const size_t h = g.size() / 2;
        split(std::vector<int>(g.begin(), g.begin() + (long)h));
        split(std::vector<int>(g.begin() + (long)h, g.end()));
    };
    if (!rest.empty()) split(rest);
    const int G = (int)groups.size();
    // worth it only when the groups can skip a fair share of the leaf tests
    // (README: 21 of 23 leaves grouped; Cornell: 2 of 8, not grouped)
    const int min_frac2 = kn.cull_min;   // grouped leaves must be at least half of all (PBRT_CULL_MIN=0: any)
    if (G == 0 || G > kMaxCullGroups || min_frac2 * (int)rest.size() < (int)leaves.size()) return 0;
    boxes.assign((size_t)G * 6, 0.0);
    for (int gi = 0; gi < G; gi++) {
        for (int k = 0; k < 3; k++) {
            boxes[(size_t)gi * 6 + k] = kInf;
            boxes[(size_t)gi * 6 + 3 + k] = -kInf;
        }
        for (int v : groups[(size_t)gi]) {
            group_of[(size_t)v] = gi;
            for (int k = 0; k < 3; k++) {
                boxes[(size_t)gi * 6 + k] = std::min(boxes[(size_t)gi * 6 + k], s->nodes[v].bmin[k]);
                boxes[(size_t)gi * 6 + 3 + k] = std::max(boxes[(size_t)gi * 6 + 3 + k], s->nodes[v].bmax[k]);
            }
        }
    }
    masks.assign((size_t)8 * (G + 1), 0u);
    const int nl = (int)leaves.size();
    for (int oct = 0; oct < 8; oct++)
        for (int j = 0; j < nl; j++) {
            const uint32_t node = order[(size_t)8 * n + (size_t)oct * n + (size_t)j];
            const int gi = group_of[node];
            masks[(size_t)oct * (G + 1) + (size_t)(gi < 0 ? G : gi)] |= 1u << j;
        }
    return G;
}

std::vector<DevPrim> dev_prims(const pbrt_scene_desc* s) {
    std::vector<DevPrim> v((size_t)(s->n_prims > 0 ? s->n_prims : 1));
    std::memset(v.data(), 0, v.size() * sizeof(DevPrim));
    for (int i = 0; i < s->n_prims; i++) {
        const pbrt_primitive_desc& p = s->prims[i];
        v[i].shape = s->shapes[p.shape];
        v[i].prim_to_world = p.prim_to_world;
        v[i].kind = p.kind;
        v[i].material = p.material;
        v[i].prim_identity = is_identity(p.prim_to_world.m) ? 1 : 0;
        v[i].fast = xf_fast_kind(p.prim_to_world.m_inv) | xf_fast_kind(v[i].shape.object_to_world.m_inv) << 8;
    }
    return v;
}

int validate_scene(const pbrt_scene_desc* s) {
    if (!s) return PBRT_E_INVALID;
    if (s->n_prims < 0 || s->n_nodes < 0 || s->n_lights < 0 || s->n_shapes < 0 || s->n_materials < 0)
        return PBRT_E_INVALID;
    if (s->n_nodes > 32767) return PBRT_E_UNSUPPORTED;   // 15-bit node index in the preorder tables
    for (int i = 0; i < s->n_prims; i++) {
        const pbrt_primitive_desc& p = s->prims[i];
        if (p.shape < 0 || p.shape >= s->n_shapes || p.material < 0 || p.material >= s->n_materials)
            return PBRT_E_INVALID;
        if (p.kind != PBRT_PRIM_GEOMETRIC && p.kind != PBRT_PRIM_TRANSFORMED) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_shapes; i++)
        if (s->shapes[i].type != PBRT_SHAPE_SPHERE && s->shapes[i].type != PBRT_SHAPE_DISK) return PBRT_E_UNSUPPORTED;
    for (int i = 0; i < s->n_nodes; i++) {
        const pbrt_bvh_node& n = s->nodes[i];
        if (n.n_prims > 0 && (int64_t)n.offset + n.n_prims > s->n_prims) return PBRT_E_INVALID;
        if (n.n_prims == 0 && (n.offset >= (uint32_t)s->n_nodes || n.axis > 2)) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_materials; i++)
        if (s->materials[i].type < PBRT_MAT_MATTE || s->materials[i].type > PBRT_MAT_GLASS) return PBRT_E_UNSUPPORTED;
    if (s->n_meshes < 0 || (s->n_meshes > 0 && !s->meshes)) return PBRT_E_INVALID;
    for (int i = 0; i < s->n_meshes; i++) {
        const pbrt_mesh_desc& m = s->meshes[i];
        if (m.n_vertices < 0 || m.n_triangles < 0 || m.material < 0 || m.material >= s->n_materials ||
            (m.n_triangles > 0 && (!m.p || !m.indices)))
            return PBRT_E_INVALID;
        for (int64_t k = 0; k < 3 * (int64_t)m.n_triangles; k++)
            if (m.indices[k] < 0 || m.indices[k] >= m.n_vertices) return PBRT_E_INVALID;
    }
    for (int i = 0; i < s->n_lights; i++) {
        const pbrt_light_desc& l = s->lights[i];
        if (l.type < PBRT_LIGHT_POINT || l.type > PBRT_LIGHT_DIFFUSE_AREA) return PBRT_E_UNSUPPORTED;
        if (l.type == PBRT_LIGHT_DIFFUSE_AREA &&
            (l.shape < 0 || l.shape >= s->n_shapes || s->shapes[l.shape].type != PBRT_SHAPE_SPHERE))
            return PBRT_E_UNSUPPORTED;
    }
    const pbrt_film_desc& f = s->film;
    if (f.crop_max_x <= f.crop_min_x || f.crop_max_y <= f.crop_min_y) return PBRT_E_INVALID;
    return PBRT_OK;
}

const PcgJump& pcg_jump_table() {
    static PcgJump J = [] {
        PcgJump t;
        uint64_t a = 0x5851f42d4c957f2dULL, b = 1;   // one step: s' = a*s + inc*1
        for (int i = 0; i < 64; i++) {
            t.a[i] = a;
            t.b[i] = b;
            b = b * (a + 1);   // two applications of the 2^i jump
            a = a * a;
        }
        return t;
    }();
    return J;
}

int paths_ci_pixels(const pbrt_gpu_ctx* c, const RenderParams& rp);
bool paths_wf_enabled(const pbrt_gpu_ctx* c);
// Can the wave-parallel kernels replay this render exactly? (conditions: pbrt_spec.h)
#ifndef PBRT_SP_SERIAL_KB
// above this many KB of raw StartPixel draws, StartPixel runs on one lane and
// its buffers leave LDS (build option). 4: config C's 256-spp pixels (9.5 KB
// of draws) then cost a k_chain_ci workgroup 11 KB of LDS instead of 27, 12
// workgroups share a CU and the chain runs the 3-wave build: C 6.50 -> 5.14 s
// (a pixel's serial StartPixel, ~20 us, is under 0.5% of a C tile's chain)
#define PBRT_SP_SERIAL_KB 4
#endif
#ifndef PBRT_SP_WINDOW_KB
#define PBRT_SP_WINDOW_KB 6   // LDS for the windowed StartPixel's picks, permutations and draw ring (build option)
#endif
#ifndef PBRT_CI_STAGE_KB
#define PBRT_CI_STAGE_KB 8   // k_chain_ci stages StartPixel's stratified values in LDS up to this (build option)
#endif
bool wave_eligible(const pbrt_gpu_ctx* c, const pbrt_render_desc* rd, const RenderParams& rp, ChainLayout& L,
                   ChainLayout& Lci) {
    if (rd->flags & PBRT_FLAG_PANIC_FIDELITY) return false;   // the serial kernel traces the extra rays
    const bool dl = rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING;
    // Mirror, smooth Glass and OrenNayar: Path renders run the kX instantiations
    // of the wave pipeline (trajectories and paths over BSDFX, with etaScale):
    // k_chain_ci for LDS-staged trees, then k_paths_ci (P = 4, 8) or the path
    // wavefront (mesh scenes); rough glass (whose every BSDF sample panics) and
    // larger trees stay on the serial kernel
    // DirectLighting over these materials runs k_dl_samples<kX> (the recursion per
    // sample; maxDepth <= 64 as the serial kernel), rough glass stays serial
    if (c->non_matte && (c->rough_glass || (dl && rd->max_depth > 64) ||
                         (!dl && (c->host_scene.n_nodes > kLdsNodes ||
                                  (!paths_wf_enabled(c) && paths_ci_pixels(c, rp) > 0 && paths_ci_pixels(c, rp) < 4)))))
        return false;
    if (dl) {   // k_dl_*: the camera ray must be per pixel (pFilm stratified; pLens stratified or unused)
        if (rd->n_dims < 1 || (rd->n_dims < 2 && c->host_scene.camera.lens_radius > 0)) return false;
    } else if (rd->integrator != PBRT_INTEGRATOR_PATH || rd->max_depth > 2048) {
        return false;   // D < 2^32
    } else if (rd->n_dims < 2 && !(rd->n_dims == 1 && c->host_scene.camera.lens_radius == 0)) {
        // the camera ray must be the pixel's (k_wf_primary): pFilm stratified
        // (n_dims >= 1), and pLens stratified (n_dims >= 2) or unused (a pinhole)
        return false;
    }
    const int nl = c->host_scene.n_lights;
    if (!dl && nl > kMaxCachedLights) return false;
    if (!dl && nl > 0) {
        const pbrt_distribution_desc& d = c->host_dist;
        if (!(d.func_int > 0)) return false;
        for (int i = 0; i < d.count; i++)
            if (!(d.func[i] > 0)) return false;   // a zero-pdf light changes the draw count
    }
    // k_film stages the tile film's running sums and a run of source pixels in LDS
    // (any filter radius below the tile size: footprints beyond 2x2 included)
    // (+ its static per-run nvalid array, k_frame.hip)
    if ((size_t)film_lds_bytes(rp) + kFilmThreads * sizeof(int) > c->lds_per_block) return false;
    const int64_t n = rp.spp, nd = rp.ndims;
    if (n > 4096 || nd * n > 8192) return false;
    int64_t off = 0;
    auto put = [&](int64_t bytes) {
        int64_t o = off;
        off += (bytes + 15) & ~int64_t(15);
        return (int)o;
    };
    L.s1d = put(nd * n * 8);
    L.other = put(nd * n * 2);
    L.sbuf = put(kWave * 8);
    L.dbuf = put(kWave * 4);
    L.vbuf = put(sp_vbuf_bytes(rp));
    L.total = (int)off;
    L.ring = 0;
    // k_chain_ci: the same staging without the window buffers, then the ring
    off = 0;
    // the pixel's stratified values are staged in LDS while the staging of one
    // 1-wave tile (aliased with the ring) stays <= PBRT_CI_STAGE_KB; above,
    // StartPixel writes them straight to the pixel's global record (always with
    // the serial StartPixel, large spp): the trajectories read them from there
    // anyway, and a smaller workgroup lets more share a CU (config C at 8 KB:
    // 6.50 -> 5.25 s)
    const int64_t al16 = 15;
    const int64_t lds_staging = ((nd * n * 8 + al16) & ~al16) + ((nd * n * 2 + al16) & ~al16) +
                                ((sp_vbuf_bytes(rp) + al16) & ~al16);
    if (rp.sp_window) {   // the windowed StartPixel: picks in LDS, values straight to the global record
        Lci.s1d = -1;
        Lci.other = put(nd * n * 2);
    } else if (rp.sp_serial) {
        Lci.s1d = -1;
        Lci.other = put(16);
    } else if (lds_staging > PBRT_CI_STAGE_KB * 1024) {
        Lci.s1d = -1;
        Lci.other = put(nd * n * 2);
    } else {
        Lci.s1d = put(nd * n * 8);
        Lci.other = put(nd * n * 2);
    }
    Lci.sbuf = Lci.dbuf = 0;
    Lci.vbuf = put(sp_vbuf_bytes(rp));
    Lci.staging = (int)off;
    Lci.ring = put(kCiRingBytes);
    Lci.total = (int)off;
    return L.total <= 48 * 1024;
}

// k_chain_ci's LDS layout for w waves per tile and G tiles per wave. With one
// tile per workgroup (G == 1) the StartPixel staging aliases the offset ring:
// a group starts a pixel only after its chain has dropped every candidate,
// so the two are never live together (config C, 256 spp: 19 KB of staging).
// Multi-wave Matte tiles (nps: k_chain_ci's next-pixel speculation) keep
// trajectories of the next pixel in flight through its StartPixel: two rings
// (one per pixel parity) after the staging.
ChainLayout ci_layout(const ChainLayout& base, int w, int G, unsigned& lds_bytes, bool nps = false) {
    ChainLayout l = base;
    if (nps) {
        l.ring = (base.staging + 15) & ~15;
        lds_bytes = (unsigned)(l.ring + 2 * w * kCiRingBytes);
    } else if (G == 1) {
        l.ring = 0;
        lds_bytes = (unsigned)std::max(base.staging, w * kCiRingBytes);
    } else {
        lds_bytes = (unsigned)(base.total + (w - 1) * kCiRingBytes);
    }
    // then two ChainCache per lane group (pixel parities; only the groups in use: G, not kCiMaxGroups)
    l.pcs = (int)((lds_bytes + 15u) & ~15u);
    lds_bytes = (unsigned)l.pcs + (unsigned)(2 * G * sizeof(ChainCache));
    l.total = (int)lds_bytes;
    return l;
}

// Waves per tile of k_chain_ci for a launch of nb tiles. The frame's EXACT
// time is bounded below by its slowest tile's chain, so when the tiles of a
// launch cannot keep every wave slot busy (2 waves/SIMD) a tile gets 2 or 4
// waves. PBRT_CI_WAVES (1, 2, 4) overrides.
int ci_waves(const pbrt_gpu_ctx* c, int64_t nb) {
    if (c->knobs.ci_waves) return c->non_matte ? std::min(c->knobs.ci_waves, 4) : c->knobs.ci_waves;
    if (c->tiles_per_wave > 1) return 1;
    // measured on config B shards (tools/shard_sim.py): 8160 tiles -> 1,
    // 4080 -> 2, 2040 and 1020 -> 4
    const int64_t slots = (int64_t)c->n_simd * 2;   // 2 waves/SIMD
    if (nb <= slots) return 4;
    if (nb <= 2 * slots) return 2;
    return 1;
}

// k_chain_ci schedule. An EXACT frame lasts at least as long as its slowest
// tile's chain, and workgroups start in launch order, so a heavy tile that
// starts late stretches the frame. Each EXACT frame records every tile's
// chain time; the next frame of the same configuration on this context
// launches its tiles heaviest first (LPT). Only the schedule changes, never
// a result. PBRT_CI_ORDER=0 disables it.
// Multi-GPU shards (launches that would run 2 or 4 waves per tile): the
// heaviest tiles of the previous frame get 4 waves in a launch of their own
// and the rest 1 wave each in a concurrent one (1/4- and 1/2-frame shards:
// 387 -> 305 ms and 524 -> 472 ms per rank). PBRT_CI_SPLIT=0 disables it;
// PBRT_CI_HEAVY=K forces the heavy count (tests).
bool ci_split_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_split; }
// Does a one-wave Matte k_chain_ci workgroup with `dyn_lds` bytes of dynamic
// LDS leave room for 3 waves per SIMD (12 workgroups on a CU's LDS)?
bool ci_eu3_fits(const pbrt_gpu_ctx* c, unsigned dyn_lds, bool lds_nodes) {
    hipFuncAttributes fa;
    const void* f = lds_nodes ? reinterpret_cast<const void*>(&k_chain_ci<1>)
                              : reinterpret_cast<const void*>(&k_chain_ci<1, 64>);
    size_t stat = 0;
    if (hipFuncGetAttributes(&fa, f) == hipSuccess) stat = fa.sharedSizeBytes;
    const size_t per_wg = stat + dyn_lds;
    return per_wg > 0 && c->lds_per_cu / per_wg >= 12;
}
int64_t ci_heavy_override(const pbrt_gpu_ctx* c) { return c->knobs.ci_heavy; }
// k_chain_ci candidate stride: 2 issues candidates at the chain head's parity
// only (dropped when an odd draw count flips it), 1 at every offset (twice
// the candidates, none dropped). PBRT_CI_STRIDE = 1 / 2 overrides.
int ci_stride(const pbrt_gpu_ctx* c, int w) {
    if (c->knobs.ci_stride) return c->knobs.ci_stride;
    return w > 1 ? 1 : 2;
}
// PBRT_CI_HEAVY_WAVES = 4 (default) or 8: waves per heavy tile of the split
int ci_heavy_waves(const pbrt_gpu_ctx* c) { return c->non_matte ? 4 : c->knobs.ci_heavy_waves; }
bool ci_order_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_order; }
// PBRT_CI_ORDER_CACHE=0: no process-wide schedule cache (each context learns its own)
bool ci_order_cache(const pbrt_gpu_ctx* c) { return c->knobs.ci_order_cache; }
// PBRT_CI_PROBE=0: a fresh context's first frame runs in launch order (no k_tile_cost)
bool ci_probe_enabled(const pbrt_gpu_ctx* c) { return c->knobs.ci_probe; }
uint64_t schedule_key(const RenderParams& rp, int kw) {
    const int64_t v[] = {rp.film_min_x, rp.film_min_y, rp.film_w,   rp.film_h,    rp.tile_size, rp.tile_begin,
                         rp.tile_stride, rp.n_slots,   rp.spp,      rp.ndims,     rp.jitter,    rp.max_depth,
                         rp.flags,       kw,           (int64_t)(rp.rr_threshold * 1e9)};
    uint64_t h = 1469598103934665603ull;
    for (int64_t x : v) h = (h ^ (uint64_t)x) * 1099511628211ull;
    return h;
}

// k_paths_ci (lane refill over kPathsPixels pixels per wave) where it fits:
// LDS-staged nodes, the pixels' stratified values in 16 KB of LDS and one
// lane per (pixel, light) for the bounce-1 estimates; 0: the path wavefront
// (k_pw_*) runs the paths. PBRT_PATHS_CI=0 forces that.
// Returns the pixels per wave (2, 4 or 8; PBRT_PATHS_CI overrides, 0 = off).
// k_paths_ci stages the stratified values of its P pixels in LDS when they take <= 16 KB
// Off by default: read from their global records (L2-resident; config B
// 111.0 -> 109.9 ms EXACT, 136.0 -> 134.8 ms THROUGHPUT against LDS staging).
// PBRT_PATHS_S1D=lds stages them where they fit (experiments).
bool paths_ci_s1d_lds(const pbrt_gpu_ctx* c, const RenderParams& rp, int P) {
    return c->knobs.paths_s1d_lds && (int64_t)P * rp.ndims * rp.spp * 8 <= 16 * 1024;
}
int paths_ci_pixels(const pbrt_gpu_ctx* c, const RenderParams& rp) {
    int pp = 4;
    bool forced = false;
    if (c->knobs.paths_ci == 0) return 0;
    if (c->knobs.paths_ci > 0) pp = c->knobs.paths_ci, forced = true;
    auto fits = [&](int p) {
        return c->host_scene.n_nodes <= kLdsNodes && p * c->host_scene.n_lights <= kWave;
    };
    if (forced) return fits(pp) ? pp : 0;
    // 8 pixels per wave where their lights fit one wave, else 4; stratified
    // values read from global memory (config B EXACT paths 109.9 -> 104.8 ms
    // for 8 against 4; config C at 256 spp 872 -> 869 ms, where 4 pixels with
    // global values already beat 2 with LDS values, 1150 ms)
    return fits(8) ? 8 : fits(4) ? 4 : 0;
}

// The full-path stage on the path wavefront (k_pw_*) instead of k_paths_ci:
// PBRT_PATHS_WF=1 / 0 forces it on / off; by default it runs for scenes with
// triangle meshes, where it measured faster (config D: 385 -> 343 ms EXACT,
// 420 -> 381 ms THROUGHPUT), and not for the analytic scenes, where the
// monolithic lane-refill kernel is twice as fast (config B: 118 vs 212-245 ms;
// profiles/r02/path_wavefront_ab.json). PBRT_PW_SORT=1 adds the material sort
// between trace and shade: a loss on every scene measured (B 212 -> 245 ms: a
// few matte materials leave no shading divergence to remove), so off by default.
// Triangle meshes and no analytic primitive: the kMeshOnly kernels (k_chain_ci
// kDepth < 0, k_pw_trace / k_pw_shadow<true>) compile the analytic walk out.
bool mesh_only_scene(const pbrt_gpu_ctx* c) {
    return c->host_scene.n_prims == 0 && c->mesh.n_nodes > 0 && !c->non_matte;
}

bool paths_wf_enabled(const pbrt_gpu_ctx* c) {
    if (c->knobs.paths_wf >= 0) return c->knobs.paths_wf == 1;
    return c->mesh.n_nodes > 0;
}
int paths_wavefront(pbrt_gpu_ctx* c, const DevScene& sc, int64_t sb, int64_t nb) {
    const RenderParams& rp = c->rp;
    const int64_t nrec = nb * c->wb.ppt, per = rp.spp - 1;
    const int nl = sc.n_lights;
    const int sort = c->knobs.pw_sort ? 1 : 0;
    const int n_keys = std::max(1, std::min(c->host_scene.n_materials, kPwMaxKeys));
    const double gb = c->knobs.pw_gb;
    const int64_t per_path = (int64_t)sizeof(PwPath) + 4 * 4;   // record + 4 queue slots
    int64_t chunk = per > 0 ? std::max<int64_t>(1, (int64_t)(gb * 1073741824.0) / (per_path * per)) : nrec;
    chunk = std::min(chunk, nrec);
    if (per > 0) chunk = std::min<int64_t>(chunk, (int64_t)0xFFFFFFF0 / per);
    const int64_t cap = std::max<int64_t>(1, chunk * std::max<int64_t>(per, 1));
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    const int64_t ncnt = 3 + 2 * kPwMaxKeys;
    const size_t need = (size_t)(al(cap * (int64_t)sizeof(PwPath)) + 4 * al(cap * 4) + al(ncnt * 4) +
                                 al(chunk * std::max(nl, 1) * (int64_t)sizeof(Spec)) + al(chunk * std::max(nl, 1) * 4) +
                                 al(nrec * 8));
    if (c->pw_cap < need || !c->d_pw) {
        if (c->d_pw) (void)hipFree(c->d_pw);
        c->d_pw = nullptr;
        c->pw_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_pw, need));
        c->pw_cap = need;
    }
    unsigned char* p = c->d_pw;
    auto take = [&](int64_t bytes) {
        unsigned char* q = p;
        p += al(bytes);
        return q;
    };
    PwPath* paths = (PwPath*)take(cap * (int64_t)sizeof(PwPath));
    PwQueues qs;
    for (int i = 0; i < 3; i++) qs.q[i] = (uint32_t*)take(cap * 4);
    qs.sorted = (uint32_t*)take(cap * 4);
    qs.cnt = (uint32_t*)take(ncnt * 4);
    qs.cap = cap;
    Spec* ldc = (Spec*)take(chunk * std::max(nl, 1) * (int64_t)sizeof(Spec));
    int* ldp = (int*)take(chunk * std::max(nl, 1) * 4);
    unsigned long long* pkey = (unsigned long long*)take(nrec * 8);
    const unsigned G = (unsigned)std::max<int64_t>(64, (int64_t)c->n_simd * 8);   // grid-stride blocks
    HIPCHK(c, hipMemsetAsync(pkey, 0xFF, (size_t)nrec * 8, c->stream));
    const bool mb = rp.mode == PBRT_MODE_THROUGHPUT;
    const bool kx = c->non_matte;   // Mirror / smooth Glass / OrenNayar: the kX instantiations
    for (int64_t r0 = 0; r0 < nrec; r0 += chunk) {
        const int64_t nr = std::min(chunk, nrec - r0);
        if (per > 0) {
            HIPCHK(c, hipMemsetAsync(qs.cnt, 0, (size_t)ncnt * 4, c->stream));
            if (nl > 0)
                hipLaunchKernelGGL(kx ? k_pw_cache<true> : k_pw_cache<false>,
                                   dim3((unsigned)((nr * nl + kWave - 1) / kWave)), dim3(kWave), 0,
                                   c->stream, sc, c->wb, r0, nr, ldc, ldp);
            auto start = kx ? (mb ? k_pw_start<true, true> : k_pw_start<false, true>)
                            : (mb ? k_pw_start<true> : k_pw_start<false>);
            hipLaunchKernelGGL(start, dim3((unsigned)((nr * per + kWave - 1) / kWave)), dim3(kWave), 0, c->stream,
                               sc, rp, c->wb, sb, r0, nr, ldc, ldp, paths, qs, pkey);
            for (int pass = 0; pass + 1 < rp.max_depth; pass++) {
                hipLaunchKernelGGL(mesh_only_scene(c) ? k_pw_trace<true> : k_pw_trace<false>, dim3(G), dim3(kWave), 0, c->stream, sc, rp, c->wb, paths, qs, 0,
                                   n_keys, pkey);
                if (sort && n_keys > 1) {
                    hipLaunchKernelGGL(k_pw_scan, dim3(1), dim3(1), 0, c->stream, qs, n_keys);
                    hipLaunchKernelGGL(k_pw_scatter, dim3(G / 4), dim3(256), 0, c->stream, paths, qs);
                }
                hipLaunchKernelGGL(kx ? k_pw_shade<true> : k_pw_shade<false>, dim3(G), dim3(kWave), 0, c->stream, sc,
                                   rp, c->wb, sb, paths, qs,
                                   sort && n_keys > 1 ? 1 : 0, pkey);
                hipLaunchKernelGGL(mesh_only_scene(c) ? k_pw_shadow<true> : k_pw_shadow<false>, dim3(G), dim3(kWave), 0, c->stream, sc, rp, c->wb, paths, qs, pkey);
            }
        }
        hipLaunchKernelGGL(k_pw_panics, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, c->stream, rp, c->wb, sb, r0,
                           nr, pkey, c->d_ctr);
    }
    HIPCHK(c, hipGetLastError());
    return PBRT_OK;
}

// Carve the per-batch buffers of the wave path. Budget: PBRT_WAVE_BUFFER_GB,
// default min(96 GB, half the free HBM) -- config C (1080p, 256 spp, ~34 GB)
// and one rank's 1/8 shard of config E (4K, 1024 spp, ~68 GB) are then one
// batch on a 288 GB MI355X, so the whole frame is one launch per kernel and
// gets the heaviest-first schedule.
int wave_buffers(pbrt_gpu_ctx* c) {
    const RenderParams& rp = c->rp;
    const int64_t ppt = rp.tile_size * rp.tile_size, n = rp.spp, nd = rp.ndims > 0 ? rp.ndims : 1;
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    // k_chain_ci<kX>'s RR decision records, one per ring entry (Path renders of non-Matte scenes)
    const int64_t rrb_bytes = c->non_matte ? (int64_t)kCiMaxRing * (int64_t)sizeof(RrBranches) : 0;
    const int64_t per_tile = al(ppt * (int64_t)sizeof(PixelRec)) + al(ppt * nd * n * 8) + al(ppt * n * 8) +
                             al(ppt * n * 24) + al(ppt * n * 4) + al(ppt * (int64_t)sizeof(PanicRec)) + al(4) +
                             al(rrb_bytes);
    double gb = 96.0;
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
            gb = std::min(gb, 0.5 * (double)(free_b + c->wave_cap) / 1073741824.0);
    }
    if (c->knobs.wave_buffer_gb > 0) gb = c->knobs.wave_buffer_gb;
    int64_t batch = (int64_t)(gb * 1073741824.0) / per_tile;
    if (batch < 1) batch = 1;
    if (batch > rp.n_slots) batch = rp.n_slots > 0 ? rp.n_slots : 1;
    const size_t need = (size_t)(batch * per_tile);
    if (c->wave_cap < need || !c->d_wave) {
        if (c->d_wave) (void)hipFree(c->d_wave);
        c->d_wave = nullptr;
        c->wave_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_wave, need));
        c->wave_cap = need;
    }
    WaveBufs& wb = c->wb;
    unsigned char* p = c->d_wave;
    auto take = [&](int64_t bytes_per_tile) {
        unsigned char* q = p;
        p += batch * al(bytes_per_tile);
        return q;
    };
    wb.prec = (PixelRec*)take(ppt * (int64_t)sizeof(PixelRec));
    wb.s1d = (double*)take(ppt * nd * n * 8);
    wb.memb = (uint64_t*)take(ppt * n * 8);
    wb.L = (double*)take(ppt * n * 24);
    wb.rays = (uint32_t*)take(ppt * n * 4);
    wb.ppanic = (PanicRec*)take(ppt * (int64_t)sizeof(PanicRec));
    wb.tile_npx = (int32_t*)take(4);
    wb.rrb = rrb_bytes ? (RrBranches*)take(rrb_bytes) : nullptr;
    wb.ppt = ppt;
    wb.s1d_stride = nd * n;
    c->wave_batch = batch;
    return PBRT_OK;
}

int prepare(pbrt_gpu_ctx* c, const pbrt_render_desc* rd) {
    if (!rd) return set_err(c, PBRT_E_INVALID, "null render desc");
    if (rd->tile_size <= 0 || rd->sampler_x <= 0 || rd->sampler_y <= 0 || rd->n_dims < 0 || rd->n_dims > 64)
        return set_err(c, PBRT_E_INVALID, "bad sampler / tile size");
    if ((int64_t)rd->sampler_x * rd->sampler_y > (1 << 20)) return set_err(c, PBRT_E_INVALID, "spp too large");
    if (rd->integrator != PBRT_INTEGRATOR_PATH && rd->integrator != PBRT_INTEGRATOR_DIRECT_LIGHTING)
        return set_err(c, PBRT_E_UNSUPPORTED, "unknown integrator");
    if (rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING && rd->dl_strategy != PBRT_DL_UNIFORM_SAMPLE_ALL &&
        rd->dl_strategy != PBRT_DL_UNIFORM_SAMPLE_ONE)
        return set_err(c, PBRT_E_UNSUPPORTED, "unknown DirectLighting strategy");
    if (rd->mode != PBRT_MODE_EXACT && rd->mode != PBRT_MODE_THROUGHPUT)
        return set_err(c, PBRT_E_INVALID, "unknown mode");
    const pbrt_film_desc& f = c->host_scene.film;
    if (f.filter_radius_x <= 0 || f.filter_radius_y <= 0 || f.filter_radius_x >= (double)rd->tile_size ||
        f.filter_radius_y >= (double)rd->tile_size)
        return set_err(c, PBRT_E_UNSUPPORTED, "filter radius must be in (0, tile_size)");
    if ((rd->flags & PBRT_FLAG_PANIC_FIDELITY) && c->non_matte)
        return set_err(c, PBRT_E_UNSUPPORTED, "panic fidelity covers Matte scenes only");
    if (rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING && c->non_matte && rd->max_depth > 2 * kDlMaxLevels)
        return set_err(c, PBRT_E_UNSUPPORTED, "DirectLighting through glass: maxDepth must be <= 64");
    RenderParams& rp = c->rp;
    std::memset(&rp, 0, sizeof(rp));
    rp.film_min_x = f.crop_min_x;
    rp.film_min_y = f.crop_min_y;
    rp.film_w = f.crop_max_x - f.crop_min_x;
    rp.film_h = f.crop_max_y - f.crop_min_y;
    rp.tile_size = rd->tile_size;
    rp.ntx = (rp.film_w + rd->tile_size - 1) / rd->tile_size;
    rp.nty = (rp.film_h + rd->tile_size - 1) / rd->tile_size;
    int64_t total = rp.ntx * rp.nty;
    int64_t begin = rd->tile_begin < 0 ? 0 : rd->tile_begin;
    int64_t end = rd->tile_end > 0 && rd->tile_end < total ? rd->tile_end : total;
    int64_t stride = rd->tile_stride > 0 ? rd->tile_stride : 1;
    rp.tile_begin = begin;
    rp.tile_stride = stride;
    rp.n_slots = begin < end ? (end - begin + stride - 1) / stride : 0;
    rp.slot_w = rd->tile_size + 2 * ((int64_t)f.filter_radius_x + 1);
    rp.slot_h = rd->tile_size + 2 * ((int64_t)f.filter_radius_y + 1);
    rp.xs = rd->sampler_x;
    rp.ys = rd->sampler_y;
    rp.spp = rd->sampler_x * rd->sampler_y;
    rp.ndims = rd->n_dims;
    rp.jitter = rd->jitter ? 1 : 0;
    rp.integrator = rd->integrator;
    rp.max_depth = rd->max_depth;
    rp.dl_strategy = rd->dl_strategy;
    rp.rr_threshold = rd->rr_threshold;
    rp.lanes_per_wave = c->lanes_per_wave;
    rp.flags = rd->flags;
    rp.mode = rd->mode;
    rp.ci_nps = 0;   // set per k_chain_ci launch (launch_ci)
    rp.ci_scap = c->knobs.ci_scap;
    pbrt_distribution_desc& dist = c->host_dist;
    std::memset(&dist, 0, sizeof(dist));
    if (rd->integrator == PBRT_INTEGRATOR_PATH) {
        int rc = pbrt_scene_light_distribution(&c->host_scene, rd->light_strategy, &dist);
        if (rc != PBRT_OK) return set_err(c, rc, "unsupported light sample strategy");
        HIPCHK(c, hipMemcpyAsync(c->d_dist, &dist, sizeof(dist), hipMemcpyHostToDevice, c->stream));
    }
    {
        const int64_t n = rp.spp, s1 = rp.jitter ? 2 * n : n, s2 = rp.jitter ? 3 * n : n;
        const int64_t E = (int64_t)rp.ndims * (s1 + s2), V = E + 64 + E / 8;
        rp.sp_events = (int32_t)E;
        rp.sp_draws = (int32_t)V;
        rp.sp_serial = V * 4 <= PBRT_SP_SERIAL_KB * 1024 ? 0 : 1;
        // the windowed wave StartPixel where the serial one would run, without
        // jitter (values are functions of their index), while its picks and
        // permutations fit PBRT_SP_WINDOW_KB of LDS (config C; E's 1024 spp stay serial)
        // (k_chain_ci instantiates it for Matte scenes of LDS-staged trees, the
        // analytic walk: the host runs those kernels below)
        rp.sp_window = c->knobs.sp_window && rp.sp_serial && !rp.jitter && !c->non_matte && c->host_scene.n_nodes <= kLdsNodes &&
                       c->mesh.n_nodes == 0 &&
                       (int64_t)rp.ndims * n * 4 + kSpRing * 4 <= PBRT_SP_WINDOW_KB * 1024 ? 1 : 0;
    }
    c->use_spec = c->kernel_req != PBRT_KERNEL_SERIAL && wave_eligible(c, rd, rp, c->lay, c->lay_ci);
    if ((c->kernel_req == PBRT_KERNEL_WAVE || c->kernel_req == PBRT_KERNEL_WAVEFRONT ||
         c->kernel_req == PBRT_KERNEL_WAVE_CI) && !c->use_spec)
        return set_err(c, PBRT_E_UNSUPPORTED, "render not eligible for the wave-parallel kernels");
    c->use_dl = c->use_spec && rd->integrator == PBRT_INTEGRATOR_DIRECT_LIGHTING;
    if (c->use_dl && c->kernel_req != PBRT_KERNEL_AUTO && c->kernel_req != PBRT_KERNEL_WAVE_DL)
        return set_err(c, PBRT_E_UNSUPPORTED, "DirectLighting runs on the serial or the k_dl_* kernels");
    if (!c->use_dl && c->kernel_req == PBRT_KERNEL_WAVE_DL)
        return set_err(c, PBRT_E_UNSUPPORTED, "render not eligible for the DirectLighting wave kernels");
    // the chain stage of the wave pipeline is k_chain_ci (PBRT_KERNEL_WAVE and
    // _WAVEFRONT, whose window and wavefront chains it replaced, select it too)
    c->use_ci = c->use_spec && !c->use_dl;
    if (c->use_spec && rp.n_slots > 0) {
        int rcw = wave_buffers(c);
        if (rcw != PBRT_OK) return rcw;
        // tiles per k_chain_ci wave (opts.lanes_per_wave = 1, 2 or 4; default 1).
        // One tile per wave is fastest on MI355X: its 64 trajectories leave the
        // same bounce-1 point, so their traversals stay coherent; packing tiles
        // cuts speculation but a window lasts as long as its slowest lane, and
        // mixed-tile windows measured 2.5x slower per window.
        int G = 1;
        if (c->lanes_per_wave_set && c->lanes_per_wave >= 1 && c->lanes_per_wave <= kCiMaxGroups &&
            (c->lanes_per_wave & (c->lanes_per_wave - 1)) == 0)
            G = c->lanes_per_wave;
        c->tiles_per_wave = G;
    }
    size_t nslot = (size_t)(rp.n_slots > 0 ? rp.n_slots : 1);
    int rc;
    if ((rc = ensure(c, &c->d_films, &c->films_cap, nslot * (size_t)(rp.slot_w * rp.slot_h * 3)))) return rc;
    if ((rc = ensure(c, &c->d_s1d, &c->s1d_cap, nslot * (size_t)(rp.ndims > 0 ? rp.ndims : 1) * (size_t)rp.spp)))
        return rc;
    if ((rc = ensure(c, &c->d_panics, &c->panics_cap, nslot))) return rc;
    if ((rc = ensure(c, &c->d_out, &c->out_cap, (size_t)(rp.film_w * rp.film_h * 3)))) return rc;
    return PBRT_OK;
}

}  // namespace

extern "C" {

int pbrt_gpu_create(const pbrt_scene_desc* scene, const pbrt_gpu_opts* opts, pbrt_gpu_ctx** out) {
    if (!out) return PBRT_E_INVALID;
    *out = nullptr;
    int rc = validate_scene(scene);
    if (rc != PBRT_OK) return rc;
    auto* c = new pbrt_gpu_ctx();
    c->knobs = Knobs::from_env();
    c->device = (opts && opts->device >= 0) ? opts->device : -1;
    if (opts && opts->lanes_per_wave > 0 && opts->lanes_per_wave <= 64) {
        c->lanes_per_wave = opts->lanes_per_wave;
        c->lanes_per_wave_set = true;
    }
    if (opts && (opts->occupancy == 2 || opts->occupancy == 4 || opts->occupancy == 8)) c->min_waves = opts->occupancy;
    if (opts) c->occ_req = opts->occupancy;
    if (opts && (opts->kernel < PBRT_KERNEL_AUTO || opts->kernel > PBRT_KERNEL_WAVE_DL)) {
        delete c;
        return PBRT_E_INVALID;
    }
    if (opts) c->kernel_req = opts->kernel;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        delete c;
        return PBRT_E_HIP;
    }
    if (c->device >= 0) {
        if (hipSetDevice(c->device) != hipSuccess) { delete c; return PBRT_E_HIP; }
    } else {
        (void)hipGetDevice(&c->device);
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0) {
            c->n_simd = 4 * prop.multiProcessorCount;
            c->lds_per_block = prop.sharedMemPerBlock;
            if (prop.maxSharedMemoryPerMultiProcessor > 0) c->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
        }
    }
    std::vector<uint32_t> order;
    if (!dev_order(scene, order)) {
        delete c;
        return PBRT_E_INVALID;
    }
    c->host_scene = *scene;
    c->scene_hash = scene_content_hash(scene);
    c->non_matte = false;
    for (int i = 0; i < scene->n_materials; i++)   // Mirror, Glass or OrenNayar (Matte with sigma != 0)
        c->non_matte |= scene->materials[i].type != PBRT_MAT_MATTE ||
                        !(std::min(std::max(scene->materials[i].sigma, 0.0), 90.0) == 0);
    c->rough_glass = false;
    for (int i = 0; i < scene->n_materials; i++)
        c->rough_glass |= scene->materials[i].type == PBRT_MAT_GLASS &&
                          !(scene->materials[i].u_roughness == 0 && scene->materials[i].v_roughness == 0);
    c->h_node_prims.resize((size_t)scene->n_nodes);
    for (int i = 0; i < scene->n_nodes; i++) c->h_node_prims[i] = scene->nodes[i].n_prims;
    c->host_scene.shapes = nullptr;
    c->host_scene.materials = nullptr;
    c->host_scene.prims = nullptr;
    c->host_scene.nodes = nullptr;
    c->host_lights.assign(scene->lights, scene->lights + scene->n_lights);
    c->host_scene.lights = c->host_lights.data();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_split, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        pbrt_gpu_destroy(c);
        return PBRT_E_HIP;
    }

    if (hipHostMalloc((void**)&c->h_cancel, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->d_cancel, c->h_cancel, 0) != hipSuccess) {
        pbrt_gpu_destroy(c);
        return PBRT_E_HIP;
    }
    __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    if ((rc = upload(c, &c->d_shapes, scene->shapes, scene->n_shapes)) ||
        (rc = upload(c, &c->d_materials, scene->materials, scene->n_materials)) ||
        (rc = upload(c, &c->d_prims, scene->prims, scene->n_prims)) ||
        (rc = upload(c, &c->d_nodes, dev_nodes(scene).data(), scene->n_nodes)) ||
        (rc = upload(c, &c->d_order, order.data(), order.size())) ||
        (rc = upload(c, &c->d_fprims, dev_prims(scene).data(), scene->n_prims)) ||
        (rc = upload(c, &c->d_lights, scene->lights, scene->n_lights)) ||
        (rc = upload(c, &c->d_camera, &scene->camera, 1)) || (rc = upload(c, &c->d_film, &scene->film, 1)) ||
        (rc = upload<pbrt_distribution_desc>(c, &c->d_dist, nullptr, 1)) ||
        (rc = upload<Counters>(c, &c->d_ctr, nullptr, 1)) || (rc = upload<int>(c, &c->d_cancel_seen, nullptr, 1)) ||
        (rc = upload<PcgJump>(c, &c->d_jump, &pcg_jump_table(), 1))) {
        pbrt_gpu_destroy(c);
        return rc;
    }
    {   // leaf culling groups of the LDS-staged walk
        std::vector<double> gb;
        std::vector<uint32_t> gm;
        c->n_groups = cull_groups(c->knobs, scene, order, gb, gm);
        if (!c->knobs.cull_groups) c->n_groups = 0;   // PBRT_CULL_GROUPS=0: test every leaf (A/B)
        if (c->n_groups > 0 && ((rc = upload(c, &c->d_groups, gb.data(), gb.size())) ||
                                (rc = upload(c, &c->d_gmasks, gm.data(), gm.size())))) {
            pbrt_gpu_destroy(c);
            return rc;
        }
    }
    if (scene->n_meshes > 0) {   // triangle meshes: LBVH built on the device (mesh_bvh.hip)
        std::string err;
        rc = mesh_bvh_build(scene, c->stream, c->mesh, err);
        if (rc != PBRT_OK) {
            pbrt_gpu_destroy(c);
            return rc;
        }
    }
    c->host_scene.meshes = nullptr;
    *out = c;
    return PBRT_OK;
}

namespace {
int render_enqueue(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_device);
}

int pbrt_gpu_render_async_into(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_device) {
    if (!c) return PBRT_E_INVALID;
    {   // from here on this render is the one pbrt_gpu_cancel cancels: a cancel
        // that lands while prepare() sizes and allocates the buffers is kept
        std::lock_guard<std::mutex> lk(c->cancel_mu);
        c->in_flight = true;
        c->cancel_req = false;
        __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    if (rd) c->last_rd = *rd;   // kept for a re-render (pbrt_gpu_synchronize)
    c->last_film_device = film_device;
    const int rc = render_enqueue(c, rd, film_device);
    if (rc != PBRT_OK) {   // nothing was launched (or the launch failed): no render is in flight
        std::lock_guard<std::mutex> lk(c->cancel_mu);
        c->in_flight = false;
        c->cancel_req = false;
        __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    return rc;
}

namespace {
int render_enqueue(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_device) {
    HIPCHK(c, hipSetDevice(c->device));
    c->t_start = std::chrono::steady_clock::now();
    int rc = prepare(c, rd);
    if (rc != PBRT_OK) return rc;
    const RenderParams& rp = c->rp;
    double* out = film_device ? film_device : c->d_out;
    c->film_target = out;
    c->last_heavy = 0;
    c->sched_src = PBRT_SCHED_LAUNCH_ORDER;
    HIPCHK(c, hipMemsetAsync(c->d_ctr, 0, sizeof(Counters), c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_cancel_seen, 0, sizeof(int), c->stream));
    if (rp.n_slots > 0) HIPCHK(c, hipMemsetAsync(c->d_panics, 0, sizeof(PanicRec) * (size_t)rp.n_slots, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if (rp.n_slots > 0) {
        DevScene sc = dev_scene(c, rd->integrator == PBRT_INTEGRATOR_PATH);
        if (c->use_spec) {
            c->last_kernel = c->use_dl ? PBRT_KERNEL_WAVE_DL
                             : rp.mode == PBRT_MODE_THROUGHPUT ? PBRT_KERNEL_WAVE : PBRT_KERNEL_WAVE_CI;
            const bool lds_nodes = c->host_scene.n_nodes <= kLdsNodes;
            const bool kx = c->non_matte;   // Mirror / smooth Glass / OrenNayar: the kX instantiations
            const bool mesh_only = mesh_only_scene(c);   // triangle meshes and nothing else: no analytic walk
            c->n_batches = (int)((rp.n_slots + c->wave_batch - 1) / c->wave_batch);
            while ((int)c->bev.size() < 3 * c->n_batches) {
                hipEvent_t e;
                HIPCHK(c, hipEventCreate(&e));
                c->bev.push_back(e);
            }
            for (int64_t sb = 0, bi = 0; sb < rp.n_slots; sb += c->wave_batch, bi++) {
                const int64_t nb = std::min<int64_t>(c->wave_batch, rp.n_slots - sb);
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 0], c->stream));
                const int G = c->tiles_per_wave;
                // EXACT k_paths_ci over n slots (ord: the slots' order, else slots 0 .. n - 1)
                const bool paths_ci_exact = !c->use_dl && rp.mode != PBRT_MODE_THROUGHPUT &&
                                            !(paths_wf_enabled(c) || paths_ci_pixels(c, rp) == 0);
                auto launch_paths = [&](const uint32_t* ord, int64_t n, hipStream_t st) {
                    const int pp = paths_ci_pixels(c, rp);
                    const int per = rp.ndims * rp.spp;
                    auto kern = kx ? (pp == 8 ? k_paths_ci<8, false, true> : k_paths_ci<4, false, true>)
                                   : (pp == 8 ? k_paths_ci<8> : pp == 2 ? k_paths_ci<2> : k_paths_ci<4>);
                    const int sl = paths_ci_s1d_lds(c, rp, pp) ? 1 : 0;
                    const int lds = pp == 8 ? paths_group_lds<8>(sl * per) : pp == 2 ? paths_group_lds<2>(sl * per)
                                                                                     : paths_group_lds<4>(sl * per);
                    // ordered: whole slots, ceil(ppt / pp) workgroups each (pp need not divide ppt)
                    const int64_t groups = ord ? n * ((c->wb.ppt + pp - 1) / pp) : (n * c->wb.ppt + pp - 1) / pp;
                    hipLaunchKernelGGL(kern, dim3((unsigned)groups), dim3(kWave),
                                       (unsigned)lds, st, with_slot(sc, 3), rp, c->wb, sb, n * c->wb.ppt,
                                       c->d_ctr, sl, ord);
                };
                c->ov_done = 0;
                if (c->use_dl) {
                    hipLaunchKernelGGL(kx ? k_wf_primary<true> : k_wf_primary<false>, dim3((unsigned)((nb * c->wb.ppt + kWave - 1) / kWave)),
                                       dim3(kWave), 0, c->stream, with_slot(sc, 1), rp, c->wb, sb, nb);
                    unsigned lds = 0;
                    const ChainLayout lw = ci_layout(c->lay_ci, 1, 1, lds);
                    hipLaunchKernelGGL(k_dl_setup, dim3((unsigned)nb), dim3(kWave), lds, c->stream, sc, rp, lw,
                                       c->d_jump, c->wb, sb, nb);
                } else if (rp.mode == PBRT_MODE_THROUGHPUT) {
                    // no offset chain: every sample's stream is known up front
                } else {
                    hipLaunchKernelGGL(kx ? k_wf_primary<true> : k_wf_primary<false>,
                                       dim3((unsigned)((nb * c->wb.ppt + kWave - 1) / kWave)),
                                       dim3(kWave), 0, c->stream, with_slot(sc, 1), rp, c->wb, sb, nb);
                    const int kw = ci_waves(c, nb);
                    const uint32_t* order = nullptr;
                    bool learned = false;   // order from the last frame's measured chain times
                    uint32_t* ticks = nullptr;
                    if ((kw > 1 || G == 1) && c->n_batches == 1 && ci_order_enabled(c)) {
                        if (c->ticks_cap < nb) {
                            if (c->d_ticks) (void)hipFree(c->d_ticks);
                            if (c->d_slot_order) (void)hipFree(c->d_slot_order);
                            c->d_ticks = c->d_slot_order = nullptr;
                            c->ticks_cap = 0;
                            HIPCHK(c, hipMalloc((void**)&c->d_ticks, sizeof(uint32_t) * (size_t)nb * kTickPlanes));
                            HIPCHK(c, hipMalloc((void**)&c->d_slot_order, sizeof(uint32_t) * (size_t)nb));
                            c->ticks_cap = nb;
                        }
                        const uint64_t key = schedule_key(rp, kw);
                        c->sched_src = PBRT_SCHED_LAUNCH_ORDER;
                        if (!(c->order_key == key && (int64_t)c->h_slot_order.size() == nb) && ci_order_cache(c)) {
                            SchedEntry e;   // a fresh context: another context's measured order for this scene
                            if (sched_cache_get(c, key, nb, e)) {
                                c->h_slot_order = std::move(e.order);
                                c->heavy_k = e.heavy_k;
                                c->order_key = key;
                                c->sched_src = PBRT_SCHED_CACHED;
                            }
                        }
                        if (c->order_key == key && (int64_t)c->h_slot_order.size() == nb) {
                            if (c->sched_src != PBRT_SCHED_CACHED) c->sched_src = PBRT_SCHED_LEARNED;
                            HIPCHK(c, hipMemcpyAsync(c->d_slot_order, c->h_slot_order.data(), sizeof(uint32_t) * (size_t)nb,
                                                     hipMemcpyHostToDevice, c->stream));
                            order = c->d_slot_order;
                            learned = true;
                        }
                        c->probed = false;
                        if (!order && ci_probe_enabled(c) && nb <= (int64_t)1 << 24) {
                            // no measured order for this configuration yet: estimate it
                            int64_t npad = 2048;
                            while (npad < nb) npad <<= 1;
                            if (c->cost_cap < npad) {
                                if (c->d_cost) (void)hipFree(c->d_cost);
                                if (c->d_cost_keys) (void)hipFree(c->d_cost_keys);
                                c->d_cost = nullptr;
                                c->d_cost_keys = nullptr;
                                c->cost_cap = 0;
                                HIPCHK(c, hipMalloc((void**)&c->d_cost, sizeof(float) * 4 * (size_t)npad));
                                HIPCHK(c, hipMalloc((void**)&c->d_cost_keys, sizeof(uint64_t) * (size_t)npad));
                                c->cost_cap = npad;
                            }
                            HIPCHK(c, hipMemsetAsync(c->d_cost_keys, 0xFF, sizeof(uint64_t) * (size_t)npad, c->stream));
                            hipLaunchKernelGGL(kx ? k_tile_cost<true> : k_tile_cost<false>, dim3((unsigned)nb),
                                               dim3(kWave), 0, c->stream, with_slot(sc, 0),
                                               rp, c->wb, sb, nb, c->d_cost, c->d_cost_keys);
                            bitonic_sort_u64(c->d_cost_keys, (uint32_t)npad, c->stream);
                            hipLaunchKernelGGL(k_order_of_keys, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
                                               c->stream, c->d_cost_keys, nb, c->d_slot_order);
                            order = c->d_slot_order;
                            c->probed = true;
                            c->sched_src = PBRT_SCHED_PROBE;
                            c->cost_n = nb;
                        }
                        ticks = c->d_ticks;
                        c->ticks_pending = true;
                        c->ticks_key = key;
                        c->ticks_n = nb;
                    }
                    // one launch of n workgroups, workgroup b on slot ord[b] (identity if null)
                    bool split_launch = false;   // launch_ci's launch is the heavy half of a split
                    // waves per tile of a split's light launch
                    // (set below, before any launch_ci call)
                    bool light_kw = kw > 1 && c->knobs.ci_light_kw;
                    int light_w = light_kw ? kw : 1;
                    int heavy_w = ci_heavy_waves(c);
                    auto launch_ci = [&](int w, int64_t n, const uint32_t* ord, hipStream_t st, uint32_t* prog) {
                        if (w > 1) {   // one tile per workgroup of w waves; the ring grows with the lanes
                            const int ring = w * kCiRingBytes / (int)sizeof(RingEnt);
                            unsigned lds = 0;
                            // next-pixel speculation (k_chain_ci kNps: Matte, stride 1) for launches of
                            // multi-wave tiles only: not for the heavy launch of a split, where
                            // its two rings' LDS cost the light tiles beside it (1/4 shard of B
                            // 132 -> 145 ms; a 1/8 shard, no split: 131.5 -> 127.2 ms)
                            RenderParams rpl = rp;
                            rpl.ci_nps = (!kx && (!split_launch || light_kw) && ci_stride(c, w) == 1) ? c->knobs.ci_nps : 0;
                            const ChainLayout lw = ci_layout(c->lay_ci, w, 1, lds, rpl.ci_nps > 0);
                            // kX: LDS-staged trees only, at most 4 waves per tile (wave_eligible, ci_waves)
                            auto kern = kx ? (w == 2 ? k_chain_ci<2, 0, true> : k_chain_ci<4, 0, true>)
                                        : mesh_only ? (w == 2 ? k_chain_ci<2, -1> : w == 4 ? k_chain_ci<4, -1> : k_chain_ci<8, -1>)
                                        : rp.sp_window ? (w == 2 ? k_chain_ci<2, 0, false, 0, true>
                                                          : w == 4 ? k_chain_ci<4, 0, false, 0, true>
                                                                   : k_chain_ci<8, 0, false, 0, true>)
                                           : (w == 2   ? (lds_nodes ? k_chain_ci<2> : k_chain_ci<2, 64>)
                                              : w == 4 ? (lds_nodes ? k_chain_ci<4> : k_chain_ci<4, 64>)
                                                       : (lds_nodes ? k_chain_ci<8> : k_chain_ci<8, 64>));
                            hipLaunchKernelGGL(kern, dim3((unsigned)n), dim3(kWave * w), lds, st, with_slot(sc, 2), rpl, lw,
                                               c->d_jump, c->wb, sb, nb, kWave * w, ring, c->d_ctr, ord, ticks,
                                               ci_stride(c, w), prog);
                        } else {
                            const int Gc = std::min(G, kCiMaxGroups);
                            const int ring = kCiRingBytes / (int)sizeof(RingEnt) / Gc;
                            unsigned lds = 0;
                            const ChainLayout lw = ci_layout(c->lay_ci, 1, Gc, lds);
                            // Matte analytic scenes: the 3-waves/SIMD build unless the
                            // workgroup's LDS (large spp: StartPixel staging) caps the CU
                            // below 3 waves/SIMD, where the 2-wave build (no spills) is faster
                            // (config C: 6.53 vs 7.41 s)
                            const bool eu2 = !kx && !mesh_only &&
                                             (c->knobs.ci_eu == 2 || (c->knobs.ci_eu != 3 && !ci_eu3_fits(c, lds, lds_nodes)));
                            c->ci_wps = (kx || eu2) ? 2 : 3;
                            auto kern1 = kx ? k_chain_ci<1, 0, true>
                                         : mesh_only ? k_chain_ci<1, -1>
                                         : rp.sp_window ? (eu2 ? k_chain_ci<1, 0, false, 2, true> : k_chain_ci<1, 0, false, 0, true>)
                                         : eu2 ? (lds_nodes ? k_chain_ci<1, 0, false, 2> : k_chain_ci<1, 64, false, 2>)
                                               : (lds_nodes ? k_chain_ci<1> : k_chain_ci<1, 64>);
                            hipLaunchKernelGGL(kern1, dim3((unsigned)((n + Gc - 1) / Gc)), dim3(kWave),
                                               lds, st, with_slot(sc, 2), rp, lw, c->d_jump, c->wb, sb,
                                               nb, kWave / Gc, ring, c->d_ctr, Gc == 1 ? ord : nullptr,
                                               Gc == 1 ? ticks : nullptr, ci_stride(c, 1), prog);
                        }
                    };
                    // the heaviest tiles of the last frame get 4 waves each; they are
                    // launched first, on the main stream, and the rest concurrently on
                    // stream2 (same-stream launches would serialise)
                    // (multi-GPU shards, where kw > 1: the rest then run at 1 wave per
                    // tile, the most efficient per lane)
                    // measured wins at 1/2 and 1/4 shards (nb > n_simd); a loss at 1/8
                    // (1020 tiles: 294 -> 307 ms), so smaller launches never split
                    // one GPU (kw == 1): since the Matte chain runs 3 waves/SIMD the whole
                    // frame's lane time is below its heaviest tile's chain, so the heaviest
                    // tiles get 4 waves there too (config B: chain 328.5 -> 313.3 ms)
                    // (measured a loss on the mesh chain, D 825 -> 920 ms, and on kX, G 509 -> 517 ms:
                    // one GPU splits only the 3-wave Matte analytic chain)
                    bool split1 = false;
                    if (kw == 1 && G == 1 && !kx && !mesh_only) {
                        unsigned lds1 = 0;
                        (void)ci_layout(c->lay_ci, 1, 1, lds1);
                        split1 = ci_eu3_fits(c, lds1, lds_nodes);
                    }
                    int64_t heavy = (learned && G == 1 && (kw > 1 ? nb > c->n_simd : split1) && ci_split_enabled(c))
                                        ? std::min<int64_t>(c->heavy_k, nb) : 0;
                    if (ci_heavy_override(c) >= 0 && learned && G == 1)   // tests and experiments force the split
                        heavy = std::min<int64_t>(ci_heavy_override(c), nb);
                    // a multi-wave Matte shard that fits the wave slots (1/8 of B: 1020 tiles at 4 waves)
                    // is bound by its heaviest tiles' pixel-serial chains: those at 8 waves, the
                    // rest at kw, next-pixel speculation in both (the N=8 shards' max 121.9 ->
                    // ~107 ms with 32; 4-32 within a few ms; all tiles at 8 waves: 178 ms)
                    if (heavy == 0 && ci_heavy_override(c) < 0 && learned && G == 1 && kw > 1 && nb <= c->n_simd &&
                        !kx && !mesh_only && ci_split_enabled(c) && c->knobs.ci_split8 > 0) {
                        heavy = std::min<int64_t>(c->knobs.ci_split8, nb / 16);
                        light_kw = true;
                        light_w = kw;
                        heavy_w = 8;
                    }
                    if (heavy >= nb) heavy = 0;   // nothing left for the light launch: one launch at kw
                    c->last_heavy = heavy;
                    if (ticks) {   // label every slot with the waves it actually runs at
                        c->h_slot_kw.assign((size_t)nb, (uint8_t)(heavy > 0 ? light_w : kw));
                        for (int64_t i = 0; i < heavy; i++) c->h_slot_kw[c->h_slot_order[(size_t)i]] = (uint8_t)heavy_w;
                    }
                    // PBRT_PATHS_OVERLAP (a learned split, G == 1): the completion-driven path stage.
                    //  - the heavy launch on the main stream (normal priority);
                    //  - the light launch on stream3 (high priority: it wins every slot that frees
                    //    while it has workgroups left), behind a k_gate that opens once every heavy
                    //    workgroup has started, so it never delays a heavy tile's start;
                    //  - the path stage on stream2 (normal priority): chunks of the tiles in their
                    //    chains' completion order (k_chain_ci's completion list), each behind a k_gate
                    //    that opens when its tiles' chains have ended. The chunks halve (1/2, 1/4, ...
                    //    of the tiles; the last 1/2^(K-1)), so most path work is queued while the
                    //    chains run and takes the slots they free once no chain workgroup waits.
                    // Progress-driven, not timed (it replaces round 5's timed wait); only the
                    // schedule changes, never a result.
                    const bool ov_ok = c->knobs.paths_overlap > 0 && paths_ci_exact && learned && !c->ov_retry &&
                                       c->ov_stalls < 2;
                    const bool overlap = heavy > 0 && ov_ok;
                    // no split: the one chain launch on stream3 (its workgroups win the slots the
                    // path chunks also wait for); the completion list needs one tile per workgroup
                    const bool overlap1 = heavy == 0 && ov_ok && c->knobs.paths_overlap_all && (kw > 1 || G == 1);
                    if ((overlap || overlap1) && !c->stream3) {   // created on first use
                        int least = 0, greatest = 0;
                        HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
                        HIPCHK(c, hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, greatest));
                        HIPCHK(c, hipEventCreateWithFlags(&c->ev_l2, hipEventDisableTiming));
                        HIPCHK(c, hipEventCreateWithFlags(&c->ev_p1, hipEventDisableTiming));
                    }
                    if ((overlap || overlap1) && c->prog_cap < nb + kProgHead) {
                        if (c->d_prog) (void)hipFree(c->d_prog);
                        c->d_prog = nullptr;
                        c->prog_cap = 0;
                        HIPCHK(c, hipMalloc((void**)&c->d_prog, sizeof(uint32_t) * (size_t)(nb + kProgHead)));
                        c->prog_cap = nb + kProgHead;
                    }
                    auto paths = [&]() -> int {   // the path chunks on stream2, each behind its k_gate
                        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_split, 0));
                        for (int64_t s0 = 0, j = 0; s0 < nb; j++) {
                            const int64_t e0 = j + 1 >= c->knobs.paths_overlap ? nb
                                                                              : s0 + std::max<int64_t>(1, (nb - s0) / 2);
                            hipLaunchKernelGGL(k_gate, dim3(1), dim3(kWave), 0, c->stream2, c->d_prog, (uint32_t)s0,
                                               (uint32_t)e0, c->d_ctr);
                            launch_paths(c->d_prog + kProgHead + s0, e0 - s0, c->stream2);
                            s0 = e0;
                        }
                        HIPCHK(c, hipEventRecord(c->ev_p1, c->stream2));
                        return PBRT_OK;
                    };
                    if (overlap || overlap1) {
                        HIPCHK(c, hipMemsetAsync(c->d_prog, 0, kProgHead * sizeof(uint32_t), c->stream));
                        HIPCHK(c, hipMemsetAsync(c->d_prog + kProgHead, 0xFF, sizeof(uint32_t) * (size_t)nb, c->stream));
                        HIPCHK(c, hipEventRecord(c->ev_split, c->stream));
                    }
                    if (overlap1) {
                        HIPCHK(c, hipStreamWaitEvent(c->stream3, c->ev_split, 0));
                        launch_ci(kw, nb, order, c->stream3, c->d_prog);
                        HIPCHK(c, hipGetLastError());
                        HIPCHK(c, hipEventRecord(c->ev_l2, c->stream3));
                        const int r = paths();
                        if (r != PBRT_OK) return r;
                        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_l2, 0));
                        c->ov_done = nb;
                    } else if (overlap) {
                        split_launch = true;
                        launch_ci(heavy_w, heavy, order, c->stream, c->d_prog);
                        split_launch = false;
                        HIPCHK(c, hipGetLastError());   // the gates below wait for these workgroups
                        auto light = [&]() -> int {
                            HIPCHK(c, hipStreamWaitEvent(c->stream3, c->knobs.gate_hold ? c->ev_p1 : c->ev_split, 0));
                            hipLaunchKernelGGL(k_gate, dim3(1), dim3(kWave), 0, c->stream3, c->d_prog,
                                               (uint32_t)heavy, (uint32_t)heavy, c->d_ctr);
                            launch_ci(light_w, nb - heavy, order + heavy, c->stream3, c->d_prog);
                            HIPCHK(c, hipGetLastError());
                            HIPCHK(c, hipEventRecord(c->ev_l2, c->stream3));
                            return PBRT_OK;
                        };
                        const int r1 = c->knobs.gate_hold ? paths() : light();
                        if (r1 != PBRT_OK) return r1;
                        const int r2 = c->knobs.gate_hold ? light() : paths();
                        if (r2 != PBRT_OK) return r2;
                        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_l2, 0));
                        c->ov_done = nb;
                    } else if (heavy > 0) {
                        HIPCHK(c, hipEventRecord(c->ev_split, c->stream));
                        split_launch = true;
                        launch_ci(heavy_w, heavy, order, c->stream, nullptr);
                        split_launch = false;
                        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_split, 0));
                        launch_ci(light_w, nb - heavy, order + heavy, c->stream2, nullptr);
                        HIPCHK(c, hipEventRecord(c->ev_join, c->stream2));
                        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
                    } else {
                        launch_ci(kw, nb, order, c->stream, nullptr);
                    }
                }
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 1], c->stream));
                if (c->use_dl) {
                    const int64_t nrec = nb * c->wb.ppt;
                    if (rp.spp > 1)
                        hipLaunchKernelGGL(kx ? k_dl_samples<true> : k_dl_samples<false>,
                                           dim3((unsigned)std::min<int64_t>((nrec * (rp.spp - 1) + kWave - 1) / kWave,
                                                                            (int64_t)c->n_simd * 64)),
                                           dim3(kWave), 0, c->stream, with_slot(sc, 3), rp, c->wb, sb, nrec);
                    hipLaunchKernelGGL(k_dl_panics, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, c->stream, rp,
                                       c->wb, sb, nrec, c->d_ctr);
                } else if (paths_wf_enabled(c) || paths_ci_pixels(c, rp) == 0) {
                    // the path wavefront: mesh scenes, and whatever k_paths_ci cannot
                    // take (a tree beyond LDS, more than 64 / P lights)
                    if (rp.mode == PBRT_MODE_THROUGHPUT)
                        hipLaunchKernelGGL(kx ? k_mb_setup<true> : k_mb_setup<false>, dim3((unsigned)(nb * c->wb.ppt)), dim3(kWave),
                                           (unsigned)c->lay.total, c->stream, with_slot(sc, 4), rp, c->lay, c->d_jump,
                                           c->wb, sb, nb);
                    const int rcp = paths_wavefront(c, with_slot(sc, rp.mode == PBRT_MODE_THROUGHPUT ? 5 : 3), sb, nb);
                    if (rcp != PBRT_OK) return rcp;
                } else if (rp.mode == PBRT_MODE_THROUGHPUT && paths_ci_pixels(c, rp) > 0) {
                    // setup (StartPixel + bounce 1 per pixel), then lane-refill paths
                    hipLaunchKernelGGL(kx ? k_mb_setup<true> : k_mb_setup<false>, dim3((unsigned)(nb * c->wb.ppt)),
                                       dim3(kWave), (unsigned)c->lay.total, c->stream, with_slot(sc, 4), rp, c->lay,
                                       c->d_jump, c->wb, sb, nb);
                    const int pp = paths_ci_pixels(c, rp);
                    const int per = rp.ndims * rp.spp;
                    auto kern = kx ? (pp == 8 ? k_paths_ci<8, true, true> : k_paths_ci<4, true, true>)
                                   : (pp == 8 ? k_paths_ci<8, true> : pp == 2 ? k_paths_ci<2, true> : k_paths_ci<4, true>);
                    const int sl = paths_ci_s1d_lds(c, rp, pp) ? 1 : 0;
                    const int lds = pp == 8 ? paths_group_lds<8>(sl * per) : pp == 2 ? paths_group_lds<2>(sl * per)
                                                                                     : paths_group_lds<4>(sl * per);
                    hipLaunchKernelGGL(kern, dim3((unsigned)((nb * c->wb.ppt + pp - 1) / pp)), dim3(kWave),
                                       (unsigned)lds, c->stream, with_slot(sc, 5), rp, c->wb, sb, nb * c->wb.ppt,
                                       c->d_ctr, sl, nullptr);
                }
                else if (c->ov_done > 0) {   // the completion-driven path stage (stream2) ends the chain stage
                    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_p1, 0));
                } else {
                    launch_paths(nullptr, nb, c->stream);
                }
                HIPCHK(c, hipEventRecord(c->bev[3 * bi + 2], c->stream));
                hipLaunchKernelGGL(k_film, dim3((unsigned)nb), dim3(kFilmThreads), (unsigned)film_lds_bytes(rp), c->stream,
                                   c->d_film, rp, c->wb, sb, nb, c->d_films, c->d_cancel_seen, c->d_ctr);
                hipLaunchKernelGGL(k_panic_reduce, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, c->stream, c->wb,
                                   sb, nb, c->d_panics, c->d_ctr);

            }
        } else {
            c->last_kernel = PBRT_KERNEL_SERIAL;
            c->n_batches = 0;
            int64_t blocks = (rp.n_slots + rp.lanes_per_wave - 1) / rp.lanes_per_wave;
            auto kern = k_render_exact<1>;
            if (c->min_waves == 2) kern = k_render_exact<2>;
            else if (c->min_waves == 4) kern = k_render_exact<4>;
            else if (c->min_waves == 8) kern = k_render_exact<8>;
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kWave), 0, c->stream, with_slot(sc, 6), rp, c->d_films,
                               c->d_s1d, c->d_panics, c->d_ctr);
        }
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    int64_t npx = rp.film_w * rp.film_h;
    hipLaunchKernelGGL(k_merge_film, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, c->stream, c->d_film, rp,
                       c->d_films, out, c->d_cancel_seen);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    c->rendered = true;
    return PBRT_OK;
}
}  // namespace

int pbrt_gpu_render_async(pbrt_gpu_ctx* c, const pbrt_render_desc* rd) {
    return pbrt_gpu_render_async_into(c, rd, nullptr);
}

int pbrt_gpu_synchronize(pbrt_gpu_ctx* c, pbrt_gpu_stats* stats) {
    if (!c) return PBRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    const hipError_t se = hipStreamSynchronize(c->stream);
    bool cancelled = false;
    {   // the render has ended: its cancel flag dies with it
        std::lock_guard<std::mutex> lk(c->cancel_mu);
        cancelled = c->in_flight && c->cancel_req;
        c->in_flight = false;
        c->cancel_req = false;
        __atomic_store_n(c->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    HIPCHK(c, se);
    if (cancelled) {   // the kernels stopped early: the film and the schedule feedback are not valid
        c->ticks_pending = false;
        c->rendered = false;
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            stats->kernel = c->last_kernel;
            stats->total_ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->t_start).count();
        }
        return set_err(c, PBRT_E_CANCELLED, "cancelled by pbrt_gpu_cancel");
    }
    Counters ctr;
    HIPCHK(c, hipMemcpy(&ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost));
    if (ctr.gate_stall) {
        // the completion-driven path stage's gates saw the chains stand still
        // (k_gate): the film misses path work. Render the frame again with the path
        // stage after the chains; the chains replay the same streams, so the
        // result is the one an overlapped frame gives.
        if (++c->ov_stalls == 2)
            std::fprintf(stderr, "pbrt: k_gate stalled twice (kernels serialised across streams, e.g. by a "
                                 "counter-collecting profiler): the path stage now runs after the chains\n");
        c->ov_retry = true;
        const int rr = render_enqueue(c, &c->last_rd, c->last_film_device);
        c->ov_retry = false;
        if (rr != PBRT_OK) return rr;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(&ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost));
        if (ctr.gate_stall) return set_err(c, PBRT_E_HIP, "k_gate stalled without the overlap");
    } else if (c->ov_done > 0) {
        c->ov_stalls = 0;
    }
    float ms = 0, ms_merge = 0;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    (void)hipEventElapsedTime(&ms_merge, c->ev1, c->ev2);
    int rc = PBRT_OK;
    pbrt_gpu_stats st;
    std::memset(&st, 0, sizeof(st));
    st.tiles_rendered = (uint64_t)c->rp.n_slots;
    st.camera_samples = ctr.camera_samples;
    st.paths_traced = ctr.paths;
    st.kernel_ms = ms;
    st.merge_ms = ms_merge;
    st.kernel = c->last_kernel;
    st.batches = c->n_batches;
    st.rays_closest = ctr.closest_rays;
    st.rays_shadow = ctr.shadow_rays;
    for (int b = 0; b < c->n_batches; b++) {
        float a = 0, p = 0;
        (void)hipEventElapsedTime(&a, c->bev[3 * b + 0], c->bev[3 * b + 1]);
        (void)hipEventElapsedTime(&p, c->bev[3 * b + 1], c->bev[3 * b + 2]);
        st.chain_ms += a;
        st.paths_ms += p;
    }
    if (c->ticks_pending) {   // heaviest-first slot order for the next frame of this configuration
        c->ticks_pending = false;
        std::vector<uint32_t> t((size_t)c->ticks_n);
        HIPCHK(c, hipMemcpy(t.data(), c->d_ticks, sizeof(uint32_t) * t.size(), hipMemcpyDeviceToHost));
        c->h_last_ticks = t;   // pbrt_gpu_tile_ticks
        if (kTickPlanes > 1) {   // diagnostics builds: start and end clocks (pbrt_gpu_tile_clocks)
            c->h_tick_clocks.resize(2 * t.size());
            HIPCHK(c, hipMemcpy(c->h_tick_clocks.data(), c->d_ticks + t.size(), sizeof(uint32_t) * 2 * t.size(),
                                hipMemcpyDeviceToHost));
        }
        // cost at 1 wave per tile: 2 and 4 waves measured 1.3x / 1.8x faster per tile
        std::vector<double> cost(t.size());
        double sum = 0;
        for (size_t i = 0; i < t.size(); i++) {
            const int w = i < c->h_slot_kw.size() ? c->h_slot_kw[i] : 1;
            cost[i] = (double)t[i] * (w == 8 ? 2.3 : w == 4 ? 1.8 : w == 2 ? 1.3 : 1.0);
            sum += cost[i];
        }
        c->h_slot_order.resize(t.size());
        for (size_t i = 0; i < t.size(); i++) c->h_slot_order[i] = (uint32_t)i;
        std::stable_sort(c->h_slot_order.begin(), c->h_slot_order.end(),
                         [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
        // heavy: tiles whose 1-wave chain alone would take over 0.7x the
        // frame's throughput bound (summed cost over the chain's waves/SIMD)
        const double thr = 0.7 * sum / ((double)c->ci_wps * (double)c->n_simd);
        int64_t k = 0;
        while (k < (int64_t)t.size() && cost[c->h_slot_order[(size_t)k]] > thr) k++;
        // at most a quarter of the wave slots; at most 1/16 of them when the tiles
        // outnumber the one-wave slots (one GPU, 1/2 shards), whose light launch then
        // fills the GPU longer than the heavy tiles take (1/2 of B: 216 -> 202 ms with
        // 64 against 256; 1/4 of B: best at 256, 126-129 ms against 131-142 at 128-384)
        const int64_t cap = (int64_t)t.size() > (int64_t)c->ci_wps * c->n_simd ? c->n_simd / 16 : c->n_simd / 4;
        c->heavy_k = std::min<int64_t>(k, cap);
        if (ci_heavy_override(c) >= 0) c->heavy_k = ci_heavy_override(c);
        c->order_key = c->ticks_key;
        if (ci_order_cache(c)) sched_cache_put(c, c->ticks_key, c->h_slot_order, c->heavy_k);
    }
    if (ctr.any_panic) {
        std::vector<PanicRec> pr((size_t)c->rp.n_slots);
        HIPCHK(c, hipMemcpy(pr.data(), c->d_panics, sizeof(PanicRec) * pr.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < pr.size(); i++) {
            if (pr[i].kind == 0) continue;
            st.panic_kind = pr[i].kind;
            st.panic_tile = (int32_t)(c->rp.tile_begin + (int64_t)i * c->rp.tile_stride);
            st.panic_pixel_x = pr[i].px;
            st.panic_pixel_y = pr[i].py;
            st.panic_sample = pr[i].sample;
            st.panic_bounce = pr[i].bounce;
            break;
        }
        if (st.panic_kind == -1) {
            rc = set_err(c, PBRT_E_UNSUPPORTED, "unsupported material");
            st.panic_kind = 0;
        } else {
            rc = set_err(c, PBRT_E_REF_PANIC, "the Go reference panics on this input");
        }
    }
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->t_start).count();
    if (stats) *stats = st;
    return rc;
}

int pbrt_gpu_render(pbrt_gpu_ctx* c, const pbrt_render_desc* rd, double* film_xyz, pbrt_gpu_stats* stats) {
    if (!c) return PBRT_E_INVALID;
    int rc = pbrt_gpu_render_async(c, rd);
    if (rc != PBRT_OK) return rc;
    rc = pbrt_gpu_synchronize(c, stats);
    if (rc != PBRT_OK) return rc;
    if (film_xyz) return pbrt_gpu_film_download(c, film_xyz);
    return PBRT_OK;
}

double* pbrt_gpu_film_device(pbrt_gpu_ctx* c) { return c ? c->d_out : nullptr; }
void* pbrt_gpu_stream(pbrt_gpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

int pbrt_gpu_film_download(pbrt_gpu_ctx* c, double* film_xyz) {
    if (!c || !film_xyz || !c->rendered) return PBRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(film_xyz, c->film_target ? c->film_target : c->d_out,
                        sizeof(double) * (size_t)(c->rp.film_w * c->rp.film_h * 3),
                        hipMemcpyDeviceToHost));
    return PBRT_OK;
}

static int intersect_batch(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, int any, pbrt_hit_soa* hits,
                           uint8_t* occluded) {
    if (!c || !rays || (!hits && !occluded)) return PBRT_E_INVALID;
    if (n == 0) return PBRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<double> packed(n * 7);
    for (size_t i = 0; i < n; i++) {
        double* q = &packed[7 * i];
        q[0] = rays->ox[i]; q[1] = rays->oy[i]; q[2] = rays->oz[i];
        q[3] = rays->dx[i]; q[4] = rays->dy[i]; q[5] = rays->dz[i];
        q[6] = rays->tmax ? rays->tmax[i] : gomath::kInf;
    }
    size_t nout = any ? n : 9 * n;
    double *d_in = nullptr, *d_o = nullptr;
    HIPCHK(c, hipMalloc((void**)&d_in, sizeof(double) * packed.size()));
    if (hipMalloc((void**)&d_o, sizeof(double) * nout) != hipSuccess) {
        (void)hipFree(d_in);
        return set_err(c, PBRT_E_HIP, "hipMalloc");
    }
    std::vector<double> o(nout);
    hipError_t e = hipMemcpyAsync(d_in, packed.data(), sizeof(double) * packed.size(), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        DevScene sc = dev_scene(c, false);
        hipLaunchKernelGGL(k_intersect, dim3((unsigned)((n + kWave - 1) / kWave)), dim3(kWave), 0, c->stream,
                           with_slot(sc, 7),
                           (int64_t)n, d_in, d_o, any);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(o.data(), d_o, sizeof(double) * nout, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_in);
    (void)hipFree(d_o);
    if (e != hipSuccess) return set_err(c, PBRT_E_HIP, hipGetErrorString(e));
    int rc = PBRT_OK;
    for (size_t i = 0; i < n; i++) {
        if (any) {
            if (gomath::is_nan(o[i])) rc = PBRT_E_REF_PANIC;
            occluded[i] = o[i] == 1.0;
        } else {
            const double* r = &o[9 * i];
            if (gomath::is_nan(r[0])) { rc = PBRT_E_REF_PANIC; hits->hit[i] = 0; continue; }
            hits->hit[i] = r[0] == 1.0;
            if (hits->t_max) hits->t_max[i] = r[1];
            if (hits->prim) hits->prim[i] = (int32_t)r[2];
            if (hits->px) hits->px[i] = r[3];
            if (hits->py) hits->py[i] = r[4];
            if (hits->pz) hits->pz[i] = r[5];
            if (hits->nx) hits->nx[i] = r[6];
            if (hits->ny) hits->ny[i] = r[7];
            if (hits->nz) hits->nz[i] = r[8];
        }
    }
    if (rc != PBRT_OK) set_err(c, rc, "the Go reference panics on at least one ray");
    return rc;
}

int pbrt_gpu_intersect(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, pbrt_hit_soa* hits) {
    return intersect_batch(c, rays, n, 0, hits, nullptr);
}
int pbrt_gpu_intersect_p(pbrt_gpu_ctx* c, const pbrt_ray_soa* rays, size_t n, uint8_t* occluded) {
    return intersect_batch(c, rays, n, 1, nullptr, occluded);
}

void pbrt_gpu_cancel(pbrt_gpu_ctx* c) {
    if (!c) return;
    std::lock_guard<std::mutex> lk(c->cancel_mu);
    if (!c->in_flight) return;   // nothing to cancel: no render is in flight
    c->cancel_req = true;
    __atomic_store_n(c->h_cancel, 1, __ATOMIC_SEQ_CST);
}
const char* pbrt_gpu_last_error(const pbrt_gpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

void pbrt_gpu_destroy(pbrt_gpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (hipStream_t st : {c->stream, c->stream2, c->stream3})
        if (st) (void)hipStreamSynchronize(st);
    void* bufs[] = {c->d_shapes, c->d_materials, c->d_prims, c->d_nodes, c->d_order, c->d_lights, c->d_camera, c->d_film,
                    c->d_dist,   c->d_films,     c->d_s1d,   c->d_panics, c->d_ctr,   c->d_out,    c->d_jump,
                    c->d_wave,   c->d_fprims, c->d_ticks, c->d_slot_order, c->d_groups,
                    c->d_gmasks, c->d_cost,   c->d_cost_keys, c->d_pw, c->d_cancel_seen, c->d_prog};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    mesh_bvh_free(c->mesh);
    for (hipEvent_t e : c->bev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->ev_split) (void)hipEventDestroy(c->ev_split);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    for (hipEvent_t e : {c->ev_l2, c->ev_p1})
        if (e) (void)hipEventDestroy(e);
    if (c->stream3) {
        (void)hipStreamSynchronize(c->stream3);
        (void)hipStreamDestroy(c->stream3);
    }
    if (c->stream2) {
        (void)hipStreamSynchronize(c->stream2);
        (void)hipStreamDestroy(c->stream2);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->h_cancel) (void)hipHostFree(c->h_cancel);
    delete c;
}

// film.go:142-179 WriteImage pixel conversion
int pbrt_film_to_rgba8(const double* film, int64_t w, int64_t h, uint8_t* rgba) {
    if (!film || !rgba || w <= 0 || h <= 0) return PBRT_E_INVALID;
    for (int64_t i = 0; i < w * h; i++) {
        for (int c = 0; c < 3; c++)
            rgba[i * 4 + c] = (uint8_t)(gomath::to_int(gomath::clamp(film[i * 3 + c], 0, 1) * 255) & 0xFF);
        rgba[i * 4 + 3] = 255;
    }
    return PBRT_OK;
}

}  // extern "C"

// ============================================================ diagnostics

namespace {
__global__ void k_probe(int op, const double* __restrict__ in, int64_t n, int in_stride, double* __restrict__ out,
                        int out_stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* a = in + i * in_stride;
    double* o = out + i * out_stride;
    switch (op) {
        case PBRT_PROBE_SIN: o[0] = gomath::sin(a[0]); break;
        case PBRT_PROBE_COS: o[0] = gomath::cos(a[0]); break;
        case PBRT_PROBE_TAN: o[0] = gomath::tan(a[0]); break;
        case PBRT_PROBE_ATAN: o[0] = gomath::atan(a[0]); break;
        case PBRT_PROBE_ATAN2: o[0] = gomath::atan2(a[0], a[1]); break;
        case PBRT_PROBE_ASIN: o[0] = gomath::asin(a[0]); break;
        case PBRT_PROBE_ACOS: o[0] = gomath::acos(a[0]); break;
        case PBRT_PROBE_SQRT: o[0] = gomath::sqrt(a[0]); break;
        case PBRT_PROBE_DIV: o[0] = a[0] / a[1]; break;
        case PBRT_PROBE_NEXTAFTER: o[0] = gomath::nextafter(a[0], a[1]); break;
        case PBRT_PROBE_MAX: o[0] = gomath::max(a[0], a[1]); break;
        case PBRT_PROBE_MIN: o[0] = gomath::min(a[0], a[1]); break;
        case PBRT_PROBE_OFFSET_RAY_ORIGIN: {
            V3 r = offset_ray_origin(load3(a), load3(a + 3), load3(a + 6), load3(a + 9));
            o[0] = r.x; o[1] = r.y; o[2] = r.z;
            break;
        }
        case PBRT_PROBE_EFLOAT_ADD: {
            int panic = 0;
            EF r = ef_add(ef_new(a[0], a[1], panic), ef_new(a[2], a[3], panic), panic);
            o[0] = r.v; o[1] = r.lo; o[2] = r.hi; o[3] = panic;
            break;
        }
        case PBRT_PROBE_TRANSFORM_RAY: {
            pbrt_matrix4x4 m;
            for (int k = 0; k < 16; k++) m.m[k / 4][k % 4] = a[k];
            Ray r{load3(a + 16), load3(a + 19), gomath::kInf, 0};
            Ray w = xf_ray(m, r, nullptr, nullptr);
            o[0] = w.o.x; o[1] = w.o.y; o[2] = w.o.z; o[3] = w.d.x; o[4] = w.d.y; o[5] = w.d.z;
            break;
        }
        case PBRT_PROBE_SPAWN_RAY_TO: {
            V3 p0 = load3(a), e0 = load3(a + 3), n0 = load3(a + 6), p1 = load3(a + 9), e1 = load3(a + 12),
               n1 = load3(a + 15);
            V3 origin = offset_ray_origin(p0, e0, n0, p1 - p0);
            V3 target = offset_ray_origin(p1, e1, n1, origin - p1);
            V3 d = target - origin;
            o[0] = p0.x; o[1] = p0.y; o[2] = p0.z; o[3] = d.x; o[4] = d.y; o[5] = d.z; o[6] = 1 - 0.0001;
            break;
        }
        case PBRT_PROBE_PCG: {
            Pcg r;
            pcg_seed(r, (uint64_t)a[0]);
            for (int k = 0; k < out_stride; k++) o[k] = pcg_float(r);
            break;
        }
        case PBRT_PROBE_MIN_NONAN: o[0] = gomath::min_nonan(a[0], a[1]); break;
        case PBRT_PROBE_MAX_NONAN: o[0] = gomath::max_nonan(a[0], a[1]); break;
        case PBRT_PROBE_EFLOAT_MUL:
        case PBRT_PROBE_EFLOAT_DIV: {
            int panic = 0;
            EF x = ef_new(a[0], a[1], panic), y = ef_new(a[2], a[3], panic);
            EF r = op == PBRT_PROBE_EFLOAT_MUL ? ef_mul(x, y, panic) : ef_div(x, y, panic);
            o[0] = r.v; o[1] = r.lo; o[2] = r.hi; o[3] = panic;
            break;
        }
        case PBRT_PROBE_NEXT_FLOAT_UP: o[0] = gomath::next_up(a[0]); break;
        case PBRT_PROBE_NEXT_FLOAT_DOWN: o[0] = gomath::next_down(a[0]); break;
        default: o[0] = gomath::nan();
    }
}
}  // namespace

extern "C" int pbrt_gpu_probe(int device, int op, const double* in, size_t n, int in_stride, double* out,
                              int out_stride) {
    if (!in || !out || in_stride <= 0 || out_stride <= 0) return PBRT_E_INVALID;
    if (n == 0) return PBRT_OK;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return PBRT_E_HIP;
    double *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc((void**)&d_in, sizeof(double) * n * in_stride) != hipSuccess) return PBRT_E_HIP;
    if (hipMalloc((void**)&d_out, sizeof(double) * n * out_stride) != hipSuccess) {
        (void)hipFree(d_in);
        return PBRT_E_HIP;
    }
    hipError_t e = hipMemcpy(d_in, in, sizeof(double) * n * in_stride, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, d_in, (int64_t)n,
                           in_stride, d_out, out_stride);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(double) * n * out_stride, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return e == hipSuccess ? PBRT_OK : PBRT_E_HIP;
}

extern "C" int pbrt_gpu_counters(pbrt_gpu_ctx* c, uint64_t* out, int n) {
    if (!c || !out) return PBRT_E_INVALID;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) return PBRT_E_HIP;
    Counters ctr;
    if (hipMemcpy(&ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost) != hipSuccess) return PBRT_E_HIP;
    const uint64_t v[kNumCounters] = {ctr.paths,    ctr.camera_samples, ctr.closest_rays, ctr.shadow_rays,
                                      (uint64_t)ctr.any_panic, ctr.windows, ctr.phase[0], ctr.phase[1],
                                      ctr.phase[2], ctr.phase[3], ctr.phase[4], ctr.phase[5],
                                      ctr.phase[6], ctr.phase[7]};
    for (int i = 0; i < n && i < kNumCounters; i++)
        out[i] = i < 14 ? v[i] : i < 78 ? (uint64_t)ctr.dhist[i - 14] : i == 78 ? ctr.busy : i == 79 ? ctr.nps_issued
                                                                                                   : ctr.odd_d;
    return kNumCounters;
}

extern "C" int pbrt_gpu_mesh_info(pbrt_gpu_ctx* c, double* out, int n) {
    if (!c || !out) return -PBRT_E_INVALID;
    const double v[] = {(double)c->mesh.n_tris, (double)c->mesh.n_nodes, (double)c->mesh.depth, c->mesh.build_ms,
                        (double)c->mesh.n_meshes, (double)PBRT_MESH_WIDE};
    const int m = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = v[i];
    return m;
}
extern "C" int pbrt_gpu_mesh_counters(uint64_t* out, int n, int reset) {
#ifdef PBRT_MESH_COUNT
    unsigned long long h[kMeshCountSlots * 6];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mesh_count), sizeof(h)) != hipSuccess) return -PBRT_E_HIP;
    for (int i = 0; i < n && i < kMeshCountSlots * 6; i++) out[i] = h[i];
    if (reset) {
        std::memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_mesh_count), h, sizeof(h)) != hipSuccess) return -PBRT_E_HIP;
    }
    return kMeshCountSlots * 6;
#else
    (void)out; (void)n; (void)reset;
    return 0;
#endif
}

extern "C" int pbrt_gpu_mesh_download(pbrt_gpu_ctx* c, void* nodes, int32_t* gid, float* tris) {
    if (!c) return PBRT_E_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) return PBRT_E_HIP;
    const size_t nn = mesh_node_bytes(c->mesh.n_nodes), nt = (size_t)c->mesh.n_tris;
    if (nodes && nn && hipMemcpy(nodes, c->mesh.nodes, nn, hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    if (gid && nt && hipMemcpy(gid, c->mesh.gid, nt * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    if (tris && nt && hipMemcpy(tris, c->mesh.tris, nt * 9 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        return PBRT_E_HIP;
    return PBRT_OK;
}

extern "C" int64_t pbrt_gpu_tile_clocks(pbrt_gpu_ctx* c, uint32_t* start, uint32_t* end, int64_t n) {
    if (!c) return -PBRT_E_INVALID;
    const int64_t m = (int64_t)c->h_tick_clocks.size() / 2;
    for (int64_t i = 0; i < m && i < n; i++) {
        if (start) start[i] = c->h_tick_clocks[(size_t)i];
        if (end) end[i] = c->h_tick_clocks[(size_t)(m + i)];
    }
    return m;
}

extern "C" int64_t pbrt_gpu_tile_ticks(pbrt_gpu_ctx* c, uint32_t* out, int64_t n, int64_t* heavy) {
    if (!c) return -PBRT_E_INVALID;
    if (heavy) *heavy = c->last_heavy;
    const int64_t m = (int64_t)c->h_last_ticks.size();
    for (int64_t i = 0; out && i < n && i < m; i++) out[i] = c->h_last_ticks[(size_t)i];
    return m;
}

extern "C" void pbrt_gpu_schedule_cache_clear(void) {
    std::lock_guard<std::mutex> lk(g_sched_mu);
    g_sched.clear();
}

extern "C" int64_t pbrt_gpu_overlap_slots(pbrt_gpu_ctx* c) {
    if (!c) return -PBRT_E_INVALID;
    return c->ov_done;
}

extern "C" int pbrt_gpu_schedule_source(pbrt_gpu_ctx* c) {
    if (!c) return -PBRT_E_INVALID;
    return c->sched_src;
}

extern "C" int64_t pbrt_gpu_tile_costs(pbrt_gpu_ctx* c, float* out, int64_t n) {
    if (!c) return -PBRT_E_INVALID;
    if (!c->probed || !c->d_cost) return 0;
    if (out && n > 0) {
        const int64_t m = std::min<int64_t>(n, c->cost_n);
        if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(out, c->d_cost, sizeof(float) * 4 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess)
            return -PBRT_E_HIP;
    }
    return c->cost_n;
}

// Region cycles of trajectory steps (PBRT_STEP_TIMING builds only; else zeros):
// [0] loop top / light-sample draws, [1] closest-hit traversal + interaction,
// [2] BSDF setup, [3] light sampling (full paths), [4] BSDF sample + spawn + RR.
extern "C" int pbrt_gpu_step_cycles(uint64_t* out, int n, int reset) {
#ifdef PBRT_STEP_TIMING
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_step_cycles), sizeof(h)) != hipSuccess) return PBRT_E_HIP;
    for (int i = 0; i < n && i < 8; i++) out[i] = h[i];
    if (reset) {
        std::memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_cycles), h, sizeof(h)) != hipSuccess) return PBRT_E_HIP;
    }
#else
    for (int i = 0; i < n && i < 8; i++) out[i] = 0;
    (void)reset;
#endif
    return 8;
}

#ifndef PBRT_BUILD_ID
#define PBRT_BUILD_ID "unknown"
#endif
extern "C" const char* pbrt_gpu_build_id(void) { return PBRT_BUILD_ID; }

extern "C" int pbrt_abi_sizes(size_t* out, int n) {
    const size_t s[] = {sizeof(pbrt_matrix4x4),   sizeof(pbrt_transform),    sizeof(pbrt_shape_desc),
                        sizeof(pbrt_material_desc), sizeof(pbrt_primitive_desc), sizeof(pbrt_bvh_node),
                        sizeof(pbrt_light_desc),  sizeof(pbrt_camera_desc),  sizeof(pbrt_film_desc),
                        sizeof(pbrt_distribution_desc), sizeof(pbrt_scene_desc), sizeof(pbrt_render_desc),
                        sizeof(pbrt_gpu_stats),   sizeof(pbrt_ray_soa),      sizeof(pbrt_hit_soa),
                        sizeof(pbrt_gpu_opts),    sizeof(pbrt_mesh_desc)};
    int m = (int)(sizeof(s) / sizeof(s[0]));
    for (int i = 0; i < n && i < m; i++) out[i] = s[i];
    return m;
}
