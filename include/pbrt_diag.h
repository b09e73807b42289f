/*
 * pbrt_diag.h — diagnostics of the device path (not part of the reference
 * interface). Evaluates individual device functions on a batch of inputs so
 * the reference's known-answer tests and large random sweeps can be checked
 * against the oracle on the GPU itself (Go-math trig, correctly rounded
 * division / sqrt, OffsetRayOrigin, EFloat, TransformRay, SpawnRayToInteraction,
 * PCG32 stream).
 */
#ifndef PBRT_DIAG_H
#define PBRT_DIAG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    PBRT_PROBE_SIN = 1,        /* in a          -> out Sin(a)                 */
    PBRT_PROBE_COS = 2,
    PBRT_PROBE_TAN = 3,
    PBRT_PROBE_ATAN = 4,
    PBRT_PROBE_ATAN2 = 5,      /* in y, x                                    */
    PBRT_PROBE_ASIN = 6,
    PBRT_PROBE_ACOS = 7,
    PBRT_PROBE_SQRT = 8,
    PBRT_PROBE_DIV = 9,        /* in a, b       -> a / b                      */
    PBRT_PROBE_NEXTAFTER = 10, /* in x, y                                    */
    PBRT_PROBE_MAX = 11,
    PBRT_PROBE_MIN = 12,
    PBRT_PROBE_OFFSET_RAY_ORIGIN = 13, /* in p[3] perr[3] n[3] w[3] -> out[3]    */
    PBRT_PROBE_EFLOAT_ADD = 14,        /* in v1 e1 v2 e2 -> value low high panic */
    PBRT_PROBE_TRANSFORM_RAY = 15,     /* in m[16] o[3] d[3] -> o'[3] d'[3]      */
    PBRT_PROBE_SPAWN_RAY_TO = 16,      /* in p0 perr0 n0 p1 perr1 n1 -> o d tmax */
    PBRT_PROBE_PCG = 17,               /* in seed -> out[out_stride] first floats */
    PBRT_PROBE_NEXT_FLOAT_UP = 18,     /* in v -> NextFloatUp(v)   (math.go:122-124) */
    PBRT_PROBE_NEXT_FLOAT_DOWN = 19,   /* in v -> NextFloatDown(v) (math.go:126-128) */
    PBRT_PROBE_MIN_NONAN = 20,         /* in x, y (not NaN) -> device min used by EFloat */
    PBRT_PROBE_MAX_NONAN = 21,         /* in x, y (not NaN) -> device max used by EFloat */
    PBRT_PROBE_EFLOAT_MUL = 22,        /* in v1 e1 v2 e2 -> value low high panic */
    PBRT_PROBE_EFLOAT_DIV = 23         /* in v1 e1 v2 e2 -> value low high panic */
};

/* Host instantiation of the float64 vector / spectrum operations the kernels
 * use (csrc/pbrt_core.h, compiled for host and device from one source), for
 * the reference's pkg/geometry/xyz_test.go and pkg/pbrt/spectrum_test.go
 * known answers. a, b: 3 doubles; s: scalar; out: 3 doubles (scalars in out[0]). */
enum {
    PBRT_VOP_ABS = 1, PBRT_VOP_ABSDOT = 2, PBRT_VOP_ADD = 3, PBRT_VOP_CROSS = 4, PBRT_VOP_DISTANCE = 5,
    PBRT_VOP_DISTANCE_SQUARED = 6, PBRT_VOP_DIV = 7, PBRT_VOP_DIV_SCALAR = 8, PBRT_VOP_DOT = 9,
    PBRT_VOP_LENGTH = 10, PBRT_VOP_LENGTH_SQUARED = 11, PBRT_VOP_MUL = 12, PBRT_VOP_MUL_SCALAR = 13,
    PBRT_VOP_NORMALIZED = 14, PBRT_VOP_SUB = 15,
    PBRT_SOP_ADD = 16, PBRT_SOP_MUL = 17, PBRT_SOP_DIV_SCALAR = 18, PBRT_SOP_IS_BLACK = 19,
    PBRT_SOP_MUL_SCALAR = 20
};
int pbrt_diag_vec_op(int op, const double* a, const double* b, double s, double* out);

/* The BVH builder's PartitionPrimitiveInfoAt (bvh.go:163-175, Lomuto around
 * in[pivot] moved to `end`) on records (prim[i], centroid x = cx[i]) with the
 * less-than-on-centroid-x predicate of pkg/accelerator/bvh_test.go:143-264;
 * permutes both arrays in place and returns the pivot's final index. */
int64_t pbrt_diag_partition_at(int32_t* prim, double* cx, int64_t n, int64_t start, int64_t end, int64_t pivot);

/* Inputs: n records of in_stride doubles; outputs: n records of out_stride. */
int pbrt_gpu_probe(int device, int op, const double* in, size_t n, int in_stride, double* out, int out_stride);

/* Device counters of the last render (after it completed), in this order:
 * paths, camera_samples, closest_rays, shadow_rays, any_panic, windows
 * (WAVE kernel speculation rounds), then lane-0 clock64 cycles summed over
 * tiles in: StartPixel swaps, bounce 1, speculative trajectories, full paths,
 * film add, StartPixel draws, chain walk, (spare); then 64 bins of the
 * continuous-issue chain's on-chain draw counts D (bin D/2, last bin >= 126),
 * then the chain's lane-steps spent tracing (utilisation = busy / (steps x
 * lanes)), its next-pixel speculation candidates and its odd on-chain draw
 * counts (diagnostics builds).
 * Returns the number of counters available. */
struct pbrt_gpu_ctx;
int pbrt_gpu_counters(struct pbrt_gpu_ctx* ctx, uint64_t* out, int n);

/* Per-slot chain time of the last EXACT continuous-issue frame (wall_clock64
 * ticks at 100 MHz, slot i = tile tile_begin + i * tile_stride), the input of
 * the next frame's heaviest-first schedule. Copies min(n, slots) values and
 * returns the slot count (0 if the last frame recorded none). *heavy = tiles of
 * the last launch that ran at 4 waves in the heavy/light split (0: no split). */
int64_t pbrt_gpu_tile_ticks(struct pbrt_gpu_ctx* ctx, uint32_t* out, int64_t n, int64_t* heavy);

/* Diagnostics builds (make diag): the start and end wall_clock64 values (low 32
 * bits, 100 MHz) of each slot's chain in the last EXACT frame, for the
 * occupancy timeline of the launch (tools/tile_timeline.py). Copies min(n,
 * slots) values into each non-null array and returns the slot count (0 in
 * other builds). */
int64_t pbrt_gpu_tile_clocks(struct pbrt_gpu_ctx* ctx, uint32_t* start, uint32_t* end, int64_t n);

/* Where the last EXACT continuous-issue frame's tile schedule came from:
 * PBRT_SCHED_LAUNCH_ORDER (none: identity order), PBRT_SCHED_PROBE (the
 * cold-frame k_tile_cost estimate), PBRT_SCHED_LEARNED (this context's
 * previous frame), PBRT_SCHED_CACHED (the process-wide cache: another context's
 * measured frame of the same scene content and configuration). */
enum { PBRT_SCHED_LAUNCH_ORDER = 0, PBRT_SCHED_PROBE = 1, PBRT_SCHED_LEARNED = 2, PBRT_SCHED_CACHED = 3 };
int pbrt_gpu_schedule_source(struct pbrt_gpu_ctx* ctx);
/* Empties the process-wide schedule cache (the next fresh context of any scene
 * starts from the probe again). PBRT_CI_ORDER_CACHE=0 disables the cache for
 * contexts created while it is set. */
void pbrt_gpu_schedule_cache_clear(void);
/* Slots of the last EXACT frame (its last batch) whose path stage ran
 * completion-driven, released tile by tile as their chains ended
 * (PBRT_PATHS_OVERLAP); 0: the path stage ran after the chain stage. */
int64_t pbrt_gpu_overlap_slots(struct pbrt_gpu_ctx* ctx);

/* Cold-frame schedule estimate of the last EXACT frame, if that frame ran
 * render.hip's k_tile_cost probe (a fresh context or a new configuration):
 * per slot {chain work (lane-bounces), hit pixels, pixels, cost}. Copies
 * min(n, slots) records of 4 floats and returns the slot count (0: no probe). */
int64_t pbrt_gpu_tile_costs(struct pbrt_gpu_ctx* ctx, float* out, int64_t n);

/* Triangle meshes of the context (extension): out = {triangles in the tree
 * (zero-area ones are left out), nodes per ordering, deepest leaf, device
 * build ms, meshes}. Returns the number of values. */
int pbrt_gpu_mesh_info(struct pbrt_gpu_ctx* ctx, double* out, int n);
/* Copies the device LBVH: nodes = 8 * nodes-per-ordering records of 32 bytes
 * (float bmin[3], uint32 escape, float bmax[3], uint32 leaf: 0xFFFFFFFF for an
 * interior node, else first_slot << 3 | count), gid = the global triangle
 * index of each leaf slot, tris = 9 floats per slot. Any pointer may be NULL. */
int pbrt_gpu_mesh_download(struct pbrt_gpu_ctx* ctx, void* nodes, int32_t* gid, float* tris);

/* Mesh-traversal counters of libraries built with -DPBRT_MESH_COUNT (make
 * meshcount; 0 values otherwise): [8 kernel slots][closest, any][walks, nodes
 * fetched, triangles tested], slots as render.hip's with_slot(). Returns the
 * count (48), or 0 in a normal build. */
int pbrt_gpu_mesh_counters(uint64_t* out, int n, int reset);

/* Region cycles inside path steps, summed over waves (only in libraries built
 * with -DPBRT_STEP_TIMING; zeros otherwise). Returns the count (8). */
int pbrt_gpu_step_cycles(uint64_t* out, int n, int reset);

/* sizeof() of every ABI struct, for binding checks (index order as in pbrt_gpu.h). */
int pbrt_abi_sizes(size_t* out, int n);

/* Content hash of the sources this library was built from (Makefile: the first
 * 16 hex digits of sha256 over csrc/, the headers and the Makefile), so that
 * profiles and bench lines can name the build they measured. */
const char* pbrt_gpu_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
