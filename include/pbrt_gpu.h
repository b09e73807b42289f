/*
 * pbrt_gpu.h — C ABI of the MI355X-native go-pbrt hot path.
 *
 * This is the drop-in boundary for go-pbrt's ray–scene intersection and
 * path-tracing inner loop. A cgo shim binds exactly these entry points (see
 * INTEGRATION.md). Every call is frame- or batch-granular: the reference's
 * per-ray interfaces (pbrt.Integrator.Li, pbrt.Aggregate.Intersect) cost a
 * cgo hop each and can never be the device boundary.
 *
 * Reference interfaces replaced (paths relative to ssttuu/go-pbrt):
 *   pbrt_gpu_render       <- pbrt.Render(ctx, Integrator, Scene, tileSize)
 *                            pkg/pbrt/integrator.go:291-350 (with Path.Li
 *                            pkg/integrator/path.go:32-157 and
 *                            DirectLighting.Li pkg/integrator/directlighting.go:62-104
 *                            executed on the device)
 *   pbrt_gpu_intersect    <- (*accelerator.BVH).Intersect  pkg/accelerator/bvh.go:659-712
 *   pbrt_gpu_intersect_p  <- (*accelerator.BVH).IntersectP pkg/accelerator/bvh.go:713-765
 *   pbrt_gpu_cancel       <- ctx.Done() / errgroup cancellation, integrator.go:305-345
 *   PBRT_E_REF_PANIC      <- the places where the reference panics instead of
 *                            returning: integrator.go:73-75 (Ld > 10),
 *                            pkg/efloat/efloat.go:102-111 (EFloat Check)
 *
 * Conventions: plain C11, no exceptions across the ABI, caller-owned output
 * buffers, every function returns a pbrt_status (0 = OK). All arithmetic is
 * IEEE-754 binary64 with Go (amd64) semantics; descriptors carry matrices
 * exactly as the Go host computed them.
 */
#ifndef PBRT_GPU_H
#define PBRT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
typedef enum pbrt_status {
    PBRT_OK = 0,
    PBRT_E_INVALID = 1,      /* bad descriptor / argument                     */
    PBRT_E_HIP = 2,          /* HIP runtime failure                           */
    PBRT_E_RCCL = 3,         /* collective failure (multi-GPU film reduce)    */
    PBRT_E_CANCELLED = 4,    /* pbrt_gpu_cancel() observed                    */
    PBRT_E_REF_PANIC = 5,    /* the Go reference would have panicked here     */
    PBRT_E_UNSUPPORTED = 6   /* descriptor uses a feature not on the hot path */
} pbrt_status;

/* panic kinds reported in pbrt_gpu_stats.panic_kind */
enum {
    PBRT_PANIC_NONE = 0,
    PBRT_PANIC_LD_GT_10 = 1,     /* integrator.go:73-75                      */
    PBRT_PANIC_EFLOAT = 2,       /* efloat.go:102-111                        */
    PBRT_PANIC_BVH_STACK = 3,    /* bvh.go:670 fixed [64] stack overflow     */
    PBRT_PANIC_NIL_DEREF = 4     /* rough Glass: TrowbridgeReitz.SampleWH returns nil
                                    (its wh is shadowed, microfacet.go:79-115), so a
                                    microfacet BxDF's SampleF dereferences nil in
                                    Reflect/Refract (reflection.go:102-118, 706-811) */
};

/* --------------------------------------------------------------- transform */
/* pkg/pbrt/transform.go:27 Matrix4x4, :144 Transform{Matrix, MatrixInverse} */
typedef struct pbrt_matrix4x4 { double m[4][4]; } pbrt_matrix4x4;
typedef struct pbrt_transform { pbrt_matrix4x4 m, m_inv; } pbrt_transform;

/* ------------------------------------------------------------------ shapes */
enum { PBRT_SHAPE_SPHERE = 1, PBRT_SHAPE_DISK = 2 };

/* pkg/pbrt/sphere.go:8-17 Sphere, pkg/shapes/disk.go:14-20 Disk.
 * world_to_object is object_to_world.Inverse() (matrix/inverse swapped). */
typedef struct pbrt_shape_desc {
    int32_t type;
    int32_t reverse_orientation;
    int32_t transform_swaps_handedness;
    int32_t pad0;
    pbrt_transform object_to_world;
    double radius;
    double z_min, z_max, theta_min, theta_max, phi_max;   /* sphere           */
    double height, inner_radius;                          /* disk             */
} pbrt_shape_desc;

/* --------------------------------------------------------------- materials */
enum { PBRT_TEX_CONSTANT = 1, PBRT_TEX_CHECKERBOARD2D = 2 };
enum { PBRT_MAT_MATTE = 0, PBRT_MAT_MIRROR = 1, PBRT_MAT_GLASS = 2 };

/* type PBRT_MAT_MATTE: pkg/materials/matte.go:8-37 MatteMaterial with Kd either a
 * ConstantSpectrumTexture (pkg/pbrt/texture.go:133-145) or a Checkerboard2D
 * over PlanarMapping2D (pkg/textures/checkerboard.go, texture.go:105-123) whose
 * two sub-textures are constants. sigma is a ConstantFloatTexture.
 * type PBRT_MAT_MIRROR: pkg/materials/mirror.go:9-32 (constant Kr; NewMirror uses 0.9).
 * type PBRT_MAT_GLASS: pkg/materials/glass.go:15-75 with constant Kr, Kt, index
 * (eta) and roughness textures. Path.Li asks for multiple lobes (path.go:74), so
 * smooth glass (both roughnesses 0) is one FresnelSpecular lobe; rough glass is
 * MicrofacetReflection + MicrofacetTransmission over TrowbridgeReitz(u, v)
 * (microfacet.go, reflection.go:670-835), whose sampling panics in the reference
 * (PBRT_PANIC_NIL_DEREF). Path renders of Mirror, smooth Glass and OrenNayar
 * scenes run on the wave pipeline (its kX instantiations, LDS-sized trees);
 * rough glass, DirectLighting through these materials and panic fidelity run
 * on the serial kernel. */
typedef struct pbrt_material_desc {
    int32_t kd_type;
    int32_t type;                  /* PBRT_MAT_* (0 = Matte)                  */
    double kd[3];
    double vs[3], vt[3], ds, dt;
    double tex1[3], tex2[3];
    double sigma;
    double kr[3], kt[3];           /* Mirror: Kr; Glass: Kr, Kt               */
    double eta, u_roughness, v_roughness;   /* Glass                          */
} pbrt_material_desc;

/* -------------------------------------------------------------- primitives */
enum { PBRT_PRIM_GEOMETRIC = 1, PBRT_PRIM_TRANSFORMED = 2 };

/* GeometricPrimitive (pkg/pbrt/primitive.go:22-78), optionally wrapped in a
 * TransformedPrimitive with a non-animated AnimatedTransform (primitive.go:89-129). */
typedef struct pbrt_primitive_desc {
    int32_t kind;
    int32_t shape;
    int32_t material;
    int32_t pad0;
    pbrt_transform prim_to_world;
} pbrt_primitive_desc;

/* flattened BVH node, pkg/accelerator/bvh.go:80-87 LinearBVHNode */
typedef struct pbrt_bvh_node {
    double bmin[3], bmax[3];
    uint32_t offset;      /* primitiveOffset (leaf) | secondChildOffset (interior) */
    uint16_t n_prims;     /* 0 => interior */
    uint8_t axis;
    uint8_t pad0;
} pbrt_bvh_node;

/* ----------------------------------------------------------- triangle meshes */
/* EXTENSION (BASELINE configs D/E): go-pbrt has no triangle shape (pkg/shapes
 * holds only disk.go) and its BVH builder is O(n^2) (bvh.go:272-411), so a
 * triangle mesh is not part of the reference's semantics. Semantics here are
 * pbrt-v3's Triangle::Intersect (watertight, Woop et al.; default uv), in
 * float64 after exact widening of float32 world-space vertices, with error
 * bounds from the real machine epsilon 2^-53 (go-pbrt's own Gamma() is
 * denormal). Meshes are traversed through their own BVH, built
 * on the device (LBVH); a closest hit is the smallest (t, triangle index)
 * over all triangles, so results do not depend on that BVH. Triangles of
 * mesh m carry the global index mesh_first(m) + i and report prim =
 * n_prims + that index. */
typedef struct pbrt_mesh_desc {
    int32_t n_vertices, n_triangles;
    int32_t material;              /* index into materials                      */
    int32_t reverse_orientation;   /* flips the geometric normal                */
    const float* p;                /* n_vertices * 3 world-space positions     */
    const int32_t* indices;        /* n_triangles * 3 vertex indices            */
} pbrt_mesh_desc;

/* ------------------------------------------------------------------ lights */
enum { PBRT_LIGHT_POINT = 1, PBRT_LIGHT_DISTANT = 2, PBRT_LIGHT_DIFFUSE_AREA = 3 };

/* pkg/lights/{point,distant,diffuse}.go */
typedef struct pbrt_light_desc {
    int32_t type;
    int32_t shape;          /* DIFFUSE_AREA: index into shapes (a sphere)    */
    int32_t two_sided;      /* DIFFUSE_AREA                                  */
    int32_t pad0;
    double spectrum[3];     /* Point.I | Distant.L | DiffuseAreaLight.LEmit  */
    double p_light[3];      /* Point: lightToWorld(0,0,0)                    */
    double w_light[3];      /* Distant: normalized world direction           */
    double world_radius;    /* Distant: set by Preprocess (BoundingSphere)   */
} pbrt_light_desc;

/* ------------------------------------------------------------------ camera */
/* PerspectiveCamera (pkg/pbrt/camera.go:128-242). shutter_close is stored as
 * the reference leaves it: NewProjectiveCamera passes shutterOpen twice
 * (camera.go:116), so both fields hold shutterOpen. */
typedef struct pbrt_camera_desc {
    pbrt_transform camera_to_world;
    pbrt_transform raster_to_camera;
    double lens_radius, focal_distance, shutter_open, shutter_close;
} pbrt_camera_desc;

/* -------------------------------------------------------------------- film */
/* pkg/pbrt/film.go:27-76 (CroppedPixelBounds, BoxFilter radius, filter table) */
typedef struct pbrt_film_desc {
    int64_t res_x, res_y;
    int64_t crop_min_x, crop_min_y, crop_max_x, crop_max_y;
    double filter_radius_x, filter_radius_y;
    double max_sample_luminance;
    double filter_table[16 * 16];
} pbrt_film_desc;

/* light-selection distribution (pkg/pbrt/sampling.go:5-55 Distribution1D),
 * computed by the host from the integrator's LightSampleStrategy
 * (lightdistribution.go). func has n entries, cdf n+1. */
#define PBRT_MAX_DIST 64
typedef struct pbrt_distribution_desc {
    int32_t count;
    int32_t pad0;
    double func_int;
    double func[PBRT_MAX_DIST];
    double cdf[PBRT_MAX_DIST + 1];
} pbrt_distribution_desc;

/* ------------------------------------------------------------------- scene */
typedef struct pbrt_scene_desc {
    int32_t n_shapes, n_materials, n_prims, n_nodes, n_lights, pad0;
    const pbrt_shape_desc* shapes;
    const pbrt_material_desc* materials;
    const pbrt_primitive_desc* prims;      /* BVH order (orderedPrims)        */
    const pbrt_bvh_node* nodes;            /* depth-first, bvh.go:632-651     */
    const pbrt_light_desc* lights;
    pbrt_camera_desc camera;
    pbrt_film_desc film;
    double world_min[3], world_max[3];     /* Scene.WorldBound (BVH root)     */
    int32_t n_meshes, pad1;                /* extension: triangle meshes      */
    const pbrt_mesh_desc* meshes;
} pbrt_scene_desc;

/* ------------------------------------------------------------------ render */
enum { PBRT_INTEGRATOR_PATH = 1, PBRT_INTEGRATOR_DIRECT_LIGHTING = 2 };
enum { PBRT_LIGHT_STRATEGY_UNIFORM = 1, PBRT_LIGHT_STRATEGY_POWER = 2 };
enum { PBRT_DL_UNIFORM_SAMPLE_ALL = 1, PBRT_DL_UNIFORM_SAMPLE_ONE = 2 };

/* Execution modes.
 *  EXACT: the reference's per-tile RNG stream replayed bit-for-bit
 *         (integrator.go:318,328; one sampler clone per 16-px tile).
 *  THROUGHPUT: identical arithmetic, but every (pixel, sample) path gets its
 *         own PCG32 stream => statistically (not bitwise) equal images. */
enum { PBRT_MODE_EXACT = 0, PBRT_MODE_THROUGHPUT = 1 };

typedef struct pbrt_render_desc {
    /* sampler: sampler.NewStratified(x, y, jitter, nDims) (stratified.go:12-19) */
    int32_t sampler_x, sampler_y, jitter, n_dims;
    /* integrator */
    int32_t integrator;      /* PBRT_INTEGRATOR_*                               */
    int32_t max_depth;
    int32_t light_strategy;  /* Path: PBRT_LIGHT_STRATEGY_*                     */
    int32_t dl_strategy;     /* DirectLighting: PBRT_DL_*                       */
    double rr_threshold;
    int64_t tile_size;       /* pbrt.Render tileSize (16 in internal/render)    */
    /* tile subset (multi-GPU sharding): tiles t = tile_begin, tile_begin +
     * tile_stride, ... < tile_end (tile_end <= 0 means all tiles). */
    int64_t tile_begin, tile_end, tile_stride;
    int32_t mode;            /* PBRT_MODE_*                                     */
    int32_t flags;           /* PBRT_FLAG_* (diagnostics), normally 0           */
} pbrt_render_desc;

typedef struct pbrt_gpu_stats {
    uint64_t tiles_rendered;
    uint64_t camera_samples;     /* W*H*(spp-1) over rendered tiles           */
    uint64_t paths_traced;       /* camera rays that reached Li               */
    double kernel_ms;            /* device time of the tile render kernel      */
    double merge_ms;             /* device time of the film merge kernel       */
    double total_ms;             /* host wall time of the call                */
    int32_t panic_kind;          /* PBRT_PANIC_*                              */
    int32_t panic_tile;
    int64_t panic_pixel_x, panic_pixel_y;
    int32_t panic_sample, panic_bounce;
    int32_t kernel;          /* PBRT_KERNEL_SERIAL / _WAVE / _WAVEFRONT (last render) */
    int32_t batches;         /* WAVE/WAVEFRONT: tile batches of the frame         */
    double chain_ms;         /* WAVE/WAVEFRONT: sample-offset chain time, summed  */
    double paths_ms;         /* WAVE/WAVEFRONT: k_paths time (full paths), summed */
    /* The reference's ray segments for the rendered paths, counted in-kernel
     * (SURVEY 8(d)): closest-hit queries of Path.Li's loop (path.go:44-45, one per
     * iteration, incl. the one at bounces == maxDepth; DirectLighting: one per
     * Li call, directlighting.go:67) and any-hit visibility rays of light
     * sampling (VisibilityTester.Unoccluded, integrator.go:112-119), on every
     * kernel. EstimateDirect's BSDF-sampled ray, which always adds 0, is not
     * counted. Equal to the oracle's counts. */
    uint64_t rays_closest;
    uint64_t rays_shadow;
} pbrt_gpu_stats;

/* ----------------------------------------------------------- ray batches */
typedef struct pbrt_ray_soa {
    const double *ox, *oy, *oz, *dx, *dy, *dz;
    const double *tmax;          /* may be NULL => +Inf                      */
} pbrt_ray_soa;

typedef struct pbrt_hit_soa {
    uint8_t* hit;
    double* t_max;               /* ray.TMax after Intersect (tHit if hit)    */
    int32_t* prim;               /* index into scene prims (BVH order), -1    */
    double *px, *py, *pz;        /* SurfaceInteraction.Point                  */
    double *nx, *ny, *nz;        /* SurfaceInteraction.Normal (geometric)     */
} pbrt_hit_soa;

/* ------------------------------------------------------------------ opts */
typedef struct pbrt_gpu_opts {
    int32_t device;              /* HIP device ordinal (-1 => current)       */
    int32_t lanes_per_wave;      /* serial kernel: tiles per 64-lane wave (0=auto) */
    int32_t occupancy;           /* serial kernel: waves/SIMD build variant (0,1,2,4,8) */
    int32_t kernel;              /* PBRT_KERNEL_*                               */
    int32_t reserved[4];
} pbrt_gpu_opts;

/* Kernels. All replay the reference bit for bit:
 *  SERIAL     one lane per tile, the tile's PCG32 stream consumed in order
 *             (any render; the only one for n_dims < 3 Path renders,
 *             zero-pdf lights, filter radius >= 1.5 and PBRT_FLAG_PANIC_FIDELITY);
 *  WAVE_CI    the wave pipeline (Path integrator, n_dims >= 3, every light
 *             pdf > 0, filter radius < 1.5, no rough glass; Mirror / smooth
 *             Glass / OrenNayar on trees of <= 64 nodes): per-pixel shared bounce 1, the
 *             tile's path offsets found by a continuous-issue chain of
 *             speculative trajectories + jump-ahead (k_chain_ci), then the
 *             samples as full paths (k_paths_ci, or the per-bounce path
 *             wavefront k_pw_* for mesh scenes and large trees);
 *  WAVE_DL    DirectLighting (n_dims >= 1): pixel-order StartPixel +
 *             jump-ahead, one lane per sample;
 *  WAVE, WAVEFRONT  (round 1's window and wavefront chains, since replaced)
 *             request the wave pipeline; st.kernel reports WAVE_CI.
 * THROUGHPUT mode reports WAVE for the wave pipeline (no chain). */
/* WAVE kernel: always replay StartPixel serially (the path normally taken
 * only after a pcg_bounded rejection); results are identical. */
#define PBRT_FLAG_SERIAL_START_PIXEL 1
/* Panic fidelity: also trace the rays whose results never reach the film but
 * whose traversal can panic in the reference -- EstimateDirect's BSDF-sampled
 * MIS ray for an area light (integrator.go:132-192, incl. Sphere.PdfWi) and
 * the closest hit at bounces == maxDepth (path.go:44-45,66). Serial kernel. */
#define PBRT_FLAG_PANIC_FIDELITY 2

enum { PBRT_KERNEL_AUTO = 0, PBRT_KERNEL_SERIAL = 1, PBRT_KERNEL_WAVE = 2, PBRT_KERNEL_WAVEFRONT = 3,
       PBRT_KERNEL_WAVE_CI = 4, /* wave pipeline, continuous-issue offset chain */
       PBRT_KERNEL_WAVE_DL = 5  /* DirectLighting: pixel-order StartPixel + jump-ahead, one lane per sample */ };

typedef struct pbrt_gpu_ctx pbrt_gpu_ctx;

/* Copies the scene to device memory. The descriptor may be freed afterwards. */
int pbrt_gpu_create(const pbrt_scene_desc* scene, const pbrt_gpu_opts* opts,
                    pbrt_gpu_ctx** out);

/* Renders the frame (or the tile subset in rd) and writes the fp64 XYZ film,
 * res_x*res_y*3 doubles in raster order, to film_xyz (host memory) before
 * returning. Equivalent of pbrt.Render minus WriteImage. */
int pbrt_gpu_render(pbrt_gpu_ctx* ctx, const pbrt_render_desc* rd,
                    double* film_xyz, pbrt_gpu_stats* stats);

/* Same, but leaves the film in device memory (pbrt_gpu_film_device) and does
 * not synchronize with the host: the bench's timed region. */
int pbrt_gpu_render_async(pbrt_gpu_ctx* ctx, const pbrt_render_desc* rd);
/* Same, merging the film into a caller-owned device buffer of res_x*res_y*3
 * doubles (e.g. a torch tensor that is then reduced over RCCL). */
int pbrt_gpu_render_async_into(pbrt_gpu_ctx* ctx, const pbrt_render_desc* rd, double* film_device);
int pbrt_gpu_synchronize(pbrt_gpu_ctx* ctx, pbrt_gpu_stats* stats);
/* device pointer to the res_x*res_y*3 fp64 film of the last render */
double* pbrt_gpu_film_device(pbrt_gpu_ctx* ctx);
int pbrt_gpu_film_download(pbrt_gpu_ctx* ctx, double* film_xyz);
/* HIP stream the context launches on (hipStream_t as void*) */
void* pbrt_gpu_stream(pbrt_gpu_ctx* ctx);

/* Batch closest hit / any hit through the device BVH (Aggregate interface). */
int pbrt_gpu_intersect(pbrt_gpu_ctx* ctx, const pbrt_ray_soa* rays, size_t n,
                       pbrt_hit_soa* hits);
int pbrt_gpu_intersect_p(pbrt_gpu_ctx* ctx, const pbrt_ray_soa* rays, size_t n,
                         uint8_t* occluded);

/* Cancels the render in flight on ctx (from pbrt_gpu_render[_async[_into]]
 * entry until its pbrt_gpu_synchronize returns): the kernels poll a flag between
 * units of work (a pixel's chain, every 128 chain steps, a workgroup of paths),
 * so the frame stops within milliseconds and its synchronize returns
 * PBRT_E_CANCELLED (the caller's film buffer is then left undefined: the final
 * merge is skipped when the kernels saw the cancel). Like the reference's
 * errgroup, which stops issuing tiles once ctx is done (integrator.go:332-335),
 * it ends that render only: the flag is cleared when the render ends, so the
 * next render on the context runs normally. With no render in flight it does
 * nothing. Thread-safe. */
void pbrt_gpu_cancel(pbrt_gpu_ctx* ctx);
const char* pbrt_gpu_last_error(const pbrt_gpu_ctx* ctx);
void pbrt_gpu_destroy(pbrt_gpu_ctx* ctx);

/* PNG-byte conversion of film.go:142-179 WriteImage: uint8(clamp(XYZ,0,1)*255),
 * no XYZ->RGB and no gamma, exactly as the reference. rgba: w*h*4 bytes. */
int pbrt_film_to_rgba8(const double* film_xyz, int64_t w, int64_t h, uint8_t* rgba);

#ifdef __cplusplus
}
#endif
#endif /* PBRT_GPU_H */
