"""ctypes mirrors of include/pbrt_gpu.h (the C ABI of the device path).

These structures are plain data layouts; they carry no behaviour. Field order
and types must match include/pbrt_gpu.h exactly (checked by
tests/test_abi.py against the sizes the library reports).
"""
import ctypes as C

PBRT_OK = 0
PBRT_E_INVALID = 1
PBRT_E_HIP = 2
PBRT_E_RCCL = 3
PBRT_E_CANCELLED = 4
PBRT_E_REF_PANIC = 5
PBRT_E_UNSUPPORTED = 6

PBRT_SHAPE_SPHERE = 1
PBRT_SHAPE_DISK = 2
PBRT_TEX_CONSTANT = 1
PBRT_TEX_CHECKERBOARD2D = 2
PBRT_MAT_MATTE, PBRT_MAT_MIRROR, PBRT_MAT_GLASS = 0, 1, 2
PBRT_PRIM_GEOMETRIC = 1
PBRT_PRIM_TRANSFORMED = 2
PBRT_LIGHT_POINT = 1
PBRT_LIGHT_DISTANT = 2
PBRT_LIGHT_DIFFUSE_AREA = 3
PBRT_INTEGRATOR_PATH = 1
PBRT_INTEGRATOR_DIRECT_LIGHTING = 2
PBRT_LIGHT_STRATEGY_UNIFORM = 1
PBRT_LIGHT_STRATEGY_POWER = 2
PBRT_DL_UNIFORM_SAMPLE_ALL = 1
PBRT_DL_UNIFORM_SAMPLE_ONE = 2
PBRT_MODE_EXACT = 0
PBRT_MODE_THROUGHPUT = 1
PBRT_KERNEL_AUTO = 0
PBRT_KERNEL_SERIAL = 1
PBRT_KERNEL_WAVE = 2
PBRT_KERNEL_WAVEFRONT = 3
PBRT_KERNEL_WAVE_CI = 4
PBRT_KERNEL_WAVE_DL = 5
PBRT_FLAG_SERIAL_START_PIXEL = 1
PBRT_FLAG_PANIC_FIDELITY = 2

PBRT_PANIC_NONE = 0
PBRT_PANIC_LD_GT_10 = 1
PBRT_PANIC_EFLOAT = 2
PBRT_PANIC_BVH_STACK = 3
PBRT_PANIC_NIL_DEREF = 4

PBRT_MAX_DIST = 64


class Matrix4x4(C.Structure):
    _fields_ = [("m", (C.c_double * 4) * 4)]


class Transform(C.Structure):
    _fields_ = [("m", Matrix4x4), ("m_inv", Matrix4x4)]


class ShapeDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("reverse_orientation", C.c_int32),
        ("transform_swaps_handedness", C.c_int32),
        ("pad0", C.c_int32),
        ("object_to_world", Transform),
        ("radius", C.c_double),
        ("z_min", C.c_double),
        ("z_max", C.c_double),
        ("theta_min", C.c_double),
        ("theta_max", C.c_double),
        ("phi_max", C.c_double),
        ("height", C.c_double),
        ("inner_radius", C.c_double),
    ]


class MaterialDesc(C.Structure):
    _fields_ = [
        ("kd_type", C.c_int32),
        ("type", C.c_int32),
        ("kd", C.c_double * 3),
        ("vs", C.c_double * 3),
        ("vt", C.c_double * 3),
        ("ds", C.c_double),
        ("dt", C.c_double),
        ("tex1", C.c_double * 3),
        ("tex2", C.c_double * 3),
        ("sigma", C.c_double),
        ("kr", C.c_double * 3),
        ("kt", C.c_double * 3),
        ("eta", C.c_double),
        ("u_roughness", C.c_double),
        ("v_roughness", C.c_double),
    ]


class PrimitiveDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("shape", C.c_int32),
        ("material", C.c_int32),
        ("pad0", C.c_int32),
        ("prim_to_world", Transform),
    ]


class BVHNode(C.Structure):
    _fields_ = [
        ("bmin", C.c_double * 3),
        ("bmax", C.c_double * 3),
        ("offset", C.c_uint32),
        ("n_prims", C.c_uint16),
        ("axis", C.c_uint8),
        ("pad0", C.c_uint8),
    ]


class LightDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("shape", C.c_int32),
        ("two_sided", C.c_int32),
        ("pad0", C.c_int32),
        ("spectrum", C.c_double * 3),
        ("p_light", C.c_double * 3),
        ("w_light", C.c_double * 3),
        ("world_radius", C.c_double),
    ]


class CameraDesc(C.Structure):
    _fields_ = [
        ("camera_to_world", Transform),
        ("raster_to_camera", Transform),
        ("lens_radius", C.c_double),
        ("focal_distance", C.c_double),
        ("shutter_open", C.c_double),
        ("shutter_close", C.c_double),
    ]


class FilmDesc(C.Structure):
    _fields_ = [
        ("res_x", C.c_int64),
        ("res_y", C.c_int64),
        ("crop_min_x", C.c_int64),
        ("crop_min_y", C.c_int64),
        ("crop_max_x", C.c_int64),
        ("crop_max_y", C.c_int64),
        ("filter_radius_x", C.c_double),
        ("filter_radius_y", C.c_double),
        ("max_sample_luminance", C.c_double),
        ("filter_table", C.c_double * 256),
    ]


class DistributionDesc(C.Structure):
    _fields_ = [
        ("count", C.c_int32),
        ("pad0", C.c_int32),
        ("func_int", C.c_double),
        ("func", C.c_double * PBRT_MAX_DIST),
        ("cdf", C.c_double * (PBRT_MAX_DIST + 1)),
    ]


class MeshDesc(C.Structure):
    """pbrt_mesh_desc: extension (configs D/E), include/pbrt_gpu.h."""
    _fields_ = [
        ("n_vertices", C.c_int32),
        ("n_triangles", C.c_int32),
        ("material", C.c_int32),
        ("reverse_orientation", C.c_int32),
        ("p", C.POINTER(C.c_float)),
        ("indices", C.POINTER(C.c_int32)),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("n_shapes", C.c_int32),
        ("n_materials", C.c_int32),
        ("n_prims", C.c_int32),
        ("n_nodes", C.c_int32),
        ("n_lights", C.c_int32),
        ("pad0", C.c_int32),
        ("shapes", C.POINTER(ShapeDesc)),
        ("materials", C.POINTER(MaterialDesc)),
        ("prims", C.POINTER(PrimitiveDesc)),
        ("nodes", C.POINTER(BVHNode)),
        ("lights", C.POINTER(LightDesc)),
        ("camera", CameraDesc),
        ("film", FilmDesc),
        ("world_min", C.c_double * 3),
        ("world_max", C.c_double * 3),
        ("n_meshes", C.c_int32),
        ("pad1", C.c_int32),
        ("meshes", C.POINTER(MeshDesc)),
    ]


class RenderDesc(C.Structure):
    _fields_ = [
        ("sampler_x", C.c_int32),
        ("sampler_y", C.c_int32),
        ("jitter", C.c_int32),
        ("n_dims", C.c_int32),
        ("integrator", C.c_int32),
        ("max_depth", C.c_int32),
        ("light_strategy", C.c_int32),
        ("dl_strategy", C.c_int32),
        ("rr_threshold", C.c_double),
        ("tile_size", C.c_int64),
        ("tile_begin", C.c_int64),
        ("tile_end", C.c_int64),
        ("tile_stride", C.c_int64),
        ("mode", C.c_int32),
        ("flags", C.c_int32),
    ]


class GpuStats(C.Structure):
    _fields_ = [
        ("tiles_rendered", C.c_uint64),
        ("camera_samples", C.c_uint64),
        ("paths_traced", C.c_uint64),
        ("kernel_ms", C.c_double),
        ("merge_ms", C.c_double),
        ("total_ms", C.c_double),
        ("panic_kind", C.c_int32),
        ("panic_tile", C.c_int32),
        ("panic_pixel_x", C.c_int64),
        ("panic_pixel_y", C.c_int64),
        ("panic_sample", C.c_int32),
        ("panic_bounce", C.c_int32),
        ("kernel", C.c_int32),
        ("batches", C.c_int32),
        ("chain_ms", C.c_double),
        ("paths_ms", C.c_double),
        ("rays_closest", C.c_uint64),
        ("rays_shadow", C.c_uint64),
    ]


class RaySoA(C.Structure):
    _fields_ = [(n, C.POINTER(C.c_double)) for n in ("ox", "oy", "oz", "dx", "dy", "dz", "tmax")]


class HitSoA(C.Structure):
    _fields_ = [
        ("hit", C.POINTER(C.c_uint8)),
        ("t_max", C.POINTER(C.c_double)),
        ("prim", C.POINTER(C.c_int32)),
        ("px", C.POINTER(C.c_double)),
        ("py", C.POINTER(C.c_double)),
        ("pz", C.POINTER(C.c_double)),
        ("nx", C.POINTER(C.c_double)),
        ("ny", C.POINTER(C.c_double)),
        ("nz", C.POINTER(C.c_double)),
    ]


class GpuOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("lanes_per_wave", C.c_int32), ("occupancy", C.c_int32),
                ("kernel", C.c_int32), ("reserved", C.c_int32 * 4)]


def render_desc(spp_x=8, spp_y=8, jitter=False, n_dims=4, integrator=PBRT_INTEGRATOR_PATH,
                max_depth=10, rr_threshold=1.0, light_strategy=PBRT_LIGHT_STRATEGY_UNIFORM,
                dl_strategy=PBRT_DL_UNIFORM_SAMPLE_ALL, tile_size=16, tile_begin=0, tile_end=0,
                tile_stride=1, mode=PBRT_MODE_EXACT, flags=0):
    """RenderDesc with the defaults of internal/render/server.go:142,162,164."""
    rd = RenderDesc()
    rd.sampler_x, rd.sampler_y, rd.jitter, rd.n_dims = spp_x, spp_y, int(bool(jitter)), n_dims
    rd.integrator, rd.max_depth = integrator, max_depth
    rd.light_strategy, rd.dl_strategy = light_strategy, dl_strategy
    rd.rr_threshold = rr_threshold
    rd.tile_size, rd.tile_begin, rd.tile_end, rd.tile_stride = tile_size, tile_begin, tile_end, tile_stride
    rd.mode, rd.flags = mode, flags
    return rd
