"""ctypes loader for the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module, and only as the checker / CPU timing.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
from pbrtgpu import abi  # noqa: E402

ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
ORACLE_FLOPS_SO = os.path.join(ORACLE_DIR, "_build", "liboracle_flops.so")

_lib = None
_lib_flops = None


class OracleStats(C.Structure):
    _fields_ = [
        ("tiles", C.c_uint64),
        ("paths", C.c_uint64),
        ("camera_samples", C.c_uint64),
        ("closest_rays", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("flops", C.c_uint64),
        ("panic_kind", C.c_int32),
        ("panic_tile", C.c_int64),
        ("panic_px", C.c_int64),
        ("panic_py", C.c_int64),
        ("panic_sample", C.c_int64),
        ("panic_bounce", C.c_int64),
        ("flops_light", C.c_uint64),
    ]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib(flops=False):
    """The oracle library; flops=True loads the FLOP-accounting build."""
    global _lib, _lib_flops
    if flops:
        if _lib_flops is None:
            if not os.path.exists(ORACLE_FLOPS_SO):
                build()
            _lib_flops = _bind(C.CDLL(ORACLE_FLOPS_SO))
        return _lib_flops
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        _lib = _bind(C.CDLL(ORACLE_SO))
    return _lib


def _bind(L):
    if True:  # noqa: SIM108 (one indented block of bindings)
        d = C.c_double
        P = C.POINTER
        for name in ("sin", "cos", "tan", "atan", "asin", "acos", "radians"):
            f = getattr(L, "oracle_go_" + name)
            f.argtypes, f.restype = [d], d
        for name in ("atan2", "nextafter", "max", "min"):
            f = getattr(L, "oracle_go_" + name)
            f.argtypes, f.restype = [d, d], d
        L.oracle_go_f2i.argtypes, L.oracle_go_f2i.restype = [d], C.c_int64
        L.oracle_fr_dielectric.argtypes, L.oracle_fr_dielectric.restype = [d, d, d], d
        for name in ("oracle_efloat_add", "oracle_efloat_mul", "oracle_efloat_div"):
            getattr(L, name).argtypes = [d, d, d, d, P(d)]
            getattr(L, name).restype = C.c_int
        L.oracle_translate.argtypes = [d, d, d, P(abi.Transform)]
        L.oracle_scale.argtypes = [d, d, d, P(abi.Transform)]
        L.oracle_rotate.argtypes = [C.c_int, d, P(abi.Transform)]
        L.oracle_xf_mul.argtypes = [P(abi.Transform)] * 3
        L.oracle_matrix_inverse.argtypes = [P(abi.Matrix4x4), P(abi.Matrix4x4)]
        L.oracle_look_at.argtypes = [P(d), P(d), P(d), P(abi.Transform)]
        L.oracle_perspective.argtypes = [d, d, d, P(abi.Transform)]
        L.oracle_transform_point.argtypes = [P(abi.Transform), P(d), P(d), P(d), P(d)]
        L.oracle_transform_ray.argtypes = [P(abi.Transform), P(d), P(d), P(d), P(d)]
        L.oracle_offset_ray_origin.argtypes = [P(d)] * 5
        L.oracle_make_sphere.argtypes = [P(abi.Transform), C.c_int, d, d, d, d, P(abi.ShapeDesc)]
        L.oracle_make_disk.argtypes = [P(abi.Transform), d, d, d, d, P(abi.ShapeDesc)]
        L.oracle_pcg_stream.argtypes = [C.c_uint64, C.c_int, P(C.c_uint32)]
        L.oracle_pcg_floats.argtypes = [C.c_uint64, C.c_int, P(d)]
        for name in ("oracle_scene_new",):
            getattr(L, name).restype = C.c_void_p
        L.oracle_scene_readme.argtypes = [C.c_int64, C.c_int64]
        L.oracle_scene_readme.restype = C.c_void_p
        L.oracle_scene_cornell.argtypes = [C.c_int64, C.c_int64]
        L.oracle_scene_cornell.restype = C.c_void_p
        L.oracle_scene_heightfield.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_uint64]
        L.oracle_scene_heightfield.restype = C.c_void_p
        L.oracle_scene_readme_glass.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_int]
        L.oracle_scene_readme_glass.restype = C.c_void_p
        L.oracle_scene_add_shape.argtypes = [C.c_void_p, P(abi.ShapeDesc)]
        L.oracle_scene_add_material.argtypes = [C.c_void_p, P(abi.MaterialDesc)]
        L.oracle_scene_add_primitive.argtypes = [C.c_void_p, P(abi.PrimitiveDesc)]
        L.oracle_scene_add_light.argtypes = [C.c_void_p, P(abi.LightDesc)]
        L.oracle_scene_set_camera_film.argtypes = [C.c_void_p, P(abi.CameraDesc), P(abi.FilmDesc)]
        L.oracle_scene_finalize.argtypes = [C.c_void_p, C.c_int]
        L.oracle_scene_desc.argtypes = [C.c_void_p, P(abi.SceneDesc)]
        L.oracle_scene_order.argtypes = [C.c_void_p, P(C.c_int32)]
        L.oracle_scene_free.argtypes = [C.c_void_p]
        L.oracle_render.argtypes = [P(abi.SceneDesc), P(abi.RenderDesc), C.c_int, C.c_int, P(d), P(OracleStats)]
        L.oracle_num_tiles.argtypes = [P(abi.SceneDesc), P(abi.RenderDesc)]
        L.oracle_num_tiles.restype = C.c_int64
        L.oracle_intersect.argtypes = [P(abi.SceneDesc), P(d), C.c_size_t, C.c_int, P(d)]
        L.oracle_tile_draws.argtypes = [P(abi.SceneDesc), P(abi.RenderDesc), C.c_int64, P(C.c_int64)]
        L.oracle_light_distribution.argtypes = [P(abi.SceneDesc), P(abi.RenderDesc), P(abi.DistributionDesc)]
        L.oracle_spawn_ray_to.argtypes = [P(d), P(d)]
        L.oracle_triangle_hit.argtypes = [P(d), P(d), P(d)]
        L.oracle_vec_op.argtypes = [C.c_int, P(d), P(d), d, P(d)]
        L.oracle_partition_at.argtypes = [P(C.c_int32), P(d), C.c_int64, C.c_int64, C.c_int64, C.c_int64]
        L.oracle_partition_at.restype = C.c_int64
    return L


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleScene:
    """Owns an oracle-built scene; .desc is a pbrt_scene_desc view of it."""

    def __init__(self, handle):
        self.h = handle
        self.desc = abi.SceneDesc()
        lib().oracle_scene_desc(self.h, C.byref(self.desc))

    @classmethod
    def readme(cls, w, h):
        return cls(lib().oracle_scene_readme(w, h))

    @classmethod
    def cornell(cls, w, h):
        return cls(lib().oracle_scene_cornell(w, h))

    @classmethod
    def heightfield(cls, w, h, quads=707, seed=1):
        """The height-field extension scene (configs D/E) from the oracle's own
        generator (oracle_scene.c orc_scene_heightfield)."""
        hnd = lib().oracle_scene_heightfield(w, h, quads, seed)
        if not hnd:
            raise ValueError("quads out of range")
        return cls(hnd)

    @classmethod
    def readme_glass(cls, w, h, special="glass", mirror=True):
        """server.go:67-91's glass sphere (+ a mirror) on the README scene, built
        by the oracle's own constructor (oracle_scene.c orc_scene_readme_glass)."""
        return cls(lib().oracle_scene_readme_glass(w, h, 1 if special == "glass" else 0, 1 if mirror else 0))

    def order(self):
        out = (C.c_int32 * self.desc.n_prims)()
        lib().oracle_scene_order(self.h, out)
        return list(out)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.oracle_scene_free(self.h)
            self.h = None


def render(desc, rd, threads=None, flags=0, flops=False):
    """Returns (rc, film[H,W,3] float64, OracleStats)."""
    threads = threads or os.cpu_count() or 1
    W = desc.film.crop_max_x - desc.film.crop_min_x
    H = desc.film.crop_max_y - desc.film.crop_min_y
    film = np.zeros((H, W, 3), dtype=np.float64)
    st = OracleStats()
    rc = lib(flops).oracle_render(C.byref(desc), C.byref(rd), threads, flags, dptr(film), C.byref(st))
    return rc, film, st


def tile_draws(desc, rd, tile):
    """PCG32 draws per pixel of `tile` (StartPixel + its samples), row-major with the
    tile's own width, in a tile_size^2 array (a ragged tile leaves the tail 0).
    Returns (rc, counts)."""
    ts = int(rd.tile_size)
    out = np.zeros(ts * ts, dtype=np.int64)
    rc = lib().oracle_tile_draws(C.byref(desc), C.byref(rd), tile, out.ctypes.data_as(C.POINTER(C.c_int64)))
    return rc, out


def intersect(desc, rays, closest=True):
    rays = np.ascontiguousarray(rays, dtype=np.float64)
    n = rays.shape[0]
    out = np.zeros((n, 9) if closest else (n,), dtype=np.float64)
    lib().oracle_intersect(C.byref(desc), dptr(rays), n, 1 if closest else 0, dptr(out))
    return out


def triangle_hit(v, ray):
    """orc_triangle_hit (triangle extension): (hit, t, b0, b1, b2)."""
    v = np.ascontiguousarray(v, dtype=np.float64)
    ray = np.ascontiguousarray(ray, dtype=np.float64)
    out = np.zeros(4)
    h = lib().oracle_triangle_hit(dptr(v), dptr(ray), dptr(out))
    return bool(h), out[0], out[1], out[2], out[3]
