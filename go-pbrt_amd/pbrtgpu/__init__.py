"""pbrtgpu — Python host wrapper over the C ABI of the MI355X hot path.

The product is the C-ABI library lib/libpbrt_gpu.so (include/pbrt_gpu.h,
include/pbrt_scene.h). This module only loads it with ctypes and mirrors the
reference's driver-side vocabulary so tests and bench read like go-pbrt:

    scene = Scene.readme(1920, 1080)            # internal/render/server.go:29-164
    with Renderer(scene) as r:                  # pbrt_gpu_create
        film, stats = r.render(render_desc())   # pbrt.Render -> fp64 XYZ film

There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible, construction raises.
"""
import ctypes as C
import os
import struct
import zlib

import numpy as np

from . import abi
from .abi import *  # noqa: F401,F403  (re-export the ABI constants/structs)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("PBRT_GPU_LIB") or os.path.join(PKG_DIR, "lib", "libpbrt_gpu.so")

_lib = None


class PbrtError(RuntimeError):
    def __init__(self, code, msg, stats=None):
        super().__init__(f"pbrt status {code}: {msg}")
        self.code = code
        self.stats = stats


def lib():
    """Load lib/libpbrt_gpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C go-pbrt_amd` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.pbrt_gpu_build_id.restype = C.c_char_p
    L.pbrt_gpu_build_id.argtypes = []
    P, d, i64 = C.POINTER, C.c_double, C.c_int64
    T = P(abi.Transform)
    L.pbrt_gpu_create.argtypes = [P(abi.SceneDesc), P(abi.GpuOpts), P(C.c_void_p)]
    L.pbrt_gpu_render.argtypes = [C.c_void_p, P(abi.RenderDesc), P(d), P(abi.GpuStats)]
    L.pbrt_gpu_render_async.argtypes = [C.c_void_p, P(abi.RenderDesc)]
    L.pbrt_gpu_render_async_into.argtypes = [C.c_void_p, P(abi.RenderDesc), C.c_void_p]
    L.pbrt_gpu_synchronize.argtypes = [C.c_void_p, P(abi.GpuStats)]
    L.pbrt_gpu_film_device.argtypes = [C.c_void_p]
    L.pbrt_gpu_film_device.restype = C.c_void_p
    L.pbrt_gpu_film_download.argtypes = [C.c_void_p, P(d)]
    L.pbrt_gpu_stream.argtypes = [C.c_void_p]
    L.pbrt_gpu_stream.restype = C.c_void_p
    L.pbrt_gpu_intersect.argtypes = [C.c_void_p, P(abi.RaySoA), C.c_size_t, P(abi.HitSoA)]
    L.pbrt_gpu_intersect_p.argtypes = [C.c_void_p, P(abi.RaySoA), C.c_size_t, P(C.c_uint8)]
    L.pbrt_gpu_cancel.argtypes = [C.c_void_p]
    L.pbrt_gpu_cancel.restype = None
    L.pbrt_gpu_last_error.argtypes = [C.c_void_p]
    L.pbrt_gpu_last_error.restype = C.c_char_p
    L.pbrt_gpu_destroy.argtypes = [C.c_void_p]
    L.pbrt_gpu_destroy.restype = None
    L.pbrt_film_to_rgba8.argtypes = [P(d), i64, i64, P(C.c_uint8)]
    L.pbrt_gpu_tile_ticks.argtypes = [C.c_void_p, P(C.c_uint32), i64, P(i64)]
    L.pbrt_gpu_tile_ticks.restype = i64
    L.pbrt_gpu_tile_costs.argtypes = [C.c_void_p, P(C.c_float), i64]
    L.pbrt_gpu_tile_costs.restype = i64
    L.pbrt_gpu_counters.argtypes = [C.c_void_p, P(C.c_uint64), C.c_int]
    L.pbrt_gpu_schedule_source.argtypes = [C.c_void_p]
    L.pbrt_gpu_schedule_cache_clear.argtypes = []
    L.pbrt_gpu_overlap_slots.argtypes = [C.c_void_p]
    L.pbrt_gpu_overlap_slots.restype = C.c_int64
    L.pbrt_gpu_schedule_cache_clear.restype = None
    for name in ("pbrt_translate", "pbrt_scale"):
        getattr(L, name).argtypes = [d, d, d, T]
        getattr(L, name).restype = None
    for name in ("pbrt_rotate_x", "pbrt_rotate_y", "pbrt_rotate_z"):
        getattr(L, name).argtypes = [d, T]
        getattr(L, name).restype = None
    L.pbrt_transform_mul.argtypes = [T, T, T]
    L.pbrt_transform_mul.restype = None
    L.pbrt_transform_inverse.argtypes = [T, T]
    L.pbrt_transform_inverse.restype = None
    L.pbrt_matrix_inverse.argtypes = [P(abi.Matrix4x4), P(abi.Matrix4x4)]
    L.pbrt_new_transform.argtypes = [P(abi.Matrix4x4), T]
    L.pbrt_look_at.argtypes = [P(d), P(d), P(d), T]
    L.pbrt_perspective.argtypes = [d, d, d, T]
    L.pbrt_perspective.restype = None
    L.pbrt_transform_point.argtypes = [T, P(d), P(d), P(d), P(d)]
    L.pbrt_transform_point.restype = None
    L.pbrt_transform_ray.argtypes = [T, P(d), P(d), P(d), P(d)]
    L.pbrt_transform_ray.restype = None
    L.pbrt_make_sphere.argtypes = [T, C.c_int, d, d, d, d, P(abi.ShapeDesc)]
    L.pbrt_make_sphere.restype = None
    L.pbrt_make_disk.argtypes = [T, d, d, d, d, P(abi.ShapeDesc)]
    L.pbrt_make_disk.restype = None
    L.pbrt_make_matte_constant.argtypes = [d, d, d, d, P(abi.MaterialDesc)]
    L.pbrt_make_matte_constant.restype = None
    L.pbrt_make_matte_checkerboard.argtypes = [P(d), P(d), d, d, P(d), P(d), d, P(abi.MaterialDesc)]
    L.pbrt_make_matte_checkerboard.restype = None
    L.pbrt_random_sampler.argtypes = [C.c_int32, P(abi.RenderDesc)]
    L.pbrt_random_sampler.restype = None
    L.pbrt_make_mirror.argtypes = [P(d), P(abi.MaterialDesc)]
    L.pbrt_make_mirror.restype = None
    L.pbrt_make_glass.argtypes = [P(d), P(d), d, d, d, P(abi.MaterialDesc)]
    L.pbrt_make_glass.restype = None
    L.pbrt_make_point_light.argtypes = [T, P(d), P(abi.LightDesc)]
    L.pbrt_make_point_light.restype = None
    L.pbrt_make_distant_light.argtypes = [T, P(d), P(d), P(abi.LightDesc)]
    L.pbrt_make_distant_light.restype = None
    L.pbrt_make_diffuse_area_light.argtypes = [P(d), C.c_int, C.c_int, P(abi.LightDesc)]
    L.pbrt_make_diffuse_area_light.restype = None
    L.pbrt_sb_create.restype = C.c_void_p
    L.pbrt_sb_destroy.argtypes = [C.c_void_p]
    L.pbrt_sb_destroy.restype = None
    L.pbrt_sb_add_shape.argtypes = [C.c_void_p, P(abi.ShapeDesc)]
    L.pbrt_sb_add_material.argtypes = [C.c_void_p, P(abi.MaterialDesc)]
    L.pbrt_sb_add_primitive.argtypes = [C.c_void_p, P(abi.PrimitiveDesc)]
    L.pbrt_sb_add_light.argtypes = [C.c_void_p, P(abi.LightDesc)]
    L.pbrt_sb_set_film.argtypes = [C.c_void_p, i64, i64, P(d), d, d, d]
    L.pbrt_sb_set_perspective_camera.argtypes = [C.c_void_p, T, P(d), d, d, d, d, d]
    L.pbrt_sb_build.argtypes = [C.c_void_p, C.c_int, P(P(abi.SceneDesc))]
    L.pbrt_sb_prim_order.argtypes = [C.c_void_p, P(C.c_int32), C.c_int]
    L.pbrt_scene_light_distribution.argtypes = [P(abi.SceneDesc), C.c_int, P(abi.DistributionDesc)]
    L.pbrt_scene_readme.argtypes = [i64, i64, P(C.c_void_p)]
    L.pbrt_scene_cornell.argtypes = [i64, i64, P(C.c_void_p)]
    L.pbrt_scene_heightfield.argtypes = [i64, i64, C.c_int32, C.c_uint64, C.c_int32, P(C.c_void_p)]
    L.pbrt_sb_add_mesh.argtypes = [C.c_void_p, C.c_int32, P(C.c_float), C.c_int32, P(C.c_int32), C.c_int32,
                                   C.c_int32]
    L.pbrt_gpu_mesh_info.argtypes = [C.c_void_p, P(d), C.c_int]
    L.pbrt_gpu_mesh_download.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int32), P(C.c_float)]
    _lib = L
    return L


def build_id():
    """Content hash of the sources the loaded library was built from."""
    return lib().pbrt_gpu_build_id().decode()


def _d3(v):
    return (C.c_double * 3)(*v)


# ------------------------------------------------------------------ transforms
def translate(x, y, z):
    t = abi.Transform()
    lib().pbrt_translate(x, y, z, C.byref(t))
    return t


def scale(x, y, z):
    t = abi.Transform()
    lib().pbrt_scale(x, y, z, C.byref(t))
    return t


def rotate(axis, degrees):
    t = abi.Transform()
    getattr(lib(), "pbrt_rotate_" + "xyz"[axis])(degrees, C.byref(t))
    return t


def mul(a, b):
    t = abi.Transform()
    lib().pbrt_transform_mul(C.byref(a), C.byref(b), C.byref(t))
    return t


def look_at(pos, look, up):
    t = abi.Transform()
    rc = lib().pbrt_look_at(_d3(pos), _d3(look), _d3(up), C.byref(t))
    if rc:
        raise PbrtError(rc, "LookAt: up parallel to view direction")
    return t


def transform_ray(t, o, d):
    oo, od = (C.c_double * 3)(), (C.c_double * 3)()
    lib().pbrt_transform_ray(C.byref(t), _d3(o), _d3(d), oo, od)
    return list(oo), list(od)


# ------------------------------------------------------------------------ scene
class Scene:
    """A pbrt_scene_builder plus its built pbrt_scene_desc."""

    def __init__(self, handle=None):
        self.h = handle if handle is not None else lib().pbrt_sb_create()
        self.desc_ptr = None

    @classmethod
    def readme(cls, w, h):
        hb = C.c_void_p()
        rc = lib().pbrt_scene_readme(w, h, C.byref(hb))
        if rc:
            raise PbrtError(rc, "pbrt_scene_readme")
        s = cls(hb.value)
        s._fetch()
        return s

    @classmethod
    def cornell(cls, w, h):
        hb = C.c_void_p()
        rc = lib().pbrt_scene_cornell(w, h, C.byref(hb))
        if rc:
            raise PbrtError(rc, "pbrt_scene_cornell")
        s = cls(hb.value)
        s._fetch()
        return s

    @classmethod
    def readme_glass(cls, w, h, special="glass", mirror=True):
        """internal/render/server.go:67-91 (commented out): the README scene plus
        a sphere of radius 5 at (50, 2.5, 50) of NewGlass(Kr = Kt = 0.5, index
        1.5) -- the commented code attaches the checkerboard `m`, the glass it
        defines is what image.png shows. special = "black": that sphere a black
        Matte instead. mirror: a Mirror (Kr 0.9) sphere beside it at (35, 5, 45).
        Built (BVH, 2 primitives per node as server.go:162)."""
        s = cls.readme(w, h)
        m = s.add_glass() if special == "glass" else s.add_matte((0.0, 0.0, 0.0))
        spheres = [((50, 2.5, 50), m)]
        if mirror:
            spheres.append(((35, 5.0, 45), s.add_mirror()))
        for (pos, mat) in spheres:
            sph = s.add_sphere(translate(0, 0, 0), 5.0)
            s.add_primitive(sph, mat, translate(*pos))
        s.build(2)
        return s

    @classmethod
    def heightfield(cls, w, h, quads=707, seed=1, spheres=False):
        """BASELINE config D (quads 707: 999 698 triangles) / E (2236): the
        height-field extension scene (include/pbrt_scene.h)."""
        hb = C.c_void_p()
        rc = lib().pbrt_scene_heightfield(w, h, quads, seed, 1 if spheres else 0, C.byref(hb))
        if rc:
            raise PbrtError(rc, "pbrt_scene_heightfield")
        s = cls(hb.value)
        s._fetch()
        return s

    # builder API (pbrt_sb_*) -------------------------------------------------
    def add_mesh(self, p, indices, material, reverse=False):
        """p: (nv, 3) float32 world positions; indices: (nt, 3) int32."""
        p = np.ascontiguousarray(p, dtype=np.float32)
        idx = np.ascontiguousarray(indices, dtype=np.int32)
        r = lib().pbrt_sb_add_mesh(self.h, p.shape[0], p.ctypes.data_as(C.POINTER(C.c_float)), idx.shape[0],
                                   idx.ctypes.data_as(C.POINTER(C.c_int32)), material, int(reverse))
        if r < 0:
            raise PbrtError(-r, "pbrt_sb_add_mesh")
        return r

    def add_sphere(self, o2w, radius, reverse=False, z_min=None, z_max=None, phi_max=360.0):
        sd = abi.ShapeDesc()
        lib().pbrt_make_sphere(C.byref(o2w), int(reverse), radius, -radius if z_min is None else z_min,
                               radius if z_max is None else z_max, phi_max, C.byref(sd))
        return lib().pbrt_sb_add_shape(self.h, C.byref(sd))

    def add_disk(self, o2w, height, radius, inner=0.0, phi_max=360.0):
        sd = abi.ShapeDesc()
        lib().pbrt_make_disk(C.byref(o2w), height, radius, inner, phi_max, C.byref(sd))
        return lib().pbrt_sb_add_shape(self.h, C.byref(sd))

    def add_matte(self, rgb, sigma=0.0):
        m = abi.MaterialDesc()
        lib().pbrt_make_matte_constant(rgb[0], rgb[1], rgb[2], sigma, C.byref(m))
        return lib().pbrt_sb_add_material(self.h, C.byref(m))

    def add_checker(self, vs, vt, ds, dt, tex1, tex2, sigma=0.0):
        m = abi.MaterialDesc()
        lib().pbrt_make_matte_checkerboard(_d3(vs), _d3(vt), ds, dt, _d3(tex1), _d3(tex2), sigma, C.byref(m))
        return lib().pbrt_sb_add_material(self.h, C.byref(m))

    def add_mirror(self, kr=(0.9, 0.9, 0.9)):
        """materials.NewMirror (mirror.go:9-14; Kr 0.9 by default)."""
        m = abi.MaterialDesc()
        lib().pbrt_make_mirror(_d3(kr), C.byref(m))
        return lib().pbrt_sb_add_material(self.h, C.byref(m))

    def add_glass(self, kr=(0.5, 0.5, 0.5), kt=(0.5, 0.5, 0.5), u_roughness=0.0, v_roughness=0.0, eta=1.5):
        """materials.NewGlass (glass.go:15-26); defaults are server.go:80-87's glass."""
        m = abi.MaterialDesc()
        lib().pbrt_make_glass(_d3(kr), _d3(kt), u_roughness, v_roughness, eta, C.byref(m))
        return lib().pbrt_sb_add_material(self.h, C.byref(m))

    def add_primitive(self, shape, material, prim_to_world=None):
        p = abi.PrimitiveDesc()
        p.shape, p.material = shape, material
        if prim_to_world is None:
            p.kind = abi.PBRT_PRIM_GEOMETRIC
        else:
            p.kind = abi.PBRT_PRIM_TRANSFORMED
            p.prim_to_world = prim_to_world
        return lib().pbrt_sb_add_primitive(self.h, C.byref(p))

    def add_point_light(self, l2w, I):
        ld = abi.LightDesc()
        lib().pbrt_make_point_light(C.byref(l2w), _d3(I), C.byref(ld))
        return lib().pbrt_sb_add_light(self.h, C.byref(ld))

    def add_distant_light(self, l2w, L, w):
        ld = abi.LightDesc()
        lib().pbrt_make_distant_light(C.byref(l2w), _d3(L), _d3(w), C.byref(ld))
        return lib().pbrt_sb_add_light(self.h, C.byref(ld))

    def add_area_light(self, Lemit, shape, two_sided=False):
        ld = abi.LightDesc()
        lib().pbrt_make_diffuse_area_light(_d3(Lemit), shape, int(two_sided), C.byref(ld))
        return lib().pbrt_sb_add_light(self.h, C.byref(ld))

    def set_film(self, w, h, crop=(0, 0, 1, 1), filter_radius=(1.0, 1.0), max_lum=1.0):
        rc = lib().pbrt_sb_set_film(self.h, w, h, (C.c_double * 4)(*crop), filter_radius[0], filter_radius[1], max_lum)
        if rc:
            raise PbrtError(rc, "set_film")

    def set_camera(self, cam2world, screen=(0, 0, 1, 1), shutter=(0.0, 1.0), lens=0.0, focal=20.0, fov=100.0):
        rc = lib().pbrt_sb_set_perspective_camera(self.h, C.byref(cam2world), (C.c_double * 4)(*screen),
                                                  shutter[0], shutter[1], lens, focal, fov)
        if rc:
            raise PbrtError(rc, "set_camera")

    def build(self, max_prims_in_node=2):
        """accelerator.NewBVH(prims, maxPrimsInNode, SplitSAH) + pbrt.NewScene."""
        ptr = C.POINTER(abi.SceneDesc)()
        rc = lib().pbrt_sb_build(self.h, max_prims_in_node, C.byref(ptr))
        if rc:
            raise PbrtError(rc, "pbrt_sb_build")
        self.desc_ptr = ptr
        return self

    def _fetch(self):
        # fixtures are already built (maxPrimsInNode 2); rebuilding is idempotent
        self.build(2)

    @property
    def desc(self):
        return self.desc_ptr.contents

    def prim_order(self):
        n = self.desc.n_prims
        out = (C.c_int32 * max(n, 1))()
        lib().pbrt_sb_prim_order(self.h, out, n)
        return list(out)[:n]

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.pbrt_sb_destroy(self.h)
            self.h = None


# --------------------------------------------------------------------- renderer
class Renderer:
    """pbrt_gpu_ctx: the scene resident on one GPU."""

    KERNELS = {"auto": abi.PBRT_KERNEL_AUTO, "serial": abi.PBRT_KERNEL_SERIAL, "wave": abi.PBRT_KERNEL_WAVE,
               "wavefront": abi.PBRT_KERNEL_WAVEFRONT, "wave_ci": abi.PBRT_KERNEL_WAVE_CI,
               "wave_dl": abi.PBRT_KERNEL_WAVE_DL}

    def __init__(self, scene, device=-1, lanes_per_wave=0, occupancy=0, kernel="auto"):
        desc = scene.desc if isinstance(scene, Scene) else scene
        self._scene = scene  # keep the descriptor alive
        opts = abi.GpuOpts()
        opts.device, opts.lanes_per_wave = device, lanes_per_wave
        opts.occupancy, opts.kernel = occupancy, self.KERNELS[kernel]
        h = C.c_void_p()
        rc = lib().pbrt_gpu_create(C.byref(desc), C.byref(opts), C.byref(h))
        if rc:
            raise PbrtError(rc, "pbrt_gpu_create failed (no GPU visible?)")
        self.h = h.value
        self.w = desc.film.crop_max_x - desc.film.crop_min_x
        self.hgt = desc.film.crop_max_y - desc.film.crop_min_y

    def _check(self, rc, stats=None):
        if rc:
            raise PbrtError(rc, lib().pbrt_gpu_last_error(self.h).decode(), stats)

    def render(self, rd):
        film = np.zeros((self.hgt, self.w, 3), dtype=np.float64)
        st = abi.GpuStats()
        rc = lib().pbrt_gpu_render(self.h, C.byref(rd), film.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st))
        self._check(rc, st)
        return film, st

    def render_async(self, rd, film_device_ptr=None):
        """Enqueue a frame; film_device_ptr = caller device buffer (e.g. tensor.data_ptr())."""
        if film_device_ptr is None:
            self._check(lib().pbrt_gpu_render_async(self.h, C.byref(rd)))
        else:
            self._check(lib().pbrt_gpu_render_async_into(self.h, C.byref(rd), C.c_void_p(film_device_ptr)))

    def synchronize(self):
        st = abi.GpuStats()
        self._check(lib().pbrt_gpu_synchronize(self.h, C.byref(st)), st)
        return st

    def film(self):
        film = np.zeros((self.hgt, self.w, 3), dtype=np.float64)
        self._check(lib().pbrt_gpu_film_download(self.h, film.ctypes.data_as(C.POINTER(C.c_double))))
        return film

    def film_device_ptr(self):
        return lib().pbrt_gpu_film_device(self.h)

    def stream(self):
        return lib().pbrt_gpu_stream(self.h)

    def mesh_info(self):
        """{tris, nodes, depth, build_ms, meshes, wide} of the context's device LBVH
        (wide: the 4-ary layout, MeshNode4; else eight threaded binary orderings)."""
        out = (C.c_double * 8)()
        lib().pbrt_gpu_mesh_info(self.h, out, 8)
        return {"tris": int(out[0]), "nodes": int(out[1]), "depth": int(out[2]), "build_ms": out[3],
                "meshes": int(out[4]), "wide": bool(out[5])}

    def mesh_download(self):
        """(nodes, gid [tris], tris [tris, 9]) of the device LBVH; nodes is a [n]
        MeshNode4 structured array for the wide layout, else [8, n] MeshNode."""
        info = self.mesh_info()
        if info["wide"]:
            dt = np.dtype([("lo", np.float32, (3, 4)), ("hi", np.float32, (3, 4)), ("child", np.uint32, 4),
                           ("parent", np.uint32), ("axis", np.uint32), ("count", np.uint32), ("pad", np.uint32)])
            nodes = np.zeros(info["nodes"], dtype=dt)
        else:
            dt = np.dtype([("bmin", np.float32, 3), ("escape", np.uint32), ("bmax", np.float32, 3),
                           ("leaf", np.uint32)])
            nodes = np.zeros(8 * info["nodes"], dtype=dt)
        gid = np.zeros(info["tris"], dtype=np.int32)
        tris = np.zeros((info["tris"], 9), dtype=np.float32)
        rc = lib().pbrt_gpu_mesh_download(self.h, nodes.ctypes.data_as(C.c_void_p),
                                          gid.ctypes.data_as(C.POINTER(C.c_int32)),
                                          tris.ctypes.data_as(C.POINTER(C.c_float)))
        self._check(rc)
        return (nodes if info["wide"] else nodes.reshape(8, info["nodes"])), gid, tris

    def tile_ticks(self):
        """(per-slot chain ticks of the last EXACT frame at 100 MHz, heavy slots of its split)."""
        heavy = C.c_int64(0)
        n = lib().pbrt_gpu_tile_ticks(self.h, None, 0, C.byref(heavy))
        out = np.zeros(max(n, 0), dtype=np.uint32)
        if n > 0:
            lib().pbrt_gpu_tile_ticks(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n, C.byref(heavy))
        return out, int(heavy.value)

    def tile_costs(self):
        """(n_slots, 4) cold-frame cost features of the last EXACT frame's probe
        (chain work, hit pixels, pixels, cost); empty if that frame had a learned order."""
        n = lib().pbrt_gpu_tile_costs(self.h, None, 0)
        out = np.zeros((max(n, 0), 4), dtype=np.float32)
        if n > 0:
            rc = lib().pbrt_gpu_tile_costs(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), n)
            if rc < 0:
                self._check(-rc)
        return out

    SCHEDULE_SOURCES = {0: "launch order", 1: "probe", 2: "learned", 3: "cached"}

    def schedule_source(self):
        """Where the last EXACT frame's tile schedule came from: 'launch order', 'probe'
        (cold-frame estimate), 'learned' (this context's previous frame) or 'cached'
        (the process-wide cache: another context's frame of the same scene and configuration)."""
        return self.SCHEDULE_SOURCES[lib().pbrt_gpu_schedule_source(self.h)]

    def overlap_slots(self):
        """Slots of the last EXACT frame whose path stage ran completion-driven
        (pbrt_gpu_overlap_slots; 0: after the chain stage)."""
        return lib().pbrt_gpu_overlap_slots(self.h)

    def counters(self):
        """pbrt_gpu_counters of the last render (include/pbrt_diag.h order)."""
        out = np.zeros(128, dtype=np.uint64)
        n = lib().pbrt_gpu_counters(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), 128)
        return out[:max(n, 0)]

    def intersect(self, rays):
        """rays: (n,7) [ox,oy,oz,dx,dy,dz,tmax] -> (n,9) like the oracle."""
        rays = np.ascontiguousarray(rays, dtype=np.float64)
        n = rays.shape[0]
        cols = [np.ascontiguousarray(rays[:, k]) for k in range(7)]
        soa = abi.RaySoA(*[c.ctypes.data_as(C.POINTER(C.c_double)) for c in cols])
        hit = np.zeros(n, np.uint8)
        tmax = np.zeros(n)
        prim = np.zeros(n, np.int32)
        p = [np.zeros(n) for _ in range(6)]
        hs = abi.HitSoA(hit.ctypes.data_as(C.POINTER(C.c_uint8)), tmax.ctypes.data_as(C.POINTER(C.c_double)),
                        prim.ctypes.data_as(C.POINTER(C.c_int32)),
                        *[a.ctypes.data_as(C.POINTER(C.c_double)) for a in p])
        rc = lib().pbrt_gpu_intersect(self.h, C.byref(soa), n, C.byref(hs))
        out = np.stack([hit.astype(np.float64), tmax, prim.astype(np.float64)] + p, axis=1)
        return rc, out

    def intersect_p(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float64)
        n = rays.shape[0]
        cols = [np.ascontiguousarray(rays[:, k]) for k in range(7)]
        soa = abi.RaySoA(*[c.ctypes.data_as(C.POINTER(C.c_double)) for c in cols])
        occ = np.zeros(n, np.uint8)
        rc = lib().pbrt_gpu_intersect_p(self.h, C.byref(soa), n, occ.ctypes.data_as(C.POINTER(C.c_uint8)))
        return rc, occ

    def close(self):
        if getattr(self, "h", None):
            lib().pbrt_gpu_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        self.close()


def schedule_cache_clear():
    """Empty the process-wide schedule cache (pbrt_gpu_schedule_cache_clear)."""
    lib().pbrt_gpu_schedule_cache_clear()


def film_to_rgba8(film):
    """film.go:142-179 WriteImage pixel conversion (no XYZ->RGB, no gamma)."""
    film = np.ascontiguousarray(film, dtype=np.float64)
    h, w, _ = film.shape
    out = np.zeros((h, w, 4), np.uint8)
    rc = lib().pbrt_film_to_rgba8(film.ctypes.data_as(C.POINTER(C.c_double)), w, h,
                                  out.ctypes.data_as(C.POINTER(C.c_uint8)))
    if rc:
        raise PbrtError(rc, "film_to_rgba8")
    return out


def write_png(path, film):
    """Film.WriteImage (film.go:142-179): the fp64 XYZ film as an 8-bit PNG.

    Pixels are pbrt_film_to_rgba8's (uint8(Clamp(v, 0, 1) * 255) per channel,
    no XYZ->RGB, no gamma, alpha 255). Every pixel is opaque, so the image is
    written as 8-bit truecolour without alpha, the colour type Go's png.Encode
    picks for an opaque NRGBA image; scanlines use filter 0 (Go picks filters
    adaptively, so the file bytes differ while the decoded pixels are the same)."""
    rgba = film_to_rgba8(film)
    h, w, _ = rgba.shape
    raw = np.zeros((h, 1 + 3 * w), np.uint8)
    raw[:, 1:] = rgba[:, :, :3].reshape(h, 3 * w)

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
           + chunk(b"IDAT", zlib.compress(raw.tobytes(), 6)) + chunk(b"IEND", b""))
    with open(path, "wb") as f:
        f.write(png)
    return rgba


def read_png_rgb(path):
    """Decode an 8-bit truecolour PNG with filter-0 scanlines (write_png's) -> (h, w, 3) uint8."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3)
