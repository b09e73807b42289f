"""The C-ABI library loads on a CPU-only host and exports every function the
public headers declare; the ctypes mirrors match the C struct layouts.
(No compute call is made here: that needs a GPU.)"""
import ctypes as C
import os
import re

import pytest

import pbrtgpu as G
from pbrtgpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["pbrt_gpu.h", "pbrt_scene.h", "pbrt_diag.h"]


def declared_functions():
    names = []
    for h in HEADERS:
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(pbrt_\w+)\s*\(", src, flags=re.M):
            names.append(m.group(1))
    return sorted(set(names))


def test_headers_declare_the_boundary():
    names = declared_functions()
    for required in ("pbrt_gpu_create", "pbrt_gpu_render", "pbrt_gpu_intersect", "pbrt_gpu_intersect_p",
                     "pbrt_gpu_cancel", "pbrt_gpu_last_error", "pbrt_gpu_destroy", "pbrt_scene_readme"):
        assert required in names


@pytest.mark.parametrize("name", declared_functions())
def test_symbol_exported(name):
    L = G.lib()
    assert hasattr(L, name), f"{name} declared in include/ but not exported by libpbrt_gpu.so"


def test_struct_sizes_match_ctypes():
    mirrors = [abi.Matrix4x4, abi.Transform, abi.ShapeDesc, abi.MaterialDesc, abi.PrimitiveDesc, abi.BVHNode,
               abi.LightDesc, abi.CameraDesc, abi.FilmDesc, abi.DistributionDesc, abi.SceneDesc, abi.RenderDesc,
               abi.GpuStats, abi.RaySoA, abi.HitSoA, abi.GpuOpts, abi.MeshDesc]
    sizes = (C.c_size_t * 32)()
    n = G.lib().pbrt_abi_sizes(sizes, 32)
    assert n == len(mirrors)
    for i, T in enumerate(mirrors):
        assert C.sizeof(T) == sizes[i], f"{T.__name__}: ctypes {C.sizeof(T)} != C {sizes[i]}"


def test_create_rejects_bad_descriptor_without_gpu_work():
    """Validation happens before any device call: a null scene is INVALID."""
    h = C.c_void_p()
    rc = G.lib().pbrt_gpu_create(None, None, C.byref(h))
    assert rc == abi.PBRT_E_INVALID and not h.value


def test_product_does_not_link_the_oracle():
    """The product library must not depend on the test oracle."""
    so = open(G.LIB_PATH, "rb").read()
    assert b"liboracle" not in so and b"oracle_render" not in so
