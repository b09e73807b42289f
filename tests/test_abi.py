"""The C-ABI library loads on a CPU-only host and exports every function the
public headers declare; the ctypes mirrors match the C struct layouts.
(No compute call is made here: that needs a GPU.)"""
import ctypes as C
import os
import re

import numpy as np
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


def go_uint8_of_clamped(v):
    """film.go:157-159 uint8(math.Clamp(v, 0, 1) * 255): Clamp (pkg/math/math.go:42-50)
    passes NaN through (both comparisons false); Go's float->uint8 conversion on
    amd64 truncates via CVTTSD2SQ, which gives math.MinInt64 (low byte 0) for NaN."""
    out = np.zeros(v.shape, np.uint8)
    ok = ~np.isnan(v)
    c = np.where(v < 0, 0.0, np.where(v > 1, 1.0, v))
    out[ok] = np.trunc(c[ok] * 255).astype(np.int64).astype(np.uint8)
    return out


def test_film_to_rgba8_matches_write_image_semantics():
    """pbrt_film_to_rgba8 is a host-only conversion (no GPU call): NaN, negative,
    -0, exactly 1.0, values above 1, infinities and rounding-edge values."""
    edge = [np.nan, -1.0, -0.0, 0.0, 1.0, 1.5, np.inf, -np.inf, 0.5, 0.999, 1.0 / 255, 254.5 / 255,
            np.nextafter(1.0, 0.0), 5e-324, 0.0039215686274509803]
    rng = np.random.default_rng(7)
    vals = np.concatenate([np.array(edge), rng.uniform(-0.5, 1.5, 3 * 64 * 32 - len(edge))])
    film = vals.reshape(32, 64, 3)
    rgba = G.film_to_rgba8(film)
    assert rgba.shape == (32, 64, 4) and (rgba[:, :, 3] == 255).all()
    assert np.array_equal(rgba[:, :, :3], go_uint8_of_clamped(film))
    assert list(rgba.reshape(-1, 4)[0]) == [0, 0, 0, 255]        # NaN, -1, -0
    assert list(rgba.reshape(-1, 4)[1]) == [0, 255, 255, 255]    # 0, 1.0, 1.5
    assert list(rgba.reshape(-1, 4)[2]) == [255, 0, 127, 255]    # +Inf, -Inf, 0.5
    assert list(rgba.reshape(-1, 4)[3]) == [254, 1, 254, 255]    # 0.999, 1/255, 254.5/255


def test_write_png_round_trip(tmp_path):
    """Film.WriteImage: the PNG decodes to the converted pixels (opaque -> RGB 8-bit)."""
    rng = np.random.default_rng(3)
    film = rng.uniform(-0.2, 1.3, (27, 41, 3))
    film[3, 5, 1] = np.nan
    path = str(tmp_path / "film.png")
    rgba = G.write_png(path, film)
    back = G.read_png_rgb(path)
    assert back.shape == (27, 41, 3)
    assert np.array_equal(back, rgba[:, :, :3])
    assert back[3, 5, 1] == 0
