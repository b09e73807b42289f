"""Round-4 frozen fixtures (tests/golden/golden_materials.json, made by
`python tests/golden/make_golden.py materials`): the scenes that were checked
only live against the oracle, so that an edit of the oracle's material code
(compute_bsdf_x / specular_bounce, restating pkg/materials/glass.go:44-72,
mirror.go, matte.go:30-35 and pkg/pbrt/reflection.go:465-668) cannot move the
oracle and the device together unnoticed:

- Mirror + smooth Glass + Matte spheres with an area light, Path(10);
- OrenNayar (Matte sigma 20), Path(6);
- DirectLighting through server.go:67-91's glass sphere (+ a mirror), maxDepth 5
  (directlighting.go:97-101, integrator.go:383-422);
- a glass triangle mesh, and the height-field generator at 64x64 quads
  (extension: parity unpinned against Go, frozen here);
- a 64x64 crop of config G's 1080p frame (README + glass + mirror,
  Stratified(8,8), Path(10)) on the glass sphere, on the kX wave pipeline.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
import scenes
from pbrtgpu import abi

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
META = json.load(open(os.path.join(GOLD, "golden_materials.json")))

# The oracle renders its own construction of the glass scenes (oracle_scene.c
# orc_scene_readme_glass), the device the product's (pbrt_scene.h builder), so a
# construction error on either side breaks the frozen match.
ORACLE_BUILD = {
    "readme_glass_64x48_s3x3_direct5": lambda: O.OracleScene.readme_glass(64, 48, mirror=True),
    "heightfield_q64_48x32_s2x2_path": lambda: O.OracleScene.heightfield(48, 32, quads=64),
}
BUILD = {
    "materials_48x32_s4x4_path": lambda: scenes.material_scene("both", 48, 32),
    "materials_48x32_s3x3_oren20_path6": lambda: scenes.material_scene("matte", 48, 32, sigma=20.0),
    "readme_glass_64x48_s3x3_direct5": lambda: G.Scene.readme_glass(64, 48, mirror=True),
    "mesh_glass_48x32_s2x2_path": lambda: scenes.mesh_material_scene("glass", 48, 32),
    "heightfield_q64_48x32_s2x2_path": lambda: G.Scene.heightfield(48, 32, quads=64),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("special", ["glass", "black"])
@pytest.mark.parametrize("mirror", [True, False])
def test_glass_scene_constructions_agree(special, mirror):
    """The product's scene builder and the oracle's independent constructor
    produce the same scene: BVH nodes, primitives in BVH order with their shapes
    and materials, lights, camera and film, byte for byte."""
    p = G.Scene.readme_glass(96, 64, special=special, mirror=mirror)
    o = O.OracleScene.readme_glass(96, 64, special=special, mirror=mirror)
    pd, od = p.desc, o.desc
    b = lambda x: bytes(memoryview(x))   # noqa: E731
    assert (pd.n_prims, pd.n_nodes, pd.n_lights) == (od.n_prims, od.n_nodes, od.n_lights)
    for i in range(pd.n_nodes):
        assert b(pd.nodes[i]) == b(od.nodes[i]), i
    for i in range(pd.n_prims):
        x, y = pd.prims[i], od.prims[i]
        assert (x.kind, b(x.prim_to_world)) == (y.kind, b(y.prim_to_world)), i
        assert b(pd.shapes[x.shape]) == b(od.shapes[y.shape]), i
        assert b(pd.materials[x.material]) == b(od.materials[y.material]), i
    for i in range(pd.n_lights):
        x, y = pd.lights[i], od.lights[i]
        if x.type == abi.PBRT_LIGHT_DIFFUSE_AREA:
            assert b(pd.shapes[x.shape]) == b(od.shapes[y.shape]), i
        assert b(x) == b(y) or x.type == abi.PBRT_LIGHT_DIFFUSE_AREA, i
    assert b(pd.camera) == b(od.camera) and b(pd.film) == b(od.film)


@pytest.mark.parametrize("quads", [64, 707])
def test_heightfield_constructions_agree(quads):
    """The height-field extension (configs D/E): the product's generator
    (pbrt_scene_heightfield) and the oracle's independent one agree on every
    vertex (float32 bits), every index, the material, lights, camera, film and
    the world bound (which sets the distant light's radius)."""
    p = G.Scene.heightfield(96, 64, quads=quads, seed=1)
    o = O.OracleScene.heightfield(96, 64, quads=quads, seed=1)
    pd, od = p.desc, o.desc
    b = lambda x: bytes(memoryview(x))   # noqa: E731
    assert pd.n_meshes == od.n_meshes == 1 and pd.n_prims == od.n_prims == 0
    pm, om = pd.meshes[0], od.meshes[0]
    assert (pm.n_vertices, pm.n_triangles, pm.reverse_orientation) == (om.n_vertices, om.n_triangles, 0)
    pv = np.ctypeslib.as_array(pm.p, shape=(3 * pm.n_vertices,)).view(np.uint32)
    ov = np.ctypeslib.as_array(om.p, shape=(3 * om.n_vertices,)).view(np.uint32)
    assert np.array_equal(pv, ov)
    assert np.array_equal(np.ctypeslib.as_array(pm.indices, shape=(3 * pm.n_triangles,)),
                          np.ctypeslib.as_array(om.indices, shape=(3 * om.n_triangles,)))
    assert b(pd.materials[pm.material]) == b(od.materials[om.material])
    for i in range(pd.n_lights):
        x, y = pd.lights[i], od.lights[i]
        if x.type == abi.PBRT_LIGHT_DIFFUSE_AREA:
            assert b(pd.shapes[x.shape]) == b(od.shapes[y.shape])
        else:
            assert b(x) == b(y), i
    assert b(pd.camera) == b(od.camera) and b(pd.film) == b(od.film)
    assert list(pd.world_min) == list(od.world_min) and list(pd.world_max) == list(od.world_max)


def test_fixture_set():
    assert set(META["cases"]) == set(BUILD)
    for name in BUILD:
        assert os.path.exists(os.path.join(GOLD, name + ".npz"))


@pytest.mark.parametrize("name", sorted(BUILD))
def test_oracle_material_fixtures(name):
    case = META["cases"][name]
    sc = ORACLE_BUILD.get(name, BUILD[name])()   # the scene owns the memory its desc points into
    rc, film, st = O.render(sc.desc, abi.render_desc(**case["render"]), threads=8)
    assert rc == 0 and st.paths == case["paths"]
    assert sha(film) == case["sha256"]
    assert np.array_equal(film, np.load(os.path.join(GOLD, name + ".npz"))["film"])


def crop_g_tiles():
    c = META["crop_g"]
    ntx = (c["w"] + 15) // 16
    return [abi.render_desc(**dict(c["render"], tile_begin=ty * ntx + c["tx0"], tile_end=ty * ntx + c["tx0"] + c["n"]))
            for ty in range(c["ty0"], c["ty0"] + c["n"])]


def crop_g_window(film):
    x0, y0, n = META["crop_g"]["window"]
    return film[y0:y0 + n, x0:x0 + n]


def test_oracle_config_g_crop():
    c = META["crop_g"]
    sc = O.OracleScene.readme_glass(c["w"], c["h"], mirror=True)
    acc, paths = None, 0
    for rd in crop_g_tiles():
        rc, f, st = O.render(sc.desc, rd, threads=8)
        assert rc == 0
        acc = f if acc is None else acc + f
        paths += st.paths
    assert paths == c["paths"] and sha(crop_g_window(acc)) == c["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BUILD))
def test_device_material_fixtures(name):
    case = META["cases"][name]
    sc = BUILD[name]()
    with G.Renderer(sc) as r:
        film, st = r.render(abi.render_desc(**case["render"]))
    assert st.paths_traced == case["paths"]
    assert sha(film) == case["sha256"]


@pytest.mark.gpu
def test_device_config_g_crop():
    c = META["crop_g"]
    sc = G.Scene.readme_glass(c["w"], c["h"], mirror=True)
    acc = None
    with G.Renderer(sc) as r:
        for rd in crop_g_tiles():
            f, st = r.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            acc = f if acc is None else acc + f
    assert sha(crop_g_window(acc)) == c["sha256"]
