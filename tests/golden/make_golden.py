"""Generates tests/golden/*.npz from the CPU oracle (oracle/, pinned by the
reference's own known-answer tests in tests/test_reference_kats.py).

These are build-generated golden vectors, not reference-generated: go-pbrt has
no Go toolchain in this image and no render-level goldens of its own (SURVEY
§4, §8c). Re-run after an intentional oracle change:
    python tests/golden/make_golden.py              # golden.json and its films
    python tests/golden/make_golden.py materials    # golden_materials.json (round 4)
The material / mesh scenes are built with the product's host-side scene
builder (pbrt_sb_*, no GPU) and rendered by the oracle.
"""
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
import oracle_lib as O  # noqa: E402
import pbrtgpu as G  # noqa: E402
import scenes  # noqa: E402
from pbrtgpu import abi  # noqa: E402

CASES = {
    # name: (scene, w, h, render_desc kwargs)
    "readme_64x64_s2x2_path": ("readme", 64, 64, dict(spp_x=2, spp_y=2)),
    "readme_48x32_s4x4_path": ("readme", 48, 32, dict(spp_x=4, spp_y=4)),
    "readme_64x48_s2x2_direct": ("readme", 64, 48, dict(spp_x=2, spp_y=2,
                                                       integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)),
    "readme_40x24_s3x2_jitter": ("readme", 40, 24, dict(spp_x=3, spp_y=2, jitter=True)),
    "cornell_48x32_s2x2_path8": ("cornell", 48, 32, dict(spp_x=2, spp_y=2, max_depth=8)),
}


def render_case(name):
    scene, w, h, kw = CASES[name]
    sc = O.OracleScene.readme(w, h) if scene == "readme" else O.OracleScene.cornell(w, h)
    rd = abi.render_desc(**kw)
    rc, film, st = O.render(sc.desc, rd, threads=4)
    assert rc == 0, (name, rc)
    return film, st


def pcg_vectors():
    out = {}
    import ctypes as C
    for seed in (0, 1, 8159):
        buf = (C.c_uint32 * 16)()
        O.lib().oracle_pcg_stream(seed, 16, buf)
        out[str(seed)] = list(buf)
    return out


# SURVEY 8(c)'s build-generated fixtures (round 3): frozen known answers that
# do not move when the oracle is edited
TILE_FILMS = {   # 256x256 README frames whose every tile is pinned on its own
    "readme_256x256_s2x2_path": dict(spp_x=2, spp_y=2),
    "readme_256x256_s4x4_path": dict(spp_x=4, spp_y=4),
}
# config B's frame (1920x1080, Stratified(8,8), Path(10)): the 4x4 tiles whose
# pixels are x 928..991, y 480..543 -- a 64x64 crop of the headline frame
CROP_B = dict(w=1920, h=1080, tx0=58, ty0=30, n=4, render=dict(spp_x=8, spp_y=8))
DRAW_TILES = (0, 4080, 8159)   # per-pixel PCG32 draw counts of these config-B tiles
N_RAYS = 10000                 # batch-intersect hit records (bvh.go:659-765)


def tile_films(name, kw):
    sc = O.OracleScene.readme(256, 256)
    rd = abi.render_desc(**kw)
    rc, film, st = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    n = int(O.lib().oracle_num_tiles(C.byref(sc.desc), C.byref(rd)))
    hashes = []
    for t in range(n):
        rc, ft, _ = O.render(sc.desc, abi.render_desc(**dict(kw, tile_begin=t, tile_end=t + 1)), threads=1)
        assert rc == 0
        hashes.append(hashlib.sha256(ft.tobytes()).hexdigest())
    return film, st, hashes


def crop_b():
    c = CROP_B
    sc = O.OracleScene.readme(c["w"], c["h"])
    ntx = (c["w"] + 15) // 16
    acc = None
    paths = 0
    for ty in range(c["ty0"], c["ty0"] + c["n"]):
        t0 = ty * ntx + c["tx0"]
        rc, f, st = O.render(sc.desc, abi.render_desc(**dict(c["render"], tile_begin=t0, tile_end=t0 + c["n"])),
                             threads=8)
        assert rc == 0
        acc = f if acc is None else acc + f
        paths += st.paths
    x0, y0 = c["tx0"] * 16 - 1, c["ty0"] * 16 - 1   # the block's pixels plus the 1-px filter apron
    win = acc[y0:y0 + 16 * c["n"] + 2, x0:x0 + 16 * c["n"] + 2].copy()
    return win, paths


def draw_counts():
    sc = O.OracleScene.readme(1920, 1080)
    rd = abi.render_desc(8, 8)
    out = {}
    for t in DRAW_TILES:
        rc, d = O.tile_draws(sc.desc, rd, t)
        assert rc == 0
        out[str(t)] = [int(v) for v in d]
    return out


def hit_records():
    """10^4 seeded random rays in the README scene: origins in a box around the
    spheres, directions uniform on the sphere, TMax +Inf or a random finite value."""
    rng = np.random.default_rng(20261017)
    o = rng.uniform([-20.0, 0.5, -20.0], [110.0, 60.0, 110.0], size=(N_RAYS, 3))
    d = rng.normal(size=(N_RAYS, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = np.where(rng.uniform(size=N_RAYS) < 0.5, np.inf, rng.uniform(1.0, 200.0, size=N_RAYS))
    rays = np.concatenate([o, d, tmax[:, None]], axis=1)
    sc = O.OracleScene.readme(64, 64)
    closest = O.intersect(sc.desc, rays, closest=True)
    anyhit = O.intersect(sc.desc, rays, closest=False)
    return rays, closest, anyhit


# Round 4: frozen films of the scenes that were checked only live against the
# oracle (VERDICT r3 missing #4): Mirror / smooth Glass, OrenNayar, DirectLighting
# through glass, triangle meshes, and a 64x64 crop of config G.
MAT_CASES = {
    # name: (scene builder, render_desc kwargs)
    "materials_48x32_s4x4_path": (lambda: scenes.material_scene("both", 48, 32), dict(spp_x=4, spp_y=4)),
    "materials_48x32_s3x3_oren20_path6": (lambda: scenes.material_scene("matte", 48, 32, sigma=20.0),
                                          dict(spp_x=3, spp_y=3, max_depth=6)),
    # the oracle's own construction of server.go:67-91's glass sphere + a mirror
    # (oracle_scene.c orc_scene_readme_glass), independent of the product's builder
    "readme_glass_64x48_s3x3_direct5": (lambda: O.OracleScene.readme_glass(64, 48, mirror=True),
                                        dict(spp_x=3, spp_y=3, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING,
                                             max_depth=5)),
    "mesh_glass_48x32_s2x2_path": (lambda: scenes.mesh_material_scene("glass", 48, 32), dict(spp_x=2, spp_y=2)),
    # the oracle's own height-field generator (oracle_scene.c orc_scene_heightfield)
    "heightfield_q64_48x32_s2x2_path": (lambda: O.OracleScene.heightfield(48, 32, quads=64), dict(spp_x=2, spp_y=2)),
}
# config G (README + server.go:67-91's glass sphere + a mirror, 1920x1080,
# Stratified(8,8), Path(10)): the 4x4 tiles of pixels x 1216..1279, y 768..831,
# on the glass sphere
CROP_G = dict(w=1920, h=1080, tx0=76, ty0=48, n=4, render=dict(spp_x=8, spp_y=8))


def crop_g():
    c = CROP_G
    sc = O.OracleScene.readme_glass(c["w"], c["h"], mirror=True)
    ntx = (c["w"] + 15) // 16
    acc = None
    paths = 0
    for ty in range(c["ty0"], c["ty0"] + c["n"]):
        t0 = ty * ntx + c["tx0"]
        rc, f, st = O.render(sc.desc, abi.render_desc(**dict(c["render"], tile_begin=t0, tile_end=t0 + c["n"])),
                             threads=8)
        assert rc == 0
        acc = f if acc is None else acc + f
        paths += st.paths
    x0, y0 = c["tx0"] * 16 - 1, c["ty0"] * 16 - 1
    return acc[y0:y0 + 16 * c["n"] + 2, x0:x0 + 16 * c["n"] + 2].copy(), paths


def main_materials():
    commit = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    meta = {"generator": "tests/golden/make_golden.py materials", "oracle_commit": commit, "cases": {}}
    for name, (build, kw) in MAT_CASES.items():
        sc = build()
        rd = abi.render_desc(**kw)
        rc, film, st = O.render(sc.desc, rd, threads=8)
        assert rc == 0, (name, rc)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), film=film)
        meta["cases"][name] = {"sha256": hashlib.sha256(film.tobytes()).hexdigest(), "paths": int(st.paths),
                               "render": {k: (int(v) if isinstance(v, bool) else v) for k, v in kw.items()}}
    win, paths = crop_g()
    np.savez_compressed(os.path.join(HERE, "readme_glass_1920x1080_s8x8_crop64.npz"), film=win)
    meta["crop_g"] = dict(CROP_G, sha256=hashlib.sha256(win.tobytes()).hexdigest(), paths=int(paths),
                          window=[CROP_G["tx0"] * 16 - 1, CROP_G["ty0"] * 16 - 1, 16 * CROP_G["n"] + 2])
    with open(os.path.join(HERE, "golden_materials.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(MAT_CASES), "material cases and the config-G crop")


def main():
    commit = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    meta = {"generator": "tests/golden/make_golden.py", "oracle_commit": commit, "cases": {}}
    for name in CASES:
        film, st = render_case(name)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), film=film)
        meta["cases"][name] = {"sha256": hashlib.sha256(film.tobytes()).hexdigest(), "paths": int(st.paths),
                               "scene": CASES[name][0], "w": CASES[name][1], "h": CASES[name][2],
                               "render": {k: (int(v) if isinstance(v, bool) else v) for k, v in CASES[name][3].items()}}
    meta["pcg32_first16"] = pcg_vectors()
    meta["tile_films"] = {}
    for name, kw in TILE_FILMS.items():
        film, st, hashes = tile_films(name, kw)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), film=film)
        meta["tile_films"][name] = {"sha256": hashlib.sha256(film.tobytes()).hexdigest(), "paths": int(st.paths),
                                    "render": kw, "tile_sha256": hashes}
    win, paths = crop_b()
    np.savez_compressed(os.path.join(HERE, "readme_1920x1080_s8x8_crop64.npz"), film=win)
    meta["crop_b"] = dict(CROP_B, sha256=hashlib.sha256(win.tobytes()).hexdigest(), paths=int(paths),
                          window=[CROP_B["tx0"] * 16 - 1, CROP_B["ty0"] * 16 - 1, 16 * CROP_B["n"] + 2])
    meta["draw_counts_1920x1080_s8x8"] = draw_counts()
    rays, closest, anyhit = hit_records()
    np.savez_compressed(os.path.join(HERE, "readme_hits_1e4.npz"), rays=rays, closest=closest, anyhit=anyhit)
    meta["hits"] = {"n": N_RAYS, "sha256_closest": hashlib.sha256(closest.tobytes()).hexdigest(),
                    "sha256_anyhit": hashlib.sha256(anyhit.tobytes()).hexdigest(),
                    "hit_fraction": float(closest[:, 0].mean())}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(CASES), "cases")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "materials":
        main_materials()
    else:
        main()
