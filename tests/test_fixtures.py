"""SURVEY 8(c)'s build-generated golden fixtures (tests/golden/make_golden.py):
frozen known answers for the oracle (CPU) and the device (GPU), so an oracle
edit cannot silently move both sides at once.

- 256x256 README frames at Stratified(2,2) and (4,4): the film, and every tile's
  own contribution (a one-tile render) by hash;
- a 64x64 crop of config B's frame (1920x1080, Stratified(8,8), Path(10)): the
  4x4 tiles of pixels x 928..991, y 480..543, with their 1-px filter apron;
- per-pixel PCG32 draw counts of config-B tiles 0, 4080 and 8159 (StartPixel +
  every sample's path, the quantity the wave pipeline's chain reconstructs);
- batch-intersect hit records of 10^4 seeded random rays (bvh.go:659-765).
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
META = json.load(open(os.path.join(GOLD, "golden.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def crop_tiles():
    c = META["crop_b"]
    ntx = (c["w"] + 15) // 16
    return [abi.render_desc(**dict(c["render"], tile_begin=ty * ntx + c["tx0"], tile_end=ty * ntx + c["tx0"] + c["n"]))
            for ty in range(c["ty0"], c["ty0"] + c["n"])]


def crop_window(film):
    x0, y0, n = META["crop_b"]["window"]
    return film[y0:y0 + n, x0:x0 + n]


# ---------------------------------------------------------------- the oracle
@pytest.mark.parametrize("name", sorted(META["tile_films"]))
def test_oracle_tile_films(name):
    case = META["tile_films"][name]
    sc = O.OracleScene.readme(256, 256)
    rc, film, st = O.render(sc.desc, abi.render_desc(**case["render"]), threads=8)
    assert rc == 0 and sha(film) == case["sha256"] and st.paths == case["paths"]
    assert np.array_equal(film, np.load(os.path.join(GOLD, name + ".npz"))["film"])
    for t in (0, 17, 128, 255):
        rc, ft, _ = O.render(sc.desc, abi.render_desc(**dict(case["render"], tile_begin=t, tile_end=t + 1)), threads=1)
        assert rc == 0 and sha(ft) == case["tile_sha256"][t]


def test_oracle_config_b_crop():
    sc = O.OracleScene.readme(1920, 1080)
    acc = None
    for rd in crop_tiles():
        rc, f, _ = O.render(sc.desc, rd, threads=8)
        assert rc == 0
        acc = f if acc is None else acc + f
    win = crop_window(acc)
    assert sha(win) == META["crop_b"]["sha256"]


def test_oracle_draw_counts():
    sc = O.OracleScene.readme(1920, 1080)
    for t, want in META["draw_counts_1920x1080_s8x8"].items():
        rc, d = O.tile_draws(sc.desc, abi.render_desc(8, 8), int(t))
        assert rc == 0 and list(d) == want
    # StartPixel alone is 8 dims x 64 UniformUInt32B draws (+ rejections); every
    # traced sample adds the path's draws
    # (tile 8159 is in the ragged last row: 16 x 8 pixels, the rest of its array is 0)
    assert min(min(x for x in v if x) for v in META["draw_counts_1920x1080_s8x8"].values()) >= 512
    assert sum(1 for x in META["draw_counts_1920x1080_s8x8"]["8159"] if x) == 128


def test_oracle_hit_records():
    z = np.load(os.path.join(GOLD, "readme_hits_1e4.npz"))
    sc = O.OracleScene.readme(64, 64)
    closest = O.intersect(sc.desc, z["rays"], closest=True)
    anyhit = O.intersect(sc.desc, z["rays"], closest=False)
    assert sha(closest) == META["hits"]["sha256_closest"] and sha(anyhit) == META["hits"]["sha256_anyhit"]
    assert 0.2 < closest[:, 0].mean() < 0.9


# ---------------------------------------------------------------- the device
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(META["tile_films"]))
@pytest.mark.parametrize("kernel", ["serial", "auto"])
def test_device_tile_films(name, kernel):
    case = META["tile_films"][name]
    sc = G.Scene.readme(256, 256)
    with G.Renderer(sc, kernel=kernel) as r:
        film, st = r.render(abi.render_desc(**case["render"]))
        assert sha(film) == case["sha256"] and st.paths_traced == case["paths"]
        for t in range(0, 256, 5):   # every fifth tile on its own
            ft, _ = r.render(abi.render_desc(**dict(case["render"], tile_begin=t, tile_end=t + 1)))
            assert sha(ft) == case["tile_sha256"][t], t


@pytest.mark.gpu
def test_device_config_b_crop():
    sc = G.Scene.readme(1920, 1080)
    acc = None
    with G.Renderer(sc) as r:
        for rd in crop_tiles():
            f, st = r.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            acc = f if acc is None else acc + f
    assert sha(crop_window(acc)) == META["crop_b"]["sha256"]


@pytest.mark.gpu
def test_device_hit_records():
    z = np.load(os.path.join(GOLD, "readme_hits_1e4.npz"))
    sc = G.Scene.readme(64, 64)
    with G.Renderer(sc) as r:
        rc, closest = r.intersect(z["rays"])
        assert rc == 0
        rc, occ = r.intersect_p(z["rays"])
        assert rc == 0
    want = z["closest"]
    ok = ~np.isnan(want[:, 0])   # a NaN row: the reference panics on that ray
    assert ok.mean() > 0.99
    assert np.array_equal(closest[ok, :3], want[ok, :3])
    hit = ok & (want[:, 0] == 1)
    assert np.array_equal(closest[hit].view(np.uint64), want[hit].view(np.uint64))
    assert np.array_equal(occ[ok].astype(np.float64), z["anyhit"][ok])
