"""Configs C and D at full size in the STEADY STATE, against the oracle's own
scene constructions.

The bench times steady-state frames: the learned heaviest-first (LPT) tile
order, the heavy/light split, the completion-driven path stage. These tests
render a fresh context's cold frame and two steady-state frames of the full
1080p configuration on the device (product scene builder), and an evenly
spread sample of 65 tiles (tile_stride 127) on the oracle from its OWN scene
construction (oracle_scene.c: orc_scene_cornell, orc_scene_heightfield), and
compare the interiors of the sampled tiles (the pixels only that tile's samples
reach) bit for bit in every frame.

References: Render's tile loop and per-tile sampler clone
(/root/reference/pkg/pbrt/integrator.go:228-350), Film.MergeFilmTile
(pkg/pbrt/film.go:115-132).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))
STRIDE = 127   # 65 of the 8160 tiles of a 1080p frame, spread over the frame


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def interiors_equal(frame, ofilm, W, H, tiles, tile=16):
    """Tiles whose interior pixels (box filter radius 1: a sample at pixel p
    reaches film pixels p - 1 and p) differ between the two films."""
    ntx = (W + tile - 1) // tile
    bad = []
    for t in tiles:
        x0, y0 = (t % ntx) * tile, (t // ntx) * tile
        x1, y1 = min(x0 + tile, W), min(y0 + tile, H)
        if not np.array_equal(bits(frame[y0:y1 - 1, x0:x1 - 1]), bits(ofilm[y0:y1 - 1, x0:x1 - 1])):
            bad.append(t)
    return bad


def steady_state_check(scene, oscene, rd_kw, W, H, expect_heavy):
    n_tiles = ((W + 15) // 16) * ((H + 15) // 16)
    tiles = list(range(0, n_tiles, STRIDE))
    rc, ofilm, ost = O.render(oscene.desc, abi.render_desc(**rd_kw, tile_begin=0, tile_stride=STRIDE),
                              threads=THREADS)
    assert rc == 0 and ost.tiles == len(tiles)
    rd = abi.render_desc(**rd_kw)
    with G.Renderer(scene) as r:
        for frame in range(3):
            film, st = r.render(rd)
            _, heavy = r.tile_ticks()
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI and st.tiles_rendered == n_tiles
            if expect_heavy:   # the steady-state frames run the heavy/light split
                assert (heavy > 0) == (frame > 0), (frame, heavy)
            bad = interiors_equal(film, ofilm, W, H, tiles)
            print(f"frame {frame} (heavy {heavy}): {len(tiles) - len(bad)}/{len(tiles)} sampled tiles bit-exact")
            assert not bad, (frame, bad[:8])


def test_config_C_steady_state_sampled_tiles_vs_oracle_scene():
    W, H = 1920, 1080
    steady_state_check(G.Scene.cornell(W, H), O.OracleScene.cornell(W, H), dict(spp_x=16, spp_y=16, max_depth=8),
                       W, H, expect_heavy=False)


def test_config_D_steady_state_sampled_tiles_vs_oracle_scene():
    W, H = 1920, 1080
    steady_state_check(G.Scene.heightfield(W, H, quads=707, seed=1), O.OracleScene.heightfield(W, H, quads=707, seed=1),
                       dict(spp_x=8, spp_y=8), W, H, expect_heavy=False)
