"""BASELINE configs B and C at their full size, through the C ABI.

Config B (README scene, 1920x1080, Stratified(8,8), Path(10)): the WHOLE frame
against the oracle -- per-pixel RMS of the fp64 XYZ film and the fraction of
bit-identical tiles (BASELINE.md:47-48), both at their exact-parity values.

Config C (Cornell, 1920x1080, Stratified(16,16) = 255 traced paths/px,
Path(maxDepth 8); SURVEY 8(d), internal/render/server.go:142 for the
sampler): full-frame properties, and a bit-exact oracle check of the first,
middle and last tiles plus the frame's heaviest tiles by measured chain time.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def tile_parity(film, ofilm, tile=16):
    """(per-pixel RMS over the XYZ film, fraction of tiles whose pixels are bit-identical)."""
    rms = float(np.sqrt(np.mean((film - ofilm) ** 2)))
    H, W, _ = film.shape
    same = (bits(film) == bits(ofilm)).all(axis=2)
    ok = n = 0
    for y in range(0, H, tile):
        for x in range(0, W, tile):
            n += 1
            ok += bool(same[y:y + tile, x:x + tile].all())
    return rms, ok / n


def test_config_B_split_without_paths_overlap_vs_oracle(monkeypatch):
    """PBRT_PATHS_OVERLAP=0: the heavy/light split with one light launch and
    the whole path stage after the chains (the default overlaps the path stage
    of the heavy tiles and the light launch's first round with the rest of the
    chain, test_config_B_whole_frame_vs_oracle). Every frame is the oracle's,
    bit for bit."""
    monkeypatch.setenv("PBRT_PATHS_OVERLAP", "0")
    scene = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(8, 8)
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0
    with G.Renderer(scene) as r:
        for frame in range(3):
            film, st = r.render(rd)
            _, heavy = r.tile_ticks()
            assert (heavy > 0) == (frame > 0), (frame, heavy)
            assert st.paths_traced == ost.paths
            assert np.array_equal(bits(film), bits(ofilm)), frame


def test_config_B_whole_frame_vs_oracle():
    """The cold frame of a fresh context (probe order) and the steady-state
    frames the bench times: from the second frame on, the learned LPT order and
    the one-GPU heavy/light split (the heaviest tiles at 4 waves on one stream
    beside the rest at 1 wave, render.hip launch_ci), with the path stage of the
    heavy tiles and the light launch's first round overlapping the rest of the
    chain (PBRT_PATHS_OVERLAP, default on). Every frame is the oracle's, bit
    for bit."""
    scene = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(8, 8)
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0
    with G.Renderer(scene) as r:
        for frame in range(3):
            film, st = r.render(rd)
            _, heavy = r.tile_ticks()
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            assert st.tiles_rendered == 8160 and st.paths_traced == 1920 * 1080 * 63
            assert ost.paths == st.paths_traced
            # the first frame has no measured schedule; later ones split
            assert (heavy > 0) == (frame > 0), (frame, heavy)
            rms, frac = tile_parity(film, ofilm)
            print(f"config B frame {frame} (heavy tiles {heavy}): rms {rms:.3e}, bit-identical tiles {frac:.6f}")
            assert rms == 0.0 and frac == 1.0, (frame, rms, frac)
            assert np.array_equal(bits(film), bits(ofilm)), frame


def tile_interior_equal(frame, tile_film, rd_tile, W, tile=16):
    """Pixels of tile t that only tile t's samples reach (box filter radius
    < 1.5: a sample at pixel p lands on film pixels p-1 and p) are equal in a
    whole frame and in the one-tile render of t."""
    ntx = (W + tile - 1) // tile
    t = rd_tile.tile_begin
    x0, y0 = (t % ntx) * tile, (t // ntx) * tile
    x1, y1 = min(x0 + tile, frame.shape[1]), min(y0 + tile, frame.shape[0])
    a = frame[y0:y1 - 1, x0:x1 - 1]
    b = tile_film[y0:y1 - 1, x0:x1 - 1]
    return bool(np.all(a == b)) and a.size > 0


def test_config_C_full_size_properties_and_heaviest_tiles():
    W, H = 1920, 1080
    scene = G.Scene.cornell(W, H)
    rd = abi.render_desc(16, 16, max_depth=8)
    with G.Renderer(scene) as r:
        film, st = r.render(rd)
        ticks, _ = r.tile_ticks()
        film2, st2 = r.render(rd)   # the steady-state frame: learned heaviest-first order
    assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
    assert st.tiles_rendered == 8160 and st.paths_traced == W * H * 255
    assert st2.paths_traced == st.paths_traced
    assert st.batches == 1
    assert np.isfinite(film).all() and (film >= 0).all() and film.max() > 0
    assert len(ticks) == 8160 and ticks.min() > 0
    heaviest = [int(t) for t in np.argsort(ticks)[::-1][:3]]
    tiles = sorted({0, 4080, 8159, *heaviest})
    for t in tiles:
        one = abi.render_desc(16, 16, max_depth=8, tile_begin=t, tile_end=t + 1)
        with G.Renderer(scene) as r:
            g, _ = r.render(one)
        rc, o, _ = O.render(scene.desc, one, threads=1)
        assert rc == 0
        assert np.array_equal(bits(g), bits(o)), t
        assert tile_interior_equal(film, o, one, W), ("cold frame", t)
        assert tile_interior_equal(film2, o, one, W), ("second frame", t)
    print(f"config C: bit-exact tiles {tiles} (heaviest by chain time: {heaviest}), cold and second frame")
