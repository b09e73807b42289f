"""Path renders with fewer than three sampled dimensions on the wave pipeline.

Stratified(x, y, jitter, n) with n < 3 (pkg/sampler/stratified.go:12-19): the
CameraSample still reads pFilm (2D dim 0) and time (1D dim 0) from the
stratified arrays, so every sample of a pixel traces the pixel's camera ray
(pLens, 2D dim 1, is a PCG32 draw at n = 1, which a pinhole never reads:
sampler.go:75-80, pixel.go:60-80). What changes is bounce 1: its light sample
uLight (2D dim 2) is a PCG32 draw of each sample, so the bounce-1 estimate is
per sample (path_step's first step traces its own shadow ray) instead of the
pixel's cached (0,0) estimate. The chain is unchanged: a path's draw count
still depends only on its RNG offset.

Bit-exact against the oracle: README / Cornell scenes, both modes, the path
wavefront, the materials pipeline (kX), a triangle mesh, and config N's frame
(1080p, Stratified(8,8) with 2 sampled dims) on spread tiles.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu

THREADS = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))
MB = abi.PBRT_MODE_THROUGHPUT


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def check(scene, rd, want=abi.PBRT_KERNEL_WAVE_CI, nonzero=True):
    with G.Renderer(scene) as r:
        film, st = r.render(rd)
    if want is not None:
        assert st.kernel == want, st.kernel
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0 and st.paths_traced == ost.paths
    assert np.array_equal(bits(film), bits(ofilm)), int((film != ofilm).sum())
    if nonzero:
        assert film.max() > 0
    return film


@pytest.mark.parametrize("n_dims", [1, 2])
@pytest.mark.parametrize("kw", [dict(spp_x=8, spp_y=8), dict(spp_x=5, spp_y=7, jitter=True),
                                dict(spp_x=4, spp_y=4, max_depth=12, rr_threshold=0.5),
                                dict(spp_x=4, spp_y=4, light_strategy=abi.PBRT_LIGHT_STRATEGY_POWER),
                                dict(spp_x=16, spp_y=16, max_depth=4)])
@pytest.mark.parametrize("scene", ["readme", "cornell"])
def test_low_dims_exact(scene, kw, n_dims):
    sc = G.Scene.readme(64, 48) if scene == "readme" else G.Scene.cornell(64, 48)
    # Power light selection runs the wave pipeline only when every light's pdf is > 0
    power = kw.get("light_strategy") == abi.PBRT_LIGHT_STRATEGY_POWER
    check(sc, abi.render_desc(n_dims=n_dims, **kw), want=None if power else abi.PBRT_KERNEL_WAVE_CI,
          nonzero=not power)   # README's lights under Power: the oracle's film is black too


@pytest.mark.parametrize("n_dims", [1, 2])
def test_low_dims_throughput_mode(n_dims):
    check(G.Scene.readme(64, 48), abi.render_desc(6, 6, n_dims=n_dims, mode=MB), want=abi.PBRT_KERNEL_WAVE)


@pytest.mark.parametrize("n_dims", [1, 2])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, MB])
def test_low_dims_path_wavefront(n_dims, mode, monkeypatch):
    """PBRT_PATHS_WF=1: bounce 1's per-sample shadow ray in k_pw_start."""
    monkeypatch.setenv("PBRT_PATHS_WF", "1")
    check(G.Scene.readme(48, 40), abi.render_desc(5, 5, n_dims=n_dims, mode=mode),
          want=abi.PBRT_KERNEL_WAVE_CI if mode == abi.PBRT_MODE_EXACT else abi.PBRT_KERNEL_WAVE)


@pytest.mark.parametrize("n_dims", [1, 2])
@pytest.mark.parametrize("ci_waves", ["1", "4"])
def test_low_dims_materials(n_dims, ci_waves, monkeypatch):
    """Mirror / smooth glass (kX chain and paths)."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    check(G.Scene.readme_glass(64, 40), abi.render_desc(6, 6, n_dims=n_dims))


@pytest.mark.parametrize("n_dims", [1, 2])
def test_low_dims_mesh(n_dims):
    check(G.Scene.heightfield(48, 32, quads=24, seed=1, spheres=True), abi.render_desc(4, 4, n_dims=n_dims))


@pytest.mark.slow
def test_config_N_sampled_tiles():
    """Config N: the README scene at 1920x1080, Stratified(8,8) with 2 sampled
    dimensions, Path(10): 24 spread tiles bit for bit (tile_stride 340)."""
    sc = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(8, 8, n_dims=2, tile_begin=7, tile_stride=340)
    check(sc, rd)
