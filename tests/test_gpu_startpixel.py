"""The windowed wave StartPixel (render_common.h start_pixel_wave, rp.sp_window).

Stratified.StartPixel (/root/reference/pkg/sampler/stratified.go:21-48, with
StratifiedSample1D/2D and Shuffle, sampling.go:101-145) at sample counts whose
raw draws do not fit a k_chain_ci workgroup's LDS (config C: 256 spp). Without
jitter the windowed version resolves the same pcg_bounded rejections through
a 256-entry ring of raw draws, shuffles uint16 indices in LDS and writes each
value (i + 0.5) / n once; with jitter (or beyond PBRT_SP_WINDOW_KB) the lane-0
replay runs as before. Every film below is the oracle's, bit for bit, on the
chain (EXACT), THROUGHPUT's setup and DirectLighting's setup kernels.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu

THREADS = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def check(scene, rd, kernel):
    with G.Renderer(scene) as r:
        film, st = r.render(rd)
    assert st.kernel == kernel, st.kernel
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0 and st.paths_traced == ost.paths
    assert np.array_equal(bits(film), bits(ofilm)), int((film != ofilm).sum())
    assert film.max() > 0


# (spp_x, spp_y, n_dims, jitter): 144 and 256 spp run the windowed StartPixel
# at n_dims 4 and 2; 1 dim at a pinhole; 400 spp x 4 dims and jitter stay on
# the lane-0 replay
CASES = [(12, 12, 4, False), (16, 16, 4, False), (16, 16, 2, False), (16, 16, 1, False), (20, 20, 4, False),
         (11, 13, 3, False), (16, 16, 4, True)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}-d{c[2]}{'-j' if c[3] else ''}")
@pytest.mark.parametrize("waves", ["1", "4"])
def test_windowed_start_pixel_exact(case, waves, monkeypatch):
    monkeypatch.setenv("PBRT_CI_WAVES", waves)
    sx, sy, nd, jit = case
    check(G.Scene.cornell(32, 32), abi.render_desc(sx, sy, n_dims=nd, jitter=jit, max_depth=8), abi.PBRT_KERNEL_WAVE_CI)


@pytest.mark.parametrize("case", CASES[:2] + CASES[-1:], ids=lambda c: f"{c[0]}x{c[1]}-d{c[2]}{'-j' if c[3] else ''}")
def test_windowed_start_pixel_throughput_and_direct_lighting(case):
    sx, sy, nd, jit = case
    check(G.Scene.readme(48, 32), abi.render_desc(sx, sy, n_dims=nd, jitter=jit, mode=abi.PBRT_MODE_THROUGHPUT),
          abi.PBRT_KERNEL_WAVE)
    check(G.Scene.readme(48, 32), abi.render_desc(sx, sy, n_dims=nd, jitter=jit, max_depth=3,
                                                  integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING),
          abi.PBRT_KERNEL_WAVE_DL)
