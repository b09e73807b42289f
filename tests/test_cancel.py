"""Cancellation (pbrt_gpu_cancel, include/pbrt_gpu.h): the reference's render
stops issuing tiles once its context is done (pkg/pbrt/integrator.go:305-345,
errgroup + ctx). Here a cancel from another thread stops the frame in flight
within about 100 ms on every kernel family, its render returns
PBRT_E_CANCELLED, and the context stays usable: the next render is bit-exact.
"""
import os
import threading
import time

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def full_time(r, rd):
    t0 = time.time()
    r.render(rd)
    return time.time() - t0


def check_cancel_then_render(sc, rd, small_rd, kernel, delay=0.4, bound=0.25):
    """Enqueue the frame (render_async returns with the render in flight), cancel
    it from another thread after `delay`, and require synchronize to return
    PBRT_E_CANCELLED within `bound` seconds of the cancel, from the kernel
    family `kernel` (pbrt_gpu_stats.kernel of the cancelled render)."""
    with G.Renderer(sc) as r:
        G.lib().pbrt_gpu_cancel(r.h)   # nothing in flight: a no-op
        r.render_async(rd)
        t_cancel = []

        def fire():
            t_cancel.append(time.time())
            G.lib().pbrt_gpu_cancel(r.h)

        timer = threading.Timer(delay, fire)
        timer.start()
        with pytest.raises(G.PbrtError) as ei:
            r.synchronize()
        t_done = time.time()
        timer.join()
        assert ei.value.code == abi.PBRT_E_CANCELLED
        assert ei.value.stats is not None and ei.value.stats.kernel == kernel
        dt = t_done - t_cancel[0]
        assert dt < bound, f"the frame ran {dt:.3f} s past the cancel"
        # the cancel died with its render: the next one is exact
        film, st = r.render(small_rd)
    rc, of, _ = O.render(sc.desc, small_rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0 and np.array_equal(bits(film), bits(of))
    return dt


def test_cancel_config_c_chain_then_render_again():
    """config C (Cornell, 1080p, Stratified(16,16), Path(8)): ~10 s of k_chain_ci."""
    sc = G.Scene.cornell(1920, 1080)
    check_cancel_then_render(sc, abi.render_desc(16, 16, max_depth=8),
                             abi.render_desc(2, 2, max_depth=8, tile_end=48), abi.PBRT_KERNEL_WAVE_CI)


def test_cancel_throughput_mode_paths():
    sc = G.Scene.cornell(1920, 1080)
    check_cancel_then_render(sc, abi.render_desc(32, 32, max_depth=8, mode=abi.PBRT_MODE_THROUGHPUT),
                             abi.render_desc(2, 2, max_depth=8, tile_end=48), abi.PBRT_KERNEL_WAVE, delay=0.3)


def test_cancel_serial_kernel():
    """Stratified with n_dims = 0 (pFilm from the RNG: the camera ray is per
    sample) renders on the serial kernel (one lane per tile), whose pixels poll
    the flag by wall clock."""
    sc = G.Scene.readme(1920, 1080)
    check_cancel_then_render(sc, abi.render_desc(8, 8, n_dims=0), abi.render_desc(2, 2, n_dims=0, tile_end=32),
                             abi.PBRT_KERNEL_SERIAL, delay=0.3)


def test_cancel_direct_lighting_wave():
    """k_dl_* is fast: size the frame from a timed 8x8 render so it lasts >= ~1 s."""
    sc = G.Scene.cornell(1920, 1080)
    dl = dict(integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)
    with G.Renderer(sc) as r:
        t8 = full_time(r, abi.render_desc(8, 8, **dl))
    side = 8
    while side < 32 and t8 * (side / 8) ** 2 < 1.0:   # the k_dl_* kernels stage <= 8192 stratified values
        side *= 2
    check_cancel_then_render(sc, abi.render_desc(side, side, **dl),
                             abi.render_desc(2, 2, tile_end=48, **dl), abi.PBRT_KERNEL_WAVE_DL,
                             delay=min(0.1, t8 * (side / 8) ** 2 / 4))


def test_cancel_outside_a_render_is_a_no_op():
    sc = G.Scene.readme(64, 48)
    rd = abi.render_desc(2, 2)
    with G.Renderer(sc) as r:
        f1, _ = r.render(rd)
        G.lib().pbrt_gpu_cancel(r.h)
        f2, _ = r.render(rd)
    assert np.array_equal(bits(f1), bits(f2))
