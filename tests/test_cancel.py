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


def cancel_after(r, seconds):
    t = threading.Timer(seconds, lambda: G.lib().pbrt_gpu_cancel(r.h))
    t.start()
    return t


def full_time(r, rd):
    t0 = time.time()
    r.render(rd)
    return time.time() - t0


def check_cancel_then_render(sc, rd, small_rd, delay=0.4, bound=0.25):
    with G.Renderer(sc) as r:
        G.lib().pbrt_gpu_cancel(r.h)   # nothing in flight: a no-op
        t0 = time.time()
        timer = cancel_after(r, delay)
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
        dt = time.time() - t0
        timer.join()
        assert ei.value.code == abi.PBRT_E_CANCELLED
        assert dt < delay + bound, f"the frame ran {dt - delay:.3f} s past the cancel"
        # the cancel died with its render: the next one is exact
        film, st = r.render(small_rd)
    rc, of, _ = O.render(sc.desc, small_rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0 and np.array_equal(bits(film), bits(of))
    return dt


def test_cancel_config_c_chain_then_render_again():
    """config C (Cornell, 1080p, Stratified(16,16), Path(8)): ~10 s of k_chain_ci."""
    sc = G.Scene.cornell(1920, 1080)
    check_cancel_then_render(sc, abi.render_desc(16, 16, max_depth=8),
                             abi.render_desc(2, 2, max_depth=8, tile_end=48))


def test_cancel_throughput_mode_paths():
    sc = G.Scene.cornell(1920, 1080)
    check_cancel_then_render(sc, abi.render_desc(32, 32, max_depth=8, mode=abi.PBRT_MODE_THROUGHPUT),
                             abi.render_desc(2, 2, max_depth=8, tile_end=48), delay=0.3)


def test_cancel_serial_kernel():
    """A scene holding glass renders on the serial kernel (one lane per tile)."""
    sc = G.Scene.readme(1920, 1080)
    glass = sc.add_glass()
    sph = sc.add_sphere(G.translate(0, 0, 0), 5.0)
    sc.add_primitive(sph, glass, G.translate(50, 2.5, 50))
    sc.build(2)
    check_cancel_then_render(sc, abi.render_desc(8, 8), abi.render_desc(2, 2, tile_end=32), delay=0.3)


def test_cancel_direct_lighting_wave():
    sc = G.Scene.cornell(1920, 1080)
    rd = abi.render_desc(32, 32, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)
    check_cancel_then_render(sc, rd, abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING,
                                                     tile_end=48), delay=0.2)


def test_cancel_outside_a_render_is_a_no_op():
    sc = G.Scene.readme(64, 48)
    rd = abi.render_desc(2, 2)
    with G.Renderer(sc) as r:
        f1, _ = r.render(rd)
        G.lib().pbrt_gpu_cancel(r.h)
        f2, _ = r.render(rd)
    assert np.array_equal(bits(f1), bits(f2))
