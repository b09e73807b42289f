"""The process-wide schedule cache (render.hip, sched_cache_*).

internal/render/server.go:29-164 builds a fresh scene, integrator and renderer
for every request. A fresh context therefore starts from the schedule another
context measured on the same scene content and configuration, instead of the
cold-frame probe. Only the schedule changes: every frame of every context is
the oracle's, bit for bit.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


def oracle_film(scene, rd):
    rc, film, _ = O.render(scene.desc, rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0
    return film


def test_fresh_context_starts_from_another_contexts_schedule(monkeypatch):
    monkeypatch.setenv("PBRT_CI_ORDER_CACHE", "1")
    G.schedule_cache_clear()
    rd = abi.render_desc(8, 8)
    scene = G.Scene.readme(320, 192)
    want = oracle_film(scene, rd)
    with G.Renderer(scene) as a:   # the first request of the process: probe, then its own measurement
        for frame, src in enumerate(["probe", "learned"]):
            film, st = a.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            assert a.schedule_source() == src, frame
            assert same_bits(film, want), frame
    # a later request: a new scene object with the same content, a new context
    scene2 = G.Scene.readme(320, 192)
    with G.Renderer(scene2) as b:
        for frame, src in enumerate(["cached", "learned"]):
            film, _ = b.render(rd)
            assert b.schedule_source() == src, frame
            assert same_bits(film, want), frame
    # other content or another configuration: no match
    with G.Renderer(G.Scene.readme(320, 176)) as c:
        c.render(rd)
        assert c.schedule_source() == "probe"
    rd_shard = abi.render_desc(8, 8, tile_begin=1, tile_stride=2)
    with G.Renderer(scene2) as d:
        film, _ = d.render(rd_shard)
        assert d.schedule_source() == "probe"
        assert same_bits(film, oracle_film(scene2, rd_shard))
    G.schedule_cache_clear()
    with G.Renderer(scene2) as e:
        e.render(rd)
        assert e.schedule_source() == "probe"


def test_schedule_cache_off(monkeypatch):
    monkeypatch.setenv("PBRT_CI_ORDER_CACHE", "1")
    G.schedule_cache_clear()
    rd = abi.render_desc(4, 4)
    scene = G.Scene.readme(160, 96)
    with G.Renderer(scene) as a:
        a.render(rd)
        a.render(rd)
    monkeypatch.setenv("PBRT_CI_ORDER_CACHE", "0")
    with G.Renderer(scene) as b:
        b.render(rd)
        assert b.schedule_source() == "probe"
    G.schedule_cache_clear()


def test_completion_driven_path_stage_ragged_tiles_and_mode_switch(monkeypatch):
    """the completion-driven path stage launches k_paths_ci
    over whole slots in completion order, ceil(ppt / P) groups per slot. With
    tile size 13 (169 pixels: P = 8 does not divide it) and the one-GPU split
    forced (one-wave tiles, 6 heavy tiles), the steady-state frames are the
    oracle's bit for bit, also after a THROUGHPUT frame in between has
    overwritten the wave buffers."""
    monkeypatch.setenv("PBRT_CI_WAVES", "1")
    monkeypatch.setenv("PBRT_CI_HEAVY", "6")
    scene = G.Scene.readme(320, 240)
    rd = abi.render_desc(4, 4, tile_size=13)
    want = oracle_film(scene, rd)
    with G.Renderer(scene) as r:
        for frame, mode in enumerate(["exact", "exact", "throughput", "exact"]):
            if mode == "throughput":
                r.render(abi.render_desc(4, 4, tile_size=13, mode=abi.PBRT_MODE_THROUGHPUT))
                continue
            film, st = r.render(rd)
            _, heavy = r.tile_ticks()
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            assert (heavy > 0) == (frame > 0), (frame, heavy)
            assert same_bits(film, want), frame


def test_gate_stall_renders_the_frame_again(monkeypatch, capfd):
    """A dispatcher that serialises kernels across streams (rocprofv3 counter
    collection does) never runs the chains beside the k_gate waiting for them.
    PBRT_GATE_HOLD=1 builds that order on purpose: the light chain launch waits
    for the whole path stage. k_gate sees no chain progress for 1 s, opens every
    gate of the frame, and pbrt_gpu_synchronize renders the frame again with the
    path stage after the chains; after two such frames the context keeps the
    overlap off. Every frame is the oracle's, bit for bit."""
    monkeypatch.setenv("PBRT_CI_WAVES", "1")
    monkeypatch.setenv("PBRT_CI_HEAVY", "6")
    monkeypatch.setenv("PBRT_GATE_HOLD", "1")
    scene = G.Scene.readme(320, 240)
    rd = abi.render_desc(4, 4)
    want = oracle_film(scene, rd)
    with G.Renderer(scene) as r:
        for frame in range(4):
            film, st = r.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            assert same_bits(film, want), frame
            assert r.overlap_slots() == 0, frame   # the re-render (and the probe frame) ran without it
            err = capfd.readouterr().err
            assert ("k_gate stalled twice" in err) == (frame == 2), (frame, err)


@pytest.mark.parametrize("overlap_all", ["1", "0"])
def test_completion_driven_path_stage_without_split(monkeypatch, overlap_all):
    """Frames without a heavy/light split (no tile heavy enough, or a shard of
    multi-wave tiles) run the completion-driven path stage too
    (PBRT_PATHS_OVERLAP_ALL, default on): one chain launch, the path chunks
    released by its completion list. Ragged 13-pixel tiles, one and two waves
    per tile; every frame is the oracle's, bit for bit, with the stage on and
    off."""
    monkeypatch.setenv("PBRT_PATHS_OVERLAP_ALL", overlap_all)
    monkeypatch.setenv("PBRT_CI_SPLIT", "0")
    scene = G.Scene.readme(320, 240)
    for waves in ("1", "2"):
        monkeypatch.setenv("PBRT_CI_WAVES", waves)
        rd = abi.render_desc(4, 4, tile_size=13, tile_begin=1, tile_stride=3)
        want = oracle_film(scene, rd)
        with G.Renderer(scene) as r:
            for frame in range(3):
                film, st = r.render(rd)
                _, heavy = r.tile_ticks()
                assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
                assert heavy == 0, (waves, frame, heavy)
                # frame 0 is the probe's (no completion-driven stage before a learned schedule)
                assert r.overlap_slots() == (st.tiles_rendered if frame > 0 and overlap_all == "1" else 0), \
                    (waves, frame)
                assert same_bits(film, want), (waves, frame)


def test_multiwave_shard_heavy_tiles_at_8_waves(monkeypatch):
    """A learned multi-wave Matte shard that fits the wave slots (as 1/8 of B
    does) runs its heaviest tiles, min(PBRT_CI_SPLIT8, slots / 16), at 8 waves
    beside the rest at its own waves per tile; off with PBRT_CI_SPLIT8=0. Every
    frame is the oracle's, bit for bit."""
    monkeypatch.setenv("PBRT_CI_WAVES", "4")
    scene = G.Scene.readme(320, 240)
    rd = abi.render_desc(4, 4, tile_begin=2, tile_stride=3)   # 100 of the 300 tiles
    want = oracle_film(scene, rd)
    for k, expect in (("32", 100 // 16), ("0", 0)):
        monkeypatch.setenv("PBRT_CI_SPLIT8", k)
        with G.Renderer(scene) as r:
            for frame in range(3):
                film, st = r.render(rd)
                _, heavy = r.tile_ticks()
                assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
                assert heavy == (expect if frame > 0 else 0), (k, frame, heavy)
                assert same_bits(film, want), (k, frame)


def test_completion_driven_path_stage_over_several_batches(monkeypatch):
    """A frame split into several tile batches (a small wave-buffer budget):
    each batch runs its own chain and path stage, the next batch only after
    both. Three frames of one context, each the oracle's bit for bit."""
    monkeypatch.setenv("PBRT_WAVE_BUFFER_GB", "0.02")
    scene = G.Scene.readme(320, 240)
    rd = abi.render_desc(4, 4)
    want = oracle_film(scene, rd)
    with G.Renderer(scene) as r:
        for frame in range(3):
            film, st = r.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
            assert st.batches > 1, st.batches
            assert same_bits(film, want), frame
