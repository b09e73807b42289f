"""In-kernel ray counters ("rays/s (closest-hit + any-hit
segments, counted in-kernel)"; pbrt_gpu_stats.rays_closest / rays_shadow).

The counted segments are the reference's: one closest-hit query per iteration
of Path.Li's loop (pkg/integrator/path.go:44-45, also at bounces == maxDepth,
where path.go:66 breaks after the query), one per DirectLighting.Li call
(directlighting.go:67, incl. the SpecularTransmit recursion), and one any-hit
ray per traced VisibilityTester (integrator.go:112-119). Every kernel family
(serial, the wave pipeline's k_paths_ci, the path wavefront k_pw_*, k_dl_*)
must report exactly the oracle's counts, which restate those sites.
"""
import os

import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu


def counts(sc, rd, kernel="auto", lanes=0):
    rc, _, ost = O.render(sc.desc, rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0
    with G.Renderer(sc, kernel=kernel) as r:
        _, st = r.render(rd)
    return st, ost


@pytest.mark.parametrize("kernel", ["serial", "auto"])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("depth", [1, 2, 10])
def test_path_ray_counts_match_the_oracle(kernel, mode, depth):
    sc = G.Scene.readme(64, 48)
    st, ost = counts(sc, abi.render_desc(3, 3, max_depth=depth, mode=mode), kernel)
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
    assert st.rays_closest >= st.paths_traced > 0


@pytest.mark.parametrize("kernel", ["serial", "auto"])
@pytest.mark.parametrize("strategy", [abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE])
def test_direct_lighting_ray_counts(kernel, strategy):
    sc = G.Scene.cornell(48, 32)
    rd = abi.render_desc(3, 3, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy)
    st, ost = counts(sc, rd, kernel)
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
    assert st.rays_closest == st.paths_traced   # one query per sample, no recursion through Matte


def test_glass_recursion_ray_counts():
    """DirectLighting through glass: every recursion level is one more query."""
    sc = G.Scene.readme(96, 64)
    glass = sc.add_glass()
    sph = sc.add_sphere(G.translate(0, 0, 0), 5.0)
    sc.add_primitive(sph, glass, G.translate(50, 2.5, 50))
    sc.build(2)
    rd = abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, max_depth=6)
    st, ost = counts(sc, rd)
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
    assert st.rays_closest > st.paths_traced


def test_mesh_path_wavefront_ray_counts():
    """k_pw_* (the default for mesh scenes) counts like the rest."""
    sc = G.Scene.heightfield(48, 32, quads=40, seed=1, spheres=True)
    for mode in (abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT):
        st, ost = counts(sc, abi.render_desc(3, 3, mode=mode))
        assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)


def test_cornell_wave_ray_counts_multi_batch():
    """Counts accumulate over the wave pipeline's tile batches."""
    sc = G.Scene.cornell(80, 48)
    os.environ["PBRT_WAVE_BUFFER_GB"] = "0.0005"
    try:
        st, ost = counts(sc, abi.render_desc(4, 4, max_depth=8))
    finally:
        del os.environ["PBRT_WAVE_BUFFER_GB"]
    assert st.batches > 1
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
