"""Panic fidelity (PBRT_FLAG_PANIC_FIDELITY): the rays the hot path skips
because their results never reach the film, but whose traversal can panic in
the reference:

- EstimateDirect's BSDF-sampled MIS half for an area light, Sphere.PdfWi
  included (pkg/pbrt/integrator.go:132-192, sphere.go:350-363);
- the closest hit at bounces == maxDepth (pkg/integrator/path.go:44-45, 66).

The scene puts a sphere of radius 5e159 about 1e160 away in one direction
octant: any ray that reaches its leaf box overflows EFloat in
Sphere.Intersect and panics (efloat.go:102-111), while the camera rays (down
onto a floor disk) and the shadow rays (a short segment to an area-light
sphere) never reach it. With maxDepth 2 the only rays that can are the two
above, so the film renders without the flag and panics with it. Expected
panic sites come from the oracle (no Go toolchain here: "parity unpinned"
against Go itself, pinned oracle-vs-device).
"""
import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

FID = abi.PBRT_FLAG_PANIC_FIDELITY


def fidelity_scene(octant):
    s = G.Scene()
    m = s.add_matte((0.5, 0.5, 0.5))
    floor = s.add_disk(G.mul(G.translate(0, 0, 0), G.rotate(0, 90)), 0.0, 100.0)
    s.add_primitive(floor, m)
    c = [o * 5.77e159 for o in octant]
    big = s.add_sphere(G.translate(*c), 5e159)
    s.add_primitive(big, m)
    light = s.add_sphere(G.translate(0, 5, 0), 0.5)
    s.add_area_light((5, 5, 5), light)
    s.set_film(32, 32)
    s.set_camera(G.look_at((0, 20, 20), (0, 0, 0), (0, 1, 0)), fov=60)
    return s.build(max_prims_in_node=1)


# (octant of the panic sphere, n_dims, the bounce of the expected panic):
# MIS ray (bounce 1: its u_scattering comes from the RNG when n_dims <= 3, the
# 2D stratified values being (0,0), ledger #3), or the maxDepth hit (bounce 2)
CASES = [((1, 1, 1), 2, 1), ((-1, -1, 1), 0, 1), ((1, 1, -1), 4, 2), ((-1, -1, -1), 4, 2)]


def panic_site(st):
    return (st.panic_kind, st.panic_tile, st.panic_px, st.panic_py, st.panic_sample, st.panic_bounce)


@pytest.mark.parametrize("octant,nd,bounce", CASES)
def test_oracle_panics_only_with_the_fidelity_rays(octant, nd, bounce):
    sc = fidelity_scene(octant)
    rc, film, _ = O.render(sc.desc, abi.render_desc(3, 3, max_depth=2, n_dims=nd), threads=4)
    assert rc == 0 and np.isfinite(film).all() and film.max() > 0
    rc, _, st = O.render(sc.desc, abi.render_desc(3, 3, max_depth=2, n_dims=nd, flags=FID), threads=4)
    assert rc == abi.PBRT_E_REF_PANIC and st.panic_kind == abi.PBRT_PANIC_EFLOAT
    assert st.panic_bounce == bounce


def test_oracle_fidelity_rays_leave_films_unchanged():
    """On scenes that do not panic the extra rays change no film value."""
    for scene, rd in ((O.OracleScene.readme(48, 32), abi.render_desc(3, 3)),
                      (O.OracleScene.cornell(32, 32), abi.render_desc(3, 3, max_depth=4))):
        _, f0, _ = O.render(scene.desc, rd, threads=4)
        rd.flags = FID
        rc, f1, _ = O.render(scene.desc, rd, threads=4)
        assert rc == 0 and np.array_equal(f0.view(np.uint64), f1.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("octant,nd,bounce", CASES)
def test_device_panic_fidelity_matches_the_oracle(octant, nd, bounce):
    sc = fidelity_scene(octant)
    rd = abi.render_desc(3, 3, max_depth=2, n_dims=nd)
    rc, ofilm, _ = O.render(sc.desc, rd, threads=4)
    assert rc == 0
    with G.Renderer(sc) as r:   # without the flag: the wave kernels where eligible, the oracle's film
        film, st = r.render(rd)
    assert np.array_equal(film.view(np.uint64), ofilm.view(np.uint64))
    rd.flags = FID
    rc, _, ost = O.render(sc.desc, rd, threads=4)
    assert rc == abi.PBRT_E_REF_PANIC
    with G.Renderer(sc) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    assert ei.value.code == abi.PBRT_E_REF_PANIC
    st = ei.value.stats
    assert st.kernel == abi.PBRT_KERNEL_SERIAL
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample,
            st.panic_bounce) == panic_site(ost)


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [abi.PBRT_INTEGRATOR_PATH, abi.PBRT_INTEGRATOR_DIRECT_LIGHTING])
def test_device_fidelity_rays_leave_films_unchanged(integrator):
    scene = G.Scene.cornell(32, 24)
    rd = abi.render_desc(3, 3, max_depth=3, integrator=integrator)
    with G.Renderer(scene) as r:
        f0, _ = r.render(rd)
    rd.flags = FID
    with G.Renderer(scene) as r:
        f1, st = r.render(rd)
    assert st.kernel == abi.PBRT_KERNEL_SERIAL
    _, of, _ = O.render(scene.desc, rd, threads=4)
    assert np.array_equal(f0.view(np.uint64), f1.view(np.uint64))
    assert np.array_equal(f1.view(np.uint64), of.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["serial", "auto"])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
def test_device_efloat_panic_in_regular_tracing(kernel, mode):
    """maxDepth 3: the regular bounce-2 rays reach the panic sphere, so the
    reference panics in EFloat.Check without any flag; the device reports the
    same kind (PBRT_PANIC_EFLOAT) and site on every kernel."""
    sc = fidelity_scene((1, 1, -1))
    rd = abi.render_desc(3, 3, max_depth=3, mode=mode)
    rc, _, ost = O.render(sc.desc, rd, threads=4)
    assert rc == abi.PBRT_E_REF_PANIC and ost.panic_kind == abi.PBRT_PANIC_EFLOAT
    with G.Renderer(sc, kernel=kernel) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample,
            st.panic_bounce) == panic_site(ost)
