"""Mirror and smooth Glass: pkg/materials/mirror.go:9-32,
pkg/materials/glass.go:15-75 and their BxDFs in pkg/pbrt/reflection.go
(FrDielectric :21-42, Refract :106-118, FresnelSpecular :465-536,
SpecularReflection :538-574), driven by Path.Li's specular bookkeeping
(pkg/integrator/path.go:82-117).

Quirks restated (and therefore tested here):
- SpecularReflection is typed Reflection|Diffuse, so a Mirror still samples a
  light (its F and Pdf are 0) and its sampled type is 0 (no specular bounce);
- FresnelSpecular's radiance scale is etaI^2 / (etaT / etaT) = etaI^2;
- smooth glass is a single specular lobe: no light sample, so its paths consume
  fewer draws per bounce;
- DirectLighting asks for one lobe per BxDF (directlighting.go:76), so smooth
  glass is SpecularReflection + SpecularTransmission there (glass.go:58-72):
  SpecularReflect matches no lobe (SpecularReflection is Reflection|Diffuse),
  SpecularTransmit refracts and recurses into Li at depth + 2; a Mirror renders
  under DirectLighting exactly like a black Matte;
- rough glass (MicrofacetReflection + MicrofacetTransmission over
  TrowbridgeReitz, pkg/pbrt/microfacet.go, reflection.go:670-835): SampleWH
  shadows its result and returns nil, so any BSDF.SampleF on it dereferences
  nil in Reflect/Refract -- in Path.Li's bounce sampling and in EstimateDirect's
  BSDF-sampled half, which runs for every area light (integrator.go:134-139).
  The reference panics there (PBRT_PANIC_NIL_DEREF); with delta lights only,
  DirectLighting renders rough glass through the microfacet F and Pdf, whose
  own quirks (D's alphaX*alphaY, MicrofacetTransmission.F's inverted hemisphere
  test, its unset TransportMode) are restated.

Path renders of these scenes (smooth glass, mirror, OrenNayar; n_dims >= 1)
run on the wave pipeline's kX instantiations (k_wf_primary / k_chain_ci /
k_paths_ci / k_mb_setup over BSDFX, with Path.Li's etaScale); everything else
(n_dims 0, DirectLighting's specular recursion, rough glass) on the serial
kernel. Both are checked bit for bit against the oracle.

No reference test covers these materials and there is no Go toolchain here:
device-vs-oracle parity is bit-exact but "parity unpinned" against Go itself.
The oracle's FrDielectric is pinned by closed forms below.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi
from scenes import material_scene, mesh_material_scene  # noqa: F401


def bits(a):
    return a.view(np.uint64)


# ------------------------------------------------------------------ CPU tests
def test_fr_dielectric_closed_forms():
    """FrDielectric at normal incidence is ((eta-1)/(eta+1))^2, total internal
    reflection returns 1 (reflection.go:21-42)."""
    L = O.lib()
    f = L.oracle_fr_dielectric
    assert f(1.0, 1.0, 1.5) == pytest.approx(0.04, rel=1e-15)
    assert f(-1.0, 1.0, 1.5) == pytest.approx(0.04, rel=1e-15)   # leaving: the indices swap
    assert f(-0.2, 1.0, 1.5) == 1.0                              # sin_t = 1.5 * 0.98 > 1
    assert 0.04 < f(0.3, 1.0, 1.5) < 1.0


def test_oracle_materials_render_deterministically():
    sc = material_scene()
    rd = abi.render_desc(3, 3, max_depth=6)
    rc, f1, st = O.render(sc.desc, rd, threads=1)
    assert rc == 0 and np.isfinite(f1).all() and f1.max() > 0
    rc, f8, _ = O.render(sc.desc, rd, threads=8)
    assert np.array_equal(bits(f1), bits(f8))
    scm = material_scene("matte")   # the builder owns the desc: keep it alive
    _, fm, _ = O.render(scm.desc, rd, threads=8)
    assert not np.array_equal(f1, fm)   # the glass and mirror spheres are in view


def test_oracle_direct_lighting_mirror_is_black_matte():
    """A Mirror's SpecularReflection is typed Reflection|Diffuse (reflection.go:538-544):
    DirectLighting's SpecularReflect (Reflection|Specular) and SpecularTransmit match
    no lobe, its F is 0, and it renders exactly like a black Matte (same draws)."""
    for strategy in (abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE):
        rd = abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy)
        sa, sb = material_scene(kt=(0, 0, 0), glass_kr=(0, 0, 0)), material_scene("black")
        rc, fa, _ = O.render(sa.desc, rd, threads=8)
        rc2, fb, _ = O.render(sb.desc, rd, threads=8)
        assert rc == rc2 == 0 and np.array_equal(bits(fa), bits(fb))


def readme_glass_scene(w=96, h=64, special="glass", mirror=False):
    """internal/render/server.go:67-91's commented-out glass sphere added to the
    README scene (pbrtgpu.Scene.readme_glass; bench.py config G)."""
    return G.Scene.readme_glass(w, h, special=special, mirror=mirror)


@pytest.mark.parametrize("strategy", [abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE])
def test_oracle_direct_lighting_refracts_through_smooth_glass(strategy):
    """DirectLighting asks for one lobe per BxDF (allowMultipleLobes false,
    directlighting.go:76): smooth glass is SpecularReflection + SpecularTransmission
    (glass.go:58-72), and SpecularTransmit (integrator.go:383-422) follows the
    Transmission|Specular lobe into Li at depth + 2 (#23). So:
    - the glass sphere is not a black Matte: light refracted from the scene;
    - with maxDepth 1 no specular call runs and glass renders as a black Matte;
    - the recursion's light samples consume draws: pixels that see the glass
      draw more PCG32 numbers than with a black Matte sphere."""
    rd = abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy, max_depth=5)
    sg, sb = readme_glass_scene(), readme_glass_scene(special="black")
    rc, fg, _ = O.render(sg.desc, rd, threads=8)
    rc2, fb, _ = O.render(sb.desc, rd, threads=8)
    assert rc == rc2 == 0 and np.isfinite(fg).all()
    assert (fg.sum(axis=2) > fb.sum(axis=2)).sum() > 100   # light through the glass sphere
    rd1 = abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy, max_depth=1)
    _, g1, _ = O.render(sg.desc, rd1, threads=8)
    _, b1, _ = O.render(sb.desc, rd1, threads=8)
    assert np.array_equal(bits(g1), bits(b1))
    ntiles = O.lib().oracle_num_tiles(C.byref(sg.desc), C.byref(rd))
    more = same = 0
    for tile in range(ntiles):
        rcg, dg = O.tile_draws(sg.desc, rd, tile)
        rcb, db = O.tile_draws(sb.desc, rd, tile)
        assert rcg == rcb == 0
        more += int((dg - db > 4).sum())           # a recursion level draws >= 5 numbers
        same += int((np.abs(dg - db) <= 2).sum())  # StartPixel rejections move by a draw or two
    assert more > 20 and same > more   # only the pixels that see the glass draw more


def test_oracle_rough_glass_panics_like_the_reference():
    sc = material_scene(rough=0.3)
    for rd in (abi.render_desc(2, 2),
               abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)):
        rc, _, st = O.render(sc.desc, rd, threads=4)
        assert rc == abi.PBRT_E_REF_PANIC and st.panic_kind == abi.PBRT_PANIC_NIL_DEREF
        assert st.panic_bounce == 1
    sp = material_scene(rough=0.3, area=False)   # Path.Li still samples a bounce
    rc, _, st = O.render(sp.desc, abi.render_desc(2, 2), threads=4)
    assert rc == abi.PBRT_E_REF_PANIC and st.panic_kind == abi.PBRT_PANIC_NIL_DEREF


def test_oracle_rough_glass_direct_lighting_with_delta_lights():
    """DirectLighting without area lights never samples the BSDF: rough glass
    renders through its microfacet F (reflection and transmission lobes)."""
    rd = abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)
    sr, sb = material_scene(rough=0.3, area=False), material_scene("black", area=False)
    rc, fr, _ = O.render(sr.desc, rd, threads=8)
    _, fb, _ = O.render(sb.desc, rd, threads=8)
    assert rc == 0 and np.isfinite(fr).all()
    assert (fr.sum(axis=2) > fb.sum(axis=2)).sum() > 10   # glossy highlights on the glass sphere


def test_material_desc_layout():
    m = abi.MaterialDesc()
    G.lib().pbrt_make_glass((G.C.c_double * 3)(0.5, 0.4, 0.3), (G.C.c_double * 3)(0.2, 0.1, 0.0), 0.0, 0.0, 1.5,
                            G.C.byref(m))
    assert m.type == abi.PBRT_MAT_GLASS and list(m.kr) == [0.5, 0.4, 0.3] and list(m.kt) == [0.2, 0.1, 0.0]
    assert m.eta == 1.5 and m.u_roughness == 0 and m.v_roughness == 0
    G.lib().pbrt_make_mirror((G.C.c_double * 3)(0.9, 0.9, 0.9), G.C.byref(m))
    assert m.type == abi.PBRT_MAT_MIRROR and list(m.kr) == [0.9, 0.9, 0.9] and m.eta == 0


# ------------------------------------------------------------------ GPU tests
def path_kernel(nd, mode):
    """The kernel a Path render of a Mirror/Glass/OrenNayar scene runs on (a
    pinhole camera: n_dims >= 1 keeps the camera ray the pixel's)."""
    if nd < 1:
        return abi.PBRT_KERNEL_SERIAL
    return abi.PBRT_KERNEL_WAVE_CI if mode == abi.PBRT_MODE_EXACT else abi.PBRT_KERNEL_WAVE


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("spp,nd,depth", [(3, 4, 6), (2, 2, 8), (4, 0, 5), (4, 5, 10), (2, 3, 2)])
def test_device_materials_bitexact_vs_oracle(mode, spp, nd, depth):
    sc = material_scene()
    rd = abi.render_desc(spp, spp, n_dims=nd, max_depth=depth, mode=mode)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    assert st.kernel == path_kernel(nd, mode)
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("ci_waves", ["1", "2", "4", "8"])
def test_device_materials_chain_waves_vs_oracle(monkeypatch, ci_waves):
    """k_chain_ci<kW, 32, kX> for every waves-per-tile count, and the serial
    kernel on the same render: all bit-identical to the oracle."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    sc = material_scene(w=48, h=40)
    rd = abi.render_desc(4, 4, max_depth=8)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
        film2, _ = r.render(rd)   # the second frame runs in the measured tile order
    assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
    assert np.array_equal(bits(film), bits(of)) and np.array_equal(bits(film2), bits(of))
    with G.Renderer(sc, kernel="serial") as r:
        fs, sts = r.render(rd)
    assert sts.kernel == abi.PBRT_KERNEL_SERIAL and np.array_equal(bits(fs), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
def test_device_materials_stats_match_oracle(mode):
    """Path counts and the in-kernel ray counters of the kX pipeline equal the
    oracle's (glass bounces sample no light: fewer shadow rays per bounce)."""
    sc = material_scene(w=40, h=32)
    rd = abi.render_desc(3, 3, max_depth=7, mode=mode)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    assert st.kernel == path_kernel(4, mode)
    assert np.array_equal(bits(film), bits(of))
    assert st.paths_traced == ost.paths
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", [abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE])
def test_device_materials_direct_lighting_vs_oracle(strategy):
    sc = material_scene()
    rd = abi.render_desc(3, 3, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    assert st.kernel == abi.PBRT_KERNEL_WAVE_DL
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", [abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE])
def test_device_direct_lighting_glass_at_8x8_spp_and_tile_ranges(strategy):
    """server.go:160's DirectLighting(UniformSampleAll, 10) through its glass
    sphere (server.go:67-94) at Stratified(8,8) on a 160x96 film, on the
    k_dl_* kernels: the whole film and a tile range bit-identical to the oracle,
    with the reference ray counts."""
    sc = readme_glass_scene(160, 96, mirror=False)
    rd = abi.render_desc(8, 8, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy, max_depth=10)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
        assert st.kernel == abi.PBRT_KERNEL_WAVE_DL and st.paths_traced == ost.paths
        assert np.array_equal(bits(film), bits(of))
        assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
        rd2 = abi.render_desc(8, 8, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy,
                              max_depth=10, tile_begin=7, tile_end=41, tile_stride=3)
        f2, _ = r.render(rd2)
    rc, of2, _ = O.render(sc.desc, rd2, threads=8)
    assert rc == 0 and np.array_equal(bits(f2), bits(of2))


@pytest.mark.gpu
def test_device_materials_power_strategy_and_rr():
    sc = material_scene(w=40, h=40)
    rd = abi.render_desc(3, 3, max_depth=12, rr_threshold=0.5, light_strategy=abi.PBRT_LIGHT_STRATEGY_POWER)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, _ = r.render(rd)
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [abi.PBRT_INTEGRATOR_PATH, abi.PBRT_INTEGRATOR_DIRECT_LIGHTING])
@pytest.mark.parametrize("area", [True, False])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
def test_device_rough_glass_vs_oracle(integrator, area, mode):
    """Rough glass: the reference's nil-dereference panic site, or (DirectLighting
    with delta lights) the microfacet film, bit-exact."""
    sc = material_scene(rough=0.3, area=area)
    rd = abi.render_desc(3, 3, integrator=integrator, mode=mode)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    with G.Renderer(sc) as r:
        if rc == 0:
            film, _ = r.render(rd)
            assert np.array_equal(bits(film), bits(of))
            return
        assert rc == abi.PBRT_E_REF_PANIC and ost.panic_kind == abi.PBRT_PANIC_NIL_DEREF
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    assert ei.value.code == abi.PBRT_E_REF_PANIC
    st = ei.value.stats
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == \
        (ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


@pytest.mark.gpu
def test_device_fidelity_on_mirror_glass_is_unsupported():
    sc = material_scene()
    with G.Renderer(sc) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(abi.render_desc(2, 2, flags=abi.PBRT_FLAG_PANIC_FIDELITY))
    assert ei.value.code == abi.PBRT_E_UNSUPPORTED


@pytest.mark.gpu
def test_device_matte_scene_keeps_the_wave_kernels():
    """A scene without Mirror/Glass still takes the wave pipeline."""
    sc = material_scene("matte")
    with G.Renderer(sc) as r:
        film, st = r.render(abi.render_desc(3, 3, max_depth=6))
    assert st.kernel != abi.PBRT_KERNEL_SERIAL
    scm = material_scene("matte")
    _, of, _ = O.render(scm.desc, abi.render_desc(3, 3, max_depth=6), threads=8)
    assert np.array_equal(bits(film), bits(of))


# ------------------------------------------------------------------ OrenNayar
# Matte with sigma != 0 (matte.go:30-35): OrenNayar (reflection.go:609-668) with
# the reference's B = 0.45 sigma^2 / (sigma^2 * 0.09) and its else-branch
# tanBeta = sinThetaO / |cos wo|; sampled like a Lambertian.
def test_oracle_oren_nayar_renders_and_clamps_sigma():
    rd = abi.render_desc(3, 3, max_depth=5)
    s0, s20, s90, s120, sneg = (material_scene("matte", sigma=v) for v in (0.0, 20.0, 90.0, 120.0, -5.0))
    f0 = O.render(s0.desc, rd, threads=8)[1]
    rc, f20, _ = O.render(s20.desc, rd, threads=8)
    assert rc == 0 and np.isfinite(f20).all() and not np.array_equal(f0, f20)
    assert np.array_equal(bits(O.render(s90.desc, rd, threads=8)[1]), bits(O.render(s120.desc, rd, threads=8)[1]))
    assert np.array_equal(bits(O.render(sneg.desc, rd, threads=8)[1]), bits(f0))   # Clamp(-5, 0, 90) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [abi.PBRT_INTEGRATOR_PATH, abi.PBRT_INTEGRATOR_DIRECT_LIGHTING])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("sigma", [20.0, 90.0])
def test_device_oren_nayar_vs_oracle(integrator, mode, sigma):
    sc = material_scene("matte", sigma=sigma)
    rd = abi.render_desc(3, 3, max_depth=6, integrator=integrator, mode=mode)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    expect = path_kernel(4, mode) if integrator == abi.PBRT_INTEGRATOR_PATH else abi.PBRT_KERNEL_WAVE_DL
    assert st.kernel == expect
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("kernel", ["auto", "serial"])
def test_device_readme_scene_with_the_commented_out_glass_sphere(mode, kernel):
    """internal/render/server.go:67-91 (commented out): a glass sphere of radius 5
    at (50, 2.5, 50) with Kr = Kt = 0.5 and index 1.5, added to the README scene;
    plus a mirror sphere beside it. The wave pipeline (kX) and the serial
    kernel, both bit-exact."""
    sc = readme_glass_scene(mirror=True)
    rd = abi.render_desc(2, 2, mode=mode)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc, kernel=kernel) as r:
        film, st = r.render(rd)
    assert st.kernel == (path_kernel(4, mode) if kernel == "auto" else abi.PBRT_KERNEL_SERIAL)
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
def test_device_readme_glass_scene_at_8x8_spp_bitexact():
    """The README scene with server.go's glass sphere and a mirror at config B's
    sampler (Stratified(8,8), Path(10)) on a 256x160 film: the kX chain (one wave
    per tile and the default) and paths, every tile bit-identical."""
    sc = readme_glass_scene(256, 160, mirror=True)
    rd = abi.render_desc(8, 8)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    assert st.kernel == abi.PBRT_KERNEL_WAVE_CI and st.paths_traced == ost.paths
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", [abi.PBRT_DL_UNIFORM_SAMPLE_ALL, abi.PBRT_DL_UNIFORM_SAMPLE_ONE])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("depth", [2, 5, 10, 64])
def test_device_direct_lighting_through_glass_vs_oracle(strategy, mode, depth):
    """DirectLighting's SpecularTransmit recursion through smooth glass
    (directlighting.go:76,97-101, integrator.go:383-422, glass.go:58-72), on the
    README scene with server.go's glass sphere and a mirror: device vs oracle
    bit-exact (the device folds the linear recursion in the reference's order)."""
    sc = readme_glass_scene(mirror=True)
    rd = abi.render_desc(3, 3, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, dl_strategy=strategy,
                         max_depth=depth, mode=mode)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    # round 4: the recursion runs per sample on k_dl_samples<kX> (its chain of
    # levels, hence the draw count, is the pixel's); the serial kernel too
    for kernel, want in (("auto", abi.PBRT_KERNEL_WAVE_DL), ("serial", abi.PBRT_KERNEL_SERIAL)):
        with G.Renderer(sc, kernel=kernel) as r:
            film, st = r.render(rd)
        assert st.kernel == want
        assert np.array_equal(bits(film), bits(of)), kernel
        assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays), kernel


@pytest.mark.gpu
def test_device_direct_lighting_through_glass_depth_limit():
    """The device keeps at most 32 recursion levels: maxDepth > 64 through glass is
    refused (PBRT_E_UNSUPPORTED), never truncated."""
    sc = readme_glass_scene()
    with G.Renderer(sc) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, max_depth=65))
    assert ei.value.code == abi.PBRT_E_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("material", ["glass", "mirror", "oren"])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
def test_device_mesh_with_specular_material_vs_oracle(monkeypatch, material, mode):
    """A triangle mesh of Glass / Mirror / OrenNayar: the kX chain and the kX
    path wavefront (k_pw_*, the path stage of mesh scenes), unsorted and
    material-sorted, and the serial kernel, all bit-exact against the oracle,
    which resolves the mesh's material the same way (oracle_render.c)."""
    sc = mesh_material_scene(material)
    rd = abi.render_desc(3, 3, max_depth=6, mode=mode)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0 and np.isfinite(of).all()
    for sort in ("0", "1"):
        monkeypatch.setenv("PBRT_PW_SORT", sort)
        with G.Renderer(sc) as r:
            film, st = r.render(rd)
        assert st.kernel == path_kernel(4, mode)
        assert np.array_equal(bits(film), bits(of))
    with G.Renderer(sc, kernel="serial") as r:
        film, st = r.render(rd)
    assert st.kernel == abi.PBRT_KERNEL_SERIAL
    assert np.array_equal(bits(film), bits(of))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("sort", ["0", "1"])
def test_device_glass_scene_on_the_path_wavefront(monkeypatch, mode, sort):
    """The README + glass + mirror scene with the path stage forced onto the kX
    path wavefront (PBRT_PATHS_WF=1), unsorted and sorted by material between
    trace and shade: bit-exact against the oracle."""
    monkeypatch.setenv("PBRT_PATHS_WF", "1")
    monkeypatch.setenv("PBRT_PW_SORT", sort)
    sc = readme_glass_scene(mirror=True)
    rd = abi.render_desc(3, 3, mode=mode)
    rc, of, _ = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    assert st.kernel == path_kernel(4, mode)
    assert np.array_equal(bits(film), bits(of))


def test_oracle_mesh_material_changes_the_image():
    """The mesh's material is honoured by the oracle: a glass or mirror mesh
    renders differently from an OrenNayar one."""
    rd = abi.render_desc(2, 2, max_depth=5)
    films = {}
    for m in ("glass", "mirror", "oren"):
        sc = mesh_material_scene(m)
        rc, films[m], _ = O.render(sc.desc, rd, threads=8)
        assert rc == 0
    assert not np.array_equal(films["glass"], films["mirror"])
    assert not np.array_equal(films["glass"], films["oren"])


@pytest.mark.gpu
@pytest.mark.parametrize("ci_waves", ["1", "2", "4"])
@pytest.mark.parametrize("nd,depth,rr", [(4, 10, 1.0), (6, 24, 1.0), (10, 32, 0.7), (3, 16, 1.0)])
def test_device_glass_rr_on_stratified_dims_vs_oracle(monkeypatch, ci_waves, nd, depth, rr):
    """Russian roulette after >= 3 glass bounces reads stratified 1D values (a
    glass bounce samples no light): speculative trajectories record up to three
    such decisions and the chain head resolves them with its sample index; a
    fourth falls back to a re-run at the head. Deep paths through the glass
    sphere and 3 to 10 sampled dims cover the recorded, exhausted and mixed
    cases, at every ring size (waves per tile)."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    sc = readme_glass_scene(64, 48)
    rd = abi.render_desc(4, 4, n_dims=nd, max_depth=depth, rr_threshold=rr)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    assert rc == 0
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
        film2, _ = r.render(rd)   # the measured tile order
    assert st.kernel == abi.PBRT_KERNEL_WAVE_CI and st.paths_traced == ost.paths
    assert np.array_equal(bits(film), bits(of)) and np.array_equal(bits(film2), bits(of))
    assert (st.rays_closest, st.rays_shadow) == (ost.closest_rays, ost.shadow_rays)
