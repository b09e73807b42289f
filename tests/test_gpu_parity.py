"""Parity of the HIP path (through the C ABI) with the CPU oracle.

Bar: bit-identical fp64 films (integer-exact comparison of the IEEE bits) for
every configuration the oracle finishes in seconds, plus the committed golden
fixtures; at full 1080p size, size-independent properties and a bit-exact
check of a sample of tiles.
"""
import ctypes as C
import hashlib
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


KERNELS = ["serial", "auto"]   # auto = the wave-parallel kernel wherever it is eligible


def gpu_render(scene, rd, lanes_per_wave=0, kernel="auto"):
    with G.Renderer(scene, lanes_per_wave=lanes_per_wave, kernel=kernel) as r:
        film, st = r.render(rd)
    if kernel == "serial":
        assert st.kernel == abi.PBRT_KERNEL_SERIAL
    elif kernel in ("wave", "wavefront"):   # requests of the window / wavefront chains run k_chain_ci
        assert st.kernel in (abi.PBRT_KERNEL_WAVE_CI, abi.PBRT_KERNEL_WAVE)
    elif kernel == "wave_ci":
        assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
    elif kernel == "wave_dl":
        assert st.kernel == abi.PBRT_KERNEL_WAVE_DL
    return film, st


def wave_eligible(rd):
    """Path renders whose camera ray is the pixel's (pFilm stratified: n_dims
    >= 1; the scenes here are pinholes, so pLens may be a draw)."""
    return (rd.integrator == abi.PBRT_INTEGRATOR_PATH and rd.n_dims >= 1
            and rd.light_strategy == abi.PBRT_LIGHT_STRATEGY_UNIFORM)


def dl_wave_eligible(rd):
    """DirectLighting on k_dl_*: the camera ray per pixel (the scenes here are pinhole)."""
    return rd.integrator == abi.PBRT_INTEGRATOR_DIRECT_LIGHTING and rd.n_dims >= 1


def oracle_render(scene, rd):
    rc, film, st = O.render(scene.desc, rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0
    return film, st


def check(scene, rd, **kw):
    film, st = gpu_render(scene, rd, **kw)
    if kw.get("kernel", "auto") == "auto":
        want = (abi.PBRT_KERNEL_WAVE, abi.PBRT_KERNEL_WAVE_CI) if wave_eligible(rd) else \
            (abi.PBRT_KERNEL_WAVE_DL,) if dl_wave_eligible(rd) else (abi.PBRT_KERNEL_SERIAL,)
        assert st.kernel in want
    ofilm, ost = oracle_render(scene, rd)
    assert st.paths_traced == ost.paths
    assert same_bits(film, ofilm), f"{int((film != ofilm).sum())} film values differ"
    return film, st


# ----------------------------------------------------------- device math KATs
def probe(op, inp, out_stride=1):
    inp = np.ascontiguousarray(inp, dtype=np.float64)
    if inp.ndim == 1:
        inp = inp[:, None]
    out = np.zeros((inp.shape[0], out_stride))
    rc = G.lib().pbrt_gpu_probe(-1, op, inp.ctypes.data_as(C.POINTER(C.c_double)), inp.shape[0], inp.shape[1],
                                out.ctypes.data_as(C.POINTER(C.c_double)), out_stride)
    assert rc == 0
    return out


def setup_module(module):
    G.lib().pbrt_gpu_probe.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_int,
                                       C.POINTER(C.c_double), C.c_int]


def test_device_go_cos_golden():
    """transform_test.go:80 on the device: Cos(Pi/180*90) == 6.123233995736757e-17."""
    out = probe(abi.PBRT_PROBE_COS if hasattr(abi, "PBRT_PROBE_COS") else 2, np.array([math.pi / 180.0 * 90]))
    assert out[0, 0] == 6.123233995736757e-17


def test_device_trig_matches_oracle():
    """Go-math trig on the device equals the oracle bit for bit on 2e5 inputs per
    function over the ranges the hot path uses (phi, theta, concentric-disk angles)."""
    rng = np.random.default_rng(1)
    L = O.lib()
    n = 200_000
    xs = np.concatenate([rng.uniform(-7, 7, n // 2), rng.uniform(-1, 1, n // 4), rng.uniform(-1e3, 1e3, n // 4)])
    for op, f in ((1, L.oracle_go_sin), (2, L.oracle_go_cos), (4, L.oracle_go_atan)):
        got = probe(op, xs)[:, 0]
        want = np.array([f(x) for x in xs])
        assert same_bits(got, want), op
    u = rng.uniform(-1, 1, n)
    for op, f in ((6, L.oracle_go_asin), (7, L.oracle_go_acos)):
        got = probe(op, u)[:, 0]
        want = np.array([f(x) for x in u])
        assert same_bits(got, want), op
    yx = rng.normal(size=(n, 2)) * rng.choice([1e-3, 1, 1e3], size=(n, 1))
    got = probe(5, yx)[:, 0]
    want = np.array([L.oracle_go_atan2(y, x) for y, x in yx])
    assert same_bits(got, want)


def special_values(n, seed):
    rng = np.random.default_rng(seed)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
                   1.0, -1.0, 2.0 ** 53, -(2.0 ** 53), 2.0 ** 53 - 1, 2.0 ** 60, 1.7976931348623157e308,
                   -1.7976931348623157e308, 0.5, 1e-300, -1e-300])
    rnd = rng.standard_normal(n) * 10.0 ** rng.integers(-320, 300, n)
    return np.concatenate([sp, rnd])


def test_device_next_float_up_down_and_go_max_min_special_values():
    """Branch-free device forms of NextFloatUp/Down (pkg/math/math.go:122-128 =
    math.Nextafter(v, v±1)) and Go math.Max/Min: bit-identical to the oracle's
    Go restatement on ±0, ±Inf, NaN, denormals, |v| >= 2^53 and random values."""
    L = O.lib()
    v = special_values(4000, 11)
    up = probe(18, v)[:, 0]
    dn = probe(19, v)[:, 0]
    want_up = np.array([L.oracle_go_nextafter(x, x + 1) for x in v])
    want_dn = np.array([L.oracle_go_nextafter(x, x - 1) for x in v])
    assert same_bits(up, want_up) and same_bits(dn, want_dn)
    a = np.repeat(v[:60], 60)
    b = np.tile(v[:60], 60)
    pairs = np.stack([np.concatenate([a, v]), np.concatenate([b, v[::-1]])], axis=1)
    mx = probe(11, pairs)[:, 0]
    mn = probe(12, pairs)[:, 0]
    assert same_bits(mx, np.array([L.oracle_go_max(x, y) for x, y in pairs]))
    assert same_bits(mn, np.array([L.oracle_go_min(x, y) for x, y in pairs]))


def test_device_nonan_min_max_order_signed_zeros_like_go():
    """The device min/max used inside EFloat.Mul (v_min_f64 / v_max_f64) equal
    Go's Min/Max on every non-NaN pair, incl. -0 vs +0 and infinities."""
    L = O.lib()
    v = special_values(3000, 12)
    v = v[~np.isnan(v)]
    a = np.concatenate([np.repeat(v[:40], 40), v, [0.0, -0.0, 0.0, -0.0]])
    b = np.concatenate([np.tile(v[:40], 40), v[::-1], [-0.0, 0.0, 0.0, -0.0]])
    pairs = np.stack([a, b], axis=1)
    assert same_bits(probe(20, pairs)[:, 0], np.array([L.oracle_go_min(x, y) for x, y in pairs]))
    assert same_bits(probe(21, pairs)[:, 0], np.array([L.oracle_go_max(x, y) for x, y in pairs]))


@pytest.mark.parametrize("op,name", [(22, "oracle_efloat_mul"), (23, "oracle_efloat_div")])
def test_device_efloat_mul_div_match_oracle(op, name):
    """EFloat Mul / Div (efloat.go) incl. Check() panics, on random, signed-zero,
    straddling-zero and overflowing intervals."""
    rng = np.random.default_rng(op)
    n = 20000
    v1 = rng.standard_normal(n) * 10.0 ** rng.integers(-200, 200, n)
    v2 = rng.standard_normal(n) * 10.0 ** rng.integers(-200, 200, n)
    e1 = np.abs(v1) * 10.0 ** rng.integers(-17, 1, n) * (rng.uniform(size=n) < 0.8)
    e2 = np.abs(v2) * 10.0 ** rng.integers(-17, 1, n) * (rng.uniform(size=n) < 0.8)
    sp = np.array([0.0, -0.0, 1.0, -1.0, 5e-324, 1e308, -1e308])
    k = len(sp)
    with np.errstate(over="ignore"):
        extra = np.array([[x, 0.0, y, 0.0] for x in sp for y in sp] +
                         [[x, abs(x) * 2, y, 0.0] for x in sp for y in sp])
    inp = np.concatenate([np.stack([v1, e1, v2, e2], axis=1), extra])
    got = probe(op, inp, 4)
    fn = getattr(O.lib(), name)
    for i, (a, ea, b, eb) in enumerate(inp):
        out = (C.c_double * 3)()
        pan = fn(a, ea, b, eb, out)
        if pan:
            assert got[i, 3] != 0, (i, inp[i])
        else:
            assert got[i, 3] == 0, (i, inp[i])
            assert same_bits(got[i, :3], np.array(list(out))), (i, inp[i], got[i], list(out))


def test_device_div_sqrt_correctly_rounded():
    """gfx950 fp64 '/' and sqrt must be correctly rounded (SURVEY §9 'verify on
    gfx950'): 2e6 random operands incl. denormals vs the host (IEEE)."""
    rng = np.random.default_rng(2)
    n = 1_000_000
    a = rng.normal(size=n) * np.exp2(rng.integers(-1070, 1000, n))
    b = rng.normal(size=n) * np.exp2(rng.integers(-60, 60, n))
    got = probe(9, np.stack([a, b], 1))[:, 0]
    with np.errstate(over="ignore", under="ignore"):
        assert same_bits(got, a / b)
    s = np.abs(rng.normal(size=n)) * np.exp2(rng.integers(-1074, 1000, n))
    got = probe(8, s)[:, 0]
    assert same_bits(got, np.sqrt(s))


def test_device_offset_ray_origin_golden():
    """ray_test.go:10-19 on the device (fp64 denormals preserved)."""
    eps = 5e-324
    out = probe(13, np.array([[0, 0, 0, eps, eps, eps, 1, 1, 1, 1, 1, 1]]), 3)
    assert list(out[0]) == [1.5183e-320] * 3


def test_device_efloat_add_golden():
    """efloat_test.go:9-13 on the device."""
    out = probe(14, np.array([[1.0, 0.0, 1.0, 0.0]]), 4)
    assert list(out[0]) == [2.0, 1.9999999999999998, 2.0000000000000004, 0.0]


def test_device_transform_ray_golden():
    """transform_test.go:77-81 on the device."""
    x = G.mul(G.rotate(1, 90), G.translate(5, 4, 3))
    m = [x.m.m[i][j] for i in range(4) for j in range(4)]
    out = probe(15, np.array([m + [0, 0, 0, 1, 0, 0]]), 6)
    assert list(out[0]) == [3.0000000000000004, 4, -5, 6.123233995736757e-17, 0, -1]


def test_device_visibility_tester_golden():
    """light_test.go:10-44 on the device."""
    out = probe(16, np.array([[0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 0, 0, 0, 0, 0, 0, 0, 0]]), 7)
    assert list(out[0]) == [0, 0, 0, 10, 0, 0, 0.9999]


def test_device_pcg_matches_golden():
    gold = GOLDEN["pcg32_first16"]
    L = O.lib()
    for seed in (0, 1, 8159):
        buf = (C.c_double * 16)()
        L.oracle_pcg_floats(seed, 16, buf)
        out = probe(17, np.array([float(seed)]), 16)
        assert same_bits(out[0], np.array(list(buf)))
        # and the oracle floats derive from the committed u32 golden stream
        assert list(buf) == [min(0.9999999999999999, u * 2.3283064365386963e-10) for u in gold[str(seed)]]


# ---------------------------------------------------------------- film parity
@pytest.mark.parametrize("kernel", KERNELS + ["wavefront", "wave_ci"])
@pytest.mark.parametrize("name", sorted(GOLDEN["cases"]))
def test_golden_fixtures(name, kernel):
    case = GOLDEN["cases"][name]
    w, h = case["w"], case["h"]
    scene = G.Scene.readme(w, h) if case["scene"] == "readme" else G.Scene.cornell(w, h)
    rd = abi.render_desc(**case["render"])
    if kernel in ("wavefront", "wave_ci") and not wave_eligible(rd):
        if dl_wave_eligible(rd):
            kernel = "wave_dl"   # DirectLighting's wave kernels instead of the path chain
        else:
            pytest.skip("not eligible for the wave-parallel kernels")
    film, st = gpu_render(scene, rd, kernel=kernel)
    gold = np.load(os.path.join(HERE, "golden", name + ".npz"))["film"]
    assert same_bits(film, gold)
    assert hashlib.sha256(film.tobytes()).hexdigest() == case["sha256"]
    assert st.paths_traced == case["paths"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_readme_256_path_bitexact(kernel):
    check(G.Scene.readme(256, 256), abi.render_desc(2, 2), kernel=kernel)


def test_config_A_traces_nothing():
    """Config A: Stratified(1,1) traces 0 paths (sampler.go:29-34): all-zero film."""
    film, st = gpu_render(G.Scene.readme(256, 256),
                          abi.render_desc(1, 1, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING))
    assert st.paths_traced == 0 and st.tiles_rendered == 256
    assert not film.any()


@pytest.mark.parametrize("kernel", KERNELS)
def test_config_A_prime_direct_lighting(kernel):
    check(G.Scene.readme(256, 256), abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING),
          kernel=kernel)


@pytest.mark.parametrize("kernel", KERNELS)
def test_direct_lighting_sample_one(kernel):
    check(G.Scene.readme(64, 64), abi.render_desc(2, 2, integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING,
                                                  dl_strategy=abi.PBRT_DL_UNIFORM_SAMPLE_ONE), kernel=kernel)


DL = abi.PBRT_INTEGRATOR_DIRECT_LIGHTING


@pytest.mark.parametrize("kw", [
    dict(spp_x=8, spp_y=8),
    dict(spp_x=5, spp_y=3, jitter=True),
    dict(spp_x=4, spp_y=4, n_dims=1),
    dict(spp_x=4, spp_y=4, n_dims=2),
    dict(spp_x=4, spp_y=4, n_dims=7),
    dict(spp_x=4, spp_y=4, max_depth=1),
    dict(spp_x=4, spp_y=4, dl_strategy=abi.PBRT_DL_UNIFORM_SAMPLE_ONE, n_dims=2),
    dict(spp_x=3, spp_y=3, tile_size=13),
    dict(spp_x=3, spp_y=3, tile_begin=2, tile_stride=3),
    dict(spp_x=24, spp_y=24, max_depth=3),
    dict(spp_x=4, spp_y=4, mode=abi.PBRT_MODE_THROUGHPUT),
    dict(spp_x=4, spp_y=4, mode=abi.PBRT_MODE_THROUGHPUT, dl_strategy=abi.PBRT_DL_UNIFORM_SAMPLE_ONE),
])
@pytest.mark.parametrize("scene", ["readme", "cornell"])
def test_direct_lighting_wave_kernel_bitexact(scene, kw):
    """DirectLighting on k_dl_setup + k_dl_samples (pixel-order StartPixel and
    jump-ahead, then one lane per sample): bit for bit the oracle's serial
    replay, in both modes, both strategies and every sampler shape it takes."""
    sc = G.Scene.readme(72, 40) if scene == "readme" else G.Scene.cornell(72, 40)
    rd = abi.render_desc(integrator=DL, **kw)
    film, st = check(sc, rd, kernel="wave_dl")
    assert st.kernel == abi.PBRT_KERNEL_WAVE_DL
    if rd.sampler_x * rd.sampler_y > 1:
        assert film.max() > 0


def test_direct_lighting_wave_kernel_n_dims_0_falls_back_to_serial():
    """n_dims = 0: pFilm comes from the RNG, so the camera ray is per sample."""
    rd = abi.render_desc(3, 3, integrator=DL, n_dims=0)
    film, st = check(G.Scene.readme(40, 24), rd)
    assert st.kernel == abi.PBRT_KERNEL_SERIAL
    with G.Renderer(G.Scene.readme(40, 24), kernel="wave_dl") as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    assert ei.value.code == abi.PBRT_E_UNSUPPORTED


def test_direct_lighting_wave_kernel_1080p_64spp_vs_oracle():
    """Config B's frame under DirectLighting (UniformSampleAll): the whole
    1080p / 64 spp film bit for bit."""
    scene = G.Scene.readme(1920, 1080)
    check(scene, abi.render_desc(8, 8, integrator=DL), kernel="wave_dl")


@pytest.mark.parametrize("kw", [
    dict(spp_x=4, spp_y=4),
    dict(spp_x=3, spp_y=5, jitter=True),
    dict(spp_x=2, spp_y=2, n_dims=0),
    dict(spp_x=2, spp_y=2, n_dims=7),
    dict(spp_x=2, spp_y=2, max_depth=1),
    dict(spp_x=2, spp_y=2, max_depth=2),
    dict(spp_x=2, spp_y=2, max_depth=5, rr_threshold=0.0),
    dict(spp_x=2, spp_y=2, rr_threshold=1e9),
    dict(spp_x=2, spp_y=2, light_strategy=abi.PBRT_LIGHT_STRATEGY_POWER),
    dict(spp_x=2, spp_y=2, tile_size=8),
    dict(spp_x=2, spp_y=2, tile_size=13),
])
@pytest.mark.parametrize("kernel", KERNELS)
def test_readme_variants_bitexact(kw, kernel):
    check(G.Scene.readme(72, 40), abi.render_desc(**kw), kernel=kernel)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("w,h", [(1, 1), (17, 3), (37, 23), (16, 16)])
def test_ragged_images(w, h, kernel):
    check(G.Scene.readme(w, h), abi.render_desc(3, 3), kernel=kernel)


WAVE_VARIANTS = [
    dict(spp_x=9, spp_y=9),                      # 80 traced samples: two 64-lane batches
    dict(spp_x=8, spp_y=8, n_dims=3),            # bounce-1 uScattering from the RNG
    dict(spp_x=5, spp_y=5, n_dims=5),            # bounce-1 BSDF sample stratified (0,0)
    dict(spp_x=4, spp_y=6, jitter=True),
    dict(spp_x=6, spp_y=6, flags=abi.PBRT_FLAG_SERIAL_START_PIXEL),
    dict(spp_x=4, spp_y=4, max_depth=3),
    dict(spp_x=4, spp_y=4, max_depth=12, rr_threshold=0.0),
    dict(spp_x=4, spp_y=4, max_depth=2),
    dict(spp_x=8, spp_y=8, n_dims=2),            # bounce-1 light sample from the RNG (per sample)
    dict(spp_x=6, spp_y=5, n_dims=1, jitter=True),   # pLens from the RNG too (a pinhole: same ray)
]


@pytest.mark.parametrize("kw", WAVE_VARIANTS)
@pytest.mark.parametrize("kernel", ["wave", "wave_ci"])
def test_wave_kernel_variants(kw, kernel):
    check(G.Scene.readme(48, 40), abi.render_desc(**kw), kernel=kernel)


def test_wavefront_cornell_64spp_and_readme_256():
    check(G.Scene.cornell(32, 32), abi.render_desc(8, 8, max_depth=10), kernel="wavefront")
    check(G.Scene.readme(256, 256), abi.render_desc(2, 2), kernel="wavefront")
    check(G.Scene.readme(112, 80), abi.render_desc(4, 4), kernel="wavefront")


def test_wavefront_panic_is_reported_like_the_oracle():
    scene = panic_scene()
    rd = abi.render_desc(2, 2)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    assert rc == abi.PBRT_E_REF_PANIC
    with G.Renderer(scene, kernel="wavefront") as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert ei.value.code == abi.PBRT_E_REF_PANIC and st.kernel == abi.PBRT_KERNEL_WAVE_CI
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


@pytest.mark.parametrize("tiles_per_wave", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("kernel", ["wave", "wave_ci"])
def test_wave_kernel_tiles_per_wave(tiles_per_wave, kernel):
    """k_chain_ci packs up to 4 tiles per wave (64 / L lanes each; larger
    requests run one tile per wave); 37 tiles leave partial last waves."""
    check(G.Scene.readme(112, 80), abi.render_desc(4, 4), kernel=kernel, lanes_per_wave=tiles_per_wave)


@pytest.mark.parametrize("kernel", ["wave", "wave_ci"])
def test_wave_kernel_cornell_64spp(kernel):
    check(G.Scene.cornell(32, 32), abi.render_desc(8, 8, max_depth=10), kernel=kernel)


@pytest.mark.parametrize("tiles_per_wave", [1, 4])
def test_wave_ci_readme_256_and_odd_draw_counts(tiles_per_wave):
    """Continuous-issue chain on larger frames: D is odd for ~1% of paths
    (no RR draw), which flips the chain's offset parity mid-pixel."""
    check(G.Scene.readme(256, 256), abi.render_desc(2, 2), kernel="wave_ci", lanes_per_wave=tiles_per_wave)
    check(G.Scene.readme(112, 80), abi.render_desc(8, 8), kernel="wave_ci", lanes_per_wave=tiles_per_wave)
    check(G.Scene.cornell(48, 32), abi.render_desc(6, 6, max_depth=12, rr_threshold=0.5), kernel="wave_ci",
          lanes_per_wave=tiles_per_wave)


@pytest.mark.parametrize("ci_waves", ["1", "2", "4", "8"])
@pytest.mark.parametrize("kw", WAVE_VARIANTS)
def test_wave_ci_waves_per_tile(kw, ci_waves, monkeypatch):
    """k_chain_ci with 1, 2 or 4 waves cooperating on one tile's chain
    (idle lanes ranked across waves, StartPixel on the first wave)."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    check(G.Scene.readme(48, 40), abi.render_desc(**kw), kernel="wave_ci")


@pytest.mark.parametrize("ci_waves", ["1", "4"])
def test_wave_ci_stride_1_keeps_bits(ci_waves, monkeypatch):
    """PBRT_CI_STRIDE=1: chain candidates at every offset (both parities), so
    an odd draw count drops nothing; only the schedule changes."""
    monkeypatch.setenv("PBRT_CI_STRIDE", "1")
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    check(G.Scene.readme(112, 80), abi.render_desc(8, 8), kernel="wave_ci")
    check(G.Scene.readme(48, 40), abi.render_desc(4, 4, jitter=True), kernel="wave_ci")
    check(G.Scene.cornell(48, 32), abi.render_desc(6, 6, max_depth=12, rr_threshold=0.5), kernel="wave_ci")


@pytest.mark.parametrize("ci_waves", ["1", "2", "4", "8"])
def test_wave_ci_waves_per_tile_larger_frames(ci_waves, monkeypatch):
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    check(G.Scene.readme(112, 80), abi.render_desc(8, 8), kernel="wave_ci")
    check(G.Scene.cornell(48, 32), abi.render_desc(6, 6, max_depth=12, rr_threshold=0.5), kernel="wave_ci")


@pytest.mark.parametrize("ci_waves", ["1", "2", "4", "8"])
def test_wave_ci_heaviest_first_schedule_keeps_bits(ci_waves, monkeypatch):
    """The second frame of a configuration launches its tiles in the
    heaviest-first order measured on the first; only the schedule changes."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    scene = G.Scene.readme(112, 80)
    rds = [abi.render_desc(8, 8), abi.render_desc(4, 4, tile_begin=1, tile_stride=2)]
    with G.Renderer(scene, kernel="wave_ci") as r:
        for rd in rds:
            ofilm, _ = oracle_render(scene, rd)
            for _ in range(3):
                film, st = r.render(rd)
                assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
                assert same_bits(film, ofilm)


@pytest.mark.parametrize("heavy", ["3", "12"])
@pytest.mark.parametrize("ci_waves", ["2", "4", "8"])
def test_wave_ci_heavy_light_split_keeps_bits(ci_waves, heavy, monkeypatch):
    heavy_env = heavy
    """Shard mode: from the second frame the heaviest tiles run at 4 waves in
    one launch and the rest at 1 wave in a concurrent launch on a second
    stream; only the schedule changes."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    monkeypatch.setenv("PBRT_CI_HEAVY", heavy)
    if ci_waves == "8":   # heavy tiles at 8 waves (PBRT_CI_HEAVY_WAVES)
        monkeypatch.setenv("PBRT_CI_HEAVY_WAVES", "8")
    scene = G.Scene.readme(112, 80)
    rds = [abi.render_desc(8, 8), abi.render_desc(4, 4, tile_begin=1, tile_stride=2),
           abi.render_desc(6, 6, max_depth=12, rr_threshold=0.5)]
    with G.Renderer(scene, kernel="wave_ci") as r:
        for rd in rds:
            ofilm, _ = oracle_render(scene, rd)
            for frame in range(3):
                film, st = r.render(rd)
                assert st.kernel == abi.PBRT_KERNEL_WAVE_CI
                assert same_bits(film, ofilm)
                ticks, heavy = r.tile_ticks()
                assert len(ticks) == st.tiles_rendered and ticks.min() > 0
                # the split runs from the second frame on (the first has no schedule yet)
                assert (heavy > 0) == (frame > 0 and int(heavy_env) < st.tiles_rendered), (frame, heavy)


@pytest.mark.parametrize("probe", ["0", "1"])
def test_wave_ci_cold_frame_probe_order_keeps_bits(probe, monkeypatch):
    """A fresh context's first frame launches its tiles in the order of the
    k_tile_cost estimate (no measured chain times yet); later frames use the
    measured order. Only the schedule changes: every frame is the oracle's."""
    monkeypatch.setenv("PBRT_CI_PROBE", probe)
    scene = G.Scene.readme(160, 96)
    rd = abi.render_desc(5, 5)
    ofilm, _ = oracle_render(scene, rd)
    with G.Renderer(scene, kernel="wave_ci") as r:
        for frame in range(2):
            film, st = r.render(rd)
            assert same_bits(film, ofilm)
            costs = r.tile_costs()
            if frame == 0 and probe == "1":
                assert costs.shape == (st.tiles_rendered, 4)
                assert (costs[:, 3] > 0).all() and (costs[:, 2] == 256).all()
                assert costs[:, 1].sum() > 0   # hit pixels were probed
            else:
                assert len(costs) == 0


def test_wave_ci_split_default_heuristic_on_a_quarter_shard():
    """Without PBRT_CI_HEAVY: a 1/4 shard of the 1080p frame (2040 tiles, 4
    waves per tile) gets the heavy/light split from its second frame; bits
    stay the oracle's."""
    scene = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(2, 2, tile_begin=1, tile_stride=4)
    ofilm, _ = oracle_render(scene, rd)
    with G.Renderer(scene) as r:
        for frame in range(3):
            film, st = r.render(rd)
            assert st.kernel == abi.PBRT_KERNEL_WAVE_CI and st.tiles_rendered == 2040
            assert same_bits(film, ofilm)
            _, heavy = r.tile_ticks()
            assert (heavy > 0) == (frame > 0), (frame, heavy)


@pytest.mark.parametrize("ci_waves", ["1", "4"])
def test_wave_ci_panic_is_reported_like_the_oracle(ci_waves, monkeypatch):
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    scene = panic_scene()
    rd = abi.render_desc(2, 2)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    assert rc == abi.PBRT_E_REF_PANIC
    with G.Renderer(scene, kernel="wave_ci") as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert ei.value.code == abi.PBRT_E_REF_PANIC and st.kernel == abi.PBRT_KERNEL_WAVE_CI
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


def test_wave_kernel_rejects_ineligible_render():
    with G.Renderer(G.Scene.readme(16, 16), kernel="wave") as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(abi.render_desc(2, 2, n_dims=0))
    assert ei.value.code == abi.PBRT_E_UNSUPPORTED


@pytest.mark.parametrize("lpw", [1, 4, 16, 64])
def test_lanes_per_wave_invariant(lpw):
    check(G.Scene.readme(96, 48), abi.render_desc(2, 2), lanes_per_wave=lpw)


@pytest.mark.parametrize("kernel", KERNELS)
def test_cornell_bitexact(kernel):
    check(G.Scene.cornell(64, 48), abi.render_desc(3, 3, max_depth=8), kernel=kernel)


def test_tile_shards_sum_to_full_frame():
    """Multi-GPU sharding (tile t -> rank t mod N): the sum of the shard films
    equals the single-device film; only pixels covered by tiles of different
    shards can differ, and then only by float association order."""
    scene = G.Scene.readme(80, 48)
    full, _ = gpu_render(scene, abi.render_desc(2, 2))
    for n in (2, 3):
        parts = [gpu_render(scene, abi.render_desc(2, 2, tile_begin=r, tile_stride=n))[0] for r in range(n)]
        acc = np.zeros_like(full)
        for p in parts:
            acc += p
        np.testing.assert_allclose(acc, full, rtol=1e-14, atol=0)
        # each shard equals the oracle's render of the same shard, bit for bit
        for r in range(n):
            ofilm, _ = oracle_render(scene, abi.render_desc(2, 2, tile_begin=r, tile_stride=n))
            assert same_bits(parts[r], ofilm)


def test_tile_range_subset():
    scene = G.Scene.readme(64, 64)
    rd = abi.render_desc(2, 2, tile_begin=3, tile_end=11, tile_stride=1)
    film, st = gpu_render(scene, rd)
    assert st.tiles_rendered == 8
    ofilm, _ = oracle_render(scene, rd)
    assert same_bits(film, ofilm)


# --------------------------------------------------------- batch intersection
def random_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-60, 140, size=(n, 3))
    o[:, 1] = rng.uniform(-5, 120, size=n)
    d = rng.normal(size=(n, 3))
    tmax = np.where(rng.uniform(size=n) < 0.2, rng.uniform(1, 200, size=n), np.inf)
    return np.concatenate([o, d, tmax[:, None]], axis=1)


def test_intersect_matches_oracle():
    """Aggregate.Intersect/IntersectP (bvh.go:659-765) on 2e4 random rays, bit-exact
    hit flags, hit prim, TMax, point and normal."""
    scene = G.Scene.readme(64, 64)
    rays = random_rays(20_000, 3)
    with G.Renderer(scene) as r:
        rc, got = r.intersect(rays)
        rc_p, occ = r.intersect_p(rays)
    assert rc == 0 and rc_p == 0
    want = O.intersect(scene.desc, rays, closest=True)
    wocc = O.intersect(scene.desc, rays, closest=False)
    assert same_bits(got, want)
    assert np.array_equal(occ.astype(bool), wocc.astype(bool))
    assert 0.2 < got[:, 0].mean() < 0.95   # the sample exercises hits and misses


# ------------------------------------------------------------ reference panics
def panic_scene():
    """A point light so bright that EstimateDirect returns > 10 on the first
    lit hit: UniformSampleOneLight panics (integrator.go:73-75)."""
    s = G.Scene()
    chk = s.add_matte((0.8, 0.8, 0.8))
    t = G.mul(G.translate(0, 0, 0), G.rotate(0, 90))
    d = s.add_disk(t, 0.0, 100.0)
    s.add_primitive(d, chk)
    s.add_point_light(G.translate(0, 5, 0), (1e5, 1e5, 1e5))
    s.set_film(32, 32)
    s.set_camera(G.look_at((0, 20, 20), (0, 0, 0), (0, 1, 0)), fov=60)
    return s.build()


@pytest.mark.parametrize("kernel", KERNELS)
def test_reference_panic_is_reported_like_the_oracle(kernel):
    scene = panic_scene()
    rd = abi.render_desc(2, 2)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    assert rc == abi.PBRT_E_REF_PANIC and ost.panic_kind == abi.PBRT_PANIC_LD_GT_10
    with G.Renderer(scene, kernel=kernel) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert ei.value.code == abi.PBRT_E_REF_PANIC
    assert st.panic_kind == abi.PBRT_PANIC_LD_GT_10
    assert (st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


# ------------------------------------------------------------ full-size (1080p)
@pytest.mark.slow
def test_1080p_64spp_properties_and_sampled_tiles():
    """BASELINE config B at full size: 8160 tiles, W*H*63 paths, finite film;
    a sample of tiles is re-rendered by the oracle and must match bit for bit."""
    scene = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(8, 8)
    with G.Renderer(scene) as r:
        film, st = r.render(rd)
    assert st.tiles_rendered == 8160
    assert st.paths_traced == 1920 * 1080 * 63
    assert np.isfinite(film).all()
    # tiles 0, 4080, 8159 (first, middle, last) alone, oracle vs GPU
    for t in (0, 4080, 8159):
        one = abi.render_desc(8, 8, tile_begin=t, tile_end=t + 1)
        with G.Renderer(scene) as r:
            g, _ = r.render(one)
        o, _ = oracle_render(scene, one)
        assert same_bits(g, o), t


# ------------------------------------------------- THROUGHPUT mode (Mode B)
MB = abi.PBRT_MODE_THROUGHPUT
MB_CASES = [
    ("readme", 64, 48, dict(spp_x=2, spp_y=2)),
    ("readme", 112, 80, dict(spp_x=8, spp_y=8)),
    ("readme", 37, 23, dict(spp_x=3, spp_y=5, jitter=True)),
    ("readme", 48, 40, dict(spp_x=4, spp_y=4, n_dims=7, max_depth=12)),
    ("readme", 48, 40, dict(spp_x=4, spp_y=4, tile_size=13, rr_threshold=0.5)),
    ("cornell", 48, 32, dict(spp_x=6, spp_y=6, max_depth=8)),
]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("case", MB_CASES, ids=lambda c: f"{c[0]}{c[1]}x{c[2]}-{c[3]}")
def test_throughput_mode_bitexact_vs_oracle(case, kernel):
    """Mode B on both device paths (serial lane-per-tile replay with reseeding,
    and the chain-free wave-per-pixel k_paths<true>) equals the oracle's Mode B
    restatement bit for bit."""
    name, w, h, kw = case
    scene = G.Scene.readme(w, h) if name == "readme" else G.Scene.cornell(w, h)
    check(scene, abi.render_desc(**kw, mode=MB), kernel=kernel)


@pytest.mark.parametrize("kw", [dict(n_dims=0), dict(integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, n_dims=0),
                                dict(light_strategy=abi.PBRT_LIGHT_STRATEGY_POWER)])
def test_throughput_mode_serial_fallback(kw):
    """Renders the wave path cannot take run Mode B on the serial kernel."""
    check(G.Scene.readme(40, 24), abi.render_desc(3, 3, mode=MB, **kw))


@pytest.mark.parametrize("kernel", KERNELS)
def test_throughput_mode_panic_is_reported_like_the_oracle(kernel):
    scene = panic_scene()
    rd = abi.render_desc(2, 2, mode=MB)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    assert rc == abi.PBRT_E_REF_PANIC
    with G.Renderer(scene, kernel=kernel) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert ei.value.code == abi.PBRT_E_REF_PANIC
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


def test_throughput_mode_1080p_sampled_tiles_and_shards():
    """Config B size in Mode B: every path traced, finite film, sampled tiles
    bit-exact vs the oracle, and 3 interleaved shards sum to the frame's tiles."""
    scene = G.Scene.readme(1920, 1080)
    rd = abi.render_desc(8, 8, mode=MB)
    with G.Renderer(scene) as r:
        film, st = r.render(rd)
        assert st.tiles_rendered == 8160 and st.paths_traced == 1920 * 1080 * 63
        assert np.isfinite(film).all()
        for t in (0, 4321, 8159):
            g, _ = r.render(abi.render_desc(8, 8, tile_begin=t, tile_end=t + 1, mode=MB))
            o, _ = oracle_render(scene, abi.render_desc(8, 8, tile_begin=t, tile_end=t + 1, mode=MB))
            assert same_bits(g, o), t


# ------------------------------------------- config C sampler (256 spp) at small size
@pytest.mark.parametrize("ci_waves", ["1", "2", "4", "8"])
def test_cornell_256spp_wave_ci(ci_waves, monkeypatch):
    """Stratified(16,16) as config C: the continuous-issue chain with its
    StartPixel staging aliased on the offset ring (19 KB of LDS) and k_paths_ci
    at 2 pixels per wave; 1, 2 and 4 waves per tile."""
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    check(G.Scene.cornell(48, 32), abi.render_desc(16, 16, max_depth=8), kernel="wave_ci")


def test_cornell_256spp_wave_ci_tiles_per_wave():
    """Several tiles per wave (no staging/ring aliasing) at 256 spp."""
    check(G.Scene.cornell(64, 32), abi.render_desc(16, 16, max_depth=8), kernel="wave_ci", lanes_per_wave=4)


def test_cornell_256spp_throughput_mode():
    check(G.Scene.cornell(48, 32), abi.render_desc(16, 16, max_depth=8, mode=MB))


@pytest.mark.parametrize("cull", ["0", "1"])
def test_leaf_culling_groups_keep_bits(cull, monkeypatch):
    """The README tree's leaf culling groups (cull_groups in render.hip) only
    skip leaf tests that fail; with and without them the films are the
    oracle's (EXACT and THROUGHPUT)."""
    monkeypatch.setenv("PBRT_CULL_GROUPS", cull)
    scene = G.Scene.readme(96, 64)
    check(scene, abi.render_desc(4, 4))
    check(scene, abi.render_desc(3, 3, mode=MB))


@pytest.mark.parametrize("spp", [24, 32])
def test_wave_ci_large_spp_global_start_pixel_values(spp):
    """Stratified(24,24) / (32,32): StartPixel's draws exceed the wave kernel's
    LDS staging, so it runs serially and k_chain_ci writes the pixel's
    stratified values straight to their global record (config E's sampler).
    Several batches; bit for bit the oracle's."""
    scene = G.Scene.readme(40, 24)
    rd = abi.render_desc(spp, spp, max_depth=6)
    film, st = check(scene, rd, kernel="wave_ci")
    assert st.kernel == abi.PBRT_KERNEL_WAVE_CI


@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("kernel", ["serial", "wave_dl"])
def test_direct_lighting_panic_is_reported_like_the_oracle(kernel, mode):
    """DirectLighting with UniformSampleOne on the panic scene: Ld > 10
    (integrator.go:73-75); kind, tile, pixel, sample and bounce as the oracle's."""
    scene = panic_scene()
    rd = abi.render_desc(3, 3, integrator=DL, dl_strategy=abi.PBRT_DL_UNIFORM_SAMPLE_ONE, mode=mode)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    assert rc == abi.PBRT_E_REF_PANIC and ost.panic_kind == abi.PBRT_PANIC_LD_GT_10
    with G.Renderer(scene, kernel=kernel) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert ei.value.code == abi.PBRT_E_REF_PANIC
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)


PW_CASES = [
    ("readme", 96, 64, dict(spp_x=4, spp_y=4)),
    ("readme", 64, 48, dict(spp_x=3, spp_y=3, max_depth=12, rr_threshold=0.5)),
    ("readme", 40, 24, dict(spp_x=2, spp_y=2, max_depth=1)),
    ("readme", 48, 32, dict(spp_x=24, spp_y=24, max_depth=4)),
    ("cornell", 48, 32, dict(spp_x=4, spp_y=4, max_depth=8)),
    ("cornell", 32, 32, dict(spp_x=3, spp_y=3, light_strategy=abi.PBRT_LIGHT_STRATEGY_POWER)),
]


@pytest.mark.parametrize("sort", ["1", "0"])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("case", PW_CASES, ids=lambda c: f"{c[0]}{c[1]}x{c[2]}-{c[3]}")
def test_path_wavefront_bitexact(case, mode, sort, monkeypatch):
    """PBRT_PATHS_WF=1: the full paths as per-bounce compacted queues, sorted
    by material between trace and shade (PBRT_PW_SORT) -- bit for bit the
    oracle's film in both modes."""
    monkeypatch.setenv("PBRT_PATHS_WF", "1")
    monkeypatch.setenv("PBRT_PW_SORT", sort)
    name, w, h, kw = case
    scene = G.Scene.readme(w, h) if name == "readme" else G.Scene.cornell(w, h)
    check(scene, abi.render_desc(**kw, mode=mode))


@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
def test_path_wavefront_chunked_and_panics(mode, monkeypatch):
    """A path-record budget small enough to force several chunks; and the
    panic scene's report through the wavefront."""
    monkeypatch.setenv("PBRT_PATHS_WF", "1")
    monkeypatch.setenv("PBRT_PW_GB", "0.01")
    check(G.Scene.readme(80, 48), abi.render_desc(5, 5, mode=mode))
    scene = panic_scene()
    rd = abi.render_desc(2, 2, mode=mode)
    rc, _, ost = O.render(scene.desc, rd, threads=1)
    with G.Renderer(scene) as r:
        with pytest.raises(G.PbrtError) as ei:
            r.render(rd)
    st = ei.value.stats
    assert (st.panic_kind, st.panic_tile, st.panic_pixel_x, st.panic_pixel_y, st.panic_sample, st.panic_bounce) == (
        ost.panic_kind, ost.panic_tile, ost.panic_px, ost.panic_py, ost.panic_sample, ost.panic_bounce)



def many_spheres_scene(n, seed):
    """n Matte spheres scattered in front of the README camera: a BVH far
    beyond the 64 LDS-staged nodes, so k_chain_ci walks with the reference's
    [64] stack and the full paths run on the path wavefront."""
    rng = np.random.default_rng(seed)
    s = G.Scene()
    mats = [s.add_matte(tuple(rng.uniform(0.2, 0.9, 3))) for _ in range(3)]
    floor = s.add_disk(G.mul(G.translate(0, -1, 0), G.rotate(0, 90)), 0.0, 50.0)
    s.add_primitive(floor, mats[0])
    for i in range(n):
        c = (rng.uniform(-6, 6), rng.uniform(-0.5, 4), rng.uniform(-6, 6))
        sph = s.add_sphere(G.translate(*c), rng.uniform(0.2, 0.8), reverse=bool(i % 7 == 3))
        s.add_primitive(sph, mats[i % 3])
    s.add_point_light(G.translate(0, 8, 0), (40, 40, 40))
    s.add_distant_light(G.translate(0, 0, 0), (0.6, 0.6, 0.6), (1, 2, 1))
    s.set_film(64, 48)
    s.set_camera(G.look_at((0, 5, 14), (0, 0, 0), (0, 1, 0)), fov=50)
    return s.build()


@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("ci_waves", ["1", "4"])
def test_large_bvh_wave_pipeline_bitexact(mode, ci_waves, monkeypatch):
    monkeypatch.setenv("PBRT_CI_WAVES", ci_waves)
    scene = many_spheres_scene(90, 5)
    assert scene.desc.n_nodes > 64
    film, st = check(scene, abi.render_desc(3, 3, max_depth=6, mode=mode))
    assert st.kernel == (abi.PBRT_KERNEL_WAVE_CI if mode == abi.PBRT_MODE_EXACT else abi.PBRT_KERNEL_WAVE)
    assert film.max() > 0


def test_throughput_mode_statistical_equivalence_at_config_B():
    """THROUGHPUT (Mode B, the >= 6x scaling vehicle) is checked
    for statistical equivalence with EXACT on config B's frame (1080p, 64 spp):
    against a high-spp EXACT render (Stratified(16,16)) its clipped RMS error
    matches EXACT's own (same spp) within 10%, and its clipped mean / median
    sit inside the spread of EXACT renders with different tile seeds. The
    estimator is heavy-tailed (BSDF.SampleF returns the local wi, ledger #7),
    hence the clipped statistics."""
    scene = G.Scene.readme(1920, 1080)
    with G.Renderer(scene) as r:
        a16, _ = r.render(abi.render_desc(8, 8))
        a8, _ = r.render(abi.render_desc(8, 8, tile_size=8))
        b16, st = r.render(abi.render_desc(8, 8, mode=abi.PBRT_MODE_THROUGHPUT))
        ref, _ = r.render(abi.render_desc(16, 16))
    assert st.paths_traced == 1920 * 1080 * 63
    inner = (slice(1, -1), slice(1, -1))
    a16, a8, b16 = a16[inner], a8[inner], b16[inner]
    ref = ref[inner] * (63.0 / 255.0)   # film sums: scale the 255-path reference to 63 paths
    cap = np.percentile(ref, 95)
    clip = lambda x: np.clip(x, 0, cap)   # noqa: E731
    err_a = np.sqrt(np.mean((clip(a16) - clip(ref)) ** 2))
    err_b = np.sqrt(np.mean((clip(b16) - clip(ref)) ** 2))
    assert 0.9 < err_b / err_a < 1.1, (err_a, err_b)
    for stat in (np.median, lambda x: clip(x).mean()):
        sa16, sa8, sb = stat(a16), stat(a8), stat(b16)
        spread = abs(sa16 - sa8) + 0.002 * abs(sa16)
        assert abs(sb - 0.5 * (sa16 + sa8)) < 3 * spread, (sa16, sa8, sb)
