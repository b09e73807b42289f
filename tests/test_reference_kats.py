"""Known-answer tests authored by the reference (go-pbrt's own unit tests),
checked against the oracle and the product's host-side Go-math layer.

Each test cites the reference test it restates. These are the only
reference-authored known answers for the hot path; they pin
the oracle before it is trusted as the parity checker.
"""
import ctypes as C
import math
import struct

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

D3 = C.c_double * 3
EPS = 5e-324  # math.MachineEpsilon = NextFloatUp(0) (pkg/math/math.go:17)


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


# ---------------------------------------------------------------- Go math
def test_cos_pi_over_2_is_go_not_libm():
    """pkg/pbrt/transform_test.go:80 pins Go's Cos(Pi/180*90) = 6.123233995736757e-17."""
    L = O.lib()
    x = L.oracle_go_radians(90)
    assert x == 1.5707963267948966
    assert L.oracle_go_cos(x) == 6.123233995736757e-17
    assert L.oracle_go_sin(x) == 1.0
    assert math.cos(x) == 6.123233995736766e-17  # libm differs: the oracle must not use it


def test_go_sin_pi_widely_observed_value():
    """Go's Sin(Pi) = 1.2246467991473515e-16 (libm: ...532e-16); parity anchor of SURVEY App. A."""
    assert O.lib().oracle_go_sin(math.pi) == 1.2246467991473515e-16


def test_go_max_min_special_cases():
    """src/math/dim.go semantics used by go-pbrt (parity ledger #25)."""
    L = O.lib()
    assert math.isinf(L.oracle_go_max(math.inf, math.nan))
    assert math.isnan(L.oracle_go_max(1.0, math.nan))
    assert math.copysign(1, L.oracle_go_max(-0.0, 0.0)) == 1
    assert math.copysign(1, L.oracle_go_min(-0.0, 0.0)) == -1
    assert L.oracle_go_min(-math.inf, math.nan) == -math.inf


def test_go_nextafter_and_int_conversion():
    L = O.lib()
    assert L.oracle_go_nextafter(0.0, 1.0) == EPS
    assert L.oracle_go_nextafter(2.0**53, 2.0**53 + 1) == 2.0**53  # NextFloatUp no-op (#24)
    assert L.oracle_go_f2i(math.nan) == -(2**63)
    assert L.oracle_go_f2i(-1.5) == -1


# --------------------------------------------------------------- ray_test.go
def _offset(impl, p, e, n, w):
    out = D3()
    if impl == "oracle":
        O.lib().oracle_offset_ray_origin(D3(*p), D3(*e), D3(*n), D3(*w), out)
        return list(out)
    raise ValueError(impl)


def test_offset_ray_origin_denormal():
    """pkg/pbrt/ray_test.go:10-19: OffsetRayOrigin(0, (eps,eps,eps), (1,1,1), (1,1,1)) == 1.5183e-320 x3."""
    out = _offset("oracle", (0, 0, 0), (EPS, EPS, EPS), (1, 1, 1), (1, 1, 1))
    assert out == [1.5183e-320] * 3


# ------------------------------------------------------------ efloat_test.go
def test_efloat_add():
    """pkg/efloat/efloat_test.go:9-13."""
    out = D3()
    assert O.lib().oracle_efloat_add(1.0, 0.0, 1.0, 0.0, out) == 0
    assert list(out) == [2.0, 1.9999999999999998, 2.0000000000000004]


# --------------------------------------------------------- transform_test.go
def _mat(rows):
    m = abi.Matrix4x4()
    for i in range(4):
        for j in range(4):
            m.m[i][j] = rows[i][j]
    return m


def _rows(m):
    return [[m.m[i][j] for j in range(4)] for i in range(4)]


@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_matrix_inverse(impl):
    """pkg/pbrt/transform_test.go:17-36."""
    m = _mat([[1, 0, 0, 0], [0, 1, 1, 0], [0, 0, 1, 0], [0, 0, 2, 1]])
    out = abi.Matrix4x4()
    rc = (O.lib().oracle_matrix_inverse if impl == "oracle" else G.lib().pbrt_matrix_inverse)(C.byref(m), C.byref(out))
    assert rc == 0
    assert _rows(out) == [[1, 0, 0, 0], [0, 1, -1, 0], [0, 0, 1, 0], [0, 0, -2, 1]]


@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_transform_point(impl):
    """pkg/pbrt/transform_test.go:66-75."""
    t = abi.Transform()
    p, e = D3(), D3()
    if impl == "oracle":
        O.lib().oracle_translate(5, 4, 3, C.byref(t))
        O.lib().oracle_transform_point(C.byref(t), D3(0, 0, 0), D3(0, 0, 0), p, e)
    else:
        G.lib().pbrt_translate(5, 4, 3, C.byref(t))
        G.lib().pbrt_transform_point(C.byref(t), D3(0, 0, 0), D3(0, 0, 0), p, e)
    assert list(p) == [5, 4, 3]
    ident = abi.Transform()
    ident.m = _mat([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
    ident.m_inv = ident.m
    f = O.lib().oracle_transform_point if impl == "oracle" else G.lib().pbrt_transform_point
    f(C.byref(ident), D3(0, 0, 0), D3(0, 0, 0), p, e)
    assert list(p) == [0, 0, 0] and list(e) == [0, 0, 0]


@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_transform_ray_pins_go_cos(impl):
    """pkg/pbrt/transform_test.go:77-81: RotateY(90)*Translate(5,4,3) on o=0, d=x gives
    o=(3.0000000000000004, 4, -5), d=(6.123233995736757e-17, 0, -1)."""
    if impl == "oracle":
        L = O.lib()
        ry, tr, x = abi.Transform(), abi.Transform(), abi.Transform()
        L.oracle_rotate(1, 90, C.byref(ry))
        L.oracle_translate(5, 4, 3, C.byref(tr))
        L.oracle_xf_mul(C.byref(ry), C.byref(tr), C.byref(x))
        oo, od = D3(), D3()
        L.oracle_transform_ray(C.byref(x), D3(0, 0, 0), D3(1, 0, 0), oo, od)
        oo, od = list(oo), list(od)
    else:
        x = G.mul(G.rotate(1, 90), G.translate(5, 4, 3))
        oo, od = G.transform_ray(x, (0, 0, 0), (1, 0, 0))
    assert oo == [3.0000000000000004, 4, -5]
    assert od == [6.123233995736757e-17, 0, -1]


# ------------------------------------------------------------ light_test.go
def test_visibility_tester_shadow_ray():
    """pkg/pbrt/light_test.go:10-44: p0=0, p1=(10,0,0), zero normals and errors ->
    Ray{Origin 0, Direction (10,0,0), TMax 0.9999}."""
    out = (C.c_double * 7)()
    O.lib().oracle_spawn_ray_to((C.c_double * 18)(0, 0, 0, 0, 0, 0, 0, 0, 0, 10, 0, 0, 0, 0, 0, 0, 0, 0), out)
    assert list(out) == [0, 0, 0, 10, 0, 0, 0.9999]


# ------------------------------------------------------- reflection_test.go
def test_matches_flags():
    """pkg/pbrt/reflection_test.go:8-14 (MatchesFlags(t, f) = t&f == t)."""
    R, T, Dif, Gl, S = 1, 2, 4, 8, 16
    ALL = R | T | Dif | Gl | S
    mf = lambda t, f: (t & f) == t  # noqa: E731
    assert mf(Dif, Dif) and mf(Dif, Dif | R) and mf(R, Dif | R) and not mf(R, Dif) and mf(R, ALL)
    # the hot path relies on it: Lambertian (R|D) matches BSDFAll and All&^Specular
    assert mf(R | Dif, ALL) and mf(R | Dif, ALL & ~S) and not mf(R | Dif, R | S)


# ---------------------------------------- simple_test.go / bvh_test.go scene
def _three_spheres(builder):
    """pkg/accelerator/simple_test.go:10-38: spheres r=1 at (0,0,5), (0,0,10), (10,10,10, reversed)."""
    specs = [((0, 0, 5), False), ((0, 0, 10), False), ((10, 10, 10), True)]
    return specs


def _oracle_three_spheres(max_prims):
    L = O.lib()
    h = L.oracle_scene_new()
    m = abi.MaterialDesc()
    m.kd_type = abi.PBRT_TEX_CONSTANT
    m.kd[0] = m.kd[1] = m.kd[2] = 0.5
    L.oracle_scene_add_material(h, C.byref(m))
    for (x, y, z), rev in _three_spheres(None):
        t, sd = abi.Transform(), abi.ShapeDesc()
        L.oracle_translate(x, y, z, C.byref(t))
        L.oracle_make_sphere(C.byref(t), int(rev), 1.0, -1.0, 1.0, 360.0, C.byref(sd))
        s = L.oracle_scene_add_shape(h, C.byref(sd))
        p = abi.PrimitiveDesc()
        p.kind, p.shape, p.material = abi.PBRT_PRIM_GEOMETRIC, s, 0
        L.oracle_scene_add_primitive(h, C.byref(p))
    assert L.oracle_scene_finalize(h, max_prims) == 0
    return O.OracleScene(h)


def _rays():
    # the four rays of simple_test.go:60-108 / bvh_test.go:43-141
    return np.array([
        [0, 0, 0, 0, 0, 1.0, np.inf],
        [0, 0, 0, 0, 0, -1.0, np.inf],
        [0, 0, 500, 0, 0, -1.0, np.inf],
        [10, 10, 500, 0, 0, -1.0, np.inf],
    ])


@pytest.mark.parametrize("max_prims", [255, 2])
def test_bvh_intersect_primitive_identity(max_prims):
    """bvh_test.go:43-106: hits prims[0], miss, prims[1], prims[2]."""
    sc = _oracle_three_spheres(max_prims)
    order = sc.order()
    out = O.intersect(sc.desc, _rays(), closest=True)
    hit = out[:, 0].astype(bool)
    assert list(hit) == [True, False, True, True]
    prim_original = [order[int(p)] if h else -1 for p, h in zip(out[:, 2], hit)]
    assert prim_original == [0, -1, 1, 2]


@pytest.mark.parametrize("max_prims", [255, 2])
def test_bvh_intersect_p_table(max_prims):
    """bvh_test.go:108-141 and simple_test.go:69-108."""
    sc = _oracle_three_spheres(max_prims)
    occ = O.intersect(sc.desc, _rays(), closest=False)
    assert list(occ.astype(bool)) == [True, False, True, True]


def test_sphere_hit_point_exact():
    """simple_test.go:40-57: ray from (15,15,15) along normalize(-1,-1,-1) hits the reversed
    sphere at (10,10,10) + normalize(1,1,1), compared exactly."""
    sc = _oracle_three_spheres(255)
    inv = 1.0 / math.sqrt(3.0)
    d = [-1 * inv, -1 * inv, -1 * inv]  # Normalize(): multiply by 1/sqrt
    out = O.intersect(sc.desc, np.array([[15, 15, 15, d[0], d[1], d[2], np.inf]]), closest=True)
    assert out[0, 0] == 1.0
    expected = 10 + inv  # (10,10,10).AddAssign(normalize(1,1,1))
    assert list(out[0, 3:6]) == [expected] * 3


def test_bvh_build_matches_product_builder():
    """The product's host BVH (pbrt_sb_build) equals the oracle's restatement of
    RecursiveBuild/flattenBVHTree (bvh.go:272-411, 632-651) for the test scene."""
    for max_prims in (255, 2):
        sc = _oracle_three_spheres(max_prims)
        s = G.Scene()
        m = s.add_matte((0.5, 0.5, 0.5))
        for (x, y, z), rev in _three_spheres(None):
            sh = s.add_sphere(G.translate(x, y, z), 1.0, reverse=rev)
            s.add_primitive(sh, m)
        s.set_film(16, 16)
        s.set_camera(G.look_at((0, 0, -10), (0, 0, 0), (0, 1, 0)))
        s.build(max_prims)
        assert s.desc.n_nodes == sc.desc.n_nodes
        a = C.string_at(C.cast(s.desc.nodes, C.c_void_p).value, s.desc.n_nodes * C.sizeof(abi.BVHNode))
        b = C.string_at(C.cast(sc.desc.nodes, C.c_void_p).value, sc.desc.n_nodes * C.sizeof(abi.BVHNode))
        assert a == b
        assert s.prim_order() == sc.order()


# ------------------------------------------------ pkg/geometry/xyz_test.go
def _vop(impl, op, a, b=None, s=0.0):
    a = np.ascontiguousarray(a, dtype=np.float64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.zeros(3)
    P = C.POINTER(C.c_double)
    f = O.lib().oracle_vec_op if impl == "oracle" else G.lib().pbrt_diag_vec_op
    f.argtypes = [C.c_int, P, P, C.c_double, P]
    rc = f(op, a.ctypes.data_as(P), None if bb is None else bb.ctypes.data_as(P), s, out.ctypes.data_as(P))
    assert rc == 0
    return out


XYZ_KATS = [
    # (xyz_test.go function, op, a, b, scalar, expected (vector or scalar))
    ("Abs :9-13", "ABS", (-1, -2, -3), None, 0, (1, 2, 3)),
    ("AbsDot :15-18", "ABSDOT", (-1, -2, -3), (1, 2, 3), 0, 14.0),
    ("Add :20-23", "ADD", (1, 2, 3), (1, 2, 3), 0, (2, 4, 6)),
    ("Cross :37-40", "CROSS", (1, 2, 3), (1, 2, 4), 0, (2, -1, 0)),
    ("Distance :42-45", "DISTANCE", (1, 2, 3), (1, 2, 4), 0, 1.0),
    ("DistanceSquared :47-50", "DISTANCE_SQUARED", (1, 2, 3), (1, 2, 5), 0, 4.0),
    ("Div :52-55", "DIV", (3, 9, 27), (3, 3, 3), 0, (1, 3, 9)),
    ("DivScalar :63-66", "DIV_SCALAR", (3, 9, 27), None, 3.0, (1, 3, 9)),
    ("Dot :68-72", "DOT", (3, 9, 27), (2, 4, 6), 0, 204.0),
    ("Length :87-90", "LENGTH", (0, 3, 0), None, 0, 3.0),
    ("LengthSquared :92-95", "LENGTH_SQUARED", (0, 3, 0), None, 0, 9.0),
    ("Mul :97-101", "MUL", (1, 2, 3), (1, 2, 3), 0, (1, 4, 9)),
    ("MulScalar :109-112", "MUL_SCALAR", (1, 2, 3), None, 2.0, (2, 4, 6)),
    ("Normalize :114-118", "NORMALIZED", (0, 0, 3), None, 0, (0, 0, 1)),
    ("Normalized :120-123", "NORMALIZED", (0, 0, 3), None, 0, (0, 0, 1)),
    ("Sub :154-157", "SUB", (2, 4, 6), (1, 3, 5), 0, (1, 1, 1)),
]


@pytest.mark.parametrize("impl", ["oracle", "product"])
@pytest.mark.parametrize("kat", XYZ_KATS, ids=lambda k: k[0].split()[0])
def test_xyz_kats(kat, impl):
    """pkg/geometry/xyz_test.go (exact equality, as testify's assert.Equal), on
    the oracle and on the product's pbrt_core.h (host instantiation)."""
    name, op, a, b, s, want = kat
    out = _vop(impl, _VOPS[op], a, b, s)
    if isinstance(want, tuple):
        assert tuple(out) == tuple(float(w) for w in want), name
    else:
        assert out[0] == want, name


SPEC_KATS = [
    # spectrum_test.go: NewSpectrum(v) = (v, v, v)
    ("Add :9-18", "SPEC_ADD", (1, 1, 1), (2, 2, 2), 0, (3, 3, 3)),
    ("DivScalar :51-54", "SPEC_DIV_SCALAR", (3, 3, 3), None, 3.0, (1, 1, 1)),
    ("Mul :56-59", "SPEC_MUL", (3, 3, 3), (4, 4, 4), 0, (12, 12, 12)),
    ("IsBlack :61-66 rgb(1,0,1)", "SPEC_IS_BLACK", (1, 0, 1), None, 0, 0.0),
    ("IsBlack :61-66 1", "SPEC_IS_BLACK", (1, 1, 1), None, 0, 0.0),
    ("IsBlack :61-66 0.0001", "SPEC_IS_BLACK", (0.0001, 0.0001, 0.0001), None, 0, 0.0),
    ("IsBlack :61-66 0", "SPEC_IS_BLACK", (0, 0, 0), None, 0, 1.0),
]

_VOPS = {"ABS": 1, "ABSDOT": 2, "ADD": 3, "CROSS": 4, "DISTANCE": 5, "DISTANCE_SQUARED": 6, "DIV": 7,
         "DIV_SCALAR": 8, "DOT": 9, "LENGTH": 10, "LENGTH_SQUARED": 11, "MUL": 12, "MUL_SCALAR": 13,
         "NORMALIZED": 14, "SUB": 15, "SPEC_ADD": 16, "SPEC_MUL": 17, "SPEC_DIV_SCALAR": 18, "SPEC_IS_BLACK": 19,
         "SPEC_MUL_SCALAR": 20}


@pytest.mark.parametrize("impl", ["oracle", "product"])
@pytest.mark.parametrize("kat", SPEC_KATS, ids=lambda k: k[0].replace(" ", "_"))
def test_spectrum_kats(kat, impl):
    """pkg/pbrt/spectrum_test.go. AddScalar, AddAssign and Clone are Go value /
    aliasing semantics of methods the hot path does not call (Spectrum values
    are passed by value in both restatements)."""
    name, op, a, b, s, want = kat
    out = _vop(impl, _VOPS[op], a, b, s)
    if isinstance(want, tuple):
        assert tuple(out) == tuple(float(w) for w in want), name
    else:
        assert out[0] == want, name


# ------------------------------------ pkg/accelerator/bvh_test.go:143-264
PARTITION_KATS = [
    ([5, 4, 3, 2, 1], 0, 4, 2, [1, 2, 3, 4, 5]),
    ([5, 1, 2, 4, 3], 0, 4, 1, [1, 3, 2, 4, 5]),
]


@pytest.mark.parametrize("impl", ["oracle", "product"])
@pytest.mark.parametrize("kat", PARTITION_KATS, ids=["Test0", "Test1"])
def test_partition_primitive_info_at(kat, impl):
    """TestPartitionPrimitiveInfoAt: primitiveNumber k has centroid (k, 0, 0);
    the less-than-on-x predicate; the expected primitive order after the
    Lomuto pass. (RadixSortInPlace, bvh_test.go:20-41, serves HLBVH only,
    which nil-derefs in the reference and is not restated.)"""
    prims, start, end, pivot, want = kat
    p = np.array(prims, dtype=np.int32)
    cx = p.astype(np.float64)
    f = O.lib().oracle_partition_at if impl == "oracle" else G.lib().pbrt_diag_partition_at
    f.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_int64, C.c_int64, C.c_int64, C.c_int64]
    f.restype = C.c_int64
    m = f(p.ctypes.data_as(C.POINTER(C.c_int32)), cx.ctypes.data_as(C.POINTER(C.c_double)), len(p), start, end,
          pivot)
    assert list(p) == want
    assert cx.tolist() == [float(x) for x in want]
    assert 0 <= m <= end and p[m] == prims[pivot]
