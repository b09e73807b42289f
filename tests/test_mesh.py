"""Triangle-mesh extension (BASELINE configs D/E), CPU side: the oracle's
triangle test, its accelerator against brute force, and the height-field
fixture. go-pbrt has no triangle shape, so parity here is "unpinned": the
triangle test restates pbrt-v3's Triangle::Intersect and these tests check
its known answers and the oracle's own consistency; the GPU path is then
checked against this oracle (tests/test_gpu_mesh.py).
"""
import math

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G

TRI = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], dtype=np.float64)


def test_triangle_known_answer():
    hit, t, b0, b1, b2 = O.triangle_hit(TRI, [0.25, 0.25, 1, 0, 0, -1, math.inf])
    assert hit and t == 1.0
    assert (b0, b1, b2) == (0.5, 0.25, 0.25)
    # from below, same t; grazing outside the triangle misses; behind the origin misses
    assert O.triangle_hit(TRI, [0.25, 0.25, -2, 0, 0, 1, math.inf])[:2] == (True, 2.0)
    assert not O.triangle_hit(TRI, [0.75, 0.75, 1, 0, 0, -1, math.inf])[0]
    assert not O.triangle_hit(TRI, [0.25, 0.25, 1, 0, 0, 1, math.inf])[0]


def test_triangle_edges_are_watertight():
    """Rays through the shared edge of two triangles hit at least one of them
    (the watertight test's guarantee)."""
    a = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], dtype=np.float64)
    b = np.array([1, 0, 0, 1, 1, 0, 0, 1, 0], dtype=np.float64)
    rng = np.random.default_rng(7)
    for s in rng.uniform(0, 1, size=500):
        o = [1 - s, s, 3.0]
        d = rng.normal(size=3) * 1e-3 + np.array([0, 0, -1.0])
        p = np.array(o) + d * (3.0 / -d[2])   # where the ray crosses z = 0
        o = list(np.array(o) - (p - np.array([1 - s, s, 0.0])))
        ray = o + list(d) + [math.inf]
        assert O.triangle_hit(a, ray)[0] or O.triangle_hit(b, ray)[0]


def brute_closest(tris, rays):
    """Smallest (t, index) over all triangles with t < tmax."""
    out = []
    for r in rays:
        best = (r[6], -1)
        for g in range(tris.shape[0]):
            h, t, *_ = O.triangle_hit(tris[g], r)
            if h and (t < best[0] or (t == best[0] and best[1] >= 0 and g < best[1])):
                best = (t, g)
        out.append(best)
    return out


def mesh_tris(scene):
    d = scene.desc
    m = d.meshes[0]
    p = np.ctypeslib.as_array(m.p, shape=(m.n_vertices * 3,)).reshape(-1, 3).astype(np.float64)
    idx = np.ctypeslib.as_array(m.indices, shape=(m.n_triangles * 3,)).reshape(-1, 3)
    return p[idx].reshape(-1, 9)


def test_heightfield_fixture():
    s = G.Scene.heightfield(32, 24, quads=8, seed=1)
    d = s.desc
    assert d.n_meshes == 1 and d.meshes[0].n_triangles == 2 * 8 * 8 and d.meshes[0].n_vertices == 81
    assert d.n_prims == 0 and d.n_lights == 4
    tris = mesh_tris(s)
    assert tris[:, 0::3].min() == -100 and tris[:, 0::3].max() == 200
    assert abs(tris[:, 1::3]).max() < 5.01
    # geometric normals point up (+y), the fixture's winding
    e1 = tris[:, 3:6] - tris[:, 0:3]
    e2 = tris[:, 6:9] - tris[:, 0:3]
    assert (np.cross(e1, e2)[:, 1] < 0).all() or (np.cross(e1, e2)[:, 1] > 0).all()
    # the world bound covers the mesh (Distant light radius, distant.go:36-38)
    assert d.world_min[0] == -100 and d.world_max[2] == 200
    # deterministic: the same seed gives the same vertices, another seed others
    s1, s2 = G.Scene.heightfield(8, 8, quads=8, seed=1), G.Scene.heightfield(8, 8, quads=8, seed=2)
    assert np.array_equal(mesh_tris(s1), tris)
    assert not np.array_equal(mesh_tris(s2), tris)
    big = G.Scene.heightfield(8, 8, quads=707)
    assert big.desc.meshes[0].n_triangles == 999698


@pytest.mark.parametrize("spheres", [False, True])
def test_oracle_mesh_closest_matches_brute_force(spheres):
    s = G.Scene.heightfield(16, 16, quads=6, seed=3, spheres=spheres)
    tris = mesh_tris(s)
    rng = np.random.default_rng(11)
    n = 300
    o = np.stack([rng.uniform(-120, 220, n), rng.uniform(5, 60, n), rng.uniform(-120, 220, n)], axis=1)
    d = rng.normal(size=(n, 3))
    d[:, 1] = -np.abs(d[:, 1]) - 0.2
    tmax = np.where(rng.uniform(size=n) < 0.3, rng.uniform(1, 100, n), np.inf)
    rays = np.concatenate([o, d, tmax[:, None]], axis=1)
    got = O.intersect(s.desc, rays, closest=True)
    anyh = O.intersect(s.desc, rays, closest=False)
    want = brute_closest(tris, rays)
    n_tri_hits = 0
    for i, (t, g) in enumerate(want):
        if spheres and got[i, 0] and got[i, 2] < s.desc.n_prims:
            assert g < 0 or got[i, 1] <= t   # an analytic primitive in front
            continue
        assert bool(got[i, 0]) == (g >= 0), i
        if g >= 0:
            n_tri_hits += 1
            assert got[i, 1] == t and int(got[i, 2]) == s.desc.n_prims + g, i
        assert bool(anyh[i]) >= bool(got[i, 0])
    assert n_tri_hits > n // 3


def test_oracle_renders_a_mesh_scene():
    s = G.Scene.heightfield(32, 24, quads=16, seed=1, spheres=True)
    rc, film, st = O.render(s.desc, G.render_desc(2, 2), threads=4)
    assert rc == 0 and st.paths == 32 * 24 * 3
    assert np.isfinite(film).all() and film.max() > 0
