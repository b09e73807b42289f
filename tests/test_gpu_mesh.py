"""Triangle-mesh extension on the GPU (BASELINE configs D/E): the device LBVH's
structure, batch intersection and renders, bit for bit against the oracle's
independent restatement (oracle/oracle_mesh.c, its own median-split BVH).
go-pbrt has no triangle shape, so this parity is "unpinned" (no reference
arithmetic to pin the triangle test to; tests/test_mesh.py checks the
oracle's known answers and its accelerator against brute force).
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


def same_bits(a, b):
    return np.array_equal(bits(a), bits(b))


def mesh_tris(scene):
    m = scene.desc.meshes[0]
    p = np.ctypeslib.as_array(m.p, shape=(m.n_vertices * 3,)).reshape(-1, 3)
    idx = np.ctypeslib.as_array(m.indices, shape=(m.n_triangles * 3,)).reshape(-1, 3)
    return p[idx].reshape(-1, 9)


def check_wide_tree(nodes, tris, nt, info):
    """The 4-ary layout (pbrt_mesh.h MeshNode4): one tree; every node but the
    root is the child of exactly one node and names it as parent; slots
    0..count-1 hold a node or a triangle, the rest are empty; child boxes
    contain their subtree's boxes and triangles; the slots are in ascending
    centre order along the node's axis; every triangle is one slot; the depth
    is the builder's level count and at most 32."""
    EMPTY, TRI = 0xFFFFFFFF, 0x80000000
    n = len(nodes)
    assert n >= 1 and nodes[0]["parent"] == EMPTY
    seen = np.zeros(n, dtype=np.int32)
    covered = np.zeros(nt, dtype=np.int32)
    levels = 0
    stack = [(0, 1, None)]
    while stack:
        i, lev, box = stack.pop()
        seen[i] += 1
        levels = max(levels, lev)
        nd = nodes[i]
        cnt, ax = int(nd["count"]), int(nd["axis"])
        assert 1 <= cnt <= 4 and ax < 3
        lo, hi = nd["lo"], nd["hi"]   # [3][4]
        if box is not None:
            assert (lo[:, :cnt] >= box[0][:, None]).all() and (hi[:, :cnt] <= box[1][:, None]).all()
        cen = lo[ax, :cnt] + hi[ax, :cnt]
        assert (np.diff(cen) >= 0).all()
        for k in range(4):
            c = int(nd["child"][k])
            if k >= cnt:
                assert c == EMPTY
                continue
            if c & TRI:
                s = c & ~TRI
                covered[s] += 1
                t = tris[s].reshape(3, 3)
                assert (t >= lo[:, k]).all() and (t <= hi[:, k]).all()
            else:
                assert 0 < c < n and nodes[c]["parent"] == i
                stack.append((c, lev + 1, (lo[:, k], hi[:, k])))
    assert (seen == 1).all() and (covered == 1).all()
    assert levels == info["depth"] <= 32


@pytest.mark.parametrize("quads", [1, 2, 3, 16, 100])
def test_lbvh_structure(quads):
    """Every ordering is a depth-first threading of one binary tree: leaves
    escape to the next node, the second child of an interior node starts at its
    first child's escape and ends at the node's; leaves partition the triangle
    slots; boxes nest and contain their triangles; gid is a permutation."""
    scene = G.Scene.heightfield(16, 16, quads=quads, seed=5)
    tris_in = mesh_tris(scene)
    with G.Renderer(scene) as r:
        info = r.mesh_info()
        nodes, gid, tris = r.mesh_download()
    nt = 2 * quads * quads
    assert info["tris"] == nt and info["meshes"] == 1
    assert sorted(gid.tolist()) == list(range(nt))
    assert np.array_equal(tris, tris_in[gid])
    n = info["nodes"]
    if info["wide"]:
        check_wide_tree(nodes, tris, nt, info)
        return
    assert nodes.shape == (8, n) and n >= 1
    recs = None
    for o in range(8):
        N = nodes[o]
        covered = np.zeros(nt, dtype=np.int32)

        def walk(i, lo, hi):   # returns the escape of node i
            nd = N[i]
            assert (nd["bmin"] >= lo).all() and (nd["bmax"] <= hi).all()
            if nd["leaf"] != 0xFFFFFFFF:
                first, cnt = int(nd["leaf"]) >> 3, int(nd["leaf"]) & 7
                assert 1 <= cnt <= 4
                covered[first:first + cnt] += 1
                t = tris[first:first + cnt].reshape(-1, 3, 3)
                assert (t >= nd["bmin"]).all() and (t <= nd["bmax"]).all()
                assert nd["escape"] == i + 1
                return i + 1
            e1 = walk(i + 1, nd["bmin"], nd["bmax"])
            e2 = walk(e1, nd["bmin"], nd["bmax"])
            assert e2 == nd["escape"]
            return e2

        inf = np.float32(np.inf)
        assert walk(0, -inf, inf) == n
        assert (covered == 1).all()
        rec = sorted((tuple(N[i]["bmin"]), tuple(N[i]["bmax"]), int(N[i]["leaf"])) for i in range(n))
        recs = rec if recs is None else recs
        assert rec == recs   # the eight orderings hold the same nodes


def random_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = np.stack([rng.uniform(-150, 250, n), rng.uniform(-10, 120, n), rng.uniform(-150, 250, n)], axis=1)
    d = rng.normal(size=(n, 3))
    d[rng.uniform(size=n) < 0.02, 0] = 0.0   # axis-parallel directions (d == 0 slabs)
    tmax = np.where(rng.uniform(size=n) < 0.2, rng.uniform(1, 200, n), np.inf)
    return np.concatenate([o, d, tmax[:, None]], axis=1)


@pytest.mark.parametrize("spheres", [False, True])
@pytest.mark.parametrize("quads", [8, 200])
def test_intersect_mesh_matches_oracle(quads, spheres):
    scene = G.Scene.heightfield(32, 32, quads=quads, seed=1, spheres=spheres)
    rays = random_rays(20_000, 9)
    with G.Renderer(scene) as r:
        rc, got = r.intersect(rays)
        rc_p, occ = r.intersect_p(rays)
    assert rc == 0 and rc_p == 0
    want = O.intersect(scene.desc, rays, closest=True)
    wocc = O.intersect(scene.desc, rays, closest=False)
    assert same_bits(got, want), int((bits(got) != bits(want)).any(axis=1).sum())
    assert np.array_equal(occ.astype(bool), wocc.astype(bool))
    tri_hits = (got[:, 0] == 1) & (got[:, 2] >= scene.desc.n_prims)
    assert tri_hits.mean() > 0.1


MESH_CASES = [
    (8, False, dict(spp_x=2, spp_y=2)),
    (32, True, dict(spp_x=2, spp_y=2)),
    (64, False, dict(spp_x=4, spp_y=4, max_depth=6)),
    (16, True, dict(spp_x=3, spp_y=3, rr_threshold=0.5, max_depth=12)),
]


@pytest.mark.parametrize("paths_wf", ["default", "0"])
@pytest.mark.parametrize("kernel", ["serial", "auto"])
@pytest.mark.parametrize("mode", [abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT])
@pytest.mark.parametrize("case", MESH_CASES, ids=lambda c: f"q{c[0]}{'s' if c[1] else ''}-{c[2]}")
def test_render_mesh_bitexact(case, mode, kernel, paths_wf, monkeypatch):
    """Mesh scenes run their full paths on the path wavefront by default
    (k_pw_*); PBRT_PATHS_WF=0 keeps k_paths_ci. Both bit for bit."""
    if paths_wf != "default":
        if kernel == "serial":
            pytest.skip("the serial kernel has no path stage")
        monkeypatch.setenv("PBRT_PATHS_WF", paths_wf)
    quads, spheres, kw = case
    scene = G.Scene.heightfield(48, 32, quads=quads, seed=1, spheres=spheres)
    rd = abi.render_desc(**kw, mode=mode)
    with G.Renderer(scene, kernel=kernel) as r:
        film, st = r.render(rd)
    if kernel == "auto":
        assert st.kernel in (abi.PBRT_KERNEL_WAVE, abi.PBRT_KERNEL_WAVE_CI)
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0 and st.paths_traced == ost.paths
    assert same_bits(film, ofilm), int((film != ofilm).sum())
    assert film.max() > 0


@pytest.mark.slow
def test_config_D_full_size_properties_and_heaviest_tiles():
    """BASELINE config D: 999 698 triangles, 1920x1080, Stratified(8,8),
    Path(10): every path traced, finite film, the device BVH build time, and
    the first / middle / last tiles plus the heaviest three bit-exact."""
    W, H = 1920, 1080
    scene = G.Scene.heightfield(W, H, quads=707, seed=1)
    rd = abi.render_desc(8, 8)
    with G.Renderer(scene) as r:
        info = r.mesh_info()
        film, st = r.render(rd)
        ticks, _ = r.tile_ticks()
        film2, _ = r.render(rd)   # the steady-state frame: learned heaviest-first order
    assert info["tris"] == 999698
    print(f"config D LBVH: {info}")
    assert st.tiles_rendered == 8160 and st.paths_traced == W * H * 63
    assert np.isfinite(film).all() and film.max() > 0
    assert len(ticks) == 8160
    heaviest = [int(t) for t in np.argsort(ticks)[::-1][:3]]
    for t in sorted({0, 4080, 8159, *heaviest}):
        one = abi.render_desc(8, 8, tile_begin=t, tile_end=t + 1)
        with G.Renderer(scene) as r:
            g, _ = r.render(one)
        rc, o, _ = O.render(scene.desc, one, threads=1)
        assert rc == 0 and same_bits(g, o), t
        # pixels only tile t's samples reach, in the cold and the second frame
        x0, y0 = (t % 120) * 16, (t // 120) * 16
        for f in (film, film2):
            assert np.all(f[y0:y0 + 15, x0:x0 + 15] == o[y0:y0 + 15, x0:x0 + 15]), t


@pytest.mark.slow
def test_config_E_full_mesh_sampled_tiles_bitexact():
    """BASELINE config E: the 9 999 392-triangle height field, 3840x2160,
    Stratified(32,32) (1023 traced paths per pixel), Path(10). The device
    LBVH of the full mesh renders an evenly spread sample of 24 of the 32 400
    tiles (tile_stride 1350, several batches at 1023 spp), bit for bit against
    the oracle's own BVH over the same mesh."""
    W, H = 3840, 2160
    scene = G.Scene.heightfield(W, H, quads=2236, seed=1)
    rd = abi.render_desc(32, 32, tile_begin=0, tile_stride=1350)
    with G.Renderer(scene) as r:
        info = r.mesh_info()
        film, st = r.render(rd)
    assert info["tris"] == 9999392
    print(f"config E LBVH: {info}; sampled frame: {st.kernel_ms:.0f} ms, {st.batches} batches")
    assert st.tiles_rendered == 24 and st.paths_traced == 24 * 256 * 1023
    assert np.isfinite(film).all() and film.max() > 0
    rc, ofilm, ost = O.render(scene.desc, rd, threads=THREADS)
    assert rc == 0 and ost.paths == st.paths_traced
    assert same_bits(film, ofilm), int((bits(film) != bits(ofilm)).any(axis=2).sum())
