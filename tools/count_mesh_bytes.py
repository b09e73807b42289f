"""Algorithmic HBM bytes of the mesh traversal (configs D/E), per kernel: one
frame rendered with the counting build (make -C go-pbrt_amd meshcount), whose
mesh walks count the node bytes they fetch in 32-byte blocks (a binary node is
one block; a wide node visit reads four, going back up through a wide parent
one) and the triangles they test (36 B each). Needs a GPU. The result is committed under profiles/ and read by
bench.py --config D for the HBM roofline (achieved = these bytes / the
kernel's measured time).

    PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_meshcount.so \\
        python tools/count_mesh_bytes.py [--quads 707 --width 1920 --height 1080 --spp 8]
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
os.environ.setdefault("PBRT_GPU_LIB", os.path.join(REPO, "go-pbrt_amd", "lib", "exp", "libpbrt_gpu_meshcount.so"))

SLOTS = {1: "k_wf_primary", 2: "k_chain_ci", 3: "k_paths_ci", 4: "k_mb_setup", 5: "k_paths_ci_mb",
         6: "k_render_exact", 7: "k_intersect"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quads", type=int, default=707)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--mode", default="exact", choices=["exact", "throughput"])
    ap.add_argument("--max-depth", type=int, default=10)
    ap.add_argument("--shard", default="", help="R/N: count the tiles t mod N == R only (per-path figures)")
    a = ap.parse_args()
    import pbrtgpu as G
    L = G.lib()
    L.pbrt_gpu_mesh_counters.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int]
    buf = (C.c_uint64 * 48)()
    assert L.pbrt_gpu_mesh_counters(buf, 48, 1) == 48, "not the counting build (make meshcount)"
    scene = G.Scene.heightfield(a.width, a.height, quads=a.quads, seed=1)
    mode = G.abi.PBRT_MODE_EXACT if a.mode == "exact" else G.abi.PBRT_MODE_THROUGHPUT
    with G.Renderer(scene) as r:
        info = r.mesh_info()
        r0, n0 = (int(x) for x in a.shard.split("/")) if a.shard else (0, 1)
        _, st = r.render(G.render_desc(a.spp, a.spp, mode=mode, max_depth=a.max_depth, tile_begin=r0,
                                       tile_stride=n0))
    L.pbrt_gpu_mesh_counters(buf, 48, 1)
    v = list(buf)
    out = {"scene": f"heightfield quads={a.quads} seed=1", "triangles": info["tris"], "nodes": info["nodes"],
           "depth": info["depth"], "width": a.width, "height": a.height, "sampler": f"Stratified({a.spp},{a.spp})",
           "mode": a.mode, "paths": int(st.paths_traced), "tiles": a.shard or "all", "bytes_per_node": 32, "bytes_per_triangle": 36,
           "layout": "wide (MeshNode4, 128 B)" if info.get("wide") else "binary (8 threaded orderings, 32 B)",
           "definition": "per launch: node blocks fetched x 32 B + triangles tested x 36 B over every mesh "
                         "walk of the kernel (libpbrt_gpu_meshcount.so counters; 'nodes' counts 32-byte "
                         "blocks: a wide node visit is 4, a wide parent read 1)", "kernels": {}}
    for slot, name in SLOTS.items():
        k = {}
        for q, qn in ((0, "closest"), (1, "any")):
            walks, nodes, tris = v[(slot * 2 + q) * 3:(slot * 2 + q) * 3 + 3]
            if walks:
                k[qn] = {"walks": walks, "nodes": nodes, "triangles": tris,
                         "nodes_per_walk": nodes / walks, "triangles_per_walk": tris / walks}
        if k:
            b = sum(x["nodes"] * 32 + x["triangles"] * 36 for x in k.values())
            k["bytes_per_launch"] = b
            k["bytes_per_path"] = b / max(1, int(st.paths_traced))
            out["kernels"][name] = k
    path = os.path.join(REPO, "profiles",
                        f"meshbytes_heightfield{a.quads}_{a.width}x{a.height}_s{a.spp}x{a.spp}_{a.mode}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
