"""Estimate bench.py's multi-GPU scaling on one GPU: render the tile shard each
rank of an N-GPU job would get (tiles t with t mod N == r) and time it.

    python tools/shard_sim.py [--ns 1,2,4,8] [--ranks 0,7] [--mode exact]

Prints one JSON line per (N, r): the shard's kernel ms and paths. The N-GPU
frame time is the max over ranks plus the film reduce (not simulated here).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-pbrt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--ranks", default="0,-1")
    ap.add_argument("--mode", default="exact", choices=["exact", "throughput"])
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rows", action="store_true", help="time each tile row alone instead (the row's slowest tile)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE knob (read when the context is created)")
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import torch
    import pbrtgpu as G
    W, H = 1920, 1080
    scene = G.Scene.readme(W, H)
    r = G.Renderer(scene, device=0, kernel=a.kernel)
    film = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    mode = G.abi.PBRT_MODE_EXACT if a.mode == "exact" else G.abi.PBRT_MODE_THROUGHPUT
    if a.rows:
        ntx, nty = (W + 15) // 16, (H + 15) // 16
        for ty in range(nty):
            rd = G.render_desc(spp_x=8, spp_y=8, tile_begin=ty * ntx, tile_end=(ty + 1) * ntx, tile_stride=1,
                               mode=mode)
            r.render_async(rd, film.data_ptr())
            st = r.synchronize()
            print(json.dumps({"row": ty, "chain_ms": st.chain_ms, "paths_ms": st.paths_ms,
                              "paths": int(st.paths_traced)}), flush=True)
        return
    for n in [int(x) for x in a.ns.split(",")]:
        for rr in [int(x) for x in a.ranks.split(",")]:
            rank = rr % n
            rd = G.render_desc(spp_x=8, spp_y=8, tile_begin=rank, tile_stride=n, mode=mode)
            r.render_async(rd, film.data_ptr())
            r.synchronize()
            best = None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.render_async(rd, film.data_ptr())
                st = r.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            print(json.dumps({"n": n, "rank": rank, "wall_ms": best * 1e3, "kernel_ms": st.kernel_ms,
                              "chain_ms": st.chain_ms, "paths_ms": st.paths_ms, "paths": int(st.paths_traced),
                              "kernel": int(st.kernel), "env": a.env}), flush=True)


if __name__ == "__main__":
    main()
