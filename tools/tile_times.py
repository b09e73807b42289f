"""Distribution of the per-tile k_chain_ci times of one frame (wall_clock64 ticks
at 100 MHz, recorded by every EXACT frame for the next frame's schedule).

    python tools/tile_times.py [--config B|G|C] [--top 20]

Prints one JSON line: the chain's kernel ms, the tile-time mean / p50 / p99 / max
(ms), the sum over tiles divided by the concurrent tile slots (the lane-time
bound), and the heaviest tiles with their (x, y) tile coordinates.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-pbrt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B", choices=["B", "G", "C"])
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE knob (read when the context is created)")
    ap.add_argument("--frames", type=int, default=2, help="frames rendered; the last one is reported")
    ap.add_argument("--dump", action="store_true", help="add every tile's ms (slot order) to the JSON line")
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import pbrtgpu as G
    W, H = 1920, 1080
    scene = {"B": G.Scene.readme, "G": G.Scene.readme_glass, "C": G.Scene.cornell}[a.config](W, H)
    spp, depth = (16, 8) if a.config == "C" else (8, 10)
    rd = G.render_desc(spp_x=spp, spp_y=spp, max_depth=depth)
    with G.Renderer(scene) as r:
        for _ in range(a.frames):   # from the second frame on: the measured order of the previous one
            _, st = r.render(rd)
        ticks, heavy = r.tile_ticks()
    t = np.asarray(ticks, dtype=np.float64) / 1e5   # 100 MHz ticks -> ms
    ntx = (W + 15) // 16
    order = np.argsort(-t)[:a.top]
    print(json.dumps({
        "config": a.config, "env": a.env, "chain_ms": st.chain_ms, "tiles": int(t.size), "heavy_slots": heavy,
        "tile_ms": {"mean": float(t.mean()), "p50": float(np.median(t)), "p99": float(np.percentile(t, 99)),
                    "max": float(t.max())},
        "sum_over_2048_slots_ms": float(t.sum() / 2048.0),
        "heaviest": [{"tile": int(i), "tx": int(i % ntx), "ty": int(i // ntx), "ms": float(t[i])} for i in order],
        **({"all_ms": [round(float(x), 3) for x in t]} if a.dump else {}),
    }))


if __name__ == "__main__":
    main()
