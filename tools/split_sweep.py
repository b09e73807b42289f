"""k_chain_ci schedule experiments on one GPU: for a list of environment
settings (PBRT_CI_WAVES / PBRT_CI_HEAVY / PBRT_CI_SPLIT ...), render a config-B
shard (tiles t mod N == rank) on a fresh context for a few frames and report
the chain time of each frame, plus the per-tile chain-time distribution of the
last frame (sum over 2 waves/SIMD = the throughput bound, max = the latency bound).

    python tools/split_sweep.py --n 1 --settings "default;PBRT_CI_WAVES=4,PBRT_CI_HEAVY=32"
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--settings", default="default")
    a = ap.parse_args()
    import pbrtgpu as G
    scene = G.Scene.readme(1920, 1080)
    rd = G.render_desc(spp_x=8, spp_y=8, tile_begin=a.rank, tile_stride=a.n)
    for setting in a.settings.split(";"):
        env = {} if setting == "default" else dict(kv.split("=") for kv in setting.split(","))
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        with G.Renderer(scene, device=0) as r:
            chain = []
            for _ in range(a.frames):
                r.render_async(rd)
                st = r.synchronize()
                chain.append(round(st.chain_ms, 1))
            ticks, heavy = r.tile_ticks()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        t = np.sort(ticks.astype(np.float64) / 1e5)[::-1]   # ms at 100 MHz
        print(json.dumps({"n": a.n, "rank": a.rank, "setting": setting, "chain_ms": chain,
                          "paths_ms": round(st.paths_ms, 1), "heavy": heavy, "tiles": len(t),
                          "tile_ms_sum_over_2048_slots": round(t.sum() / 2048, 1),
                          "tile_ms_top10": [round(x, 1) for x in t[:10]],
                          "tile_ms_p50": round(float(np.median(t)), 1)}), flush=True)


if __name__ == "__main__":
    main()
