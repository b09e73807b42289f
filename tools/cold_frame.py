"""Cold-frame schedule check (render.hip k_tile_cost): chain time of a fresh
context's first frame with the probe order, without it (PBRT_CI_PROBE=0, launch
order) and of the following frames (measured order), plus how well the probe's
cost predicts the measured per-tile chain times (Spearman rank correlation and a
least-squares fit of ticks on the probe features).

    python tools/cold_frame.py [--config B|C|D] [--frames 3] > gpurun_out/cold.json
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
sys.path.insert(0, REPO)


def rank(a):
    r = np.empty(len(a))
    r[np.argsort(a, kind="stable")] = np.arange(len(a))
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B")
    ap.add_argument("--frames", type=int, default=3)
    args = ap.parse_args()
    import pbrtgpu as G
    from bench import CONFIGS, make_scene

    cfg = CONFIGS[args.config]
    scene = make_scene(G, cfg, 1920, 1080)
    rd = G.render_desc(spp_x=cfg["spp"], spp_y=cfg["spp"], max_depth=cfg["max_depth"])
    out = {"config": args.config}
    for probe in (0, 1):
        os.environ["PBRT_CI_PROBE"] = str(probe)
        with G.Renderer(scene, device=0) as r:
            chain = []
            for f in range(args.frames):
                r.render_async(rd)
                st = r.synchronize()
                chain.append(st.chain_ms)
                if f == 0:
                    ticks, _ = r.tile_ticks()
                    costs = r.tile_costs()
            out[f"probe{probe}_chain_ms"] = chain
            if probe and len(costs):
                t = ticks.astype(np.float64)
                X = np.c_[costs[:, 0], costs[:, 1], costs[:, 2], np.ones(len(t))].astype(np.float64)
                coef, *_ = np.linalg.lstsq(X, t, rcond=None)
                pred = X @ coef
                out["spearman_cost_ticks"] = float(np.corrcoef(rank(costs[:, 3]), rank(t))[0, 1])
                out["spearman_work_ticks"] = float(np.corrcoef(rank(costs[:, 0]), rank(t))[0, 1])
                out["lstsq_ticks_on_work_hits_px_1"] = coef.tolist()
                out["lstsq_r2"] = float(1 - ((t - pred) ** 2).sum() / ((t - t.mean()) ** 2).sum())
                top = np.argsort(-t)[:20]
                out["top20_ticks"] = t[top].tolist()
                out["top20_cost_rank"] = [int(x) for x in (len(t) - 1 - rank(costs[:, 3]))[top]]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
