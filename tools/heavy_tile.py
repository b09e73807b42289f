"""Latency of single tiles of a frame (the heaviest tiles bound a multi-GPU shard's
chain): each tile rendered alone (tile_begin = t, tile_end = t + 1) at the given
k_chain_ci waves per tile and candidate strides.

    python tools/heavy_tile.py [--config B] [--tiles 5389,4648] [--waves 1,2,4,8] [--strides 0]

One JSON line per (tile, waves, stride): the chain ms (best of --reps frames) and,
with a diagnostics build (PBRT_GPU_LIB=lib/libpbrt_gpu_diag.so), the chain's
phase clocks (lane 0 of every wave; shares of their sum) and steps.
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-pbrt_amd"))

PHASES = ["start_pixel", "issue", "traversal", "hit", "walk"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B", choices=["B", "G", "C"])
    ap.add_argument("--tiles", default="5389,4648")
    ap.add_argument("--waves", default="1,2,4,8")
    ap.add_argument("--strides", default="0")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE knob (read when a context is created)")
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import pbrtgpu as G
    from pbrtgpu import abi
    W, H = 1920, 1080
    scene = {"B": G.Scene.readme, "G": G.Scene.readme_glass, "C": G.Scene.cornell}[a.config](W, H)
    spp, depth = (16, 8) if a.config == "C" else (8, 10)
    for t in [int(x) for x in a.tiles.split(",")]:
        for w in [int(x) for x in a.waves.split(",")]:
            for cs in [int(x) for x in a.strides.split(",")]:
                os.environ["PBRT_CI_WAVES"] = str(w)
                if cs:
                    os.environ["PBRT_CI_STRIDE"] = str(cs)
                else:
                    os.environ.pop("PBRT_CI_STRIDE", None)
                rd = abi.render_desc(spp, spp, max_depth=depth, tile_begin=t, tile_end=t + 1)
                best, vals = None, None
                with G.Renderer(scene) as r:
                    for _ in range(a.reps):
                        _, st = r.render(rd)
                        if best is None or st.chain_ms < best:
                            best = st.chain_ms
                            out = (C.c_uint64 * 80)()
                            n = G.lib().pbrt_gpu_counters(C.c_void_p(r.h), out, 80)
                            vals = list(out)[:n]
                rec = {"config": a.config, "env": a.env, "tile": t, "waves": w, "stride": cs, "chain_ms": best}
                if vals and len(vals) >= 11 and sum(vals[6:11]) > 0:
                    ph = vals[6:11]
                    tot = float(sum(ph))
                    rec["steps"] = vals[5]
                    rec["phase_share"] = {k: round(v / tot, 4) for k, v in zip(PHASES, ph)}
                    rec["steps_per_pixel"] = vals[5] / 256.0
                    rec["issued_per_pixel"] = vals[11] / 256.0
                    rec["on_chain_per_pixel"] = sum(vals[14:78]) / 256.0
                    if len(vals) >= 80:   # lane utilisation; next-pixel speculation candidates
                        rec["lane_util"] = vals[78] / max(1, vals[5] * 64 * w)
                        rec["nps_issued_per_pixel"] = vals[79] / 256.0
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
