"""Render one frame and print the wave kernel's phase counters (diagnostics).

    python tools/phase_stats.py [--width W --height H --spp S --kernel auto|serial]
                                [--scene cornell --max-depth 8 --tile-stride 16]

With the diagnostics build (make diag) it also prints, per pixel, the chain
steps, the candidate trajectories issued and the on-chain ones (the on-chain
D histogram's total), and the count of on-chain draw counts above the tail
cap's bound dmax (k_chain.h; must be 0).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go-pbrt_amd"))
import pbrtgpu as G  # noqa: E402
from pbrtgpu import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=8)
ap.add_argument("--max-depth", type=int, default=10)
ap.add_argument("--tile-stride", type=int, default=1, help="render every k-th tile only (an evenly spread sample)")
ap.add_argument("--kernel", default="auto")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--occupancy", type=int, default=0)
ap.add_argument("--tiles-per-wave", type=int, default=0)
ap.add_argument("--scene", default="readme", choices=["readme", "readme_glass", "cornell", "heightfield"])
ap.add_argument("--quads", type=int, default=707, help="height field cells per side (heightfield: 707 = config D, 2236 = E)")
ap.add_argument("--tile-begin", type=int, default=0)
a = ap.parse_args()

if a.scene == "heightfield":
    scene = G.Scene.heightfield(a.width, a.height, quads=a.quads, seed=1)
else:
    scene = {"readme": G.Scene.readme, "readme_glass": G.Scene.readme_glass, "cornell": G.Scene.cornell}[a.scene](
        a.width, a.height)
names = ["paths", "camera_samples", "closest_rays", "shadow_rays", "any_panic", "windows",
         "cyc_start_pixel", "cyc_issue_first_scatter", "cyc_traversal", "cyc_hit_processing",
         "cyc_barrier_walk", "issued", "d_over_dmax", "cyc_7"]
with G.Renderer(scene, kernel=a.kernel, occupancy=a.occupancy, lanes_per_wave=a.tiles_per_wave) as r:
    rd = abi.render_desc(a.spp, a.spp, max_depth=a.max_depth, tile_begin=a.tile_begin, tile_stride=a.tile_stride)
    for i in range(a.reps):
        t0 = time.perf_counter()
        r.render_async(rd)
        st = r.synchronize()
        dt = time.perf_counter() - t0
        out = (C.c_uint64 * 81)()
        n = G.lib().pbrt_gpu_counters(C.c_void_p(r.h), out, 81)
        vals = dict(zip(names, list(out)[:14]))
        dh = list(out)[14:n]
        tot = sum(vals[k] for k in names[6:11]) or 1
        print(f"rep {i}: {dt * 1e3:.1f} ms kernel {st.kernel_ms:.1f} ms chain {st.chain_ms:.1f} ms "
              f"kernel={st.kernel} Mpaths/s={st.paths_traced / dt / 1e6:.2f}")
        px = a.width * a.height / a.tile_stride   # pixels rendered (about, for a tile sample)
        print("  windows/pixel %.2f" % (vals["windows"] / px))
        dh, busy, odd = dh[:64], (dh[64] if len(dh) > 64 else 0), (dh[66] if len(dh) > 66 else 0)
        if odd:
            print("  odd on-chain draw counts: %.1f%%" % (100.0 * odd / max(1, sum(dh))))
        if busy and vals["windows"]:
            print("  lane utilisation (lane-steps tracing / steps x 64) %.3f" % (busy / (vals["windows"] * 64.0)))
        onchain = sum(dh)
        if onchain:
            print("  issued candidates/pixel %.1f, on-chain/pixel %.1f (%.1f%%), on-chain D above the tail "
                  "cap's dmax: %d" % (vals["issued"] / px, onchain / px, 100.0 * onchain / max(vals["issued"], 1),
                                      vals["d_over_dmax"]))
            mean_d = sum((2 * b + 1) * c for b, c in enumerate(dh)) / onchain
            print("  on-chain D histogram (bin = D // 2; mean D ~ %.1f): %s" % (
                mean_d, json.dumps({2 * b: c for b, c in enumerate(dh) if c})))
        sc_ = (C.c_uint64 * 8)()
        G.lib().pbrt_gpu_step_cycles(sc_, 8, 1)
        tot_s = sum(sc_[:5])
        print("  step cycles (raw): " + " ".join(str(int(v)) for v in sc_))
        if tot_s:
            labels = ["loop top", "closest hit + SI", "BSDF setup", "light sampling", "BSDF sample+spawn+RR"]
            print("  step regions: " + ", ".join(f"{l} {v / tot_s * 100:.1f}%" for l, v in zip(labels, sc_[:5])))
        tt = sum(sc_[5:8])
        if tt:   # the steptime build records the traversal regions on their own
            print("  closest-hit traversal: node walk %.1f%%, leaf tests %.1f%%, interaction %.1f%%" % tuple(
                v / tt * 100 for v in sc_[5:8]))
        for k in names[6:11]:
            print(f"  {k:16s} {vals[k] / tot * 100:5.1f}%  {vals[k] / px:10.0f} cyc/pixel")
