"""Occupancy timeline of config B's chain stage, from the diagnostics build's
per-slot start and end clocks (pbrt_gpu_tile_clocks, wall_clock64 at 100 MHz):
renders the frame twice on one context (the second is the steady state the
bench times: learned order, heavy/light split) and prints, for the steady
frame, the number of tiles in flight over time and the idle capacity of the
one-wave launch's slots once it stops being full -- the room a path stage
overlapped with the chain's tail could use.

    PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_diag.so python tools/tile_timeline.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
os.environ.setdefault("PBRT_GPU_LIB", os.path.join(REPO, "go-pbrt_amd", "lib", "exp", "libpbrt_gpu_diag.so"))


def main():
    import pbrtgpu as G
    L = G.lib()
    L.pbrt_gpu_tile_clocks.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int64]
    L.pbrt_gpu_tile_clocks.restype = C.c_int64
    W, H = 1920, 1080
    scene = G.Scene.readme(W, H)
    rd = G.render_desc(8, 8)
    out = {}
    with G.Renderer(scene) as r:
        for frame in range(2):
            _, st = r.render(rd)
            n = L.pbrt_gpu_tile_clocks(r.h, None, None, 0)
            assert n > 0, "not the diagnostics build (make diag)"
            s = np.zeros(n, dtype=np.uint32)
            e = np.zeros(n, dtype=np.uint32)
            L.pbrt_gpu_tile_clocks(r.h, s.ctypes.data_as(C.POINTER(C.c_uint32)),
                                   e.ctypes.data_as(C.POINTER(C.c_uint32)), n)
            _, heavy = r.tile_ticks()
            t0 = int(s.min())
            ss = (s.astype(np.int64) - t0) / 1e5   # ms (100 MHz)
            ee = (e.astype(np.int64) - t0) / 1e5
            end = float(ee.max())
            grid = np.arange(0.0, end + 1.0, 1.0)
            active = np.array([int(((ss <= t) & (ee > t)).sum()) for t in grid])
            full = int(active[: max(1, len(active) // 4)].max())   # tiles in flight while the launch is full
            t_drop = float(grid[np.argmax((active < 0.98 * full) & (grid > 10))])
            idle = float(((full - active[grid >= t_drop]).clip(min=0)).sum() / full)   # full-launch ms left idle
            out[f"frame{frame}"] = {
                "chain_ms": st.chain_ms, "heavy": heavy, "tiles": int(n), "span_ms": end,
                "in_flight_when_full": full, "drops_below_98pct_at_ms": t_drop,
                "idle_full_launch_ms_after_drop": idle,
                "busy_tile_ms_over_full": float((ee - ss).sum() / full),
                "in_flight_every_10ms": {int(t): int(a) for t, a in zip(grid[::10], active[::10])},
            }
            print(json.dumps({k: v for k, v in out[f"frame{frame}"].items() if k != "in_flight_every_10ms"}),
                  flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
