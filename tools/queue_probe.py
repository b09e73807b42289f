"""Does the renderer's lazily created third stream (the completion-driven path
stage's chain stream, render.hip) get a hardware queue of its own when other
streams were created after the context (RCCL's, torch's)? GPU_MAX_HW_QUEUES is
4 on the pool's boxes. Renders rank r's shard of config B (tile_begin=r,
tile_stride=N) for a few frames, optionally after creating --extra torch
streams and running a kernel on each, and prints the steady frame times.

    python tools/queue_probe.py [--extra 2] [--n 8] [--rank 5] [--frames 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-pbrt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extra", type=int, default=0)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=5)
    ap.add_argument("--frames", type=int, default=5)
    a = ap.parse_args()
    import torch
    import pbrtgpu as G
    torch.cuda.set_device(0)
    film = torch.zeros((1080, 1920, 3), dtype=torch.float64, device="cuda")
    scene = G.Scene.readme(1920, 1080)
    r = G.Renderer(scene, device=0)
    streams = []
    for _ in range(a.extra):   # as RCCL and torch create theirs after the renderer
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            (film[:1] + 1.0).sum().item()
        streams.append(s)
    rd = G.render_desc(8, 8, max_depth=10, tile_begin=a.rank, tile_stride=a.n)
    out = []
    for f in range(a.frames):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = r.render_async(rd, film.data_ptr())
        st = r.synchronize()
        out.append(round((time.perf_counter() - t0) * 1e3, 1))
    _, heavy = r.tile_ticks()
    print(json.dumps({"extra": a.extra, "n": a.n, "rank": a.rank, "frame_ms": out, "heavy": heavy,
                      "overlap_slots": r.overlap_slots()}))


if __name__ == "__main__":
    main()
