"""Sweep lanes_per_wave (tiles per 64-lane wave) on a 1080p frame subset."""
import sys, os, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
import pbrtgpu as G
W, H = 1920, 1080
scene = G.Scene.readme(W, H)
for lpw in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 16, 32, 64]:
    with G.Renderer(scene, lanes_per_wave=lpw) as r:
        rd = G.render_desc(8, 8)
        r.render(G.render_desc(2, 2, tile_end=64))  # warm
        t = time.time(); film, st = r.render(rd); dt = time.time() - t
    print(f"lpw={lpw:3d} kernel={st.kernel_ms:9.1f} ms  wall={dt:6.2f}s  Mpaths/s={st.paths_traced/dt/1e6:7.2f}", flush=True)
