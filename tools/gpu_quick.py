"""Quick GPU bring-up: fp64 div/sqrt rounding check + README parity vs oracle."""
import sys, os, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import pbrtgpu as G
import oracle_lib as O

def run(w, h, sx, sy, integ=G.PBRT_INTEGRATOR_PATH, lpw=0, **kw):
    s = G.Scene.readme(w, h)
    rd = G.render_desc(sx, sy, integrator=integ, **kw)
    t = time.time()
    with G.Renderer(s, lanes_per_wave=lpw) as r:
        film, st = r.render(rd)
        t_gpu = time.time() - t
        t = time.time()
        rc, ofilm, ost = O.render(s.desc, rd)
        t_cpu = time.time() - t
    same = np.array_equal(film.view(np.uint64), ofilm.view(np.uint64))
    nd = int((film != ofilm).sum())
    print(f"{w}x{h} {sx}x{sy} integ={integ} lpw={lpw}: bitexact={same} ndiff={nd} gpu={t_gpu:.3f}s kern={st.kernel_ms:.1f}ms cpu={t_cpu:.2f}s paths={st.paths_traced}/{ost.paths} rc={rc}", flush=True)
    if not same:
        idx = np.argwhere(film != ofilm)[:5]
        for i in idx: print("  ", i, film[tuple(i)], ofilm[tuple(i)])
    return same

ok = run(64, 64, 2, 2)
ok &= run(256, 256, 2, 2)
ok &= run(128, 96, 4, 4, lpw=8)
ok &= run(96, 64, 2, 2, integ=G.PBRT_INTEGRATOR_DIRECT_LIGHTING)
print("ALL_OK" if ok else "MISMATCH")
