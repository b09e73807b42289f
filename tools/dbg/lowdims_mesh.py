"""Debug: mesh scene parity under n_dims 1/2/4, path wavefront on/off, both modes."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np
import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

sc = G.Scene.heightfield(48, 32, quads=24, seed=1, spheres=True)
for wf in ("1", "0"):
    os.environ["PBRT_PATHS_WF"] = wf
    for nd in (4, 2, 1):
        for mode in (abi.PBRT_MODE_EXACT, abi.PBRT_MODE_THROUGHPUT):
            rd = abi.render_desc(4, 4, n_dims=nd, mode=mode)
            with G.Renderer(sc) as r:
                film, st = r.render(rd)
            rc, of, ost = O.render(sc.desc, rd, threads=8)
            bad = (film.view(np.uint64) != of.view(np.uint64)).any(axis=2)
            ys, xs = np.nonzero(bad)
            print(f"wf={wf} nd={nd} mode={mode} kernel={st.kernel} paths {st.paths_traced}/{ost.paths} "
                  f"bad px {bad.sum()} first {list(zip(xs[:4].tolist(), ys[:4].tolist()))}", flush=True)
