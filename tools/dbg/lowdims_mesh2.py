"""Debug: which chain configurations break n_dims = 1 on the mesh scene."""
import os, sys, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1:   # child: one configuration
    sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
    import numpy as np
    import oracle_lib as O
    import pbrtgpu as G
    from pbrtgpu import abi
    name, nd = sys.argv[1], int(sys.argv[2])
    sc = {"hf_sph": lambda: G.Scene.heightfield(48, 32, quads=24, seed=1, spheres=True),
          "hf": lambda: G.Scene.heightfield(48, 32, quads=24, seed=1),
          "readme": lambda: G.Scene.readme(96, 64),
          "cornell": lambda: G.Scene.cornell(96, 64)}[name]()
    rd = abi.render_desc(4, 4, n_dims=nd)
    with G.Renderer(sc) as r:
        film, st = r.render(rd)
    rc, of, ost = O.render(sc.desc, rd, threads=8)
    bad = (film.view(np.uint64) != of.view(np.uint64)).any(axis=2)
    print(f"{name} nd={nd} env={os.environ.get('DBG_ENV','')} kernel={st.kernel} bad px {int(bad.sum())}", flush=True)
    sys.exit(0)
for env in ("", "PBRT_CI_STRIDE=1", "PBRT_CI_WAVES=4", "PBRT_CI_ORDER=0", "PBRT_CULL_GROUPS=0"):
    for name in ("hf_sph", "hf", "readme", "cornell"):
        for nd in (1, 2):
            e = dict(os.environ, DBG_ENV=env)
            if env:
                k, v = env.split("=")
                e[k] = v
            subprocess.run([sys.executable, __file__, name, str(nd)], env=e, timeout=120)
