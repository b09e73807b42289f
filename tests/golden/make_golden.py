"""Generates tests/golden/*.npz from the CPU oracle (oracle/, pinned by the
reference's own known-answer tests in tests/test_reference_kats.py).

These are build-generated golden vectors, not reference-generated: go-pbrt has
no Go toolchain in this image and no render-level goldens of its own (SURVEY
§4, §8c). Re-run after an intentional oracle change:
    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
import oracle_lib as O  # noqa: E402
from pbrtgpu import abi  # noqa: E402

CASES = {
    # name: (scene, w, h, render_desc kwargs)
    "readme_64x64_s2x2_path": ("readme", 64, 64, dict(spp_x=2, spp_y=2)),
    "readme_48x32_s4x4_path": ("readme", 48, 32, dict(spp_x=4, spp_y=4)),
    "readme_64x48_s2x2_direct": ("readme", 64, 48, dict(spp_x=2, spp_y=2,
                                                       integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING)),
    "readme_40x24_s3x2_jitter": ("readme", 40, 24, dict(spp_x=3, spp_y=2, jitter=True)),
    "cornell_48x32_s2x2_path8": ("cornell", 48, 32, dict(spp_x=2, spp_y=2, max_depth=8)),
}


def render_case(name):
    scene, w, h, kw = CASES[name]
    sc = O.OracleScene.readme(w, h) if scene == "readme" else O.OracleScene.cornell(w, h)
    rd = abi.render_desc(**kw)
    rc, film, st = O.render(sc.desc, rd, threads=4)
    assert rc == 0, (name, rc)
    return film, st


def pcg_vectors():
    out = {}
    import ctypes as C
    for seed in (0, 1, 8159):
        buf = (C.c_uint32 * 16)()
        O.lib().oracle_pcg_stream(seed, 16, buf)
        out[str(seed)] = list(buf)
    return out


def main():
    commit = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    meta = {"generator": "tests/golden/make_golden.py", "oracle_commit": commit, "cases": {}}
    for name in CASES:
        film, st = render_case(name)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), film=film)
        meta["cases"][name] = {"sha256": hashlib.sha256(film.tobytes()).hexdigest(), "paths": int(st.paths),
                               "scene": CASES[name][0], "w": CASES[name][1], "h": CASES[name][2],
                               "render": {k: (int(v) if isinstance(v, bool) else v) for k, v in CASES[name][3].items()}}
    meta["pcg32_first16"] = pcg_vectors()
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(CASES), "cases")


if __name__ == "__main__":
    main()
