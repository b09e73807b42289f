"""Algorithmic fp64 FLOPs of a full frame, counted by the FLOP-accounting oracle
build (oracle/_build/liboracle_flops.so: every fp64 add/sub/mul/div/sqrt of the
reference algorithm that reaches an output = 1 FLOP; compare/Max/Min/abs/
Nextafter bit steps = 0). Deterministic for (scene, config); the result is
committed under profiles/ and read by bench.py for the roofline.

    python tools/count_flops.py [--scene readme|cornell --width 1920 --height 1080 --spp 8 --max-depth 10
                                 --tile-stride 1]

--tile-stride S counts every S-th tile (an evenly spread sample; per-path
figures are then sample means, stated in the output).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))
import oracle_lib as O  # noqa: E402
from pbrtgpu import abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--scene", default="readme", choices=["readme", "cornell", "readme_glass"],
                    help="readme_glass: bench.py config G (the README scene + server.go's glass sphere "
                         "+ a mirror), built by the product's scene builder (scene data only)")
    ap.add_argument("--max-depth", type=int, default=10)
    ap.add_argument("--tile-stride", type=int, default=1)
    a = ap.parse_args()
    if a.scene == "readme_glass":
        import pbrtgpu as G
        sc = G.Scene.readme_glass(a.width, a.height)
    else:
        sc = getattr(O.OracleScene, a.scene)(a.width, a.height)
    rd = abi.render_desc(a.spp, a.spp, max_depth=a.max_depth, tile_begin=0, tile_stride=a.tile_stride)
    t = time.time()
    rc, film, st = O.render(sc.desc, rd, threads=a.threads, flops=True)
    dt = time.time() - t
    assert rc == 0
    out = {
        "scene": a.scene, "width": a.width, "height": a.height, "sampler": f"Stratified({a.spp},{a.spp})",
        "integrator": f"Path({a.max_depth}, rr=1, Uniform)", "tiles": int(st.tiles), "paths": int(st.paths),
        "tile_sample": "every tile" if a.tile_stride == 1 else f"every {a.tile_stride}-th tile (tile_stride)",
        "flops": int(st.flops), "flops_per_path": st.flops / st.paths,
        "flops_light_per_path": st.flops_light / st.paths,
        "flops_trajectory_per_path": (st.flops - st.flops_light) / st.paths,
        "closest_rays_per_path": st.closest_rays / st.paths, "shadow_rays_per_path": st.shadow_rays / st.paths,
        "count_build_wall_s": dt, "threads": a.threads,
        "definition": "fp64 add/sub/mul/div/sqrt executed by the reference algorithm on values that reach "
                      "the film (oracle/_build/liboracle_flops.so)",
    }
    path = os.path.join(REPO, "profiles", f"flops_{a.scene}_{a.width}x{a.height}_s{a.spp}x{a.spp}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
