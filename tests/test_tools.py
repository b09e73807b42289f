"""CPU checks of host-side helpers added in round 3: bench.py's config G scene
(README + server.go:67-91's glass sphere + a mirror) and the kernel-resource
parser of tools/kernel_resources.py (device assembly `.set` directives)."""
import importlib.util
import os
import sys

import numpy as np

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def test_config_G_scene_has_glass_and_mirror():
    bench = _load(os.path.join(REPO, "bench.py"), "bench_for_test")
    cfg = bench.CONFIGS["G"]
    assert cfg["scene"] == "readme_glass" and cfg["spp"] == 8 and cfg["max_depth"] == 10
    sc = bench.make_scene(G, cfg, 48, 32)
    base = G.Scene.readme(48, 32)
    d, b = sc.desc, base.desc
    assert d.n_prims == b.n_prims + 2 and d.n_materials == b.n_materials + 2
    kinds = {d.materials[i].type for i in range(d.n_materials)}
    assert {abi.PBRT_MAT_GLASS, abi.PBRT_MAT_MIRROR} <= kinds
    # the oracle renders the product-built descriptor (scene data); glass changes the image
    rd = abi.render_desc(2, 2, max_depth=5)
    rc, fg, _ = O.render(d, rd, threads=4)
    rc2, fb, _ = O.render(b, rd, threads=4)
    assert rc == rc2 == 0 and np.isfinite(fg).all() and not np.array_equal(fg, fb)


def test_kernel_resources_parser(tmp_path):
    kr = _load(os.path.join(REPO, "tools", "kernel_resources.py"), "kernel_resources_for_test")
    sym = "_ZN12_GLOBAL__N_110k_chain_ciILi1ELi0ELb0EEEvN4pbrt8DevSceneE"
    callee = "_ZN4pbrt7path_liE"
    asm = (f"\t.set {callee}.num_vgpr, 200\n"
           f"\t.set {sym}.num_vgpr, max(128, {callee}.num_vgpr)\n"
           f"\t.set {sym}.num_agpr, 0\n"
           f"\t.set {sym}.numbered_sgpr, 100\n"
           f"\t.amdhsa_kernel {sym}\n"
           "\t\t.amdhsa_group_segment_fixed_size 6640\n"
           "\t\t.amdhsa_private_segment_fixed_size 28\n"
           "\t.end_amdhsa_kernel\n")
    p = tmp_path / "k.s"
    p.write_text(asm)
    kr._cache.clear()
    assert kr.resolve(asm, sym + ".num_vgpr") == 200
    out_file = tmp_path / "out.json"
    import io
    import json
    from contextlib import redirect_stdout
    buf = io.StringIO()
    sys.argv = ["kernel_resources.py", str(p)]
    with redirect_stdout(buf):
        kr.main()
    res = json.loads(buf.getvalue())
    (name, v), = res.items()
    assert name.startswith("k_chain_ci<1, 0, false>")
    assert v == {"arch_vgpr": 200, "acc_vgpr": 0, "sgpr": 100, "scratch_bytes_per_lane": 28,
                 "lds_static_bytes": 6640, "waves_per_simd_by_registers": 2}
    out_file.write_text(buf.getvalue())
