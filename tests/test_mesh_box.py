"""The mesh walk's float32 box test (go-pbrt_amd/csrc/pbrt_mesh.h,
mesh_box32_hit, build option PBRT_MESH_F32) against the float64 slab test it
stands in for (mesh_box_hit): on random, aimed, grazing, axis-parallel,
far-origin/tiny-box, origin-on-face and origin-off-face rays, and TMax within
ulps of the entry distance, every box the float64 test keeps is kept (a few
more are: a node visit, never a different closest hit). Rays with a nonzero
|d_i| outside [1e-30, 1e30] run the float64 test. CPU only (g++ on the
product header)."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_float32_box_test_keeps_every_float64_box(tmp_path):
    exe = tmp_path / "mbc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Werror",
                    "-Wno-unknown-pragmas", "-o", str(exe), os.path.join(REPO, "tests", "mesh_box_check.cpp")],
                   check=True)
    r = subprocess.run([str(exe), "200000"], capture_output=True, text=True)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout
    fams = {line.split()[0]: {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", line)}
            for line in r.stdout.splitlines() if "cases=" in line}
    assert set(fams) == {"random", "aimed", "tmax_at_entry", "grazing", "axis_parallel", "far_small",
                         "tiny_huge_dir", "origin_on_face", "origin_ulps_off_face"}
    for name, f in fams.items():
        assert f["bad"] == 0, name
    # the families exercise what they name
    assert fams["aimed"]["kept64"] > 100000
    assert fams["tmax_at_entry"]["extra32"] > 0 and fams["tmax_at_entry"]["kept64"] > 0
    assert fams["tiny_huge_dir"]["f64path"] == fams["tiny_huge_dir"]["cases"]
    assert fams["grazing"]["f64path"] > 0
    # the widening is small: the float32 test keeps few boxes the float64 test culls
    assert fams["random"]["extra32"] <= fams["random"]["cases"] // 1000
