"""The cgo shim (integration/go/pbrtgpu/pbrtgpu.go) against the C ABI.

No Go toolchain exists here, so the Go side is not compiled. This test
compiles the shim's cgo preamble with gcc and checks that every C identifier
the Go code uses (functions, types, constants, and the struct fields it sets
or reads) exists in include/pbrt_gpu.h / include/pbrt_scene.h, so the shim
cannot drift from the headers.
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM_DIR = os.path.join(REPO, "integration", "go", "pbrtgpu")
SHIMS = sorted(os.path.join(SHIM_DIR, f) for f in os.listdir(SHIM_DIR) if f.endswith(".go"))
PATCHES = os.path.join(REPO, "integration", "go", "patches")
REFERENCE = "/root/reference"
# cgo pseudo-identifiers and C scalar types, not ABI names
CGO_BUILTINS = {"GoString", "CString", "GoBytes", "int", "int32_t", "int64_t", "uint8_t", "double", "size_t",
                "uint64_t", "float", "char", "int32_t", "malloc", "free"}


def shim_parts():
    src = "\n".join(open(f).read() for f in SHIMS)
    pre = "\n".join(l[3:] for l in src.splitlines() if l.startswith("// #") and not l.startswith("// #cgo"))
    names = set(re.findall(r"\bC\.([A-Za-z_]\w*)", src)) - CGO_BUILTINS
    fields = set()
    for fn in re.split(r"\nfunc ", src):   # a `var x C.T` is scoped to its function
        for var, ty in re.findall(r"\bvar (\w+) C\.(\w+)", fn):
            for f in re.findall(r"\b%s\.(\w+)\b" % re.escape(var), fn):
                fields.add((ty, f))
    return pre, names, fields


def test_shim_identifiers_exist_in_the_headers(tmp_path):
    pre, names, fields = shim_parts()
    assert "pbrt_gpu.h" in pre and "pbrt_scene.h" in pre
    hdr = open(os.path.join(REPO, "include", "pbrt_gpu.h")).read() + open(
        os.path.join(REPO, "include", "pbrt_scene.h")).read()
    funcs = set(re.findall(r"\b(pbrt_\w+)\s*\(", hdr))
    body = []
    for n in sorted(names):
        if n.isupper() or n.startswith("PBRT_"):
            body.append(f"    (void)({n});")
        elif n in funcs:
            body.append(f"    (void)&{n};")
        else:
            body.append(f"    {{ {n}* p_ = 0; (void)p_; }}")   # opaque handles included
    for ty, f in sorted(fields):
        body.append(f"    (void)sizeof((({ty}*)0)->{f});")
    c = tmp_path / "shim_check.c"
    c.write_text(pre + "\n\nvoid shim_check(void) {\n" + "\n".join(body) + "\n}\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(REPO, "include"),
                        str(c)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert len(names) > 30 and len(fields) >= 10


def test_shim_covers_the_render_entry_points():
    _, names, _ = shim_parts()
    for n in ("pbrt_gpu_create", "pbrt_gpu_render", "pbrt_gpu_cancel", "pbrt_gpu_last_error", "pbrt_gpu_destroy",
              "pbrt_gpu_intersect", "pbrt_gpu_intersect_p", "pbrt_film_to_rgba8", "pbrt_sb_build",
              "pbrt_make_glass", "pbrt_make_mirror", "pbrt_random_sampler"):
        assert n in names, n


def test_dropin_types_cover_the_reference_interfaces():
    """pbrtgpu.Path is a pbrt.Integrator (integrator.go:12-21) with
    RenderFrame, pbrtgpu.BVH a pbrt.Aggregate (primitive.go:9-20) with batch methods;
    both embed the CPU implementation for the per-ray methods."""
    src = open(os.path.join(SHIM_DIR, "dropin.go")).read()
    assert re.search(r"type Path struct \{\s*pbrt\.Integrator", src)
    assert re.search(r"type BVH struct \{\s*\*accelerator\.BVH", src)
    assert "func (p *Path) RenderFrame(ctx context.Context, scene pbrt.Scene, tileSize int64) error" in src
    for m in ("IntersectBatch", "IntersectPBatch"):
        assert f"func (b *BVH) {m}(" in src
    for ctor in ("NewSphereShape", "NewDisk", "NewMatte", "NewCheckerMatte", "NewMirror", "NewGlass",
                 "NewGeometricPrimitive", "NewTransformedPrimitive", "NewBVH", "NewPoint", "NewDistant",
                 "NewDiffuseAreaLight", "NewScene", "NewFilm", "NewPerspectiveCamera", "NewPath"):
        assert f"func (r *Recorder) {ctor}(" in src, ctor


@pytest.mark.skipif(not os.path.isdir(REFERENCE) or not os.path.exists("/usr/bin/patch"),
                    reason="the reference checkout (or patch(1)) is not on this machine")
def test_patches_apply_to_the_reference(tmp_path):
    """integration/go/patches/*.patch apply cleanly to the reference checkout
    (dry run: nothing under /root/reference is written), and the hook patch puts
    the FrameRenderer check at the top of pbrt.Render (integrator.go:291)."""
    pats = sorted(f for f in os.listdir(PATCHES) if f.endswith(".patch"))
    assert len(pats) == 2
    for f in pats:
        r = subprocess.run(["patch", "--dry-run", "-p1", "-d", REFERENCE, "-i", os.path.join(PATCHES, f)],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    hook = open(os.path.join(PATCHES, pats[0])).read()
    assert "+\tif fr, ok := s.(FrameRenderer); ok {" in hook and "+func RenderTiles(" in hook
    server = open(os.path.join(PATCHES, pats[1])).read()
    assert "+\tdli := rec.NewPath(10, camera, sampler, pixelBounds, 1, pbrt.Uniform, 0)" in server


def test_batch_arrays_live_in_c_memory():
    """cgo forbids passing C a Go value that points at Go memory:
    pbrt_ray_soa / pbrt_hit_soa hold array pointers, so the batch methods build
    their arrays in one C.malloc'd arena, and the render watcher goroutine is
    joined before RenderFrame returns (no pbrt_gpu_cancel after Close)."""
    src = open(os.path.join(SHIM_DIR, "dropin.go")).read()
    for m in ("IntersectBatch", "IntersectPBatch"):
        body = src[src.index(f"func (b *BVH) {m}("):]
        body = body[:body.index("\n}\n")]
        assert "newArena(" in body and "defer a.free()" in body, m
        assert "make([]" not in body, m   # no Go-allocated array reaches the SoA structs
    assert "C.malloc(" in src and "C.free(" in src
    shim = open(os.path.join(SHIM_DIR, "pbrtgpu.go")).read()
    rf = shim[shim.index("func (r *Renderer) RenderFrame("):]
    rf = rf[:rf.index("\n}\n")]
    assert "<-exited" in rf and rf.index("close(done)") < rf.index("<-exited") < rf.index("switch rc")
