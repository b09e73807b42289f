"""The reference interface's edge cases on the GPU: every descriptor field the
README scene leaves at its default, rendered device vs oracle bit for bit on
the serial kernel and on whatever kernel the auto route picks (asserted).

- partial spheres: zMin / zMax / phiMax (sphere.go:105-135), incl. rays whose
  near hit is clipped and fall through to t1, and the shadowed phi (:127);
- disks with innerRadius and phiMax (disk.go:64-126);
- a thin-lens camera (lensRadius > 0, camera.go:192-242; with stratified dims
  pLens is (0, 0), #3; with none it comes from the RNG per sample);
- a film crop window and a non-unit screen window (film.go:42-76,
  camera.go:106-124);
- BoxFilter radius 0.5, 1.5 and 2 (film.go:211-248: 1, 4 or 9+ pixels per sample);
- a two-sided area light (diffuse.go:36-41) on a reversed light sphere;
- negative-scale (handedness-swapping) transforms: go-pbrt never sets
  transformSwapsHandedness (sphere.go:19-32, disk.go:22-35), so
  reverseOrientation != transformSwapsHandedness (interaction.go:179-181) is
  reverseOrientation alone while the transformed normals flip.

No reference test covers these fields; the oracle's restatement of them is the
checker ("parity unpinned" against Go itself, as for every render-level test).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def edge_scene(w=48, h=32, partial=False, disk_edges=False, lens=0.0, focal=10.0, crop=(0, 0, 1, 1),
               screen=None, filter_radius=1.0, two_sided=None, neg_scale=False):
    """A floor, three spheres, a point light and an area-light sphere; the flags
    switch on one edge case each (see the module docstring)."""
    s = G.Scene()
    chk = s.add_checker((0.2, 0, 0), (0, 0, 0.2), 0, 0, (1, 1, 1), (0.18, 0.18, 0.18))
    red, green, blue = s.add_matte((0.7, 0.1, 0.1)), s.add_matte((0.1, 0.7, 0.1)), s.add_matte((0.1, 0.1, 0.7))
    if disk_edges:
        # the floor with a hole and a missing sector, and an upright ring with a gap
        floor = s.add_disk(G.rotate(0, 90), 0.0, 30.0, inner=3.0, phi_max=300.0)
        s.add_primitive(floor, chk)
        ring = s.add_disk(G.mul(G.translate(0, 3, -4), G.rotate(2, 30)), 0.0, 4.0, inner=1.5, phi_max=250.0)
        s.add_primitive(ring, green)
        under = s.add_disk(G.rotate(0, 90), -0.5, 40.0)   # seen through the hole
        s.add_primitive(under, blue)
    else:
        floor = s.add_disk(G.rotate(0, 90), 0.0, 100.0)
        s.add_primitive(floor, chk)
    if partial:
        # z axis up (RotateX(-90)); a cap cut off at z = 1.2 shows the inside (t1)
        cap = s.add_sphere(G.rotate(0, -90), 2.0, z_min=-1.0, z_max=1.2, phi_max=270.0)
        s.add_primitive(cap, red, G.translate(-2.5, 2.0, 0.0))
        band = s.add_sphere(G.rotate(0, -90), 2.0, z_min=-0.6, z_max=0.9, phi_max=200.0, reverse=True)
        s.add_primitive(band, green, G.translate(2.5, 2.0, 0.0))
    else:
        for (x, m) in ((-2.5, red), (2.5, green)):
            sph = s.add_sphere(G.translate(0, 0, 0), 2.0)
            s.add_primitive(sph, m, G.translate(x, 2.0, 0.0))
    if neg_scale:
        # mirrored TransformedPrimitive and a mirrored object-to-world
        sph = s.add_sphere(G.scale(1, 1, -1), 1.5)
        s.add_primitive(sph, blue, G.mul(G.translate(0.0, 1.5, -4.0), G.scale(-1, 1, 1)))
        # an upright disk facing the camera (one Mul: Transform.Mul's inverse
        # order, #18, commutes here since the translation has no x part)
        d = s.add_disk(G.mul(G.translate(0, 1.0, 3), G.scale(-1, 1, 1)), 0.0, 1.0)
        s.add_primitive(d, red)
    else:
        sph = s.add_sphere(G.translate(0, 0, 0), 1.5)
        s.add_primitive(sph, blue, G.translate(0.0, 1.5, -4.0))
        d = s.add_disk(G.translate(0, 1.0, 3), 0.0, 1.0)
        s.add_primitive(d, red)
    if two_sided is None:
        light = s.add_sphere(G.translate(0, 9, 2), 0.75)
        s.add_area_light((6, 6, 6), light)
    else:
        # a reversed light sphere: one-sided it faces inwards (dark), two-sided it shines
        light = s.add_sphere(G.translate(0, 9, 2), 0.75, reverse=True)
        s.add_area_light((6, 6, 6), light, two_sided=two_sided)
    s.add_point_light(G.translate(-6, 10, 8), (60, 60, 60))
    s.set_film(w, h, crop=crop, filter_radius=(filter_radius, filter_radius))
    cam = G.look_at((0, 6, 14), (0, 1.5, 0), (0, 1, 0))
    if screen is None:
        s.set_camera(cam, lens=lens, focal=focal, fov=55)
    else:
        s.set_camera(cam, screen=screen, lens=lens, focal=focal, fov=55)
    return s.build(max_prims_in_node=1)


def check(sc, rd, expect_auto):
    """device (serial and auto) vs oracle, bit-exact; expect_auto: the kernel the auto route must take"""
    rc, of, _ = O.render(sc.desc, rd, threads=min(16, os.cpu_count() or 1))
    assert rc == 0 and np.isfinite(of).all()
    for kernel in ("serial", "auto"):
        with G.Renderer(sc, kernel=kernel) as r:
            film, st = r.render(rd)
        want = abi.PBRT_KERNEL_SERIAL if kernel == "serial" else expect_auto
        assert st.kernel == want, (kernel, st.kernel)
        assert np.array_equal(bits(film), bits(of)), kernel
    return of


PATH_RD = dict(max_depth=5)
DL_RD = dict(integrator=abi.PBRT_INTEGRATOR_DIRECT_LIGHTING, max_depth=5)
PATH_AUTO, DL_AUTO = abi.PBRT_KERNEL_WAVE_CI, abi.PBRT_KERNEL_WAVE_DL


@pytest.mark.parametrize("integ", ["path", "dl"])
def test_partial_spheres(integ):
    sc = edge_scene(partial=True)
    kw, auto = (PATH_RD, PATH_AUTO) if integ == "path" else (DL_RD, DL_AUTO)
    of = check(sc, abi.render_desc(3, 3, **kw), auto)
    full = edge_scene()
    _, ff, _ = O.render(full.desc, abi.render_desc(3, 3, **kw), threads=8)
    assert not np.array_equal(of, ff)   # the clipping is in view


@pytest.mark.parametrize("integ", ["path", "dl"])
def test_disk_inner_radius_and_phi_max(integ):
    sc = edge_scene(disk_edges=True)
    kw, auto = (PATH_RD, PATH_AUTO) if integ == "path" else (DL_RD, DL_AUTO)
    of = check(sc, abi.render_desc(3, 3, **kw), auto)
    assert of.max() > 0


@pytest.mark.parametrize("n_dims", [4, 2, 1, 0])
def test_thin_lens_camera(n_dims):
    """lensRadius > 0: with stratified dims pLens = (0, 0) maps to a fixed lens
    point (ConcentricSampleDisk(0, 0) = -(cos, sin)(pi/4)); with n_dims 0 or 1
    every sample draws its own lens point from the RNG (serial kernel only)."""
    sc = edge_scene(lens=0.4, focal=12.0)
    auto = PATH_AUTO if n_dims >= 2 else abi.PBRT_KERNEL_SERIAL
    of = check(sc, abi.render_desc(3, 3, n_dims=n_dims, **PATH_RD), auto)
    pin = edge_scene()
    _, pf, _ = O.render(pin.desc, abi.render_desc(3, 3, n_dims=n_dims, **PATH_RD), threads=8)
    assert not np.array_equal(of, pf)


def test_thin_lens_direct_lighting():
    sc = edge_scene(lens=0.4, focal=12.0)
    check(sc, abi.render_desc(2, 2, n_dims=4, **DL_RD), DL_AUTO)
    # n_dims 1: pLens comes from the RNG, so the camera ray is per sample: serial
    check(sc, abi.render_desc(2, 2, n_dims=1, **DL_RD), abi.PBRT_KERNEL_SERIAL)


@pytest.mark.parametrize("crop,screen", [((0.25, 0.1, 0.8, 0.9), None),
                                         ((0, 0, 1, 1), (-1.5, -1.0, 1.5, 1.0)),
                                         ((0.3, 0.2, 0.95, 0.7), (-0.8, -0.5, 1.2, 0.9))])
def test_crop_and_screen_window(crop, screen):
    """CroppedPixelBounds from the crop window (film.go:42-76) offsets every tile
    and pixel; the screen window changes RasterToCamera (camera.go:106-124)."""
    sc = edge_scene(w=64, h=40, crop=crop, screen=screen)
    W = sc.desc.film.crop_max_x - sc.desc.film.crop_min_x
    H = sc.desc.film.crop_max_y - sc.desc.film.crop_min_y
    if crop != (0, 0, 1, 1):
        assert (W, H) != (64, 40) and sc.desc.film.crop_min_x > 0
    for kw, auto in ((PATH_RD, PATH_AUTO), (DL_RD, DL_AUTO)):
        of = check(sc, abi.render_desc(2, 2, **kw), auto)
        assert of.shape == (H, W, 3)


@pytest.mark.parametrize("radius", [0.5, 1.3, 1.5, 2.0, 2.7])
def test_filter_radius(radius):
    """BoxFilter radius r: a sample at the pixel corner covers a footprint of
    2x2 (r < 1.5), 4x4 (1.5 <= r < 2.5) or 6x6 film pixels; the tile films'
    aprons grow with r. k_film runs every radius below the tile size."""
    sc = edge_scene(filter_radius=radius)
    check(sc, abi.render_desc(2, 2, **PATH_RD), PATH_AUTO)
    check(sc, abi.render_desc(2, 2, **DL_RD), DL_AUTO)
    check(sc, abi.render_desc(3, 2, n_dims=2, **PATH_RD), PATH_AUTO)


def test_two_sided_area_light():
    """DiffuseAreaLight.L (diffuse.go:36-41): on a reversed light sphere the
    sampled point's normal faces away, so one-sided it adds nothing and
    two-sided it lights the scene."""
    one, two = edge_scene(two_sided=False), edge_scene(two_sided=True)
    for kw, auto in ((PATH_RD, PATH_AUTO), (DL_RD, DL_AUTO)):
        f1 = check(one, abi.render_desc(2, 2, **kw), auto)
        f2 = check(two, abi.render_desc(2, 2, **kw), auto)
        assert f2.sum() > f1.sum()


@pytest.mark.parametrize("integ", ["path", "dl"])
def test_negative_scale_transforms(integ):
    sc = edge_scene(neg_scale=True)
    assert all(sc.desc.shapes[i].transform_swaps_handedness == 0 for i in range(sc.desc.n_shapes))
    kw, auto = (PATH_RD, PATH_AUTO) if integ == "path" else (DL_RD, DL_AUTO)
    of = check(sc, abi.render_desc(3, 3, **kw), auto)
    if integ == "path":
        # the mirrored shading frames (ss from the transformed dpdu) change the
        # local-frame bounce directions (#7)
        plain = edge_scene()
        _, pf, _ = O.render(plain.desc, abi.render_desc(3, 3, **kw), threads=8)
        assert not np.array_equal(of, pf)


def test_all_edges_at_once_throughput_mode():
    """Every edge case in one scene, THROUGHPUT mode (its own streams, same arithmetic)."""
    sc = edge_scene(partial=True, disk_edges=True, lens=0.3, crop=(0.1, 0.05, 0.9, 1.0),
                    screen=(-1.2, -0.9, 1.3, 1.0), two_sided=True, neg_scale=True)
    check(sc, abi.render_desc(3, 3, mode=abi.PBRT_MODE_THROUGHPUT, **PATH_RD), abi.PBRT_KERNEL_WAVE)
