"""Scene builders shared by the tests and tests/golden/make_golden.py (host-side
pbrt_sb_* builder only: no GPU needed to build a scene)."""
import numpy as np

import pbrtgpu as G


def material_scene(kind="both", w=32, h=24, rough=0.0, area=True, kt=(0.5, 0.5, 0.5), sigma=0.0,
                   glass_kr=(0.5, 0.5, 0.5)):
    """A floor, a glass sphere, a mirror sphere and a matte sphere, lit by a
    point light and an area-light sphere. kind: "both" | "matte" (the two
    special spheres matte) | "black" (the two special spheres black matte)."""
    s = G.Scene()
    chk = s.add_checker((0.2, 0, 0), (0, 0, 0.2), 0, 0, (1, 1, 1), (0.18, 0.18, 0.18))
    floor = s.add_disk(G.rotate(0, 90), 0.0, 100.0)
    s.add_primitive(floor, chk)
    red = s.add_matte((0.6, 0.1, 0.1), sigma=sigma)
    if kind == "both":
        glass = s.add_glass(kr=glass_kr, kt=kt, u_roughness=rough, v_roughness=0.5 * rough)   # server.go:80-87
        mirror = s.add_mirror()
    elif kind == "matte":
        glass = mirror = s.add_matte((0.5, 0.5, 0.5))
    else:
        glass = mirror = s.add_matte((0.0, 0.0, 0.0))
    for (x, z, m) in ((-2.5, 0.0, glass), (2.5, 0.0, mirror), (0.0, -4.0, red)):
        sph = s.add_sphere(G.translate(0, 0, 0), 2.0)
        s.add_primitive(sph, m, G.translate(x, 2.0, z))
    if area:
        light = s.add_sphere(G.translate(0, 9, 2), 0.75)
        s.add_area_light((6, 6, 6), light)
    s.add_point_light(G.translate(-6, 10, 8), (60, 60, 60))
    s.set_film(w, h)
    s.set_camera(G.look_at((0, 7, 12), (0, 1.5, 0), (0, 1, 0)), fov=55)
    return s.build(max_prims_in_node=1)


def mesh_material_scene(material, w=40, h=32):
    """A small triangle mesh (a tilted 4x4-quad grid) made of `material`
    ("glass" | "mirror" | "oren"), over the checker floor, beside a matte
    sphere; include/pbrt_gpu.h lets a mesh take any material."""
    s = G.Scene()
    chk = s.add_checker((0.2, 0, 0), (0, 0, 0.2), 0, 0, (1, 1, 1), (0.18, 0.18, 0.18))
    s.add_primitive(s.add_disk(G.rotate(0, 90), 0.0, 100.0), chk)
    m = {"glass": lambda: s.add_glass(), "mirror": lambda: s.add_mirror(),
         "oren": lambda: s.add_matte((0.5, 0.6, 0.4), sigma=30.0)}[material]()
    n = 4
    xs = np.linspace(-3.0, 3.0, n + 1)
    p = np.array([(x, 1.0 + 0.4 * x + 0.3 * z, z) for z in xs for x in xs], dtype=np.float32)
    idx = []
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i, (j + 1) * (n + 1) + i + 1
            idx += [(a, b, d), (a, d, c)]
    s.add_mesh(p, np.array(idx, dtype=np.int32), m)
    s.add_primitive(s.add_sphere(G.translate(0, 0, 0), 1.5), s.add_matte((0.6, 0.1, 0.1)), G.translate(0, 1.5, -4))
    s.add_point_light(G.translate(-6, 10, 8), (60, 60, 60))
    s.add_area_light((6, 6, 6), s.add_sphere(G.translate(0, 9, 2), 0.75))
    s.set_film(w, h)
    s.set_camera(G.look_at((0, 7, 12), (0, 1.5, 0), (0, 1, 0)), fov=55)
    return s.build(max_prims_in_node=1)
