#!/usr/bin/env python3
"""Benchmark of the MI355X hot path on BASELINE.json's headline workload.

One step = one full frame of config B: the README sphere scene
(internal/render/server.go:29-164) at 1920x1080, Stratified(8,8) (63 traced
paths per pixel: sample 0 is never traced, sampler.go:29-34), Path(maxDepth 10,
rr 1, Uniform), 16-px tiles, EXACT mode (the reference's per-tile RNG replayed
bit for bit). Inputs (scene, BVH) are resident on the GPU before timing.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: one process per GPU; tiles are sharded t -> rank (t mod N) and the
per-rank fp64 XYZ films are summed on rank 0 with one RCCL reduce (the
additive Film.MergeFilmTile, film.go:115-132). Total work is fixed -> "strong".

Prints ONE JSON line on rank 0 (value = Mpaths/s over all GPUs).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-pbrt_amd"))

METRIC = ("Mpaths/s (samples×pixels/s) at 1920×1080, 64 spp; 1/2/4/8-GPU scaling + HBM GB/s vs "
          "roofline")
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 vector peak (datasheet, an FMA = 2 FLOP); the path is fp64-VALU bound
# the parity build forbids contraction (-ffp-contract=off: Go evaluates a*b+c as
# two rounded ops), so the attainable add/mul issue rate is half the FMA peak
FP64_PEAK_NOFMA_TFLOPS = FP64_PEAK_TFLOPS / 2
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=0, help="0 = the config's (1920, or 3840 for E)")
    ap.add_argument("--height", type=int, default=0, help="0 = the config's (1080, or 2160 for E)")
    ap.add_argument("--shard", default="", help="R/N: on ONE GPU, render only tiles t mod N == R, the share of "
                                                "rank R of an N-GPU job (reported as such)")
    ap.add_argument("--config", default="B", choices=["B", "C", "D", "E", "G", "H", "F", "N"],
                    help="BASELINE config: B = README sphere scene, Stratified(8,8), Path(10); "
                         "C = Cornell (SURVEY 8(d)), Stratified(16,16), Path(8); "
                         "D = 999 698-triangle height field (extension), Stratified(8,8), Path(10); "
                         "E = 9 999 392-triangle height field, 3840x2160, Stratified(32,32), Path(10); "
                         "G = README scene + server.go's commented-out glass sphere + a mirror, "
                         "Stratified(8,8), Path(10); serial-kernel cases: H = DirectLighting(10) through "
                         "server.go's glass sphere, F = B with BoxFilter radius 1.5, N = B with 2 sampled dims")
    ap.add_argument("--spp", type=int, default=0, help="Stratified(spp, spp) (0 = the config's)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "serial", "wave", "wavefront", "wave_ci"])
    ap.add_argument("--tiles-per-wave", type=int, default=0, help="k_chain_ci tiles per wave (0 = library default)")
    ap.add_argument("--occupancy", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0 = nproc / 8, the host's share per GPU of an 8-GPU node, "
                         "capped by the CPUs this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="exact", choices=["exact", "throughput"],
                    help="mode of the headline line (exact = the reference's per-tile RNG, bit-exact)")
    ap.add_argument("--no-side-mode", action="store_true",
                    help="skip the extra frames in the other mode (reported under side_mode)")
    ap.add_argument("--no-rpc", action="store_true",
                    help="skip the per-request leg (rpc: fresh scene + context + frame + film download + RGBA8)")
    return ap.parse_args()


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def host_cpu():
    """nproc, the affinity mask, the cgroup CPU quota and the CPU model of this host."""
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    quota = None   # CPUs' worth of time the cgroup grants (cgroup v2 cpu.max), if limited
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return {"nproc": nproc, "affinity": affinity, "cgroup_cpus": quota, "cpu_model": model}


def cpu_rate(sc, rd_kwargs, threads, seconds):
    """Oracle Mpaths/s on `threads` threads over an evenly spread tile sample of
    the frame (bit-reversed stride-64 batches: every prefix is spread over the
    frame), stopping after `seconds` of wall time or the whole frame."""
    import oracle_lib as O
    from pbrtgpu import abi

    n_tiles = int(O.lib().oracle_num_tiles(sc.desc, abi.render_desc(**rd_kwargs)))
    stride = 64
    offsets = [int(format(i, "06b")[::-1], 2) for i in range(stride)]
    paths = tiles = 0
    t0 = time.perf_counter()
    for off in offsets:
        rd = abi.render_desc(**dict(rd_kwargs, tile_begin=off, tile_stride=stride))
        rc, _, st = O.render(sc.desc, rd, threads=threads)
        if rc != 0:
            raise RuntimeError(f"oracle rc {rc}")
        paths += st.paths
        tiles += st.tiles
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    what = "the whole frame" if tiles == n_tiles else \
        f"{tiles} of {n_tiles} tiles of the same frame (evenly spread, stride {stride})"
    return paths / dt / 1e6, f"{what}: {paths} paths in {dt:.2f} s on {threads} threads"


def effective_cpus(cpu):
    """CPUs this process can actually run on: the affinity mask, capped by the
    cgroup's CPU quota (cgroup v2 cpu.max) when there is one."""
    eff = cpu["affinity"]
    if cpu["cgroup_cpus"]:
        eff = min(eff, max(1, int(cpu["cgroup_cpus"])))
    return eff


def cpu_baseline(args, scene_name, rd_kwargs, W, H, product_scene=None, gpus_per_host=8):
    """The oracle (C restatement of the Go path, oracle/) on the same frame's
    tiles, on this box's host CPUs (one worker per host core).

    The threads are the per-GPU share of the node (nproc / 8: the node has 8
    GPUs), capped by what this process may use (min of the affinity mask and
    the cgroup quota). Where the cap binds, the per-GPU share cannot be timed
    here: the line says so and adds a linear extrapolation (labelled as one).
    When the box grants more CPUs than the share, a second timing on all of
    them is added under `all_granted`."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O

    cpu = host_cpu()
    eff = effective_cpus(cpu)
    if scene_name in ("heightfield", "readme_glass", "readme_glass1", "readme_filter15"):
        # scene data: the oracle renders the product-built descriptor
        sc = product_scene
    else:
        sc = (O.OracleScene.readme if scene_name == "readme" else O.OracleScene.cornell)(W, H)
    node_share = max(1, cpu["nproc"] // gpus_per_host)
    share = args.cpu_threads or min(node_share, eff)
    budget = args.cpu_seconds / 2
    v_share, s_share = cpu_rate(sc, rd_kwargs, share, budget)
    capped = share < node_share
    out = {
        "value": v_share,
        "unit": "Mpaths/s",
        "cores": share,
        "kind": "port",
        "nproc": cpu["nproc"],
        "affinity": cpu["affinity"],
        "cgroup_cpus": cpu["cgroup_cpus"],
        "effective_cpus": eff,
        "cpu_model": cpu["cpu_model"],
        "per_core": v_share / share,
        "sample": f"{s_share}; "
                  + (f"the node's per-GPU share is nproc {cpu['nproc']} / {gpus_per_host} GPUs = {node_share} CPUs, "
                     f"but this box grants {eff} (affinity {cpu['affinity']}, cgroup quota {cpu['cgroup_cpus']}): "
                     f"timed on all {share} granted CPUs" if capped else
                     f"the per-GPU share of the host: nproc {cpu['nproc']} / {gpus_per_host} GPUs")
                  + "; oracle/ C restatement of the Go path, which has no Go per-op heap allocation, so it is "
                    "expected to be faster than go-pbrt",
    }
    if capped:
        out["per_gpu_share"] = {"cpus": node_share, "value_extrapolated": v_share / share * node_share,
                                "note": f"linear extrapolation of the {share}-CPU timing to the node's per-GPU "
                                        f"share ({node_share} CPUs); not measured"}
    elif eff > share:
        v_all, s_all = cpu_rate(sc, rd_kwargs, eff, budget)
        out["all_granted"] = {"value": v_all, "unit": "Mpaths/s", "cores": eff, "per_core": v_all / eff,
                              "sample": s_all + f" (all {eff} CPUs this box grants)"}
    return out


def roofline(scene_name, W, H, S, paths_per_launch, kernel_kind, kern_ms, chain_ms, paths_ms, merge_ms,
             mode="exact"):
    """Roofline of the dominant kernel, priced in ALGORITHMIC fp64 FLOPs: the
    reference's own arithmetic per path, counted by the FLOP-accounting oracle
    (profiles/flops_*.json, tools/count_flops.py) x the paths of one launch,
    over the kernel's duration measured here with HIP events on its stream.

    WAVE pipeline: k_chain is dominant; what it must reproduce per path is
    the trajectory (everything but light sampling: flops_trajectory_per_path).
    Its speculative, discarded trajectories are not algorithmic work, so they
    lower `frac` -- that is the point of the measure."""
    fl = load_json(os.path.join(REPO, "profiles", f"flops_{scene_name}_{W}x{H}_s{S}x{S}.json"))
    if not fl:
        return None
    pmc = load_json(os.path.join(REPO, "profiles", f"pmc_{scene_name}_{W}x{H}_s{S}x{S}.json")) or {}
    total = fl["flops_per_path"] * paths_per_launch
    if mode == "throughput" and kernel_kind == 2:   # no chain: k_paths<true> runs the whole path
        algo, name, ms = total, "k_paths_mb", paths_ms
    elif kernel_kind in (2, 3, 4) and chain_ms > 0:   # PBRT_KERNEL_WAVE / _WAVEFRONT / _WAVE_CI
        algo = fl.get("flops_trajectory_per_path", fl["flops_per_path"]) * paths_per_launch
        name, ms = {2: "k_chain", 3: "wf_chain", 4: "k_chain_ci"}[kernel_kind], chain_ms
    else:
        algo, name, ms = total, "k_render_exact", kern_ms
    achieved = algo / (ms / 1e3) / 1e12
    return {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS,
            # the add/mul peak the no-contraction parity build can reach
            "peak_nofma": FP64_PEAK_NOFMA_TFLOPS, "frac_nofma": achieved / FP64_PEAK_NOFMA_TFLOPS,
            "kernel": name, "kernel_ms": ms, "flops_per_launch": algo,
            "flops_source": f"profiles/flops_{scene_name}_{W}x{H}_s{S}x{S}.json",
            **pmc_fields(pmc, name, ms, kern_ms),
            "pipeline": {"kernels_ms": kern_ms, "k_paths_ms": paths_ms, "merge_ms": merge_ms,
                         "achieved_tflops": total / (kern_ms / 1e3) / 1e12,
                         "flops_per_path": fl["flops_per_path"]}}


def pmc_fields(pmc, name, ms, frame_ms):
    """`traffic` and the north_star's "HBM GB/s vs peak" from the PMC passes
    (profiles/pmc_*.json: rocprofv3 FETCH_SIZE / WRITE_SIZE runs of the same
    bench command, tools/pmc_traffic.py), named by the library build they
    measured: `traffic_same_build` says whether that is the build running now.
    `traffic` is the kernel family's stage bytes per steady-state frame: the
    sum over its launches of one frame (the N=1 chain stage is two concurrent
    k_chain_ci launches), against the stage time `ms`."""
    stages = pmc.get("stages") or {}
    traffic = (stages.get(name) or {}).get("hbm_bytes_per_frame")
    frame_bytes = sum(v.get("hbm_bytes_per_frame", 0) for v in stages.values())
    pmc_build = pmc.get("build_id")
    return {"traffic": traffic,
            "traffic_unit": "HBM bytes per frame of the stage (PMC FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
            "traffic_instantiations": (stages.get(name) or {}).get("instantiations"),
            "traffic_source": pmc.get("source"), "traffic_build_id": pmc_build,
            "traffic_same_build": bool(pmc_build) and pmc_build == BUILD_ID,
            "hbm": {"kernel_gbs": traffic / (ms / 1e3) / 1e9 if traffic else None,
                    "frame_gbs": frame_bytes / (frame_ms / 1e3) / 1e9 if frame_bytes else None,
                    "peak_gbs": HBM_PEAK_GBS,
                    "kernel_frac": traffic / (ms / 1e3) / 1e9 / HBM_PEAK_GBS if traffic else None}}


BUILD_ID = None   # pbrt_gpu_build_id() of the loaded library (set in main)


CONFIGS = {
    # BASELINE.json configs[1]: internal/render/server.go:29-164 verbatim
    "B": dict(scene="readme", spp=8, max_depth=10,
              text="README sphere scene {W}x{H}, Stratified({S},{S}) = {T} traced paths/px, "
                   "Path(maxDepth 10, rr 1, Uniform), tile 16"),
    # BASELINE.json configs[2]: SURVEY 8(d) Cornell fixture
    "C": dict(scene="cornell", spp=16, max_depth=8,
              text="Cornell 6 disks + 2 spheres {W}x{H}, Stratified({S},{S}) = {T} traced paths/px, "
                   "Path(maxDepth 8, rr 1, Uniform), tile 16"),
    # BASELINE.json configs[3] on one GPU: the triangle extension (include/pbrt_scene.h)
    "D": dict(scene="heightfield", quads=707, spp=8, max_depth=10,
              text="height field 999698 triangles (device LBVH) + README lights/camera {W}x{H}, "
                   "Stratified({S},{S}) = {T} traced paths/px, Path(maxDepth 10, rr 1, Uniform), tile 16"),
    # BASELINE.json configs[4] (8 GPUs): the same generator at 2236 x 2236 quads, 4K, 1024 spp
    "E": dict(scene="heightfield", quads=2236, spp=32, max_depth=10, width=3840, height=2160,
              text="height field 9999392 triangles (device LBVH) + README lights/camera {W}x{H}, "
                   "Stratified({S},{S}) = {T} traced paths/px, Path(maxDepth 10, rr 1, Uniform), tile 16"),
    # the README scene with server.go:67-91's commented-out glass sphere and a mirror
    "G": dict(scene="readme_glass", spp=8, max_depth=10,
              text="README sphere scene + glass sphere (server.go:67-91) + mirror sphere {W}x{H}, "
                   "Stratified({S},{S}) = {T} traced paths/px, Path(maxDepth 10, rr 1, Uniform), tile 16"),
    # The reference behaviours that run on the serial kernel, at 1080p:
    # H: server.go:160's commented-out DirectLighting(UniformSampleAll, 10) with the
    #    commented-out glass sphere (server.go:67-94)
    "H": dict(scene="readme_glass1", spp=8, max_depth=10, integrator="direct",
              text="README sphere scene + glass sphere (server.go:67-94) {W}x{H}, Stratified({S},{S}) = {T} traced "
                   "samples/px, DirectLighting(UniformSampleAll, maxDepth 10), tile 16"),
    # F: config B with a BoxFilter of radius 1.5 (film.go:211-248: 4-9 film pixels per sample)
    "F": dict(scene="readme_filter15", spp=8, max_depth=10,
              text="README sphere scene {W}x{H}, BoxFilter radius 1.5, Stratified({S},{S}) = {T} traced paths/px, "
                   "Path(maxDepth 10, rr 1, Uniform), tile 16"),
    # N: config B with Stratified(8, 8, false, 2): two sampled dimensions (stratified.go:12-19)
    "N": dict(scene="readme", spp=8, max_depth=10, n_dims=2,
              text="README sphere scene {W}x{H}, Stratified({S},{S}) with 2 sampled dimensions = {T} traced "
                   "paths/px, Path(maxDepth 10, rr 1, Uniform), tile 16"),
}


def make_scene(G, cfg, W, H):
    if cfg["scene"] == "readme":
        return G.Scene.readme(W, H)
    if cfg["scene"] == "readme_glass":
        return G.Scene.readme_glass(W, H)
    if cfg["scene"] == "readme_glass1":
        return G.Scene.readme_glass(W, H, mirror=False)
    if cfg["scene"] == "readme_filter15":
        s = G.Scene.readme(W, H)
        s.set_film(W, H, filter_radius=(1.5, 1.5))
        return s.build(2)
    if cfg["scene"] == "cornell":
        return G.Scene.cornell(W, H)
    return G.Scene.heightfield(W, H, quads=cfg["quads"], seed=1)


def mesh_roofline(cfg, W, H, S, mode, stats_ms, paths, rays_closest, rays_shadow):
    """HBM roofline of the mesh traversal, priced on the REFERENCE's rays: the
    frame's closest-hit queries beyond the camera ray (the chain's on-chain
    trajectories and the path stage trace exactly these; the camera ray is
    traced once per pixel by k_wf_primary) and its visibility rays, each at
    the bytes one reference walk fetches (nodes x 32 B + triangles x 36 B,
    the path stage's per-walk means, counted by tools/count_mesh_bytes.py into
    profiles/meshbytes_*.json), over the dominant stage's time measured here
    with HIP events. The chain's speculative off-chain walks are not
    algorithmic work: they lower `frac`."""
    mb = load_json(os.path.join(REPO, "profiles", f"meshbytes_heightfield{cfg['quads']}_{W}x{H}_s{S}x{S}_{mode}.json"))
    if not mb:
        return None
    pmc = load_json(os.path.join(REPO, "profiles", f"pmc_heightfield{cfg['quads']}_{W}x{H}_s{S}x{S}.json")) or {}
    cand = [("k_chain_ci", stats_ms["chain"]), ("k_paths_ci", stats_ms["paths"])] if mode == "exact" else \
        [("k_paths_ci_mb", stats_ms["paths"])]
    name, ms = max(cand, key=lambda x: x[1])
    ref = mb["kernels"].get("k_paths_ci") or {}
    if "closest" not in ref or ms <= 0:
        return None
    per_closest = ref["closest"]["nodes_per_walk"] * mb["bytes_per_node"] + \
        ref["closest"]["triangles_per_walk"] * mb["bytes_per_triangle"]
    anyw = ref.get("any") or {"nodes_per_walk": 0.0, "triangles_per_walk": 0.0}
    per_any = anyw["nodes_per_walk"] * mb["bytes_per_node"] + anyw["triangles_per_walk"] * mb["bytes_per_triangle"]
    traced_closest = max(rays_closest - paths, 0.0)   # the camera ray's query is per pixel on the device
    if name == "k_chain_ci":   # the trajectories: closest-hit walks only
        algo = traced_closest * per_closest
    else:
        algo = traced_closest * per_closest + rays_shadow * per_any
    achieved = algo / (ms / 1e3) / 1e9
    # the same pricing with every reference closest-hit query, the per-sample camera
    # ray included (the reference traces it per sample; the device once per pixel)
    algo_cam = (rays_closest * per_closest if name == "k_chain_ci"
                else rays_closest * per_closest + rays_shadow * per_any)
    fam = {"k_chain_ci": "k_chain_ci", "k_paths_ci": "k_paths_ci", "k_paths_ci_mb": "k_paths_ci"}[name]
    pf = pmc_fields(pmc, fam, ms, stats_ms["kernels"])
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, **pf, "kernel": name, "kernel_ms": ms,
            "bytes_per_launch": algo,
            "frac_incl_camera_rays": algo_cam / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
            "algorithmic": {"reference_closest_walks_beyond_camera": traced_closest,
                            "reference_shadow_walks": rays_shadow,
                            "bytes_per_closest_walk": per_closest, "bytes_per_shadow_walk": per_any,
                            "source": f"profiles/meshbytes_heightfield{cfg['quads']}_{W}x{H}_s{S}x{S}_{mode}.json "
                                      f"(k_paths_ci per-walk means)"},
            "kernel_walks": {q: {"nodes": k[q]["nodes_per_walk"], "triangles": k[q]["triangles_per_walk"],
                                 "walks": k[q]["walks"]}
                             for kn, k in mb["kernels"].items() for q in ("closest", "any") if q in k
                             and kn == name.replace("_mb", "")},
            "pipeline": {"kernels_ms": stats_ms["kernels"], "k_chain_ms": stats_ms["chain"],
                         "k_paths_ms": stats_ms["paths"]}}


class GpuBackend:
    """One process per GPU: torch owns the device, RCCL (the "nccl" backend)
    reduces the films over xGMI, the renderer's stream is ordered after
    torch's current stream before every frame."""

    def __init__(self, local):
        import torch
        self.torch = torch
        self.local = local
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.rstream = None

    def init_process_group(self):
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=self.dev)   # RCCL over xGMI

    def zeros(self, shape):
        return self.torch.zeros(shape, dtype=self.torch.float64, device=self.dev)

    def attach(self, renderer):
        # the renderer launches on its own non-blocking HIP stream
        self.rstream = self.torch.cuda.ExternalStream(renderer.stream(), device=self.dev)

    def order(self):
        # everything queued on torch's stream (the film's zero fill, the previous
        # frame's RCCL reduce, which dist.reduce made torch's stream wait for)
        # precedes the frame
        self.rstream.wait_stream(self.torch.cuda.current_stream(self.dev))

    def synchronize(self):
        self.torch.cuda.synchronize()

    def barrier(self, world):
        if world > 1:
            import torch.distributed as dist
            dist.barrier(device_ids=[self.local])

    def tensor(self, vals):
        return self.torch.tensor(vals, dtype=self.torch.float64, device=self.dev)


def rpc_leg(G, cfg, W, H, rd, local, args, steady_ms):
    """What the reference's caller pays per request: internal/render/server.go:29-164
    builds the scene, the integrator and (through the cgo shim) a renderer for
    every RPC, renders one frame and writes the image. Timed here end to end on
    the host clock: scene construction (host BVH build), pbrt_gpu_create, one
    frame through pbrt_gpu_render (which includes the device-to-host film copy)
    and pbrt_film_to_rgba8 (Film.WriteImage's pixel conversion). Two requests:
    `cold` with the process-wide schedule cache emptied (the first request a
    process serves: the cold-frame probe schedules it) and `cached` (a later
    request: it starts from the schedule the bench's own context measured)."""
    out = {}
    for label in ("cached", "cold"):
        if label == "cold":
            G.schedule_cache_clear()
        t0 = time.perf_counter()
        scene = make_scene(G, cfg, W, H)
        t1 = time.perf_counter()
        r = G.Renderer(scene, device=local, kernel=args.kernel, lanes_per_wave=args.tiles_per_wave,
                       occupancy=args.occupancy)
        t2 = time.perf_counter()
        film, st = r.render(rd)
        t3 = time.perf_counter()
        G.film_to_rgba8(film)
        t4 = time.perf_counter()
        src = r.schedule_source()
        r.close()
        out[label] = {"rpc_ms": (t4 - t0) * 1e3, "scene_ms": (t1 - t0) * 1e3, "create_ms": (t2 - t1) * 1e3,
                      "render_ms": (t3 - t2) * 1e3, "frame_kernels_ms": st.kernel_ms, "chain_ms": st.chain_ms,
                      "rgba8_ms": (t4 - t3) * 1e3, "schedule": src}
    out["rpc_ms"] = out["cached"]["rpc_ms"]
    out["cached_frame_over_steady"] = out["cached"]["render_ms"] / steady_ms if steady_ms else None
    out["note"] = ("per request of internal/render/server.go: scene + pbrt_gpu_create + pbrt_gpu_render (frame + "
                   "D2H film copy) + pbrt_film_to_rgba8, host wall clock; `cached`: a fresh context that starts "
                   "from the process-wide schedule cache; `cold`: the cache emptied (the probe schedules it)")
    return out


def make_step(renderer, backend, film, rd, world):
    """One frame: the rank's shard into its full-size film, then (N > 1) one
    SUM reduce of the films onto rank 0 -- the additive MergeFilmTile."""
    import torch.distributed as dist

    def step():
        backend.order()
        renderer.render_async(rd, film.data_ptr())
        st = renderer.synchronize()
        if world > 1:
            dist.reduce(film, dst=0, op=dist.ReduceOp.SUM)
        return st
    return step


def timed(step, backend, world, rank, steps, warmup, label="exact", log=sys.stderr):
    """W untimed warmup frames, then K frames bracketed by barrier +
    synchronize on both sides; elapsed is the MAX over ranks, paths the SUM."""
    import torch.distributed as dist

    for i in range(warmup):
        st = step()
        if rank == 0:
            print(f"[bench] {label} warmup {i}: kernels {st.kernel_ms:.0f} ms", file=log, flush=True)
    backend.barrier(world)
    backend.synchronize()
    t0 = time.perf_counter()
    stats = []
    for i in range(steps):
        stats.append(step())
        if rank == 0:   # progress on stderr (long frames: config E); stdout holds the one JSON line
            print(f"[bench] {label} step {i}: kernels {stats[-1].kernel_ms:.0f} ms", file=log, flush=True)
    backend.synchronize()
    backend.barrier(world)
    elapsed = time.perf_counter() - t0
    paths_local = sum(int(s.paths_traced) for s in stats)
    agg = backend.tensor([elapsed, float(paths_local)])
    if world > 1:
        mx = agg.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = agg.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, paths_total = float(mx[0]), float(sm[1])
    else:
        paths_total = float(paths_local)
    return elapsed, paths_local, paths_total, stats


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    import torch.distributed as dist

    backend = GpuBackend(local)

    import pbrtgpu as G

    global BUILD_ID
    BUILD_ID = G.build_id()
    cfg = CONFIGS[args.config]
    W, H = args.width or cfg.get("width", 1920), args.height or cfg.get("height", 1080)
    shard_r, shard_n = rank, world
    if args.shard:
        if world > 1:
            raise SystemExit("--shard is a one-GPU simulation of a rank; not under torch.distributed")
        shard_r, shard_n = (int(x) for x in args.shard.split("/"))
    S = args.spp or cfg["spp"]
    rd_kwargs = dict(spp_x=S, spp_y=S, max_depth=cfg["max_depth"])
    if cfg.get("integrator") == "direct":
        rd_kwargs["integrator"] = G.abi.PBRT_INTEGRATOR_DIRECT_LIGHTING
    if "n_dims" in cfg:
        rd_kwargs["n_dims"] = cfg["n_dims"]
    scene = make_scene(G, cfg, W, H)
    # the renderer (and its two HIP streams) before RCCL's own streams, so the
    # heavy/light chain launches get hardware queues of their own
    renderer = G.Renderer(scene, device=local, kernel=args.kernel, lanes_per_wave=args.tiles_per_wave,
                          occupancy=args.occupancy)
    if world > 1:
        backend.init_process_group()
    modes = {"exact": G.abi.PBRT_MODE_EXACT, "throughput": G.abi.PBRT_MODE_THROUGHPUT}
    film = backend.zeros((H, W, 3))
    backend.attach(renderer)

    def rd_of(mode):
        return G.render_desc(**rd_kwargs, tile_begin=shard_r, tile_stride=shard_n, mode=modes[mode])

    # cold frame: a fresh context's first frame (no schedule learned yet), as
    # internal/render/server.go pays it when it builds a scene per RPC
    backend.barrier(world)
    backend.synchronize()
    t0 = time.perf_counter()
    first = make_step(renderer, backend, film, rd_of(args.mode), world)()
    backend.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    if world > 1:
        fm = backend.tensor([first_ms])
        dist.all_reduce(fm, op=dist.ReduceOp.MAX)
        first_ms = float(fm[0])

    elapsed, paths_local, paths_total, stats = timed(make_step(renderer, backend, film, rd_of(args.mode), world),
                                                     backend, world, rank, args.steps, args.warmup, args.mode)
    kern_ms = sum(s.kernel_ms for s in stats) / len(stats)
    merge_ms = sum(s.merge_ms for s in stats) / len(stats)
    chain_ms = sum(s.chain_ms for s in stats) / len(stats)
    paths_ms = sum(s.paths_ms for s in stats) / len(stats)
    kernel_kind = int(stats[0].kernel)
    rays_c = sum(int(s.rays_closest) for s in stats)
    rays_s = sum(int(s.rays_shadow) for s in stats)
    side = None
    if not args.no_side_mode:
        other = "throughput" if args.mode == "exact" else "exact"
        e2, _, p2, st2 = timed(make_step(renderer, backend, film, rd_of(other), world), backend, world, rank,
                               2, 1, other)
        side = {"mode": other, "value": p2 / e2 / 1e6, "unit": "Mpaths/s", "ms_per_step": e2 / 2 * 1e3,
                "chain_ms": sum(s.chain_ms for s in st2) / 2, "k_paths_ms": sum(s.paths_ms for s in st2) / 2,
                "note": "THROUGHPUT = one PCG32 stream per (pixel, sample): same arithmetic, statistically "
                        "(not bitwise) the reference image; EXACT is the headline"}

    rpc = None
    if world == 1 and not args.no_rpc:
        rpc = rpc_leg(G, cfg, W, H, rd_of(args.mode), local, args, elapsed / args.steps * 1e3)

    if rank == 0:
        value = paths_total / elapsed / 1e6
        if cfg.get("integrator") or "n_dims" in cfg or cfg["scene"] == "readme_filter15":
            roof = None   # no algorithmic-FLOP count of these variants (profiles/flops_* are B, C, G)
        elif cfg["scene"] == "heightfield":
            roof = mesh_roofline(cfg, W, H, S, args.mode, {"chain": chain_ms, "paths": paths_ms, "kernels": kern_ms},
                                 paths_local / len(stats), rays_c / len(stats), rays_s / len(stats))
        else:
            roof = roofline(cfg["scene"], W, H, S, paths_local / len(stats), kernel_kind, kern_ms, chain_ms,
                            paths_ms, merge_ms, args.mode)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "timed_region": "render_async_into a device-resident film + synchronize per frame (inputs resident "
                            "in HBM); the 50 MB device-to-host film copy of pbrt_gpu_render is excluded here and "
                            "included in rpc.*.render_ms",
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": {"readme": "synthetic (the reference's hard-coded README scene; no external data)",
                     "cornell": "synthetic (SURVEY 8(d) Cornell fixture built from reference types)",
                     "heightfield": "synthetic (procedural height field, seed 1; triangle extension)",
                     "readme_glass": "synthetic (README scene + server.go's commented-out glass sphere + a mirror)",
                     "readme_glass1": "synthetic (README scene + server.go's commented-out glass sphere)",
                     "readme_filter15": "synthetic (the README scene with a radius-1.5 box filter)",
                     }[cfg["scene"]],
            "config": {
                "workload": cfg["text"].format(W=W, H=H, S=S, T=S * S - 1) + ", "
                            + ("EXACT per-tile RNG" if args.mode == "exact" else "THROUGHPUT per-path RNG"),
                "baseline_config": args.config,
                "width": W, "height": H, "spp": S * S, "traced_spp": S * S - 1, "max_depth": cfg["max_depth"],
                "paths_per_frame": int(paths_total / args.steps), "mode": args.mode,
                "parallelism": f"tiles mod {world}" + (" + RCCL film reduce" if world > 1 else "")
                               + (f"; ONE GPU rendering rank {shard_r}'s shard of {shard_n} (tiles t mod {shard_n} == "
                                  f"{shard_r})" if args.shard else ""),
                "kernel": {1: "serial", 2: "wave", 3: "wavefront", 4: "wave_ci", 5: "wave_dl"}.get(kernel_kind, "?"),
            },
            "pipeline_ms": {"kernels": kern_ms, "chain": chain_ms, "paths": paths_ms, "merge": merge_ms},
            # nominal W*H*spp, and the reference's ray segments counted in-kernel
            # (closest-hit queries of Path.Li's loop + visibility rays; pbrt_gpu_stats.rays_*)
            "nominal_samples_per_frame": W * H * S * S,
            "rays": {"closest_per_frame": rays_c / len(stats) * (world if world > 1 else 1),
                     "shadow_per_frame": rays_s / len(stats) * (world if world > 1 else 1),
                     "per_s": (rays_c + rays_s) * (world if world > 1 else 1) / elapsed,
                     "unit": "rays/s", "note": "reference ray segments (rank 0's count x N for N > 1)"},
            "build_id": BUILD_ID,
            "first_frame_ms": first_ms,
            "first_frame_chain_ms": first.chain_ms,
            "roofline": roof,
        }
        if side:
            out["side_mode"] = side
        if rpc:
            out["rpc"] = rpc
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline(args, cfg["scene"], rd_kwargs, W, H, scene)
            cb["gpu_over_cpu"] = value / cb["value"]
            if "per_gpu_share" in cb:
                cb["per_gpu_share"]["gpu_over_cpu_extrapolated"] = value / cb["per_gpu_share"]["value_extrapolated"]
            if "all_granted" in cb:
                cb["all_granted"]["gpu_over_cpu"] = value / cb["all_granted"]["value"]
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    renderer.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
