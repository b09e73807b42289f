"""CPU dry run of bench.py's N > 1 code (gloo, world size 2).

bench.py's multi-GPU frame is make_step (stream ordering, the rank's shard
render into its full-size film, one SUM reduce onto rank 0) driven by timed
(warmup, barrier + synchronize brackets, MAX elapsed and SUM paths over ranks).
Here the same two functions run under torch.distributed with the gloo backend;
the GPU backend is swapped for a CPU one (same methods, no streams) and the
renderer for one that renders the rank's shard with the oracle, the same tile
subset bench.py hands the device (tiles t mod N == rank). Checked: rank 0's
reduced film is the full frame (bit-exact where one rank owns every covering
tile, fp64 association order elsewhere), paths are summed, elapsed is the max
over ranks, and every rank ran the same number of frames and reduces.
"""
import ctypes as C
import json
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from pbrtgpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP = 48, 40, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class CpuBackend:
    """bench.GpuBackend's interface on the CPU (gloo): no streams to order."""

    def __init__(self):
        self.orders = 0

    def init_process_group(self):
        dist.init_process_group("gloo")

    def zeros(self, shape):
        return torch.zeros(shape, dtype=torch.float64)

    def attach(self, renderer):
        pass

    def order(self):
        self.orders += 1

    def synchronize(self):
        pass

    def barrier(self, world):
        if world > 1:
            dist.barrier()

    def tensor(self, vals):
        return torch.tensor(vals, dtype=torch.float64)


class Stats:
    def __init__(self, st, ms):
        self.paths_traced = st.paths
        self.kernel_ms = ms
        self.merge_ms = self.chain_ms = self.paths_ms = 0.0
        self.kernel = 1


class OracleShardRenderer:
    """pbrtgpu.Renderer's render_async / synchronize over the oracle: the film
    at film_device_ptr is overwritten with the shard's merged XYZ, as
    k_merge_film overwrites the device film."""

    def __init__(self, scene, rank):
        self.sc = scene
        self.rank = rank
        self.pending = None

    def render_async(self, rd, film_ptr):
        t0 = time.perf_counter()
        rc, film, st = O.render(self.sc.desc, rd, threads=2)
        assert rc == 0
        dst = np.ctypeslib.as_array((C.c_double * film.size).from_address(film_ptr))
        dst[:] = film.ravel()
        if self.rank == 1:
            time.sleep(0.05)   # rank 1 is slower: elapsed must be the max over ranks
        self.pending = Stats(st, (time.perf_counter() - t0) * 1e3)

    def synchronize(self):
        st, self.pending = self.pending, None
        return st


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, REPO)
    import bench

    backend = CpuBackend()
    backend.init_process_group()
    try:
        sc = O.OracleScene.readme(W, H)
        renderer = OracleShardRenderer(sc, rank)
        film = backend.zeros((H, W, 3))
        backend.attach(renderer)
        rd = abi.render_desc(SPP, SPP, tile_begin=rank, tile_stride=world)
        step = bench.make_step(renderer, backend, film, rd, world)
        t0 = time.perf_counter()
        elapsed, paths_local, paths_total, stats = bench.timed(step, backend, world, rank, 3, 1, "exact",
                                                               log=open(os.devnull, "w"))
        wall = time.perf_counter() - t0
        res = {"elapsed": elapsed, "paths_local": paths_local, "paths_total": paths_total, "frames": len(stats),
               "orders": backend.orders, "wall": wall}
        json.dump(res, open(os.path.join(out_dir, f"rank{rank}.json"), "w"))
        if rank == 0:
            np.save(os.path.join(out_dir, "reduced.npy"), film.numpy())
        backend.barrier(world)
    finally:
        dist.destroy_process_group()


def test_bench_multi_rank_branch_gloo(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    sc = O.OracleScene.readme(W, H)
    rc, full, st = O.render(sc.desc, abi.render_desc(SPP, SPP), threads=2)
    assert rc == 0
    # paths: each rank its shard, the SUM over ranks is the frame's, per timed frame
    assert sum(r["paths_local"] for r in res) == 3 * st.paths
    assert all(r["paths_total"] == 3 * st.paths for r in res)
    # elapsed: the MAX over ranks (rank 1 sleeps in every frame), the same on every rank
    assert res[0]["elapsed"] == res[1]["elapsed"] >= 3 * 0.05
    # 1 warmup + 3 timed frames, each ordered after the torch stream and reduced
    assert all(r["frames"] == 3 and r["orders"] == 4 for r in res)
    # rank 0 holds the reduced film of the LAST frame: the full frame
    reduced = np.load(tmp_path / "reduced.npy")
    np.testing.assert_allclose(reduced, full, rtol=1e-14, atol=0)
    shard_films = [O.render(sc.desc, abi.render_desc(SPP, SPP, tile_begin=r, tile_stride=world), threads=2)[1]
                   for r in range(world)]
    owners = sum((f != 0).any(axis=2).astype(int) for f in shard_films)
    assert np.array_equal(reduced[owners <= 1], full[owners <= 1])
