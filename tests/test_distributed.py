"""Multi-process sharding of a frame, on CPU with gloo.

bench.py / the multi-GPU path: rank r renders tiles t with t mod N == r into a
full-frame fp64 XYZ film and the films are summed on rank 0 with one reduce
(the additive Film.MergeFilmTile, film.go:115-132). Here the per-rank render
is the oracle (the device path's shards are checked bit-exact against the
oracle in test_gpu_parity.py::test_tile_shards_sum_to_full_frame), so this
test covers the process-group plumbing and the reduction semantics:

  * every shard film equals the oracle's render of that shard, bit for bit;
  * the reduced film equals the single-process frame up to fp64 association
    order at pixels covered by tiles of different ranks (rtol 1e-14), and
    exactly everywhere else.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from pbrtgpu import abi

W, H = 48, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir, spp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = O.OracleScene.readme(W, H)
        rd = abi.render_desc(spp, spp, tile_begin=rank, tile_stride=world)
        rc, film, st = O.render(sc.desc, rd, threads=2)
        assert rc == 0
        np.save(os.path.join(out_dir, f"shard{rank}.npy"), film)
        t = torch.from_numpy(film.copy())
        dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        paths = torch.tensor([float(st.paths)], dtype=torch.float64)
        dist.all_reduce(paths, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.save(os.path.join(out_dir, "reduced.npy"), t.numpy())
            np.save(os.path.join(out_dir, "paths.npy"), paths.numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_tile_shards_reduce_to_full_frame(tmp_path, world):
    spp = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path), spp), nprocs=world, join=True,
                       start_method="spawn")
    sc = O.OracleScene.readme(W, H)
    rc, full, st = O.render(sc.desc, abi.render_desc(spp, spp), threads=2)
    assert rc == 0
    reduced = np.load(tmp_path / "reduced.npy")
    assert float(np.load(tmp_path / "paths.npy")[0]) == st.paths == W * H * (spp * spp - 1)
    np.testing.assert_allclose(reduced, full, rtol=1e-14, atol=0)
    # pixels covered by one rank's tiles only are bit-exact
    shards = [np.load(tmp_path / f"shard{r}.npy") for r in range(world)]
    owners = sum((s != 0).any(axis=2).astype(int) for s in shards)
    single = owners <= 1
    assert np.array_equal(reduced[single], full[single])
    # and each shard is the oracle's own render of that tile subset
    for r in range(world):
        rc, want, _ = O.render(sc.desc, abi.render_desc(spp, spp, tile_begin=r, tile_stride=world), threads=2)
        assert rc == 0 and np.array_equal(shards[r], want)
