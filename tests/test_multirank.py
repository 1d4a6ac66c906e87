"""The N>1 path on CPU: two ranks over gloo (shard queries, no data-path
collective, barrier + max-over-ranks timing, weak-scaling aggregate).  Each rank plans its own shard
with the CPU oracle standing in for its GPU; the union of the shards must equal the single-process
result, and the reduced wall time must be the slowest rank's."""
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle import oracle as O
    from python_motion_planning_amd import shard, workloads as wl

    r, w, _ = shard.env_rank()
    assert (r, w) == (rank, world)
    dist = shard.init("gloo")
    # strong-scaling split of one batch: 96 queries on a 64^2 grid
    occ = wl.random_grid(64, 64, 0.2, seed=5)
    cells = wl.largest_component_cells(occ)
    rng = np.random.default_rng(6)
    starts = cells[rng.integers(0, len(cells), 96)].astype(np.int32)
    goals = cells[rng.integers(0, len(cells), 96)].astype(np.int32)
    lo, hi = shard.shard_range(rank, world, len(starts))
    shard.barrier(dist)
    t0 = time.perf_counter()
    res = O.astar2d_batch(occ, starts[lo:hi], goals[lo:hi], path_cap=4096, nthreads=1)
    time.sleep(0.05 * (rank + 1))  # make the ranks' times differ
    shard.barrier(dist)
    mine = time.perf_counter() - t0
    (slowest,) = shard.max_over_ranks(dist, [mine])
    # weak scaling: every rank's own C2-style batch from a rank-offset pair seed
    _, s_w, g_w = wl.c2_workload(nq=8, W=64, H=64, pair_seed=shard.weak_seed(1, rank))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), lo=lo, hi=hi, cost=res["cost"], mine=mine, slowest=slowest,
             s_w=s_w, g_w=g_w)
    dist.destroy_process_group()


def test_two_ranks_gloo(tmp_path):
    from oracle import oracle as O
    from python_motion_planning_amd import shard, workloads as wl

    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    z = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    # the shards tile the batch exactly
    assert int(z[0]["lo"]) == 0 and int(z[0]["hi"]) == int(z[1]["lo"]) and int(z[1]["hi"]) == 96
    occ = wl.random_grid(64, 64, 0.2, seed=5)
    cells = wl.largest_component_cells(occ)
    rng = np.random.default_rng(6)
    starts = cells[rng.integers(0, len(cells), 96)].astype(np.int32)
    goals = cells[rng.integers(0, len(cells), 96)].astype(np.int32)
    ref = O.astar2d_batch(occ, starts, goals, path_cap=4096, nthreads=1)
    assert np.array_equal(np.concatenate([z[0]["cost"], z[1]["cost"]]), ref["cost"])
    # max over ranks is the slowest rank's time, the same on every rank
    assert float(z[0]["slowest"]) == float(z[1]["slowest"]) == max(float(z[0]["mine"]), float(z[1]["mine"]))
    # weak-scaling shards are distinct batches
    assert not np.array_equal(z[0]["s_w"], z[1]["s_w"])
    assert shard.shard_range(0, 1, 96) == (0, 96)
    assert [shard.shard_range(r, 3, 10) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]


def test_single_process_defaults(monkeypatch):
    from python_motion_planning_amd import shard

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert shard.env_rank() == (0, 1, 0)
    assert shard.init("gloo") is None
    assert shard.max_over_ranks(None, [1.5, 2]) == [1.5, 2.0]
