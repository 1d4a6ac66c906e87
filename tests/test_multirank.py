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


def _c2_small():
    from python_motion_planning_amd import workloads as wl

    return wl.c2_workload(nq=72, W=96, H=96, pair_seed=11)


def _c5_small():
    from python_motion_planning_amd import workloads as wl

    return wl.c5_workload(nq=40, first_seed=100)


def _plan2d(s, g, occ):
    import torch

    from oracle import oracle as O

    r = O.astar2d_batch(occ, s, g, path_cap=2048, nthreads=1)
    return {k: torch.as_tensor(r[k]) for k in ("cost", "status", "n_expanded", "path_len", "path")}


def _plan3d(s, g, occ):
    import torch

    from oracle import oracle as O

    cost, st = O.astar3d_batch(occ, s, g, nthreads=1)
    return {"cost": torch.as_tensor(cost), "status": torch.as_tensor(st)}


def _sharded_main(rank, world, port, outdir):
    """One rank of the strong-scaling path (shard.run_sharded): lpt_deal share -> the per-rank planner
    (the oracle standing in for this rank's GPU) -> all_gather_rows into input order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from python_motion_planning_amd import shard

    dist = shard.init("gloo")
    occ, s, g = _c2_small()
    r2 = shard.run_sharded(dist, lambda a, b: _plan2d(a, b, occ), s, g)
    occ3, s3, g3 = _c5_small()
    r3 = shard.run_sharded(dist, lambda a, b, occ: _plan3d(a, b, occ), s3, g3, per_query={"occ": occ3})
    mine = shard.lpt_deal(shard.octile(s, g), world, rank)
    np.savez(os.path.join(outdir, f"sharded{rank}.npz"), mine=mine,
             **{"c2_" + k: v.numpy() for k, v in r2.items()}, **{"c5_" + k: v.numpy() for k, v in r3.items()})
    dist.destroy_process_group()


def test_two_ranks_run_sharded_gather(tmp_path):
    """world-size-2 gloo ranks through shard.run_sharded (lpt_deal + all_gather_rows): every rank's
    gathered records equal one single-process run's, in input order, for a C2-style batch (96^2
    grid, 72 queries) and a C5 batch (per-query 3D grids, 40 queries)."""
    world = 2
    mp.start_processes(_sharded_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    z = [np.load(tmp_path / f"sharded{r}.npz") for r in range(world)]
    occ, s, g = _c2_small()
    ref2 = {k: v.numpy() for k, v in _plan2d(s, g, occ).items()}
    occ3, s3, g3 = _c5_small()
    ref3 = {k: v.numpy() for k, v in _plan3d(s3, g3, occ3).items()}
    assert (ref2["status"] == 0).all() and (ref3["status"] == 0).all()
    for r in range(world):
        for k, v in ref2.items():
            assert np.array_equal(z[r]["c2_" + k], v), (r, k)
        for k, v in ref3.items():
            assert np.array_equal(z[r]["c5_" + k], v), (r, k)
    # the deal really split the batch: disjoint, covering, both ranks busy
    m0, m1 = z[0]["mine"], z[1]["mine"]
    assert len(m0) and len(m1) and not set(m0) & set(m1) and len(m0) + len(m1) == len(s)


def test_single_process_defaults(monkeypatch):
    from python_motion_planning_amd import shard

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert shard.env_rank() == (0, 1, 0)
    assert shard.init("gloo") is None
    assert shard.max_over_ranks(None, [1.5, 2]) == [1.5, 2.0]


def _bench_json(*argv):
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=300, env=env, cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_flag_spawns_ranks(n):
    """`python bench.py --gpus N --scaling strong` (no torch.distributed.run around it) starts N ranks
    itself; the strong-scaling deal + all_gather over those ranks reproduces the single-rank records
    for every strong-scaling workload: the C2 batch, the C5 batch (BASELINE config 5: queries sharded
    over the GPUs) and the C4 agents (config 4: sharded by agent), DWA and LQR steps."""
    out = _bench_json("--gpus", str(n), "--dry-run", "--scaling", "strong")
    assert out["n_gpus"] == n and out["scaling"] == "strong"
    assert out["gathered_equal"] == {"c2": True, "c5": True, "c4_dwa": True, "c4_lqr": True}
    assert out["gathered_equal_single_rank"] is True


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=repo)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_lpt_deal_and_local_gather():
    import torch

    from python_motion_planning_amd import shard

    work = np.array([5.0, 1.0, 9.0, 3.0, 7.0, 2.0, 8.0])
    parts = [shard.lpt_deal(work, 3, r) for r in range(3)]
    # the longest three go one to each rank, then the next three, ...
    assert sorted(np.concatenate(parts).tolist()) == list(range(7))
    assert [sorted(work[p].tolist(), reverse=True)[0] for p in parts] == [9.0, 8.0, 7.0]
    assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1
    # octile distance: max + (sqrt2 - 1) min in 2D
    assert np.allclose(shard.octile(np.array([[0, 0]]), np.array([[3, 4]])), [4 + (np.sqrt(2) - 1) * 3])
    idx = np.array([4, 0, 2])
    g = shard.all_gather_rows(None, idx, {"v": torch.tensor([40.0, 0.5, 20.0])}, 5)
    assert g["v"].tolist() == [0.5, 0.0, 20.0, 0.0, 40.0]
