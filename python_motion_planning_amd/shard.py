"""Multi-GPU plumbing for the batched planners: one process per GPU, independent shards.

Every workload on the hot path shards trivially (independent start/goal queries, independent
agents), so there is no collective on the compute path: each rank plans its own shard.  The cross-
rank traffic is the barrier around a timed region, the max-over-ranks of its wall time, and -- for a
batch split over ranks (strong scaling, `run_sharded`) -- one all-gather of the fixed-size per-query
result records at the end.  torch.distributed supplies the process group: "nccl"
(RCCL over xGMI) on GPUs, "gloo" on CPUs for the tests.

`launch_ranks` starts the N rank processes itself when a program is run as a single process with
`--gpus N` (no torch.distributed.run around it): the parent never touches the GPU, each child gets
RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT, and the parent exits with the first
non-zero child exit code.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np


def env_rank():
    """(rank, world_size, local_rank) from the torch.distributed.run environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv=None, extra_env=None) -> int:
    """Run `python <argv>` as n rank processes on this node (one per GPU) and wait for all of them.

    Called before anything touches the GPU.  Children inherit stdout/stderr, so rank 0's output is
    the program's output.  The children are polled: on the first non-zero exit the survivors (which
    may be blocked in a collective waiting for the dead rank, up to the process-group timeout) are
    terminated, and that exit code is returned; 0 when every rank exits 0."""
    import time

    argv = list(sys.argv if argv is None else argv)
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable] + argv, env=env))
    while True:
        rcs = [p.poll() for p in procs]
        bad = [c for c in rcs if c is not None and c != 0]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(c == 0 for c in rcs):
            return 0
        time.sleep(0.05)


def init(backend: str = "nccl", always: bool = False):
    """Initialise the process group when WORLD_SIZE > 1 (or at any world size with always=True, which
    the 1-GPU tests use to drive the RCCL branch); returns the torch.distributed module or None."""
    rank, world, local = env_rank()
    if world <= 1 and not always:
        return None
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist


def shard_range(rank: int, world: int, n: int):
    """Contiguous block [lo, hi) of n items owned by `rank` (equal split, remainder to the first ranks)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def octile(starts, goals) -> np.ndarray:
    """Octile start-goal distance per query: the work estimate of a grid search."""
    d = np.abs(np.asarray(starts, np.int64) - np.asarray(goals, np.int64)).reshape(len(starts), -1)
    d.sort(axis=1)
    # 2D: max + (sqrt2 - 1) min; 3D: the same chain over the sorted axes
    w = np.array([np.sqrt(3.0) - np.sqrt(2.0), np.sqrt(2.0) - 1.0, 1.0])[-d.shape[1]:]
    return (d * w).sum(axis=1)


def lpt_deal(work, world: int, rank: int) -> np.ndarray:
    """Indices of the items rank `rank` owns when the items, sorted by descending `work` (stable),
    are dealt round-robin over `world` ranks: every rank gets the same number of long and short
    queries (longest-processing-time-first)."""
    order = np.argsort(-np.asarray(work, np.float64), kind="stable")
    return np.sort(order[rank::world])


def weak_seed(base: int, rank: int, per_rank: int = 1) -> int:
    """Seed of rank r's own shard in weak scaling (every rank a fresh batch of the same size)."""
    return base + rank * per_rank


def max_over_ranks(dist, values, device="cpu"):
    """Element-wise max of a list of floats over all ranks (identity without a process group)."""
    if dist is None:
        return [float(v) for v in values]
    import torch

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def sum_over_ranks(dist, values, device="cpu"):
    """Element-wise sum of a list of floats over all ranks (identity without a process group)."""
    if dist is None:
        return [float(v) for v in values]
    import torch

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def barrier(dist):
    if dist is not None:
        dist.barrier()


def all_gather_rows(dist, idx, rows: dict, n: int, device="cpu") -> dict:
    """Gather per-query result records from every rank into full [n, ...] tensors on every rank.

    idx: this rank's query indices (any order, disjoint across ranks, together covering 0..n-1);
    rows: name -> tensor [len(idx), ...] holding those queries' records.  One padded all_gather per
    record field (the shards differ in size by at most one row under lpt_deal); the result puts row
    k of rank r at index idx_r[k].  Without a process group the rows are scattered locally."""
    import torch

    idx_t = torch.as_tensor(np.asarray(idx, np.int64), device=device)
    out = {}
    if dist is None:
        for k, v in rows.items():
            full = torch.zeros((n,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
            full[idx_t.to(v.device)] = v
            out[k] = full
        return out
    world = dist.get_world_size()
    cnt = torch.tensor([idx_t.numel()], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    cnts = [int(c.item()) for c in cnts]
    m = max(cnts)

    def gather(t):
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=device)
        pad[: t.shape[0]] = t.to(device)
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        return torch.cat([p[:c] for p, c in zip(parts, cnts)])

    all_idx = gather(idx_t)
    for k, v in rows.items():
        g = gather(v)
        full = torch.zeros((n,) + tuple(v.shape[1:]), dtype=v.dtype, device=device)
        full[all_idx] = g
        out[k] = full
    return out


def run_sharded(dist, plan_fn, starts, goals, device="cpu", work=None, per_query=None):
    """Strong-scaling split of ONE batch of queries over the ranks of `dist`, plus the result gather.

    Each rank takes its lpt_deal share of the queries (by octile distance unless `work` is given),
    calls plan_fn(local_starts, local_goals, **local_per_query) -> dict of [n_local, ...] tensors,
    and all ranks return the full-batch records in the input order.  `per_query` holds further
    per-query inputs (e.g. C5's per-query occupancy grids), sliced like the starts.  Equal to
    plan_fn(starts, goals, **per_query) on one rank."""
    n = len(starts)
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    w = octile(starts, goals) if work is None else work
    idx = lpt_deal(w, world, rank)
    extra = {k: np.asarray(v)[idx] for k, v in (per_query or {}).items()}
    rows = plan_fn(np.asarray(starts)[idx], np.asarray(goals)[idx], **extra)
    return all_gather_rows(dist, idx, rows, n, device)
