"""Multi-GPU plumbing for the batched planners: one process per GPU, independent shards.

Every workload on the hot path shards trivially (independent start/goal queries, independent
agents), so there is no collective on the data path: each rank builds and plans its own shard,
and the only cross-rank traffic is the barrier around a timed region and the max-over-ranks of
its wall time.  torch.distributed supplies the process group: "nccl" (RCCL over
xGMI) on GPUs, "gloo" on CPUs for the tests.
"""
from __future__ import annotations

import os


def env_rank():
    """(rank, world_size, local_rank) from the torch.distributed.run environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl"):
    """Initialise the process group when WORLD_SIZE > 1; returns the torch.distributed module or None."""
    rank, world, local = env_rank()
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist

    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist


def shard_range(rank: int, world: int, n: int):
    """Contiguous block [lo, hi) of n items owned by `rank` (strong-scaling split)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


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


def barrier(dist):
    if dist is not None:
        dist.barrier()
