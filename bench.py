"""Benchmark of the hot path (BASELINE.json): batched A* plans/s on a 1024^2 Grid (config 2).

python bench.py --gpus N --steps K --warmup W      (N>1: launched by torch.distributed.run)

One step = one pass of the hot path over one batch: 4096 start/goal pairs on the C2 grid
(SURVEY.md §8(d) generator), inputs resident in HBM, outputs (cost, path, n_expanded, status)
written to HBM.  Multi-GPU: weak scaling, rank r plans its own 4096 pairs (pair seed 1 + r) on
the same grid; no collective on the data path.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def astar_algorithmic_bytes(counters: np.ndarray) -> float:
    """per plan B = 19*E + 16*(P + Q); E expansions (3x3 occupancy 9 B + 3x3 closed
    9 B + 1 B parent write), P heap pushes, Q heap pops, 16 B per heap entry."""
    P, Q, E = counters[:, 0].astype(np.float64), counters[:, 1].astype(np.float64), counters[:, 2].astype(np.float64)
    return float(np.sum(19.0 * E + 16.0 * (P + Q)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nq", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=1024, help="queries in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workers", type=int, default=2048, help="persistent A* workers (waves) per launch")
    ap.add_argument("--streams", type=int, default=3,
                    help="batches in flight: consecutive steps go to different HIP streams (own scratch "
                         "context each), so one batch's long-query tail overlaps the next batch")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from python_motion_planning_amd import _lib, batch, workloads as wl

    nq = args.nq
    occ, starts, goals = wl.c2_workload(nq=nq, pair_seed=1 + rank)
    W, H = occ.shape
    L = _lib.load_library()
    occ_bits = batch.occ_bits_device(occ, torch)
    s_d = torch.as_tensor(starts, device="cuda")
    g_d = torch.as_tensor(goals, device="cuda")
    path_cap = 4096
    S = max(1, args.streams)
    lanes = []
    for _ in range(S):
        ctx = L.pmp_create(torch.cuda.current_device())
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, args.workers, 0), "reserve")
        lanes.append(dict(
            ctx=ctx, stream=torch.cuda.Stream(),
            cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
            plen=torch.empty(nq, dtype=torch.int32, device="cuda"),
            path=torch.empty((nq, path_cap), dtype=torch.int32, device="cuda"),
            nexp=torch.empty(nq, dtype=torch.int32, device="cuda"),
            status=torch.empty(nq, dtype=torch.int32, device="cuda")))
    ctr = torch.empty((nq, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step(i, counters=None):
        b = lanes[i % S]
        rc = L.pmp_astar2d_batch(b["ctx"], b["stream"].cuda_stream, occ_bits.data_ptr(), W, H, 0, s_d.data_ptr(),
                                 g_d.data_ptr(), nq, b["cost"].data_ptr(), b["plen"].data_ptr(), b["path"].data_ptr(),
                                 path_cap, b["nexp"].data_ptr(), None, 0, counters, b["status"].data_ptr())
        if rc:
            _lib.check(b["ctx"], rc, "pmp_astar2d_batch")
        return b

    # warmup: every stream once (the first pass also records the deterministic push/pop/expansion counts)
    step(0, ctr.data_ptr())
    for i in range(1, max(args.warmup, S)):
        step(i)
    torch.cuda.synchronize()
    counters = ctr.cpu().numpy()
    cost = lanes[0]["cost"]
    for b in lanes:
        st = b["status"].cpu().numpy()
        assert (st == 0).all(), f"unexpected statuses {np.unique(st)}"
        assert torch.equal(b["cost"], cost)
    bytes_per_launch = astar_algorithmic_bytes(counters)

    # timed region
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        b = lanes[i % S]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(b["stream"])
        step(i)
        e1.record(b["stream"])
        evs.append((e0, e1))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if dist:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = torch.tensor([kern_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        kern_ms = float(k.item())

    plans = nq * args.steps * world
    value = plans / elapsed
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        threads = min(16, os.cpu_count() or 1)
        ns = min(args.cpu_sample, nq)
        O.lib()
        t = time.perf_counter()
        ref = O.astar2d_batch(occ, starts[:ns], goals[:ns], path_cap=path_cap, nthreads=threads)
        dt = time.perf_counter() - t
        assert np.array_equal(ref["cost"], cost[:ns].cpu().numpy()), "GPU/oracle cost mismatch"
        cpu = {"value": ns / dt, "unit": "plans/s", "cores": threads, "kind": "port",
               "sample": f"first {ns} of the 4096 C2 pairs, C restatement (oracle/pmp_oracle.c) with OpenMP over "
                         f"queries, {dt:.1f} s wall"}

    if rank == 0:
        out = {
            "metric": "A* plans/sec on 1024^2 grid (4096 random start/goal pairs per GPU)",
            "value": value,
            "unit": "plans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) C2 generator: default_rng(0) 20% obstacles, default_rng(1+rank) pairs)",
            "config": {"workload": "C2 batched A* 1024x1024 Grid, 4096 start/goal pairs per GPU, euclidean",
                       "grid": [W, H], "queries_per_gpu": nq, "parallelism": f"query-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None},
            "cpu_baseline": cpu,
            "detail": {"kernel_ms_per_launch": kern_ms,
                       "algorithmic_bytes_per_launch": bytes_per_launch,
                       "expansions_per_launch": int(counters[:, 2].sum()),
                       "max_expansions_query": int(counters[:, 2].max()),
                       "pushes_per_launch": int(counters[:, 0].sum()),
                       "pops_per_launch": int(counters[:, 1].sum()),
                       "max_heap_entries": int(counters[:, 3].max()),
                       "workers": args.workers, "streams": S},
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
