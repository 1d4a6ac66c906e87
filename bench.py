"""Benchmark of the hot path (BASELINE.json): batched A* plans/s on a 1024^2 Grid (config 2).

python bench.py --gpus N --steps K --warmup W      (N>1: launched by torch.distributed.run)

One step = one pass of the hot path over one batch: 4096 start/goal pairs on the C2 grid
(SURVEY.md §8(d) generator), inputs resident in HBM, outputs (cost, path, n_expanded, status)
written to HBM.  Multi-GPU: weak scaling, rank r plans its own 4096 pairs (pair seed 1 + r) on
the same grid; no collective on the data path.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
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


def control_leg(args, torch, dist, world, rank):
    """BASELINE.json's second metric: MPC-style sampled control steps/s at H=30 x 4096 samples (C4):
    256 agents per GPU on the README grid, each step = one DWA.plan iteration (dwa.py:72-93) with a
    64 x 64 (v, w) window, predict_time 3.0 (H = 30).  One timed step = one launch over all agents."""
    from python_motion_planning_amd import _lib, batch, local_planner, workloads as wl

    na = args.agents
    occ, states, goals = wl.c4_workload(na, seed=2 + rank)
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (na, 1)).astype(np.int32),
                            path_cap=2048)
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    Hg = occ.shape[1]
    paths = []
    for i in range(na):
        cells = P[i, : pl[i]][::-1]
        paths.append(np.column_stack([cells // Hg, cells % Hg]).astype(np.float64))
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(local_planner.LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, 64, 64)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    st0 = torch.tensor(states, dtype=torch.float64, device="cuda")
    st = st0.clone()
    ox, oy, gocc = grid
    occ_bits = batch.occ_bits_device(gocc, torch)
    gd = torch.tensor(goals, dtype=torch.float64, device="cuda")
    xyd = torch.tensor(xy, dtype=torch.float64, device="cuda")
    offd = torch.tensor(off, dtype=torch.int32, device="cuda")
    L = _lib.load_library()
    ctx = _lib.context()
    u = torch.empty((na, 2), dtype=torch.float64, device="cuda")
    best = torch.empty(na, dtype=torch.int32, device="cuda")
    status = torch.empty(na, dtype=torch.int32, device="cuda")
    nst = torch.empty(na, dtype=torch.int32, device="cuda")

    def step():
        rc = L.pmp_dwa_step_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), ox, oy, gocc.shape[0], gocc.shape[1],
                                  ctypes.byref(lp), ctypes.byref(dp), na, st.data_ptr(), gd.data_ptr(), xyd.data_ptr(),
                                  offd.data_ptr(), 1, u.data_ptr(), best.data_ptr(), status.data_ptr(),
                                  nst.data_ptr(), None, None, None)
        if rc:
            _lib.check(ctx, rc, "pmp_dwa_step_batch")

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    st.copy_(st0)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    evs = []
    K = args.control_steps
    t0 = time.perf_counter()
    for i in range(K):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
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
    steps_done = na * K * world
    # ~8.2 MFLOP per agent-step in the stencil formulation
    flops_per_step = 4096 * 30 * (12 + 2 * 20) + 4096 * 30 * 9 * 6 + 4096 * 20
    achieved_tf = flops_per_step * na / (kern_ms * 1e-3) / 1e12
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        threads = min(16, os.cpu_count() or 1)
        ns = min(32, na)
        obs = np.argwhere(occ).astype(np.float64)
        xs, offs = batch.pack_paths(paths[:ns])
        t = time.perf_counter()
        O.dwa_step_batch(obs, xs, offs, goals[:ns], states[:ns], nthreads=threads)
        dt = time.perf_counter() - t
        cpu = {"value": ns / dt, "unit": "agent-steps/s", "cores": threads, "kind": "port",
               "sample": f"first {ns} C4 agents, one step each, C restatement of DWA.evaluation (brute-force "
                         f"cdist like the reference) with OpenMP over agents, {dt:.1f} s wall"}
    return {"metric": "MPC steps/sec (H=30, 4096 samples): sampled-rollout control step (DWA form)",
            "value": steps_done / elapsed, "unit": "agent-steps/s", "agents_per_gpu": na, "steps": K,
            "ms_per_step": elapsed / K * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "config": {"workload": "C4: README 51x31 grid, 64x64 (v,w) samples, H=30, weights 0.2/0.1/0.05"},
            "roofline": {"bound": "fp64-valu", "achieved": achieved_tf, "peak": 78.6, "unit": "TFLOP/s",
                         "frac": achieved_tf / 78.6, "traffic": None,
                         "flops_per_agent_step": flops_per_step},
            "cpu_baseline": cpu}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nq", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=1024, help="queries in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--agents", type=int, default=256, help="C4 agents per GPU (control-step leg)")
    ap.add_argument("--control-steps", type=int, default=20, help="timed control steps")
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

    control = control_leg(args, torch, dist, world, rank)

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
            "secondary": control,
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
