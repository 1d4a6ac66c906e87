"""Benchmark of the hot path (BASELINE.json): batched A* plans/s on a 1024^2 Grid (config 2) as the
headline, and the other configs as secondary legs in the same JSON line.

python bench.py --gpus N --steps K --warmup W      (N>1: launched by torch.distributed.run)

Headline step = one pass of the hot path over one batch: 4096 start/goal pairs on the C2 grid
(SURVEY.md §8(d) generator), inputs resident in HBM, outputs (cost, path, n_expanded, status)
written to HBM.  Secondary legs (--legs): the H=30 x 4096-sample control step (C4, DWA form), RRT*
on the C3 512^2 map (65,536 samples), 3D A* on C5 (8192 queries), and the LQR / MPC tracking steps
on the C4 agents.  Multi-GPU: --scaling weak (default), every rank runs its own shard (rank-offset
seeds) of every leg; --scaling strong, one fixed batch per leg is dealt over the ranks (C2 pairs and
C5 queries longest-first round-robin, C4 agents round-robin) and the records are all_gathered back
into input order at the end (rank 0 checks them against a replay of the whole batch on its GPU).  No
collective on the data path.  Rank 0 prints one JSON line.
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
L2_PEAK_GBS = 34500.0  # MI355X L2, 8 XCDs x 4 MiB, aggregate (MI355X_MICROARCH.md, L2 per XCD)


def astar_algorithmic_bytes(counters: np.ndarray) -> float:
    """per plan B = 19*E + 16*(P + Q); E expansions (3x3 occupancy 9 B + 3x3 closed
    9 B + 1 B parent write), P heap pushes, Q heap pops, 16 B per heap entry."""
    P, Q, E = counters[:, 0].astype(np.float64), counters[:, 1].astype(np.float64), counters[:, 2].astype(np.float64)
    return float(np.sum(19.0 * E + 16.0 * (P + Q)))


def c4_share(args, na, world, rank):
    """C4 agents of this rank: weak scaling, `na` agents of its own (default_rng(2 + rank)); strong
    scaling, its round-robin share of one fixed set of `na` agents (default_rng(2)).  Returns
    (occ, states, goals, indices into the fixed set or None)."""
    from python_motion_planning_amd import shard, workloads as wl

    if args.scaling == "strong":
        occ, states, goals = wl.c4_workload(na, seed=2)
        mine = shard.lpt_deal(np.ones(na), world, rank)  # equal work per agent: round-robin
        return occ, states[mine], goals[mine], mine
    occ, states, goals = wl.c4_workload(na, seed=2 + rank)
    return occ, states, goals, None


def dwa_inputs(torch, occ, states, goals):
    """The C4 agents' global paths (start -> goal): A* from each agent's cell to (45, 25) on the GPU."""
    from python_motion_planning_amd import batch

    na = len(states)
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (na, 1)).astype(np.int32),
                            path_cap=2048)
    pl, P = r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
    Hg = occ.shape[1]
    paths = [np.column_stack([P[i, : pl[i]][::-1] // Hg, P[i, : pl[i]][::-1] % Hg]).astype(np.float64)
             for i in range(na)]
    return paths


def control_replay(args, torch, occ, states, goals, K):
    """K DWA steps of all the given agents in one launch each (untimed): the strong-scaling check."""
    from python_motion_planning_amd import _lib, batch, local_planner

    paths = dwa_inputs(torch, occ, states, goals)
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(local_planner.LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, 64, 64)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    st = torch.tensor(states, dtype=torch.float64, device="cuda")
    o = None
    for _ in range(K):
        o = batch.dwa_step_batch(grid, lp, dp, st, goals, xy, off)
    torch.cuda.synchronize()
    return {"state": st, "u": o["u"], "best": o["best"]}


def control_leg(args, torch, dist, world, rank):
    """BASELINE.json's second metric: MPC-style sampled control steps/s at H=30 x 4096 samples (C4):
    256 agents per GPU on the README grid, each step = one DWA.plan iteration (dwa.py:72-93) with a
    64 x 64 (v, w) window, predict_time 3.0 (H = 30).  One timed step = one launch over all agents."""
    from python_motion_planning_amd import _lib, batch, local_planner, shard

    occ, states, goals, mine = c4_share(args, args.agents, world, rank)
    na = len(states)
    paths = dwa_inputs(torch, occ, states, goals)
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
    K = args.control_steps
    # every step writes its own output rows (the state advances in place), so each timed step is
    # checked below against the same step of an untimed replay
    u_all = torch.empty((K, na, 2), dtype=torch.float64, device="cuda")
    best_all = torch.empty((K, na), dtype=torch.int32, device="cuda")
    status_all = torch.empty((K, na), dtype=torch.int32, device="cuda")
    nst = torch.empty(na, dtype=torch.int32, device="cuda")
    _LABEL[0] = "mpc_sampled_dwa"

    def step(k):
        rc = L.pmp_dwa_step_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), ox, oy, gocc.shape[0], gocc.shape[1],
                                  ctypes.byref(lp), ctypes.byref(dp), na, st.data_ptr(), gd.data_ptr(), xyd.data_ptr(),
                                  offd.data_ptr(), 1, u_all[k].data_ptr(), best_all[k].data_ptr(),
                                  status_all[k].data_ptr(), nst.data_ptr(), None, None, None)
        if rc:
            _lib.check(ctx, rc, "pmp_dwa_step_batch")

    for _ in range(max(1, args.warmup)):
        step(0)
    torch.cuda.synchronize()
    st.copy_(st0)
    poison([u_all, best_all, status_all])
    elapsed, kern_ms = timed(torch, dist, step, K)
    # the timed work checked: an untimed replay of the same K steps from the same states gives the same
    # controls, argmax and status at every step and the same final agent states (the first step's
    # evaluation is pinned to the oracle by tests/test_dwa_gpu.py)
    timed_rows = [{"u": u_all[k].clone(), "best": best_all[k].clone(), "status": status_all[k].clone()}
                  for k in range(K)]
    st_timed = st.clone()
    st.copy_(st0)
    for k in range(K):
        step(k)
    torch.cuda.synchronize()
    checked = 0
    for k in range(K):
        checked += check_timed("dwa", {"u": u_all[k], "best": best_all[k], "status": status_all[k]}, [timed_rows[k]])
    check_timed("dwa", {"state": st}, [{"state": st_timed}])
    ref_out = {"state": st_timed, "u": u_all[K - 1], "best": best_all[K - 1]}
    steps_done = (args.agents if args.scaling == "strong" else na * world) * K
    gathered = None
    if args.scaling == "strong":
        # the fixed agent set's records from every rank, in agent order; rank 0 replays all the agents
        # on its own GPU (untimed) and compares
        g = shard.all_gather_rows(dist, mine, {k: ref_out[k] for k in ("state", "u", "best")}, args.agents,
                                  device="cuda")
        gathered = {"agents": args.agents, "agents_this_rank": na}
        if rank == 0:
            occ1, st1, gl1, _ = c4_share(args, args.agents, 1, 0)
            full = control_replay(args, torch, occ1, st1, gl1, K)
            gathered["gathered_equal_single_rank"] = all(torch.equal(g[k], full[k]) for k in ("state", "u", "best"))
    # SURVEY.md §8(d) C4 in the stencil formulation, transcendental calls not counted: per sample and
    # step 12 flops of rollout (x, y, th updates) + a 3x3 stencil of 6 flops per cell; 20 per sample
    # for normalisation and scoring -> 8.2 MFLOP per agent-step
    flops_per_step = 4096 * 30 * 12 + 4096 * 30 * 9 * 6 + 4096 * 20
    achieved_tf = flops_per_step * na / (kern_ms * 1e-3) / 1e12
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        threads = cpu_threads()
        obs = np.argwhere(occ).astype(np.float64)
        xs, offs = batch.pack_paths(paths)

        # the kernel's formulation on the CPU (obstacle term over the cells within R): all cores, 1 core
        def run(nth, k=na):
            return lambda i: O.dwa_step_batch(obs, xs, offs[: k + 1], goals[:k], states[:k], nthreads=nth, grid=occ)
        reps, dt = timed_cpu(run(threads), args.cpu_seconds)
        ns1 = min(16, na)
        reps1, dt1 = timed_cpu(run(1, ns1), 2.0)
        # the reference's own formulation (cdist over all 215 obstacles per trajectory point): all cores
        nb = min(32, na)
        xb, ob = batch.pack_paths(paths[:nb])
        repsb, dtb = timed_cpu(lambda i: O.dwa_step_batch(obs, xb, ob, goals[:nb], states[:nb], nthreads=threads),
                               2.0)
        cpu = {"value": na * reps / dt, "unit": "agent-steps/s", "cores": threads, "kind": "port",
               "host": host_cpu(),
               "sample": f"all {na} C4 agents x {reps} steps, C restatement of DWA.evaluation with the obstacle "
                         f"term over the cells within the inflation radius (the kernel's formulation; identical "
                         f"values), OpenMP over agents, {dt:.1f} s wall",
               "one_core": {"value": ns1 * reps1 / dt1, "sample": f"{ns1} agents x {reps1} steps, {dt1:.1f} s"},
               "reference_formulation": {"value": nb * repsb / dtb, "cores": threads,
                                         "sample": f"{nb} agents x {repsb} steps, cdist over every obstacle like "
                                                   f"dwa.py:164, {dtb:.1f} s"}}
    _LABEL[0] = "setup"
    return {"metric": "MPC steps/sec (H=30, 4096 samples): sampled-rollout control step (DWA form)",
            "value": steps_done / elapsed, "unit": "agent-steps/s", "agents_per_gpu": na, "steps": K,
            "scaling": args.scaling, "strong_scaling_gather": gathered,
            "ms_per_step": elapsed / K * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "timed_launches_checked": checked,
            "config": {"workload": "C4: README 51x31 grid, 64x64 (v,w) samples, H=30, weights 0.2/0.1/0.05"},
            "roofline": with_issue(with_traffic({"bound": "fp64-valu", "achieved": achieved_tf, "peak": 78.6,
                                                 "unit": "TFLOP/s", "frac": achieved_tf / 78.6, "traffic": None,
                                                 "frac_basis": "model flops (SURVEY.md 8(d) stencil form), not the "
                                                               "instructions executed: see issue",
                                                 "flops_per_agent_step": flops_per_step,
                                                 "flops_note": "SURVEY.md 8(d) stencil formulation, sin/cos/atan2 "
                                                               "not counted; the kernel's 2x2 nibble stencil and "
                                                               "per-w rotation table execute fewer"},
                                                "dwa_split_kernel", "mpc_sampled_dwa"),
                                   "dwa_split_kernel", "mpc_sampled_dwa", na, "agent-step"),
            "cpu_baseline": cpu}


# ---- launch manifest -------------------------------------------------------------------------
# Which workload (leg) made each dispatch of each kernel, in launch order, so the rocprofv3 kernel
# trace and PMC passes can be keyed per (kernel, workload) (tools/prof_summary.py): every C-ABI
# planner call is counted through a wrapper on the library, under the label of the leg running.
_MANIFEST = []  # [label, kernel short name, dispatches], consecutive equal (label, kernel) merged
_LABEL = ["setup"]
_G2D = {0: "astar2d_kernel", 1: "dijkstra2d_kernel", 2: "gbfs2d_kernel", 3: "theta2d_kernel", 4: "lazy_theta2d_kernel"}
ENTRY_KERNEL = {  # C-ABI entry -> (short name of the kernel it launches, as tools/prof_summary.short)
    "pmp_astar2d_batch": lambda a: "astar2d_kernel",
    "pmp_graph2d_batch": lambda a: _G2D[int(a[2])],
    "pmp_astar3d_batch": lambda a: "astar3d_kernel",
    "pmp_graph3d_batch": lambda a: "astar3d_kernel",
    # D* 2D: the first pass and the re-run at the bound (default first capacity: two dispatches per call)
    "pmp_dstar2d_batch": lambda a: [("dstar_kernel", 1), ("dstar_rerun_kernel", 1)],
    "pmp_dstar2d_onpress_batch": lambda a: [("dstar_kernel", 1), ("dstar_rerun_kernel", 1)],
    "pmp_dstar3d_batch": lambda a: "dstar3d_kernel",
    "pmp_lpastar3d_batch": lambda a: "lpa3d_kernel",
    "pmp_lpastar2d_batch": lambda a: "lpa_kernel",
    "pmp_dstarlite2d_batch": lambda a: "lpa_kernel",
    "pmp_lpastar2d_replan_batch": lambda a: "lpa_kernel",
    "pmp_dstarlite2d_replan_batch": lambda a: "lpa_kernel",
    "pmp_dwa_step_batch": lambda a: _dwa_kernels(a),
    "pmp_rrt_batch": lambda a: "rrt_kernel",
    "pmp_totp3d_batch": lambda a: "totp3d_kernel",
    # MPC: per plan iteration a step and a solve dispatch, then a last step (track.hip)
    "pmp_track_step_batch": lambda a: "track_kernel_lqr" if int(a[2]) == 0 else
                                      [("track_mpc_step", int(a[12]) + 1), ("track_mpc_solve", int(a[12]))],
    "pmp_lqr_control_batch": lambda a: "lqr_control_kernel",
    "pmp_mpc_control_batch": lambda a: "mpc_control_kernel",
}


def _dwa_kernels(a):
    """pmp_dwa_step_batch's dispatches (dwa.hip): fixed windows (nv, nw > 0) launch dwa_split_kernel once
    per plan iteration (k parts, or k = 1); resolution-sized windows one dwa_kernel for all iterations."""
    dp = getattr(a[8], "_obj", a[8])
    if dp.nv > 0 and dp.nw > 0:
        return [("dwa_split_kernel", int(a[14]))]
    return "dwa_kernel"


def count_launches(L):
    """Wrap the planner entry points of the (singleton) library object so every successful call is
    logged in _MANIFEST under the current label.  Idempotent."""
    if getattr(L, "_pmp_counted", False):
        return L
    for name, kern in ENTRY_KERNEL.items():
        fn = getattr(L, name)

        def wrapped(*a, _fn=fn, _k=kern):
            rc = _fn(*a)
            if rc == 0:
                ks = _k(a)
                for k, n in ([(ks, 1)] if isinstance(ks, str) else ks):  # an entry may dispatch several kernels
                    if _MANIFEST and _MANIFEST[-1][0] == _LABEL[0] and _MANIFEST[-1][1] == k:
                        _MANIFEST[-1][2] += n
                    else:
                        _MANIFEST.append([_LABEL[0], k, n])
            return rc
        setattr(L, name, wrapped)
    L._pmp_counted = True
    return L


class leg_label:
    """with leg_label("dstar_256"): ... -- the launches inside belong to that workload."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = _LABEL[0]
        _LABEL[0] = self.name

    def __exit__(self, *exc):
        _LABEL[0] = self.prev


def _newest_profile(fname):
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", fname)),
                   key=lambda p: int(os.path.basename(os.path.dirname(p))[1:] or 0))
    return files[-1] if files else None


def pmc_traffic(workload: str, kernel: str):
    """HBM bytes per dispatch of `kernel` in the leg `workload`, from the newest committed
    profiles/r*/pmc_traffic.json (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, keyed per
    (kernel, workload) through the bench's launch manifest by tools/prof_summary.py, gfx950
    correction applied).  A summary entry whose kernel or workload does not match is refused.
    (bytes, source) or (None, reason)."""
    path = _newest_profile("pmc_traffic.json")
    if not path:
        return None, "no committed pmc_traffic.json"
    with open(path) as f:
        d = json.load(f).get("workloads", {}).get(workload)
    src = os.path.relpath(path, REPO)
    if not d:
        return None, f"{src} has no entry for workload {workload}"
    if d.get("kernel") != kernel:
        return None, f"{src} [{workload}] is kernel {d.get('kernel')}, not {kernel}: refused"
    b = d.get("hbm_bytes_per_dispatch")
    return (float(b) if b is not None else None), f"{src} [{workload}: {kernel}]"


def with_traffic(roof: dict, kernel: str, workload: str) -> dict:
    t, src = pmc_traffic(workload, kernel)
    roof["traffic"] = t
    roof["traffic_source"] = src
    alg = roof.get("algorithmic_bytes_per_launch")
    if t and alg:
        roof["traffic_over_algorithmic"] = t / alg
    return roof


def with_issue(roof: dict, kernel: str, workload: str, units_per_dispatch: float, unit: str) -> dict:
    """The binding resource of an issue-bound leg beside its memory roof: instructions per unit of
    work and the VALU issue fraction of `kernel`'s dispatches in the leg `workload`, from the newest
    committed profiles/r*/pmc_issue.json (the SQ issue pass of tools/profile_round.sh, keyed per
    workload by tools/prof_summary.py).  valu_issue_frac = SQ_INSTS_VALU / (1024 SIMDs x
    GRBM_GUI_ACTIVE / 8 XCDs / 2 cycles per wave64 VALU instruction)."""
    path = _newest_profile("pmc_issue.json")
    if not path:
        roof["issue"] = {"source": "no committed pmc_issue.json"}
        return roof
    src = os.path.relpath(path, REPO)
    with open(path) as f:
        d = json.load(f).get("workloads", {}).get(workload)
    if not d or d.get("kernel") != kernel:
        roof["issue"] = {"source": f"{src} has no {kernel} entry for workload {workload}: refused"}
        return roof
    per = 1.0 / float(units_per_dispatch) if units_per_dispatch else None
    roof["issue"] = {
        "unit": unit,
        "valu_insts_per_unit": d["SQ_INSTS_VALU_per_dispatch"] * per if per else None,
        "salu_insts_per_unit": d.get("SQ_INSTS_SALU_per_dispatch", 0.0) * per if per else None,
        "lds_insts_per_unit": d.get("SQ_INSTS_LDS_per_dispatch", 0.0) * per if per else None,
        "valu_issue_frac": d.get("valu_issue_frac"),
        "wave_issue_frac": d.get("wave_issue_frac"), "wave_wait_frac": d.get("wave_wait_frac"),
        "units_per_dispatch": units_per_dispatch,
        "source": f"{src} [{workload}: {kernel}, SQ pass of the short bench; units from this run]"}
    return roof


def with_mfma(roof: dict, kernel: str) -> dict:
    """MFMA utilisation of `kernel` from the newest committed profiles/r*/pmc_mfma.json (the separate
    rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE, tools/profile_round.sh):
    busy cycles over 1024 SIMDs x the dispatch's GPU cycles, in percent (rocprofv3's MfmaUtil)."""
    path = _newest_profile("pmc_mfma.json")
    roof["mfma_util_pct"] = None
    if path:
        with open(path) as f:
            d = json.load(f).get(kernel) or {}
        if d.get("mfma_util_pct") is not None:
            roof["mfma_util_pct"] = float(d["mfma_util_pct"])
            roof["mfma_source"] = f"{os.path.relpath(path, REPO)} [{kernel}]"
    return roof


_STREAM_POOL = []


_SHARED_CTX = []  # the headline's context kept for the Theta* legs (--theta-share-ctx)


def pool_stream(torch, i):
    """Stream i of one pool shared by every leg.  HIP maps each new stream to the next of its
    GPU_MAX_HW_QUEUES hardware queues round-robin, so streams created leg after leg eventually share
    a queue and two 'batches in flight' serialise behind each other; the legs therefore reuse the
    same few streams (at most 6, each on its own queue of the 8 this bench asks for)."""
    while len(_STREAM_POOL) <= i:
        _STREAM_POOL.append(torch.cuda.Stream())
    return _STREAM_POOL[i]


def timed(torch, dist, fn, steps, stream=None, streams=None, last=None):
    """Barrier + sync, run `steps` launches with HIP events around each (on `stream`; or, with
    `streams`, launch i runs with streams[i % len] current: batches in flight, each on its own
    stream and so its own per-stream pmp_ctx), barrier + sync; returns (wall seconds, max over
    ranks; mean event ms per launch).  With a list `last`, the return values of the final launch
    on each stream are appended to it (for the check of the timed work, `check_timed`)."""
    import contextlib

    from python_motion_planning_amd import shard

    shard.barrier(dist)
    torch.cuda.synchronize()
    evs = []
    rets = {}
    t0 = time.perf_counter()
    for i in range(steps):
        sm = streams[i % len(streams)] if streams else stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if sm is None:
            e0.record()
        else:
            e0.record(sm)
        with (torch.cuda.stream(sm) if streams else contextlib.nullcontext()):
            r = fn(i)
        if last is not None:
            rets[i % len(streams) if streams else 0] = r
        if sm is None:
            e1.record()
        else:
            e1.record(sm)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    shard.barrier(dist)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
    if last is not None:
        last.extend(rets.values())
    return elapsed, kern_ms


LPA_BYTES_NOTE = ("LPA* / D* Lite: per expansion the 3x3 block of (g, rhs) 9 x 16 B + 9 B occupancy + 8 B g write "
                  "= 161 B; per U insertion 20 B (k1, k2 f64 + cell)")


def lpa_bytes(expansions, pushes) -> float:
    """Algorithmic bytes of the LPA* / D* Lite 2D list machine (lpa_star.py:39-230, d_star_lite.py:14-187):
    161 B per expansion + 20 B per U insertion (LPA_BYTES_NOTE)."""
    return 161.0 * float(expansions) + 20.0 * float(pushes)


def hbm_roof(alg_bytes, kern_ms, note):
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": None, "algorithmic_bytes_per_launch": alg_bytes, "bytes_note": note}


def dyn3d_roof(kind, n, pushes, kern_ms):
    """DStar3D (d_star3d.py:60-281): per processState the 3x3x3 block of voxel states (h, k f64 + tag /
    parent: 27 x 24 B) + 27 B occupancy + 2 OPEN entries x 16 B = 707 B.  LPAStar3D
    (lpa_star3d.py:40-225): per expansion 27 x 16 B (g, rhs) + 27 B occupancy + 8 B g write = 467 B,
    + 20 B per U insertion (counted by the kernel; when absent, one per expansion)."""
    if kind == "dstar3d":
        return hbm_roof(707.0 * n, kern_ms, "707 B per processState (27 x 24 B voxel states + 27 B occupancy + 2 OPEN "
                                            "entries x 16 B)")
    p = n if pushes is None else pushes
    return hbm_roof(467.0 * n + 20.0 * p, kern_ms, "467 B per expansion (27 x 16 B g/rhs + 27 B occupancy + 8 B write) "
                                                   "+ 20 B per U insertion")


def poison(bufs):
    """Overwrite output buffers before a timed region (NaN / -1), so that check_timed proves the
    timed launches wrote them."""
    for t in bufs:
        if t.is_floating_point():
            t.fill_(float("nan"))
        else:
            t.fill_(-1)


def check_timed(name, ref: dict, outs) -> int:
    """The work of the timed launches is checked, not trusted: every stream's last timed output
    equals the warmup launch's (which the legs check against the oracle / invariants) field for
    field.  Returns the number of launches checked; raises on a mismatch."""
    import torch

    n = 0
    for o in outs:
        for k, v in ref.items():
            got = o[k]
            if not torch.equal(got.to(v.device), v):
                raise AssertionError(f"{name}: timed launch output '{k}' differs from the warmup launch's")
        n += 1
    if n == 0:
        raise AssertionError(f"{name}: no timed output to check")
    return n


def cgroup_cpus():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max or v1 cfs quota), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else max(1, -(-q // per))
    except (OSError, ValueError):
        return None


def cpu_threads():
    """The CPU baselines' thread count: every core this job may use -- its affinity mask, capped by
    the cgroup CPU quota (a gpurun box hands the job a share of the machine: more threads than the
    quota only time-slice against each other)."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    return min(n, q) if q else n


def host_cpu():
    """The CPU-baseline host as the bench sees it: model, os.cpu_count() (the machine) and the
    affinity mask (the cores this job may use; gpurun boxes hand a share of the machine)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "os_cpu_count": os.cpu_count(), "affinity_cores": len(os.sched_getaffinity(0)),
            "cgroup_quota_cpus": cgroup_cpus(), "threads_used": cpu_threads()}


def timed_cpu(fn, min_seconds):
    """Run fn() until at least min_seconds of wall time have passed; returns (calls, seconds)."""
    t = time.perf_counter()
    reps = 0
    while True:
        fn(reps)
        reps += 1
        dt = time.perf_counter() - t
        if dt >= min_seconds:
            return reps, dt


def rrt_leg(args, torch, dist, world, rank):
    """C3: RRT* on the 512^2 Map (40 rects + 40 circles, default_rng(7)), start (5,5), goal (505,505),
    65,536 samples, max_dist 0.5, r 10, goal rate 0.05; query q draws from np.random.seed(q) (rank
    offset).  One timed step = one launch over all queries of the rank."""
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import _lib, batch, workloads as wl

    nq, sn = args.rrt_queries, args.rrt_samples
    env = pmp.Map(512, 512)
    rects, circs = wl.c3_map()
    env.update(obs_rect=rects, obs_circ=circs)
    seeds = np.arange(nq) + rank * nq
    rnd = np.stack([np.random.RandomState(int(q)).random_sample(3 * sn + 1) for q in seeds])
    rnd_d = torch.as_tensor(rnd, device="cuda")
    starts, goals = np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1))
    _LABEL[0] = "rrt_star_warmup"  # launches of other sizes than the timed ones: keyed apart in the profile
    out = batch.rrt_batch(env, starts, goals, rnd_d, sn, star=True, counters=True)  # warmup + counters
    torch.cuda.synchronize()
    ctr = out["counters"].cpu().numpy()
    status = out["status"].cpu().numpy()
    assert np.isin(status, (0, 1)).all(), f"unexpected RRT* statuses {np.unique(status)}"
    # One workgroup grows one tree and a query's time grows with the square of its iterations
    # (12 k - 42 k per C3 query: the whole-tree scans), so a 256-query launch lasts as long as its
    # slowest query.  Continuous batching: --rrt-batches batches of the 256 queries go to the planner
    # as ONE launch (grid = every query of them, one workgroup per CU at a time), and the hardware
    # dispatcher hands each CU its next query as its last one finishes; --rrt-streams launches in
    # flight on their own streams (own pmp_ctx each) overlap the launches' tails.
    nb = max(1, args.rrt_batches)
    nql = nq * nb
    L = _lib.load_library()
    rect, circ, bnd = batch.map_arrays(env, torch)
    s_d = torch.as_tensor(np.tile(starts, (nb, 1)), device="cuda")
    g_d = torch.as_tensor(np.tile(goals, (nb, 1)), device="cuda")
    rnd_l = rnd_d.repeat(nb, 1) if nb > 1 else rnd_d
    cap = sn + 2
    P = _lib.RRTParams(512.0, 512.0, 0.5, 0.5, 10.0, 0.05, sn, 1)
    lanes = []
    for _ in range(max(1, args.rrt_streams)):
        f64 = dict(dtype=torch.float64, device="cuda")
        i32 = dict(dtype=torch.int32, device="cuda")
        lanes.append(dict(ctx=L.pmp_create(torch.cuda.current_device()), stream=pool_stream(torch, len(lanes)),
                          txy=torch.empty((nql, cap, 2), **f64), tg=torch.empty((nql, cap), **f64),
                          tpar=torch.empty((nql, cap), **i32), nn=torch.empty(nql, **i32), cost=torch.empty(nql, **f64),
                          plen=torch.empty(nql, **i32), path=torch.empty((nql, cap, 2), **f64),
                          draws=torch.empty(nql, dtype=torch.int64, device="cuda"), st=torch.empty(nql, **i32)))
        if args.rrt_resident > 0:  # the LDS tree share: room for this many workgroups per CU
            _lib.check(lanes[-1]["ctx"], L.pmp_set_resident_per_cu(lanes[-1]["ctx"], args.rrt_resident),
                       "pmp_set_resident_per_cu")

    def launch(i):
        b = lanes[i % len(lanes)]
        rc = L.pmp_rrt_batch(b["ctx"], b["stream"].cuda_stream, ctypes.byref(P), rect.data_ptr(), int(rect.shape[0]),
                             circ.data_ptr(), int(circ.shape[0]), bnd.data_ptr(), int(bnd.shape[0]), s_d.data_ptr(),
                             g_d.data_ptr(), nql, rnd_l.data_ptr(), int(rnd_l.shape[1]), cap, b["txy"].data_ptr(),
                             b["tg"].data_ptr(), b["tpar"].data_ptr(), b["nn"].data_ptr(), b["cost"].data_ptr(),
                             b["plen"].data_ptr(), b["path"].data_ptr(), cap, b["draws"].data_ptr(), b["st"].data_ptr(),
                             None)
        if rc:
            _lib.check(b["ctx"], rc, "pmp_rrt_batch")

    for i in range(len(lanes)):  # warm every lane's scratch
        launch(i)
    torch.cuda.synchronize()
    for b in lanes:  # every repeat of the batch equals the warmup's 256 queries
        assert torch.equal(b["nn"], out["n_nodes"].repeat(nb)) and torch.equal(b["st"], out["status"].repeat(nb))
        assert torch.equal(b["cost"], out["cost"].repeat(nb)) and torch.equal(b["draws"], out["draws"].repeat(nb))
    rkeys = ("nn", "st", "cost", "plen", "draws")
    ref_out = {k: lanes[0][k].clone() for k in rkeys}
    _LABEL[0] = "rrt_star"
    for b in lanes:
        poison([b[k] for k in rkeys])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for i in range(args.rrt_steps):
        b = lanes[i % len(lanes)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(b["stream"])
        launch(i)
        e1.record(b["stream"])
        evs.append((e0, e1))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    from python_motion_planning_amd import shard

    elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
    checked = check_timed("rrt_star", ref_out, lanes[: min(len(lanes), args.rrt_steps)])
    for b in lanes:  # the lanes' per-query lists and coarse copies (about 14 GB each): not needed later
        L.pmp_destroy(b["ctx"])
    # the bytes the kernel loads: 4 B per node scanned (the 16-bit fixed-point
    # coordinate copy of the coarse nearest / radius scans) + 24 B per in-radius candidate (exact
    # f64 x, y and g).  The trees (4 B x 65,537 nodes per query) stay in L2 / Infinity Cache, so the
    # roof is the L2 bandwidth (MI355X_MICROARCH.md: ~34.5 TB/s aggregate)
    alg_bytes = float(4.0 * ctr[:, 1].sum() + 24.0 * ctr[:, 2].sum()) * nb
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    # SURVEY.md §8(d)'s own accounting: 16 B of xy per node scanned + 8 B of g per in-radius node
    sv_bytes = float(16.0 * ctr[:, 1].sum() + 8.0 * ctr[:, 2].sum()) * nb
    sv_gbs = sv_bytes / (kern_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        th = cpu_threads()
        ns = min(args.rrt_cpu_sample, nq)
        t = time.perf_counter()
        ref = O.rrt_batch(True, rects, circs, 512, 512, starts[:ns], goals[:ns], rnd[:ns], sn, nthreads=th)
        dt = time.perf_counter() - t
        assert np.array_equal(ref["status"], status[:ns]) and np.array_equal(ref["n_nodes"], out["n_nodes"][:ns].cpu().numpy())
        cpu = {"value": ns / dt, "unit": "plans/s", "cores": th, "kind": "port",
               "sample": f"first {ns} C3 queries at the full 65,536 samples, C restatement of RRT* "
                         f"(oracle/pmp_oracle.c, same O(N^2) loops as the reference) with OpenMP over queries, "
                         f"{dt:.1f} s wall"}
    return {"metric": "RRT* plans/sec on 512x512 Map, 65536 samples", "value": nql * args.rrt_steps * world / elapsed,
            "unit": "plans/s", "queries_per_gpu": nq, "steps": args.rrt_steps, "batches_per_launch": nb,
            "queries_per_launch": nql,
            "ms_per_step": elapsed / args.rrt_steps * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "streams": len(lanes), "timed_launches_checked": checked,
            "config": {"workload": "C3: Map(512,512), 40 rects + 40 circles (default_rng(7)), (5,5)->(505,505), "
                                   "65536 samples, max_dist 0.5, r 10, goal rate 0.05"},
            # frac on SURVEY.md 8(d)'s algorithmic bytes (the line's model, "bytes_model"), against the L2
            # roof (the trees are L2 / Infinity-Cache resident); the kernel's own loads beside it
            "roofline": with_issue(with_traffic({"bound": "l2", "achieved": sv_gbs, "peak": L2_PEAK_GBS, "unit": "GB/s",
                                      "frac": sv_gbs / L2_PEAK_GBS, "traffic": None,
                                      "algorithmic_bytes_per_launch": sv_bytes,
                                      "bytes_model": "8d: 16 B xy/node scanned + 8 B g/in-radius node",
                                      "frac_hbm": sv_gbs / HBM_PEAK_GBS,
                                      "bytes_note": "SURVEY.md 8(d): 16 B xy per node scanned + 8 B g per in-radius "
                                                    "node; traffic = HBM bytes (PMC), far below: the trees are "
                                                    "cache-resident",
                                      "as_loaded": {"bytes_per_launch": alg_bytes, "achieved": achieved,
                                                    "frac_l2": achieved / L2_PEAK_GBS,
                                                    "note": "the kernel's own loads: 4 B per node scanned (16-bit "
                                                            "fixed-point coarse copy) + 24 B per in-radius candidate"}},
                                                "rrt_kernel", "rrt_star"),
                                   "rrt_kernel", "rrt_star", float(ctr[:, 0].sum()) * nb, "iteration"),
            "detail": {"found": int((status == 0).sum()), "mean_nodes": float(out["n_nodes"].float().mean().item()),
                       "iterations_per_launch": int(ctr[:, 0].sum()) * nb,
                       "nodes_scanned_per_launch": int(ctr[:, 1].sum()) * nb,
                       "collision_tests_per_launch": int(ctr[:, 3].sum()) * nb,
                       "iterations_per_query_q50_max": [float(np.percentile(ctr[:, 0], 50)), int(ctr[:, 0].max())]},
            "cpu_baseline": cpu}


def astar3d_leg(args, torch, dist, world, rank):
    """C5: AStar3D on Grid3D(26,20,16) door scenario, 8192 queries per GPU (random.seed(i) pairs,
    safety bubbles carved per query, so each query has its own occupancy)."""
    from python_motion_planning_amd import _lib, batch, shard, workloads as wl

    if args.scaling == "strong":  # one fixed 8192-query batch dealt longest-first round-robin
        occ_all, s_all, g_all = wl.c5_workload(args.a3_queries, first_seed=0)
        mine = shard.lpt_deal(shard.octile(s_all, g_all), world, rank)
        occ, s, g = occ_all[mine], s_all[mine], g_all[mine]
    else:
        occ, s, g = wl.c5_workload(args.a3_queries, first_seed=rank * args.a3_queries)
        mine = None
    nq = len(s)
    _LABEL[0] = "astar3d"
    X, Y, Z = occ.shape[1:]
    words = np.stack([batch.pack_bits(o) for o in occ])
    occ_d = torch.as_tensor(np.ascontiguousarray(words).view(np.int32), device="cuda")
    s_d = torch.as_tensor(s, device="cuda")
    g_d = torch.as_tensor(g, device="cuda")
    L = _lib.load_library()
    cap = 512  # C5 paths are far shorter (the kernel reports PMP_PATH_OVERFLOW otherwise)
    # Batches per launch (as the headline): B of the steps' batches per launch, streamed through the
    # launch's persistent workers longest first; B = 1 with several streams = batches in flight.
    B = max(1, min(args.a3_batches_per_launch or args.a3_steps, args.a3_steps))
    nlaunch = -(-args.a3_steps // B)
    S = max(1, min(args.a3_streams, nlaunch))
    occ_r, s_r, g_r = occ_d.repeat(B, 1), s_d.repeat(B, 1), g_d.repeat(B, 1)
    wpc = args.a3_workers_per_cu if B == 1 else args.a3_residency
    lanes = []
    for _ in range(S):
        ctx = L.pmp_create(torch.cuda.current_device())
        _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, wpc), "workers")
        _lib.check(ctx, L.pmp_set_resident_per_cu(ctx, args.a3_residency), "residency")
        lanes.append(dict(ctx=ctx, stream=pool_stream(torch, len(lanes)),
                          cost=torch.empty(B * nq, dtype=torch.float64, device="cuda"),
                          plen=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
                          path=torch.empty((B * nq, cap), dtype=torch.int32, device="cuda"),
                          nexp=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
                          st=torch.empty(B * nq, dtype=torch.int32, device="cuda")))
    ctr = torch.empty((B * nq, 4), dtype=torch.int64, device="cuda")

    def run(i, nb, counters=None):
        b = lanes[i % len(lanes)]
        rc = L.pmp_astar3d_batch(b["ctx"], b["stream"].cuda_stream, occ_r.data_ptr(), 1, X, Y, Z, 0, s_r.data_ptr(),
                                 g_r.data_ptr(), nq * nb, b["cost"].data_ptr(), b["plen"].data_ptr(),
                                 b["path"].data_ptr(), cap, b["nexp"].data_ptr(), None, 0, counters, b["st"].data_ptr())
        if rc:
            _lib.check(b["ctx"], rc, "pmp_astar3d_batch")

    wb = max(1, min(B, 2))
    _LABEL[0] = "astar3d_warmup"  # smaller launches than the timed ones: keyed apart in the profile
    run(0, wb, ctr.data_ptr())
    for i in range(1, len(lanes)):
        run(i, wb)
    torch.cuda.synchronize()
    _LABEL[0] = f"astar3d_x{B}"  # keyed by batches per launch: a profile of other launches is refused
    c = ctr[:nq].cpu().numpy()
    akeys = ("cost", "plen", "nexp", "st")
    ref_out = {k: lanes[0][k][:nq].clone() for k in akeys}
    assert np.isin(ref_out["st"].cpu().numpy(), (0, 1)).all(), "unexpected 3D A* statuses"
    plen, path = ref_out["plen"], lanes[0]["path"][:nq].clone()
    for b in lanes:
        for j in range(wb):
            assert torch.equal(b["cost"][j * nq:(j + 1) * nq], ref_out["cost"])
        poison([b[k] for k in akeys])
    shard.barrier(dist)
    torch.cuda.synchronize()
    evs = []
    nbs = [min(B, args.a3_steps - i * B) for i in range(nlaunch)]
    t0 = time.perf_counter()
    for i in range(nlaunch):
        b = lanes[i % len(lanes)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(b["stream"])
        run(i, nbs[i])
        e1.record(b["stream"])
        evs.append((e0, e1))
    torch.cuda.synchronize()
    shard.barrier(dist)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(e) for a, e in evs]))
    elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
    outs = []
    for li, b in enumerate(lanes[: min(S, nlaunch)]):
        last_nb = nbs[max(i for i in range(nlaunch) if i % S == li)]
        outs += [{k: b[k][j * nq:(j + 1) * nq] for k in akeys} for j in range(last_nb)]
    checked = check_timed("astar3d", ref_out, outs)
    cost = ref_out["cost"]
    gathered = None
    if args.scaling == "strong":
        # the fixed batch's records from every rank in input order; rank 0 plans the whole batch on its
        # own GPU (untimed) and compares
        gk = ("cost", "st", "nexp", "plen")
        gth = shard.all_gather_rows(dist, mine, {k: ref_out[k] for k in gk}, args.a3_queries, device="cuda")
        gathered = {"queries": args.a3_queries, "queries_this_rank": nq}
        if rank == 0:
            full = batch.astar3d_batch(occ_all, s_all, g_all, path_cap=cap)
            torch.cuda.synchronize()
            gathered["gathered_equal_single_rank"] = all(
                torch.equal(gth[k], full[f]) for k, f in zip(gk, ("cost", "status", "n_expanded", "path_len")))
    # per plan 55*E3 + 16*(P3 + Q3), with P3 the reference's pushes and Q3 <= P3
    # (every pushed entry popped at most once): 55*E3 + 32*P3
    alg_bytes = float(np.sum(55.0 * c[:, 2] + 32.0 * c[:, 0])) * float(np.mean(nbs))
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        th = cpu_threads()
        t = time.perf_counter()
        reps = 0
        while True:
            rc_, rs_ = O.astar3d_batch(occ, s, g, nthreads=th)
            if reps == 0:
                assert np.array_equal(rc_, cost.cpu().numpy()), "GPU/oracle 3D cost mismatch"
            reps += 1
            if time.perf_counter() - t > args.cpu_seconds:
                break
        dt = time.perf_counter() - t
        cpu = {"value": nq * reps / dt, "unit": "plans/s", "cores": th, "kind": "port",
               "sample": f"all {nq} C5 queries, repeated {reps}x, C restatement of AStar3D (oracle/pmp_oracle.c) "
                         f"with OpenMP over queries, {dt:.1f} s wall"}
    _LABEL[0] = "totp3d"
    traj = totp3d_leg(args, torch, dist, world, rank, plen, path, (X, Y, Z)) if "totp" in args.legs.split(",") else None
    _LABEL[0] = "setup"
    torch.cuda.synchronize()
    for b in lanes:  # the lanes' scratch (about 15 GB each) is not needed by the other legs
        L.pmp_destroy(b["ctx"])
    plans = (args.a3_queries if args.scaling == "strong" else nq * world) * args.a3_steps
    return {"metric": "3D A* plans/sec, Grid3D(26,20,16) door scenario, 8192 queries", "value": plans / elapsed,
            "unit": "plans/s", "queries_per_gpu": nq, "steps": args.a3_steps,
            "scaling": args.scaling, "strong_scaling_gather": gathered,
            "ms_per_step": elapsed / args.a3_steps * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "streams": len(lanes), "batches_per_launch": B, "timed_launches_checked": checked,
            "workers_per_cu": wpc, "resident_per_cu": args.a3_residency,
            "config": {"workload": "C5: Grid3D(26,20,16) door, random.seed(i) pairs, safety bubbles r=1, euclidean"},
            "roofline": with_issue(with_traffic({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                                 "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                                                 "algorithmic_bytes_per_launch": alg_bytes},
                                                "astar3d_kernel", f"astar3d_x{B}"),
                                   "astar3d_kernel", f"astar3d_x{B}", float(c[:, 2].sum()) * B, "expansion"),
            "detail": {"expansions_per_batch": int(c[:, 2].sum()), "reference_pushes_per_batch": int(c[:, 0].sum()),
                       "heap_pops_per_batch": int(c[:, 1].sum()), "max_heap_entries": int(c[:, 3].max())},
            "cpu_baseline": cpu, "trajectory": traj}


def totp3d_leg(args, torch, dist, world, rank, plen, path, dims):
    """C5's step after planning (examples/3d_example.py:93-128): TimeOptimalTrajectory3D.generate() on
    every path the 3D A* leg planned, with the example's constraints (max velocity 2 / 2 / 1.5,
    max acceleration 1.5 / 1.5 / 1.0, time step 0.05, path_resolution 0.05).  One step = one launch
    over all the paths; the oracle (C restatement, OpenMP) timed on the same paths beside it."""
    from python_motion_planning_amd import _lib, batch

    X, Y, Z = dims
    pl = plen.cpu().numpy()
    P = path.cpu().numpy()
    paths = []
    for q in range(len(pl)):
        v = P[q, : pl[q]].astype(np.int64)
        if len(v) >= 2:
            paths.append(np.stack([v // (Y * Z), (v // Z) % Y, v % Z], axis=1).astype(np.float64))
    cons = dict(max_velocity=(2.0, 2.0, 1.5), max_acceleration=(1.5, 1.5, 1.0), min_time_step=0.05,
                path_resolution=0.05)
    prm = _lib.TotpParams.make(**cons)
    first = batch.totp3d_batch(paths, prm)
    torch.cuda.synchronize()
    n_pts = first["n_points"].cpu().numpy()
    n_smp = first["n_samples"].cpu().numpy()
    assert (first["status"].cpu().numpy() == 0).all()
    pc = int(n_pts.max())
    L = _lib.load_library()
    ctx = _lib.context()
    npath = len(paths)
    off = np.zeros(npath + 1, np.int32)
    off[1:] = np.cumsum([len(a) for a in paths])
    flat = torch.as_tensor(np.concatenate(paths), device="cuda")
    off_d = torch.as_tensor(off, device="cuda")
    nmax = int(max(len(a) for a in paths))
    sc = int(first["s_values"].shape[1])
    out = {k: torch.empty_like(first[k]) for k in ("s_values", "s_dot", "s_ddot", "time", "n_samples", "n_points",
                                                   "total_time", "status")}
    pts = torch.empty((npath, pc, 12), dtype=torch.float64, device="cuda")

    def run(i):
        rc = L.pmp_totp3d_batch(ctx, _lib.stream_ptr(), ctypes.byref(prm), npath, flat.data_ptr(), off_d.data_ptr(),
                                nmax, sc, out["s_values"].data_ptr(), out["s_dot"].data_ptr(), out["s_ddot"].data_ptr(),
                                out["time"].data_ptr(), out["n_samples"].data_ptr(), pc, pts.data_ptr(),
                                out["n_points"].data_ptr(), out["total_time"].data_ptr(), out["status"].data_ptr(),
                                None, 0)
        if rc:
            _lib.check(ctx, rc, "pmp_totp3d_batch")

    elapsed, kern_ms = timed(torch, dist, run, args.a3_steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        th = cpu_threads()
        op = O.TotpParams.make(cons["max_velocity"], cons["max_acceleration"], cons["min_time_step"],
                               cons["path_resolution"])
        ref = O.totp3d_batch(paths, op, sample_cap=sc, point_cap=pc, nthreads=th)
        assert np.array_equal(ref["n_points"], out["n_points"].cpu().numpy()), "GPU/oracle trajectory length mismatch"
        np.testing.assert_allclose(ref["total_time"], out["total_time"].cpu().numpy(), rtol=1e-9)
        reps, dt = timed_cpu(lambda r: O.totp3d_batch(paths, op, sample_cap=sc, point_cap=pc, nthreads=th),
                             args.cpu_seconds)
        sub = paths[: max(1, npath // 16)]
        reps1, dt1 = timed_cpu(lambda r: O.totp3d_batch(sub, op, sample_cap=sc, point_cap=pc, nthreads=1), 1.0)
        cpu = {"value": npath * reps / dt, "unit": "trajectories/s", "cores": th, "kind": "port", "host": host_cpu(),
               "sample": f"all {npath} C5 paths x {reps}, C restatement of TimeOptimalTrajectory3D.generate() "
                         f"(oracle/pmp_oracle.c) with OpenMP over paths, {dt:.1f} s wall",
               "one_core": {"value": len(sub) * reps1 / dt1, "sample": f"{len(sub)} paths x {reps1}, {dt1:.1f} s"}}
    return {"metric": "C5 time-optimal trajectories/sec (TimeOptimalTrajectory3D.generate on the 3D A* paths)",
            "value": npath * args.a3_steps * world / elapsed, "unit": "trajectories/s", "paths_per_gpu": npath,
            "steps": args.a3_steps, "ms_per_step": elapsed / args.a3_steps * 1e3, "kernel_ms_per_launch": kern_ms,
            "dtype": "f64", "config": {"workload": "C5 paths, 3d_example.py constraints, path_resolution 0.05"},
            "roofline": None,
            "roofline_note": "latency-bound: two sequential velocity recurrences per path (each step depends on the "
                             "last through the centripetal term), one wave per path; no HBM or MFMA roofline applies",
            "detail": {"samples_per_launch": int(n_smp.sum()), "points_per_launch": int(n_pts.sum()),
                       "max_points": pc},
            "cpu_baseline": cpu}


def graphs_leg(args, torch, dist, world, rank):
    """Widened planners on the same measurement bar: ThetaStar /
    LazyThetaStar 2D on C2 queries (1024^2 grid, astar2d.hip THETA = 1 / 2), and LPAStar / DStarLite
    on README-grid queries (lpa.hip).  Each: plans/s over `--graph-steps` launches, HIP-event kernel
    time, and the oracle (C restatement, OpenMP or a loop) timed on a bounded sample beside it."""
    from python_motion_planning_amd import _lib, batch, shard, workloads as wl

    L = _lib.load_library()
    out = {}
    occ2, s2, g2 = wl.c2_workload(4096, pair_seed=1 + rank)
    nq = args.theta_queries
    s2, g2 = s2[:nq], g2[:nq]
    occ_bits = batch.occ_bits_device(occ2, torch)
    s2d, g2d = torch.as_tensor(s2, device="cuda"), torch.as_tensor(g2, device="cuda")
    # Batches per launch (as the headline): B of the steps' batches per launch, streamed through the
    # launch's persistent workers longest first; B = 1 with several streams = batches in flight.
    B = max(1, min(args.theta_batches_per_launch or args.graph_steps, args.graph_steps))
    nlaunch = -(-args.graph_steps // B)
    S = max(1, min(args.theta_streams, nlaunch))
    s_rep, g_rep = s2d.repeat(B, 1), g2d.repeat(B, 1)
    tw = args.theta_workers if B == 1 else 256 * args.theta_residency
    for algo in ("theta_star", "lazy_theta_star"):
        _LABEL[0] = algo + "_2d_warmup"
        lanes = []
        for _ in range(S):
            shared = not lanes and bool(_SHARED_CTX)
            ctx = _SHARED_CTX[0] if shared else L.pmp_create(torch.cuda.current_device())
            _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, args.theta_engine, 1 if args.theta_engine == 2 else 0),
                       "engine")
            _lib.check(ctx, L.pmp_astar2d_reserve(ctx, 1024, 1024, tw, 0), "reserve")
            if args.theta_residency:
                _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, args.theta_residency), "residency")
            lanes.append(dict(ctx=ctx, shared=shared, stream=pool_stream(torch, len(lanes)),
                              cost=torch.empty(B * nq, dtype=torch.float64, device="cuda"),
                              plen=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
                              path=torch.empty((B * nq, 8192), dtype=torch.int32, device="cuda"),
                              nexp=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
                              st=torch.empty(B * nq, dtype=torch.int32, device="cuda")))
        ctr = torch.empty((nq, 4), dtype=torch.int64, device="cuda")

        def run(i, nb, algo=algo, counters=None):
            b = lanes[i % len(lanes)]
            rc = L.pmp_graph2d_batch(b["ctx"], b["stream"].cuda_stream, _lib.ALGOS[algo], occ_bits.data_ptr(), 1024, 1024,
                                     0, s_rep.data_ptr(), g_rep.data_ptr(), nq * nb, b["cost"].data_ptr(),
                                     b["plen"].data_ptr(), b["path"].data_ptr(), 8192, b["nexp"].data_ptr(), None, 0,
                                     counters, b["st"].data_ptr())
            if rc:
                _lib.check(b["ctx"], rc, "pmp_graph2d_batch")

        run(0, 1, counters=ctr.data_ptr())
        for i in range(1, len(lanes)):
            run(i, 1)
        # a warmup of the timed launch's size: it first-touches every slot's per-query state (Theta*'s
        # CLOSED parents are not the headline's: a 4096-query warmup left two thirds of the 12,288
        # slots' 4 MB to be touched inside the timed launch -- Theta* then read below Lazy Theta*)
        if B > 1:
            for i in range(len(lanes)):
                run(i, B)
        torch.cuda.synchronize()
        _LABEL[0] = f"{algo}_2d_x{B}"
        r = {"cost": lanes[0]["cost"][:nq].clone(), "status": lanes[0]["st"][:nq].clone()}
        assert (r["status"] == 0).all(), f"unexpected {algo} statuses"
        for b in lanes[1:]:
            assert torch.equal(b["cost"][:nq], r["cost"])
        gkeys = ("cost", "plen", "nexp", "st")
        ref_out = {k: lanes[0][k][:nq].clone() for k in gkeys}
        for b in lanes:
            poison([b[k] for k in gkeys])
        c = ctr.cpu().numpy()
        shard.barrier(dist)
        torch.cuda.synchronize()
        evs = []
        nbs = [min(B, args.graph_steps - i * B) for i in range(nlaunch)]
        t0 = time.perf_counter()
        for i in range(nlaunch):
            b = lanes[i % len(lanes)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(b["stream"])
            run(i, nbs[i])
            e1.record(b["stream"])
            evs.append((e0, e1))
        torch.cuda.synchronize()
        shard.barrier(dist)
        elapsed = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(e) for a, e in evs]))
        elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
        outs = []
        for li, b in enumerate(lanes[: min(S, nlaunch)]):
            last_nb = nbs[max(i for i in range(nlaunch) if i % S == li)]
            outs += [{k: b[k][j * nq:(j + 1) * nq] for k in gkeys} for j in range(last_nb)]
        checked = check_timed(algo, ref_out, outs)
        for b in lanes:  # their scratch (about 40 GB each with the Theta* parents) is not needed later
            if not b["shared"]:
                L.pmp_destroy(b["ctx"])
        lanes.clear()
        alg = astar_algorithmic_bytes(c) * float(np.mean(nbs))
        achieved = alg / (kern_ms * 1e-3) / 1e9
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            ns, th = nq, cpu_threads()  # the whole batch: about 3.5 s of wall on the box's 16 cores
            t = time.perf_counter()
            ref = O.astar2d_batch(occ2, s2[:ns], g2[:ns], path_cap=8192, nthreads=th, algo=algo)
            dt = time.perf_counter() - t
            assert np.array_equal(ref["cost"], r["cost"][:ns].cpu().numpy()), f"GPU/oracle {algo} cost mismatch"
            cpu = {"value": ns / dt, "unit": "plans/s", "cores": th, "kind": "port",
                   "sample": f"first {ns} of the {nq} queries, C restatement (oracle/pmp_oracle.c) with OpenMP over "
                             f"queries, {dt:.1f} s wall"}
        out[algo + "_2d"] = {
            "metric": f"{algo} 2D plans/sec on the C2 1024^2 grid", "value": nq * args.graph_steps * world / elapsed,
            "unit": "plans/s", "queries_per_gpu": nq, "steps": args.graph_steps, "streams": S,
            "batches_per_launch": B, "workers": tw, "resident_per_cu": args.theta_residency,
            "engine": "multi-query (4 per wave, astar2d_mq.hip)" if args.theta_engine == 2 else "one query per wave",
            "timed_launches_checked": checked,
            "ms_per_step": elapsed / args.graph_steps * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "roofline": with_traffic({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": achieved / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": alg,
                                      "note": "A*'s 19E + 16(P+Q) bytes; the line-of-sight cells are not counted"},
                                     "theta2d_kernel" if algo == "theta_star" else "lazy_theta2d_kernel", f"{algo}_2d_x{B}"),
            "detail": {"expansions_per_batch": int(c[:, 2].sum()), "pushes_per_batch": int(c[:, 0].sum())},
            "cpu_baseline": cpu}
    while _SHARED_CTX:
        L.pmp_destroy(_SHARED_CTX.pop())

    occ = wl.readme_grid()
    free = np.argwhere(occ == 0)
    rng = np.random.default_rng(3 + rank)
    nl = args.lpa_queries
    sl = free[rng.integers(len(free), size=nl)].astype(np.int32)
    gl = free[rng.integers(len(free), size=nl)].astype(np.int32)
    s_d, g_d = torch.as_tensor(sl, device="cuda"), torch.as_tensor(gl, device="cuda")
    lpa_streams = [pool_stream(torch, i) for i in range(max(1, args.lpa_streams))]
    if args.lpa_workers_per_cu:
        for sm in [torch.cuda.current_stream()] + lpa_streams:
            with torch.cuda.stream(sm):
                _lib.check(_lib.context(), _lib.load_library().pmp_set_workers_per_cu(
                    _lib.context(), args.lpa_workers_per_cu), "workers")
    for lite in (False, True):
        _LABEL[0] = "dstar_lite" if lite else "lpa_star"

        def run(i, lite=lite, counters=False):
            return batch.lpastar2d_batch(occ, s_d, g_d, counters=counters, lite=lite)
        r = run(0, counters=True)
        for sm in lpa_streams:  # each stream's context and scratch, before the timed region
            with torch.cuda.stream(sm):
                run(0)
        torch.cuda.synchronize()
        c = r["counters"].cpu().numpy()
        last = []
        elapsed, kern_ms = timed(torch, dist, run, args.graph_steps, streams=lpa_streams, last=last)
        checked = check_timed("lpa", {k: r[k] for k in ("cost", "n_expanded", "status", "path_len")}, last)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            th = cpu_threads()
            t = time.perf_counter()
            reps = 0
            while True:
                ref = O.lpastar2d_batch(occ, sl, gl, lite=lite, nthreads=th)
                if reps == 0:
                    assert np.array_equal(ref["cost"], r["cost"].cpu().numpy()), "GPU/oracle LPA* cost mismatch"
                reps += 1
                if time.perf_counter() - t > 2.0:
                    break
            dt = time.perf_counter() - t
            cpu = {"value": nl * reps / dt, "unit": "plans/s", "cores": th, "kind": "port",
                   "sample": f"all {nl} queries, repeated {reps}x, C restatement (oracle/pmp_oracle.c) with OpenMP "
                             f"over queries, {dt:.1f} s wall"}
        name = "dstar_lite" if lite else "lpa_star"
        alg = lpa_bytes(c[:, 1].sum(), c[:, 0].sum())
        out[name] = {
            "metric": f"{name} plans/sec on the README 51x31 grid ({nl} random free-cell pairs)",
            "value": nl * args.graph_steps * world / elapsed, "unit": "plans/s", "queries_per_gpu": nl,
            "steps": args.graph_steps, "ms_per_step": elapsed / args.graph_steps * 1e3, "kernel_ms_per_launch": kern_ms,
            "timed_launches_checked": checked, "dtype": "f64",
            "roofline": with_traffic(hbm_roof(alg, kern_ms, LPA_BYTES_NOTE), "lpa_kernel", name),
            "roofline_note": "latency-bound list machine (U scans / shifts of a few hundred entries per expansion, "
                             "L2-resident): a small frac is the expected reading",
            "detail": {"expansions_per_launch": int(c[:, 1].sum()), "pushes_per_launch": int(c[:, 0].sum()),
                       "max_U": int(c[:, 3].max())},
            "cpu_baseline": cpu}

    # incremental replanning: plan() + 4 OnPress obstacle edits per query, each followed by a re-plan
    nt = 4
    inner = np.argwhere(np.ones((occ.shape[0] - 2, occ.shape[1] - 2), bool)) + 1
    T = inner[rng.integers(len(inner), size=(nl, nt))].astype(np.int32)
    t_d = torch.as_tensor(T, device="cuda")
    for lite in (False, True):
        _LABEL[0] = ("dstar_lite" if lite else "lpa_star") + "_replan"

        def run(i, lite=lite, counters=False):
            return batch.lpastar2d_replan_batch(occ, s_d, g_d, t_d, lite=lite, counters=counters)
        for sm in lpa_streams:
            with torch.cuda.stream(sm):
                run(0)
        r = run(0, counters=True)
        torch.cuda.synchronize()
        ne = r["n_expanded"].cpu().numpy()
        cr = r["counters"].cpu().numpy()
        last = []
        elapsed, kern_ms = timed(torch, dist, run, args.graph_steps, streams=lpa_streams, last=last)
        checked = check_timed("lpa_replan", {k: r[k] for k in ("cost", "n_expanded", "status", "path_len")}, last)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            th = cpu_threads()
            ref = O.lpastar2d_replan_batch(occ, sl, gl, T, lite=lite, nthreads=th)
            assert np.array_equal(ref["cost"], r["cost"].cpu().numpy()), "GPU/oracle replan cost mismatch"
            reps, dt = timed_cpu(lambda i: O.lpastar2d_replan_batch(occ, sl, gl, T, lite=lite, nthreads=th), 2.0)
            ns1 = min(2048, nl)
            reps1, dt1 = timed_cpu(lambda i: O.lpastar2d_replan_batch(occ, sl[:ns1], gl[:ns1], T[:ns1], lite=lite,
                                                                      nthreads=1), 2.0)
            cpu = {"value": nl * (nt + 1) * reps / dt, "unit": "plans/s", "cores": th, "kind": "port",
                   "sample": f"all {nl} sessions ({nt} edits each) x {reps}, C restatement with OpenMP over "
                             f"sessions, {dt:.1f} s wall",
                   "one_core": {"value": ns1 * (nt + 1) * reps1 / dt1,
                                "sample": f"{ns1} sessions x {reps1}, {dt1:.1f} s"}}
        name = ("dstar_lite" if lite else "lpa_star") + "_replan"
        out[name] = {
            "metric": f"{name} plans/sec (plan() + {nt} OnPress edits per session, README grid, {nl} sessions)",
            "value": nl * (nt + 1) * args.graph_steps * world / elapsed, "unit": "plans/s", "sessions_per_gpu": nl,
            "steps": args.graph_steps, "ms_per_step": elapsed / args.graph_steps * 1e3,
            "kernel_ms_per_launch": kern_ms, "timed_launches_checked": checked, "dtype": "f64",
            "roofline": with_traffic(hbm_roof(lpa_bytes(cr[:, 1].sum(), cr[:, 0].sum()), kern_ms, LPA_BYTES_NOTE),
                                     "lpa_kernel", name),
            "roofline_note": "latency-bound list machine, as lpa_star",
            "detail": {"expansions_per_launch": int(np.maximum(ne, 0).sum())}, "cpu_baseline": cpu}
    _LABEL[0] = "setup"
    return out


def dstar_leg(args, torch, dist, world, rank):
    """DStar.plan (d_star.py:75-156, processState loop over the list-semantics OPEN) on C2-style grids:
    10 % random obstacles, boundary walls, start/goal pairs from the largest free component, at 256^2
    and 512^2 (SURVEY.md §6 measured the reference there).  One timed step = one launch over the
    rank's queries."""
    from python_motion_planning_amd import _lib, batch, shard, workloads as wl

    L = _lib.load_library()
    out = {}
    for W, nq in ((256, args.dstar_queries), (512, args.dstar_queries)):
        occ, s, g = wl.c2_workload(nq=nq, W=W, H=W, density=0.1, grid_seed=4, pair_seed=5 + rank)
        _LABEL[0] = f"dstar_{W}_warmup"
        s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
        bits = batch.occ_bits_device(occ, torch)
        # B batches per launch (continuous batching, as the headline), or B = 1 with batches in flight
        # on their own streams (own pmp_ctx each)
        B = max(1, min(args.dstar_batches_per_launch or args.dstar_steps, args.dstar_steps))
        nlaunch = -(-args.dstar_steps // B)
        S = max(1, min(args.dstar_streams, nlaunch))
        s_rep, g_rep = s_d.repeat(B, 1), g_d.repeat(B, 1)
        lanes = []
        for _ in range(S):
            ctx = L.pmp_create(torch.cuda.current_device())
            _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, args.dstar_workers_per_cu), "workers")
            _lib.check(ctx, L.pmp_set_resident_per_cu(ctx, args.dstar_residency), "residency")
            lanes.append(dict(ctx=ctx, stream=pool_stream(torch, len(lanes)),
                              cost=torch.empty(B * nq, dtype=torch.float64, device="cuda"),
                              plen=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
                              path=torch.empty((B * nq, 4 * W), dtype=torch.int32, device="cuda"),
                              npr=torch.empty(B * nq, dtype=torch.int64, device="cuda"),
                              st=torch.empty(B * nq, dtype=torch.int32, device="cuda")))

        def run(i, nb):
            b = lanes[i % len(lanes)]
            rc = L.pmp_dstar2d_batch(b["ctx"], b["stream"].cuda_stream, bits.data_ptr(), W, W, s_rep.data_ptr(),
                                     g_rep.data_ptr(), nq * nb, b["cost"].data_ptr(), b["plen"].data_ptr(),
                                     b["path"].data_ptr(), 4 * W, b["npr"].data_ptr(), b["st"].data_ptr(), 0)
            if rc:
                _lib.check(b["ctx"], rc, "pmp_dstar2d_batch")

        for i in range(len(lanes)):
            run(i, 1)
        torch.cuda.synchronize()
        _LABEL[0] = f"dstar_{W}"
        r = {"cost": lanes[0]["cost"][:nq], "n_process": lanes[0]["npr"][:nq], "status": lanes[0]["st"][:nq]}
        for b in lanes[1:]:
            assert torch.equal(b["cost"][:nq], r["cost"]) and torch.equal(b["npr"][:nq], r["n_process"])
        npr = r["n_process"].cpu().numpy()
        st = r["status"].cpu().numpy()
        dkeys = ("cost", "plen", "npr", "st")
        ref_out = {k: lanes[0][k][:nq].clone() for k in dkeys}
        for b in lanes:
            poison([b[k] for k in dkeys])
        shard.barrier(dist)
        torch.cuda.synchronize()
        evs = []
        nbs = [min(B, args.dstar_steps - i * B) for i in range(nlaunch)]
        t0 = time.perf_counter()
        for i in range(nlaunch):
            b = lanes[i % len(lanes)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(b["stream"])
            run(i, nbs[i])
            e1.record(b["stream"])
            evs.append((e0, e1))
        torch.cuda.synchronize()
        shard.barrier(dist)
        elapsed = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(e) for a, e in evs]))
        elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
        outs = []
        for li, b in enumerate(lanes[: min(S, nlaunch)]):
            last_nb = nbs[max(i for i in range(nlaunch) if i % S == li)]
            outs += [{k: b[k][j * nq:(j + 1) * nq] for k in dkeys} for j in range(last_nb)]
        checked = check_timed(f"dstar_{W}", ref_out, outs)
        r = {"cost": ref_out["cost"], "n_process": ref_out["npr"], "status": ref_out["st"]}
        torch.cuda.synchronize()
        for b in lanes:
            L.pmp_destroy(b["ctx"])
        lanes.clear()
        # algorithmic bytes per processState: the 3x3 block of cell states (h, k f64 + tag / parent:
        # 24 B each) read + ~2 OPEN entries (16 B) inserted / removed
        alg = float(npr.sum()) * (9 * 24 + 2 * 16) * float(np.mean(nbs))
        achieved = alg / (kern_ms * 1e-3) / 1e9
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            th = cpu_threads()
            ns = min(nq, 4 * th)
            ref = O.dstar2d_batch(occ, s[:ns], g[:ns], nthreads=th)
            assert np.array_equal(ref["cost"], r["cost"][:ns].cpu().numpy()), "GPU/oracle D* cost mismatch"
            assert np.array_equal(ref["n_process"], npr[:ns]), "GPU/oracle D* processState-count mismatch"
            reps, dt = timed_cpu(lambda i: O.dstar2d_batch(occ, s[:ns], g[:ns], nthreads=th), 2.0)
            reps1, dt1 = timed_cpu(lambda i: O.dstar2d_batch(occ, s[:2], g[:2], nthreads=1), 1.0)
            cpu = {"value": ns * reps / dt, "unit": "plans/s", "cores": th, "kind": "port",
                   "sample": f"first {ns} of the {nq} queries x {reps}, C restatement of DStar (list OPEN, "
                             f"first-minimum scans like d_star.py:220-259) with OpenMP over queries, {dt:.1f} s wall",
                   "one_core": {"value": 2 * reps1 / dt1, "sample": f"2 queries x {reps1}, {dt1:.1f} s"}}
        out[f"dstar_{W}"] = {
            "metric": f"DStar plans/sec on a {W}x{W} grid (10% obstacles, {nq} random start/goal pairs)",
            "value": nq * args.dstar_steps * world / elapsed, "unit": "plans/s", "queries_per_gpu": nq,
            "steps": args.dstar_steps, "ms_per_step": elapsed / args.dstar_steps * 1e3, "kernel_ms_per_launch": kern_ms,
            "dtype": "f64", "streams": S, "batches_per_launch": B, "timed_launches_checked": checked,
            "roofline": with_traffic({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                                      "algorithmic_bytes_per_launch": alg,
                                      "bytes_note": "248 B per processState (3x3 cell states 9 x 24 B + 2 OPEN "
                                                    "entries x 16 B); latency-bound, one wave per query"},
                                     "dstar_kernel", f"dstar_{W}:dstar_kernel"),
            "detail": {"process_state_per_launch": int(npr.sum()), "max_process_state_query": int(npr.max()),
                       "statuses": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}},
            "cpu_baseline": cpu}
    _LABEL[0] = "setup"
    return out


def dyn3d_leg(args, torch, dist, world, rank):
    """The 3D incremental planners on the C5 workload (Grid3D(26,20,16) door, per-query safety
    bubbles, random.seed(i) pairs): DStar3D (d_star3d.py:100-149, dstar3d.hip) and LPAStar3D
    (lpa_star3d.py:78-124, lpa3d.hip), each as plan() alone and as a replanning session (plan() + 2
    dynamic-obstacle calls: DStar3D.apply_dynamic_obstacles of 2 voxels, LPAStar3D.apply_change
    blocking a voxel).  One timed step = one launch over the rank's queries."""
    from python_motion_planning_amd import _lib, batch, shard, workloads as wl

    nq = args.dyn3d_queries
    occ, s, g = wl.c5_workload(nq, first_seed=rank * nq)
    X, Y, Z = occ.shape[1:]
    rng = np.random.default_rng(40 + rank)
    inner = rng.integers(1, [X - 1, Y - 1, Z - 1], size=(nq, 2, 2, 3)).astype(np.int32)
    changes = np.concatenate([inner[:, :, 0, :], np.ones((nq, 2, 1), np.int32)], axis=2)
    s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
    # the grids packed once (device words), outside the timed region
    bits = torch.as_tensor(np.ascontiguousarray(np.stack([batch.pack_bits(o) for o in occ])).view(np.int32),
                           device="cuda")
    # B batches per launch (continuous batching through the launch's persistent workers, longest
    # first), or B = 1 with batches in flight: consecutive launches on different streams (the
    # per-stream contexts of _lib.context), so the next launch's workers fill the CUs the finished ones free
    B = max(1, min(args.dyn3d_batches_per_launch or args.dyn3d_steps, args.dyn3d_steps))
    nlaunch = -(-args.dyn3d_steps // B)
    streams = [pool_stream(torch, i) for i in range(max(1, min(args.dyn3d_streams, nlaunch)))]
    s_rep, g_rep, bits_rep = s_d.repeat(B, 1), g_d.repeat(B, 1), bits.repeat(B, 1)
    out = {}
    for kind, rounds in (("dstar3d", None), ("dstar3d", inner), ("lpastar3d", None), ("lpastar3d", changes)):
        _LABEL[0] = kind + ("" if rounds is None else "_replan") + "_warmup"
        rd = None if rounds is None else torch.as_tensor(rounds, device="cuda")
        rd_rep = None if rd is None else rd.repeat(B, *([1] * (rd.dim() - 1)))

        def run(i, nb=1, kind=kind, rd_rep=rd_rep, counters=False):
            m = nq * nb
            r_ = None if rd_rep is None else rd_rep[:m]
            with torch.cuda.stream(streams[i % len(streams)]):
                if kind == "lpastar3d" and args.lpa3d_workers_per_cu:
                    _lib.check(_lib.context(), _lib.load_library().pmp_set_workers_per_cu(
                        _lib.context(), args.lpa3d_workers_per_cu), "workers")
                if kind == "dstar3d":
                    return batch.dstar3d_batch(occ.shape, s_rep[:m], g_rep[:m], r_, path_cap=X * Y * Z + 1,
                                               occ_bits=bits_rep[:m])
                return batch.lpastar3d_batch(occ.shape, s_rep[:m], g_rep[:m], r_, path_cap=X * Y * Z + 1,
                                             occ_bits=bits_rep[:m], counters=counters)

        r = run(0, counters=True)
        torch.cuda.synchronize()
        nkey = "n_process" if kind == "dstar3d" else "n_expanded"
        nexp = r[nkey].cpu().numpy()
        pushes = int(r["counters"][:, 0].sum().item()) if r.get("counters") is not None else None
        st = r["status"].cpu().numpy()
        cost0 = r["cost"].cpu().numpy()
        ref_out = {k: r[k].clone() for k in ("cost", nkey, "status", "path_len")}
        del r
        # one untimed launch per stream whose outputs are freed: the timed launches then reuse those
        # blocks from the stream's caching-allocator pool instead of allocating (and synchronising)
        nbs = [min(B, args.dyn3d_steps - i * B) for i in range(nlaunch)]
        for i in range(len(streams)):
            run(i, nbs[i])
        torch.cuda.synchronize()
        _LABEL[0] = kind + ("" if rounds is None else "_replan") + f"_x{B}"
        shard.barrier(dist)
        torch.cuda.synchronize()
        evs = []
        lastr = {}
        t0 = time.perf_counter()
        for i in range(nlaunch):
            sm = streams[i % len(streams)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sm)
            lastr[i % len(streams)] = (run(i, nbs[i]), nbs[i])
            e1.record(sm)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        shard.barrier(dist)
        elapsed = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(e) for a, e in evs]))
        elapsed, kern_ms = shard.max_over_ranks(dist, [elapsed, kern_ms], "cuda")
        outs = [{k: rr[k][j * nq:(j + 1) * nq] for k in ref_out} for rr, nb_ in lastr.values() for j in range(nb_)]
        checked = check_timed(kind, ref_out, outs)
        del lastr, outs
        R = 1 if rounds is None else rounds.shape[1] + 1
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            th = cpu_threads()
            ns = min(nq, 64 * th)
            ref = O.graph3d_dynamic_batch(kind, occ[:ns], s[:ns], g[:ns], None if rounds is None else rounds[:ns],
                                          nthreads=th)
            assert np.array_equal(ref["n"], nexp[:ns]), f"GPU/oracle {kind} expansion-count mismatch"
            assert np.array_equal(ref["cost"], cost0[:ns]), f"GPU/oracle {kind} cost mismatch"
            reps, dt = timed_cpu(lambda i: O.graph3d_dynamic_batch(kind, occ[:ns], s[:ns], g[:ns],
                                                                   None if rounds is None else rounds[:ns], nthreads=th),
                                 2.0)
            reps1, dt1 = timed_cpu(lambda i: O.graph3d_dynamic_batch(kind, occ[:16], s[:16], g[:16],
                                                                     None if rounds is None else rounds[:16],
                                                                     nthreads=1), 1.0)
            cpu = {"value": ns * R * reps / dt, "unit": "plans/s", "cores": th, "kind": "port",
                   "sample": f"first {ns} of the {nq} queries x {reps}, C restatement (list-semantics OPEN / U, "
                             f"as the reference) with OpenMP over queries, {dt:.1f} s wall",
                   "one_core": {"value": 16 * R * reps1 / dt1, "sample": f"16 queries x {reps1}, {dt1:.1f} s"}}
        name = kind + ("" if rounds is None else "_replan")
        out[name] = {
            "metric": f"{kind} plans/sec on C5 (Grid3D 26x20x16 door, {nq} queries"
                      + ("" if rounds is None else f", plan + {R - 1} dynamic-obstacle calls per session") + ")",
            "value": nq * R * args.dyn3d_steps * world / elapsed, "unit": "plans/s", "queries_per_gpu": nq,
            "timed_launches_checked": checked,
            "steps": args.dyn3d_steps, "ms_per_step": elapsed / args.dyn3d_steps * 1e3, "kernel_ms_per_launch": kern_ms,
            "dtype": "f64",
            "roofline": with_issue(with_traffic(dyn3d_roof(kind, int(np.maximum(nexp, 0).sum() * np.mean(nbs)),
                                                           None if pushes is None else int(pushes * np.mean(nbs)),
                                                           kern_ms),
                                                "dstar3d_kernel" if kind == "dstar3d" else "lpa3d_kernel", f"{name}_x{B}"),
                                   "dstar3d_kernel" if kind == "dstar3d" else "lpa3d_kernel", f"{name}_x{B}",
                                   float(np.maximum(nexp, 0).sum() * np.mean(nbs)),
                                   "processState" if kind == "dstar3d" else "expansion"),
            "roofline_note": "latency-bound list machines (OPEN / U with Python-list semantics): a small frac is "
                             "the expected reading",
            "streams": len(streams), "batches_per_launch": B,
            "detail": {"expansions_per_batch": int(np.maximum(nexp, 0).sum()),
                       "statuses": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}},
            "cpu_baseline": cpu}
    _LABEL[0] = "setup"
    return out


def latency_leg(args, torch, dist, world, rank):
    """Single-query latency of the drop-in AStar.plan() end to end (the
    set -> bit-grid ingestion, the kernel, the path / CLOSED-Node marshalling): C1 (the README
    query, 51x31, 579 expansions) and one C2 query (1024^2 grid given as a 213k-tuple obstacle set).
    Median wall time of repeated calls, with the parts timed separately; the reference measured
    14.8-26.8 ms for C1 and 2.76 s mean per C2 query in CPython."""
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import batch, workloads as wl

    out = {}
    cases = [("c1_readme", wl.readme_grid(), (5, 5), (45, 25), 50)]
    occ2, s2, g2 = wl.c2_workload(nq=64)
    # a C2 query of median length: the 32nd longest of 64 by octile distance
    from python_motion_planning_amd import shard

    k = int(np.argsort(shard.octile(s2, g2))[32])
    cases.append(("c2_1024_one_query", occ2, tuple(int(v) for v in s2[k]), tuple(int(v) for v in g2[k]), 5))
    for name, occ, s, g, reps in cases:
        _LABEL[0] = name
        W, H = occ.shape
        env = pmp.Grid(W, H)
        env.update({(int(x), int(y)) for x, y in np.argwhere(occ)})
        planner = pmp.AStar(s, g, env)
        planner.plan()  # warm: library, context, allocator
        torch.cuda.synchronize()
        walls, ingest, kern, nodes = [], [], [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            cost, path, expand = planner.plan()
            walls.append(time.perf_counter() - t0)
        for _ in range(min(reps, 5)):
            t0 = time.perf_counter()
            words = env.occupancy_words()
            t1 = time.perf_counter()
            occ_bits = torch.as_tensor(words.view(np.int32), device="cuda")
            r = batch.astar2d_batch((W, H), np.array([s]), np.array([g]), path_cap=W * H + 1, expand_cap=W * H,
                                    occ_bits=occ_bits)
            ne = int(r["n_expanded"][0])
            t2 = time.perf_counter()
            exp = r["expand"][0, :ne].cpu().numpy().astype(np.uint32)
            planner._expand_nodes(exp, H)
            t3 = time.perf_counter()
            ingest.append(t1 - t0)
            kern.append(t2 - t1)
            nodes.append(t3 - t2)
        cpu = None
        if rank == 0 and not args.no_cpu_baseline:
            from oracle import oracle as O

            t0 = time.perf_counter()
            n1 = 0
            while True:
                O.astar2d(occ, s, g)
                n1 += 1
                if time.perf_counter() - t0 > 1.0:
                    break
            cpu = {"value": (time.perf_counter() - t0) / n1 * 1e3, "unit": "ms", "cores": 1, "kind": "port",
                   "sample": f"{n1} calls of the C restatement (oracle/pmp_oracle.c astar2d with the CLOSED order)"}
        out[name] = {"metric": f"drop-in AStar.plan() latency, {name}", "value": float(np.median(walls)) * 1e3,
                     "unit": "ms", "higher_is_better": False, "calls": reps, "expansions": len(expand),
                     "parts_ms": {"set_to_bitgrid": float(np.median(ingest)) * 1e3,
                                  "kernel_and_sync": float(np.median(kern)) * 1e3,
                                  "closed_node_list": float(np.median(nodes)) * 1e3,
                                  "note": "plan() packs the set while the kernel runs on the Grid's last upload "
                                          "(re-run if the set changed); one pinned D2H per query"},
                     "reference_python_ms": "14.8-26.8 (SURVEY.md §6)" if name == "c1_readme" else
                                            "2760 mean per C2 query (SURVEY.md §6)",
                     "cpu_baseline": cpu}
    _LABEL[0] = "setup"
    return out


def track_leg(args, torch, dist, world, rank, kind):
    """LQR / MPC tracking (lqr.py:58-86 / mpc.py:66-94) for the C4 agents: one timed step = one launch
    running `iters` plan iterations of every agent (MPC at p = 30, m = 8, ADMM to 1e-9)."""
    from python_motion_planning_amd import _lib, batch, local_planner, shard

    iters = args.track_iters
    occ, states, goals, mine = c4_share(args, args.track_agents, world, rank)
    na = len(states)
    paths = dwa_inputs(torch, occ, states, goals)
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(local_planner.LocalPlanner.DEFAULTS)
    kw = dict(lqr_params=_lib.LQRParams.make()) if kind == "lqr" else dict(mpc_params=_lib.MPCParams.make(p=30))
    st0 = torch.tensor(states, dtype=torch.float64, device="cuda")
    st = st0.clone()
    up = torch.zeros((na, 2), dtype=torch.float64, device="cuda")
    gd = torch.tensor(goals, dtype=torch.float64, device="cuda")
    xyd = torch.tensor(xy, dtype=torch.float64, device="cuda")
    offd = torch.tensor(off, dtype=torch.int32, device="cuda")
    _LABEL[0] = "lqr" if kind == "lqr" else "mpc_qp"
    # the first (untimed) launch also counts the QP solves it runs (pmp_set_stats): the MFMA work of
    # a launch is one assembly pass per solve, not per agent-step (rotation steps solve nothing)
    solves_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    sctx = _lib.context()
    L = _lib.load_library()
    _lib.check(sctx, L.pmp_set_stats(sctx, solves_d.data_ptr()), "pmp_set_stats")
    o = batch.track_step_batch(kind, lp, st, gd, xyd, offd, iters=iters, u_p=up, **kw)
    torch.cuda.synchronize()
    _lib.check(sctx, L.pmp_set_stats(sctx, None), "pmp_set_stats")
    qp_solves = int(solves_d.item())
    stepped = int(o["n_steps"].sum().item())
    admm = int(o["admm_iters"].sum().item())

    ref_out = {"u": o["u"].clone(), "n_steps": o["n_steps"].clone(), "admm_iters": o["admm_iters"].clone(),
               "state": st.clone(), "u_p": up.clone()}

    # every timed launch starts from its own copy of the initial states (made before the timed
    # region) and keeps its outputs, so each one is checked against the first launch's
    st_k = [st0.clone() for _ in range(args.track_steps)]
    up_k = [torch.zeros_like(up) for _ in range(args.track_steps)]
    outs = []

    def run(i):
        r = batch.track_step_batch(kind, lp, st_k[i], gd, xyd, offd, iters=iters, u_p=up_k[i], **kw)
        outs.append({"u": r["u"], "n_steps": r["n_steps"], "admm_iters": r["admm_iters"], "state": st_k[i],
                     "u_p": up_k[i]})
        return outs[-1]

    elapsed, kern_ms = timed(torch, dist, run, args.track_steps)
    checked = check_timed(kind, ref_out, outs)
    gathered = None
    steps_all = stepped * world
    if args.scaling == "strong":
        # the fixed agent set's records from every rank in agent order; rank 0 replays all the agents on
        # its own GPU (untimed, one launch) and compares
        g = shard.all_gather_rows(dist, mine, {k: ref_out[k] for k in ("u", "n_steps", "state", "u_p")},
                                  args.track_agents, device="cuda")
        steps_all = int(g["n_steps"].sum().item())
        gathered = {"agents": args.track_agents, "agents_this_rank": na, "agent_steps": steps_all}
        if rank == 0:
            occ1, st1, gl1, _ = c4_share(args, args.track_agents, 1, 0)
            xy1, off1 = batch.pack_paths(dwa_inputs(torch, occ1, st1, gl1))
            st1d = torch.tensor(st1, dtype=torch.float64, device="cuda")
            up1 = torch.zeros((len(st1), 2), dtype=torch.float64, device="cuda")
            o1 = batch.track_step_batch(kind, lp, st1d, torch.tensor(gl1, dtype=torch.float64, device="cuda"),
                                        torch.tensor(xy1, dtype=torch.float64, device="cuda"),
                                        torch.tensor(off1, dtype=torch.int32, device="cuda"), iters=iters, u_p=up1,
                                        **kw)
            torch.cuda.synchronize()
            full = {"u": o1["u"], "n_steps": o1["n_steps"], "state": st1d, "u_p": up1}
            gathered["gathered_equal_single_rank"] = all(torch.equal(g[k], full[k]) for k in full)
    mfma = None
    if kind == "mpc":
        # per ADMM iteration ~ 16x16 inverse matvec (512) + scans/projections (~150); assembly 2*16*16*3p (MFMA)
        flops = admm * 662.0 + qp_solves * 2 * 16 * 16 * 90
        # the assembly's matrix-core work (track.hip mpc_rows): per QP solve ceil(3p / 16) row blocks
        # x (2 MFMAs of y = S_x x + 4 K-slices x 2 MFMAs of H and g), 16 x 16 x 4 x 2 flops each
        per_solve = (-(-90 // 16)) * 10
        mfma_flops = qp_solves * per_solve * 16 * 16 * 4 * 2.0
        mfma_tf = mfma_flops / (kern_ms * 1e-3) / 1e12
        mfma = {"mfma_tflops": mfma_tf, "mfma_frac_of_fp64_peak": mfma_tf / 78.6,
                "mfma_util_pct_analytic": 100.0 * mfma_tf / 78.6,
                "qp_solves_per_launch": qp_solves, "mfma_instructions_per_launch": qp_solves * per_solve,
                "mfma_flops_per_qp_solve": per_solve * 16 * 16 * 4 * 2,
                "note": "H = S_u' Q S_u, y = S_x x, g = (S_u' Q) y on v_mfma_f64_16x16x4_f64, one assembly per QP "
                        "solve (pmp_set_stats count); the ADMM runs on the VALU (one 16x16 inverse per agent). "
                        "mfma_tflops is over the whole launch (track_mpc_step + track_mpc_solve kernels); "
                        "roofline.mfma_util_pct is the rocprofv3 busy-cycle figure of track_mpc_solve alone"}
    else:
        flops = stepped * 1200.0  # 3x3 Riccati update, 2x2 inverse, K e (lqr.py:116-141)
    achieved_tf = flops / (kern_ms * 1e-3) / 1e12
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        th = cpu_threads()
        t = time.perf_counter()
        tot, reps = 0, 0
        while True:  # repeat the batch until ~8 s of CPU wall time (the first pass is also checked)
            ost, oup, ou, ostat, onst, n_ = O.track_batch(
                kind, xy, off, goals, states, iters=iters, nthreads=th,
                mpc=O.MPCParams.default(p=30, eps_abs=1e-9, eps_rel=1e-9))
            if reps == 0:
                assert int(n_) == stepped, "GPU/oracle step-count mismatch"
            tot += int(n_)
            reps += 1
            if time.perf_counter() - t > args.cpu_seconds or reps >= 100000:
                break
        dt = time.perf_counter() - t
        cpu = {"value": tot / dt, "unit": "agent-steps/s", "cores": th, "kind": "port",
               "sample": f"all {na} C4 agents x {iters} plan iterations, repeated {reps}x, C restatement "
                         f"(oracle/pmp_oracle.c) with OpenMP over agents, {dt:.1f} s wall"}
    _LABEL[0] = "setup"
    name = "LQR" if kind == "lqr" else "MPC (p=30, m=8, ADMM QP)"
    return {"metric": f"{name} tracking agent-steps/sec", "value": steps_all * args.track_steps / elapsed,
            "unit": "agent-steps/s", "agents_per_gpu": na, "iterations_per_launch": iters, "steps": args.track_steps,
            "scaling": args.scaling, "strong_scaling_gather": gathered,
            "ms_per_step": elapsed / args.track_steps * 1e3, "kernel_ms_per_launch": kern_ms, "dtype": "f64",
            "config": {"workload": f"C4 agents on the README grid ({na} per launch), {iters} LQR/MPC plan iterations "
                                   f"per launch"},
            "roofline": with_mfma(with_traffic({"bound": "fp64-valu", "achieved": achieved_tf, "peak": 78.6,
                                                "unit": "TFLOP/s", "frac": achieved_tf / 78.6, "traffic": None},
                                               "track_kernel_lqr" if kind == "lqr" else "track_mpc_solve",
                                               "lqr" if kind == "lqr" else "mpc_qp"),
                                  "track_kernel_lqr" if kind == "lqr" else "track_mpc_solve"),
            "timed_launches_checked": checked, "mfma": mfma,
            "detail": {"agent_steps_per_launch": stepped, "admm_iterations_per_launch": admm},
            "cpu_baseline": cpu}


def _sig(v, n=4):
    """A number rounded to n significant digits (the compact line's precision)."""
    if v is None or not isinstance(v, (int, float)) or v == 0 or v != v:
        return v
    return float(f"{v:.{n}g}")


def compact_leg(rec: dict) -> dict:
    """One secondary leg in the headline line: value, unit, roofline frac and CPU-baseline value
    (the full record goes to the detail file)."""
    roof = rec.get("roofline") or {}
    cpu = rec.get("cpu_baseline") or {}
    out = {"value": _sig(rec.get("value")), "unit": rec.get("unit"), "frac": _sig(roof.get("frac"), 3),
           "cpu": _sig(cpu.get("value"))}
    if roof.get("traffic") and roof.get("algorithmic_bytes_per_launch"):
        out["traffic_x"] = _sig(roof["traffic"] / roof["algorithmic_bytes_per_launch"], 3)
    if rec.get("timed_launches_checked") is not None:
        out["checked"] = rec["timed_launches_checked"]
    if roof.get("mfma_util_pct") is not None:  # rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES pass (profiles/)
        out["mfma_util_pct"] = _sig(roof["mfma_util_pct"], 3)
    if rec.get("mfma"):  # the matrix-core share of the leg's own arithmetic, live
        out["mfma_tflops"] = _sig(rec["mfma"]["mfma_tflops"], 3)
        # the same work as a percentage of the f64 MFMA peak, comparable with mfma_util_pct
        out["mfma_util_pct_analytic"] = _sig(rec["mfma"]["mfma_util_pct_analytic"], 3)
    if roof.get("bytes_model"):
        out["bytes_model"] = roof["bytes_model"]
    iss = roof.get("issue") or {}
    if iss.get("valu_issue_frac") is not None:  # the SQ issue pass (profiles/): the binding resource
        out["valu_issue_frac"] = _sig(iss["valu_issue_frac"], 3)
        out["valu_per_unit"] = _sig(iss.get("valu_insts_per_unit"), 4)
        out["unit_of_issue"] = iss.get("unit")
    return out


def write_detail(args, out: dict):
    """The full per-leg records (every field of every leg) as JSON: --detail-out, default
    gpurun_out/bench_detail.json (merged back from a GPU box by gpurun).  Returns the path or None."""
    path = args.detail_out or os.path.join(REPO, "gpurun_out", "bench_detail.json")
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(path, REPO)
    except OSError:
        return None


def headline_line(out: dict, detail_path) -> dict:
    """The driver-parsed last stdout line (<= 4 KB): the headline with its roofline and CPU baseline,
    and a compact map of the secondary legs."""
    roof = dict(out["roofline"])
    roof = {k: (_sig(v) if isinstance(v, float) else v) for k, v in roof.items()}
    if isinstance(roof.get("issue"), dict):
        roof["issue"] = {k: (_sig(v, 4) if isinstance(v, float) else v) for k, v in roof["issue"].items()}
    cpu = out["cpu_baseline"]
    if cpu:
        host = cpu.get("host") or {}
        cpu = {"value": _sig(cpu["value"]), "unit": cpu["unit"], "cores": cpu["cores"], "kind": cpu["kind"],
               "sample": cpu["sample"], "cpu_model": host.get("model"),
               "one_core": _sig((cpu.get("one_core") or {}).get("value"))}
    d = out["detail"]
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    line["roofline"] = roof
    line["cpu_baseline"] = cpu
    line["detail"] = {"kernel_ms_per_launch": _sig(d["kernel_ms_per_launch"]), "streams": d["streams"],
                      "engine": d["engine"],
                      "batches_per_launch": d["batches_per_launch"],
                      "expansions_per_batch": d["expansions_per_batch"],
                      "timed_launches_checked": d["timed_launches_checked"], "detail_file": detail_path}
    line["secondary"] = {k: compact_leg(v) for k, v in out["secondary"].items()}
    s = json.dumps(line)
    # keep the line inside the driver's window whatever the leg set: drop optional fields first
    for drop in (("secondary", "unit_of_issue"), ("secondary", "traffic_x"), ("secondary", "checked"),
                 ("cpu_baseline", "sample")):
        if len(s) <= 4000:
            break
        if drop[0] == "secondary":
            for v in line["secondary"].values():
                v.pop(drop[1], None)
        elif line.get("cpu_baseline"):
            line["cpu_baseline"].pop(drop[1], None)
        s = json.dumps(line)
    return line


def dry_run(args, rank, world):
    """--dry-run: the multi-rank plumbing without a GPU.  Ranks come from launch_ranks (or
    torch.distributed.run) and join a gloo group.  Each strong-scaling workload is dealt over the ranks
    exactly as the GPU legs deal it -- C2 (96 queries, 64^2 grid) and C5 (48 per-query 3D grids)
    longest-first round-robin by octile distance, the C4 agents (12 DWA, 16 LQR) round-robin
    (c4_share) -- planned with the CPU oracle standing in for the kernels, and all_gathered; rank 0
    checks every gathered record set against one single-process oracle run and prints a JSON line of
    the bench's shape (n_gpus = world)."""
    import torch  # noqa: F401  (torch.distributed)

    from oracle import oracle as O
    from python_motion_planning_amd import batch, shard, workloads as wl

    dist = shard.init("gloo")
    occ, starts, goals = wl.c2_workload(nq=96, W=64, H=64, pair_seed=6)

    def plan(s, g):
        r = O.astar2d_batch(occ, s, g, path_cap=4096, nthreads=1)
        return {"cost": torch.as_tensor(r["cost"]), "status": torch.as_tensor(r["status"]),
                "n_expanded": torch.as_tensor(r["n_expanded"]), "path_len": torch.as_tensor(r["path_len"])}

    occ3, s3, g3 = wl.c5_workload(48, first_seed=0)

    def plan3(s, g, occ):
        cost, st = O.astar3d_batch(occ, s, g, nthreads=1)
        return {"cost": torch.as_tensor(cost), "status": torch.as_tensor(st)}

    def c4_paths(occ4, states):
        r = O.astar2d_batch(occ4, states[:, :2].astype(np.int32), np.tile([45, 25], (len(states), 1)).astype(np.int32),
                            path_cap=2048, nthreads=1)
        H4 = occ4.shape[1]
        paths = [np.column_stack([r["path"][i, : r["path_len"][i]][::-1] // H4,
                                  r["path"][i, : r["path_len"][i]][::-1] % H4]).astype(np.float64)
                 for i in range(len(states))]
        return batch.pack_paths(paths)

    def dwa(occ4, states, goals4):
        xy, off = c4_paths(occ4, states)
        st, u, status = O.dwa_step_batch(np.argwhere(occ4).astype(np.float64), xy, off, goals4, states, nthreads=1,
                                         grid=occ4)
        return {"state": torch.as_tensor(st), "u": torch.as_tensor(u), "status": torch.as_tensor(status)}

    def lqr(occ4, states, goals4):
        xy, off = c4_paths(occ4, states)
        st, up, u, status, nst, _ = O.track_batch("lqr", xy, off, goals4, states, iters=5, nthreads=1)
        return {"state": torch.as_tensor(st), "u": torch.as_tensor(u), "n_steps": torch.as_tensor(nst)}

    shard.barrier(dist)
    t0 = time.perf_counter()
    out = shard.run_sharded(dist, plan, starts, goals)
    shard.barrier(dist)
    (elapsed,) = shard.max_over_ranks(dist, [time.perf_counter() - t0])
    out3 = shard.run_sharded(dist, plan3, s3, g3, per_query={"occ": occ3})
    c4 = {}
    for name, fn, na in (("c4_dwa", dwa, 12), ("c4_lqr", lqr, 16)):
        occ4, st4, gl4, mine = c4_share(args, na, world, rank)
        c4[name] = shard.all_gather_rows(dist, mine, fn(occ4, st4, gl4), na)
    if rank == 0:
        ref = O.astar2d_batch(occ, starts, goals, path_cap=4096, nthreads=1)
        eq = {"c2": all(np.array_equal(out[k].numpy(), ref[k]) for k in ("cost", "status", "n_expanded", "path_len"))}
        ref3 = plan3(s3, g3, occ3)
        eq["c5"] = all(torch.equal(out3[k], ref3[k]) for k in ref3)
        for name, fn, na in (("c4_dwa", dwa, 12), ("c4_lqr", lqr, 16)):
            occ4, st4, gl4, _ = c4_share(args, na, 1, 0)
            ref4 = fn(occ4, st4, gl4)
            eq[name] = all(torch.equal(c4[name][k], ref4[k]) for k in ref4)
        print(json.dumps({"metric": "dry run: A* plans/sec (CPU oracle stand-in, 64^2 grid, 96 queries)",
                          "value": 96 / elapsed, "unit": "plans/s", "n_gpus": world, "steps": 1, "warmup": 0,
                          "scaling": "strong", "dry_run": True, "gathered_equal_single_rank": all(eq.values()),
                          "gathered_equal": eq, "higher_is_better": True}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def c2_share_mode(args):
    """--strong-share R/N (diagnostic, one GPU, one process): rank R's share of C2 under the N-rank
    strong split (shard.lpt_deal of the default_rng(1) pairs by octile distance, as --scaling strong
    deals it) repeated --steps times in one launch, the share's per-rank launch time measured; with
    --tail-sq K the K longest of the launch's queries (octile) run on the single-query engine
    (astar2d_sq.hip: a workgroup and a CU's LDS per query) on a second stream beside the multi-query
    launch of the rest.  Every query's outputs are checked against an all-multi-query run."""
    import torch

    from python_motion_planning_amd import _lib, batch, shard, workloads as wl

    R, N = (int(v) for v in args.strong_share.split("/"))
    torch.cuda.set_device(0)
    occ, s_all, g_all = wl.c2_workload(nq=args.nq, pair_seed=1)
    mine = shard.lpt_deal(shard.octile(s_all, g_all), N, R)
    starts, goals = np.tile(s_all[mine], (args.steps, 1)), np.tile(g_all[mine], (args.steps, 1))
    nq, W, H = len(starts), occ.shape[0], occ.shape[1]
    L = _lib.load_library()
    occ_bits = batch.occ_bits_device(occ, torch)
    path_cap = 4096
    ctxs = []

    def mk(engine, workers):
        ctx = L.pmp_create(0)
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, engine, 1), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, workers, 0), "reserve")
        _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, 60), "residency")
        ctxs.append(ctx)
        return ctx

    def outs(n):
        return {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
                (("cost", torch.float64), ("plen", torch.int32), ("nexp", torch.int32), ("status", torch.int32))}

    def launch(ctx, stream, idx, o):
        s_d = torch.as_tensor(starts[idx], device="cuda")
        g_d = torch.as_tensor(goals[idx], device="cuda")
        path = torch.empty((len(idx), path_cap), dtype=torch.int32, device="cuda")
        keep.append((s_d, g_d, path))
        rc = L.pmp_astar2d_batch(ctx, stream.cuda_stream, occ_bits.data_ptr(), W, H, 0, s_d.data_ptr(), g_d.data_ptr(),
                                 len(idx), o["cost"].data_ptr(), o["plen"].data_ptr(), path.data_ptr(), path_cap,
                                 o["nexp"].data_ptr(), None, 0, None, o["status"].data_ptr())
        _lib.check(ctx, rc, "pmp_astar2d_batch")

    keep = []
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    mq = mk(1, 15360)
    allidx = np.arange(nq)
    # reference: every query on the multi-query engine (also the warmup that touches its slots)
    ref = outs(nq)
    launch(mq, sA, allidx, ref)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch(mq, sA, allidx, ref)
    torch.cuda.synchronize()
    t_mq = time.perf_counter() - t0
    rec = {"metric": f"C2 strong-split share: rank {R} of {N}, {len(mine)} pairs x {args.steps} in one launch",
           "queries": nq, "launch_s_multi_query_only": t_mq}
    K = args.tail_sq
    if K > 0:
        order = np.argsort(-shard.octile(starts, goals), kind="stable")
        heavy, light = np.sort(order[:K]), np.sort(order[K:])
        sq = mk(3, K)
        oh, ol = outs(K), outs(nq - K)
        for rep_i in range(2):  # the first pass touches the single-query slots
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            launch(sq, sB, heavy, oh)   # the long queries first: a CU each
            launch(mq, sA, light, ol)
            torch.cuda.synchronize()
            t_split = time.perf_counter() - t0
        for k in ref:
            assert torch.equal(oh[k], ref[k][torch.as_tensor(heavy, device="cuda")]), k
            assert torch.equal(ol[k], ref[k][torch.as_tensor(light, device="cuda")]), k
        rec.update({"tail_sq": K, "launch_s_with_tail_on_single_query_engine": t_split,
                    "heavy_expansions": int(oh["nexp"].sum().item()), "all_expansions": int(ref["nexp"].sum().item())})
    assert (ref["status"] == 0).all()
    for c in ctxs:
        L.pmp_destroy(c)
    print(json.dumps(rec))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--strong-share", default="",
                    help="diagnostic R/N: rank R's share of C2 under the N-rank strong split on this GPU (c2_share_mode)")
    ap.add_argument("--tail-sq", type=int, default=0,
                    help="with --strong-share: the K longest queries on the single-query engine on a second stream")
    ap.add_argument("--nq", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=4096, help="queries in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="minimum CPU-baseline wall time of the short legs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--agents", type=int, default=256, help="C4 agents per GPU (control-step leg)")
    ap.add_argument("--control-steps", type=int, default=20, help="timed control steps")
    ap.add_argument("--engine", type=int, default=1, choices=[0, 1, 2],
                    help="A* 2D engine: 1 = four queries per wave (astar2d_mq.hip) for the C2 batches, 2 = that for "
                         "every batch, 0 = one query per wave (astar2d.hip)")
    ap.add_argument("--t2lds", type=int, default=1,
                    help="multi-query engine: level-10..12 heap bits in LDS (1; heaps <= 16383) or level-10..14 in HBM (0)")
    ap.add_argument("--workers", type=int, default=0,
                    help="A* queries in flight per launch (persistent 16-lane groups on engine 1, waves on engine 0); "
                         "0 = the engine's default")
    ap.add_argument("--theta-workers", type=int, default=768, help="persistent Theta* 2D workers per launch")
    ap.add_argument("--theta-engine", type=int, default=2,
                    help="Theta* 2D engine: 2 = four queries per wave (astar2d_mq.hip, round 5), 0 = one per wave")
    ap.add_argument("--keep-headline-ctx", type=int, default=0,
                    help="dev A/B: keep the headline's context (and its scratch) until exit")
    ap.add_argument("--theta-share-ctx", type=int, default=1,
                    help="1: the Theta* 2D legs plan on the headline's context (its scratch, as one long-lived "
                         "planner would) instead of fresh ones; 0: fresh contexts -- their new ~100 GB of scratch, "
                         "allocated right after the headline's is freed, ran Theta* 1.85x slower on every box tried "
                         "(7.2 s vs 3.9 s per 12-batch launch, tools/calls/r5_call15.sh)")
    ap.add_argument("--theta-residency", type=int, default=48,
                    help="Theta* 2D queries resident per CU (as --residency; with one multi-batch launch: 256 x this "
                         "many groups; multi-query engine on the headline's context, round 5: 24 / 32 / 40 / 48 -> "
                         "Theta* 10.7 / 13.4 / 14.5 / 18.0 k, Lazy 9.8 / 12.2 / 13.1 / 16.2 k plans/s; 48 = 12 waves "
                         "per CU, the Theta* build's 3 per SIMD)")
    ap.add_argument("--residency", type=int, default=0,
                    help="A* queries resident per CU over all batches in flight (sets each one's LDS heap share; "
                         "0 = the engine's default)")
    ap.add_argument("--legs", default="dwa,rrt,astar3d,totp,lqr,mpc,graphs,dstar,dyn3d,latency",
                    help="secondary legs to run (comma list of dwa, rrt, astar3d, totp (C5 trajectories on the "
                         "astar3d leg's paths), lqr, mpc, graphs, dstar, dyn3d, latency; 'none' for none)")
    ap.add_argument("--dyn3d-queries", type=int, default=8192, help="C5 queries per DStar3D / LPAStar3D launch")
    ap.add_argument("--dyn3d-steps", type=int, default=24)
    ap.add_argument("--dyn3d-streams", type=int, default=4, help="DStar3D / LPAStar3D launches in flight")
    ap.add_argument("--lpa-workers-per-cu", type=int, default=0,
                    help="LPA* / D* Lite 2D persistent workers per CU (0 = the library default)")
    ap.add_argument("--lpa3d-workers-per-cu", type=int, default=0,
                    help="LPAStar3D persistent workers per CU (0 = the library default)")
    ap.add_argument("--dyn3d-batches-per-launch", type=int, default=6,
                    help="DStar3D / LPAStar3D batches per launch (0 = all the timed steps in one launch; LPAStar3D "
                         "169 k / 315 k / 321 k plans/s at 1 x 6 streams / 24 x 1 / 6 x 4)")
    ap.add_argument("--dstar-queries", type=int, default=4096, help="queries per D* batch (256^2 and 512^2 grids)")
    ap.add_argument("--dstar-batches-per-launch", type=int, default=1,
                    help="D* batches per launch (0 = all the timed steps in one launch; 1 = one per launch on "
                         "--dstar-streams: faster here, 4,180 vs 2,650-3,090 plans/s at 512^2, D* has no "
                         "longest-first order)")
    ap.add_argument("--dstar-steps", type=int, default=9)
    ap.add_argument("--lpa-streams", type=int, default=3, help="LPA* / D* Lite 2D batches in flight")
    ap.add_argument("--theta-streams", type=int, default=6, help="Theta* 2D batches in flight (own stream + context each)")
    ap.add_argument("--dstar-streams", type=int, default=3, help="D* batches in flight (own stream + context each)")
    ap.add_argument("--theta-queries", type=int, default=4096, help="C2 queries per Theta* / Lazy Theta* 2D batch")
    ap.add_argument("--theta-batches-per-launch", type=int, default=0,
                    help="Theta* 2D batches per launch (0 = all the timed steps in one launch, streamed through "
                         "256 x --theta-residency persistent workers; 1 = one batch per launch on --theta-streams)")
    ap.add_argument("--lpa-queries", type=int, default=65536,
                    help="README-grid queries per LPA* / D* Lite launch (4 per worker wave: the queue balances the "
                         "tail; 16,384 / 65,536 per launch: 1.11 M / 1.19 M plans/s, replanning 4.16 M / 4.81 M)")
    ap.add_argument("--graph-steps", type=int, default=12)
    ap.add_argument("--rrt-queries", type=int, default=256)
    ap.add_argument("--rrt-samples", type=int, default=65536)
    ap.add_argument("--rrt-steps", type=int, default=4)
    ap.add_argument("--rrt-streams", type=int, default=2, help="RRT* launches in flight (own stream + context each)")
    ap.add_argument("--rrt-batches", type=int, default=16,
                    help="RRT* batches (of --rrt-queries) per launch: continuous batching, one launch over all of them")
    ap.add_argument("--rrt-cpu-sample", type=int, default=16)
    ap.add_argument("--rrt-resident", type=int, default=0,
                    help="RRT* workgroups per CU the LDS tree copy leaves room for (0: one, the whole LDS)")
    ap.add_argument("--a3-queries", type=int, default=8192)
    ap.add_argument("--a3-steps", type=int, default=32)
    ap.add_argument("--a3-streams", type=int, default=6, help="3D A* batches in flight (own stream + context each)")
    ap.add_argument("--a3-batches-per-launch", type=int, default=0,
                    help="3D A* batches per launch (0 = all the timed steps in one launch)")
    ap.add_argument("--a3-workers-per-cu", type=int, default=4, help="3D A* persistent workers per CU")
    ap.add_argument("--a3-residency", type=int, default=20,
                    help="3D A* workers resident per CU over all batches in flight (LDS share; 0 = per launch); "
                         "round 4 sweep, one box: 20 / 24 / 28 / 32 -> 1.848 / 1.816 / 1.810 / 1.794 M plans/s")
    ap.add_argument("--dstar-workers-per-cu", type=int, default=0, help="D* persistent workers per CU (0 = default)")
    ap.add_argument("--dstar-residency", type=int, default=0,
                    help="D* workers resident per CU over all batches in flight (LDS share; 0 = per launch)")
    ap.add_argument("--track-agents", type=int, default=32768,
                    help="agents per LQR / MPC tracking launch (four per wave, one per 16-lane row: 8192 waves)")
    ap.add_argument("--track-iters", type=int, default=20)
    ap.add_argument("--track-steps", type=int, default=5)
    ap.add_argument("--schedule", choices=["lpt", "input"], default="lpt",
                    help="A* query order across workers: longest start-goal distance first, or input order")
    ap.add_argument("--prio", type=int, default=64,
                    help="longest-first only: the first N (longest) queries of a batch run at raised wave priority")
    ap.add_argument("--batches-per-launch", type=int, default=0,
                    help="batches (steps) one launch plans, streamed through its persistent workers longest first; "
                         "0 = all the timed steps in one launch (engine 1) or one per launch (engine 0)")
    ap.add_argument("--streams", type=int, default=6,
                    help="batches in flight: consecutive steps go to different HIP streams (own scratch "
                         "context each), so one batch's long-query tail overlaps the next batch")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="HIP hardware queues per process (GPU_MAX_HW_QUEUES, <= 32), set before the GPU is "
                         "touched: with HIP's default of 4 a fourth batch in flight shares a queue with "
                         "another and serialises behind it (0: keep the environment's value)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: every rank plans its own --nq batch; strong: one --nq batch dealt over the ranks "
                         "(longest-first round-robin) with an all_gather of the results")
    ap.add_argument("--detail-out", default=None,
                    help="file for the full per-leg records (default gpurun_out/bench_detail.json); stdout's last "
                         "line is the compact headline")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the rank launcher, the strong-scaling deal and the result all_gather "
                         "over gloo with the CPU oracle standing in for the kernels (tests/test_multirank.py)")
    args = ap.parse_args()
    # engine defaults: engine 1 (multi-query, one heap operation per group per step, two-level spill
    # blocks) -- 15,360 groups in flight, 60 per CU = 3.75 waves per SIMD (round 4, same box,
    # alternating, three rounds: 56 / 60 / 64 per CU 17.38-17.41 k / 17.70-17.82 k / 16.69-18.06 k
    # plans/s; before the block layout 56 was best); engine 0 -- 768 waves, 18 per CU (round 2)
    # round 6 (tiled cell states): 56 per CU, 14,336 groups -- the LDS share then holds 127 heap positions,
    # exactly levels 0-6, so the spill starts at a level boundary (56 / 60 / 64 per CU: 19.04-19.16 k /
    # 18.56-18.72 k / 18.65 k plans/s on one box, tools/calls/r6_call8.sh, r6_call9.sh)
    if not args.workers:
        args.workers = 14336 if args.engine else 768
    if not args.residency:
        args.residency = 56 if args.engine else 18
    if not args.batches_per_launch and args.engine == 0:
        args.batches_per_launch = 1
    if args.strong_share:
        return c2_share_mode(args)

    from python_motion_planning_amd import shard

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # a bare `python bench.py --gpus N`: start the N rank processes here, before anything touches
        # a GPU, and leave with their exit code (rank 0 prints the JSON line)
        sys.exit(shard.launch_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    rank, world, local = shard.env_rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, rank, world)

    # must be in the environment before the HIP runtime initialises (the first torch.cuda call)
    # (the GPU box exports GPU_MAX_HW_QUEUES=4, HIP's default: override it; --hw-queues 0 keeps it)
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(4, args.hw_queues)))
    import torch

    dist = shard.init("nccl")  # RCCL over xGMI; None for a single process
    if dist is None:
        torch.cuda.set_device(0)

    from python_motion_planning_amd import _lib, batch, workloads as wl

    if args.scaling == "strong":
        # one fixed batch (the C2 pairs of default_rng(1)) dealt longest-first round-robin over the ranks
        occ, starts_all, goals_all = wl.c2_workload(nq=args.nq, pair_seed=1)
        mine = shard.lpt_deal(shard.octile(starts_all, goals_all), world, rank)
        starts, goals = starts_all[mine], goals_all[mine]
    else:
        occ, starts, goals = wl.c2_workload(nq=args.nq, pair_seed=1 + rank)
        mine = np.arange(args.nq)
    nq = len(starts)
    W, H = occ.shape
    L = count_launches(_lib.load_library())
    _LABEL[0] = "astar2d_c2"
    occ_bits = batch.occ_bits_device(occ, torch)
    s_d = torch.as_tensor(starts, device="cuda")
    g_d = torch.as_tensor(goals, device="cuda")
    path_cap = 4096
    # Batches per launch (B): the steps' batches go to the planner B at a time, each launch's
    # persistent workers streaming through its B x 4096 queries longest first (continuous batching:
    # a query of batch k+1 starts as soon as a worker frees up, instead of behind batch k's longest
    # query).  B = 1 with several streams is the round-2 schedule (one launch per batch, batches in
    # flight on their own streams).  Every batch keeps its own outputs; every timed batch is checked.
    B = max(1, min(args.batches_per_launch or args.steps, args.steps))
    nlaunch = -(-args.steps // B)
    S = max(1, min(args.streams, nlaunch))
    s_rep = s_d.repeat(B, 1)
    g_rep = g_d.repeat(B, 1)
    lanes = []
    for _ in range(S):
        ctx = L.pmp_create(torch.cuda.current_device())
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, args.engine, args.t2lds), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, args.workers, 0), "reserve")
        _lib.check(ctx, L.pmp_astar2d_set_schedule(ctx, 1 if args.schedule == "lpt" else 0), "schedule")
        _lib.check(ctx, L.pmp_astar2d_set_priority(ctx, args.prio), "priority")
        if args.residency:
            _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, args.residency), "residency")
        lanes.append(dict(
            ctx=ctx, stream=pool_stream(torch, len(lanes)),
            cost=torch.empty(B * nq, dtype=torch.float64, device="cuda"),
            plen=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
            path=torch.empty((B * nq, path_cap), dtype=torch.int32, device="cuda"),
            nexp=torch.empty(B * nq, dtype=torch.int32, device="cuda"),
            status=torch.empty(B * nq, dtype=torch.int32, device="cuda")))
    ctr = torch.empty((B * nq, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step(i, nb, counters=None):
        """Launch i (on lane i % S): nb batches of the nq pairs, as one call of the C-ABI."""
        b = lanes[i % S]
        rc = L.pmp_astar2d_batch(b["ctx"], b["stream"].cuda_stream, occ_bits.data_ptr(), W, H, 0, s_rep.data_ptr(),
                                 g_rep.data_ptr(), nq * nb, b["cost"].data_ptr(), b["plen"].data_ptr(),
                                 b["path"].data_ptr(), path_cap, b["nexp"].data_ptr(), None, 0, counters,
                                 b["status"].data_ptr())
        if rc:
            _lib.check(b["ctx"], rc, "pmp_astar2d_batch")
        return b

    # warmup: every lane once (the first launch also records the deterministic push/pop/expansion counts);
    # its launches are smaller than the timed ones, so the profile keys them apart
    # (at least as many batches as the launch has query slots: a launch that first-touches the ~150 GB
    # of per-slot scratch runs ~1.3 s slower, tools/ab_headline.py)
    wb = max(1, min(B, max(args.warmup, -(-args.workers // nq) if args.engine else 1)))
    _LABEL[0] = "astar2d_c2_warmup"
    step(0, wb, ctr.data_ptr())
    for i in range(1, S):
        step(i, wb)
    torch.cuda.synchronize()
    _LABEL[0] = f"astar2d_c2_x{B}"  # keyed by batches per launch: a profile of other launches is refused
    counters = ctr[:nq].cpu().numpy()
    ref_out = {k: lanes[0][k][:nq].clone() for k in ("cost", "plen", "nexp", "status")}
    st0 = ref_out["status"].cpu().numpy()
    assert (st0 == 0).all(), f"unexpected statuses {np.unique(st0)}"
    for b in lanes:
        for j in range(wb):
            assert torch.equal(b["cost"][j * nq:(j + 1) * nq], ref_out["cost"])
    bytes_per_batch = astar_algorithmic_bytes(counters)
    for b in lanes:
        poison([b["cost"], b["plen"], b["nexp"], b["status"]])
    torch.cuda.synchronize()

    # timed region.  kernel_ms = HIP events on each launch's own stream (= rocprofv3's dispatch
    # duration).  Each launch also records its device execution span (first worker start .. last
    # worker end, pmp_set_timing) for the detail block.
    spans = torch.empty((nlaunch, 2), dtype=torch.int64, device="cuda")
    spans[:, 0] = -1  # UINT64_MAX
    spans[:, 1] = 0
    khz = ctypes.c_int(0)
    _lib.check(lanes[0]["ctx"], L.pmp_wall_clock_khz(lanes[0]["ctx"], ctypes.byref(khz)), "wall clock")
    shard.barrier(dist)
    torch.cuda.synchronize()
    evs = []
    nbs = [min(B, args.steps - i * B) for i in range(nlaunch)]
    t0 = time.perf_counter()
    for i in range(nlaunch):
        b = lanes[i % S]
        L.pmp_set_timing(b["ctx"], spans[i].data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(b["stream"])
        step(i, nbs[i])
        e1.record(b["stream"])
        evs.append((e0, e1))
    torch.cuda.synchronize()
    shard.barrier(dist)
    elapsed = time.perf_counter() - t0
    for b in lanes:
        L.pmp_set_timing(b["ctx"], None)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    sp = spans.cpu().numpy().view(np.uint64)
    span_ms = float(np.mean((sp[:, 1] - sp[:, 0]).astype(np.float64)) / khz.value)
    # every batch of the last launch on every lane equals the warmup's first batch
    outs = []
    for li, b in enumerate(lanes[: min(S, nlaunch)]):
        last_nb = nbs[max(i for i in range(nlaunch) if i % S == li)]
        outs += [{k: b[k][j * nq:(j + 1) * nq] for k in ("cost", "plen", "nexp", "status")} for j in range(last_nb)]
    timed_checked = check_timed("astar2d", ref_out, outs)
    elapsed, kern_ms, span_ms = shard.max_over_ranks(dist, [elapsed, kern_ms, span_ms], "cuda")
    # the ranks plan different pair sets (weak: default_rng(1 + rank); strong: dealt shares): the roofline
    # is per GPU, on the mean over ranks of each rank's own algorithmic bytes against the max-over-ranks
    # kernel time
    bytes_per_batch = shard.sum_over_ranks(dist, [bytes_per_batch], "cuda")[0] / world
    bytes_per_launch = bytes_per_batch * float(np.mean(nbs))
    plans = (args.nq if args.scaling == "strong" else nq * world) * args.steps
    value = plans / elapsed
    gathered = None
    if args.scaling == "strong" and dist is not None:
        # the survey's end-of-run result exchange: every rank's records into the full batch, input order
        g = shard.all_gather_rows(dist, mine, {"cost": ref_out["cost"], "status": ref_out["status"],
                                               "n_expanded": ref_out["nexp"]}, args.nq, device="cuda")
        gathered = {"queries": args.nq, "found": int((g["status"] == 0).sum().item()),
                    "sum_expansions": int(g["n_expanded"].sum().item())}
    counters_all = shard.all_gather_rows(dist, mine, {"c": torch.as_tensor(counters, device="cuda")},
                                         args.nq, device="cuda")["c"].cpu().numpy() if (
        args.scaling == "strong" and dist is not None) else counters
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    # the headline's scratch (about 30 GB per batch in flight) is not needed by the other legs, except
    # with --theta-share-ctx: the Theta* legs then plan on the headline's context (its grow-only
    # scratch already holds their per-slot state, so they allocate only the CLOSED-parent array)
    torch.cuda.synchronize()
    cost = ref_out["cost"].cpu()
    for i, b in enumerate(lanes):
        if i == 0 and ((args.theta_share_ctx and "graphs" in args.legs.split(",")) or args.keep_headline_ctx):
            _SHARED_CTX.append(b["ctx"])
        else:
            L.pmp_destroy(b["ctx"])
    lanes.clear()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        threads = cpu_threads()
        ns = min(args.cpu_sample, nq)
        O.lib()
        t = time.perf_counter()
        ref = O.astar2d_batch(occ, starts[:ns], goals[:ns], path_cap=path_cap, nthreads=threads)
        dt = time.perf_counter() - t
        assert np.array_equal(ref["cost"], cost[:ns].numpy()), "GPU/oracle cost mismatch"
        # one core: every 32nd query of the batch (the same mix of short and long queries)
        sub = np.arange(0, nq, 32)[: max(1, args.cpu_sample // 32)]
        t = time.perf_counter()
        O.astar2d_batch(occ, starts[sub], goals[sub], path_cap=path_cap, nthreads=1)
        dt1 = time.perf_counter() - t
        cpu = {"value": ns / dt, "unit": "plans/s", "cores": threads, "kind": "port", "host": host_cpu(),
               "sample": f"first {ns} of the 4096 C2 pairs, C restatement (oracle/pmp_oracle.c) with OpenMP over "
                         f"queries on every core of the affinity mask, {dt:.1f} s wall",
               "one_core": {"value": len(sub) / dt1, "sample": f"every 32nd pair ({len(sub)}), {dt1:.1f} s"}}

    _LABEL[0] = "setup"
    legs = [x for x in args.legs.split(",") if x and x != "none"]
    secondary = {}
    if "dwa" in legs:
        secondary["mpc_sampled_dwa"] = control_leg(args, torch, dist, world, rank)
    if "rrt" in legs:
        with leg_label("rrt_star"):
            secondary["rrt_star"] = rrt_leg(args, torch, dist, world, rank)
    if "astar3d" in legs:
        secondary["astar3d"] = astar3d_leg(args, torch, dist, world, rank)
        if secondary["astar3d"].get("trajectory"):
            secondary["totp3d"] = secondary["astar3d"].pop("trajectory")
    if "lqr" in legs:
        secondary["lqr"] = track_leg(args, torch, dist, world, rank, "lqr")
    if "mpc" in legs:
        secondary["mpc_qp"] = track_leg(args, torch, dist, world, rank, "mpc")
    if "graphs" in legs:
        secondary.update(graphs_leg(args, torch, dist, world, rank))
    if "dstar" in legs:
        secondary.update(dstar_leg(args, torch, dist, world, rank))
    if "dyn3d" in legs:
        secondary.update(dyn3d_leg(args, torch, dist, world, rank))
    if "latency" in legs:
        secondary.update(latency_leg(args, torch, dist, world, rank))

    if rank == 0:
        out = {
            "metric": "A* plans/sec on 1024^2 grid (4096 random start/goal pairs per GPU)" if args.scaling == "weak"
                      else f"A* plans/sec on 1024^2 grid ({args.nq} random start/goal pairs over {world} GPUs)",
            "value": value,
            "unit": "plans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) C2 generator: default_rng(0) 20% obstacles, default_rng(1+rank) pairs)",
            "config": {"workload": "C2 batched A* 1024x1024 Grid, 4096 start/goal pairs per GPU, euclidean"
                                   if args.scaling == "weak" else
                                   f"C2 batched A* 1024x1024 Grid, one {args.nq}-pair batch split over the GPUs",
                       "grid": [W, H], "queries_per_gpu": nq, "parallelism": f"query-sharded x{world}"},
            "roofline": with_issue(with_traffic({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                                                 "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                                                 "algorithmic_bytes_per_launch": bytes_per_launch,
                                                 # launches in flight overlap: bytes of one batch per step interval
                                                 "achieved_aggregate": bytes_per_batch / (elapsed / args.steps) / 1e9,
                                                 "frac_aggregate": bytes_per_batch / (elapsed / args.steps) / 1e9
                                                                   / HBM_PEAK_GBS},
                                                "astar2d_kernel", f"astar2d_c2_x{B}"),
                                   "astar2d_kernel", f"astar2d_c2_x{B}", float(counters[:, 2].sum()) * B, "expansion"),
            "cpu_baseline": cpu,
            "secondary": secondary,
            "detail": {"kernel_ms_per_launch": kern_ms,
                       "kernel_ms_source": "HIP events on the launch's stream (= rocprofv3 dispatch duration)",
                       "execution_span_ms_per_launch": span_ms, "schedule": args.schedule,
                       "algorithmic_bytes_per_launch": bytes_per_launch,
                       "batches_per_launch": B, "launches": nlaunch,
                       "expansions_per_batch": int(counters[:, 2].sum()),
                       "max_expansions_query": int(counters[:, 2].max()),
                       "pushes_per_batch": int(counters[:, 0].sum()),
                       "pops_per_batch": int(counters[:, 1].sum()),
                       "algorithmic_bytes_note": "per GPU: mean over ranks of each rank's own batch bytes",
                       "max_heap_entries": int(counters[:, 3].max()),
                       "expansions_all_ranks_per_step": int(counters_all[:, 2].sum()) if args.scaling == "strong" else None,
                       "strong_scaling_gather": gathered,
                       "engine": "multi-query (4 per wave, astar2d_mq.hip)" if args.engine else
                                 "one query per wave (astar2d.hip)", "t2_lds": args.t2lds,
                       "queries_in_flight_per_launch": args.workers, "streams": S, "priority_queries": args.prio,
                       "resident_per_cu": args.residency,
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "timed_launches_checked": timed_checked},
            "launch_manifest": _MANIFEST,
        }
        path = write_detail(args, out)
        line = json.dumps(headline_line(out, path))
        print(line, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
