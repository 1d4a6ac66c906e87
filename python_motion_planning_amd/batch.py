"""Batched entry points over the C-ABI (include/pmp.h).  Inputs/outputs are torch device tensors.

These are the calls the drop-in planner classes, the bench and the parity tests go through;
each one launches the gfx950 kernels of libpmp_hip.so asynchronously on the current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .env import pack_bits


def _dev(torch, a, dtype):
    if isinstance(a, torch.Tensor):
        return a.to(device="cuda", dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


def occ_bits_device(occ, torch=None):
    """uint8 [W, H] (x-major) numpy occupancy -> bit-packed uint32 device tensor (as int32)."""
    torch = torch or _lib.device_check()
    words = pack_bits(occ)
    return torch.as_tensor(words.view(np.int32), device="cuda")


def astar2d_batch(occ, starts, goals, heuristic: str = "euclidean", path_cap: int | None = None,
                  expand_cap: int = 0, counters: bool = False, occ_bits=None, reserve_slots: int | None = None,
                  heap_cap: int = 0, retry_overflow: bool = True, algo: str = "astar"):
    """Batched AStar.plan (a_star.py:39-83); algo "dijkstra" / "gbfs" run Dijkstra.plan
    (dijkstra.py:36-85) / GBFS.plan (gbfs.py:36-86) on the same kernel (pmp_graph2d_batch).

    occ: numpy uint8 [W, H] (or pass occ=(W, H) with a prebuilt `occ_bits` device tensor).
    starts, goals: [nq, 2] int (numpy or device tensors).
    Returns dict of device tensors: cost f64 [nq], path_len i32 [nq], path i32 [nq, path_cap]
    (cell ids x*H+y, goal first), n_expanded i32, status i32, optional expand / counters.

    A query whose heap outgrows the reserved capacity stops with STATUS_CAP_OVERFLOW; with
    retry_overflow those queries are planned again on the GPU with the full bound (8 W H + 8
    entries) on fewer workers -- one host sync to read the statuses.
    """
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    if occ_bits is None:
        W, H = int(occ.shape[0]), int(occ.shape[1])
        occ_bits = occ_bits_device(occ, torch)
    else:
        W, H = (int(occ[0]), int(occ[1])) if isinstance(occ, tuple) else (int(occ.shape[0]), int(occ.shape[1]))
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    if path_cap is None:
        path_cap = min(W * H + 1, 1 << 16)
    out = dict(
        cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
        path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
        path=torch.empty((nq, path_cap), dtype=torch.int32, device="cuda"),
        n_expanded=torch.empty(nq, dtype=torch.int32, device="cuda"),
        status=torch.empty(nq, dtype=torch.int32, device="cuda"),
    )
    out["expand"] = torch.empty((nq, expand_cap), dtype=torch.int32, device="cuda") if expand_cap else None
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    if reserve_slots:
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, int(reserve_slots), int(heap_cap)), "pmp_astar2d_reserve")
    rc = L.pmp_graph2d_batch(ctx, _lib.stream_ptr(), _lib.ALGOS[algo], occ_bits.data_ptr(), W, H,
                             1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq,
                             out["cost"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(), path_cap,
                             out["n_expanded"].data_ptr(), _lib.ptr(out["expand"]), int(expand_cap),
                             _lib.ptr(out["counters"]), out["status"].data_ptr())
    _lib.check(ctx, rc, "pmp_graph2d_batch")
    if retry_overflow:
        redo = torch.nonzero(out["status"] == _lib.STATUS_CAP_OVERFLOW).flatten()
        if redo.numel():
            r = astar2d_full_bound((W, H), s[redo], g[redo], heuristic, path_cap, expand_cap, counters, occ_bits,
                                   algo=algo)
            for k in ("cost", "path_len", "path", "n_expanded", "status", "expand", "counters"):
                if out[k] is not None:
                    out[k][redo] = r[k]
    out["W"], out["H"] = W, H
    return out


def astar2d_full_bound(occ, starts, goals, heuristic="euclidean", path_cap=None, expand_cap=0, counters=False,
                       occ_bits=None, algo="astar"):
    """The overflow re-plan: the queries (a few) planned with the full heap bound (8 W H + 8 entries,
    which no search exceeds) on at most 256 workers, then the context's geometry restored as it was --
    the host's own reservation (its explicit heap_cap, or the default when it asked for none, so the
    engine choice of later batches is unchanged) or launch-sized scratch."""
    W, H = (int(occ[0]), int(occ[1])) if isinstance(occ, tuple) else (int(occ.shape[0]), int(occ.shape[1]))
    L, ctx = _lib.load_library(), _lib.context()
    nq = int(starts.shape[0])
    geo = np.zeros(6, np.int32)  # the geometry in force, restored after the re-run
    _lib.check(ctx, L.pmp_astar2d_geometry(ctx, geo.ctypes.data), "pmp_astar2d_geometry")
    _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, max(1, min(nq, 256)), 8 * W * H + 8), "pmp_astar2d_reserve")
    try:
        return astar2d_batch(occ if occ_bits is None else (W, H), starts, goals, heuristic, path_cap, expand_cap,
                             counters, occ_bits, retry_overflow=False, algo=algo)
    finally:
        if geo[5] or not geo[0]:  # sized by the launches: keep it that way (grows with the batches)
            _lib.check(ctx, L.pmp_astar2d_reserve_auto(ctx), "pmp_astar2d_reserve_auto")
        else:  # the host's own reservation, with the capacity it asked for (0 = the default)
            cap = int(geo[3]) if geo[4] & 2 else 0
            _lib.check(ctx, L.pmp_astar2d_reserve(ctx, int(geo[0]), int(geo[1]), int(geo[2]), cap),
                       "pmp_astar2d_reserve")


_ONE = {}


class SingleQuery:
    """One drop-in query (AStar.plan, a_star.py:39-83) with one host round trip: start/goal go up in
    one pinned copy, the kernel writes (status, n_expanded, path_len | path | CLOSED records) into one
    int32 device block, and the block comes back in one pinned copy and one stream sync.  The
    buffers are kept per (context, capacities) and reused call after call."""

    def __init__(self, torch, path_cap: int, expand_cap: int) -> None:
        self.path_cap, self.expand_cap = path_cap, expand_cap
        n = 4 + path_cap + expand_cap
        self.dev = torch.empty(n, dtype=torch.int32, device="cuda")
        self.host = torch.empty(n, dtype=torch.int32, pin_memory=True)
        self.sg_host = torch.empty(4, dtype=torch.int32, pin_memory=True)
        self.sg_dev = torch.empty(4, dtype=torch.int32, device="cuda")
        self.cost = torch.empty(1, dtype=torch.float64, device="cuda")

    def launch(self, torch, W: int, H: int, occ_bits, start, goal, heuristic: str, algo: str) -> None:
        L, ctx = _lib.load_library(), _lib.context()
        self.sg_host.numpy()[:] = (start[0], start[1], goal[0], goal[1])
        self.sg_dev.copy_(self.sg_host, non_blocking=True)
        d, pc = self.dev.data_ptr(), self.path_cap
        rc = L.pmp_graph2d_batch(ctx, _lib.stream_ptr(), _lib.ALGOS[algo], occ_bits.data_ptr(), W, H,
                                 1 if heuristic == "manhattan" else 0, self.sg_dev.data_ptr(),
                                 self.sg_dev.data_ptr() + 8, 1, self.cost.data_ptr(), d + 8, d + 16, pc, d + 4,
                                 d + 16 + 4 * pc, self.expand_cap, None, d)
        _lib.check(ctx, rc, "pmp_graph2d_batch")
        self.host.copy_(self.dev, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()

    def result(self):
        """(status, n_expanded, path cells goal->start, CLOSED records) as numpy, after the sync."""
        self.event.synchronize()
        h = self.host.numpy()
        st, nexp, plen = int(h[0]), int(h[1]), int(h[2])
        path = h[4: 4 + min(max(plen, 0), self.path_cap)].copy()
        exp = h[4 + self.path_cap: 4 + self.path_cap + min(max(nexp, 0), self.expand_cap)].view(np.uint32).copy()
        return st, nexp, plen, path, exp


def single_query(torch, path_cap: int, expand_cap: int) -> SingleQuery:
    key = (_lib.context(), path_cap, expand_cap)
    q = _ONE.get(key)
    if q is None:
        if len(_ONE) > 16:
            _ONE.clear()
        q = _ONE[key] = SingleQuery(torch, path_cap, expand_cap)
    return q


_RECORDS = ("cost", "path_len", "path", "n_expanded", "status")


def astar2d_sharded(occ, starts, goals, dist=None, path_cap: int | None = None, algo: str = "astar", **kw):
    """One batch of 2D grid queries split over all ranks of the process group `dist` (one GPU each):
    every rank plans its longest-first round-robin share on its own GPU with astar2d_batch and every
    rank returns the full batch's records (cost, path_len, path, n_expanded, status) in input order,
    gathered with one all_gather per field over RCCL.  dist=None: one rank."""
    from . import shard

    torch = _lib.device_check()
    occ_np = np.asarray(occ)
    occ_bits = occ_bits_device(occ_np, torch)
    shape = (int(occ_np.shape[0]), int(occ_np.shape[1]))

    def plan(s, g):
        r = astar2d_batch(shape, s, g, path_cap=path_cap, occ_bits=occ_bits, algo=algo, **kw)
        return {k: r[k] for k in _RECORDS}

    return shard.run_sharded(dist, plan, np.asarray(starts), np.asarray(goals), device="cuda")


def astar3d_sharded(occ, starts, goals, dist=None, path_cap: int | None = None, algo: str = "astar", **kw):
    """astar2d_sharded for AStar3D (C5: 8192 queries over the node's GPUs).  occ: shared [X,Y,Z] or
    per-query [nq,X,Y,Z] grids (per-query grids are sliced with the rank's queries)."""
    from . import shard

    _lib.device_check()
    occ_np = np.asarray(occ)
    s_all, g_all = np.asarray(starts), np.asarray(goals)
    per_query = occ_np.ndim == 4
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    idx = shard.lpt_deal(shard.octile(s_all, g_all), world, rank)
    r = astar3d_batch(occ_np[idx] if per_query else occ_np, s_all[idx], g_all[idx], path_cap=path_cap, algo=algo, **kw)
    return shard.all_gather_rows(dist, idx, {k: r[k] for k in _RECORDS}, len(s_all), device="cuda")


def obstacle_grid(obstacles):
    """Obstacle set of (x, y) integer tuples -> (ox, oy, occ[W, H]) covering its bounding box."""
    if not obstacles:
        return 0, 0, np.zeros((1, 1), np.uint8)
    a = np.fromiter((c for t in obstacles for c in t), np.int64, count=2 * len(obstacles)).reshape(-1, 2)
    ox, oy = int(a[:, 0].min()), int(a[:, 1].min())
    W, H = int(a[:, 0].max()) - ox + 1, int(a[:, 1].max()) - oy + 1
    occ = np.zeros((W, H), np.uint8)
    occ[a[:, 0] - ox, a[:, 1] - oy] = 1
    return ox, oy, occ


def pack_paths(paths):
    """list of [P_i, 2] paths -> (path_xy [sum P, 2] f64, path_off [n+1] i32) numpy arrays."""
    off = np.zeros(len(paths) + 1, np.int32)
    for i, p in enumerate(paths):
        off[i + 1] = off[i] + len(p)
    xy = np.concatenate([np.asarray(p, np.float64).reshape(-1, 2) for p in paths]) if off[-1] else np.zeros((0, 2))
    return xy, off


def dwa_step_batch(grid, lp_params, dwa_params, state, goal, path_xy, path_off, iters: int = 1,
                   want_eval: bool = False, want_traj: bool = False, want_hist: bool = False, parts: int = 0):
    """Batched DWA.plan iterations (dwa.py:72-93) on the gfx950 kernel dwa.hip.

    grid: (ox, oy, occ[W, H]) from obstacle_grid() (or with occ already a device bit tensor plus W, H).
    lp_params: _lib.LPParams; dwa_params: _lib.DWAParams.
    state [na, 5] f64 device tensor, updated in place; goal [na, 3]; path_xy / path_off from pack_paths().
    parts: workgroups per agent (pmp_dwa_set_split: 0 auto, 1 one per agent, k); results are identical.
    Returns dict of device tensors (u, best, status, n_steps, optional hist_pose, eval, best_traj).
    """
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    ox, oy, occ = grid[:3]
    if isinstance(occ, np.ndarray):
        W, H = occ.shape
        occ_bits = occ_bits_device(occ, torch)
    else:
        occ_bits, (W, H) = occ, grid[3]
    na = int(state.shape[0])
    goal = _dev(torch, goal, torch.float64).reshape(-1, 3)
    path_xy = _dev(torch, path_xy, torch.float64).reshape(-1, 2)
    path_off = _dev(torch, path_off, torch.int32)
    H_steps = int(dwa_params.predict_time / lp_params.dt)
    out = dict(u=torch.empty((na, 2), dtype=torch.float64, device="cuda"),
               best=torch.empty(na, dtype=torch.int32, device="cuda"),
               status=torch.empty(na, dtype=torch.int32, device="cuda"),
               n_steps=torch.empty(na, dtype=torch.int32, device="cuda"))
    out["hist_pose"] = torch.zeros((na, iters, 3), dtype=torch.float64, device="cuda") if want_hist else None
    out["eval"] = torch.zeros((na, 4096, 3), dtype=torch.float64, device="cuda") if want_eval else None
    out["best_traj"] = (torch.zeros((na, iters, max(H_steps, 1), 5), dtype=torch.float64, device="cuda")
                        if want_traj else None)
    _lib.check(ctx, L.pmp_dwa_set_split(ctx, int(parts)), "pmp_dwa_set_split")
    rc = L.pmp_dwa_step_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(),
                              ox, oy, W, H, ctypes.byref(lp_params), ctypes.byref(dwa_params), na, state.data_ptr(),
                              goal.data_ptr(), path_xy.data_ptr(), path_off.data_ptr(), int(iters),
                              out["u"].data_ptr(), out["best"].data_ptr(), out["status"].data_ptr(),
                              out["n_steps"].data_ptr(), _lib.ptr(out["hist_pose"]), _lib.ptr(out["eval"]),
                              _lib.ptr(out["best_traj"]))
    _lib.check(ctx, rc, "pmp_dwa_step_batch")
    return out


def lqr_control_batch(lp_params, lqr_params, s, s_d, u_r, robot_vw):
    """Batched LQR.lqrControl (lqr.py:103-145).  s, s_d [n,3], u_r [n,2], robot_vw [n,2] (the
    robot's current v, w).  Returns u [n,2] (device tensor)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    s = _dev(torch, s, torch.float64).reshape(-1, 3)
    n = int(s.shape[0])
    s_d = _dev(torch, s_d, torch.float64).reshape(-1, 3)
    u_r = _dev(torch, u_r, torch.float64).reshape(-1, 2)
    vw = _dev(torch, robot_vw, torch.float64).reshape(-1, 2)
    u = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    rc = L.pmp_lqr_control_batch(ctx, _lib.stream_ptr(), ctypes.byref(lp_params),
                                 ctypes.byref(lqr_params), n, s.data_ptr(), s_d.data_ptr(), u_r.data_ptr(),
                                 vw.data_ptr(), u.data_ptr())
    _lib.check(ctx, rc, "pmp_lqr_control_batch")
    return u


def mpc_control_batch(lp_params, mpc_params, s, s_d, u_r, u_p, robot_vw, want_qp: bool = False):
    """Batched MPC.mpcControl (mpc.py:111-214).  u_p [n,2] device tensor updated in place (the new
    u_p the reference returns).  Returns dict: u [n,2], iters, status, and with want_qp the assembled
    QP (H [n,2m,2m], g [n,2m], lu [n,2,4m]) and its solution du [n,2m]."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    s = _dev(torch, s, torch.float64).reshape(-1, 3)
    n = int(s.shape[0])
    nv = 2 * int(mpc_params.m)
    s_d = _dev(torch, s_d, torch.float64).reshape(-1, 3)
    u_r = _dev(torch, u_r, torch.float64).reshape(-1, 2)
    vw = _dev(torch, robot_vw, torch.float64).reshape(-1, 2)
    f64 = dict(dtype=torch.float64, device="cuda")
    out = dict(u=torch.empty((n, 2), **f64), iters=torch.empty(n, dtype=torch.int32, device="cuda"),
               status=torch.empty(n, dtype=torch.int32, device="cuda"))
    out.update(H=torch.zeros((n, nv, nv), **f64), g=torch.zeros((n, nv), **f64), lu=torch.zeros((n, 2, 2 * nv), **f64),
               du=torch.zeros((n, nv), **f64)) if want_qp else out.update(H=None, g=None, lu=None, du=None)
    rc = L.pmp_mpc_control_batch(ctx, _lib.stream_ptr(), ctypes.byref(lp_params),
                                 ctypes.byref(mpc_params), n, s.data_ptr(), s_d.data_ptr(), u_r.data_ptr(),
                                 u_p.data_ptr(), vw.data_ptr(), out["u"].data_ptr(), _lib.ptr(out["H"]),
                                 _lib.ptr(out["g"]), _lib.ptr(out["lu"]), _lib.ptr(out["du"]), out["iters"].data_ptr(),
                                 out["status"].data_ptr())
    _lib.check(ctx, rc, "pmp_mpc_control_batch")
    return out


def track_step_batch(kind: str, lp_params, state, goal, path_xy, path_off, iters: int = 1, lqr_params=None,
                     mpc_params=None, u_p=None, want_hist: bool = False):
    """Batched LQR.plan / MPC.plan iterations (lqr.py:58-86, mpc.py:66-94), kind "lqr" or "mpc".
    state [na,5] f64 device tensor (updated in place); u_p [na,2] device tensor (MPC, in place).
    Returns dict of device tensors (u, status, n_steps, admm_iters, optional hist_pose)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    k = {"lqr": _lib.TRACK_LQR, "mpc": _lib.TRACK_MPC}[kind]
    na = int(state.shape[0])
    goal = _dev(torch, goal, torch.float64).reshape(-1, 3)
    path_xy = _dev(torch, path_xy, torch.float64).reshape(-1, 2)
    path_off = _dev(torch, path_off, torch.int32)
    if k == _lib.TRACK_MPC and u_p is None:
        raise ValueError("MPC needs the carried u_p tensor [na, 2]")
    out = dict(u=torch.empty((na, 2), dtype=torch.float64, device="cuda"),
               status=torch.empty(na, dtype=torch.int32, device="cuda"),
               n_steps=torch.empty(na, dtype=torch.int32, device="cuda"),
               admm_iters=torch.empty(na, dtype=torch.int32, device="cuda"))
    out["hist_pose"] = torch.zeros((na, iters, 3), dtype=torch.float64, device="cuda") if want_hist else None
    rc = L.pmp_track_step_batch(ctx, _lib.stream_ptr(), k, ctypes.byref(lp_params),
                                ctypes.byref(lqr_params) if lqr_params is not None else None,
                                ctypes.byref(mpc_params) if mpc_params is not None else None, na, state.data_ptr(),
                                _lib.ptr(u_p), goal.data_ptr(), path_xy.data_ptr(), path_off.data_ptr(), int(iters),
                                out["u"].data_ptr(), out["status"].data_ptr(), out["n_steps"].data_ptr(),
                                _lib.ptr(out["hist_pose"]), out["admm_iters"].data_ptr())
    _lib.check(ctx, rc, "pmp_track_step_batch")
    return out


def dstar2d_batch(occ, starts, goals, path_cap: int | None = None, max_process: int = 0):
    """Batched DStar.plan (d_star.py:75-156) on one Grid.  occ uint8 [W, H] (x-major).
    Returns dict of device tensors: cost, path_len, path [nq, path_cap] (cells x*H+y, start -> goal),
    n_process (processState calls), status (4 = the reference raises: start unreachable)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ = np.asarray(occ)
    W, H = occ.shape
    occ_bits = occ_bits_device(occ, torch)
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    path_cap = W * H + 1 if path_cap is None else int(path_cap)
    out = dict(cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
               path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
               path=torch.empty((nq, path_cap), dtype=torch.int32, device="cuda"),
               n_process=torch.empty(nq, dtype=torch.int64, device="cuda"),
               status=torch.empty(nq, dtype=torch.int32, device="cuda"))
    rc = L.pmp_dstar2d_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), W, H,
                             s.data_ptr(), g.data_ptr(), nq, out["cost"].data_ptr(), out["path_len"].data_ptr(),
                             out["path"].data_ptr(), path_cap, out["n_process"].data_ptr(), out["status"].data_ptr(),
                             int(max_process))
    _lib.check(ctx, rc, "pmp_dstar2d_batch")
    return out


def dstar2d_onpress_batch(occ, starts, goals, presses, path_cap: int | None = None, max_process: int = 0):
    """Batched DStar.plan followed by one DStar.OnPress per press (d_star.py:75-134) on one Grid,
    pmp_dstar2d_onpress_batch.  presses [nq, npress, 2] int cells (x, y).
    Returns dict of device tensors, per call r (0 = plan): cost [nq, R], path_len [nq, R],
    path [nq, R, path_cap] (cells x*H+y; plan start -> goal, presses the walk without the goal),
    n_process [nq, R] (len(EXPAND)), status [nq, R] (include/pmp.h)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ = np.asarray(occ)
    W, H = occ.shape
    occ_bits = occ_bits_device(occ, torch)
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    pr = _dev(torch, presses, torch.int32)
    if pr.dim() != 3 or pr.shape[0] != nq or pr.shape[2] != 2:
        raise ValueError("presses must be [nq, npress, 2]")
    R = int(pr.shape[1]) + 1
    path_cap = 4 * W * H + 8 if path_cap is None else int(path_cap)
    i32 = dict(dtype=torch.int32, device="cuda")
    out = dict(cost=torch.empty((nq, R), dtype=torch.float64, device="cuda"), path_len=torch.empty((nq, R), **i32),
               path=torch.empty((nq, R, path_cap), **i32),
               n_process=torch.empty((nq, R), dtype=torch.int64, device="cuda"), status=torch.empty((nq, R), **i32))
    rc = L.pmp_dstar2d_onpress_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), W, H, s.data_ptr(), g.data_ptr(), nq,
                                     pr.data_ptr(), R - 1, out["cost"].data_ptr(), out["path_len"].data_ptr(),
                                     out["path"].data_ptr(), path_cap, out["n_process"].data_ptr(),
                                     out["status"].data_ptr(), int(max_process))
    _lib.check(ctx, rc, "pmp_dstar2d_onpress_batch")
    return out


def lpastar2d_batch(occ, starts, goals, heuristic: str = "euclidean", path_cap: int = 1001, counters: bool = False,
                    lite: bool = False):
    """Batched LPAStar.plan (lpa_star.py:78-87: computeShortestPath + extractPath) on one Grid;
    lite=True runs DStarLite.plan (d_star_lite.py:14-187, pmp_dstarlite2d_batch).
    occ uint8 [W, H] (x-major).  Returns dict of device tensors: cost, path_len, path [nq, path_cap]
    (cells x*H+y, start -> goal), n_expanded (len(EXPAND)), status (1 = extractPath gave up after
    1000 steps, 4 = the reference raises), optional counters [nq, 4]."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ = np.asarray(occ)
    W, H = occ.shape
    occ_bits = occ_bits_device(occ, torch)
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    out = dict(cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
               path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
               path=torch.empty((nq, int(path_cap)), dtype=torch.int32, device="cuda"),
               n_expanded=torch.empty(nq, dtype=torch.int32, device="cuda"),
               status=torch.empty(nq, dtype=torch.int32, device="cuda"))
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    fn = L.pmp_dstarlite2d_batch if lite else L.pmp_lpastar2d_batch
    rc = fn(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), W, H,
                               1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq,
                               out["cost"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(),
                               int(path_cap), out["n_expanded"].data_ptr(), _lib.ptr(out["counters"]),
                               out["status"].data_ptr())
    _lib.check(ctx, rc, "pmp_dstarlite2d_batch" if lite else "pmp_lpastar2d_batch")
    return out


def lpastar2d_replan_batch(occ, starts, goals, toggles, heuristic: str = "euclidean", path_cap: int = 1001,
                           counters: bool = False, lite: bool = False):
    """LPAStar.plan() then one LPAStar.OnPress edit (lpa_star.py:101-137) per toggle, each followed by
    plan() on the kept state, for every query (pmp_lpastar2d_replan_batch); lite=True: DStarLite.plan()
    then DStarLite.OnPress per toggle (d_star_lite.py:61-97, pmp_dstarlite2d_replan_batch).  toggles [nq, nt, 2].
    Returns cost / n_expanded / status [nq, nt + 1] (status -1 = not run) and the last plan's path."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ = np.asarray(occ)
    W, H = occ.shape
    occ_bits = occ_bits_device(occ, torch)
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    t = _dev(torch, toggles, torch.int32).reshape(nq, -1, 2)
    nt = int(t.shape[1])
    if nt < 1:
        raise ValueError("lpastar2d_replan_batch needs at least one toggle per query")
    if bool(((t[..., 0] < 0) | (t[..., 0] >= W) | (t[..., 1] < 0) | (t[..., 1] >= H)).any()):
        raise ValueError("toggle cells must lie in the grid (OnPress rejects others, lpa_star.py:108-109)")
    out = dict(cost=torch.empty((nq, nt + 1), dtype=torch.float64, device="cuda"),
               n_expanded=torch.empty((nq, nt + 1), dtype=torch.int32, device="cuda"),
               status=torch.empty((nq, nt + 1), dtype=torch.int32, device="cuda"),
               path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
               path=torch.empty((nq, int(path_cap)), dtype=torch.int32, device="cuda"))
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    fn = L.pmp_dstarlite2d_replan_batch if lite else L.pmp_lpastar2d_replan_batch
    rc = fn(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), W, H,
                                      1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq,
                                      t.data_ptr(), nt, out["cost"].data_ptr(), out["n_expanded"].data_ptr(),
                                      out["status"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(),
                                      int(path_cap), _lib.ptr(out["counters"]))
    _lib.check(ctx, rc, "pmp_dstarlite2d_replan_batch" if lite else "pmp_lpastar2d_replan_batch")
    return out


def map_arrays(env, torch=None):
    """Map obstacle lists (env.py:83-117) -> device f64 tensors rect [nr,4], circ [nc,3], bnd [nb,4]."""
    torch = torch or _lib.device_check()

    def t(lst, k):
        a = np.asarray(lst if lst else np.zeros((0, k)), np.float64).reshape(-1, k)
        return torch.as_tensor(np.ascontiguousarray(a), device="cuda")

    return t(env.obs_rect, 4), t(env.obs_circ, 3), t(env.boundary, 4)


def rrt_batch(env, starts, goals, rnd, sample_num: int, star: bool = True, max_dist: float = 0.5,
              radius: float = 10.0, goal_sample_rate: float = 0.05, delta: float = 0.5, path_cap: int | None = None,
              counters: bool = False):
    """Batched RRT / RRT* plans (rrt.py:49-151, rrt_star.py:43-76) on one Map.
    rnd: [nq, stride] f64 random streams (RandomState.random_sample order; 3*sample_num+1 per query).
    Returns dict of device tensors: tree_xy [nq,cap,2], tree_g, tree_parent, n_nodes, cost, path_len,
    path [nq,path_cap,2] (goal -> start), draws, status."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    rect, circ, bnd = map_arrays(env, torch)
    s = _dev(torch, starts, torch.float64).reshape(-1, 2)
    g = _dev(torch, goals, torch.float64).reshape(-1, 2)
    nq = int(s.shape[0])
    rnd = _dev(torch, rnd, torch.float64).reshape(nq, -1)
    cap = int(sample_num) + 2
    path_cap = cap if path_cap is None else int(path_cap)
    f64 = dict(dtype=torch.float64, device="cuda")
    i32 = dict(dtype=torch.int32, device="cuda")
    out = dict(tree_xy=torch.empty((nq, cap, 2), **f64), tree_g=torch.empty((nq, cap), **f64),
               tree_parent=torch.empty((nq, cap), **i32), n_nodes=torch.empty(nq, **i32),
               cost=torch.empty(nq, **f64), path_len=torch.empty(nq, **i32),
               path=torch.empty((nq, max(path_cap, 1), 2), **f64), draws=torch.empty(nq, dtype=torch.int64, device="cuda"),
               status=torch.empty(nq, **i32),
               counters=torch.zeros((nq, 4), dtype=torch.int64, device="cuda") if counters else None)
    P = _lib.RRTParams(float(env.x_range), float(env.y_range), float(delta), float(max_dist), float(radius),
                       float(goal_sample_rate), int(sample_num), int(bool(star)))
    rc = L.pmp_rrt_batch(ctx, _lib.stream_ptr(), ctypes.byref(P), rect.data_ptr(),
                         int(rect.shape[0]), circ.data_ptr(), int(circ.shape[0]), bnd.data_ptr(), int(bnd.shape[0]),
                         s.data_ptr(), g.data_ptr(), nq, rnd.data_ptr(), int(rnd.shape[1]), cap,
                         out["tree_xy"].data_ptr(), out["tree_g"].data_ptr(), out["tree_parent"].data_ptr(),
                         out["n_nodes"].data_ptr(), out["cost"].data_ptr(), out["path_len"].data_ptr(),
                         out["path"].data_ptr(), path_cap, out["draws"].data_ptr(), out["status"].data_ptr(),
                         _lib.ptr(out["counters"]))
    _lib.check(ctx, rc, "pmp_rrt_batch")
    return out


def astar3d_batch(occ, starts, goals, heuristic: str = "euclidean", path_cap: int | None = None,
                  expand_cap: int = 0, counters: bool = False, algo: str = "astar"):
    """Batched AStar3D.plan (a_star3d.py:33-106); algo "dijkstra" / "gbfs" run Dijkstra3D.plan
    (dijkstra3d.py:39-87) / GBFS3D.plan (gbfs3d.py:34-82) on the same kernel (pmp_graph3d_batch).

    occ: uint8 [X, Y, Z] shared grid or [nq, X, Y, Z] per-query grids (numpy).
    Returns dict of device tensors: cost (inf if unreachable), path_len, path [nq, path_cap]
    (cells (x*Y+y)*Z+z, start -> goal), n_expanded (len(CLOSED)), status, optional expand / counters.
    """
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ = np.asarray(occ)
    per_query = occ.ndim == 4
    X, Y, Z = occ.shape[-3:]
    if per_query:
        words = np.stack([pack_bits(o) for o in occ])
    else:
        words = pack_bits(occ)
    occ_bits = torch.as_tensor(np.ascontiguousarray(words).view(np.int32), device="cuda")
    s = _dev(torch, starts, torch.int32).reshape(-1, 3)
    g = _dev(torch, goals, torch.int32).reshape(-1, 3)
    nq = int(s.shape[0])
    if path_cap is None:
        path_cap = min(X * Y * Z + 1, 1 << 16)
    out = dict(cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
               path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
               path=torch.empty((nq, path_cap), dtype=torch.int32, device="cuda"),
               n_expanded=torch.empty(nq, dtype=torch.int32, device="cuda"),
               status=torch.empty(nq, dtype=torch.int32, device="cuda"))
    out["expand"] = torch.empty((nq, expand_cap), dtype=torch.int32, device="cuda") if expand_cap else None
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    rc = L.pmp_graph3d_batch(ctx, _lib.stream_ptr(), _lib.ALGOS[algo], occ_bits.data_ptr(), 1 if per_query else 0,
                             X, Y, Z, 1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq,
                             out["cost"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(), path_cap,
                             out["n_expanded"].data_ptr(), _lib.ptr(out["expand"]), int(expand_cap),
                             _lib.ptr(out["counters"]), out["status"].data_ptr())
    _lib.check(ctx, rc, "pmp_graph3d_batch")
    out["dims"] = (X, Y, Z)
    return out


def dstar3d_batch(occ, starts, goals, blocks=None, path_cap: int | None = None, expand_cap: int = 0,
                  max_process: int = 0, occ_bits=None):
    """Batched DStar3D (d_star3d.py:60-281): plan() and then one apply_dynamic_obstacles() per round
    of `blocks` [nq, nrounds, nblk, 3] (int voxels; outside the grid = ignored), on pmp_dstar3d_batch.

    occ: uint8 [X, Y, Z] shared grid or [nq, X, Y, Z] per-query grids (numpy).
    Returns dict of device tensors, per round r (0 = plan): cost [nq, R], path_len [nq, R],
    path [nq, R, path_cap] (voxels (x*Y+y)*Z+z, start -> goal), n_process [nq, R] (len(EXPAND)),
    status [nq, R] (include/pmp.h), optional expand [nq, expand_cap] (plan()'s EXPAND voxels).
    occ_bits: optional device words of `occ` already packed (occ may then be just its shape)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ_bits, per_query, (X, Y, Z) = _occ3d_bits(torch, occ, occ_bits)
    s = _dev(torch, starts, torch.int32).reshape(-1, 3)
    g = _dev(torch, goals, torch.int32).reshape(-1, 3)
    nq = int(s.shape[0])
    if blocks is None:
        nr, nb, b = 0, 0, None
    else:
        b = _dev(torch, blocks, torch.int32)
        if b.dim() != 4 or b.shape[0] != nq or b.shape[3] != 3:
            raise ValueError("blocks must be [nq, nrounds, nblk, 3]")
        nr, nb = int(b.shape[1]), int(b.shape[2])
    R = nr + 1
    path_cap = min(X * Y * Z + 1, 1 << 16) if path_cap is None else int(path_cap)
    i32 = dict(dtype=torch.int32, device="cuda")
    out = dict(cost=torch.empty((nq, R), dtype=torch.float64, device="cuda"), path_len=torch.empty((nq, R), **i32),
               path=torch.empty((nq, R, path_cap), **i32),
               n_process=torch.empty((nq, R), dtype=torch.int64, device="cuda"), status=torch.empty((nq, R), **i32))
    out["expand"] = torch.empty((nq, expand_cap), **i32) if expand_cap else None
    rc = L.pmp_dstar3d_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), 1 if per_query else 0, X, Y, Z, s.data_ptr(),
                             g.data_ptr(), nq, _lib.ptr(b), nr, nb, out["cost"].data_ptr(), out["path_len"].data_ptr(),
                             out["path"].data_ptr(), path_cap, out["n_process"].data_ptr(), out["status"].data_ptr(),
                             _lib.ptr(out["expand"]), int(expand_cap), int(max_process))
    _lib.check(ctx, rc, "pmp_dstar3d_batch")
    out["dims"] = (X, Y, Z)
    return out


def _occ3d_bits(torch, occ, occ_bits=None):
    """(device words, per_query, (X, Y, Z)) of a shared [X, Y, Z] or per-query [nq, X, Y, Z] grid; with
    occ_bits given, `occ` only supplies the shape."""
    shape = tuple(occ) if isinstance(occ, tuple) else np.asarray(occ).shape
    per_query = len(shape) == 4
    if occ_bits is None:
        occ = np.asarray(occ)
        words = np.stack([pack_bits(o) for o in occ]) if per_query else pack_bits(occ)
        occ_bits = torch.as_tensor(np.ascontiguousarray(words).view(np.int32), device="cuda")
    return occ_bits, per_query, tuple(int(d) for d in shape[-3:])


def lpastar3d_batch(occ, starts, goals, changes=None, heuristic: str = "euclidean", path_cap: int | None = None,
                    counters: bool = False, max_expansions: int = 0, occ_bits=None):
    """Batched LPAStar3D (lpa_star3d.py:40-225): plan() and then one apply_change() per row of
    `changes` [nq, nr, 4] = (x, y, z, mode) with mode 0 = blocked None (toggle), 1 = True, 2 = False,
    on pmp_lpastar3d_batch.  occ: uint8 [X, Y, Z] shared or [nq, X, Y, Z] per-query grids.
    Returns dict of device tensors per call r (0 = plan): cost [nq, R], path_len [nq, R],
    path [nq, R, path_cap] (voxels (x*Y+y)*Z+z, start -> goal), n_expanded [nq, R] (len(EXPAND)),
    status [nq, R] (include/pmp.h), optional counters [nq, 4].
    occ_bits: optional device words of `occ` already packed (occ may then be just its shape)."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    occ_bits, per_query, (X, Y, Z) = _occ3d_bits(torch, occ, occ_bits)
    s = _dev(torch, starts, torch.int32).reshape(-1, 3)
    g = _dev(torch, goals, torch.int32).reshape(-1, 3)
    nq = int(s.shape[0])
    if changes is None:
        nr, ch = 0, None
    else:
        ch = _dev(torch, changes, torch.int32)
        if ch.dim() != 3 or ch.shape[0] != nq or ch.shape[2] != 4:
            raise ValueError("changes must be [nq, nr, 4]")
        nr = int(ch.shape[1])
    R = nr + 1
    path_cap = min(X * Y * Z + 1, 1 << 16) if path_cap is None else int(path_cap)
    i32 = dict(dtype=torch.int32, device="cuda")
    out = dict(cost=torch.empty((nq, R), dtype=torch.float64, device="cuda"), path_len=torch.empty((nq, R), **i32),
               path=torch.empty((nq, R, path_cap), **i32),
               n_expanded=torch.empty((nq, R), dtype=torch.int64, device="cuda"), status=torch.empty((nq, R), **i32))
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    rc = L.pmp_lpastar3d_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), 1 if per_query else 0, X, Y, Z,
                               1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq, _lib.ptr(ch), nr,
                               out["cost"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(), path_cap,
                               out["n_expanded"].data_ptr(), out["status"].data_ptr(), _lib.ptr(out["counters"]),
                               int(max_expansions))
    _lib.check(ctx, rc, "pmp_lpastar3d_batch")
    out["dims"] = (X, Y, Z)
    return out


def totp3d_batch(paths, params, point_cap: int | None = None, eval_t=None, retry_overflow: bool = True):
    """Batched TimeOptimalTrajectory3D(path, constraints, path_resolution).generate()
    (trajectory/time_optimal_trajectory.py:260-302) on pmp_totp3d_batch.  paths: list of [n, 3]
    waypoint arrays (reference order); params: _lib.TotpParams.  With eval_t (1-D times), evaluate(t)
    (:304-335) at those times instead of generate()'s sampling.
    Returns dict of device tensors: s_values / s_dot / s_ddot / time [nq, sample_cap], n_samples,
    points [nq, point_cap, 12] (time, position, velocity, acceleration, yaw, yaw rate; NaN = None),
    n_points, total_time, status (include/pmp.h).  Queries whose points overflow the first cap are
    re-run with their exact count when retry_overflow."""
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    arrs = [np.asarray(p, np.float64).reshape(-1, 3) for p in paths]
    nq = len(arrs)
    off = np.zeros(nq + 1, np.int32)
    off[1:] = np.cumsum([len(a) for a in arrs])
    nmax = max(2, max((len(a) for a in arrs), default=2))
    # n_samples = max(int(L / res), 100) with L summed in the kernel's (the reference's) order
    res = float(params.path_resolution)
    ns = [max(int(np.cumsum(np.sqrt(np.sum(np.diff(a, axis=0) ** 2, axis=1)))[-1] / res), 100) if len(a) > 1 else 1
          for a in arrs]
    sample_cap = max(ns, default=1) + 1
    flat = torch.as_tensor(np.concatenate(arrs) if nq else np.zeros((0, 3)), device="cuda")
    off_d = torch.as_tensor(off, device="cuda")
    et = None if eval_t is None else torch.as_tensor(np.asarray(eval_t, np.float64).ravel(), device="cuda")
    n_eval = 0 if et is None else int(et.numel())
    if point_cap is None:
        point_cap = n_eval + 1 if et is not None else 2048

    def launch(idx_paths, offs, pc):
        m = len(offs) - 1
        f64 = dict(dtype=torch.float64, device="cuda")
        i32 = dict(dtype=torch.int32, device="cuda")
        o = dict(s_values=torch.empty((m, sample_cap), **f64), s_dot=torch.empty((m, sample_cap), **f64),
                 s_ddot=torch.empty((m, sample_cap), **f64), time=torch.empty((m, sample_cap), **f64),
                 n_samples=torch.empty(m, **i32), points=torch.empty((m, pc, 12), **f64), n_points=torch.empty(m, **i32),
                 total_time=torch.empty(m, **f64), status=torch.empty(m, **i32))
        if m:
            rc = L.pmp_totp3d_batch(ctx, _lib.stream_ptr(), ctypes.byref(params), m, idx_paths.data_ptr(),
                                    offs.data_ptr(), nmax, sample_cap, o["s_values"].data_ptr(), o["s_dot"].data_ptr(),
                                    o["s_ddot"].data_ptr(), o["time"].data_ptr(), o["n_samples"].data_ptr(), pc,
                                    o["points"].data_ptr(), o["n_points"].data_ptr(), o["total_time"].data_ptr(),
                                    o["status"].data_ptr(), _lib.ptr(et), n_eval)
            _lib.check(ctx, rc, "pmp_totp3d_batch")
        return o

    out = launch(flat, off_d, int(point_cap))
    if retry_overflow and nq:
        st = out["status"].cpu().numpy()
        npt = out["n_points"].cpu().numpy()
        redo = np.nonzero((st == _lib.STATUS_PATH_OVERFLOW) & (npt > point_cap))[0]
        if len(redo):
            pc = int(npt[redo].max())
            sub = [arrs[i] for i in redo]
            so = np.zeros(len(sub) + 1, np.int32)
            so[1:] = np.cumsum([len(a) for a in sub])
            r = launch(torch.as_tensor(np.concatenate(sub), device="cuda"), torch.as_tensor(so, device="cuda"), pc)
            big = torch.full((nq, pc, 12), float("nan"), dtype=torch.float64, device="cuda")
            big[:, : int(point_cap)] = out["points"]
            idx = torch.as_tensor(redo, device="cuda", dtype=torch.long)
            big[idx] = r["points"]
            out["points"] = big
            for k in ("s_values", "s_dot", "s_ddot", "time", "n_samples", "n_points", "total_time", "status"):
                out[k][idx] = r[k]
    return out
