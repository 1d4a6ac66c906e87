"""ctypes front-end of the CPU oracle (oracle/pmp_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package python_motion_planning_amd never imports this.
Each wrapper names the reference function it restates (see pmp_oracle.c for file:line).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
# tests/test_oracle_sanitized.py points this at the ASan/UBSan build (make -C oracle san)
_SAN_PATH = os.environ.get("PMP_ORACLE_LIB")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "pmp_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "-B" if force else "liboracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if _SAN_PATH:
            L = ctypes.CDLL(_SAN_PATH)
        else:
            build()
            L = ctypes.CDLL(_LIB_PATH)
        L.oracle_hypot.restype = ctypes.c_double
        L.oracle_hypot.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oracle_hypot_many.restype = None
        L.oracle_hypot_many.argtypes = [_dp, _dp, _dp, ctypes.c_int64]
        L.oracle_graph2d.restype = ctypes.c_int
        L.oracle_graph2d.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     _dp, _i32p, ctypes.c_int, _i32p, _i32p, ctypes.c_int, _i32p, _i64p]
        L.oracle_graph3d.restype = ctypes.c_int
        L.oracle_graph3d.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     _i32p, _i32p, _dp, _i32p, ctypes.c_int, _i32p, _i32p, ctypes.c_int,
                                     _i32p, _i64p]
        L.oracle_dstar2d.restype = ctypes.c_int
        L.oracle_dstar2d.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, _dp, _i32p, ctypes.c_int, _i32p,
                                     _i64p, ctypes.c_int64]
        L.oracle_graph2d_batch.restype = ctypes.c_int
        L.oracle_graph2d_batch.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p,
                                           _i32p, ctypes.c_int, _dp, _i32p, ctypes.c_int, _i32p, _i32p, _i64p,
                                           _i32p, ctypes.c_int]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def hypot(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64).ravel()
    b = np.ascontiguousarray(b, dtype=np.float64).ravel()
    out = np.empty_like(a)
    lib().oracle_hypot_many(_p(a, _dp), _p(b, _dp), _p(out, _dp), a.size)
    return out


# planners sharing the AStar loop (pmp_oracle.c oracle_graph2d / oracle_graph3d)
ALGOS = {"astar": 0, "dijkstra": 1, "gbfs": 2}
# 2D only: ThetaStar / LazyThetaStar on the same loop (3D Theta* is theta3d below)
ALGOS2D = dict(ALGOS, theta_star=3, lazy_theta_star=4)


def astar2d(occ: np.ndarray, start, goal, heuristic: str = "euclidean", with_expand: bool = True,
            path_cap: int | None = None, expand_cap: int | None = None, algo: str = "astar"):
    """Restatement of AStar.plan (a_star.py:39-83); algo "dijkstra" / "gbfs" restate Dijkstra.plan
    (dijkstra.py:36-85) / GBFS.plan (gbfs.py:36-86), "theta_star" / "lazy_theta_star" ThetaStar.plan
    (theta_star.py:44-94) / LazyThetaStar.plan (lazy_theta_star.py:38-101).  occ: uint8 [W, H],
    occ[x, y] != 0 blocked.
    Returns dict(status, cost, path (goal->start list of (x,y)), expand (closure order), counters)."""
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    path_cap = path_cap or W * H + 1
    expand_cap = expand_cap or (W * H if with_expand else 0)
    path = np.zeros(path_cap, np.int32)
    expand = np.zeros(max(expand_cap, 1), np.int32)
    cost = ctypes.c_double(0)
    plen = ctypes.c_int32(0)
    nexp = ctypes.c_int32(0)
    ctr = np.zeros(4, np.int64)
    st = lib().oracle_graph2d(ALGOS2D[algo], _p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0,
                              int(start[0]), int(start[1]), int(goal[0]), int(goal[1]),
                              ctypes.byref(cost), _p(path, _i32p), path_cap, ctypes.byref(plen),
                              _p(expand, _i32p) if with_expand else None, expand_cap,
                              ctypes.byref(nexp), _p(ctr, _i64p))
    cells = path[: plen.value]
    out = dict(status=st, cost=cost.value, n_expanded=nexp.value,
               path=[(int(c) // H, int(c) % H) for c in cells], path_cells=cells.copy(),
               n_push=int(ctr[0]), n_pop=int(ctr[1]), max_heap=int(ctr[3]))
    if with_expand:
        e = expand[: min(nexp.value, expand_cap)]
        out["expand_cells"] = e.copy()
    return out


def astar3d(occ: np.ndarray, start, goal, heuristic: str = "euclidean", with_expand: bool = True,
            algo: str = "astar"):
    """Restatement of AStar3D.plan (a_star3d.py:33-78); algo "dijkstra" / "gbfs" restate
    Dijkstra3D.plan (dijkstra3d.py:39-87) / GBFS3D.plan (gbfs3d.py:34-82).  occ: uint8 [X, Y, Z]."""
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    X, Y, Z = occ.shape
    n = X * Y * Z
    path = np.zeros(n + 1, np.int32)
    expand = np.zeros(n, np.int32)
    s = np.asarray(start, np.int32)
    g = np.asarray(goal, np.int32)
    cost = ctypes.c_double(0)
    plen = ctypes.c_int32(0)
    nexp = ctypes.c_int32(0)
    ctr = np.zeros(4, np.int64)
    st = lib().oracle_graph3d(ALGOS[algo], _p(occ, _u8p), X, Y, Z, 1 if heuristic == "manhattan" else 0,
                              _p(s, _i32p), _p(g, _i32p), ctypes.byref(cost), _p(path, _i32p), n + 1,
                              ctypes.byref(plen), _p(expand, _i32p) if with_expand else None, n,
                              ctypes.byref(nexp), _p(ctr, _i64p))

    def dec(c):
        c = int(c)
        return (c // (Y * Z), (c // Z) % Y, c % Z)

    out = dict(status=st, cost=cost.value, n_expanded=nexp.value,
               path=[dec(c) for c in path[: plen.value]], path_cells=path[: plen.value].copy(),
               n_push=int(ctr[0]), n_pop=int(ctr[1]), n_iter=int(ctr[2]), max_heap=int(ctr[3]))
    if with_expand:
        out["expand_cells"] = expand[: nexp.value].copy()
    return out


def dstar2d(occ: np.ndarray, start, goal, max_process: int = 0):
    """Restatement of DStar.plan (d_star.py:75-89).  Returns path start->goal."""
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    path = np.zeros(W * H + 1, np.int32)
    cost = ctypes.c_double(0)
    plen = ctypes.c_int32(0)
    nproc = ctypes.c_int64(0)
    st = lib().oracle_dstar2d(_p(occ, _u8p), W, H, int(start[0]), int(start[1]), int(goal[0]),
                              int(goal[1]), ctypes.byref(cost), _p(path, _i32p), W * H + 1,
                              ctypes.byref(plen), ctypes.byref(nproc), max_process)
    cells = path[: plen.value]
    return dict(status=st, cost=cost.value, n_process=nproc.value,
                path=[(int(c) // H, int(c) % H) for c in cells], path_cells=cells.copy())


def dstar2d_batch(occ: np.ndarray, starts, goals, nthreads: int = 0):
    """OpenMP batch of the DStar.plan restatement: cost, status, n_process per query."""
    L = lib()
    if not getattr(L, "_dsb_set", False):
        L.oracle_dstar2d_batch.restype = None
        L.oracle_dstar2d_batch.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, _i32p, _i32p, ctypes.c_int, _dp, _i32p,
                                           _i64p, ctypes.c_int]
        L._dsb_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 2)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 2)
    nq = len(s)
    out = dict(cost=np.zeros(nq), status=np.zeros(nq, np.int32), n_process=np.zeros(nq, np.int64))
    L.oracle_dstar2d_batch(_p(occ, _u8p), W, H, _p(s, _i32p), _p(g, _i32p), nq, _p(out["cost"], _dp),
                           _p(out["status"], _i32p), _p(out["n_process"], _i64p), int(nthreads))
    return out


def astar2d_batch(occ: np.ndarray, starts, goals, heuristic: str = "euclidean", path_cap: int = 4096,
                  nthreads: int = 0, algo: str = "astar"):
    """OpenMP batch of the AStar.plan (or Dijkstra / GBFS) restatement (one grid, many queries)."""
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 2)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 2)
    nq = len(s)
    out = dict(cost=np.zeros(nq), path=np.zeros((nq, path_cap), np.int32), path_len=np.zeros(nq, np.int32),
               n_expanded=np.zeros(nq, np.int32), counters=np.zeros((nq, 4), np.int64),
               status=np.zeros(nq, np.int32))
    lib().oracle_graph2d_batch(ALGOS2D[algo], _p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0, _p(s, _i32p),
                               _p(g, _i32p), nq, _p(out["cost"], _dp), _p(out["path"], _i32p), path_cap,
                               _p(out["path_len"], _i32p), _p(out["n_expanded"], _i32p),
                               _p(out["counters"], _i64p), _p(out["status"], _i32p), int(nthreads))
    return out


# ------------------------------------------------------------------------------------------------
# local planners
class LPParams(ctypes.Structure):
    """LocalPlanner.params (local_planner.py:39-55)."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "dt", "lookahead_time", "max_lookahead", "min_lookahead", "max_v_inc", "min_v_inc", "max_v", "min_v",
        "max_w_inc", "min_w_inc", "max_w", "min_w", "goal_dist_tol", "rotate_tol")]

    @classmethod
    def default(cls, **kw):
        import math

        d = dict(dt=0.1, lookahead_time=1.0, max_lookahead=2.5, min_lookahead=1.0, max_v_inc=1.0, min_v_inc=-1.0,
                 max_v=0.5, min_v=0.0, max_w_inc=math.pi, min_w_inc=-math.pi, max_w=math.pi / 2, min_w=-math.pi / 2,
                 goal_dist_tol=0.5, rotate_tol=0.5)
        d.update(kw)
        return cls(**d)


class LQRParams(ctypes.Structure):
    """LQR settings (lqr.py:35-38); mirrors pmp_lqr_params."""
    _fields_ = [("q", ctypes.c_double * 3), ("r", ctypes.c_double * 2), ("iters", ctypes.c_int32),
                ("eps", ctypes.c_double)]

    @classmethod
    def default(cls, **kw):
        d = dict(q=(1.0, 1.0, 1.0), r=(1.0, 1.0), iters=100, eps=0.1)
        d.update(kw)
        return cls((ctypes.c_double * 3)(*d["q"]), (ctypes.c_double * 2)(*d["r"]), d["iters"], d["eps"])


class MPCParams(ctypes.Structure):
    """MPC horizons/weights (mpc.py:37-40) + ADMM settings (OSQP defaults); mirrors pmp_mpc_params."""
    _fields_ = [("p", ctypes.c_int32), ("m", ctypes.c_int32), ("q", ctypes.c_double * 3), ("r", ctypes.c_double * 2),
                ("rho", ctypes.c_double), ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double), ("adaptive_tol", ctypes.c_double),
                ("max_iter", ctypes.c_int32), ("check_every", ctypes.c_int32), ("adaptive_every", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]

    @classmethod
    def default(cls, **kw):
        d = dict(p=12, m=8, q=(0.8, 0.8, 0.5), r=(2.0, 2.0), rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3,
                 eps_rel=1e-3, adaptive_tol=5.0, max_iter=4000, check_every=25, adaptive_every=25)
        d.update(kw)
        return cls(d["p"], d["m"], (ctypes.c_double * 3)(*d["q"]), (ctypes.c_double * 2)(*d["r"]), d["rho"],
                   d["sigma"], d["alpha"], d["eps_abs"], d["eps_rel"], d["adaptive_tol"], d["max_iter"],
                   d["check_every"], d["adaptive_every"], 0)


def _lp_lib():
    L = lib()
    if not getattr(L, "_lp_bound", False):
        P = ctypes.POINTER(LPParams)
        L.oracle_np_sum.restype = ctypes.c_double
        L.oracle_np_sum.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64]
        L.oracle_lookahead.restype = ctypes.c_int
        L.oracle_lookahead.argtypes = [_dp, ctypes.c_int, _dp, P, _dp, _dp, _dp]
        L.oracle_dwa_window.restype = None
        L.oracle_dwa_window.argtypes = [ctypes.c_double, ctypes.c_double, P, _dp]
        L.oracle_dwa_eval.restype = ctypes.c_int
        L.oracle_dwa_eval.argtypes = [_dp, ctypes.c_int, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp, _i32p, _dp]
        L.oracle_dwa_step.restype = ctypes.c_int
        L.oracle_dwa_step.argtypes = [_dp, ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, P, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp]
        L.oracle_reach_goal.restype = ctypes.c_int
        L.oracle_reach_goal.argtypes = [_dp, _dp, P]
        L.oracle_lqr_control.restype = None
        L.oracle_lqr_control.argtypes = [_dp, _dp, _dp, ctypes.c_double, ctypes.c_double, P,
                                         ctypes.POINTER(LQRParams), _dp]
        MP = ctypes.POINTER(MPCParams)
        L.oracle_mpc_assemble.restype = None
        L.oracle_mpc_assemble.argtypes = [_dp, _dp, _dp, _dp, P, MP, _dp, _dp, _dp, _dp]
        L.oracle_qp_admm.restype = ctypes.c_int
        L.oracle_qp_admm.argtypes = [ctypes.c_int, _dp, _dp, _dp, _dp, MP, _dp, _i32p, _dp]
        L.oracle_mpc_control.restype = ctypes.c_int
        L.oracle_mpc_control.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double, P, MP, _dp, _i32p]
        L.oracle_track_step.restype = ctypes.c_int
        L.oracle_track_step.argtypes = [ctypes.c_int, _dp, ctypes.c_int, _dp, _dp, _dp, P, ctypes.POINTER(LQRParams),
                                        MP, _dp, _i32p]
        L.oracle_track_batch.restype = ctypes.c_int64
        L.oracle_track_batch.argtypes = [ctypes.c_int, _dp, _i32p, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int, P,
                                         ctypes.POINTER(LQRParams), MP, _dp, _i32p, _i32p, ctypes.c_int]
        L._lp_bound = True
    return L


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def np_sum(a, stride=1):
    a = _d(a)
    n = (a.size + stride - 1) // stride
    return _lp_lib().oracle_np_sum(_p(a, _dp), n, stride)


def lookahead(path, robot_xyv, params=None):
    """getLookaheadPoint (local_planner.py:103-170) -> (status, (x, y), theta, kappa)."""
    path = _d(path).reshape(-1, 2)
    r = _d(robot_xyv)
    pt = np.zeros(2)
    th = ctypes.c_double(0)
    ka = ctypes.c_double(0)
    st = _lp_lib().oracle_lookahead(_p(path, _dp), len(path), _p(r, _dp), ctypes.byref(params or LPParams.default()),
                                    _p(pt, _dp), ctypes.byref(th), ctypes.byref(ka))
    return st, (float(pt[0]), float(pt[1])), th.value, ka.value


def dwa_window(v, w, params=None):
    out = np.zeros(4)
    _lp_lib().oracle_dwa_window(v, w, ctypes.byref(params or LPParams.default()), _p(out, _dp))
    return out


def dwa_eval(obstacles, state, goal_xy, vr, v_res=0.05, w_res=0.05, nv=0, nw=0, predict_time=1.5, dt=0.1,
             weights=(0.2, 0.1, 0.05), inflation=1.0):
    """DWA.evaluation (dwa.py:137-190): returns (eval3 [N,3] = eval_win @ factor, best, best_traj [H,5])."""
    obs = _d(obstacles).reshape(-1, 2)
    st = _d(state)
    g = _d(goal_xy)
    vr = _d(vr)
    nv_ = nv if nv > 0 else int((vr[1] - vr[0]) / v_res)
    nw_ = nw if nw > 0 else int((vr[3] - vr[2]) / w_res)
    N = max(nv_ * nw_, 0)
    H = int(predict_time / dt)
    e3 = np.zeros((max(N, 1), 3))
    bt = np.zeros((max(H, 1), 5))
    best = ctypes.c_int32(0)
    n = _lp_lib().oracle_dwa_eval(_p(obs, _dp), len(obs), _p(st, _dp), _p(g, _dp), _p(vr, _dp), v_res, w_res, nv, nw,
                                  predict_time, dt, weights[0], weights[1], weights[2], inflation, _p(e3, _dp),
                                  ctypes.byref(best), _p(bt, _dp))
    return e3[:n], best.value, bt[:H]


def dwa_step(obstacles, path, goal, state, params=None, v_res=0.05, w_res=0.05, nv=0, nw=0, predict_time=1.5,
             weights=(0.2, 0.1, 0.05), inflation=1.0):
    """One DWA.plan iteration (dwa.py:72-93); returns (status, new_state, u)."""
    obs = _d(obstacles).reshape(-1, 2)
    path = _d(path).reshape(-1, 2)
    g = _d(goal)
    st = _d(state).copy()
    u = np.zeros(2)
    rc = _lp_lib().oracle_dwa_step(_p(obs, _dp), len(obs), _p(path, _dp), len(path), _p(g, _dp), _p(st, _dp),
                                   ctypes.byref(params or LPParams.default()), v_res, w_res, nv, nw, predict_time,
                                   weights[0], weights[1], weights[2], inflation, _p(u, _dp))
    return rc, st, u


def lqr_control(s, s_d, u_r, robot_v, robot_w, params=None, lqr=None):
    """LQR.lqrControl (lqr.py:103-145) with the robot's current (v, w)."""
    u = np.zeros(2)
    _lp_lib().oracle_lqr_control(_p(_d(s), _dp), _p(_d(s_d), _dp), _p(_d(u_r), _dp), robot_v, robot_w,
                                 ctypes.byref(params or LPParams.default()), ctypes.byref(lqr or LQRParams.default()),
                                 _p(u, _dp))
    return u


def mpc_assemble(s, s_d, u_r, u_p, params=None, mpc=None):
    """MPC.mpcControl QP assembly (mpc.py:124-200) -> (H [2m,2m], g [2m], l [4m], u [4m])."""
    mpc = mpc or MPCParams.default()
    n = 2 * mpc.m
    H, g, lo, hi = np.zeros((n, n)), np.zeros(n), np.zeros(2 * n), np.zeros(2 * n)
    _lp_lib().oracle_mpc_assemble(_p(_d(s), _dp), _p(_d(s_d), _dp), _p(_d(u_r), _dp), _p(_d(u_p), _dp),
                                  ctypes.byref(params or LPParams.default()), ctypes.byref(mpc), _p(H, _dp), _p(g, _dp),
                                  _p(lo, _dp), _p(hi, _dp))
    return H, g, lo, hi


def qp_admm(H, g, lo, hi, mpc=None):
    """ADMM solve of min 1/2 x'Hx + g'x, lo <= [kron(tril(1),I2); I] x <= hi -> (x, status, iters, rho)."""
    mpc = mpc or MPCParams.default()
    x = np.zeros(2 * mpc.m)
    it = ctypes.c_int32(0)
    rho = ctypes.c_double(0)
    st = _lp_lib().oracle_qp_admm(mpc.m, _p(_d(H), _dp), _p(_d(g), _dp), _p(_d(lo), _dp), _p(_d(hi), _dp),
                                  ctypes.byref(mpc), _p(x, _dp), ctypes.byref(it), ctypes.byref(rho))
    return x, st, it.value, rho.value


def mpc_control(s, s_d, u_r, u_p, robot_v, robot_w, params=None, mpc=None):
    """MPC.mpcControl (mpc.py:111-214) -> (u [2], new u_p [2], admm status, iters)."""
    up = _d(u_p).copy()
    u = np.zeros(2)
    it = ctypes.c_int32(0)
    st = _lp_lib().oracle_mpc_control(_p(_d(s), _dp), _p(_d(s_d), _dp), _p(_d(u_r), _dp), _p(up, _dp), robot_v,
                                      robot_w, ctypes.byref(params or LPParams.default()),
                                      ctypes.byref(mpc or MPCParams.default()), _p(u, _dp), ctypes.byref(it))
    return u, up, st, it.value


def track_step(kind, path, goal, state, u_p=(0.0, 0.0), params=None, lqr=None, mpc=None):
    """One LQR.plan (kind "lqr") / MPC.plan ("mpc") iteration -> (status, new_state, new_u_p, u, admm_iters)."""
    path = _d(path).reshape(-1, 2)
    st = _d(state).copy()
    up = _d(u_p).copy()
    u = np.zeros(2)
    it = ctypes.c_int32(0)
    rc = _lp_lib().oracle_track_step(0 if kind == "lqr" else 1, _p(path, _dp), len(path), _p(_d(goal), _dp),
                                     _p(st, _dp), _p(up, _dp), ctypes.byref(params or LPParams.default()),
                                     ctypes.byref(lqr or LQRParams.default()), ctypes.byref(mpc or MPCParams.default()),
                                     _p(u, _dp), ctypes.byref(it))
    return rc, st, up, u, it.value


def track_batch(kind, path_xy, path_off, goals, states, u_p=None, iters=1, params=None, lqr=None, mpc=None,
                nthreads=0):
    """`iters` LQR/MPC plan iterations for each agent (OpenMP) -> (states, u_p, u, status, n_steps, total)."""
    xy = _d(path_xy).reshape(-1, 2)
    off = np.ascontiguousarray(path_off, np.int32)
    g = _d(goals).reshape(-1, 3)
    st = _d(states).reshape(-1, 5).copy()
    na = len(st)
    up = np.zeros((na, 2)) if u_p is None else _d(u_p).reshape(-1, 2).copy()
    u = np.zeros((na, 2))
    status = np.zeros(na, np.int32)
    nst = np.zeros(na, np.int32)
    tot = _lp_lib().oracle_track_batch(0 if kind == "lqr" else 1, _p(xy, _dp), _p(off, _i32p), _p(g, _dp), _p(st, _dp),
                                       _p(up, _dp), na, iters, ctypes.byref(params or LPParams.default()),
                                       ctypes.byref(lqr or LQRParams.default()), ctypes.byref(mpc or MPCParams.default()),
                                       _p(u, _dp), _p(status, _i32p), _p(nst, _i32p), nthreads)
    return st, up, u, status, nst, tot


def dwa_step_batch(obstacles, path_xy, path_off, goals, states, params=None, nv=64, nw=64, predict_time=3.0,
                   v_res=0.05, w_res=0.05, weights=(0.2, 0.1, 0.05), inflation=1.0, nthreads=0, grid=None):
    """OpenMP batch of one DWA.plan iteration per agent.  grid: optional uint8 [W, H] occupancy of the
    same obstacles -- the obstacle term is then taken over the cells within the inflation radius
    (identical values; the CPU form of the kernel's stencil) instead of the reference's loop over
    every obstacle."""
    L = _lp_lib()
    L.oracle_dwa_set_grid.restype = None
    L.oracle_dwa_set_grid.argtypes = [_u8p, ctypes.c_int, ctypes.c_int]
    if grid is not None:
        grid = np.ascontiguousarray(grid, dtype=np.uint8)
        L.oracle_dwa_set_grid(_p(grid, _u8p), grid.shape[0], grid.shape[1])
    try:
        return _dwa_step_batch(L, obstacles, path_xy, path_off, goals, states, params, nv, nw, predict_time,
                               v_res, w_res, weights, inflation, nthreads)
    finally:
        if grid is not None:
            L.oracle_dwa_set_grid(None, 0, 0)


def _dwa_step_batch(L, obstacles, path_xy, path_off, goals, states, params, nv, nw, predict_time, v_res, w_res,
                    weights, inflation, nthreads):
    if not getattr(L, "_dwab", False):
        L.oracle_dwa_step_batch.restype = ctypes.c_int
        L.oracle_dwa_step_batch.argtypes = [_dp, ctypes.c_int, _dp, _i32p, _dp, _dp, ctypes.c_int,
                                            ctypes.POINTER(LPParams), ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_double, _dp, _i32p, ctypes.c_int]
        L._dwab = True
    obs = _d(obstacles).reshape(-1, 2)
    xy = _d(path_xy).reshape(-1, 2)
    off = np.ascontiguousarray(path_off, np.int32)
    g = _d(goals).reshape(-1, 3)
    st = _d(states).reshape(-1, 5).copy()
    na = len(st)
    u = np.zeros((na, 2))
    status = np.zeros(na, np.int32)
    L.oracle_dwa_step_batch(_p(obs, _dp), len(obs), _p(xy, _dp), _p(off, _i32p), _p(g, _dp), _p(st, _dp), na,
                            ctypes.byref(params or LPParams.default()), v_res, w_res, nv, nw, predict_time,
                            weights[0], weights[1], weights[2], inflation, _p(u, _dp), _p(status, _i32p),
                            int(nthreads))
    return st, u, status


# ------------------------------------------------------------------------------------------------
# sample search (RRT / RRT*)
def _rrt_bind():
    L = lib()
    if not getattr(L, "_rrt_bound", False):
        L.oracle_rrt.restype = ctypes.c_int
        L.oracle_rrt.argtypes = [ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, _dp, ctypes.c_int64, _dp, ctypes.c_int, _i32p, _i64p]
        L.oracle_rrt_batch.restype = ctypes.c_int
        L.oracle_rrt_batch.argtypes = [ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp, _dp, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp,
                                       ctypes.c_int64, _dp, ctypes.c_int, _i32p, _i32p, ctypes.c_int]
        L.oracle_map_collision.restype = ctypes.c_int
        L.oracle_map_collision.argtypes = [_dp, ctypes.c_int, _dp, ctypes.c_int, _dp, ctypes.c_int, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L._rrt_bound = True
    return L


def _map_arrays(rects, circs, X, Y, boundary=None):
    if boundary is None:
        boundary = [[0, 0, 1, Y], [0, Y, X, 1], [1, 0, X, 1], [X, 1, 1, Y]]
    r = _d(np.asarray(rects, np.float64).reshape(-1, 4))
    c = _d(np.asarray(circs, np.float64).reshape(-1, 3))
    b = _d(np.asarray(boundary, np.float64).reshape(-1, 4))
    return r, c, b


def map_collision(rects, circs, X, Y, p1, p2, delta=0.5):
    r, c, b = _map_arrays(rects, circs, X, Y)
    return bool(_rrt_bind().oracle_map_collision(_p(r, _dp), len(r), _p(c, _dp), len(c), _p(b, _dp), len(b), delta,
                                                 p1[0], p1[1], p2[0], p2[1]))


def rrt(star, rects, circs, X, Y, start, goal, rnd, sample_num=10000, max_dist=0.5, radius=10.0, goal_rate=0.05,
        delta=0.5, cap=None):
    """RRT / RRT* plan (rrt.py:49-83, rrt_star.py:43-76) on a Map, consuming the double stream
    `rnd` -> dict(status, tree [n,4] (x, y, g, parent), draws)."""
    r, c, b = _map_arrays(rects, circs, X, Y)
    rnd = _d(rnd)
    cap = cap or sample_num + 2
    tree = np.zeros((cap, 4))
    nn = ctypes.c_int32(0)
    dr = ctypes.c_int64(0)
    st = _rrt_bind().oracle_rrt(int(bool(star)), _p(r, _dp), len(r), _p(c, _dp), len(c), _p(b, _dp), len(b), delta,
                                X, Y, start[0], start[1], goal[0], goal[1], sample_num, max_dist, radius, goal_rate,
                                _p(rnd, _dp), len(rnd), _p(tree, _dp), cap, ctypes.byref(nn), ctypes.byref(dr))
    return dict(status=st, tree=tree[: nn.value].copy(), draws=dr.value)


def rrt_batch(star, rects, circs, X, Y, starts, goals, rnd, sample_num, max_dist=0.5, radius=10.0, goal_rate=0.05,
              delta=0.5, cap=None, nthreads=0):
    """Independent RRT(*) queries with OpenMP; rnd [nq, stride] streams."""
    r, c, b = _map_arrays(rects, circs, X, Y)
    rnd = _d(rnd)
    nq, stride = rnd.shape
    cap = cap or sample_num + 2
    tree = np.zeros((nq, cap, 4))
    nn = np.zeros(nq, np.int32)
    st = np.zeros(nq, np.int32)
    s = _d(np.asarray(starts, np.float64).reshape(-1, 2))
    g = _d(np.asarray(goals, np.float64).reshape(-1, 2))
    _rrt_bind().oracle_rrt_batch(int(bool(star)), _p(r, _dp), len(r), _p(c, _dp), len(c), _p(b, _dp), len(b), delta,
                                 X, Y, _p(s, _dp), _p(g, _dp), nq, sample_num, max_dist, radius, goal_rate,
                                 _p(rnd, _dp), stride, _p(tree, _dp), cap, _p(nn, _i32p), _p(st, _i32p), nthreads)
    return dict(status=st, n_nodes=nn, tree=tree)


def astar3d_batch(occ, starts, goals, heuristic: str = "euclidean", nthreads: int = 0, algo: str = "astar"):
    """AStar3D (or Dijkstra3D / GBFS3D) over per-query grids occ [nq, X, Y, Z] with OpenMP
    -> (cost [nq], status [nq])."""
    L = lib()
    if not getattr(L, "_a3b", False):
        L.oracle_graph3d_batch.restype = ctypes.c_int
        L.oracle_graph3d_batch.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           _i32p, _i32p, ctypes.c_int, _dp, _i32p, ctypes.c_int]
        L._a3b = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    nq, X, Y, Z = occ.shape
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 3)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 3)
    cost = np.zeros(nq)
    st = np.zeros(nq, np.int32)
    L.oracle_graph3d_batch(ALGOS[algo], _p(occ, _u8p), X, Y, Z, 1 if heuristic == "manhattan" else 0, _p(s, _i32p),
                           _p(g, _i32p), nq, _p(cost, _dp), _p(st, _i32p), nthreads)
    return cost, st


def theta3d(occ: np.ndarray, start, goal, lazy: bool = False, heuristic: str = "euclidean",
            with_expand: bool = True):
    """Restatement of ThetaStar3D.plan (theta_star3d.py:38-94) or, with lazy, LazyThetaStar3D.plan
    (lazy_theta_star3d.py:41-112).  occ: uint8 [X, Y, Z].  Path start -> goal."""
    L = lib()
    if not getattr(L, "_th3", False):
        L.oracle_theta3d.restype = ctypes.c_int
        L.oracle_theta3d.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     _i32p, _i32p, _dp, _i32p, ctypes.c_int, _i32p, _i32p, ctypes.c_int, _i32p, _i64p]
        L._th3 = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    X, Y, Z = occ.shape
    n = X * Y * Z
    path = np.zeros(n + 1, np.int32)
    expand = np.zeros(n, np.int32)
    s = np.asarray(start, np.int32)
    g = np.asarray(goal, np.int32)
    cost = ctypes.c_double(0)
    plen = ctypes.c_int32(0)
    nexp = ctypes.c_int32(0)
    ctr = np.zeros(4, np.int64)
    st = L.oracle_theta3d(int(bool(lazy)), _p(occ, _u8p), X, Y, Z, 1 if heuristic == "manhattan" else 0,
                          _p(s, _i32p), _p(g, _i32p), ctypes.byref(cost), _p(path, _i32p), n + 1, ctypes.byref(plen),
                          _p(expand, _i32p) if with_expand else None, n, ctypes.byref(nexp), _p(ctr, _i64p))
    out = dict(status=st, cost=cost.value, n_expanded=nexp.value, path_cells=path[: plen.value].copy(),
               n_push=int(ctr[0]), n_pop=int(ctr[1]), n_iter=int(ctr[2]), max_heap=int(ctr[3]))
    if with_expand:
        out["expand_cells"] = expand[: nexp.value].copy()
    return out


def lpastar2d(occ: np.ndarray, start, goal, heuristic: str = "euclidean", lite: bool = False):
    """Restatement of LPAStar.plan (lpa_star.py:78-87, computeShortestPath :139-160, extractPath
    :209-230) with the reference's list semantics for U; lite=True restates DStarLite.plan
    (d_star_lite.py:14-187).  Path start -> goal.  status 4 = the reference raises (ValueError from
    min() of an empty U / neighbour list, or KeyError)."""
    L = lib()
    if not getattr(L, "_lpa_set", False):
        for fn in (L.oracle_lpastar2d, L.oracle_dstarlite2d):
            fn.restype = ctypes.c_int
            fn.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, _dp, _i32p, ctypes.c_int, _i32p, _i64p]
        L._lpa_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    path = np.zeros(1002, np.int32)
    cost = ctypes.c_double(0)
    plen = ctypes.c_int32(0)
    ctr = np.zeros(4, np.int64)
    st = (L.oracle_dstarlite2d if lite else L.oracle_lpastar2d)(_p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0, int(start[0]), int(start[1]),
                            int(goal[0]), int(goal[1]), ctypes.byref(cost), _p(path, _i32p), 1002, ctypes.byref(plen),
                            _p(ctr, _i64p))
    cells = path[: plen.value]
    return dict(status=st, cost=cost.value, path=[(int(c) // H, int(c) % H) for c in cells], path_cells=cells.copy(),
                n_push=int(ctr[0]), n_expanded=int(ctr[1]), steps=int(ctr[2]), max_u=int(ctr[3]))


def lpastar2d_replan(occ: np.ndarray, start, goal, toggles, heuristic: str = "euclidean", lite: bool = False):
    """LPAStar.plan() then one LPAStar.OnPress edit (lpa_star.py:101-137) per toggle cell, each
    followed by plan() on the kept state; lite=True: DStarLite.plan() then DStarLite.OnPress
    (d_star_lite.py:61-97: walk, km, edit, computeShortestPath, walk on) per toggle.  Returns per-plan cost / n_expanded / status arrays
    (status -1 = not run because an earlier plan raised) and the last plan's path."""
    L = lib()
    if not getattr(L, "_lpar_set", False):
        L.oracle_lpastar2d_replan.restype = ctypes.c_int
        L.oracle_lpastar2d_replan.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, ctypes.c_int, _dp,
                                              _i32p, _i32p, _i32p, ctypes.c_int, _i32p, _i64p]
        L._lpar_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    t = np.ascontiguousarray(toggles, np.int32).reshape(-1, 2)
    nt = len(t)
    cost = np.zeros(nt + 1)
    nexp = np.zeros(nt + 1, np.int32)
    st = np.zeros(nt + 1, np.int32)
    path = np.zeros(1002, np.int32)
    plen = ctypes.c_int32(0)
    ctr = np.zeros(4, np.int64)
    L.oracle_lpastar2d_replan(int(bool(lite)), _p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0, int(start[0]), int(start[1]),
                              int(goal[0]), int(goal[1]), _p(t, _i32p), nt, _p(cost, _dp), _p(nexp, _i32p),
                              _p(st, _i32p), _p(path, _i32p), 1002, ctypes.byref(plen), _p(ctr, _i64p))
    return dict(cost=cost, n_expanded=nexp, status=st, path_cells=path[: plen.value].copy())


def lpastar2d_batch(occ: np.ndarray, starts, goals, heuristic: str = "euclidean", lite: bool = False,
                    nthreads: int = 0):
    """OpenMP batch of the LPAStar.plan (or, lite, DStarLite.plan) restatement: cost, status, n_expanded."""
    L = lib()
    if not getattr(L, "_lpab_set", False):
        L.oracle_lpastar2d_batch.restype = None
        L.oracle_lpastar2d_batch.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p,
                                             _i32p, ctypes.c_int, _dp, _i32p, _i32p, ctypes.c_int]
        L._lpab_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 2)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 2)
    nq = len(s)
    out = dict(cost=np.zeros(nq), status=np.zeros(nq, np.int32), n_expanded=np.zeros(nq, np.int32))
    L.oracle_lpastar2d_batch(int(bool(lite)), _p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0, _p(s, _i32p),
                             _p(g, _i32p), nq, _p(out["cost"], _dp), _p(out["status"], _i32p),
                             _p(out["n_expanded"], _i32p), int(nthreads))
    return out


def lpastar2d_replan_batch(occ: np.ndarray, starts, goals, toggles, heuristic: str = "euclidean", lite: bool = False,
                           nthreads: int = 0):
    """OpenMP batch of lpastar2d_replan: toggles [nq, nt, 2]; returns cost / n_expanded / status [nq, nt + 1]."""
    L = lib()
    if not getattr(L, "_lparb_set", False):
        L.oracle_lpastar2d_replan_batch.restype = None
        L.oracle_lpastar2d_replan_batch.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    _i32p, _i32p, ctypes.c_int, _i32p, ctypes.c_int, _dp, _i32p,
                                                    _i32p, ctypes.c_int]
        L._lparb_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 2)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 2)
    nq = len(s)
    t = np.ascontiguousarray(toggles, np.int32).reshape(nq, -1, 2)
    nt = t.shape[1]
    out = dict(cost=np.zeros((nq, nt + 1)), n_expanded=np.zeros((nq, nt + 1), np.int32),
               status=np.zeros((nq, nt + 1), np.int32))
    L.oracle_lpastar2d_replan_batch(int(bool(lite)), _p(occ, _u8p), W, H, 1 if heuristic == "manhattan" else 0,
                                    _p(s, _i32p), _p(g, _i32p), nq, _p(t, _i32p), nt, _p(out["cost"], _dp),
                                    _p(out["n_expanded"], _i32p), _p(out["status"], _i32p), int(nthreads))
    return out


def dstar3d(occ: np.ndarray, start, goal, blocks=None, path_cap: int = 0, max_process: int = 0):
    """Restatement of DStar3D.plan (d_star3d.py:100-109) followed by one apply_dynamic_obstacles
    (:115-149) per entry of blocks [nrounds][nblk][3] (voxels outside the grid are ignored).
    Returns per round (0 = plan): cost, status (0 reached the goal, 1 stopped at a parentless node,
    3 cap), n_process (len(EXPAND)), path (voxel ids x*Y*Z + y*Z + z, start -> goal)."""
    L = lib()
    if not getattr(L, "_d3_set", False):
        L.oracle_dstar3d.restype = ctypes.c_int
        L.oracle_dstar3d.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p, _i32p, ctypes.c_int,
                                     ctypes.c_int, _dp, _i32p, _i64p, _i32p, ctypes.c_int, _i32p, ctypes.c_int64]
        L._d3_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    X, Y, Z = occ.shape
    b = np.zeros((0, 0, 3), np.int32) if blocks is None else np.ascontiguousarray(blocks, np.int32)
    nr, nb = (b.shape[0], b.shape[1]) if b.size else (len(b), 0)
    path_cap = path_cap or X * Y * Z + 1
    s = np.ascontiguousarray(start, np.int32)
    g = np.ascontiguousarray(goal, np.int32)
    cost = np.zeros(nr + 1)
    st = np.zeros(nr + 1, np.int32)
    npr = np.zeros(nr + 1, np.int64)
    path = np.zeros((nr + 1, path_cap), np.int32)
    plen = np.zeros(nr + 1, np.int32)
    rc = L.oracle_dstar3d(_p(occ, _u8p), X, Y, Z, _p(s, _i32p), _p(g, _i32p), _p(b, _i32p) if b.size else None, nr, nb,
                          _p(cost, _dp), _p(st, _i32p), _p(npr, _i64p), _p(path, _i32p), path_cap, _p(plen, _i32p),
                          int(max_process))
    return dict(rc=rc, cost=cost, status=st, n_process=npr,
                paths=[path[r, : min(plen[r], path_cap)].copy() for r in range(nr + 1)], path_len=plen)


def dstar2d_onpress(occ: np.ndarray, start, goal, presses, path_cap: int = 0, max_process: int = 0):
    """Restatement of DStar.plan followed by one OnPress per press (x, y) (d_star.py:75-134).
    Returns per call (0 = plan): cost, status (include/pmp.h pmp_dstar2d_onpress_batch), n_process
    (len(EXPAND)), paths (cells x*H + y; plan: start -> goal, presses: the walk without the goal)."""
    L = lib()
    if not getattr(L, "_d2p_set", False):
        L.oracle_dstar2d_onpress.restype = ctypes.c_int
        L.oracle_dstar2d_onpress.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, _i32p, ctypes.c_int, _dp, _i32p, ctypes.c_int, _i32p, _i64p,
                                             _i32p, ctypes.c_int64]
        L._d2p_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    W, H = occ.shape
    pr = np.ascontiguousarray(presses, np.int32).reshape(-1, 2)
    n = len(pr)
    path_cap = path_cap or 4 * W * H + 8
    cost = np.zeros(n + 1)
    st = np.zeros(n + 1, np.int32)
    npr = np.zeros(n + 1, np.int64)
    plen = np.zeros(n + 1, np.int32)
    path = np.zeros((n + 1, path_cap), np.int32)
    L.oracle_dstar2d_onpress(_p(occ, _u8p), W, H, int(start[0]), int(start[1]), int(goal[0]), int(goal[1]),
                             _p(pr, _i32p), n, _p(cost, _dp), _p(path, _i32p), path_cap, _p(plen, _i32p), _p(npr, _i64p),
                             _p(st, _i32p), int(max_process))
    return dict(cost=cost, status=st, n_process=npr, path_len=plen, first=path[:, 0].copy(),
                paths=[path[r, : max(0, min(plen[r], path_cap))].copy() for r in range(n + 1)])


def lpastar3d(occ: np.ndarray, start, goal, changes=None, heuristic: str = "euclidean", path_cap: int = 0,
              max_exp: int = 0):
    """Restatement of LPAStar3D.plan (lpa_star3d.py:78-82) followed by one apply_change per row of
    changes [nr][4] = (x, y, z, mode) (mode 0 toggle = blocked None, 1 block, 2 free; :93-124).
    Returns per call (0 = plan): cost, status (0 path, 1 empty path, 2 overflow, 3 cap, -1 not run),
    n_expanded (len(EXPAND)), paths (voxel ids, start -> goal)."""
    L = lib()
    if not getattr(L, "_l3_set", False):
        L.oracle_lpastar3d.restype = ctypes.c_int
        L.oracle_lpastar3d.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p,
                                       _i32p, ctypes.c_int, _dp, _i32p, _i64p, _i32p, ctypes.c_int, _i32p,
                                       ctypes.c_int64]
        L._l3_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    X, Y, Z = occ.shape
    ch = np.zeros((0, 4), np.int32) if changes is None else np.ascontiguousarray(changes, np.int32).reshape(-1, 4)
    nr = len(ch)
    path_cap = path_cap or X * Y * Z + 1
    cost = np.zeros(nr + 1)
    st = np.zeros(nr + 1, np.int32)
    ne = np.zeros(nr + 1, np.int64)
    plen = np.zeros(nr + 1, np.int32)
    path = np.zeros((nr + 1, path_cap), np.int32)
    L.oracle_lpastar3d(_p(occ, _u8p), X, Y, Z, 1 if heuristic == "manhattan" else 0,
                       _p(np.ascontiguousarray(start, np.int32), _i32p), _p(np.ascontiguousarray(goal, np.int32), _i32p),
                       _p(ch, _i32p) if nr else None, nr, _p(cost, _dp), _p(st, _i32p), _p(ne, _i64p), _p(path, _i32p),
                       path_cap, _p(plen, _i32p), int(max_exp))
    return dict(cost=cost, status=st, n_expanded=ne, path_len=plen,
                paths=[path[r, : min(plen[r], path_cap)].copy() for r in range(nr + 1)])


def graph3d_dynamic_batch(kind: str, occ, starts, goals, rounds=None, heuristic: str = "euclidean", nthreads: int = 0):
    """OpenMP batch of the DStar3D (kind "dstar3d", rounds = blocks [nq, nr, nblk, 3]) or LPAStar3D
    (kind "lpastar3d", rounds = changes [nq, nr, 4]) restatement over per-query [nq, X, Y, Z] or
    shared [X, Y, Z] grids.  Returns cost / status / n [nq, nr + 1] (n = len(EXPAND))."""
    L = lib()
    if not getattr(L, "_g3db_set", False):
        L.oracle_dstar3d_batch.restype = None
        L.oracle_dstar3d_batch.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p,
                                           ctypes.c_int, _i32p, ctypes.c_int, ctypes.c_int, _dp, _i32p, _i64p,
                                           ctypes.c_int]
        L.oracle_lpastar3d_batch.restype = None
        L.oracle_lpastar3d_batch.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, _i32p, _i32p, ctypes.c_int, _i32p, ctypes.c_int, _dp, _i32p,
                                             _i64p, ctypes.c_int]
        L._g3db_set = True
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    per_query = occ.ndim == 4
    X, Y, Z = occ.shape[-3:]
    s = np.ascontiguousarray(starts, np.int32).reshape(-1, 3)
    g = np.ascontiguousarray(goals, np.int32).reshape(-1, 3)
    nq = len(s)
    rd = None if rounds is None else np.ascontiguousarray(rounds, np.int32)
    nr = 0 if rd is None else rd.shape[1]
    out = dict(cost=np.zeros((nq, nr + 1)), status=np.zeros((nq, nr + 1), np.int32), n=np.zeros((nq, nr + 1), np.int64))
    if kind == "dstar3d":
        nb = 0 if rd is None else rd.shape[2]
        L.oracle_dstar3d_batch(_p(occ, _u8p), int(per_query), X, Y, Z, _p(s, _i32p), _p(g, _i32p), nq,
                               _p(rd, _i32p) if rd is not None else None, nr, nb, _p(out["cost"], _dp),
                               _p(out["status"], _i32p), _p(out["n"], _i64p), int(nthreads))
    else:
        L.oracle_lpastar3d_batch(_p(occ, _u8p), int(per_query), X, Y, Z, 1 if heuristic == "manhattan" else 0,
                                 _p(s, _i32p), _p(g, _i32p), nq, _p(rd, _i32p) if rd is not None else None, nr,
                                 _p(out["cost"], _dp), _p(out["status"], _i32p), _p(out["n"], _i64p), int(nthreads))
    return out


class TotpParams(ctypes.Structure):
    """totp_params_t: TrajectoryConstraints (trajectory_base.py) + path_resolution"""
    _fields_ = [("vmax", ctypes.c_double * 3), ("amax", ctypes.c_double * 3), ("tstep", ctypes.c_double),
                ("res", ctypes.c_double)]

    @classmethod
    def make(cls, vmax=(2.0, 2.0, 2.0), amax=(1.0, 1.0, 1.0), tstep=0.01, res=0.01):
        return cls((ctypes.c_double * 3)(*vmax), (ctypes.c_double * 3)(*amax), tstep, res)


def totp3d_batch(paths, params: TotpParams, sample_cap: int = 0, point_cap: int = 0, nthreads: int = 0):
    """TimeOptimalTrajectory3D(path, constraints, path_resolution).generate() for every path
    (time_optimal_trajectory.py:8-353) with OpenMP over paths.  Caps of 0 size the buffers from a
    first pass.  Returns profiles [nq, sample_cap] + n_samples, points [nq, point_cap, 12] (time,
    position, velocity, acceleration, yaw, yaw rate; NaN = None) + n_points, total_time, status."""
    L = lib()
    if not getattr(L, "_totp", False):
        L.oracle_totp3d_batch.restype = ctypes.c_int
        L.oracle_totp3d_batch.argtypes = [_dp, _i64p, ctypes.c_int, ctypes.POINTER(TotpParams), ctypes.c_int, _dp, _dp,
                                          _dp, _dp, _i32p, ctypes.c_int, _dp, _i32p, _dp, _i32p, ctypes.c_int]
        L._totp = True
    flat = np.ascontiguousarray(np.concatenate([np.asarray(p, np.float64).reshape(-1, 3) for p in paths]))
    off = np.zeros(len(paths) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p in paths])
    nq = len(paths)

    def run(sc, pc):
        out = dict(s_values=np.zeros((nq, sc)), s_dot=np.zeros((nq, sc)), s_ddot=np.zeros((nq, sc)),
                   time=np.zeros((nq, sc)), n_samples=np.zeros(nq, np.int32), points=np.zeros((nq, pc, 12)),
                   n_points=np.zeros(nq, np.int32), total_time=np.zeros(nq), status=np.zeros(nq, np.int32))
        L.oracle_totp3d_batch(_p(flat, _dp), _p(off, _i64p), nq, ctypes.byref(params), sc, _p(out["s_values"], _dp),
                              _p(out["s_dot"], _dp), _p(out["s_ddot"], _dp), _p(out["time"], _dp),
                              _p(out["n_samples"], _i32p), pc, _p(out["points"], _dp), _p(out["n_points"], _i32p),
                              _p(out["total_time"], _dp), _p(out["status"], _i32p), nthreads)
        return out

    if sample_cap <= 0 or point_cap <= 0:
        first = run(1, 1)
        sample_cap = sample_cap if sample_cap > 0 else max(1, int(first["n_samples"].max()))
        point_cap = point_cap if point_cap > 0 else max(1, int(first["n_points"].max()))
    return run(sample_cap, point_cap)
