"""ctypes binding of libpmp_hip.so (C-ABI declared in include/pmp.h).

The product path has no CPU fallback: if the HIP library or a HIP device is missing, every
planning call raises.  PyTorch is used only for device memory and the current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PMP_HIP_LIB") or os.path.join(_HERE, "libpmp_hip.so")  # override: diagnostics only

_vp = ctypes.c_void_p
_i = ctypes.c_int

# name -> (restype, argtypes); pointers are passed as raw device addresses (c_void_p)
SIGNATURES = {
    "pmp_create": (_vp, [_i]),
    "pmp_destroy": (None, [_vp]),
    "pmp_last_error": (ctypes.c_char_p, [_vp]),
    "pmp_version": (ctypes.c_char_p, []),
    "pmp_astar2d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _i,
                               _vp, _vp]),
    "pmp_graph2d_batch": (_i, [_vp, _vp, _i, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _i,
                               _vp, _vp]),
    "pmp_graph3d_batch": (_i, [_vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp,
                               _i, _vp, _vp]),
    "pmp_astar2d_reserve": (_i, [_vp, _i, _i, _i, _i]),
    "pmp_astar2d_geometry": (_i, [_vp, _vp]),
    "pmp_astar2d_reserve_auto": (_i, [_vp]),
    "pmp_set_timing": (_i, [_vp, _vp]),
    "pmp_wall_clock_khz": (_i, [_vp, _vp]),
    "pmp_set_stats": (_i, [_vp, _vp]),
    "pmp_dwa_set_split": (_i, [_vp, _i]),
    "pmp_astar2d_sq_cap": (_i, [_i, _i]),
    "pmp_astar2d_set_schedule": (_i, [_vp, _i]),
    "pmp_astar2d_set_priority": (_i, [_vp, _i]),
    "pmp_astar2d_set_residency": (_i, [_vp, _i]),
    "pmp_astar2d_set_engine": (_i, [_vp, _i, _i]),
    "pmp_set_resident_per_cu": (_i, [_vp, _i]),
    "pmp_set_workers_per_cu": (_i, [_vp, _i]),
    "pmp_dstar_set_first_cap": (_i, [_vp, _i]),
    "pmp_astar3d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _i,
                               _vp, _vp]),
    "pmp_dwa_step_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp]),
    "pmp_lqr_control_batch": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "pmp_mpc_control_batch": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp]),
    "pmp_dstar2d_batch": (_i, [_vp, _vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, ctypes.c_int64]),
    "pmp_dstar2d_onpress_batch": (_i, [_vp, _vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp,
                                       ctypes.c_int64]),
    "pmp_dstar3d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _vp, _vp,
                               _vp, _i, ctypes.c_int64]),
    "pmp_lpastar3d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _i, _vp,
                                 _vp, _vp, ctypes.c_int64]),
    "pmp_lpastar2d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "pmp_dstarlite2d_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "pmp_lpastar2d_replan_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i,
                                        _vp]),
    "pmp_dstarlite2d_replan_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i,
                                          _vp]),
    "pmp_rrt_batch": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _i, _vp, _i, _vp, _vp, _i, _vp, ctypes.c_int64, _i, _vp, _vp,
                           _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "pmp_track_step_batch": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp,
                                  _vp]),
    "pmp_totp3d_batch": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp,
                              _vp, _i]),
}


class LPParams(ctypes.Structure):
    """pmp_lp_params == LocalPlanner.params (local_planner/local_planner.py:39-55)."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "dt", "lookahead_time", "max_lookahead", "min_lookahead", "max_v_inc", "min_v_inc", "max_v", "min_v",
        "max_w_inc", "min_w_inc", "max_w", "min_w", "goal_dist_tol", "rotate_tol")]

    @classmethod
    def from_params(cls, p: dict):
        return cls(p["TIME_STEP"], p["LOOKAHEAD_TIME"], p["MAX_LOOKAHEAD_DIST"], p["MIN_LOOKAHEAD_DIST"],
                   p["MAX_V_INC"], p["MIN_V_INC"], p["MAX_V"], p["MIN_V"], p["MAX_W_INC"], p["MIN_W_INC"],
                   p["MAX_W"], p["MIN_W"], p["GOAL_DIST_TOL"], p["ROTATE_TOL"])


class DWAParams(ctypes.Structure):
    """pmp_dwa_params == the DWA constructor's parameters (local_planner/dwa.py:45-56)."""
    _fields_ = [("heading_weight", ctypes.c_double), ("obstacle_weight", ctypes.c_double),
                ("velocity_weight", ctypes.c_double), ("predict_time", ctypes.c_double),
                ("inflation", ctypes.c_double), ("v_resolution", ctypes.c_double),
                ("w_resolution", ctypes.c_double), ("nv", ctypes.c_int32), ("nw", ctypes.c_int32)]

class LQRParams(ctypes.Structure):
    """pmp_lqr_params == LQR's Q, R, lqr_iteration, eps_iter (local_planner/lqr.py:35-38)."""
    _fields_ = [("q", ctypes.c_double * 3), ("r", ctypes.c_double * 2), ("iters", ctypes.c_int32),
                ("eps", ctypes.c_double)]

    @classmethod
    def make(cls, q=(1.0, 1.0, 1.0), r=(1.0, 1.0), iters: int = 100, eps: float = 0.1):
        return cls((ctypes.c_double * 3)(*[float(v) for v in q]), (ctypes.c_double * 2)(*[float(v) for v in r]),
                   int(iters), float(eps))


# ADMM settings of the MPC QP solve.  OSQP's defaults (OSQP is what mpc.py:196-203 calls) stop at
# eps 1e-3; the drop-in solves to 1e-9 by default so results do not depend on solver internals.
OSQP_DEFAULTS = dict(rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, adaptive_tol=5.0, max_iter=4000,
                     check_every=25, adaptive_every=25)
ADMM_DEFAULTS = dict(OSQP_DEFAULTS, eps_abs=1e-9, eps_rel=1e-9)


class MPCParams(ctypes.Structure):
    """pmp_mpc_params == MPC's p, m, Q, R (local_planner/mpc.py:37-40) + the ADMM settings."""
    _fields_ = [("p", ctypes.c_int32), ("m", ctypes.c_int32), ("q", ctypes.c_double * 3), ("r", ctypes.c_double * 2),
                ("rho", ctypes.c_double), ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double), ("adaptive_tol", ctypes.c_double),
                ("max_iter", ctypes.c_int32), ("check_every", ctypes.c_int32), ("adaptive_every", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]

    @classmethod
    def make(cls, p: int = 12, m: int = 8, q=(0.8, 0.8, 0.5), r=(2.0, 2.0), **admm):
        a = dict(ADMM_DEFAULTS)
        a.update(admm)
        return cls(int(p), int(m), (ctypes.c_double * 3)(*[float(v) for v in q]),
                   (ctypes.c_double * 2)(*[float(v) for v in r]), a["rho"], a["sigma"], a["alpha"], a["eps_abs"],
                   a["eps_rel"], a["adaptive_tol"], int(a["max_iter"]), int(a["check_every"]),
                   int(a["adaptive_every"]), 0)


class RRTParams(ctypes.Structure):
    """pmp_rrt_params == Map size, delta (sample_search.py:22), RRT kwargs (rrt.py:36-44), RRT* r."""
    _fields_ = [("x_range", ctypes.c_double), ("y_range", ctypes.c_double), ("delta", ctypes.c_double),
                ("max_dist", ctypes.c_double), ("radius", ctypes.c_double), ("goal_sample_rate", ctypes.c_double),
                ("sample_num", ctypes.c_int32), ("star", ctypes.c_int32)]


class TotpParams(ctypes.Structure):
    """pmp_totp_params == TrajectoryConstraints (trajectory/trajectory_base.py:30-45) max_velocity,
    max_acceleration, min_time_step + TimeOptimalTrajectory3D's path_resolution."""
    _fields_ = [("max_velocity", ctypes.c_double * 3), ("max_acceleration", ctypes.c_double * 3),
                ("min_time_step", ctypes.c_double), ("path_resolution", ctypes.c_double)]

    @classmethod
    def make(cls, max_velocity=(2.0, 2.0, 2.0), max_acceleration=(1.0, 1.0, 1.0), min_time_step: float = 0.01,
             path_resolution: float = 0.01):
        return cls((ctypes.c_double * 3)(*[float(v) for v in max_velocity]),
                   (ctypes.c_double * 3)(*[float(v) for v in max_acceleration]), float(min_time_step),
                   float(path_resolution))


TRACK_LQR, TRACK_MPC = 0, 1

STATUS_FOUND, STATUS_NO_PATH, STATUS_PATH_OVERFLOW, STATUS_CAP_OVERFLOW, STATUS_REF_RAISES = range(5)


class PMPError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()
_ctx = {}


# planners sharing the AStar loop (include/pmp.h PMP_ALGO_*)
ALGO_ASTAR, ALGO_DIJKSTRA, ALGO_GBFS, ALGO_THETA, ALGO_LAZY_THETA = 0, 1, 2, 3, 4
ALGOS = {"astar": ALGO_ASTAR, "dijkstra": ALGO_DIJKSTRA, "gbfs": ALGO_GBFS, "theta_star": ALGO_THETA,
         "lazy_theta_star": ALGO_LAZY_THETA}


def load_library(path: str = LIB_PATH):
    """Load libpmp_hip.so and bind every C-ABI symbol.  Works without a GPU (no HIP call)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise PMPError(f"{path} is missing: build it with `make -C {_HERE}/csrc` "
                               "(python_motion_planning_amd has no CPU fallback)")
            L = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def device_check():
    import torch

    if not torch.cuda.is_available():
        raise PMPError("python_motion_planning_amd needs a HIP device (MI355X); none is visible")
    return torch


def context(device: int | None = None):
    """Per-(thread, device, current stream) pmp_ctx.  A context's scratch (work queue, per-worker
    state) belongs to the launches of one stream: keyed by the stream too, launches the caller puts
    on different torch streams never share scratch, and every batch call allocates its tensors and
    launches on the same current stream, so the caching allocator orders their reuse."""
    torch = device_check()
    L = load_library()
    dev = torch.cuda.current_device() if device is None else int(device)
    key = (threading.get_ident(), dev, torch.cuda.current_stream(dev).cuda_stream)
    c = _ctx.get(key)
    if c is None:
        c = L.pmp_create(dev)
        if not c:
            raise PMPError(f"pmp_create({dev}) failed")
        _ctx[key] = c
    return c


def check(ctx, rc: int, what: str):
    if rc != 0:
        msg = load_library().pmp_last_error(ctx)
        raise PMPError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def stream_ptr():
    import torch

    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()
