"""Local planners: drop-in Robot / LocalPlanner / DWA (local_planner/ and utils/agent/ of the reference).

plan() keeps the reference's return conventions; the per-iteration control step runs in the
gfx950 kernels (dwa.hip).  step() is one iteration of the reference's plan loop; plan_batch()
runs many independent agents at once.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib, batch
from .env import Env
from .factory import SearchFactory
from .planner import Planner


class Robot:
    """utils/agent/agent.py:37-134 -- unicycle state [x, y, theta, v, w] + pose history."""

    def __init__(self, px, py, theta, v, w) -> None:
        self.px, self.py, self.theta = px, py, theta
        self.v, self.w = v, w
        self.history_pose = []
        self.parameters = None

    def __str__(self) -> str:
        return "Robot"

    @property
    def position(self):
        return (self.px, self.py)

    @property
    def state(self):
        return np.array([[self.px], [self.py], [self.theta], [self.v], [self.w]])

    def reset(self) -> None:
        self.v = 0
        self.w = 0
        self.history_pose = []


class LocalPlanner(Planner):
    """local_planner/local_planner.py:12-261 (parameters, global path, goal test)."""

    DEFAULTS = dict(TIME_STEP=0.1, MAX_ITERATION=1500, LOOKAHEAD_TIME=1.0, MAX_LOOKAHEAD_DIST=2.5,
                    MIN_LOOKAHEAD_DIST=1.0, MAX_V_INC=1.0, MIN_V_INC=-1.0, MAX_V=0.5, MIN_V=0.0,
                    MAX_W_INC=math.pi, MIN_W_INC=-math.pi, MAX_W=math.pi / 2, MIN_W=-math.pi / 2,
                    GOAL_DIST_TOL=0.5, ROTATE_TOL=0.5)

    def __init__(self, start: tuple, goal: tuple, env: Env, heuristic_type: str = "euclidean", **params) -> None:
        assert len(start) == 3 and len(goal) == 3, "Start and goal parameters must be (x, y, theta)"
        self.start, self.goal = start, goal
        self.heuristic_type = heuristic_type
        self.env = env
        self.obstacles = self.env.obstacles
        self.plot = None
        self.robot = Robot(start[0], start[1], start[2], 0, 0)
        self.params = {k: params.get(k, v) for k, v in self.DEFAULTS.items()}
        self.g_planner_ = None
        self.path = None
        self.search_factory_ = SearchFactory()

    @property
    def g_planner(self):
        return str(self.g_planner_)

    @g_planner.setter
    def g_planner(self, config):
        if "planner_name" in config:
            self.g_planner_ = self.search_factory_(**config)
        else:
            raise RuntimeError("Please set planner name!")

    @property
    def g_path(self):
        if self.g_planner_ is None:
            raise AttributeError("Global path searcher is None, please set it first!")
        cost, path, _ = self.g_planner_.plan()
        return path

    @property
    def lookahead_dist(self):
        p = self.params
        return min(max(abs(self.robot.v) * p["LOOKAHEAD_TIME"], p["MIN_LOOKAHEAD_DIST"]), p["MAX_LOOKAHEAD_DIST"])

    def dist(self, start: tuple, end: tuple) -> float:
        return math.hypot(end[0] - start[0], end[1] - start[1])

    def angle(self, start: tuple, end: tuple) -> float:
        return math.atan2(end[1] - start[1], end[0] - start[0])

    def regularizeAngle(self, angle: float):
        return angle - 2.0 * math.pi * math.floor((angle + math.pi) / (2.0 * math.pi))

    def reachGoal(self, cur: tuple, goal: tuple) -> bool:
        e_theta = self.regularizeAngle(cur[2] - goal[2])
        return not (self.dist((cur[0], cur[1]), (goal[0], goal[1])) > self.params["GOAL_DIST_TOL"]
                    or abs(e_theta) > self.params["ROTATE_TOL"])

    # ---- kernel plumbing --------------------------------------------------------------------------
    def _lp_params(self):
        return _lib.LPParams.from_params(self.params)

    def _grid(self):
        return batch.obstacle_grid(self.env.obstacles)


class DWA(LocalPlanner):
    """Dynamic Window Approach (local_planner/dwa.py:15-212) on the gfx950 kernel dwa.hip."""

    def __init__(self, start: tuple, goal: tuple, env: Env, heuristic_type: str = "euclidean",
                 heading_weight: float = 0.2, obstacle_weight: float = 0.1, velocity_weight: float = 0.05,
                 predict_time: float = 1.5, obstacle_inflation_radius: float = 1.0,
                 v_resolution: float = 0.05, w_resolution: float = 0.05, **params) -> None:
        super().__init__(start, goal, env, heuristic_type, **params)
        self.heading_weight = heading_weight
        self.obstacle_weight = obstacle_weight
        self.velocity_weight = velocity_weight
        self.predict_time = predict_time
        self.obstacle_inflation_radius = obstacle_inflation_radius
        self.v_resolution = v_resolution
        self.w_resolution = w_resolution
        self.g_planner = {"planner_name": "a_star", "start": (start[0], start[1]), "goal": (goal[0], goal[1]),
                          "env": env}
        self.path = self.g_path[::-1]

    def __str__(self) -> str:
        return "Dynamic Window Approach(DWA)"

    def _dwa_params(self, nv: int = 0, nw: int = 0):
        return _lib.DWAParams(self.heading_weight, self.obstacle_weight, self.velocity_weight, self.predict_time,
                              self.obstacle_inflation_radius, self.v_resolution, self.w_resolution, nv, nw)

    def _run(self, iters: int):
        torch = _lib.device_check()
        r = self.robot
        state = torch.tensor([[r.px, r.py, r.theta, r.v, r.w]], dtype=torch.float64, device="cuda")
        xy, off = batch.pack_paths([np.asarray(self.path, np.float64)])
        out = batch.dwa_step_batch(self._grid(), self._lp_params(), self._dwa_params(), state,
                                   np.array([self.goal], np.float64), xy, off, iters=iters, want_traj=True,
                                   want_hist=True)
        n = int(out["n_steps"][0])
        st = int(out["status"][0])
        hist = out["hist_pose"][0, :n].cpu().numpy()
        traj = out["best_traj"][0, :n].cpu().numpy()
        s = state[0].cpu().numpy()
        for p in hist:
            r.history_pose.append((float(p[0]), float(p[1]), float(p[2])))
        r.px, r.py, r.theta, r.v, r.w = (float(v) for v in s)
        return st, n, list(traj)

    def step(self):
        """One iteration of DWA.plan (dwa.py:74-93).  Returns 'reached', 'stepped' or raises."""
        st, n, _ = self._run(1)
        if st == _lib.STATUS_REF_RAISES:
            raise IndexError("DWA evaluation window is empty / lookahead failed (reference raises)")
        return "reached" if st == 1 else "stepped"

    def plan(self) -> tuple:
        """(True, history_traj, history_pose) or (False, None, None) (dwa.py:67-93)."""
        st, n, traj = self._run(int(self.params["MAX_ITERATION"]))
        if st == 1:
            return True, traj, self.robot.history_pose
        if st == _lib.STATUS_REF_RAISES:
            raise IndexError("DWA evaluation window is empty / lookahead failed (reference raises)")
        return False, None, None

    def run(self):
        return self.plan()


class _Tracker(LocalPlanner):
    """Shared plan loop of LQR / MPC (lqr.py:58-86, mpc.py:66-94) on the gfx950 kernel track.hip."""

    KIND = "lqr"

    def __init__(self, start: tuple, goal: tuple, env: Env, heuristic_type: str = "euclidean", **params) -> None:
        super().__init__(start, goal, env, heuristic_type, **params)
        self.g_planner = {"planner_name": "a_star", "start": (start[0], start[1]), "goal": (goal[0], goal[1]),
                          "env": env}
        self.path = self.g_path[::-1]
        self._u_p = (0.0, 0.0)

    def _kernel_params(self):
        return {}

    def _run(self, iters: int):
        torch = _lib.device_check()
        r = self.robot
        state = torch.tensor([[r.px, r.py, r.theta, r.v, r.w]], dtype=torch.float64, device="cuda")
        u_p = torch.tensor([self._u_p], dtype=torch.float64, device="cuda")
        xy, off = batch.pack_paths([np.asarray(self.path, np.float64)])
        out = batch.track_step_batch(self.KIND, self._lp_params(), state, np.array([self.goal], np.float64), xy, off,
                                     iters=iters, u_p=u_p, want_hist=True, **self._kernel_params())
        n = int(out["n_steps"][0])
        st = int(out["status"][0])
        for p in out["hist_pose"][0, :n].cpu().numpy():
            r.history_pose.append((float(p[0]), float(p[1]), float(p[2])))
        r.px, r.py, r.theta, r.v, r.w = (float(v) for v in state[0].cpu().numpy())
        self._u_p = tuple(float(v) for v in u_p[0].cpu().numpy())
        return st

    def step(self):
        """One iteration of the plan loop.  Returns 'reached' or 'stepped'; raises where the reference does."""
        st = self._run(1)
        if st == _lib.STATUS_REF_RAISES:
            raise IndexError("getLookaheadPoint failed (reference raises)")
        return "reached" if st == 1 else "stepped"

    def plan(self):
        """(True, history_pose) or (False, None)."""
        self._u_p = (0.0, 0.0)  # mpc.py:64 starts every plan() from u_p = (0, 0)
        st = self._run(int(self.params["MAX_ITERATION"]))
        if st == 1:
            return True, self.robot.history_pose
        if st == _lib.STATUS_REF_RAISES:
            raise IndexError("getLookaheadPoint failed (reference raises)")
        return False, None

    def run(self):
        return self.plan()


class LQR(_Tracker):
    """Linear Quadratic Regulator (local_planner/lqr.py:12-145)."""

    KIND = "lqr"

    def __init__(self, start: tuple, goal: tuple, env: Env, heuristic_type: str = "euclidean", **params) -> None:
        self.Q = np.diag([1, 1, 1])
        self.R = np.diag([1, 1])
        self.lqr_iteration = 100
        self.eps_iter = 1e-1
        super().__init__(start, goal, env, heuristic_type, **params)

    def __str__(self) -> str:
        return "Linear Quadratic Regulator (LQR)"

    def _lqr_params(self):
        return _lib.LQRParams.make(np.diag(self.Q), np.diag(self.R), self.lqr_iteration, self.eps_iter)

    def _kernel_params(self):
        return dict(lqr_params=self._lqr_params())

    def lqrControl(self, s: tuple, s_d: tuple, u_r: tuple) -> np.ndarray:
        """lqr.py:103-145 on the device; returns [[v], [w]]."""
        u = batch.lqr_control_batch(self._lp_params(), self._lqr_params(), [s], [s_d], [u_r],
                                    [(self.robot.v, self.robot.w)])
        return u.cpu().numpy().reshape(2, 1)


class MPC(_Tracker):
    """Model Predictive Control (local_planner/mpc.py:14-214).  The OSQP solve of mpc.py:196-203 is
    the device ADMM of track.hip (settings in self.admm; OSQP itself is not available)."""

    KIND = "mpc"

    def __init__(self, start: tuple, goal: tuple, env: Env, heuristic_type: str = "euclidean", **params) -> None:
        self.p = 12
        self.m = 8
        self.Q = np.diag([0.8, 0.8, 0.5])
        self.R = np.diag([2, 2])
        self.admm = dict(_lib.ADMM_DEFAULTS)
        super().__init__(start, goal, env, heuristic_type, **params)
        self.u_min = np.array([[self.params["MIN_V"]], [self.params["MIN_W"]]])
        self.u_max = np.array([[self.params["MAX_V"]], [self.params["MAX_W"]]])
        self.du_min = np.array([[self.params["MIN_V_INC"]], [self.params["MIN_W_INC"]]])
        self.du_max = np.array([[self.params["MAX_V_INC"]], [self.params["MAX_W_INC"]]])

    def __str__(self) -> str:
        return "Model Predicted Control (MPC)"

    def _mpc_params(self):
        return _lib.MPCParams.make(self.p, self.m, np.diag(self.Q), np.diag(self.R), **self.admm)

    def _kernel_params(self):
        return dict(mpc_params=self._mpc_params())

    def mpcControl(self, s: tuple, s_d: tuple, u_r: tuple, u_p: tuple):
        """mpc.py:111-214 on the device: returns ([[v], [w]], new u_p)."""
        torch = _lib.device_check()
        up = torch.tensor([u_p], dtype=torch.float64, device="cuda")
        out = batch.mpc_control_batch(self._lp_params(), self._mpc_params(), [s], [s_d], [u_r], up,
                                      [(self.robot.v, self.robot.w)])
        u = out["u"].cpu().numpy().reshape(2, 1)
        return u, tuple(float(v) for v in up[0].cpu().numpy())
