"""Drop-in TimeOptimalTrajectory3D (trajectory/time_optimal_trajectory.py:8-353 of the reference)
on the gfx950 kernel pmp_totp3d_batch: the config-5 step after 3D planning
(examples/3d_example.py:93-128).

Same constructor, attributes and return values as the reference (TrajectoryPoint /
TrajectoryConstraints dataclasses as in trajectory/trajectory_base.py:8-45); generate() and
evaluate() run on the GPU.  For many paths at once use batch.totp3d_batch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib, batch


@dataclass
class TrajectoryPoint:
    """trajectory_base.py:8-22"""
    time: float
    position: np.ndarray
    velocity: np.ndarray
    acceleration: np.ndarray
    jerk: Optional[np.ndarray] = None
    yaw: Optional[float] = None
    yaw_rate: Optional[float] = None

    def to_tuple(self):
        return tuple(self.position)


@dataclass
class TrajectoryConstraints:
    """trajectory_base.py:25-45"""
    max_velocity: np.ndarray
    max_acceleration: np.ndarray
    max_jerk: Optional[np.ndarray] = None
    min_time_step: float = 0.01

    def __post_init__(self):
        self.max_velocity = np.asarray(self.max_velocity)
        self.max_acceleration = np.asarray(self.max_acceleration)
        if self.max_jerk is not None:
            self.max_jerk = np.asarray(self.max_jerk)


def _params(constraints: TrajectoryConstraints, path_resolution: float):
    return _lib.TotpParams.make(np.asarray(constraints.max_velocity, np.float64),
                                np.asarray(constraints.max_acceleration, np.float64), float(constraints.min_time_step),
                                float(path_resolution))


def _points(rows: np.ndarray, with_yaw: bool = True) -> List[TrajectoryPoint]:
    out = []
    for r in rows:
        out.append(TrajectoryPoint(time=float(r[0]), position=r[1:4].copy(), velocity=r[4:7].copy(),
                                   acceleration=r[7:10].copy(),
                                   yaw=None if not with_yaw or np.isnan(r[10]) else float(r[10]),
                                   yaw_rate=None if not with_yaw or np.isnan(r[11]) else float(r[11])))
    return out


class TimeOptimalTrajectory3D:
    """time_optimal_trajectory.py:8-39 (path-velocity decomposition along a waypoint path)."""

    def __init__(self, path, constraints: Optional[TrajectoryConstraints] = None, path_resolution: float = 0.01):
        if not path:
            raise ValueError("Path cannot be empty")
        # _process_path (trajectory_base.py:64-80): 2D points get z = 0
        self.dimension = 3
        self.path = np.array([[p[0], p[1], 0.0] if len(p) == 2 else list(p) for p in path], dtype=float)
        if constraints is None:
            constraints = TrajectoryConstraints(np.array([2.0] * 3), np.array([1.0] * 3))
        self.constraints = constraints
        self.path_resolution = path_resolution
        self.trajectory_points: List[TrajectoryPoint] = []
        self.total_time = 0.0
        self.segment_times: List[float] = []
        self.s_values = None
        self.path_length = 0.0
        self.s_dot_profile = None
        self.s_ddot_profile = None
        self.time_profile = None

    def _run(self, eval_t=None):
        if len(self.path) < 2:
            raise ValueError("Need at least 2 waypoints for trajectory generation")
        r = batch.totp3d_batch([self.path], _params(self.constraints, self.path_resolution), eval_t=eval_t)
        st = int(r["status"][0].item())
        if st == _lib.STATUS_REF_RAISES:
            raise ValueError("`x` must be strictly increasing sequence.")
        if st != _lib.STATUS_FOUND:
            raise _lib.PMPError(f"pmp_totp3d_batch status {st}")
        return r

    def generate(self) -> List[TrajectoryPoint]:
        """generate() (:260-302) + compute_yaw_from_velocity (trajectory_base.py:245-261)."""
        r = self._run()
        ns = int(r["n_samples"][0].item())
        self.s_values = r["s_values"][0, :ns].cpu().numpy()
        self.path_length = float(self.s_values[-1])
        self.s_dot_profile = r["s_dot"][0, :ns].cpu().numpy()
        self.s_ddot_profile = r["s_ddot"][0, :ns].cpu().numpy()
        self.time_profile = r["time"][0, :ns].cpu().numpy()
        self.total_time = float(r["total_time"][0].item())
        npt = int(r["n_points"][0].item())
        self.trajectory_points = _points(r["points"][0, :npt].cpu().numpy())
        return self.trajectory_points

    def evaluate(self, t: float) -> TrajectoryPoint:
        """evaluate(t) (:304-335) after generate()."""
        if self.time_profile is None:
            raise AttributeError("'TimeOptimalTrajectory3D' object has no attribute 's_of_t' (call generate() first)")
        r = self._run(eval_t=[float(t)])
        return _points(r["points"][0, :1].cpu().numpy(), with_yaw=False)[0]

    # TrajectoryBase accessors (trajectory_base.py:97-148)
    def get_positions(self) -> np.ndarray:
        if not self.trajectory_points:
            self.generate()
        return np.array([tp.position for tp in self.trajectory_points])

    def get_velocities(self) -> np.ndarray:
        if not self.trajectory_points:
            self.generate()
        return np.array([tp.velocity for tp in self.trajectory_points])

    def get_accelerations(self) -> np.ndarray:
        if not self.trajectory_points:
            self.generate()
        return np.array([tp.acceleration for tp in self.trajectory_points])

    def get_times(self) -> np.ndarray:
        if not self.trajectory_points:
            self.generate()
        return np.array([tp.time for tp in self.trajectory_points])

    def get_path_length(self) -> float:
        return float(sum(np.linalg.norm(self.path[i] - self.path[i - 1]) for i in range(1, len(self.path))))

    def check_constraints(self) -> dict:
        """trajectory_base.py:150-190"""
        if not self.trajectory_points:
            self.generate()
        res = {"velocity_satisfied": True, "acceleration_satisfied": True, "jerk_satisfied": True}
        if np.any(np.max(np.abs(self.get_velocities()), axis=0) > self.constraints.max_velocity):
            res["velocity_satisfied"] = False
        if np.any(np.max(np.abs(self.get_accelerations()), axis=0) > self.constraints.max_acceleration):
            res["acceleration_satisfied"] = False
        return res
