"""Sample-search planners: drop-in RRT / RRTStar (global_planner/sample_search/) on the gfx950
kernel rrt.hip.

plan() keeps the reference's signature, return convention and its use of the global numpy RNG:
the draws generateRandomNode (rrt.py:91-103) would make are read from a copy of np.random's
state, and afterwards the global generator is advanced by exactly the number the kernel
consumed, so a caller's later np.random draws are unchanged.
"""
from __future__ import annotations

import math

import numpy as np

from . import batch
from .env import Map, Node
from .planner import Planner


def random_stream(sample_num: int, state=None) -> np.ndarray:
    """The doubles generateRandomNode would draw from np.random (or from `state`): at most
    3 per iteration, in RandomState.random_sample order."""
    rs = np.random.RandomState()
    rs.set_state(np.random.get_state() if state is None else state)
    return rs.random_sample(3 * int(sample_num) + 1)


class SampleSearcher(Planner):
    """global_planner/sample_search/sample_search.py:13-135 (collision tests run on the device)."""

    def __init__(self, start: tuple, goal: tuple, env: Map, delta: float = 0.5) -> None:
        super().__init__(start, goal, env)
        self.delta = delta


class RRT(SampleSearcher):
    """Rapidly-exploring Random Tree (rrt.py:14-151)."""

    STAR = False

    def __init__(self, start: tuple, goal: tuple, env: Map, max_dist: float = 0.5, sample_num: int = 10000,
                 goal_sample_rate: float = 0.05) -> None:
        super().__init__(start, goal, env)
        self.max_dist = max_dist
        self.sample_num = sample_num
        self.goal_sample_rate = goal_sample_rate
        self.r = 10.0

    def __str__(self) -> str:
        return "Rapidly-exploring Random Tree(RRT)"

    def plan(self) -> tuple:
        """(cost, path goal->start, expand list of Node) or (0, None, expand) (rrt.py:49-83)."""
        rnd = random_stream(self.sample_num)
        out = batch.rrt_batch(self.env, [self.start.current], [self.goal.current], rnd[None], self.sample_num,
                              star=self.STAR, max_dist=self.max_dist, radius=self.r,
                              goal_sample_rate=self.goal_sample_rate, delta=self.delta)
        st = int(out["status"][0])
        draws = int(out["draws"][0])
        if draws:
            np.random.random_sample(draws)  # advance the global RNG exactly as the reference's loop does
        if st not in (0, 1):
            raise RuntimeError(f"RRT kernel status {st}")
        n = int(out["n_nodes"][0])
        xy = out["tree_xy"][0, :n].cpu().numpy()
        g = out["tree_g"][0, :n].cpu().numpy()
        par = out["tree_parent"][0, :n].cpu().numpy()
        expand = []
        for i in range(n):
            cur = (float(xy[i, 0]), float(xy[i, 1]))
            expand.append(Node(cur, (float(xy[par[i], 0]), float(xy[par[i], 1])), float(g[i]), 0))
        # the start and goal keep the caller's coordinates (ints in the README examples)
        expand[0] = self.start
        if st == 1:
            return 0, None, expand
        self.goal.parent = expand[int(par[n - 1])].current
        self.goal.g = float(g[n - 1])
        expand[-1] = self.goal
        plen = int(out["path_len"][0])
        pts = out["path"][0, :plen].cpu().numpy()
        path = [(float(x), float(y)) for x, y in pts]
        path[0], path[-1] = self.goal.current, self.start.current
        return float(out["cost"][0]), path, expand

    def run(self):
        return self.plan()

    @staticmethod
    def plan_batch(env: Map, starts, goals, rnd, sample_num: int, star: bool = False, **kw):
        """Independent queries on one Map; rnd [nq, stride] random streams.  Device-tensor dict."""
        return batch.rrt_batch(env, starts, goals, rnd, sample_num, star=star, **kw)


class RRTStar(RRT):
    """RRT* (rrt_star.py:11-76): choose-parent and rewire within radius r."""

    STAR = True

    def __init__(self, start: tuple, goal: tuple, env: Map, max_dist: float = 0.5, sample_num: int = 10000,
                 r: float = 10.0, goal_sample_rate: float = 0.05) -> None:
        super().__init__(start, goal, env, max_dist, sample_num, goal_sample_rate)
        self.r = r

    def __str__(self) -> str:
        return "RRT*"

    @staticmethod
    def plan_batch(env: Map, starts, goals, rnd, sample_num: int, star: bool = True, **kw):
        return batch.rrt_batch(env, starts, goals, rnd, sample_num, star=star, **kw)
