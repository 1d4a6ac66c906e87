"""Planner ABCs: drop-in for utils/planner/planner.py:12-39 and planner3d.py:12-51.

Plotting (the reference's Plot / Plot3D, created in every Planner.__init__ at planner.py:20)
is out of scope: `self.plot` is None and run() returns the plan() result.
"""
from __future__ import annotations

import math
from abc import ABC, abstractmethod

from .env import Env, Env3D, Node, Node3D


class Planner(ABC):
    def __init__(self, start: tuple, goal: tuple, env: Env) -> None:
        self.start = Node(start, start, 0, 0)
        self.goal = Node(goal, goal, 0, 0)
        self.env = env
        self.plot = None

    def dist(self, node1: Node, node2: Node) -> float:
        return math.hypot(node2.x - node1.x, node2.y - node1.y)

    def angle(self, node1: Node, node2: Node) -> float:
        return math.atan2(node2.y - node1.y, node2.x - node1.x)

    @abstractmethod
    def plan(self):
        """Interface for planning."""

    def run(self):
        """Reference: plan + animation.  Animation is out of scope; returns plan()."""
        return self.plan()


class Planner3D(ABC):
    def __init__(self, start: tuple, goal: tuple, env: Env3D) -> None:
        self.start = Node3D(start, start, 0, 0)
        self.goal = Node3D(goal, goal, 0, 0)
        self.env = env
        self.plot = None

    def dist(self, node1: Node3D, node2: Node3D) -> float:
        return math.sqrt((node2.x - node1.x) ** 2 + (node2.y - node1.y) ** 2 + (node2.z - node1.z) ** 2)

    def angle(self, node1: Node3D, node2: Node3D):
        dx, dy, dz = node2.x - node1.x, node2.y - node1.y, node2.z - node1.z
        return math.atan2(dy, dx), math.atan2(dz, math.hypot(dx, dy))

    @abstractmethod
    def plan(self):
        """Interface for planning."""

    def run(self):
        return self.plan()
