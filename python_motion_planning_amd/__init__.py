"""python_motion_planning_amd -- MI355X-native batched motion-planning core.

Drop-in for the hot path of python_motion_planning (Slenderman00 fork): the same class names
and plan() conventions, with the inner loops running as gfx950 HIP kernels (libpmp_hip.so,
C-ABI in include/pmp.h).  There is no CPU fallback: without the library or a HIP device the
planners raise.
"""
from .env import Env, Env3D, Grid, Grid3D, Map, Map3D, Node, Node3D, pack_bits  # noqa: F401
from .graph_search import (AStar, AStar3D, Dijkstra, Dijkstra3D, DStar, GBFS, GBFS3D, GraphSearcher,  # noqa: F401
                           GraphSearcher3D, DStar3D, DNode3D, LPAStar3D, LNode3D, DStarLite, LazyThetaStar, LazyThetaStar3D, LPAStar, ThetaStar, ThetaStar3D)
from .factory import ControlFactory, SearchFactory  # noqa: F401
from .local_planner import DWA, LQR, MPC, LocalPlanner, Robot  # noqa: F401
from .planner import Planner, Planner3D  # noqa: F401
from .sample_search import RRT, RRTStar, SampleSearcher  # noqa: F401
from . import batch, workloads  # noqa: F401

__all__ = ["Env", "Env3D", "Grid", "Grid3D", "Map", "Map3D", "Node", "Node3D", "Planner", "Planner3D",
           "GraphSearcher", "AStar", "Dijkstra", "GBFS", "ThetaStar", "LazyThetaStar", "LPAStar", "DStarLite", "DStar", "GraphSearcher3D", "DStar3D", "DNode3D", "LPAStar3D", "LNode3D", "AStar3D", "Dijkstra3D", "GBFS3D", "ThetaStar3D", "LazyThetaStar3D", "SearchFactory", "ControlFactory", "LocalPlanner", "Robot", "DWA", "LQR", "MPC", "SampleSearcher", "RRT", "RRTStar",
           "batch", "workloads"]
