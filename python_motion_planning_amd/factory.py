"""Name registries: drop-in SearchFactory (utils/planner/search_factory.py:13-51) and ControlFactory
(utils/planner/control_factory.py:13-27) for the planners this package accelerates.  Names of
reference planners outside the accelerated hot path raise NotImplementedError (not silently
substituted)."""
from __future__ import annotations

_SEARCH_OUT_OF_SCOPE = {"jps", "voronoi", "s_theta_star", "anya", "rrt_connect", "informed_rrt", "aco", "pso"}
_CONTROL_OUT_OF_SCOPE = {"pid", "apf", "rpp"}


class SearchFactory(object):
    def __call__(self, planner_name, **config):
        from . import graph_search

        table = {"a_star": "AStar", "dijkstra": "Dijkstra", "gbfs": "GBFS", "d_star": "DStar", "rrt": "RRT",
                 "rrt_star": "RRTStar", "theta_star": "ThetaStar", "lazy_theta_star": "LazyThetaStar",
                 "lpa_star": "LPAStar", "d_star_lite": "DStarLite"}
        if planner_name in table:
            mod = graph_search if planner_name in ("a_star", "dijkstra", "gbfs", "d_star", "theta_star", "lazy_theta_star", "lpa_star", "d_star_lite") else __import__(
                __package__ + ".sample_search", fromlist=["x"])
            cls = getattr(mod, table[planner_name], None)
            if cls is None:
                raise NotImplementedError(f"{planner_name} is not implemented yet in python_motion_planning_amd")
            return cls(**config)
        if planner_name in _SEARCH_OUT_OF_SCOPE:
            raise NotImplementedError(f"{planner_name} is outside the accelerated hot path of python_motion_planning_amd")
        raise ValueError("The `planner_name` must be set correctly.")


class ControlFactory(object):
    def __call__(self, planner_name, **config):
        from . import local_planner

        table = {"dwa": "DWA", "lqr": "LQR", "mpc": "MPC"}
        if planner_name in table:
            cls = getattr(local_planner, table[planner_name], None)
            if cls is None:
                raise NotImplementedError(f"{planner_name} is not implemented yet in python_motion_planning_amd")
            return cls(**config)
        if planner_name in _CONTROL_OUT_OF_SCOPE:
            raise NotImplementedError(f"{planner_name} is outside the accelerated hot path of python_motion_planning_amd")
        raise ValueError("The `planner_name` must be set correctly.")
