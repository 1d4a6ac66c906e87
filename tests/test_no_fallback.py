"""The product path has no CPU fallback: without libpmp_hip.so, or without a HIP device, every
planner raises instead of silently computing on the CPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_missing_library_raises():
    code = ("import python_motion_planning_amd._lib as L\n"
            "try:\n    L.load_library()\nexcept L.PMPError as e:\n    print('raised:', e)\n")
    env = dict(os.environ, PMP_HIP_LIB="/nonexistent/libpmp_hip.so")
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert "raised:" in out.stdout and "no CPU fallback" in out.stdout, out.stdout + out.stderr


def _no_gpu():
    import torch

    return not torch.cuda.is_available()


@pytest.mark.skipif(not _no_gpu(), reason="checks the behaviour on a host without a HIP device")
def test_planners_raise_without_device():
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import _lib, workloads as wl

    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
    with pytest.raises(_lib.PMPError):
        pmp.AStar((5, 5), (45, 25), env).plan()
    with pytest.raises(_lib.PMPError):
        pmp.DStar((5, 5), (45, 25), env).plan()
    m = pmp.Map(51, 31)
    m.update(obs_rect=wl.README_MAP_RECT, obs_circ=wl.README_MAP_CIRC)
    with pytest.raises(_lib.PMPError):
        pmp.RRTStar((18, 8), (37, 18), m).plan()
    with pytest.raises(_lib.PMPError):
        pmp.SearchFactory()("a_star", start=(5, 5), goal=(45, 25), env=env).plan()
    # local planners build their global path with the A* kernel in the constructor
    with pytest.raises(_lib.PMPError):
        pmp.DWA((5, 5, 0), (45, 25, 0), env)
    with pytest.raises(_lib.PMPError):
        pmp.MPC((5, 5, 0), (45, 25, 0), env)


def test_out_of_scope_names_raise():
    import python_motion_planning_amd as pmp

    with pytest.raises(NotImplementedError):
        pmp.SearchFactory()("jps", start=(1, 1), goal=(2, 2), env=None)
    with pytest.raises(NotImplementedError):
        pmp.ControlFactory()("pid", start=(1, 1, 0), goal=(2, 2, 0), env=None)


def test_factory_names_dijkstra_gbfs():
    import python_motion_planning_amd as pmp

    env = pmp.Grid(51, 31)
    assert type(pmp.SearchFactory()("dijkstra", start=(5, 5), goal=(45, 25), env=env)).__name__ == "Dijkstra"
    assert type(pmp.SearchFactory()("gbfs", start=(5, 5), goal=(45, 25), env=env)).__name__ == "GBFS"


def test_factory_names_theta_2d():
    import python_motion_planning_amd as pmp

    env = pmp.Grid(51, 31)
    assert type(pmp.SearchFactory()("theta_star", start=(5, 5), goal=(45, 25), env=env)).__name__ == "ThetaStar"
    assert type(pmp.SearchFactory()("lazy_theta_star", start=(5, 5), goal=(45, 25), env=env)).__name__ == "LazyThetaStar"
