"""Wall time of the drop-in DWA.plan (README map, (5,5,0) -> (45,25,0); resolution-sized windows, every
plan iteration in one dwa_kernel launch).  Usage: python tools/dwa_plan_time.py [reps]"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import python_motion_planning_amd as pmp  # noqa: E402
from python_motion_planning_amd import workloads as wl  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
env = pmp.Grid(51, 31)
env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
ts = []
for r in range(reps + 1):
    planner = pmp.DWA((5, 5, 0), (45, 25, 0), env)
    t = time.perf_counter()
    ok, traj, poses = planner.plan()
    ts.append(time.perf_counter() - t)
print({"ok": ok, "steps": len(poses), "ms": [round(1e3 * x, 2) for x in ts[1:]]})
