"""Dev probe (diagnostic build): where a 2D A* expansion spends its cycles on the C2 batch, for a
few worker counts.  Run with PMP_HIP_LIB=python_motion_planning_amd/libpmp_hip_stamps.so.
counters[q] = {pop cycles, 3x3 wait cycles, push-phase cycles (incl. the wait), total cycles}."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
nq = int(os.environ.get("NQ", "4096"))
occ, s, g = wl.c2_workload(nq)
for workers in [int(w) for w in os.environ.get("WORKERS", "1024,2048,4096").split(",")]:
    t = time.time()
    r = batch.astar2d_batch(occ, s, g, counters=True, reserve_slots=workers)
    torch.cuda.synchronize()
    dt = time.time() - t
    st = r["counters"].cpu().numpy().astype(np.float64)
    ne = r["n_expanded"].cpu().numpy().astype(np.float64)
    E = ne.sum()
    # oracle ratios on C2: 2.59 pops and 2.65 pushes per expansion
    print(f"workers {workers}: {dt:.2f} s  per expansion cycles: pop {st[:, 0].sum() / E:.0f} "
          f"(/pop {st[:, 0].sum() / E / 2.59:.0f})  wait {st[:, 1].sum() / E:.0f}  push-phase {st[:, 2].sum() / E:.0f} "
          f"(/push {(st[:, 2].sum() - st[:, 1].sum()) / E / 2.65:.0f})  total {st[:, 3].sum() / E:.0f}", flush=True)
