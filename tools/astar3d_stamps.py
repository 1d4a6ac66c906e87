"""Dev probe (diagnostic build): where a 3D A* expansion spends its cycles (C5 batch).
Run with PMP_HIP_LIB=python_motion_planning_amd/libpmp_hip_stamps.so."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
occ, s, g = wl.c5_workload(8192)
ref = batch.astar3d_batch(occ, s, g, counters=True)  # the stamps build reports cycles in counters
torch.cuda.synchronize()
st = ref["counters"].cpu().numpy().astype(np.float64)
ne = ref["n_expanded"].cpu().numpy().astype(np.float64)
print(f"per expansion cycles: pop {st[:, 0].sum() / ne.sum():.0f}  after-pop wait {st[:, 1].sum() / ne.sum():.0f}  "
      f"push loop {st[:, 2].sum() / ne.sum():.0f}  total {st[:, 3].sum() / ne.sum():.0f}; "
      f"per query total {st[:, 3].mean():.0f} cycles, expansions {ne.mean():.0f}")
i = int(np.argmax(st[:, 3]))
print(f"slowest query {i}: {st[i, 3]:.0f} cycles, {ne[i]:.0f} expansions ({st[i, 3] / max(ne[i], 1):.0f} per expansion; "
      f"pop {st[i, 0] / max(ne[i], 1):.0f} wait {st[i, 1] / max(ne[i], 1):.0f} push {st[i, 2] / max(ne[i], 1):.0f})")
