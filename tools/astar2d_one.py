"""Dev probe for PMC passes: one A* 2D launch on the C2 workload.
MODE=longest: the longest C2 query alone (1 worker); MODE=batch: the 4096-query batch at WORKERS."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
occ, s, g = wl.c2_workload(4096)
ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_counters.npy"))
mode = os.environ.get("MODE", "longest")
idx = np.argsort(-ref[:, 2])[:1] if mode == "longest" else np.arange(4096)
w = 1 if mode == "longest" else int(os.environ.get("WORKERS", "3072"))
r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=4096, counters=True, reserve_slots=w)
torch.cuda.synchronize()
c = ref[idx]
print(mode, "pushes", c[:, 0].sum(), "pops", c[:, 1].sum(), "exp", c[:, 2].sum(), flush=True)
