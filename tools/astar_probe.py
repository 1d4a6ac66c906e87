"""Dev probe: A* kernel latency per expansion, alone vs in a batch (C2 workload)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402


def run(occ, s, g, workers, reps=1):
    L = _lib.load_library()
    ctx = _lib.context()
    W, H = occ.shape
    _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, workers, 0), "reserve")
    r = batch.astar2d_batch(occ, s, g, path_cap=4096, counters=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        r = batch.astar2d_batch(occ, s, g, path_cap=4096, counters=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, r["counters"].cpu().numpy()


occ, s, g = wl.c2_workload(4096)
torch.cuda.set_device(0)
dt, c = run(occ, s, g, 1024)
order = np.argsort(-c[:, 2])
print("batch 4096 @1024 workers: %.3f s, max exp %d" % (dt, c[:, 2].max()), flush=True)
for k in (1, 8, 64):
    idx = order[:k]
    dt, ck = run(occ, s[idx], g[idx], k)
    print("longest %d alone: %.4f s  -> %.3f us/expansion (max %d)" % (k, dt, dt / ck[:, 2].max() * 1e6, ck[:, 2].max()), flush=True)
idx = order[2000:2064]
dt, ck = run(occ, s[idx], g[idx], 64)
print("64 median queries alone: %.4f s -> %.3f us/exp" % (dt, dt / ck[:, 2].max() * 1e6), flush=True)
for w in (256, 512, 2048):
    dt, c = run(occ, s, g, w)
    print("batch 4096 @%d workers: %.3f s" % (w, dt), flush=True)
