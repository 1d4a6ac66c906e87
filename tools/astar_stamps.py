"""Dev probe (diagnostic build): where an A* expansion spends its cycles.
Run with PMP_HIP_LIB=python_motion_planning_amd/libpmp_hip_stamps.so."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

occ, s, g = wl.c2_workload(4096)
torch.cuda.set_device(0)
c = np.load(os.path.join(os.path.dirname(__file__), "c2_counters.npy")) if os.path.exists(
    os.path.join(os.path.dirname(__file__), "c2_counters.npy")) else None
order = np.argsort(-c[:, 2]) if c is not None else np.arange(4096)
for label, idx in (("longest alone", order[:1]), ("64 median alone", order[2000:2064]), ("full batch", np.arange(4096))):
    L = _lib.load_library()
    ctx = _lib.context()
    _lib.check(ctx, L.pmp_astar2d_reserve(ctx, 1024, 1024, min(1024, len(idx)), 0), "reserve")
    r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=4096, counters=True)
    torch.cuda.synchronize()
    st = r["counters"].cpu().numpy().astype(np.float64)
    ne = r["n_expanded"].cpu().numpy().astype(np.float64)
    pops = c[idx, 1] if c is not None else ne
    print(f"{label}: per pop cycles: pop+issue {st[:,0].sum()/pops.sum():.0f}  3x3-wait {st[:,1].sum()/pops.sum():.0f}  "
          f"per expansion push {st[:,2].sum()/ne.sum():.0f}  total/expansion {st[:,3].sum()/ne.sum():.0f}", flush=True)
