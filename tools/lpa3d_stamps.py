"""LPAStar3D phase cycles per expansion (libpmp_hip_stamps.so: counters = cycles of min scan,
g block + rhs minima, membership scan, sequential updates), one query alone and at full load."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

assert "stamps" in os.environ.get("PMP_HIP_LIB", "")
occ, s, g = wl.c5_workload(2048)
ref = batch.lpastar3d_batch(occ, s, g)  # n_expanded from the same build (counters hold cycles)
ne = ref["n_expanded"][:, 0].cpu().numpy().astype(np.float64)
for nq in (1, 64, 2048):
    r = batch.lpastar3d_batch(occ[:nq], s[:nq], g[:nq], counters=True)
    torch.cuda.synchronize()
    c = r["counters"].cpu().numpy().astype(np.float64)
    e = ne[:nq].sum()
    print(nq, "cycles per expansion: min-scan %.0f  block+rhs %.0f  membership %.0f  updates %.0f" %
          tuple(c[:, k].sum() / e for k in range(4)), flush=True)
