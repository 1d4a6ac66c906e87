"""Dev probe: one LPA* (or D* Lite, LITE=1) launch of the bench's README-grid queries (65,536), timed,
with the reference counters (pushes, expansions) for traffic-per-algorithmic-byte ratios under
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/lpa_traffic.sh)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
lite = os.environ.get("LITE", "0") == "1"
occ = wl.readme_grid()
free = np.argwhere(occ == 0)
rng = np.random.default_rng(3)
nl = int(os.environ.get("NQ", "65536"))
s = torch.as_tensor(free[rng.integers(len(free), size=nl)].astype(np.int32), device="cuda")
g = torch.as_tensor(free[rng.integers(len(free), size=nl)].astype(np.int32), device="cuda")
batch.lpastar2d_batch(occ, s[:64], g[:64], lite=lite)  # warm
torch.cuda.synchronize()
t0 = time.perf_counter()
r = batch.lpastar2d_batch(occ, s, g, counters=True, lite=lite)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
c = r["counters"].cpu().numpy()
P, E = int(c[:, 0].sum()), int(c[:, 1].sum())
print(f"{'dstar_lite' if lite else 'lpa_star'} {nl} queries {dt * 1e3:.1f} ms ({nl / dt:.0f} plans/s) pushes {P} "
      f"expansions {E} max|U| {int(c[:, 3].max())} alg_bytes {161.0 * E + 20.0 * P:.0f}", flush=True)
