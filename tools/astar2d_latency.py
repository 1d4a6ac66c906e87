"""Dev probe (C2 workload): A* 2D latency per expansion / per heap op, alone and under load.
With PMP_HIP_LIB=.../libpmp_hip_stamps.so the counters are cycle sums {pop, 3x3 wait, push, total}
per query; with the normal library they are {pushes, pops, expansions, max heap}."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
stamps = "stamps" in os.environ.get("PMP_HIP_LIB", "")
occ, s, g = wl.c2_workload(4096)
ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_counters.npy"))  # push, pop, exp, maxn
order = np.argsort(-ref[:, 2])


def run(idx, workers, reps=1):
    r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=4096, counters=True, reserve_slots=workers)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=4096, counters=True, reserve_slots=workers)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, r["counters"].cpu().numpy().astype(np.float64)


def report(name, idx, workers, reps=1):
    dt, c = run(idx, workers, reps)
    rc = ref[idx].astype(np.float64)
    E, P, Q = rc[:, 2].sum(), rc[:, 0].sum(), rc[:, 1].sum()
    line = f"{name}: {dt * 1e3:.1f} ms  E={E:.0f} ops={P + Q:.0f}"
    if stamps:
        line += (f"  cycles/exp: pop {c[:, 0].sum() / E:.0f} wait {c[:, 1].sum() / E:.0f} push-phase {c[:, 2].sum() / E:.0f}"
                 f" total {c[:, 3].sum() / E:.0f}  | /pop {c[:, 0].sum() / Q:.0f}  /push {(c[:, 2].sum() - c[:, 1].sum()) / P:.0f}")
    else:
        mx = rc[:, 2].max()
        line += f"  longest-query us/exp {dt / mx * 1e6:.3f}  us/op {dt / (rc[:, 0] + rc[:, 1]).max() * 1e6:.3f}"
    print(line, flush=True)


report("longest 1 alone", order[:1], 1)
report("longest 8 alone", order[:8], 8)
report("median 64 alone", order[2000:2064], 64)
report("median 1024 alone", order[1500:2524], 1024)
for w in [int(x) for x in os.environ.get("WORKERS", "1024,3072").split(",")]:
    report(f"batch 4096 @{w}", np.arange(4096), w)
