"""Dev probe: one A* 2D launch on the C2 workload, timed, for engine A/B and PMC passes.
ENGINE=1|0 (multi-query / one query per wave), T2LDS=0|1, WORKERS (queries in flight), RESIDENCY
(per CU; 0 = the launch's own), MODE=batch (4096 queries) | longest (the longest C2 query alone) |
longest4 (the 4 longest, one wave on engine 1) | c2med (one median C2 query) | c1.  Prints the launch time and the ops count."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
mode = os.environ.get("MODE", "batch")
occ, s, g = wl.c2_workload(4096)
ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_counters.npy"))
if mode == "c1":  # the README query alone (the drop-in latency case): counters from the oracle's C1 run
    occ, s, g = wl.readme_grid(), np.array([[5, 5]], np.int32), np.array([[45, 25]], np.int32)
    ref = np.array([[2314, 1890, 579, 438]], np.int64)
W, H = occ.shape
engine, t2 = int(os.environ.get("ENGINE", "1")), int(os.environ.get("T2LDS", "0"))
if mode == "c1":
    idx = np.zeros(1, np.int64)
elif mode == "longest":
    idx = np.argsort(-ref[:, 2])[:1]
elif mode == "c2med":  # a C2 query of median start-goal distance (the bench's latency row picks likewise)
    from python_motion_planning_amd import shard
    idx = np.argsort(shard.octile(s, g))[2048:2049]
elif mode == "longest4":
    idx = np.argsort(-ref[:, 2])[:4]
else:
    idx = np.tile(np.arange(4096), int(os.environ.get("REPEAT", "1")))  # MODE=batch, REPEAT=K: K batches as one launch
w = int(os.environ.get("WORKERS", "2048" if engine == 1 else "768"))
w = min(w, len(idx))
L, ctx = _lib.load_library(), _lib.context()
_lib.check(ctx, L.pmp_astar2d_set_engine(ctx, engine, t2), "engine")
_lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, w, 0), "reserve")
res = int(os.environ.get("RESIDENCY", "0"))
if res:
    _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, res), "residency")
bits = batch.occ_bits_device(occ, torch)
for rep in range(int(os.environ.get("REPS", "2"))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = batch.astar2d_batch((W, H), s[idx], g[idx], path_cap=4096, counters=True, occ_bits=bits,
                            retry_overflow=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    c = r["counters"].cpu().numpy()
    if os.environ.get("PMP_HIP_LIB", "").endswith("stamps.so"):  # cycle sums per query (PMP_STAMPS build)
        rr = ref[idx]
        tot = c[:, 3].astype(np.float64)
        print(f"stamps: pop {c[:, 0].sum() / tot.sum():.3f} expand {c[:, 1].sum() / tot.sum():.3f} "
              f"push {c[:, 2].sum() / tot.sum():.3f} of the query cycles; cycles per pop "
              f"{tot.sum() / rr[:, 1].sum():.0f}; per-query max {tot.max():.3e}", flush=True)
        continue
    assert np.array_equal(c[:, :3], ref[idx][:, :3]), "counter mismatch"
    print(f"{mode} x{len(idx) // 4096 if mode == 'batch' else 1} ({len(idx) / dt:.0f} plans/s) engine {engine} t2lds {t2} workers {w} residency {res}: {dt * 1e3:.1f} ms "
          f"pushes {c[:, 0].sum()} pops {c[:, 1].sum()} exp {c[:, 2].sum()}", flush=True)
