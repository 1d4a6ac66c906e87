"""Dev probe: LPAStar3D on C5 (8192 queries x 6 per launch, as the bench's dyn3d leg) -- kernel time
against the workers per CU (pmp_set_workers_per_cu), U's peak length against the LDS share, and with
a PMP_STAMPS build the cycle split (min scan, g block + rhs minima, membership scan, updates)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
nq = 8192
occ, s, g = wl.c5_workload(nq, first_seed=0)
rep = 6
s6, g6 = np.tile(s, (rep, 1)), np.tile(g, (rep, 1))
bits = torch.as_tensor(np.ascontiguousarray(np.stack([batch.pack_bits(o) for o in occ])).view(np.int32),
                       device="cuda").repeat(rep, 1)
L = _lib.load_library()
ctx = _lib.context()
stamps = "stamps" in os.environ.get("PMP_HIP_LIB", "")
for w in [int(x) for x in (sys.argv[1:] or ["16"])]:
    _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, w), "workers")
    r = batch.lpastar3d_batch(occ.shape, s6, g6, path_cap=int(np.prod(occ.shape[1:])) + 1, occ_bits=bits, counters=True)
    torch.cuda.synchronize()
    ms = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = batch.lpastar3d_batch(occ.shape, s6, g6, path_cap=int(np.prod(occ.shape[1:])) + 1, occ_bits=bits, counters=True)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    c = r["counters"].cpu().numpy()
    if os.environ.get("PMP_PROBE_OUT"):  # per-query counters and expansions, for offline joins
        np.savez(os.environ["PMP_PROBE_OUT"], counters=c, n_expanded=r["n_expanded"].cpu().numpy())
    print(f"workers/CU {w}: {np.median(ms):.1f} ms per {rep * nq}-query launch ({rep * nq / np.median(ms) * 1e3:.0f} plans/s "
          f"one launch alone)", flush=True)
    if stamps:
        tot = c.sum(axis=0).astype(np.float64)
        ne = float(r["n_expanded"].sum().item())
        if "stamps2" in os.environ.get("PMP_HIP_LIB", ""):
            print("  ticks per expansion: removes %.0f pushes %.0f whole block %.0f whole query %.0f" % tuple(tot / ne),
                  flush=True)
        else:
            print("  cycle share: min-scan %.3f block+rhs %.3f membership %.3f updates %.3f" % tuple(tot / tot.sum()),
                  flush=True)
            print("  ticks per expansion: min-scan %.0f block+rhs %.0f membership %.0f updates %.0f" % tuple(tot / ne),
                  flush=True)
    else:
        nexp = c[:, 1]
        mx = c[:, 3]
        print(f"  expansions mean {nexp.mean():.0f} max {nexp.max()}; pushes mean {c[:, 0].mean():.0f}; "
              f"peak |U| quantiles 50/90/99/max {np.percentile(mx, 50):.0f}/{np.percentile(mx, 90):.0f}/"
              f"{np.percentile(mx, 99):.0f}/{mx.max()}", flush=True)
