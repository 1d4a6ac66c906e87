"""Dev probe: DStar3D / LPAStar3D (plan only) on the C5 workload vs workers per CU
(pmp_set_workers_per_cu on each stream's context) and batches in flight."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
L = _lib.load_library()
nq = 8192
occ, s, g = wl.c5_workload(nq, first_seed=0)
X, Y, Z = occ.shape[1:]
bits = torch.as_tensor(np.ascontiguousarray(np.stack([batch.pack_bits(o) for o in occ])).view(np.int32), device="cuda")
s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
if os.environ.get("DUMMY_GB"):  # probe: one large allocation touched and freed before the first config
    d = torch.ones(int(float(os.environ["DUMMY_GB"]) * 2**30 // 8), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    del d
for kind in os.environ.get("KINDS", "dstar3d,lpastar3d").split(","):
    ref = None
    for pc in [int(x) for x in os.environ.get("PER_CU", "4,8,16").split(",")]:
        S = int(os.environ.get("STREAMS", "4"))
        streams = [torch.cuda.Stream() for _ in range(S)]
        for sm in streams:
            with torch.cuda.stream(sm):
                _lib.check(_lib.context(), L.pmp_set_workers_per_cu(_lib.context(), pc), "workers")

        def run(i):
            with torch.cuda.stream(streams[i % S]):
                if kind == "dstar3d":
                    return batch.dstar3d_batch(occ.shape, s_d, g_d, None, path_cap=X * Y * Z + 1, occ_bits=bits)
                return batch.lpastar3d_batch(occ.shape, s_d, g_d, None, path_cap=X * Y * Z + 1, occ_bits=bits)
        outs = [run(i) for i in range(S)]
        torch.cuda.synchronize()
        c = outs[0]["cost"].cpu().numpy()
        del outs
        for i in range(S):  # freed outputs: the timed launches reuse the blocks (no allocation inside)
            run(i)
        torch.cuda.synchronize()
        K = 3 * S
        t = time.perf_counter()
        for i in range(K):
            run(i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / K
        if ref is None:
            ref = c.copy()
        print(f"{kind} per_cu {pc} streams {S}: {dt * 1e3:.1f} ms/batch  {nq / dt:.0f} plans/s  "
              f"equal={np.array_equal(c, ref)}", flush=True)
