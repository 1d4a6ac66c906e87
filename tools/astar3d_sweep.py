"""Dev probe: C5 3D A* throughput vs persistent workers per CU (pmp_set_workers_per_cu) and batches
in flight (one stream + context each), checked against the first configuration's costs."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
nq = 8192
occ, s, g = wl.c5_workload(nq, first_seed=0)
X, Y, Z = occ.shape[1:]
words = np.stack([batch.pack_bits(o) for o in occ])
occ_d = torch.as_tensor(np.ascontiguousarray(words).view(np.int32), device="cuda")
s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
L = _lib.load_library()
cap = X * Y * Z + 1
ref = None
for pc in [int(x) for x in os.environ.get("PER_CU", "4,8,16").split(",")]:
    for S in [int(x) for x in os.environ.get("STREAMS", "1,3").split(",")]:
        lanes = []
        for _ in range(S):
            ctx = L.pmp_create(0)
            _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, pc), "workers")
            lanes.append(dict(ctx=ctx, st=torch.cuda.Stream(), cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
                              plen=torch.empty(nq, dtype=torch.int32, device="cuda"),
                              path=torch.empty((nq, cap), dtype=torch.int32, device="cuda"),
                              nexp=torch.empty(nq, dtype=torch.int32, device="cuda"),
                              status=torch.empty(nq, dtype=torch.int32, device="cuda")))

        def run(i):
            b = lanes[i % S]
            _lib.check(b["ctx"], L.pmp_astar3d_batch(b["ctx"], b["st"].cuda_stream, occ_d.data_ptr(), 1, X, Y, Z, 0,
                                                     s_d.data_ptr(), g_d.data_ptr(), nq, b["cost"].data_ptr(),
                                                     b["plen"].data_ptr(), b["path"].data_ptr(), cap, b["nexp"].data_ptr(),
                                                     None, 0, None, b["status"].data_ptr()), "astar3d")
        for i in range(2 * S):
            run(i)
        torch.cuda.synchronize()
        K = 12
        t = time.perf_counter()
        for i in range(K):
            run(i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / K
        c = lanes[0]["cost"].cpu().numpy()
        if ref is None:
            ref = c.copy()
        print(f"per_cu {pc} streams {S}: {dt * 1e3:.2f} ms/batch  {nq / dt:.0f} plans/s  equal={np.array_equal(c, ref)}",
              flush=True)
        for b in lanes:
            L.pmp_destroy(b["ctx"])
        del lanes
        torch.cuda.empty_cache()
