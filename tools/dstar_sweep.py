"""Dev probe: D* (C2-style 256^2 / 512^2 grids, the bench's dstar leg workload) launch throughput vs
workers per CU (pmp_set_workers_per_cu) and batches in flight (own stream + context each)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
L = _lib.load_library()
nq = int(os.environ.get("NQ", "1024"))
for W in [int(x) for x in os.environ.get("DIMS", "256,512").split(",")]:
    occ, s, g = wl.c2_workload(nq=nq, W=W, H=W, density=0.1, grid_seed=4, pair_seed=5)
    bits = batch.occ_bits_device(occ, torch)
    s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
    ref = None
    for pc in [int(x) for x in os.environ.get("PER_CU", "4,8,16").split(",")]:
        for S in [int(x) for x in os.environ.get("STREAMS", "1,3").split(",")]:
            lanes = []
            for _ in range(S):
                ctx = L.pmp_create(0)
                _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, pc), "workers")
                lanes.append(dict(ctx=ctx, st=torch.cuda.Stream(), cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
                                  plen=torch.empty(nq, dtype=torch.int32, device="cuda"),
                                  path=torch.empty((nq, 4 * W), dtype=torch.int32, device="cuda"),
                                  npr=torch.empty(nq, dtype=torch.int64, device="cuda"),
                                  status=torch.empty(nq, dtype=torch.int32, device="cuda")))

            def run(i):
                b = lanes[i % S]
                _lib.check(b["ctx"], L.pmp_dstar2d_batch(b["ctx"], b["st"].cuda_stream, bits.data_ptr(), W, W,
                                                         s_d.data_ptr(), g_d.data_ptr(), nq, b["cost"].data_ptr(),
                                                         b["plen"].data_ptr(), b["path"].data_ptr(), 4 * W,
                                                         b["npr"].data_ptr(), b["status"].data_ptr(), 0), "dstar")
            for i in range(S):
                run(i)
            torch.cuda.synchronize()
            K = max(2 * S, 4)
            t = time.perf_counter()
            for i in range(K):
                run(i)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / K
            c = lanes[0]["cost"].cpu().numpy()
            if ref is None:
                ref = c.copy()
            print(f"{W}^2 per_cu {pc} streams {S}: {dt * 1e3:.1f} ms/batch  {nq / dt:.0f} plans/s  "
                  f"equal={np.array_equal(c, ref)}", flush=True)
            for b in lanes:
                L.pmp_destroy(b["ctx"])
            del lanes
            torch.cuda.empty_cache()
