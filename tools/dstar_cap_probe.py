"""Dev probe: D* (pmp_dstar2d_batch) on the bench's 256^2 / 512^2 workloads (4096 queries, one launch
on one context): status histogram and kernel time -- for builds with a smaller heap / entry capacity
per cell (PMP_DSTAR_HEAP_PER_CELL), whose overflowing queries report STATUS_CAP_OVERFLOW.
usage (GPU box): PMP_HIP_LIB=... python tools/dstar_cap_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

L = _lib.load_library()
for W in (256, 512):
    nq = 4096
    occ, s, g = wl.c2_workload(nq=nq, W=W, H=W, density=0.1, grid_seed=4, pair_seed=5)
    bits = batch.occ_bits_device(occ, torch)
    s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
    ctx = L.pmp_create(0)
    cost = torch.empty(nq, dtype=torch.float64, device="cuda")
    plen = torch.empty(nq, dtype=torch.int32, device="cuda")
    path = torch.empty((nq, 4 * W), dtype=torch.int32, device="cuda")
    npr = torch.empty(nq, dtype=torch.int64, device="cuda")
    st = torch.empty(nq, dtype=torch.int32, device="cuda")
    times = []
    for r in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.pmp_dstar2d_batch(ctx, torch.cuda.current_stream().cuda_stream, bits.data_ptr(), W, W, s_d.data_ptr(),
                                 g_d.data_ptr(), nq, cost.data_ptr(), plen.data_ptr(), path.data_ptr(), 4 * W,
                                 npr.data_ptr(), st.data_ptr(), 0)
        _lib.check(ctx, rc, "pmp_dstar2d_batch")
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    u, c = np.unique(st.cpu().numpy(), return_counts=True)
    print(f"W={W}: statuses {dict(zip(u.tolist(), c.tolist()))}, kernel ms {[round(t, 1) for t in times]}, "
          f"n_process sum {int(npr.sum())}, cost sum {float(cost.sum()):.6f}", flush=True)
    L.pmp_destroy(ctx)
