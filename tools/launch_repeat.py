"""Dev probe: is a slow launch a property of the scratch allocation or of the moment?  Runs one
multi-batch launch (A* or Theta* 2D on the C2 pairs, engine 2) several times on one context, then on
a fresh context (new scratch), printing each launch's kernel time (HIP events around the call).
usage: python3 tools/launch_repeat.py <astar|theta_star|lazy_theta_star> <batches> <residency> <reps> <contexts>"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

algo, B, res, reps, nctx = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
torch.cuda.set_device(0)
L = _lib.load_library()
occ, s, g = wl.c2_workload(4096)[:3]
bits = batch.occ_bits_device(occ, torch)
s_d = torch.as_tensor(np.tile(s, (B, 1)), dtype=torch.int32, device="cuda")
g_d = torch.as_tensor(np.tile(g, (B, 1)), dtype=torch.int32, device="cuda")
for c in range(nctx):
    ctx = _lib.context()
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 2, 1), "engine")
    _lib.check(ctx, L.pmp_astar2d_reserve(ctx, 1024, 1024, 256 * res, 0), "reserve")
    _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, res), "residency")
    for r in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = batch.astar2d_batch((1024, 1024), s_d, g_d, path_cap=8192, occ_bits=bits, algo=algo)
        e1.record()
        torch.cuda.synchronize()
        print(f"{algo} context {c} launch {r}: {e0.elapsed_time(e1):.0f} ms for {B} batches", flush=True)
    torch.cuda.synchronize()
    L.pmp_destroy(ctx)  # a fresh context (new scratch allocations) for the next round
    _lib._ctx.clear()
