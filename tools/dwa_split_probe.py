"""Dev probe: DWA step kernel time (HIP events, mean of 50 launches) against the workgroups per agent
(pmp_dwa_set_split) for the 8-GPU strong split's per-rank share (32 of C4's 256 agents) and for all
256; every setting's states / controls checked equal to one workgroup per agent."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, local_planner, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
lp = _lib.LPParams.from_params(local_planner.LocalPlanner.DEFAULTS)
dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, 64, 64)
occ, states, goals = wl.c4_workload(256)
r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (256, 1)).astype(np.int32),
                        path_cap=2048)
pl, P = r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
H = occ.shape[1]
paths = [np.column_stack([P[i, : pl[i]][::-1] // H, P[i, : pl[i]][::-1] % H]).astype(np.float64) for i in range(256)]
grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
for na, parts_list in ((32, (1, 2, 4, 8, 16)), (256, (1, 2, 4))):
    xy, off = batch.pack_paths(paths[:na])
    ref = None
    for parts in parts_list:
        st0 = torch.tensor(states[:na], dtype=torch.float64, device="cuda")
        st = st0.clone()
        o = batch.dwa_step_batch(grid, lp, dp, st, goals[:na], xy, off, iters=1, parts=parts)
        torch.cuda.synchronize()
        got = (st.cpu().numpy(), o["u"].cpu().numpy(), o["best"].cpu().numpy())
        if ref is None:
            ref = got
        assert all(np.array_equal(a, b) for a, b in zip(got, ref)), (na, parts)
        evs = []
        for _ in range(50):
            st.copy_(st0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch.dwa_step_batch(grid, lp, dp, st, goals[:na], xy, off, iters=1, parts=parts)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in evs[5:]]))
        print(f"agents {na} parts {parts}: {ms * 1e3:.1f} us per step (event span incl. the wrapper's launches)",
              flush=True)

if os.environ.get("PMP_HIP_LIB", "").endswith("dwastamps.so"):
    # phase stamps of one 32-agent step at 8 parts (s_memtime ticks, tid 0 of every workgroup)
    na, parts = 32, 8
    xy, off = batch.pack_paths(paths[:na])
    st = torch.tensor(states[:na], dtype=torch.float64, device="cuda")
    for rep in range(3):
        st.copy_(torch.tensor(states[:na], dtype=torch.float64, device="cuda"))
        o = batch.dwa_step_batch(grid, lp, dp, st, goals[:na], xy, off, iters=1, want_traj=True, parts=parts)
        torch.cuda.synchronize()
    raw = o["best_traj"].reshape(-1).cpu().numpy().view(np.uint64)[: na * parts * 10].reshape(na * parts, 10)
    raw = raw.astype(np.int64)
    raw = raw[raw[:, 0] > 0]  # parts that ran (a stopped agent's parts return before stamping)
    t0 = raw[:, 0].min()
    names = ["start", "occ", "rollout+lookahead", "columns", "leafsums", "arrive", "sums", "scores", "end"]
    part = raw[:, :6] - t0
    print("all parts, mean ticks since the first start:", {n: int(part[:, i].mean()) for i, n in enumerate(names[:6])})
    last = raw[raw[:, 6] > 0] - t0
    print("per-phase mean ticks, all parts:", np.diff(raw[:, :6], axis=1).mean(axis=0).round().tolist())
    print("per-phase mean ticks, last parts:", np.diff(raw[raw[:, 6] > 0][:, :9], axis=1).mean(axis=0).round().tolist())
    print("last parts, mean ticks since the first start:", {n: int(last[:, i].mean()) for i, n in enumerate(names)})
    print("last part end, max ticks:", int(last[:, 8].max()))

if os.environ.get("PMP_HIP_LIB", "").endswith("dwastamps.so"):
    # phase stamps of one 256-agent step on the one-workgroup (LOCAL, k = 1) kernel
    na = 256
    xy, off = batch.pack_paths(paths[:na])
    st = torch.tensor(states[:na], dtype=torch.float64, device="cuda")
    for rep in range(3):
        st.copy_(torch.tensor(states[:na], dtype=torch.float64, device="cuda"))
        o = batch.dwa_step_batch(grid, lp, dp, st, goals[:na], xy, off, iters=1, want_traj=True, parts=1)
        torch.cuda.synchronize()
    raw = o["best_traj"].reshape(-1).cpu().numpy().view(np.uint64)[: na * 10].reshape(na, 10).astype(np.int64)
    raw = raw[raw[:, 8] > 0]
    names = ["occ+nib", "rollout+lookahead", "columns", "leafsums", "sums", "scores", "end"]
    cols = [0, 1, 2, 3, 4, 6, 7, 8]
    d = np.diff(raw[:, cols], axis=1).mean(axis=0).round().astype(int).tolist()
    print("LOCAL 256 agents, per-phase mean ticks:", dict(zip(names, d)), "total", int((raw[:, 8] - raw[:, 0]).mean()),
          "span", int(raw[:, 8].max() - raw[:, 0].min()))
