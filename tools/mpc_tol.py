"""Dev probe: the largest MPC state / u_p differences between the GPU plan loop and the oracle on the
256 C4 agents x 40 iterations (test_track_gpu.py's case) and on the smoke's 8 agents x 5, absolute and
relative, so the tests' tolerances are set from measurement (north_star: 1e-5 relative)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from python_motion_planning_amd import _lib, batch, local_planner, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
lp = _lib.LPParams.from_params(local_planner.LocalPlanner.DEFAULTS)
for na, iters in ((8, 5), (256, 40)):
    occ, states, goals = wl.c4_workload(na)
    ap = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (na, 1)).astype(np.int32),
                             path_cap=2048)
    pl, PP = ap["path_len"].cpu().numpy(), ap["path"].cpu().numpy()
    paths = [np.column_stack([PP[i, : pl[i]][::-1] // 31, PP[i, : pl[i]][::-1] % 31]).astype(np.float64)
             for i in range(na)]
    xy, off = batch.pack_paths(paths)
    st = torch.tensor(states, dtype=torch.float64, device="cuda")
    up = torch.zeros((na, 2), dtype=torch.float64, device="cuda")
    batch.track_step_batch("mpc", lp, st, goals, xy, off, iters=iters, u_p=up, mpc_params=_lib.MPCParams.make(p=30))
    ost, oup = O.track_batch("mpc", xy, off, goals, states, iters=iters,
                             mpc=O.MPCParams.default(p=30, eps_abs=1e-9, eps_rel=1e-9))[:2]
    for name, a, b in (("state", st.cpu().numpy(), ost), ("u_p", up.cpu().numpy(), oup)):
        d = np.abs(a - b)
        rel = d / np.maximum(np.abs(b), 1e-300)
        nz = np.abs(b) > 0
        print(f"{na} agents x {iters}: {name} max abs {d.max():.3e}, max rel (nonzero ref) "
              f"{rel[nz].max() if nz.any() else 0:.3e}, exact zeros kept {bool((a[~nz] == 0).all())}", flush=True)
