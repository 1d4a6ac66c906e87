"""Stage-by-stage wall time of the drop-in AStar.plan() (a_star.py:39-83) on one GPU: where the
single-query latency goes (C1 README query, one C2 query).  Dev tool: `python tools/latency_parts.py`."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import python_motion_planning_amd as pmp  # noqa: E402
from python_motion_planning_amd import _lib, batch, shard  # noqa: E402
from python_motion_planning_amd import workloads as wl  # noqa: E402


def main():
    occ2, s2, g2 = wl.c2_workload(nq=64)
    cases = [("c1", wl.readme_grid(), (5, 5), (45, 25))]
    if occ2 is not None:
        k = int(np.argsort(shard.octile(s2, g2))[32])
        cases.append(("c2", occ2, tuple(int(v) for v in s2[k]), tuple(int(v) for v in g2[k])))
    for name, occ, s, g in cases:
        W, H = occ.shape
        env = pmp.Grid(W, H)
        env.update({(int(x), int(y)) for x, y in np.argwhere(occ)})
        planner = pmp.AStar(s, g, env)
        planner.plan()
        torch.cuda.synchronize()
        walls = []
        for _ in range(20):
            t0 = time.perf_counter()
            planner.plan()
            walls.append(time.perf_counter() - t0)
        ab = {"speculative": [], "cold_upload": []}
        for _ in range(10):  # A/B in one process: launch on the cached upload vs pack-then-upload first
            t0 = time.perf_counter()
            planner.plan()
            ab["speculative"].append(time.perf_counter() - t0)
            env._pmp_occ = None
            t0 = time.perf_counter()
            planner.plan()
            ab["cold_upload"].append(time.perf_counter() - t0)
        print(name, "plan() A/B median ms", {k: round(float(np.median(v)) * 1e3, 3) for k, v in ab.items()},
              flush=True)
        parts = {}

        def tick(key, t):
            parts.setdefault(key, []).append(time.perf_counter() - t)
            return time.perf_counter()

        for _ in range(10):
            t = time.perf_counter()
            words = env.occupancy_words()
            t = tick("occupancy_words", t)
            ob = torch.as_tensor(words.view(np.int32), device="cuda")
            torch.cuda.synchronize()
            t = tick("occ_h2d", t)
            r = batch.astar2d_batch((W, H), np.array([s]), np.array([g]), path_cap=min(W * H + 1, 1 << 14),
                                    expand_cap=min(W * H, 1 << 18), occ_bits=ob, retry_overflow=False)
            t = tick("batch_call_async", t)
            torch.cuda.synchronize()
            t = tick("kernel_wait", t)
            st = torch.stack([r["status"][0], r["n_expanded"][0], r["path_len"][0]]).cpu().tolist()
            t = tick("meta_d2h", t)
            cells = r["path"][0, : st[2]].cpu().numpy()
            exp = r["expand"][0, : st[1]].cpu().numpy().astype(np.uint32)
            t = tick("path_expand_d2h", t)
            planner._expand_nodes(exp, H)
            t = tick("closed_node_list", t)
        out = {k: round(float(np.median(v)) * 1e3, 4) for k, v in parts.items()}
        print(name, "plan() median ms", round(float(np.median(walls)) * 1e3, 4), out, flush=True)


if __name__ == "__main__":
    _lib.device_check()
    main()
