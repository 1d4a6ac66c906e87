"""Dev probe: the C2 batch (REPEAT copies) split between the two A* 2D engines running at the same
time on two streams -- the one-query-per-wave engine (astar2d.hip, scalar-issue bound) and the
multi-query engine (astar2d_mq.hip, vector-issue bound) -- so a CU's scalar and vector pipes both
work.  FRAC = share of the queries on the multi-query engine (by descending octile distance, dealt
so both get the same length mix); RES_MQ / RES_W = queries resident per CU of each (their LDS
shares must fit together: 160 KiB per CU); W_MQ / W_W = groups / waves per launch.  Checks every
query's counters against the C2 reference counters and prints plans/s."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, shard, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
occ, s, g = wl.c2_workload(4096)
ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_counters.npy"))
rep = int(os.environ.get("REPEAT", "10"))
S, G = np.tile(s, (rep, 1)), np.tile(g, (rep, 1))
R = np.tile(ref, (rep, 1))
L = _lib.load_library()
bits = batch.occ_bits_device(occ, torch)


def split(frac):
    order = np.argsort(-shard.octile(S, G), kind="stable")
    k = int(round(1.0 / frac)) if frac > 0 else 0
    if frac <= 0:
        return np.zeros(0, np.int64), order
    if frac >= 1:
        return order, np.zeros(0, np.int64)
    # deal: a FRAC share of every block of the sorted order to the multi-query engine
    take = (np.arange(len(order)) * frac) % 1.0 < frac
    return order[take], order[~take]


def lane(engine, workers, res):
    ctx = L.pmp_create(0)
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, engine, 1), "engine")
    _lib.check(ctx, L.pmp_astar2d_reserve(ctx, 1024, 1024, workers, 0), "reserve")
    if res:
        _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, res), "residency")
    return ctx


def run(ctx, stream, idx):
    nq = len(idx)
    out = dict(cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
               pl=torch.empty(nq, dtype=torch.int32, device="cuda"),
               path=torch.empty((nq, 4096), dtype=torch.int32, device="cuda"),
               ne=torch.empty(nq, dtype=torch.int32, device="cuda"),
               ctr=torch.empty((nq, 4), dtype=torch.int64, device="cuda"),
               st=torch.empty(nq, dtype=torch.int32, device="cuda"))
    s_d = torch.as_tensor(S[idx], device="cuda")
    g_d = torch.as_tensor(G[idx], device="cuda")
    out["s"], out["g"] = s_d, g_d
    return out


def launch(ctx, stream, o):
    nq = o["cost"].numel()
    if nq == 0:
        return
    rc = L.pmp_astar2d_batch(ctx, stream.cuda_stream, bits.data_ptr(), 1024, 1024, 0, o["s"].data_ptr(), o["g"].data_ptr(),
                             nq, o["cost"].data_ptr(), o["pl"].data_ptr(), o["path"].data_ptr(), 4096, o["ne"].data_ptr(),
                             None, 0, o["ctr"].data_ptr(), o["st"].data_ptr())
    _lib.check(ctx, rc, "astar2d_batch")


for spec in os.environ.get("SPECS", "1.0:32:0:8192:768,0.5:16:9:4096:2304").split(","):
    frac, res_mq, res_w, w_mq, w_w = spec.split(":")
    frac, res_mq, res_w, w_mq, w_w = float(frac), int(res_mq), int(res_w), int(w_mq), int(w_w)
    i_mq, i_w = split(frac)
    c_mq, c_w = lane(2, w_mq, res_mq + res_w), lane(0, w_w, res_w + res_mq)
    st_mq, st_w = torch.cuda.Stream(), torch.cuda.Stream()
    o_mq, o_w = run(c_mq, st_mq, i_mq), run(c_w, st_w, i_w)
    for it in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch(c_mq, st_mq, o_mq)
        launch(c_w, st_w, o_w)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    ok = True
    for o, idx in ((o_mq, i_mq), (o_w, i_w)):
        if len(idx):
            c = o["ctr"].cpu().numpy()
            ok &= bool(np.array_equal(c[:, :3], R[idx][:, :3])) and bool((o["st"].cpu().numpy() == 0).all())
    print(f"frac_mq {frac} res {res_mq}+{res_w} workers {w_mq}/{w_w}: {len(S) / dt:.0f} plans/s ({dt * 1e3:.0f} ms) "
          f"counters_ok {ok}", flush=True)
    L.pmp_destroy(c_mq)
    L.pmp_destroy(c_w)
