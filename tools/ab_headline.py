"""Same-process A/B of libpmp_hip builds on the A* headline launch (C2, engine 1, the bench's
geometry): each build is loaded with its own ctypes handle (RTLD_LOCAL: the same C-ABI symbols
resolve per handle), and the builds take turns -- create a context, one warmup launch (5 batches:
every slot first-touched, as the driver's --warmup 5), R timed
launches of B batches (HIP events on the launch stream), destroy the context (its ~150 GB of
per-slot scratch) -- so box-level drift hits every build alike.  Outputs are checked equal across
builds.
usage (GPU box): python tools/ab_headline.py libA.so libB.so [--rounds 3 --reps 2 --batches 5]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def bind(path):
    from python_motion_planning_amd import _lib

    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--warmup-batches", type=int, default=5,
                    help="the first launch on a fresh context: >= workers / 4096 batches touches every slot's "
                         "scratch (a launch that first-touches ~150 GB runs ~1.3 s slower)")
    ap.add_argument("--workers", type=int, default=14336)
    ap.add_argument("--residency", type=int, default=56)
    ap.add_argument("--prio", type=int, default=64)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from python_motion_planning_amd import batch, workloads as wl

    torch.cuda.set_device(0)
    occ, starts, goals = wl.c2_workload(nq=4096, pair_seed=1)
    W, H = occ.shape
    nq, B = len(starts), args.batches
    occ_bits = batch.occ_bits_device(occ, torch)
    s_rep = torch.as_tensor(starts, device="cuda").repeat(max(B, args.warmup_batches), 1)
    g_rep = torch.as_tensor(goals, device="cuda").repeat(max(B, args.warmup_batches), 1)
    path_cap = 4096
    NB = max(B, args.warmup_batches)
    out = {k: torch.empty(NB * nq, dtype=dt, device="cuda") for k, dt in
           (("cost", torch.float64), ("plen", torch.int32), ("nexp", torch.int32), ("status", torch.int32))}
    path = torch.empty((NB * nq, path_cap), dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()
    libs = [(os.path.basename(p), bind(p)) for p in args.libs]
    times = {n: [] for n, _ in libs}
    ref = None
    for r in range(args.rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for name, L in order:
            ctx = L.pmp_create(0)

            def chk(rc, what):
                if rc:
                    raise RuntimeError(f"{name}: {what}: {L.pmp_last_error(ctx).decode()}")

            chk(L.pmp_astar2d_set_engine(ctx, 1, 1), "engine")
            chk(L.pmp_astar2d_reserve(ctx, W, H, args.workers, 0), "reserve")
            chk(L.pmp_astar2d_set_schedule(ctx, 1), "schedule")
            chk(L.pmp_astar2d_set_priority(ctx, args.prio), "priority")
            chk(L.pmp_astar2d_set_residency(ctx, args.residency), "residency")

            def launch(nb):
                return L.pmp_astar2d_batch(ctx, stream.cuda_stream, occ_bits.data_ptr(), W, H, 0, s_rep.data_ptr(),
                                           g_rep.data_ptr(), nq * nb, out["cost"].data_ptr(), out["plen"].data_ptr(),
                                           path.data_ptr(), path_cap, out["nexp"].data_ptr(), None, 0, None,
                                           out["status"].data_ptr())

            chk(launch(min(B, args.warmup_batches)), "warmup")
            torch.cuda.synchronize()
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                chk(launch(B), "launch")
                e1.record(stream)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1))
                got = {k: v[:B * nq].cpu().numpy().copy() for k, v in out.items()}
                if ref is None:
                    ref = got
                    assert (ref["status"] == 0).all()
                for k in ref:
                    assert np.array_equal(got[k], ref[k]), (name, k)
            L.pmp_destroy(ctx)
            torch.cuda.synchronize()
            print(name, "round", r, "ms", [round(t, 1) for t in times[name][-args.reps:]], flush=True)
    res = {}
    for name, ts in times.items():
        ms = float(np.median(ts))
        res[name] = {"median_ms": ms, "plans_per_s": nq * B / ms * 1e3, "all_ms": ts}
        print(f"{name}: median {ms:.1f} ms per {B}-batch launch -> {nq * B / ms * 1e3:.0f} plans/s "
              f"(min {min(ts):.1f}, max {max(ts):.1f})")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
