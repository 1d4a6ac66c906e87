"""Batched entry points over the C-ABI (include/pmp.h).  Inputs/outputs are torch device tensors.

These are the calls the drop-in planner classes, the bench and the parity tests go through;
each one launches the gfx950 kernels of libpmp_hip.so asynchronously on the current stream.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .env import pack_bits


def _dev(torch, a, dtype):
    if isinstance(a, torch.Tensor):
        return a.to(device="cuda", dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


def occ_bits_device(occ, torch=None):
    """uint8 [W, H] (x-major) numpy occupancy -> bit-packed uint32 device tensor (as int32)."""
    torch = torch or _lib.device_check()
    words = pack_bits(occ)
    return torch.as_tensor(words.view(np.int32), device="cuda")


def astar2d_batch(occ, starts, goals, heuristic: str = "euclidean", path_cap: int | None = None,
                  expand_cap: int = 0, counters: bool = False, occ_bits=None, reserve_slots: int | None = None,
                  heap_cap: int = 0):
    """Batched AStar.plan (a_star.py:39-83).

    occ: numpy uint8 [W, H] (or pass occ=(W, H) with a prebuilt `occ_bits` device tensor).
    starts, goals: [nq, 2] int (numpy or device tensors).
    Returns dict of device tensors: cost f64 [nq], path_len i32 [nq], path i32 [nq, path_cap]
    (cell ids x*H+y, goal first), n_expanded i32, status i32, optional expand / counters.
    """
    torch = _lib.device_check()
    L = _lib.load_library()
    ctx = _lib.context()
    if occ_bits is None:
        W, H = int(occ.shape[0]), int(occ.shape[1])
        occ_bits = occ_bits_device(occ, torch)
    else:
        W, H = (int(occ[0]), int(occ[1])) if isinstance(occ, tuple) else (int(occ.shape[0]), int(occ.shape[1]))
    s = _dev(torch, starts, torch.int32).reshape(-1, 2)
    g = _dev(torch, goals, torch.int32).reshape(-1, 2)
    nq = int(s.shape[0])
    if path_cap is None:
        path_cap = min(W * H + 1, 1 << 16)
    out = dict(
        cost=torch.empty(nq, dtype=torch.float64, device="cuda"),
        path_len=torch.empty(nq, dtype=torch.int32, device="cuda"),
        path=torch.empty((nq, path_cap), dtype=torch.int32, device="cuda"),
        n_expanded=torch.empty(nq, dtype=torch.int32, device="cuda"),
        status=torch.empty(nq, dtype=torch.int32, device="cuda"),
    )
    out["expand"] = torch.empty((nq, expand_cap), dtype=torch.int32, device="cuda") if expand_cap else None
    out["counters"] = torch.empty((nq, 4), dtype=torch.int64, device="cuda") if counters else None
    if reserve_slots:
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, int(reserve_slots), int(heap_cap)), "pmp_astar2d_reserve")
    rc = L.pmp_astar2d_batch(ctx, _lib.stream_ptr(), occ_bits.data_ptr(), W, H,
                             1 if heuristic == "manhattan" else 0, s.data_ptr(), g.data_ptr(), nq,
                             out["cost"].data_ptr(), out["path_len"].data_ptr(), out["path"].data_ptr(), path_cap,
                             out["n_expanded"].data_ptr(), _lib.ptr(out["expand"]), int(expand_cap),
                             _lib.ptr(out["counters"]), out["status"].data_ptr())
    _lib.check(ctx, rc, "pmp_astar2d_batch")
    out["W"], out["H"] = W, H
    return out
