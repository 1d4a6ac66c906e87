"""Maintainer-side binding of libpmp_hip.so for the reference's AStar.plan (Option B).

A maintainer of python_motion_planning would add this module next to
global_planner/graph_search/a_star.py and replace the OPEN/CLOSED loop (a_star.py:47-83) with a
call into the C ABI (include/pmp.h, pmp_astar2d_batch).  It depends only on ctypes, numpy and
torch (device buffers), not on python_motion_planning_amd:

    from .a_star_hip import make_plan
    AStar.plan = make_plan(Node)          # Node = python_motion_planning.utils.Node

tests/test_integration_stub.py runs it against the README query.
"""
import ctypes
import math
import os

import numpy as np

_L = None
_ctx = None


def _lib(path=None):
    global _L, _ctx
    if _L is None:
        path = path or os.environ.get("PMP_HIP_LIB", "libpmp_hip.so")
        _L = ctypes.CDLL(path)
        _L.pmp_create.restype = ctypes.c_void_p
        _L.pmp_create.argtypes = [ctypes.c_int]
        _L.pmp_last_error.restype = ctypes.c_char_p
        _L.pmp_last_error.argtypes = [ctypes.c_void_p]
        _L.pmp_astar2d_batch.restype = ctypes.c_int
        _L.pmp_astar2d_batch.argtypes = ([ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2 +
                                         [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] +
                                         [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 2)
        _ctx = _L.pmp_create(0)
    return _L, _ctx


def make_plan(Node, lib_path=None):
    """An AStar.plan replacement with the reference's return convention (a_star.py:39-83):
    (cost, path goal -> start, CLOSED nodes in closure order) or ([], [], [])."""

    def plan(self):
        import torch

        L, ctx = _lib(lib_path)
        W, H = self.env.x_range, self.env.y_range
        occ = np.zeros(W * H, np.uint8)  # x-major cells x*H + y, the in-grid obstacles
        for (x, y) in self.env.obstacles:
            if 0 <= x < W and 0 <= y < H:
                occ[x * H + y] = 1
        packed = np.packbits(occ, bitorder="little")
        packed = np.concatenate([packed, np.zeros((-len(packed)) % 4, np.uint8)])  # whole u32 words
        bits = torch.as_tensor(packed.view("<u4").view(np.int32), device="cuda")
        s = torch.tensor([self.start.current], dtype=torch.int32, device="cuda")
        g = torch.tensor([self.goal.current], dtype=torch.int32, device="cuda")
        i32 = dict(dtype=torch.int32, device="cuda")
        cost = torch.empty(1, dtype=torch.float64, device="cuda")
        plen, nexp, st = torch.empty(1, **i32), torch.empty(1, **i32), torch.empty(1, **i32)
        path = torch.empty((1, W * H + 1), **i32)
        exp = torch.empty((1, W * H), **i32)
        rc = L.pmp_astar2d_batch(ctx, torch.cuda.current_stream().cuda_stream, bits.data_ptr(), W, H,
                                 0 if self.heuristic_type == "euclidean" else 1, s.data_ptr(), g.data_ptr(), 1,
                                 cost.data_ptr(), plen.data_ptr(), path.data_ptr(), W * H + 1, nexp.data_ptr(),
                                 exp.data_ptr(), W * H, None, st.data_ptr())
        if rc != 0:
            raise RuntimeError(L.pmp_last_error(ctx).decode())
        if int(st[0]) != 0:
            return [], [], []
        cells = path[0, : int(plen[0])].cpu().numpy()
        records = exp[0, : int(nexp[0])].cpu().numpy().astype(np.uint32)
        # CLOSED nodes: record = cell | parent_motion << 28 (8 = the start); g re-accumulated with the
        # motions' own costs (Node.__add__, node.py:39-41), h = self.h as the search set it
        motions = self.env.motions
        gmap, expand = {}, []
        for e in records.tolist():
            cell, d = e & 0x0FFFFFFF, e >> 28
            cur = (cell // H, cell % H)
            if d == 8:
                node = Node(cur, cur, 0, 0)
            else:
                m = motions[d]
                par = (cur[0] - m.x, cur[1] - m.y)
                node = Node(cur, par, gmap[par] + m.g, self.h(Node(cur), self.goal))
            gmap[cur] = node.g
            expand.append(node)
        pth = [(int(c) // H, int(c) % H) for c in cells]
        c = 0
        for a, b in zip(pth[:-1], pth[1:]):  # extractPath's summation order (goal -> start)
            c += math.hypot(b[0] - a[0], b[1] - a[1])
        return c, pth, expand

    return plan
