"""Generate golden vectors by running the REFERENCE (python_motion_planning @ /root/reference).

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py [section ...]

Sections: astar_readme astar_small astar_1024 dstar astar3d graph2d graph3d theta3d theta2d lpa dstarlite lpa_replan dstarlite_replan rrt dwa lqr mpc hypot totp
Outputs are small fixtures (inputs + expected outputs) under tests/golden/.  The reference is
imported with stubs for the modules absent from this image (osqp, pyvista), per SURVEY.md §8(c).
"""
from __future__ import annotations

import csv
import hashlib
import json
import math
import os
import sys
import types
import unittest.mock
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def import_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    if REF + "/src" not in sys.path:
        sys.path.insert(0, REF + "/src")
    if "osqp" not in sys.modules:
        sys.modules["osqp"] = types.ModuleType("osqp")
    sys.modules["pyvista"] = unittest.mock.MagicMock()
    import logging

    import python_motion_planning as pmp  # noqa: E402

    logging.disable(logging.CRITICAL)
    return pmp


def close_figs():
    import matplotlib.pyplot as plt

    plt.close("all")


def obstacles_of(occ):
    return {(int(x), int(y)) for x, y in np.argwhere(occ)}


def occ_hash(cells):
    return hashlib.sha1(np.asarray(cells, np.int32).tobytes()).hexdigest()


def ragged(lists, dtype=np.int32):
    off = np.zeros(len(lists) + 1, np.int64)
    for i, l in enumerate(lists):
        off[i + 1] = off[i] + len(l)
    flat = np.concatenate([np.asarray(l, dtype).ravel() for l in lists]) if off[-1] else np.zeros(0, dtype)
    return flat, off


# ----------------------------------------------------------------------------------------------
def run_astar(args):
    occ, start, goal, heur, keep_expand = args
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    p = pmp.AStar(tuple(start), tuple(goal), env, heur)
    cost, path, expand = p.plan()
    close_figs()
    cells = [x * H + y for (x, y) in path]
    ecells = [n.current[0] * H + n.current[1] for n in expand]
    return dict(found=bool(path), cost=float(cost) if path else float("nan"), path=cells,
                n_expanded=len(expand), expand=ecells if keep_expand else [], expand_sha1=occ_hash(ecells))


def sec_astar_readme():
    from python_motion_planning_amd import workloads as wl

    occ = wl.readme_grid()
    r = run_astar((occ, (5, 5), (45, 25), "euclidean", True))
    r2 = run_astar((occ, (5, 5), (45, 25), "manhattan", True))
    out = dict(W=51, H=31, start=[5, 5], goal=[45, 25], obstacles=np.argwhere(occ).tolist(),
               euclidean=dict(cost_hex=float(r["cost"]).hex(), cost_repr=repr(r["cost"]), path=r["path"],
                              expand=r["expand"]),
               manhattan=dict(cost_hex=float(r2["cost"]).hex(), path=r2["path"], expand=r2["expand"]))
    with open(os.path.join(HERE, "astar_readme.json"), "w") as f:
        json.dump(out, f)
    print("astar_readme", r["cost"], len(r["path"]), r["n_expanded"])


def sec_astar_small(n=200):
    rng = np.random.default_rng(12345)
    cases = []
    for i in range(n):
        W = int(rng.integers(8, 97))
        H = int(rng.integers(8, 97))
        dens = float(rng.uniform(0.0, 0.35))
        occ = (rng.random((W, H)) < dens).astype(np.uint8)
        occ[:, 0] = occ[:, H - 1] = 1
        occ[0, :] = occ[W - 1, :] = 1
        free = np.argwhere(occ == 0)
        if len(free) < 2:
            occ[1, 1] = occ[W - 2, H - 2] = 0
            free = np.argwhere(occ == 0)
        s = free[rng.integers(len(free))]
        g = free[rng.integers(len(free))]
        kind = i % 20
        if kind == 7:          # start == goal
            g = s
        elif kind == 11:       # goal is an obstacle
            occ[g[0], g[1]] = 1
        elif kind == 13:       # start is an obstacle
            occ[s[0], s[1]] = 1
        heur = "manhattan" if i % 5 == 3 else "euclidean"
        cases.append((occ, tuple(int(v) for v in s), tuple(int(v) for v in g), heur, True))
    with Pool(8) as pool:
        res = pool.map(run_astar, cases, chunksize=4)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "astar_small.npz"),
        dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        manhattan=np.array([c[3] == "manhattan" for c in cases]),
        found=np.array([r["found"] for r in res]), cost=np.array([r["cost"] for r in res], np.float64),
        path=path_flat, path_off=path_off, expand=exp_flat, expand_off=exp_off,
        n_expanded=np.array([r["n_expanded"] for r in res], np.int32))
    print("astar_small", sum(r["found"] for r in res), "found of", n)


def sec_astar_1024(nq=48):
    from python_motion_planning_amd import workloads as wl

    occ, starts, goals = wl.c2_workload(nq=4096)
    idx = np.arange(nq)
    cases = [(occ, tuple(starts[i]), tuple(goals[i]), "euclidean", False) for i in idx]
    with Pool(8) as pool:
        res = pool.map(run_astar, cases, chunksize=1)
    path_flat, path_off = ragged([r["path"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "astar_1024.npz"),
        occ_sha1=np.array(occ_hash(np.argwhere(occ).ravel())), query_index=idx.astype(np.int32),
        start=starts[idx], goal=goals[idx], found=np.array([r["found"] for r in res]),
        cost=np.array([r["cost"] for r in res], np.float64), path=path_flat, path_off=path_off,
        n_expanded=np.array([r["n_expanded"] for r in res], np.int32),
        expand_sha1=np.array([r["expand_sha1"] for r in res]))
    print("astar_1024 expansions", [r["n_expanded"] for r in res][:10])


# ----------------------------------------------------------------------------------------------
def run_dstar(args):
    occ, start, goal = args
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    p = pmp.DStar(tuple(start), tuple(goal), env)
    try:
        cost, path, _ = p.plan()
        close_figs()
        return dict(raised="", cost=float(cost), path=[x * H + y for (x, y) in path], n_process=len(p.EXPAND))
    except Exception as e:  # the reference raises for unreachable starts (d_star.py:234)
        close_figs()
        return dict(raised=type(e).__name__, cost=float("nan"), path=[], n_process=len(p.EXPAND))


def sec_dstar():
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(777)
    cases = [(wl.readme_grid(), (5, 5), (45, 25))]
    for i in range(23):
        W = int(rng.integers(10, 48))
        H = int(rng.integers(10, 48))
        occ = wl.random_grid(W, H, float(rng.uniform(0, 0.3)), int(rng.integers(1 << 30)))
        free = np.argwhere(occ == 0)
        s = tuple(int(v) for v in free[rng.integers(len(free))])
        g = tuple(int(v) for v in free[rng.integers(len(free))])
        cases.append((occ, s, g))
    with Pool(8) as pool:
        res = pool.map(run_dstar, cases)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "dstar_small.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        raised=np.array([r["raised"] for r in res]), cost=np.array([r["cost"] for r in res]),
        path=path_flat, path_off=path_off, n_process=np.array([r["n_process"] for r in res], np.int64))
    print("dstar", [(r["raised"], r["n_process"]) for r in res])


# ----------------------------------------------------------------------------------------------
def run_astar3d(args):
    occ, start, goal = args
    pmp = import_reference()
    X, Y, Z = occ.shape
    env = pmp.Grid3D(X, Y, Z)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
    p = pmp.AStar3D(tuple(start), tuple(goal), env)
    cost, path, expand = p.plan()
    close_figs()
    enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
    return dict(cost=float(cost), path=[enc(t) for t in path], expand=[enc(n.current) for n in expand])


def sec_astar3d():
    sys.path.insert(0, REF + "/examples")
    import scenarios as S  # reference examples/scenarios.py (only `random` imported)

    pmp = import_reference()
    from python_motion_planning_amd import workloads as wl

    # (a) scenario bitmaps as the reference builds them (checks workloads.py semantics)
    bitmaps = {}
    for (X, Y, Z) in [(21, 15, 11), (26, 20, 16)]:
        for name, fn in S.scenarios.items():
            g = pmp.Grid3D(X, Y, Z)
            obs = fn(g)
            occ = np.zeros((X, Y, Z), np.uint8)
            for (a, b, c) in obs:
                if 0 <= a < X and 0 <= b < Y and 0 <= c < Z:
                    occ[a, b, c] = 1
            bitmaps[f"{name}_{X}x{Y}x{Z}"] = np.packbits(occ.ravel())
    # carve check
    g = pmp.Grid3D(26, 20, 16)
    obs = S.scenarios["door"](g)
    S.carve_safety_bubble(obs, (13, 10, 8), radius=2)
    occ = np.zeros((26, 20, 16), np.uint8)
    for (a, b, c) in obs:
        occ[a, b, c] = 1
    bitmaps["door_26x20x16_carved_13_10_8_r2"] = np.packbits(occ.ravel())
    np.savez_compressed(os.path.join(HERE, "scenarios3d.npz"), **bitmaps)

    # (b) the reference's published CSV rows for AStar3D (every 10th row = distinct seeds)
    rows = []
    with open(os.path.join(REF, "3d_pathfinding_results.csv"), newline="") as f:
        rd = csv.reader(f)
        next(rd)
        for k, r in enumerate(rd):
            if r[1] == "astar" and k % 10 == 0:
                rows.append(dict(scenario=r[0], cost=r[3], visited=int(r[4]),
                                 start=list(eval(r[5])), goal=list(eval(r[6])), seed=int(r[7])))  # noqa: S307
    with open(os.path.join(HERE, "astar3d_csv.json"), "w") as f:
        json.dump(rows, f)

    # (c) full reference runs (path + expand order) for a subset, both grid sizes
    cases = []
    for name in S.scenarios:
        for seed in range(0, 100, 10):
            s, gq = wl.bench3d_query(seed, 21, 15, 11)
            o = wl.SCENARIOS_3D[name](21, 15, 11)
            wl.carve_safety_bubble(o, s, 2)
            wl.carve_safety_bubble(o, gq, 2)
            cases.append((o, s, gq))
    for seed in range(40):
        s, gq = wl.bench3d_query(seed, 26, 20, 16)
        o = wl.SCENARIOS_3D["door"](26, 20, 16)
        wl.carve_safety_bubble(o, s, 1)
        wl.carve_safety_bubble(o, gq, 1)
        cases.append((o, s, gq))
    with Pool(8) as pool:
        res = pool.map(run_astar3d, cases)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "astar3d_runs.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        cost=np.array([r["cost"] for r in res]), path=path_flat, path_off=path_off,
        expand=exp_flat, expand_off=exp_off)
    print("astar3d csv rows", len(rows), "runs", len(res))


# ----------------------------------------------------------------------------------------------
def readme_env(pmp):
    from python_motion_planning_amd import workloads as wl

    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
    return env


def dwa_eval_case(args):
    """One DWA.evaluation (dwa.py:137-190) at a chosen robot state; 64x64 or default resolution."""
    state, grid64, predict_time = args
    pmp = import_reference()
    env = readme_env(pmp)
    p = pmp.DWA((5, 5, 0), (45, 25, 0), env, predict_time=predict_time)
    r = p.robot
    r.px, r.py, r.theta, r.v, r.w = state
    la, theta_trj, kappa = p.getLookaheadPoint()
    vr = p.calDynamicWin()
    if grid64:
        p.v_resolution = (vr[1] - vr[0]) / 64.5
        p.w_resolution = (vr[3] - vr[2]) / 64.5
    ev, tw = p.evaluation(vr, la)
    best = int(np.argmax(ev[:, -1]))
    close_figs()
    return dict(state=list(state), lookahead=[float(la[0]), float(la[1])], theta_trj=float(theta_trj),
                kappa=float(kappa), vr=[float(v) for v in vr], v_res=float(p.v_resolution),
                w_res=float(p.w_resolution), eval=np.asarray(ev, np.float64), best=best,
                best_traj=np.asarray(tw[best], np.float64), path=np.asarray(p.path, np.float64))


def sec_dwa():
    pmp = import_reference()
    rng = np.random.default_rng(31)
    from python_motion_planning_amd import workloads as wl

    occ = wl.readme_grid()
    free = np.argwhere(occ == 0)
    cases = []
    for i in range(24):
        c = free[rng.integers(len(free))]
        st = (float(c[0] + rng.uniform(-0.4, 0.4)), float(c[1] + rng.uniform(-0.4, 0.4)), float(rng.uniform(-np.pi, np.pi)),
              float(rng.uniform(0, 0.5)), float(rng.uniform(-np.pi / 2, np.pi / 2)))
        cases.append((st, i < 12, 3.0 if i % 3 else 1.5))
    with Pool(8) as pool:
        res = pool.map(dwa_eval_case, cases)
    out = {}
    for k in ("state", "lookahead", "vr"):
        out[k] = np.array([r[k] for r in res], np.float64)
    for k in ("theta_trj", "kappa", "v_res", "w_res"):
        out[k] = np.array([r[k] for r in res], np.float64)
    out["predict_time"] = np.array([c[2] for c in cases])
    out["best"] = np.array([r["best"] for r in res], np.int32)
    ev_flat, ev_off = ragged([r["eval"].ravel() for r in res], np.float64)
    bt_flat, bt_off = ragged([r["best_traj"].ravel() for r in res], np.float64)
    out.update(eval=ev_flat, eval_off=ev_off, best_traj=bt_flat, best_traj_off=bt_off, path=res[0]["path"])
    np.savez_compressed(os.path.join(HERE, "dwa_eval.npz"), **out)
    print("dwa eval", [r["eval"].shape[0] for r in res])


def run_local_plan(args):
    kind, start, goal, kw = args
    pmp = import_reference()
    env = readme_env(pmp)
    cls = {"dwa": pmp.DWA, "lqr": pmp.LQR}[kind]
    p = cls(start, goal, env, **kw)
    if kind == "dwa":
        ok, hist_traj, hist_pose = p.plan()
        u = np.array([t[0, 3:5] for t in hist_traj]) if ok else np.zeros((0, 2))
    else:
        ok, hist_pose = p.plan()
        u = np.zeros((0, 2))
    close_figs()
    return dict(ok=bool(ok), poses=np.asarray(hist_pose if ok else [], np.float64).reshape(-1, 3), u=u,
                path=np.asarray(p.path, np.float64))


def sec_local_plans():
    cases = [("dwa", (5, 5, 0), (45, 25, 0), {}), ("dwa", (8, 24, -1.0), (45, 25, 0), {"predict_time": 3.0}),
             ("lqr", (5, 5, 0), (45, 25, 0), {}), ("lqr", (8, 24, -1.0), (45, 25, 0.5), {})]
    with Pool(4) as pool:
        res = pool.map(run_local_plan, cases)
    out = {}
    for i, (c, r) in enumerate(zip(cases, res)):
        out[f"c{i}_kind"] = np.array(c[0])
        out[f"c{i}_start"] = np.array(c[1], np.float64)
        out[f"c{i}_goal"] = np.array(c[2], np.float64)
        out[f"c{i}_predict_time"] = np.array(c[3].get("predict_time", 1.5))
        out[f"c{i}_ok"] = np.array(r["ok"])
        out[f"c{i}_poses"] = r["poses"]
        out[f"c{i}_u"] = r["u"]
        out[f"c{i}_path"] = r["path"]
    np.savez_compressed(os.path.join(HERE, "local_plans.npz"), **out)
    print("local plans", [(c[0], r["ok"], len(r["poses"])) for c, r in zip(cases, res)])


def sec_lqr():
    pmp = import_reference()
    env = readme_env(pmp)
    p = pmp.LQR((5, 5, 0), (45, 25, 0), env)
    rng = np.random.default_rng(77)
    n = 1000
    S = np.column_stack([rng.uniform(0, 50, n), rng.uniform(0, 30, n), rng.uniform(-np.pi, np.pi, n)])
    SD = S + np.column_stack([rng.normal(0, 1, n), rng.normal(0, 1, n), rng.normal(0, 0.5, n)])
    UR = np.column_stack([rng.uniform(0, 0.5, n), rng.uniform(-1, 1, n)])
    V = rng.uniform(0, 0.5, n)
    Wv = rng.uniform(-1.5, 1.5, n)
    U = np.zeros((n, 2))
    for i in range(n):
        p.robot.v, p.robot.w = float(V[i]), float(Wv[i])
        U[i] = p.lqrControl(tuple(S[i]), tuple(SD[i]), tuple(UR[i])).ravel()
    close_figs()
    np.savez_compressed(os.path.join(HERE, "lqr_control.npz"), s=S, s_d=SD, u_r=UR, v=V, w=Wv, u=U)
    print("lqr", U[:3])


class _RecordingOSQP:
    """Stand-in for the absent `osqp` module: records the QP that MPC.mpcControl (mpc.py:196-203)
    hands to OSQP and returns a zero step.  Only the QP ASSEMBLY is pinned by these vectors; the
    OSQP solve itself is parity-unpinned (OSQP is not installed in this image)."""
    last = None

    def setup(self, P, q, A, l, u, **kw):
        _RecordingOSQP.last = dict(P=P.toarray(), q=np.asarray(q, np.float64).ravel(), A=A.toarray(),
                                   l=np.asarray(l, np.float64).ravel(), u=np.asarray(u, np.float64).ravel())

    def solve(self):
        class R:
            pass
        r = R()
        r.x = np.zeros(_RecordingOSQP.last["P"].shape[0])
        return r


def sec_mpc():
    pmp = import_reference()
    import python_motion_planning.local_planner.mpc as mpcmod

    mpcmod.osqp = types.SimpleNamespace(OSQP=_RecordingOSQP)
    env = readme_env(pmp)
    p = pmp.MPC((5, 5, 0), (45, 25, 0), env)
    rng = np.random.default_rng(99)
    out = {}
    for horizon in (12, 30):
        p.p = horizon
        n = 100
        S = np.column_stack([rng.uniform(0, 50, n), rng.uniform(0, 30, n), rng.uniform(-np.pi, np.pi, n)])
        SD = S + np.column_stack([rng.normal(0, 1, n), rng.normal(0, 1, n), rng.normal(0, 0.5, n)])
        UR = np.column_stack([rng.uniform(0, 0.5, n), rng.uniform(-1, 1, n)])
        UP = np.column_stack([rng.uniform(-0.2, 0.2, n), rng.uniform(-0.5, 0.5, n)])
        Ps, qs, As, ls, us = [], [], [], [], []
        for i in range(n):
            p.robot.v, p.robot.w = 0.2, 0.1
            p.mpcControl(tuple(S[i]), tuple(SD[i]), tuple(UR[i]), tuple(UP[i]))
            rec = _RecordingOSQP.last
            Ps.append(rec["P"]); qs.append(rec["q"]); As.append(rec["A"]); ls.append(rec["l"]); us.append(rec["u"])
        out[f"p{horizon}_s"] = S
        out[f"p{horizon}_s_d"] = SD
        out[f"p{horizon}_u_r"] = UR
        out[f"p{horizon}_u_p"] = UP
        out[f"p{horizon}_P"] = np.array(Ps)
        out[f"p{horizon}_q"] = np.array(qs)
        out[f"p{horizon}_A"] = np.array(As[0])
        out[f"p{horizon}_l"] = np.array(ls)
        out[f"p{horizon}_u"] = np.array(us)
    close_figs()
    np.savez_compressed(os.path.join(HERE, "mpc_qp.npz"), **out)
    print("mpc qp", out["p12_P"].shape, out["p30_P"].shape)


def run_rrt(args):
    """One RRT / RRT* plan with np.random.seed(seed): result, the whole tree (insertion order,
    parent as an index) and the next global draw (pins how many draws plan() consumed)."""
    kind, mapname, seed, sample_num, start, goal = args
    pmp = import_reference()
    from python_motion_planning_amd import workloads as wl

    if mapname == "readme":
        env = pmp.Map(51, 31)
        env.update(obs_rect=[list(r) for r in wl.README_MAP_RECT], obs_circ=[list(c) for c in wl.README_MAP_CIRC])
    else:
        env = pmp.Map(512, 512)
        rects, circs = wl.c3_map()
        env.update(obs_rect=rects, obs_circ=circs)
    cls = pmp.RRTStar if kind == "rrt_star" else pmp.RRT
    planner = cls(start, goal, env, sample_num=sample_num)
    np.random.seed(seed)
    cost, path, expand = planner.plan()
    nxt = np.random.random()
    index = {n.current: i for i, n in enumerate(expand)}
    tree = np.array([[n.x, n.y, n.g, index[n.parent] if n.parent in index else -1] for n in expand], np.float64)
    close_figs()
    return dict(cost=float(cost), found=path is not None, path=np.array(path if path else [], np.float64).reshape(-1, 2),
                tree=tree, next=nxt)


def sec_rrt():
    cases = []
    for kind in ("rrt", "rrt_star"):
        for s in range(10):
            cases.append((kind, "readme", s, 10000, (18, 8), (37, 18)))
    for s in range(4):
        cases.append(("rrt_star", "c3", s, 2000, (5, 5), (505, 505)))
    cases.append(("rrt_star", "c3", 11, 5000, (5, 5), (505, 505)))
    with Pool(8) as pool:
        res = pool.map(run_rrt, cases)
    out = {}
    for i, (c, r) in enumerate(zip(cases, res)):
        out[f"c{i}_kind"] = np.array(c[0])
        out[f"c{i}_map"] = np.array(c[1])
        out[f"c{i}_seed"] = np.array(c[2])
        out[f"c{i}_sample_num"] = np.array(c[3])
        out[f"c{i}_start"] = np.array(c[4], np.float64)
        out[f"c{i}_goal"] = np.array(c[5], np.float64)
        for k, v in r.items():
            out[f"c{i}_{k}"] = np.asarray(v)
    out["n_cases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "rrt.npz"), **out)
    print("rrt", [(c[0], c[1], c[2], r["found"], len(r["tree"]), round(r["cost"], 6)) for c, r in zip(cases, res)])


# ----------------------------------------------------------------------------------------------
# Dijkstra / GBFS (2D: dijkstra.py, gbfs.py; 3D: dijkstra3d.py, gbfs3d.py) -- SURVEY.md §8(f) rank 1
def run_graph2d(args):
    occ, start, goal, heur, algo = args
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    cls = dict(dijkstra=pmp.Dijkstra, gbfs=pmp.GBFS)[algo]
    p = cls(tuple(start), tuple(goal), env, heur)
    cost, path, expand = p.plan()
    close_figs()
    return dict(found=bool(path), cost=float(cost) if path else float("nan"), path=[x * H + y for (x, y) in path],
                expand=[n.current[0] * H + n.current[1] for n in expand])


def sec_graph2d(n=120):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(2468)
    cases = []
    occ = wl.readme_grid()
    for algo in ("dijkstra", "gbfs"):
        for heur in ("euclidean", "manhattan"):
            cases.append((occ, (5, 5), (45, 25), heur, algo))
    for i in range(n):
        W = int(rng.integers(8, 81))
        H = int(rng.integers(8, 81))
        dens = float(rng.uniform(0.0, 0.35))
        occ = (rng.random((W, H)) < dens).astype(np.uint8)
        occ[:, 0] = occ[:, H - 1] = 1
        occ[0, :] = occ[W - 1, :] = 1
        free = np.argwhere(occ == 0)
        if len(free) < 2:
            occ[1, 1] = occ[W - 2, H - 2] = 0
            free = np.argwhere(occ == 0)
        s = free[rng.integers(len(free))]
        g = free[rng.integers(len(free))]
        if i % 17 == 5:
            g = s
        heur = "manhattan" if i % 4 == 3 else "euclidean"
        cases.append((occ, tuple(int(v) for v in s), tuple(int(v) for v in g), heur, "gbfs" if i % 2 else "dijkstra"))
    with Pool(8) as pool:
        res = pool.map(run_graph2d, cases, chunksize=4)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "graph2d_small.npz"),
        dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        manhattan=np.array([c[3] == "manhattan" for c in cases]), algo=np.array([c[4] for c in cases]),
        found=np.array([r["found"] for r in res]), cost=np.array([r["cost"] for r in res], np.float64),
        path=path_flat, path_off=path_off, expand=exp_flat, expand_off=exp_off)
    print("graph2d", sum(r["found"] for r in res), "found of", len(cases), "readme costs",
          [r["cost"] for r in res[:4]])


def run_graph3d(args):
    occ, start, goal, algo = args
    pmp = import_reference()
    X, Y, Z = occ.shape
    env = pmp.Grid3D(X, Y, Z)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
    cls = dict(dijkstra=pmp.Dijkstra3D, gbfs=pmp.GBFS3D)[algo]
    p = cls(tuple(start), tuple(goal), env)
    cost, path, expand = p.plan()
    close_figs()
    enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
    return dict(cost=float(cost), path=[enc(t) for t in path], expand=[enc(n.current) for n in expand])


def sec_graph3d():
    from python_motion_planning_amd import workloads as wl

    # (a) the reference's published CSV rows for Dijkstra3D / GBFS3D (every 10th row = distinct seeds)
    rows = []
    with open(os.path.join(REF, "3d_pathfinding_results.csv"), newline="") as f:
        rd = csv.reader(f)
        next(rd)
        for k, r in enumerate(rd):
            if r[1] in ("dijkstra", "gbfs") and k % 10 == 0:
                rows.append(dict(algo=r[1], scenario=r[0], cost=r[3], visited=int(r[4]),
                                 start=list(eval(r[5])), goal=list(eval(r[6])), seed=int(r[7])))  # noqa: S307
    with open(os.path.join(HERE, "graph3d_csv.json"), "w") as f:
        json.dump(rows, f)
    # (b) full reference runs (path + expand order): every scenario, both planners
    cases = []
    for algo in ("dijkstra", "gbfs"):
        for name in wl.SCENARIOS_3D:
            for seed in range(3, 100, 16):
                s, gq = wl.bench3d_query(seed, 21, 15, 11)
                o = wl.SCENARIOS_3D[name](21, 15, 11)
                wl.carve_safety_bubble(o, s, 2)
                wl.carve_safety_bubble(o, gq, 2)
                cases.append((o, s, gq, algo))
    with Pool(8) as pool:
        res = pool.map(run_graph3d, cases)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "graph3d_runs.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        algo=np.array([c[3] for c in cases]), cost=np.array([r["cost"] for r in res]), path=path_flat,
        path_off=path_off, expand=exp_flat, expand_off=exp_off)
    print("graph3d csv rows", len(rows), "runs", len(res))


# ----------------------------------------------------------------------------------------------
# ThetaStar3D / LazyThetaStar3D (theta_star3d.py, lazy_theta_star3d.py) -- SURVEY.md §8(f) rank 4
def run_theta3d(args):
    occ, start, goal, lazy = args
    pmp = import_reference()
    X, Y, Z = occ.shape
    env = pmp.Grid3D(X, Y, Z)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
    from python_motion_planning.global_planner.graph_search import LazyThetaStar3D, ThetaStar3D

    p = (LazyThetaStar3D if lazy else ThetaStar3D)(tuple(start), tuple(goal), env)
    cost, path, expand = p.plan()
    close_figs()
    enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
    return dict(cost=float(cost), path=[enc(t) for t in path], expand=[enc(n.current) for n in expand])


def sec_theta3d():
    from python_motion_planning_amd import workloads as wl

    rows = []
    with open(os.path.join(REF, "3d_pathfinding_results.csv"), newline="") as f:
        rd = csv.reader(f)
        next(rd)
        for k, r in enumerate(rd):
            if r[1] in ("theta_star", "lazy_theta_star") and k % 10 == 0:
                rows.append(dict(algo=r[1], scenario=r[0], cost=r[3], visited=int(r[4]),
                                 start=list(eval(r[5])), goal=list(eval(r[6])), seed=int(r[7])))  # noqa: S307
    with open(os.path.join(HERE, "theta3d_csv.json"), "w") as f:
        json.dump(rows, f)
    cases = []
    for lazy in (False, True):
        for name in wl.SCENARIOS_3D:
            for seed in range(5, 100, 16):
                s, gq = wl.bench3d_query(seed, 21, 15, 11)
                o = wl.SCENARIOS_3D[name](21, 15, 11)
                wl.carve_safety_bubble(o, s, 2)
                wl.carve_safety_bubble(o, gq, 2)
                cases.append((o, s, gq, lazy))
    with Pool(8) as pool:
        res = pool.map(run_theta3d, cases)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "theta3d_runs.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        lazy=np.array([c[3] for c in cases]), cost=np.array([r["cost"] for r in res]), path=path_flat,
        path_off=path_off, expand=exp_flat, expand_off=exp_off)
    print("theta3d csv rows", len(rows), "runs", len(res))


# ----------------------------------------------------------------------------------------------
# ThetaStar / LazyThetaStar 2D (theta_star.py, lazy_theta_star.py) -- SURVEY.md §8(f) rank 4
def run_theta2d(args):
    occ, start, goal, heur, algo = args
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    cls = dict(theta_star=pmp.ThetaStar, lazy_theta_star=pmp.LazyThetaStar)[algo]
    p = cls(tuple(start), tuple(goal), env, heur)
    cost, path, expand = p.plan()
    close_figs()
    return dict(found=bool(path), cost=float(cost) if path else float("nan"), path=[x * H + y for (x, y) in path],
                expand=[n.current[0] * H + n.current[1] for n in expand],
                exp_parent=[n.parent[0] * H + n.parent[1] for n in expand], exp_g=[float(n.g) for n in expand])


def sec_theta2d(n=160):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(1357)
    cases = []
    occ = wl.readme_grid()
    for algo in ("theta_star", "lazy_theta_star"):
        for heur in ("euclidean", "manhattan"):
            cases.append((occ, (5, 5), (45, 25), heur, algo))
    for i in range(n):
        big = i % 20 == 7
        W = int(rng.integers(96, 161)) if big else int(rng.integers(8, 81))
        H = int(rng.integers(96, 161)) if big else int(rng.integers(8, 81))
        dens = float(rng.uniform(0.0, 0.35))
        occ = (rng.random((W, H)) < dens).astype(np.uint8)
        occ[:, 0] = occ[:, H - 1] = 1
        occ[0, :] = occ[W - 1, :] = 1
        free = np.argwhere(occ == 0)
        if len(free) < 2:
            occ[1, 1] = occ[W - 2, H - 2] = 0
            free = np.argwhere(occ == 0)
        s = free[rng.integers(len(free))]
        g = free[rng.integers(len(free))]
        if i % 17 == 5:
            g = s
        heur = "manhattan" if i % 4 == 3 else "euclidean"
        cases.append((occ, tuple(int(v) for v in s), tuple(int(v) for v in g), heur,
                      "lazy_theta_star" if i % 2 else "theta_star"))
    with Pool(8) as pool:
        res = pool.map(run_theta2d, cases, chunksize=2)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    exp_flat, exp_off = ragged([r["expand"] for r in res])
    par_flat, _ = ragged([r["exp_parent"] for r in res])
    g_flat, _ = ragged([r["exp_g"] for r in res], np.float64)
    np.savez_compressed(
        os.path.join(HERE, "theta2d_small.npz"),
        dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        manhattan=np.array([c[3] == "manhattan" for c in cases]), algo=np.array([c[4] for c in cases]),
        found=np.array([r["found"] for r in res]), cost=np.array([r["cost"] for r in res], np.float64),
        path=path_flat, path_off=path_off, expand=exp_flat, expand_off=exp_off, exp_parent=par_flat, exp_g=g_flat)
    print("theta2d", sum(r["found"] for r in res), "found of", len(cases), "readme costs",
          [r["cost"] for r in res[:4]])


# ----------------------------------------------------------------------------------------------
# LPAStar (lpa_star.py) -- SURVEY.md §8(f) rank 3 (the initial computeShortestPath + extractPath)
def run_lpa(args):
    occ, start, goal, heur = args[:4]
    lite = len(args) > 4 and args[4]
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    p = (pmp.DStarLite if lite else pmp.LPAStar)(tuple(start), tuple(goal), env, heur)
    try:
        cost, path, _ = p.plan()
        err = ""
    except (ValueError, KeyError) as e:
        cost, path, err = float("nan"), [], type(e).__name__
    close_figs()
    return dict(cost=float(cost), path=[x * H + y for (x, y) in path], n_expand=len(p.EXPAND), err=err)


def sec_lpa(n=120, lite=False):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(8642)
    cases = [(wl.readme_grid(), (5, 5), (45, 25), "euclidean"), (wl.readme_grid(), (5, 5), (45, 25), "manhattan")]
    for i in range(n):
        W = int(rng.integers(6, 41))
        H = int(rng.integers(6, 41))
        dens = float(rng.uniform(0.0, 0.35))
        occ = (rng.random((W, H)) < dens).astype(np.uint8)
        occ[:, 0] = occ[:, H - 1] = 1
        occ[0, :] = occ[W - 1, :] = 1
        free = np.argwhere(occ == 0)
        if len(free) < 2:
            occ[1, 1] = occ[W - 2, H - 2] = 0
            free = np.argwhere(occ == 0)
        s = free[rng.integers(len(free))]
        g = free[rng.integers(len(free))]
        if i % 19 == 4:
            g = s
        cases.append((occ, tuple(int(v) for v in s), tuple(int(v) for v in g), "manhattan" if i % 4 == 3 else "euclidean"))
    cases = [c + (lite,) for c in cases]
    with Pool(8) as pool:
        res = pool.map(run_lpa, cases, chunksize=2)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    np.savez_compressed(
        os.path.join(HERE, "dstarlite_small.npz" if lite else "lpa_small.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        manhattan=np.array([c[3] == "manhattan" for c in cases]), cost=np.array([r["cost"] for r in res]),
        path=path_flat, path_off=path_off, n_expand=np.array([r["n_expand"] for r in res], np.int64),
        err=np.array([r["err"] for r in res]))
    print("dstarlite" if lite else "lpa", sum(1 for r in res if r["path"]), "with path,", sum(1 for r in res if r["err"]), "raise, of", len(res),
          "readme", res[0]["cost"], res[0]["n_expand"])


# LPAStar.OnPress replanning (lpa_star.py:101-137) without the figure: the same edits on the planner
def dstarlite_onpress(p, x, y):
    """DStarLite.OnPress (d_star_lite.py:61-97) without the figure and the prints."""
    cur_start, new_start = p.start, p.start
    update_start = True
    cost, count = 0, 0
    path = [p.start.current]
    p.EXPAND = []
    while cur_start != p.goal:
        neighbors = [node_n for node_n in p.getNeighbor(cur_start) if not p.isCollision(cur_start, node_n)]
        next_node = min(neighbors, key=lambda n: n.g)
        path.append(next_node.current)
        cost += p.cost(cur_start, next_node)
        count += 1
        cur_start = next_node
        if count > 20000:
            raise RuntimeError("walk does not end")
        if update_start:
            update_start = False
            p.km = p.h(cur_start, new_start)
            new_start = cur_start
            node_change = p.map[(x, y)]
            if (x, y) not in p.obstacles:
                p.obstacles.add((x, y))
            else:
                p.obstacles.remove((x, y))
                p.updateVertex(node_change)
            p.env.update(p.obstacles)
            for node_n in p.getNeighbor(node_change):
                p.updateVertex(node_n)
            p.computeShortestPath()
    return cost, path


def run_lpa_replan(args):
    occ, start, goal, toggles = args[:4]
    lite = len(args) > 4 and args[4]
    pmp = import_reference()
    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    p = (pmp.DStarLite if lite else pmp.LPAStar)(tuple(start), tuple(goal), env, "euclidean")
    costs, nexp, errs, path = [], [], [], []
    try:
        cost, path, _ = p.plan()
        costs.append(float(cost)); nexp.append(len(p.EXPAND)); errs.append("")
        for (x, y) in toggles:
            if lite:
                cost, path = dstarlite_onpress(p, x, y)
                costs.append(float(cost)); nexp.append(len(p.EXPAND)); errs.append("")
                continue
            p.EXPAND = []
            node_change = p.map[(x, y)]
            if (x, y) not in p.obstacles:
                p.obstacles.add((x, y))
            else:
                p.obstacles.remove((x, y))
                p.updateVertex(node_change)
            p.env.update(p.obstacles)
            for node_n in p.getNeighbor(node_change):
                p.updateVertex(node_n)
            cost, path, _ = p.plan()
            costs.append(float(cost)); nexp.append(len(p.EXPAND)); errs.append("")
    except (ValueError, KeyError, RuntimeError) as e:
        costs.append(float("nan")); nexp.append(len(p.EXPAND)); errs.append(type(e).__name__)
        path = []
    close_figs()
    return dict(cost=costs, nexp=nexp, err=errs, path=[x * H + y for (x, y) in path])


def sec_lpa_replan(n=60, nt=4, lite=False):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(9753)
    cases = []
    for i in range(n):
        if i < 4:
            occ = wl.readme_grid()
        else:
            W, H = int(rng.integers(10, 41)), int(rng.integers(10, 41))
            occ = (rng.random((W, H)) < float(rng.uniform(0.0, 0.3))).astype(np.uint8)
            occ[:, 0] = occ[:, -1] = 1
            occ[0, :] = occ[-1, :] = 1
        W, H = occ.shape
        free = np.argwhere(occ == 0)
        s = tuple(int(v) for v in free[rng.integers(len(free))])
        g = tuple(int(v) for v in free[rng.integers(len(free))])
        if i < 4:
            s, g = (5, 5), (45, 25)
        inner = np.argwhere(np.ones((W - 2, H - 2), bool)) + 1
        tg = [tuple(int(v) for v in inner[rng.integers(len(inner))]) for _ in range(nt)]
        cases.append((occ, s, g, tg, lite))
    with Pool(8) as pool:
        res = pool.map(run_lpa_replan, cases, chunksize=2)
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([r["path"] for r in res])
    pad = lambda v, f: [list(x) + [f] * (nt + 1 - len(x)) for x in v]  # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "dstarlite_replan.npz" if lite else "lpa_replan.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        toggles=np.array([c[3] for c in cases], np.int32),
        cost=np.array(pad([r["cost"] for r in res], float("nan"))), nexp=np.array(pad([r["nexp"] for r in res], 0)),
        err=np.array(pad([r["err"] for r in res], "-")), path=path_flat, path_off=path_off)
    print("dstarlite_replan" if lite else "lpa_replan", len(res), "cases;", sum(1 for r in res if r["err"][-1]), "raise")


# ----------------------------------------------------------------------------------------------
# DStar3D plan + apply_dynamic_obstacles (d_star3d.py:100-149) -- SURVEY.md §8(f) rank 3
def run_dstar3d(args):
    occ, start, goal, rounds = args
    pmp = import_reference()
    X, Y, Z = occ.shape
    env = pmp.Grid3D(X, Y, Z)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
    p = pmp.DStar3D(tuple(start), tuple(goal), env)
    enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
    cost, path, expand = p.plan()
    out = dict(cost=[float(cost)], path=[[enc(t) for t in path]], nexp=[len(expand)])
    for blk in rounds:
        cost, path = p.apply_dynamic_obstacles([tuple(int(v) for v in b) for b in blk])
        out["cost"].append(float(cost))
        out["path"].append([enc(t) for t in path])
        out["nexp"].append(len(p.EXPAND))
    close_figs()
    return out


def sec_dstar3d(n_per=8, nr=3):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(4242)
    cases = []
    for name in wl.SCENARIOS_3D:
        for j in range(n_per):
            X, Y, Z = (21, 15, 11) if j % 4 else (26, 20, 16)
            seed = int(rng.integers(1000))
            s, g = wl.bench3d_query(seed, X, Y, Z)
            o = wl.SCENARIOS_3D[name](X, Y, Z)
            wl.carve_safety_bubble(o, s, 2 if X == 21 else 1)
            wl.carve_safety_bubble(o, g, 2 if X == 21 else 1)
            inner = np.argwhere(o[1:-1, 1:-1, 1:-1] == 0) + 1
            rounds = []
            for _ in range(nr):
                blk = [inner[rng.integers(len(inner))] for _ in range(3)]
                rounds.append([[int(v) for v in b] for b in blk])
            cases.append((o, s, g, rounds))
    # blocks on the planned path (forces the modify / processState repair): taken from a first plan
    res = []
    with Pool(8) as pool:
        first = pool.map(run_dstar3d, [(c[0], c[1], c[2], []) for c in cases])
        jobs = []
        for c, f in zip(cases, first):
            o, s, g, rounds = c
            X, Y, Z = o.shape
            path = f["path"][0]
            if len(path) > 3:
                v = path[len(path) // 2]
                rounds[0][0] = [v // (Y * Z), (v // Z) % Y, v % Z]
            jobs.append(pool.apply_async(run_dstar3d, (c,)))
        keep = []
        for c, j in zip(cases, jobs):
            try:
                res.append(j.get(timeout=120))
                keep.append(c)
            except Exception as e:  # a walk that never ends in the reference (no step bound there)
                print("dstar3d case dropped:", type(e).__name__)
        cases = keep
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    paths = [p for r in res for p in r["path"]]
    path_flat, path_off = ragged(paths)
    np.savez_compressed(
        os.path.join(HERE, "dstar3d_runs.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        blocks=np.array([c[3] for c in cases], np.int32), cost=np.array([r["cost"] for r in res]),
        nexp=np.array([r["nexp"] for r in res], np.int64), path=path_flat, path_off=path_off)
    # the reference's published CSV rows for DStar3D (every 10th row = distinct seeds, 120 inf rows in all)
    rows = []
    with open(os.path.join(REF, "3d_pathfinding_results.csv"), newline="") as f:
        rd = csv.reader(f)
        next(rd)
        for k, r in enumerate(rd):
            if r[1] == "dstar" and k % 10 == 0:
                rows.append(dict(algo=r[1], scenario=r[0], cost=r[3], visited=int(r[4]),
                                 start=list(eval(r[5])), goal=list(eval(r[6])), seed=int(r[7])))  # noqa: S307
    with open(os.path.join(HERE, "dstar3d_csv.json"), "w") as f:
        json.dump(rows, f)
    print("dstar3d runs", len(res), "csv rows", len(rows), "inf rounds",
          sum(1 for r in res for c in r["cost"] if math.isinf(c)))


# ----------------------------------------------------------------------------------------------
# DStar.plan + OnPress(event) (d_star.py:75-134): the reference's own OnPress with a stand-in event
# and a recording plot (the walk's path / cost are what it hands to plot.animation)
def run_dstar_onpress(args):
    occ, start, goal, presses = args
    pmp = import_reference()
    import contextlib
    import io

    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))
    p = pmp.DStar(tuple(start), tuple(goal), env)
    out = dict(cost=[], path=[], nexp=[], kind=[])
    try:
        cost, path, _ = p.plan()
    except Exception as e:  # noqa: BLE001  unreachable start: AttributeError (d_star.py:234)
        out["cost"].append(float("nan")); out["path"].append([]); out["nexp"].append(len(p.EXPAND))
        out["kind"].append(type(e).__name__)
        close_figs()
        return out
    out["cost"].append(float(cost)); out["path"].append([x * H + y for (x, y) in path])
    out["nexp"].append(len(p.EXPAND)); out["kind"].append("")
    p.plot = unittest.mock.MagicMock()
    for (x, y) in presses:
        ev = types.SimpleNamespace(xdata=float(x) + 0.25, ydata=float(y) + 0.25)
        p.plot.animation.reset_mock()
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                p.OnPress(ev)
        except Exception as e:  # noqa: BLE001  KeyError on a parentless node, AttributeError on an emptied OPEN
            out["cost"].append(float("nan")); out["path"].append([]); out["nexp"].append(len(p.EXPAND))
            out["kind"].append(type(e).__name__)
            break
        if p.plot.animation.called:
            wpath, _, wcost, _ = p.plot.animation.call_args[0]
            out["cost"].append(float(wcost)); out["path"].append([x * H + y for (x, y) in wpath])
            out["nexp"].append(len(p.EXPAND)); out["kind"].append("")
        else:
            out["cost"].append(0.0); out["path"].append([]); out["nexp"].append(len(p.EXPAND)); out["kind"].append("noop")
    close_figs()
    return out


def sec_dstar_onpress(n=48, npress=4):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(31337)
    cases = []
    for i in range(n):
        if i < 6:
            occ = wl.readme_grid()
            s, g = ((5, 5), (45, 25)) if i < 3 else tuple(tuple(int(v) for v in np.argwhere(occ == 0)[rng.integers(
                (occ == 0).sum())]) for _ in range(2))
        else:
            W, H = int(rng.integers(10, 41)), int(rng.integers(10, 41))
            occ = wl.random_grid(W, H, float(rng.uniform(0.0, 0.25)), int(rng.integers(1 << 30)))
            free = np.argwhere(occ == 0)
            s = tuple(int(v) for v in free[rng.integers(len(free))])
            g = tuple(int(v) for v in free[rng.integers(len(free))])
        cases.append([occ, s, g, None])
    res = []
    with Pool(8) as pool:
        first = pool.map(run_dstar_onpress, [(c[0], c[1], c[2], []) for c in cases])
        jobs = []
        for c, f in zip(cases, first):
            occ, s, g, _ = c
            W, H = occ.shape
            path = f["path"][0]
            pr = []
            for k in range(npress):
                if path and k < 2 and len(path) > 4:  # on the planned path: forces the modify / processState repair
                    v = path[int(rng.integers(1, len(path) - 1))]
                    pr.append((v // H, v % H))
                else:  # anywhere (off-path, obstacles and off-grid presses included)
                    pr.append((int(rng.integers(-1, W + 1)), int(rng.integers(-1, H + 1))))
            c[3] = pr
            jobs.append(pool.apply_async(run_dstar_onpress, (tuple(c),)))
        keep = []
        for c, j in zip(cases, jobs):
            try:
                res.append(j.get(timeout=60))
                keep.append(c)
            except Exception as e:  # noqa: BLE001  an OnPress walk that never ends in the reference
                print("dstar onpress case dropped:", type(e).__name__)
        cases = keep
    R = npress + 1
    pad = lambda v, f: list(v) + [f] * (R - len(v))  # noqa: E731
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([p for r in res for p in pad(r["path"], [])])
    np.savez_compressed(
        os.path.join(HERE, "dstar_onpress.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        presses=np.array([c[3] for c in cases], np.int32),
        cost=np.array([pad(r["cost"], float("nan")) for r in res]), nexp=np.array([pad(r["nexp"], -1) for r in res]),
        kind=np.array([pad(r["kind"], "-") for r in res]), path=path_flat, path_off=path_off)
    kinds = [k for r in res for k in r["kind"]]
    print("dstar_onpress", len(res), "cases;", {k: kinds.count(k) for k in set(kinds)})


# ----------------------------------------------------------------------------------------------
# LPAStar3D plan + apply_change (lpa_star3d.py:78-124) -- SURVEY.md §8(f) rank 3
def run_lpastar3d(args):
    occ, start, goal, changes = args
    pmp = import_reference()
    X, Y, Z = occ.shape
    env = pmp.Grid3D(X, Y, Z)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
    p = pmp.LPAStar3D(tuple(start), tuple(goal), env)
    enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
    cost, path, expand = p.plan()
    out = dict(cost=[float(cost)], path=[[enc(t) for t in path]], nexp=[len(expand)])
    for (x, y, z, mode) in changes:
        blocked = None if mode == 0 else (mode == 1)
        cost, path, expand = p.apply_change((int(x), int(y), int(z)), blocked)
        out["cost"].append(float(cost))
        out["path"].append([enc(t) for t in path])
        out["nexp"].append(len(expand))
    close_figs()
    return out


def sec_lpastar3d(n_per=8, nr=4):
    from python_motion_planning_amd import workloads as wl

    rng = np.random.default_rng(5151)
    cases = []
    for name in wl.SCENARIOS_3D:
        for j in range(n_per):
            X, Y, Z = (21, 15, 11) if j % 4 else (26, 20, 16)
            seed = int(rng.integers(1000))
            s, g = wl.bench3d_query(seed, X, Y, Z)
            if j == 7 and name == "empty":
                g = s  # start == goal: map[goal] overwrites map[start] (lpa_star3d.py:62-63)
            o = wl.SCENARIOS_3D[name](X, Y, Z)
            wl.carve_safety_bubble(o, s, 2 if X == 21 else 1)
            wl.carve_safety_bubble(o, g, 2 if X == 21 else 1)
            cases.append([o, s, g, None])
    res = []
    with Pool(8) as pool:
        first = pool.map(run_lpastar3d, [(c[0], c[1], c[2], []) for c in cases])
        jobs = []
        for c, f in zip(cases, first):
            o, s, g, _ = c
            X, Y, Z = o.shape
            path = f["path"][0]
            ch = []
            for k in range(nr):
                if k < 2 and len(path) > 3:  # block a voxel of the current path
                    v = path[int(rng.integers(1, len(path) - 1))]
                    ch.append([v // (Y * Z), (v // Z) % Y, v % Z, 1 if k == 0 else 0])
                elif k == 2:  # free an obstacle voxel (the wall or a scenario block)
                    obs = np.argwhere(o)
                    v = obs[rng.integers(len(obs))]
                    ch.append([int(v[0]), int(v[1]), int(v[2]), 2])
                else:  # toggle anywhere (off-grid included)
                    ch.append([int(rng.integers(-1, X + 1)), int(rng.integers(0, Y)), int(rng.integers(0, Z)), 0])
            c[3] = ch
            jobs.append(pool.apply_async(run_lpastar3d, (tuple(c),)))
        keep = []
        for c, j in zip(cases, jobs):
            try:
                res.append(j.get(timeout=180))
                keep.append(c)
            except Exception as e:  # noqa: BLE001
                print("lpastar3d case dropped:", type(e).__name__, e)
        cases = keep
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    path_flat, path_off = ragged([p for r in res for p in r["path"]])
    np.savez_compressed(
        os.path.join(HERE, "lpastar3d_runs.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        changes=np.array([c[3] for c in cases], np.int32), cost=np.array([r["cost"] for r in res]),
        nexp=np.array([r["nexp"] for r in res], np.int64), path=path_flat, path_off=path_off)
    rows = []
    with open(os.path.join(REF, "3d_pathfinding_results.csv"), newline="") as f:
        rd = csv.reader(f)
        next(rd)
        for k, r in enumerate(rd):
            if r[1] == "lpastar" and k % 10 == 0:
                rows.append(dict(algo=r[1], scenario=r[0], cost=r[3], visited=int(r[4]),
                                 start=list(eval(r[5])), goal=list(eval(r[6])), seed=int(r[7])))  # noqa: S307
    with open(os.path.join(HERE, "lpastar3d_csv.json"), "w") as f:
        json.dump(rows, f)
    print("lpastar3d runs", len(res), "csv rows", len(rows), "empty paths",
          sum(1 for r in res for p in r["path"] if not p))


# ----------------------------------------------------------------------------------------------
# the CLOSED Node objects AStar / Dijkstra / GBFS return (a_star.py:64): current, parent, g, h with
# their Python types (g stays int while every step is straight) -- pins the native marshalling
def sec_astar_nodes():
    from python_motion_planning_amd import workloads as wl

    pmp = import_reference()
    occ = wl.readme_grid()
    env = pmp.Grid(51, 31)
    env.update(obstacles_of(occ))
    out = []
    for name, cls in (("astar", pmp.AStar), ("dijkstra", pmp.Dijkstra), ("gbfs", pmp.GBFS)):
        for heur in ("euclidean", "manhattan"):
            cost, path, expand = cls((5, 5), (45, 25), env, heur).plan()
            out.append(dict(algo=name, heuristic=heur, cost=repr(cost),
                            nodes=[[list(n.current), list(n.parent), repr(n.g), type(n.g).__name__, repr(n.h),
                                    type(n.h).__name__] for n in expand]))
    close_figs()
    with open(os.path.join(HERE, "astar_nodes.json"), "w") as f:
        json.dump(out, f)
    print("astar nodes", [(o["algo"], o["heuristic"], len(o["nodes"])) for o in out])


# ----------------------------------------------------------------------------------------------
# TimeOptimalTrajectory3D (trajectory/time_optimal_trajectory.py:8-353) on C5 paths: the 3d_example
# set-up (examples/3d_example.py:104-128: constraints, path_resolution 0.05, path from AStar3D.plan)
# plus the defaults (2 / 1 m/s(^2), resolution 0.01) and the 2- and 3-waypoint special cases of
# scipy's CubicSpline
def run_totp(args):
    path, vmax, amax, tstep, res = args
    pmp = import_reference()
    from python_motion_planning.trajectory import TimeOptimalTrajectory3D, TrajectoryConstraints

    cons = None if vmax is None else TrajectoryConstraints(max_velocity=np.array(vmax), max_acceleration=np.array(amax),
                                                           min_time_step=tstep)
    tr = TimeOptimalTrajectory3D(path=[tuple(p) for p in path], constraints=cons, path_resolution=res)
    pts = tr.generate()
    nan = float("nan")
    return dict(total_time=float(tr.total_time), s_values=np.asarray(tr.s_values, np.float64),
                s_dot=np.asarray(tr.s_dot_profile, np.float64), s_ddot=np.asarray(tr.s_ddot_profile, np.float64),
                time=np.asarray(tr.time_profile, np.float64),
                pts=np.array([[q.time, *q.position, *q.velocity, *q.acceleration,
                               nan if q.yaw is None else q.yaw, nan if q.yaw_rate is None else q.yaw_rate]
                              for q in pts], np.float64))


def sec_totp():
    from python_motion_planning_amd import workloads as wl

    pmp = import_reference()
    ex = ([2.0, 2.0, 1.5], [1.5, 1.5, 1.0], 0.05, 0.05)  # 3d_example.py:104-109, :124-128
    cases = []
    for seed in range(32):
        s, gq = wl.bench3d_query(seed, 26, 20, 16)
        o = wl.SCENARIOS_3D["door"](26, 20, 16)
        wl.carve_safety_bubble(o, s, 1)
        wl.carve_safety_bubble(o, gq, 1)
        env = pmp.Grid3D(26, 20, 16)
        env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(o)})
        cost, path, _ = pmp.AStar3D(tuple(s), tuple(gq), env).plan()
        close_figs()
        if len(path) >= 2:
            cases.append((np.array(path, np.float64),) + (ex if seed % 4 else (None, None, None, 0.01)))
    # scipy CubicSpline special cases (n = 2: line, n = 3: parabola) and a short diagonal run
    cases.append((np.array([[1, 1, 1], [2, 2, 1]], np.float64),) + ex)
    cases.append((np.array([[1, 1, 1], [2, 2, 1], [3, 2, 2]], np.float64),) + ex)
    cases.append((np.array([[5, 5, 5], [4, 4, 4], [3, 3, 3], [2, 3, 3], [1, 3, 4]], np.float64),) + ex)
    cases.append((np.array([[5, 5, 5], [4, 4, 4], [3, 3, 3], [2, 3, 3], [1, 3, 4]], np.float64), None, None, None, 0.01))
    with Pool(8) as pool:
        res = pool.map(run_totp, cases)
    path_flat, path_off = ragged([c[0] for c in cases], np.float64)
    prof_off = np.concatenate([[0], np.cumsum([len(r["s_values"]) for r in res])]).astype(np.int64)
    # trajectory points: all of them up to 1500 per case, else every 10th and the last (fixture size);
    # pts_idx = the point's index in the reference's list, n_pts = the list's length
    keep = [np.arange(len(r["pts"])) if len(r["pts"]) <= 1500 else
            np.unique(np.append(np.arange(0, len(r["pts"]), 10), len(r["pts"]) - 1)) for r in res]
    pts_off = np.concatenate([[0], np.cumsum([len(k) for k in keep])]).astype(np.int64)
    cons = np.array([(c[1] or [2.0] * 3) + (c[2] or [1.0] * 3) + [c[3] if c[3] is not None else 0.01, c[4]]
                     for c in cases], np.float64)
    np.savez_compressed(
        os.path.join(HERE, "totp.npz"), path=path_flat.reshape(-1, 3), path_off=path_off, cons=cons,
        total_time=np.array([r["total_time"] for r in res]), prof_off=prof_off,
        s_values=np.concatenate([r["s_values"] for r in res]), s_dot=np.concatenate([r["s_dot"] for r in res]),
        s_ddot=np.concatenate([r["s_ddot"] for r in res]), time=np.concatenate([r["time"] for r in res]),
        pts_off=pts_off, pts=np.concatenate([r["pts"][k] for r, k in zip(res, keep)]),
        pts_idx=np.concatenate(keep).astype(np.int32), n_pts=np.array([len(r["pts"]) for r in res], np.int32))
    print("totp cases", len(cases), "samples", prof_off[-1], "points", pts_off[-1])


def run_dstar_nowall(args):
    """run_dstar_onpress on a grid whose border cells are free: getNeighbor (d_star.py:276-291) of a
    border node looks up an out-of-grid key and raises KeyError -- recorded with its key."""
    occ, start, goal, presses = args
    pmp = import_reference()
    import contextlib
    import io

    W, H = occ.shape
    env = pmp.Grid(W, H)
    env.update(obstacles_of(occ))  # no border walls
    p = pmp.DStar(tuple(start), tuple(goal), env)
    out = dict(cost=[], path=[], nexp=[], kind=[], key=[])

    def fail(e):
        out["cost"].append(float("nan")); out["path"].append([]); out["nexp"].append(len(p.EXPAND))
        out["kind"].append(type(e).__name__)
        k = e.args[0] if isinstance(e, KeyError) and e.args else None
        out["key"].append(tuple(int(v) for v in k) if isinstance(k, tuple) else (-1, -1))

    try:
        cost, path, _ = p.plan()
    except Exception as e:  # noqa: BLE001
        fail(e)
        close_figs()
        return out
    out["cost"].append(float(cost)); out["path"].append([x * H + y for (x, y) in path])
    out["nexp"].append(len(p.EXPAND)); out["kind"].append(""); out["key"].append((-1, -1))
    p.plot = unittest.mock.MagicMock()
    for (x, y) in presses:
        ev = types.SimpleNamespace(xdata=float(x) + 0.25, ydata=float(y) + 0.25)
        p.plot.animation.reset_mock()
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                p.OnPress(ev)
        except Exception as e:  # noqa: BLE001
            fail(e)
            break
        if p.plot.animation.called:
            wpath, _, wcost, _ = p.plot.animation.call_args[0]
            out["cost"].append(float(wcost)); out["path"].append([x * H + y for (x, y) in wpath])
            out["nexp"].append(len(p.EXPAND)); out["kind"].append(""); out["key"].append((-1, -1))
        else:
            out["cost"].append(0.0); out["path"].append([]); out["nexp"].append(len(p.EXPAND)); out["kind"].append("noop")
            out["key"].append((-1, -1))
    close_figs()
    return out


def sec_dstar_nowall(n=48, npress=3):
    """D* plan + OnPress on grids without border walls (round 6): the border KeyError."""
    rng = np.random.default_rng(4242)
    cases = []
    for i in range(n):
        W, H = int(rng.integers(8, 31)), int(rng.integers(8, 31))
        occ = (rng.random((W, H)) < float(rng.uniform(0.0, 0.25))).astype(np.uint8)
        free = np.argwhere(occ == 0)
        if i % 2:  # start and goal near the middle: the plan can finish before any border node
            mid = free[(np.abs(free[:, 0] - W // 2) <= 2) & (np.abs(free[:, 1] - H // 2) <= 2)]
            pick = mid if len(mid) >= 2 else free
        else:
            pick = free
        s = tuple(int(v) for v in pick[rng.integers(len(pick))])
        g = tuple(int(v) for v in pick[rng.integers(len(pick))])
        cases.append([occ, s, g, None])
    with Pool(8) as pool:
        first = pool.map(run_dstar_nowall, [(c[0], c[1], c[2], []) for c in cases])
        for c, f in zip(cases, first):
            W, H = c[0].shape
            path = f["path"][0]
            pr = []
            for k in range(npress):
                if path and len(path) > 3:
                    v = path[int(rng.integers(1, len(path) - 1))]
                    pr.append((v // H, v % H))
                else:
                    pr.append((int(rng.integers(0, W)), int(rng.integers(0, H))))
            c[3] = pr
        res = pool.map(run_dstar_nowall, [tuple(c) for c in cases])
    dims = np.array([c[0].shape for c in cases], np.int32)
    occ_flat, occ_off = ragged([np.packbits(c[0].ravel()) for c in cases], np.uint8)
    R = npress + 1
    kinds = np.full((n, R), "", dtype="<U16")
    keys = np.full((n, R, 2), -1, np.int32)
    cost = np.full((n, R), np.nan)
    nexp = np.full((n, R), -1, np.int64)
    paths = []
    for i, r in enumerate(res):
        for k in range(R):
            if k < len(r["kind"]):
                kinds[i, k] = r["kind"][k]
                keys[i, k] = r["key"][k]
                cost[i, k] = r["cost"][k]
                nexp[i, k] = r["nexp"][k]
                paths.append(r["path"][k])
            else:
                kinds[i, k] = "notrun"
                paths.append([])
    path_flat, path_off = ragged(paths)
    np.savez_compressed(
        os.path.join(HERE, "dstar_nowall.npz"), dims=dims, occ_bits=occ_flat, occ_off=occ_off,
        start=np.array([c[1] for c in cases], np.int32), goal=np.array([c[2] for c in cases], np.int32),
        presses=np.array([c[3] for c in cases], np.int32), kind=kinds, key=keys, cost=cost, nexp=nexp,
        path=path_flat, path_off=path_off)
    print("dstar_nowall", [list(r["kind"]) for r in res])


SECTIONS = dict(dstar_nowall=sec_dstar_nowall, rrt=sec_rrt, mpc=sec_mpc, dwa=sec_dwa, local_plans=sec_local_plans, lqr=sec_lqr, astar_readme=sec_astar_readme, astar_small=sec_astar_small, astar_1024=sec_astar_1024,
                dstar=sec_dstar, astar3d=sec_astar3d,
                graph2d=sec_graph2d, graph3d=sec_graph3d, theta3d=sec_theta3d, theta2d=sec_theta2d, lpa=sec_lpa,
                dstarlite=lambda: sec_lpa(lite=True), lpa_replan=sec_lpa_replan,
                dstarlite_replan=lambda: sec_lpa_replan(lite=True), dstar3d=sec_dstar3d,
                dstar_onpress=sec_dstar_onpress, lpastar3d=sec_lpastar3d,
                astar_nodes=sec_astar_nodes, totp=sec_totp)

if __name__ == "__main__":
    want = sys.argv[1:] or list(SECTIONS)
    for w in want:
        SECTIONS[w]()
