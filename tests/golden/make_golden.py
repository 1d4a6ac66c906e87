"""Generate golden vectors by running the REFERENCE (python_motion_planning @ /root/reference).

Run in the build container only (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py [section ...]

Sections: astar_readme astar_small astar_1024 dstar astar3d rrt dwa lqr mpc hypot
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


SECTIONS = dict(astar_readme=sec_astar_readme, astar_small=sec_astar_small, astar_1024=sec_astar_1024,
                dstar=sec_dstar, astar3d=sec_astar3d)

if __name__ == "__main__":
    want = sys.argv[1:] or list(SECTIONS)
    for w in want:
        SECTIONS[w]()
