"""HIP LPAStar3D (lpa3d.hip via the C-ABI): plan() and apply_change() rounds against the
reference's published CSV rows, replayed reference runs and the oracle (lpa_star3d.py:40-225).

Bar: bit-exact -- every call's cost, len(EXPAND) and path."""
import os

import numpy as np
import pytest

from golden_io import grid_cases, load_json, seg

pytestmark = pytest.mark.gpu


def _csv_batch(rows):
    from python_motion_planning_amd import workloads as wl

    occ = np.zeros((len(rows), 21, 15, 11), np.uint8)
    S = np.zeros((len(rows), 3), np.int32)
    G = np.zeros((len(rows), 3), np.int32)
    for i, r in enumerate(rows):
        s, g = wl.bench3d_query(r["seed"], 21, 15, 11)
        o = wl.SCENARIOS_3D[r["scenario"]](21, 15, 11)
        wl.carve_safety_bubble(o, s, 2)
        wl.carve_safety_bubble(o, g, 2)
        occ[i], S[i], G[i] = o, s, g
    return occ, S, G


def test_lpastar3d_published_csv_rows():
    """The 500 distinct LPAStar3D rows of 3d_pathfinding_results.csv in one launch."""
    from python_motion_planning_amd import batch

    rows = load_json("lpastar3d_csv.json")
    occ, S, G = _csv_batch(rows)
    out = batch.lpastar3d_batch(occ, S, G)
    cost = out["cost"][:, 0].cpu().numpy()
    ne = out["n_expanded"][:, 0].cpu().numpy()
    for i, r in enumerate(rows):
        assert repr(float(cost[i])) == r["cost"], (i, r)
        assert ne[i] == r["visited"], (i, r)


def test_lpastar3d_apply_change_against_reference():
    """40 replayed reference sessions: plan() + 4 apply_change() calls each (block on the path,
    toggle on the path, free an obstacle, toggle anywhere), one launch per session."""
    from python_motion_planning_amd import batch

    n = 0
    for i, occ, z in grid_cases("lpastar3d_runs.npz"):
        R = z["changes"].shape[1] + 1
        out = batch.lpastar3d_batch(occ, z["start"][i][None], z["goal"][i][None], z["changes"][i][None])
        for r in range(R):
            assert float(out["cost"][0, r]) == z["cost"][i][r], (i, r)
            assert int(out["n_expanded"][0, r]) == z["nexp"][i][r], (i, r)
            pl = int(out["path_len"][0, r])
            assert np.array_equal(out["path"][0, r, :pl].cpu().numpy(), seg(z["path"], z["path_off"], i * R + r)), (i, r)
        n += 1
    assert n >= 38


def test_lpastar3d_c5_batch_against_oracle():
    """C5 shape (26x20x16 door): 256 queries, 3 changes each (two blocks on the planned path, a
    toggle anywhere), every output against the oracle."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, s, g = wl.c5_workload(256)
    X, Y, Z = occ.shape[1:]
    r0 = batch.lpastar3d_batch(occ, s, g)
    pl0, p0 = r0["path_len"][:, 0].cpu().numpy(), r0["path"][:, 0].cpu().numpy()
    rng = np.random.default_rng(17)
    ch = np.zeros((len(s), 3, 4), np.int32)
    for q in range(len(s)):
        for k in range(3):
            if k < 2 and pl0[q] > 3:
                v = int(p0[q, rng.integers(1, pl0[q] - 1)])
                ch[q, k] = (v // (Y * Z), (v // Z) % Y, v % Z, 1)
            else:
                ch[q, k] = (rng.integers(1, X - 1), rng.integers(1, Y - 1), rng.integers(1, Z - 1), 0)
    out = batch.lpastar3d_batch(occ, s, g, ch, counters=True)
    cost, ne, st = out["cost"].cpu().numpy(), out["n_expanded"].cpu().numpy(), out["status"].cpu().numpy()
    pl, path = out["path_len"].cpu().numpy(), out["path"].cpu().numpy()
    for q in range(len(s)):
        ref = O.lpastar3d(occ[q], s[q], g[q], ch[q])
        for r in range(4):
            assert st[q, r] == ref["status"][r] and ne[q, r] == ref["n_expanded"][r], (q, r)
            assert cost[q, r] == ref["cost"][r], (q, r)
            assert np.array_equal(path[q, r, : pl[q, r]], ref["paths"][r]), (q, r)


def test_lpastar3d_dropin_sequence():
    """The drop-in class: plan() then apply_change() calls, as the reference object."""
    import python_motion_planning_amd as pmp

    for i, occ, z in grid_cases("lpastar3d_runs.npz"):
        if i % 5:
            continue
        X, Y, Z = occ.shape
        env = pmp.Grid3D(X, Y, Z)
        env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
        p = pmp.LPAStar3D(tuple(int(v) for v in z["start"][i]), tuple(int(v) for v in z["goal"][i]), env)
        enc = lambda t: (t[0] * Y + t[1]) * Z + t[2]  # noqa: E731
        R = z["changes"].shape[1] + 1
        cost, path, expand = p.plan()
        assert cost == z["cost"][i][0] and len(expand) == z["nexp"][i][0]
        assert [enc(t) for t in path] == seg(z["path"], z["path_off"], i * R).tolist()
        for r in range(1, R):
            x, y, zz, mode = (int(v) for v in z["changes"][i][r - 1])
            cost, path, expand = p.apply_change((x, y, zz), None if mode == 0 else mode == 1)
            assert cost == z["cost"][i][r] and len(expand) == z["nexp"][i][r], (i, r)
            assert [enc(t) for t in path] == seg(z["path"], z["path_off"], i * R + r).tolist(), (i, r)


@pytest.mark.gpu
def test_lpastar3d_longest_first_schedule_full_c5():
    """All 8192 C5 queries with 1 worker per CU (256 workers): the longest-first order and the
    raised priority of the longest queries are active; costs and len(EXPAND) equal the oracle's."""
    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, s, g = wl.c5_workload(8192)
    L, ctx = _lib.load_library(), _lib.context()
    _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, 1), "workers")
    try:
        out = batch.lpastar3d_batch(occ, s, g)
    finally:
        _lib.check(ctx, L.pmp_set_workers_per_cu(ctx, 0), "workers")
    ref = O.graph3d_dynamic_batch("lpastar3d", occ, s, g, None, nthreads=min(16, os.cpu_count() or 1))
    assert np.array_equal(out["n_expanded"][:, 0].cpu().numpy(), ref["n"][:, 0])
    assert np.array_equal(out["cost"][:, 0].cpu().numpy(), ref["cost"][:, 0])


@pytest.mark.gpu
def test_lpastar3d_stuck_extract_cycle():
    """C5 query 7349's greedy extractPath (lpa_star3d.py:199-225) falls into a 2-cycle of sqrt(3)
    steps and walks to the 100000-step guard: (cost, []).  The kernel finds the cycle and adds the
    remaining steps' costs in order -- cost bits equal to the oracle's full walk, plus neighbouring
    queries and apply_change rounds that toggle voxels next to the stuck goal."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, s, g = wl.c5_workload(8192)
    idx = np.array([7349, 7348, 7350, 0])
    occ, s, g = occ[idx], s[idx], g[idx]
    ch = np.zeros((len(idx), 2, 4), np.int32)
    for q in range(len(idx)):
        ch[q, 0] = (g[q][0], g[q][1], min(g[q][2] + 1, occ.shape[3] - 1), 0)
        ch[q, 1] = (g[q][0], g[q][1], min(g[q][2] + 1, occ.shape[3] - 1), 0)
    out = batch.lpastar3d_batch(occ, s, g, ch)
    cost, st, ne = out["cost"].cpu().numpy(), out["status"].cpu().numpy(), out["n_expanded"].cpu().numpy()
    assert cost[0, 0] > 1e5  # the 100000-step walk
    for q in range(len(idx)):
        ref = O.lpastar3d(occ[q], s[q], g[q], ch[q])
        for r in range(3):
            assert st[q, r] == ref["status"][r] and ne[q, r] == ref["n_expanded"][r], (q, r)
            assert cost[q, r] == ref["cost"][r], (q, r, cost[q, r], ref["cost"][r])
