"""HIP 3D A* (astar3d.hip via the C-ABI) vs the reference's published CSV, full runs and the oracle.

Bar: bit-exact cost, path, visited count and closure order."""
import numpy as np
import pytest

from golden_io import grid_cases, load_json, seg

pytestmark = pytest.mark.gpu


def test_published_csv_rows():
    """The 500 AStar3D rows of the reference's own 3d_pathfinding_results.csv (21x15x11, r=2 bubbles)."""
    from python_motion_planning_amd import batch, workloads as wl

    rows = load_json("astar3d_csv.json")
    occ = np.zeros((len(rows), 21, 15, 11), np.uint8)
    S = np.zeros((len(rows), 3), np.int32)
    G = np.zeros((len(rows), 3), np.int32)
    for i, r in enumerate(rows):
        s, g = wl.bench3d_query(r["seed"], 21, 15, 11)
        o = wl.SCENARIOS_3D[r["scenario"]](21, 15, 11)
        wl.carve_safety_bubble(o, s, 2)
        wl.carve_safety_bubble(o, g, 2)
        occ[i], S[i], G[i] = o, s, g
    out = batch.astar3d_batch(occ, S, G)
    cost = out["cost"].cpu().numpy()
    ne = out["n_expanded"].cpu().numpy()
    for i, r in enumerate(rows):
        assert repr(float(cost[i])) == r["cost"], (i, r)
        assert ne[i] == r["visited"], (i, r)


def test_full_runs_against_reference():
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("astar3d_runs.npz"):
        X, Y, Z = occ.shape
        out = batch.astar3d_batch(occ, z["start"][i][None], z["goal"][i][None], expand_cap=X * Y * Z)
        assert float(out["cost"][0]) == z["cost"][i]
        pl = int(out["path_len"][0])
        assert np.array_equal(out["path"][0, :pl].cpu().numpy(), seg(z["path"], z["path_off"], i))
        ne = int(out["n_expanded"][0])
        assert np.array_equal(out["expand"][0, :ne].cpu().numpy(), seg(z["expand"], z["expand_off"], i))


def test_dropin_class():
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import workloads as wl

    s, g = wl.bench3d_query(3, 21, 15, 11)
    o = wl.SCENARIOS_3D["maze"](21, 15, 11)
    wl.carve_safety_bubble(o, s, 2)
    wl.carve_safety_bubble(o, g, 2)
    env = pmp.Grid3D(21, 15, 11)
    env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(o)})
    cost, path, expand = pmp.AStar3D(s, g, env).plan()
    from oracle import oracle as O

    ref = O.astar3d(o, s, g)
    assert cost == ref["cost"] and path == ref["path"] and len(expand) == ref["n_expanded"]


def test_c5_batch_against_oracle():
    """C5: 8192 door-scenario queries on 26x20x16 (per-query carve) in one launch, every one against
    the oracle (status, cost bits, expansions, path, the reference's push count)."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, S, G = wl.c5_workload(8192)
    out = batch.astar3d_batch(occ, S, G, counters=True)
    st = out["status"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    ne = out["n_expanded"].cpu().numpy()
    pl = out["path_len"].cpu().numpy()
    P = out["path"].cpu().numpy()
    ctr = out["counters"].cpu().numpy()
    for q in range(8192):  # every query against the oracle
        ref = O.astar3d(occ[q], S[q], G[q], with_expand=False)
        assert st[q] == ref["status"] and cost[q] == ref["cost"] and ne[q] == ref["n_expanded"], q
        assert np.array_equal(P[q, : pl[q]], ref["path_cells"]), q
        # pushes counted the reference's way; the kernel's heap drops dead duplicates, so it is never larger
        assert ctr[q, 0] == ref["n_push"] and ctr[q, 3] <= ref["max_heap"], q
    assert (st == 0).all()
