"""Dijkstra / GBFS (2D: dijkstra.py, gbfs.py; 3D: dijkstra3d.py, gbfs3d.py) and Theta* / Lazy Theta*
3D (theta_star3d.py, lazy_theta_star3d.py) on the HIP kernels astar2d.hip / astar3d.hip (C-ABI
pmp_graph2d_batch / pmp_graph3d_batch) vs the reference's own outputs (tests/golden/graph2d_small.npz,
graph3d_csv.json, graph3d_runs.npz, theta3d_csv.json, theta3d_runs.npz) and the oracle.

Bar: bit-exact -- cost bits, path cells, closure (expand) order, visited counts."""
import numpy as np
import pytest

from golden_io import grid_cases, load_json, seg

pytestmark = pytest.mark.gpu


def test_graph2d_against_reference():
    from python_motion_planning_amd import batch

    n = 0
    for i, occ, z in grid_cases("graph2d_small.npz"):
        W, H = occ.shape
        heur = "manhattan" if z["manhattan"][i] else "euclidean"
        r = batch.astar2d_batch(occ, z["start"][i][None], z["goal"][i][None], heur, path_cap=W * H + 1,
                                expand_cap=W * H, algo=str(z["algo"][i]))
        st = int(r["status"][0])
        if not z["found"][i]:
            assert st == 1, i
            continue
        assert st == 0, i
        assert float(r["cost"][0]) == z["cost"][i], i
        plen = int(r["path_len"][0])
        assert np.array_equal(r["path"][0, :plen].cpu().numpy(), seg(z["path"], z["path_off"], i)), i
        ne = int(r["n_expanded"][0])
        e = (r["expand"][0, :ne].cpu().numpy().astype(np.uint32) & 0x0FFFFFFF).astype(np.int32)
        assert np.array_equal(e, seg(z["expand"], z["expand_off"], i)), i
        n += 1
    assert n > 100


def test_readme_dropin_classes():
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import workloads as wl
    from oracle import oracle as O

    occ = wl.readme_grid()
    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(occ)})
    for cls, algo in ((pmp.Dijkstra, "dijkstra"), (pmp.GBFS, "gbfs")):
        for heur in ("euclidean", "manhattan"):
            cost, path, expand = cls((5, 5), (45, 25), env, heur).plan()
            ref = O.astar2d(occ, (5, 5), (45, 25), heur, algo=algo)
            assert cost == ref["cost"] and path == ref["path"], (algo, heur)
            assert [n.current[0] * 31 + n.current[1] for n in expand] == ref["expand_cells"].tolist()
            if algo == "gbfs":
                assert all(n.g == 0 for n in expand)
            else:
                assert all(n.h == 0 for n in expand)


def test_c2_subset_against_oracle():
    """Dijkstra / GBFS on the C2 1024x1024 grid (20 % obstacles): 24 queries each, bit-exact."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, s, g = wl.c2_workload(4096)
    idx = np.arange(0, 4096, 171)[:24]
    for algo in ("dijkstra", "gbfs"):
        r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=8192, counters=True, algo=algo)
        ref = O.astar2d_batch(occ, s[idx], g[idx], path_cap=8192, algo=algo)
        assert np.array_equal(r["status"].cpu().numpy(), ref["status"]), algo
        assert np.array_equal(r["cost"].cpu().numpy(), ref["cost"]), algo
        assert np.array_equal(r["n_expanded"].cpu().numpy(), ref["n_expanded"]), algo
        # pushes, pops, expansions and the largest heap (24 queries: the single-query engine, which
        # samples the heap size after each expansion's pushes, as the oracle's maximum lands there)
        assert np.array_equal(r["counters"].cpu().numpy(), ref["counters"]), algo
        P = r["path"].cpu().numpy()
        for k in range(len(idx)):
            n = ref["path_len"][k]
            assert np.array_equal(P[k, :n], ref["path"][k, :n]), (algo, k)


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


def test_graph3d_published_csv_rows():
    """The 1000 Dijkstra3D / GBFS3D rows of the reference's 3d_pathfinding_results.csv."""
    from python_motion_planning_amd import batch

    rows = load_json("graph3d_csv.json")
    for algo in ("dijkstra", "gbfs"):
        sub = [r for r in rows if r["algo"] == algo]
        occ, S, G = _csv_batch(sub)
        out = batch.astar3d_batch(occ, S, G, algo=algo)
        cost = out["cost"].cpu().numpy()
        ne = out["n_expanded"].cpu().numpy()
        for i, r in enumerate(sub):
            assert repr(float(cost[i])) == r["cost"], (algo, i, r)
            assert ne[i] == r["visited"], (algo, i, r)


def test_graph3d_full_runs_and_dropin():
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("graph3d_runs.npz"):
        X, Y, Z = occ.shape
        algo = str(z["algo"][i])
        out = batch.astar3d_batch(occ, z["start"][i][None], z["goal"][i][None], expand_cap=X * Y * Z, algo=algo)
        assert float(out["cost"][0]) == z["cost"][i], (algo, i)
        pl = int(out["path_len"][0])
        assert np.array_equal(out["path"][0, :pl].cpu().numpy(), seg(z["path"], z["path_off"], i)), (algo, i)
        ne = int(out["n_expanded"][0])
        assert np.array_equal(out["expand"][0, :ne].cpu().numpy(), seg(z["expand"], z["expand_off"], i)), (algo, i)
        if i % 9 == 0:  # the drop-in classes on the same case
            env = pmp.Grid3D(X, Y, Z)
            env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
            cls = pmp.Dijkstra3D if algo == "dijkstra" else pmp.GBFS3D
            cost, path, expand = cls(tuple(z["start"][i]), tuple(z["goal"][i]), env).plan()
            assert cost == z["cost"][i] and len(expand) == ne


def test_theta3d_published_csv_rows():
    """The 1000 ThetaStar3D / LazyThetaStar3D rows of the reference's 3d_pathfinding_results.csv."""
    from python_motion_planning_amd import batch

    rows = load_json("theta3d_csv.json")
    for algo in ("theta_star", "lazy_theta_star"):
        sub = [r for r in rows if r["algo"] == algo]
        occ, S, G = _csv_batch(sub)
        out = batch.astar3d_batch(occ, S, G, algo=algo)
        cost = out["cost"].cpu().numpy()
        ne = out["n_expanded"].cpu().numpy()
        st = out["status"].cpu().numpy()
        for i, r in enumerate(sub):
            assert repr(float(cost[i])) == r["cost"], (algo, i, r, st[i])
            assert ne[i] == r["visited"], (algo, i, r)


def test_theta3d_full_runs_and_dropin():
    import python_motion_planning_amd as pmp
    from oracle import oracle as O
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("theta3d_runs.npz"):
        X, Y, Z = occ.shape
        lazy = bool(z["lazy"][i])
        algo = "lazy_theta_star" if lazy else "theta_star"
        out = batch.astar3d_batch(occ, z["start"][i][None], z["goal"][i][None], expand_cap=X * Y * Z, counters=True,
                                  algo=algo)
        assert float(out["cost"][0]) == z["cost"][i], (algo, i)
        pl = int(out["path_len"][0])
        assert np.array_equal(out["path"][0, :pl].cpu().numpy(), seg(z["path"], z["path_off"], i)), (algo, i)
        ne = int(out["n_expanded"][0])
        assert np.array_equal(out["expand"][0, :ne].cpu().numpy(), seg(z["expand"], z["expand_off"], i)), (algo, i)
        ref = O.theta3d(occ, z["start"][i], z["goal"][i], lazy=lazy, with_expand=False)
        assert int(out["counters"][0, 0]) == ref["n_push"] and int(out["counters"][0, 2]) == ref["n_iter"], (algo, i)
        if i % 7 == 0:
            env = pmp.Grid3D(X, Y, Z)
            env.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(occ)})
            cls = pmp.LazyThetaStar3D if lazy else pmp.ThetaStar3D
            cost, path, expand = cls(tuple(z["start"][i]), tuple(z["goal"][i]), env).plan()
            assert cost == z["cost"][i] and len(expand) == ne


def test_theta3d_c5_batch_against_oracle():
    """Theta* / Lazy Theta* on the C5 door workload (26x20x16, per-query carve), 2048 queries each."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, S, G = wl.c5_workload(2048)
    for lazy in (False, True):
        out = batch.astar3d_batch(occ, S, G, algo="lazy_theta_star" if lazy else "theta_star")
        cost = out["cost"].cpu().numpy()
        ne = out["n_expanded"].cpu().numpy()
        pl = out["path_len"].cpu().numpy()
        P = out["path"].cpu().numpy()
        for q in np.random.default_rng(5).choice(2048, 120, replace=False):
            ref = O.theta3d(occ[q], S[q], G[q], lazy=lazy, with_expand=False)
            assert cost[q] == ref["cost"] and ne[q] == ref["n_expanded"], (lazy, q)
            assert np.array_equal(P[q, : pl[q]], ref["path_cells"]), (lazy, q)


@pytest.fixture(params=[(1, 0), (0, 0), (2, 1), (2, 0)], ids=["auto", "wave", "mq_t2lds", "mq"])
def theta_engine(request):
    """The 2D graph engine the Theta* tests run on: engine 0 (one query per wave, astar2d.hip) or
    engine 2 (four queries per wave, astar2d_mq.hip; the small-batch runs take its lone-group mode)."""
    from python_motion_planning_amd import _lib

    L, ctx = _lib.load_library(), _lib.context()
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, *request.param), "engine")
    yield request.param
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 0), "engine")


def test_theta2d_against_reference(theta_engine):
    """ThetaStar / LazyThetaStar 2D (theta_star.py, lazy_theta_star.py) on astar2d.hip / astar2d_mq.hip vs
    the reference's runs (tests/golden/theta2d_small.npz): cost bits, path, closure order; the drop-in
    classes rebuild the reference's CLOSED nodes (parent, g) from the kernel's expand records."""
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import batch

    n = 0
    for i, occ, z in grid_cases("theta2d_small.npz"):
        W, H = occ.shape
        heur = "manhattan" if z["manhattan"][i] else "euclidean"
        algo = str(z["algo"][i])
        r = batch.astar2d_batch(occ, z["start"][i][None], z["goal"][i][None], heur, path_cap=W * H + 1,
                                expand_cap=W * H, algo=algo)
        st = int(r["status"][0])
        if not z["found"][i]:
            assert st == 1, i
            continue
        assert st == 0, i
        assert float(r["cost"][0]) == z["cost"][i], i
        plen = int(r["path_len"][0])
        assert np.array_equal(r["path"][0, :plen].cpu().numpy(), seg(z["path"], z["path_off"], i)), i
        ne = int(r["n_expanded"][0])
        e = (r["expand"][0, :ne].cpu().numpy().astype(np.uint32) & 0x03FFFFFF).astype(np.int32)
        assert np.array_equal(e, seg(z["expand"], z["expand_off"], i)), i
        if i % 5 == 0:  # drop-in class: the CLOSED nodes' parents and g as the reference holds them
            env = pmp.Grid(W, H)
            env.update({(int(a), int(b)) for a, b in np.argwhere(occ)})
            cls = pmp.LazyThetaStar if algo == "lazy_theta_star" else pmp.ThetaStar
            cost, path, expand = cls(tuple(z["start"][i]), tuple(z["goal"][i]), env, heur).plan()
            assert cost == z["cost"][i] and [a * H + b for a, b in path] == seg(z["path"], z["path_off"], i).tolist()
            par = seg(z["exp_parent"], z["expand_off"], i).tolist()
            assert [nd.parent[0] * H + nd.parent[1] for nd in expand] == par, i
            assert [nd.g for nd in expand] == seg(z["exp_g"], z["expand_off"], i).tolist(), i
        n += 1
    assert n > 140


def test_theta2d_c2_subset_against_oracle(theta_engine):
    """ThetaStar / LazyThetaStar on the C2 1024x1024 grid (20 % obstacles): 16 queries each, bit-exact
    cost, path, closure count and push/pop counts, on each engine."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, s, g = wl.c2_workload(4096)
    idx = np.arange(0, 4096, 257)[:16]
    for algo in ("theta_star", "lazy_theta_star"):
        r = batch.astar2d_batch(occ, s[idx], g[idx], path_cap=8192, counters=True, algo=algo)
        ref = O.astar2d_batch(occ, s[idx], g[idx], path_cap=8192, algo=algo)
        assert np.array_equal(r["status"].cpu().numpy(), ref["status"]), algo
        assert np.array_equal(r["cost"].cpu().numpy(), ref["cost"]), algo
        assert np.array_equal(r["n_expanded"].cpu().numpy(), ref["n_expanded"]), algo
        # pushes, pops, expansions, and the largest heap except on engine 2 (which samples it once
        # per step, after a step's pop may already have shrunk the heap)
        cols = 3 if theta_engine[0] == 2 else 4
        assert np.array_equal(r["counters"].cpu().numpy()[:, :cols], ref["counters"][:, :cols]), algo
        P = r["path"].cpu().numpy()
        for k in range(len(idx)):
            n = ref["path_len"][k]
            assert np.array_equal(P[k, :n], ref["path"][k, :n]), (algo, k)


def test_theta2d_c2_batch_multiquery_against_oracle():
    """The Theta* bench's shape on the multi-query engine: 1,024 C2 queries in one launch at 24 groups
    per CU (longest first, heaps spilled past the LDS share), every query against the oracle (cost
    bits, path, closure count, push / pop counts); Lazy Theta* the same on 512."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, s, g = wl.c2_workload(4096)
    L = _lib.load_library()
    for algo, nq in (("theta_star", 1024), ("lazy_theta_star", 512)):
        ctx = L.pmp_create(torch.cuda.current_device())
        try:
            _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 2, 1), "engine")
            _lib.check(ctx, L.pmp_astar2d_reserve(ctx, 1024, 1024, 256 * 24, 0), "reserve")
            _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, 24), "residency")
            sd, gd = torch.as_tensor(s[:nq], device="cuda"), torch.as_tensor(g[:nq], device="cuda")
            out = {k: torch.empty(nq, dtype=t, device="cuda") for k, t in
                   (("cost", torch.float64), ("plen", torch.int32), ("nexp", torch.int32), ("st", torch.int32))}
            path = torch.empty((nq, 8192), dtype=torch.int32, device="cuda")
            ctr = torch.empty((nq, 4), dtype=torch.int64, device="cuda")
            bits = batch.occ_bits_device(occ, torch)
            rc = L.pmp_graph2d_batch(ctx, torch.cuda.current_stream().cuda_stream, _lib.ALGOS[algo], bits.data_ptr(),
                                     1024, 1024, 0, sd.data_ptr(), gd.data_ptr(), nq, out["cost"].data_ptr(),
                                     out["plen"].data_ptr(), path.data_ptr(), 8192, out["nexp"].data_ptr(), None, 0,
                                     ctr.data_ptr(), out["st"].data_ptr())
            _lib.check(ctx, rc, "pmp_graph2d_batch")
            torch.cuda.synchronize()
        finally:
            L.pmp_destroy(ctx)
        ref = O.astar2d_batch(occ, s[:nq], g[:nq], path_cap=8192, algo=algo)
        assert np.array_equal(out["st"].cpu().numpy(), ref["status"]), algo
        assert np.array_equal(out["cost"].cpu().numpy(), ref["cost"]), algo
        assert np.array_equal(out["nexp"].cpu().numpy(), ref["n_expanded"]), algo
        assert np.array_equal(ctr.cpu().numpy()[:, :3], ref["counters"][:, :3]), algo  # pushes, pops, expansions
        P, pl = path.cpu().numpy(), out["plen"].cpu().numpy()
        for k in range(nq):
            assert np.array_equal(P[k, : pl[k]], ref["path"][k, : ref["path_len"][k]]), (algo, k)


@pytest.mark.parametrize("lite", [False, True])
def test_lpastar_against_reference(lite):
    """LPAStar.plan (lpa_star.py:78-230) / DStarLite.plan (d_star_lite.py:14-187) on lpa.hip vs the
    reference's runs (tests/golden/lpa_small.npz, dstarlite_small.npz): cost bits, path, len(EXPAND),
    and the raising runs (status 4 / ValueError from the drop-in)."""
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import batch

    n = 0
    for i, occ, z in grid_cases("dstarlite_small.npz" if lite else "lpa_small.npz"):
        W, H = occ.shape
        heur = "manhattan" if z["manhattan"][i] else "euclidean"
        r = batch.lpastar2d_batch(occ, z["start"][i][None], z["goal"][i][None], heur, lite=lite)
        st = int(r["status"][0])
        assert int(r["n_expanded"][0]) == z["n_expand"][i], i
        if str(z["err"][i]):
            assert st == 4, i
            continue
        path = seg(z["path"], z["path_off"], i)
        assert st == (0 if len(path) else 1), i
        assert float(r["cost"][0]) == z["cost"][i], i
        assert np.array_equal(r["path"][0, : int(r["path_len"][0])].cpu().numpy(), path), i
        if i % 6 == 0:
            env = pmp.Grid(W, H)
            env.update({(int(a), int(b)) for a, b in np.argwhere(occ)})
            cls = pmp.DStarLite if lite else pmp.LPAStar
            cost, p, _ = cls(tuple(z["start"][i]), tuple(z["goal"][i]), env, heur).plan()
            assert cost == z["cost"][i] and [a * H + b for a, b in p] == path.tolist(), i
        n += 1
    assert n > 90


@pytest.mark.parametrize("lite", [False, True])
def test_lpastar_batch_against_oracle(lite):
    """256 LPA* / D* Lite queries on one 96x80 grid (25 % obstacles) in one launch vs the oracle:
    status, cost, path, len(EXPAND), pushes and max |U|."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch

    rng = np.random.default_rng(11)
    occ = (rng.random((96, 80)) < 0.25).astype(np.uint8)
    occ[:, 0] = occ[:, -1] = 1
    occ[0, :] = occ[-1, :] = 1
    free = np.argwhere(occ == 0)
    S = free[rng.integers(len(free), size=256)].astype(np.int32)
    G = free[rng.integers(len(free), size=256)].astype(np.int32)
    r = batch.lpastar2d_batch(occ, S, G, counters=True, lite=lite)
    st = r["status"].cpu().numpy()
    cost = r["cost"].cpu().numpy()
    ne = r["n_expanded"].cpu().numpy()
    ctr = r["counters"].cpu().numpy()
    P = r["path"].cpu().numpy()
    pl = r["path_len"].cpu().numpy()
    for q in range(256):
        ref = O.lpastar2d(occ, S[q], G[q], lite=lite)
        assert st[q] == ref["status"] and ne[q] == ref["n_expanded"], q
        assert ctr[q, 0] == ref["n_push"] and ctr[q, 3] == ref["max_u"], q
        if ref["status"] in (0, 1):
            assert cost[q] == ref["cost"], q
        if ref["status"] == 0:
            assert np.array_equal(P[q, : pl[q]], ref["path_cells"]), q


@pytest.mark.parametrize("lite", [False, True])
def test_lpastar_long_lists(lite):
    """Lists far longer than the README grid's: 24 queries on a 256^2 grid (10 % obstacles), some
    with |U| > 496, against the oracle (status, cost, path, len(EXPAND), pushes, max |U|)."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch

    rng = np.random.default_rng(12)
    occ = (rng.random((256, 256)) < 0.1).astype(np.uint8)
    occ[:, 0] = occ[:, -1] = 1
    occ[0, :] = occ[-1, :] = 1
    free = np.argwhere(occ == 0)
    S = free[rng.integers(len(free), size=24)].astype(np.int32)
    G = free[rng.integers(len(free), size=24)].astype(np.int32)
    r = batch.lpastar2d_batch(occ, S, G, counters=True, lite=lite)
    st, cost = r["status"].cpu().numpy(), r["cost"].cpu().numpy()
    ne, ctr = r["n_expanded"].cpu().numpy(), r["counters"].cpu().numpy()
    P, pl = r["path"].cpu().numpy(), r["path_len"].cpu().numpy()
    long_lists = 0
    for q in range(len(S)):
        ref = O.lpastar2d(occ, S[q], G[q], lite=lite)
        long_lists += ref["max_u"] > 496
        assert st[q] == ref["status"] and ne[q] == ref["n_expanded"], q
        assert ctr[q, 0] == ref["n_push"] and ctr[q, 3] == ref["max_u"], q
        if ref["status"] in (0, 1):
            assert cost[q] == ref["cost"], q
        if ref["status"] == 0:
            assert np.array_equal(P[q, : pl[q]], ref["path_cells"]), q
    assert long_lists > 0


@pytest.mark.parametrize("lite", [False, True])
def test_lpastar_lists_beyond_lds_share(lite):
    """U moving from the wave's LDS share to HBM mid-query (lpa.hip u_push: copy-out, then every
    u_find / u_remove / min scan on the HBM arrays).  The context leaves LDS room for 32 workers per CU
    (pmp_set_resident_per_cu), so a query's share is (160 KiB / 32 / 20 B) & ~15 = 256 entries, and the
    256^2 queries' lists outgrow it; every query against the oracle (status, cost, path, len(EXPAND),
    pushes, max |U|)."""
    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch

    ucap = ((160 * 1024) // 32 // 20) & ~15
    rng = np.random.default_rng(12)
    occ = (rng.random((256, 256)) < 0.1).astype(np.uint8)
    occ[:, 0] = occ[:, -1] = 1
    occ[0, :] = occ[-1, :] = 1
    free = np.argwhere(occ == 0)
    S = free[rng.integers(len(free), size=24)].astype(np.int32)
    G = free[rng.integers(len(free), size=24)].astype(np.int32)
    L, ctx = _lib.load_library(), _lib.context()
    _lib.check(ctx, L.pmp_set_resident_per_cu(ctx, 32), "resident")
    try:
        r = batch.lpastar2d_batch(occ, S, G, counters=True, lite=lite)
        st, cost = r["status"].cpu().numpy(), r["cost"].cpu().numpy()
        ne, ctr = r["n_expanded"].cpu().numpy(), r["counters"].cpu().numpy()
        P, pl = r["path"].cpu().numpy(), r["path_len"].cpu().numpy()
    finally:
        _lib.check(ctx, L.pmp_set_resident_per_cu(ctx, 0), "resident")
    spilled = 0
    for q in range(len(S)):
        ref = O.lpastar2d(occ, S[q], G[q], lite=lite)
        spilled += ref["max_u"] > ucap
        assert st[q] == ref["status"] and ne[q] == ref["n_expanded"], q
        assert ctr[q, 0] == ref["n_push"] and ctr[q, 3] == ref["max_u"], q
        if ref["status"] in (0, 1):
            assert cost[q] == ref["cost"], q
        if ref["status"] == 0:
            assert np.array_equal(P[q, : pl[q]], ref["path_cells"]), q
    assert spilled >= 4, spilled


@pytest.mark.parametrize("lite", [False, True])
def test_lpastar_replan_against_reference_and_oracle(lite):
    """LPA* incremental replanning (pmp_lpastar2d_replan_batch: plan() + OnPress edits, lpa_star.py:101-137)
    vs the reference's replays (tests/golden/lpa_replan.npz), all 60 cases in one launch, then a 256-query
    batch with 6 edits each on a 64x48 grid vs the oracle."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("dstarlite_replan.npz" if lite else "lpa_replan.npz"):
        r = batch.lpastar2d_replan_batch(occ, z["start"][i][None], z["goal"][i][None], z["toggles"][i][None], lite=lite)
        st = r["status"][0].cpu().numpy()
        ne = r["n_expanded"][0].cpu().numpy()
        cost = r["cost"][0].cpu().numpy()
        errs = z["err"][i].tolist()
        for ph, e in enumerate(errs):
            if e == "-":
                assert st[ph] == -1, (i, ph)
                continue
            assert ne[ph] == z["nexp"][i][ph], (i, ph)
            want = 3 if e == "RuntimeError" else 4
            assert (st[ph] == want) if e else (st[ph] in (0, 1) and cost[ph] == z["cost"][i][ph]), (i, ph)
        if not any(errs):
            pl = int(r["path_len"][0])
            assert np.array_equal(r["path"][0, :pl].cpu().numpy(), seg(z["path"], z["path_off"], i)), i

    rng = np.random.default_rng(21)
    occ = (rng.random((64, 48)) < 0.2).astype(np.uint8)
    occ[:, 0] = occ[:, -1] = 1
    occ[0, :] = occ[-1, :] = 1
    free = np.argwhere(occ == 0)
    S = free[rng.integers(len(free), size=256)].astype(np.int32)
    G = free[rng.integers(len(free), size=256)].astype(np.int32)
    T = (np.argwhere(np.ones((62, 46), bool)) + 1)[rng.integers(62 * 46, size=(256, 6))].astype(np.int32)
    r = batch.lpastar2d_replan_batch(occ, S, G, T, lite=lite)
    st, ne, cost = (r[k].cpu().numpy() for k in ("status", "n_expanded", "cost"))
    for q in range(256):
        ref = O.lpastar2d_replan(occ, S[q], G[q], T[q], lite=lite)
        assert np.array_equal(st[q], ref["status"]) and np.array_equal(ne[q], ref["n_expanded"]), q
        assert np.array_equal(cost[q], ref["cost"]), q
