"""HIP 2D A* (libpmp_hip.so, via the C-ABI) vs the reference's golden vectors and the oracle.

Bar: bit-exact -- cost bits, path cells, closure (expand) order, expansion counts."""
import hashlib

import numpy as np
import pytest

from golden_io import grid_cases, load_json, load_npz, seg

pytestmark = pytest.mark.gpu


def _pmp():
    import python_motion_planning_amd as pmp

    return pmp


# (engine, tier-2 bits in LDS): 2 = four queries per wave (astar2d_mq.hip) for every batch, 0 = one
# query per wave (astar2d.hip; grid state in LDS on small grids), 3 = one query per workgroup with the
# heap in LDS and its choice bits in registers (astar2d_sq.hip), 1 = the default choice between them
# by batch and grid size; all must give the reference's answers bit for bit
ENGINES = [(2, 0), (2, 1), (0, 0), (3, 0), (1, 0)]


@pytest.fixture(params=ENGINES, ids=["mq", "mq_t2lds", "wave", "sq", "auto"])
def engine(request):
    from python_motion_planning_amd import _lib

    L, ctx = _lib.load_library(), _lib.context()
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, *request.param), "engine")
    yield request.param
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 0), "engine")


def test_readme_dropin_class():
    pmp = _pmp()
    fx = load_json("astar_readme.json")
    env = pmp.Grid(51, 31)
    obstacles = env.obstacles
    for x, y in fx["obstacles"]:
        obstacles.add((x, y))
    env.update(obstacles)
    for heur in ("euclidean", "manhattan"):
        planner = pmp.AStar((5, 5), (45, 25), env, heur)
        cost, path, expand = planner.plan()
        exp = fx[heur]
        assert cost == float.fromhex(exp["cost_hex"])
        assert [x * 31 + y for (x, y) in path] == exp["path"]
        assert [n.current[0] * 31 + n.current[1] for n in expand] == exp["expand"]
    cost, path, expand = pmp.AStar((5, 5), (45, 25), env).plan()
    assert repr(cost) == "54.04163056034261" and len(path) == 48 and len(expand) == 579
    # expand nodes carry parent / g / h like the reference's CLOSED values
    assert expand[0].current == (5, 5) and expand[0].parent == (5, 5) and expand[0].g == 0


def test_dropin_obstacle_set_changes_between_calls():
    """plan() launches on the Grid's last uploaded bit grid while it packs the obstacle set again:
    an obstacle added or removed between two calls must re-run the query on the new set."""
    from oracle import oracle as O

    pmp = _pmp()
    fx = load_json("astar_readme.json")
    env = pmp.Grid(51, 31)
    for x, y in fx["obstacles"]:
        env.obstacles.add((x, y))
    env.update(env.obstacles)
    planner = pmp.AStar((5, 5), (45, 25), env)
    cost0, path0, _ = planner.plan()
    block = path0[len(path0) // 2]
    for step in range(3):
        if step == 1:
            env.obstacles.add(block)  # in place: same set object, same Grid
        elif step == 2:
            env.obstacles.discard(block)
        cost, path, expand = planner.plan()
        ref = O.astar2d(env.occupancy(), (5, 5), (45, 25))
        assert ref["status"] == 0 and cost == ref["cost"] and path == ref["path"], step
        assert [n.current[0] * 31 + n.current[1] for n in expand] == ref["expand_cells"].tolist(), step
        if step != 1:
            assert cost == cost0 and path == path0
        else:
            assert block not in path


def test_small_grids_against_reference(engine):
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("astar_small.npz"):
        W, H = occ.shape
        heur = "manhattan" if z["manhattan"][i] else "euclidean"
        r = batch.astar2d_batch(occ, z["start"][i][None], z["goal"][i][None], heur, path_cap=W * H + 1,
                                expand_cap=W * H)
        st = int(r["status"][0])
        if not z["found"][i]:
            assert st == 1, i
            continue
        assert st == 0, i
        assert float(r["cost"][0]) == z["cost"][i], i
        plen = int(r["path_len"][0])
        assert np.array_equal(r["path"][0, :plen].cpu().numpy(), seg(z["path"], z["path_off"], i)), i
        ne = int(r["n_expanded"][0])
        assert ne == z["n_expanded"][i]
        e = (r["expand"][0, :ne].cpu().numpy().astype(np.uint32) & 0x0FFFFFFF).astype(np.int32)
        assert np.array_equal(e, seg(z["expand"], z["expand_off"], i)), i


def test_c2_subset_against_reference(engine):
    from python_motion_planning_amd import batch, workloads as wl

    z = load_npz("astar_1024.npz")
    occ, starts, goals = wl.c2_workload(nq=4096)
    idx = z["query_index"]
    r = batch.astar2d_batch(occ, starts[idx], goals[idx], path_cap=4096, expand_cap=280000)
    assert (r["status"].cpu().numpy() == 0).all()
    assert np.array_equal(r["n_expanded"].cpu().numpy(), z["n_expanded"])
    assert np.array_equal(r["cost"].cpu().numpy(), z["cost"])
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    E = r["expand"].cpu().numpy().astype(np.uint32)
    for i in range(len(idx)):
        assert np.array_equal(P[i, :pl[i]], seg(z["path"], z["path_off"], i)), i
        e = (E[i, : z["n_expanded"][i]] & 0x0FFFFFFF).astype(np.int32)
        assert hashlib.sha1(e.tobytes()).hexdigest() == str(z["expand_sha1"][i]), i


_C2_REF = {}


def _c2_oracle():
    """The oracle on all 4096 C2 queries (OpenMP over the host's cores; a few seconds), computed once."""
    from oracle import oracle as O
    from python_motion_planning_amd import workloads as wl

    if not _C2_REF:
        occ, starts, goals = wl.c2_workload(nq=4096)
        _C2_REF.update(occ=occ, starts=starts, goals=goals,
                       ref=O.astar2d_batch(occ, starts, goals, path_cap=4096))
    return _C2_REF


def _assert_c2_equal(ref, r, copies=1):
    nq = len(ref["cost"])
    cost = r["cost"].cpu().numpy()
    ne = r["n_expanded"].cpu().numpy()
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    ctr = r["counters"].cpu().numpy() if r.get("counters") is not None else None
    for c in range(copies):
        sl = slice(c * nq, (c + 1) * nq)
        assert (r["status"].cpu().numpy()[sl] == 0).all()
        assert np.array_equal(ref["cost"], cost[sl])
        assert np.array_equal(ref["n_expanded"], ne[sl])
        assert np.array_equal(ref["path_len"], pl[sl])
        if ctr is not None:
            assert np.array_equal(ref["counters"][:, :2], ctr[sl, :2])  # pushes and pops
        for q in range(nq):
            assert np.array_equal(ref["path"][q, : ref["path_len"][q]], P[c * nq + q, : pl[c * nq + q]]), (c, q)


def test_c2_full_batch_against_oracle_and_properties():
    """All 4096 C2 queries in one launch, every one bit-exact vs the oracle (cost bits, expansion and
    heap-operation counts, path), and size-independent properties on every query."""
    from python_motion_planning_amd import batch

    c2 = _c2_oracle()
    occ, starts, goals, ref = c2["occ"], c2["starts"], c2["goals"], c2["ref"]
    W, H = occ.shape
    r = batch.astar2d_batch(occ, starts, goals, path_cap=4096, counters=True)
    st = r["status"].cpu().numpy()
    assert (st == 0).all()
    cost = r["cost"].cpu().numpy()
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    ne = r["n_expanded"].cpu().numpy()
    ctr = r["counters"].cpu().numpy()
    _assert_c2_equal(ref, r)
    # properties on every query
    sq2 = 2.0 ** 0.5
    for q in range(4096):
        p = P[q, : pl[q]]
        xs, ys = p // H, p % H
        assert xs[0] == goals[q, 0] and ys[0] == goals[q, 1]
        assert xs[-1] == starts[q, 0] and ys[-1] == starts[q, 1]
        dx, dy = np.diff(xs), np.diff(ys)
        assert (np.maximum(np.abs(dx), np.abs(dy)) == 1).all()
        assert not occ[xs, ys].any()
        c = 0.0
        for a, b in zip(np.abs(dx).tolist(), np.abs(dy).tolist()):
            c += sq2 if (a and b) else 1.0
        assert c == cost[q]
    assert (ctr[:, 2] == ne).all() and (ctr[:, 1] <= ctr[:, 0]).all()


def test_edge_cases(engine):
    import torch

    from python_motion_planning_amd import batch, workloads as wl

    occ = wl.readme_grid()
    starts = np.array([[5, 5], [5, 5], [-3, 4], [5, 5], [20, 5], [5, 5]], np.int32)
    goals = np.array([[45, 25], [5, 5], [45, 25], [60, 2], [45, 25], [20, 5]], np.int32)
    r = batch.astar2d_batch(occ, starts, goals, path_cap=2048)
    st = r["status"].cpu().numpy().tolist()
    assert st == [0, 0, 1, 1, 1, 1]  # (20,5) is a wall cell: start blocked / goal blocked
    assert int(r["path_len"][1]) == 1 and float(r["cost"][1]) == 0.0
    # path_cap overflow is reported, never silently truncated
    r = batch.astar2d_batch(occ, starts[:1], goals[:1], path_cap=10)
    assert int(r["status"][0]) == 2 and int(r["path_len"][0]) == 48
    # tiny heap capacity -> status 3 from the kernel ...
    r = batch.astar2d_batch(occ, starts[:1], goals[:1], path_cap=64, reserve_slots=1, heap_cap=4,
                            retry_overflow=False)
    assert int(r["status"][0]) == 3
    # ... and the host re-runs the overflowed queries with the full bound: same answers as the oracle
    from oracle import oracle as O

    r = batch.astar2d_batch(occ, starts, goals, path_cap=2048, reserve_slots=4, heap_cap=8, expand_cap=4096)
    assert r["status"].cpu().numpy().tolist() == [0, 0, 1, 1, 1, 1]
    ref = O.astar2d(occ, tuple(starts[0]), tuple(goals[0]))
    assert float(r["cost"][0]) == ref["cost"] and int(r["n_expanded"][0]) == ref["n_expanded"]
    torch.cuda.synchronize()
    # restore default scratch sizing for later tests
    batch.astar2d_batch(occ, starts[:1], goals[:1], path_cap=64, reserve_slots=64, heap_cap=0)


def test_explicit_heap_cap_and_overflow_retry_keep_geometry():
    """An explicit heap_cap above the multi-query engine's limit is kept (the one-query engine is
    reserved for it, not the limit); a batch's overflow re-run restores the geometry in force: the
    host's reservation, or launch-sized (auto) scratch on a context the host never reserved."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch

    L, ctx = _lib.load_library(), _lib.context()

    def geometry():
        geo = np.zeros(6, np.int32)
        _lib.check(ctx, L.pmp_astar2d_geometry(ctx, geo.ctypes.data), "geometry")
        return geo.tolist()

    W = 70
    occ = np.zeros((W, W), np.uint8)
    occ[0, :] = occ[-1, :] = occ[:, 0] = occ[:, -1] = 1
    occ[30, 5:60] = 1
    starts = np.array([[3, 3], [60, 60], [10, 50]], np.int32)
    goals = np.array([[65, 65], [2, 2], [50, 10]], np.int32)
    ref = O.astar2d_batch(occ, starts, goals, path_cap=W * W + 1)
    try:
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 1), "engine")  # multi-query limit 16383
        limit = 16383
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, W, 4, limit + 1000), "reserve")
        assert geometry()[3] == limit + 1000 and geometry()[4] == 2  # kept (explicit); one-query engine
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, W, 4096, 0), "reserve")
        assert geometry()[3] == limit and geometry()[4] == 1  # the default is the limit (multi-query)
        # an overflow re-run on a default reservation restores the default (not the cut limit as an
        # explicit cap, which would move later small batches off the single-query engine)
        before = geometry()
        r = batch.astar2d_full_bound(occ, torch.as_tensor(starts, device="cuda"),
                                     torch.as_tensor(goals, device="cuda"), path_cap=W * W + 1)
        assert np.array_equal(r["cost"].cpu().numpy(), ref["cost"])
        assert geometry() == before
        # a tiny explicit cap overflows every query; the re-run (full bound 8 W H + 8 = 39,208 > the
        # limit) must not be cut back to the limit, and the host's geometry comes back afterwards
        r = batch.astar2d_batch(occ, starts, goals, path_cap=W * W + 1, reserve_slots=4, heap_cap=8)
        assert np.array_equal(r["status"].cpu().numpy(), ref["status"])
        assert np.array_equal(r["cost"].cpu().numpy(), ref["cost"])
        assert np.array_equal(r["n_expanded"].cpu().numpy(), ref["n_expanded"])
        geo = geometry()
        assert geo[:4] == [W, W, 4, 8] and geo[4] & 2 and geo[5] == 0
        # a launch-sized context stays launch-sized after a re-run
        _lib.check(ctx, L.pmp_astar2d_reserve_auto(ctx), "reserve_auto")
        assert geometry()[0] == 0
        r = batch.astar2d_batch(occ, starts, goals, path_cap=W * W + 1)
        assert np.array_equal(r["cost"].cpu().numpy(), ref["cost"])
        assert geometry()[5] == 1
    finally:
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 0), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve_auto(ctx), "reserve_auto")


def test_unreachable_and_empty_batch(engine):
    from python_motion_planning_amd import batch

    occ = np.zeros((16, 16), np.uint8)
    occ[:, 0] = occ[:, 15] = occ[0, :] = occ[15, :] = 1
    occ[8, :] = 1  # wall splits the grid
    r = batch.astar2d_batch(occ, np.array([[2, 2]]), np.array([[12, 12]]), path_cap=300)
    assert int(r["status"][0]) == 1
    from oracle import oracle as O

    assert int(r["n_expanded"][0]) == O.astar2d(occ, (2, 2), (12, 12))["n_expanded"]
    r = batch.astar2d_batch(occ, np.zeros((0, 2), np.int32), np.zeros((0, 2), np.int32), path_cap=4)
    assert r["status"].numel() == 0


def test_heap_above_32767_entries_uses_hbm_bit_tiers():
    """A heap past 32767 entries walks levels >= 14, whose direction-bit blocks live in HBM
    (astar2d.hip, tiers >= 3).  An open 2900x2900 grid whose goal is walled in explores every
    cell and peaks at ~36k heap entries: counts and the closure must match the oracle exactly."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch

    W = 2900
    occ = np.zeros((W, W), np.uint8)
    occ[0, :] = occ[-1, :] = occ[:, 0] = occ[:, -1] = 1
    g = (W // 2, W // 2)
    occ[g[0] - 1:g[0] + 2, g[1] - 1:g[1] + 2] = 1
    occ[g] = 0
    s = np.array([[1, 1]], np.int32)
    ref = O.astar2d_batch(occ, s, np.array([g], np.int32))
    assert ref["counters"][0, 3] > 32767
    r = batch.astar2d_batch(occ, s, np.array([g], np.int32), path_cap=16, counters=True, reserve_slots=1,
                            heap_cap=1 << 17)
    assert int(r["status"][0]) == 1
    assert int(r["n_expanded"][0]) == int(ref["n_expanded"][0])
    assert r["counters"].cpu().numpy()[0].tolist() == ref["counters"][0].tolist()
    batch.astar2d_batch(occ[:64, :64], s, s, path_cap=4, reserve_slots=64, heap_cap=0)  # default sizing again


@pytest.mark.parametrize("eng,per_cu", [(2, 48), (2, 18), (0, 18), (0, 1)])
def test_residency_batches_in_flight(eng, per_cu):
    """The bench's headline schedule: several contexts, each a smaller persistent-worker launch on
    its own stream with the LDS heap share of 18 resident workers per CU (pmp_astar2d_set_residency,
    368 LDS positions, the rest of each heap spilled), all in flight together.  Every batch equals
    the oracle's CLOSED order / cost / path."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, s, g = wl.c2_workload(nq=96, W=256, H=256, pair_seed=21)
    if per_cu == 1:  # a 60x60 grid: the one-query-per-wave engine keeps the grid state in LDS
        occ, s, g = occ[:60, :60].copy(), np.clip(s, 1, 58).astype(np.int32), np.clip(g, 1, 58).astype(np.int32)
        occ[s[:, 0], s[:, 1]] = 0
        occ[g[:, 0], g[:, 1]] = 0
    W, H = occ.shape
    L = _lib.load_library()
    bits = batch.occ_bits_device(occ, torch)
    s_d, g_d = torch.as_tensor(s, device="cuda"), torch.as_tensor(g, device="cuda")
    nq, pc = len(s), 4096
    lanes = []
    for _ in range(3):
        ctx = L.pmp_create(torch.cuda.current_device())
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, eng, 0), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, 32, 0), "reserve")
        _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, per_cu), "residency")
        assert L.pmp_astar2d_set_residency(ctx, 129) != 0
        lanes.append(dict(ctx=ctx, stream=torch.cuda.Stream(),
                          out=[torch.empty(nq, dtype=torch.float64, device="cuda"),
                               torch.empty(nq, dtype=torch.int32, device="cuda"),
                               torch.empty((nq, pc), dtype=torch.int32, device="cuda"),
                               torch.empty(nq, dtype=torch.int32, device="cuda"),
                               torch.empty(nq, dtype=torch.int32, device="cuda")]))
    torch.cuda.synchronize()
    for b in lanes:
        c, pl, p, ne, st = b["out"]
        rc = L.pmp_astar2d_batch(b["ctx"], b["stream"].cuda_stream, bits.data_ptr(), W, H, 0, s_d.data_ptr(),
                                 g_d.data_ptr(), nq, c.data_ptr(), pl.data_ptr(), p.data_ptr(), pc, ne.data_ptr(),
                                 None, 0, None, st.data_ptr())
        _lib.check(b["ctx"], rc, "pmp_astar2d_batch")
    torch.cuda.synchronize()
    ref = O.astar2d_batch(occ, s, g, path_cap=pc)
    for b in lanes:
        c, pl, p, ne, st = (t.cpu().numpy() for t in b["out"])
        assert (st == ref["status"]).all()
        assert (c == ref["cost"]).all() and (ne == ref["n_expanded"]).all() and (pl == ref["path_len"]).all()
        for q in range(nq):
            assert (p[q, : pl[q]] == ref["path"][q, : pl[q]]).all()
        L.pmp_destroy(b["ctx"])


@pytest.mark.parametrize("per_cu", [56, 60], ids=["56_per_cu", "60_per_cu"])
def test_c2_headline_schedule_against_oracle(per_cu):
    """The bench's headline schedule (engine 2, 14,336 groups = 56 per CU since round 6, and round 5's
    60 per CU; several batches streamed through one launch longest first): two copies of the 4096 C2
    queries in one launch, every query bit-exact vs the oracle."""
    import torch

    from python_motion_planning_amd import _lib, batch

    c2 = _c2_oracle()
    occ, starts, goals, ref = c2["occ"], c2["starts"], c2["goals"], c2["ref"]
    W, H = occ.shape
    L, ctx = _lib.load_library(), _lib.context()
    try:
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 1), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve(ctx, W, H, 256 * per_cu, 0), "reserve")
        _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, per_cu), "residency")
        r = batch.astar2d_batch(occ, np.tile(starts, (2, 1)), np.tile(goals, (2, 1)), path_cap=4096, counters=True)
        torch.cuda.synchronize()
        _assert_c2_equal(ref, r, copies=2)
    finally:
        _lib.check(ctx, L.pmp_astar2d_set_residency(ctx, 0), "residency")
        _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, 1, 0), "engine")
        _lib.check(ctx, L.pmp_astar2d_reserve_auto(ctx), "reserve_auto")


def test_dropin_heap_beyond_single_query_capacity():
    """The drop-in AStar.plan() on a query whose heap (16,913 entries) outgrows the single-query
    engine's LDS heap: the kernel reports PMP_CAP_OVERFLOW and plan() re-runs it with the full bound
    (graph_search.AStar.plan) -- the answer, path and CLOSED order still equal the oracle's."""
    from oracle import oracle as O
    from python_motion_planning_amd import _lib

    pmp = _pmp()
    W = 1400
    occ = np.zeros((W, W), np.uint8)
    occ[0, :] = occ[-1, :] = occ[:, 0] = occ[:, -1] = 1
    occ[W // 2, 1:W - 40] = 1  # a wall across most of the grid: A* floods the near half first
    s, g = (W // 4, W // 2), (3 * W // 4, W // 2)
    ref = O.astar2d(occ, s, g)
    sq_cap = _lib.load_library().pmp_astar2d_sq_cap(W, W)
    assert sq_cap == 13632  # (160 KiB - 256 B) / 12 B, a multiple of 16 (no grid block at 1400^2)
    assert ref["status"] == 0 and ref["max_heap"] > sq_cap  # beyond the single-query engine's LDS heap
    env = pmp.Grid(W, W)
    env.update({(int(a), int(b)) for a, b in np.argwhere(occ)})
    cost, path, expand = pmp.AStar(s, g, env).plan()
    assert cost == ref["cost"] and path == ref["path"]
    assert [n.current[0] * W + n.current[1] for n in expand] == ref["expand_cells"].tolist()
