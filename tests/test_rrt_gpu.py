"""HIP RRT / RRT* (rrt.hip via the C-ABI) vs the reference's trees and the oracle.

Bar: every tree node's parent index and the draw count equal; coordinates and costs within 1e-12
relative (the device atan2/cos/sin are <= 1 ulp from glibc, which steering feeds into the node
coordinates)."""
import numpy as np
import pytest

from golden_io import load_npz

pytestmark = pytest.mark.gpu


def _map(kind):
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import workloads as wl

    if kind == "readme":
        env = pmp.Map(51, 31)
        env.update(obs_rect=wl.README_MAP_RECT, obs_circ=wl.README_MAP_CIRC)
    else:
        env = pmp.Map(512, 512)
        rects, circs = wl.c3_map()
        env.update(obs_rect=rects, obs_circ=circs)
    return env


def _check_tree(out, q, ref, what):
    n = int(out["n_nodes"][q])
    assert n == len(ref), (what, n, len(ref))
    xy = out["tree_xy"][q, :n].cpu().numpy()
    g = out["tree_g"][q, :n].cpu().numpy()
    par = out["tree_parent"][q, :n].cpu().numpy()
    assert np.array_equal(par, ref[:, 3].astype(np.int32)), what
    np.testing.assert_allclose(xy, ref[:, :2], rtol=1e-12, atol=0, err_msg=what)
    np.testing.assert_allclose(g, ref[:, 2], rtol=1e-12, atol=0, err_msg=what)
    return bool(np.array_equal(xy, ref[:, :2]) and np.array_equal(g, ref[:, 2]))


def test_trees_against_reference():
    """All 25 captured reference runs (README map RRT/RRT* seeds 0..9, C3 RRT* 2000/5000 samples)."""
    from python_motion_planning_amd import batch

    z = load_npz("rrt.npz")
    groups = {}
    for i in range(int(z["n_cases"])):
        key = (str(z[f"c{i}_kind"]), str(z[f"c{i}_map"]), int(z[f"c{i}_sample_num"]))
        groups.setdefault(key, []).append(i)
    exact = 0
    for (kind, mp, sn), idx in groups.items():
        env = _map(mp)
        rnd = np.stack([np.random.RandomState(int(z[f"c{i}_seed"])).random_sample(3 * sn + 1) for i in idx])
        out = batch.rrt_batch(env, [z[f"c{i}_start"] for i in idx], [z[f"c{i}_goal"] for i in idx], rnd, sn,
                              star=kind == "rrt_star")
        for q, i in enumerate(idx):
            exact += _check_tree(out, q, z[f"c{i}_tree"], (kind, mp, i))
            assert (int(out["status"][q]) == 0) == bool(z[f"c{i}_found"])
            assert rnd[q, int(out["draws"][q])] == z[f"c{i}_next"]
            if bool(z[f"c{i}_found"]):
                assert abs(float(out["cost"][q]) - float(z[f"c{i}_cost"])) <= 1e-12 * float(z[f"c{i}_cost"])
                plen = int(out["path_len"][q])
                np.testing.assert_allclose(out["path"][q, :plen].cpu().numpy(), z[f"c{i}_path"], rtol=1e-12)
    print(f"{exact}/{int(z['n_cases'])} trees bit-exact")


def test_rrt_star_dropin_readme():
    """pmp.RRTStar((18, 8), (37, 18), README map).plan() with np.random.seed(0): the reference's
    cost, path, node count, and the global RNG left where the reference leaves it."""
    import python_motion_planning_amd as pmp

    z = load_npz("rrt.npz")
    i = 10  # rrt_star, readme, seed 0
    assert str(z[f"c{i}_kind"]) == "rrt_star" and int(z[f"c{i}_seed"]) == 0
    planner = pmp.RRTStar((18, 8), (37, 18), _map("readme"))
    np.random.seed(0)
    cost, path, expand = planner.plan()
    assert np.random.random() == z[f"c{i}_next"]
    assert abs(cost - 26.33608540485134) <= 1e-12 * cost
    assert len(expand) == len(z[f"c{i}_tree"]) and len(path) == len(z[f"c{i}_path"])
    np.testing.assert_allclose(np.array(path, np.float64), z[f"c{i}_path"], rtol=1e-12)
    assert path[0] == (37, 18) and path[-1] == (18, 8)


def test_c3_batch_against_oracle():
    """C3 map, 32 queries (np.random.seed(q)) x 3000 samples: every tree vs the oracle."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    env = _map("c3")
    rects, circs = wl.c3_map()
    nq, sn = 32, 3000
    rnd = np.stack([np.random.RandomState(q).random_sample(3 * sn + 1) for q in range(nq)])
    starts, goals = np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1))
    out = batch.rrt_batch(env, starts, goals, rnd, sn, star=True)
    ref = O.rrt_batch(True, rects, circs, 512, 512, starts, goals, rnd, sn)
    for q in range(nq):
        _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], q)
        assert int(out["status"][q]) == ref["status"][q]


def test_c3_midsize_against_oracle():
    """C3 map, 8 queries x 12,000 samples (trees of ~9.4k nodes, past the 3,000-sample batch test and
    into the sizes where rewiring lists are long): whole RRT* trees (parents, draw counts; coordinates
    to 1e-12) equal to the oracle's, and four plain-RRT trees."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    env = _map("c3")
    rects, circs = wl.c3_map()
    nq, sn = 8, 12000
    rnd = np.stack([np.random.RandomState(500 + q).random_sample(3 * sn + 1) for q in range(nq)])
    starts, goals = np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1))
    out = batch.rrt_batch(env, starts, goals, rnd, sn, star=True)
    ref = O.rrt_batch(True, rects, circs, 512, 512, starts, goals, rnd, sn)
    assert (ref["n_nodes"] > 3000).all()
    for q in range(nq):
        _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], q)
        assert int(out["status"][q]) == ref["status"][q]
    # plain RRT through the same index (nearest only)
    out = batch.rrt_batch(env, starts[:4], goals[:4], rnd[:4], sn, star=False)
    ref = O.rrt_batch(False, rects, circs, 512, 512, starts[:4], goals[:4], rnd[:4], sn)
    for q in range(4):
        _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], q)
        assert int(out["status"][q]) == ref["status"][q]


def test_rrt_star_dense_ball_against_oracle():
    """README map with the goal inside an obstacle (never connected, so the tree takes every sample):
    6,000 samples on 51x31 put hundreds of nodes in one r = 10 ball, past the kernel's 512 staged
    coarse hits -- the rescan path (rrt.hip 4a) -- and the trees equal the oracle's."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    env = _map("readme")
    nq, sn = 4, 6000
    rnd = np.stack([np.random.RandomState(900 + q).random_sample(3 * sn + 1) for q in range(nq)])
    starts, goals = np.tile([5.0, 5.0], (nq, 1)), np.tile([27.0, 13.0], (nq, 1))  # inside rect (26, 7, 2, 12)
    out = batch.rrt_batch(env, starts, goals, rnd, sn, star=True, counters=True)
    ref = O.rrt_batch(True, wl.README_MAP_RECT, wl.README_MAP_CIRC, 51, 31, starts, goals, rnd, sn)
    assert (ref["n_nodes"] > 3500).all()
    # in-radius candidates per iteration: a ball of this tree holds hundreds of nodes
    c = out["counters"].cpu().numpy()
    assert (c[:, 2] / np.maximum(c[:, 0], 1)).max() > 200
    for q in range(nq):
        _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], q)
        assert int(out["status"][q]) == ref["status"][q]


def test_c3_full_size_properties():
    """C3 at BASELINE size (65,536 samples), 4 queries: the four whole trees against the oracle, and tree
    invariants on every node of all four -- parents reach the start without cycles, g >= g(parent) +
    edge length (rewires never raise a cost), sampled edges collision-free under the oracle's
    isCollision, draw counts consistent."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    env = _map("c3")
    rects, circs = wl.c3_map()
    nq, sn = 4, 65536
    rnd = np.stack([np.random.RandomState(100 + q).random_sample(3 * sn + 1) for q in range(nq)])
    out = batch.rrt_batch(env, np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1)), rnd, sn, star=True)
    # all four trees against the oracle at full size (the oracle's OpenMP runs them in parallel)
    ref = O.rrt_batch(True, rects, circs, 512, 512, np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1)),
                      rnd, sn)
    for q in range(nq):
        _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], q)
        assert int(out["status"][q]) == ref["status"][q]
    rng = np.random.default_rng(0)
    for q in range(nq):
        assert int(out["status"][q]) in (0, 1)
        n = int(out["n_nodes"][q])
        xy = out["tree_xy"][q, :n].cpu().numpy()
        g = out["tree_g"][q, :n].cpu().numpy()
        par = out["tree_parent"][q, :n].cpu().numpy().astype(np.int64)
        assert par[0] == 0 and g[0] == 0
        assert n > 10000 and int(out["draws"][q]) <= 3 * sn + 1
        # every node reaches the start: pointer doubling over the parent array
        p = par.copy()
        for _ in range(20):
            p = p[p]
        assert np.all(p == 0)
        edge = np.hypot(xy[:, 0] - xy[par, 0], xy[:, 1] - xy[par, 1])
        assert np.all(g[1:] >= g[par[1:]] + edge[1:] - 1e-9)
        for j in rng.choice(np.arange(1, n), 200, replace=False):
            assert not O.map_collision(rects, circs, 512, 512, xy[j], xy[par[j]])


@pytest.mark.parametrize("case", ["long_segments", "many_obstacles"])
def test_collision_bins_edge_cases_against_oracle(case):
    """The obstacle bins (rrt.hip, round 5) on the paths the C3 runs do not take: segments whose
    bounding box meets more than 9 bins (max_dist 60, radius 80: the full item list instead), and a
    map of more than 128 obstacles (no bins at all).  RRT* and RRT trees vs the oracle."""
    import python_motion_planning_amd as pmp
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    if case == "long_segments":
        rects, circs = wl.c3_map()
        kw = dict(max_dist=60.0, radius=80.0)
        sn = 600
    else:
        rects, circs = wl.c3_map(n_rect=80, n_circ=60, seed=11)
        kw = {}
        sn = 1500
    env = pmp.Map(512, 512)
    env.update(obs_rect=rects, obs_circ=circs)
    nq = 16
    rnd = np.stack([np.random.RandomState(500 + q).random_sample(3 * sn + 1) for q in range(nq)])
    starts, goals = np.tile([5.0, 5.0], (nq, 1)), np.tile([505.0, 505.0], (nq, 1))
    for star in (True, False):
        out = batch.rrt_batch(env, starts, goals, rnd, sn, star=star, **kw)
        ref = O.rrt_batch(star, rects, circs, 512, 512, starts, goals, rnd, sn, **kw)
        for q in range(nq):
            _check_tree(out, q, ref["tree"][q, : ref["n_nodes"][q]], (case, star, q))
            assert int(out["status"][q]) == ref["status"][q]
