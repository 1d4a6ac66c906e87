"""Host marshalling (csrc/hostio.c, the _hostio extension) -- SURVEY.md §8(f) rank 2: the obstacle
set -> bit-grid conversion and the CLOSED Node lists, against the reference's own objects.  CPU only."""
import numpy as np

from golden_io import load_json


def test_set_to_words_matches_numpy():
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import _hostio, workloads as wl

    occ, _, _ = wl.c2_workload(nq=1, W=333, H=257)
    obs = {(int(x), int(y)) for x, y in np.argwhere(occ)}
    obs |= {(-1, 3), (333, 0), (5, 257), (np.int64(7), np.int32(9))}  # off-grid and numpy-int entries
    ref = occ.copy()
    ref[7, 9] = 1
    w = np.empty((333 * 257 + 31) // 32, np.uint32)
    n = _hostio.set_to_words(obs, (333, 257), w)
    assert n == int(ref.sum())
    assert np.array_equal(w, pmp.pack_bits(ref))
    env = pmp.Grid(333, 257)
    env.update(obs)
    assert np.array_equal(env.occupancy(), ref)
    # 3D
    o3 = (np.random.default_rng(1).random((13, 7, 5)) < 0.3).astype(np.uint8)
    e3 = pmp.Grid3D(13, 7, 5)
    e3.update({(int(a), int(b), int(c)) for a, b, c in np.argwhere(o3)} | {(13, 0, 0)})
    assert np.array_equal(e3.occupancy(), o3)


def test_expand_nodes_match_reference_objects():
    """The reference's CLOSED nodes for the README query (AStar / Dijkstra / GBFS, both
    heuristics): current, parent, repr and type of g and h, rebuilt from (cell | dir << 28)."""
    import python_motion_planning_amd as pmp
    from python_motion_planning_amd import _hostio

    env = pmp.Grid(51, 31)
    motions = env.motions
    dirs = {(m.x, m.y): d for d, m in enumerate(motions)}
    kinds = {("astar", "euclidean"): 0, ("astar", "manhattan"): 1, ("dijkstra", "euclidean"): 2,
             ("dijkstra", "manhattan"): 2, ("gbfs", "euclidean"): 3, ("gbfs", "manhattan"): 4}
    for case in load_json("astar_nodes.json"):
        rec = []
        for cur, par, *_ in case["nodes"]:
            d = 8 if cur == par else dirs[(cur[0] - par[0], cur[1] - par[1])]
            rec.append((cur[0] * 31 + cur[1]) | (d << 28))
        rec = np.array(rec, np.uint32)
        nodes = _hostio.expand_nodes(rec, len(rec), 31, [(m.x, m.y) for m in motions], [m.g for m in motions],
                                     (45, 25), kinds[(case["algo"], case["heuristic"])], pmp.Node)
        assert len(nodes) == len(case["nodes"])
        for n, (cur, par, g, gt, h, ht) in zip(nodes, case["nodes"]):
            assert list(n.current) == cur and list(n.parent) == par
            assert repr(n.g) == g and type(n.g).__name__ == gt, (case["algo"], cur)
            assert repr(n.h) == h and type(n.h).__name__ == ht, (case["algo"], cur)
