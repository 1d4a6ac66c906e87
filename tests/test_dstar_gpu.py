"""HIP D* (dstar.hip via the C-ABI) vs the reference's golden runs and the oracle.

Bar: bit-exact -- processState count, cost bits, path cells; unreachable starts raise."""
import numpy as np
import pytest

from golden_io import grid_cases, seg

pytestmark = pytest.mark.gpu


def test_dstar_against_reference():
    from python_motion_planning_amd import batch

    for i, occ, z in grid_cases("dstar_small.npz"):
        r = batch.dstar2d_batch(occ, z["start"][i][None], z["goal"][i][None])
        st = int(r["status"][0])
        assert int(r["n_process"][0]) == z["n_process"][i], i
        if z["raised"][i]:
            assert st == 4, i
            continue
        assert st == 0, i
        assert float(r["cost"][0]) == z["cost"][i], i
        plen = int(r["path_len"][0])
        assert np.array_equal(r["path"][0, :plen].cpu().numpy(), seg(z["path"], z["path_off"], i)), i


@pytest.mark.parametrize("W,density,nq", [(96, 0.25, 48), (256, 0.15, 8)])
def test_dstar_batch_against_oracle(W, density, nq):
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ = wl.random_grid(W, W, density, seed=W)
    cells = wl.largest_component_cells(occ)
    rng = np.random.default_rng(W + 1)
    s = cells[rng.integers(0, len(cells), nq)]
    g = cells[rng.integers(0, len(cells), nq)]
    # a few unreachable starts: free cells outside the largest component
    free = np.argwhere(occ == 0)
    lab = {tuple(c) for c in cells.tolist()}
    outside = np.array([c for c in free.tolist() if tuple(c) not in lab][:2] or [s[0]])
    s[: len(outside)] = outside
    r = batch.dstar2d_batch(occ, s, g)
    st, npr = r["status"].cpu().numpy(), r["n_process"].cpu().numpy()
    cost, plen, path = r["cost"].cpu().numpy(), r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
    for q in range(nq):
        o = O.dstar2d(occ, s[q], g[q])
        assert st[q] == o["status"] and npr[q] == o["n_process"], q
        if o["status"] == 0:
            assert cost[q] == o["cost"]
            assert np.array_equal(path[q, : plen[q]], o["path_cells"])


def test_dstar_dropin_readme():
    import python_motion_planning_amd as pmp
    from oracle import oracle as O
    from python_motion_planning_amd import workloads as wl

    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
    cost, path, none = pmp.DStar((5, 5), (45, 25), env).plan()
    o = O.dstar2d(wl.readme_grid(), (5, 5), (45, 25))
    assert none is None and cost == o["cost"] and path == o["path"]
    assert path[0] == (5, 5) and path[-1] == (45, 25)
