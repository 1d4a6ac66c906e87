"""HIP DWA control step (dwa.hip via the C-ABI) vs the reference's golden vectors and the oracle.

Bar (north_star): trajectories within 1e-12 relative (device sin/cos/atan2 are <= 1 ulp from glibc);
discrete decisions (argmax) equal, or -- only on a near-tie -- a score within 1e-12 of the best."""
import numpy as np
import pytest

from golden_io import load_npz, seg

pytestmark = pytest.mark.gpu


def _pmp():
    import python_motion_planning_amd as pmp

    return pmp


def _readme_env(pmp):
    from python_motion_planning_amd import workloads as wl

    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
    return env


def test_evaluation_against_reference():
    import torch

    pmp = _pmp()
    from python_motion_planning_amd import _lib, batch

    z = load_npz("dwa_eval.npz")
    env = _readme_env(pmp)
    grid = batch.obstacle_grid(env.obstacles)
    xy, off = batch.pack_paths([z["path"]])
    lp = _lib.LPParams.from_params(pmp.LocalPlanner.DEFAULTS)
    for i in range(len(z["state"])):
        dp = _lib.DWAParams(0.2, 0.1, 0.05, float(z["predict_time"][i]), 1.0, float(z["v_res"][i]),
                            float(z["w_res"][i]), 0, 0)
        state = torch.tensor(z["state"][i][None], dtype=torch.float64, device="cuda")
        out = batch.dwa_step_batch(grid, lp, dp, state, np.array([[45.0, 25.0, 0.0]]), xy, off, iters=1,
                                   want_eval=True, want_traj=True)
        assert int(out["status"][0]) == 0
        ref = seg(z["eval"], z["eval_off"], i).reshape(-1, 3)
        ev = out["eval"][0, : len(ref)].cpu().numpy()
        np.testing.assert_allclose(ev, ref, rtol=1e-12, atol=1e-15)
        b = int(out["best"][0])
        if b != z["best"][i]:  # tie-aware: only a near-tie may pick another sample
            assert abs(ref[b, 2] - ref[z["best"][i], 2]) <= 1e-12 * abs(ref[z["best"][i], 2])
        else:
            bt = out["best_traj"][0, 0].cpu().numpy()
            np.testing.assert_allclose(bt, seg(z["best_traj"], z["best_traj_off"], i).reshape(-1, 5), rtol=1e-12)


def test_dwa_plan_dropin_against_reference():
    pmp = _pmp()
    z = load_npz("local_plans.npz")
    env = _readme_env(pmp)
    planner = pmp.DWA((5, 5, 0), (45, 25, 0), env)
    assert np.array_equal(np.asarray(planner.path, np.float64), z["c0_path"])
    ok, hist_traj, hist_pose = planner.plan()
    assert ok and bool(z["c0_ok"])
    ref = z["c0_poses"]
    assert len(hist_pose) == len(ref)
    np.testing.assert_allclose(np.array(hist_pose), ref, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(np.array([t[0, 3:5] for t in hist_traj]), z["c0_u"], rtol=1e-9, atol=1e-12)


def test_c4_batch_against_oracle():
    """C4: 256 agents x 4096 samples x H=30, one step; every agent checked against the oracle, and
    properties on all."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, states, goals = wl.c4_workload(256)
    ref_paths = []
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (256, 1)).astype(np.int32),
                            path_cap=2048)
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    H = occ.shape[1]
    for i in range(256):
        cells = P[i, : pl[i]][::-1]
        ref_paths.append(np.column_stack([cells // H, cells % H]).astype(np.float64))
    xy, off = batch.pack_paths(ref_paths)
    lp = _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, 64, 64)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
    out = batch.dwa_step_batch(grid, lp, dp, st_d, goals, xy, off, iters=1, want_eval=True)
    status = out["status"].cpu().numpy()
    new_st = st_d.cpu().numpy()
    u = out["u"].cpu().numpy()
    obs = np.argwhere(occ).astype(np.float64)
    for i in range(256):  # every agent against the oracle
        rc, ost, ou = O.dwa_step(obs, ref_paths[i], goals[i], states[i], nv=64, nw=64, predict_time=3.0)
        assert rc == status[i], i
        if rc != 0:
            continue
        np.testing.assert_allclose(new_st[i], ost, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(u[i], ou, rtol=1e-12, atol=1e-14)
    # properties: stepped agents moved with an admissible control from their dynamic window
    for i in range(256):
        if status[i] != 0:
            continue
        vr = O.dwa_window(states[i, 3], states[i, 4])
        assert vr[0] - 1e-12 <= u[i, 0] <= vr[1] + 1e-12 and vr[2] - 1e-12 <= u[i, 1] <= vr[3] + 1e-12


@pytest.mark.parametrize("inflation", [3.0, 9.5, 20.0])
def test_large_inflation_against_oracle(inflation):
    """The obstacle stencil covers any inflation radius (dwa.py:162-164: min(cdist(...), R) over all
    obstacles): radii above 8 cells need several bit runs per stencil row."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, states, goals = wl.c4_workload(16, seed=5)
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (16, 1)).astype(np.int32),
                            path_cap=2048)
    pl, P = r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
    H = occ.shape[1]
    paths = [np.column_stack([P[i, : pl[i]][::-1] // H, P[i, : pl[i]][::-1] % H]).astype(np.float64)
             for i in range(16)]
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, inflation, 0.05, 0.05, 32, 32)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
    out = batch.dwa_step_batch(grid, lp, dp, st_d, goals, xy, off, iters=1)
    status = out["status"].cpu().numpy()
    new_st, u = st_d.cpu().numpy(), out["u"].cpu().numpy()
    obs = np.argwhere(occ).astype(np.float64)
    for i in range(16):
        rc, ost, ou = O.dwa_step(obs, paths[i], goals[i], states[i], nv=32, nw=32, predict_time=3.0,
                                 inflation=inflation)
        assert rc == status[i], i
        if rc == 0:
            np.testing.assert_allclose(new_st[i], ost, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(u[i], ou, rtol=1e-12, atol=1e-14)


def _c4_inputs(na, seed=None):
    from python_motion_planning_amd import batch, workloads as wl

    occ, states, goals = wl.c4_workload(256) if seed is None else wl.c4_workload(na, seed=seed)
    occ, states, goals = occ, states[:na], goals[:na]
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (na, 1)).astype(np.int32),
                            path_cap=2048)
    pl, P = r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
    H = occ.shape[1]
    paths = [np.column_stack([P[i, : pl[i]][::-1] // H, P[i, : pl[i]][::-1] % H]).astype(np.float64)
             for i in range(na)]
    return occ, states, goals, paths


def test_c4_split_32_agents_against_oracle():
    """The 8-GPU strong split's per-rank share (32 of C4's 256 agents): with fewer agents than CUs the
    default splits each agent's 4096 samples over several workgroups (leaf-aligned parts of numpy's
    pairwise tree, dwa.py:176-181; first-index argmax across parts, dwa.py:89).  Every agent against
    the oracle, and the evaluation rows bit-equal to one workgroup per agent."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch

    occ, states, goals, paths = _c4_inputs(32)
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, 64, 64)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    outs = {}
    for parts in (0, 1):
        st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
        o = batch.dwa_step_batch(grid, lp, dp, st_d, goals, xy, off, iters=1, want_eval=True, want_traj=True,
                                 parts=parts)
        torch.cuda.synchronize()
        outs[parts] = {k: v.cpu().numpy() for k, v in o.items() if v is not None}
        outs[parts]["state"] = st_d.cpu().numpy()
    for k in outs[1]:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    obs = np.argwhere(occ).astype(np.float64)
    for i in range(32):
        rc, ost, ou = O.dwa_step(obs, paths[i], goals[i], states[i], nv=64, nw=64, predict_time=3.0)
        assert rc == outs[0]["status"][i], i
        if rc == 0:
            np.testing.assert_allclose(outs[0]["state"][i], ost, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(outs[0]["u"][i], ou, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("nv", [64, 40])
def test_split_parts_bit_equal(nv):
    """Any number of parts (incl. uneven leaf counts, more requested parts than leaves, a 40 x 40 window
    whose pairwise tree has uneven leaves) gives the bits of one workgroup per agent over several plan
    iterations, including an agent that starts at its goal (status 1 at iteration 0)."""
    import torch

    from python_motion_planning_amd import _lib, batch

    occ, states, goals, paths = _c4_inputs(24, seed=3)
    states = states.copy()
    states[5, :3] = goals[5]  # at the goal: reachGoal stops it before any step
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, 1.0, 0.05, 0.05, nv, nv)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    ref = None
    for parts in (1, 2, 3, 5, 8, 16, 64):
        st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
        o = batch.dwa_step_batch(grid, lp, dp, st_d, goals, xy, off, iters=4, want_eval=True, want_traj=True,
                                 want_hist=True, parts=parts)
        torch.cuda.synchronize()
        got = {k: v.cpu().numpy() for k, v in o.items() if v is not None}
        got["state"] = st_d.cpu().numpy()
        assert got["status"][5] == 1 and got["n_steps"][5] == 0
        if ref is None:
            ref = got
            assert (got["n_steps"] > 0).sum() >= 20
            continue
        for k in ref:
            assert np.array_equal(got[k], ref[k]), (parts, k)


@pytest.mark.parametrize("inflation", [0.0, 0.5, 1.0, 1.5, 1.999])
def test_small_radius_dense_obstacles_against_oracle(inflation):
    """Radii below 2 take the 3 x 3 stencil behind the dilated-occupancy skip (dwa.hip rollout_small):
    a grid with extra random obstacles (most trajectory points near one, several cells per stencil),
    every agent against the oracle (dwa.py:162-164 over the obstacle list), one workgroup and the
    k-split kernel both."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, states, goals = wl.c4_workload(48, seed=7)
    rng = np.random.default_rng(11)
    occ = occ.copy()
    occ |= rng.random(occ.shape) < 0.12
    keep = [i for i in range(48)]
    for i in keep:
        occ[int(states[i, 0]), int(states[i, 1])] = False
    occ[45, 25] = False
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (48, 1)).astype(np.int32),
                            path_cap=2048)
    pl, P = r["path_len"].cpu().numpy(), r["path"].cpu().numpy()
    keep = [i for i in range(48) if pl[i] > 1][:24]
    assert len(keep) >= 12
    H = occ.shape[1]
    paths = [np.column_stack([P[i, : pl[i]][::-1] // H, P[i, : pl[i]][::-1] % H]).astype(np.float64) for i in keep]
    states, goals = states[keep], goals[keep]
    xy, off = batch.pack_paths(paths)
    lp = _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)
    dp = _lib.DWAParams(0.2, 0.1, 0.05, 3.0, inflation, 0.05, 0.05, 32, 32)
    grid = batch.obstacle_grid({(int(a), int(b)) for a, b in np.argwhere(occ)})
    obs = np.argwhere(occ).astype(np.float64)
    for parts in (1, 4):
        st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
        out = batch.dwa_step_batch(grid, lp, dp, st_d, goals, xy, off, iters=1, parts=parts)
        status, new_st, u = out["status"].cpu().numpy(), st_d.cpu().numpy(), out["u"].cpu().numpy()
        for i in range(len(keep)):
            rc, ost, ou = O.dwa_step(obs, paths[i], goals[i], states[i], nv=32, nw=32, predict_time=3.0,
                                     inflation=inflation)
            assert rc == status[i], (parts, i)
            if rc == 0:
                np.testing.assert_allclose(new_st[i], ost, rtol=1e-12, atol=1e-14)
                np.testing.assert_allclose(u[i], ou, rtol=1e-12, atol=1e-14)
