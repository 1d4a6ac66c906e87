"""HIP LQR / MPC tracking controllers (track.hip via the C-ABI) vs the reference's golden vectors,
the oracle and -- for the MPC solve, whose OSQP parity is unpinned -- a KKT optimality certificate.

Bars: LQR controls and trajectories within 1e-12 / 1e-9 (device sin/cos <= 1 ulp from glibc);
MPC QP assembly within 1e-12 of max|H|, |g| (different but exact summation orders); the ADMM
solution within 1e-7 of the certified optimum and of the oracle's run of the same algorithm."""
import numpy as np
import pytest

from golden_io import kkt_certificate, load_npz

pytestmark = pytest.mark.gpu


def _pmp():
    import python_motion_planning_amd as pmp

    return pmp


def _readme_env(pmp):
    from python_motion_planning_amd import workloads as wl

    env = pmp.Grid(51, 31)
    env.update({(int(x), int(y)) for x, y in np.argwhere(wl.readme_grid())})
    return env


def _lp():
    from python_motion_planning_amd import _lib

    return _lib.LPParams.from_params(_pmp().LocalPlanner.DEFAULTS)


def test_lqr_control_against_reference():
    from python_motion_planning_amd import _lib, batch

    z = load_npz("lqr_control.npz")
    u = batch.lqr_control_batch(_lp(), _lib.LQRParams.make(), z["s"], z["s_d"], z["u_r"],
                                np.column_stack([z["v"], z["w"]])).cpu().numpy()
    np.testing.assert_allclose(u, z["u"], rtol=1e-12, atol=1e-14)


def test_lqr_plan_dropin_against_reference():
    pmp = _pmp()
    z = load_npz("local_plans.npz")
    env = _readme_env(pmp)
    ran = 0
    for c in range(4):
        if str(z[f"c{c}_kind"]) != "lqr":
            continue
        planner = pmp.LQR(tuple(z[f"c{c}_start"]), tuple(z[f"c{c}_goal"]), env)
        assert np.array_equal(np.asarray(planner.path, np.float64), z[f"c{c}_path"])
        ok, hist = planner.plan()
        assert ok == bool(z[f"c{c}_ok"])
        np.testing.assert_allclose(np.array(hist), z[f"c{c}_poses"], rtol=1e-9, atol=1e-9)
        ran += 1
    assert ran == 2


@pytest.mark.parametrize("P", [12, 30])
def test_mpc_control_against_reference_qp(P):
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch

    z = load_npz("mpc_qp.npz")
    n = len(z[f"p{P}_s"])
    vw = np.tile([0.2, 0.1], (n, 1))  # robot (v, w) when the vectors were captured
    for eps in (1e-9, 1e-3):  # drop-in default, OSQP's default
        mp = _lib.MPCParams.make(p=P, eps_abs=eps, eps_rel=eps)
        up = torch.tensor(z[f"p{P}_u_p"], dtype=torch.float64, device="cuda")
        out = batch.mpc_control_batch(_lp(), mp, z[f"p{P}_s"], z[f"p{P}_s_d"], z[f"p{P}_u_r"], up, vw, want_qp=True)
        H, g, lu = (out[k].cpu().numpy() for k in ("H", "g", "lu"))
        du, u, it, st = (out[k].cpu().numpy() for k in ("du", "u", "iters", "status"))
        up = up.cpu().numpy()
        omp = O.MPCParams.default(p=P, eps_abs=eps, eps_rel=eps)
        for i in range(n):
            Hr, gr = z[f"p{P}_P"][i], z[f"p{P}_q"][i]
            np.testing.assert_allclose(H[i], Hr, rtol=0, atol=1e-12 * np.abs(Hr).max())
            np.testing.assert_allclose(g[i], gr, rtol=0, atol=1e-12 * max(np.abs(gr).max(), 1e-300))
            assert np.array_equal(lu[i, 0], z[f"p{P}_l"][i]) and np.array_equal(lu[i, 1], z[f"p{P}_u"][i])
            assert st[i] == 0
            ou, oup, ost, oit = O.mpc_control(z[f"p{P}_s"][i], z[f"p{P}_s_d"][i], z[f"p{P}_u_r"][i],
                                              z[f"p{P}_u_p"][i], 0.2, 0.1, mpc=omp)
            assert ost == 0 and oit == it[i], (i, oit, it[i])
            np.testing.assert_allclose(u[i], ou, rtol=0, atol=1e-9)
            np.testing.assert_allclose(up[i], oup, rtol=0, atol=1e-9)
            if eps < 1e-6:
                xs = kkt_certificate(Hr, gr, z[f"p{P}_A"], z[f"p{P}_l"][i], z[f"p{P}_u"][i], du[i])
                assert xs is not None, i
                np.testing.assert_allclose(du[i], xs, rtol=0, atol=1e-7)


def _c4_paths(occ, states):
    from python_motion_planning_amd import batch

    na = len(states)
    r = batch.astar2d_batch(occ, states[:, :2].astype(np.int32), np.tile([45, 25], (na, 1)).astype(np.int32),
                            path_cap=2048)
    pl = r["path_len"].cpu().numpy()
    P = r["path"].cpu().numpy()
    H = occ.shape[1]
    return [np.column_stack([P[i, : pl[i]][::-1] // H, P[i, : pl[i]][::-1] % H]).astype(np.float64)
            for i in range(na)]


@pytest.mark.parametrize("kind", ["lqr", "mpc"])
def test_c4_track_batch_against_oracle(kind):
    """256 C4 agents, 40 plan iterations each, every agent checked against the oracle."""
    import torch

    from oracle import oracle as O
    from python_motion_planning_amd import _lib, batch, workloads as wl

    occ, states, goals = wl.c4_workload(256)
    paths = _c4_paths(occ, states)
    xy, off = batch.pack_paths(paths)
    st_d = torch.tensor(states, dtype=torch.float64, device="cuda")
    up_d = torch.zeros((256, 2), dtype=torch.float64, device="cuda")
    kw = dict(lqr_params=_lib.LQRParams.make()) if kind == "lqr" else dict(mpc_params=_lib.MPCParams.make(p=30))
    out = batch.track_step_batch(kind, _lp(), st_d, goals, xy, off, iters=40, u_p=up_d, want_hist=True, **kw)
    ost, oup, ou, ostat, onst, _ = O.track_batch(kind, xy, off, goals, states, iters=40,
                                                 mpc=O.MPCParams.default(p=30, eps_abs=1e-9, eps_rel=1e-9))
    assert np.array_equal(out["status"].cpu().numpy(), ostat)
    assert np.array_equal(out["n_steps"].cpu().numpy(), onst)
    tol = 1e-9 if kind == "lqr" else 1e-6
    np.testing.assert_allclose(st_d.cpu().numpy(), ost, rtol=0, atol=tol)
    if kind == "mpc":
        np.testing.assert_allclose(up_d.cpu().numpy(), oup, rtol=0, atol=tol)
        assert int(out["admm_iters"].sum()) > 0


def test_mpc_plan_dropin_against_oracle():
    """MPC.plan on the README scenario (mpc.py:56-94) vs the oracle's plan loop (parity with the
    reference's OSQP-based run is unpinned; the loop around the solve is pinned by the LQR runs)."""
    from oracle import oracle as O

    pmp = _pmp()
    env = _readme_env(pmp)
    planner = pmp.MPC((5, 5, 0), (45, 25, 0), env)
    ok, hist = planner.plan()
    st = np.array([5.0, 5.0, 0.0, 0.0, 0.0])
    up = np.zeros(2)
    poses = []
    for _ in range(1500):
        rc, st2, up, u, _ = O.track_step("mpc", np.asarray(planner.path, np.float64), (45, 25, 0), st, up,
                                         mpc=O.MPCParams.default(eps_abs=1e-9, eps_rel=1e-9))
        if rc == 1:
            break
        assert rc == 0
        poses.append(st[:3].copy())
        st = st2
    assert ok == (rc == 1)
    assert len(hist) == len(poses)
    np.testing.assert_allclose(np.array(hist), np.array(poses), rtol=0, atol=1e-6)
