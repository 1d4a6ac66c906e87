"""TimeOptimalTrajectory3D on gfx950 (pmp_totp3d_batch) against the reference's own runs
(tests/golden/totp.npz, make_golden.py sec_totp) and the CPU restatement (oracle/pmp_oracle.c)."""
import numpy as np
import pytest

from golden_io import totp_cases, totp_compare

pytestmark = pytest.mark.gpu


def _prm(vmax, amax, tstep, res):
    from python_motion_planning_amd import _lib

    return _lib.TotpParams.make(vmax, amax, tstep, res)


def test_totp_against_reference_runs():
    from python_motion_planning_amd import batch

    for i, path, p, z in totp_cases():
        r = batch.totp3d_batch([path], _prm(*p))
        assert int(r["status"][0]) == 0
        npt = int(r["n_points"][0])
        prof = {k: r[k][0].cpu().numpy() for k in ("s_values", "s_dot", "s_ddot", "time")}
        totp_compare(z, i, int(r["n_samples"][0]), prof, npt, r["points"][0, :npt].cpu().numpy(),
                     float(r["total_time"][0]), rtol=1e-9)


def test_totp_batch_equals_single_runs():
    """All fixture paths of one parameter set in one launch give the per-path results."""
    from python_motion_planning_amd import batch

    cases = [(i, path, p) for i, path, p, _ in totp_cases() if p[3] == 0.05]
    r = batch.totp3d_batch([c[1] for c in cases], _prm(*cases[0][2]))
    for j, (i, path, p) in enumerate(cases):
        s = batch.totp3d_batch([path], _prm(*p))
        n = int(s["n_points"][0])
        assert int(r["n_points"][j]) == n
        a = r["points"][j, :n].cpu().numpy()
        b = s["points"][0, :n].cpu().numpy()
        assert np.array_equal(np.isnan(a), np.isnan(b))
        assert np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)])


def test_totp_c5_paths_vs_oracle():
    """256 C5 door paths planned by the 3D A* kernel, trajectories vs the CPU restatement."""
    from oracle import oracle as O
    from python_motion_planning_amd import batch, workloads as wl

    occ, s, g = wl.c5_workload(256)
    a = batch.astar3d_batch(occ, s, g)
    X, Y, Z = occ.shape[-3:]
    pl = a["path_len"].cpu().numpy()
    P = a["path"].cpu().numpy()
    paths = []
    for q in range(len(pl)):
        v = P[q, : pl[q]].astype(np.int64)
        if len(v) >= 2:
            paths.append(np.stack([v // (Y * Z), (v // Z) % Y, v % Z], axis=1).astype(np.float64))
    prm_args = ((2.0, 2.0, 1.5), (1.5, 1.5, 1.0), 0.05, 0.05)
    r = batch.totp3d_batch(paths, _prm(*prm_args))
    o = O.totp3d_batch(paths, O.TotpParams.make(*prm_args))
    assert (r["status"].cpu().numpy() == 0).all() and (o["status"] == 0).all()
    assert np.array_equal(r["n_samples"].cpu().numpy(), o["n_samples"])
    assert np.array_equal(r["n_points"].cpu().numpy(), o["n_points"])
    rp = r["points"].cpu().numpy()
    for q in range(len(paths)):
        n = int(o["n_points"][q])
        a_, b_ = rp[q, :n], o["points"][q, :n]
        assert np.array_equal(np.isnan(a_), np.isnan(b_)), q
        m = ~np.isnan(b_)
        assert np.max(np.abs(a_[m] - b_[m]) / np.maximum(1.0, np.abs(b_[m]))) <= 1e-9, q
    np.testing.assert_allclose(r["total_time"].cpu().numpy(), o["total_time"], rtol=1e-12)


def test_totp_point_overflow_is_retried():
    from python_motion_planning_amd import batch

    for i, path, p, z in totp_cases():
        if z["n_pts"][i] > 3000:
            r = batch.totp3d_batch([path], _prm(*p), point_cap=100)
            assert int(r["status"][0]) == 0 and int(r["n_points"][0]) == int(z["n_pts"][i])
            assert r["points"].shape[1] >= int(z["n_pts"][i])
            break


def test_totp_raises_like_reference():
    from python_motion_planning_amd import _lib, batch
    from python_motion_planning_amd.trajectory import TimeOptimalTrajectory3D

    r = batch.totp3d_batch([np.array([[1.0, 1.0, 1.0]]), np.array([[1.0, 1.0, 1.0], [1.0, 1.0, 1.0], [2.0, 1.0, 1.0]])],
                           _lib.TotpParams.make())
    assert r["status"].cpu().numpy().tolist() == [4, 4]
    with pytest.raises(ValueError):
        TimeOptimalTrajectory3D([(1, 1, 1)]).generate()


def test_dropin_time_optimal_trajectory():
    """The drop-in class as examples/3d_example.py:104-128 uses it."""
    from python_motion_planning_amd.trajectory import TimeOptimalTrajectory3D, TrajectoryConstraints

    for i, path, p, z in totp_cases():
        if p[3] != 0.05 or z["n_pts"][i] > 1500:
            continue
        cons = TrajectoryConstraints(max_velocity=np.array(p[0]), max_acceleration=np.array(p[1]),
                                     max_jerk=np.array([1.0, 1.0, 0.8]), min_time_step=p[2])
        tr = TimeOptimalTrajectory3D(path=[tuple(v) for v in path], constraints=cons, path_resolution=p[3])
        pts = tr.generate()
        pto = z["pts_off"]
        ref = z["pts"][pto[i]:pto[i + 1]]
        assert len(pts) == len(ref)
        for a, b in zip(pts, ref):
            assert abs(a.time - b[0]) <= 1e-9 * max(1, abs(b[0]))
            assert np.allclose(a.position, b[1:4], rtol=1e-9, atol=1e-9)
            assert (a.yaw is None) == np.isnan(b[10])
            assert (a.yaw_rate is None) == np.isnan(b[11])
        assert abs(tr.total_time - z["total_time"][i]) <= 1e-9 * tr.total_time
        # evaluate(t) at a sample time equals the generated point (yaw is generate()'s)
        e = tr.evaluate(pts[3].time)
        assert np.allclose(e.velocity, pts[3].velocity, rtol=1e-12, atol=1e-12) and e.yaw is None
        assert tr.check_constraints()["velocity_satisfied"] in (True, False)
        break
