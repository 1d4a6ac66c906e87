"""Loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def seg(flat, off, i):
    return flat[off[i]:off[i + 1]]


def grid_cases(name):
    """Yield (i, occ[W,H] or [X,Y,Z] uint8, fixture) for packed-occupancy fixtures."""
    z = load_npz(name)
    dims = z["dims"]
    for i in range(len(dims)):
        shape = tuple(int(v) for v in dims[i])
        n = int(np.prod(shape))
        occ = np.unpackbits(seg(z["occ_bits"], z["occ_off"], i))[:n].reshape(shape).astype(np.uint8)
        yield i, occ, z


def kkt_certificate(H, g, A, lo, hi, x, tol=1e-7):
    """Optimality certificate for min 1/2 x'Hx + g'x, lo <= Ax <= hi (H > 0): take the active set
    of x, solve the equality-constrained KKT system exactly, check feasibility and multiplier
    signs.  Returns the certified optimum x* (or None)."""
    Ax = A @ x
    act_hi = np.abs(Ax - hi) <= tol * (1 + np.abs(hi))
    act_lo = np.abs(Ax - lo) <= tol * (1 + np.abs(lo))
    act = act_hi | act_lo
    Aa = A[act]
    n, k = len(x), int(act.sum())
    K = np.block([[H, Aa.T], [Aa, np.zeros((k, k))]])
    b = np.concatenate([-g, np.where(act_hi[act], hi[act], lo[act])])
    sol = np.linalg.lstsq(K, b, rcond=None)[0]
    xs, lam = sol[:n], sol[n:]
    ok = (np.all(A @ xs <= hi + 1e-9) and np.all(A @ xs >= lo - 1e-9) and np.all(lam[act_hi[act]] >= -1e-9)
          and np.all(lam[act_lo[act]] <= 1e-9))
    return xs if ok else None


def totp_cases():
    """Yield (i, path [n, 3], params tuple (vmax, amax, tstep, res), fixture) for tests/golden/totp.npz
    (TimeOptimalTrajectory3D runs of the reference, make_golden.py sec_totp)."""
    z = load_npz("totp.npz")
    for i in range(len(z["total_time"])):
        c = z["cons"][i]
        yield i, seg(z["path"], z["path_off"], i), (tuple(c[0:3]), tuple(c[3:6]), float(c[6]), float(c[7])), z


def totp_compare(z, i, n_samples, prof, n_points, pts, total_time, rtol=1e-9):
    """Compare one trajectory with fixture case i: sample / point counts exact, profiles and points
    within rtol (relative to max(1, |ref|)), the NaN (= None) pattern of yaw / yaw rate exact."""
    po, pto = z["prof_off"], z["pts_off"]
    ns = int(po[i + 1] - po[i])
    assert int(n_samples) == ns
    assert int(n_points) == int(z["n_pts"][i])

    def close(a, b, what):
        a = np.asarray(a, np.float64)
        b = np.asarray(b, np.float64)
        assert a.shape == b.shape, what
        assert (np.isnan(a) == np.isnan(b)).all(), what
        m = ~np.isnan(b)
        err = np.abs(a[m] - b[m]) / np.maximum(1.0, np.abs(b[m]))
        assert err.size == 0 or err.max() <= rtol, (what, float(err.max()))

    for k in ("s_values", "s_dot", "s_ddot", "time"):
        close(prof[k][:ns], z[k][po[i]:po[i + 1]], f"case {i} {k}")
    idx = z["pts_idx"][pto[i]:pto[i + 1]]
    close(np.asarray(pts)[idx], z["pts"][pto[i]:pto[i + 1]], f"case {i} points")
    close([total_time], [z["total_time"][i]], f"case {i} total_time")
