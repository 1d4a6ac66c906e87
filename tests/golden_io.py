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
