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
