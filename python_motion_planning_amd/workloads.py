"""Synthetic workloads of BASELINE.json's configs, generated from fixed seeds.

These build the INPUTS of the hot path (occupancy grids, start/goal pairs, agent states);
no planning happens here.  Layout convention everywhere: occupancy ``occ[x, y]`` (x-major,
cell id ``x * H + y``), matching the reference's ``(x, y)`` obstacle tuples
(utils/environment/env.py:41-80).
"""
from __future__ import annotations

import random

import numpy as np


# --------------------------------------------------------------------------------------------
# 2D grids
# --------------------------------------------------------------------------------------------
def boundary_grid(W: int, H: int) -> np.ndarray:
    """Grid.init (env.py:57-76): the four boundary rows/columns are obstacles."""
    occ = np.zeros((W, H), np.uint8)
    occ[:, 0] = occ[:, H - 1] = 1
    occ[0, :] = occ[W - 1, :] = 1
    return occ


def readme_grid() -> np.ndarray:
    """C1: Grid(51, 31) plus the README / examples/global_examples.py:23-33 walls."""
    occ = boundary_grid(51, 31)
    for i in range(10, 21):
        occ[i, 15] = 1
    for i in range(15):
        occ[20, i] = 1
    for i in range(15, 30):
        occ[30, i] = 1
    for i in range(16):
        occ[40, i] = 1
    return occ


def random_grid(W: int, H: int, density: float, seed: int) -> np.ndarray:
    occ = (np.random.default_rng(seed).random((W, H)) < density).astype(np.uint8)
    occ[:, 0] = occ[:, H - 1] = 1
    occ[0, :] = occ[W - 1, :] = 1
    return occ


def largest_component_cells(occ: np.ndarray) -> np.ndarray:
    """Free cells of the largest 4-connected free component (reachability under the
    no-corner-cutting rule of graph_search.py:78-86 is exactly 4-connectivity)."""
    from scipy import ndimage

    lab, n = ndimage.label(occ == 0)
    if n == 0:
        return np.zeros((0, 2), np.int64)
    sizes = np.bincount(lab.ravel())
    sizes[0] = 0
    return np.argwhere(lab == int(np.argmax(sizes)))


def c2_workload(nq: int = 4096, W: int = 1024, H: int = 1024, density: float = 0.2,
                grid_seed: int = 0, pair_seed: int = 1):
    """C2: 1024^2 grid, 20 % random obstacles (default_rng(0)), boundary walls, nq start/goal
    pairs drawn from the largest free component with default_rng(1)."""
    occ = random_grid(W, H, density, grid_seed)
    cells = largest_component_cells(occ)
    rng = np.random.default_rng(pair_seed)
    starts = cells[rng.integers(0, len(cells), nq)].astype(np.int32)
    goals = cells[rng.integers(0, len(cells), nq)].astype(np.int32)
    return occ, starts, goals


def occ_from_obstacles(obstacles, W: int, H: int) -> np.ndarray:
    occ = np.zeros((W, H), np.uint8)
    if obstacles:
        a = np.asarray(list(obstacles), dtype=np.int64).reshape(-1, 2)
        m = (a[:, 0] >= 0) & (a[:, 0] < W) & (a[:, 1] >= 0) & (a[:, 1] < H)
        occ[a[m, 0], a[m, 1]] = 1
    return occ


# --------------------------------------------------------------------------------------------
# 3D scenarios: semantics of examples/scenarios.py (shell, door, floors, maze, city) and
# carve_safety_bubble, re-implemented on a dense uint8 [X, Y, Z] array.
# --------------------------------------------------------------------------------------------
def shell3d(X: int, Y: int, Z: int) -> np.ndarray:
    occ = np.zeros((X, Y, Z), np.uint8)
    occ[[0, X - 1], :, :] = 1
    occ[:, [0, Y - 1], :] = 1
    occ[:, :, [0, Z - 1]] = 1
    return occ


def scenario_door(X, Y, Z, door_size=2):
    occ = shell3d(X, Y, Z)
    x0 = X // 2
    occ[x0, 1:Y - 1, 1:Z - 1] = 1
    ym, zm = Y // 2, Z // 2
    for dy in range(-(door_size // 2), door_size - door_size // 2):
        for dz in range(-(door_size // 2), door_size - door_size // 2):
            occ[x0, ym + dy, zm + dz] = 0
    return occ


def scenario_floors(X, Y, Z, floors=3, hole_size=2):
    occ = shell3d(X, Y, Z)
    zs = [Z * (i + 1) // (floors + 1) for i in range(floors)]
    for i, z0 in enumerate(zs):
        occ[1:X - 1, 1:Y - 1, z0] = 1
        hx = 2 + (i * 3) % (X - 4)
        hy = 2 + (i * 2) % (Y - 4)
        for dx in range(hole_size):
            for dy in range(hole_size):
                occ[min(X - 2, hx + dx), min(Y - 2, hy + dy), z0] = 0
    return occ


def scenario_maze(X, Y, Z, seed=0, vertical_connector_prob=0.12):
    rng = random.Random(seed)

    def odd_interior(x, y, z):
        return (1 <= x < X - 1 and 1 <= y < Y - 1 and 1 <= z < Z - 1
                and x % 2 == 1 and y % 2 == 1 and z % 2 == 1)

    start = (1, 1, 1)
    if not odd_interior(*start):
        return shell3d(X, Y, Z)
    stack = [start]
    visited = {start}
    passages = {start}
    dirs = [(2, 0, 0), (-2, 0, 0), (0, 2, 0), (0, -2, 0), (0, 0, 2), (0, 0, -2)]
    while stack:
        cx, cy, cz = stack[-1]
        rng.shuffle(dirs)
        advanced = False
        for dx, dy, dz in dirs:
            nx, ny, nz = cx + dx, cy + dy, cz + dz
            if not odd_interior(nx, ny, nz) or (nx, ny, nz) in visited:
                continue
            passages.add((cx + dx // 2, cy + dy // 2, cz + dz // 2))
            passages.add((nx, ny, nz))
            visited.add((nx, ny, nz))
            stack.append((nx, ny, nz))
            advanced = True
            break
        if not advanced:
            stack.pop()
    if Z >= 5 and vertical_connector_prob > 0:
        for x in range(1, X - 1, 2):
            for y in range(1, Y - 1, 2):
                for z in range(3, Z - 2, 2):
                    if (x, y, z) in passages and (x, y, z - 2) in passages and rng.random() < vertical_connector_prob:
                        passages.add((x, y, z - 1))
                    if (x, y, z) in passages and (x, y, z + 2) in passages and rng.random() < vertical_connector_prob:
                        passages.add((x, y, z + 1))
    occ = shell3d(X, Y, Z)
    occ[1:X - 1, 1:Y - 1, 1:Z - 1] = 1
    for (x, y, z) in passages:
        if 1 <= x < X - 1 and 1 <= y < Y - 1 and 1 <= z < Z - 1:
            occ[x, y, z] = 0
    return occ


def scenario_city(X, Y, Z, skyscraper_density=1, seed=2):
    rng = random.Random(seed)
    occ = shell3d(X, Y, Z)
    num = int((X - 2) * (Y - 2) * skyscraper_density)
    pos = [(x, y) for x in range(2, X - 2) for y in range(2, Y - 2) if x % 3 != 0 and y % 3 != 0]
    rng.shuffle(pos)
    for x, y in pos[:num]:
        height = rng.randint(3, Z - 2) if Z > 3 else 1
        for z in range(1, 1 + height):
            if z < Z - 1:
                occ[x, y, z] = 1
    return occ


SCENARIOS_3D = {
    "empty": lambda X, Y, Z: shell3d(X, Y, Z),
    "door": lambda X, Y, Z: scenario_door(X, Y, Z, door_size=2),
    "floors": lambda X, Y, Z: scenario_floors(X, Y, Z, floors=3, hole_size=2),
    "maze": lambda X, Y, Z: scenario_maze(X, Y, Z, seed=0),
    "city": lambda X, Y, Z: scenario_city(X, Y, Z, skyscraper_density=0.18, seed=0),
}


def carve_safety_bubble(occ: np.ndarray, center, radius=1):
    """examples/scenarios.py carve_safety_bubble: clear the cube around center, never the
    bounding box of the obstacle set (computed from the current obstacles)."""
    nz = np.argwhere(occ)
    if len(nz):
        mn, mx = nz.min(0), nz.max(0)
    else:
        mn, mx = np.array([0, 0, 0]), np.array([999999] * 3)
    cx, cy, cz = center
    for dx in range(-radius, radius + 1):
        for dy in range(-radius, radius + 1):
            for dz in range(-radius, radius + 1):
                x, y, z = cx + dx, cy + dy, cz + dz
                if mn[0] < x < mx[0] and mn[1] < y < mx[1] and mn[2] < z < mx[2]:
                    occ[x, y, z] = 0
    return occ


def bench3d_query(i: int, X: int, Y: int, Z: int):
    """examples/benchmark.py:50-69: random.seed(i); start, goal by randint(1, R-2); redraw goal."""
    random.seed(i)
    s = (random.randint(1, X - 2), random.randint(1, Y - 2), random.randint(1, Z - 2))
    g = (random.randint(1, X - 2), random.randint(1, Y - 2), random.randint(1, Z - 2))
    while g == s:
        g = (random.randint(1, X - 2), random.randint(1, Y - 2), random.randint(1, Z - 2))
    return s, g


def c5_workload(nq: int = 8192, X: int = 26, Y: int = 20, Z: int = 16, scenario: str = "door",
                radius: int = 1, first_seed: int = 0):
    """C5: Grid3D(26,20,16) (examples/3d_example.py:32-34), scenario door, query i uses
    random.seed(i), carve_safety_bubble(r=1) at both ends (3d_example.py:84-85) -> per-query
    occupancy.  Returns occ [nq, X, Y, Z] uint8, starts [nq,3], goals [nq,3]."""
    base = SCENARIOS_3D[scenario](X, Y, Z)
    occ = np.empty((nq, X, Y, Z), np.uint8)
    starts = np.empty((nq, 3), np.int32)
    goals = np.empty((nq, 3), np.int32)
    for q in range(nq):
        s, g = bench3d_query(first_seed + q, X, Y, Z)
        o = base.copy()
        carve_safety_bubble(o, s, radius)
        carve_safety_bubble(o, g, radius)
        occ[q] = o
        starts[q] = s
        goals[q] = g
    return occ, starts, goals


def c4_workload(na: int = 256, seed: int = 2):
    """C4: README grid, `na` agents on free cells drawn with default_rng(seed),
    theta ~ U(-pi, pi), v ~ U(0, 0.5), w ~ U(-pi/2, pi/2); goal (45, 25, 0).  Returns
    (occ, states [na, 5], goals [na, 3]); the global path of agent i is A* from its cell to (45, 25)."""
    occ = readme_grid()
    free = np.argwhere(occ == 0)
    rng = np.random.default_rng(seed)
    cells = free[rng.integers(0, len(free), na)]
    states = np.zeros((na, 5))
    states[:, 0:2] = cells
    states[:, 2] = rng.uniform(-np.pi, np.pi, na)
    states[:, 3] = rng.uniform(0.0, 0.5, na)
    states[:, 4] = rng.uniform(-np.pi / 2, np.pi / 2, na)
    goals = np.tile(np.array([45.0, 25.0, 0.0]), (na, 1))
    return occ, states, goals


# --------------------------------------------------------------------------------------------
# Continuous maps (utils/environment/env.py:83-117 Map) for the sample-search planners
# --------------------------------------------------------------------------------------------
README_MAP_RECT = [[14, 12, 8, 2], [18, 22, 8, 3], [26, 7, 2, 12], [32, 14, 10, 2]]
README_MAP_CIRC = [[7, 12, 3], [46, 20, 2], [15, 5, 2], [37, 7, 3], [37, 23, 3]]


def map_boundary(X: int, Y: int):
    """Map.init (env.py:99-110): the four boundary rectangles."""
    return [[0, 0, 1, Y], [0, Y, X, 1], [1, 0, X, 1], [X, 1, 1, Y]]


def c3_map(X: int = 512, Y: int = 512, n_rect: int = 40, n_circ: int = 40, seed: int = 7):
    """C3: Map(512, 512); default_rng(7) draws 40 rectangles then 40 circles as
    floats from 7 vectorised integer draws: x, y in [10, 480), w, h in [5, 40), then cx, cy in
    [10, 500), r in [3, 20).  Returns (obs_rect, obs_circ) as lists of float lists."""
    rng = np.random.default_rng(seed)
    rx = rng.integers(10, 480, n_rect)
    ry = rng.integers(10, 480, n_rect)
    rw = rng.integers(5, 40, n_rect)
    rh = rng.integers(5, 40, n_rect)
    cx = rng.integers(10, 500, n_circ)
    cy = rng.integers(10, 500, n_circ)
    cr = rng.integers(3, 20, n_circ)
    rects = [[float(a), float(b), float(c), float(d)] for a, b, c, d in zip(rx, ry, rw, rh)]
    circs = [[float(a), float(b), float(c)] for a, b, c in zip(cx, cy, cr)]
    return rects, circs
