"""World model: drop-in Grid / Map / Grid3D / Node / Node3D (utils/environment/ of the reference).

The reference stores a Grid's obstacles as a Python set of (x, y) tuples and rebuilds a
cKDTree on every update (env.py:78-80).  Here the set stays the user-facing truth (same
attribute names, same mutation idiom) and is converted to the bit-packed x-major occupancy
the kernels read (cell id x*H + y, bit c of word c>>5).
"""
from __future__ import annotations

from math import sqrt

import numpy as np

from . import _hostio  # native set -> bit-grid marshalling (csrc/hostio.c); no Python fallback


class Node:
    """utils/environment/node.py:8-84 -- search node (current, parent, g, h)."""

    __slots__ = ("current", "parent", "g", "h")

    def __init__(self, current: tuple, parent: tuple = None, g: float = 0, h: float = 0) -> None:
        self.current = current
        self.parent = parent
        self.g = g
        self.h = h

    def __add__(self, node):
        assert isinstance(node, Node)
        return Node((self.x + node.x, self.y + node.y), self.parent, self.g + node.g, self.h)

    def __eq__(self, node) -> bool:
        if not isinstance(node, Node):
            return False
        return self.current == node.current

    def __ne__(self, node) -> bool:
        return not self.__eq__(node)

    def __lt__(self, node) -> bool:
        assert isinstance(node, Node)
        return self.g + self.h < node.g + node.h or (self.g + self.h == node.g + node.h and self.h < node.h)

    def __hash__(self) -> int:
        return hash(self.current)

    def __str__(self) -> str:
        return "Node({}, {}, {}, {})".format(self.current, self.parent, self.g, self.h)

    __repr__ = __str__

    @property
    def x(self):
        return self.current[0]

    @property
    def y(self):
        return self.current[1]

    @property
    def px(self):
        return self.parent[0] if self.parent else None

    @property
    def py(self):
        return self.parent[1] if self.parent else None


class Node3D(Node):
    """utils/environment/node3d.py -- 3D search node."""

    __slots__ = ()

    def __add__(self, node):
        assert isinstance(node, Node3D)
        return Node3D((self.x + node.x, self.y + node.y, self.z + node.z), self.parent, self.g + node.g, self.h)

    def __eq__(self, node) -> bool:
        if not isinstance(node, Node3D):
            return False
        return self.current == node.current

    def __hash__(self) -> int:
        return hash(self.current)

    @property
    def z(self):
        return self.current[2]

    @property
    def pz(self):
        return self.parent[2] if self.parent else None


class Env:
    """utils/environment/env.py:14-38."""

    def __init__(self, x_range: int, y_range: int, eps: float = 1e-6) -> None:
        self.x_range = x_range
        self.y_range = y_range
        self.eps = eps

    @property
    def grid_map(self) -> set:
        return {(i, j) for i in range(self.x_range) for j in range(self.y_range)}


def pack_bits(occ: np.ndarray) -> np.ndarray:
    """uint8/bool occupancy (any shape, C order) -> little-endian bit-packed uint32 words."""
    flat = np.ascontiguousarray(occ, dtype=np.uint8).ravel() != 0
    b = np.packbits(flat, bitorder="little")
    pad = (-len(b)) % 4
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    return b.view("<u4").copy()


class Grid(Env):
    """utils/environment/env.py:41-80 -- discrete 2D grid, 8-connected motions."""

    def __init__(self, x_range: int, y_range: int) -> None:
        super().__init__(x_range, y_range)
        self.motions = [Node((-1, 0), None, 1, None), Node((-1, 1), None, sqrt(2), None),
                        Node((0, 1), None, 1, None), Node((1, 1), None, sqrt(2), None),
                        Node((1, 0), None, 1, None), Node((1, -1), None, sqrt(2), None),
                        Node((0, -1), None, 1, None), Node((-1, -1), None, sqrt(2), None)]
        self.obstacles = None
        self.init()

    def init(self) -> None:
        x, y = self.x_range, self.y_range
        obstacles = set()
        for i in range(x):
            obstacles.add((i, 0))
            obstacles.add((i, y - 1))
        for i in range(y):
            obstacles.add((0, i))
            obstacles.add((x - 1, i))
        self.update(obstacles)

    def update(self, obstacles):
        self.obstacles = obstacles

    @property
    def obstacles_tree(self):
        """The reference keeps a cKDTree of the obstacles (env.py:78-80); built on demand here."""
        from scipy.spatial import cKDTree

        return cKDTree(np.array(list(self.obstacles)))

    # ---- kernel-facing views ------------------------------------------------------------------
    def occupancy_words(self) -> np.ndarray:
        """The kernels' bit-packed x-major occupancy (uint32 words, bit c of word c >> 5 for cell
        c = x*H + y) of the in-range obstacle cells, from one native pass over the set."""
        W, H = self.x_range, self.y_range
        words = np.empty((W * H + 31) // 32, np.uint32)
        _hostio.set_to_words(self.obstacles or (), (W, H), words)
        return words

    def occupancy(self) -> np.ndarray:
        """uint8 [x_range, y_range], occ[x, y] = 1 for (x, y) in obstacles (in-range cells)."""
        W, H = self.x_range, self.y_range
        bits = np.unpackbits(self.occupancy_words().view(np.uint8), bitorder="little")
        return bits[: W * H].reshape(W, H)

    @classmethod
    def from_occupancy(cls, occ: np.ndarray) -> "Grid":
        g = cls.__new__(cls)
        Env.__init__(g, int(occ.shape[0]), int(occ.shape[1]))
        g.motions = Grid(2, 2).motions
        g.obstacles = {(int(x), int(y)) for x, y in np.argwhere(occ)}
        return g


class Map(Env):
    """utils/environment/env.py:83-117 -- continuous 2D map with rect/circle obstacles."""

    def __init__(self, x_range: int, y_range: int) -> None:
        super().__init__(x_range, y_range)
        self.boundary = None
        self.obs_circ = None
        self.obs_rect = None
        self.init()

    def init(self):
        x, y = self.x_range, self.y_range
        self.boundary = [[0, 0, 1, y], [0, y, x, 1], [1, 0, x, 1], [x, 1, 1, y]]
        self.obs_rect = []
        self.obs_circ = []

    def update(self, boundary=None, obs_circ=None, obs_rect=None):
        self.boundary = boundary if boundary else self.boundary
        self.obs_circ = obs_circ if obs_circ else self.obs_circ
        self.obs_rect = obs_rect if obs_rect else self.obs_rect


class Env3D:
    """utils/environment/env3d.py:14-40."""

    def __init__(self, x_range: int, y_range: int, z_range: int, eps: float = 1e-6) -> None:
        self.x_range = x_range
        self.y_range = y_range
        self.z_range = z_range
        self.eps = eps

    @property
    def grid_map(self) -> set:
        return {(i, j, o) for i in range(self.x_range) for j in range(self.y_range) for o in range(self.z_range)}


class Grid3D(Env3D):
    """utils/environment/env3d.py:43-103 -- discrete 3D grid, 26 motions in the reference order."""

    def __init__(self, x_range: int, y_range: int, z_range: int) -> None:
        super().__init__(x_range, y_range, z_range)
        s2, s3 = sqrt(2), sqrt(3)
        dirs = [(-1, 0, 0), (-1, 1, 0), (0, 1, 0), (1, 1, 0), (1, 0, 0), (1, -1, 0), (0, -1, 0), (-1, -1, 0),
                (0, 0, 1), (0, 0, -1),
                (-1, 0, 1), (-1, 1, 1), (0, 1, 1), (1, 1, 1), (1, 0, 1), (1, -1, 1), (0, -1, 1), (-1, -1, 1),
                (-1, 0, -1), (-1, 1, -1), (0, 1, -1), (1, 1, -1), (1, 0, -1), (1, -1, -1), (0, -1, -1),
                (-1, -1, -1)]
        cost = {1: 1, 2: s2, 3: s3}
        self.motions = [Node3D(d, None, cost[sum(1 for c in d if c)], None) for d in dirs]
        self.obstacles = None
        self.init()

    def init(self) -> None:
        # env3d.py:77-97 including its z-1 offset on the side walls
        x, y, z = self.x_range, self.y_range, self.z_range
        obstacles = set()
        for _z in range(z):
            for i in range(x):
                obstacles.add((i, 0, _z - 1))
                obstacles.add((i, y - 1, _z - 1))
            for i in range(y):
                obstacles.add((0, i, _z - 1))
                obstacles.add((x - 1, i, _z - 1))
        for _x in range(x):
            for _y in range(y):
                obstacles.add((_x, _y, 0))
                obstacles.add((_x, _y, z - 1))
        self.update(obstacles)

    def update(self, obstacles):
        self.obstacles = obstacles

    def occupancy_words(self) -> np.ndarray:
        """Bit-packed occupancy (cell (x*Y + y)*Z + z) of the in-range obstacle voxels (native pass)."""
        X, Y, Z = self.x_range, self.y_range, self.z_range
        words = np.empty((X * Y * Z + 31) // 32, np.uint32)
        _hostio.set_to_words(self.obstacles or (), (X, Y, Z), words)
        return words

    def occupancy(self) -> np.ndarray:
        """uint8 [x_range, y_range, z_range] of the in-range obstacle voxels."""
        X, Y, Z = self.x_range, self.y_range, self.z_range
        bits = np.unpackbits(self.occupancy_words().view(np.uint8), bitorder="little")
        return bits[: X * Y * Z].reshape(X, Y, Z)


class Map3D(Env3D):
    """utils/environment/env3d.py:106-147 (kept for API completeness; no in-scope planner uses it)."""

    def __init__(self, x_range: int, y_range: int, z_range: int) -> None:
        super().__init__(x_range, y_range, z_range)
        self.boundary = None
        self.obs_circ = None
        self.obs_rect = None
        self.init()

    def init(self):
        x, y, z = self.x_range, self.y_range, self.z_range
        self.boundary = [[0, 0, 0, x, y, 0], [0, 0, z, x, y, z], [0, 0, 0, x, 0, z],
                         [0, y, 0, x, y, z], [0, 0, 0, 0, y, z], [x, 0, 0, x, y, z]]
        self.obs_rect = []
        self.obs_circ = []

    def update(self, boundary=None, obs_circ=None, obs_rect=None):
        self.boundary = boundary if boundary else self.boundary
        self.obs_circ = obs_circ if obs_circ else self.obs_circ
        self.obs_rect = obs_rect if obs_rect else self.obs_rect
