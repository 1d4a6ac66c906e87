"""Graph-search planners: drop-in AStar (global_planner/graph_search/a_star.py) on the HIP kernels.

plan() keeps the reference's signature and return convention; plan_batch() is the batched form
(many start/goal pairs on one Grid) that the kernels are built for.
"""
from __future__ import annotations

import math
from collections.abc import Sequence

import numpy as np

from . import batch
from .env import Grid, Node
from .planner import Planner


class LazyExpand(Sequence):
    """The CLOSED Node list of a plan, built on first access (AStar.lazy_expand = True): len() is
    known without building it."""

    def __init__(self, build, n: int) -> None:
        self._build, self._n, self._nodes = build, n, None

    def _get(self) -> list:
        if self._nodes is None:
            self._nodes = self._build()
        return self._nodes

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        return self._get()[i]

    def __eq__(self, other) -> bool:
        return list(self._get()) == list(other)


class GraphSearcher(Planner):
    """global_planner/graph_search/graph_search.py:11-87."""

    def __init__(self, start: tuple, goal: tuple, env: Grid, heuristic_type: str = "euclidean") -> None:
        super().__init__(start, goal, env)
        self.heuristic_type = heuristic_type
        self.motions = self.env.motions
        self.obstacles = self.env.obstacles

    def h(self, node: Node, goal: Node) -> float:
        if self.heuristic_type == "manhattan":
            return abs(goal.x - node.x) + abs(goal.y - node.y)
        elif self.heuristic_type == "euclidean":
            return math.hypot(goal.x - node.x, goal.y - node.y)

    def cost(self, node1: Node, node2: Node) -> float:
        if self.isCollision(node1, node2):
            return float("inf")
        return self.dist(node1, node2)

    def isCollision(self, node1: Node, node2: Node) -> bool:
        obs = self.env.obstacles
        if node1.current in obs or node2.current in obs:
            return True
        x1, y1 = node1.x, node1.y
        x2, y2 = node2.x, node2.y
        if x1 != x2 and y1 != y2:
            return (x1, y2) in obs or (x2, y1) in obs
        return False


class AStar(GraphSearcher):
    """A* (a_star.py:13-124) -- the OPEN/CLOSED loop runs in the gfx950 kernel astar2d.hip."""

    _algo = "astar"

    def __str__(self) -> str:
        return "A*"

    #: return the CLOSED Node list lazily (materialised on first use); the reference builds it eagerly
    lazy_expand = False

    def plan(self) -> tuple:
        """Returns (cost, path goal->start, expand list of Node) or ([], [], []) (a_star.py:39-83).

        The Grid's obstacle set is bit-packed natively (no per-call Python loop); the path and
        CLOSED-record buffers are sized for the common case and the query re-runs with exact sizes
        only when one overflows.  One host round trip per query (batch.SingleQuery); the bit grid
        uploaded by the previous call on this Grid is launched on at once while the obstacle set is
        packed again on the host, and the query re-runs on a fresh upload if the set changed."""
        from . import _lib

        torch = _lib.device_check()  # no CPU fallback: raises PMPError without a HIP device
        W, H = self.env.x_range, self.env.y_range
        dev = torch.cuda.current_device()
        s, g = self.start.current, self.goal.current
        path_cap, expand_cap = min(W * H + 1, 1 << 14), min(W * H, 1 << 18)
        cached = getattr(self.env, "_pmp_occ", None)
        if cached is not None and cached[0] != (W, H, dev):
            cached = None
        while True:
            q = batch.single_query(torch, path_cap, expand_cap)
            if cached is not None:  # speculative launch on the last upload, checked below
                q.launch(torch, W, H, cached[2], s, g, self.heuristic_type, self._algo)
            words = self.env.occupancy_words()
            if cached is None or not np.array_equal(words, cached[1]):
                cached = ((W, H, dev), words, torch.as_tensor(words.view(np.int32), device="cuda"))
                self.env._pmp_occ = cached
                q.launch(torch, W, H, cached[2], s, g, self.heuristic_type, self._algo)
            st, nexp, plen, cells, exp = q.result()
            if st == 2 or nexp > expand_cap:  # PMP_PATH_OVERFLOW / truncated CLOSED records: exact sizes
                path_cap, expand_cap = max(path_cap, plen), max(expand_cap, nexp)
                continue
            break
        if st == _lib.STATUS_CAP_OVERFLOW:  # heap outgrew the reservation: the batch path's full-bound re-plan
            # sized for any outcome (a path visits a cell at most once, a cell closes at most once): the
            # full search may close more cells than the overflowed run had reached
            # (straight to the full bound: a plain batch call would first re-run the same engine at the
            # same limit and overflow again)
            path_cap, expand_cap = W * H + 1, W * H
            sg = torch.as_tensor(np.array([[s[0], s[1]], [g[0], g[1]]], np.int32), device="cuda")
            r = batch.astar2d_full_bound((W, H), sg[:1], sg[1:], self.heuristic_type, path_cap=path_cap,
                                         expand_cap=expand_cap, algo=self._algo, occ_bits=cached[2])
            st, nexp, plen = (int(v) for v in torch.stack([r["status"][0], r["n_expanded"][0],
                                                            r["path_len"][0]]).cpu().tolist())
            cells = r["path"][0, :plen].cpu().numpy()
            exp = r["expand"][0, :nexp].cpu().numpy().astype(np.uint32)
        if st != 0:
            if st == 1:
                return [], [], []
            raise RuntimeError(f"{self} kernel status {st}")
        path = [(int(c) // H, int(c) % H) for c in cells]
        cost = 0
        for a, b in zip(path[:-1], path[1:]):
            cost += math.hypot(b[0] - a[0], b[1] - a[1])
        if self.lazy_expand:
            return cost, path, LazyExpand(lambda: self._expand_nodes(exp, H), nexp)
        return cost, path, self._expand_nodes(exp, H)

    def _expand_nodes(self, exp: np.ndarray, H: int) -> list:
        """Rebuild the reference's CLOSED Node objects (current, parent, g, h) from the kernel's
        closure-ordered (cell | parent_dir << 28) records, natively (csrc/hostio.c): g accumulated
        with Python's `+` on the motion costs as Node.__add__ does (node.py:39-41), h as
        GraphSearcher.h; Dijkstra's h = 0 (dijkstra.py:74), GBFS's g = 0 (gbfs.py:75)."""
        from ._hostio import expand_nodes

        manhattan = self.heuristic_type == "manhattan"
        kind = {"astar": 1 if manhattan else 0, "dijkstra": 2, "gbfs": 4 if manhattan else 3}[self._algo]
        motions = self.env.motions
        return expand_nodes(np.ascontiguousarray(exp, np.uint32), len(exp), H, [(m.x, m.y) for m in motions],
                            [m.g for m in motions], tuple(int(v) for v in self.goal.current), kind, Node)

    @classmethod
    def plan_batch(cls, occ: np.ndarray, starts, goals, heuristic_type: str = "euclidean", **kw):
        """Batched plan over one occupancy grid; returns the device-tensor dict of
        batch.astar2d_batch (cost, path_len, path goal->start, n_expanded, status)."""
        return batch.astar2d_batch(occ, starts, goals, heuristic_type, algo=cls._algo, **kw)


class Dijkstra(AStar):
    """Dijkstra (dijkstra.py:13-85): AStar's loop with node_n.h = 0 (:73-74), on the same kernel."""

    _algo = "dijkstra"

    def __str__(self) -> str:
        return "Dijkstra"


class GBFS(AStar):
    """Greedy Best First Search (gbfs.py:13-86): AStar's loop with node_n.g = 0 (:73-75), so the
    heap orders by h alone; the same kernel."""

    _algo = "gbfs"

    def __str__(self) -> str:
        return "Greedy Best First Search(GBFS)"


class ThetaStar(AStar):
    """Theta* (theta_star.py:13-171): AStar's loop where a neighbour takes the expanded node's parent
    as its own when that parent sees it (Bresenham lineOfSight) and is no farther (updateVertex,
    :96-108).  Same kernel as AStar, with any-cell parents kept per CLOSED cell."""

    _algo = "theta_star"

    def __str__(self) -> str:
        return "Theta*"

    def _expand_nodes(self, exp: np.ndarray, H: int) -> list:
        """CLOSED Node objects from the kernel's (cell | code << 26) records.  code: 0-7 = path 1
        through motion d, 8 = start, 16 + d = path 2 (the pusher's own parent), 24 + d = Lazy Theta*'s
        re-parenting to the CLOSED neighbour in motion d; + 32 = no parent found (g = inf)."""
        motions = self.env.motions
        nodes, gmap, pmap = [], {}, {}
        for e in exp.tolist():
            cell, code = e & 0x03FFFFFF, e >> 26
            cur = (cell // H, cell % H)
            d = code & 7
            m = motions[d]
            if code == 8:
                node = Node(cur, cur, 0, 0)
            else:
                base = code & 31
                if base >= 24:
                    par = (cur[0] + m.x, cur[1] + m.y)
                    g = gmap[par] + m.g
                else:
                    pusher = (cur[0] - m.x, cur[1] - m.y)
                    if base >= 16:
                        par = pmap[pusher]
                        g = gmap[par] + self.dist(Node(cur), Node(par))
                    else:
                        par = pusher
                        g = gmap[par] + m.g
                if code & 32:
                    g = float("inf")
                node = Node(cur, par, g, self.h(Node(cur), self.goal))
            gmap[cur], pmap[cur] = node.g, node.parent
            nodes.append(node)
        return nodes


class LazyThetaStar(ThetaStar):
    """Lazy Theta* (lazy_theta_star.py:13-114): updateVertex without the line of sight at the push;
    the line of sight is checked when the node pops (:55-65).  Same kernel."""

    _algo = "lazy_theta_star"

    def __str__(self) -> str:
        return "Lazy Theta*"


class LPAStar(GraphSearcher):
    """Lifelong Planning A* (lpa_star.py:39-230): plan() is the initial computeShortestPath +
    extractPath on the gfx950 kernel lpa.hip (U with the reference's list semantics).  Interactive
    replanning (OnPress) needs a figure and is not provided."""

    _lite = False

    def __str__(self) -> str:
        return "Lifelong Planning A*"

    def plan(self) -> tuple:
        """Returns (cost, path start->goal, None); (cost, [], None) when extractPath gives up after
        1000 steps; raises ValueError where the reference's min() of an empty list does."""
        occ = self.env.occupancy()
        W, H = occ.shape
        r = batch.lpastar2d_batch(occ, np.array([self.start.current]), np.array([self.goal.current]),
                                  self.heuristic_type, counters=True, lite=self._lite)
        st = int(r["status"][0])
        self.n_expanded = int(r["n_expanded"][0])
        if st == 4:
            raise ValueError("min() arg is an empty sequence (LPAStar: U emptied before the goal was consistent)")
        if st == 1:
            return float(r["cost"][0]), [], None
        if st != 0:
            raise RuntimeError(f"{self} kernel status {st}")
        plen = int(r["path_len"][0])
        cells = r["path"][0, :plen].cpu().numpy()
        return float(r["cost"][0]), [(int(c) // H, int(c) % H) for c in cells], None


class DStarLite(LPAStar):
    """D* Lite (d_star_lite.py:14-187): LPAStar's plan() searched from the goal toward the start
    (keys with h(node, start) + km, km = 0), on the same kernel (pmp_dstarlite2d_batch).  Interactive
    replanning (OnPress) needs a figure and is not provided."""

    _lite = True

    def __str__(self) -> str:
        return "D* Lite"


def dstar_border_key(cell: int, W: int, H: int) -> tuple:
    """The key DStar.getNeighbor (d_star.py:276-291) fails on for a node on the grid's border: the
    first motion (env.py:52-55 order) whose target is outside the grid (self.map holds the in-grid
    cells only).  The kernel reports that node as status 4 with path_len -2 and path[0] = its cell."""
    x, y = divmod(int(cell), H)
    for dx, dy in ((-1, 0), (-1, 1), (0, 1), (1, 1), (1, 0), (1, -1), (0, -1), (-1, -1)):
        if not (0 <= x + dx < W and 0 <= y + dy < H):
            return (x + dx, y + dy)
    raise ValueError(f"cell {cell} is not on the border of a {W}x{H} grid")


class DStar(GraphSearcher):
    """Dynamic A* (d_star.py:37-291) -- the static plan (processState until the start is CLOSED)
    runs in the gfx950 kernel dstar.hip with the reference's list-semantics OPEN."""

    def __init__(self, start: tuple, goal: tuple, env: Grid) -> None:
        super().__init__(start, goal, env, None)
        self.EXPAND = []

    def __str__(self) -> str:
        return "Dynamic A*(D*)"

    def plan(self) -> tuple:
        """(cost, path start->goal, None) (d_star.py:75-89); raises AttributeError when the start is
        unreachable, like the reference (min_k of an empty OPEN, :234)."""
        occ = self.env.occupancy()
        self._occ0, self._presses = occ, []
        W, H = occ.shape
        r = batch.dstar2d_batch(occ, np.array([self.start.current]), np.array([self.goal.current]))
        st = int(r["status"][0])
        self.n_process = int(r["n_process"][0])
        if st == 4:
            if int(r["path_len"][0]) == -2:  # getNeighbor of a border node (a grid without walls)
                raise KeyError(dstar_border_key(int(r["path"][0, 0]), W, H))
            raise AttributeError("'NoneType' object has no attribute 'k'")
        if st != 0:
            raise RuntimeError(f"D* kernel status {st}")
        cells = r["path"][0, : int(r["path_len"][0])].cpu().numpy()
        return float(r["cost"][0]), [(int(c) // H, int(c) % H) for c in cells], None

    def run(self):
        return self.plan()

    def OnPress(self, event) -> None:
        """Mouse callback (d_star.py:102-134) without the figure: a press on a free in-grid cell adds
        the obstacle and repairs the plan from the start's back-pointer chain; the walk's cost and
        path (which stops before the goal, as the reference's) are kept in self.cost / self.path and
        len(self.EXPAND) is the processState count of that repair.  The kernel is stateless, so the
        plan and every earlier press are replayed on the device."""
        x, y = int(event.xdata), int(event.ydata)
        if x < 0 or x > self.env.x_range - 1 or y < 0 or y > self.env.y_range - 1:
            print("Please choose right area!")
            return
        if (x, y) in self.obstacles:
            return
        print("Add obstacle at: ({}, {})".format(x, y))
        if not hasattr(self, "_occ0"):
            self._occ0, self._presses = self.env.occupancy(), []
        self.obstacles.add((x, y))
        self.env.update(self.obstacles)
        self._presses.append((x, y))
        W, H = self._occ0.shape
        r = batch.dstar2d_onpress_batch(self._occ0, np.array([self.start.current]), np.array([self.goal.current]),
                                        np.array([self._presses], np.int32))
        k = len(self._presses)
        st = int(r["status"][0, k])
        if st == 4:
            if int(r["path_len"][0, k]) == -2:  # getNeighbor of a border node (a grid without walls)
                raise KeyError(dstar_border_key(int(r["path"][0, k, 0]), W, H))
            if int(r["path_len"][0, k]) < 0:
                raise KeyError(None)  # self.map[node.parent] of a parentless node
            raise AttributeError("'NoneType' object has no attribute 'k'")  # min_k of an emptied OPEN
        if st not in (0, 1):
            raise RuntimeError(f"D* kernel status {st} (a walk or repair the reference never finishes)")
        n = int(r["path_len"][0, k])
        self.cost = float(r["cost"][0, k])
        self.path = [(int(c) // H, int(c) % H) for c in r["path"][0, k, :n].cpu().numpy()]
        self.EXPAND = [None] * int(r["n_process"][0, k])

    @staticmethod
    def plan_batch(occ: np.ndarray, starts, goals, **kw):
        return batch.dstar2d_batch(occ, starts, goals, **kw)

    @staticmethod
    def onpress_batch(occ: np.ndarray, starts, goals, presses, **kw):
        return batch.dstar2d_onpress_batch(occ, starts, goals, presses, **kw)


class GraphSearcher3D:
    """global_planner/graph_search/graph_search_3d.py:11-107 (Planner3D base)."""

    def __init__(self, start: tuple, goal: tuple, env, heuristic_type: str = "euclidean") -> None:
        from .env import Node3D

        self.start = Node3D(start, start, 0, 0)
        self.goal = Node3D(goal, goal, 0, 0)
        self.env = env
        self.plot = None
        self.heuristic_type = heuristic_type
        self.motions = self.env.motions
        self.obstacles = self.env.obstacles

    def h(self, node, goal) -> float:
        dx, dy, dz = abs(goal.x - node.x), abs(goal.y - node.y), abs(goal.z - node.z)
        if self.heuristic_type == "manhattan":
            return dx + dy + dz
        return math.sqrt(dx ** 2 + dy ** 2 + dz ** 2)

    def dist(self, node1, node2) -> float:
        return math.sqrt((node2.x - node1.x) ** 2 + (node2.y - node1.y) ** 2 + (node2.z - node1.z) ** 2)

    def run(self):
        return self.plan()


class AStar3D(GraphSearcher3D):
    """A* for 3D grids (a_star3d.py:18-111) -- the search runs in the gfx950 kernel astar3d.hip."""

    _algo = "astar"

    def __str__(self) -> str:
        return "A*"

    def plan(self) -> tuple:
        """(cost, path start->goal, expand) -- (inf, [], expand) when unreachable (a_star3d.py:33-78).
        expand: one Node3D per CLOSED cell in first-insertion order (its `current`; parent/g/h None)."""
        from .env import Node3D

        occ = self.env.occupancy()
        X, Y, Z = occ.shape
        r = batch.astar3d_batch(occ, np.array([self.start.current]), np.array([self.goal.current]),
                                self.heuristic_type, path_cap=X * Y * Z + 1, expand_cap=X * Y * Z, algo=self._algo)
        st = int(r["status"][0])
        ne = int(r["n_expanded"][0])
        ex = r["expand"][0, :ne].cpu().numpy()
        expand = [Node3D((int(c) // (Y * Z), (int(c) // Z) % Y, int(c) % Z), None, None, None) for c in ex]
        if st == 1:
            return float("inf"), [], expand
        if st != 0:
            raise RuntimeError(f"{self} kernel status {st}")
        cells = r["path"][0, : int(r["path_len"][0])].cpu().numpy()
        path = [(int(c) // (Y * Z), (int(c) // Z) % Y, int(c) % Z) for c in cells]
        return float(r["cost"][0]), path, expand

    @classmethod
    def plan_batch(cls, occ, starts, goals, heuristic_type: str = "euclidean", **kw):
        return batch.astar3d_batch(occ, starts, goals, heuristic_type, algo=cls._algo, **kw)


class Dijkstra3D(AStar3D):
    """Dijkstra for 3D grids (dijkstra3d.py:18-147): key (g, 0.0, counter), start h = 0; its
    getNeighbor (:89-126) is isCollision plus an in-bounds test.  The same kernel with h = 0."""

    _algo = "dijkstra"

    def __init__(self, start: tuple, goal: tuple, env) -> None:
        super().__init__(start, goal, env, "euclidean")  # dijkstra3d.py:31 passes no heuristic

    def __str__(self) -> str:
        return "Dijkstra (3D)"


class GBFS3D(AStar3D):
    """Greedy Best First Search for 3D grids (gbfs3d.py:20-114): key (h, counter), CLOSED membership
    tests.  The same kernel with every g = 0."""

    _algo = "gbfs"

    def __str__(self) -> str:
        return "Greedy Best First Search (GBFS) 3D"


class ThetaStar3D(AStar3D):
    """Theta* for 3D voxel grids (theta_star3d.py:24-232): AStar3D's loop where a neighbour takes the
    expanding node's CLOSED parent as its own when lineOfSight (integer Bresenham, :139-213) allows a
    cheaper straight segment.  Same kernel (astar3d.hip, THETA = 1); paths are any-voxel."""

    _algo = "theta_star"

    def __str__(self) -> str:
        return "Theta* 3D"


class LazyThetaStar3D(AStar3D):
    """Lazy Theta* for 3D grids (lazy_theta_star3d.py:24-252): the parent update without the line of
    sight test, which is deferred to the pop (a failure re-parents the node to its best CLOSED
    neighbour).  Same kernel (astar3d.hip, THETA = 2)."""

    _algo = "lazy_theta_star"

    def __str__(self) -> str:
        return "Lazy Theta* 3D"


class DNode3D:
    """D* bookkeeping node of DStar3D (d_star3d.py:21-57): coordinates in `current`, parent
    coordinates, tag t, h and k.  Equality and hashing by coordinates (Node3D, node3d.py:43-57)."""

    __slots__ = ("current", "parent", "t", "h", "k")

    def __init__(self, current, parent, t, h, k) -> None:
        self.current, self.parent, self.t, self.h, self.k = current, parent, t, h, k

    def __eq__(self, other) -> bool:
        return isinstance(other, DNode3D) and self.current == other.current

    def __hash__(self) -> int:
        return hash(self.current)

    def __repr__(self) -> str:
        return f"DNode3D(current={self.current}, parent={self.parent}, t={self.t}, h={self.h}, k={self.k})"


class DStar3D(GraphSearcher3D):
    """Dynamic A* in 3D voxel grids (d_star3d.py:60-281).  plan() and apply_dynamic_obstacles() run
    in the gfx950 kernel dstar3d.hip with the reference's list-semantics OPEN.  The kernel is
    stateless, so the planner keeps the history of blocked-voxel batches and every call replays the
    plan and the earlier rounds on the device (the reference's in-place state is a function of that
    history)."""

    def __init__(self, start: tuple, goal: tuple, env) -> None:
        super().__init__(start, goal, env, None)
        self._rounds = []
        self.EXPAND = []
        self._occ0 = None

    def __str__(self) -> str:
        return "Dynamic A* (D*) 3D"

    def _run(self, want_expand: bool):
        occ = self._occ0
        X, Y, Z = occ.shape
        nb = max((len(r) for r in self._rounds), default=0)
        blocks = None
        if self._rounds:
            blocks = np.full((1, len(self._rounds), max(nb, 1), 3), -1, np.int32)
            for i, r in enumerate(self._rounds):
                if r:
                    blocks[0, i, : len(r)] = np.asarray(r, np.int32).reshape(-1, 3)
        r = batch.dstar3d_batch(occ, np.array([self.start.current]), np.array([self.goal.current]), blocks,
                                path_cap=4 * X * Y * Z + 8, expand_cap=(8 * X * Y * Z + 8) if want_expand else 0)
        st = r["status"][0].cpu().numpy()
        if (st >= 2).any():
            raise RuntimeError(f"{self} kernel status {st.tolist()}")
        return r

    def _cells(self, r, k):
        X, Y, Z = r["dims"]
        n = int(r["path_len"][0, k])
        return [(int(c) // (Y * Z), (int(c) // Z) % Y, int(c) % Z) for c in r["path"][0, k, :n].cpu().numpy()]

    def plan(self) -> tuple:
        """(cost, path start->goal, EXPAND) (d_star3d.py:100-109).  An unreachable start gives
        (0.0, [start], EXPAND), as the reference's extractPath breaks at the parentless start.
        EXPAND: one DNode3D per processState, `current` set (state fields not materialised)."""
        self._occ0 = self.env.occupancy()
        self._rounds = []
        r = self._run(True)
        ne = int(r["n_process"][0, 0])
        X, Y, Z = r["dims"]
        ex = r["expand"][0, :ne].cpu().numpy()
        self.EXPAND = [DNode3D((int(c) // (Y * Z), (int(c) // Z) % Y, int(c) % Z), None, None, None, None) for c in ex]
        return float(r["cost"][0, 0]), self._cells(r, 0), list(self.EXPAND)

    def apply_dynamic_obstacles(self, newly_blocked) -> tuple:
        """Block the voxels and repair from the start's back-pointer chain (d_star3d.py:115-149).
        Returns (cost, path); self.EXPAND holds this call's processState count."""
        if self._occ0 is None:
            self.plan()
        blk = [tuple(int(v) for v in t) for t in newly_blocked]
        for v in blk:
            self.obstacles.add(v)
        self.env.update(self.obstacles)
        self._rounds.append(blk)
        r = self._run(False)
        k = len(self._rounds)
        self.EXPAND = [None] * int(r["n_process"][0, k])
        return float(r["cost"][0, k]), self._cells(r, k)

    @staticmethod
    def plan_batch(occ, starts, goals, blocks=None, **kw):
        return batch.dstar3d_batch(occ, starts, goals, blocks, **kw)


class LNode3D:
    """LPA* node of LPAStar3D (lpa_star3d.py:13-43): coordinates in `current`, g, rhs, key."""

    __slots__ = ("current", "g", "rhs", "key", "parent")

    def __init__(self, current, g, rhs, key) -> None:
        self.current, self.g, self.rhs, self.key, self.parent = current, g, rhs, key, None

    def __eq__(self, other) -> bool:
        return isinstance(other, LNode3D) and self.current == other.current

    def __hash__(self) -> int:
        return hash(self.current)


class LPAStar3D(GraphSearcher3D):
    """Lifelong Planning A* on 3D voxel grids (lpa_star3d.py:40-225): plan() and apply_change() run
    in the gfx950 kernel lpa3d.hip with the reference's list-semantics U.  The kernel is stateless,
    so the planner keeps the history of changes and every call replays plan() and the earlier
    changes on the device (the reference's kept g / rhs / U are a function of that history)."""

    def __init__(self, start: tuple, goal: tuple, env, heuristic_type: str = "euclidean") -> None:
        super().__init__(start, goal, env, heuristic_type)
        self.EXPAND = []
        self._changes = []
        self._occ0 = None

    def __str__(self) -> str:
        return "Lifelong Planning A* 3D"

    def _call(self):
        ch = np.asarray(self._changes, np.int32).reshape(1, -1, 4) if self._changes else None
        X, Y, Z = self._occ0.shape
        r = batch.lpastar3d_batch(self._occ0, np.array([self.start.current]), np.array([self.goal.current]), ch,
                                  self.heuristic_type, path_cap=X * Y * Z + 1)
        k = len(self._changes)
        st = int(r["status"][0, k])
        if st not in (0, 1):
            raise RuntimeError(f"{self} kernel status {st}")
        n = int(r["path_len"][0, k])
        cells = r["path"][0, k, :n].cpu().numpy()
        path = [(int(c) // (Y * Z), (int(c) // Z) % Y, int(c) % Z) for c in cells]
        self.EXPAND = [None] * int(r["n_expanded"][0, k])
        return float(r["cost"][0, k]), path, self.EXPAND

    def plan(self) -> tuple:
        """(cost, path start->goal, EXPAND) (lpa_star3d.py:78-82); (cost, [], EXPAND) when the greedy
        extraction finds no path.  EXPAND holds len(EXPAND) placeholders (the node objects are not
        materialised).  A second plan() without changes expands nothing and keeps EXPAND, as there."""
        if self._occ0 is None:
            self._occ0 = self.env.occupancy()
            return self._call()
        # a no-op round: computeShortestPath on the kept state; plan() does not clear EXPAND
        prev = list(self.EXPAND)
        self._changes.append((-1, -1, -1, 0))
        cost, path, new = self._call()
        self.EXPAND = prev + new
        return cost, path, self.EXPAND

    def apply_change(self, coord: tuple, blocked=None) -> tuple:
        """Toggle / set the voxel and re-plan incrementally (lpa_star3d.py:93-124)."""
        if self._occ0 is None:
            self.plan()
        c = tuple(int(v) for v in coord)
        if blocked is None:
            if c in self.obstacles:
                self.obstacles.remove(c)
            else:
                self.obstacles.add(c)
        elif blocked:
            self.obstacles.add(c)
        elif c in self.obstacles:
            self.obstacles.remove(c)
        self.env.update(self.obstacles)
        self._changes.append((c[0], c[1], c[2], 0 if blocked is None else (1 if blocked else 2)))
        return self._call()

    @staticmethod
    def plan_batch(occ, starts, goals, changes=None, **kw):
        return batch.lpastar3d_batch(occ, starts, goals, changes, **kw)
