"""The path form of CPython's heapq that the multi-query A* kernel runs (astar2d_mq.hip, path_op /
pop_leaf): one operation = a path of positions q_L (lane L <-> level L), a ballot for the boundary
level b, a one-level shift of the path and the new element at b, plus the _siftup choice bits of the
changed levels' parents.  Checked here against Lib/heapq.py itself (heappush / heappop on items
ordered like Node.__lt__, node.py:51-54, with many exact ties) on random operation sequences: the
heap array, the direction bits, root and last element must equal CPython's after every operation."""
import heapq
import random


class Item:
    __slots__ = ("f", "h", "tag")

    def __init__(self, f, h, tag):
        self.f, self.h, self.tag = f, h, tag

    def __lt__(self, other):  # Node.__lt__: (g + h, h); ties fall back to the heap's structure
        return self.f < other.f or (self.f == other.f and self.h < other.h)


def lt(a, b):
    return a < b


def bit_of(heap, p):
    """_siftup's choice at node p: 1 = the right child (2p + 2) when not (left < right)."""
    return 0 if lt(heap[2 * p + 1], heap[2 * p + 2]) else 1


class PathHeap:
    """The kernel's formulation: the array, direction bits for nodes with two children, root, last."""

    def __init__(self):
        self.a, self.bits = [], {}

    def _set_bit(self, parent, child_new, sib):
        # choice_bit_k: bit(parent) = !(left < right) with the child's new content
        child_pos = child_new[0]
        v, s = child_new[1], sib
        self.bits[parent] = int(not lt(v, s)) if child_pos & 1 else int(not lt(s, v))

    def _path_op(self, pop, Q, Kd, n, X):
        v_last = self.a[n - 1] if pop else None  # lane 15's load
        q = [(Q >> (Kd - L)) - 1 for L in range(Kd + 1)]
        V = [self.a[p] if p < len(self.a) else None for p in q]
        if pop:
            cnt = sum(1 for L in range(1, Kd + 1) if not lt(X, V[L]))
            b = cnt
        else:
            cnt = sum(1 for L in range(0, Kd) if lt(X, V[L]))
            b = Kd - cnt
        new = list(V)
        for L in range(Kd + 1):
            if L == b:
                new[L] = X
            elif pop and L < b:
                new[L] = V[L + 1]
            elif not pop and L > b:
                new[L] = V[L - 1]
        while len(self.a) < n + (0 if pop else 1):
            self.a.append(None)
        for L in range(Kd + 1):
            if (pop and L <= b) or (not pop and L >= b):
                self.a[q[L]] = new[L]
        size = n if pop else n + 1
        for L in range(1, Kd + 1):
            s = ((q[L] - 1) ^ 1) + 1
            if s < (n if pop else n) and ((pop and L <= b) or (not pop and L >= b)):
                self._set_bit(q[L - 1], (q[L], new[L]), self.a[s])
        del self.a[size:]
        # the kernel's registers: root = level 0's new content; last = a push's level Kd (position n),
        # a pop's old heap[n - 1] unless X landed on it (the leaf, b == Kd)
        self.root = new[0]
        if pop:
            if not (b == Kd and Q == n):
                self.last = v_last
        else:
            self.last = new[Kd]
        return b

    def push(self, x):
        n = len(self.a)
        Q = n + 1
        self._path_op(False, Q, Q.bit_length() - 1, n, x)

    def pop_leaf(self, n):
        """_siftup's leaf from the bits: levels 0..D-2 unconditionally, then one conditional step."""
        D = n.bit_length() - 1
        P, K = 1, 0
        for _ in range(max(D - 1, 0)):
            P = 2 * P + self.bits[P - 1]
            K += 1
        if 2 * P <= n:
            c = self.bits[P - 1] if 2 * P < n else 0
            P = 2 * P + c
            K += 1
        return P, K

    def pop(self):
        root = self.a[0]
        last = self.a[-1]
        n = len(self.a) - 1
        if n == 0:
            self.a.pop()
            return root
        self.a.pop()
        self.last = last  # X
        P, K = self.pop_leaf(n)
        self._path_op(True, P, K, n, last)
        return root


def check_bits(h):
    for p in range(len(h.a)):
        if 2 * p + 2 < len(h.a):
            assert h.bits[p] == bit_of(h.a, p), p


def test_path_form_equals_cpython_heapq():
    rng = random.Random(7)
    for trial in range(60):
        ref, ph = [], PathHeap()
        tag = 0
        for step in range(rng.randint(50, 1500)):
            if ref and rng.random() < 0.45:
                r = heapq.heappop(ref)
                m = ph.pop()
                assert r is m, (trial, step)
            else:
                it = Item(float(rng.randint(0, 12)), rng.randint(0, 3), tag)
                tag += 1
                heapq.heappush(ref, it)
                ph.push(it)
            assert len(ref) == len(ph.a) and all(x is y for x, y in zip(ref, ph.a)), (trial, step)
            if ref:
                assert ph.root is ref[0] and ph.last is ref[-1], (trial, step)
            check_bits(ph)
