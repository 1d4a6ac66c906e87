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

    def push_pair(self, x1, x2):
        """astar2d_mq.hip's push pair (round 6): the first push at position n (odd: a left child) and
        the second at n + 1, its sibling, in one operation -- the second insertion runs on the chain
        (levels 0..Kd-1) the first produced, X2 at the top of the chain's run of levels greater than
        it, the chain's old bottom (or X2) in the new leaf; the first leaf's parent bit compares the
        two leaves."""
        n = len(self.a)
        assert n % 2 == 1
        Q = n + 1
        Kd = Q.bit_length() - 1
        q = [(Q >> (Kd - L)) - 1 for L in range(Kd + 1)]
        V = [self.a[p] if p < n else None for p in q]
        b = Kd - sum(1 for L in range(Kd) if lt(x1, V[L]))
        new = [x1 if L == b else (V[L - 1] if L > b else V[L]) for L in range(Kd + 1)]
        cnt2 = sum(1 for L in range(Kd) if lt(x2, new[L]))
        b2 = Kd - cnt2
        chain = [x2 if L == b2 else (new[L - 1] if L > b2 else new[L]) for L in range(Kd)] + [new[Kd]]
        leaf2 = new[Kd - 1] if cnt2 > 0 else x2
        bst = min(b, b2)
        self.a.extend([None, None])
        for L in range(bst, Kd + 1):
            self.a[q[L]] = chain[L]
        self.a[n + 1] = leaf2
        for L in range(max(1, bst), Kd):
            s = ((q[L] - 1) ^ 1) + 1
            if s < n:
                self._set_bit(q[L - 1], (q[L], chain[L]), self.a[s])
        self._set_bit(q[Kd - 1], (q[Kd], chain[Kd]), leaf2)
        self.root = chain[0]
        self.last = leaf2
        return bst

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


def test_push_pairs_equal_two_cpython_heappushes():
    """The multi-query kernel's push pairs (two pending pushes at sibling positions n, n + 1 in one
    path operation, heaps of >= 16 entries) against two heapq.heappush calls, interleaved with pops
    and single pushes: array, bits, root and last after every operation."""
    rng = random.Random(11)
    pairs = 0
    for trial in range(60):
        ref, ph = [], PathHeap()
        tag = 0
        for step in range(rng.randint(100, 1500)):
            n = len(ref)
            r = rng.random()
            if ref and r < 0.4:
                assert heapq.heappop(ref) is ph.pop(), (trial, step)
            elif n >= 16 and n % 2 == 1 and r < 0.8:
                x1 = Item(float(rng.randint(0, 12)), rng.randint(0, 3), tag)
                x2 = Item(float(rng.randint(0, 12)), rng.randint(0, 3), tag + 1)
                tag += 2
                heapq.heappush(ref, x1)
                heapq.heappush(ref, x2)
                ph.push_pair(x1, x2)
                pairs += 1
            else:
                it = Item(float(rng.randint(0, 12)), rng.randint(0, 3), tag)
                tag += 1
                heapq.heappush(ref, it)
                ph.push(it)
            assert len(ref) == len(ph.a) and all(x is y for x, y in zip(ref, ph.a)), (trial, step)
            if ref:
                assert ph.root is ref[0] and ph.last is ref[-1], (trial, step)
            check_bits(ph)
    assert pairs > 5000
