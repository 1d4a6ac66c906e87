"""The 3D A* kernel's decrease-key in place (astar3d.hip with heap16.h POS operations): a binary
min-heap on a total order with a cell -> position map kept current by every move, and the kernel's
way of keeping the positions it loaded at the start of an expansion current through that expansion's
operations (the pop moves the path below the root up one level and the old last entry to the hole; a
sift-up from p0 moves the ancestors of p0 from its landing position down one level toward p0).
Checked here against a plain reference on random sequences: the pop order equals the sorted order of
live keys, the map always points at each cell's entry, and the corrected positions equal the map."""
import random


class PosHeap:
    def __init__(self):
        self.a = []      # entries (key, cell)
        self.pos = {}    # cell -> position

    def _put(self, p, e):
        self.a[p] = e
        self.pos[e[1]] = p

    def pop(self):
        """heap16.pop: the hole descends along the smaller child while that child < last."""
        root = self.a[0]
        last = self.a.pop()
        del self.pos[root[1]]
        n = len(self.a)
        if n == 0:
            return root, 0
        hole = 0
        while True:
            c = 2 * hole + 1
            if c >= n:
                break
            if c + 1 < n and self.a[c + 1][0] < self.a[c][0]:
                c += 1
            if not (self.a[c][0] < last[0]):
                break
            self._put(hole, self.a[c])
            hole = c
        self._put(hole, last)
        return root, hole

    def sift_up(self, p0, e):
        """heap16.sift_up: a push at p0 = n or a decrease-key of the entry at p0."""
        if p0 == len(self.a):
            self.a.append(None)
        p = p0
        while p > 0 and e[0] < self.a[(p - 1) >> 1][0]:
            self._put(p, self.a[(p - 1) >> 1])
            p = (p - 1) >> 1
        self._put(p, e)
        return p


def level(p):
    return (p + 1).bit_length() - 1


def fix_after_pop(npos, n, hole):
    """astar3d.hip after the pop (n = the decremented size)."""
    if npos is None or n == 0:
        return npos
    d = level(hole) - level(npos)
    if npos == n:
        return hole
    if npos != 0 and d >= 0 and ((hole + 1) >> d) == npos + 1:
        return (npos - 1) >> 1
    return npos


def fix_after_sift(npos, p0, ip):
    if npos is None:
        return None
    d = level(p0) - level(npos)
    if d >= 1 and ((p0 + 1) >> d) == npos + 1 and level(npos) >= level(ip):
        return ((p0 + 1) >> (d - 1)) - 1
    return npos


def test_decrease_key_positions_and_order():
    rng = random.Random(11)
    for trial in range(40):
        h = PosHeap()
        live = {}  # cell -> key
        ctr = 0
        cells = list(range(400))
        for c in rng.sample(cells, 40):
            ctr += 1
            k = (rng.randint(0, 60), ctr)
            live[c] = k
            h.sift_up(len(h.a), (k, c))
        for step in range(300):
            if not h.a:
                break
            # one expansion: positions of some cells loaded first, then the pop, then a batch of
            # pushes / decrease-keys, each followed by the corrections
            batch = rng.sample(cells, 8)
            npos = {c: h.pos.get(c) for c in batch}
            n_before = len(h.a)
            root, hole = h.pop()
            assert root[0] == min(live.values()) and live.pop(root[1]) == root[0]
            npos = {c: (None if c == root[1] else fix_after_pop(p, n_before - 1, hole)) for c, p in npos.items()}
            for c in batch:
                assert npos[c] == h.pos.get(c), (trial, step, c)
            for c in batch:
                if c == root[1]:
                    continue
                ctr += 1
                k = (rng.randint(0, 60), ctr)
                if c in live and not (k < live[c]):
                    continue  # not an improvement: dead on arrival
                p0 = npos[c] if c in live else len(h.a)
                ip = h.sift_up(p0, (k, c))
                live[c] = k
                npos[c] = ip
                for o in batch:
                    if o != c:
                        npos[o] = fix_after_sift(npos[o], p0, ip)
                for o in batch:
                    assert npos[o] == h.pos.get(o), (trial, step, o)
            for p, e in enumerate(h.a):
                assert h.pos[e[1]] == p
                if p:
                    assert not (e[0] < h.a[(p - 1) >> 1][0])


def test_batch_store_then_sift_up_below_parent():
    """astar3d.hip's batch: an expansion's live items stored at n, n + 1, ... together, then only the
    ones below their (pre-batch) parent -- or whose parent is another new item -- sift up, in position
    order.  The result must be a valid heap holding every entry, and the skipped items must still be
    not below their parents at the end (a sift-up only lowers the parents of later positions)."""
    import heapq

    rng = random.Random(5)
    for trial in range(300):
        h = PosHeap()
        ref = []
        ctr = 0
        for _ in range(rng.randint(0, 60)):
            ctr += 1
            e = ((rng.randint(0, 30), ctr), ctr)
            h.sift_up(len(h.a), e)
            heapq.heappush(ref, e)
        for _ in range(20):
            n0 = len(h.a)
            k = rng.randint(1, 26)
            items = []
            for _ in range(k):
                ctr += 1
                items.append(((rng.randint(0, 30), ctr), ctr))
            below = []
            for r, e in enumerate(items):
                pos, pp = n0 + r, (n0 + r - 1) >> 1
                below.append(not (pos > 0 and pp < n0) or e[0] < h.a[pp][0])
            for e in items:
                h.a.append(e)
                h.pos[e[1]] = len(h.a) - 1
            for r, e in enumerate(items):
                if below[r]:
                    h.sift_up(n0 + r, e)
            for e in items:
                heapq.heappush(ref, e)
            assert sorted(h.a) == sorted(ref)
            for p in range(1, len(h.a)):
                assert not (h.a[p][0] < h.a[(p - 1) >> 1][0]), (trial, p)
            for _ in range(rng.randint(0, 10)):
                if h.a:
                    a, _ = h.pop()
                    b = heapq.heappop(ref)
                    assert a == b
