"""The 3D A* kernel's batch store of an expansion's pushes (astar3d.hip, heap16.h push_batch) on a
binary min-heap of a total order, modelled here (heap16.h pop / sift_up) and checked against
Lib/heapq.py on random sequences.  (Round 4's decrease-key-in-place variant was slower and was
removed in round 5, with its model.)"""
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
