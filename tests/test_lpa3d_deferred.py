"""CPU model of lpa3d.hip's deferred U.remove (kDefer): inside one expansion's block a remove leaves a
hole, logical list positions map to the physical array through the pending holes' boundaries, the
pushes (CPython heapq.heappush on whatever order the list has, lpa_star3d.py:154-157) sift through
that map, and the block ends with one compaction.  The model follows the kernel's index arithmetic
(remove_at / phys / push_t / compact_t and the one-hole membership scan of update_block) and is
checked against the reference's own list semantics: `list.remove` and `heapq.heappush`."""
import heapq
import random

import pytest


class DeferredU:
    def __init__(self, items):
        self.a = list(items)  # physical array
        self.n = len(items)   # logical length
        self.hb = []          # hole boundaries b_j (live entries before hole j)

    def phys(self, L):
        return L + sum(1 for b in self.hb if L >= b)

    def remove_at(self, i):
        self.hb = [b - 1 if b > i else b for b in self.hb] + [i]
        self.n -= 1

    def push(self, item):
        np1 = self.n + 1
        D = np1.bit_length() - 1
        pj = [self.phys((np1 >> j) - 1) for j in range(D + 1)]  # lane j: path position (np1 >> j) - 1
        anc = [None] + [self.a[pj[j]] for j in range(1, D + 1)]
        s = 0
        while s + 1 <= D and item < anc[s + 1]:  # trailing "item < ancestor" run from the parent up
            s += 1
        need = pj[0] + 1 - len(self.a)
        if need > 0:
            self.a.extend([None] * need)
        for j in range(1, s + 1):
            self.a[pj[j - 1]] = anc[j]
        self.a[pj[s]] = item
        self.n += 1

    def scan_logical(self):
        """update_block's membership scan with at most one hole: physical walk, hole skipped."""
        assert len(self.hb) <= 1
        hole = self.hb[0] if self.hb else 1 << 30
        out = []
        for k in range(self.n + len(self.hb)):
            if k == hole:
                continue
            out.append((k - (1 if k > hole else 0), self.a[k]))
        return out

    def compact(self):
        if not self.hb:
            return
        frm = min(self.hb)
        n = self.n
        for base in range(frm, n, 256):
            L = [min(base + l, n - 1) for l in range(256)]
            P = [self.phys(x) for x in L]
            vals = [self.a[p] for p in P]  # every load of the round before its stores
            for l in range(256):
                if base + l < n and P[l] != L[l]:
                    self.a[L[l]] = vals[l]
        del self.a[n:]
        self.hb = []


def _run(seed, n0, steps):
    rng = random.Random(seed)
    keys = [(rng.randint(0, 6), rng.randint(0, 3), c) for c in range(n0)]
    ref = list(keys)
    rng.shuffle(ref)  # U is a list in arbitrary (not heap) order, as the reference's is
    mod = DeferredU(ref)
    nxt = n0
    # one popped node removed first (expand), then updateVertex-like remove / push pairs
    i = rng.randrange(len(ref))
    del ref[i]
    mod.remove_at(i)
    assert mod.scan_logical() == list(enumerate(ref))
    for _ in range(steps):
        if ref and rng.random() < 0.6:
            i = rng.randrange(len(ref))
            del ref[i]
            mod.remove_at(i)
        if rng.random() < 0.7:
            item = (rng.randint(0, 6), rng.randint(0, 3), nxt)
            nxt += 1
            heapq.heappush(ref, item)
            mod.push(item)
        assert [mod.a[mod.phys(L)] for L in range(mod.n)] == ref
    mod.compact()
    assert mod.a == ref


@pytest.mark.parametrize("seed", range(40))
def test_deferred_removes_match_list_semantics(seed):
    _run(seed, n0=[1, 2, 5, 40, 300, 700][seed % 6], steps=27)


def test_deferred_removes_long_lists():
    for seed in range(5):
        _run(1000 + seed, n0=1500, steps=27)
