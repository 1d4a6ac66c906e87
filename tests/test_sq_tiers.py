"""The single-query A* kernel's register form of the _siftup choice bits (astar2d_sq.hip: sq_pop_leaf,
sq_bits): levels 0-5 one bit per lane, levels 6-11 one 64-bit block word per lane, level 12 one word
per lane; a heappop's leaf from two "ballots" (each lane tests its own leaf of a 6-level block) and
the bits rebuilt lane by lane from the S / U ballots of an operation.  Modelled here lane for lane and
checked against Lib/heapq.py on random operation sequences with many exact ties, including heaps that
reach levels 12-13 (the third tier)."""
import heapq
import random

from test_heap_path_form import Item, bit_of, lt


def leaf_masks():
    M, V = [], []
    for lane in range(64):
        m = v = 0
        r = 1
        for k in range(6):
            bt = (lane >> (5 - k)) & 1
            m |= 1 << r
            v |= bt << r
            r = 2 * r + bt
        M.append(m)
        V.append(v)
    return M, V


MASK_M, MASK_V = leaf_masks()


def ballot(pred):
    return sum(1 << L for L in range(64) if pred(L))


def ffs(x):
    return (x & -x).bit_length() - 1


class SqHeap:
    def __init__(self):
        self.a = []
        self.t0 = [0] * 64
        self.w1 = [0] * 64
        self.w2 = [0] * 64

    # ---- sq_pop_leaf
    def pop_leaf(self, n):
        D = n.bit_length() - 1
        if D == 0:
            return 1, 0
        w0 = ballot(lambda L: self.t0[L] != 0)
        j0 = ffs(ballot(lambda L: ((w0 ^ MASK_V[L]) & MASK_M[L]) == 0))
        full = (1 << 13) | (j0 << 7)
        if D >= 7:
            w1 = self.w1[j0]
            j1 = ffs(ballot(lambda L: ((w1 ^ MASK_V[L]) & MASK_M[L]) == 0))
            full |= j1 << 1
            if D >= 13:
                full |= (self.w2[j0] >> j1) & 1
        u = full >> (14 - D)
        if 2 * u <= n:
            ch = (full >> (13 - D)) & 1 if 2 * u + 1 <= n else 0
            return 2 * u + ch, D
        return u, D - 1

    # ---- sq_bits
    def bits(self, Q, Kd, S, U):
        if U & 0x7E:
            for k in range(1, 64):
                lk = k.bit_length() - 1
                sh = Kd - lk
                if sh >= 1 and (Q >> sh) == k and (U >> (lk + 1)) & 1:
                    self.t0[k] = (S >> (lk + 1)) & 1
        if U & (0x3F << 7):
            j = (Q >> (Kd - 6)) - 64
            w = self.w1[j]
            new = 0
            for k in range(1, 64):
                lk = k.bit_length() - 1
                l = 6 + lk
                sh = Kd - l
                on = sh >= 1 and (((Q >> sh) ^ k) & ((1 << lk) - 1)) == 0 and (U >> (l + 1)) & 1
                bit = (S >> (l + 1)) & 1 if on else (w >> k) & 1
                new |= bit << k
            self.w1[j] = new
        if (U >> 13) & 1:
            u12 = Q >> (Kd - 12)
            j, i = (u12 >> 6) - 64, u12 & 63
            w = self.w2[j]
            self.w2[j] = (w & ~(1 << i)) | (((S >> 13) & 1) << i)

    # ---- sq_op
    def op(self, pop, Q, Kd, n, X):
        q = [(Q >> (Kd - L)) - 1 for L in range(Kd + 1)]
        V = [self.a[p] if p < len(self.a) else None for p in q]
        last15 = self.a[n - 1] if pop else None
        if pop:
            b = sum(1 for L in range(1, Kd + 1) if not lt(X, V[L]))
        else:
            b = Kd - sum(1 for L in range(Kd) if lt(X, V[L]))
        new = list(V)
        for L in range(Kd + 1):
            if L == b:
                new[L] = X
            elif pop and L < b:
                new[L] = V[L + 1]
            elif not pop and L > b:
                new[L] = V[L - 1]
        S = U = 0
        sib = {}
        for L in range(1, Kd + 1):
            s = ((q[L] - 1) ^ 1) + 1
            if s < n:
                sib[L] = self.a[s]
        if not pop:
            self.a.append(None)
        for L in range(Kd + 1):
            chg = L <= b if pop else L >= b
            if chg:
                self.a[q[L]] = new[L]
                if L >= 1 and L in sib:
                    v, s = new[L], sib[L]
                    bit = int(not lt(v, s)) if q[L] & 1 else int(not lt(s, v))
                    U |= 1 << L
                    S |= bit << L
        self.bits(Q, Kd, S, U)
        self.root = new[0]
        if pop:
            if not (b == Kd and Q == n):
                self.last = last15
        else:
            self.last = new[Kd]

    # ---- sq_bit1: one node's bit (a trivial push's parent)
    def bit1(self, u, bit):
        lv = u.bit_length() - 1
        if lv <= 5:
            self.t0[u] = bit
        elif lv <= 11:
            r = lv - 6
            j, k = (u >> r) - 64, (1 << r) | (u & ((1 << r) - 1))
            self.w1[j] = (self.w1[j] & ~(1 << k)) | (bit << k)
        else:
            j, i = (u >> 6) - 64, u & 63
            self.w2[j] = (self.w2[j] & ~(1 << i)) | (bit << i)

    def push(self, x):
        n = len(self.a)
        if n > 0 and not lt(x, self.a[(n - 1) >> 1]):  # the kernel's trivial-push path
            self.a.append(x)
            if n % 2 == 0:
                self.bit1(((n - 1) >> 1) + 1, int(not lt(self.last, x)))
            self.last = x
            return
        Q = n + 1
        self.op(False, Q, Q.bit_length() - 1, n, x)

    def push_batch(self, items):
        """An expansion's pushes in motion order: the leading run of trivial ones (each item not
        less than its parent, a position < n) stored together, then one by one (the kernel's batch)."""
        n = len(self.a)
        k = 0
        if n > 0:
            for i, x in enumerate(items):
                pos = n + i
                pp = (pos - 1) >> 1
                if pp >= n or lt(x, self.a[pp]):
                    break
                k += 1
            for i in range(k):
                pos = n + i
                self.a.append(items[i])
                if pos % 2 == 0:
                    left = self.last if i == 0 else items[i - 1]
                    self.bit1(((pos - 1) >> 1) + 1, int(not lt(left, items[i])))
            if k:
                self.last = items[k - 1]
        for x in items[k:]:
            self.push(x)

    def pop(self):
        root = self.a[0]
        last = self.a.pop()
        n = len(self.a)
        if n == 0:
            return root
        self.last = last
        Q, Kd = self.pop_leaf(n)
        self.op(True, Q, Kd, n, last)
        return root

    def bit(self, p):
        u = p + 1
        lv = u.bit_length() - 1
        if lv <= 5:
            return self.t0[u]
        if lv <= 11:
            r = lv - 6
            return (self.w1[(u >> r) - 64] >> ((1 << r) | (u & ((1 << r) - 1)))) & 1
        return (self.w2[(u >> 6) - 64] >> (u & 63)) & 1


def run(seed, steps, p_pop, grow_to=None):
    rng = random.Random(seed)
    ref, h = [], SqHeap()
    tag = 0
    for step in range(steps):
        fill = grow_to is not None and len(ref) < grow_to
        if ref and not fill and rng.random() < p_pop:
            r = heapq.heappop(ref)
            m = h.pop()
            assert r is m, (seed, step)
        elif rng.random() < 0.5:
            it = Item(float(rng.randint(0, 40)), rng.randint(0, 3), tag)
            tag += 1
            heapq.heappush(ref, it)
            h.push(it)
        else:  # an expansion's batch of up to 8 pushes
            items = []
            for _ in range(rng.randint(1, 8)):
                items.append(Item(float(rng.randint(0, 40)), rng.randint(0, 3), tag))
                tag += 1
            for it in items:
                heapq.heappush(ref, it)
            h.push_batch(items)
        assert len(ref) == len(h.a), (seed, step)
        if ref:
            assert h.root is ref[0] and h.last is ref[-1], (seed, step)
        if step % 97 == 0 or len(ref) < 80:
            assert all(x is y for x, y in zip(ref, h.a)), (seed, step)
            for p in range(len(ref)):
                if 2 * p + 2 < len(ref):
                    assert h.bit(p) == bit_of(ref, p), (seed, step, p)


def test_sq_tiers_small_heaps():
    for seed in range(20):
        run(seed, 800, 0.45)


def test_sq_tiers_levels_6_to_11():
    run(101, 6000, 0.35)
    run(102, 6000, 0.48)


def test_sq_tiers_level_12_13():
    # fill past 8191 entries (level 13), then mix pops and pushes at that depth
    run(201, 12500, 0.55, grow_to=9000)
