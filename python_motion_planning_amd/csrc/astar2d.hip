// Batched 2D A* for gfx950, bit-exact with the reference AStar.plan
// (global_planner/graph_search/a_star.py:39-83) including CPython heapq's tie behaviour
// (Lib/heapq.py heappush/_siftdown, heappop/_siftup) under Node.__lt__ (utils/environment/node.py:51-54).
//
// Execution model: persistent workers, one wave64 each, pull query indices from an atomic queue.
// A worker keeps the query's whole CPython heap array in LDS (positions >= lds_cap spill to a
// per-worker HBM array) and a 4-bit-per-cell state array in HBM (0 = open, dir+1 = closed with
// parent motion `dir`), reused across the queries it processes.
//
// Heap entry (12 B in LDS as SoA: f64 f[] | u32 cm[]):
//   cm = dx << 18 | dy << 4 | dir, with (dx, dy) = goal - cell as 14-bit two's-complement fields and
//   dir = the motion index (env.py:52-55) that reached the cell from its parent, 8 = start.  The
//   start entry stores (dx, dy) = (0, 0): its h is 0 (planner.py:15); its real cell is the query's.
//   f = g + h as Node.__lt__ computes it (euclidean h = hypot(dx, dy) == sqrt(d2) exactly for
//   |d| <= 16384, pinned against CPython's vector_norm; manhattan h = |dx| + |dy|).
//   Node.__lt__: f < f' or (f == f' and h < h'); h order == hkey order (dx^2 + dy^2, or |dx| + |dy|),
//   four integer ops from cm, so loading an entry costs no transcendental.
//   g of a popped node = G[parent] + motion cost (node.py:39-41), G written when the parent closed,
//   loaded in the same HBM round as the node's 3x3 occupancy / CLOSED block.
//
// heappop (CPython: pop last, put it at the root, _siftup walks the smaller child -- right child
// when not left < right -- to a leaf, then _siftdown moves it back up).  The final array equals a
// top-down walk along that same child path that moves each chosen child up while
// !(last < child) and drops `last` at the first child it is less than (the path is sorted, so the
// "not less" set is a prefix).  The path comes from per-node child-choice bits (below) in a scalar
// walk of two instructions per level; one LDS round loads the path; a ballot popcount places last.
// heappush (_siftdown): the ancestors load in one round, one ballot finds how many move down.
// Both operations are written for a low instruction count: the kernel is issue-bound (one wave per
// query, a few waves per SIMD), so every instruction on the heap path costs wall time.
#include "pmp_internal.h"
#include "grid2d.h"

// Diagnostic build only (make stamps -> libpmp_hip_stamps.so): per-query cycle sums of the
// expansion segments go to counters[4q+0..3] = {pop, 3x3 wait, push, total} instead of the counts.
#ifdef PMP_STAMPS
#define STAMP(v) uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define STAMP(v)
#endif

namespace {

constexpr int kMaxDim = 8192;
constexpr double kSqrt2 = 1.4142135623730951;  // math.sqrt(2) == math.hypot(1, 1)

// motions in the order of env.py:52-55: (-1,0),(-1,1),(0,1),(1,1),(1,0),(1,-1),(0,-1),(-1,-1),
// as 2-bit fields of (m + 1)
constexpr uint32_t kMx1 = 0x1A90u, kMy1 = 0x01A9u;
__device__ __forceinline__ int mot_x(int d) { return (int)((kMx1 >> (2 * d)) & 3u) - 1; }
__device__ __forceinline__ int mot_y(int d) { return (int)((kMy1 >> (2 * d)) & 3u) - 1; }

// HEUR (a template parameter, so key computations carry no runtime branch): bits 0-1 = the
// heuristic -- 0 euclidean, 1 manhattan (GraphSearcher.h, graph_search.py:41-44), 2 zero (Dijkstra's
// node_n.h = 0, dijkstra.py:74); bit 2 = the Theta* entry layout: a 5-bit code instead of the 4-bit
// dir (code 16 + dir = "path 2": the parent is the pusher's own parent, theta_star.py:104-108) and a
// 13-bit dy field (H <= 4096).
constexpr int kThetaLayout = 4;
template <int HEUR> constexpr int hkind() { return HEUR & 3; }
template <int HEUR> constexpr int dbits() { return (HEUR & kThetaLayout) ? 5 : 4; }
template <int HEUR>
__device__ __forceinline__ uint32_t pack_cm(int dx, int dy, int dir)
{
    constexpr int S = dbits<HEUR>();
    return ((uint32_t)dx << 18) | (((uint32_t)dy & ((1u << (18 - S)) - 1u)) << S) | (uint32_t)dir;
}
template <int HEUR> __device__ __forceinline__ int cm_dx(uint32_t cm) { return (int)cm >> 18; }
template <int HEUR> __device__ __forceinline__ int cm_dy(uint32_t cm) { return (int)(cm << 14) >> (14 + dbits<HEUR>()); }
template <int HEUR> __device__ __forceinline__ int cm_dir(uint32_t cm) { return (int)(cm & ((1u << dbits<HEUR>()) - 1u)); }

// The order key of h.
template <int HEUR>
__device__ __forceinline__ uint32_t hkey(uint32_t cm)
{
    if (hkind<HEUR>() == 2) return 0u;
    const int dx = cm_dx<HEUR>(cm), dy = cm_dy<HEUR>(cm);
    if (hkind<HEUR>() == 1) return (uint32_t)(abs(dx) + abs(dy));
    return (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
}
template <int HEUR>
__device__ __forceinline__ double h_of_key(uint32_t hk)
{
    return hkind<HEUR>() == 2 ? 0.0 : (hkind<HEUR>() == 1 ? (double)hk : __dsqrt_rn((double)hk));
}

// Node.__lt__ (node.py:51-54) -- evaluated without short-circuit branches
__device__ __forceinline__ bool key_lt(double fa, uint32_t ka, double fb, uint32_t kb)
{
    return (fa < fb) | ((fa == fb) & (ka < kb));
}

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Direction bits.  For every node p with two children the heap also keeps CPython _siftup's child
// choice bit(p) = !(heap[2p+1] < heap[2p+2]) (Lib/heapq.py: "if rightpos < endpos and not
// heap[childpos] < heap[rightpos]: childpos = rightpos"), so the whole sift path of a heappop is
// known from bits alone.  Bits live in 5-level subtree blocks: the u32 block of tier t (levels
// 5t..5t+4) rooted at node a keeps node (a's descendant r levels down, offset o) at bit (1<<r)-1+o.
// LDS word 0 = tier 0, words 1..32 = tier 1, words 33..1056 = tier 2; tiers >= 3 (heaps of more than
// 32767 entries) in HBM.  A bit is only meaningful while its node has two children: it is rewritten
// whenever a push gives a node its right child or a push/pop changes one of its children, and the
// walk ignores it for a node with one child.
constexpr int kBitsLdsWords = 1057;
constexpr int kBitsLdsBytes = 4240;  // 1057 words, padded to 16 B
static_assert(kBitsLdsBytes >= 4 * kBitsLdsWords, "bit blocks overflow their LDS region");
constexpr int kBigHeap = 32767;  // from this size on, levels >= 15 exist: bit tiers >= 3 in HBM

struct Heap {
    lds_f64* F;        // LDS f[lds_cap]
    lds_u32* C;        // LDS cm[lds_cap]
    lds_u32* B;        // LDS direction-bit blocks of tiers 0..2
    uint32_t* hb;      // HBM direction-bit blocks of tiers >= 3
    __amdgpu_buffer_rsrc_t spill;  // HBM entries {f lo, f hi, cm, 0} for positions >= lds_cap
    int cap;
};

// per lane: bit `lane` of mask ? a : b
__device__ __forceinline__ uint32_t sel_lanes(uint64_t mask, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
    return r;
}

// Entry load in two phases, so a round of several loads is issued before any value is used.
// SPILL = false: every position touched is < cap (pure ds_read code).  SPILL: both an LDS read
// (clamped address) and a buffer read are issued and the right one selected; a position < cap
// gives a negative buffer offset, which is out of range and reads 0 -- no branch.
template <bool SPILL>
struct Ld {
    double fl;
    uint32_t cl;
    uint4 v;
    bool in;
    __device__ __forceinline__ void issue(const Heap& h, int p)
    {
        if constexpr (!SPILL) {
            fl = h.F[p];
            cl = h.C[p];
        } else {
            in = p < h.cap;
            const int pl = in ? p : 0;
            // 12 of the entry's 16 bytes: a b128 load left a 4th destination register that the compiler
            // reused for the LDS load below, a write-after-write that waited for the HBM load at once
            const auto w = __builtin_amdgcn_raw_buffer_load_b96(h.spill, (p - h.cap) * 16, 0, 0);
            v = make_uint4(w[0], w[1], w[2], 0u);
            fl = h.F[pl];
            cl = h.C[pl];
        }
    }
    // the select as explicit v_cndmask: left to itself the compiler turns it into an LDS load
    // predicated into the buffer load's registers, which must first wait for the buffer load
    __device__ __forceinline__ void get(double& f, uint32_t& c) const
    {
        if constexpr (!SPILL) {
            f = fl;
            c = cl;
        } else {
            const uint64_t m = ballot(in);
            const uint64_t b = (uint64_t)__double_as_longlong(fl);
            f = __hiloint2double((int)sel_lanes(m, (uint32_t)(b >> 32), v.y), (int)sel_lanes(m, (uint32_t)b, v.x));
            c = sel_lanes(m, cl, v.z);
        }
    }
};
template <bool SPILL>
__device__ __forceinline__ void hld(const Heap& h, int p, double& f, uint32_t& c)
{
    Ld<SPILL> l;
    l.issue(h, p);
    l.get(f, c);
}
// Entry store by the lanes with `on`; the buffer store of a lane that does not spill gets an
// out-of-range offset and is dropped by the hardware.
template <bool SPILL>
__device__ __forceinline__ void hst(const Heap& h, bool on, int p, double f, uint32_t c)
{
    if constexpr (!SPILL) {
        if (on) {
            h.F[p] = f;
            h.C[p] = c;
        }
    } else {
        if (on && p < h.cap) {
            h.F[p] = f;
            h.C[p] = c;
        }
        const uint64_t b = (uint64_t)__double_as_longlong(f);
        const uint4 v = make_uint4((uint32_t)b, (uint32_t)(b >> 32), c, 0u);
        const int off = (on && p >= h.cap) ? (p - h.cap) * 16 : -16;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                               h.spill, off, 0, 0);
    }
}

// HBM word of tier t >= 3 for the block whose root has path number R (= root position + 1):
// tier t starts after sum_{s=3}^{t-1} 32^s = (32^t - 32^3) / 31 words
__device__ __forceinline__ size_t hb_word(int t, uint32_t R)
{
    const size_t base = (size_t)1 << (5 * t);
    return (base - 32768u) / 31u + (size_t)(R - (uint32_t)base);
}

// LDS atomic masked OR: word = (word & ~mask) | val, no return value (nothing waits on it).  LDS
// operations of one wave complete in order, so later ds_reads of the word see it.
__device__ __forceinline__ void ds_mskor(lds_u32* w, uint32_t mask, uint32_t val)
{
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)w), "v"(mask), "v"(val) : "memory");
}

// Block coordinates of a level: tier t = level / 5, r = level - 5t, mr = 2^r - 1 and the LDS word
// offset of the tier's blocks (word = block root path number + off).
struct Lvl {
    int t, r;
    uint32_t mr;
    int off;
};
__device__ __forceinline__ Lvl lvl_of(int level)
{
    Lvl l;
    l.t = (int)((uint32_t)__mul24(level, 13) >> 6);  // level / 5 for level < 64
    l.r = level - __mul24(l.t, 5);
    l.mr = (1u << l.r) - 1u;
    l.off = l.t == 0 ? -1 : (l.t == 1 ? -31 : -991);
    return l;
}

// Set the direction bit of the node whose path number (position + 1) is Pl, at the level `L`
// describes, on the lanes with `on`; the bit value is this lane's bit of `bits`.  Lanes may share a
// block word, hence the atomics.
template <bool BIG>
__device__ __forceinline__ void bit_write(const Heap& h, bool on, const Lvl& L, uint32_t Pl, uint64_t bits)
{
    const uint32_t R = Pl >> L.r;
    const uint32_t m = 1u << ((Pl & L.mr) + L.mr);  // node (R's descendant, offset Pl - R 2^r) of the block
    const uint32_t v = sel_lanes(bits, m, 0u);
    if (!BIG || L.t <= 2) {
        if (on) ds_mskor(h.B + (int)R + L.off, m, v);
    } else if (on) {
        uint32_t* w = h.hb + hb_word(L.t, R);
        if (v) __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_and(w, ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// bit_write for one wave-uniform bit value, by lane 0 (any heap size)
__device__ __forceinline__ void bit_write1(const Heap& h, int lane, const Lvl& L, uint32_t Pl, bool bit)
{
    const uint32_t R = Pl >> L.r;
    const uint32_t m = 1u << ((Pl & L.mr) + L.mr);
    if (lane != 0) return;
    if (L.t <= 2) {
        ds_mskor(h.B + (int)R + L.off, m, bit ? m : 0u);
    } else {
        uint32_t* w = h.hb + hb_word(L.t, R);
        if (bit) __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_and(w, ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Lane mask of the lanes where a < b under Node.__lt__ (node.py:51-54) on (f, h) pairs, h ordered by
// hkey(cm); compares go straight to lane masks (no bool round trips through VGPRs).
template <int HEUR>
__device__ __forceinline__ uint64_t lt_mask(bool on, double fa, uint32_t ca, double fb, uint32_t cb)
{
    const uint64_t lt = ballot(on && fa < fb);
    const uint64_t eq = ballot(on && fa == fb);
    return lt | (eq & ballot(hkey<HEUR>(ca) < hkey<HEUR>(cb)));
}
// CPython _siftup's choice bit of a parent whose child `child` (a position) now holds (vf, vc) and
// whose other child holds (sf, sc): bit = !(left < right).  Returns the lane mask of bits.
template <int HEUR>
__device__ __forceinline__ uint64_t choice_bits(int child, double vf, uint32_t vc, double sf, uint32_t sc)
{
    const uint64_t eq = ballot(vf == sf);
    const uint32_t vk = hkey<HEUR>(vc), sk = hkey<HEUR>(sc);
    const uint64_t vlt = ballot(vf < sf) | (eq & ballot(vk < sk));
    const uint64_t slt = ballot(sf < vf) | (eq & ballot(sk < vk));
    const uint64_t left = ballot((child & 1) != 0);  // odd positions are left children
    return (left & ~vlt) | (~left & ~slt);
}

// Five levels of the _siftup path inside one bit block: w2 = block word << 1 (node Pr of the
// block, Pr = 1 at its root, is bit Pr); returns Pr after five steps (32..63).  Each step is
// SCC = bit Pr of w2; Pr = 2 Pr + SCC.  Steps past the block's last real level are harmless:
// the caller keeps the prefix it needs (Pr >> (5 - steps)).
__device__ __forceinline__ uint32_t walk5(uint32_t w2)
{
    uint32_t pr = 1;
    asm("s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, %0\n\t"
        "s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, %0\n\t"
        "s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, %0\n\t"
        "s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, %0\n\t"
        "s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, %0"
        : "+s"(pr)
        : "s"(w2)
        : "scc");
    return pr;
}

__device__ __forceinline__ void wave_sync_mem()
{
    // Orders this wave's LDS and HBM accesses across its lanes.  A wave's memory operations are
    // performed in order, so wavefront scope needs no s_waitcnt (LLVM AMDGPU memory model): this
    // is a compiler barrier only and never stalls on outstanding HBM stores.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// heappop on a heap of n (> 0, already decremented) entries whose old last element sits at
// position n; the old root has been taken by the caller.  Updates the wave-uniform root (heap[0]).
//  1. the _siftup path p_0 = 0, p_1, .., p_K (a leaf) from the direction bits: tier-0/1 words come
//     with `last` in one LDS round, the 32 tier-2 candidates in a second round issued as soon as the
//     tier-1 block is known; the walk itself is scalar;
//  2. one round: lane i in 1..K loads heap[p_i], heap[p_{i+1}] and heap[sibling(p_i)];
//  3. the children that move up are the prefix with !(last < heap[p_i]) (the path is sorted), so a
//     ballot popcount m places `last` at p_m -- the array CPython's _siftup + _siftdown produce;
//  4. lanes 1..m rewrite the bits of p_0..p_{m-1}, whose children changed.
// What a pop wrote, for callers that hold heap values loaded before it (the parent window): the
// leaf's path number P and level K, the mover count m (p_{j-1} <- A_j for j <= m, p_m <- last) and
// lane j's A_j = heap[p_j] before the pop.
struct PopOut {
    uint32_t P;
    int K, m;
    double Af;
    uint32_t Ac;
};

template <bool SPILL, bool BIG, int HEUR>
__device__ __forceinline__ void heap_pop(const Heap& h, int n, uint32_t v01, double& lastf, uint32_t& lastc, double& rootf,
                                         uint32_t& rootc, const Lvl& pl, int lane, PopOut& po)
{
    n = uni(n);
    // `last` = heap[n] is kept in registers by the caller (no load round); v01 = the tier-0 word
    // (lane 0) and tier-1 words (lanes 1..32), loaded by the caller ahead of time
    const double lf = lastf;
    const uint32_t lc = lastc;

    // ---- 1. the path.  Levels 0..D-1 are full (D = floor(log2 n)), so every node above level D-1
    //      has two children and the walk takes D-1 unconditional steps; the last step (level D-1 ->
    //      D) exists only below a node with a child.  P = path number (position + 1); (w, prel) =
    //      the block word (<< 1) and the block-relative number of the current node.
    const int D = 31 - __clz(n);
    const int full = D - 1;
    uint32_t P = 1, prel = 1, w = rl_u32(v01, 0) << 1;
    int lvl = 0;
    if (full > 0) {
        const int s0 = min(5, full);
        const uint32_t pr0 = walk5(w);
        prel = pr0 >> (5 - s0);
        P = prel;
        lvl = s0;
        if (s0 == 5) {  // P roots a tier-1 block
            const uint32_t R1 = P;
            uint32_t v2 = 0;
            if (full >= 10) v2 = h.B[33 + (R1 << 5) - 1024 + (uint32_t)(lane & 31)];
            w = rl_u32(v01, (int)R1 - 31) << 1;
            prel = 1;
            if (full > 5) {
                const int s1 = min(5, full - 5);
                const uint32_t pr1 = walk5(w);
                prel = pr1 >> (5 - s1);
                P = (R1 << s1) + prel - (1u << s1);
                lvl = 5 + s1;
                if (s1 == 5) {  // P roots a tier-2 block
                    const uint32_t R2 = P;
                    w = rl_u32(v2, (int)(R2 - (R1 << 5))) << 1;
                    prel = 1;
                    if (full > 10) {
                        const int s2 = min(5, full - 10);
                        const uint32_t pr2 = walk5(w);
                        prel = pr2 >> (5 - s2);
                        P = (R2 << s2) + prel - (1u << s2);
                        lvl = 10 + s2;
                        if constexpr (BIG) {
                            // tiers >= 3 (heaps above 32767 entries): L2-coherent reads of the HBM blocks
                            int s = s2;
                            for (int t = 3; s == 5; t++) {
                                w = (uint32_t)uni((int)__hip_atomic_fetch_or(h.hb + hb_word(t, P), 0u, __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT)) << 1;
                                prel = 1;
                                if (full <= lvl) break;
                                s = min(5, full - lvl);
                                const uint32_t pr = walk5(w);
                                prel = pr >> (5 - s);
                                P = (P << s) + prel - (1u << s);
                                lvl += s;
                            }
                        }
                    }
                }
            }
        }
    }
    // the last step: below the node at level D-1 if it has a child (position 2P - 1 < n); the bit
    // counts only when it also has a right child
    if (2u * P <= (uint32_t)n) {
        const uint32_t c = (2u * P < (uint32_t)n) ? ((w >> prel) & 1u) : 0u;
        P = 2u * P + c;
        lvl++;
    }
    const int K = lvl;

    // ---- 2. one load round; lane 0 loads heap[n - 1], the next `last`
    const bool on = lane >= 1 && lane <= K;
    const int sh = on ? K - lane : 0;
    const int pi = on ? (int)(P >> sh) - 1 : (lane == 0 ? n - 1 : 0);
    const bool hasb = on && lane < K;
    const int pn = hasb ? (int)(P >> (sh - 1)) - 1 : 0;
    const int si = ((pi - 1) ^ 1) + 1;  // sibling: odd (left) p -> p + 1, even (right) p -> p - 1
    const bool hass = on && si < n;
    double Af, Bf, Sf;
    uint32_t Ac, Bc, Sc;
    {
        Ld<SPILL> la, lb, ls;
        la.issue(h, pi);
        lb.issue(h, pn);
        ls.issue(h, hass ? si : 0);
        la.get(Af, Ac);
        lb.get(Bf, Bc);
        ls.get(Sf, Sc);
    }

    // ---- 3. movers: lanes 1..m store heap[p_i] at p_{i-1}; lane 0 stores last at p_m
    const uint64_t onm = ballot(on);
    const int m = __popcll(onm & ~lt_mask<HEUR>(on, lf, lc, Af, Ac));
    {
        const bool l0 = lane == 0;
        const bool st = l0 || (on && lane <= m);
        const int dst = (int)(P >> (l0 ? K - m : sh + 1)) - 1;
        hst<SPILL>(h, st, dst, l0 ? lf : Af, l0 ? lc : Ac);
    }
    if (m >= 1) {
        rootf = rl_f64(Af, 1);
        rootc = rl_u32(Ac, 1);
    } else {
        rootf = lf;
        rootc = lc;
    }
    // the new last element heap[n - 1]: n - 1 has no children, so of the path it can only be the
    // leaf p_K, which this pop rewrites only when last itself lands there
    if (!(m == K && P == (uint32_t)n)) {
        lastf = rl_f64(Af, 0);
        lastc = rl_u32(Ac, 0);
    }

    // ---- 4. bits of p_0 .. p_{m-1}: the new heap[p_i] against its sibling
    {
        const bool useb = lane < m;
        const uint64_t bits = choice_bits<HEUR>(pi, useb ? Bf : lf, useb ? Bc : lc, Sf, Sc);
        bit_write<BIG>(h, hass && lane <= m, pl, P >> (sh + 1), bits);
    }
    po.P = P;
    po.K = K;
    po.m = m;
    po.Af = Af;
    po.Ac = Ac;
    wave_sync_mem();
}

// heappush of `it` onto a heap of n entries (position n is free): the ancestors a_j = parent^j(n)
// load in one round (with the siblings of a_{j-1}, for the bits); a ballot popcount t gives how
// many move down; lanes 1..t+1 rewrite the bits of a_1..a_{t+1}, whose children changed.
template <bool SPILL, bool BIG, int HEUR>
__device__ __forceinline__ void heap_push(const Heap& h, int n, double itf, uint32_t itc, uint32_t itk, double& lastf,
                                          uint32_t& lastc, double& rootf, uint32_t& rootc, int lane, int& t_out,
                                          double& a1f, uint32_t& a1c)
{
    n = uni(n);
    const uint32_t np1 = (uint32_t)n + 1u;
    const int D = 31 - __clz((int)np1);  // depth of position n
    const bool on = lane >= 1 && lane <= D;
    const int l1 = on ? lane : 1;
    const int aj = (int)(np1 >> l1) - 1;        // a_j
    const int x = (int)(np1 >> (l1 - 1)) - 1;   // a_{j-1}
    const int sx = ((x - 1) ^ 1) + 1;
    const bool hass = on && sx < n;  // a_{j-1} = n (lane 1) has a sibling only when n is even
    double Af, Sf;
    uint32_t Ac, Sc;
    {
        Ld<SPILL> la, ls;
        la.issue(h, on ? aj : 0);
        ls.issue(h, hass ? sx : 0);
        la.get(Af, Ac);
        ls.get(Sf, Sc);
    }
    const int t = __popcll(lt_mask<HEUR>(on, itf, itc, Af, Ac));  // the "less" set is a prefix from the parent up
    const int ipos = (int)(np1 >> t) - 1;
    // the new heap[a_1] (the parent): the item when it stops there, else a_2's old entry
    t_out = t;
    a1f = t >= 2 ? rl_f64(Af, 2) : itf;
    a1c = t >= 2 ? rl_u32(Ac, 2) : itc;
    {
        const bool l0 = lane == 0;
        const bool st = l0 || (on && lane <= t);
        hst<SPILL>(h, st, l0 ? ipos : x, l0 ? itf : Af, l0 ? itc : Ac);
    }
    if (ipos == 0) {
        rootf = itf;
        rootc = itc;
    }
    // the new last element heap[n]: the item, or the parent that moved down into n
    if (t == 0) {
        lastf = itf;
        lastc = itc;
    } else {
        lastf = rl_f64(Af, 1);
        lastc = rl_u32(Ac, 1);
    }
    {
        const bool usea = lane - 1 < t;  // the new heap[a_{j-1}]
        const uint64_t bits = choice_bits<HEUR>(x, usea ? Af : itf, usea ? Ac : itc, Sf, Sc);
        bit_write<BIG>(h, hass && lane <= t + 1, lvl_of(D - l1), np1 >> l1, bits);
    }
    wave_sync_mem();
}

template <int HEUR>
__device__ __forceinline__ void pop_any(const Heap& h, int n, uint32_t v01, double& lastf, uint32_t& lastc, double& rootf,
                                        uint32_t& rootc, const Lvl& pl, int lane, PopOut& po)
{
    if (n < h.cap) heap_pop<false, false, HEUR>(h, n, v01, lastf, lastc, rootf, rootc, pl, lane, po);
    else if (n < kBigHeap) heap_pop<true, false, HEUR>(h, n, v01, lastf, lastc, rootf, rootc, pl, lane, po);
    else heap_pop<true, true, HEUR>(h, n, v01, lastf, lastc, rootf, rootc, pl, lane, po);
}
template <int HEUR>
__device__ __forceinline__ void push_any(const Heap& h, int n, double itf, uint32_t itc, uint32_t itk, double& lastf,
                                         uint32_t& lastc, double& rootf, uint32_t& rootc, int lane, int& t,
                                         double& a1f, uint32_t& a1c)
{
    if (n < h.cap) heap_push<false, false, HEUR>(h, n, itf, itc, itk, lastf, lastc, rootf, rootc, lane, t, a1f, a1c);
    else if (n < kBigHeap) heap_push<true, false, HEUR>(h, n, itf, itc, itk, lastf, lastc, rootf, rootc, lane, t, a1f, a1c);
    else heap_push<true, true, HEUR>(h, n, itf, itc, itk, lastf, lastc, rootf, rootc, lane, t, a1f, a1c);
}



// 4-bit cell state: word i >> 3, nibble i & 7
template <typename P>
__device__ __forceinline__ uint32_t cst_at(P cst, uint32_t i) { return (cst[i >> 3] >> ((i & 7) * 4)) & 15u; }

// LDSG (small grids): the worker's occupancy bits, cell-state nibbles and G live in its LDS share
// behind the heap, so an expansion's 3x3 round, G[parent] and the CLOSED write are LDS accesses (one
// query's latency is a chain of these rounds: the drop-in single-query path)
template <bool LDSG> struct GridMem {
    typedef const uint32_t* Occ;
    typedef uint32_t* Cst;
    typedef double* Gv;
};
template <> struct GridMem<true> {
    typedef const lds_u32* Occ;
    typedef lds_u32* Cst;
    typedef lds_f64* Gv;
};
// LDS bytes of the LDSG grid block (occupancy words, state words, G), each part 16-B aligned
__host__ __device__ constexpr size_t ldsg_occ_bytes(size_t ncell) { return (((ncell + 31) / 32) * 4 + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t ldsg_cst_words(size_t ncell) { return ((ncell + 7) / 8 + 3) & ~(size_t)3; }
__host__ __device__ constexpr size_t ldsg_bytes(size_t ncell) { return ldsg_occ_bytes(ncell) + ldsg_cst_words(ncell) * 4 + ncell * 8; }

// GZERO: GBFS (gbfs.py:73-75) -- every pushed node gets g = 0, so f = h and G is never needed.
// THETA: 1 = ThetaStar (theta_star.py:44-108), 2 = LazyThetaStar (lazy_theta_star.py:38-114); the
// parent of a node is any cell, kept per CLOSED cell in P_all (HEUR carries the Theta* layout).
template <int HEUR, bool GZERO, int THETA, bool LDSG = false>
__global__ __launch_bounds__(64) void astar2d_kernel(
    const uint32_t* __restrict__ occ, int W, int H, const int32_t* __restrict__ start_xy,
    const int32_t* __restrict__ goal_xy, const int32_t* __restrict__ order, int nq, double* __restrict__ cost_out,
    int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out, int path_cap,
    int32_t* __restrict__ nexp_out, uint32_t* __restrict__ expand_out, int expand_cap,
    int64_t* __restrict__ counters, int32_t* __restrict__ status_out, int* __restrict__ queue,
    uint4* __restrict__ spill_all, int heap_cap, int lds_cap, uint32_t* __restrict__ cst_all, size_t cst_words,
    double* __restrict__ G_all, uint32_t* __restrict__ hbits_all, size_t hbits_words, int prio_n,
    unsigned long long* __restrict__ span, uint32_t* __restrict__ P_all)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    span_begin(span);
    Heap hp;
    hp.B = (lds_u32*)smem;
    hp.F = (lds_f64*)(smem + kBitsLdsBytes);
    hp.C = (lds_u32*)(smem + kBitsLdsBytes + (size_t)8 * lds_cap);
    hp.hb = hbits_all + (size_t)worker * hbits_words;
    {
        const size_t spill_n = (size_t)(heap_cap > lds_cap ? heap_cap - lds_cap : 0);
        hp.spill = __builtin_amdgcn_make_buffer_rsrc(spill_all + (size_t)worker * spill_n, 0, (int)(spill_n * 16), 0x00020000);
    }
    hp.cap = lds_cap;
    typename GridMem<LDSG>::Occ occg;
    typename GridMem<LDSG>::Cst cst;
    typename GridMem<LDSG>::Gv G;
    if constexpr (LDSG) {
        // grid block after the heap: occupancy (copied once per worker), state words, G
        const size_t ncell = (size_t)W * (size_t)H;
        unsigned char* gb = smem + kBitsLdsBytes + (size_t)12 * lds_cap;
        lds_u32* ow = (lds_u32*)gb;
        const uint32_t nw = (uint32_t)((ncell + 31) / 32);
        for (uint32_t i = lane; i < nw; i += 64) ow[i] = occ[i];
        occg = ow;
        cst = (lds_u32*)(gb + ldsg_occ_bytes(ncell));
        G = (lds_f64*)(gb + ldsg_occ_bytes(ncell) + ldsg_cst_words(ncell) * 4);
    } else {
        occg = occ;
        cst = cst_all + (size_t)worker * cst_words;
        G = G_all + (size_t)worker * ((size_t)W * (size_t)H);
    }
    uint32_t* Pc = THETA ? P_all + (size_t)worker * ((size_t)W * (size_t)H) : nullptr;  // CLOSED parent cell

    // ---- per-lane constants
    // this lane's cell of the 3x3 block: lane i < 9 -> occupancy of (x + i/3 - 1, y + i%3 - 1),
    // lane 9 + i -> its CLOSED-state nibble, lane 18 -> G[parent]
    const int blk_i = lane < 9 ? lane : (lane < 18 ? lane - 9 : 4);
    const int blk_dx = blk_i / 3 - 1, blk_dy = blk_i % 3 - 1;
    // motion of lane m < 8: offset, cost, and the 3x3 cells isCollision needs free
    // (graph_search.py:66-87: both endpoints; for a diagonal both corner cells)
    const int mo = lane & 7;
    const int mx = mot_x(mo), my = mot_y(mo);
    const double mcost = GZERO ? 0.0 : ((mo & 1) ? kSqrt2 : 1.0);
    const int par_off = mx * H + my;  // lane d: linear offset of motion d (parent = cell - offset)
    uint32_t need = 16u | (1u << ((mx + 1) * 3 + (my + 1)));
    if (mo & 1) need |= (1u << (3 + (my + 1))) | (1u << ((mx + 1) * 3 + 1));
    const uint32_t self_bit = 1u << ((mx + 1) * 3 + (my + 1));
    // pop lane i (1..15) rewrites the bit of the path node at level i - 1
    const Lvl pop_lvl = lvl_of(lane >= 1 ? lane - 1 : 0);

    for (;;) {
        // readfirstlane (not __shfl): the compiler must SEE the query index as wave-uniform, or
        // every value derived from it (coordinates, heap size, walk state) lands in VGPRs and the
        // scalar heap walk is compiled as a divergent loop.
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = uni(order ? order[qi] : qi);
        // the longest queries (first in the longest-first order) get issue priority on their SIMD:
        // they set the launch's tail, the short ones fill the cycles they leave idle
        if (qi < prio_n) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);

        // reset this worker's cell-state array
        if constexpr (LDSG) {
            for (size_t i = lane; i < cst_words; i += 64) cst[i] = 0u;
        } else {
            uint4* c4 = reinterpret_cast<uint4*>(cst);
            const size_t n4 = cst_words / 4;
            for (size_t i = lane; i < n4; i += 64) c4[i] = make_uint4(0u, 0u, 0u, 0u);
            for (size_t i = n4 * 4 + lane; i < cst_words; i += 64) cst[i] = 0u;
        }
        wave_sync_mem();

        const int sx = uni(start_xy[2 * q]), sy = uni(start_xy[2 * q + 1]);
        const int gx = uni(goal_xy[2 * q]), gy = uni(goal_xy[2 * q + 1]);
        const bool s_in = (unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H;
        const bool g_in = (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
        if (!s_in || !g_in) {  // outside the grid: blocked -> no neighbours -> no path
            // every lane stores the same values: no lane-0-only block right before the continue
            status_out[q] = PMP_NO_PATH;
            cost_out[q] = 0.0;
            path_len_out[q] = 0;
            nexp_out[q] = s_in ? 1 : 0;
            if (counters) {
                counters[4 * q] = 1; counters[4 * q + 1] = 1; counters[4 * q + 2] = s_in ? 1 : 0; counters[4 * q + 3] = 1;
            }
            continue;
        }

        // heap[0] in registers (wave-uniform): Node(start, start, 0, 0), key (0, h = 0)
        double rootf = 0.0;
        uint32_t rootc = pack_cm<HEUR>(0, 0, 8);
        double lastf = rootf;  // heap[n - 1]
        uint32_t lastc = rootc;
        if (lane == 0) hst<true>(hp, true, 0, rootf, rootc);
        wave_sync_mem();

        int n = 1;
        int64_t npush = 1, npop = 0;
        int nexp = 0, maxn = 1;
        int st = PMP_NO_PATH;
        double goal_cost = 0.0;
        int plen = 0;

#ifdef PMP_STAMPS
        uint64_t cyc_pop = 0, cyc_wait = 0, cyc_push = 0, cyc_hbm = 0;
        const uint64_t cyc_q0 = __builtin_amdgcn_s_memtime();
#endif
        while (n > 0) {
            STAMP(ts0);
            const uint32_t ncm = rootc;
            const uint32_t v01 = hp.B[lane <= 32 ? lane : 0];  // bit words for the pop below
            npop++;
            n -= 1;
            const int ndir = cm_dir<HEUR>(ncm);
            const int x = ndir == 8 ? sx : gx - cm_dx<HEUR>(ncm);
            const int y = ndir == 8 ? sy : gy - cm_dy<HEUR>(ncm);
            const uint32_t nlin = (uint32_t)x * (uint32_t)H + (uint32_t)y;

            // ---- HBM round, issued before the LDS pop so the two overlap: one unconditional load
            //      per lane (raw word kept until after the pop, so no wait is placed before it)
            uint32_t blk_word, blk_sh;
            bool blk_in;
            {
                const int cx = x + blk_dx, cy = y + blk_dy;
                blk_in = lane < 18 && (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
                const uint32_t ci = blk_in ? (uint32_t)cx * (uint32_t)H + (uint32_t)cy : 0u;
                const auto ptr = lane < 9 ? occg + (ci >> 5) : cst + (ci >> 3);
                blk_sh = lane < 9 ? (ci & 31u) : (ci & 7u) * 4u;
                blk_word = *ptr;
            }
            double gpar = 0.0;  // G[parent] (the parent closed earlier); the start has g = 0
            uint32_t ppar = 0u;  // Theta* path 2: the pusher's CLOSED parent
            if (THETA) {
                if (ndir != 8) {
                    const uint32_t plin = nlin - (uint32_t)rl_u32((uint32_t)par_off, ndir & 7);
                    if (lane == 18) gpar = G[plin];
                    if (lane == 19 && ndir >= 16) ppar = Pc[plin];
                }
            } else if (!GZERO && ndir < 8) {
                const uint32_t plin = nlin - (uint32_t)rl_u32((uint32_t)par_off, ndir);
                if (lane == 18) gpar = G[plin];
            }
#ifdef PMP_STAMPS_SPLIT  // diagnostic: wait for the HBM round before the pop, time the two apart
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(blk_word), "v"(gpar) : "memory");
            STAMP(tsB);
            cyc_hbm += tsB - ts0;
            ts0 = tsB;
#endif

            // ---- heappop (a_star.py:54): `last` = heap[n] sifts down the CPython path
            PopOut po;
            if (n > 0) pop_any<HEUR>(hp, n, v01, lastf, lastc, rootf, rootc, pop_lvl, lane, po);

            STAMP(ts1);
            // 3x3 masks: bit k = cell (x + k/3 - 1, y + k%3 - 1); the node is k = 4
            const uint32_t occ9 = (uint32_t)ballot(lane < 9 && (!blk_in || ((blk_word >> blk_sh) & 1u))) & 0x1ffu;
            const uint32_t cls9 =
                (uint32_t)(ballot(lane >= 9 && lane < 18 && blk_in && ((blk_word >> blk_sh) & 15u) != 0u) >> 9) & 0x1ffu;
#ifdef PMP_STAMPS
            {
                STAMP(ts2);
                cyc_pop += ts1 - ts0;
                cyc_wait += ts2 - ts1;
            }
#endif
            if (cls9 & 16u) continue;  // node.current in CLOSED (a_star.py:57-58)

            // The parents of the positions this expansion's pushes can take (n .. n + 7) load in one
            // round now, under the neighbour computation below, instead of one probe round per push.
            // Valid while the 8 positions share a depth: a push that sifts up (t >= 1) rewrites only
            // the ancestors of its position, and of those only its parent is the parent of another
            // position of the batch (its right sibling's), which is refreshed below.
            const int n0 = n;
            const bool pcache = n0 > 0 && (31 - __clz(n0 + 1)) == (31 - __clz(n0 + 8));
            double pf8 = 0.0;
            uint32_t pc8 = 0u;
            Ld<true> pld;
            if (pcache) pld.issue(hp, lane < 8 ? ((n0 + lane - 1) >> 1) : 0);


            // CLOSED[node.current] = node (a_star.py:82).  The node's state word was loaded by lane 13
            // and only this wave writes it: store it back now (fire-and-forget, off the critical path).
            double gnode = (GZERO || ndir == 8) ? 0.0 : rl_f64(gpar, 18) + ((ndir & 1) ? kSqrt2 : 1.0);
            // Theta*: the node's parent (cell, coordinates, g) and its expand-record code
            uint32_t par_lin = nlin;
            int px = x, py = y, ecode = ndir;
            double gp_g = 0.0;
            if (THETA && ndir != 8) {
                const uint32_t pusher = nlin - (uint32_t)rl_u32((uint32_t)par_off, ndir & 7);
                gp_g = rl_f64(gpar, 18);
                par_lin = pusher;
                if (ndir >= 16) {  // path 2: node.g = parent.g + dist (theta_star.py:106-108)
                    par_lin = rl_u32(ppar, 19);
                    double t = 0.0;
                    if (lane == 18) t = G[par_lin];
                    gp_g = rl_f64(t, 18);
                }
                px = (int)(par_lin / (uint32_t)H);
                py = (int)(par_lin - (uint32_t)px * (uint32_t)H);
                gnode = gp_g + ((ndir >= 16) ? __dsqrt_rn((double)((x - px) * (x - px) + (y - py) * (y - py)))
                                             : ((ndir & 1) ? kSqrt2 : 1.0));
                if (THETA == 2 && !grid2d::los2d(occ, H, px, py, x, y)) {
                    // set vertex (lazy_theta_star.py:55-65): the first CLOSED, collision-free
                    // neighbour minimising its g + dist becomes the parent; g = inf if there is none
                    const bool cand = lane < 8 && (occ9 & need) == 0u && (cls9 & self_bit) != 0u;
                    double gn = 0.0;
                    if (cand) gn = G[nlin + (uint32_t)par_off];
                    const double gc = gn + mcost;
                    uint64_t cmask = ballot(cand) & 0xffull;
                    double best = __longlong_as_double(0x7ff0000000000000ll);
                    int bm = -1;
                    while (cmask) {
                        const int m = __ffsll((long long)cmask) - 1;
                        cmask &= cmask - 1;
                        const double c = rl_f64(gc, m);
                        if (best > c) { best = c; bm = m; }
                    }
                    gnode = best;
                    if (bm >= 0) {
                        gp_g = rl_f64(gn, bm);
                        px = x + mot_x(bm);
                        py = y + mot_y(bm);
                        par_lin = (uint32_t)px * (uint32_t)H + (uint32_t)py;
                        ecode = 24 + bm;
                    } else {
                        ecode |= 32;
                    }
                }
            }
            if (lane == 13) cst[nlin >> 3] = blk_word | ((uint32_t)(THETA ? 1 : ndir + 1) << blk_sh);
            if (!GZERO && lane == 14) G[nlin] = gnode;
            if (THETA && lane == 15) Pc[nlin] = par_lin;
            if (lane == 0 && expand_out && nexp < expand_cap)
                expand_out[(size_t)q * expand_cap + nexp] = THETA ? (nlin | ((uint32_t)ecode << 26)) : (nlin | ((uint32_t)ndir << 28));
            nexp++;

            if (x == gx && y == gy) {  // goal found (a_star.py:61-64)
                st = PMP_FOUND;
                wave_sync_mem();
                if (THETA && lane == 0) {  // extractPath via the CLOSED parents (any cell), hypot per hop
                    uint32_t li = nlin;
                    int cx = x, cy = y;
                    double cost = 0.0;
                    int len = 0;
                    uint32_t* pth = path_out + (size_t)q * path_cap;
                    for (;;) {
                        if (len < path_cap) pth[len] = li;
                        len++;
                        if (cx == sx && cy == sy) break;
                        const uint32_t pl = Pc[li];
                        const int qx = (int)(pl / (uint32_t)H), qy = (int)(pl - (uint32_t)qx * (uint32_t)H);
                        cost += __dsqrt_rn((double)((cx - qx) * (cx - qx) + (cy - qy) * (cy - qy)));
                        cx = qx;
                        cy = qy;
                        li = pl;
                    }
                    goal_cost = cost;
                    plen = len;
                } else if (lane == 0) {  // extractPath (a_star.py:98-117): goal -> start, cost in that order
                    int cx = x, cy = y;
                    double cost = 0.0;
                    int len = 0;
                    uint32_t* pth = path_out + (size_t)q * path_cap;
                    for (;;) {
                        const uint32_t li = (uint32_t)cx * (uint32_t)H + (uint32_t)cy;
                        if (len < path_cap) pth[len] = li;
                        len++;
                        if (cx == sx && cy == sy) break;
                        const int d = (int)cst_at(cst, li) - 1;
                        cost += (d & 1) ? kSqrt2 : 1.0;
                        cx -= mot_x(d);
                        cy -= mot_y(d);
                    }
                    goal_cost = cost;
                    plen = len;
                }
                break;
            }

            // ---- getNeighbor + the push loop in motion order; push the goal and stop (a_star.py:66-80)
            const int ndx = gx - x - mx, ndy = gy - y - my;  // goal - neighbour of lane m
            const bool nb_ok = lane < 8 && (occ9 & need) == 0u && (cls9 & self_bit) == 0u;
            uint64_t vm = ballot(nb_ok) & 0xffull;
            const uint64_t gm = ballot(nb_ok && ndx == 0 && ndy == 0) & 0xffull;
            if (gm) vm &= (gm << 1) - 1;
            // Node + motion (node.py:39-41), h = GraphSearcher.h (graph_search.py:41-44)
            double ig = gnode + mcost;
            int icode = mo;
            if (THETA && ndir != 8) {
                // updateVertex(CLOSED[node.parent], node_n) (theta_star.py:96-108; lazy_theta_star.py:
                // 103-114 without the line of sight): path 2 when parent.g + dist <= node_n.g
                const int nxl = x + mx, nyl = y + my;
                const double g2 =
                    gp_g + __dsqrt_rn((double)((px - nxl) * (px - nxl) + (py - nyl) * (py - nyl)));
                if (lane < 8 && (vm >> lane & 1ull) && g2 <= ig && (THETA == 2 || grid2d::los2d(occ, H, nxl, nyl, px, py))) {
                    ig = g2;
                    icode = 16 + mo;
                }
            }
            const uint32_t icm = pack_cm<HEUR>(ndx, ndy, icode);
            const uint32_t ik = hkey<HEUR>(icm);
            const double ifv = ig + h_of_key<HEUR>(ik);
            bool overflow = false;
            if (pcache) pld.get(pf8, pc8);
            while (vm) {
                const int m = __ffsll((long long)vm) - 1;
                vm &= vm - 1;
                if (n >= heap_cap) { overflow = true; break; }
                const double itf = rl_f64(ifv, m);
                const uint32_t itc = rl_u32(icm, m), itk = rl_u32(ik, m);
                // CPython's _siftdown stops at once when the item is not less than its parent (73 % of
                // C2's pushes): compare with the parent first, and run the full push only when it moves
                double pf;
                uint32_t pc;
                if (pcache) {
                    pf = rl_f64(pf8, n - n0);
                    pc = rl_u32(pc8, n - n0);
                } else {
                    hld<true>(hp, n > 0 ? (n - 1) >> 1 : 0, pf, pc);
                    pf = rl_f64(pf, 0);
                    pc = rl_u32(pc, 0);
                }
                if (n > 0 && !key_lt(itf, itk, pf, hkey<HEUR>(pc))) {
                    // t = 0: heap[n] = item; a right child (n even) sets its parent's bit against its
                    // left sibling heap[n - 1] = last
                    if ((n & 1) == 0)
                        bit_write1(hp, lane, lvl_of(30 - __clz(n + 1)), ((uint32_t)n + 1u) >> 1,
                                   !key_lt(lastf, hkey<HEUR>(lastc), itf, itk));
                    hst<true>(hp, lane == 0, n, itf, itc);
                    lastf = itf;
                    lastc = itc;
                    wave_sync_mem();
                } else {
                    int t;
                    double a1f;
                    uint32_t a1c;
                    push_any<HEUR>(hp, n, itf, itc, itk, lastf, lastc, rootf, rootc, lane, t, a1f, a1c);
                    // a left child's right sibling (the next position) has the same parent, now a1
                    if (pcache && (n & 1) && lane == n - n0 + 1) {
                        pf8 = a1f;
                        pc8 = a1c;
                    }
                }
                n += 1;
                npush++;
            }
            if (n > maxn) maxn = n;
#ifdef PMP_STAMPS
            {
                STAMP(ts3);
                cyc_push += ts3 - ts1;
            }
#endif
            if (overflow) { st = PMP_CAP_OVERFLOW; break; }
        }

        if (lane == 0) {
            int s = st;
            if (s == PMP_FOUND && plen > path_cap) s = PMP_PATH_OVERFLOW;
            status_out[q] = s;
            cost_out[q] = (st == PMP_FOUND) ? goal_cost : 0.0;
            path_len_out[q] = (st == PMP_FOUND) ? plen : 0;
            nexp_out[q] = nexp;
            if (counters) {
#ifdef PMP_STAMPS
                counters[4 * q + 0] = (int64_t)cyc_pop;
#ifdef PMP_STAMPS_SPLIT
                counters[4 * q + 1] = (int64_t)cyc_hbm;
#else
                counters[4 * q + 1] = (int64_t)cyc_wait;
#endif
                counters[4 * q + 2] = (int64_t)cyc_push;
                counters[4 * q + 3] = (int64_t)(__builtin_amdgcn_s_memtime() - cyc_q0);
#else
                counters[4 * q + 0] = npush;
                counters[4 * q + 1] = npop;
                counters[4 * q + 2] = nexp;
                counters[4 * q + 3] = maxn;
#endif
            }
        }
        wave_sync_mem();
    }
    span_end(span);
}

// ---- longest-first schedule: counting sort of the queries by descending start-goal distance ----
__device__ __forceinline__ int lpt_key(const int32_t* s, const int32_t* g, int q)
{
    const double dx = (double)s[2 * q] - g[2 * q], dy = (double)s[2 * q + 1] - g[2 * q + 1];
    const double d = __dsqrt_rn(dx * dx + dy * dy);  // expansions grow ~ with distance^2
    return d < 2147483647.0 ? (int)d : 2147483647;  // callers clamp to the histogram's last bin
}

__global__ void lpt_hist(const int32_t* s, const int32_t* g, int nq, int nb, int* hist)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) atomicAdd(&hist[min(lpt_key(s, g, q), nb - 1)], 1);
}

// offsets[k] = number of queries with a larger key (descending order); one thread, nb <= 16384
__global__ void lpt_scan(int nb, int* hist)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int run = 0;
    for (int k = nb - 1; k >= 0; k--) {
        const int c = hist[k];
        hist[k] = run;
        run += c;
    }
}

__global__ void lpt_scatter(const int32_t* s, const int32_t* g, int nq, int nb, int* offs, int32_t* order)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) order[atomicAdd(&offs[min(lpt_key(s, g, q), nb - 1)], 1)] = q;
}

int default_workers() { return 256 * 4; }
int default_lds_cap(int workers_per_cu)
{
    // 160 KiB LDS per CU shared by the resident workers: the direction-bit blocks, then 12 B per
    // heap entry; keep a little slack (< 16: the share is too small, the caller refuses)
    int bytes = (160 * 1024) / workers_per_cu - 256 - kBitsLdsBytes;
    return bytes < 16 * 12 ? 0 : (bytes / 12) & ~15;
}
// HBM words of the direction-bit tiers >= 3 for heaps of up to heap_cap entries
size_t hbits_words(int heap_cap)
{
    const int maxlvl = 31 - __builtin_clz((unsigned)heap_cap);
    size_t w = 0;
    for (int t = 3; 5 * t <= maxlvl; t++) w += (size_t)1 << (5 * t);
    return w ? w : 1;
}
// The heap never holds more than 8 * expansions + 1 <= 8 W H + 1 entries; the default cap is far
// below that bound (C2's largest heap is ~10k entries).  A query that outgrows its cap stops with
// PMP_CAP_OVERFLOW and the host re-runs it with a larger reservation (batch.astar2d_batch).
size_t max_heap(int W, int H) { return 8 * (size_t)W * H + 8; }
int default_heap_cap(int W, int H)
{
    const size_t c = max_heap(W, H);
    return (int)(c < (size_t)(1 << 16) ? c : (size_t)(1 << 16));
}
// per-context scratch budget: workers are reduced to fit (heap spill + cell state + G per worker)
constexpr size_t kScratchBudget = (size_t)64 << 30;

// longest-first order of a batch in the context's SCR_PDIR scratch (counting sort, descending
// start-goal distance)
int lpt_order2d(pmp_ctx* ctx, hipStream_t s, const int32_t* start_xy, const int32_t* goal_xy, int nq, int W, int H,
                int32_t** order)
{
    const int nb = (int)ceil(sqrt((double)W * W + (double)H * H)) + 1;
    int* hist = (int*)pmp_scratch(ctx, SCR_PDIR, sizeof(int) * ((size_t)nb + (size_t)nq));
    if (!hist) return PMP_ENOMEM;
    *order = hist + nb;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(hist, 0, sizeof(int) * (size_t)nb, s));
    hipLaunchKernelGGL(lpt_hist, dim3((nq + 255) / 256), dim3(256), 0, s, start_xy, goal_xy, nq, nb, hist);
    hipLaunchKernelGGL(lpt_scan, dim3(1), dim3(64), 0, s, nb, hist);
    hipLaunchKernelGGL(lpt_scatter, dim3((nq + 255) / 256), dim3(256), 0, s, start_xy, goal_xy, nq, nb, hist, *order);
    return PMP_OK;
}

}  // namespace

// The multi-query engine (astar2d_mq.hip) serves A* / Dijkstra / GBFS when the context selects it
// and the reserved heap capacity fits its limit (a query that outgrows it is re-run by the host with
// the full bound, which selects this file's engine).
static int astar2d_reserve_impl(pmp_ctx* ctx, int W, int H, int workers, int heap_cap)
{
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim || workers < 1)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_reserve: bad dims/workers");
    const int mq_cap = pmp_astar2d_mq_cap(ctx->astar_mq_t2lds != 0);
    const bool dflt = heap_cap <= 0;
    if (dflt) heap_cap = default_heap_cap(W, H);
    if ((size_t)heap_cap > max_heap(W, H)) heap_cap = (int)max_heap(W, H);
    // the default capacity on the multi-query engine is its limit; a capacity the host asked for (an
    // explicit one, or the full bound of an overflow re-run) is kept and, above that limit, reserves
    // the one-query-per-wave engine instead
    ctx->astar_heap_cap_wave = heap_cap;  // small batches on a multi-query reservation (pmp_graph2d_batch)
    ctx->astar_cap_explicit = dflt ? 0 : 1;
    if (ctx->astar_engine >= 1 && dflt && heap_cap > mq_cap) heap_cap = mq_cap;
    if (ctx->astar_engine >= 1 && heap_cap <= mq_cap) {
        // workers = queries in flight (16-lane groups, 4 per wave); scratch is taken at launch
        const size_t per_slot = (size_t)W * H + g_slot_cells(W, H) * 8 + (size_t)mq_cap * 16 + 4096 + 256;
        const size_t fit = kScratchBudgetMq / per_slot;
        if (fit < 4) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_astar2d_reserve: one wave exceeds the scratch budget");
        if ((size_t)workers > fit) workers = (int)(fit & ~(size_t)3);
        const int per_cu = ctx->astar_resident_per_cu > 0 ? ctx->astar_resident_per_cu : (workers + 255) / 256;
        int lds_cap = pmp_astar2d_mq_lds_cap(per_cu, ctx->astar_mq_t2lds != 0);
        if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
        if (lds_cap < 16)
            return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_reserve: residency leaves no LDS heap share");
        if (!pmp_scratch(ctx, SCR_AUX0, 256)) return PMP_ENOMEM;
        ctx->astar_W = W;
        ctx->astar_H = H;
        ctx->astar_workers = workers;
        ctx->astar_heap_cap = heap_cap;
        ctx->astar_lds_cap = lds_cap;
        ctx->astar_reserved_mq = 1;
        return PMP_OK;
    }
    ctx->astar_reserved_mq = 0;
    const size_t ncell = (size_t)W * H;
    const size_t cst_words = ((ncell + 7) / 8 + 3) & ~(size_t)3;
    {
        const size_t per_worker = (size_t)heap_cap * 16 + cst_words * 4 + ncell * 8 + hbits_words(heap_cap) * 4;
        const size_t fit = kScratchBudget / per_worker;
        if (fit < 1) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_astar2d_reserve: one worker exceeds the scratch budget");
        if ((size_t)workers > fit) workers = (int)fit;
    }
    const int per_cu = ctx->astar_resident_per_cu > 0 ? ctx->astar_resident_per_cu : (workers + 255) / 256;
    int lds_cap = default_lds_cap(per_cu < 1 ? 1 : per_cu);
    if (lds_cap < 16)  // the share cannot hold the bit blocks and a minimal heap: refuse, never wrap
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_reserve: residency leaves no LDS heap share (one query per wave)");
    if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    const size_t spill = heap_cap > lds_cap ? (size_t)(heap_cap - lds_cap) : 0;
    if (!pmp_scratch(ctx, SCR_HEAP, (size_t)workers * spill * 16 + 16)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_CLOSED, (size_t)workers * cst_words * 4)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_AUX0, 256)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_G, (size_t)workers * ncell * 8)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_BITS, (size_t)workers * hbits_words(heap_cap) * 4)) return PMP_ENOMEM;
    ctx->astar_W = W;
    ctx->astar_H = H;
    ctx->astar_workers = workers;
    ctx->astar_heap_cap = heap_cap;
    ctx->astar_lds_cap = lds_cap;
    return PMP_OK;
}

extern "C" int pmp_astar2d_reserve(pmp_ctx* ctx, int W, int H, int workers, int heap_cap)
{
    if (!ctx) return PMP_EINVAL;
    const int rc = astar2d_reserve_impl(ctx, W, H, workers, heap_cap);
    if (rc == PMP_OK) ctx->astar_auto = 0;  // the host's own geometry: launches keep it
    return rc;
}

extern "C" int pmp_astar2d_geometry(pmp_ctx* ctx, int32_t* out6)
{
    if (!ctx || !out6) return PMP_EINVAL;
    out6[0] = ctx->astar_W;
    out6[1] = ctx->astar_H;
    out6[2] = ctx->astar_workers;
    out6[3] = ctx->astar_heap_cap;
    out6[4] = (ctx->astar_reserved_mq ? 1 : 0) | (ctx->astar_cap_explicit ? 2 : 0);
    out6[5] = ctx->astar_auto;
    return PMP_OK;
}

extern "C" int pmp_astar2d_reserve_auto(pmp_ctx* ctx)
{
    if (!ctx) return PMP_EINVAL;
    ctx->astar_W = ctx->astar_H = 0;  // the next launch reserves for its batch (pmp_graph2d_batch)
    ctx->astar_auto = 1;
    return PMP_OK;
}

extern "C" int pmp_astar2d_set_engine(pmp_ctx* ctx, int engine, int t2_lds)
{
    if (!ctx) return PMP_EINVAL;
    if (engine < 0 || engine > 3)
        return pmp_set_err(ctx, PMP_EINVAL,
                           "pmp_astar2d_set_engine: engine must be 0 (one query per wave), 1 (multi-query for large "
                           "batches, single-query for small ones), 2 (multi-query always) or 3 (single-query always)");
    ctx->astar_engine = engine;
    ctx->astar_mq_t2lds = t2_lds ? 1 : 0;
    if (ctx->astar_W == 0) return PMP_OK;
    return astar2d_reserve_impl(ctx, ctx->astar_W, ctx->astar_H, ctx->astar_workers, 0);
}

extern "C" int pmp_astar2d_set_residency(pmp_ctx* ctx, int per_cu)
{
    if (!ctx) return PMP_EINVAL;
    // queries resident per CU: at most 32 one-query waves, or 128 queries of 32 four-query waves
    if (per_cu < 0 || per_cu > 128)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_set_residency: per_cu must be in [0, 128]");
    ctx->astar_resident_per_cu = per_cu;
    if (ctx->astar_W == 0) return PMP_OK;  // applied by the next reserve
    return astar2d_reserve_impl(ctx, ctx->astar_W, ctx->astar_H, ctx->astar_workers, ctx->astar_heap_cap);
}

namespace {
// Batches below this size run on the one-query-per-wave engine even on a multi-query context: with
// fewer queries than the chip has waves, a query's own latency sets the launch time, and a wave
// serves one query faster than a quarter of one.
constexpr int kMqMinBatch = 1024;
// Batches up to this size run on the single-query engine (one query per workgroup with a CU's LDS)
// when it holds the heap: fewer queries than CUs, so each query's latency is the launch time.
constexpr int kSqMaxBatch = 256;
// The LDSG variant needs at least this many heap positions in LDS beside the grid block.
constexpr int kLdsgMinHeap = 64;
}  // namespace

extern "C" int pmp_graph2d_batch(pmp_ctx* ctx, void* stream, int algo, const uint32_t* occ_bits, int W, int H,
                                 int heuristic, const int32_t* start_xy, const int32_t* goal_xy, int nq,
                                 double* cost, int32_t* path_len, uint32_t* path, int path_cap,
                                 int32_t* n_expanded, uint32_t* expand, int expand_cap, int64_t* counters,
                                 int32_t* status)
{
    if (!ctx) return PMP_EINVAL;
    if (algo < PMP_ALGO_ASTAR || algo > PMP_ALGO_LAZY_THETA)
        return pmp_set_err(ctx, PMP_EINVAL,
                           "pmp_graph2d_batch: algo must be 0 (AStar), 1 (Dijkstra), 2 (GBFS), 3 (ThetaStar) or 4 (LazyThetaStar)");
    const bool theta = algo == PMP_ALGO_THETA || algo == PMP_ALGO_LAZY_THETA;
    if (theta && H > 4096)  // the Theta* entry layout keeps a 13-bit dy (and expand records 26-bit cells)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_graph2d_batch: ThetaStar / LazyThetaStar need H <= 4096");
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: W and H must be in [1, 8192]");
    if (heuristic != 0 && heuristic != 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: heuristic must be 0 or 1");
    if (nq < 0 || path_cap < 1 || (expand && expand_cap < 1))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: bad nq/path_cap/expand_cap");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xy || !goal_xy || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    {
        // a geometry made here (not by the host's pmp_astar2d_reserve) follows the batches: sized to
        // the first batch, it grows when a larger one arrives
        const int auto_w = ctx->astar_engine >= 1 ? 4 * default_workers() : default_workers();
        const bool grow = ctx->astar_auto && ctx->astar_workers < nq && ctx->astar_workers < auto_w;
        if (!(ctx->astar_W == W && ctx->astar_H == H) || grow) {
            const int rc = astar2d_reserve_impl(ctx, W, H, nq < auto_w ? nq : auto_w, 0);
            if (rc) return rc;
            ctx->astar_auto = 1;
        }
    }
    const size_t ncell = (size_t)W * H;
    const size_t cst_words = ((ncell + 7) / 8 + 3) & ~(size_t)3;
    // one-query-per-wave launch geometry: the reservation's, or on a multi-query reservation this
    // engine's defaults for the batch (with the heap capacity asked for, or this engine's default: not the multi-query limit)
    int heap_cap = ctx->astar_heap_cap;
    int workers, per_cu, lds_cap;
    if (!ctx->astar_reserved_mq) {
        workers = ctx->astar_workers < nq ? ctx->astar_workers : nq;
        per_cu = ctx->astar_resident_per_cu > 0 ? ctx->astar_resident_per_cu : (ctx->astar_workers + 255) / 256;
        lds_cap = ctx->astar_lds_cap;
    } else {
        heap_cap = ctx->astar_heap_cap_wave;
        workers = default_workers() < nq ? default_workers() : nq;
        per_cu = ctx->astar_resident_per_cu > 0 ? ctx->astar_resident_per_cu : (workers + 255) / 256;
        if (per_cu > 32) per_cu = 32;
        lds_cap = default_lds_cap(per_cu);
        if (lds_cap < 16)
            return pmp_set_err(ctx, PMP_EINVAL, "pmp_graph2d_batch: residency leaves no LDS heap share (one query per wave)");
        if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    }
    // small grids: the grid block in LDS when the share holds it beside a useful heap
    bool ldsg = false;
    if (!theta) {
        const long long share = (long long)(160 * 1024) / (per_cu < 1 ? 1 : per_cu) - 256;
        long long cap_g = (share - kBitsLdsBytes - (long long)ldsg_bytes(ncell)) / 12;
        cap_g &= ~15ll;
        if (cap_g >= kLdsgMinHeap) {
            ldsg = true;
            lds_cap = cap_g > heap_cap ? (heap_cap + 15) & ~15 : (int)cap_g;
        }
    }
    if (!theta && (ctx->astar_engine == 3 || (ctx->astar_engine == 1 && nq <= kSqMaxBatch))) {
        // the single-query engine, when its LDS holds the heap capacity asked for (the default
        // capacity is cut to what it holds: a query that outgrows it reports PMP_CAP_OVERFLOW and the
        // host re-runs it with the full bound, which lands on this file's engine)
        const int sq_cap = pmp_astar2d_sq_cap(W, H);
        const int want = ctx->astar_reserved_mq ? ctx->astar_heap_cap_wave : ctx->astar_heap_cap;
        // one query slot (cell states + G, unless the grid sits in LDS) per query of the batch
        const bool fits = (size_t)nq * (ncell * 9 + 256) <= kScratchBudgetMq;
        if (sq_cap > 0 && fits && (!ctx->astar_cap_explicit || want <= sq_cap))
            return pmp_astar2d_sq_launch(ctx, (hipStream_t)stream, algo, occ_bits, W, H, heuristic, start_xy, goal_xy, nq,
                                         want < sq_cap ? want : sq_cap, cost, path_len, path, path_cap, n_expanded,
                                         expand, expand_cap, counters, status);
    }
    // the multi-query engine (A* / Dijkstra / GBFS, and Theta* / Lazy Theta* since round 5)
    if (ctx->astar_reserved_mq && (ctx->astar_engine == 2 || (!ldsg && nq >= kMqMinBatch))) {
        const int groups = ctx->astar_workers < nq ? ctx->astar_workers : nq;
        int* queue = (int*)ctx->buf[SCR_AUX0];
        hipStream_t s = (hipStream_t)stream;
        PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
        int32_t* order = nullptr;
        if (ctx->astar_lpt && nq > groups) {
            const int rc = lpt_order2d(ctx, s, start_xy, goal_xy, nq, W, H, &order);
            if (rc) return rc;
        }
        return pmp_astar2d_mq_launch(ctx, s, algo, occ_bits, W, H, heuristic, start_xy, goal_xy, order, nq, cost,
                                     path_len, path, path_cap, n_expanded, expand, expand_cap, counters, status, queue);
    }
    // this engine's scratch for the launch (grow-only: no-ops on its own reservation)
    const size_t spill = heap_cap > lds_cap ? (size_t)(heap_cap - lds_cap) : 0;
    if (!pmp_scratch(ctx, SCR_HEAP, (size_t)workers * spill * 16 + 16)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_BITS, (size_t)workers * hbits_words(heap_cap) * 4)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_AUX0, 256)) return PMP_ENOMEM;
    uint32_t* cst = nullptr;
    double* G = nullptr;
    if (!ldsg) {
        cst = (uint32_t*)pmp_scratch(ctx, SCR_CLOSED, (size_t)workers * cst_words * 4);
        G = (double*)pmp_scratch(ctx, SCR_G, (size_t)workers * ncell * 8);
        if (!cst || !G) return PMP_ENOMEM;
    }
    uint4* spill_p = (uint4*)ctx->buf[SCR_HEAP];
    int* queue = (int*)ctx->buf[SCR_AUX0];
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)kBitsLdsBytes + (size_t)lds_cap * 12 + (ldsg ? ldsg_bytes(ncell) : 0);
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    int32_t* order = nullptr;
    if (ctx->astar_lpt && nq > workers) {
        const int rc = lpt_order2d(ctx, s, start_xy, goal_xy, nq, W, H, &order);
        if (rc) return rc;
    }
    uint32_t* par = nullptr;
    if (theta) {
        par = (uint32_t*)pmp_scratch(ctx, SCR_PAR, (size_t)workers * ncell * 4);
        if (!par) return PMP_ENOMEM;
    }
    constexpr int TL = kThetaLayout;
    auto kern = algo == PMP_ALGO_DIJKSTRA ? astar2d_kernel<2, false, 0>
              : algo == PMP_ALGO_GBFS     ? (heuristic == 1 ? astar2d_kernel<1, true, 0> : astar2d_kernel<0, true, 0>)
              : algo == PMP_ALGO_THETA    ? (heuristic == 1 ? astar2d_kernel<TL | 1, false, 1> : astar2d_kernel<TL, false, 1>)
              : algo == PMP_ALGO_LAZY_THETA ? (heuristic == 1 ? astar2d_kernel<TL | 1, false, 2> : astar2d_kernel<TL, false, 2>)
                                          : (heuristic == 1 ? astar2d_kernel<1, false, 0> : astar2d_kernel<0, false, 0>);
    if (ldsg)
        kern = algo == PMP_ALGO_DIJKSTRA ? astar2d_kernel<2, false, 0, true>
             : algo == PMP_ALGO_GBFS     ? (heuristic == 1 ? astar2d_kernel<1, true, 0, true> : astar2d_kernel<0, true, 0, true>)
                                         : (heuristic == 1 ? astar2d_kernel<1, false, 0, true> : astar2d_kernel<0, false, 0, true>);
    hipLaunchKernelGGL(kern, dim3(workers), dim3(64), lds, s, occ_bits, W, H, start_xy,
                       goal_xy, (const int32_t*)order, nq, cost, path_len, path, path_cap, n_expanded, expand,
                       expand_cap, counters, status, queue, spill_p, heap_cap, lds_cap, cst, cst_words, G,
                       (uint32_t*)ctx->buf[SCR_BITS], hbits_words(heap_cap), order ? ctx->astar_prio_n : 0, ctx->span,
                       par);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

extern "C" int pmp_astar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                                 int heuristic, const int32_t* start_xy, const int32_t* goal_xy, int nq,
                                 double* cost, int32_t* path_len, uint32_t* path, int path_cap,
                                 int32_t* n_expanded, uint32_t* expand, int expand_cap, int64_t* counters,
                                 int32_t* status)
{
    return pmp_graph2d_batch(ctx, stream, PMP_ALGO_ASTAR, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, cost,
                             path_len, path, path_cap, n_expanded, expand, expand_cap, counters, status);
}
