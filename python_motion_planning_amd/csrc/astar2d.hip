// Batched 2D A* for gfx950, bit-exact with the reference AStar.plan
// (global_planner/graph_search/a_star.py:39-83) including CPython heapq's tie behaviour
// (Lib/heapq.py heappush/_siftdown, heappop/_siftup) under Node.__lt__ (utils/environment/node.py:51-54).
//
// Execution model: persistent workers, one wave64 each, pull query indices from an atomic queue.
// A worker keeps the query's whole CPython heap array in LDS (positions >= lds_cap spill to a
// per-worker HBM array) and a 4-bit-per-cell state array in HBM (0 = open, dir+1 = closed with
// parent motion `dir`), reused across the queries it processes.
//
// Heap entry (12 B in LDS as SoA: f64 f[] | u32 cm[]):  cm = (x << 13 | y) << 4 | dir
//   dir = motion index (env.py:52-55) that reached the cell from its parent, 8 = start.
//   f = g + h as Node.__lt__ computes it (euclidean h = hypot(dx, dy) == sqrt(d2) exactly for
//   |d| <= 16384, pinned against CPython's vector_norm; manhattan h = |dx| + |dy|).
//   Node.__lt__: f < f' or (f == f' and h < h'); h order == hkey order (d2, or |dx|+|dy|), and hkey
//   is rebuilt from the cell with integer ops, so loading an entry costs no transcendental.
//   g of a popped node = G[parent] + motion cost (node.py:39-41), G written when the parent closed,
//   loaded in the same HBM round as the node's 3x3 occupancy / CLOSED block.
//
// heappop (CPython: pop last, put it at the root, _siftup walks the smaller child -- right child
// when not left < right -- to a leaf, then _siftdown moves it back up).  The final array equals a
// top-down walk along that same child path that moves each chosen child up while
// !(last < child) and drops `last` at the first child it is less than (the path is sorted, so the
// "not less" set is a prefix).  A chunk = 6 levels below the hole: lane l < 63 loads one sibling
// pair, decides the CPython child choice and the two "may move up" bits; three ballots give the
// masks; the walk itself is scalar; movers store in parallel.
// heappush (_siftdown): the ancestors load in one round, one ballot finds how many move down.
#include "pmp_internal.h"

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

__device__ __constant__ int c_mx[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
__device__ __constant__ int c_my[8] = {0, 1, 1, 1, 0, -1, -1, -1};

struct Q {  // per-query wave-uniform constants
    int gx, gy;
};

struct Ent {
    double f;
    uint32_t cm, hk;
};

// HEUR: 0 euclidean, 1 manhattan (GraphSearcher.h, graph_search.py:41-44) -- a template parameter,
// so key computations carry no runtime branch.
template <int HEUR>
__device__ __forceinline__ uint32_t hkey_raw(const Q& q, uint32_t cm)
{
    const int x = (int)(cm >> 17), y = (int)((cm >> 4) & 8191u);
    const int dx = q.gx - x, dy = q.gy - y;
    return HEUR == 1 ? (uint32_t)(abs(dx) + abs(dy)) : (uint32_t)(dx * dx + dy * dy);
}

// h of a pushed node and its integer order key
template <int HEUR>
__device__ __forceinline__ double h_and_key(const Q& q, uint32_t cm, uint32_t& hk)
{
    hk = hkey_raw<HEUR>(q, cm);
    return HEUR == 1 ? (double)hk : __dsqrt_rn((double)hk);
}

// order key of a stored entry; the start node has h = 0 (planner.py:15)
template <int HEUR>
__device__ __forceinline__ uint32_t key_of(const Q& q, uint32_t cm)
{
    const uint32_t k = hkey_raw<HEUR>(q, cm);
    return (cm & 15u) == 8u ? 0u : k;
}

// Node.__lt__ (node.py:51-54) -- evaluated without short-circuit branches
__device__ __forceinline__ bool key_lt(double fa, uint32_t ka, double fb, uint32_t kb)
{
    return (fa < fb) | ((fa == fb) & (ka < kb));
}
__device__ __forceinline__ bool ent_lt(const Ent& a, const Ent& b) { return key_lt(a.f, a.hk, b.f, b.hk); }

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// The CPython heap array: positions < lds_cap in LDS (explicit address space 3, so every access is
// a ds_read/ds_write), positions >= lds_cap in a per-worker HBM spill reached only through buffer
// instructions (a distinct instruction class, so the compiler can never fold the two paths into
// one flat access that waits on both counters).
//
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

struct Heap {
    lds_f64* lg;       // LDS f[lds_cap]
    lds_u32* lcm;      // LDS cm[lds_cap]
    lds_u32* lb;       // LDS direction-bit blocks of tiers 0..2
    uint32_t* hb;      // HBM direction-bit blocks of tiers >= 3
    __amdgpu_buffer_rsrc_t spill;  // HBM entries {f lo, f hi, cm, 0} for positions >= lds_cap
    int lds_cap;

    __device__ __forceinline__ void load(int p, double& g, uint32_t& cm) const
    {
        if (p < lds_cap) {
            g = lg[p];
            cm = lcm[p];
        } else {
            const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(spill, (p - lds_cap) * 16, 0, 0));
            g = __hiloint2double((int)v.y, (int)v.x);
            cm = v.z;
        }
    }
    __device__ __forceinline__ void store(int p, double g, uint32_t cm) const
    {
        if (p < lds_cap) {
            lg[p] = g;
            lcm[p] = cm;
        } else {
            const uint64_t b = (uint64_t)__double_as_longlong(g);
            const uint4 v = make_uint4((uint32_t)b, (uint32_t)(b >> 32), cm, 0u);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                                   spill, (p - lds_cap) * 16, 0, 0);
        }
    }
};

// HBM word of tier t >= 3 for the block whose root has path number R (= root position + 1):
// tier t starts after sum_{s=3}^{t-1} 32^s = (32^t - 32^3) / 31 words
__device__ __forceinline__ size_t hb_word(int t, uint32_t R)
{
    const size_t base = (size_t)1 << (5 * t);
    return (base - 32768u) / 31u + (size_t)(R - (uint32_t)base);
}

// Set the direction bit of the node at `level` whose path number (position + 1) is Pl.  Lanes may
// share a block word, so the update is an atomic and/or (no return value: nothing waits on it).
__device__ __forceinline__ void bit_write(const Heap& hp, int level, uint32_t Pl, uint32_t bit)
{
    const int t = level / 5, r = level - 5 * t;
    const uint32_t R = Pl >> r;
    const uint32_t m = 1u << ((1u << r) - 1u + (Pl & ((1u << r) - 1u)));
    if (t <= 2) {
        lds_u32* w = hp.lb + (t == 0 ? 0u : (t == 1 ? R - 31u : R - 991u));
        if (bit) __atomic_fetch_or(w, m, __ATOMIC_RELAXED);
        else __atomic_fetch_and(w, ~m, __ATOMIC_RELAXED);
    } else {
        uint32_t* w = hp.hb + hb_word(t, R);
        if (bit) __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_and(w, ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// 4-bit cell state: word i >> 3, nibble i & 7
__device__ __forceinline__ uint32_t cst_at(const uint32_t* cst, uint32_t i) { return (cst[i >> 3] >> ((i & 7) * 4)) & 15u; }

__device__ __forceinline__ void wave_sync_mem()
{
    // Orders this wave's LDS and HBM accesses across its lanes.  A wave's memory operations are
    // performed in order, so wavefront scope needs no s_waitcnt (LLVM AMDGPU memory model): this
    // is a compiler barrier only and never stalls on outstanding HBM stores.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// SPILL = false: every position touched is < lds_cap (pure ds_read/ds_write code, no vmcnt waits).
template <bool SPILL>
__device__ __forceinline__ void hload(const Heap& hp, int p, double& g, uint32_t& cm)
{
    if constexpr (SPILL) {
        hp.load(p, g, cm);
    } else {
        g = hp.lg[p];
        cm = hp.lcm[p];
    }
}
template <bool SPILL>
__device__ __forceinline__ void hstore(const Heap& hp, int p, double g, uint32_t cm)
{
    if constexpr (SPILL) {
        hp.store(p, g, cm);
    } else {
        hp.lg[p] = g;
        hp.lcm[p] = cm;
    }
}
// predicated load: SPILL lanes branch (a buffer load only where needed), LDS-only code loads a
// clamped valid address unconditionally
template <bool SPILL>
__device__ __forceinline__ void hload_if(const Heap& hp, bool v, int p, double& g, uint32_t& cm)
{
    if constexpr (SPILL) {
        g = 0.0;
        cm = 0u;
        if (v) hp.load(p, g, cm);
    } else {
        hload<false>(hp, v ? p : 0, g, cm);
    }
}

// heappop on a heap of n (> 0, already decremented) entries whose old last element sits at
// position n; the old root has been taken by the caller.  Updates `root` (wave-uniform heap[0]).
//  1. the _siftup path p_0 = 0, p_1, .., p_K (a leaf) from the direction bits: a scalar walk over
//     prefetched block words (tiers 0/1 in one LDS round, the 32 tier-2 candidates below p_5 in a
//     second round that overlaps the tier-1 walk);
//  2. one round: lane i in 1..K loads heap[p_i], heap[p_{i+1}] and heap[sibling(p_i)];
//  3. the children that move up are the prefix with !(last < heap[p_i]) (the path is sorted), so a
//     ballot popcount m places `last` at p_m -- the array CPython's _siftup + _siftdown produce;
//  4. lanes 1..m rewrite the bits of p_0..p_{m-1}, whose children changed.
template <bool SPILL, int HEUR>
__device__ __forceinline__ void heap_pop(const Heap& hp, const Q& qc, int n, Ent& root, int lane)
{
    n = uni(n);  // wave-uniform by construction; say so, so the walk below stays on the SALU
    Ent last;
    hload<SPILL>(hp, n, last.f, last.cm);  // uniform address, but an LDS load is not known-uniform:
    const uint32_t v01 = hp.lb[lane <= 32 ? lane : 0];  // tier-0 word (lane 0), tier-1 words (1..32)
    last.f = rl_f64(last.f, 0);            // readlane makes `last` (and the root / node derived from
    last.cm = rl_u32(last.cm, 0);          // it) SGPR values, keeping the whole walk scalar
    last.hk = key_of<HEUR>(qc, last.cm);

    // ---- 1. the path.  Levels 0..D-1 are full (D = floor(log2 n)), so every node above level D-1
    //      has two children and the walk takes D-1 unconditional steps; the last step (level D-1 ->
    //      D) exists only below a node with a child.  Per step: c = bit, P = 2P + c (P = position + 1
    //      of the current node), Pr = the same relative to the current block's root (bit index Pr-1).
    const int D = 31 - __clz(n);
    uint32_t P = 1, R1 = 0, v2 = 0;
    int K = 0;
    {
        // w2 = block word << 1, so node Pr of the block (Pr = 1 at its root) is bit Pr of w2
        uint32_t w2 = rl_u32(v01, 0) << 1, Pr = 1;
        const int full = D - 1;
        int lvl = 0;  // level of the current node
        for (int t = 0; lvl < full; t++) {
            const int steps = min(5, full - lvl);  // unconditional steps inside this block
            for (int r = 0; r < steps; r++) Pr = 2u * Pr + ((w2 >> Pr) & 1u);
            P = (P << steps) + Pr - (1u << steps);
            lvl += steps;
            if (steps < 5) break;
            // the node reached roots the block of tier t + 1: fetch its word
            Pr = 1u;
            if (t == 0) {
                w2 = rl_u32(v01, (int)P - 31) << 1;
                R1 = P;
                if (full >= 10) v2 = hp.lb[33 + ((R1 << 5) - 1024u) + (uint32_t)(lane & 31)];
            } else if (t == 1) {
                w2 = rl_u32(v2, (int)(P - (R1 << 5))) << 1;
            } else {  // tiers >= 3 (heaps above 32767 entries): an L2-coherent read of the HBM block
                w2 = (uint32_t)uni((int)__hip_atomic_fetch_or(hp.hb + hb_word(t + 1, P), 0u, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)) << 1;
            }
        }
        K = lvl;
        // the last step: below a node at level D-1 with a child (2p + 1 < n, p = P - 1)
        // (w2, Pr) already describe the block holding the node at level D-1
        if (D >= 1 && 2u * P - 1u < (uint32_t)n) {
            const uint32_t c = (2u * P < (uint32_t)n) ? ((w2 >> Pr) & 1u) : 0u;
            P = 2u * P + c;
            K++;
        }
    }

    // ---- 2. one load round
    const bool on = lane >= 1 && lane <= K;
    const int sh = K - lane;
    const int pi = on ? (int)(P >> sh) - 1 : 0;
    const bool hasb = on && lane < K;
    const int pn = hasb ? (int)(P >> (sh - 1)) - 1 : 0;
    const int si = (pi & 1) ? pi + 1 : pi - 1;
    const bool hass = on && si < n;
    Ent A, B, S;
    hload_if<SPILL>(hp, on, pi, A.f, A.cm);
    hload_if<SPILL>(hp, hasb, pn, B.f, B.cm);
    hload_if<SPILL>(hp, hass, si, S.f, S.cm);
    A.hk = key_of<HEUR>(qc, A.cm);
    B.hk = key_of<HEUR>(qc, B.cm);
    S.hk = key_of<HEUR>(qc, S.cm);

    // ---- 3. movers and stores
    const int m = __popcll(ballot(on && !ent_lt(last, A)));
    if (lane >= 1 && lane <= m) hstore<SPILL>(hp, (int)(P >> (sh + 1)) - 1, A.f, A.cm);
    if (lane == 0) hstore<SPILL>(hp, (int)(P >> (K - m)) - 1, last.f, last.cm);
    if (m >= 1) {
        root.f = rl_f64(A.f, 1);
        root.cm = rl_u32(A.cm, 1);
        root.hk = rl_u32(A.hk, 1);
    } else {
        root = last;
    }

    // ---- 4. bits of p_0 .. p_{m-1}
    if (hass && lane <= m) {
        const Ent vn = lane < m ? B : last;  // the new heap[p_i]
        const bool bit = (pi & 1) ? !ent_lt(vn, S) : !ent_lt(S, vn);
        bit_write(hp, lane - 1, P >> (sh + 1), bit ? 1u : 0u);
    }
    wave_sync_mem();
}

// heappush of `it` onto a heap of n entries (position n is free): the ancestors a_j = parent^j(n)
// load in one round (with the siblings of a_{j-1}, for the bits); a ballot popcount t gives how
// many move down; lanes 1..t+1 rewrite the bits of a_1..a_{t+1}, whose children changed.
template <bool SPILL, int HEUR>
__device__ __forceinline__ void heap_push(const Heap& hp, const Q& qc, int n, const Ent& it, Ent& root, int lane)
{
    n = uni(n);
    const uint32_t np1 = (uint32_t)n + 1u;
    const int D = 31 - __clz((int)np1);  // depth of position n
    const bool on = lane >= 1 && lane <= D;
    const int aj = on ? (int)(np1 >> lane) - 1 : 0;
    const int x = on ? (int)(np1 >> (lane - 1)) - 1 : 1;  // a_{j-1}
    const int sx = (x & 1) ? x + 1 : x - 1;
    const bool hass = on && sx < n;  // a_{j-1} = n (lane 1) has a sibling only when n is even
    Ent a, S;
    hload_if<SPILL>(hp, on, aj, a.f, a.cm);
    hload_if<SPILL>(hp, hass, sx, S.f, S.cm);
    a.hk = key_of<HEUR>(qc, a.cm);
    S.hk = key_of<HEUR>(qc, S.cm);
    const int t = __popcll(ballot(on && ent_lt(it, a)));  // the "less" set is a prefix from the parent up
    if (lane >= 1 && lane <= t) hstore<SPILL>(hp, x, a.f, a.cm);
    const int ipos = (int)(np1 >> t) - 1;
    if (lane == 0) hstore<SPILL>(hp, ipos, it.f, it.cm);
    if (ipos == 0) root = it;
    if (hass && lane <= t + 1) {
        const Ent vn = lane - 1 < t ? a : it;  // the new heap[a_{j-1}]
        const bool bit = (x & 1) ? !ent_lt(vn, S) : !ent_lt(S, vn);
        bit_write(hp, D - lane, np1 >> lane, bit ? 1u : 0u);
    }
    wave_sync_mem();
}

template <int HEUR>
__global__ __launch_bounds__(64) void astar2d_kernel(
    const uint32_t* __restrict__ occ, int W, int H, const int32_t* __restrict__ start_xy,
    const int32_t* __restrict__ goal_xy, const int32_t* __restrict__ order, int nq, double* __restrict__ cost_out,
    int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out, int path_cap,
    int32_t* __restrict__ nexp_out, uint32_t* __restrict__ expand_out, int expand_cap,
    int64_t* __restrict__ counters, int32_t* __restrict__ status_out, int* __restrict__ queue,
    uint4* __restrict__ spill_all, int heap_cap, int lds_cap, uint32_t* __restrict__ cst_all, size_t cst_words,
    double* __restrict__ G_all, uint32_t* __restrict__ hbits_all, size_t hbits_words, int prio_n,
    unsigned long long* __restrict__ span)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    span_begin(span);
    Heap hp;
    hp.lb = (lds_u32*)smem;
    hp.lg = (lds_f64*)(smem + kBitsLdsBytes);
    hp.lcm = (lds_u32*)(smem + kBitsLdsBytes + (size_t)8 * lds_cap);
    hp.hb = hbits_all + (size_t)worker * hbits_words;
    {
        const size_t spill_n = (size_t)(heap_cap > lds_cap ? heap_cap - lds_cap : 0);
        hp.spill = __builtin_amdgcn_make_buffer_rsrc(spill_all + (size_t)worker * spill_n, 0, (int)(spill_n * 16), 0x00020000);
    }
    hp.lds_cap = lds_cap;
    uint32_t* cst = cst_all + (size_t)worker * cst_words;
    double* G = G_all + (size_t)worker * ((size_t)W * (size_t)H);
    // this lane's cell of the 3x3 block: lane i < 9 -> occupancy of (x + i/3 - 1, y + i%3 - 1),
    // lane 9 + i -> its CLOSED-state nibble
    const int blk_i = lane < 9 ? lane : (lane < 18 ? lane - 9 : 4);
    const int blk_dx = blk_i / 3 - 1, blk_dy = blk_i % 3 - 1;

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
        {
            uint4* c4 = reinterpret_cast<uint4*>(cst);
            const size_t n4 = cst_words / 4;
            for (size_t i = lane; i < n4; i += 64) c4[i] = make_uint4(0u, 0u, 0u, 0u);
            for (size_t i = n4 * 4 + lane; i < cst_words; i += 64) cst[i] = 0u;
        }
        wave_sync_mem();

        const int sx = start_xy[2 * q], sy = start_xy[2 * q + 1];
        Q qc;
        qc.gx = goal_xy[2 * q];
        qc.gy = goal_xy[2 * q + 1];
        const bool s_in = (unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H;
        const bool g_in = (unsigned)qc.gx < (unsigned)W && (unsigned)qc.gy < (unsigned)H;
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
        const uint32_t goal_xy13 = ((uint32_t)qc.gx << 13) | (uint32_t)qc.gy;

        Ent root;  // heap[0], kept in registers (wave-uniform)
        root.cm = ((((uint32_t)sx << 13) | (uint32_t)sy) << 4) | 8u;  // Node(start, start, 0, 0)
        root.hk = 0;
        root.f = 0.0;
        if (lane == 0) hstore<true>(hp, 0, root.f, root.cm);
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
            const Ent node = root;
            npop++;
            n -= 1;
            const int x = (int)(node.cm >> 17), y = (int)((node.cm >> 4) & 8191u);
            const int ndir = (int)(node.cm & 15u);
            const uint32_t nlin = (uint32_t)x * (uint32_t)H + (uint32_t)y;

            // ---- HBM round, issued before the LDS pop so the two overlap: one unconditional load
            //      per lane (raw word kept until after the pop, so no wait is placed before it)
            uint32_t blk_word, blk_sh;
            bool blk_in;
            {
                const int cx = x + blk_dx, cy = y + blk_dy;
                blk_in = lane < 18 && (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
                const uint32_t ci = blk_in ? (uint32_t)cx * (uint32_t)H + (uint32_t)cy : 0u;
                const uint32_t* ptr = lane < 9 ? occ + (ci >> 5) : cst + (ci >> 3);
                blk_sh = lane < 9 ? (ci & 31u) : (ci & 7u) * 4u;
                blk_word = *ptr;
            }
            double gpar = 0.0;  // G[parent] (the parent closed earlier); the start has g = 0
            if (lane == 18 && ndir < 8) gpar = G[(uint32_t)(x - c_mx[ndir]) * (uint32_t)H + (uint32_t)(y - c_my[ndir])];
#ifdef PMP_STAMPS_SPLIT  // diagnostic: wait for the HBM round before the pop, time the two apart
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(blk_word), "v"(gpar) : "memory");
            STAMP(tsB);
            cyc_hbm += tsB - ts0;
            ts0 = tsB;
#endif

            // ---- heappop (a_star.py:54): `last` = heap[n] sifts down the CPython path
            if (n > 0) {
                if (n < lds_cap) heap_pop<false, HEUR>(hp, qc, n, root, lane);
                else heap_pop<true, HEUR>(hp, qc, n, root, lane);
            }

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

            // CLOSED[node.current] = node (a_star.py:82).  The node's state word was loaded by lane 13
            // and only this wave writes it: store it back now (fire-and-forget, off the critical path).
            const double gnode = ndir == 8 ? 0.0 : rl_f64(gpar, 18) + ((ndir & 1) ? kSqrt2 : 1.0);
            if (lane == 13) cst[nlin >> 3] = blk_word | ((uint32_t)(ndir + 1) << blk_sh);
            if (lane == 14) G[nlin] = gnode;
            if (lane == 0 && expand_out && nexp < expand_cap)
                expand_out[(size_t)q * expand_cap + nexp] = nlin | ((uint32_t)ndir << 28);
            nexp++;

            if (node.cm >> 4 == goal_xy13) {  // goal found (a_star.py:61-64)
                st = PMP_FOUND;
                wave_sync_mem();
                if (lane == 0) {  // extractPath (a_star.py:98-117): goal -> start, cost in that order
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
                        cx -= c_mx[d];
                        cy -= c_my[d];
                    }
                    goal_cost = cost;
                    plen = len;
                }
                break;
            }

            // ---- getNeighbor + the push loop in motion order; push the goal and stop (a_star.py:66-80)
            bool nb_ok = false;
            uint32_t nbxy = 0;
            if (lane < 8) {
                const int ax = c_mx[lane] + 1, ay = c_my[lane] + 1;
                uint32_t need = 16u | (1u << (ax * 3 + ay));                     // both endpoints
                if (lane & 1) need |= (1u << (3 + ay)) | (1u << (ax * 3 + 1));  // both corner cells
                nb_ok = (occ9 & need) == 0u && ((cls9 >> (ax * 3 + ay)) & 1u) == 0u;
                nbxy = ((uint32_t)(x + c_mx[lane]) << 13) | (uint32_t)(y + c_my[lane]);
            }
            uint64_t vm = ballot(nb_ok) & 0xffull;
            const uint64_t gm = ballot(nb_ok && nbxy == goal_xy13) & 0xffull;
            if (gm) vm &= (gm << 1) - 1;
            Ent item;  // node + motion (node.py:39-41), h = GraphSearcher.h (graph_search.py:41-44)
            {
                const int m = lane & 7;
                item.cm = (nbxy << 4) | (uint32_t)m;
                item.f = 0.0;
                item.hk = 0u;
                if (lane < 8) item.f = (gnode + ((m & 1) ? kSqrt2 : 1.0)) + h_and_key<HEUR>(qc, item.cm, item.hk);
            }
            bool overflow = false;
            while (vm) {
                const int m = __ffsll((long long)vm) - 1;
                vm &= vm - 1;
                if (n >= heap_cap) { overflow = true; break; }
                Ent it;
                it.f = rl_f64(item.f, m);
                it.cm = rl_u32(item.cm, m);
                it.hk = rl_u32(item.hk, m);
                if (n < lds_cap) heap_push<false, HEUR>(hp, qc, n, it, root, lane);
                else heap_push<true, HEUR>(hp, qc, n, it, root, lane);
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
    const int dx = s[2 * q] - g[2 * q], dy = s[2 * q + 1] - g[2 * q + 1];
    return (int)__dsqrt_rn((double)dx * dx + (double)dy * dy);  // expansions grow ~ with distance^2
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
    // heap entry; keep a little slack
    int bytes = (160 * 1024) / workers_per_cu - 256 - kBitsLdsBytes;
    return (bytes / 12) & ~15;
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

}  // namespace

extern "C" int pmp_astar2d_reserve(pmp_ctx* ctx, int W, int H, int workers, int heap_cap)
{
    if (!ctx) return PMP_EINVAL;
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim || workers < 1)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_reserve: bad dims/workers");
    if (heap_cap <= 0) heap_cap = default_heap_cap(W, H);
    if ((size_t)heap_cap > max_heap(W, H)) heap_cap = (int)max_heap(W, H);
    const size_t ncell = (size_t)W * H;
    const size_t cst_words = ((ncell + 7) / 8 + 3) & ~(size_t)3;
    {
        const size_t per_worker = (size_t)heap_cap * 16 + cst_words * 4 + ncell * 8 + hbits_words(heap_cap) * 4;
        const size_t fit = kScratchBudget / per_worker;
        if (fit < 1) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_astar2d_reserve: one worker exceeds the scratch budget");
        if ((size_t)workers > fit) workers = (int)fit;
    }
    const int per_cu = (workers + 255) / 256;
    int lds_cap = default_lds_cap(per_cu < 1 ? 1 : per_cu);
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

extern "C" int pmp_astar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                                 int heuristic, const int32_t* start_xy, const int32_t* goal_xy, int nq,
                                 double* cost, int32_t* path_len, uint32_t* path, int path_cap,
                                 int32_t* n_expanded, uint32_t* expand, int expand_cap, int64_t* counters,
                                 int32_t* status)
{
    if (!ctx) return PMP_EINVAL;
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: W and H must be in [1, 8192]");
    if (heuristic != 0 && heuristic != 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: heuristic must be 0 or 1");
    if (nq < 0 || path_cap < 1 || (expand && expand_cap < 1))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: bad nq/path_cap/expand_cap");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xy || !goal_xy || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    if (!(ctx->astar_W == W && ctx->astar_H == H)) {
        int workers = default_workers();
        if (workers > nq) workers = nq;
        int rc = pmp_astar2d_reserve(ctx, W, H, workers, 0);
        if (rc) return rc;
    }
    const int workers = ctx->astar_workers < nq ? ctx->astar_workers : nq;
    const size_t ncell = (size_t)W * H;
    const size_t cst_words = ((ncell + 7) / 8 + 3) & ~(size_t)3;
    uint4* spill = (uint4*)ctx->buf[SCR_HEAP];
    uint32_t* cst = (uint32_t*)ctx->buf[SCR_CLOSED];
    int* queue = (int*)ctx->buf[SCR_AUX0];
    double* G = (double*)ctx->buf[SCR_G];
    hipStream_t s = (hipStream_t)stream;
    const size_t lds = (size_t)kBitsLdsBytes + (size_t)ctx->astar_lds_cap * 12;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    int32_t* order = nullptr;
    if (ctx->astar_lpt && nq > workers) {
        const int nb = (int)ceil(sqrt((double)W * W + (double)H * H)) + 1;
        int* hist = (int*)pmp_scratch(ctx, SCR_PDIR, sizeof(int) * ((size_t)nb + (size_t)nq));
        if (!hist) return PMP_ENOMEM;
        order = hist + nb;
        PMP_HIP_CHECK(ctx, hipMemsetAsync(hist, 0, sizeof(int) * (size_t)nb, s));
        hipLaunchKernelGGL(lpt_hist, dim3((nq + 255) / 256), dim3(256), 0, s, start_xy, goal_xy, nq, nb, hist);
        hipLaunchKernelGGL(lpt_scan, dim3(1), dim3(64), 0, s, nb, hist);
        hipLaunchKernelGGL(lpt_scatter, dim3((nq + 255) / 256), dim3(256), 0, s, start_xy, goal_xy, nq, nb, hist, order);
    }
    auto kern = heuristic == 1 ? astar2d_kernel<1> : astar2d_kernel<0>;
    hipLaunchKernelGGL(kern, dim3(workers), dim3(64), lds, s, occ_bits, W, H, start_xy,
                       goal_xy, (const int32_t*)order, nq, cost, path_len, path, path_cap, n_expanded, expand,
                       expand_cap, counters, status, queue, spill, ctx->astar_heap_cap, ctx->astar_lds_cap, cst, cst_words, G,
                       (uint32_t*)ctx->buf[SCR_BITS], hbits_words(ctx->astar_heap_cap), order ? ctx->astar_prio_n : 0, ctx->span);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
