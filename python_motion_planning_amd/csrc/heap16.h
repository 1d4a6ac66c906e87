// Wave64 binary min-heap of 16-byte entries for strictly (totally) ordered keys, shared by the
// 3D A* (astar3d.hip) and D* (dstar.hip) kernels.  Positions < lds_cap live in LDS as three SoA
// arrays (f64 g, u32 a, u32 b); deeper positions spill to HBM through buffer instructions (one
// 16 B record each).  With a total order any correct heap pops the same sequence, so the shape is
// free; the operations are organised for one wave:
//   pop:  the hole walks down 6 levels per LDS round -- 63 lanes each load one sibling pair of the
//         next 6 levels, three ballots give "right child is smaller" and "child < last" per pair,
//         the walk over those masks is scalar, and the movers store in parallel;
//   push: the ancestors load in one round; the "less than the new item" set is a prefix of the
//         root path, so a ballot popcount gives the sift-up distance;
//   push_batch: an expansion's pushes stored together, only those below their parent sifted up;
// The key is supplied by a policy type K: K::derive(e) fills e.f / e.hk from the stored fields and
// K::lt(x, y) is the strict order.  K::kStoredF: f is stored beside the entry (24 B in LDS: g, f, a,
// b; 32 B spill records) instead of derived on every load, so a key costs no square root.
#pragma once
#include "pmp_internal.h"

namespace heap16 {

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

struct Ent {
    double g;       // stored
    uint32_t a, b;  // stored
    double f;       // derived (K::derive)
    uint32_t hk;    // derived
};

struct Heap {
    lds_f64* lg;
    lds_f64* lf;  // stored-f heaps only
    lds_u32* la;
    lds_u32* lb;
    __amdgpu_buffer_rsrc_t spill;  // {g lo, g hi, a, b} (+ {f lo, f hi} with stored f) for positions >= lds_cap
    int lds_cap;
};

// LDS and spill bytes per entry
template <bool SF> constexpr int lds_entry_bytes() { return SF ? 24 : 16; }
template <bool SF> constexpr int spill_entry_bytes() { return SF ? 32 : 16; }

template <bool SF = false>
__device__ __forceinline__ Heap make_heap(unsigned char* smem, int lds_cap, uint4* spill_base, size_t spill_n)
{
    Heap hp;
    hp.lg = (lds_f64*)smem;
    hp.lf = SF ? (lds_f64*)(smem + (size_t)8 * lds_cap) : nullptr;
    hp.la = (lds_u32*)(smem + (size_t)(SF ? 16 : 8) * lds_cap);
    hp.lb = (lds_u32*)(smem + (size_t)(SF ? 20 : 12) * lds_cap);
    hp.lds_cap = lds_cap;
    hp.spill = __builtin_amdgcn_make_buffer_rsrc(spill_base, 0, (int)(spill_n * spill_entry_bytes<SF>()), 0x00020000);
    return hp;
}

template <bool SPILL, bool SF = false>
__device__ __forceinline__ void load(const Heap& hp, int p, Ent& e)
{
    if (!SPILL || p < hp.lds_cap) {
        e.g = hp.lg[p];
        if (SF) e.f = hp.lf[p];
        e.a = hp.la[p];
        e.b = hp.lb[p];
    } else {
        const int off = (p - hp.lds_cap) * spill_entry_bytes<SF>();
        const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(hp.spill, off, 0, 0));
        e.g = __hiloint2double((int)v.y, (int)v.x);
        e.a = v.z;
        e.b = v.w;
        if (SF) {
            const uint2 w = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(hp.spill, off + 16, 0, 0));
            e.f = __hiloint2double((int)w.y, (int)w.x);
        }
    }
}

template <bool SPILL, bool SF = false>
__device__ __forceinline__ void store(const Heap& hp, int p, const Ent& e)
{
    if (!SPILL || p < hp.lds_cap) {
        hp.lg[p] = e.g;
        if (SF) hp.lf[p] = e.f;
        hp.la[p] = e.a;
        hp.lb[p] = e.b;
    } else {
        const int off = (p - hp.lds_cap) * spill_entry_bytes<SF>();
        const uint64_t bits = (uint64_t)__double_as_longlong(e.g);
        const uint4 v = make_uint4((uint32_t)bits, (uint32_t)(bits >> 32), e.a, e.b);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                               hp.spill, off, 0, 0);
        if (SF) {
            const uint64_t fb = (uint64_t)__double_as_longlong(e.f);
            const uint2 w = make_uint2((uint32_t)fb, (uint32_t)(fb >> 32));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, w),
                                                  hp.spill, off + 16, 0, 0);
        }
    }
}

__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

__device__ __forceinline__ Ent rl_ent(const Ent& e, int lane)
{
    Ent r;
    r.g = rl_f64(e.g, lane);
    r.f = rl_f64(e.f, lane);
    r.a = rl_u32(e.a, lane);
    r.b = rl_u32(e.b, lane);
    r.hk = rl_u32(e.hk, lane);
    return r;
}

// Per-lane constants of the 6-level pop chunk: lane l < 63 owns the sibling pair at level jl,
// offset ol of the chunk below the hole.
__device__ __forceinline__ void pop_lane_consts(int lane, int& jl, int& ol)
{
    jl = 32 - __clz(lane + 1);
    ol = lane + 1 - (1 << (jl - 1));
}

// Lane-parallel form of the 6-level walk (pop<..., PAR = true>): lane l < 63 owns sibling pair l
// (level jl, offset ol) and knows its strict ancestor pairs (`anc`) and which child of each leads to
// it (`dir`).  The walk visits the pair iff every ancestor chose the child toward it and that child
// moved up (it is < last); so "visited and my chosen child moves" is a handful of 64-bit mask tests
// per lane instead of the 6-step scalar chain (the scalar unit is shared by the CU's four SIMDs).
struct Walk6 {
    uint64_t anc, dir;
};
__device__ __forceinline__ Walk6 walk6_consts(int lane, int jl, int ol)
{
    Walk6 w{0ull, 0ull};
    if (lane < 63)
        for (int i = 1; i < jl; i++) {
            const int idx = (1 << (i - 1)) - 1 + (ol >> (jl - i));
            w.anc |= 1ull << idx;
            w.dir |= (uint64_t)((ol >> (jl - i - 1)) & 1) << idx;
        }
    return w;
}

// Extract-min on a heap whose size was already decremented to n (> 0); the old last element sits
// at position n.  `root` receives the new minimum (wave-uniform).  PAR: the walk over each 6-level
// chunk is evaluated lane-parallel from `w` (same result as the scalar walk).  Returns the final hole
// (where the old last element landed): the entries on the path from the root's child down to it moved
// up one level.
template <class K, bool SPILL, bool PAR = false>
__device__ __forceinline__ int pop(const Heap& hp, const K& key, int n, Ent& root, int lane, int jl, int ol,
                                    const Walk6& w = Walk6{0ull, 0ull})
{
    constexpr bool SF = K::kStoredF;
    n = uni(n);
    Ent last;
    load<SPILL, SF>(hp, n, last);
    last.g = rl_f64(last.g, 0);
    if (SF) last.f = rl_f64(last.f, 0);
    last.a = rl_u32(last.a, 0);
    last.b = rl_u32(last.b, 0);
    key.derive(last);
    int hole = 0;
    bool first = true;
    for (;;) {
        const int li = ((hole + 1) << jl) - 1 + 2 * ol;
        const bool vl = (lane < 63) & (li < n);
        const bool vr = (lane < 63) & (li + 1 < n);
        Ent L, R;
        L.g = R.g = 0.0;
        L.f = R.f = 0.0;
        L.a = R.a = 0u;
        L.b = R.b = 0u;
        if constexpr (SPILL) {
            if (vl) load<true, SF>(hp, li, L);
            if (vr) load<true, SF>(hp, li + 1, R);
        } else {
            load<false, SF>(hp, vl ? li : 0, L);
            load<false, SF>(hp, vr ? li + 1 : 0, R);
        }
        key.derive(L);
        key.derive(R);
        const uint64_t dmask = ballot(vr & K::lt(R, L));       // the smaller child
        const uint64_t mlmask = ballot(vl & K::lt(L, last));  // moves up while child < last
        const uint64_t mrmask = ballot(vr & K::lt(R, last));
        int cur = uni(hole), oc = 0;
        uint64_t mover = 0, movr = 0;
        uint32_t go = 1u;
        if constexpr (PAR) {
            // chosen child of each pair moves up (< last; validity is in the masks)
            const uint64_t cl = (dmask & mrmask) | (~dmask & mlmask);
            const bool vis = lane < 63 && ((dmask ^ w.dir) & w.anc) == 0ull && (cl & w.anc) == w.anc;
            mover = ballot(vis && ((cl >> lane) & 1ull));
            movr = mover & dmask;
            go = (mover >> 31) != 0ull ? 1u : 0u;  // a level-6 pair (indices 31..62) moved
            if (mover) cur = __builtin_amdgcn_readlane(li + (int)((dmask >> lane) & 1ull), 63 - __clzll((long long)mover));
        } else {
        // branch-free scalar walk: every step is a select, so the 6 levels are one straight-line
        // SALU sequence (taken branches cost more than the arithmetic they skip)
#pragma unroll
        for (int lv = 1; lv <= 6; lv++) {
            const int c = 2 * cur + 1;
            const int pl = (1 << (lv - 1)) - 1 + oc;
            const uint32_t r = (uint32_t)(dmask >> pl) & 1u;
            const uint64_t mm = r ? mrmask : mlmask;
            go = go & (uint32_t)(c < n) & ((uint32_t)(mm >> pl) & 1u);
            const uint64_t bit = (uint64_t)go << pl;
            mover |= bit;
            movr |= (uint64_t)(go & r) << pl;
            cur = go ? c + (int)r : cur;
            oc = go ? 2 * oc + (int)r : oc;
        }
        }
        if ((mover >> lane) & 1ull) {
            const bool rr = (movr >> lane) & 1ull;
            const int dst = ((rr ? li + 1 : li) - 1) >> 1;
            store<SPILL, SF>(hp, dst, rr ? R : L);
        }
        if (first && (mover & 1ull)) root = rl_ent((movr & 1ull) ? R : L, 0);
        first = false;
        hole = cur;
        if (!go) break;
        wsync();
    }
    if (lane == 0) store<SPILL, SF>(hp, hole, last);
    if (hole == 0) root = last;
    wsync();
    return hole;
}

// Sift `it` (wave-uniform, derived) up from position p0 (a push at p0 = n).  `root` is updated if it
// becomes the minimum.  Returns the position it lands at; the ancestors of p0 from there down moved
// one level toward p0.
template <class K, bool SPILL>
__device__ __forceinline__ int sift_up(const Heap& hp, const K& key, int p0, const Ent& it, Ent& root, int lane)
{
    constexpr bool SF = K::kStoredF;
    const int np1 = uni(p0) + 1;
    const int depth = 31 - __clz(np1);
    const bool valid = lane < depth;
    const int apos = valid ? (np1 >> (lane + 1)) - 1 : 0;
    Ent a;
    a.g = 0.0;
    a.f = 0.0;
    a.a = a.b = 0u;
    if constexpr (SPILL) {
        if (valid) load<true, SF>(hp, apos, a);
    } else {
        load<false, SF>(hp, apos, a);
    }
    key.derive(a);
    const int t = __popcll(ballot(valid & K::lt(it, a)));
    if (lane < t) store<SPILL, SF>(hp, (np1 >> lane) - 1, a);
    const int ipos = (np1 >> t) - 1;
    if (lane == 0) store<SPILL, SF>(hp, ipos, it);
    if (ipos == 0) root = it;
    wsync();
    return ipos;
}
// Insert `it` into a heap of n entries.
template <class K, bool SPILL>
__device__ __forceinline__ int push(const Heap& hp, const K& key, int n, const Ent& it, Ent& root, int lane)
{
    return sift_up<K, SPILL>(hp, key, n, it, root, lane);
}

// Push the items of the lanes in pm (wave-uniform mask; each lane's `it` derived) into a heap of n
// entries, for a total order (the heap's shape is free): all stored together at n, n + 1, ... (lane
// order) in one round, then only the ones below their pre-batch parent (or whose parent is another
// new item) sift up, in position order -- a sift-up only lowers the parents of later positions, so
// an item found not below its parent stays valid.  Returns the new size.
template <class K>
__device__ __forceinline__ int push_batch(const Heap& hp, const K& key, int n, uint64_t pm, const Ent& it, Ent& root,
                                          int lane)
{
    constexpr bool SF = K::kStoredF;
    n = uni(n);
    const bool mine = (pm >> lane) & 1ull;
    const int pos = n + __popcll(pm & ((1ull << lane) - 1ull)), pp = (pos - 1) >> 1;
    const bool hasp = mine && pos > 0 && pp < n;
    Ent par;
    load<true, SF>(hp, hasp ? pp : 0, par);
    key.derive(par);
    const bool below = !hasp || K::lt(it, par);
    if (mine) store<true, SF>(hp, pos, it);
    wsync();
    uint64_t sm = ballot(mine && below);
    while (sm) {
        const int m = __ffsll((long long)sm) - 1;
        sm &= sm - 1ull;
        const Ent x = rl_ent(it, m);
        const int p0 = n + __popcll(pm & ((1ull << m) - 1ull));
        if (p0 < hp.lds_cap) sift_up<K, false>(hp, key, p0, x, root, lane);
        else sift_up<K, true>(hp, key, p0, x, root, lane);
    }
    return n + __popcll(pm);
}

}  // namespace heap16
