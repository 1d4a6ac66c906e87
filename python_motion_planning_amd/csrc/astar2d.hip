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
struct Heap {
    lds_f64* lg;       // LDS f[lds_cap]
    lds_u32* lcm;      // LDS cm[lds_cap]
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

// heappop on a heap of n (>0, already decremented) entries whose old last element sits at position
// n; the old root has been taken by the caller.  Updates `root` (wave-uniform copy of heap[0]).
// jl / ol: this lane's pair level (1..6) and pair offset inside a chunk (lane 63: idle).
template <bool SPILL, int HEUR>
__device__ __forceinline__ void heap_pop(const Heap& hp, const Q& qc, int n, Ent& root, int lane, int jl, int ol)
{
    n = uni(n);  // wave-uniform by construction; say so, so the walk below stays on the SALU
    Ent last;
    hload<SPILL>(hp, n, last.f, last.cm);  // uniform address, but an LDS load is not known-uniform:
    last.f = rl_f64(last.f, 0);            // readlane makes `last` (and the root / node derived from
    last.cm = rl_u32(last.cm, 0);          // it) SGPR values, keeping the whole walk scalar
    last.hk = key_of<HEUR>(qc, last.cm);
    int hole = 0;
    bool first = true;
    for (;;) {
        const int li = ((hole + 1) << jl) - 1 + 2 * ol;  // left child position of this lane's pair
        const bool vl = (lane < 63) & (li < n);
        const bool vr = (lane < 63) & (li + 1 < n);
        Ent L, R;
        if constexpr (SPILL) {
            L.f = R.f = 0.0;
            L.cm = R.cm = 0u;
            if (vl) hload<true>(hp, li, L.f, L.cm);
            if (vr) hload<true>(hp, li + 1, R.f, R.cm);
        } else {  // unconditional loads from clamped (valid) addresses: no branch
            const int a = vl ? li : 0, b = vr ? li + 1 : 0;
            L.f = hp.lg[a];
            L.cm = hp.lcm[a];
            R.f = hp.lg[b];
            R.cm = hp.lcm[b];
        }
        L.hk = key_of<HEUR>(qc, L.cm);
        R.hk = key_of<HEUR>(qc, R.cm);
        const uint64_t dmask = ballot(vr & !ent_lt(L, R));    // heapq._siftup: right unless left < right
        const uint64_t mlmask = ballot(vl & !ent_lt(last, L));  // child may move up past `last`
        const uint64_t mrmask = ballot(vr & !ent_lt(last, R));
        // scalar walk through the chunk's 6 levels (all SGPR, unrolled)
        int cur = uni(hole), oc = 0;
        uint64_t mover = 0, movr = 0;
        bool go = true;
#pragma unroll
        for (int lv = 1; lv <= 6; lv++) {
            const int c = 2 * cur + 1;
            const int pl = (1 << (lv - 1)) - 1 + oc;  // pair lane
            const int r = (int)((dmask >> pl) & 1ull);
            const uint64_t mm = r ? mrmask : mlmask;
            go = go & (c < n) & (((mm >> pl) & 1ull) != 0ull);
            if (go) {
                mover |= 1ull << pl;
                movr |= (uint64_t)r << pl;
                cur = c + r;
                oc = 2 * oc + r;
            }
        }
        if ((mover >> lane) & 1ull) {  // the chosen child moves up one level
            const bool rr = (movr >> lane) & 1ull;
            hstore<SPILL>(hp, ((rr ? li + 1 : li) - 1) >> 1, rr ? R.f : L.f, rr ? R.cm : L.cm);
        }
        if (first && (mover & 1ull)) {  // the child that moved into the root is the new root
            const bool r0 = movr & 1ull;
            root.f = rl_f64(r0 ? R.f : L.f, 0);
            root.cm = rl_u32(r0 ? R.cm : L.cm, 0);
            root.hk = rl_u32(r0 ? R.hk : L.hk, 0);
        }
        first = false;
        hole = cur;
        if (!go) break;
        wave_sync_mem();
    }
    if (lane == 0) hstore<SPILL>(hp, hole, last.f, last.cm);
    if (hole == 0) root = last;
    wave_sync_mem();
}

// heappush of `it` onto a heap of n entries (position n is free).
template <bool SPILL, int HEUR>
__device__ __forceinline__ void heap_push(const Heap& hp, const Q& qc, int n, const Ent& it, Ent& root, int lane)
{
    n = uni(n);
    const int np1 = n + 1;
    const int depth = 31 - __clz(np1);  // ancestors of position n
    const bool valid = lane < depth;
    const int apos = valid ? (np1 >> (lane + 1)) - 1 : 0;
    Ent a;
    if constexpr (SPILL) {
        a.f = 0.0;
        a.cm = 0u;
        if (valid) hload<true>(hp, apos, a.f, a.cm);
    } else {
        a.f = hp.lg[apos];
        a.cm = hp.lcm[apos];
    }
    a.hk = key_of<HEUR>(qc, a.cm);
    const int t = __popcll(ballot(valid & ent_lt(it, a)));  // the "less" set is a prefix from the parent up
    if (lane < t) hstore<SPILL>(hp, (np1 >> lane) - 1, a.f, a.cm);
    const int ipos = (np1 >> t) - 1;
    if (lane == 0) hstore<SPILL>(hp, ipos, it.f, it.cm);
    if (ipos == 0) root = it;
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
    double* __restrict__ G_all, unsigned long long* __restrict__ span)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    span_begin(span);
    Heap hp;
    hp.lg = (lds_f64*)(smem);
    hp.lcm = (lds_u32*)(smem + (size_t)8 * lds_cap);
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
    // this lane's sibling pair inside a pop chunk: level jl = 1..6 below the hole, offset ol
    const int pop_jl = 32 - __clz(lane + 1);
    const int pop_ol = lane + 1 - (1 << (pop_jl - 1));

    for (;;) {
        // readfirstlane (not __shfl): the compiler must SEE the query index as wave-uniform, or
        // every value derived from it (coordinates, heap size, walk state) lands in VGPRs and the
        // scalar heap walk is compiled as a divergent loop.
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = uni(order ? order[qi] : qi);

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
        uint64_t cyc_pop = 0, cyc_wait = 0, cyc_push = 0;
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

            // ---- heappop (a_star.py:54): `last` = heap[n] sifts down the CPython path
            if (n > 0) {
                if (n < lds_cap) heap_pop<false, HEUR>(hp, qc, n, root, lane, pop_jl, pop_ol);
                else heap_pop<true, HEUR>(hp, qc, n, root, lane, pop_jl, pop_ol);
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
                counters[4 * q + 1] = (int64_t)cyc_wait;
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
    // 160 KiB LDS per CU shared by the resident workers; 12 B per entry, keep a little slack
    int bytes = (160 * 1024) / workers_per_cu - 256;
    return (bytes / 12) & ~15;
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
        const size_t per_worker = (size_t)heap_cap * 16 + cst_words * 4 + ncell * 8;
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
    const size_t lds = (size_t)ctx->astar_lds_cap * 12;
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
                       ctx->span);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
