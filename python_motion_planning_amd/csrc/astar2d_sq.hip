// Single-query 2D A* (and Dijkstra / GBFS) for gfx950: the drop-in AStar.plan() latency engine.
// Bit-exact with the reference AStar.plan (global_planner/graph_search/a_star.py:39-83) including
// CPython heapq's tie behaviour (Lib/heapq.py heappush/_siftdown, heappop/_siftup) under
// Node.__lt__ (utils/environment/node.py:51-54) -- the algorithm of astar2d.hip / astar2d_mq.hip,
// laid out for ONE query's latency instead of a batch's throughput.
//
// One query per workgroup of one wave, which owns the CU's whole LDS:
//  - the heap lives entirely in LDS (f64 f[], u32 code[] as SoA; up to 16,383 entries, levels 0-13;
//    a query that outgrows the LDS capacity stops with PMP_CAP_OVERFLOW and the host re-runs it on
//    astar2d.hip);
//  - CPython _siftup's child-choice bits (bit(p) = !(heap[2p+1] < heap[2p+2])) live in REGISTERS:
//    levels 0-5 one bit per lane (lane u = node u, 1-based), levels 6-11 one 64-bit word per lane
//    (lane j = the 6-level block under node 64 + j), level 12 one 64-bit word per lane (lane j = the
//    64 level-12 nodes under block j).  A heappop's leaf is two ballots (each lane tests its own leaf
//    of a 6-level block against masks fixed per lane) and two readlanes -- no memory round trip;
//  - every heap operation is one rotation of one root-to-node path (tests/test_heap_path_form.py):
//    lane L holds path level L; one LDS load round (the path and its siblings), one ballot for the
//    boundary level, a DPP shift, the stores, and the choice bits of the changed levels' parents,
//    rebuilt as ballots into the register tiers;
//  - small grids (the README grid) keep occupancy, CLOSED motions and G in LDS too (LDSG), so an
//    expansion's 3x3 round is an LDS round; larger grids (C2's 1024^2) read them from HBM/L2, issued
//    before the heap pop so the two overlap, with the per-slot epoch cell states of astar2d_mq.hip.
// Control flow is uniform (one query per wave): pops and pushes take scalar branches, not selects.
#include "pmp_internal.h"

namespace {

constexpr double kSqrt2 = 1.4142135623730951;  // math.sqrt(2) == math.hypot(1, 1)
constexpr int kSqCapMax = 16383;                // heap positions 0..16382: levels 0..13
constexpr int kSqMinCap = 1024;                 // the smallest LDS heap worth this engine

// motions in the order of env.py:52-55: (-1,0),(-1,1),(0,1),(1,1),(1,0),(1,-1),(0,-1),(-1,-1)
constexpr uint32_t kMx1 = 0x1A90u, kMy1 = 0x01A9u;
__device__ __forceinline__ int mot_x(int d) { return (int)((kMx1 >> (2 * d)) & 3u) - 1; }
__device__ __forceinline__ int mot_y(int d) { return (int)((kMy1 >> (2 * d)) & 3u) - 1; }

// entry code: goal-relative offset and the motion that reached the cell (8 = the start)
__device__ __forceinline__ uint32_t pack_cm(int dx, int dy, int dir)
{
    return ((uint32_t)dx << 18) | (((uint32_t)dy & 0x3FFFu) << 4) | (uint32_t)dir;
}
__device__ __forceinline__ int cm_dx(uint32_t cm) { return (int)cm >> 18; }
__device__ __forceinline__ int cm_dy(uint32_t cm) { return (int)(cm << 14) >> 18; }
__device__ __forceinline__ int cm_dir(uint32_t cm) { return (int)(cm & 15u); }
// HEUR: 0 euclidean, 1 manhattan (graph_search.py:41-44), 2 zero (Dijkstra); the h order key
template <int HEUR>
__device__ __forceinline__ uint32_t hkey(uint32_t cm)
{
    if (HEUR == 2) return 0u;
    const int dx = cm_dx(cm), dy = cm_dy(cm);
    if (HEUR == 1) return (uint32_t)(abs(dx) + abs(dy));
    return (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
}
template <int HEUR>
__device__ __forceinline__ double h_of_key(uint32_t hk)
{
    return HEUR == 2 ? 0.0 : (HEUR == 1 ? (double)hk : __dsqrt_rn((double)hk));
}
// Node.__lt__ (node.py:51-54): (g + h, h)
__device__ __forceinline__ bool key_lt(double fa, uint32_t ka, double fb, uint32_t kb)
{
    return (fa < fb) | ((fa == fb) & (ka < kb));
}

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

__device__ __forceinline__ uint64_t rl64(uint64_t v, int j)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), j) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)v, j);
}
// lane j's copy of v replaced by the (wave-uniform) val
__device__ __forceinline__ uint64_t wl64(uint64_t v, uint64_t val, int j) { return lane_id() == j ? val : v; }
// lane + 1 / lane - 1 of my 16-lane row (the path lives in row 0)
__device__ __forceinline__ uint32_t shl1(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t shr1(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false); }
__device__ __forceinline__ double shl1f(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)shl1((uint32_t)(b >> 32)) << 32) | shl1((uint32_t)b));
}
__device__ __forceinline__ double shr1f(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)shr1((uint32_t)(b >> 32)) << 32) | shr1((uint32_t)b));
}
__device__ __forceinline__ void wave_sync_mem() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// LDS grid block of the LDSG variant: occupancy words, one motion byte per cell (0 = open), G
__host__ __device__ constexpr size_t sq_occ_bytes(size_t ncell) { return (((ncell + 31) / 32) * 4 + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t sq_cst_bytes(size_t ncell) { return (ncell + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t sq_grid_bytes(size_t ncell) { return sq_occ_bytes(ncell) + sq_cst_bytes(ncell) + ncell * 8; }
constexpr int kSqLdsBytes = 160 * 1024 - 256;

// The heap and its choice-bit tiers (registers).  n = heap size.
struct SqHeap {
    lds_f64* F;
    lds_u32* C;
    uint32_t t0;  // lane u (1..63): bit of node u (levels 0-5)
    uint64_t w1;  // lane j: bits of the 6-level block rooted at node 64 + j (bit r = block node r)
    uint64_t w2;  // lane j: bits of level-12 nodes 4096 + 64 j + i (bit i)
};

// per-lane constants
struct SqLane {
    int lane, lk;   // lane, floor(log2(lane)) (lane >= 1)
    uint64_t M, V;  // leaf `lane` of a 6-level block: the block nodes on its path, and their bits
};

// _siftup's leaf for a heappop on a heap of n (>= 1) entries: 1-based node Q at level Kd
__device__ __forceinline__ void sq_pop_leaf(const SqHeap& h, const SqLane& c, int n, uint32_t& Q, int& Kd)
{
    const int D = 31 - __clz(n);  // level of the last position (node n)
    if (D == 0) {
        Q = 1u;
        Kd = 0;
        return;
    }
    const uint64_t w0 = __ballot(h.t0 != 0u);
    const int j0 = __ffsll((long long)__ballot(((w0 ^ c.V) & c.M) == 0ull)) - 1;
    uint32_t full = (1u << 13) | ((uint32_t)j0 << 7);  // the level-13 node along the bits
    if (D >= 7) {
        const uint64_t w1 = rl64(h.w1, j0);
        const int j1 = __ffsll((long long)__ballot(((w1 ^ c.V) & c.M) == 0ull)) - 1;
        full |= (uint32_t)j1 << 1;
        if (D >= 13) full |= (uint32_t)(rl64(h.w2, j0) >> j1) & 1u;
    }
    const uint32_t u = full >> (14 - D);  // node at level D - 1
    if (2u * u <= (uint32_t)n) {
        const uint32_t ch = (2u * u + 1u <= (uint32_t)n) ? (full >> (13 - D)) & 1u : 0u;
        Q = 2u * u + ch;
        Kd = D;
    } else {
        Q = u;
        Kd = D - 1;
    }
}

// CPython _siftup's choice bit of the parent of `child` (a position) whose new content is v and
// whose sibling holds s: bit = !(left < right), odd positions are left children
__device__ __forceinline__ bool choice_bit(int child, double vf, uint32_t vk, double sf, uint32_t sk)
{
    return (child & 1) ? !key_lt(vf, vk, sf, sk) : !key_lt(sf, sk, vf, vk);
}

// Rebuild the choice bits of the path nodes whose bits changed.  Lane L (1..Kd) of the operation
// produced its parent's (level L - 1) new bit: bit L of S, valid where bit L of U is set.
__device__ __forceinline__ void sq_bits(SqHeap& h, const SqLane& c, uint32_t Q, int Kd, uint64_t S, uint64_t U)
{
    if (U & 0x7Eull) {  // levels 0-5: lane k = node k
        const int sh = Kd - c.lk;
        const bool on = c.lane >= 1 && sh >= 1 && (Q >> sh) == (uint32_t)c.lane && ((U >> (c.lk + 1)) & 1ull);
        h.t0 = on ? (uint32_t)((S >> (c.lk + 1)) & 1ull) : h.t0;
    }
    if (U & (0x3Full << 7)) {  // levels 6-11: one block word, lane k = block node k
        const int j = (int)(Q >> (Kd - 6)) - 64;
        const uint64_t w = rl64(h.w1, j);
        const int l = 6 + c.lk;
        const int sh = Kd - l;
        const bool on = c.lane >= 1 && sh >= 1 && (((Q >> sh) ^ (uint32_t)c.lane) & ((1u << c.lk) - 1u)) == 0u &&
                        ((U >> (l + 1)) & 1ull);
        const bool bit = on ? ((S >> (l + 1)) & 1ull) : ((w >> c.lane) & 1ull);
        h.w1 = wl64(h.w1, __ballot(c.lane >= 1 && bit), j);
    }
    if ((U >> 13) & 1ull) {  // level 12
        const uint32_t u12 = Q >> (Kd - 12);
        const int j = (int)(u12 >> 6) - 64, i = (int)(u12 & 63u);
        uint64_t w = rl64(h.w2, j);
        w = (w & ~(1ull << i)) | (((S >> 13) & 1ull) << i);
        h.w2 = wl64(h.w2, w, j);
    }
}

// Set the choice bit of one node (1-based u, wave-uniform) -- a trivial push's parent
__device__ __forceinline__ void sq_bit1(SqHeap& h, uint32_t u, uint32_t bit)
{
    const int l = 31 - __clz((int)u);
    if (l <= 5) {
        h.t0 = lane_id() == (int)u ? bit : h.t0;
    } else if (l <= 11) {
        const int r = l - 6;
        const int j = (int)(u >> r) - 64;
        const uint32_t k = (1u << r) | (u & ((1u << r) - 1u));
        const uint64_t w = rl64(h.w1, j);
        h.w1 = wl64(h.w1, (w & ~(1ull << k)) | ((uint64_t)bit << k), j);
    } else {
        const int j = (int)(u >> 6) - 64;
        const uint32_t i = u & 63u;
        const uint64_t w = rl64(h.w2, j);
        h.w2 = wl64(h.w2, (w & ~(1ull << i)) | ((uint64_t)bit << i), j);
    }
}
__device__ __forceinline__ double uni_f64(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)(uint32_t)uni((int)(b >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)b));
}

// One heap operation on the path q_L = (Q >> (Kd - L)) - 1 (lane L <-> level L, row 0):
//  pop  (heap already shrunk to n; X = the old last element): the prefix of levels 1..b with
//       !(X < heap[q_L]) moves up one level, X lands at level b; lane 15 loads the new last;
//  push (X = the item at position n = q_Kd, n = the size before it): the levels b..Kd-1 with
//       X < heap[q_L] move down one level, X lands at level b.
template <bool POP, int HEUR>
__device__ __forceinline__ void sq_op(SqHeap& h, const SqLane& c, uint32_t Q, int Kd, int n, double Xf, uint32_t Xc,
                                      double& rootf, uint32_t& rootc, double& lastf, uint32_t& lastc)
{
    const int L = c.lane;
    const uint32_t Xk = hkey<HEUR>(Xc);
    const bool lvl = L <= Kd;
    const int q = lvl ? (int)(Q >> (Kd - L)) - 1 : 0;
    const bool lda = POP ? (L >= 1 && lvl) : (L < Kd);
    const int ai = lda ? q : ((POP && L == 15) ? n - 1 : 0);
    const int si = ((q - 1) ^ 1) + 1;
    const bool hass = L >= 1 && lvl && si < n;
    const double Vf = h.F[ai];
    const uint32_t Vc = h.C[ai];
    const double Sf = h.F[hass ? si : 0];
    const uint32_t Sc = h.C[hass ? si : 0];
    __builtin_amdgcn_sched_barrier(0);  // all four loads in flight before the first use
    const uint32_t Vk = hkey<HEUR>(Vc);
    // the boundary level b
    const bool lt = key_lt(Xf, Xk, Vf, Vk);
    const int cnt = __popcll(__ballot(lda && (POP ? !lt : lt)));
    const int b = POP ? cnt : Kd - cnt;
    const bool atb = L == b, shift = POP ? L < b : (L > b && lvl);
    double nf;
    uint32_t nc;
    if (POP) {
        const double uf = shl1f(Vf);
        const uint32_t uc = shl1(Vc);
        nf = atb ? Xf : (shift ? uf : Vf);
        nc = atb ? Xc : (shift ? uc : Vc);
    } else {
        const double df = shr1f(Vf);
        const uint32_t dc = shr1(Vc);
        nf = atb ? Xf : (shift ? df : Vf);
        nc = atb ? Xc : (shift ? dc : Vc);
    }
    const bool chg = POP ? L <= b : (L >= b && lvl);
    if (chg) {
        h.F[q] = nf;
        h.C[q] = nc;
    }
    // the bits of the changed levels' parents: lane L from its new content and its sibling
    const bool upd = chg && hass;
    const bool bit = choice_bit(q, nf, hkey<HEUR>(nc), Sf, hkey<HEUR>(Sc));
    const uint64_t U = __ballot(upd), S = __ballot(upd && bit);
    sq_bits(h, c, Q, Kd, S, U);
    // root = level 0's new content; last: a pop's heap[n - 1] unless X stayed on it, a push's heap[n]
    rootf = rl_f64(nf, 0);
    rootc = rl_u32(nc, 0);
    if (POP) {
        if (!(b == Kd && Q == (uint32_t)n)) {
            lastf = rl_f64(Vf, 15);
            lastc = rl_u32(Vc, 15);
        }
    } else {
        lastf = rl_f64(nf, Kd);
        lastc = rl_u32(nc, Kd);
    }
    wave_sync_mem();
}

template <bool LDSG> struct SqGrid {
    typedef const uint32_t* Occ;
    typedef uint8_t* Cst;
    typedef double* Gv;
};
template <> struct SqGrid<true> {
    typedef const lds_u32* Occ;
    typedef lds_u8* Cst;
    typedef lds_f64* Gv;
};

// One query per workgroup (blockIdx.x); LDS: F[cap], C[cap][, LDSG grid block].
template <int HEUR, bool GZERO, bool LDSG>
__global__ __launch_bounds__(64) void astar2d_sq_kernel(
    const uint32_t* __restrict__ occ, int W, int H, const int32_t* __restrict__ start_xy,
    const int32_t* __restrict__ goal_xy, double* __restrict__ cost_out, int32_t* __restrict__ path_len_out,
    uint32_t* __restrict__ path_out, int path_cap, int32_t* __restrict__ nexp_out, uint32_t* __restrict__ expand_out,
    int expand_cap, int64_t* __restrict__ counters, int32_t* __restrict__ status_out, int heap_cap, int lds_cap,
    uint8_t* __restrict__ cst_all, size_t cst_slot_bytes, double* __restrict__ G_all, uint32_t* __restrict__ epoch_all,
    unsigned long long* __restrict__ span)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int q = blockIdx.x;
    span_begin(span);
    SqLane c;
    c.lane = lane;
    c.lk = lane >= 1 ? 31 - __clz(lane) : 0;
    c.M = c.V = 0ull;
    {
        uint32_t r = 1u;
        for (int k = 0; k < 6; k++) {
            const uint32_t bt = (uint32_t)(lane >> (5 - k)) & 1u;
            c.M |= 1ull << r;
            c.V |= (uint64_t)bt << r;
            r = 2u * r + bt;
        }
    }
    SqHeap hp;
    hp.F = (lds_f64*)smem;
    hp.C = (lds_u32*)(smem + (size_t)8 * lds_cap);
    hp.t0 = 0u;
    hp.w1 = hp.w2 = 0ull;

    const size_t ncell = (size_t)W * (size_t)H;
    typename SqGrid<LDSG>::Occ occg;
    typename SqGrid<LDSG>::Cst cst;
    typename SqGrid<LDSG>::Gv G;
    uint32_t ep = 1u;
    // cell-state byte of (x, y): row-major, in the LDS grid block and in the per-slot HBM states it
    // shares with the multi-query engine (which tiles them, cst_idx: a query only reads bytes of its
    // own epoch, written by itself, so engines with different layouts can share a slot; the tiled
    // index costs this latency-bound single wave 4 % on a C2 query and gains it nothing -- one query's
    // states stay in L2)
    auto cidx = [&](int x, int y) -> uint32_t { return (uint32_t)x * (uint32_t)H + (uint32_t)y; };
    if constexpr (LDSG) {
        unsigned char* gb = smem + (size_t)12 * lds_cap;
        lds_u32* ow = (lds_u32*)gb;
        const uint32_t nw = (uint32_t)((ncell + 31) / 32);
        for (uint32_t i = lane; i < nw; i += 64) ow[i] = occ[i];
        occg = ow;
        cst = (lds_u8*)(gb + sq_occ_bytes(ncell));
        lds_u32* cw = (lds_u32*)cst;
        for (uint32_t i = lane; i < sq_cst_bytes(ncell) / 4; i += 64) cw[i] = 0u;
        G = (lds_f64*)(gb + sq_occ_bytes(ncell) + sq_cst_bytes(ncell));
    } else {
        occg = occ;
        cst = cst_all + (size_t)q * cst_slot_bytes;
        G = G_all + (size_t)q * g_slot_cells(W, H);  // (the shared slot stride; row-major inside)
        // next epoch; every 15th query (and a fresh slot, epoch 0) clears the cell states
        ep = epoch_all[q];
        if (ep == 0u || ep >= 15u) {
            uint4* c4 = reinterpret_cast<uint4*>(cst);
            for (size_t i = lane; i < cst_slot_bytes / 16; i += 64) c4[i] = make_uint4(0u, 0u, 0u, 0u);
            ep = 1u;
        } else {
            ep++;
        }
    }
    wave_sync_mem();

    // per-lane constants of the 3x3 round: lanes 0..8 occupancy of cell (x + i/3 - 1, y + i%3 - 1),
    // lanes 9..17 its motion byte, lane 18 G[parent]
    const int blk_i = lane < 9 ? lane : (lane < 18 ? lane - 9 : 4);
    const int blk_dx = blk_i / 3 - 1, blk_dy = blk_i % 3 - 1;
    // lane m < 8 is motion m: offset, cost, the 3x3 cells isCollision needs free (graph_search.py:66-87)
    const int mo = lane & 7;
    const int mx = mot_x(mo), my = mot_y(mo);
    const double mcost = GZERO ? 0.0 : ((mo & 1) ? kSqrt2 : 1.0);
    uint32_t need = 16u | (1u << ((mx + 1) * 3 + (my + 1)));
    if (mo & 1) need |= (1u << (3 + (my + 1))) | (1u << ((mx + 1) * 3 + 1));
    const uint32_t self_bit = 1u << ((mx + 1) * 3 + (my + 1));

    const int sx = uni(start_xy[2 * q]), sy = uni(start_xy[2 * q + 1]);
    const int gx = uni(goal_xy[2 * q]), gy = uni(goal_xy[2 * q + 1]);
    const bool s_in = (unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H;
    const bool g_in = (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
    int st = PMP_NO_PATH;
    double goal_cost = 0.0;
    int plen = 0, nexp = 0, maxn = 1;
    int64_t npush = 1, npop = 0;
    if (!s_in || !g_in) {  // outside the grid: blocked -> no neighbours -> no path
        nexp = s_in ? 1 : 0;
        npop = 1;
        if (lane == 0) {
            status_out[q] = PMP_NO_PATH;
            cost_out[q] = 0.0;
            path_len_out[q] = 0;
            nexp_out[q] = nexp;
            if (counters) {
                counters[4 * q] = 1; counters[4 * q + 1] = 1; counters[4 * q + 2] = nexp; counters[4 * q + 3] = 1;
            }
            if (!LDSG) epoch_all[q] = ep;
        }
        span_end(span);
        return;
    }

    // heap[0] = Node(start, start, 0, 0), key (0, h = 0)
    double rootf = 0.0, lastf = 0.0;
    uint32_t rootc = pack_cm(0, 0, 8), lastc = rootc;
    if (lane == 0) {
        hp.F[0] = rootf;
        hp.C[0] = rootc;
    }
    wave_sync_mem();
    int n = 1;
#ifdef PMP_STAMPS  // diagnostic build: cycles in the pop, the 3x3 wait and the pushes, per query
    uint64_t cyc_pop = 0, cyc_wait = 0, cyc_push = 0;
    const uint64_t cyc_q0 = __builtin_amdgcn_s_memtime();
#define SQ_STAMP(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#else
#define SQ_STAMP(t)
#endif

    while (n > 0) {
        SQ_STAMP(ts0);
        // ---- heappop (a_star.py:54): the popped node is the root
        const uint32_t ncm = rootc;
        npop++;
        n -= 1;
        const int ndir = cm_dir(ncm);
        const int x = ndir == 8 ? sx : gx - cm_dx(ncm);
        const int y = ndir == 8 ? sy : gy - cm_dy(ncm);
        const uint32_t nlin = (uint32_t)x * (uint32_t)H + (uint32_t)y;
        // the 3x3 round, issued before the heap pop so the two overlap
        uint32_t ow, cb;
        bool blk_in;
        double gpar = 0.0;
        {
            const int cx = x + blk_dx, cy = y + blk_dy;
            blk_in = lane < 18 && (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
            const uint32_t ci = blk_in ? (uint32_t)cx * (uint32_t)H + (uint32_t)cy : 0u;
            ow = occg[ci >> 5] >> (ci & 31u);
            cb = cst[blk_in ? cidx(cx, cy) : 0u];
            const uint32_t gi = (!GZERO && lane == 18 && ndir < 8) ? nlin - (uint32_t)(mot_x(ndir) * H + mot_y(ndir)) : 0u;
            if (!GZERO) gpar = G[gi];
        }
        if (n > 0) {
            uint32_t Q;
            int Kd;
            sq_pop_leaf(hp, c, n, Q, Kd);
            Q = (uint32_t)uni((int)Q);
            Kd = uni(Kd);
            sq_op<true, HEUR>(hp, c, Q, Kd, n, lastf, lastc, rootf, rootc, lastf, lastc);
        }
        SQ_STAMP(ts1);
        // 3x3 masks: bit k = cell (x + k/3 - 1, y + k%3 - 1); the node is k = 4
        const uint32_t occ9 = (uint32_t)__ballot(lane < 9 && (!blk_in || (ow & 1u))) & 0x1FFu;
        const bool closed = LDSG ? cb != 0u : ((cb >> 4) == ep && (cb & 15u) != 0u);
        const uint32_t cls9 = (uint32_t)(__ballot(lane >= 9 && lane < 18 && blk_in && closed) >> 9) & 0x1FFu;
#ifdef PMP_STAMPS
        {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            SQ_STAMP(ts2);
            cyc_pop += ts1 - ts0;
            cyc_wait += ts2 - ts1;
        }
#endif
        if (cls9 & 16u) continue;  // node.current in CLOSED (a_star.py:57-58)

        // CLOSED[node.current] = node (a_star.py:82)
        const double gnode = (GZERO || ndir == 8) ? 0.0 : rl_f64(gpar, 18) + ((ndir & 1) ? kSqrt2 : 1.0);
        if (lane == 0) cst[cidx(x, y)] = (uint8_t)(LDSG ? (uint32_t)(ndir + 1) : ((ep << 4) | (uint32_t)(ndir + 1)));
        if (!GZERO && lane == 1) G[nlin] = gnode;
        if (lane == 2 && expand_out && nexp < expand_cap) expand_out[(size_t)q * expand_cap + nexp] = nlin | ((uint32_t)ndir << 28);
        nexp++;

        if (x == gx && y == gy) {  // goal found (a_star.py:61-64): extractPath, goal -> start
            st = PMP_FOUND;
            wave_sync_mem();
            if (lane == 0) {
                int px = x, py = y;
                double cost = 0.0;
                int len = 0;
                uint32_t* pth = path_out + (size_t)q * path_cap;
                for (;;) {
                    const uint32_t li = (uint32_t)px * (uint32_t)H + (uint32_t)py;
                    if (len < path_cap) pth[len] = li;
                    len++;
                    if (px == sx && py == sy) break;
                    const int d = (int)(cst[cidx(px, py)] & 15u) - 1;
                    cost += (d & 1) ? kSqrt2 : 1.0;
                    px -= mot_x(d);
                    py -= mot_y(d);
                }
                goal_cost = cost;
                plen = len;
            }
            break;
        }

        // ---- getNeighbor + the pushes in motion order; push the goal and stop (a_star.py:66-80)
        const int ndx = gx - x - mx, ndy = gy - y - my;
        const bool nb_ok = lane < 8 && (occ9 & need) == 0u && (cls9 & self_bit) == 0u;
        uint64_t vm = __ballot(nb_ok) & 0xFFull;
        const uint64_t gm = __ballot(nb_ok && ndx == 0 && ndy == 0) & 0xFFull;
        if (gm) vm &= (gm << 1) - 1ull;
        const uint32_t icm = pack_cm(ndx, ndy, mo);
        const double ifv = gnode + mcost + h_of_key<HEUR>(hkey<HEUR>(icm));
        if (n + __popcll(vm) > heap_cap) {  // a push would find n >= heap_cap
            st = PMP_CAP_OVERFLOW;
            break;
        }
        // The leading run of trivial pushes (CPython's _siftdown stops at once: the item is not less
        // than its parent, a position < n the run does not change) is stored together: the parents
        // of the positions n, n + 1, ... load in one LDS round
        if (vm && n > 0) {
            const uint32_t below = (uint32_t)vm & ((1u << mo) - 1u);
            const int pos = n + __popc(below);
            const int pp = (pos - 1) >> 1;
            const bool mine = lane < 8 && ((vm >> mo) & 1ull);
            const double pf = hp.F[mine ? pp : 0];
            const uint32_t pc = hp.C[mine ? pp : 0];
            const uint32_t ik = hkey<HEUR>(icm);
            const bool triv = mine && pp < n && !key_lt(ifv, ik, pf, hkey<HEUR>(pc));
            const uint64_t nt = vm & ~(__ballot(triv) & 0xFFull);
            const uint64_t run = nt ? vm & ((nt & (0ull - nt)) - 1ull) : vm;
            if (run) {
                const bool inrun = lane < 8 && ((run >> mo) & 1ull);
                if (inrun) {
                    hp.F[pos] = ifv;
                    hp.C[pos] = icm;
                }
                // a right child (even position) sets its parent's bit against its left sibling: the
                // previous item of the run, or `last` for the first
                const int prev = below ? 31 - __clz(below) : 0;
                const double pvf = __shfl(ifv, prev);
                const uint32_t pvc = (uint32_t)__shfl((int)icm, prev);
                const double leftf = below ? pvf : lastf;
                const uint32_t leftk = below ? hkey<HEUR>(pvc) : hkey<HEUR>(lastc);
                const uint64_t rb = __ballot(inrun && !key_lt(leftf, leftk, ifv, ik));
                uint64_t rc = __ballot(inrun && (pos & 1) == 0);
                while (rc) {
                    const int m = __ffsll((long long)rc) - 1;
                    rc &= rc - 1ull;
                    sq_bit1(hp, (uint32_t)__builtin_amdgcn_readlane(pp, m) + 1u, (uint32_t)((rb >> m) & 1ull));
                }
                const int top = 63 - __clzll((long long)run);
                lastf = rl_f64(ifv, top);
                lastc = rl_u32(icm, top);
                const int k = __popcll(run);
                n += k;
                npush += k;
                vm &= ~run;
                wave_sync_mem();
            }
        }
        while (vm) {
            const int m = __ffsll((long long)vm) - 1;
            vm &= vm - 1ull;
            const double Xf = rl_f64(ifv, m);
            const uint32_t Xc = rl_u32(icm, m);
            // CPython's _siftdown stops at once when the item is not less than its parent (most
            // pushes): store it, and set its parent's bit against its left sibling (= last)
            const int pp = n > 0 ? (n - 1) >> 1 : 0;
            const double pf = uni_f64(hp.F[pp]);
            const uint32_t pc = (uint32_t)uni((int)hp.C[pp]);
            const uint32_t Xk = hkey<HEUR>(Xc);
            if (n > 0 && !key_lt(Xf, Xk, pf, hkey<HEUR>(pc))) {
                if (lane == 0) {
                    hp.F[n] = Xf;
                    hp.C[n] = Xc;
                }
                if ((n & 1) == 0) sq_bit1(hp, (uint32_t)pp + 1u, !key_lt(lastf, hkey<HEUR>(lastc), Xf, Xk) ? 1u : 0u);
                lastf = Xf;
                lastc = Xc;
                wave_sync_mem();
            } else {
                const uint32_t Q = (uint32_t)n + 1u;
                const int Kd = 31 - __clz((int)Q);
                sq_op<false, HEUR>(hp, c, Q, Kd, n, Xf, Xc, rootf, rootc, lastf, lastc);
            }
            n++;
            npush++;
        }
        if (n > maxn) maxn = n;
#ifdef PMP_STAMPS
        {
            SQ_STAMP(ts3);
            cyc_push += ts3 - ts1;
        }
#endif
    }

    if (lane == 0) {
        int s = st;
        if (s == PMP_FOUND && plen > path_cap) s = PMP_PATH_OVERFLOW;
        status_out[q] = s;
        cost_out[q] = st == PMP_FOUND ? goal_cost : 0.0;
        path_len_out[q] = st == PMP_FOUND ? plen : 0;
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
        if (!LDSG) epoch_all[q] = ep;
    }
    span_end(span);
}
#undef SQ_STAMP

bool sq_ldsg(size_t ncell) { return sq_grid_bytes(ncell) + (size_t)12 * kSqMinCap <= (size_t)kSqLdsBytes; }

}  // namespace

// Heap positions the single-query engine holds in LDS for a W x H grid (0: none worth it).
extern "C" int pmp_astar2d_sq_cap(int W, int H)
{
    const size_t ncell = (size_t)W * H;
    const size_t grid = sq_ldsg(ncell) ? sq_grid_bytes(ncell) : 0;
    const long long cap = ((long long)kSqLdsBytes - (long long)grid) / 12;
    if (cap < kSqMinCap) return 0;
    return cap > kSqCapMax ? kSqCapMax : (int)(cap & ~15ll);
}

// One workgroup per query; heap_cap <= pmp_astar2d_sq_cap(W, H).
int pmp_astar2d_sq_launch(pmp_ctx* ctx, hipStream_t s, int algo, const uint32_t* occ_bits, int W, int H, int heuristic,
                          const int32_t* start_xy, const int32_t* goal_xy, int nq, int heap_cap, double* cost,
                          int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                          int expand_cap, int64_t* counters, int32_t* status)
{
    const int cap = pmp_astar2d_sq_cap(W, H);
    if (cap == 0 || heap_cap < 1 || heap_cap > cap)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_sq_launch: heap capacity outside the single-query engine's");
    const size_t ncell = (size_t)W * H;
    const bool ldsg = sq_ldsg(ncell);
    const int lds_cap = (heap_cap + 15) & ~15;
    uint8_t* cstp = nullptr;
    size_t cst_bytes = 0;
    double* G = nullptr;
    uint32_t* ep = nullptr;
    if (!ldsg) {
        const int rc = pmp_astar2d_slot_scratch(ctx, s, (size_t)nq, W, H, &cstp, &cst_bytes, &G, &ep);
        if (rc) return rc;
    }
    const size_t lds = (size_t)12 * lds_cap + (ldsg ? sq_grid_bytes(ncell) : 0);
#define SQ_LAUNCH(HE, GZ, LG)                                                                                        \
    hipLaunchKernelGGL((astar2d_sq_kernel<HE, GZ, LG>), dim3(nq), dim3(64), lds, s, occ_bits, W, H, start_xy, goal_xy, \
                       cost, path_len, path, path_cap, n_expanded, expand, expand_cap, counters, status, heap_cap,      \
                       lds_cap, cstp, cst_bytes, G, ep, ctx->span)
    const int he = algo == PMP_ALGO_DIJKSTRA ? 2 : heuristic;
    const bool gz = algo == PMP_ALGO_GBFS;
    if (ldsg) {
        if (gz) { if (he == 1) SQ_LAUNCH(1, true, true); else SQ_LAUNCH(0, true, true); }
        else if (he == 2) SQ_LAUNCH(2, false, true);
        else if (he == 1) SQ_LAUNCH(1, false, true);
        else SQ_LAUNCH(0, false, true);
    } else {
        if (gz) { if (he == 1) SQ_LAUNCH(1, true, false); else SQ_LAUNCH(0, true, false); }
        else if (he == 2) SQ_LAUNCH(2, false, false);
        else if (he == 1) SQ_LAUNCH(1, false, false);
        else SQ_LAUNCH(0, false, false);
    }
#undef SQ_LAUNCH
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
