// Batched LPA* in 3D for gfx950, exact with LPAStar3D (global_planner/graph_search/lpa_star3d.py:40-225):
// plan() (:78-82: computeShortestPath :127-145 + extractPath :185-225) and any number of
// apply_change(coord, blocked) rounds (:93-124) per query, over Grid3D with GraphSearcher3D's
// asymmetric isCollision (graph_search_3d.py:66-107).
//
// U is the reference's Python list, kept element for element:
//   * min(U, key) = the FIRST minimal key in list order (list `<` on [k1, k2], :130);
//   * U.remove(node) shifts the tail left (the list never holds a node twice: updateVertex removes
//     before it pushes, :154-157);
//   * heapq.heappush appends and sifts with CPython _siftdown on whatever order the list has.
// U lives in LDS (one wave per query, 8 per CU; positions past the LDS share spill to HBM), so the
// scans, shifts and sifts are LDS rounds.  g / rhs per voxel stay in HBM.
//
// One expansion touches one 5x5x5 block: updateVertex never changes g, so after the expanded
// node's own g update every rhs the expansion recomputes (the node's and its 26 neighbours') reads
// g values of that block, staged in LDS in two load rounds, and the 27 rhs minima (26 candidates
// each, cost(n, node) with isCollision(n, node)) are computed lane-parallel.  The membership of the
// 27 voxels in U comes from one scan; the sequential remove / push of updateVertex in motion order
// (:145, :154-157) then only adjusts the 27 tracked positions (a remove shifts the ones past it, a
// push's sift moves its ancestor chain).
//
// start == goal: map[goal] overwrites map[start] (:62-63), the start object is detached, and the
// reference's result is fixed: plan() expands it once and returns (0.0, [goal]); every
// apply_change then expands nothing.
#include <algorithm>
#include "pmp_internal.h"

namespace {

constexpr int kMaxDim = 256;
// Write-traffic attribution (dev builds, tools/build_variant.sh): every store of the selected
// categories is issued twice, the copy into a mirror of the worker's arrays, so the extra WRITE_SIZE
// over the plain build is that category's traffic.  Bits: 1 U's spilled positions (shifts, pushes),
// 2 the g / rhs values, 4 the written-this-query bits (ORs and the per-query clear).
#ifndef PMP_L3_MIRROR
#define PMP_L3_MIRROR 0
#endif
constexpr int kL3Mirror = PMP_L3_MIRROR;
// Deferred removes (round 6): U.remove inside one expansion's block leaves a hole instead of shifting
// the tail; positions stay logical (the reference's list indices) and map to the physical array
// through the pending holes; the block's end closes every hole in one compaction pass.  0: the
// round-5 form (every remove shifts the tail at once).
#ifndef PMP_L3_DEFER
#define PMP_L3_DEFER 1
#endif
constexpr bool kDefer = PMP_L3_DEFER != 0;
constexpr double kInf = __builtin_huge_val();

__device__ __constant__ int8_t c_m[26][3] = {
    {-1, 0, 0}, {-1, 1, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0}, {1, -1, 0}, {0, -1, 0}, {-1, -1, 0},
    {0, 0, 1}, {0, 0, -1},
    {-1, 0, 1}, {-1, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, -1, 1}, {-1, -1, 1},
    {-1, 0, -1}, {-1, 1, -1}, {0, 1, -1}, {1, 1, -1}, {1, 0, -1}, {1, -1, -1}, {0, -1, -1}, {-1, -1, -1}};

// the same table as a compile-time constant (indexed only by unrolled loop counters)
constexpr int8_t kM[26][3] = {
    {-1, 0, 0}, {-1, 1, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0}, {1, -1, 0}, {0, -1, 0}, {-1, -1, 0},
    {0, 0, 1}, {0, 0, -1},
    {-1, 0, 1}, {-1, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, -1, 1}, {-1, -1, 1},
    {-1, 0, -1}, {-1, 1, -1}, {0, 1, -1}, {1, 1, -1}, {1, 0, -1}, {1, -1, -1}, {0, -1, -1}, {-1, -1, -1}};

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef __attribute__((address_space(3))) double lds_f64;

__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// list `<` on [k1, k2]; branch-free (the short-circuit form compiled to exec-mask branches)
__device__ __forceinline__ bool key_lt(double a1, double a2, double b1, double b2)
{
    return (a1 < b1) | ((a1 == b1) & (a2 < b2));
}

// c / d for 0 <= c < 2^24 through an f32 reciprocal (error <= 1 before the correction): a handful
// of instructions instead of an integer division
__device__ __forceinline__ int fdiv(int c, int d, float inv)
{
    int q = (int)((float)c * inv);
    const int r = c - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

struct Geo {
    int X, Y, Z;
    float invY, invZ;
    __device__ __forceinline__ bool in(int x, int y, int z) const
    {
        return (unsigned)x < (unsigned)X && (unsigned)y < (unsigned)Y && (unsigned)z < (unsigned)Z;
    }
    __device__ __forceinline__ int id(int x, int y, int z) const { return (x * Y + y) * Z + z; }
    __device__ __forceinline__ void xyz(int c, int& x, int& y, int& z) const
    {
        const int r = fdiv(c, Z, invZ);
        z = c - r * Z;
        x = fdiv(r, Y, invY);
        y = r - x * Y;
    }
};

// 125-bit masks over the 5x5x5 block around a centre (bit (x*5 + y)*5 + z of block coordinates
// 0..4), wave-uniform: "in the map" and "an obstacle"
struct Mask125 {
    uint64_t lo, hi;
    __device__ __forceinline__ bool at(int b) const { return b < 64 ? (lo >> b) & 1ull : (hi >> (b - 64)) & 1ull; }
};

// working occupancy (apply_change edits it): LDS when it fits, else the worker's HBM copy;
// `p in self.obstacles` is false outside the grid
struct Occ {
    lds_u32* l;
    uint32_t* g;
    bool lds;
    Geo geo;
    __device__ __forceinline__ bool at(int x, int y, int z) const
    {
        if (!geo.in(x, y, z)) return false;
        const uint32_t c = (uint32_t)geo.id(x, y, z);
        const uint32_t w = lds ? l[c >> 5] : g[c >> 5];
        return (w >> (c & 31)) & 1u;
    }
    // isCollision(node1 = (x1,y1,z1), node2) for neighbouring voxels
    __device__ __forceinline__ bool coll(int x1, int y1, int z1, int x2, int y2, int z2) const
    {
        if (at(x1, y1, z1) || at(x2, y2, z2)) return true;
        const int dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
        const int ch = (dx != 0) + (dy != 0) + (dz != 0);
        if (ch <= 1) return false;
        if (ch == 2) {
            if (dx != 0 && dy != 0) return at(x1 + dx, y1, z1) || at(x1, y1 + dy, z1);
            if (dx != 0 && dz != 0) return at(x1 + dx, y1, z1) || at(x1, y1, z1 + dz);
            return at(x1, y1 + dy, z1) || at(x1, y1, z1 + dz);
        }
        return at(x1 + dx, y1, z1) || at(x1, y1 + dy, z1) || at(x1, y1, z1 + dz);
    }
};

__device__ __forceinline__ double dist_unit(int dx, int dy, int dz)  // Planner3D.dist of a motion
{
    return __dsqrt_rn((double)(dx * dx + dy * dy + dz * dz));
}

// U: positions < cap in LDS, the rest in the worker's HBM arrays
struct UList {
    lds_i32* lc;
    lds_f64* l1;
    lds_f64* l2;
    int32_t* gc;
    double* g1;
    double* g2;
    int32_t* mgc;  // kL3Mirror & 1: the mirror of the spilled part
    double* mg1;
    double* mg2;
    int cap;
    int n;
    // SP = false: every position touched is < cap (pure LDS code, no vector-memory waits)
    template <bool SP>
    __device__ __forceinline__ void ld(int k, int32_t& c, double& a, double& b) const
    {
        if (!SP || k < cap) {
            c = lc[k];
            a = l1[k];
            b = l2[k];
        } else {
            c = gc[k - cap];
            a = g1[k - cap];
            b = g2[k - cap];
        }
    }
    template <bool SP>
    __device__ __forceinline__ void st(int k, int32_t c, double a, double b) const
    {
        if (!SP || k < cap) {
            lc[k] = c;
            l1[k] = a;
            l2[k] = b;
        } else {
            gc[k - cap] = c;
            g1[k - cap] = a;
            g2[k - cap] = b;
            if (kL3Mirror & 1) {
                mgc[k - cap] = c;
                mg1[k - cap] = a;
                mg2[k - cap] = b;
            }
        }
    }
};

// The 27 tracked voxels of the current block (lane b < 27 = block voxel b, 26 = the centre): their
// U positions follow every remove / push
struct Track {
    int pos;  // per lane: this lane's voxel's index in U, -1 = not in U
};

struct L3 {
    Geo geo;
    Occ occ;
    UList U;
    double* g;
    double* rhs;
    // Written-this-query bits of g / rhs (one bit per voxel, the worker's own 2 x ceil(V / 32) words in
    // HBM, L2-resident; `touch`): a voxel whose bit is clear holds the query's initial value (inf;
    // rhs(start) = 0 is written), so a query starts with no reset of the two arrays (8 B x 2 per
    // voxel, more than its whole search writes otherwise).  The bits are read beside the g / rhs
    // loads (same round) with L1-bypassing agent-scope atomic loads and set by atomic ORs, so a read
    // always sees this wave's earlier sets.  (Round 5 kept them in LDS first: the 2 KB they took from
    // U's share spilled more lists to HBM -- +50 % writes, -9 % plans/s.)
    uint32_t* gt;
    uint32_t* rt;
    double* mg;     // kL3Mirror & 2: mirrors of g / rhs
    double* mrhs;
    uint32_t* mgt;  // kL3Mirror & 4: mirrors of the bits
    uint32_t* mrt;
    bool touch;
    lds_f64* cube;  // 125 g values of the 5x5x5 block around the centre
    int lane;
    // kDefer: the holes pending in U's physical array (wave-uniform count hm <= 28 -- the popped node
    // and the 27 block voxels; lane j < hm holds hole j's boundary b_j = the live entries before it).
    // Logical position L sits at physical L + #{j : b_j <= L}.
    int hb;
    int hm;
    int start, goal;  // voxel ids
    int gx, gy, gz;
    int heur;
    int64_t nexp;
    int64_t npush;
    int maxn;
    double goal_g, goal_rhs;  // the goal's g / rhs, kept in registers for the termination test
#ifdef PMP_STAMPS
    uint64_t cyc[4];  // diagnostic build: min scan, g block + rhs minima, membership scan, updates
#define LSTAMP(v) [[maybe_unused]] const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define LSTAMP(v)
#endif

    __device__ __forceinline__ static uint32_t bw(const uint32_t* t, int c)
    {
        return __hip_atomic_load(t + (c >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ bool gw(int c) const { return !touch || ((bw(gt, c) >> (c & 31)) & 1u); }
    __device__ __forceinline__ bool rw(int c) const { return !touch || ((bw(rt, c) >> (c & 31)) & 1u); }
    __device__ __forceinline__ double g_at(int c) const { return gw(c) ? g[c] : kInf; }
    __device__ __forceinline__ void mark(uint32_t* t, int c) const
    {
        if (touch) __hip_atomic_fetch_or(t + (c >> 5), 1u << (c & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((kL3Mirror & 4) && touch)
            __hip_atomic_fetch_or((t == gt ? mgt : mrt) + (c >> 5), 1u << (c & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    __device__ __forceinline__ double hval(int x, int y, int z) const
    {
        const int dx = abs(gx - x), dy = abs(gy - y), dz = abs(gz - z);
        return heur == 1 ? (double)(dx + dy + dz) : __dsqrt_rn((double)(dx * dx + dy * dy + dz * dz));
    }

    // U.remove(U[i]): the tail moves left one slot; 4 elements per lane per round (all loads of a
    // round before its stores; a round never reads what an earlier round wrote)
    template <bool SP>
    __device__ __forceinline__ void remove_at_t(int i)
    {
        // the loads of a round are unconditional (clamped to the last element) so they issue back to
        // back with one wait; only the stores are masked
        const int last = U.n - 1;
        for (int base = i; base < last; base += 256) {
            int32_t c[4];
            double a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = base + lane + 64 * j;
                U.template ld<SP>(k < last ? k + 1 : last, c[j], a[j], b[j]);
            }
            wsync();
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = base + lane + 64 * j;
                if (k < last) U.template st<SP>(k, c[j], a[j], b[j]);
            }
            wsync();
        }
    }
    __device__ __forceinline__ void remove_at(int i, Track& t)
    {
        if (kDefer) {  // a hole at logical i: later holes' boundaries past i drop by one
            if (lane < hm && hb > i) hb -= 1;
            if (lane == hm) hb = i;
            hm += 1;
        } else if (U.n <= U.cap) {
            remove_at_t<false>(i);
        } else {
            remove_at_t<true>(i);
        }
        U.n -= 1;
        if (t.pos == i) t.pos = -1;
        else if (t.pos > i) t.pos -= 1;
    }
    // physical index of logical position L (kDefer)
    __device__ __forceinline__ int phys(int L) const
    {
        int P = L;
        for (int j = 0; j < hm; j++) P += L >= __builtin_amdgcn_readlane(hb, j) ? 1 : 0;
        return P;
    }
    // close every pending hole: logical L takes physical phys(L), ascending from the first hole, 4
    // entries per lane per round, all loads of a round before its stores (a store goes to L <= its
    // source, below every later round's sources)
    template <bool SP>
    __device__ __forceinline__ void compact_t(int from)
    {
        const int n = U.n;
        for (int base = from; base < n; base += 256) {
            int L[4], P[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = base + lane + 64 * j;
                L[j] = k < n ? k : n - 1;
                P[j] = L[j];
            }
            for (int h = 0; h < hm; h++) {
                const int bh = __builtin_amdgcn_readlane(hb, h);
#pragma unroll
                for (int j = 0; j < 4; j++) P[j] += L[j] >= bh ? 1 : 0;
            }
            int32_t c[4];
            double a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; j++) U.template ld<SP>(P[j], c[j], a[j], b[j]);
            wsync();
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (base + lane + 64 * j < n && P[j] != L[j]) U.template st<SP>(L[j], c[j], a[j], b[j]);
            wsync();
        }
    }
    __device__ __forceinline__ void compact()
    {
        if (!kDefer || hm == 0) return;
        int from = U.n;
        for (int j = 0; j < hm; j++) from = min(from, __builtin_amdgcn_readlane(hb, j));
        if (U.n + hm <= U.cap) compact_t<false>(from);
        else compact_t<true>(from);
        hm = 0;
    }

    // heapq.heappush(U, node): lane j (1..D) loads ancestor j of position n; the ancestors that move
    // down are the run of "new < ancestor" from the parent up (_siftdown stops at the first one that
    // is not greater).  `me` = this lane tracks the pushed voxel.  kDefer: lane j (0..D) maps path
    // position (np1 >> j) - 1 to its physical index first.
    template <bool SP>
    __device__ __forceinline__ int push_t(int32_t c, double k1, double k2, uint32_t np1, int& s)
    {
        const int D = 31 - __clz((int)np1);
        const bool on = lane >= 1 && lane <= D;
        const int aj = on ? (int)(np1 >> lane) - 1 : 0;
        // kDefer: lane j's path position and the one below it (its store target), both mapped
        int pj = aj, pdown = 0;
        if (kDefer) {
            const int L0 = lane <= D ? (int)(np1 >> lane) - 1 : 0;
            const int L1 = on ? (int)(np1 >> (lane - 1)) - 1 : 0;
            pj = L0;
            pdown = L1;
            for (int h = 0; h < hm; h++) {
                const int bh = __builtin_amdgcn_readlane(hb, h);
                pj += L0 >= bh ? 1 : 0;
                pdown += L1 >= bh ? 1 : 0;
            }
        }
        int32_t ac = 0;
        double a1 = 0.0, a2 = 0.0;
        if (on) U.template ld<SP>(pj, ac, a1, a2);
        const uint64_t lt = ballot(on && key_lt(k1, k2, a1, a2));
        s = __builtin_ctzll(~(lt >> 1));  // trailing ones from lane 1
        wsync();
        if (kDefer) {
            if (on && lane <= s) U.template st<SP>(pdown, ac, a1, a2);
            const int pdst = __builtin_amdgcn_readlane(pj, s);
            if (lane == 0) U.template st<SP>(pdst, c, k1, k2);
        } else {
            if (on && lane <= s) U.template st<SP>((int)(np1 >> (lane - 1)) - 1, ac, a1, a2);
            if (lane == 0) U.template st<SP>((int)(np1 >> s) - 1, c, k1, k2);
        }
        wsync();
        return (int)(np1 >> s) - 1;
    }
    __device__ __forceinline__ void push(int32_t c, double k1, double k2, Track& t, bool me)
    {
        const uint32_t np1 = (uint32_t)U.n + 1u;
        int s;
        const int dst = U.n + (kDefer ? hm : 0) < U.cap ? push_t<false>(c, k1, k2, np1, s) : push_t<true>(c, k1, k2, np1, s);
        // tracked positions: ancestor j (1..s) -> ancestor j-1
        if (t.pos >= 0) {
            const int p1 = t.pos + 1;
            const int depth = 31 - __clz(np1) - (31 - __clz(p1));  // levels from p to position n
            if (depth >= 1 && depth <= s && ((int)(np1 >> depth) == p1)) t.pos = (int)(np1 >> (depth - 1)) - 1;
        }
        if (me) t.pos = dst;
        U.n += 1;
        npush += 1;
        if (U.n > maxn) maxn = U.n;
    }

    // updateVertex over the 3x3x3 block of `center` (:147-158): optionally the centre first (its own
    // updateVertex), then getNeighbor(center) in motion order.  The 5x5x5 g block is staged first;
    // g does not change inside.  expand: the centre was just popped -- computeShortestPath's
    // over/under-consistency step (:136-141) runs here on the staged g / rhs: g = rhs, or g = inf
    // and the centre's own updateVertex.  The g / rhs stores go out after the block's updates.
    __device__ void update_block(int center, bool do_center, bool expand = false)
    {
        LSTAMP(t0);
        int cx, cy, cz;
        geo.xyz(center, cx, cy, cz);
        // ---- stage g of the 5x5x5 block (inf outside the map).  Every HBM read of the block (g, and
        //      rhs of the lane's voxel below) issues first, unconditionally on in-map addresses, and
        //      the LDS stores follow: one round trip instead of a wait per load.
        double gb0, gb1;
        bool gin0, gin1;
        {
            const int x0 = cx + lane / 25 - 2, y0 = cy + (lane / 5) % 5 - 2, z0 = cz + lane % 5 - 2;
            const int b1 = lane + 64;
            const int x1 = cx + b1 / 25 - 2, y1 = cy + (b1 / 5) % 5 - 2, z1 = cz + b1 % 5 - 2;
            gin0 = geo.in(x0, y0, z0);
            gin1 = b1 < 125 && geo.in(x1, y1, z1);
            const int i0 = gin0 ? geo.id(x0, y0, z0) : center, i1 = gin1 ? geo.id(x1, y1, z1) : center;
            // loads first, unconditionally (in-map addresses): one round trip, no LDS round before it;
            // a voxel this query never wrote holds a stale value: inf by its bit
            gb0 = g[i0];
            gb1 = g[i1];
            gin0 = gin0 && gw(i0);
            gin1 = gin1 && gw(i1);
        }
        const int m = lane < 26 ? lane : 0;
        const int dx = lane < 26 ? c_m[m][0] : 0, dy = lane < 26 ? c_m[m][1] : 0, dz = lane < 26 ? c_m[m][2] : 0;
        const int px = cx + dx, py = cy + dy, pz = cz + dz;
        const bool mine = lane <= 26 && geo.in(px, py, pz);
        const int P = mine ? geo.id(px, py, pz) : 0;
        const double rvr = rhs[mine ? P : center];
        const double rvl = (mine && rw(P)) ? rvr : kInf;
        cube[lane] = gin0 ? gb0 : kInf;
        if (lane < 61) cube[lane + 64] = gin1 ? gb1 : kInf;
        // ---- block masks: in the map / obstacle, as wave-uniform bits
        Mask125 inm, obm;
        {
            bool i0 = false, o0 = false, i1 = false, o1 = false;
            {
                const int b = lane;
                const int x = cx + b / 25 - 2, y = cy + (b / 5) % 5 - 2, z = cz + b % 5 - 2;
                i0 = geo.in(x, y, z);
                o0 = i0 && occ.at(x, y, z);
            }
            if (lane < 61) {
                const int b = lane + 64;
                const int x = cx + b / 25 - 2, y = cy + (b / 5) % 5 - 2, z = cz + b % 5 - 2;
                i1 = geo.in(x, y, z);
                o1 = i1 && occ.at(x, y, z);
            }
            inm.lo = ballot(i0);
            inm.hi = ballot(i1);
            obm.lo = ballot(o0);
            obm.hi = ballot(o1);
        }
        // ---- this lane's block voxel (above): lanes 0..25 = motion m, lane 26 = the centre
        // the centre's getNeighbor(center): in the map, endpoint free
        const bool is_nb = lane < 26 && mine && !occ.at(px, py, pz);
        double rv = mine ? rvl : 0.0;
        wsync();
        double gnew = 0.0;  // the popped centre's new g (expand)
        if (expand) {
            const double g0 = cube[62], r0 = rl_f64(rv, 26);
            const bool over = g0 > r0;
            gnew = over ? r0 : kInf;
            do_center = !over;
            if (lane == 0) cube[62] = gnew;
            if (center == goal) goal_g = gnew;
            wsync();
        }
        // ---- rhs of the lane's voxel: min over its getNeighbor of g + cost(n, voxel) (:150-153)
        if (mine && P != start) {
            // block coordinates of the voxel (1..3) and of its neighbours (0..4): every occupancy
            // test of isCollision(n, voxel) falls inside the block
            const int ax = dx + 2, ay = dy + 2, az = dz + 2;
            const bool pblk = obm.at((ax * 5 + ay) * 5 + az);
            double best = kInf;
            bool any = false;
#pragma unroll
            for (int u = 0; u < 26; u++) {
                const int ex = kM[u][0], ey = kM[u][1], ez = kM[u][2];  // compile-time after unrolling
                const int qx = ax + ex, qy = ay + ey, qz = az + ez;
                const int qb = (qx * 5 + qy) * 5 + qz;
                if (!inm.at(qb) || obm.at(qb)) continue;  // getNeighbor: in the map, endpoint free
                any = true;
                // isCollision(n = q, voxel): the voxel blocked, or the face cells next to q toward it
                const int mx = -ex, my = -ey, mz = -ez;  // q -> voxel
                const int ch = (mx != 0) + (my != 0) + (mz != 0);
                bool c = pblk;
                if (!c && ch == 2) {
                    if (mx != 0 && my != 0) c = obm.at(((qx + mx) * 5 + qy) * 5 + qz) || obm.at((qx * 5 + qy + my) * 5 + qz);
                    else if (mx != 0 && mz != 0) c = obm.at(((qx + mx) * 5 + qy) * 5 + qz) || obm.at((qx * 5 + qy) * 5 + qz + mz);
                    else c = obm.at((qx * 5 + qy + my) * 5 + qz) || obm.at((qx * 5 + qy) * 5 + qz + mz);
                } else if (!c && ch == 3) {
                    c = obm.at(((qx + mx) * 5 + qy) * 5 + qz) || obm.at((qx * 5 + qy + my) * 5 + qz) ||
                        obm.at((qx * 5 + qy) * 5 + qz + mz);
                }
                const double gq = cube[qb];
                best = fmin(best, gq + (c ? kInf : (ch == 1 ? 1.0 : (ch == 2 ? 1.4142135623730951 : 1.7320508075688772))));
            }
            rv = any ? best : kInf;
        }
        const double gv = mine ? cube[(dx + 2) * 25 + (dy + 2) * 5 + (dz + 2)] : 0.0;
        const double hv = mine ? hval(px, py, pz) : 0.0;  // calculateKey's h, lane-parallel
        LSTAMP(t1);
        // ---- U positions of the 27 voxels: one scan
        Track t;
        t.pos = -1;
        // kDefer: at most one hole here (the popped node's, expand); the scan walks the physical
        // array, skips the hole and reports logical positions
        const int hole = (kDefer && hm) ? __builtin_amdgcn_readlane(hb, 0) : 0x7fffffff;
        const int nph = U.n + (kDefer ? hm : 0);
        const bool usp = nph > U.cap;
        for (int base = 0; base < nph; base += 64) {
            const int k = base + lane;
            int32_t c = -1;
            double a, b;
            {
                const int kk = k < nph ? k : nph - 1;  // an unconditional load, the result masked
                if (usp) U.template ld<true>(kk, c, a, b);
                else U.template ld<false>(kk, c, a, b);
                if (k >= nph || k == hole) c = -1;
            }
            // block index of c relative to the centre, or -1
            int bi = -1;
            if (c >= 0) {
                int x, y, z;
                geo.xyz(c, x, y, z);
                const int ex = x - cx, ey = y - cy, ez = z - cz;
                if (ex >= -1 && ex <= 1 && ey >= -1 && ey <= 1 && ez >= -1 && ez <= 1) bi = (ex + 1) * 9 + (ey + 1) * 3 + (ez + 1);
            }
            uint64_t hits = ballot(bi >= 0);
            while (hits) {
                const int l = __ffsll((long long)hits) - 1;
                hits &= hits - 1;
                const int hbi = __builtin_amdgcn_readlane(bi, l);
                const int myb = (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1);
                if (lane <= 26 && myb == hbi) t.pos = base + l - (base + l > hole ? 1 : 0);
            }
        }
        LSTAMP(t2);
        // ---- updateVertex in the reference's order: the centre (if asked), then each neighbour
        const uint64_t nbm = ballot(is_nb);
        const int nsteps = (do_center ? 1 : 0) + __popcll(nbm);
        uint64_t rem = nbm;
        for (int sidx = 0; sidx < nsteps; sidx++) {
            int who;
            if (do_center && sidx == 0) {
                who = 26;
            } else {
                who = __ffsll((long long)rem) - 1;
                rem &= rem - 1;
            }
            const int Pw = __builtin_amdgcn_readlane(P, who);
            const double rw = rl_f64(rv, who);
            const double gw = rl_f64(gv, who);
            if (Pw == goal) goal_rhs = rw;
            const int pw = __builtin_amdgcn_readlane(t.pos, who);
            LSTAMP(u0);
            if (pw >= 0) remove_at(pw, t);
            LSTAMP(u1);
            if (gw != rw) {
                const double mn = gw < rw ? gw : rw;
                push(Pw, mn + rl_f64(hv, who), mn, t, lane == who);
            }
#if defined(PMP_STAMPS) && PMP_STAMPS == 2
            LSTAMP(u2);
            cyc[0] += u1 - u0;
            cyc[1] += u2 - u1;
#endif
        }
        // deferred stores: the updated voxels' rhs (the start keeps its own), the centre's new g
        {
            // (a recomputed rhs equal to the one held -- the implicit inf of a never-written voxel
            // included -- is not stored: most of a block's updateVertex calls leave rhs as it was, and
            // each store is a partly written line)
            const bool upd = mine && P != start && (is_nb || (lane == 26 && do_center)) && rv != rvl;
            if (upd) {
                rhs[P] = rv;
                if (kL3Mirror & 2) mrhs[P] = rv;
                mark(rt, P);
            }
            if (expand && lane == 0) {
                g[center] = gnew;
                if (kL3Mirror & 2) mg[center] = gnew;
                mark(gt, center);
            }
        }
        LSTAMP(tc);
        compact();
        wsync();
#if defined(PMP_STAMPS) && PMP_STAMPS == 2  // remove, push, the whole block, the whole query
        LSTAMP(t3);
        cyc[2] += t3 - t0;
#elif defined(PMP_STAMPS)
        LSTAMP(t3);
        cyc[1] += t1 - t0;
        cyc[2] += t2 - t1;
        cyc[3] += t3 - t2;
#endif
    }
};

__host__ __device__ inline size_t l3_mirror_bytes(size_t ncell, int words)
{
    return ((2 * ncell + 2 * (ncell + 1)) * 8 + (ncell + 1) * 4 + (size_t)words * 8 + 255) & ~(size_t)255;
}

__global__ __launch_bounds__(64) void lpa3d_kernel(
    const uint32_t* __restrict__ occ_all, int per_query, int X, int Y, int Z, int heur,
    const int32_t* __restrict__ start_xyz, const int32_t* __restrict__ goal_xyz, int nq,
    const int32_t* __restrict__ changes, int nr, double* __restrict__ cost_out, int32_t* __restrict__ plen_out,
    int32_t* __restrict__ path_out, int path_cap, int64_t* __restrict__ nexp_out, int32_t* __restrict__ status_out,
    int64_t* __restrict__ counters, int64_t max_exp, int* __restrict__ queue, double* __restrict__ scr_f64,
    int32_t* __restrict__ scr_i32, uint32_t* __restrict__ occ_scr, int words, int occ_lds, int ucap,
    const int32_t* __restrict__ order, int prio_n, uint32_t* __restrict__ bits_all, unsigned char* __restrict__ mirror)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int ncell = X * Y * Z;
    L3 S;
    S.geo = Geo{X, Y, Z, 1.0f / (float)Y, 1.0f / (float)Z};
    S.lane = lane;
    S.heur = heur;
    // LDS: cube (125 f64, 1000 B -> 1024), U keys (2 x ucap f64), U cells (ucap i32), occupancy bits
    S.cube = (lds_f64*)smem;
    S.U.l1 = (lds_f64*)(smem + 1024);
    S.U.l2 = (lds_f64*)(smem + 1024 + (size_t)8 * ucap);
    S.U.lc = (lds_i32*)(smem + 1024 + (size_t)16 * ucap);
    S.U.cap = ucap;
    S.occ.l = (lds_u32*)(smem + 1024 + (size_t)20 * ucap);
    S.occ.lds = occ_lds != 0;
    S.touch = true;
    S.hb = 0;
    S.hm = 0;
    S.gt = bits_all + (size_t)blockIdx.x * 2 * (size_t)words;
    S.rt = S.gt + words;
    S.occ.g = occ_scr + (size_t)blockIdx.x * (size_t)words;
    S.occ.geo = S.geo;
    {
        const size_t spill = (size_t)ncell + 1;
        double* f = scr_f64 + (size_t)blockIdx.x * (2 * (size_t)ncell + 2 * spill);
        S.g = f;
        S.rhs = f + ncell;
        S.U.g1 = f + 2 * (size_t)ncell;
        S.U.g2 = S.U.g1 + spill;
        S.U.gc = scr_i32 + (size_t)blockIdx.x * spill;
        if (kL3Mirror) {  // the mirror: g, rhs, U keys, U cells, the two bit arrays
            double* mf = (double*)(mirror + (size_t)blockIdx.x * l3_mirror_bytes(ncell, words));
            S.mg = mf;
            S.mrhs = mf + ncell;
            S.U.mg1 = mf + 2 * (size_t)ncell;
            S.U.mg2 = S.U.mg1 + spill;
            S.U.mgc = (int32_t*)(S.U.mg2 + spill);
            S.mgt = (uint32_t*)(S.U.mgc + spill);
            S.mrt = S.mgt + words;
        }
    }
    const int R1 = nr + 1;

    for (;;) {
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = uni(order ? order[qi] : qi);
        // longest queries first, at raised priority (they set the launch's tail)
        if (qi < prio_n) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
        const int sx = uni(start_xyz[3 * q]), sy = uni(start_xyz[3 * q + 1]), sz = uni(start_xyz[3 * q + 2]);
        const int gx = uni(goal_xyz[3 * q]), gy = uni(goal_xyz[3 * q + 1]), gz = uni(goal_xyz[3 * q + 2]);
        const bool in = S.geo.in(sx, sy, sz) && S.geo.in(gx, gy, gz);
        if (!in) {  // endpoints outside the map: not supported (every lane stores the same values)
            for (int r = 0; r < R1; r++) {
                status_out[(size_t)q * R1 + r] = PMP_REF_RAISES;
                cost_out[(size_t)q * R1 + r] = 0.0;
                plen_out[(size_t)q * R1 + r] = 0;
                nexp_out[(size_t)q * R1 + r] = 0;
            }
            continue;
        }
        S.start = S.geo.id(sx, sy, sz);
        S.goal = S.geo.id(gx, gy, gz);
        S.gx = gx;
        S.gy = gy;
        S.gz = gz;
        S.npush = 0;
        S.maxn = 0;
#ifdef PMP_STAMPS
        S.cyc[0] = S.cyc[1] = S.cyc[2] = S.cyc[3] = 0;
        const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
        if (S.start == S.goal) {
            for (int r = 0; r < R1; r++) {
                status_out[(size_t)q * R1 + r] = 0;
                cost_out[(size_t)q * R1 + r] = 0.0;
                plen_out[(size_t)q * R1 + r] = 1;
                nexp_out[(size_t)q * R1 + r] = r == 0 ? 1 : 0;
                path_out[((size_t)q * R1 + r) * (size_t)path_cap] = S.goal;
            }
            if (counters && lane == 0) {
                counters[4 * q] = 1; counters[4 * q + 1] = 1; counters[4 * q + 2] = 0; counters[4 * q + 3] = 1;
            }
            continue;
        }
        // working occupancy, g = rhs = inf, rhs(start) = 0 (LNode3D(start, inf, 0.0), :58)
        {
            const uint32_t* src = occ_all + (per_query ? (size_t)q * (size_t)words : 0);
            for (int w = lane; w < words; w += 64) {
                if (S.occ.lds) S.occ.l[w] = src[w];
                else S.occ.g[w] = src[w];
            }
            if (S.touch) {
                for (int w = lane; w < words; w += 64) {
                    __hip_atomic_store(S.gt + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(S.rt + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (kL3Mirror & 4) {
                        __hip_atomic_store(S.mgt + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(S.mrt + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                wsync();
                if (lane == 0) {
                    S.rhs[S.start] = 0.0;
                    if (kL3Mirror & 2) S.mrhs[S.start] = 0.0;
                    S.mark(S.rt, S.start);
                }
            } else {
                for (int c = lane; c < ncell; c += 64) {
                    S.g[c] = kInf;
                    S.rhs[c] = c == S.start ? 0.0 : kInf;
                }
            }
        }
        wsync();
        S.U.n = 0;
        S.goal_g = kInf;
        S.goal_rhs = kInf;  // LNode3D(goal, inf, inf) (:59); goal != start here
        {
            Track t;
            t.pos = -1;
            S.push(S.start, 0.0 + S.hval(sx, sy, sz), 0.0, t, false);  // calculateKey(start)
        }
        int st = 0;
        int64_t tot_exp = 0;
        for (int r = 0; r <= nr; r++) {
            S.nexp = 0;
            if (r > 0 && st != 0 && st != PMP_NO_PATH) {
                if (lane == 0) {
                    status_out[(size_t)q * R1 + r] = -1;
                    cost_out[(size_t)q * R1 + r] = 0.0;
                    plen_out[(size_t)q * R1 + r] = 0;
                    nexp_out[(size_t)q * R1 + r] = 0;
                }
                continue;
            }
            st = 0;
            if (r > 0) {
                // apply_change(coord, blocked) (:93-124)
                const int32_t* ch = changes + ((size_t)q * nr + (r - 1)) * 4;
                const int cx = uni(ch[0]), cy = uni(ch[1]), cz = uni(ch[2]), mode = uni(ch[3]);
                if (S.geo.in(cx, cy, cz)) {
                    const int cell = S.geo.id(cx, cy, cz);
                    const bool is_obs = S.occ.at(cx, cy, cz);
                    bool freed = false;
                    if (mode == 0) freed = is_obs;
                    else if (mode == 2) freed = is_obs;
                    const bool block = (mode == 0 && !is_obs) || mode == 1;
                    wsync();
                    if (lane == 0 && (freed || block)) {
                        const uint32_t bit = 1u << (cell & 31);
                        if (S.occ.lds) {
                            if (freed) S.occ.l[cell >> 5] &= ~bit;
                            else S.occ.l[cell >> 5] |= bit;
                        } else {
                            if (freed) S.occ.g[cell >> 5] &= ~bit;
                            else S.occ.g[cell >> 5] |= bit;
                        }
                    }
                    wsync();
                    // updateVertex(map[coord]) when freed, then getNeighbor(changed)'s updateVertex
                    S.update_block(cell, freed);
                }
            }
            // ---- computeShortestPath (:127-145)
            for (;;) {
                if (S.U.n == 0) break;
#ifdef PMP_STAMPS
                [[maybe_unused]] const uint64_t ts = __builtin_amdgcn_s_memtime();
#endif
                if (max_exp > 0 && S.nexp >= max_exp) { st = PMP_CAP_OVERFLOW; break; }
                const double gg = S.goal_g, gr = S.goal_rhs;
                // min(U, key): first minimal key in list order
                double b1 = kInf, b2 = kInf;
                int bi = 0x7fffffff;
                const bool usp = S.U.n > S.U.cap;
                // two entries per lane per round, loads unconditional (clamped) and issued together
                for (int k0 = lane; k0 < S.U.n; k0 += 128) {
                    int32_t c, c2;
                    double a1, a2, e1, e2;
                    const int kb = k0 + 64 < S.U.n ? k0 + 64 : S.U.n - 1;
                    if (usp) { S.U.template ld<true>(k0, c, a1, a2); S.U.template ld<true>(kb, c2, e1, e2); }
                    else { S.U.template ld<false>(k0, c, a1, a2); S.U.template ld<false>(kb, c2, e1, e2); }
                    if (bi == 0x7fffffff || key_lt(a1, a2, b1, b2)) { b1 = a1; b2 = a2; bi = k0; }
                    if (k0 + 64 < S.U.n && key_lt(e1, e2, b1, b2)) { b1 = e1; b2 = e2; bi = k0 + 64; }
                }
                for (int o = 1; o < 64; o <<= 1) {
                    const double o1 = __shfl_xor(b1, o, 64), o2 = __shfl_xor(b2, o, 64);
                    const int oi = __shfl_xor(bi, o, 64);
                    const bool take = oi != 0x7fffffff &&
                                      (bi == 0x7fffffff || key_lt(o1, o2, b1, b2) || (o1 == b1 && o2 == b2 && oi < bi));
                    if (take) { b1 = o1; b2 = o2; bi = oi; }
                }
                bi = uni(bi);
                b1 = rl_f64(b1, 0);
                b2 = rl_f64(b2, 0);
                const double gm = gg < gr ? gg : gr;
                // node.key >= calculateKey(goal) and goal.rhs == goal.g (:131-133); h(goal, goal) = 0
#if defined(PMP_STAMPS) && PMP_STAMPS != 2
                S.cyc[0] += __builtin_amdgcn_s_memtime() - ts;
#endif
                if (!key_lt(b1, b2, gm + 0.0, gm) && gr == gg) break;
                int32_t vt = 0;
                if (lane == 0) {
                    double a, b;
                    if (usp) S.U.template ld<true>(bi, vt, a, b);
                    else S.U.template ld<false>(bi, vt, a, b);
                }
                const int v = uni(vt);
                {
                    Track t;
                    t.pos = -1;
                    S.remove_at(bi, t);
                }
                S.nexp++;
                // over-consistent: g = rhs; else g = inf and updateVertex(node); then the neighbours
                S.update_block(v, false, true);
            }
            // ---- extractPath (:185-225): greedy min-g free neighbour from the goal
            double cost = 0.0;
            int len = 0;
            int32_t* pth = path_out + ((size_t)q * R1 + r) * (size_t)path_cap;
            if (st == 0) {
                int node = S.goal;
                if (lane == 0 && len < path_cap) pth[len] = node;
                len++;
                int safety = 0;
                // Brent's cycle detection: the walk's next node is a function of the node alone (g
                // and the map are fixed here), so a repeated node is a cycle the walk never leaves
                // and the reference walks on to its 100000-step guard, returning (cost, []).  Once a
                // cycle of <= 64 steps is found, the steps left repeat its step costs: they are
                // added in order (the same f64 sums) without the per-step memory rounds (a stuck
                // C5 query took ~270 ms of one wave walking them).
                int tort = node, power = 1, lam = 0, ring = 0;
                bool chk = true, cyc = false;
                while (node != S.start) {
                    int x, y, z;
                    S.geo.xyz(node, x, y, z);
                    const int m = lane < 26 ? lane : 0;
                    const int nx = x + c_m[m][0], ny = y + c_m[m][1], nz = z + c_m[m][2];
                    bool ok = lane < 26 && S.geo.in(nx, ny, nz) && !S.occ.at(nx, ny, nz) &&
                              !S.occ.coll(x, y, z, nx, ny, nz);
                    double gn = kInf;
                    if (ok) gn = S.g_at(S.geo.id(nx, ny, nz));
                    uint64_t vm = ballot(ok);
                    if (!vm) { st = PMP_NO_PATH; break; }
                    int bm = -1;
                    double bg = 0.0;
                    while (vm) {
                        const int k = __ffsll((long long)vm) - 1;
                        vm &= vm - 1;
                        const double gk = rl_f64(gn, k);
                        if (bm < 0 || gk < bg) { bm = k; bg = gk; }
                    }
                    cost += dist_unit(c_m[bm][0], c_m[bm][1], c_m[bm][2]);
                    node = S.geo.id(x + c_m[bm][0], y + c_m[bm][1], z + c_m[bm][2]);
                    if (lane == 0 && len < path_cap) pth[len] = node;
                    len++;
                    if (++safety >= 100000) { st = PMP_NO_PATH; break; }
                    if (chk) {
                        if (lane == (safety & 63)) ring = bm;  // step t's motion at lane t & 63
                        lam++;
                        if (node == tort) {
                            if (lam <= 64) { cyc = true; break; }
                            chk = false;  // a longer cycle: walk it
                        } else if (lam == power) {
                            tort = node;
                            power <<= 1;
                            lam = 0;
                        }
                    }
                }
                if (cyc) {
                    // cycle step i (0..lam-1) = step safety - lam + 1 + i; the steps left,
                    // safety + 1 .. 99999 + 1, take them in turn
                    const int mi = __builtin_amdgcn_ds_bpermute(((safety - lam + 1 + lane) & 63) << 2, ring);
                    const int mm = lane < lam ? mi : 0;
                    const double dc = dist_unit(c_m[mm][0], c_m[mm][1], c_m[mm][2]);
                    int i = 0;
                    for (int j = safety; j < 100000; j++) {
                        cost += rl_f64(dc, i);
                        i = i + 1 == lam ? 0 : i + 1;
                    }
                    st = PMP_NO_PATH;
                }
                wsync();
                if (st == 0) {
                    if (len > path_cap) st = PMP_PATH_OVERFLOW;
                    else  // path.reverse()
                        for (int i = lane; i < len / 2; i += 64) {
                            const int32_t a = pth[i], b = pth[len - 1 - i];
                            pth[i] = b;
                            pth[len - 1 - i] = a;
                        }
                }
            }
            tot_exp += S.nexp;
            if (lane == 0) {
                status_out[(size_t)q * R1 + r] = st;
                cost_out[(size_t)q * R1 + r] = cost;
                plen_out[(size_t)q * R1 + r] = st == 0 || st == PMP_PATH_OVERFLOW ? len : 0;
                nexp_out[(size_t)q * R1 + r] = S.nexp;
            }
            wsync();
        }
        if (counters && lane == 0) {
#ifdef PMP_STAMPS
#if PMP_STAMPS == 2
            S.cyc[3] = __builtin_amdgcn_s_memtime() - tq0;
#endif
            for (int k = 0; k < 4; k++) counters[4 * q + k] = (int64_t)S.cyc[k];
#else
            counters[4 * q] = S.npush;
            counters[4 * q + 1] = tot_exp;
            counters[4 * q + 2] = 0;
            counters[4 * q + 3] = S.maxn;
#endif
        }
        wsync();
    }
}

constexpr int kOccLdsWords = 2048;                 // grids up to 65536 voxels: occupancy in LDS
constexpr size_t kScratchBudget = (size_t)16 << 30;

}  // namespace

extern "C" int pmp_lpastar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y,
                                   int Z, int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq,
                                   const int32_t* changes, int nr, double* cost, int32_t* path_len, int32_t* path,
                                   int path_cap, int64_t* n_expanded, int32_t* status, int64_t* counters,
                                   int64_t max_expansions)
{
    if (!ctx) return PMP_EINVAL;
    if (X < 1 || Y < 1 || Z < 1 || X > kMaxDim || Y > kMaxDim || Z > kMaxDim)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar3d_batch: X, Y, Z must be in [1, 256]");
    if (heuristic != 0 && heuristic != 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar3d_batch: heuristic must be 0 or 1");
    if (nq < 0 || path_cap < 1 || nr < 0 || (nr > 0 && !changes))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar3d_batch: bad nq/path_cap/nr/changes");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xyz || !goal_xyz || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar3d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t ncell = (size_t)X * Y * Z;
    const int words = (int)((ncell + 31) / 32);
    const bool occ_lds = words <= kOccLdsWords;
    // up to 16 waves per CU (tools/dyn3d_sweep.py): the LDS share of each holds the g block, U (20 B per
    // entry, the rest spills) and the occupancy
    const int per_cu = std::max(1, std::min(ctx->workers_per_cu > 0 ? ctx->workers_per_cu : 16, (nq + 255) / 256));
    const int occ_bytes = occ_lds ? ((words * 4 + 15) & ~15) : 0;
    int ucap = (((160 * 1024) / per_cu - 1024 - occ_bytes) / 20) & ~15;
    if (ucap < 64) ucap = 64;
    if ((size_t)ucap > ncell + 1) ucap = (int)((ncell + 1 + 15) & ~(size_t)15);
    const size_t lds = 1024 + (size_t)20 * ucap + occ_bytes;
    const size_t spill = ncell + 1;
    const size_t per_worker = (2 * ncell + 2 * spill) * 8 + spill * 4 + (size_t)words * 8 + (occ_lds ? 0 : (size_t)words * 4) + 256;
    int workers = 256 * per_cu;
    const size_t fit = kScratchBudget / per_worker;
    if (fit < 1) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_lpastar3d_batch: one worker exceeds the scratch budget");
    if ((size_t)workers > fit) workers = (int)fit;
    if (workers > nq) workers = nq;
    double* f = (double*)pmp_scratch(ctx, SCR_AUX2, (size_t)workers * (2 * ncell + 2 * spill) * 8 + 16);
    // U cells of the HBM part, then the written-this-query bits (2 x words per worker)
    int32_t* i32 = (int32_t*)pmp_scratch(ctx, SCR_AUX3, (size_t)workers * spill * 4 + (size_t)workers * 2 * words * 4 + 16);
    uint32_t* occw = (uint32_t*)pmp_scratch(ctx, SCR_AUX4, occ_lds ? 16 : (size_t)workers * words * 4 + 16);
    int* queue = (int*)pmp_scratch(ctx, SCR_AUX0, 256);
    if (!f || !i32 || !occw || !queue) return PMP_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    int32_t* order = nullptr;
    {
        const int rc = pmp_lpt_order3d(ctx, s, start_xyz, goal_xyz, nq, X, Y, Z, workers, &order);
        if (rc) return rc;
    }
    unsigned char* mirror = nullptr;
    if (kL3Mirror) {
        mirror = (unsigned char*)pmp_scratch(ctx, SCR_MQ_PC, (size_t)workers * l3_mirror_bytes(ncell, words));
        if (!mirror) return PMP_ENOMEM;
    }
    hipLaunchKernelGGL(lpa3d_kernel, dim3(workers), dim3(64), lds, s, occ_bits, per_query, X, Y, Z, heuristic, start_xyz,
                       goal_xyz, nq, changes, nr, cost, path_len, path, path_cap, n_expanded, status, counters,
                       max_expansions, queue, f, i32, occw, words, occ_lds ? 1 : 0, ucap, (const int32_t*)order,
                       order ? ctx->astar_prio_n : 0, (uint32_t*)(i32 + (size_t)workers * spill), mirror);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
