// Batched 3D A* for gfx950, exact with the reference AStar3D.plan
// (global_planner/graph_search/a_star3d.py:33-106) over Grid3D (utils/environment/env3d.py:43-103)
// with GraphSearcher3D.isCollision (graph_search_3d.py:66-107).
//
// The reference heap holds tuples (f, h, counter, node) -> a TOTAL order, so the pop sequence is
// the sorted order of (f, h, counter) whatever the heap shape; the kernel keeps a binary heap in
// LDS (spilling deep positions to HBM) with the same key:
//   entry = {f64 g, f64 f, u32 seq (push counter), u32 cm = (x<<16 | y<<8 | z) << 5 | dir}
//   (24 B in LDS, 32 B spill records); f = g + h computed once at the push with
//   h = math.sqrt(dx**2+dy**2+dz**2) of integers (exactly the reference's tentative_g + node_n.h),
//   hkey = d2 rebuilt from the cell on load (sqrt of integers is monotone and exact).
// Reopening semantics are the reference's: a pop is skipped if CLOSED holds the cell with g <= node.g
// (:48-50), a neighbour is skipped if CLOSED holds it with g <= tentative_g (:68-70), CLOSED is
// (over)written before the goal test (:52-63).  Path is reversed to start -> goal (:105).
// The heap engine is heap16.h (LDS + HBM spill, wave-parallel pop/push).
// One wave64 per query (persistent workers pulling an atomic queue); per-worker HBM state:
// u8 closed-dir per cell (0 = open, dir+1 = closed) + f64 closed g per cell, reset per query.
#include <algorithm>
#include "heap16.h"

namespace {

constexpr int kMaxDim3 = 256;

__device__ __constant__ int8_t c_m3[26][3] = {
    {-1, 0, 0}, {-1, 1, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0}, {1, -1, 0}, {0, -1, 0}, {-1, -1, 0},
    {0, 0, 1}, {0, 0, -1},
    {-1, 0, 1}, {-1, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, -1, 1}, {-1, -1, 1},
    {-1, 0, -1}, {-1, 1, -1}, {0, 1, -1}, {1, 1, -1}, {1, 0, -1}, {1, -1, -1}, {0, -1, -1}, {-1, -1, -1}};

using heap16::Ent;  // g = path cost, a = push counter, b = cm; derived f = g + h, hk = h order key

// (f, h, counter) tuple order of a_star3d.py:40,75.  f = tentative_g + h is computed once, at the
// push (set_f), and stored beside the entry; h's order key (an integer) is rebuilt from the cell.
struct Key3 {
    static constexpr bool kStoredF = true;
    int gx, gy, gz;
    int heur;  // 0 euclidean, 1 manhattan, 2 zero (Dijkstra3D: h = 0, dijkstra3d.py:34,83)
    int Y, Z;

    __device__ __forceinline__ uint32_t hkey(uint32_t b) const
    {
        const int x = (int)((b >> 21) & 255u), y = (int)((b >> 13) & 255u), z = (int)((b >> 5) & 255u);
        const int dx = abs(gx - x), dy = abs(gy - y), dz = abs(gz - z);
        return heur == 2 ? 0u : (heur == 1 ? (uint32_t)(dx + dy + dz) : (uint32_t)(dx * dx + dy * dy + dz * dz));
    }
    __device__ __forceinline__ void derive(Ent& e) const { e.hk = hkey(e.b); }
    // f = g + h exactly as node_n.g + node_n.h (math.sqrt of the integer square sum for euclidean)
    __device__ __forceinline__ void set_f(Ent& e) const
    {
        e.hk = hkey(e.b);
        e.f = heur == 2 ? e.g : (heur == 1 ? e.g + (double)e.hk : e.g + __dsqrt_rn((double)e.hk));
    }

    static __device__ __forceinline__ bool lt(const Ent& a, const Ent& b)
    {
        return (a.f < b.f) | ((a.f == b.f) & ((a.hk < b.hk) | ((a.hk == b.hk) & (a.a < b.a))));
    }
};

__device__ __forceinline__ bool occ3(const uint32_t* occ, int X, int Y, int Z, int x, int y, int z)
{
    if ((unsigned)x >= (unsigned)X || (unsigned)y >= (unsigned)Y || (unsigned)z >= (unsigned)Z) return true;
    const uint32_t c = ((uint32_t)x * (uint32_t)Y + (uint32_t)y) * (uint32_t)Z + (uint32_t)z;
    return (occ[c >> 5] >> (c & 31)) & 1u;
}

typedef __attribute__((address_space(3))) uint32_t lds_w32;

// occupancy bit, blocked outside the grid, from the per-query bitmap staged in LDS
__device__ __forceinline__ uint32_t occ3l(const lds_w32* occ, int X, int Y, int Z, int x, int y, int z)
{
    if ((unsigned)x >= (unsigned)X || (unsigned)y >= (unsigned)Y || (unsigned)z >= (unsigned)Z) return 1u;
    const uint32_t c = ((uint32_t)x * (uint32_t)Y + (uint32_t)y) * (uint32_t)Z + (uint32_t)z;
    return (occ[c >> 5] >> (c & 31)) & 1u;
}

constexpr int kOccLdsWords = 1024;  // grids up to 32768 cells keep their occupancy in LDS (4 KiB)

// lineOfSight (theta_star3d.py:139-213 == lazy_theta_star3d.py:158-233): integer Bresenham from a to
// b along the dominant axis; both endpoints free, every voxel after a (b included) in the grid and free.
template <bool OCC_LDS>
__device__ __forceinline__ bool los3d(const uint32_t* occ, const lds_w32* occl, int X, int Y, int Z, int x0, int y0,
                                      int z0, int x1, int y1, int z1)
{
    auto blocked = [&](int a, int b, int c) -> bool {
        return OCC_LDS ? occ3l(occl, X, Y, Z, a, b, c) != 0u : occ3(occ, X, Y, Z, a, b, c);
    };
    if (blocked(x0, y0, z0) || blocked(x1, y1, z1)) return false;
    const int dx = abs(x1 - x0), dy = abs(y1 - y0), dz = abs(z1 - z0);
    const int sx = x1 >= x0 ? 1 : -1, sy = y1 >= y0 ? 1 : -1, sz = z1 >= z0 ? 1 : -1;
    // the dominant axis becomes `u`, the other two `v`, `w` (same arithmetic as the three branches)
    const int ax = (dx >= dy && dx >= dz) ? 0 : ((dy >= dx && dy >= dz) ? 1 : 2);
    const int du = ax == 0 ? dx : (ax == 1 ? dy : dz);
    const int dv = ax == 0 ? dy : dx, dw = ax == 2 ? dy : dz;
    int x = x0, y = y0, z = z0;
    int ev = du / 2, ew = du / 2;
    for (int k = 0; k < du; k++) {
        if (ax == 0) x += sx;
        else if (ax == 1) y += sy;
        else z += sz;
        ev -= dv;
        ew -= dw;
        if (ev < 0) {
            if (ax == 0) y += sy;
            else x += sx;
            ev += du;
        }
        if (ew < 0) {
            if (ax == 2) y += sy;
            else z += sz;
            ew += du;
        }
        if (blocked(x, y, z)) return false;
    }
    return true;
}

__device__ __forceinline__ double dist3(int dx, int dy, int dz)  // Planner3D.dist (planner3d.py:22-27)
{
    return __dsqrt_rn((double)(dx * dx + dy * dy + dz * dz));
}

// THETA: 0 = AStar3D / Dijkstra3D / GBFS3D, 1 = ThetaStar3D (theta_star3d.py:38-110), 2 =
// LazyThetaStar3D (lazy_theta_star3d.py:41-128).  Theta modes keep any-voxel parents: a per-cell
// CLOSED parent (cpar) and, per push, the entry's parent in a side table indexed by the push
// counter (ppar), since an entry's parent may be its pusher's parent.
#ifndef PMP_A3_WAVES
#define PMP_A3_WAVES 5  // waves per SIMD the A* / Dijkstra / GBFS variants are compiled for (A/B switch)
#endif
template <bool OCC_LDS, int THETA>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(THETA == 0 ? PMP_A3_WAVES : 4))) void astar3d_kernel(
    const uint32_t* __restrict__ occ_all, int per_query, int X, int Y, int Z, int heuristic,
    const int32_t* __restrict__ start_xyz, const int32_t* __restrict__ goal_xyz, int nq, double* __restrict__ cost_out,
    int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out, int path_cap, int32_t* __restrict__ nexp_out,
    uint32_t* __restrict__ expand_out, int expand_cap, int64_t* __restrict__ counters, int32_t* __restrict__ status_out,
    int* __restrict__ queue, uint4* __restrict__ spill_all, int heap_cap, int lds_cap, uint8_t* __restrict__ cdir_all,
    double* __restrict__ cg_all, int gzero, uint32_t* __restrict__ cpar_all, uint32_t* __restrict__ ppar_all,
    uint32_t ppar_cap, const int32_t* __restrict__ order, int prio_n)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    const size_t ncell = (size_t)X * Y * Z;
    const size_t words = (ncell + 31) / 32;
    const size_t spill_n = (size_t)(heap_cap > lds_cap ? heap_cap - lds_cap : 0);
    heap16::Heap hp =
        heap16::make_heap<true>(smem, lds_cap, spill_all + (size_t)worker * spill_n * 2, spill_n);  // 32 B records
    lds_w32* occl = (lds_w32*)(smem + (size_t)heap16::lds_entry_bytes<true>() * lds_cap);  // OCC_LDS: the query's bitmap
    uint8_t* cdir = cdir_all + (size_t)worker * ncell;
    double* cg = cg_all + (size_t)worker * 2 * ncell;  // closed g
    double* og = cg + ncell;                            // best pending (pushed) g
    uint32_t* cpar = THETA ? cpar_all + (size_t)worker * ncell : nullptr;      // CLOSED parent cell
    uint32_t* ppar = THETA ? ppar_all + (size_t)worker * ppar_cap : nullptr;   // parent of push #seq
    int pop_jl, pop_ol;
    heap16::pop_lane_consts(lane, pop_jl, pop_ol);
    const heap16::Walk6 pop_w = heap16::walk6_consts(lane, pop_jl, pop_ol);
    // neighbour lane m < 26: motion m (env3d.py:56-70)
    const int mdx = lane < 26 ? c_m3[lane][0] : 0, mdy = lane < 26 ? c_m3[lane][1] : 0, mdz = lane < 26 ? c_m3[lane][2] : 0;
    const int mchg = (mdx != 0) + (mdy != 0) + (mdz != 0);
    // Planner3D.dist: math.sqrt(1|2|3); GBFS3D pushes every node with g = 0 (gbfs3d.py:78), so its
    // key (h, counter) is this loop's (f, h, counter) with f = 0 + h, and `g >= closed g` is always
    // true: the CLOSED membership tests of gbfs3d.py:55,74
    const double mcost = gzero ? 0.0 : __dsqrt_rn((double)mchg);

    for (;;) {
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = uni(order ? order[qi] : qi);
        // the longest queries (first in the longest-first order) run at raised priority: they set the
        // launch's tail, the short ones fill the issue slots they leave idle
        if (qi < prio_n) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
        const uint32_t* occ = occ_all + (per_query ? (size_t)q * words : 0);
        if (OCC_LDS)
            for (size_t i = lane; i < words; i += 64) occl[i] = occ[i];
        for (size_t i = lane; i < ncell; i += 64) {
            cdir[i] = 0;
            og[i] = __builtin_inf();
        }
        heap16::wsync();
        const int sx = start_xyz[3 * q], sy = start_xyz[3 * q + 1], sz = start_xyz[3 * q + 2];
        Key3 qc;
        qc.gx = goal_xyz[3 * q];
        qc.gy = goal_xyz[3 * q + 1];
        qc.gz = goal_xyz[3 * q + 2];
        qc.heur = heuristic;
        qc.Y = Y;
        qc.Z = Z;
        const bool s_in = (unsigned)sx < (unsigned)X && (unsigned)sy < (unsigned)Y && (unsigned)sz < (unsigned)Z;
        const bool g_in = (unsigned)qc.gx < (unsigned)X && (unsigned)qc.gy < (unsigned)Y && (unsigned)qc.gz < (unsigned)Z;
        if (!s_in || !g_in) {  // every lane stores the same values (no lane-0 block before the continue)
            status_out[q] = PMP_NO_PATH;
            cost_out[q] = __builtin_inf();
            path_len_out[q] = 0;
            nexp_out[q] = s_in ? 1 : 0;
            if (counters) { counters[4 * q] = 1; counters[4 * q + 1] = 1; counters[4 * q + 2] = s_in; counters[4 * q + 3] = 1; }
            continue;
        }
        const uint32_t scm = (((uint32_t)sx << 16) | ((uint32_t)sy << 8) | (uint32_t)sz) << 5 | 26u;
        const uint32_t goal_xyz24 = ((uint32_t)qc.gx << 16) | ((uint32_t)qc.gy << 8) | (uint32_t)qc.gz;
        Ent root;  // start: g = 0, h = heuristic(start), counter 0 (a_star3d.py:38-41)
        root.g = 0.0;
        root.a = 0u;
        root.b = scm;
        qc.set_f(root);
        if (lane == 0) heap16::store<true, true>(hp, 0, root);
        if (THETA && lane == 0) ppar[0] = ((uint32_t)sx * (uint32_t)Y + (uint32_t)sy) * (uint32_t)Z + (uint32_t)sz;
        heap16::wsync();
        int n = 1;
        uint32_t seq = 1;
        int64_t npush = 1, npop = 0, niter = 0;
#ifdef PMP_STAMPS
        // diagnostic build: cycles in (pop + the overlapped HBM round), after-pop wait, push loop, whole query
        uint64_t cyc_pop = 0, cyc_wait = 0, cyc_push = 0;
        const uint64_t cyc_q0 = __builtin_amdgcn_s_memtime();
#endif
        int nexp = 0, maxn = 1, st = PMP_NO_PATH, plen = 0;
        double goal_cost = __builtin_inf();

        while (n > 0) {
            const Ent node = root;
            npop++;
            n -= 1;
            const int x = (int)((node.b >> 21) & 255u), y = (int)((node.b >> 13) & 255u), z = (int)((node.b >> 5) & 255u);
            const int ndir = (int)(node.b & 31u);
            const uint32_t lin = ((uint32_t)x * (uint32_t)Y + (uint32_t)y) * (uint32_t)Z + (uint32_t)z;
            // ---- HBM round (issued before the pop): neighbour collision + CLOSED state, node's CLOSED state
            const int nx = x + mdx, ny = y + mdy, nz = z + mdz;
            bool coll = true;
            uint32_t nlin = lin;
            if (lane < 26) {
                const bool inb = (unsigned)nx < (unsigned)X && (unsigned)ny < (unsigned)Y && (unsigned)nz < (unsigned)Z;
                if (inb) nlin = ((uint32_t)nx * (uint32_t)Y + (uint32_t)ny) * (uint32_t)Z + (uint32_t)nz;
            }
            // one HBM round, independent of the collision test: CLOSED / pending state (lanes 0..25 the
            // neighbours, 26 the node).  Every lane loads (lanes > 26 the node's cell): a zero fill of
            // the destinations on the other lanes made the compiler drain vmcnt -- every store of the
            // previous expansion included -- at the top of each iteration.
            const uint32_t ncd = cdir[nlin];
            const double ncg = cg[nlin];
            const double nog = og[nlin];
            // theta: the entry's parent cell (the start's parent is the start); read by lane 27 below,
            // loaded on every lane (no zero-filled destination, see above)
            uint32_t epar = 0;
            if (THETA) epar = ppar[node.a < ppar_cap ? node.a : 0u];
            if (lane < 26) {
                if (OCC_LDS) {
#define OCC(a, b, c) occ3l(occl, X, Y, Z, a, b, c)
                    uint32_t c = OCC(x, y, z) | OCC(nx, ny, nz);
                    if (mchg == 2) {
                        if (mdx != 0 && mdy != 0) c |= OCC(x + mdx, y, z) | OCC(x, y + mdy, z);
                        else if (mdx != 0 && mdz != 0) c |= OCC(x + mdx, y, z) | OCC(x, y, z + mdz);
                        else c |= OCC(x, y + mdy, z) | OCC(x, y, z + mdz);
                    } else if (mchg == 3) {
                        c |= OCC(x + mdx, y, z) | OCC(x, y + mdy, z) | OCC(x, y, z + mdz);
                    }
                    coll = c != 0u;
#undef OCC
                } else {
                    coll = occ3(occ, X, Y, Z, x, y, z) || occ3(occ, X, Y, Z, nx, ny, nz);
                    if (mchg == 2) {
                        if (mdx != 0 && mdy != 0) coll = coll || occ3(occ, X, Y, Z, x + mdx, y, z) || occ3(occ, X, Y, Z, x, y + mdy, z);
                        else if (mdx != 0 && mdz != 0) coll = coll || occ3(occ, X, Y, Z, x + mdx, y, z) || occ3(occ, X, Y, Z, x, y, z + mdz);
                        else coll = coll || occ3(occ, X, Y, Z, x, y + mdy, z) || occ3(occ, X, Y, Z, x, y, z + mdz);
                    } else if (mchg == 3) {
                        coll = coll || occ3(occ, X, Y, Z, x + mdx, y, z) || occ3(occ, X, Y, Z, x, y + mdy, z) ||
                               occ3(occ, X, Y, Z, x, y, z + mdz);
                    }
                }
            }
            // ---- pop
#ifdef PMP_STAMPS
            const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
            if (n > 0) {
                if (n < lds_cap) heap16::pop<Key3, false, true>(hp, qc, n, root, lane, pop_jl, pop_ol, pop_w);
                else heap16::pop<Key3, true, true>(hp, qc, n, root, lane, pop_jl, pop_ol, pop_w);
            }
#ifdef PMP_STAMPS
            const uint64_t ts1 = __builtin_amdgcn_s_memtime();
#endif
            // best_closed check (a_star3d.py:48-50)
            const bool sclosed = rl_u32(ncd, 26) != 0u;
            const double scg = rl_f64(ncg, 26);
            double node_g = node.g;
            uint32_t npar = 0;  // theta: the node's parent cell
            if (THETA) {
                npar = rl_u32(epar, 27);
                if (THETA == 2) {
                    // lazy_theta_star3d.py:60-71: no line of sight from the parent -> g = inf, then the
                    // best CLOSED neighbour (first minimum in motion order) becomes the parent
                    const int px = (int)(npar / ((uint32_t)Y * Z)), py = (int)((npar / (uint32_t)Z) % (uint32_t)Y),
                              pz = (int)(npar % (uint32_t)Z);
                    if (!los3d<OCC_LDS>(occ, occl, X, Y, Z, px, py, pz, x, y, z)) {
                        const bool cand = lane < 26 && !coll && ncd != 0u;
                        const double cgv = cand ? ncg + mcost : __builtin_inf();
                        double best = cgv;  // wave min, ties to the lowest lane (= motion order)
                        int bl = cand ? lane : 64;
                        for (int o = 32; o >= 1; o >>= 1) {
                            const double ob = __shfl_xor(best, o);
                            const int ol = __shfl_xor(bl, o);
                            if (ob < best || (ob == best && ol < bl)) { best = ob; bl = ol; }
                        }
                        node_g = __builtin_inf();
                        const int bsel = uni(bl);
                        if (bsel < 64) {
                            const double bv = rl_f64(best, 0);
                            if (bv < node_g) {
                                node_g = bv;
                                npar = rl_u32(nlin, bsel);
                            }
                        }
                    }
                }
            }
#ifdef PMP_STAMPS
            const uint64_t ts2 = __builtin_amdgcn_s_memtime();
            cyc_pop += ts1 - ts0;
            cyc_wait += ts2 - ts1;
#endif
            if (sclosed && node_g >= scg) continue;
            niter++;
            // Neighbour decisions first (:66-75): they consume this round's loads before any store is
            // issued below, so the compiler never has to drain those stores (vmcnt) to read them.
            const double g1 = node_g + mcost;
            const bool ok = lane < 26 && !coll && !(ncd != 0u && g1 >= ncg);
            double tg = g1;
            uint32_t qpar = lin;
            if (THETA) {
                // updateVertex with node_p = CLOSED[node.parent] (theta_star3d.py:86-110 with
                // lineOfSight(q, node_p); lazy_theta_star3d.py:104-128 without it)
                // the reference reads CLOSED[node.parent] after inserting the node itself
                const double gp = npar == lin ? node_g : rl_f64(lane == 0 ? cg[npar] : 0.0, 0);
                const int px = (int)(npar / ((uint32_t)Y * Z)), py = (int)((npar / (uint32_t)Z) % (uint32_t)Y),
                          pz = (int)(npar % (uint32_t)Z);
                if (ok && (THETA == 2 || los3d<OCC_LDS>(occ, occl, X, Y, Z, nx, ny, nz, px, py, pz))) {
                    const double alt = gp + dist3(nx - px, ny - py, nz - pz);
                    if (alt < tg) {
                        tg = alt;
                        qpar = npar;
                    }
                }
            }
            // The key (f, h, counter) is a total order, so only the heap's contents matter.  An entry
            // whose cell already has a pending entry with g <= tg pops after it (f = g + h, equal
            // g -> earlier counter) and is then skipped by the CLOSED check (:48-50): it is dead on
            // arrival and is not inserted.  A strictly better entry is inserted and makes the old
            // one dead instead (skipped the same way when it pops).
            const bool live = THETA == 2 ? ok : (ok && tg < nog);
            const uint32_t okm = (uint32_t)ballot(ok);
            uint64_t vm = ballot(live);
            if (lane == 0) {
                if (!sclosed) {
                    if (expand_out && nexp < expand_cap) expand_out[(size_t)q * expand_cap + nexp] = lin;
                }
                cdir[lin] = (uint8_t)(ndir + 1);
                cg[lin] = node_g;
                if (THETA) cpar[lin] = npar;
            }
            if (!sclosed) nexp++;
            if (((node.b >> 5) & 0xFFFFFFu) == goal_xyz24) {  // goal check (:59-63), path via CLOSED parents
                st = PMP_FOUND;
                heap16::wsync();
                if (THETA && lane == 0) {  // extractPath via CLOSED parents (theta_star3d.py:217-232)
                    uint32_t c = lin;
                    const uint32_t st_c = ((uint32_t)sx * (uint32_t)Y + (uint32_t)sy) * (uint32_t)Z + (uint32_t)sz;
                    int len = 1;
                    double cost = 0.0;
                    while (c != st_c && len <= (int)ncell) {
                        const uint32_t p = cpar[c];
                        const int ddx = (int)(c / ((uint32_t)Y * Z)) - (int)(p / ((uint32_t)Y * Z));
                        const int ddy = (int)((c / (uint32_t)Z) % (uint32_t)Y) - (int)((p / (uint32_t)Z) % (uint32_t)Y);
                        const int ddz = (int)(c % (uint32_t)Z) - (int)(p % (uint32_t)Z);
                        cost += dist3(ddx, ddy, ddz);
                        c = p;
                        len++;
                    }
                    goal_cost = cost;
                    plen = len;
                    if (len <= path_cap) {
                        uint32_t* pth = path_out + (size_t)q * path_cap;
                        c = lin;
                        for (int i = len - 1; i >= 0; i--) {
                            pth[i] = c;
                            if (i == 0) break;
                            c = cpar[c];
                        }
                    }
                } else if (!THETA && lane == 0) {
                    int cx = x, cy = y, cz = z, len = 1;
                    double cost = 0.0;
                    while (!(cx == sx && cy == sy && cz == sz)) {  // goal -> start: cost and length
                        const uint32_t li = ((uint32_t)cx * (uint32_t)Y + (uint32_t)cy) * (uint32_t)Z + (uint32_t)cz;
                        const int d = (int)cdir[li] - 1;
                        const int chg = (c_m3[d][0] != 0) + (c_m3[d][1] != 0) + (c_m3[d][2] != 0);
                        cost += __dsqrt_rn((double)chg);
                        cx -= c_m3[d][0];
                        cy -= c_m3[d][1];
                        cz -= c_m3[d][2];
                        len++;
                    }
                    goal_cost = cost;
                    plen = len;
                    if (len <= path_cap) {  // write start -> goal (path.reverse(), :105)
                        uint32_t* pth = path_out + (size_t)q * path_cap;
                        cx = x; cy = y; cz = z;
                        for (int i = len - 1; i >= 0; i--) {
                            const uint32_t li = ((uint32_t)cx * (uint32_t)Y + (uint32_t)cy) * (uint32_t)Z + (uint32_t)cz;
                            pth[i] = li;
                            if (i == 0) break;
                            const int d = (int)cdir[li] - 1;
                            cx -= c_m3[d][0];
                            cy -= c_m3[d][1];
                            cz -= c_m3[d][2];
                        }
                    }
                }
                break;
            }
            // ---- neighbours (:66-75): push the live ones with the reference's counters
            npush += __popc(okm);  // the reference's pushes
            if (live && THETA != 2) og[nlin] = tg;
            Ent item;
            item.g = tg;
            item.a = 0u;
            item.b = ((((uint32_t)nx & 255u) << 16) | (((uint32_t)ny & 255u) << 8) | ((uint32_t)nz & 255u)) << 5 | (uint32_t)(lane < 26 ? lane : 0);
            qc.set_f(item);
            bool overflow = false;
#ifndef PMP_A3_BATCH
#define PMP_A3_BATCH 1
#endif
            if (THETA == 0 && PMP_A3_BATCH && vm) {
                // The key is a total order, so the heap's shape is free: the live neighbours are stored
                // together at n, n + 1, ... (lane order) in one round, and only the ones below their
                // parent (an entry from before this batch; else assumed below) sift up afterwards, in
                // position order -- a sift-up only lowers the parents of the later ones, so an item
                // found not below its parent stays so.  Most pushes cost no heap operation of their own.
                if (n + __popcll(vm) > heap_cap) {
                    overflow = true;
                } else {
                    Ent it = item;
                    it.a = seq + (uint32_t)__popc(okm & ((1u << (lane & 31)) - 1u));
                    n = heap16::push_batch(hp, qc, n, vm, it, root, lane);
                }
                vm = 0;
            }
            while (vm) {
                const int m = __ffsll((long long)vm) - 1;
                vm &= vm - 1;
                Ent it = heap16::rl_ent(item, m);
                // counter = the reference's push index of this neighbour
                it.a = seq + (uint32_t)__popc(okm & ((1u << m) - 1u));
                if (THETA) {
                    if (it.a >= ppar_cap) { overflow = true; break; }
                    if (lane == 0) ppar[it.a] = rl_u32(qpar, m);
                }
                if (n >= heap_cap) { overflow = true; break; }
                if (n < lds_cap) heap16::sift_up<Key3, false>(hp, qc, n, it, root, lane);
                else heap16::sift_up<Key3, true>(hp, qc, n, it, root, lane);
                n += 1;
            }
            seq += (uint32_t)__popc(okm);
#ifdef PMP_STAMPS
            cyc_push += __builtin_amdgcn_s_memtime() - ts2;
#endif
            if (n > maxn) maxn = n;
            if (overflow) { st = PMP_CAP_OVERFLOW; break; }
        }
        if (lane == 0) {
            int s = st;
            if (s == PMP_FOUND && plen > path_cap) s = PMP_PATH_OVERFLOW;
            status_out[q] = s;
            cost_out[q] = st == PMP_FOUND ? goal_cost : __builtin_inf();
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
                counters[4 * q + 2] = niter;
                counters[4 * q + 3] = maxn;
#endif
            }
        }
        heap16::wsync();
    }
}

// ---- longest-first schedule: counting sort of the queries by descending start-goal distance ----
__device__ __forceinline__ int lpt3_key(const int32_t* s, const int32_t* g, int q)
{
    // in double (endpoints may lie far outside the grid: the kernels report those queries, this
    // pre-pass must only stay in range), clamped to the histogram [0, nb - 1] by the callers
    const double dx = (double)s[3 * q] - g[3 * q], dy = (double)s[3 * q + 1] - g[3 * q + 1],
                 dz = (double)s[3 * q + 2] - g[3 * q + 2];
    const double d = __dsqrt_rn(dx * dx + dy * dy + dz * dz);
    return d < 2147483647.0 ? (int)d : 2147483647;
}
__global__ void lpt3_hist(const int32_t* s, const int32_t* g, int nq, int nb, int* hist)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) atomicAdd(&hist[min(lpt3_key(s, g, q), nb - 1)], 1);
}
__global__ void lpt3_scan(int nb, int* hist)  // offsets[k] = queries with a larger key; one thread
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int run = 0;
    for (int k = nb - 1; k >= 0; k--) {
        const int c = hist[k];
        hist[k] = run;
        run += c;
    }
}
__global__ void lpt3_scatter(const int32_t* s, const int32_t* g, int nq, int nb, int* offs, int32_t* order)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) order[atomicAdd(&offs[min(lpt3_key(s, g, q), nb - 1)], 1)] = q;
}

// per-context scratch budget of the 3D planners (heap spill + closed state + Theta* parents per worker)
#ifndef PMP_ASTAR3D_BUDGET_GIB
#define PMP_ASTAR3D_BUDGET_GIB 48  // 32: ~4,870 workers at C5 (2.05 M plans/s), 48: the 20-per-CU 5,120 (2.09-2.11 M, tools/calls/r6_call53.sh)
#endif
constexpr size_t kScratchBudget3 = (size_t)PMP_ASTAR3D_BUDGET_GIB << 30;

}  // namespace

int pmp_lpt_order3d(pmp_ctx* ctx, hipStream_t s, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, int X,
                    int Y, int Z, int workers, int32_t** order)
{
    *order = nullptr;
    if (!ctx->astar_lpt || nq <= workers) return PMP_OK;
    const int nb = (int)ceil(sqrt((double)X * X + (double)Y * Y + (double)Z * Z)) + 1;
    int* hist = (int*)pmp_scratch(ctx, SCR_PDIR, sizeof(int) * ((size_t)nb + (size_t)nq));
    if (!hist) return PMP_ENOMEM;
    int32_t* ord = hist + nb;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(hist, 0, sizeof(int) * (size_t)nb, s));
    hipLaunchKernelGGL(lpt3_hist, dim3((nq + 255) / 256), dim3(256), 0, s, start_xyz, goal_xyz, nq, nb, hist);
    hipLaunchKernelGGL(lpt3_scan, dim3(1), dim3(64), 0, s, nb, hist);
    hipLaunchKernelGGL(lpt3_scatter, dim3((nq + 255) / 256), dim3(256), 0, s, start_xyz, goal_xyz, nq, nb, hist, ord);
    *order = ord;
    return PMP_OK;
}

extern "C" int pmp_graph3d_batch(pmp_ctx* ctx, void* stream, int algo, const uint32_t* occ_bits, int per_query, int X,
                                 int Y, int Z, int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq,
                                 double* cost, int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                                 uint32_t* expand, int expand_cap, int64_t* counters, int32_t* status)
{
    if (!ctx) return PMP_EINVAL;
    if (algo < PMP_ALGO_ASTAR || algo > PMP_ALGO_LAZY_THETA)
        return pmp_set_err(ctx, PMP_EINVAL,
                           "pmp_graph3d_batch: algo must be 0 (AStar3D), 1 (Dijkstra3D), 2 (GBFS3D), 3 (ThetaStar3D) or "
                           "4 (LazyThetaStar3D)");
    if (X < 1 || Y < 1 || Z < 1 || X > kMaxDim3 || Y > kMaxDim3 || Z > kMaxDim3)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar3d_batch: X, Y, Z must be in [1, 256]");
    if (heuristic != 0 && heuristic != 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar3d_batch: heuristic must be 0 or 1");
    if (nq < 0 || path_cap < 1 || (expand && expand_cap < 1))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar3d_batch: bad nq/path_cap/expand_cap");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xyz || !goal_xyz || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar3d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t ncell = (size_t)X * Y * Z;
    // workers per CU: the configured count (default 16: C5's 8192-query batches run fastest at 16-24,
    // tools/astar3d_sweep.py), but no more than the batch fills, so small batches get a larger LDS
    // heap share per worker
    const int per_cu = std::max(1, std::min(ctx->workers_per_cu > 0 ? ctx->workers_per_cu : 16, (nq + 255) / 256));
    int workers = 256 * per_cu;
    if (workers > nq) workers = nq;
    const size_t words = (ncell + 31) / 32;
    bool occ_lds = words <= (size_t)kOccLdsWords;
    // the query's bitmap in LDS takes its own size (C5: 260 words), the rest of the share is heap
    int occ_bytes = occ_lds ? (int)((words * 4 + 15) & ~(size_t)15) : 0;
    constexpr int kEnt = heap16::lds_entry_bytes<true>(), kSpill = heap16::spill_entry_bytes<true>();
    int lds_cap = pmp_heap_lds_cap(ctx, per_cu, occ_bytes, kEnt);
    if (lds_cap < kMinLdsHeap && occ_lds) {  // the LDS share cannot hold the occupancy too: keep it in HBM
        occ_lds = false;
        occ_bytes = 0;
        lds_cap = pmp_heap_lds_cap(ctx, per_cu, 0, kEnt);
    }
    if (lds_cap < kMinLdsHeap)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_graph3d_batch: workers / resident per CU leave no LDS heap share");
    size_t hc = 26 * ncell + 8;
    if (hc > (size_t)(1 << 22)) hc = (size_t)1 << 22;
    const int heap_cap = (int)hc;
    if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    const size_t spill_n = heap_cap > lds_cap ? (size_t)(heap_cap - lds_cap) : 0;
    const int theta = algo == PMP_ALGO_THETA ? 1 : (algo == PMP_ALGO_LAZY_THETA ? 2 : 0);
    // theta modes: CLOSED parent per cell, and the parent of every push (indexed by the push counter;
    // a query that pushes more stops with PMP_CAP_OVERFLOW)
    const uint32_t ppar_cap = theta ? (uint32_t)std::min<size_t>(64 * ncell + 64, (size_t)1 << 24) : 0u;
    {
        // per-context scratch budget: fewer workers (each pulls more queries) rather than ENOMEM
        const size_t per_worker = spill_n * kSpill + ncell + ncell * 16 +
                                  (theta ? ((size_t)ncell + ppar_cap) * 4 : 0);
        const size_t fit = kScratchBudget3 / per_worker;
        if (fit < 1) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_graph3d_batch: one worker exceeds the scratch budget");
        if ((size_t)workers > fit) workers = (int)fit;
    }
    uint4* spill = (uint4*)pmp_scratch(ctx, SCR_AUX1, (size_t)workers * spill_n * kSpill + 16);
    uint8_t* cdir = (uint8_t*)pmp_scratch(ctx, SCR_AUX2, (size_t)workers * ncell + 16);
    double* cg = (double*)pmp_scratch(ctx, SCR_AUX3, (size_t)workers * ncell * 16 + 16);  // closed g + pending g
    int* queue = (int*)pmp_scratch(ctx, SCR_AUX0, 256);
    uint32_t* tpar = nullptr;  // theta: CLOSED parents + push parents
    if (theta) {
        tpar = (uint32_t*)pmp_scratch(ctx, SCR_AUX4, (size_t)workers * (ncell + ppar_cap) * 4 + 16);
        if (!tpar) return PMP_ENOMEM;
    }
    if (!spill || !cdir || !cg || !queue) return PMP_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    int32_t* order = nullptr;
    {
        const int rc = pmp_lpt_order3d(ctx, s, start_xyz, goal_xyz, nq, X, Y, Z, workers, &order);
        if (rc) return rc;
    }
    auto kern = occ_lds ? (theta == 1 ? astar3d_kernel<true, 1> : theta == 2 ? astar3d_kernel<true, 2> : astar3d_kernel<true, 0>)
                        : (theta == 1 ? astar3d_kernel<false, 1> : theta == 2 ? astar3d_kernel<false, 2> : astar3d_kernel<false, 0>);
    hipLaunchKernelGGL(kern, dim3(workers), dim3(64), (size_t)lds_cap * kEnt + occ_bytes, s, occ_bits, per_query, X, Y, Z,
                       algo == PMP_ALGO_DIJKSTRA ? 2 : heuristic, start_xyz, goal_xyz, nq, cost, path_len, path, path_cap,
                       n_expanded, expand, expand_cap, counters, status, queue, spill, heap_cap, lds_cap, cdir, cg,
                       algo == PMP_ALGO_GBFS ? 1 : 0, theta ? tpar : nullptr, theta ? tpar + (size_t)workers * ncell : nullptr,
                       ppar_cap, (const int32_t*)order, order ? ctx->astar_prio_n : 0);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

extern "C" int pmp_astar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y,
                                 int Z, int heuristic, const int32_t* start_xyz, const int32_t* goal_xyz, int nq,
                                 double* cost, int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                                 uint32_t* expand, int expand_cap, int64_t* counters, int32_t* status)
{
    return pmp_graph3d_batch(ctx, stream, PMP_ALGO_ASTAR, occ_bits, per_query, X, Y, Z, heuristic, start_xyz, goal_xyz, nq,
                             cost, path_len, path, path_cap, n_expanded, expand, expand_cap, counters, status);
}
