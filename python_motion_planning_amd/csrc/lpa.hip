// Batched LPA* for gfx950: LPAStar.plan (global_planner/graph_search/lpa_star.py:78-87) =
// computeShortestPath (:139-160) + extractPath (:209-230), bit-exact with the reference including
// its OPEN "set" U, which is a Python list:
//   * min(U, key=key) returns the FIRST minimal element in list order (:141);
//   * U.remove(node) shifts the list tail left by one (:149, :173);
//   * heapq.heappush(U, node) appends and sifts by LNode.__lt__ (key list compare, :32-33) on
//     whatever order the list holds after the removes (:178).
// So the kernel keeps the list itself, element for element: U = {cell, k1, k2} arrays in LDS (the
// wave's share; a list that outgrows it moves to HBM arrays for the rest of its query).  `node in U`
// and U.remove's search are a scan of the cells (a node is in U at most once: updateVertex removes
// it before pushing it again).
//
// DStarLite.plan (d_star_lite.py:14-187; plan() is LPAStar's) is the same loop run backwards: the
// node created with rhs = 0 is the goal, the search ends on the start's consistency, keys add
// h(node, start) + km (km = 0 in plan()), a popped node with an outdated key is only re-keyed
// (:104-106), and extractPath walks start -> goal without reversing (`lite` below).
//
// Execution model: one wave64 per query (persistent workers over an atomic queue).  The wave
// scans U for the minimum (64 lanes, first index on ties), shifts the tail 64 elements per
// instruction, sifts a push with one load round of the ancestors (the "less" prefix from the
// parent up is a ballot's trailing-ones count), and evaluates a node's 8 neighbours on lanes 0..7
// (rhs = min over them, :166-167).
#include "pmp_internal.h"

namespace {

constexpr int kMaxDim = 8192;
constexpr double kSqrt2 = 1.4142135623730951;  // math.hypot(1, 1)
constexpr double kInf = __builtin_huge_val();

// motions in the order of env.py:52-55
__constant__ int kMX[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
__constant__ int kMY[8] = {0, 1, 1, 1, 0, -1, -1, -1};

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) int32_t lds_i32;

struct Q {
    const uint32_t* occ;
    int W, H, heur;
    int32_t src, tgt;  // src: the node created with rhs = 0; tgt: ends the search, h points at it
    int gx, gy;        // tgt's coordinates
    double* g;
    double* rhs;
    int32_t* Uc;   // U in HBM (a list past the LDS share)
    double* Uk1;
    double* Uk2;
    lds_i32* Lc;   // U in LDS
    lds_f64* L1;
    lds_f64* L2;
    int cap;       // LDS entries
    bool lds;      // U is in LDS (wave-uniform)
    int n;         // |U| (wave-uniform)
    int64_t npush;
    double km;     // D* Lite's key offset (0 in plan(), set by OnPress)
};

__device__ __forceinline__ bool occ_at(const uint32_t* occ, int H, int x, int y)
{
    const uint32_t ci = (uint32_t)x * (uint32_t)H + (uint32_t)y;
    return ((occ[ci >> 5] >> (ci & 31u)) & 1u) != 0u;
}
__device__ __forceinline__ bool key_lt(double a1, double a2, double b1, double b2)
{
    return a1 < b1 || (a1 == b1 && a2 < b2);
}
__device__ __forceinline__ void wave_sync_mem() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// calculateKey's h (GraphSearcher.h, graph_search.py:41-44): hypot of integer deltas == the
// correctly rounded sqrt of the exact square sum; manhattan |dx| + |dy|
__device__ __forceinline__ double hval(const Q& S, int x, int y)
{
    const int dx = S.gx - x, dy = S.gy - y;
    return S.heur == 1 ? (double)(abs(dx) + abs(dy)) : __dsqrt_rn((double)(dx * dx + dy * dy));
}

// list entry k of U, wherever the list lives
__device__ __forceinline__ int32_t u_c(const Q& S, int k) { return S.lds ? S.Lc[k] : S.Uc[k]; }
__device__ __forceinline__ double u_k1(const Q& S, int k) { return S.lds ? S.L1[k] : S.Uk1[k]; }
__device__ __forceinline__ double u_k2(const Q& S, int k) { return S.lds ? S.L2[k] : S.Uk2[k]; }
__device__ __forceinline__ void u_set(const Q& S, int k, int32_t c, double a, double b)
{
    if (S.lds) {
        S.Lc[k] = c;
        S.L1[k] = a;
        S.L2[k] = b;
    } else {
        S.Uc[k] = c;
        S.Uk1[k] = a;
        S.Uk2[k] = b;
    }
}

// position of node v in U, or -1 (`node in U`, list.index)
__device__ __forceinline__ int u_find(const Q& S, int32_t v, int lane)
{
    for (int k0 = 0; k0 < S.n; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t m = ballot(k < S.n && u_c(S, k < S.n ? k : 0) == v);
        if (m) return k0 + __ffsll((long long)m) - 1;
    }
    return -1;
}

// U.remove(U[i]): the tail moves left one slot, 64 elements per round (every lane loads before
// any lane stores, and a round never reads what an earlier round wrote)
__device__ void u_remove(Q& S, int i, int lane)
{
    for (int base = i; base < S.n - 1; base += 64) {
        const int k = base + lane;
        const bool on = k < S.n - 1;
        int32_t c = 0;
        double a = 0.0, b = 0.0;
        if (on) {
            c = u_c(S, k + 1);
            a = u_k1(S, k + 1);
            b = u_k2(S, k + 1);
        }
        wave_sync_mem();
        if (on) u_set(S, k, c, a, b);
        wave_sync_mem();
    }
    S.n -= 1;
}

// heapq.heappush(U, (c, k1, k2)): lane j (1..D) loads ancestor j of position n; the ancestors that
// move down are the run of "new < ancestor" from the parent up (CPython _siftdown stops at the
// first one that is not greater)
__device__ void u_push(Q& S, int32_t c, double k1, double k2, int lane)
{
    if (S.lds && S.n + 1 > S.cap) {  // the list outgrows the LDS share: to HBM for the rest of the query
        for (int k = lane; k < S.n; k += 64) {
            S.Uc[k] = S.Lc[k];
            S.Uk1[k] = S.L1[k];
            S.Uk2[k] = S.L2[k];
        }
        S.lds = false;
        wave_sync_mem();
    }
    const uint32_t np1 = (uint32_t)S.n + 1u;
    const int D = 31 - __clz((int)np1);
    const bool on = lane >= 1 && lane <= D;
    const int aj = on ? (int)(np1 >> lane) - 1 : 0;
    int32_t ac = 0;
    double a1 = 0.0, a2 = 0.0;
    if (on) {
        ac = u_c(S, aj);
        a1 = u_k1(S, aj);
        a2 = u_k2(S, aj);
    }
    const uint64_t lt = ballot(on && key_lt(k1, k2, a1, a2));
    const int t = __builtin_ctzll(~(lt >> 1));  // trailing ones from lane 1
    wave_sync_mem();
    if (on && lane <= t) u_set(S, (int)(np1 >> (lane - 1)) - 1, ac, a1, a2);  // ancestor j to j - 1 (0 = position n)
    if (lane == 0) u_set(S, (int)(np1 >> t) - 1, c, k1, k2);
    wave_sync_mem();
    S.n += 1;
    S.npush += 1;
}

// updateVertex (:162-179).  Returns PMP_REF_RAISES when the reference raises (KeyError: a
// neighbour off the map; ValueError: min() of an empty neighbour list).
__device__ int update_vertex(Q& S, int32_t v, int lane)
{
    const int vx = (int)((uint32_t)v / (uint32_t)S.H), vy = v - vx * S.H;
    const int m = lane & 7;
    // Every read of this call issues up front, unconditionally (in-grid addresses on every lane):
    // the neighbour's occupancy words and g, and v's g / rhs / U position -- one round trip where
    // short-circuit tests and lane-0 blocks made several.
    const int ux = vx + kMX[m], uy = vy + kMY[m];
    const bool in = (unsigned)ux < (unsigned)S.W && (unsigned)uy < (unsigned)S.H;
    const bool act = lane < 8 && in;
    const int uxs = act ? ux : vx, uys = act ? uy : vy;
    const bool ou = occ_at(S.occ, S.H, uxs, uys), ov = occ_at(S.occ, S.H, vx, vy);
    const bool oa = occ_at(S.occ, S.H, uxs, vy), ob = occ_at(S.occ, S.H, vx, uys);
    const double gu = S.g[uxs * S.H + uys];
    const double gv = S.g[v], rsrc = S.rhs[v];
    const int p = u_find(S, v, lane);
    double rv;
    if (v != S.src) {
        // getNeighbor (:196-207): map lookup (KeyError off the grid), then the obstacle filter;
        // cost (graph_search.py:46-59): inf on isCollision(node_n, node), else hypot
        const bool valid = act && !ou;
        const bool coll = ou | ov | ((m & 1) ? (oa | ob) : false);
        const double val = act ? gu + (coll ? kInf : ((m & 1) ? kSqrt2 : 1.0)) : kInf;
        if (ballot(lane < 8 && !in)) return PMP_REF_RAISES;
        if (!ballot(valid)) return PMP_REF_RAISES;
        double best = valid ? val : kInf;
        for (int o = 1; o < 8; o <<= 1) best = fmin(best, __shfl_xor(best, o, 64));
        rv = __shfl(best, 0, 64);
        if (lane == 0) S.rhs[v] = rv;
    } else {
        rv = rsrc;
    }
    const int pu = uni(p);
    if (pu >= 0) u_remove(S, pu, lane);  // `node in U`: U.remove(node)
    if (gv != rv) {
        const double mn = gv < rv ? gv : rv;
        u_push(S, v, mn + hval(S, vx, vy) + S.km, mn, lane);
    }
    return 0;
}

// One greedy step of extractPath (lpa_star.py:209-230) / D* Lite's OnPress walk (d_star_lite.py:
// 73-83): the first minimal-g neighbour in motion order among the free ones that isCollision allows.
// Returns the motion, or -1 where the reference raises (KeyError off the grid, min() of nothing).
__device__ int greedy_step(const Q& S, int32_t c, int lane)
{
    const int H = S.H;
    const int x = (int)((uint32_t)c / (uint32_t)H), y = c - x * H;
    const int m = lane & 7;
    const int ux = x + kMX[m], uy = y + kMY[m];
    const bool in = (unsigned)ux < (unsigned)S.W && (unsigned)uy < (unsigned)H;
    // all reads issued together (in-grid addresses on every lane)
    const bool act = lane < 8 && in;
    const int uxs = act ? ux : x, uys = act ? uy : y;
    const bool o1 = occ_at(S.occ, H, uxs, uys), o2 = occ_at(S.occ, H, x, y);
    const bool o3 = occ_at(S.occ, H, uxs, y), o4 = occ_at(S.occ, H, x, uys);
    const double gu = S.g[uxs * H + uys];
    const bool valid = act && !(o1 | o2 | ((m & 1) ? (o3 | o4) : false));
    if (ballot(lane < 8 && !in)) return -1;
    uint64_t vm = ballot(valid) & 0xffull;
    int bm = -1;
    double bg = 0.0;
    while (vm) {
        const int k = __ffsll((long long)vm) - 1;
        vm &= vm - 1;
        const double gk = __shfl(gu, k, 64);
        if (bm < 0 || gk < bg) { bm = k; bg = gk; }
    }
    return bm;
}

// OnPress's obstacle edit at (tx, ty) (lpa_star.py:113-122 == d_star_lite.py:85-93): flip the cell in
// the worker's grid, updateVertex the cell if it was freed, then its free neighbours
__device__ int toggle_cell(Q& S, uint32_t* occ_w, int tx, int ty, int lane)
{
    const int H = S.H;
    const int32_t tc = tx * H + ty;
    const bool was = occ_at(S.occ, H, tx, ty);
    if (lane == 0) {
        if (was) occ_w[tc >> 5] &= ~(1u << (tc & 31));
        else occ_w[tc >> 5] |= 1u << (tc & 31);
    }
    wave_sync_mem();
    int st = 0;
    if (was) st = update_vertex(S, tc, lane);
    if (!st) {  // getNeighbor(node_change): KeyError off the grid before any update
        const int ux = tx + kMX[lane & 7], uy = ty + kMY[lane & 7];
        const bool in = (unsigned)ux < (unsigned)S.W && (unsigned)uy < (unsigned)H;
        if (ballot(lane < 8 && !in)) st = PMP_REF_RAISES;
        const uint32_t nbm = (uint32_t)ballot(lane < 8 && in && !occ_at(S.occ, H, ux, uy)) & 0xffu;
        for (int m = 0; m < 8 && !st; m++)
            if ((nbm >> m) & 1u) st = update_vertex(S, (tx + kMX[m]) * H + (ty + kMY[m]), lane);
    }
    return st;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void lpa_kernel(const uint32_t* __restrict__ occ, int W, int H, int heur,
                                                 const int32_t* __restrict__ start_xy,
                                                 const int32_t* __restrict__ goal_xy, int nq, double* __restrict__ cost_out,
                                                 int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out,
                                                 int path_cap, int32_t* __restrict__ nexp_out,
                                                 int64_t* __restrict__ counters, int32_t* __restrict__ status_out,
                                                 int* __restrict__ queue, double* __restrict__ scr_f64,
                                                 int32_t* __restrict__ scr_i32, int lite,
                                                 const int32_t* __restrict__ toggles, int nt,
                                                 double* __restrict__ rp_cost, int32_t* __restrict__ rp_nexp,
                                                 int32_t* __restrict__ rp_status, uint32_t* __restrict__ occ_scr, int ucap)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const size_t ncell = (size_t)W * (size_t)H;
    const size_t nwords = (ncell + 31) / 32;
    Q S;
    // replanning toggles obstacles, so each worker then works on its own copy of the grid
    uint32_t* occ_w = nt > 0 ? occ_scr + (size_t)blockIdx.x * nwords : nullptr;
    S.occ = nt > 0 ? occ_w : occ;
    S.W = W;
    S.H = H;
    S.heur = heur;
    {
        double* f = scr_f64 + (size_t)blockIdx.x * 4 * ncell;
        int32_t* i = scr_i32 + (size_t)blockIdx.x * 2 * ncell;
        S.g = f;
        S.rhs = f + ncell;
        S.Uk1 = f + 2 * ncell;
        S.Uk2 = f + 3 * ncell;
        S.Uc = i;
        S.L1 = (lds_f64*)smem;
        S.L2 = (lds_f64*)(smem + (size_t)8 * ucap);
        S.Lc = (lds_i32*)(smem + (size_t)16 * ucap);
        S.cap = ucap;
    }
    for (;;) {
        const int q = next_query(queue, lane);
        if (q >= nq) break;
        const int sx = uni(start_xy[2 * q]), sy = uni(start_xy[2 * q + 1]);
        const int gx = uni(goal_xy[2 * q]), gy = uni(goal_xy[2 * q + 1]);
        int st = 0;
        int64_t nexp = 0, steps = 0, maxn = 0;
        double cost = 0.0;
        int len = 0;
        S.gx = lite ? sx : gx;
        S.gy = lite ? sy : gy;
        S.n = 0;
        S.lds = true;
        S.npush = 0;
        S.km = 0.0;
        if (!((unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H && (unsigned)gx < (unsigned)W &&
              (unsigned)gy < (unsigned)H)) {
            st = PMP_REF_RAISES;  // map lookups off the grid (KeyError)
        } else {
            for (size_t i = lane; i < ncell; i += 64) {
                S.g[i] = kInf;
                S.rhs[i] = kInf;
            }
            if (nt > 0)
                for (size_t i = lane; i < nwords; i += 64) occ_w[i] = occ[i];
            wave_sync_mem();
            const int32_t start = sx * H + sy, goal = gx * H + gy;
            S.src = lite ? goal : start;
            S.tgt = lite ? start : goal;
            // start == goal: map[start] overwrote map[goal] (lpa_star.py:62-63, d_star_lite.py:58-59).
            // LPA*: self.goal is a detached LNode(goal, inf, inf), so the loop ends only when U
            // empties.  D* Lite: the detached node is the goal in U; its g = 0 never reaches a
            // neighbour's rhs, so the first expansion pushes nothing and U empties.
            const bool detached = start == goal;
            if (lane == 0) S.rhs[S.src] = 0.0;  // LNode(start, inf, 0.0) (lpa_star.py:59) / LNode(goal, inf, 0.0)
            wave_sync_mem();
            u_push(S, S.src, hval(S, lite ? gx : sx, lite ? gy : sy), 0.0, lane);
            maxn = 1;
            if (lite && detached) {
                nexp = 1;
                S.n = 0;
            }
            // phase 0: plan(); phase p >= 1: LPAStar.OnPress (lpa_star.py:101-137) at toggles[p - 1]:
            // flip the cell, updateVertex(cell) if it was freed, updateVertex on its free neighbours,
            // then plan() again on the kept g / rhs / U (EXPAND restarts)
            for (int phase = 0; phase <= nt; phase++) {
            // D* Lite's OnPress (d_star_lite.py:61-97): walk from the start along min-g neighbours; after
            // the first step set km = h(step, start), edit the cell, computeShortestPath, walk on
            int32_t wcur = S.tgt;
            if (phase > 0) {
                nexp = 0;
                steps = 0;
                cost = 0.0;
                len = 0;
                const int tx = uni(toggles[2 * ((size_t)q * nt + phase - 1)]);
                const int ty = uni(toggles[2 * ((size_t)q * nt + phase - 1) + 1]);
                if (lite) {
                    uint32_t* pth = path_out + (size_t)q * path_cap;
                    if (lane == 0 && len < path_cap) pth[len] = (uint32_t)wcur;
                    len++;
                    if (wcur != S.src) {
                        const int bm = greedy_step(S, wcur, lane);
                        if (bm < 0) {
                            st = PMP_REF_RAISES;
                        } else {
                            cost += (bm & 1) ? kSqrt2 : 1.0;
                            const int x = (int)((uint32_t)wcur / (uint32_t)H), y = wcur - x * H;
                            wcur = (x + kMX[bm]) * H + (y + kMY[bm]);
                            if (lane == 0 && len < path_cap) pth[len] = (uint32_t)wcur;
                            len++;
                            steps++;
                            // km = h(cur_start, new_start) with new_start = self.start
                            const int cx = x + kMX[bm], cy = y + kMY[bm];
                            S.km = S.heur == 1 ? (double)(abs(sx - cx) + abs(sy - cy))
                                               : __dsqrt_rn((double)((sx - cx) * (sx - cx) + (sy - cy) * (sy - cy)));
                            st = toggle_cell(S, occ_w, tx, ty, lane);
                        }
                    } else {
                        st = -2;  // the walk never starts: no edit, no search (marker, cleared below)
                    }
                } else {
                    st = toggle_cell(S, occ_w, tx, ty, lane);
                }
            }
            for (;;) {
                if (st) break;
                if (S.n == 0) { st = PMP_REF_RAISES; break; }  // min() of an empty list
                // safety bound only (LPA* on a static grid settles every cell a bounded number of
                // times): a runaway query stops with status 3 instead of holding the GPU
                if (nexp > (int64_t)64 * (int64_t)ncell + 64) { st = PMP_CAP_OVERFLOW; break; }
                // the target's g / rhs (read after the scan) issue first, beside it
                const double ggt = S.g[S.tgt], grt = S.rhs[S.tgt];
                // min(U, key=key): first minimal element in list order; 2 entries per lane in flight
                // (increasing k per lane, as the one-at-a-time loop)
                double b1 = kInf, b2 = kInf;
                int bi = 0x7fffffff;
                for (int k0 = lane; k0 < S.n; k0 += 128) {
                    double a1[2], a2[2];
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const int k = k0 + 64 * u < S.n ? k0 + 64 * u : k0;
                        a1[u] = u_k1(S, k);
                        a2[u] = u_k2(S, k);
                    }
#pragma unroll
                    for (int u = 0; u < 2; u++)
                        if (k0 + 64 * u < S.n && (bi == 0x7fffffff || key_lt(a1[u], a2[u], b1, b2))) {
                            b1 = a1[u]; b2 = a2[u]; bi = k0 + 64 * u;
                        }
                }
                for (int o = 1; o < 64; o <<= 1) {
                    const double o1 = __shfl_xor(b1, o, 64), o2 = __shfl_xor(b2, o, 64);
                    const int oi = __shfl_xor(bi, o, 64);
                    const bool take = oi != 0x7fffffff &&
                                      (bi == 0x7fffffff || key_lt(o1, o2, b1, b2) || (o1 == b1 && o2 == b2 && oi < bi));
                    if (take) { b1 = o1; b2 = o2; bi = oi; }
                }
                bi = uni(bi);
                b1 = __shfl(b1, 0, 64);
                b2 = __shfl(b2, 0, 64);
                const int32_t vt = u_c(S, bi);  // every lane the same word
                const double gg = detached ? kInf : ggt;
                const double gr = detached ? kInf : grt;
                const double gm = gg < gr ? gg : gr;
                if (!key_lt(b1, b2, gm + 0.0 + S.km, gm) && gr == gg) break;  // calculateKey(tgt): h = 0
                const int32_t v = uni(vt);
                // v's g / rhs (not touched by the list shift) load before it, on every lane
                const double gv = S.g[v], rv = S.rhs[v];
                u_remove(S, bi, lane);
                nexp++;
                const int vx = (int)((uint32_t)v / (uint32_t)H), vy = v - vx * H;
                if (lite) {  // node.key < calculateKey(node): re-key and push, nothing else (:104-106)
                    const double mn = gv < rv ? gv : rv;
                    const double c1 = mn + hval(S, vx, vy) + S.km;
                    if (key_lt(b1, b2, c1, mn)) {
                        u_push(S, v, c1, mn, lane);
                        if (S.n > maxn) maxn = S.n;
                        continue;
                    }
                }
                if (gv > rv) {
                    if (lane == 0) S.g[v] = rv;
                    wave_sync_mem();
                } else {
                    if (lane == 0) S.g[v] = kInf;
                    wave_sync_mem();
                    if ((st = update_vertex(S, v, lane))) break;
                }
                // getNeighbor(node) (:196-207): the list is fixed before the updates
                uint32_t nbm = 0u;
                {
                    const int ux = vx + kMX[lane & 7], uy = vy + kMY[lane & 7];
                    const bool in = (unsigned)ux < (unsigned)W && (unsigned)uy < (unsigned)H;
                    const uint64_t bad = ballot(lane < 8 && !in);
                    const bool ok = lane < 8 && in && !occ_at(S.occ, H, ux, uy);
                    nbm = (uint32_t)ballot(ok) & 0xffu;
                    if (bad) st = PMP_REF_RAISES;  // KeyError while the list is built: no update runs
                }
                if (st) break;
                for (int m = 0; m < 8 && nbm; m++) {
                    if (!((nbm >> m) & 1u)) continue;
                    const int r = update_vertex(S, (vx + kMX[m]) * H + (vy + kMY[m]), lane);
                    if (r) { st = r; break; }
                }
                if (st) break;
                if (S.n > maxn) maxn = S.n;
            }
            if (st == -2) st = 0;  // D* Lite walk that starts at the goal: cost 0, path [start]
            else if (st == 0) {
                // extractPath (:209-230): greedy min-g neighbour from tgt, first minimum in motion order;
                // gives up (cost kept, empty path) after 1000 steps.  D* Lite's OnPress walk continues
                // from where its first step left it, with no step limit (a bound of its own here).
                const bool onpress = lite && phase > 0;
                uint32_t* pth = path_out + (size_t)q * path_cap;
                int32_t c = onpress ? wcur : S.tgt;
                if (!onpress) {
                    if (lane == 0 && len < path_cap) pth[len] = (uint32_t)c;
                    len++;
                }
                while (c != S.src) {
                    const int bm = greedy_step(S, c, lane);
                    if (bm < 0) { st = PMP_REF_RAISES; break; }
                    cost += (bm & 1) ? kSqrt2 : 1.0;
                    const int x = (int)((uint32_t)c / (uint32_t)H), y = c - x * H;
                    c = (x + kMX[bm]) * H + (y + kMY[bm]);
                    if (lane == 0 && len < path_cap) pth[len] = (uint32_t)c;
                    len++;
                    ++steps;
                    if (!onpress && steps == 1000) { st = PMP_NO_PATH; break; }
                    if (onpress && steps > (int64_t)4 * (int64_t)ncell + 4) { st = PMP_CAP_OVERFLOW; break; }
                }
                wave_sync_mem();
                if (st == 0) {
                    if (len > path_cap) st = PMP_PATH_OVERFLOW;
                    else if (!lite)  // LPA*: list(reversed(path)); D* Lite's runs start -> goal already
                        for (int i = lane; i < len / 2; i += 64) {
                            const uint32_t a = pth[i], b = pth[len - 1 - i];
                            pth[i] = b;
                            pth[len - 1 - i] = a;
                        }
                }
            }
            if (nt > 0 && lane == 0) {
                const size_t k = (size_t)q * (nt + 1) + phase;
                rp_cost[k] = (st == 0 || st == PMP_NO_PATH) ? cost : 0.0;
                rp_nexp[k] = (int32_t)nexp;
                rp_status[k] = st;
            }
            if (st != 0 && st != PMP_NO_PATH) {  // the reference raised: no further OnPress runs
                if (lane == 0)
                    for (int p2 = phase + 1; p2 <= nt; p2++) {
                        const size_t k = (size_t)q * (nt + 1) + p2;
                        rp_cost[k] = 0.0;
                        rp_nexp[k] = 0;
                        rp_status[k] = -1;
                    }
                break;
            }
            if (st == PMP_NO_PATH && phase < nt) st = 0;  // (cost, []) is a result, not a raise
            }  // phase
        }
        if (lane == 0) {
            status_out[q] = st;
            cost_out[q] = (st == 0 || st == PMP_NO_PATH) ? cost : 0.0;
            path_len_out[q] = st == 0 ? len : 0;
            nexp_out[q] = (int32_t)nexp;
            if (counters) {
                counters[4 * q] = S.npush;
                counters[4 * q + 1] = nexp;
                counters[4 * q + 2] = steps;
                counters[4 * q + 3] = maxn;
            }
        }
        wave_sync_mem();
    }
}

}  // namespace

static int lpa_batch(int lite, pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                     const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost, int32_t* path_len,
                     uint32_t* path, int path_cap, int32_t* n_expanded, int64_t* counters, int32_t* status,
                     const int32_t* toggles = nullptr, int nt = 0, double* rp_cost = nullptr, int32_t* rp_nexp = nullptr,
                     int32_t* rp_status = nullptr)
{
    if (!ctx) return PMP_EINVAL;
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_batch / pmp_dstarlite2d_batch: W and H must be in [1, 8192]");
    if (heuristic != 0 && heuristic != 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_batch / pmp_dstarlite2d_batch: heuristic must be 0 or 1");
    if (nq < 0 || path_cap < 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_batch / pmp_dstarlite2d_batch: bad nq/path_cap");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xy || !goal_xy || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_batch / pmp_dstarlite2d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t ncell = (size_t)W * H;
    const size_t per_worker = ncell * 36;  // g, rhs, U keys (f64) + U cells (i32); U itself in LDS until it outgrows it
    // one wave per query, 24 per CU by default (the kernel is capped at 80 VGPRs for 6 waves per
    // SIMD): each query is a dependent chain of short U scans and shifts (L2-latency bound), so more
    // resident waves hide more of it (16 -> 24 per CU: LPA* 1.46 M -> 1.55 M plans/s, replanning
    // 5.86 M -> 6.66 M)
    int workers = 256 * (ctx->workers_per_cu > 0 ? ctx->workers_per_cu : 24);  // pmp_set_workers_per_cu
    const size_t max_workers = ((size_t)16 << 30) / per_worker;  // scratch under 16 GiB
    if ((size_t)workers > max_workers) workers = (int)(max_workers > 0 ? max_workers : 1);
    if (workers > nq) workers = nq;
    double* f = (double*)pmp_scratch(ctx, SCR_AUX2, (size_t)workers * ncell * 32 + 16);
    int32_t* i32 = (int32_t*)pmp_scratch(ctx, SCR_AUX3, (size_t)workers * ncell * 4 + 16);
    int* queue = (int*)pmp_scratch(ctx, SCR_AUX0, 256);
    if (!f || !i32 || !queue) return PMP_ENOMEM;
    uint32_t* occ_scr = nullptr;
    if (nt > 0) {
        occ_scr = (uint32_t*)pmp_scratch(ctx, SCR_AUX4, (size_t)workers * ((ncell + 31) / 32) * 4 + 16);
        if (!occ_scr) return PMP_ENOMEM;
    }
    hipStream_t s = (hipStream_t)stream;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    // U's LDS share: the CU's 160 KiB over its resident workers (or the residency the context was
    // told to leave room for, pmp_set_resident_per_cu), 20 B per list entry
    const int per_cu = pmp_lds_share(ctx, (workers + 255) / 256);
    int ucap = ((160 * 1024) / (per_cu < 1 ? 1 : per_cu) / 20) & ~15;
    if (ucap > 4096) ucap = 4096;
    hipLaunchKernelGGL(lpa_kernel, dim3(workers), dim3(64), (size_t)ucap * 20, s, occ_bits, W, H, heuristic, start_xy,
                       goal_xy, nq, cost, path_len, path, path_cap, n_expanded, counters, status, queue, f, i32, lite,
                       toggles, nt, rp_cost, rp_nexp, rp_status, occ_scr, ucap);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

extern "C" int pmp_lpastar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                                   const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost,
                                   int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                                   int64_t* counters, int32_t* status)
{
    return lpa_batch(0, ctx, stream, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, cost, path_len, path, path_cap,
                     n_expanded, counters, status);
}

extern "C" int pmp_dstarlite2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                                     const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost,
                                     int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded,
                                     int64_t* counters, int32_t* status)
{
    return lpa_batch(1, ctx, stream, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, cost, path_len, path, path_cap,
                     n_expanded, counters, status);
}

static int replan_batch(int lite, pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H, int heuristic,
                        const int32_t* start_xy, const int32_t* goal_xy, int nq, const int32_t* toggles, int nt,
                        double* cost, int32_t* n_expanded, int32_t* status, int32_t* path_len, uint32_t* path,
                        int path_cap, int64_t* counters)
{
    if (!ctx) return PMP_EINVAL;
    if (nt < 1 || !toggles || !cost || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_replan_batch: need nt >= 1 toggles and the per-plan outputs");
    if (nq > 0 && (!path_len || !path)) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lpastar2d_replan_batch: null path output");
    // the last plan's cost / status / len(EXPAND) also land in the single-plan outputs; scratch for them
    double* c1 = (double*)pmp_scratch(ctx, SCR_AUX1, (size_t)(nq > 0 ? nq : 1) * 16 + 16);
    if (!c1) return PMP_ENOMEM;
    int32_t* n1 = (int32_t*)(c1 + (nq > 0 ? nq : 1));
    int32_t* s1 = n1 + (nq > 0 ? nq : 1);
    return lpa_batch(lite, ctx, stream, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, c1, path_len, path, path_cap,
                     n1, counters, s1, toggles, nt, cost, n_expanded, status);
}

extern "C" int pmp_lpastar2d_replan_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                                          int heuristic, const int32_t* start_xy, const int32_t* goal_xy, int nq,
                                          const int32_t* toggles, int nt, double* cost, int32_t* n_expanded,
                                          int32_t* status, int32_t* path_len, uint32_t* path, int path_cap,
                                          int64_t* counters)
{
    return replan_batch(0, ctx, stream, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, toggles, nt, cost, n_expanded,
                        status, path_len, path, path_cap, counters);
}

extern "C" int pmp_dstarlite2d_replan_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                                            int heuristic, const int32_t* start_xy, const int32_t* goal_xy, int nq,
                                            const int32_t* toggles, int nt, double* cost, int32_t* n_expanded,
                                            int32_t* status, int32_t* path_len, uint32_t* path, int path_cap,
                                            int64_t* counters)
{
    return replan_batch(1, ctx, stream, occ_bits, W, H, heuristic, start_xy, goal_xy, nq, toggles, nt, cost, n_expanded,
                        status, path_len, path, path_cap, counters);
}
