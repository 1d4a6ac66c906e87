// Batched 2D A* for gfx950: one wave64 per query, bit-exact with the reference
// AStar.plan (global_planner/graph_search/a_star.py:39-83) including CPython heapq's tie
// behaviour (Lib/heapq.py heappush/_siftdown, heappop/_siftup) under Node.__lt__
// (utils/environment/node.py:51-54).
//
// Heap entry (16 B, one dwordx4):  f64 f = g + h | u32 cell = x<<13 | y | u32 meta = hkey<<4 | dir
//   hkey orders h exactly: euclidean h = hypot(dx,dy) == sqrt(d2) for |d| <= 16384 (verified
//   against the oracle restatement of CPython's vector_norm), so hkey = d2; manhattan hkey = h.
//   dir = motion index (env.py:52-55) that reached the cell from its parent, 8 = start.
// g of a popped node is G[parent] + motion cost (G written when the parent was closed), so the
// entry does not carry g.  Per-query scratch: heap, closed bits, parent-dir bytes, G (f64).
//
// Wave-parallel heap operations (the heap stays the CPython array, element for element):
//   heappop  -> _siftup walks the smaller-child path to a leaf: lanes prefetch the 5-level
//               subtree (62 entries) below the current position in ONE round, the walk then runs
//               in registers (readlane); _siftdown of the old last element back up that path is a
//               ballot over the path (the path is sorted, the "not less" set is a prefix).
//   heappush -> _siftdown: all ancestors load in one round, one ballot finds the stop level.
#include "pmp_internal.h"

namespace {

constexpr int kMaxDim = 8192;
constexpr int kSubLanes = 62;  // 2 + 4 + 8 + 16 + 32 entries: subtree of depth 5
constexpr double kSqrt2 = 1.4142135623730951;  // math.sqrt(2) == math.hypot(1, 1)

__device__ __constant__ int c_mx[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
__device__ __constant__ int c_my[8] = {0, 1, 1, 1, 0, -1, -1, -1};

struct Ent {
    double f;
    uint32_t cell, meta;
};

__device__ __forceinline__ bool ent_lt(const Ent& a, const Ent& b)
{
    return a.f < b.f || (a.f == b.f && (a.meta >> 4) < (b.meta >> 4));
}

__device__ __forceinline__ Ent ld_ent(const uint4* heap, int idx)
{
    uint4 v = heap[idx];
    Ent e;
    e.f = __hiloint2double((int)v.y, (int)v.x);
    e.cell = v.z;
    e.meta = v.w;
    return e;
}

__device__ __forceinline__ void st_ent(uint4* heap, int idx, const Ent& e)
{
    uint64_t b = (uint64_t)__double_as_longlong(e.f);
    heap[idx] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), e.cell, e.meta);
}

__device__ __forceinline__ Ent rl_ent(const Ent& e, int lane)
{
    Ent r;
    r.f = rl_f64(e.f, lane);
    r.cell = rl_u32(e.cell, lane);
    r.meta = rl_u32(e.meta, lane);
    return r;
}

__device__ __forceinline__ bool bit_at(const uint32_t* bits, uint32_t i) { return (bits[i >> 5] >> (i & 31)) & 1u; }

__device__ __forceinline__ bool occ_at(const uint32_t* occ, int W, int H, int x, int y)
{
    if ((unsigned)x >= (unsigned)W || (unsigned)y >= (unsigned)H) return true;
    return bit_at(occ, (uint32_t)x * (uint32_t)H + (uint32_t)y);
}

__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// lane l < 62 of a subtree prefetch below position `pos`: level j in 1..5, offset o
__device__ __forceinline__ int sub_index(int pos, int l)
{
    int j = 31 - __clz(l + 2);
    int o = l + 2 - (1 << j);
    return ((pos + 1) << j) - 1 + o;
}

__global__ __launch_bounds__(64) void astar2d_kernel(
    const uint32_t* __restrict__ occ, int W, int H, int heuristic, const int32_t* __restrict__ start_xy,
    const int32_t* __restrict__ goal_xy, int nq, int q0, double* __restrict__ cost_out,
    int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out, int path_cap,
    int32_t* __restrict__ nexp_out, uint32_t* __restrict__ expand_out, int expand_cap,
    int64_t* __restrict__ counters, int32_t* __restrict__ status_out, uint4* __restrict__ heap_all, int heap_cap,
    uint32_t* __restrict__ closed_all, size_t closed_words, uint8_t* __restrict__ pdir_all,
    double* __restrict__ G_all, size_t ncell)
{
    const int slot = blockIdx.x;
    const int q = q0 + slot;
    if (q >= nq) return;
    const int lane = lane_id();
    uint4* heap = heap_all + (size_t)slot * heap_cap;
    uint32_t* closed = closed_all + (size_t)slot * closed_words;
    uint8_t* pdir = pdir_all + (size_t)slot * ncell;
    double* G = G_all + (size_t)slot * ncell;

    const int sx = start_xy[2 * q], sy = start_xy[2 * q + 1];
    const int gx = goal_xy[2 * q], gy = goal_xy[2 * q + 1];
    const bool sin_ = (unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H;
    const bool gin_ = (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
    if (!sin_ || !gin_) {  // outside the grid: blocked -> no neighbours -> no path
        if (lane == 0) {
            status_out[q] = PMP_NO_PATH;
            cost_out[q] = 0.0;
            path_len_out[q] = 0;
            nexp_out[q] = sin_ ? 1 : 0;
            if (counters) { counters[4 * q] = 1; counters[4 * q + 1] = 1; counters[4 * q + 2] = 0; counters[4 * q + 3] = 1; }
        }
        return;
    }
    const uint32_t start_cell = ((uint32_t)sx << 13) | (uint32_t)sy;
    const uint32_t goal_cell = ((uint32_t)gx << 13) | (uint32_t)gy;

    // root of the heap lives in registers (wave-uniform); heap[0] in memory mirrors it
    Ent root;
    root.f = 0.0;           // Node(start, start, 0, 0): g = h = 0 (planner.py:15)
    root.cell = start_cell;
    root.meta = 8u;         // hkey 0, dir 8 = start
    if (lane == 0) st_ent(heap, 0, root);
    wave_fence();

    int n = 1;
    int64_t npush = 1, npop = 0;
    int nexp = 0, maxn = 1;
    int st = PMP_NO_PATH;
    double goal_cost = 0.0;
    int plen = 0;

    while (n > 0) {
        // ------------------------------------------------------------ heappop: take root
        const Ent node = root;
        npop++;
        n -= 1;
        const int x = (int)(node.cell >> 13), y = (int)(node.cell & 8191u);
        const int ndir = (int)(node.meta & 15u);
        const uint32_t nlin = (uint32_t)x * (uint32_t)H + (uint32_t)y;

        // ---- round A: subtree below root, the last element, neighbour occupancy/closed, G[parent]
        Ent v;
        v.f = 0.0; v.cell = 0; v.meta = 0;
        if (lane < kSubLanes) {
            int idx = sub_index(0, lane);
            if (idx < n) v = ld_ent(heap, idx);
        }
        Ent lastv = v;
        if (lane == 62 && n > 0) lastv = ld_ent(heap, n);
        bool nb_ok = false;
        uint32_t nbcell = 0;
        bool self_closed = false;
        if (lane < 8) {
            const int nx = x + c_mx[lane], ny = y + c_my[lane];
            bool coll = occ_at(occ, W, H, x, y) || occ_at(occ, W, H, nx, ny);
            if ((lane & 1) && !coll) coll = occ_at(occ, W, H, x, ny) || occ_at(occ, W, H, nx, y);
            if (!coll) nb_ok = !bit_at(closed, (uint32_t)nx * (uint32_t)H + (uint32_t)ny);
            nbcell = ((uint32_t)nx << 13) | (uint32_t)ny;
        } else if (lane == 8) {
            self_closed = bit_at(closed, nlin);
        }
        double gpar = 0.0;
        if (lane == 63 && ndir < 8) {
            const int px = x - c_mx[ndir], py = y - c_my[ndir];
            gpar = G[(uint32_t)px * (uint32_t)H + (uint32_t)py];
        }
        const bool is_stale = __shfl(self_closed ? 1 : 0, 8) != 0;

        // ---- finish the pop (_siftup to a leaf, _siftdown of `last` back up the path)
        if (n > 0) {
            const Ent last = rl_ent(lastv, 62);
            Ent pv;
            pv.f = 0.0; pv.cell = 0; pv.meta = 0;
            int ppos = 0;
            int k = 0;
            int cur = 0;
            for (;;) {
                int ocur = 0;
                for (int j = 1; j <= 5; j++) {
                    const int c = 2 * cur + 1;
                    if (c >= n) break;
                    const int ll = (1 << j) - 2 + 2 * ocur;
                    Ent left = rl_ent(v, ll);
                    Ent chosen = left;
                    int ch = c, och = 2 * ocur;
                    if (c + 1 < n) {
                        Ent right = rl_ent(v, ll + 1);
                        if (!ent_lt(left, right)) { chosen = right; ch = c + 1; och += 1; }
                    }
                    if (lane == k) { pv = chosen; ppos = ch; }
                    k++;
                    cur = ch;
                    ocur = och;
                }
                if (2 * cur + 1 >= n) break;
                // next round: subtree below cur
                if (lane < kSubLanes) {
                    int idx = sub_index(cur, lane);
                    if (idx < n) v = ld_ent(heap, idx);
                }
            }
            const bool notless = lane < k && !ent_lt(last, pv);
            const int m = __popcll(ballot(notless));
            // e_1..e_m move up one level, `last` lands at p_m
            if (lane < m) st_ent(heap, (ppos - 1) >> 1, pv);
            const int pm = (m == 0) ? 0 : (int)rl_u32((uint32_t)ppos, m - 1);
            if (lane == 0) st_ent(heap, pm, last);
            root = (m >= 1) ? rl_ent(pv, 0) : last;
            wave_fence();
        }
        if (is_stale) continue;  // node.current already in CLOSED (a_star.py:57-58)

        const double gnode = (ndir == 8) ? 0.0 : rl_f64(gpar, 63) + ((ndir & 1) ? kSqrt2 : 1.0);

        if (node.cell == goal_cell) {  // goal found (a_star.py:61-64)
            if (lane == 0) {
                atomicOr(&closed[nlin >> 5], 1u << (nlin & 31));
                pdir[nlin] = (uint8_t)ndir;
                G[nlin] = gnode;
                if (expand_out && nexp < expand_cap) expand_out[(size_t)q * expand_cap + nexp] = nlin | ((uint32_t)ndir << 28);
            }
            nexp++;
            st = PMP_FOUND;
            wave_fence();
            if (lane == 0) {  // extractPath (a_star.py:98-117): goal -> start, cost in that order
                uint32_t cx = (uint32_t)x, cy = (uint32_t)y;
                double cost = 0.0;
                int len = 0;
                uint32_t* pth = path_out + (size_t)q * path_cap;
                for (;;) {
                    if (len < path_cap) pth[len] = cx * (uint32_t)H + cy;
                    len++;
                    if (((cx << 13) | cy) == start_cell) break;
                    const int d = pdir[cx * (uint32_t)H + cy];
                    cost += (d & 1) ? kSqrt2 : 1.0;
                    cx = (uint32_t)((int)cx - c_mx[d]);
                    cy = (uint32_t)((int)cy - c_my[d]);
                }
                goal_cost = cost;
                plen = len;
            }
            break;
        }

        // ---- neighbours in motion order; push the goal and stop (a_star.py:66-80)
        uint64_t vm = ballot(nb_ok) & 0xffull;
        const uint64_t gm = ballot(nb_ok && nbcell == goal_cell) & 0xffull;
        if (gm) vm &= (gm << 1) - 1;  // keep motions up to and including the goal motion
        Ent item;
        {
            const int m = lane & 7;
            const int nx = x + c_mx[m], ny = y + c_my[m];
            const double gn = gnode + ((m & 1) ? kSqrt2 : 1.0);
            const int dx = gx - nx, dy = gy - ny;
            uint32_t hk;
            double h;
            if (heuristic == 1) {
                hk = (uint32_t)(abs(dx) + abs(dy));
                h = (double)hk;
            } else {
                hk = (uint32_t)(dx * dx + dy * dy);
                h = __dsqrt_rn((double)hk);
            }
            item.f = gn + h;
            item.cell = ((uint32_t)nx << 13) | (uint32_t)ny;
            item.meta = (hk << 4) | (uint32_t)m;
        }
        bool overflow = false;
        while (vm) {
            const int m = __ffsll((long long)vm) - 1;
            vm &= vm - 1;
            const Ent it = rl_ent(item, m);
            if (n >= heap_cap) { overflow = true; break; }
            // heappush -> _siftdown: ancestors of position n, one round
            const int np1 = n + 1;
            const int depth = 31 - __clz(np1);
            Ent a;
            a.f = 0.0; a.cell = 0; a.meta = 0;
            const bool valid = lane < depth;
            if (valid) a = ld_ent(heap, (np1 >> (lane + 1)) - 1);
            const bool less = valid && ent_lt(it, a);
            const int t = __popcll(ballot(less));
            if (lane < t) st_ent(heap, (np1 >> lane) - 1, a);
            const int ipos = (np1 >> t) - 1;
            if (lane == 0) st_ent(heap, ipos, it);
            if (ipos == 0) root = it;
            n += 1;
            npush++;
            wave_fence();
        }
        if (n > maxn) maxn = n;
        if (overflow) { st = PMP_CAP_OVERFLOW; break; }

        // ---- CLOSED[node.current] = node (a_star.py:82)
        if (lane == 0) {
            atomicOr(&closed[nlin >> 5], 1u << (nlin & 31));
            pdir[nlin] = (uint8_t)ndir;
            G[nlin] = gnode;
            if (expand_out && nexp < expand_cap) expand_out[(size_t)q * expand_cap + nexp] = nlin | ((uint32_t)ndir << 28);
        }
        nexp++;
        wave_fence();
    }

    if (lane == 0) {
        int s = st;
        if (s == PMP_FOUND && plen > path_cap) s = PMP_PATH_OVERFLOW;
        status_out[q] = s;
        cost_out[q] = (st == PMP_FOUND) ? goal_cost : 0.0;
        path_len_out[q] = (st == PMP_FOUND) ? plen : 0;
        nexp_out[q] = nexp;
        if (counters) {
            counters[4 * q + 0] = npush;
            counters[4 * q + 1] = npop;
            counters[4 * q + 2] = nexp;
            counters[4 * q + 3] = maxn;
        }
    }
}

}  // namespace

struct AStarCfg {
    int W = 0, H = 0, slots = 0, heap_cap = 0;
};
static AStarCfg g_astar_reserved;  // per-process default; set by pmp_astar2d_reserve

static size_t astar_slot_bytes(int W, int H, int heap_cap)
{
    size_t ncell = (size_t)W * H;
    return (size_t)heap_cap * 16 + ((ncell + 31) / 32) * 4 + ncell + ncell * 8;
}

static int astar_default_heap_cap(int W, int H)
{
    size_t ncell = (size_t)W * H;
    size_t cap = 8 * ncell + 8;
    if (cap > (size_t)(1 << 18)) cap = (size_t)1 << 18;
    return (int)cap;
}

extern "C" int pmp_astar2d_reserve(pmp_ctx* ctx, int W, int H, int max_slots, int heap_cap)
{
    if (!ctx) return PMP_EINVAL;
    if (W < 1 || H < 1 || W > kMaxDim || H > kMaxDim || max_slots < 1)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_reserve: bad dims/slots");
    if (heap_cap <= 0) heap_cap = astar_default_heap_cap(W, H);
    size_t ncell = (size_t)W * H;
    if (!pmp_scratch(ctx, SCR_HEAP, (size_t)max_slots * heap_cap * 16)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_CLOSED, (size_t)max_slots * ((ncell + 31) / 32) * 4)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_PDIR, (size_t)max_slots * ncell)) return PMP_ENOMEM;
    if (!pmp_scratch(ctx, SCR_G, (size_t)max_slots * ncell * 8)) return PMP_ENOMEM;
    g_astar_reserved.W = W;
    g_astar_reserved.H = H;
    g_astar_reserved.slots = max_slots;
    g_astar_reserved.heap_cap = heap_cap;
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
    if (!occ_bits || !start_xy || !goal_xy || !cost || !path_len || !path || !n_expanded || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_astar2d_batch: null pointer argument");
    if (nq == 0) return PMP_OK;
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;

    int heap_cap, slots;
    if (g_astar_reserved.W == W && g_astar_reserved.H == H) {
        heap_cap = g_astar_reserved.heap_cap;
        slots = g_astar_reserved.slots;
    } else {
        heap_cap = astar_default_heap_cap(W, H);
        const size_t budget = (size_t)64 << 30;  // 64 GiB of scratch by default
        size_t per = astar_slot_bytes(W, H, heap_cap);
        slots = (int)((budget / per) < (size_t)nq ? (budget / per) : (size_t)nq);
        if (slots < 1) slots = 1;
    }
    if (slots > nq) slots = nq;
    const size_t ncell = (size_t)W * H;
    const size_t closed_words = (ncell + 31) / 32;
    uint4* heap = (uint4*)pmp_scratch(ctx, SCR_HEAP, (size_t)slots * heap_cap * 16);
    uint32_t* closed = (uint32_t*)pmp_scratch(ctx, SCR_CLOSED, (size_t)slots * closed_words * 4);
    uint8_t* pdir = (uint8_t*)pmp_scratch(ctx, SCR_PDIR, (size_t)slots * ncell);
    double* G = (double*)pmp_scratch(ctx, SCR_G, (size_t)slots * ncell * 8);
    if (!heap || !closed || !pdir || !G) return PMP_ENOMEM;

    for (int q0 = 0; q0 < nq; q0 += slots) {
        const int nb = (nq - q0) < slots ? (nq - q0) : slots;
        PMP_HIP_CHECK(ctx, hipMemsetAsync(closed, 0, (size_t)nb * closed_words * 4, s));
        hipLaunchKernelGGL(astar2d_kernel, dim3(nb), dim3(64), 0, s, occ_bits, W, H, heuristic, start_xy, goal_xy,
                           nq, q0, cost, path_len, path, path_cap, n_expanded, expand, expand_cap, counters,
                           status, heap, heap_cap, closed, closed_words, pdir, G, ncell);
        PMP_HIP_CHECK(ctx, hipGetLastError());
    }
    return PMP_OK;
}
