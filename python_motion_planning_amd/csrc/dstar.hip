// Batched D* (static plan) for gfx950, exact with DStar.plan (global_planner/graph_search/d_star.py:75-291)
// over Grid with GraphSearcher.isCollision (graph_search.py:61-87).
//
// The reference's OPEN is a Python list: insert appends (duplicates allowed, :236-248), min_state is
// the FIRST entry of minimal k in list order (:220-227), delete removes the first occurrence
// (:250-259).  All entries of one node share that node's k, so the popped entry is the earliest
// remaining entry of the node minimising (k, first entry position) -- a strict total order.  The
// kernel keeps:
//   per cell (32 B): h, k, first/last remaining entry, parent cell, entry count | tag << 24;
//   per entry: the next entry of the same node (a FIFO per node, positions = append counter);
//   a lazy min-heap (heap16.h) of (k, first position, cell), validated on pop against the cell.
// processState (:158-218) runs on one wave: lanes 0..7 are the 8 motions (env.py:52-55) in order,
// the RAISE scan is a scalar loop, the LOWER/else decisions are per lane, and appended entries
// take their positions by lane-order prefix counts, exactly the reference's append order.
#include "heap16.h"

namespace {

__device__ __constant__ int c_dmx[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
__device__ __constant__ int c_dmy[8] = {0, 1, 1, 1, 0, -1, -1, -1};

constexpr uint32_t T_NEW = 0, T_OPEN = 1, T_CLOSED = 2;

struct __attribute__((aligned(16))) DCell {
    double h, k;
    int32_t first, last, parent;
    uint32_t cnt_t;  // entry count (24 bits) | tag << 24
};

using heap16::Ent;  // g = k, a = first entry position, b = cell

struct KeyD {
    __device__ __forceinline__ void derive(Ent& e) const { e.f = e.g; e.hk = 0u; }
    static __device__ __forceinline__ bool lt(const Ent& x, const Ent& y)
    {
        return (x.g < y.g) | ((x.g == y.g) & (x.a < y.a));
    }
};

__device__ __forceinline__ bool occ2(const uint32_t* occ, int W, int H, int x, int y)
{
    if ((unsigned)x >= (unsigned)W || (unsigned)y >= (unsigned)H) return true;
    const uint32_t c = (uint32_t)x * (uint32_t)H + (uint32_t)y;
    return (occ[c >> 5] >> (c & 31)) & 1u;
}

__device__ __forceinline__ DCell load_cell(const DCell* cells, int c)
{
    const uint4* p = reinterpret_cast<const uint4*>(cells + c);
    const uint4 a = p[0], b = p[1];
    DCell r;
    r.h = __hiloint2double((int)a.y, (int)a.x);
    r.k = __hiloint2double((int)a.w, (int)a.z);
    r.first = (int32_t)b.x;
    r.last = (int32_t)b.y;
    r.parent = (int32_t)b.z;
    r.cnt_t = b.w;
    return r;
}

__device__ __forceinline__ void store_cell(DCell* cells, int c, const DCell& v)
{
    uint4* p = reinterpret_cast<uint4*>(cells + c);
    const uint64_t hb = (uint64_t)__double_as_longlong(v.h), kb = (uint64_t)__double_as_longlong(v.k);
    p[0] = make_uint4((uint32_t)hb, (uint32_t)(hb >> 32), (uint32_t)kb, (uint32_t)(kb >> 32));
    p[1] = make_uint4((uint32_t)v.first, (uint32_t)v.last, (uint32_t)v.parent, v.cnt_t);
}

__device__ __forceinline__ uint32_t cnt_of(uint32_t ct) { return ct & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t tag_of(uint32_t ct) { return ct >> 24; }

__device__ __forceinline__ DCell rl_cell(const DCell& v, int lane)
{
    DCell r;
    r.h = rl_f64(v.h, lane);
    r.k = rl_f64(v.k, lane);
    r.first = (int32_t)rl_u32((uint32_t)v.first, lane);
    r.last = (int32_t)rl_u32((uint32_t)v.last, lane);
    r.parent = (int32_t)rl_u32((uint32_t)v.parent, lane);
    r.cnt_t = rl_u32(v.cnt_t, lane);
    return r;
}

__global__ __launch_bounds__(64) void dstar_kernel(const uint32_t* __restrict__ occ, int W, int H,
                                                   const int32_t* __restrict__ start_xy, const int32_t* __restrict__ goal_xy,
                                                   int nq, double* __restrict__ cost_out, int32_t* __restrict__ path_len_out,
                                                   int32_t* __restrict__ path_out, int path_cap,
                                                   int64_t* __restrict__ nproc_out, int32_t* __restrict__ status_out,
                                                   int64_t max_process, int* __restrict__ queue, uint4* __restrict__ spill_all,
                                                   int heap_cap, int lds_cap, DCell* __restrict__ cells_all,
                                                   int32_t* __restrict__ next_all, int entry_cap)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    const int ncell = W * H;
    const size_t spill_n = (size_t)(heap_cap > lds_cap ? heap_cap - lds_cap : 0);
    const heap16::Heap hp = heap16::make_heap(smem, lds_cap, spill_all + (size_t)worker * spill_n, spill_n);
    DCell* cells = cells_all + (size_t)worker * ncell;
    int32_t* nxt = next_all + (size_t)worker * entry_cap;
    int pop_jl, pop_ol;
    heap16::pop_lane_consts(lane, pop_jl, pop_ol);
    const KeyD key;
    const int mdx = c_dmx[lane & 7], mdy = c_dmy[lane & 7];
    const double mcost = (lane & 1) ? 1.4142135623730951 : 1.0;  // Planner.dist = hypot(1, 1) / hypot(1, 0)

    for (;;) {
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = qi;
        const int sx = start_xy[2 * q], sy = start_xy[2 * q + 1];
        const int gx = goal_xy[2 * q], gy = goal_xy[2 * q + 1];
        if ((unsigned)sx >= (unsigned)W || (unsigned)sy >= (unsigned)H || (unsigned)gx >= (unsigned)W ||
            (unsigned)gy >= (unsigned)H) {
            // every lane stores the same values (no lane-0 block before the continue)
            status_out[q] = PMP_REF_RAISES; cost_out[q] = 0.0; path_len_out[q] = 0; nproc_out[q] = 0;
            continue;
        }
        const int start = sx * H + sy, goal = gx * H + gy;
        // DStar.__init__ (:55-70): every cell NEW with h = k = inf, goal h = 0, insert(goal, 0)
        {
            DCell v;
            v.h = __builtin_inf();
            v.k = __builtin_inf();
            v.first = v.last = v.parent = -1;
            v.cnt_t = T_NEW << 24;
            for (int c = lane; c < ncell; c += 64) store_cell(cells, c, v);
            heap16::wsync();
            if (lane == 0) {
                v.h = 0.0;
                v.k = 0.0;
                v.first = v.last = 0;
                v.cnt_t = (T_OPEN << 24) | 1u;
                store_cell(cells, goal, v);
                nxt[0] = -1;
            }
        }
        Ent root;
        root.g = 0.0;
        root.a = 0u;
        root.b = (uint32_t)goal;
        key.derive(root);
        if (lane == 0) heap16::store<true>(hp, 0, root);
        heap16::wsync();
        int n = 1;               // heap elements (valid + stale)
        int64_t open_total = 1;  // len(OPEN)
        int ne = 1;              // entries appended so far (list positions)
        int64_t np = 0;
        int st = PMP_FOUND;
        bool start_closed = false;

        for (;;) {
            // ---- min_state: pop until an element matches its cell's (k, first) ----
            Ent top;
            DCell xc;
            for (;;) {
                top = root;
                n -= 1;
                if (n > 0) {
                    if (n < lds_cap) heap16::pop<KeyD, false>(hp, key, n, root, lane, pop_jl, pop_ol);
                    else heap16::pop<KeyD, true>(hp, key, n, root, lane, pop_jl, pop_ol);
                }
                xc = load_cell(cells, (int)top.b);
                if (cnt_of(xc.cnt_t) > 0 && (uint32_t)xc.first == top.a && xc.k == top.g) break;
                if (n == 0) { st = PMP_CAP_OVERFLOW; break; }  // cannot happen while open_total > 0
            }
            if (st != PMP_FOUND) break;
            np++;
            const int X = (int)top.b;
            const double k_old = xc.k;
            // delete (:250-259): CLOSED if OPEN, drop the first entry
            {
                uint32_t tg = tag_of(xc.cnt_t);
                if (tg == T_OPEN) tg = T_CLOSED;
                const int e = xc.first;
                xc.first = nxt[e];
                xc.cnt_t = (tg << 24) | (cnt_of(xc.cnt_t) - 1u);
                if (cnt_of(xc.cnt_t) == 0) xc.last = -1;
                open_total -= 1;
            }
            // ---- neighbours (getNeighbor, :276-291): lanes 0..7 in motion order ----
            const int x = X / H, y = X % H;
            const int nx = x + mdx, ny = y + mdy;
            bool nb = false;
            DCell yc;
            yc.h = yc.k = 0.0;
            yc.first = yc.last = yc.parent = -1;
            yc.cnt_t = 0;
            int Y = 0;
            if (lane < 8) {
                bool coll = occ2(occ, W, H, x, y) || occ2(occ, W, H, nx, ny);
                if (mdx != 0 && mdy != 0) coll = coll || occ2(occ, W, H, x, ny) || occ2(occ, W, H, nx, y);
                nb = !coll;
                if (nb) {
                    Y = nx * H + ny;
                    yc = load_cell(cells, Y);
                }
            }
            const uint64_t nbm = ballot(nb) & 0xFFull;
            // RAISE (:177-183): scalar scan in motion order
            double hX = xc.h;
            int pX = xc.parent;
            if (k_old < hX) {
                for (uint64_t m = nbm; m; m &= m - 1) {
                    const int l = __ffsll((long long)m) - 1;
                    const double hy = rl_f64(yc.h, l);
                    const double c = (l & 1) ? 1.4142135623730951 : 1.0;
                    if (hy <= k_old && hX > hy + c) {
                        pX = (int)rl_u32((uint32_t)Y, l);
                        hX = hy + c;
                    }
                }
            }
            // LOWER / else (:185-217): one decision per lane; kind 1 = insert(node_n, h_new), 2 = insert(node, h)
            int kind = 0;
            double hnew = 0.0;
            bool setpar = false;
            if (nb) {
                const uint32_t ty = tag_of(yc.cnt_t);
                const bool par_is_x = yc.parent == X;
                const double hc = hX + mcost;
                if (k_old == hX) {
                    if (ty == T_NEW || (par_is_x && yc.h != hc) || (!par_is_x && yc.h > hc)) {
                        kind = 1; hnew = hc; setpar = true;
                    }
                } else {
                    if (ty == T_NEW || (par_is_x && yc.h != hc)) {
                        kind = 1; hnew = hc; setpar = true;
                    } else if (!par_is_x && yc.h > hc) {
                        kind = 2;
                    } else if (!par_is_x && hX > yc.h + mcost && ty == T_CLOSED && yc.h > k_old) {
                        kind = 1; hnew = yc.h;
                    }
                }
            }
            const uint64_t insm = ballot(kind != 0);
            const int nins = __popcll(insm);
            if (ne + nins > entry_cap) { st = PMP_CAP_OVERFLOW; break; }
            const int myE = ne + __popcll(insm & ((1ull << lane) - 1ull));
            // insert(node_n, h_new) (:236-248) for lanes of kind 1 (distinct cells, independent)
            if (kind == 1) {
                const uint32_t ty = tag_of(yc.cnt_t);
                if (ty == T_NEW) yc.k = hnew;
                else if (ty == T_OPEN) yc.k = fmin(yc.k, hnew);
                else yc.k = fmin(yc.h, hnew);
                yc.h = hnew;
                if (setpar) yc.parent = X;
                const uint32_t cnt = cnt_of(yc.cnt_t);
                if (cnt == 0) yc.first = myE;
                else nxt[yc.last] = myE;
                nxt[myE] = -1;
                yc.last = myE;
                yc.cnt_t = (T_OPEN << 24) | (cnt + 1u);
                store_cell(cells, Y, yc);
            }
            // insert(node, node.h) for lanes of kind 2, in lane order (node is CLOSED here, so
            // k = min(h, h) = h the first time and min(k, h) = h after)
            const uint64_t xm = ballot(kind == 2);
            if (xm) {
                if (lane == 0) {
                    uint32_t cnt = cnt_of(xc.cnt_t);
                    for (uint64_t m = xm; m; m &= m - 1) {
                        const int l = __ffsll((long long)m) - 1;
                        const int e = ne + __popcll(insm & ((1ull << l) - 1ull));
                        if (cnt == 0) xc.first = e;
                        else nxt[xc.last] = e;
                        nxt[e] = -1;
                        xc.last = e;
                        cnt++;
                    }
                    xc.cnt_t = (T_OPEN << 24) | cnt;
                }
                xc.first = (int32_t)rl_u32((uint32_t)xc.first, 0);
                xc.last = (int32_t)rl_u32((uint32_t)xc.last, 0);
                xc.cnt_t = rl_u32(xc.cnt_t, 0);
                xc.k = hX;
            }
            xc.h = hX;
            xc.parent = pX;
            if (lane == 0) store_cell(cells, X, xc);
            ne += nins;
            open_total += nins;
            heap16::wsync();
            // heap pushes: every re-keyed cell (stale elements are skipped on pop)
            uint64_t pm = ballot(kind == 1);
            bool overflow = false;
            while (pm) {
                const int l = __ffsll((long long)pm) - 1;
                pm &= pm - 1;
                if (n >= heap_cap) { overflow = true; break; }
                Ent it;
                it.g = rl_f64(yc.k, l);
                it.a = rl_u32((uint32_t)yc.first, l);
                it.b = rl_u32((uint32_t)Y, l);
                key.derive(it);
                if (n == 0) {
                    if (lane == 0) heap16::store<true>(hp, 0, it);
                    root = it;
                    heap16::wsync();
                } else if (n < lds_cap) {
                    heap16::push<KeyD, false>(hp, key, n, it, root, lane);
                } else {
                    heap16::push<KeyD, true>(hp, key, n, it, root, lane);
                }
                n += 1;
            }
            if (!overflow && cnt_of(xc.cnt_t) > 0) {
                if (n >= heap_cap) {
                    overflow = true;
                } else {
                    Ent it;
                    it.g = xc.k;
                    it.a = (uint32_t)xc.first;
                    it.b = (uint32_t)X;
                    key.derive(it);
                    if (n == 0) {
                        if (lane == 0) heap16::store<true>(hp, 0, it);
                        root = it;
                        heap16::wsync();
                    } else if (n < lds_cap) {
                        heap16::push<KeyD, false>(hp, key, n, it, root, lane);
                    } else {
                        heap16::push<KeyD, true>(hp, key, n, it, root, lane);
                    }
                    n += 1;
                }
            }
            if (overflow) { st = PMP_CAP_OVERFLOW; break; }
            // start.t after this processState
            if (X == start) start_closed = tag_of(xc.cnt_t) == T_CLOSED;
            if (ballot(kind == 1 && Y == start)) start_closed = false;
            if (open_total == 0) { st = PMP_REF_RAISES; break; }  // return self.min_k on an empty OPEN
            if (start_closed) break;
            if (max_process > 0 && np >= max_process) { st = PMP_CAP_OVERFLOW; break; }
        }
        heap16::wsync();
        if (lane == 0) {
            int plen = 0;
            double cost = 0.0;
            if (st == PMP_FOUND) {
                // extractPath (:136-156): start -> goal through parents, cost via GraphSearcher.cost
                int32_t* pth = path_out + (size_t)q * path_cap;
                int c = start;
                pth[0] = c;
                plen = 1;
                while (c != goal) {
                    const int p = load_cell(cells, c).parent;
                    if (p < 0 || plen > ncell) { st = PMP_REF_RAISES; break; }
                    const int cx = c / H, cy = c % H, px = p / H, py = p % H;
                    bool coll = occ2(occ, W, H, cx, cy) || occ2(occ, W, H, px, py);
                    if (cx != px && cy != py) coll = coll || occ2(occ, W, H, cx, py) || occ2(occ, W, H, px, cy);
                    cost += coll ? __builtin_inf() : ((cx != px && cy != py) ? 1.4142135623730951 : 1.0);
                    c = p;
                    if (plen < path_cap) pth[plen] = c;
                    plen++;
                }
                if (st == PMP_FOUND && plen > path_cap) st = PMP_PATH_OVERFLOW;
            }
            status_out[q] = st;
            cost_out[q] = cost;
            path_len_out[q] = plen;
            nproc_out[q] = np;
        }
        heap16::wsync();
    }
}

}  // namespace

extern "C" int pmp_dstar2d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int W, int H,
                                 const int32_t* start_xy, const int32_t* goal_xy, int nq, double* cost,
                                 int32_t* path_len, int32_t* path, int path_cap, int64_t* n_process, int32_t* status,
                                 int64_t max_process)
{
    if (!ctx) return PMP_EINVAL;
    if (W < 1 || H < 1 || (int64_t)W * H > (1 << 26))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar2d_batch: W*H must be in [1, 2^26]");
    if (nq < 0 || path_cap < 1) return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar2d_batch: bad nq/path_cap");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xy || !goal_xy || !cost || !path_len || !path || !n_process || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar2d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t ncell = (size_t)W * H;
    // per worker: 32 B cell state + 4 entries (16 B) + 4 heap elements (64 B) per cell, over the LDS part
    const size_t hc = 4 * ncell + 64;
    const int heap_cap = (int)(hc > (size_t)(1 << 26) ? (size_t)(1 << 26) : hc);
    const int entry_cap = heap_cap;
    const int per_cu = 4;
    int lds_cap = (((160 * 1024) / per_cu - 256) / 16) & ~15;
    if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    const size_t spill_n = heap_cap > lds_cap ? (size_t)(heap_cap - lds_cap) : 0;
    const size_t per_worker = ncell * sizeof(DCell) + (size_t)entry_cap * 4 + spill_n * 16 + 4096;
    int workers = 256 * per_cu;
    const size_t max_workers = ((size_t)16 << 30) / per_worker;  // keep the scratch under 16 GiB
    if ((size_t)workers > max_workers) workers = (int)(max_workers > 0 ? max_workers : 1);
    if (workers > nq) workers = nq;
    uint4* spill = (uint4*)pmp_scratch(ctx, SCR_AUX1, (size_t)workers * spill_n * 16 + 16);
    DCell* cells = (DCell*)pmp_scratch(ctx, SCR_AUX2, (size_t)workers * ncell * sizeof(DCell) + 16);
    int32_t* nxt = (int32_t*)pmp_scratch(ctx, SCR_AUX3, (size_t)workers * entry_cap * 4 + 16);
    int* queue = (int*)pmp_scratch(ctx, SCR_AUX0, 256);
    if (!spill || !cells || !nxt || !queue) return PMP_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    hipLaunchKernelGGL(dstar_kernel, dim3(workers), dim3(64), (size_t)lds_cap * 16, s, occ_bits, W, H, start_xy, goal_xy,
                       nq, cost, path_len, path, path_cap, n_process, status, max_process, queue, spill, heap_cap, lds_cap,
                       cells, nxt, entry_cap);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
