// Batched D* in 3D for gfx950, exact with DStar3D (global_planner/graph_search/d_star3d.py:60-281):
// plan() (:100-109) and any number of apply_dynamic_obstacles() rounds (:115-149) per query, over
// Grid3D with GraphSearcher3D.isCollision (graph_search_3d.py:66-107).
//
// The reference's OPEN is a Python list of DNode3D: insert appends a node only if it is not already
// in OPEN (`node not in self.OPEN`, :245-246 -- Node3D equality is by coordinates, node3d.py:43-46),
// min_state is the FIRST entry of minimal k in list order (:220-225), delete removes the node
// (:248-253).  So every OPEN node has exactly one list position -- the append counter when it was
// (re)appended -- and the popped node minimises (k, position), a strict total order.  The kernel
// keeps per voxel {h, k, parent, position, tag} and a lazy min-heap (heap16.h) of (k, position,
// voxel), validated on pop against the voxel.
//
// processState (:168-218) runs on one wave: lanes 0..25 are the 26 motions (env3d.py:56-70) in
// order.  getNeighbor (:266-280) skips voxels outside the map and pairs with isCollision(node, n),
// which is NOT symmetric for three-axis diagonals (it checks the three face neighbours of its first
// argument), so extractPath's cost(node, parent) can be inf where the search saw no collision --
// the published CSV's inf rows.  The RAISE scan (a running strict minimum) is a first-minimum
// over the candidate lanes; the LOWER / else decisions are per lane and independent (each reads
// only its own neighbour and the node's h); appended entries take positions by lane-order prefix
// counts, exactly the reference's append order, and the node itself is appended at most once.
//
// start == goal: the constructor's map[start] = self.start detaches the goal object from the map
// (:89-90), so the goal node lives in an extra slot (ncell) that no neighbour scan reaches.
#include <algorithm>
#include "heap16.h"

namespace {

constexpr int kMaxDim = 256;

__device__ __constant__ int8_t c_m[26][3] = {
    {-1, 0, 0}, {-1, 1, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0}, {1, -1, 0}, {0, -1, 0}, {-1, -1, 0},
    {0, 0, 1}, {0, 0, -1},
    {-1, 0, 1}, {-1, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, -1, 1}, {-1, -1, 1},
    {-1, 0, -1}, {-1, 1, -1}, {0, 1, -1}, {1, 1, -1}, {1, 0, -1}, {1, -1, -1}, {0, -1, -1}, {-1, -1, -1}};

constexpr uint32_t T_NEW = 0, T_OPEN = 1, T_CLOSED = 2;

struct __attribute__((aligned(16))) DC3 {
    double h, k;
    int32_t parent;  // voxel id of the parent's coordinates, -1 = None
    uint32_t pos;    // OPEN list position (valid while tag == OPEN)
    uint32_t t;
    uint32_t pad;
};

__device__ __forceinline__ DC3 load_c(const DC3* cells, int c)
{
    const uint4* p = reinterpret_cast<const uint4*>(cells + c);
    const uint4 a = p[0], b = p[1];
    DC3 r;
    r.h = __hiloint2double((int)a.y, (int)a.x);
    r.k = __hiloint2double((int)a.w, (int)a.z);
    r.parent = (int32_t)b.x;
    r.pos = b.y;
    r.t = b.z;
    r.pad = 0u;
    return r;
}

__device__ __forceinline__ void store_c(DC3* cells, int c, const DC3& v)
{
    uint4* p = reinterpret_cast<uint4*>(cells + c);
    const uint64_t hb = (uint64_t)__double_as_longlong(v.h), kb = (uint64_t)__double_as_longlong(v.k);
    p[0] = make_uint4((uint32_t)hb, (uint32_t)(hb >> 32), (uint32_t)kb, (uint32_t)(kb >> 32));
    p[1] = make_uint4((uint32_t)v.parent, v.pos, v.t, 0u);
}

using heap16::Ent;  // g = k, a = list position, b = slot

struct KeyD {
    static constexpr bool kStoredF = false;
    __device__ __forceinline__ void derive(Ent& e) const { e.f = e.g; e.hk = 0u; }
    static __device__ __forceinline__ bool lt(const Ent& x, const Ent& y)
    {
        return (x.g < y.g) | ((x.g == y.g) & (x.a < y.a));
    }
};

typedef __attribute__((address_space(3))) uint32_t lds_w32;

// The working occupancy of one query (obstacles change in apply_dynamic_obstacles): LDS when it
// fits, else a per-worker HBM copy.  `p in self.obstacles` is false outside the grid.
template <bool LDS>
struct Occ {
    lds_w32* l;
    uint32_t* g;
    int X, Y, Z;
    __device__ __forceinline__ uint32_t word(uint32_t w) const { return LDS ? l[w] : g[w]; }
    // branch-free (word 0 read outside the grid), so a collision test's reads issue together
    __device__ __forceinline__ uint32_t at(int x, int y, int z) const
    {
        const bool in = (unsigned)x < (unsigned)X && (unsigned)y < (unsigned)Y && (unsigned)z < (unsigned)Z;
        const uint32_t c = in ? ((uint32_t)x * (uint32_t)Y + (uint32_t)y) * (uint32_t)Z + (uint32_t)z : 0u;
        return in ? (word(c >> 5) >> (c & 31)) & 1u : 0u;
    }
    __device__ __forceinline__ void set(uint32_t c) const
    {
        if (LDS) atomicOr((uint32_t*)&l[c >> 5], 1u << (c & 31));
        else atomicOr(&g[c >> 5], 1u << (c & 31));
    }
    // GraphSearcher3D.isCollision(node1 = a, node2 = b) (graph_search_3d.py:66-107)
    // All five reads are issued at once.  For a two-axis diagonal the third face cell is node1
    // itself (its delta is 0), already part of the first test, so OR-ing all three face cells
    // equals the reference's case split.
    __device__ __forceinline__ bool coll(int x1, int y1, int z1, int x2, int y2, int z2) const
    {
        const int dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
        const uint32_t ends = at(x1, y1, z1) | at(x2, y2, z2);
        const uint32_t faces = at(x1 + dx, y1, z1) | at(x1, y1 + dy, z1) | at(x1, y1, z1 + dz);
        const bool adj = max(abs(dx), max(abs(dy), abs(dz))) <= 1;
        const int ch = (dx != 0) + (dy != 0) + (dz != 0);
        return (ends | ((adj && ch >= 2) ? faces : 0u)) != 0u;
    }
};

__device__ __forceinline__ double dist3(int dx, int dy, int dz)  // Planner3D.dist
{
    return __dsqrt_rn((double)(dx * dx + dy * dy + dz * dz));
}

struct Geo {
    int X, Y, Z;
    __device__ __forceinline__ int id(int x, int y, int z) const { return (x * Y + y) * Z + z; }
    __device__ __forceinline__ void xyz(int c, int& x, int& y, int& z) const
    {
        z = c % Z;
        const int r = c / Z;
        y = r % Y;
        x = r / Y;
    }
};

// Per-query search state of one wave (wave-uniform scalars; the heap lives in LDS + HBM spill).
struct Search {
    heap16::Heap hp;
    DC3* cells;
    int heap_cap, lds_cap;
    int n;                // heap elements (valid + stale)
    int64_t open;         // len(OPEN)
    uint32_t ne;          // list positions handed out
    int64_t np;           // processState calls (len(EXPAND))
    Ent root;
    int goal_slot;        // slot of self.goal (ncell when start == goal)
    int goal_cell;        // the goal's coordinates as a voxel id
    int start_slot;
    uint32_t start_t;     // self.start.t, tracked so plan() needs no reload per processState
    bool overflow;
    int32_t* ex;          // plan()'s EXPAND as voxel ids (nullable), ex_cap entries
    int ex_cap;
};

template <bool LDS>
struct D3 {
    const Occ<LDS>& occ;
    Geo geo;
    Search& S;
    int lane, pop_jl, pop_ol;
    int mdx, mdy, mdz;
    double mcost;
    KeyD key;
    heap16::Walk6 pop_w{0ull, 0ull};  // set after construction (walk6_consts)

    __device__ __forceinline__ int coord_of(int slot) const { return slot == S.goal_slot ? S.goal_cell : slot; }

    __device__ __forceinline__ void push(double k, uint32_t pos, int slot)
    {
        if (S.n >= S.heap_cap) { S.overflow = true; return; }
        Ent it;
        it.g = k;
        it.a = pos;
        it.b = (uint32_t)slot;
        key.derive(it);
        if (S.n == 0) {
            if (lane == 0) heap16::store<true>(S.hp, 0, it);
            S.root = it;
            heap16::wsync();
        } else if (S.n < S.lds_cap) {
            heap16::push<KeyD, false>(S.hp, key, S.n, it, S.root, lane);
        } else {
            heap16::push<KeyD, true>(S.hp, key, S.n, it, S.root, lane);
        }
        S.n += 1;
    }

    __device__ __forceinline__ void pop_top()
    {
        S.n -= 1;
        if (S.n > 0) {
            if (S.n < S.lds_cap) heap16::pop<KeyD, false, true>(S.hp, key, S.n, S.root, lane, pop_jl, pop_ol, pop_w);
            else heap16::pop<KeyD, true, true>(S.hp, key, S.n, S.root, lane, pop_jl, pop_ol, pop_w);
        }
    }

    __device__ __forceinline__ bool valid(const Ent& e, const DC3& c) const
    {
        return c.t == T_OPEN && c.pos == e.a && c.k == e.g;
    }

    // drop stale heap tops; afterwards S.root is the min_state (when S.open > 0)
    // `c` = the root's cell when the loop returns early
    __device__ __forceinline__ void clean_top(DC3& c)
    {
        while (S.open > 0 && S.n > 0) {
            c = load_c(S.cells, (int)S.root.b);
            if (valid(S.root, c)) return;
            pop_top();
        }
    }
    __device__ __forceinline__ void clean_top()
    {
        DC3 c;
        clean_top(c);
    }

    // insert(node, h_new) (:233-246) for a node in slot `slot` with state c, wave-uniform
    __device__ __forceinline__ void insert_uniform(int slot, DC3 c, double hnew)
    {
        if (c.t == T_NEW) c.k = hnew;
        else if (c.t == T_OPEN) c.k = fmin(c.k, hnew);
        else c.k = fmin(c.h, hnew);
        c.h = hnew;
        const bool was_open = c.t == T_OPEN;
        c.t = T_OPEN;
        if (slot == S.start_slot) S.start_t = T_OPEN;
        if (!was_open) {
            c.pos = S.ne++;
            S.open += 1;
        }
        if (lane == 0) store_c(S.cells, slot, c);
        heap16::wsync();
        push(c.k, c.pos, slot);
    }

    // processState (:168-218).  Returns false when OPEN is empty (the reference's -1).
    __device__ __forceinline__ bool process_state()
    {
        DC3 xc;  // the popped node's cell: clean_top's load (the heap pop does not touch cells)
        clean_top(xc);
        if (S.open == 0) return false;
        const Ent top = S.root;
        const int Xs = (int)top.b;
        // the neighbours' cells load now, beside the heap pop and the collision reads
        int x, y, z;
        geo.xyz(coord_of(Xs), x, y, z);
        const int nx = x + mdx, ny = y + mdy, nz = z + mdz;
        const bool nin =
            lane < 26 && (unsigned)nx < (unsigned)geo.X && (unsigned)ny < (unsigned)geo.Y && (unsigned)nz < (unsigned)geo.Z;
        const int Yc = nin ? geo.id(nx, ny, nz) : 0;
        DC3 yc = load_c(S.cells, Yc);
        const bool nb = nin && !occ.coll(x, y, z, nx, ny, nz);
        pop_top();
        if (S.ex && lane == 0 && S.np < S.ex_cap) S.ex[S.np] = coord_of(Xs);
        S.np += 1;
        const double k_old = xc.k;
        // delete (:248-253): CLOSED (it is OPEN), off the list
        xc.t = T_CLOSED;
        S.open -= 1;
        const int Xc = coord_of(Xs);
        // getNeighbor: the voxel must be in the map and isCollision(node, n) false (nb above)
        // RAISE (:185-189): running strict minimum in motion order == first minimum of the candidates
        double hX = xc.h;
        int pX = xc.parent;
        if (k_old < hX) {
            for (uint64_t m = ballot(nb && yc.h <= k_old); m; m &= m - 1) {
                const int l = __ffsll((long long)m) - 1;
                const double v = rl_f64(yc.h, l) + rl_f64(mcost, l);
                if (hX > v) {
                    hX = v;
                    pX = (int)rl_u32((uint32_t)Yc, l);
                }
            }
        }
        // LOWER / else (:192-215): kind 1 = insert(node_n, hnew) (+ parent), 2 = insert(node, node.h)
        int kind = 0;
        double hnew = 0.0;
        bool setpar = false;
        if (nb) {
            const bool par_is_x = yc.parent == Xc;
            const double hc = hX + mcost;
            if (k_old == hX) {
                if (yc.t == T_NEW || (par_is_x && yc.h != hc) || (!par_is_x && yc.h > hc)) {
                    kind = 1; hnew = hc; setpar = true;
                }
            } else {
                if (yc.t == T_NEW || (par_is_x && yc.h != hc)) {
                    kind = 1; hnew = hc; setpar = true;
                } else if (!par_is_x && yc.h > hc) {
                    kind = 2;
                } else if (!par_is_x && hX > yc.h + mcost && yc.t == T_CLOSED && yc.h > k_old) {
                    kind = 1; hnew = yc.h;
                }
            }
        }
        // list appends in lane order: a kind-1 neighbour not yet in OPEN, and the node at its first kind-2 lane
        const uint64_t k2 = ballot(kind == 2);
        const int first2 = k2 ? __ffsll((long long)k2) - 1 : 64;
        const bool app = (kind == 1 && yc.t != T_OPEN) || (kind == 2 && lane == first2);
        const uint64_t appm = ballot(app);
        const uint32_t myE = S.ne + (uint32_t)__popcll(appm & ((1ull << lane) - 1ull));
        bool pushme = false;
        if (kind == 1) {
            const double k0 = yc.k;
            const bool was_open = yc.t == T_OPEN;
            if (yc.t == T_NEW) yc.k = hnew;
            else if (was_open) yc.k = fmin(yc.k, hnew);
            else yc.k = fmin(yc.h, hnew);
            yc.h = hnew;
            if (setpar) yc.parent = Xc;
            yc.t = T_OPEN;
            if (!was_open) yc.pos = myE;
            pushme = !was_open || yc.k != k0;
            store_c(S.cells, Yc, yc);
        }
        if (k2) {  // the node is CLOSED here: k = min(h, h) = h, t = OPEN, appended once
            xc.k = hX;
            xc.t = T_OPEN;
            xc.pos = rl_u32(myE, first2);
        }
        xc.h = hX;
        xc.parent = pX;
        if (lane == 0) store_c(S.cells, Xs, xc);
        if (Xs == S.start_slot) S.start_t = k2 ? T_OPEN : T_CLOSED;
        if (ballot(kind == 1 && Yc == S.start_slot)) S.start_t = T_OPEN;
        const int nap = __popcll(appm);
        S.ne += (uint32_t)nap;
        S.open += nap;
        heap16::wsync();
        {  // stored together, sifted up only where below the parent (heap16::push_batch: total order)
            const uint64_t pm = ballot(pushme);
            if (pm) {
                if (S.n + __popcll(pm) > S.heap_cap) {
                    S.overflow = true;
                } else {
                    Ent it;
                    it.g = yc.k;
                    it.a = yc.pos;
                    it.b = (uint32_t)Yc;
                    key.derive(it);
                    S.n = heap16::push_batch(S.hp, key, S.n, pm, it, S.root, lane);
                }
            }
        }
        if (k2 && !S.overflow) push(xc.k, xc.pos, Xs);
        return true;
    }

    // the reference's return value of processState: min k in OPEN, or -1 when it is empty
    __device__ __forceinline__ double kmin()
    {
        clean_top();
        return S.open > 0 ? S.root.g : -1.0;
    }

    // modify(node, node_parent) (:255-264)
    __device__ __forceinline__ void modify(int node, double hnew_if_closed, int64_t max_process)
    {
        DC3 c = load_c(S.cells, node);
        if (c.t == T_CLOSED) insert_uniform(node, c, hnew_if_closed);
        for (;;) {
            if (!process_state()) break;
            if (S.overflow || (max_process > 0 && S.np >= max_process)) break;
            const double km = kmin();
            if (km < 0.0 || km >= load_c(S.cells, node).h) break;
        }
    }
};

template <bool LDS>
__global__ __launch_bounds__(64) void dstar3d_kernel(
    const uint32_t* __restrict__ occ_all, int per_query, int X, int Y, int Z, const int32_t* __restrict__ start_xyz,
    const int32_t* __restrict__ goal_xyz, int nq, const int32_t* __restrict__ blocks, int nrounds, int nblk,
    double* __restrict__ cost_out, int32_t* __restrict__ plen_out, int32_t* __restrict__ path_out, int path_cap,
    int64_t* __restrict__ nproc_out, int32_t* __restrict__ status_out, int32_t* __restrict__ expand_out, int expand_cap,
    int64_t max_process, int* __restrict__ queue,
    uint4* __restrict__ spill_all, int heap_cap, int lds_cap, DC3* __restrict__ cells_all, uint32_t* __restrict__ occw_all,
    int words, const int32_t* __restrict__ order, int prio_n)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int worker = blockIdx.x;
    const int ncell = X * Y * Z;
    const size_t spill_n = (size_t)(heap_cap > lds_cap ? heap_cap - lds_cap : 0);
    Search S;
    S.hp = heap16::make_heap(smem, lds_cap, spill_all + (size_t)worker * spill_n, spill_n);
    S.cells = cells_all + (size_t)worker * (size_t)(ncell + 1);
    S.heap_cap = heap_cap;
    S.lds_cap = lds_cap;
    Occ<LDS> occ;
    occ.l = (lds_w32*)(smem + (size_t)16 * lds_cap);
    occ.g = occw_all + (size_t)worker * (size_t)words;
    occ.X = X;
    occ.Y = Y;
    occ.Z = Z;
    const Geo geo{X, Y, Z};
    D3<LDS> d{occ, geo, S, lane, 0, 0, 0, 0, 0, 0.0, KeyD()};
    heap16::pop_lane_consts(lane, d.pop_jl, d.pop_ol);
    d.pop_w = heap16::walk6_consts(lane, d.pop_jl, d.pop_ol);
    {
        const int l = lane < 26 ? lane : 0;
        d.mdx = c_m[l][0];
        d.mdy = c_m[l][1];
        d.mdz = c_m[l][2];
        d.mcost = dist3(d.mdx, d.mdy, d.mdz);
    }
    const int R1 = nrounds + 1;

    for (;;) {
        const int qi = next_query(queue, lane);
        if (qi >= nq) break;
        const int q = uni(order ? order[qi] : qi);
        // longest queries first, at raised priority (they set the launch's tail)
        if (qi < prio_n) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(0);
        const int sx = uni(start_xyz[3 * q]), sy = uni(start_xyz[3 * q + 1]), sz = uni(start_xyz[3 * q + 2]);
        const int gx = uni(goal_xyz[3 * q]), gy = uni(goal_xyz[3 * q + 1]), gz = uni(goal_xyz[3 * q + 2]);
        const bool in = (unsigned)sx < (unsigned)X && (unsigned)sy < (unsigned)Y && (unsigned)sz < (unsigned)Z &&
                        (unsigned)gx < (unsigned)X && (unsigned)gy < (unsigned)Y && (unsigned)gz < (unsigned)Z;
        if (!in) {  // endpoints outside the map: not supported (every lane stores the same values)
            for (int r = 0; r < R1; r++) {
                status_out[(size_t)q * R1 + r] = PMP_REF_RAISES;
                cost_out[(size_t)q * R1 + r] = 0.0;
                plen_out[(size_t)q * R1 + r] = 0;
                nproc_out[(size_t)q * R1 + r] = 0;
            }
            continue;
        }
        // working occupancy
        {
            const uint32_t* src = occ_all + (per_query ? (size_t)q * (size_t)words : 0);
            for (int w = lane; w < words; w += 64) {
                if (LDS) occ.l[w] = src[w];
                else occ.g[w] = src[w];
            }
        }
        const int start = geo.id(sx, sy, sz);
        S.goal_cell = geo.id(gx, gy, gz);
        S.goal_slot = start == S.goal_cell ? ncell : S.goal_cell;
        // DStar3D.__init__ (:70-93): every voxel NEW with h = k = inf; the goal object h = 0; insert(goal, 0)
        {
            DC3 v;
            v.h = v.k = __builtin_inf();
            v.parent = -1;
            v.pos = v.t = v.pad = 0u;
            for (int c = lane; c <= ncell; c += 64) store_c(S.cells, c, v);
        }
        heap16::wsync();
        S.n = 0;
        S.open = 0;
        S.ne = 0;
        S.np = 0;
        S.overflow = false;
        S.ex = expand_out ? expand_out + (size_t)q * (size_t)expand_cap : nullptr;
        S.ex_cap = expand_cap;
        S.start_slot = start;
        S.start_t = T_NEW;
        {
            DC3 gcell;
            gcell.h = 0.0;
            gcell.k = __builtin_inf();
            gcell.parent = -1;
            gcell.pos = gcell.t = gcell.pad = 0u;
            d.insert_uniform(S.goal_slot, gcell, 0.0);
        }
        // ---- plan() (:100-109)
        int st = PMP_FOUND;
        for (;;) {
            if (!d.process_state()) break;  // OPEN empty
            if (S.overflow) { st = PMP_CAP_OVERFLOW; break; }
            if (S.open == 0) break;                                  // kmin < 0
            if (S.start_t == T_CLOSED) break;                        // self.start.t == "CLOSED"
            if (max_process > 0 && S.np >= max_process) { st = PMP_CAP_OVERFLOW; break; }
        }
        S.ex = nullptr;  // the expand records are plan()'s
        for (int r = 0; r <= nrounds; r++) {
            if (r > 0) {
                // apply_dynamic_obstacles(newly_blocked) (:115-149): block, then walk from the start
                heap16::wsync();
                const int32_t* b = blocks + ((size_t)q * nrounds + (r - 1)) * (size_t)nblk * 3;
                for (int i = lane; i < nblk; i += 64) {
                    const int bx = b[3 * i], by = b[3 * i + 1], bz = b[3 * i + 2];
                    if ((unsigned)bx < (unsigned)X && (unsigned)by < (unsigned)Y && (unsigned)bz < (unsigned)Z)
                        occ.set((uint32_t)geo.id(bx, by, bz));
                }
                if (LDS) __syncthreads();
                heap16::wsync();
                S.np = 0;  // self.EXPAND.clear()
            }
            // walk from the start along the parents (plan: extractPath :153-166; rounds: the while loop
            // of :131-144 with modify on a collision); lane 0 writes the path
            int node = start;
            double cost = 0.0;
            int plen = 0;
            int32_t* pth = path_out + ((size_t)q * R1 + r) * (size_t)path_cap;
            int rst = st;
            const int64_t bound = 4 * (int64_t)ncell + 4;
            int64_t steps = 0;
            if (st == PMP_FOUND) {
                if (r == 0) {
                    if (lane == 0) pth[0] = start;
                    plen = 1;
                }
                while (node != S.goal_cell) {
                    if (++steps > bound) { rst = PMP_CAP_OVERFLOW; break; }
                    const DC3 c = load_c(S.cells, node);
                    int nxm, nym, nzm;
                    geo.xyz(node, nxm, nym, nzm);
                    if (c.parent < 0) {
                        if (r > 0) {
                            // modify(node, self.goal): cost(node, goal) may join non-adjacent voxels
                            const DC3 gc = load_c(S.cells, S.goal_slot);
                            int ax, ay, az;
                            geo.xyz(S.goal_cell, ax, ay, az);
                            const double cg = occ.coll(nxm, nym, nzm, ax, ay, az) ? __builtin_inf()
                                                                                 : dist3(ax - nxm, ay - nym, az - nzm);
                            d.modify(node, gc.h + cg, max_process);
                        }
                        rst = PMP_NO_PATH;
                        break;
                    }
                    const int p = c.parent;
                    int px, py, pz;
                    geo.xyz(p, px, py, pz);
                    const bool coll = occ.coll(nxm, nym, nzm, px, py, pz);
                    if (r > 0 && coll) {
                        // modify(node, node_parent): cost is inf (they collide)
                        const int pslot = p == S.goal_cell ? S.goal_slot : p;
                        d.modify(node, load_c(S.cells, pslot).h + __builtin_inf(), max_process);
                        if (S.overflow || (max_process > 0 && S.np >= max_process)) { rst = PMP_CAP_OVERFLOW; break; }
                        continue;
                    }
                    if (r > 0) {
                        if (plen < path_cap && lane == 0) pth[plen] = node;
                        plen++;
                    }
                    cost += coll ? __builtin_inf() : dist3(px - nxm, py - nym, pz - nzm);
                    node = p;
                    if (r == 0) {
                        if (plen < path_cap && lane == 0) pth[plen] = node;
                        plen++;
                    }
                }
                if (r > 0 && node == S.goal_cell && rst == PMP_FOUND) {
                    if (plen < path_cap && lane == 0) pth[plen] = node;
                    plen++;
                }
                if (rst == PMP_FOUND && plen > path_cap) rst = PMP_PATH_OVERFLOW;
            }
            if (lane == 0) {
                status_out[(size_t)q * R1 + r] = rst;
                cost_out[(size_t)q * R1 + r] = cost;
                plen_out[(size_t)q * R1 + r] = plen;
                nproc_out[(size_t)q * R1 + r] = S.np;
            }
            if (rst == PMP_CAP_OVERFLOW) st = PMP_CAP_OVERFLOW;
        }
        heap16::wsync();
    }
}

constexpr int kOccLdsWords = 2048;  // grids up to 65536 voxels keep the working occupancy in LDS
constexpr size_t kScratchBudget = (size_t)16 << 30;

}  // namespace

extern "C" int pmp_dstar3d_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int per_query, int X, int Y,
                                 int Z, const int32_t* start_xyz, const int32_t* goal_xyz, int nq, const int32_t* blocks,
                                 int nrounds, int nblk, double* cost, int32_t* path_len, int32_t* path, int path_cap,
                                 int64_t* n_process, int32_t* status, int32_t* expand, int expand_cap,
                                 int64_t max_process)
{
    if (!ctx) return PMP_EINVAL;
    if (X < 1 || Y < 1 || Z < 1 || X > kMaxDim || Y > kMaxDim || Z > kMaxDim)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar3d_batch: X, Y, Z must be in [1, 256]");
    if (nq < 0 || path_cap < 1 || nrounds < 0 || nblk < 0 || (nrounds > 0 && nblk > 0 && !blocks) ||
        (expand && expand_cap < 1))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar3d_batch: bad nq/path_cap/nrounds/nblk/blocks");
    if (nq == 0) return PMP_OK;
    if (!occ_bits || !start_xyz || !goal_xyz || !cost || !path_len || !path || !n_process || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar3d_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t ncell = (size_t)X * Y * Z;
    const int words = (int)((ncell + 31) / 32);
    bool lds_occ = words <= kOccLdsWords;
    const int per_cu = std::max(1, std::min(ctx->workers_per_cu > 0 ? ctx->workers_per_cu : 16, (nq + 255) / 256));
    int occ_bytes = lds_occ ? ((words * 4 + 15) & ~15) : 0;
    // heap: one valid element per OPEN voxel plus stale ones; 8 pushes per voxel bound the total
    const size_t hc = std::min<size_t>(8 * (ncell + 1) + 64, (size_t)1 << 26);
    const int heap_cap = (int)hc;
    int lds_cap = pmp_heap_lds_cap(ctx, per_cu, occ_bytes, 16);
    if (lds_cap < kMinLdsHeap && lds_occ) {  // the LDS share cannot hold the occupancy too: keep it in HBM
        lds_occ = false;
        occ_bytes = 0;
        lds_cap = pmp_heap_lds_cap(ctx, per_cu, 0, 16);
    }
    if (lds_cap < kMinLdsHeap)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dstar3d_batch: workers / resident per CU leave no LDS heap share");
    if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    const size_t spill_n = heap_cap > lds_cap ? (size_t)(heap_cap - lds_cap) : 0;
    const size_t per_worker = (ncell + 1) * sizeof(DC3) + spill_n * 16 + (lds_occ ? 0 : (size_t)words * 4) + 256;
    int workers = 256 * per_cu;
    const size_t fit = kScratchBudget / per_worker;
    if (fit < 1) return pmp_set_err(ctx, PMP_ENOMEM, "pmp_dstar3d_batch: one worker exceeds the scratch budget");
    if ((size_t)workers > fit) workers = (int)fit;
    if (workers > nq) workers = nq;
    uint4* spill = (uint4*)pmp_scratch(ctx, SCR_AUX1, (size_t)workers * spill_n * 16 + 16);
    DC3* cells = (DC3*)pmp_scratch(ctx, SCR_AUX2, (size_t)workers * (ncell + 1) * sizeof(DC3) + 16);
    uint32_t* occw = lds_occ ? nullptr : (uint32_t*)pmp_scratch(ctx, SCR_AUX3, (size_t)workers * words * 4 + 16);
    int* queue = (int*)pmp_scratch(ctx, SCR_AUX0, 256);
    if (!spill || !cells || !queue || (!lds_occ && !occw)) return PMP_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    PMP_HIP_CHECK(ctx, hipMemsetAsync(queue, 0, 16, s));
    int32_t* order = nullptr;
    {
        const int rc = pmp_lpt_order3d(ctx, s, start_xyz, goal_xyz, nq, X, Y, Z, workers, &order);
        if (rc) return rc;
    }
    auto kern = lds_occ ? dstar3d_kernel<true> : dstar3d_kernel<false>;
    hipLaunchKernelGGL(kern, dim3(workers), dim3(64), (size_t)lds_cap * 16 + occ_bytes, s, occ_bits, per_query, X, Y, Z,
                       start_xyz, goal_xyz, nq, blocks, nrounds, nblk, cost, path_len, path, path_cap, n_process, status,
                       expand, expand_cap, max_process, queue, spill, heap_cap, lds_cap, cells, occw, words,
                       (const int32_t*)order, order ? ctx->astar_prio_n : 0);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
