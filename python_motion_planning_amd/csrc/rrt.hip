// Batched RRT / RRT* for gfx950 (global_planner/sample_search/rrt.py:49-151, rrt_star.py:43-76,
// sample_search.py:27-135): one 512-thread workgroup per query grows that query's tree.
//
// Per iteration (all decisions wave-uniform, results identical to the reference's sequential loop):
//  1. sample from the query's np.random stream (generateRandomNode, rrt.py:91-103);
//  2. nearest node = first argmin of the exact CPython hypot (rrt.py:117-118).  A coarse pass over a
//     16-bit fixed-point copy of the coordinates (4 B/node) finds the minimum; only nodes within a
//     rigorous error band of it are re-evaluated exactly in f64; ties resolve to the lowest index.
//     The coarse copy lives in the workgroup's LDS (round 5: ~31k nodes beside the rest of the
//     workgroup's state; nodes beyond that in HBM/L2), so the two whole-tree scans of an iteration
//     (nearest, in-radius) read LDS instead of streaming the tree from L2.  A zero distance means
//     the sample is already in sample_list (rrt.py:67-68);
//  3. steer (hypot, atan2, cos, sin) and isCollision(new, near), the obstacle tests spread over the
//     workgroup;
//  4. RRT*: the sequential choose-parent/rewire scan (rrt_star.py:57-73) in parallel form.  With
//     G0 = the steered g and c_i = g_i + d_i for in-radius nodes i, node_new.g before node i is
//     G_{i-1} = min(G0, c_j : j < i, c_j < G0, collision-free) (a strict `>` keeps the earliest
//     minimum, so the final parent is the lowest index attaining it).  Only the few nodes with
//     c_i < G0 need a collision test to build that set; then every in-radius node decides its
//     rewire (g_i > G_{i-1} + d_i and collision-free) independently;
//  5. insert (a node landing exactly on an existing one replaces it, like the dict), goal test.
#include "localplan.h"

namespace {

// threads per query: 256, two workgroups per CU (round 6, tools/calls/r6_call37-39.sh: the iteration is a
// chain of barriers and dependent L2 rounds, so a second query per CU hides it -- 955 -> 1,475 plans/s
// over 512 x 1; 128 x 4 and a 168-VGPR 256 x 3 build are slower.  Round 5, when the whole-tree f32 scans
// dominated, 512 x 1 was the faster shape)
#ifndef PMP_RRT_NT
#define PMP_RRT_NT 256
#endif
constexpr int kNT = PMP_RRT_NT;
#ifndef PMP_RRT_PERCU
#define PMP_RRT_PERCU (512 / PMP_RRT_NT)
#endif
#ifndef PMP_RRT_MINW
#define PMP_RRT_MINW 1
#endif
constexpr int kWaves = kNT / 64;
constexpr int kMaxObs = 256;   // per obstacle kind
constexpr int kMaxBnd = 8;
// The candidate lists keep their first entries in LDS and the rest in per-query HBM lists (C3: an
// r = 10 ball holds tens of nodes), so the LDS goes to the coarse tree copy.
#ifndef PMP_RRT_KMAX
#define PMP_RRT_KMAX 128
#endif
constexpr int kMaxA = PMP_RRT_KMAX;  // collision-free improving candidates per iteration
constexpr int kMaxT = PMP_RRT_KMAX;  // candidates awaiting a collision test per phase
constexpr int kMaxK = PMP_RRT_KMAX;  // in-radius candidates kept in LDS (more spill to the HBM list)
#ifndef PMP_RRT_RND
#define PMP_RRT_RND 256
#endif
#ifndef PMP_RRT_MAXH
#define PMP_RRT_MAXH 512
#endif
constexpr int kRnd = PMP_RRT_RND;    // random doubles staged in LDS
constexpr int kMaxH = PMP_RRT_MAXH;  // coarse in-radius hits staged in LDS (more are resolved inline)
constexpr int kBins = 16;      // obstacle bins per axis over the map
constexpr int kLdsBytes = 160 * 1024;  // the CU's LDS
constexpr int kRrtMaxResident = 4;     // LDS tree shares per CU RRT honours from pmp_set_resident_per_cu

constexpr int KF_A = 1;        // c_i < G0
constexpr int KF_VALID = 2;    // ... and collision-free

struct KEntry {
    int j, flags;
    double d;
};
struct TEntry {  // a candidate awaiting a collision test: K index, G_{i-1}
    int k, pad;
    double G;
};
struct AEntry {  // a collision-free improving candidate: node, c = g + d
    int j, pad;
    double c;
};

struct RrtArgs {
    pmp_rrt_params P;
    const double *rect, *circ, *bnd;
    int nr, nc, nb;
    const double *start, *goal;
    int nq;
    const double* rnd;
    int64_t stride;
    int cap;
    double *txy, *tg;
    int32_t* tpar;
    int32_t* n_nodes;
    double* cost;
    int32_t* path_len;
    double* path;
    int path_cap;
    int64_t* draws;
    int32_t* status;
    int64_t* counters;  // nullable [nq][4]
    uint32_t* xyq;    // scratch [nq][cap]: 16-bit fixed-point x | y << 16 (the coarse copy beyond LDS)
    KEntry* klist;    // scratch [nq][cap]
    TEntry* tlist;    // scratch [nq][cap]
    AEntry* alist;    // scratch [nq][cap]
    int lcap;         // nodes of the coarse copy held in LDS
};

struct RrtShared {
    float redf[kWaves];
    double redd[kWaves];
    int redi[kWaves];
    int aj[kMaxA];
    double ac[kMaxA];
    int tk[kMaxT];      // K entries awaiting a collision test
    double tG[kMaxT];   // ... and their G_{i-1}
    // in-radius candidates (first kMaxK in LDS, with the node's coordinates and g loaded once)
    int kj[kMaxK], kf[kMaxK];
    double kd[kMaxK], kx[kMaxK], ky[kMaxK], kg[kMaxK];
    double rbuf[kRnd];  // window of the query's random stream
    // obstacle bins: bit o of bin (bx, by) = obstacle o's inflated box (plus a margin) meets the bin
    // (o: circles, then rects, then the boundary -- coll_item's order); <= 128 obstacles
    uint64_t binm[kBins * kBins][2];
    double bininv_x, bininv_y;
    int use_bins;
    uint32_t t2a[kWaves], t2b[kWaves];  // the nearest scan's per-wave top-2 ...
    int t2i[kWaves];                 // ... and the minimum's index
    double nearx, neary, nearg, nearh;
    int nK, nA, nT, nT2, slot;
    int hj[kMaxH];  // coarse in-radius hits of the scan, resolved exactly after it (one load round)
    int nH;
    double newx, newy, newG;  // the fused step's node_new (wave 0's steering)
    int fflag;                // ... 1 the sample is already in the tree, 2 the segment collides
};

// The obstacles sit at the head of the dynamic LDS (rects, 4 doubles each, then circles, 3, then the
// boundary, 4), sized to the map's counts; the coarse tree copy follows them
}  // namespace
extern __shared__ __attribute__((aligned(16))) unsigned char rrt_lds_dyn[];
namespace {
__device__ __forceinline__ const double* obs_rect() { return (const double*)rrt_lds_dyn; }
__device__ __forceinline__ const double* obs_circ(int nr) { return obs_rect() + 4 * nr; }
__device__ __forceinline__ const double* obs_bnd(int nr, int nc) { return obs_rect() + 4 * nr + 3 * nc; }
__host__ __device__ inline int obs_bytes(int nr, int nc, int nb) { return ((4 * nr + 3 * nc + 4 * nb) * 8 + 15) & ~15; }

// ---- obstacle tests (sample_search.py), same operation order as the oracle ----
__device__ inline bool in_box(const double* r, double d, double x, double y)
{
    const double px = x - (r[0] - d), py = y - (r[1] - d);
    return 0 <= px && px <= r[2] + 2 * d && 0 <= py && py <= r[3] + 2 * d;
}

__device__ inline double cross3(double p1x, double p1y, double p2x, double p2y, double p3x, double p3y)
{
    const double x1 = p2x - p1x, y1 = p2y - p1y, x2 = p3x - p1x, y2 = p3y - p1y;
    return x1 * y2 - x2 * y1;
}

__device__ bool inter_rect(const double* r, double d, double x1, double y1, double x2, double y2)
{
    const double vx[4] = {r[0] - d, r[0] + r[2] + d, r[0] + r[2] + d, r[0] - d};
    const double vy[4] = {r[1] - d, r[1] - d, r[1] + r[3] + d, r[1] + r[3] + d};
    for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++) {
            if (fmax(x1, x2) >= fmin(vx[a], vx[b]) && fmin(x1, x2) <= fmax(vx[a], vx[b]) &&
                fmax(y1, y2) >= fmin(vy[a], vy[b]) && fmin(y1, y2) <= fmax(vy[a], vy[b])) {
                if (cross3(vx[a], vy[a], vx[b], vy[b], x1, y1) * cross3(vx[a], vy[a], vx[b], vy[b], x2, y2) <= 0 &&
                    cross3(x1, y1, x2, y2, vx[a], vy[a]) * cross3(x1, y1, x2, y2, vx[b], vy[b]) <= 0)
                    return true;
            }
        }
    return false;
}

// np.dot of 2-vectors = OpenBLAS ddot: fma(a1, b1, a0 * b0)
__device__ bool inter_circle(const double* c, double d, double x, double y, double x2, double y2)
{
    const double dx = x2 - x, dy = y2 - y;
    const double d2 = fma(dy, dy, dx * dx);
    if (d2 == 0) return false;
    const double t = fma(c[1] - y, dy, (c[0] - x) * dx) / d2;
    if (0 <= t && t <= 1) {
        const double sx = x + t * dx, sy = y + t * dy;
        if (lp::py_hypot(c[0] - sx, c[1] - sy) <= c[2] + d) return true;
    }
    return false;
}

// collision test item `it` of isCollision(p1, p2): inside(p1) circles/rects/boundary, inside(p2)
// ..., rect crossings, circle crossings (sample_search.py:27-49).  Exact bounding-box rejections
// come first: |dx| > r + d already implies hypot > r + d (hypot >= |dx| exactly), and a segment
// whose bbox misses the inflated rect fails every "rapid repulsion" pair test.
__device__ inline bool coll_item(const RrtShared& S, int nr, int nc, int nb, double d, int it, double x1, double y1,
                                 double x2, double y2)
{
    const int per = nc + nr + nb;
    double x = x1, y = y1;
    if (it >= per && it < 2 * per) { it -= per; x = x2; y = y2; }
    if (it < per) {
        if (it < nc) {
            const double* c = &obs_circ(nr)[3 * it];
            const double rr = c[2] + d;
            if (fabs(x - c[0]) > rr || fabs(y - c[1]) > rr) return false;
            return lp::py_hypot(x - c[0], y - c[1]) <= rr;
        }
        it -= nc;
        if (it < nr) return in_box(&obs_rect()[4 * it], d, x, y);
        return in_box(&obs_bnd(nr, nc)[4 * (it - nr)], d, x, y);
    }
    it -= 2 * per;
    const double bx0 = fmin(x1, x2), bx1 = fmax(x1, x2), by0 = fmin(y1, y2), by1 = fmax(y1, y2);
    if (it < nr) {
        const double* r = &obs_rect()[4 * it];
        if (bx1 < r[0] - d || bx0 > r[0] + r[2] + d || by1 < r[1] - d || by0 > r[1] + r[3] + d) return false;
        return inter_rect(r, d, x1, y1, x2, y2);
    }
    it -= nr;
    const double* c = &obs_circ(nr)[3 * it];
    // the projected point lies within the segment's bbox (up to rounding): a gap of more than
    // r + d (with slack for the rounding) rules the circle out
    const double rr = (c[2] + d) * (1.0 + 1e-12) + 1e-12;
    if (bx1 < c[0] - rr || bx0 > c[0] + rr || by1 < c[1] - rr || by0 > c[1] + rr) return false;
    return inter_circle(c, d, x1, y1, x2, y2);
}

__device__ inline int coll_items(int nr, int nc, int nb) { return 2 * (nc + nr + nb) + nr + nc; }

// ---- binned collision tests: only the obstacles whose bins meet the segment's bounding box --------
// Every item coll_item can find true (p1 or p2 inside an inflated obstacle, the segment crossing
// one) lies in the segment's bounding box and in the obstacle's inflated box, so the two boxes share
// a bin (the same monotone bin map for both): the items of the other obstacles are false, and the
// OR over the rest is isCollision's answer bit for bit.
__device__ __forceinline__ int bin_of(double v, double inv)
{
    return (int)floor(fmin(fmax(v * inv, 0.0), (double)(kBins - 1)));
}

// j-th set bit of x (j < popcount(x))
__device__ __forceinline__ int select64(uint64_t x, int j)
{
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __popcll(x & ((1ull << w) - 1ull));
        if (j >= c) { j -= c; x >>= w; pos += w; }
    }
    return pos;
}

// the obstacles of the bins the box of (x1, y1)-(x2, y2) meets; false: too many bins (test all)
__device__ __forceinline__ bool bins_mask(const RrtShared& S, double x1, double y1, double x2, double y2, uint64_t& lo,
                                          uint64_t& hi)
{
    const int bx0 = bin_of(fmin(x1, x2), S.bininv_x), bx1 = bin_of(fmax(x1, x2), S.bininv_x);
    const int by0 = bin_of(fmin(y1, y2), S.bininv_y), by1 = bin_of(fmax(y1, y2), S.bininv_y);
    if (!S.use_bins || (bx1 - bx0 + 1) * (by1 - by0 + 1) > 9) return false;
    lo = 0;
    hi = 0;
    for (int by = by0; by <= by1; by++)
        for (int bx = bx0; bx <= bx1; bx++) {
            lo |= S.binm[by * kBins + bx][0];
            hi |= S.binm[by * kBins + bx][1];
        }
    return true;
}

// item t of the binned list (3 per obstacle: inside p1, inside p2, crossing) as a coll_item index, or -1
__device__ __forceinline__ int bin_item(uint64_t lo, int nlo, uint64_t hi, int t, int nr, int nc, int nb)
{
    const int j = t / 3, kind = t - 3 * j;
    const int o = j < nlo ? select64(lo, j) : 64 + select64(hi, j - nlo);
    const int per = nc + nr + nb;
    if (kind < 2) return kind * per + o;
    if (o < nc) return 2 * per + nr + o;       // circle crossing
    if (o < nc + nr) return 2 * per + (o - nc);  // rect crossing
    return -1;                                  // the boundary has no crossing test
}

// one wave cooperates on one isCollision(p1, p2); wave-uniform result
__device__ bool collision_wave(const RrtShared& S, int nr, int nc, int nb, double d, double x1, double y1, double x2,
                               double y2)
{
    bool hit = false;
    uint64_t lo, hi;
    if (bins_mask(S, x1, y1, x2, y2, lo, hi)) {
        const int nlo = __popcll(lo), items = 3 * (nlo + __popcll(hi));
        for (int t = lane_id(); t < items; t += 64) {
            const int it = bin_item(lo, nlo, hi, t, nr, nc, nb);
            if (it >= 0) hit |= coll_item(S, nr, nc, nb, d, it, x1, y1, x2, y2);
        }
    } else {
        const int items = coll_items(nr, nc, nb);
        for (int it = lane_id(); it < items; it += 64) hit |= coll_item(S, nr, nc, nb, d, it, x1, y1, x2, y2);
    }
    return ballot(hit) != 0;
}

// the same with the obstacle set given (a superset of every obstacle the segment's items can find
// true for: the extra items are exact tests that come out false); om = false: the segment's own bins
__device__ bool collision_wave_o(const RrtShared& S, int nr, int nc, int nb, double d, double x1, double y1, double x2,
                                 double y2, bool om, uint64_t lo, uint64_t hi)
{
    if (!om) return collision_wave(S, nr, nc, nb, d, x1, y1, x2, y2);
    bool hit = false;
    const int nlo = __popcll(lo), items = 3 * (nlo + __popcll(hi));
    for (int t = lane_id(); t < items; t += 64) {
        const int it = bin_item(lo, nlo, hi, t, nr, nc, nb);
        if (it >= 0) hit |= coll_item(S, nr, nc, nb, d, it, x1, y1, x2, y2);
    }
    return ballot(hit) != 0;
}

// workgroup-parallel isCollision(p1, p2); every thread gets the result
__device__ bool collision_block(const RrtShared& S, int nr, int nc, int nb, double d, double x1, double y1, double x2,
                                double y2)
{
    int hit = 0;
    uint64_t lo, hi;
    // (the bins only when the full list would take more than one pass of the workgroup)
    if (coll_items(nr, nc, nb) > kNT && bins_mask(S, x1, y1, x2, y2, lo, hi)) {
        const int nlo = __popcll(lo), items = 3 * (nlo + __popcll(hi));
        for (int t = threadIdx.x; t < items; t += kNT) {
            const int it = bin_item(lo, nlo, hi, t, nr, nc, nb);
            if (it >= 0) hit |= coll_item(S, nr, nc, nb, d, it, x1, y1, x2, y2);
        }
    } else {
        const int items = coll_items(nr, nc, nb);
        for (int it = threadIdx.x; it < items; it += kNT) hit |= coll_item(S, nr, nc, nb, d, it, x1, y1, x2, y2);
    }
    return __syncthreads_or(hit) != 0;
}

typedef short rrt_v2i16 __attribute__((ext_vector_type(2)));
// squared distance of two quantised points (x | y << 16, 15-bit coordinates): exact
__device__ __forceinline__ uint32_t cd2(uint32_t p, uint32_t q)
{
    const rrt_v2i16 d = __builtin_bit_cast(rrt_v2i16, p) - __builtin_bit_cast(rrt_v2i16, q);
    return (uint32_t)__builtin_amdgcn_sdot2(d, d, 0, false);
}

// One step of a wave's top-2 reduction (the minimum with its lowest index, the second-smallest value)
// over DPP: lanes take the value of another lane (CTRL) in the rows RM enables, the others combine
// with the neutral element.  row_ror 1, 2, 4, 8 then row_bcast 15 / 31 cover disjoint lane sets at
// every step, so lane 63 ends with the wave's top-2 (a VALU chain instead of six LDS-pipe permutes).
template <int CTRL, int RM>
__device__ __forceinline__ void top2_dpp(uint32_t& a, uint32_t& b, int& i)
{
    const uint32_t oa = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)a, CTRL, RM, 0xF, false);
    const uint32_t ob = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)b, CTRL, RM, 0xF, false);
    const int oi = __builtin_amdgcn_update_dpp(0x7fffffff, i, CTRL, RM, 0xF, false);
    b = min(min(max(oa, a), b), ob);
    const bool take = oa < a || (oa == a && oi < i);
    a = take ? oa : a;
    i = take ? oi : i;
}
__device__ __forceinline__ void wave_top2(uint32_t& a, uint32_t& b, int& i)
{
    top2_dpp<0x121, 0xF>(a, b, i);  // row_ror:1
    top2_dpp<0x122, 0xF>(a, b, i);  // row_ror:2
    top2_dpp<0x124, 0xF>(a, b, i);  // row_ror:4
    top2_dpp<0x128, 0xF>(a, b, i);  // row_ror:8
    top2_dpp<0x142, 0xA>(a, b, i);  // row_bcast:15 into rows 1, 3
    top2_dpp<0x143, 0x8>(a, b, i);  // row_bcast:31 into row 3
    a = (uint32_t)__builtin_amdgcn_readlane((int)a, 63);
    b = (uint32_t)__builtin_amdgcn_readlane((int)b, 63);
    i = __builtin_amdgcn_readlane(i, 63);
}

// The same for the lexicographic minimum of (f64 v, index i): every lane gets it
template <int CTRL, int RM>
__device__ __forceinline__ void min_di_dpp(double& v, int& i)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, RM, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0x7FF00000, (int)(uint32_t)(b >> 32), CTRL, RM, 0xF, false);
    const double ov = __longlong_as_double(((uint64_t)hi << 32) | lo);  // neutral: +inf
    const int oi = __builtin_amdgcn_update_dpp(0x7fffffff, i, CTRL, RM, 0xF, false);
    const bool take = ov < v || (ov == v && oi < i);
    v = take ? ov : v;
    i = take ? oi : i;
}
__device__ __forceinline__ void wave_min_di(double& v, int& i)
{
    min_di_dpp<0x121, 0xF>(v, i);
    min_di_dpp<0x122, 0xF>(v, i);
    min_di_dpp<0x124, 0xF>(v, i);
    min_di_dpp<0x128, 0xF>(v, i);
    min_di_dpp<0x142, 0xA>(v, i);
    min_di_dpp<0x143, 0x8>(v, i);
    v = rl_f64(v, 63);
    i = __builtin_amdgcn_readlane(i, 63);
}

// ---- workgroup reductions ----
__device__ float block_min_f(float v, RrtShared& S)
{
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) S.redf[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = S.redf[0];
    for (int w = 1; w < kWaves; w++) r = fminf(r, S.redf[w]);
    __syncthreads();
    return r;
}

// lexicographic min of (v, i)
__device__ void block_min_di(double& v, int& i, RrtShared& S)
{
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o);
        const int oi = __shfl_xor(i, o);
        if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
    }
    if ((threadIdx.x & 63) == 0) { S.redd[threadIdx.x >> 6] = v; S.redi[threadIdx.x >> 6] = i; }
    __syncthreads();
    v = S.redd[0];
    i = S.redi[0];
    for (int w = 1; w < kWaves; w++)
        if (S.redd[w] < v || (S.redd[w] == v && S.redi[w] < i)) { v = S.redd[w]; i = S.redi[w]; }
    __syncthreads();
}

struct KRec {
    int j, fl;
    double d, x, y, g;
};

// candidate k: from LDS, or (k >= kMaxK) from the HBM list plus the node arrays
__device__ __forceinline__ KRec kget(const RrtShared& S, const KEntry* kl, const double* tx, const double* tg, int k)
{
    KRec r;
    if (k < kMaxK) {
        r.j = S.kj[k]; r.fl = S.kf[k]; r.d = S.kd[k]; r.x = S.kx[k]; r.y = S.ky[k]; r.g = S.kg[k];
    } else {
        const KEntry e = kl[k];
        r.j = e.j; r.fl = e.flags; r.d = e.d; r.x = tx[2 * e.j]; r.y = tx[2 * e.j + 1]; r.g = tg[e.j];
    }
    return r;
}

__device__ __forceinline__ void kset_flags(RrtShared& S, KEntry* kl, int k, int fl)
{
    if (k < kMaxK) S.kf[k] = fl;
    else kl[k].flags = fl;
}

__device__ __forceinline__ void tset(RrtShared& S, TEntry* tl, int t, int k, double G)
{
    if (t < kMaxT) { S.tk[t] = k; S.tG[t] = G; }
    else { TEntry e; e.k = k; e.pad = 0; e.G = G; tl[t] = e; }
}
__device__ __forceinline__ int tget_k(const RrtShared& S, const TEntry* tl, int t) { return t < kMaxT ? S.tk[t] : tl[t].k; }
__device__ __forceinline__ double tget_G(const RrtShared& S, const TEntry* tl, int t) { return t < kMaxT ? S.tG[t] : tl[t].G; }
__device__ __forceinline__ void aset(RrtShared& S, AEntry* al, int a, int j, double c)
{
    if (a < kMaxA) { S.aj[a] = j; S.ac[a] = c; }
    else { AEntry e; e.j = j; e.pad = 0; e.c = c; al[a] = e; }
}
__device__ __forceinline__ int aget_j(const RrtShared& S, const AEntry* al, int a) { return a < kMaxA ? S.aj[a] : al[a].j; }
__device__ __forceinline__ double aget_c(const RrtShared& S, const AEntry* al, int a) { return a < kMaxA ? S.ac[a] : al[a].c; }

typedef __attribute__((address_space(3))) uint32_t lds_xyq;

template <bool STAR>
__global__ __launch_bounds__(kNT, PMP_RRT_MINW) void rrt_kernel(RrtArgs A)
{
    __shared__ RrtShared S;
    const int lcap = A.lcap;
    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    if (q >= A.nq) return;
    const int nr = A.nr, nc = A.nc, nb = A.nb;
    lds_xyq* xl = (lds_xyq*)(rrt_lds_dyn + obs_bytes(nr, nc, nb));  // nodes 0 .. lcap-1 of the coarse copy
    {
        double* ob = (double*)rrt_lds_dyn;
        for (int i = tid; i < 4 * nr; i += kNT) ob[i] = A.rect[i];
        for (int i = tid; i < 3 * nc; i += kNT) ob[4 * nr + i] = A.circ[i];
        for (int i = tid; i < 4 * nb; i += kNT) ob[4 * nr + 3 * nc + i] = A.bnd[i];
    }
    const pmp_rrt_params P = A.P;
    if (tid == 0) {
        S.use_bins = nc + nr + nb <= 128 && P.x_range > 0 && P.y_range > 0;
        S.bininv_x = kBins / P.x_range;
        S.bininv_y = kBins / P.y_range;
    }
    __syncthreads();
    for (int b = tid; b < kBins * kBins; b += kNT) {
        // obstacle boxes inflated by delta plus 1e-3 (far above every rounding slack of coll_item's
        // tests at map coordinates), mapped with the query's bin_of
        const int bx = b % kBins, by = b / kBins;
        uint64_t m0 = 0, m1 = 0;
        const double mg = P.delta + 1e-3;
        for (int o = 0; S.use_bins && o < nc + nr + nb; o++) {
            double x0, x1, y0, y1;
            if (o < nc) {
                const double* c = &obs_circ(nr)[3 * o];
                x0 = c[0] - c[2] - mg; x1 = c[0] + c[2] + mg; y0 = c[1] - c[2] - mg; y1 = c[1] + c[2] + mg;
            } else {
                const double* r = o < nc + nr ? &obs_rect()[4 * (o - nc)] : &obs_bnd(nr, nc)[4 * (o - nc - nr)];
                x0 = r[0] - mg; x1 = r[0] + r[2] + mg; y0 = r[1] - mg; y1 = r[1] + r[3] + mg;
            }
            if (bin_of(x0, S.bininv_x) <= bx && bx <= bin_of(x1, S.bininv_x) && bin_of(y0, S.bininv_y) <= by &&
                by <= bin_of(y1, S.bininv_y))
            {
                if (o < 64) m0 |= 1ull << o;
                else m1 |= 1ull << (o - 64);
            }
        }
        S.binm[b][0] = m0;
        S.binm[b][1] = m1;
    }
    __syncthreads();
    const double delta = P.delta;
    const int cap = A.cap;
    double* tx = A.txy + (size_t)q * cap * 2;
    double* tg = A.tg + (size_t)q * cap;
    int32_t* tpar = A.tpar + (size_t)q * cap;
    uint32_t* xyq = A.xyq + (size_t)q * cap;
    KEntry* kl = A.klist + (size_t)q * cap;
    TEntry* tl = A.tlist + (size_t)q * cap;
    AEntry* al = A.alist + (size_t)q * cap;
    // node j's coarse copy: LDS below lcap, HBM above (every node is written once, by thread 0, and
    // read after a barrier)
    auto xq_store = [&](int j, uint32_t v) {
        if (j < lcap) xl[j] = v;
        else xyq[j] = v;
    };
    const double* rnd = A.rnd + (size_t)q * A.stride;
    const double sx0 = A.start[2 * q], sy0 = A.start[2 * q + 1];
    const double gx = A.goal[2 * q], gy = A.goal[2 * q + 1];
    // Coarse coordinates: every node lies in the box spanned by the map, the start and the goal
    // (steering moves toward samples inside the map), quantised to 15 bits per axis (round 6; 16
    // before) and packed x | y << 16.  Query points (the sample, node_new, the nearest node) are
    // quantised the same way, so a coarse squared distance is exact integer arithmetic on the
    // quantised points -- one packed i16 subtraction and one dot2 (|dx|, |dy| <= 32767, the sum
    // < 2^31) -- and it is within eps_q quanta of the exact distance times qscale (each axis' two
    // roundings <= 1 quantum together: sqrt(2) < eps_q).  Candidates within 2 eps_q of the coarse
    // minimum include every exact-minimum node, and the exact f64 CPython hypot decides among them.
    const double qlo = fmin(fmin(0.0, fmin(sx0, sy0)), fmin(gx, gy));
    const double qhi = fmax(fmax(fmax(P.x_range, P.y_range), fmax(sx0, sy0)), fmax(gx, gy));
    constexpr double kQ = 32767.0;
    const double qscale = kQ / (qhi - qlo);
    auto qenc = [&](double x, double y) -> uint32_t {
        const double ux = fmin(fmax(rint((x - qlo) * qscale), 0.0), kQ);
        const double uy = fmin(fmax(rint((y - qlo) * qscale), 0.0), kQ);
        return (uint32_t)ux | ((uint32_t)uy << 16);
    };
    if (tid == 0) {
        tx[0] = sx0; tx[1] = sy0; tg[0] = 0.0; tpar[0] = 0;
        xq_store(0, qenc(sx0, sy0));
    }
    __syncthreads();
    const double lox = delta, rgx = (P.x_range - delta) - delta;
    const double loy = delta, rgy = (P.y_range - delta) - delta;
    // |coarse distance - exact distance * qscale| <= sqrt(2) (+ the f64 rounding of the quantiser)
    constexpr double eps_q = 1.5;
    // a coarse threshold: squared quanta of (a distance r in map units plus e quanta), its integer
    // part (d2 <= floor(t) for an integer d2)
    auto qthr = [&](double r, double e) -> uint32_t {
        const double t = r * qscale + e;
        const double t2 = t * t;
        return t2 >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t2;
    };
    int n = 1, status = 1;
    int64_t cur = 0;
    int64_t c_iter = 0, c_scan = 0, c_cand = 0, c_tests = 0;  // iterations, nodes scanned, in-radius, collision tests
#ifdef PMP_RRT_STAMPS
    // dev build (tools/rrt_time.py): the counters become s_memtime ticks (>> 6) summed per phase, two
    // phases per counter (low / high 32 bits) -- nearest scan + min, band + argmin, steer + collision,
    // in-radius scan, first tests, choose-parent, rewire decisions + tests, insert + goal test
    // PMP_RRT_STAMPS=2: finer phases -- nearest scan loop, its top-2 reduction, band + publish, steer +
    // collision, in-radius scan (staging), hit resolution, tests + choose + rewire, insert + goal
    uint64_t cy[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tq = 0;
#if PMP_RRT_STAMPS == 2
    constexpr int kRemap[8] = {1, 2, 3, 5, 6, 6, 6, 7};
#define RSTAMP(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); cy[kRemap[k]] += t_ - tq; tq = t_; } while (0)
#define RSTAMPF(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); cy[k] += t_ - tq; tq = t_; } while (0)
#else
#define RSTAMP(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); cy[k] += t_ - tq; tq = t_; } while (0)
#define RSTAMPF(k) do {} while (0)
#endif
#define RSTAMP_START() do { tq = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define RSTAMP(k) do {} while (0)
#define RSTAMPF(k) do {} while (0)
#define RSTAMP_START() do {} while (0)
#endif

    int64_t rb0 = 0, rb1 = 0;  // staged window [rb0, rb1) of the random stream
    for (int it = 0; it < P.sample_num; it++) {
        if (cur + 3 > A.stride) { status = PMP_CAP_OVERFLOW; break; }
        if (cur + 3 > rb1) {
            __syncthreads();
            rb0 = cur;
            rb1 = rb0 + kRnd < A.stride ? rb0 + kRnd : A.stride;
            for (int i = tid; i < (int)(rb1 - rb0); i += kNT) S.rbuf[i] = rnd[rb0 + i];
            __syncthreads();
        }
        double sx = gx, sy = gy;
        if (S.rbuf[cur++ - rb0] > P.goal_sample_rate) {
            sx = lox + rgx * S.rbuf[cur++ - rb0];
            sy = loy + rgy * S.rbuf[cur++ - rb0];
        }
        c_iter++;
        c_scan += n;
        if (tid == 0) S.nH = 0;  // (the staging of this iteration comes after a barrier)
        RSTAMP_START();
        // ---- 2. nearest ----
        const uint32_t qs = qenc(sx, sy);  // the sample, quantised (one distance formula, cd2, for every pass)
        // each thread's minimum, its first index and its second-smallest distance: the band below
        // holds only the thread's first minimum unless the second one is in it too (then the thread
        // re-scans its nodes), so the common case needs no second pass over the tree
        uint32_t best = 0xFFFFFFFFu, second = 0xFFFFFFFFu;
        int bj = 0;
        auto take = [&](uint32_t d, int j) {
            const bool lt = d < best;  // strict: increasing j keeps the first
            second = min(second, max(best, d));  // lt: the old best; else min(second, d)
            bj = lt ? j : bj;
            best = min(best, d);
        };
        const int nl = n < lcap ? n : lcap;
        {
            // 8 loads in flight per thread, the LDS part then the HBM part (L2/MALL latency), in
            // increasing j
            int j = tid;
            for (; j + 7 * kNT < nl; j += 8 * kNT) {
                uint32_t p[8];
#pragma unroll
                for (int u = 0; u < 8; u++) p[u] = xl[j + u * kNT];
#pragma unroll
                for (int u = 0; u < 8; u++) take(cd2(p[u], qs), j + u * kNT);
            }
            for (; j < nl; j += kNT) take(cd2(xl[j], qs), j);
            j = lcap + tid;
            for (; j + 7 * kNT < n; j += 8 * kNT) {
                uint32_t p[8];
#pragma unroll
                for (int u = 0; u < 8; u++) p[u] = xyq[j + u * kNT];
#pragma unroll
                for (int u = 0; u < 8; u++) take(cd2(p[u], qs), j + u * kNT);
            }
            for (; j < n; j += kNT) take(cd2(xyq[j], qs), j);
        }
        RSTAMPF(0);
        // the exact coordinates of this thread's minimum, loaded ahead of the block minimum (RRT: its
        // owner publishes them; RRT*'s fused step has wave 0 load the minimum's, so these would only
        // hold the barrier below on an L2 round -- loaded in the rare band case instead)
        double bxj = 0.0, byj = 0.0, bgj = 0.0;
        if (!STAR) { bxj = tx[2 * bj]; byj = tx[2 * bj + 1]; bgj = tg[bj]; }
        // block top-2 of the threads' f32 distances (each thread's minimum and second) and the
        // minimum's index: when nothing but the minimum lies in the band the minimum is the nearest
        // node (the band's exact re-evaluation has one candidate) and its owner publishes it
        uint32_t m, b2;
        int im;
        {
            uint32_t ta = best, tb = second;
            int ti = bj;
            wave_top2(ta, tb, ti);
            if ((tid & 63) == 0) { S.t2a[tid >> 6] = ta; S.t2b[tid >> 6] = tb; S.t2i[tid >> 6] = ti; }
            __syncthreads();
            m = S.t2a[0]; b2 = S.t2b[0]; im = S.t2i[0];
            for (int w = 1; w < kWaves; w++) {
                const uint32_t oa = S.t2a[w], ob = S.t2b[w];
                const int oi = S.t2i[w];
                const uint32_t hi2 = oa < m ? m : oa;
                b2 = hi2 < b2 ? hi2 : b2;
                b2 = ob < b2 ? ob : b2;
                if (oa < m || (oa == m && oi < im)) { m = oa; im = oi; }
            }
        }
        RSTAMP(0);
        const uint32_t T = qthr(sqrt((double)m) / qscale, 2.0 * eps_q);
        int hi = 0x7fffffff;
        double nx0, ny0, gnear, nx, ny, G0;
        bool staged = false;  // the in-radius coarse hits are staged already (the fused step)
        if (STAR && !(b2 <= T)) {
            // RRT*, one candidate: wave 0 loads the nearest node's exact coordinates (one L2 round),
            // steers and tests the segment (isCollision(node_new, node_near) on one wave, its bins),
            // while the other waves stage the in-radius coarse hits of every node_new within max_dist
            // of that node -- around its coarse position with the margin max_dist + 4 eps, a superset
            // of the exact radius test that resolves them below (round 6)
            if ((tid >> 6) == 0) {
                const double ex = tx[2 * im], ey = tx[2 * im + 1], eg = tg[im];
                int fl = 0;
                double fnx = 0.0, fny = 0.0, fG0 = 0.0;
                if (lp::py_hypot(ex - sx, ey - sy) == 0.0) {
                    fl = 1;  // node_rand.current already in sample_list
                } else {
                    double dist = lp::py_hypot(sx - ex, sy - ey);
                    const double theta = atan2(sy - ey, sx - ex);
                    if (P.max_dist < dist) dist = P.max_dist;
                    double st, ct;
                    sincos(theta, &st, &ct);  // one range reduction; the same bits as cos / sin (tools/sincos_check.hip)
                    fnx = ex + dist * ct;
                    fny = ey + dist * st;
                    fG0 = eg + dist;
                    if (collision_wave(S, nr, nc, nb, delta, fnx, fny, ex, ey)) fl = 2;
                }
                if ((tid & 63) == 0) {
                    S.nearx = ex; S.neary = ey; S.nearg = eg;
                    S.newx = fnx; S.newy = fny; S.newG = fG0; S.fflag = fl;
                }
            } else {
                const uint32_t pn = im < lcap ? xl[im] : xyq[im];
                const uint32_t Trn = qthr(P.radius + P.max_dist, eps_q + 0.01);
                constexpr int kST = kNT - 64;  // the staging threads
                for (int j0 = tid - 64; j0 < n; j0 += 8 * kST) {
                    uint32_t p[8];
                    if (j0 + 7 * kST < nl) {
#pragma unroll
                        for (int u = 0; u < 8; u++) p[u] = xl[j0 + u * kST];
                    } else {
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            const int j = j0 + u * kST;
                            p[u] = 0u;
                            if (j < nl) p[u] = xl[j];
                            else if (j < n) p[u] = xyq[j];
                        }
                    }
                    uint32_t hits = 0;
#pragma unroll
                    for (int u = 0; u < 8; u++) hits |= (uint32_t)((j0 + u * kST < n) & (cd2(p[u], pn) <= Trn)) << u;
                    for (; hits; hits &= hits - 1) {
                        const int h = atomicAdd(&S.nH, 1);
                        if (h < kMaxH) S.hj[h] = j0 + (__ffs(hits) - 1) * kST;
                    }
                }
            }
            __syncthreads();
            const int fl = S.fflag;
            if (fl == 1) continue;
            c_tests++;
            if (fl == 2) { RSTAMP(2); continue; }
            hi = im;
            nx0 = S.nearx; ny0 = S.neary; gnear = S.nearg;
            nx = S.newx; ny = S.newy; G0 = S.newG;
            staged = true;
        } else {
            if (!(b2 <= T)) {
                // one candidate: the minimum's owner publishes it (the exact distance only for the
                // sample-already-in-the-tree test; steering recomputes it)
                if (best == m && bj == im) {
                    S.nearx = bxj; S.neary = byj; S.nearg = bgj;
                    S.nearh = lp::py_hypot(bxj - sx, byj - sy);
                }
                __syncthreads();
                hi = im;
                if (S.nearh == 0.0) continue;  // node_rand.current already in sample_list
            } else {
                if (STAR) { bxj = tx[2 * bj]; byj = tx[2 * bj + 1]; bgj = tg[bj]; }
                double h = INFINITY, hx = 0.0, hy = 0.0, hg = 0.0;
                if (best <= T && !(second <= T)) {
                    h = lp::py_hypot(bxj - sx, byj - sy);
                    hi = bj; hx = bxj; hy = byj; hg = bgj;
                } else if (best <= T) {
                    // increasing j within the thread (the LDS part, then the HBM part): equal distances keep
                    // the first.  Separate loops: a select between an LDS and a global load per element
                    // would issue both.  8 loads in flight per thread, the hits of a chunk in increasing j
                    auto hit = [&](int j) {
                        const double xj = tx[2 * j], yj = tx[2 * j + 1], gj = tg[j];  // one round
                        const double e = lp::py_hypot(xj - sx, yj - sy);
                        if (e < h) { h = e; hi = j; hx = xj; hy = yj; hg = gj; }  // increasing j: keeps the first
                    };
                    for (int j0 = tid; j0 < nl; j0 += 8 * kNT) {
                        uint32_t p[8];
    #pragma unroll
                        for (int u = 0; u < 8; u++) p[u] = (j0 + u * kNT < nl) ? xl[j0 + u * kNT] : 0u;
                        uint32_t hits = 0;
    #pragma unroll
                        for (int u = 0; u < 8; u++) hits |= (uint32_t)((j0 + u * kNT < nl) & (cd2(p[u], qs) <= T)) << u;
                        for (; hits; hits &= hits - 1) hit(j0 + (__ffs(hits) - 1) * kNT);
                    }
                    for (int j0 = lcap + tid; j0 < n; j0 += 8 * kNT) {
                        uint32_t p[8];
    #pragma unroll
                        for (int u = 0; u < 8; u++) p[u] = (j0 + u * kNT < n) ? xyq[j0 + u * kNT] : 0u;
                        uint32_t hits = 0;
    #pragma unroll
                        for (int u = 0; u < 8; u++) hits |= (uint32_t)((j0 + u * kNT < n) & (cd2(p[u], qs) <= T)) << u;
                        for (; hits; hits &= hits - 1) hit(j0 + (__ffs(hits) - 1) * kNT);
                    }
                }
                const int my_hi = hi;
                block_min_di(h, hi, S);
                if (h == 0.0) continue;  // node_rand.current already in sample_list
                if (my_hi == hi) { S.nearx = hx; S.neary = hy; S.nearg = hg; }  // the owner publishes the node
                __syncthreads();
            }
            nx0 = S.nearx; ny0 = S.neary; gnear = S.nearg;
            RSTAMP(1);
            // ---- 3. steer + collision (rrt.py:121-129) ----
            double dist = lp::py_hypot(sx - nx0, sy - ny0);
            const double theta = atan2(sy - ny0, sx - nx0);
            if (P.max_dist < dist) dist = P.max_dist;
            double st, ct;
            sincos(theta, &st, &ct);
            nx = nx0 + dist * ct;
            ny = ny0 + dist * st;
            G0 = gnear + dist;
            c_tests++;
            if (collision_block(S, nr, nc, nb, delta, nx, ny, nx0, ny0)) { RSTAMP(2); continue; }
        }
        const int near = hi;
        RSTAMP(2);
        double G = G0;
        int parent = near;
        int slot = n;
        if (tid == 0) { S.nK = 0; S.nA = 0; S.nT = 0; S.nT2 = 0; S.slot = n; }
        __syncthreads();
        if (STAR) {
            const int wave = tid >> 6, lane = tid & 63;
            // ---- 4a. in-radius candidates; those with c_i < G0 queue for a collision test ----
            const uint32_t qn = qenc(nx, ny);
            const uint32_t Tr = qthr(P.radius, eps_q + 0.01);
            // node j's exact test: in the radius -> a K entry (and a T entry when c_j < G0)
            auto in_radius = [&](int j) {
                const double xj = tx[2 * j], yj = tx[2 * j + 1], gj = tg[j];  // one round
                if (xj == nx && yj == ny) atomicMin(&S.slot, j);
                const double d = lp::py_hypot(nx - xj, ny - yj);
                if (!(d < P.radius)) return;
                const int k = atomicAdd(&S.nK, 1);
                const int fl = (gj + d < G0) ? KF_A : 0;
                if (k < kMaxK) {
                    S.kj[k] = j; S.kf[k] = fl; S.kd[k] = d; S.kx[k] = xj; S.ky[k] = yj; S.kg[k] = gj;
                } else {
                    KEntry e;
                    e.j = j;
                    e.d = d;
                    e.flags = fl;
                    kl[k] = e;
                }
                if (fl & KF_A) {
                    const int t = atomicAdd(&S.nT, 1);
                    tset(S, tl, t, k, 0.0);
                }
            };
            // the obstacles any candidate -- node_new segment can meet (each lies in the box of the
            // radius disk around node_new): one mask for every test of 4b / 4c
            uint64_t olo = 0, ohi = 0;
            const bool om = bins_mask(S, nx - P.radius, ny - P.radius, nx + P.radius, ny + P.radius, olo, ohi);
            // the in-radius candidates (any order: the K list is order-free), the LDS part as 8-wide
            // chunks of the same loop body, the HBM part 8 loads in flight per thread
            for (int j0 = tid; !staged && j0 < n; j0 += 8 * kNT) {
                uint32_t p[8];
                if (j0 + 7 * kNT < nl) {
#pragma unroll
                    for (int u = 0; u < 8; u++) p[u] = xl[j0 + u * kNT];
                } else {
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int j = j0 + u * kNT;
                        p[u] = 0u;
                        if (j < nl) p[u] = xl[j];
                        else if (j < n) p[u] = xyq[j];
                    }
                }
                uint32_t hits = 0;
#pragma unroll
                for (int u = 0; u < 8; u++) hits |= (uint32_t)((j0 + u * kNT < n) & (cd2(p[u], qn) <= Tr)) << u;
              // a coarse hit is staged: its exact test waits for the scan's end, so the hits' node
              // loads go out in one round instead of one dependent round per chunk
              for (; hits; hits &= hits - 1) {
                const int h = atomicAdd(&S.nH, 1);
                if (h < kMaxH) S.hj[h] = j0 + (__ffs(hits) - 1) * kNT;
              }
            }
            if (!staged) __syncthreads();
            RSTAMPF(4);
            if (S.nH <= kMaxH) {
                for (int h = tid; h < S.nH; h += kNT) in_radius(S.hj[h]);
            } else {
                // more coarse hits than the stage holds (a dense ball): the whole scan again, each
                // hit tested where it is found
                for (int j0 = tid; j0 < n; j0 += 8 * kNT) {
                    uint32_t p[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int j = j0 + u * kNT;
                        p[u] = 0u;
                        if (j < nl) p[u] = xl[j];
                        else if (j < n) p[u] = xyq[j];
                    }
                    uint32_t hits = 0;
#pragma unroll
                    for (int u = 0; u < 8; u++) hits |= (uint32_t)((j0 + u * kNT < n) & (cd2(p[u], qn) <= Tr)) << u;
                    for (; hits; hits &= hits - 1) in_radius(j0 + (__ffs(hits) - 1) * kNT);
                }
            }
            __syncthreads();
            RSTAMP(3);
            const int nK = S.nK;
            const int nT = S.nT;
            slot = S.slot;
            c_cand += nK;
            c_scan += n;
            c_tests += nT;
            // ---- 4b. one wave per test: the collision-free improving set ----
            for (int t = wave; t < nT; t += kWaves) {
                const int k = tget_k(S, tl, t);
                const KRec e = kget(S, kl, tx, tg, k);
                if (collision_wave_o(S, nr, nc, nb, delta, e.x, e.y, nx, ny, om, olo, ohi)) continue;
                if (lane == 0) {
                    const int a = atomicAdd(&S.nA, 1);
                    aset(S, al, a, e.j, e.g + e.d);
                    kset_flags(S, kl, k, KF_A | KF_VALID);
                }
            }
            __threadfence_block();  // HBM list entries before the barrier
            __syncthreads();
            RSTAMP(4);
            const int nA = S.nA;
            // choose-parent: min (c, j) over the A list, reduced by every wave on its own (the list is
            // short), so no workgroup round
            double cb = INFINITY;
            int jb = 0x7fffffff;
            for (int a = lane; a < nA; a += 64) {
                const double c = aget_c(S, al, a);
                const int j = aget_j(S, al, a);
                if (c < cb || (c == cb && j < jb)) { cb = c; jb = j; }
            }
            wave_min_di(cb, jb);
            if (cb < G0) { G = cb; parent = jb; }
            RSTAMP(5);
            // ---- 4c. rewire decisions; untested candidates queue for a collision test ----
            for (int k = tid; k < nK; k += kNT) {
                const KRec e = kget(S, kl, tx, tg, k);
                double Gp = G0;
                for (int a = 0; a < nA; a++)
                    if (aget_j(S, al, a) < e.j) Gp = fmin(Gp, aget_c(S, al, a));
                const double gj = e.g;
                if ((e.fl & KF_VALID) && Gp > gj + e.d) continue;  // node_new re-parents here
                const double c2 = Gp + e.d;
                if (!(gj > c2)) continue;
                if (e.fl & KF_A) {
                    if (e.fl & KF_VALID) { tg[e.j] = c2; tpar[e.j] = slot; }
                    continue;
                }
                const int t = atomicAdd(&S.nT2, 1);
                tset(S, tl, t, k, Gp);
            }
            __threadfence_block();
            __syncthreads();
            const int nT2 = S.nT2;
            c_tests += nT2;
            for (int t = wave; t < nT2; t += kWaves) {
                const KRec e = kget(S, kl, tx, tg, tget_k(S, tl, t));
                if (collision_wave_o(S, nr, nc, nb, delta, e.x, e.y, nx, ny, om, olo, ohi)) continue;
                if (lane == 0) { tg[e.j] = tget_G(S, tl, t) + e.d; tpar[e.j] = slot; }
            }
            __syncthreads();  // rewires land before the insert below may overwrite a duplicate slot
        }
        RSTAMP(6);
        // ---- 5. insert + goal test (rrt.py:70-81) ----
        if (tid == 0) {
            tx[2 * slot] = nx; tx[2 * slot + 1] = ny; tg[slot] = G; tpar[slot] = parent;
            xq_store(slot, qenc(nx, ny));
        }
        if (slot == n) {
            if (n >= cap) { status = PMP_CAP_OVERFLOW; break; }
            n++;
        }
        __syncthreads();
        const double dg = lp::py_hypot(gx - nx, gy - ny);
        c_tests += dg <= P.max_dist;
        if (dg <= P.max_dist && !collision_block(S, nr, nc, nb, delta, nx, ny, gx, gy)) {
            if (n >= cap) { status = PMP_CAP_OVERFLOW; break; }
            if (tid == 0) {
                tx[2 * n] = gx; tx[2 * n + 1] = gy; tg[n] = G + lp::py_hypot(nx - gx, ny - gy); tpar[n] = slot;
                xq_store(n, qenc(gx, gy));
            }
            n++;
            status = PMP_FOUND;
            break;
        }
        RSTAMP(7);
    }
    __syncthreads();
    if (tid == 0) {
        A.n_nodes[q] = n;
        A.draws[q] = cur;
        if (A.counters) {
#ifdef PMP_RRT_STAMPS
            for (int k = 0; k < 4; k++)
                A.counters[4 * q + k] = (int64_t)(((cy[2 * k] >> 6) & 0xFFFFFFFFull) | ((cy[2 * k + 1] >> 6) << 32));
#else
            A.counters[4 * q] = c_iter;
            A.counters[4 * q + 1] = c_scan;
            A.counters[4 * q + 2] = c_cand;
            A.counters[4 * q + 3] = c_tests;
#endif
        }
        int plen = 0;
        double c = 0.0;
        if (status == PMP_FOUND) {
            c = tg[n - 1];
            // extractPath (rrt.py:133-151): goal -> start through parents
            int v = n - 1;
            bool reached = false;
            double* out = A.path + (size_t)q * A.path_cap * 2;
            for (int s = 0; s <= n; s++) {
                if (plen < A.path_cap) { out[2 * plen] = tx[2 * v]; out[2 * plen + 1] = tx[2 * v + 1]; }
                plen++;
                if (v == 0) { reached = true; break; }
                v = tpar[v];
            }
            if (!reached) status = PMP_REF_RAISES;  // parent cycle: the reference never terminates
            else if (plen > A.path_cap) status = PMP_PATH_OVERFLOW;
        }
        A.path_len[q] = plen;
        A.cost[q] = c;
        A.status[q] = status;
    }
}

}  // namespace

extern "C" int pmp_rrt_batch(pmp_ctx* ctx, void* stream, const pmp_rrt_params* p, const double* rect, int nr,
                             const double* circ, int nc, const double* bnd, int nb, const double* start_xy,
                             const double* goal_xy, int nq, const double* rnd, int64_t rnd_stride, int tree_cap,
                             double* tree_xy, double* tree_g, int32_t* tree_parent, int32_t* n_nodes, double* cost,
                             int32_t* path_len, double* path_xy, int path_cap, int64_t* draws, int32_t* status,
                             int64_t* counters)
{
    if (!ctx) return PMP_EINVAL;
    if (!p || nq < 0 || nr < 0 || nc < 0 || nb < 0 || nr > kMaxObs || nc > kMaxObs || nb > kMaxBnd)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_rrt_batch: bad params or obstacle counts (<= 256 rects, 256 circles, 8 boundary)");
    if (p->sample_num < 0 || tree_cap < 2 || rnd_stride < 1 || path_cap < 0 || !(p->delta >= 0) || !(p->max_dist >= 0))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_rrt_batch: bad sample_num / tree_cap / rnd_stride / path_cap");
    if (nq == 0) return PMP_OK;
    if ((nr && !rect) || (nc && !circ) || (nb && !bnd) || !start_xy || !goal_xy || !rnd || !tree_xy || !tree_g ||
        !tree_parent || !n_nodes || !cost || !path_len || (path_cap && !path_xy) || !draws || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_rrt_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    uint32_t* xyq = (uint32_t*)pmp_scratch(ctx, SCR_AUX0, sizeof(uint32_t) * (size_t)nq * tree_cap);
    KEntry* kl = (KEntry*)pmp_scratch(ctx, SCR_AUX1, sizeof(KEntry) * (size_t)nq * tree_cap);
    TEntry* tl = (TEntry*)pmp_scratch(ctx, SCR_AUX2, sizeof(TEntry) * (size_t)nq * tree_cap);
    AEntry* al = (AEntry*)pmp_scratch(ctx, SCR_AUX3, sizeof(AEntry) * (size_t)nq * tree_cap);
    if (!xyq || !kl || !tl || !al) return PMP_ENOMEM;
    // the coarse copy's LDS part: the workgroup's share of the CU's LDS (one workgroup per CU unless
    // pmp_set_resident_per_cu leaves room for more: several in flight) beside its static state
    // (ctx->resident_per_cu is shared with the one-wave planners, whose 16-32 per CU would leave an
    // RRT workgroup almost no tree in LDS: RRT honours at most kRrtMaxResident of it)
    int per = pmp_lds_share(ctx, 1);
    if (per > kRrtMaxResident) per = kRrtMaxResident;
    if (per < PMP_RRT_PERCU) per = PMP_RRT_PERCU;  // narrower workgroups: two per CU
    const long share = kLdsBytes / per;
    const int ob = obs_bytes(nr, nc, nb);
    int lcap = (int)(std::max(0L, share - (long)sizeof(RrtShared) - ob - 512) / 4) & ~63;
    if (lcap > tree_cap) lcap = (tree_cap + 63) & ~63;
    RrtArgs A;
    A.P = *p;
    A.rect = rect; A.circ = circ; A.bnd = bnd;
    A.nr = nr; A.nc = nc; A.nb = nb;
    A.start = start_xy; A.goal = goal_xy; A.nq = nq;
    A.rnd = rnd; A.stride = rnd_stride; A.cap = tree_cap;
    A.txy = tree_xy; A.tg = tree_g; A.tpar = tree_parent; A.n_nodes = n_nodes;
    A.cost = cost; A.path_len = path_len; A.path = path_xy; A.path_cap = path_cap;
    A.draws = draws; A.status = status; A.counters = counters; A.xyq = xyq; A.klist = kl;
    A.tlist = tl; A.alist = al; A.lcap = lcap;
    const size_t dyn = (size_t)ob + (size_t)lcap * 4;
    if (p->star)
        hipLaunchKernelGGL(rrt_kernel<true>, dim3(nq), dim3(kNT), dyn, (hipStream_t)stream, A);
    else
        hipLaunchKernelGGL(rrt_kernel<false>, dim3(nq), dim3(kNT), dyn, (hipStream_t)stream, A);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
