// Batched DWA control step for gfx950 (local_planner/dwa.py:72-212): one lane per (v, w) sample,
// H-step rollout, obstacle cost from an occupancy stencil, numpy-exact normalisation and scoring,
// first-index argmax, Robot.kinematic.  Three launch shapes (pmp_dwa_step_batch):
//  - fixed windows (nv, nw > 0), fewer agents than CUs: dwa_split_kernel, k workgroups per agent;
//  - fixed windows otherwise: the same kernel at k = 1 (LOCAL), one 1024-thread workgroup per agent;
//  - resolution-sized windows (the drop-in DWA.plan): dwa_kernel, 768 threads, every plan iteration
//    in one launch.
//
// Numerics follow the reference operation by operation (-ffp-contract=off):
//  - Robot.lookforward (agent.py:91-116): x' = x + (dt*cos th)*v, y' = y + (dt*sin th)*v,
//    th' = th + dt*w (the F@state + B@u products with 0/1 entries are exact).
//  - obstacle = min(min cdist(obstacles, traj), R): only cells with |dx|,|dy| <= R can be < R away,
//    so a stencil over the occupancy grid gives the same minimum; d = sqrt(dx*dx + dy*dy) as scipy.
//  - np.sum of a column = numpy pairwise summation (leaves of <= 128 with 8 accumulators, splits at
//    n/2 rounded down to a multiple of 8), evaluated as that exact tree.
//  - (eval_win @ factor)[:, 2] = fma(e4, vw, fma(e3, ow, fma(e2, hw, fma(e1, 0, e0*0)))) (OpenBLAS).
//  - sin/cos/atan2 are the device libm (<= 1 ulp from glibc); inside a sample's rollout cos/sin(th_k)
//    come from a rotation recurrence (within ~2e-14 of libm over H = 30 steps): trajectories agree
//    to ~1e-14 and decisions are checked tie-aware in the tests.
//  - the occupancy bitmap is staged in LDS when it fits (16 KiB).
#include "localplan.h"

namespace {

#ifndef PMP_DWA_THREADS
#define PMP_DWA_THREADS 768
#endif
constexpr int kThreads = PMP_DWA_THREADS;  // 12 waves per agent (3 per SIMD): <= 168 VGPRs, no scratch spills; 16 waves
                                           // spill to scratch, 8 hide less latency (tools/dwa_ab.sh)
constexpr int kMaxN = 4096;    // samples per step held in LDS
constexpr int kMaxLeaves = 128;

struct Linsp {  // np.linspace(a, b, n) (numpy/_core/function_base.py)
    double a, b, step, div, delta;
    int n;
};

__device__ inline Linsp make_linsp(double a, double b, int n)
{
    Linsp L;
    L.a = a;
    L.b = b;
    L.n = n;
    L.div = (double)(n - 1);
    L.delta = b - a;
    L.step = n > 1 ? L.delta / L.div : 0.0;
    return L;
}

__device__ inline double linsp_at(const Linsp& L, int i)
{
    if (L.n == 1) return L.a;
    if (i == L.n - 1) return L.b;
    return L.step == 0.0 ? ((double)i / L.div) * L.delta + L.a : (double)i * L.step + L.a;
}

typedef __attribute__((address_space(3))) uint32_t lds_w32;
constexpr int kOccLdsWords = 4096;  // grids up to 131072 cells keep their occupancy in LDS (16 KiB)
constexpr int kNibWords = 4096;     // SCHEME 3's nibble map: (W + 1) (H + 1) cells of 4 bits, <= 32768 cells

// The occupancy bits of cells (i, j0 .. j0 + n - 1) of one grid row (x-major: consecutive j are
// consecutive bits), n <= 32, all inside the grid: bit b of the result = cell (i, j0 + b).
template <class PTR>
__device__ inline uint32_t occ_run(PTR occ, int H, int i, int j0, int n)
{
    const uint32_t k = (uint32_t)i * (uint32_t)H + (uint32_t)j0;
    const uint32_t w = k >> 5, sh = k & 31u;
    uint32_t v = occ[w] >> sh;
    if (sh + (uint32_t)n > 32u) v |= occ[w + 1] << (32u - sh);
    return n >= 32 ? v : (v & ((1u << n) - 1u));
}

template <class PTR>
__device__ inline bool occ_at(PTR occ, int ox, int oy, int W, int H, int cx, int cy)
{
    const int i = cx - ox, j = cy - oy;
    if ((unsigned)i >= (unsigned)W || (unsigned)j >= (unsigned)H) return false;
    const uint32_t k = (uint32_t)i * (uint32_t)H + (uint32_t)j;
    return (occ[k >> 5] >> (k & 31)) & 1u;
}

// numpy's pairwise-sum leaf (n <= 128: eight accumulators r[j] over a[j], a[j + 8], ..., combined as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the tail; n < 8: a plain running sum) on
// eight lanes (an aligned 8-lane group, all lanes with the same a and n): lane j keeps
// accumulator r[j] (a[j], a[j + 8], ... in order: consecutive lanes read consecutive words, no LDS bank
// conflicts), the groups' shuffles combine ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) in that
// order, lane 0 adds the tail; the result is valid in lane j = 0
__device__ inline double pw_leaf8(const double* col, int lo, int n, int j)
{
    auto a = [&](int i) -> double { return col[lo + i]; };
    if (n < 8) {
        double res = 0.0;
        if (j == 0)
            for (int i = 0; i < n; i++) res += a(i);
        return res;
    }
    const int n8 = n - n % 8;
    double r = a(j);
#pragma unroll 8
    for (int i = 8; i < n8; i += 8) r += a(i + j);
    r = r + __shfl_down(r, 1, 8);  // even j: r[j] + r[j + 1]
    r = r + __shfl_down(r, 2, 8);  // j = 0, 4: (r[j] + r[j + 1]) + (r[j + 2] + r[j + 3])
    r = r + __shfl_down(r, 4, 8);  // j = 0: the two halves
    if (j == 0)
        for (int i = n8; i < n; i++) r += a(i);
    return r;
}

__device__ inline int pw_half(int n)
{
    int n2 = n / 2;
    return n2 - n2 % 8;
}

struct DwaShared {
    uint32_t occ[kOccLdsWords];      // the occupancy bitmap (when it fits)
    uint32_t nib[kNibWords];         // SCHEME 3's nibble map
    double col[3][kMaxN];            // heading, obstacle, velocity per sample
    double leafsum[3][kMaxLeaves];
    int leaf_lo[kMaxLeaves], leaf_n[kMaxLeaves];
    double redd[kThreads / 64];
    int redi[kThreads / 64];
    double sums[3];
    double sn0, cs0;                 // sin / cos of the agent's heading
    double pt[2], theta, kappa;
    int nleaves;
};

// numpy's pairwise tree for n <= kMaxN samples is at most kPwDepth splits deep (n > 128 splits at
// pw_half(n); checked over every n <= 4096), so both walks below are compile-time recursions that
// the compiler flattens into registers -- no per-lane stack arrays, no scratch memory.
constexpr int kPwDepth = 6;

// the leaves of the tree for [lo, lo + n), in left-to-right order
template <int D>
__device__ inline void pw_leaves(int lo, int n, int* leaf_lo, int* leaf_n, int& nl)
{
    if (D == 0 || n <= 128) {
        leaf_lo[nl] = lo;
        leaf_n[nl] = n;
        nl++;
        return;
    }
    if constexpr (D > 0) {
        const int n2 = pw_half(n);
        pw_leaves<D - 1>(lo, n2, leaf_lo, leaf_n, nl);
        pw_leaves<D - 1>(lo + n2, n - n2, leaf_lo, leaf_n, nl);
    }
}

// the tree's value from its leaf sums (left + right at every split, as numpy combines them)
template <int D>
__device__ inline double pw_combine(const double* leafsum, int n, int& leaf)
{
    if (D == 0 || n <= 128) return leafsum[leaf++];
    if constexpr (D > 0) {
        const int n2 = pw_half(n);
        const double l = pw_combine<D - 1>(leafsum, n2, leaf);
        const double r = pw_combine<D - 1>(leafsum, n - n2, leaf);
        return l + r;
    }
    return 0.0;
}

// One sample's H-step rollout (dwa.py:152-160 via Robot.lookforward) and the stencil's minimum
// squared obstacle distance along it.  min over cells of sqrt(d2) == sqrt(min d2): sqrt is monotone
// and correctly rounded, so one square root per sample (scipy cdist: d = sqrt(dx*dx + dy*dy), no fused
// multiply-add).  cos/sin of th_k by rotation (sd, cd = sin / cos(dt * w)): th_k = th_0 + k*(dt*w) up
// to the rounding of the running sum (which pass 3 recomputes exactly as the reference), so (cs, sn)
// stay within ~2e-14 of libm's cos/sin(th_k) over the horizon -- one sincos pair per sample.
template <bool OCC_LDS>
__device__ inline void rollout(const uint32_t* __restrict__ occ, const lds_w32* occl, int ox, int oy, int W, int H,
                               double R, double dt, int Hh, double x, double y, double sn, double cs, double sd,
                               double cd, double v, double& xo, double& yo, double& mind2o)
{
    double mind2 = INFINITY;
    for (int k = 0; k < Hh; k++) {
        const double nx = x + (dt * cs) * v, ny = y + (dt * sn) * v;
        const double ncs = cs * cd - sn * sd, nsn = sn * cd + cs * sd;
        cs = ncs;
        sn = nsn;
        x = nx;
        y = ny;
        const int x0 = (int)ceil(x - R), x1 = (int)floor(x + R);
        const int y0 = (int)ceil(y - R), y1 = (int)floor(y + R);
        // the stencil row by row: one bit run per row, distances only for its set bits (cells outside
        // the grid are not obstacles); rows of up to 32 cells per run, so any inflation radius is covered
        const int j0 = max(y0 - oy, 0), j1 = min(y1 - oy, H - 1);
        for (int jc = j0; jc <= j1; jc += 32)
            for (int cx = x0; cx <= x1; cx++) {
                const int i = cx - ox;
                if ((unsigned)i >= (unsigned)W) continue;
                const int nrun = min(32, j1 - jc + 1);
                uint32_t run = OCC_LDS ? occ_run(occl, H, i, jc, nrun) : occ_run(occ, H, i, jc, nrun);
                while (run) {
                    const int b = __ffs(run) - 1;
                    run &= run - 1;
                    const double dx = (double)cx - x, dy = (double)(oy + jc + b) - y;
                    const double d2 = dx * dx + dy * dy;
                    if (d2 < mind2) mind2 = d2;
                }
            }
    }
    xo = x;
    yo = y;
    mind2o = mind2;
}

// ---- small inflation radii (R < 2, the reference's default R = 1), occupancy in LDS -----------------
// The stencil [ceil(x - R), floor(x + R)] x [ceil(y - R), floor(y + R)] is then at most 3 x 3 cells:
// up to three columns (two unless x is within rounding of an integer), one run of <= 3 bits each (two
// words only when the run crosses one).  Two schemes:
//  - SCHEME 1 (R < 2): all six words in one LDS round (clamped addresses, masked results) instead of
//    one dependent round trip per column; the cells, and so the minimum, are rollout()'s.
//  - SCHEME 3 (R <= 1): any cell closer than R <= 1 to (x, y) is one of the four cells (fx + {0, 1},
//    fy + {0, 1}), fx, fy = floor(x, y), since |cx - x| < 1.  Cells of the box at distance >= R leave
//    min(sqrt(min d2), R) = R unchanged (dwa.py:164 caps at R), so this superset of the stencil's cells
//    gives the same obstacle term bit for bit.  A nibble map (four occupancy bits per (fx, fy), built in
//    LDS per launch) gives the four cells in one LDS read.
#ifndef PMP_DWA_ROLL_SPLIT
#define PMP_DWA_ROLL_SPLIT 3  // k-split parts (the rotation table costs a part more than it saves on 512 samples)
#endif
#ifndef PMP_DWA_ROLL_LOCAL
#define PMP_DWA_ROLL_LOCAL 4  // one 1024-thread workgroup per agent
#endif
#ifndef PMP_DWA_ROLL_PLAN
#define PMP_DWA_ROLL_PLAN 3  // dwa_kernel (resolution-sized windows, DWA.plan)
#endif

struct SmallStencil {
    const lds_w32* occ;
    const lds_w32* nib;  // SCHEME 3: nibble of (fx, fy) at index (fx + 1) (H + 1) + fy + 1, fx >= -1, fy >= -1
    int words;           // occupancy words (the last readable one: words - 1)
    int ox, oy, W, H;
    double R;
};

// SCHEME 3: the four cells' occupancy bits at (x, y) -- (fx, fy) clamped into the map and the bits
// masked when outside fx in [-1, W - 1], fy in [-1, H - 1] (none of the four cells is in the grid), so
// the read issues without a branch
struct Nib {
    uint32_t bits;
    int fx, fy;
};

// v_cvt_i32_f64 saturates out-of-range values (and gives 0 for NaN): the range test runs on integers
__device__ inline int cvt_sat_i32(double d)
{
    int r;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(d));
    return r;
}

__device__ inline Nib nib_lookup(const SmallStencil& T, double x, double y)
{
    // fx + 1 in [0, W], fy + 1 in [0, H] (unsigned compares; a saturated far-away coordinate fails them)
    const uint32_t ux = (uint32_t)cvt_sat_i32(floor(x)) - (uint32_t)(T.ox - 1);
    const uint32_t uy = (uint32_t)cvt_sat_i32(floor(y)) - (uint32_t)(T.oy - 1);
    const uint32_t in = (uint32_t)(ux <= (uint32_t)T.W) & (uint32_t)(uy <= (uint32_t)T.H);
    const uint32_t cx = in ? ux : 0u, cy = in ? uy : 0u;
    Nib n;
    n.fx = (int)cx - 1;
    n.fy = (int)cy - 1;
    const uint32_t q = cx * (uint32_t)(T.H + 1) + cy;
    n.bits = (T.nib[q >> 3] >> ((q & 7u) * 4u)) & (15u & (0u - in));
    return n;
}

__device__ inline void nib_min(const SmallStencil& T, Nib n, double x, double y, double& mind2)
{
    uint32_t nb = n.bits;
    while (nb) {
        const int b = __ffs(nb) - 1;
        nb &= nb - 1;
        const double dx = (double)(T.ox + n.fx + (b & 1)) - x, dy = (double)(T.oy + n.fy + (b >> 1)) - y;
        const double d2 = dx * dx + dy * dy;
        if (d2 < mind2) mind2 = d2;
    }
}

template <int SCHEME>
__device__ inline void stencil3(const SmallStencil& T, double x, double y, double& mind2)
{
    if constexpr (SCHEME >= 3) {
        nib_min(T, nib_lookup(T, x, y), x, y, mind2);
        return;
    }
    const int x0 = (int)ceil(x - T.R), x1 = (int)floor(x + T.R);
    const int y0 = (int)ceil(y - T.R), y1 = (int)floor(y + T.R);
    const int j0 = max(y0 - T.oy, 0), j1 = min(y1 - T.oy, T.H - 1);
    if (j0 > j1) return;
    const int nrun = j1 - j0 + 1;
    const uint32_t mask = (1u << nrun) - 1u;
    uint32_t run[3];
    if constexpr (SCHEME == 1) {
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = x0 + u - T.ox;
            const uint32_t ok = (uint32_t)(x0 + u <= x1) & (uint32_t)((unsigned)i < (unsigned)T.W);
            const uint32_t k = (uint32_t)min(max(i, 0), T.W - 1) * (uint32_t)T.H + (uint32_t)j0;
            const uint32_t w = k >> 5, w1 = min(w + 1u, (uint32_t)T.words - 1u);
            const uint64_t pair = ((uint64_t)T.occ[w1] << 32) | (uint64_t)T.occ[w];
            run[u] = (uint32_t)(pair >> (k & 31u)) & (mask & (0u - ok));
        }
    }
#pragma unroll
    for (int u = 0; u < 3; u++) {
        uint32_t r = run[u];
        while (r) {
            const int b = __ffs(r) - 1;
            r &= r - 1;
            const double dx = (double)(x0 + u) - x, dy = (double)(T.oy + j0 + b) - y;
            const double d2 = dx * dx + dy * dy;
            if (d2 < mind2) mind2 = d2;
        }
    }
}

// rollout() for R < 2: the same trajectory recurrence and cells
#ifndef PMP_DWA_PAIR
#define PMP_DWA_PAIR 1
#endif
#ifndef PMP_DWA_COLPAIR
#define PMP_DWA_COLPAIR 1
#endif
template <int SCHEME, bool PAIR = PMP_DWA_PAIR>
__device__ inline void rollout_small(const SmallStencil& T, double dt, int Hh, double x, double y, double sn,
                                     double cs, double sd, double cd, double v, double& xo, double& yo,
                                     double& mind2o)
{
    double mind2 = INFINITY;
    auto advance = [&]() {
        const double nx = x + (dt * cs) * v, ny = y + (dt * sn) * v;
        const double ncs = cs * cd - sn * sd, nsn = sn * cd + cs * sd;
        cs = ncs;
        sn = nsn;
        x = nx;
        y = ny;
    };
    int k = 0;
    if constexpr (SCHEME == 3 && PAIR) {
        // two steps per round: both lookups' LDS reads in flight together, one branch for the (rare) hits
        for (; k + 1 < Hh; k += 2) {
            advance();
            const double xa = x, ya = y;
            advance();
            const Nib na = nib_lookup(T, xa, ya), nb = nib_lookup(T, x, y);
            if (na.bits | nb.bits) {
                nib_min(T, na, xa, ya, mind2);
                nib_min(T, nb, x, y, mind2);
            }
        }
    }
    for (; k < Hh; k++) {
        advance();
        stencil3<SCHEME>(T, x, y, mind2);
    }
    xo = x;
    yo = y;
    mind2o = mind2;
}

// SCHEME 4 = SCHEME 3 with the rotation precomputed: a sample's heading sequence th_k depends only on
// its w, so (dt cos th_k, dt sin th_k) -- the rotation recurrence of rollout(), started from sincos(th0)
// with sincos(dt w), the same operations in the same order -- is tabulated once per w index in LDS
// (rot[k][iw], built by one thread per w), and each step of a rollout reads its pair: x + (dt cs) v
// with the same (dt cs) bits, one sincos per w instead of one per sample, 4 instead of 12 f64
// operations per step
constexpr int kRotMax = 2048;  // nw x Hh pairs (C4: 64 x 30)

__device__ inline void build_rot(double* rot, const Linsp& LW, int nw, int Hh, double dt, double th0, int tid, int nt)
{
    double sn0, cs0;
    sincos(th0, &sn0, &cs0);
    for (int iw = tid; iw < nw; iw += nt) {
        double sd, cd;
        sincos(dt * linsp_at(LW, iw), &sd, &cd);
        double cs = cs0, sn = sn0;
        double2* r = reinterpret_cast<double2*>(rot) + iw;
        for (int k = 0; k < Hh; k++) {
            r[k * nw] = make_double2(dt * cs, dt * sn);
            const double ncs = cs * cd - sn * sd, nsn = sn * cd + cs * sd;
            cs = ncs;
            sn = nsn;
        }
    }
}

__device__ inline void rollout_rot(const SmallStencil& T, const double* rot, int nw, int iw, int Hh, double x, double y,
                                   double v, double& xo, double& yo, double& mind2o)
{
    double mind2 = INFINITY;
    const double2* r = reinterpret_cast<const double2*>(rot) + iw;
    int k = 0;
    for (; k + 1 < Hh; k += 2) {  // two steps per round, as rollout_small
        const double2 a = r[k * nw], b = r[(k + 1) * nw];
        const double xa = x + a.x * v, ya = y + a.y * v;
        x = xa + b.x * v;
        y = ya + b.y * v;
        const Nib na = nib_lookup(T, xa, ya), nb = nib_lookup(T, x, y);
        if (na.bits | nb.bits) {
            nib_min(T, na, xa, ya, mind2);
            nib_min(T, nb, x, y, mind2);
        }
    }
    for (; k < Hh; k++) {
        const double2 a = r[k * nw];
        x = x + a.x * v;
        y = y + a.y * v;
        nib_min(T, nib_lookup(T, x, y), x, y, mind2);
    }
    xo = x;
    yo = y;
    mind2o = mind2;
}

__device__ inline SmallStencil small_stencil(const lds_w32* occl, const lds_w32* nib, int ox, int oy, int W, int H,
                                             double R)
{
    SmallStencil T;
    T.occ = occl;
    T.nib = nib;
    T.words = (int)(((size_t)W * H + 31) / 32);
    T.ox = ox;
    T.oy = oy;
    T.W = W;
    T.H = H;
    T.R = R;
    return T;
}

// SCHEME 3's nibble map from the occupancy in LDS (all threads; the caller barriers before and after)
__device__ inline void build_nib(const SmallStencil& T, lds_w32* nib, int tid, int nt)
{
    const int Hn = T.H + 1, ncell = (T.W + 1) * Hn;
    auto bit = [&](int i, int j) -> uint32_t {
        return ((unsigned)i < (unsigned)T.W && (unsigned)j < (unsigned)T.H) ? occ_at(T.occ, 0, 0, T.W, T.H, i, j) : 0u;
    };
    // rows j0 .. j0 + 8 of column i as bits 0 .. 8 (cells outside the grid: 0)
    auto col9 = [&](int i, int j0) -> uint32_t {
        if ((unsigned)i >= (unsigned)T.W) return 0u;
        const int lo = max(j0, 0), hi = min(j0 + 9, T.H);
        return hi > lo ? occ_run(T.occ, T.H, i, lo, hi - lo) << (lo - j0) : 0u;
    };
    for (int w = tid; w < (ncell + 7) / 8; w += nt) {
        uint32_t v = 0;
        const int q0 = 8 * w, fx = q0 / Hn - 1, fy = q0 % Hn - 1;
        if (q0 % Hn + 8 <= Hn && q0 + 8 <= ncell) {
            // the word's eight cells share fx: two column runs give all their bits
            const uint32_t A = col9(fx, fy), Bc = col9(fx + 1, fy);
            for (int e = 0; e < 8; e++)
                v |= (((A >> e) & 1u) | ((Bc >> e) & 1u) << 1 | ((A >> (e + 1)) & 1u) << 2 | ((Bc >> (e + 1)) & 1u) << 3)
                     << (4 * e);
            nib[w] = v;
            continue;
        }
        for (int e = 0; e < 8; e++) {
            const int q = 8 * w + e;
            if (q >= ncell) break;
            const int fx = q / Hn - 1, fy = q % Hn - 1;
            v |= (bit(fx, fy) | bit(fx + 1, fy) << 1 | bit(fx, fy + 1) << 2 | bit(fx + 1, fy + 1) << 3) << (4 * e);
        }
        nib[w] = v;
    }
}

// the host's choice of stencil scheme for a kernel built with `want` (0: rollout()); 3 becomes 4 (the
// rotation table) where the caller's fixed window fits kRotMax
int small_scheme(int want, int W, int H, double R, bool occ_lds, long rot_pairs = -1)
{
    if (want == 4) {
        const int s3 = small_scheme(3, W, H, R, occ_lds);
        return s3 == 3 && rot_pairs >= 0 && rot_pairs <= kRotMax ? 4 : s3;
    }
    if (want == 0 || !occ_lds || !(R >= 0.0) || (long)W * H <= 0) return 0;
    if (want == 3 && R <= 1.0 && ((long)(W + 1) * (H + 1) + 7) / 8 <= (long)kNibWords) return 3;
    return R < 2.0 ? 1 : 0;
}

template <bool OCC_LDS, int SCHEME>
__global__ __launch_bounds__(kThreads) void dwa_kernel(
    const uint32_t* __restrict__ occ, int ox, int oy, int W, int H, pmp_lp_params P, pmp_dwa_params D, int na,
    double* __restrict__ state, const double* __restrict__ goal, const double* __restrict__ path_xy,
    const int32_t* __restrict__ path_off, int iters, double* __restrict__ u_out, int32_t* __restrict__ best_out,
    int32_t* __restrict__ status_out, int32_t* __restrict__ nsteps_out, double* __restrict__ hist_pose,
    double* __restrict__ eval_out, double* __restrict__ best_traj)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    DwaShared& S = *reinterpret_cast<DwaShared*>(smem_raw);
    const int a = blockIdx.x;
    const int tid = threadIdx.x;
    if (a >= na) return;
    if (OCC_LDS) {
        const int words = (int)(((size_t)W * H + 31) / 32);
        for (int i = tid; i < words; i += kThreads) S.occ[i] = occ[i];
        __syncthreads();
    }
    const lds_w32* occl = (const lds_w32*)S.occ;
    const SmallStencil T = small_stencil(occl, (const lds_w32*)S.nib, ox, oy, W, H, D.inflation);
    if constexpr (OCC_LDS && SCHEME == 3) {
        build_nib(T, (lds_w32*)S.nib, tid, kThreads);
        __syncthreads();
    }
    const double* path = path_xy + 2 * (size_t)path_off[a];
    const int Pn = path_off[a + 1] - path_off[a];
    const double gl[3] = {goal[3 * a], goal[3 * a + 1], goal[3 * a + 2]};
    double st[5];
    for (int k = 0; k < 5; k++) st[k] = state[5 * a + k];
    const double dt = P.dt;
    const int Hh = (int)(D.predict_time / dt);
    const double R = D.inflation;
    int status = 0, steps = 0, best = 0;
    double u0 = st[3], u1 = st[4];

    for (int it = 0; it < iters; it++) {
        // reachGoal (dwa.py:77-78)
        if (lp::reach_goal(st, gl, P)) { status = PMP_FOUND + 1; break; }
        // getLookaheadPoint
        double pt[2] = {0, 0}, theta = 0, kappa = 0;
        const int ls = lp::lookahead_block(path, Pn, st[0], st[1], st[3], P, pt, &theta, &kappa, S.redd, S.redi);
        if (tid == 0) { S.pt[0] = pt[0]; S.pt[1] = pt[1]; }
        __syncthreads();
        if (ls) { status = PMP_REF_RAISES; break; }
        const double gx = S.pt[0], gy = S.pt[1];
        // calDynamicWin (dwa.py:111-135)
        const double vr0 = fmax(P.min_v, st[3] + P.min_v_inc * dt), vr1 = fmin(P.max_v, st[3] + P.max_v_inc * dt);
        const double vr2 = fmax(P.min_w, st[4] + P.min_w_inc * dt), vr3 = fmin(P.max_w, st[4] + P.max_w_inc * dt);
        const int nv = D.nv > 0 ? D.nv : (int)((vr1 - vr0) / D.v_resolution);
        const int nw = D.nw > 0 ? D.nw : (int)((vr3 - vr2) / D.w_resolution);
        const int N = nv * nw;
        if (nv <= 0 || nw <= 0 || N > kMaxN) { status = PMP_REF_RAISES; break; }
        const Linsp LV = make_linsp(vr0, vr1, nv), LW = make_linsp(vr2, vr3, nw);

        // evaluation (dwa.py:152-174) in three passes over the samples, one sample per thread per
        // round, so each pass carries only its own libm code (one pass with sincos, rollout and
        // atan2 together needs more registers than 16 waves per CU leave): (1) the rotation of one
        // step, sin / cos(dt * w) -> col[1], col[2]; (2) the H-step rollout -> end x, y and the
        // stencil's min d2 (a thread reads and rewrites only its own sample's slots);
        // (3) heading / obstacle / velocity.
        if (tid == 0) sincos(st[2], &S.sn0, &S.cs0);
        for (int c = tid; c < N; c += kThreads) sincos(dt * linsp_at(LW, c % nw), &S.col[1][c], &S.col[2][c]);
        __syncthreads();
        const double sn0 = S.sn0, cs0 = S.cs0;
        for (int c = tid; c < N; c += kThreads) {
            double x, y, mind2;
            if constexpr (OCC_LDS && SCHEME == 3)
                rollout_small<3, false>(T, dt, Hh, st[0], st[1], sn0, cs0, S.col[1][c], S.col[2][c], linsp_at(LV, c / nw),
                                        x, y, mind2);  // (the paired form spills at this kernel's 168 VGPRs)
            else
                rollout<OCC_LDS>(occ, occl, ox, oy, W, H, R, dt, Hh, st[0], st[1], sn0, cs0, S.col[1][c], S.col[2][c],
                                 linsp_at(LV, c / nw), x, y, mind2);
            S.col[0][c] = x;
            S.col[1][c] = mind2;
            S.col[2][c] = y;
        }
        for (int c = tid; c < N; c += kThreads) {
            const double v = linsp_at(LV, c / nw), w = linsp_at(LW, c % nw);
            double th = st[2];
            for (int k = 0; k < Hh; k++) th = th + dt * w;
            const double ang = atan2(gy - S.col[2][c], gx - S.col[0][c]);
            S.col[0][c] = lp::kPi - fabs(ang - th);
            const double mind = sqrt(S.col[1][c]);
            S.col[1][c] = mind < R ? mind : R;
            S.col[2][c] = fabs(v);
        }
        // normalisation sums (dwa.py:176-181): numpy pairwise tree, leaves in parallel
        if (tid == 0) {
            int nl = 0;
            pw_leaves<kPwDepth>(0, N, S.leaf_lo, S.leaf_n, nl);
            S.nleaves = nl;
        }
        __syncthreads();
        const int nl = S.nleaves;
        for (int g = tid >> 3; g < 3 * nl; g += kThreads >> 3) {  // one 8-lane group per (column, leaf)
            const int cidx = g / nl, l = g % nl;
            const double ls = pw_leaf8(S.col[cidx], S.leaf_lo[l], S.leaf_n[l], tid & 7);
            if ((tid & 7) == 0) S.leafsum[cidx][l] = ls;
        }
        __syncthreads();
        if (tid < 3) {
            int leaf = 0;
            S.sums[tid] = 0.0 + pw_combine<kPwDepth>(S.leafsum[tid], N, leaf);
        }
        __syncthreads();
        const double s0 = S.sums[0], s1 = S.sums[1], s2 = S.sums[2];
        // scores and first-index argmax (dwa.py:183-190, :89)
        double bs = -INFINITY;
        int bi = 0x7fffffff;
        for (int c = tid; c < N; c += kThreads) {
            const double e0 = linsp_at(LV, c / nw), e1 = linsp_at(LW, c % nw);
            const double e2 = s0 != 0 ? S.col[0][c] / s0 : S.col[0][c];
            const double e3 = s1 != 0 ? S.col[1][c] / s1 : S.col[1][c];
            const double e4 = s2 != 0 ? S.col[2][c] / s2 : S.col[2][c];
            const double sc = fma(e4, D.velocity_weight, fma(e3, D.obstacle_weight, fma(e2, D.heading_weight, fma(e1, 0.0, e0 * 0.0))));
            if (eval_out && it == iters - 1) {
                double* e = eval_out + ((size_t)a * kMaxN + c) * 3;
                e[0] = fma(e4, 0.0, fma(e3, 0.0, fma(e2, 0.0, fma(e1, 0.0, e0 * 1.0))));
                e[1] = fma(e4, 0.0, fma(e3, 0.0, fma(e2, 0.0, fma(e1, 1.0, e0 * 0.0))));
                e[2] = sc;
            }
            if (sc > bs || bi == 0x7fffffff) { bs = sc; bi = c; }
        }
        lp::block_best<false>(bs, bi, S.redd, S.redi);
        best = bi;
        u0 = linsp_at(LV, best / nw);
        u1 = linsp_at(LW, best % nw);
        if (tid == 0 && hist_pose) {
            double* hp = hist_pose + ((size_t)a * iters + it) * 3;
            hp[0] = st[0]; hp[1] = st[1]; hp[2] = st[2];
        }
        if (tid == 0 && best_traj) {
            double x = st[0], y = st[1], th = st[2];
            for (int k = 0; k < Hh; k++) {
                double sn, cs;
                sincos(th, &sn, &cs);
                const double nx = x + (dt * cs) * u0, ny = y + (dt * sn) * u0, nth = th + dt * u1;
                x = nx; y = ny; th = nth;
                double* bt = best_traj + (((size_t)a * iters + it) * Hh + k) * 5;
                bt[0] = x; bt[1] = y; bt[2] = th; bt[3] = u0; bt[4] = u1;
            }
        }
        // Robot.kinematic(u, dt) (agent.py:68-89)
        {
            double sn, cs;
            sincos(st[2], &sn, &cs);
            const double nx = st[0] + (dt * cs) * u0, ny = st[1] + (dt * sn) * u0, nth = st[2] + dt * u1;
            st[0] = nx; st[1] = ny; st[2] = nth; st[3] = u0; st[4] = u1;
        }
        steps++;
    }
    if (tid == 0) {
        for (int k = 0; k < 5; k++) state[5 * a + k] = st[k];
        u_out[2 * a] = u0;
        u_out[2 * a + 1] = u1;
        best_out[a] = best;
        status_out[a] = status;
        nsteps_out[a] = steps;
    }
}

// ---- k-split: one agent's samples over k workgroups ------------------------------------------------
// With fewer agents than CUs (the 8-GPU strong split gives a rank 32 of C4's 256 agents) the kernel
// above keeps one CU per agent and the step time at one agent's latency.  Here part p of k workgroups
// takes the numpy pairwise tree's leaves [nl p / k, nl (p + 1) / k) of the agent's N samples (dwa.py:
// 176-181: leaves of <= 128 samples, splits at multiples of 8), evaluates them and stores their three
// columns and leaf sums; the part that arrives last (an agent-scope arrival counter) combines the leaf
// sums in the tree's own order -- the same tree, so the same bits as one workgroup -- then scores all N
// samples, takes the first-index argmax (dwa.py:89) and moves the robot.  One launch per plan
// iteration (the next iteration needs the moved state); an agent that stopped (goal reached, a
// reference raise) is skipped by later launches through its status.
constexpr int kSplitRoll = 512;                 // rollout threads (waves 0..7), one sample each
constexpr int kSplitThreads = kSplitRoll + 64;  // + the control wave: lookahead and leaf table beside them
constexpr int kSplitChunk = 1024;  // samples of one part held in LDS
// k = 1 (LOCAL): one 1024-thread workgroup per agent (16 waves, 4 per SIMD at <= 128 VGPRs), all N
// samples' columns in LDS, no hand-off; the last wave computes the lookahead before its rollouts
constexpr int kLocalThreads = 1024;
#ifndef PMP_DWA_LOCAL
#define PMP_DWA_LOCAL 1  // 0: fixed windows at k = 1 on dwa_kernel (A/B builds)
#endif

// part p's samples [c[p], c[p + 1]): the host's restatement of the tree's leaves (split_bounds)
struct DwaSplitBounds {
    int c[65];
};

template <int CHUNK, int NT>
struct DwaSplitShared {
    union {
        uint32_t occ[kOccLdsWords];
        double rot[2 * kRotMax];  // SCHEME 4, over the occupancy once the nibble map is built
    };
    uint32_t nib[kNibWords];
    double col[3][CHUNK];
    double lsum[3][kMaxLeaves];  // the last part: every part's leaf sums, staged for the combine
    int leaf_lo[kMaxLeaves], leaf_n[kMaxLeaves];
    double redd[NT / 64];
    int redi[NT / 64];
    double sums[3];
    double pt[2];
    int raises;
    int nleaves;
    int last;
};

// The parts' hand-off (cdna_hip_programming.md Guideline 16, publish / consume): every column and leaf
// sum another part reads is stored write-through (an agent-scope relaxed atomic store: `sc1`), each
// storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier and the arrival counter's
// relaxed atomic add, and the last part reads them with agent-scope loads (ld_coh below) -- no
// __threadfence(), whose L2 writeback (buffer_wbl2) flushed every dirty line of the XCD and cost
// ~40 us per arrival (PMP_DWA_STAMPS, round 5).
// ISA assumption (not the HIP memory model, which gives relaxed operations no happens-before): on
// gfx950 an agent-scope relaxed store is issued with sc1 (written through to the coherent point, the
// die's memory-side cache, past every XCD's L2) and an agent-scope relaxed load with sc1 (served from
// there, never from a stale line of the reader's L2 / L1); `s_waitcnt vmcnt(0)` before the arrival
// add orders the stores' completion ahead of the count.  Other targets would need a release on the
// counter add and an acquire on the last part's read; tests/test_dwa_gpu.py's bit-equality of every
// part count against one workgroup (test_split_parts_bit_equal) guards this on the hardware.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "dwa.hip's k-split hand-off relies on gfx950's sc1 write-through stores and coherent loads"
#endif
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ void st_wt(double* p, double v)
{
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The consumer side: agent-scope relaxed loads (sc1: served coherently, not from a stale line of
// this XCD's L2 or the CU's L1), issued after the arrival counter showed every part in -- in place of
// an acquire fence (its buffer_inv sc1 over the whole cache cost 48.5 vs 42.8 us per step, round 5).
__device__ __forceinline__ double ld_coh(const double* p)
{
    return __longlong_as_double((long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

struct DwaSplitScratch {
    double* cols;     // [na][3][kMaxN]
    double* leafsum;  // [na][3][kMaxLeaves]
    int* cnt;         // [na] arrivals of this launch (reset to 0 by the last part)
};

// PMP_DWA_STAMPS (dev builds, tools/dwa_split_probe.py): every part's tid 0 writes s_memtime at its
// phase boundaries into best_traj (as raw u64), 10 slots per workgroup
#ifdef PMP_DWA_STAMPS
#define DSTAMP(i) do { if (tid == 0 && best_traj) reinterpret_cast<unsigned long long*>(best_traj)[(size_t)blockIdx.x * 10 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DSTAMP(i) do {} while (0)
#endif
template <bool LOCAL>
using PartShared = DwaSplitShared<LOCAL ? kMaxN : kSplitChunk, LOCAL ? kLocalThreads : kSplitThreads>;

template <bool OCC_LDS, int SCHEME, bool LOCAL>
__global__ __launch_bounds__(LOCAL ? kLocalThreads : kSplitThreads) void dwa_split_kernel(
    const uint32_t* __restrict__ occ, int ox, int oy, int W, int H, pmp_lp_params P, pmp_dwa_params D, int na, int k,
    int it, int iters, double* __restrict__ state, const double* __restrict__ goal, const double* __restrict__ path_xy,
    const int32_t* __restrict__ path_off, double* __restrict__ u_out, int32_t* __restrict__ best_out,
    int32_t* __restrict__ status_out, int32_t* __restrict__ nsteps_out, double* __restrict__ hist_pose,
    double* __restrict__ eval_out, double* __restrict__ best_traj, DwaSplitScratch X, DwaSplitBounds B)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    PartShared<LOCAL>& S = *reinterpret_cast<PartShared<LOCAL>*>(smem_raw);
    const int a = blockIdx.x / k, part = blockIdx.x - a * k;
    const int tid = threadIdx.x, nt = blockDim.x;
    if (a >= na) return;
    DSTAMP(0);
    // every independent load of the step in one round: the stop status, the state, the path's offsets
    const int stp = it > 0 ? status_out[a] : 0;
    double st[5];
    for (int q = 0; q < 5; q++) st[q] = state[5 * a + q];
    const int po = path_off[a], Pn = path_off[a + 1] - po;
    if (stp != 0) return;  // stopped in an earlier iteration (block-uniform)
    // a stop in this iteration: part 0 records it (at it = 0 also the outputs of a plan that never moved)
    auto stop = [&](int status) {
        if (part == 0 && tid == 0) {
            status_out[a] = status;
            if (it == 0) {
                u_out[2 * a] = st[3];
                u_out[2 * a + 1] = st[4];
                best_out[a] = 0;
                nsteps_out[a] = 0;
            }
        }
    };
    if (lp::reach_goal(st, goal + 3 * a, P)) { stop(PMP_FOUND + 1); return; }
    if (OCC_LDS) {
        const int words = (int)(((size_t)W * H + 31) / 32);
        for (int i = tid; i < words; i += nt) S.occ[i] = occ[i];
    }
    const lds_w32* occl = (const lds_w32*)S.occ;
    const SmallStencil T = small_stencil(occl, (const lds_w32*)S.nib, ox, oy, W, H, D.inflation);
    constexpr bool small = OCC_LDS && SCHEME > 0;
    const double dt = P.dt;
    const int Hh = (int)(D.predict_time / dt);
    const double R = D.inflation;
    const int nv = D.nv, nw = D.nw;  // the host splits only windows of fixed size (nv, nw > 0)
    const int N = nv * nw;
    const double vr0 = fmax(P.min_v, st[3] + P.min_v_inc * dt), vr1 = fmin(P.max_v, st[3] + P.max_v_inc * dt);
    const double vr2 = fmax(P.min_w, st[4] + P.min_w_inc * dt), vr3 = fmin(P.max_w, st[4] + P.max_w_inc * dt);
    const Linsp LV = make_linsp(vr0, vr1, nv), LW = make_linsp(vr2, vr3, nw);
    const int c0 = B.c[part], c1 = B.c[part + 1];
    __syncthreads();  // the occupancy in LDS
    if constexpr (small && SCHEME >= 3) {
        build_nib(T, (lds_w32*)S.nib, tid, nt);
        __syncthreads();
    }
    if constexpr (small && SCHEME == 4) {
        build_rot(S.rot, LW, nw, Hh, dt, st[2], tid, nt);
        __syncthreads();
    }
    DSTAMP(1);
    // the rollouts (dwa.py:152-160) and their stencil minima, one sample per thread per round; they
    // need only the state, so the control wave's lookahead runs beside them
    auto rollouts = [&](int stride) {
        double sn0, cs0;
        sincos(st[2], &sn0, &cs0);
        int c = c0 + tid;
        if constexpr (small && SCHEME == 4) {
            for (; c < c1; c += stride) {
                double x, y, mind2;
                rollout_rot(T, S.rot, nw, c % nw, Hh, st[0], st[1], linsp_at(LV, c / nw), x, y, mind2);
                S.col[0][c - c0] = x;
                S.col[1][c - c0] = mind2;
                S.col[2][c - c0] = y;
            }
            return;
        }
        for (; c < c1; c += stride) {
            double sd, cd, x, y, mind2;
            sincos(dt * linsp_at(LW, c % nw), &sd, &cd);
            if constexpr (small)
                rollout_small<SCHEME>(T, dt, Hh, st[0], st[1], sn0, cs0, sd, cd, linsp_at(LV, c / nw), x, y, mind2);
            else
                rollout<OCC_LDS>(occ, occl, ox, oy, W, H, R, dt, Hh, st[0], st[1], sn0, cs0, sd, cd,
                                 linsp_at(LV, c / nw), x, y, mind2);
            S.col[0][c - c0] = x;
            S.col[1][c - c0] = mind2;
            S.col[2][c - c0] = y;
        }
    };
    // the control wave: getLookaheadPoint (local_planner.py:103-170, lp::lookahead_block's steps) with
    // wave-level first-index reductions, its serial tail on lane 0 and the pairwise tree's leaf table on
    // lane 1
    auto control = [&](int ln) {
        const double rx = st[0], ry = st[1];
        const double L = lp::lookahead_dist(st[3], P);
        const double* path = path_xy + 2 * (size_t)po;
        double bd = INFINITY;
        int bi = 0x7fffffff;
        for (int i = ln; i < Pn; i += 64) {
            const double d = lp::py_hypot(rx - path[2 * i], ry - path[2 * i + 1]);
            if (d < bd) { bd = d; bi = i; }  // strided in increasing i: keeps the first minimum
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double ov = __shfl_xor(bd, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ov < bd || (ov == bd && oi < bi)) { bd = ov; bi = oi; }
        }
        const int idx_closest = bi;
        int fi = 0x7fffffff;  // first i >= idx_closest with dist >= L
        for (int i = idx_closest + ln; i < Pn; i += 64)
            if (lp::py_hypot(rx - path[2 * i], ry - path[2 * i + 1]) >= L) { fi = i; break; }
        for (int o = 32; o > 0; o >>= 1) {
            const int oi = __shfl_xor(fi, o, 64);
            fi = oi < fi ? oi : fi;
        }
        if (ln == 0) {
            double pt[2] = {0, 0}, theta = 0, kappa = 0;
            S.raises = lp::lookahead_tail(path, Pn, rx, ry, L, fi == 0x7fffffff ? Pn - 1 : fi, pt, &theta, &kappa);
            S.pt[0] = pt[0];
            S.pt[1] = pt[1];
        } else if (ln == 1) {
            int nl = 0;
            pw_leaves<kPwDepth>(0, N, S.leaf_lo, S.leaf_n, nl);
            S.nleaves = nl;
        }
    };
    if constexpr (LOCAL) {
        // all 16 waves roll out (N / 1024 rounds each); the last one computes the lookahead first
        if (tid >= nt - 64) control(tid - (nt - 64));
        rollouts(nt);
    } else {
        if (tid < kSplitRoll) rollouts(kSplitRoll);
        else control(tid - kSplitRoll);
    }
    __syncthreads();
    DSTAMP(2);
    if (S.raises) { stop(PMP_REF_RAISES); return; }
    const double gx = S.pt[0], gy = S.pt[1];
    const int nl = S.nleaves;
    const int l0 = (int)(((long)nl * part) / k), l1 = (int)(((long)nl * (part + 1)) / k);
    double* cols = X.cols + (size_t)a * 3 * kMaxN;
    double* lsum = X.leafsum + (size_t)a * 3 * kMaxLeaves;
    // the heading / obstacle / velocity columns (dwa.py:166-174), two samples per thread per round: th
    // after Hh steps is a chain of Hh dependent additions (th + dt*w, the rollout's order), two chains
    // interleave
    auto column = [&](int c, double th) {
        const double ang = atan2(gy - S.col[2][c - c0], gx - S.col[0][c - c0]);
        const double h = lp::kPi - fabs(ang - th);
        const double mind = sqrt(S.col[1][c - c0]);
        const double o = mind < R ? mind : R;
        const double vel = fabs(linsp_at(LV, c / nw));
        S.col[0][c - c0] = h;
        S.col[1][c - c0] = o;
        S.col[2][c - c0] = vel;
        if constexpr (!LOCAL) {
            st_wt(cols + c, h);
            st_wt(cols + kMaxN + c, o);
            st_wt(cols + 2 * kMaxN + c, vel);
        }
    };
    for (int c = c0 + tid; c < c1; c += (1 + PMP_DWA_COLPAIR) * nt) {
        const int c2 = PMP_DWA_COLPAIR && c + nt < c1 ? c + nt : c;
        const double w = linsp_at(LW, c % nw), w2 = linsp_at(LW, c2 % nw);
        double th = st[2], th2 = st[2];
        for (int q = 0; q < Hh; q++) {
            th = th + dt * w;
            th2 = th2 + dt * w2;
        }
        column(c, th);
        if (PMP_DWA_COLPAIR && c + nt < c1) column(c2, th2);
    }
    DSTAMP(3);
    __syncthreads();
    {
        // one 8-lane group per (column, leaf); groups are wave-aligned and their loop bounds uniform
        const int ml = l1 - l0;
        for (int g = tid >> 3; g < 3 * ml; g += nt >> 3) {
            const int cidx = g / ml, l = l0 + g % ml;
            const double ls = pw_leaf8(S.col[cidx], S.leaf_lo[l] - c0, S.leaf_n[l], tid & 7);
            if ((tid & 7) == 0) {
                if constexpr (LOCAL) S.lsum[cidx][l] = ls;
                else st_wt(lsum + cidx * kMaxLeaves + l, ls);
            }
        }
    }
    DSTAMP(4);
    if constexpr (!LOCAL) {
        // arrival: every wave drains its write-through stores, then one lane counts the part in; the
        // last part reads the others' columns and leaf sums with agent-scope loads
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int old = __hip_atomic_fetch_add(X.cnt + a, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.last = old == k - 1;
        }
        __syncthreads();
        DSTAMP(5);
        if (!S.last) return;
        if (tid == 0) __hip_atomic_store(X.cnt + a, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the leaf sums into LDS in one round (all threads), then the tree's combine from LDS
        for (int i = tid; i < 3 * nl; i += nt) S.lsum[i / nl][i % nl] = ld_coh(lsum + (i / nl) * kMaxLeaves + i % nl);
    }
    __syncthreads();
    if (tid < 3) {
        int leaf = 0;
        S.sums[tid] = 0.0 + pw_combine<kPwDepth>(S.lsum[tid], N, leaf);
    }
    __syncthreads();
    const double s0 = S.sums[0], s1 = S.sums[1], s2 = S.sums[2];
    DSTAMP(6);
    double bs = -INFINITY;
    int bi = 0x7fffffff;
    // the other parts' columns come from L2 / HBM: a thread's loads issue together (8 samples x 3
    // columns in flight), then the scores, in increasing c (the first index wins a tie); LOCAL reads
    // its own columns from LDS
    constexpr int kU = LOCAL ? 1 : 8;
    const bool want_eval = eval_out && it == iters - 1;
    for (int c0 = tid; c0 < N; c0 += kU * nt) {
        double hv[kU], ov[kU], vv[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int c = c0 + u * nt;
            const int cc = c < N ? c : 0;
            if constexpr (LOCAL) {
                hv[u] = S.col[0][cc];
                ov[u] = S.col[1][cc];
                vv[u] = S.col[2][cc];
            } else {
                hv[u] = ld_coh(cols + cc);
                ov[u] = ld_coh(cols + kMaxN + cc);
                vv[u] = ld_coh(cols + 2 * kMaxN + cc);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
        const int c = c0 + u * nt;
        if (c >= N) break;
        const double h = hv[u], o = ov[u], vel = vv[u];
        const double e2 = s0 != 0 ? h / s0 : h;
        const double e3 = s1 != 0 ? o / s1 : o;
        const double e4 = s2 != 0 ? vel / s2 : vel;
        // the (v, w) terms enter the score times 0: +-0 for a finite window, which changes neither the
        // score's value nor any comparison, so they are evaluated only for the eval rows
        double e0 = 0.0, e1 = 0.0, z = 0.0;
        if (want_eval) {
            e0 = linsp_at(LV, c / nw);
            e1 = linsp_at(LW, c % nw);
            z = fma(e1, 0.0, e0 * 0.0);
        }
        const double sc = fma(e4, D.velocity_weight, fma(e3, D.obstacle_weight, fma(e2, D.heading_weight, z)));
        if (want_eval) {
            double* e = eval_out + ((size_t)a * kMaxN + c) * 3;
            e[0] = fma(e4, 0.0, fma(e3, 0.0, fma(e2, 0.0, fma(e1, 0.0, e0 * 1.0))));
            e[1] = fma(e4, 0.0, fma(e3, 0.0, fma(e2, 0.0, fma(e1, 1.0, e0 * 0.0))));
            e[2] = sc;
        }
        if (sc > bs || bi == 0x7fffffff) { bs = sc; bi = c; }
        }
    }
    lp::block_best<false>(bs, bi, S.redd, S.redi);
    DSTAMP(7);
    const int best = bi;
    const double u0 = linsp_at(LV, best / nw), u1 = linsp_at(LW, best % nw);
    if (tid == 0) {
        if (hist_pose) {
            double* hp = hist_pose + ((size_t)a * iters + it) * 3;
            hp[0] = st[0]; hp[1] = st[1]; hp[2] = st[2];
        }
#ifndef PMP_DWA_STAMPS
        if (best_traj) {
#else
        if (false) {
#endif
            double x = st[0], y = st[1], th = st[2];
            for (int q = 0; q < Hh; q++) {
                double sn, cs;
                sincos(th, &sn, &cs);
                const double nx = x + (dt * cs) * u0, ny = y + (dt * sn) * u0, nth = th + dt * u1;
                x = nx; y = ny; th = nth;
                double* bt = best_traj + (((size_t)a * iters + it) * Hh + q) * 5;
                bt[0] = x; bt[1] = y; bt[2] = th; bt[3] = u0; bt[4] = u1;
            }
        }
        // Robot.kinematic(u, dt) (agent.py:68-89)
        double sn, cs;
        sincos(st[2], &sn, &cs);
        const double nx = st[0] + (dt * cs) * u0, ny = st[1] + (dt * sn) * u0, nth = st[2] + dt * u1;
        state[5 * a + 0] = nx;
        state[5 * a + 1] = ny;
        state[5 * a + 2] = nth;
        state[5 * a + 3] = u0;
        state[5 * a + 4] = u1;
        u_out[2 * a] = u0;
        u_out[2 * a + 1] = u1;
        best_out[a] = best;
        status_out[a] = 0;
        nsteps_out[a] = (it == 0 ? 0 : nsteps_out[a]) + 1;
    }
    DSTAMP(8);
}

// host restatement of pw_leaves: part p of k takes leaves [nl p / k, nl (p + 1) / k), samples
// [c[p], c[p + 1]) (c has k + 1 entries)
void split_bounds(int n, int k, int* c)
{
    int lo[kMaxLeaves], len[kMaxLeaves], nl = 0;
    struct R {
        static void go(int d, int l, int m, int* lo, int* len, int& nl)
        {
            if (d == 0 || m <= 128) { lo[nl] = l; len[nl] = m; nl++; return; }
            const int m2 = (m / 2) - (m / 2) % 8;
            go(d - 1, l, m2, lo, len, nl);
            go(d - 1, l + m2, m - m2, lo, len, nl);
        }
    };
    R::go(kPwDepth, 0, n, lo, len, nl);
    for (int p = 0; p <= k; p++) {
        const int l = (int)(((long)nl * p) / k);
        c[p] = l < nl ? lo[l] : n;
    }
}

// the largest part of n samples over k parts (leaf-aligned)
int split_max_chunk(int n, int k)
{
    int lo[kMaxLeaves], len[kMaxLeaves], nl = 0;
    struct R {
        static void go(int d, int l, int m, int* lo, int* len, int& nl)
        {
            if (d == 0 || m <= 128) { lo[nl] = l; len[nl] = m; nl++; return; }
            const int m2 = (m / 2) - (m / 2) % 8;
            go(d - 1, l, m2, lo, len, nl);
            go(d - 1, l + m2, m - m2, lo, len, nl);
        }
    };
    R::go(kPwDepth, 0, n, lo, len, nl);
    int mx = 0;
    for (int p = 0; p < k; p++) {
        const int l0 = (int)(((long)nl * p) / k), l1 = (int)(((long)nl * (p + 1)) / k);
        const int c0 = l0 < nl ? lo[l0] : n, c1 = l1 < nl ? lo[l1] : n;
        mx = c1 - c0 > mx ? c1 - c0 : mx;
    }
    return k > nl ? kMaxN + 1 : mx;  // more parts than leaves: refused
}

}  // namespace

extern "C" int pmp_dwa_set_split(pmp_ctx* ctx, int parts)
{
    if (!ctx) return PMP_EINVAL;
    if (parts < 0 || parts > 64) return pmp_set_err(ctx, PMP_EINVAL, "pmp_dwa_set_split: parts must be 0 (auto) .. 64");
    ctx->dwa_split = parts;
    return PMP_OK;
}

extern "C" int pmp_dwa_step_batch(pmp_ctx* ctx, void* stream, const uint32_t* occ_bits, int ox, int oy, int W, int H,
                                  const pmp_lp_params* lp, const pmp_dwa_params* dp, int na, double* state,
                                  const double* goal, const double* path_xy, const int32_t* path_off, int iters,
                                  double* u, int32_t* best, int32_t* status, int32_t* n_steps, double* hist_pose,
                                  double* eval, double* best_traj)
{
    if (!ctx) return PMP_EINVAL;
    if (!lp || !dp || na < 0 || iters < 1 || W < 0 || H < 0)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dwa_step_batch: bad params/na/iters/dims");
    if (na == 0) return PMP_OK;
    if (!occ_bits || !state || !goal || !path_xy || !path_off || !u || !best || !status || !n_steps)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dwa_step_batch: null pointer argument");
    if (dp->nv * dp->nw > kMaxN || !(lp->dt > 0) || !(dp->predict_time >= 0))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_dwa_step_batch: nv*nw must be <= 4096 and dt > 0");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const bool occ_lds = ((size_t)W * H + 31) / 32 <= (size_t)kOccLdsWords;
    const long rot_pairs = dp->nw > 0 ? (long)dp->nw * (long)(int)(dp->predict_time / lp->dt) : -1;
    const int scheme_split = small_scheme(PMP_DWA_ROLL_SPLIT, W, H, dp->inflation, occ_lds, rot_pairs);
    const int scheme_local = small_scheme(PMP_DWA_ROLL_LOCAL, W, H, dp->inflation, occ_lds, rot_pairs);
    // parts per agent: auto (dwa_split 0) = the CUs over the agents, at most 16; 1 = one workgroup per
    // agent.  Only windows of fixed size (nv, nw > 0) split, into leaf-aligned parts of <= kSplitChunk.
    int k = 1;
    const bool fixed = dp->nv > 0 && dp->nw > 0;
    if (fixed && dp->nv * dp->nw > 1) {
        if (ctx->dwa_split > 0) {
            k = ctx->dwa_split;
        } else {
            if (!ctx->cus) PMP_HIP_CHECK(ctx, hipDeviceGetAttribute(&ctx->cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
            k = na < ctx->cus ? ctx->cus / na : 1;
            k = k > 16 ? 16 : (k < 1 ? 1 : k);
        }
        const int n = dp->nv * dp->nw;
        while (k > 1 && split_max_chunk(n, k) > kMaxN) k--;  // more parts than leaves
        while (k > 1 && k < 64 && split_max_chunk(n, k) > kSplitChunk) k++;
        if (k > 1 && split_max_chunk(n, k) > kSplitChunk) k = 1;
    }
    if (k > 1) {
        const size_t per = (size_t)3 * kMaxN * 8 + (size_t)3 * kMaxLeaves * 8;
        char* scr = (char*)pmp_scratch(ctx, SCR_DWA, (size_t)na * per + (size_t)na * 4 + 64);
        if (!scr) return PMP_ENOMEM;
        DwaSplitScratch X;
        X.cols = (double*)scr;
        X.leafsum = (double*)(scr + (size_t)na * 3 * kMaxN * 8);
        X.cnt = (int*)(scr + (size_t)na * per);
        // the counters are zero between launches (each agent's last part resets its own); a new buffer
        // or a new layout (the counters follow the na agents' columns) starts zeroed once
        if (ctx->dwa_zeroed != scr || ctx->dwa_zeroed_n != na) {
            PMP_HIP_CHECK(ctx, hipMemsetAsync(X.cnt, 0, (size_t)na * 4, (hipStream_t)stream));
            ctx->dwa_zeroed = scr;
            ctx->dwa_zeroed_n = na;
        }
        DwaSplitBounds Bd;
        split_bounds(dp->nv * dp->nw, k, Bd.c);
        auto sk = scheme_split == 4 ? dwa_split_kernel<true, 4, false>
                  : scheme_split == 3 ? dwa_split_kernel<true, 3, false>
                  : scheme_split == 1 ? dwa_split_kernel<true, 1, false>
                  : occ_lds           ? dwa_split_kernel<true, 0, false>
                                      : dwa_split_kernel<false, 0, false>;
        for (int it = 0; it < iters; it++)
            hipLaunchKernelGGL(sk, dim3((unsigned)(na * k)), dim3(kSplitThreads), sizeof(PartShared<false>),
                               (hipStream_t)stream, occ_bits, ox, oy, W, H, *lp, *dp, na, k, it, iters, state, goal,
                               path_xy, path_off, u, best, status, n_steps, hist_pose, eval, best_traj, X, Bd);
        PMP_HIP_CHECK(ctx, hipGetLastError());
        return PMP_OK;
    }
    if (PMP_DWA_LOCAL && fixed) {
        // one workgroup per agent, one launch per plan iteration (the k-split kernel at k = 1: no scratch,
        // no hand-off)
        DwaSplitScratch X = {nullptr, nullptr, nullptr};
        DwaSplitBounds Bd;
        Bd.c[0] = 0;
        Bd.c[1] = dp->nv * dp->nw;
        auto lk = scheme_local == 4 ? dwa_split_kernel<true, 4, true>
                  : scheme_local == 3 ? dwa_split_kernel<true, 3, true>
                  : scheme_local == 1 ? dwa_split_kernel<true, 1, true>
                  : occ_lds           ? dwa_split_kernel<true, 0, true>
                                      : dwa_split_kernel<false, 0, true>;
        for (int it = 0; it < iters; it++)
            hipLaunchKernelGGL(lk, dim3((unsigned)na), dim3(kLocalThreads), sizeof(PartShared<true>), (hipStream_t)stream,
                               occ_bits, ox, oy, W, H, *lp, *dp, na, 1, it, iters, state, goal, path_xy, path_off, u, best,
                               status, n_steps, hist_pose, eval, best_traj, X, Bd);
        PMP_HIP_CHECK(ctx, hipGetLastError());
        return PMP_OK;
    }
    const int scheme_plan = small_scheme(PMP_DWA_ROLL_PLAN, W, H, dp->inflation, occ_lds) == 3 ? 3 : 0;
    auto kern = scheme_plan == 3 ? dwa_kernel<true, 3> : occ_lds ? dwa_kernel<true, 0> : dwa_kernel<false, 0>;
    hipLaunchKernelGGL(kern, dim3(na), dim3(kThreads), sizeof(DwaShared), (hipStream_t)stream, occ_bits, ox, oy, W,
                       H, *lp, *dp, na, state, goal, path_xy, path_off, iters, u, best, status, n_steps, hist_pose, eval,
                       best_traj);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
