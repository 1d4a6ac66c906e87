// Device restatements shared by the local-planner kernels (dwa.hip, lqr.hip, mpc.hip):
// CPython math.hypot, LocalPlanner helpers (local_planner/local_planner.py:86-246) and
// MathHelper (utils/helper/math_helper.py:11-65).  Compiled with -ffp-contract=off: every
// operation rounds where the reference's CPython float arithmetic rounds.
#pragma once
#include "pmp_internal.h"

namespace lp {

constexpr double kPi = 3.141592653589793;  // math.pi / np.pi

// CPython 3.10 Modules/mathmodule.c vector_norm for two coordinates (math.hypot)
__device__ inline double py_hypot(double a, double b)
{
    const double T27 = 134217729.0;
    double v0 = fabs(a), v1 = fabs(b);
    double mx = 0.0;
    bool nan_ = isnan(v0) || isnan(v1);
    if (v0 > mx) mx = v0;
    if (v1 > mx) mx = v1;
    if (isinf(mx)) return mx;
    if (nan_) return __builtin_nan("");
    if (mx == 0.0) return mx;
    int e;
    frexp(mx, &e);
    double csum = 1.0, frac = 0.0, oldcsum, x, t, hi, lo, h;
    if (e >= -1023) {
        const double scale = ldexp(1.0, -e);
        const double vv[2] = {v0, v1};
        for (int i = 0; i < 2; i++) {
            x = vv[i] * scale;
            t = x * T27;
            hi = t - (t - x);
            lo = x - hi;
            x = hi * hi;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
            x = 2.0 * hi * lo;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
            x = lo * lo;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        }
        h = sqrt(csum - 1.0 + frac);
        x = h;
        t = x * T27;
        hi = t - (t - x);
        lo = x - hi;
        x = -hi * hi;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = -2.0 * hi * lo;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = -lo * lo;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = csum - 1.0 + frac;
        return (h + x / (2.0 * h)) / scale;
    }
    const double vv[2] = {v0, v1};
    for (int i = 0; i < 2; i++) {
        x = vv[i] / mx;
        x = x * x;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
    }
    return mx * sqrt(csum - 1.0 + frac);
}

__device__ inline double regularize_angle(double a) { return a - 2.0 * kPi * floor((a + kPi) / (2.0 * kPi)); }

__device__ inline double clampd(double v, double lo, double hi)
{
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return v;
}

// LocalPlanner.reachGoal (local_planner.py:233-246)
__device__ inline bool reach_goal(const double* cur, const double* goal, const pmp_lp_params& P)
{
    const double e_theta = regularize_angle(cur[2] - goal[2]);
    const bool move = py_hypot(goal[0] - cur[0], goal[1] - cur[1]) > P.goal_dist_tol;
    const bool rot = fabs(e_theta) > P.rotate_tol;
    return !(move || rot);
}

__device__ inline double lookahead_dist(double v, const pmp_lp_params& P)
{
    return clampd(fabs(v) * P.lookahead_time, P.min_lookahead, P.max_lookahead);
}

// python index into a list of P points (negative indices wrap like path[-1])
__device__ inline int pyidx(int i, int P) { return ((i % P) + P) % P; }

// Tail of getLookaheadPoint (local_planner.py:120-170) once idx_closest / idx_goal are known.
// Returns 0, or PMP_REF_RAISES where the reference raises (IndexError / math domain error /
// ZeroDivisionError in the curvature part).
__device__ inline int lookahead_tail(const double* path, int P, double rx, double ry, double L, int idx_goal,
                                     double* pt, double* theta, double* kappa)
{
    int idx_prev = P - 2;
#define PX(i) path[2 * pyidx((i), P)]
#define PY(i) path[2 * pyidx((i), P) + 1]
    if (idx_goal == P - 1) {
        pt[0] = PX(idx_goal);
        pt[1] = PY(idx_goal);
    } else {
        if (idx_goal == 0) idx_goal = idx_goal + 1;
        idx_prev = idx_goal - 1;
        const double x1 = PX(idx_prev) - rx, y1 = PY(idx_prev) - ry;
        const double x2 = PX(idx_goal) - rx, y2 = PY(idx_goal) - ry;
        // MathHelper.circleSegmentIntersection (math_helper.py:11-37)
        const double dx = x2 - x1, dy = y2 - y1;
        const double dr2 = dx * dx + dy * dy;
        const double D = x1 * y2 - x2 * y1;
        const double d1 = x1 * x1 + y1 * y1, d2 = x2 * x2 + y2 * y2, dd = d2 - d1;
        const double delta_2 = L * L * dr2 - D * D;
        double ix, iy;
        if (delta_2 < 0) {  // MathHelper.closestPointOnLine (math_helper.py:39-58)
            const double apx = 0.0 - x1, apy = 0.0 - y1, abx = x2 - x1, aby = y2 - y1;
            const double af = (apx * abx + apy * aby) / (abx * abx + aby * aby);
            ix = x1 + af * abx;
            iy = y1 + af * aby;
        } else {
            const double delta = sqrt(delta_2);
            if (delta == 0) {
                ix = D * dy / dr2;
                iy = -D * dx / dr2;
            } else {
                const double s = copysign(1.0, dd);
                ix = (D * dy + s * dx * delta) / dr2;
                iy = (-D * dx + s * dy * delta) / dr2;
            }
        }
        pt[0] = ix + rx;
        pt[1] = iy + ry;
    }
    if (P < 2 || idx_goal >= P) return PMP_REF_RAISES;
    *theta = atan2(PY(idx_goal) - PY(idx_prev), PX(idx_goal) - PX(idx_prev));
    if (idx_goal == 1) idx_goal = idx_goal + 1;
    if (idx_goal >= P) return PMP_REF_RAISES;
    idx_prev = idx_goal - 1;
    const int idx_pprev = idx_prev - 1;
    const double a = py_hypot(PX(idx_goal) - PX(idx_prev), PY(idx_goal) - PY(idx_prev));
    const double b = py_hypot(PX(idx_goal) - PX(idx_pprev), PY(idx_goal) - PY(idx_pprev));
    const double c = py_hypot(PX(idx_prev) - PX(idx_pprev), PY(idx_prev) - PY(idx_pprev));
    if (a == 0.0 || b == 0.0 || c == 0.0) return PMP_REF_RAISES;
    const double cosB = (a * a + c * c - b * b) / (2 * a * c);
    if (cosB > 1.0 || cosB < -1.0) return PMP_REF_RAISES;
    const double sinB = sin(acos(cosB));
    const double cross = (PX(idx_prev) - PX(idx_pprev)) * (PY(idx_goal) - PY(idx_pprev)) -
                         (PY(idx_prev) - PY(idx_pprev)) * (PX(idx_goal) - PX(idx_pprev));
    *kappa = copysign(2 * sinB / b, cross);
#undef PX
#undef PY
    return 0;
}

// Block-wide first-index best of (v, i): the minimum (MIN) or maximum of v, ties to the lowest i.
// Butterflies inside each wave, then one LDS round over the waves' results: `redd` / `redi` need
// blockDim.x / 64 entries.  Every thread returns the block's result.
template <bool MIN>
__device__ inline void block_best(double& v, int& i, double* redd, int* redi)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o);
        const int oi = __shfl_xor(i, o);
        const bool take = MIN ? (ov < v || (ov == v && oi < i)) : (ov > v || (ov == v && oi < i));
        if (take) {
            v = ov;
            i = oi;
        }
    }
    const int nw = (int)(blockDim.x >> 6);
    __syncthreads();  // the previous use of redd / redi is read everywhere
    if ((threadIdx.x & 63) == 0) {
        redd[threadIdx.x >> 6] = v;
        redi[threadIdx.x >> 6] = i;
    }
    __syncthreads();
    v = redd[0];
    i = redi[0];
    for (int k = 1; k < nw; k++) {
        const double ov = redd[k];
        const int oi = redi[k];
        const bool take = MIN ? (ov < v || (ov == v && oi < i)) : (ov > v || (ov == v && oi < i));
        if (take) {
            v = ov;
            i = oi;
        }
    }
}

// getLookaheadPoint (local_planner.py:103-170) for one agent, computed by a whole workgroup:
// the distance scan, first-index argmin and the first-beyond-lookahead search are block-parallel,
// the tail runs on thread 0.  `redd` / `redi` hold >= blockDim.x / 64 entries of LDS.
__device__ inline int lookahead_block(const double* path, int P, double rx, double ry, double v, const pmp_lp_params& Pm,
                                      double* pt, double* theta, double* kappa, double* redd, int* redi)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const double L = lookahead_dist(v, Pm);
    // idx_closest = dist_to_robot.index(min(dist_to_robot))
    double bd = INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < P; i += nt) {
        const double d = py_hypot(rx - path[2 * i], ry - path[2 * i + 1]);
        if (d < bd) { bd = d; bi = i; }  // strided in increasing i: keeps the first minimum
    }
    block_best<true>(bd, bi, redd, redi);
    const int idx_closest = bi;
    // first i >= idx_closest with dist >= L
    int fi = 0x7fffffff;
    for (int i = idx_closest + tid; i < P; i += nt) {
        if (py_hypot(rx - path[2 * i], ry - path[2 * i + 1]) >= L) { fi = i; break; }
    }
    double fd = 0.0;
    block_best<true>(fd, fi, redd, redi);
    const int first = fi;
    int st = 0;
    __syncthreads();
    if (tid == 0) {
        const int idx_goal = first == 0x7fffffff ? P - 1 : first;
        st = lookahead_tail(path, P, rx, ry, L, idx_goal, pt, theta, kappa);
        redi[0] = st;
    }
    __syncthreads();
    st = redi[0];
    __syncthreads();
    return st;
}

}  // namespace lp
