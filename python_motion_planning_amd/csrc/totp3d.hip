// Batched TimeOptimalTrajectory3D.generate() for gfx950 (trajectory/time_optimal_trajectory.py:8-353,
// trajectory_base.py:245-261): the C5 step after 3D planning (examples/3d_example.py:93-128).
//
// One wave64 per path:
//  1. arc lengths (lane-parallel segment norms, a lane-0 running sum in the reference's order) and
//     scipy's not-a-knot CubicSpline per axis (lanes 0..2 each solve their axis' banded system the
//     way LAPACK's dgbtf2 / dgbtrs / dtbsv do; coefficients lane-parallel), all in LDS;
//  2. the forward and backward velocity integrations (:162-226): every step depends on the last
//     velocity through the centripetal term, so the recurrence runs on lane 0 while the other lanes
//     stage the next 64 samples' spline derivatives and velocity limits in LDS;
//  3. s_ddot (lane-parallel) and the time profile (lane-0 running sum of lane-parallel increments);
//  4. generate(): lane 0 steps t = 0, dt, ... (the reference's float accumulation), the lanes
//     evaluate 64 points at a time (interp1d linear on the time profile, spline at s), yaw and yaw
//     rate from the neighbouring lane.
// Values follow the reference's operation order (CPython / numpy float64, -ffp-contract=off), so
// results match it to rounding (the parity tests bound them at 1e-9 relative).
#include "pmp_internal.h"

namespace {

constexpr int kCh = 64;    // samples / points staged per round (one per lane)
constexpr int kStage = 8;  // doubles staged per sample

// scipy CubicSpline(x, y, bc 'not-a-knot') first derivatives at the knots (scipy/interpolate/_cubic.py,
// scipy 1.15): n == 2 both ends take the slope; n == 3 the parabola system (LAPACK dgesv, partial
// pivoting); n >= 4 the tridiagonal system with the not-a-knot end rows, LU with partial pivoting
// (dgbtf2, multipliers by the reciprocal pivot) and column-oriented back substitution (dtbsv).
// w: 5n doubles of scratch.  Same arithmetic as oracle/pmp_oracle.c cspline_slopes.
__device__ void spline_slopes(const double* x, const double* y, int n, double* s, double* w)
{
    double* dx = w;
    double* sl = w + n;
    for (int i = 0; i + 1 < n; i++) {
        dx[i] = x[i + 1] - x[i];
        sl[i] = (y[i + 1] - y[i]) / dx[i];
    }
    if (n == 2) {
        s[0] = sl[0];
        s[1] = sl[0];
        return;
    }
    if (n == 3) {
        double A[3][3] = {{1.0, 1.0, 0.0}, {dx[1], 2.0 * (dx[0] + dx[1]), dx[0]}, {0.0, 1.0, 1.0}};
        double b[3] = {2.0 * sl[0], 3.0 * (dx[0] * sl[1] + dx[1] * sl[0]), 2.0 * sl[1]};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            int p = k;
            for (int r = k + 1; r < 3; r++)
                if (fabs(A[r][k]) > fabs(A[p][k])) p = r;
            if (p != k) {
                for (int c = 0; c < 3; c++) {
                    const double t = A[k][c];
                    A[k][c] = A[p][c];
                    A[p][c] = t;
                }
                const double t = b[k];
                b[k] = b[p];
                b[p] = t;
            }
            const double rinv = 1.0 / A[k][k];
            for (int r = k + 1; r < 3; r++) {
                const double m = A[r][k] * rinv;
                for (int c = k + 1; c < 3; c++) A[r][c] -= m * A[k][c];
                b[r] -= m * b[k];
            }
        }
#pragma unroll
        for (int k = 2; k >= 0; k--) {
            s[k] = b[k] / A[k][k];
            for (int r = 0; r < k; r++) b[r] -= s[k] * A[r][k];
        }
        return;
    }
    double* D = w + 2 * n;
    double* U1 = w + 3 * n;
    double* U2 = w + 4 * n;
    double* b = s;
    for (int i = 1; i + 1 < n; i++) {
        D[i] = 2.0 * (dx[i - 1] + dx[i]);
        U1[i] = dx[i - 1];
        U2[i] = 0.0;
        b[i] = 3.0 * (dx[i] * sl[i - 1] + dx[i - 1] * sl[i]);
    }
    {
        const double d = x[2] - x[0];
        D[0] = dx[1];
        U1[0] = d;
        U2[0] = 0.0;
        b[0] = ((dx[0] + 2.0 * d) * dx[1] * sl[0] + (dx[0] * dx[0]) * sl[1]) / d;
    }
    double Lnm1;
    {
        const double d = x[n - 1] - x[n - 3];
        D[n - 1] = dx[n - 3];
        Lnm1 = d;
        U1[n - 1] = 0.0;
        U2[n - 1] = 0.0;
        b[n - 1] = ((dx[n - 2] * dx[n - 2]) * sl[n - 3] + (2.0 * d + dx[n - 2]) * dx[n - 3] * sl[n - 2]) / d;
    }
    for (int k = 0; k + 1 < n; k++) {
        double Lk1 = (k + 1 == n - 1) ? Lnm1 : dx[k + 1];
        if (fabs(Lk1) > fabs(D[k])) {
            const double t0 = D[k], t1 = U1[k], t2 = U2[k], tb = b[k];
            D[k] = Lk1;
            U1[k] = D[k + 1];
            U2[k] = U1[k + 1];
            b[k] = b[k + 1];
            Lk1 = t0;
            D[k + 1] = t1;
            U1[k + 1] = t2;
            b[k + 1] = tb;
        }
        const double m = Lk1 * (1.0 / D[k]);
        D[k + 1] -= m * U1[k];
        if (k + 2 < n) U1[k + 1] -= m * U2[k];
        b[k + 1] -= m * b[k];
    }
    for (int j = n - 1; j >= 0; j--) {
        if (b[j] != 0.0) {
            b[j] = b[j] / D[j];
            const double t = b[j];
            if (j >= 1) b[j - 1] -= t * U1[j - 1];
            if (j >= 2) b[j - 2] -= t * U2[j - 2];
        }
    }
}

// PPoly interval (scipy/interpolate/_ppoly.pyx find_interval_ascending): x[i] <= v < x[i+1], the
// last interval closed, out-of-range values to the end intervals
__device__ __forceinline__ int pp_interval(const double* x, int n, double v)
{
    if (!(x[0] <= v && v <= x[n - 1])) return v < x[0] ? 0 : n - 2;
    if (v == x[n - 1]) return n - 2;
    int lo = 0, hi = n - 2;
    if (v < x[lo + 1]) hi = lo;
    while (lo < hi) {
        const int mid = (hi + lo) / 2;
        if (v < x[mid]) hi = mid;
        else if (v >= x[mid + 1]) lo = mid + 1;
        else {
            lo = mid;
            break;
        }
    }
    return lo;
}

struct Spline {
    const double* arc;  // knots (arc lengths) [n]
    const double* C;    // [3 axes][4 rows][n - 1]
    int n;
    double L;
};

// _evaluate_path (time_optimal_trajectory.py:76-94): s clipped to [0, L]; position and the
// derivative(1) / derivative(2) PPolys (coefficients [3c0, 2c1, c2], [6c0, 2c1]) evaluated as
// evaluate_poly1 does (power sums with the power built by products)
__device__ __forceinline__ void eval_path(const Spline& S, double s, double pos[3], double q1[3], double q2[3])
{
    s = s < 0.0 ? 0.0 : (s > S.L ? S.L : s);
    const int i = pp_interval(S.arc, S.n, s), m = S.n - 1;
    const double u = s - S.arc[i], u2 = u * u, u3 = u2 * u;
#pragma unroll
    for (int d = 0; d < 3; d++) {
        const double* c = S.C + (size_t)d * 4 * m;
        const double c0 = c[i], c1 = c[m + i], c2 = c[2 * m + i], c3 = c[3 * m + i];
        pos[d] = ((c3 + c2 * u) + c1 * u2) + c0 * u3;
        q1[d] = (c2 + (2.0 * c1) * u) + (3.0 * c0) * u2;
        q2[d] = (2.0 * c1) + (6.0 * c0) * u;
    }
}

// np.linspace(0, L, ns)[i] (numpy/_core/function_base.py)
__device__ __forceinline__ double lin(double L, int ns, int i)
{
    if (i == ns - 1) return L;
    const double div = (double)(ns - 1), step = L / div;
    return step == 0.0 ? ((double)i / div) * L : (double)i * step;
}

__device__ __forceinline__ double sq(double a) { return a * a; }

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void totp3d_kernel(pmp_totp_params T, int nq, const double* __restrict__ path,
                                                    const int32_t* __restrict__ off, int nmax, int sample_cap,
                                                    double* __restrict__ sv_out, double* __restrict__ sd_out,
                                                    double* __restrict__ sdd_out, double* __restrict__ tp_out,
                                                    int32_t* __restrict__ ns_out, int point_cap, double* __restrict__ pts_out,
                                                    int32_t* __restrict__ np_out, double* __restrict__ total_out,
                                                    int32_t* __restrict__ st_out, const double* __restrict__ eval_t,
                                                    int n_eval)
{
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int q = blockIdx.x;
    const int lane = lane_id();
    if (q >= nq) return;
    const int p0 = off[q], n = off[q + 1] - p0;
    // LDS: arc [nmax] | spline coefficients [12 (nmax - 1)] | work region: the path (3 n), the solve
    // scratch (3 x 6 n), later the per-round stage (kCh x kStage)
    double* arc = sm;
    double* C = arc + nmax;
    double* R = C + 12 * (nmax > 1 ? nmax - 1 : 1);
    double* stage = R;
    if (n < 2 || n > nmax) {  // n < 2: the reference raises ValueError (time_optimal_trajectory.py:263)
        if (lane == 0) {
            st_out[q] = n < 2 ? PMP_REF_RAISES : PMP_CAP_OVERFLOW;
            ns_out[q] = 0;
            np_out[q] = 0;
            total_out[q] = 0.0;
        }
        return;
    }
    double* Y = R;  // [3][n]
    for (int i = lane; i < n; i += 64)
        for (int d = 0; d < 3; d++) Y[d * n + i] = path[3 * (size_t)(p0 + i) + d];
    __syncthreads();
    // _parameterize_path (:41-74): segment norms (np.linalg.norm = sqrt(dot)), cumulative sum
    for (int i = lane + 1; i < n; i += 64) {
        const double a = Y[i] - Y[i - 1], b = Y[n + i] - Y[n + i - 1], e = Y[2 * n + i] - Y[2 * n + i - 1];
        arc[i] = __dsqrt_rn((a * a + b * b) + e * e);
    }
    __syncthreads();
    if (lane == 0) {
        double acc = 0.0;
        arc[0] = 0.0;
        for (int i = 1; i < n; i++) {
            acc = acc + arc[i];
            arc[i] = acc;
        }
    }
    __syncthreads();
    {
        // scipy raises ValueError for knots that are not strictly increasing (repeated waypoints)
        bool bad = false;
        for (int i = lane; i + 1 < n; i += 64) bad |= !(arc[i + 1] - arc[i] > 0.0);
        if (ballot(bad)) {
            if (lane == 0) {
                st_out[q] = PMP_REF_RAISES;
                ns_out[q] = 0;
                np_out[q] = 0;
                total_out[q] = 0.0;
            }
            return;
        }
    }
    const int m = n - 1;
    double* Sl = R + 3 * n;  // slopes [3][n], then solve scratch [3][5n]
    if (lane < 3) spline_slopes(arc, Y + lane * n, n, Sl + lane * n, Sl + 3 * n + lane * 5 * n);
    __syncthreads();
    // CubicHermiteSpline coefficients (scipy/interpolate/_cubic.py)
    for (int t = lane; t < 3 * m; t += 64) {
        const int d = t / m, i = t - d * m;
        const double* y = Y + d * n;
        const double* s = Sl + d * n;
        const double dx = arc[i + 1] - arc[i], slope = (y[i + 1] - y[i]) / dx;
        const double tt = ((s[i] + s[i + 1]) - 2.0 * slope) / dx;
        double* c = C + (size_t)d * 4 * m;
        c[i] = tt / dx;
        c[m + i] = (slope - s[i]) / dx - tt;
        c[2 * m + i] = s[i];
        c[3 * m + i] = y[i];
    }
    __syncthreads();
    Spline S;
    S.arc = arc;
    S.C = C;
    S.n = n;
    S.L = arc[n - 1];
    const double L = S.L;
    int ns = (int)(L / T.path_resolution);
    if (ns < 100) ns = 100;
    if (lane == 0) {
        ns_out[q] = ns;
        np_out[q] = 0;
        total_out[q] = 0.0;
    }
    if (ns > sample_cap) {
        if (lane == 0) st_out[q] = PMP_PATH_OVERFLOW;
        return;
    }
    double* sv = sv_out + (size_t)q * sample_cap;
    double* sd = sd_out + (size_t)q * sample_cap;
    double* sdd = sdd_out + (size_t)q * sample_cap;
    double* tp = tp_out + (size_t)q * sample_cap;
    for (int i = lane; i < ns; i += 64) sv[i] = lin(L, ns, i);

    // ---- _forward_integration (:162-195)
    double sdp = 0.0;  // lane 0: s_dot_max[i - 1]
    if (lane == 0) sd[0] = 0.0;
    for (int base = 1; base < ns; base += kCh) {
        const int i = base + lane;
        if (i < ns) {
            const double s0 = lin(L, ns, i - 1), s1 = lin(L, ns, i), smid = (s1 + s0) / 2.0;
            double pos[3], q1[3], q2[3];
            // _compute_max_velocity(s_mid) (:96-118)
            eval_path(S, smid, pos, q1, q2);
            double vc = 0.0;
            bool any = false;
#pragma unroll
            for (int d = 0; d < 3; d++)
                if (fabs(q1[d]) > 1e-10) {
                    const double v = T.max_velocity[d] / fabs(q1[d]);
                    if (!any || v < vc) vc = v;
                    any = true;
                }
            if (!any) vc = fmin(fmin(T.max_velocity[0], T.max_velocity[1]), T.max_velocity[2]);
            eval_path(S, s0, pos, q1, q2);
            double* g = stage + lane * kStage;
            g[0] = q1[0]; g[1] = q1[1]; g[2] = q1[2];
            g[3] = q2[0]; g[4] = q2[1]; g[5] = q2[2];
            g[6] = vc;
            g[7] = s1 - s0;
        }
        __syncthreads();
        if (lane == 0) {
            const int cnt = min(kCh, ns - base);
            for (int l = 0; l < cnt; l++) {
                const double* g = stage + l * kStage;
                // _compute_max_acceleration (:120-160): the forward limit, with the reference's sign
                // handling for q' < 0
                double smax = __longlong_as_double(0x7ff0000000000000ll);
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const double a = g[d];
                    if (fabs(a) > 1e-10) {
                        const double cen = g[3 + d] * sdp * sdp;
                        if (a > 0) {
                            const double fw = (T.max_acceleration[d] - cen) / a;
                            if (fw < smax) smax = fw;
                        } else {
                            const double bw = (-T.max_acceleration[d] - cen) / a;
                            if (-bw < smax) smax = -bw;
                        }
                    }
                }
                const double vc = g[6];
                double nv;
                if (smax > 0) {
                    const double v2 = sdp * sdp + 2.0 * smax * g[7];
                    const double r = __dsqrt_rn(v2 > 0 ? v2 : 0.0);
                    nv = vc < r ? vc : r;
                } else {
                    nv = vc < sdp ? vc : sdp;
                }
                sd[base + l] = nv;
                sdp = nv;
            }
        }
        __syncthreads();
    }

    // ---- _backward_integration (:197-226): i = ns - 2 .. 0, limits at s_values[i + 1]
    double sdn = 0.0;  // lane 0: s_dot_final[i + 1]
    if (lane == 0) sd[ns - 1] = 0.0;
    for (int top = ns - 2; top >= 0; top -= kCh) {
        const int i = top - lane;
        if (i >= 0) {
            const double s0 = lin(L, ns, i), s1 = lin(L, ns, i + 1);
            double pos[3], q1[3], q2[3];
            eval_path(S, s1, pos, q1, q2);
            double* g = stage + lane * kStage;
            g[0] = q1[0]; g[1] = q1[1]; g[2] = q1[2];
            g[3] = q2[0]; g[4] = q2[1]; g[5] = q2[2];
            g[6] = sd[i];  // the forward profile (lane 0's stores, drained by the barrier above)
            g[7] = s1 - s0;
        }
        __syncthreads();
        if (lane == 0) {
            const int cnt = min(kCh, top + 1);
            for (int l = 0; l < cnt; l++) {
                const double* g = stage + l * kStage;
                double smin = __longlong_as_double((long long)0xfff0000000000000ull);
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    const double a = g[d];
                    if (fabs(a) > 1e-10) {
                        const double cen = g[3 + d] * sdn * sdn;
                        if (a > 0) {
                            const double bw = (-T.max_acceleration[d] - cen) / a;
                            if (bw > smin) smin = bw;
                        } else {
                            const double fw = (T.max_acceleration[d] - cen) / a;
                            if (-fw > smin) smin = -fw;
                        }
                    }
                }
                double cur = g[6];
                if (smin < 0) {
                    const double v2 = sdn * sdn - 2.0 * smin * g[7];
                    const double vb = __dsqrt_rn(v2 > 0 ? v2 : 0.0);
                    cur = vb < cur ? vb : cur;
                }
                sd[top - l] = cur;
                sdn = cur;
            }
        }
        __syncthreads();
    }

    // ---- _compute_velocity_profile (:228-258): s_ddot, then the time profile
    for (int i = lane; i < ns; i += 64) {
        double v = 0.0;
        if (i >= 1 && i + 1 < ns) {
            const double ds = lin(L, ns, i + 1) - lin(L, ns, i - 1);
            if (ds > 0) v = (sq(sd[i + 1]) - sq(sd[i - 1])) / (2.0 * ds);
        }
        sdd[i] = v;
    }
    double tacc = 0.0;  // lane 0: time_profile[i - 1]
    if (lane == 0) tp[0] = 0.0;
    for (int base = 1; base < ns; base += kCh) {
        const int i = base + lane;
        if (i < ns) {
            const double ds = lin(L, ns, i) - lin(L, ns, i - 1), avg = (sd[i] + sd[i - 1]) / 2.0;
            stage[lane] = avg > 1e-10 ? ds / avg : ds / 0.1;
        }
        __syncthreads();
        if (lane == 0) {
            const int cnt = min(kCh, ns - base);
            for (int l = 0; l < cnt; l++) {
                tacc = tacc + stage[l];
                tp[base + l] = tacc;
            }
        }
        __syncthreads();
    }
    const double total = rl_f64(tacc, 0);
    if (lane == 0) total_out[q] = total;

    // ---- generate (:260-302) / evaluate (:304-335) + compute_yaw_from_velocity (trajectory_base.py:245-261)
    double* pts = pts_out + (size_t)q * point_cap * 12;
    double* tq = stage;  // [kCh] query times
    int* meta = (int*)(stage + kCh);
    double t = 0.0, last_t = -1.0;  // lane 0: the reference's accumulated t
    int count = 0;
    bool done = false;
    double prev_t = 0.0, prev_yaw = 0.0;  // the previous point (wave-uniform)
    bool prev_has = false, prev_yaw_ok = false;
    while (!done) {
        if (lane == 0) {
            int k = 0;
            bool fin = false;
            if (eval_t) {
                for (; k < kCh && count + k < n_eval; k++) tq[k] = eval_t[count + k];
                fin = count + k >= n_eval;
            } else {
                while (k < kCh) {
                    if (t <= total) {
                        tq[k++] = t;
                        last_t = t;
                        t += T.min_time_step;
                    } else {
                        if (count + k > 0 && last_t < total) {
                            tq[k++] = total;
                            last_t = total;
                        }
                        fin = true;
                        break;
                    }
                }
            }
            meta[0] = k;
            meta[1] = fin ? 1 : 0;
        }
        __syncthreads();
        const int k = meta[0];
        done = meta[1] != 0;
        double my_t = 0.0, yaw = 0.0;
        bool has = false;
        double o[12];
        if (lane < k) {
            const double tc = tq[lane] < 0.0 ? 0.0 : (tq[lane] > total ? total : tq[lane]);
            // interp1d(kind='linear', fill_value='extrapolate') (scipy _call_linear): searchsorted
            // (left), clipped to [1, ns - 1]
            int lo = 0, hi = ns;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (tp[mid] < tc) lo = mid + 1;
                else hi = mid;
            }
            int h = lo < 1 ? 1 : (lo > ns - 1 ? ns - 1 : lo);
            const int l0 = h - 1;
            const double xl = tp[l0], xh = tp[h], dxl = tc - xl;
            const double s = (lin(L, ns, h) - lin(L, ns, l0)) / (xh - xl) * dxl + lin(L, ns, l0);
            const double sdt = (sd[h] - sd[l0]) / (xh - xl) * dxl + sd[l0];
            const double sddt = (sdd[h] - sdd[l0]) / (xh - xl) * dxl + sdd[l0];
            double pos[3], q1[3], q2[3];
            eval_path(S, s, pos, q1, q2);
            o[0] = tc;
#pragma unroll
            for (int d = 0; d < 3; d++) {
                o[1 + d] = pos[d];
                o[4 + d] = q1[d] * sdt;
                o[7 + d] = q2[d] * (sdt * sdt) + q1[d] * sddt;
            }
            my_t = tc;
            has = !eval_t && __dsqrt_rn(o[4] * o[4] + o[5] * o[5]) > 1e-6;
            yaw = has ? atan2(o[5], o[4]) : 0.0;
            o[10] = has ? yaw : __longlong_as_double(0x7ff8000000000000ll);
        }
        // yaw rate from the previous point: lane - 1, or the previous round's last point (all lanes
        // take part in the shuffles)
        const double pt = __shfl_up(my_t, 1), py = __shfl_up(yaw, 1);
        const bool ph = __shfl_up(has ? 1 : 0, 1) != 0;
        if (lane < k) {
            const double qt = lane == 0 ? prev_t : pt, qy = lane == 0 ? prev_yaw : py;
            const bool qh = lane == 0 ? (prev_has && prev_yaw_ok) : ph;
            double rate = __longlong_as_double(0x7ff8000000000000ll);
            const double dtp = my_t - qt;
            if (qh && has && dtp > 0) {
                double dy = yaw - qy;
                while (dy > M_PI) dy -= 2.0 * M_PI;
                while (dy < -M_PI) dy += 2.0 * M_PI;
                rate = dy / dtp;
            }
            o[11] = rate;
            const int idx = count + lane;
            if (idx < point_cap)
                for (int j = 0; j < 12; j++) pts[(size_t)idx * 12 + j] = o[j];
        }
        if (k > 0) {
            prev_t = rl_f64(my_t, k - 1);
            prev_yaw = rl_f64(yaw, k - 1);
            prev_yaw_ok = rl_u32(has ? 1u : 0u, k - 1) != 0;
            prev_has = true;
        }
        count += k;
        __syncthreads();
    }
    if (lane == 0) {
        np_out[q] = count;
        st_out[q] = count > point_cap ? PMP_PATH_OVERFLOW : PMP_FOUND;
    }
}

}  // namespace

extern "C" int pmp_totp3d_batch(pmp_ctx* ctx, void* stream, const pmp_totp_params* prm, int nq, const double* path_xyz,
                                const int32_t* path_off, int max_waypoints, int sample_cap, double* s_values,
                                double* s_dot, double* s_ddot, double* time_profile, int32_t* n_samples, int point_cap,
                                double* points, int32_t* n_points, double* total_time, int32_t* status,
                                const double* eval_t, int n_eval)
{
    if (!ctx) return PMP_EINVAL;
    if (!prm || nq < 0 || max_waypoints < 1 || sample_cap < 1 || point_cap < 1 || n_eval < 0 || (eval_t && n_eval < 1))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_totp3d_batch: bad params/nq/max_waypoints/caps/n_eval");
    if (!(prm->path_resolution > 0) || !(prm->min_time_step > 0))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_totp3d_batch: path_resolution and min_time_step must be > 0");
    if (nq == 0) return PMP_OK;
    if (!path_xyz || !path_off || !s_values || !s_dot || !s_ddot || !time_profile || !n_samples || !points ||
        !n_points || !total_time || !status)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_totp3d_batch: null pointer argument");
    // LDS: arc + coefficients + the path / spline-solve region (the 64-sample stage fits inside it)
    const size_t nm = (size_t)max_waypoints;
    const size_t work = 3 * nm + 3 * nm + 15 * nm;
    const size_t lds = 8 * (nm + 12 * (nm > 1 ? nm - 1 : 1) + (work > (size_t)kCh * kStage + 8 ? work : (size_t)kCh * kStage + 8));
    if (lds > 160 * 1024)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_totp3d_batch: max_waypoints too large for one CU's LDS (<= 480)");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(totp3d_kernel, dim3(nq), dim3(64), lds, (hipStream_t)stream, *prm, nq, path_xyz, path_off,
                       max_waypoints, sample_cap, s_values, s_dot, s_ddot, time_profile, n_samples, point_cap, points,
                       n_points, total_time, status, eval_t, n_eval);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
