// Batched tracking controllers for gfx950: LQR.lqrControl (local_planner/lqr.py:103-145),
// MPC.mpcControl (local_planner/mpc.py:111-214) and whole LQR.plan / MPC.plan iterations
// (lqr.py:58-86, mpc.py:66-94).
//
// LQR: one 3x3 Riccati update per call (the signed exit of lqr.py:134 stops it after one update
// under the reference's defaults), 2x2 inverse, K e.  Scalar f64 on one lane.
//
// MPC, one wave64 per agent:
//  - QP assembly in closed form.  A3 = I + N with N^2 = 0 (N = column 2 of lqr/mpc's A), so
//    A3^k = I + kN and the blocks of S_u are G_n = C A5^n B5 = sum_{k<=n} A3^k B3
//    = (n+1) B3 + n(n+1)/2 N B3; S_x's block i is [I + (i+1)N | G_i].
//  - H = S_u' Qbar S_u on the f64 MFMA (v_mfma_f64_16x16x4_f64): lane l holds
//    S_u[r = 4t + l/16][col = l%16] of the t-th K-slice, A = q_r * S_u, B = S_u; the 3p rows of S_u
//    are the K dimension, so one 16x16 accumulator tile is the whole of H.  g = S_u' Qbar S_x x
//    rides along on the VALU.
//  - ADMM (the OSQP algorithm, unscaled): lanes 0..15 own variable v and constraint rows v (the
//    cumulative-sum rows of kron(tril(1_m), I2)) and 2m+v (the identity rows).  A x is a
//    stride-2 prefix scan, A'y a stride-2 suffix scan (3 lane shuffles each); the x-update
//    multiplies by an explicit inverse of H + sigma I + rho A'A held as one row per lane, built by
//    Gauss-Jordan with readlane broadcasts of the pivot row (rebuilt only when rho adapts).
#include "localplan.h"

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// LQR.lqrControl (lqr.py:103-145) + linear/angularRegularization (local_planner.py:172-206)
// ---------------------------------------------------------------------------------------------
__device__ void lqr_control(const double s[3], const double sd[3], const double ur[2], double rv, double rw,
                            const pmp_lp_params& Pr, const pmp_lqr_params& L, double u[2])
{
    const double dt = Pr.dt;
    double sn, cs;
    sincos(sd[2], &sn, &cs);
    double A[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, B[3][2] = {{0, 0}, {0, 0}, {0, 0}};
    A[0][2] = -ur[0] * sn * dt;
    A[1][2] = ur[0] * cs * dt;
    B[0][0] = cs * dt;
    B[1][0] = sn * dt;
    B[2][1] = dt;
    double Pm[3][3] = {{L.q[0], 0, 0}, {0, L.q[1], 0}, {0, 0, L.q[2]}};
    double Pn[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int it = 0; it < L.iters; it++) {
        double PA[3][3], PB[3][2], APA[3][3], APB[3][2], BPB[2][2], BPA[2][3], S[2][2], Si[2][2];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { PA[i][j] = 0; for (int k = 0; k < 3; k++) PA[i][j] += Pm[i][k] * A[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 2; j++) { PB[i][j] = 0; for (int k = 0; k < 3; k++) PB[i][j] += Pm[i][k] * B[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { APA[i][j] = 0; for (int k = 0; k < 3; k++) APA[i][j] += A[k][i] * PA[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 2; j++) { APB[i][j] = 0; for (int k = 0; k < 3; k++) APB[i][j] += A[k][i] * PB[k][j]; }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++) { BPB[i][j] = 0; for (int k = 0; k < 3; k++) BPB[i][j] += B[k][i] * PB[k][j]; }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) { BPA[i][j] = 0; for (int k = 0; k < 3; k++) BPA[i][j] += B[k][i] * PA[k][j]; }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++) S[i][j] = (i == j ? L.r[i] : 0.0) + BPB[i][j];
        const double det = S[0][0] * S[1][1] - S[0][1] * S[1][0];
        Si[0][0] = S[1][1] / det; Si[0][1] = -S[0][1] / det; Si[1][0] = -S[1][0] / det; Si[1][1] = S[0][0] / det;
        double mx = -INFINITY;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double corr = 0;
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) corr += APB[i][a] * Si[a][b] * BPA[b][j];
                Pn[i][j] = (i == j ? L.q[i] : 0.0) + APA[i][j] - corr;
                mx = fmax(mx, Pm[i][j] - Pn[i][j]);
            }
        if (mx < L.eps) break;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Pm[i][j] = Pn[i][j];
    }
    double PB[3][2], PA[3][3], BPB[2][2], BPA[2][3], Si[2][2];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 2; j++) { PB[i][j] = 0; for (int k = 0; k < 3; k++) PB[i][j] += Pn[i][k] * B[k][j]; }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) { PA[i][j] = 0; for (int k = 0; k < 3; k++) PA[i][j] += Pn[i][k] * A[k][j]; }
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) { BPB[i][j] = (i == j ? L.r[i] : 0.0); for (int k = 0; k < 3; k++) BPB[i][j] += B[k][i] * PB[k][j]; }
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) { BPA[i][j] = 0; for (int k = 0; k < 3; k++) BPA[i][j] += B[k][i] * PA[k][j]; }
    const double det = BPB[0][0] * BPB[1][1] - BPB[0][1] * BPB[1][0];
    Si[0][0] = BPB[1][1] / det; Si[0][1] = -BPB[0][1] / det; Si[1][0] = -BPB[1][0] / det; Si[1][1] = BPB[0][0] / det;
    double K[2][3];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) { K[i][j] = 0; for (int a = 0; a < 2; a++) K[i][j] -= Si[i][a] * BPA[a][j]; }
    const double e[3] = {s[0] - sd[0], s[1] - sd[1], lp::regularize_angle(s[2] - sd[2])};
    double uu[2];
    for (int i = 0; i < 2; i++) { uu[i] = ur[i]; for (int j = 0; j < 3; j++) uu[i] += K[i][j] * e[j]; }
    u[0] = lp::clampd(rv + lp::clampd(uu[0] - rv, Pr.min_v_inc, Pr.max_v_inc), Pr.min_v, Pr.max_v);
    u[1] = lp::clampd(rw + lp::clampd(uu[1] - rw, Pr.min_w_inc, Pr.max_w_inc), Pr.min_w, Pr.max_w);
}

// ---------------------------------------------------------------------------------------------
// MPC: 16-lane scans, reductions and the explicit inverse
// ---------------------------------------------------------------------------------------------
// inclusive prefix / suffix sum over lanes of the same parity within lanes 0..15 (v = lane & 15)
__device__ __forceinline__ double prefix16(double t, int v)
{
#pragma unroll
    for (int s = 2; s < 16; s <<= 1) {
        const double o = __shfl_up(t, s);
        t += v >= s ? o : 0.0;
    }
    return t;
}

__device__ __forceinline__ double suffix16(double t, int v)
{
#pragma unroll
    for (int s = 2; s < 16; s <<= 1) {
        const double o = __shfl_down(t, s);
        t += v + s < 16 ? o : 0.0;
    }
    return t;
}

// max over lanes 0..15, returned wave-uniform
__device__ __forceinline__ double max16(double t)
{
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) t = fmax(t, __shfl_xor(t, s));
    return rl_f64(t, 0);
}

// Minv = (H + sigma I + rho A'A)^-1, row v in this lane (rows/cols >= n are the identity).
// A'A[2k+c][2k'+c'] = [c == c'] (m - max(k, k')) + [2k+c == 2k'+c'].
__device__ __forceinline__ void build_inverse(const double* Hrow, int v, int n, int m, double sigma, double rho,
                                              double (&Inv)[16])
{
    double Mr[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        const bool act = v < n && c < n;
        const int kv = v >> 1, kc = c >> 1;
        const double t = ((v & 1) == (c & 1)) ? (double)(m - (kv > kc ? kv : kc)) : 0.0;
        double val = (act ? Hrow[c] : 0.0) + rho * (t + (c == v ? 1.0 : 0.0)) + (c == v ? sigma : 0.0);
        Mr[c] = act ? val : (c == v ? 1.0 : 0.0);
        Inv[c] = c == v ? 1.0 : 0.0;
    }
    // Gauss-Jordan without pivoting (the matrix is SPD).  Before step k the pivot row's Mr is zero
    // left of k and its Inv is zero right of k, so only those columns are broadcast.
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const double f = Mr[k];
        const double inv = 1.0 / rl_f64(Mr[k], k);
        const bool piv = v == k;
#pragma unroll
        for (int c = k; c < 16; c++) {
            const double pr = rl_f64(Mr[c], k) * inv;
            Mr[c] = piv ? pr : Mr[c] - f * pr;
        }
#pragma unroll
        for (int c = 0; c <= k; c++) {
            const double pr = rl_f64(Inv[c], k) * inv;
            Inv[c] = piv ? pr : Inv[c] - f * pr;
        }
    }
}

struct MpcResult {
    double u0, u1;  // regularised control
    int iters, status;
};

// MPC.mpcControl for one agent on the calling wave (all 64 lanes, wave-uniform control flow).
// up0/up1 in/out.  Hs: 256 doubles of LDS.  Optional outputs (already offset to this call).
__device__ MpcResult mpc_control_wave(const double* s, const double* sd, const double* ur, double& up0, double& up1,
                                      double rv, double rw, const pmp_lp_params& P, const pmp_mpc_params& M,
                                      double* Hs, double* qpH, double* qpg, double* qplu, double* duo)
{
    const int lane = lane_id();
    const int m = M.m, n = 2 * m, p = M.p;
    const double dt = P.dt;
    double sn, cs;
    sincos(sd[2], &sn, &cs);
    const double a0 = -ur[0] * sn * dt, a1 = ur[0] * cs * dt;  // A[0,2], A[1,2] (mpc.py:138-139)
    const double b00 = cs * dt, b10 = sn * dt;                 // B[0,0], B[1,0] (mpc.py:143-144)
    const double e0 = s[0] - sd[0], e1 = s[1] - sd[1], e2 = s[2] - sd[2];
    const double p0 = up0, p1 = up1;

    // ---- H = S_u' Qbar S_u (MFMA f64 16x16x4) and g = S_u' Qbar S_x x ----
    const int col = lane & 15, kq = lane >> 4;
    const int jb = col >> 1, cb = col & 1;
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    double gp = 0.0;
    const int R3 = 3 * p;
    for (int k0 = 0; k0 < R3; k0 += 4) {
        const int r = k0 + kq;
        double sv = 0.0, yv = 0.0, qv = 0.0;
        if (r < R3) {
            const int i = r / 3, d = r - 3 * i;
            qv = d == 0 ? M.q[0] : (d == 1 ? M.q[1] : M.q[2]);
            const double n1 = (double)(i + 1), tri = 0.5 * (double)i * (double)(i + 1);
            if (d == 0)
                yv = ((e0 + (n1 * a0) * e2) + (n1 * b00) * p0) + (tri * a0 * dt) * p1;
            else if (d == 1)
                yv = ((e1 + (n1 * a1) * e2) + (n1 * b10) * p0) + (tri * a1 * dt) * p1;
            else
                yv = e2 + (n1 * dt) * p1;
            if (col < n && jb <= i) {
                const int nn = i - jb;
                const double m1 = (double)(nn + 1), tr = 0.5 * (double)nn * (double)(nn + 1);
                if (cb == 0)
                    sv = d == 0 ? m1 * b00 : (d == 1 ? m1 * b10 : 0.0);
                else
                    sv = d == 0 ? tr * a0 * dt : (d == 1 ? tr * a1 * dt : m1 * dt);
            }
        }
        const double av = qv * sv;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, sv, acc, 0, 0, 0);
        gp += av * yv;
    }
    gp += __shfl_xor(gp, 16);
    gp += __shfl_xor(gp, 32);
    // D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = lane/16 + 4*reg
#pragma unroll
    for (int rg = 0; rg < 4; rg++) {
        const int row = kq + 4 * rg;
        double h = acc[rg];
        if (row == col && row < n) h += (row & 1) ? M.r[1] : M.r[0];
        Hs[row * 16 + col] = h;
    }
    __syncthreads();

    const int v = col;                      // lanes 0..15: variable v, rows v and n+v
    const bool act = lane < 16 && v < n;
    const int cv = v & 1;
    const double gv = act ? gp : 0.0;
    const double l1 = act ? (cv ? P.min_w - p1 : P.min_v - p0) : 0.0;  // U_min - U_k_1
    const double h1 = act ? (cv ? P.max_w - p1 : P.max_v - p0) : 0.0;
    const double l2 = act ? (cv ? P.min_w_inc : P.min_v_inc) : 0.0;    // dU_min
    const double h2 = act ? (cv ? P.max_w_inc : P.max_v_inc) : 0.0;
    if (qpH)
        for (int idx = lane; idx < n * n; idx += kWave) qpH[idx] = Hs[(idx / n) * 16 + idx % n];
    if (qpg && act) qpg[v] = gv;
    if (qplu && act) {
        qplu[v] = l1; qplu[n + v] = l2;
        qplu[2 * n + v] = h1; qplu[3 * n + v] = h2;
    }
    // this lane's row of H stays in LDS through the ADMM (read by the inverse builds and the residual
    // checks): 32 fewer live VGPRs than a register copy, so the tracking kernel fits 2 waves per SIMD
    const double* Hrow = Hs + 16 * (v & 15);

    // ---- ADMM ----
    double rho = M.rho;
    const double sigma = M.sigma, alpha = M.alpha;
    double Inv[16];
    build_inverse(Hrow, v, n, m, sigma, rho, Inv);
    double x = 0.0, z1 = 0.0, z2 = 0.0, y1 = 0.0, y2 = 0.0;
    int status = 1, it = 0, cnt_c = 0, cnt_a = 0;
    while (it < M.max_iter) {
        it++;
        cnt_c++;
        cnt_a++;
        const double rinv = 1.0 / rho;
        const double w1 = act ? rho * z1 - y1 : 0.0, w2 = act ? rho * z2 - y2 : 0.0;
        const double rhs = sigma * x - gv + (suffix16(w1, v) + w2);
        double xt = 0.0;
#pragma unroll
        for (int c = 0; c < 16; c++) xt += Inv[c] * rl_f64(rhs, c);
        xt = act ? xt : 0.0;
        const double zt1 = prefix16(xt, v);
        x = alpha * xt + (1.0 - alpha) * x;
        double zr = alpha * zt1 + (1.0 - alpha) * z1;
        double zn = lp::clampd(zr + rinv * y1, l1, h1);
        y1 = act ? y1 + rho * (zr - zn) : 0.0;
        z1 = act ? zn : 0.0;
        zr = alpha * xt + (1.0 - alpha) * z2;
        zn = lp::clampd(zr + rinv * y2, l2, h2);
        y2 = act ? y2 + rho * (zr - zn) : 0.0;
        z2 = act ? zn : 0.0;
        const bool check = (M.check_every > 0 && cnt_c == M.check_every) || it == M.max_iter;
        const bool adapt = M.adaptive_every > 0 && cnt_a == M.adaptive_every;
        if (cnt_c == M.check_every) cnt_c = 0;
        if (cnt_a == M.adaptive_every) cnt_a = 0;
        if (!check && !adapt) continue;
        // residuals (unscaled inf norms, OSQP's termination test)
        const double ax1 = prefix16(x, v), ax2 = x;
        double hx = 0.0;
#pragma unroll
        for (int c = 0; c < 16; c++) hx += (act && c < n ? Hrow[c] : 0.0) * rl_f64(x, c);
        const double aty = suffix16(y1, v) + y2;
        const double prim = max16(act ? fmax(fabs(ax1 - z1), fabs(ax2 - z2)) : 0.0);
        const double dual = max16(act ? fabs((hx + gv) + aty) : 0.0);
        const double pscale = max16(act ? fmax(fmax(fabs(ax1), fabs(ax2)), fmax(fabs(z1), fabs(z2))) : 0.0);
        const double dscale = max16(act ? fmax(fmax(fabs(hx), fabs(aty)), fabs(gv)) : 0.0);
        if (check && prim <= M.eps_abs + M.eps_rel * pscale && dual <= M.eps_abs + M.eps_rel * dscale) {
            status = 0;
            break;
        }
        if (adapt) {
            const double pn = prim / (pscale + 1e-30), dn = dual / (dscale + 1e-30);
            const double rn = lp::clampd(rho * sqrt(pn / (dn + 1e-30)), 1e-6, 1e6);
            if (rn > rho * M.adaptive_tol || rn < rho / M.adaptive_tol) {
                rho = rn;
                build_inverse(Hrow, v, n, m, sigma, rho, Inv);
            }
        }
    }
    __syncthreads();  // Hs is reused by the caller
    if (duo && act) duo[v] = x;
    const double du0 = rl_f64(x, 0), du1 = rl_f64(x, 1);
    const double uu0 = (du0 + p0) + ur[0], uu1 = (du1 + p1) + ur[1];
    up0 = uu0 - ur[0];
    up1 = uu1 - ur[1];
    MpcResult R;
    R.u0 = lp::clampd(rv + lp::clampd(uu0 - rv, P.min_v_inc, P.max_v_inc), P.min_v, P.max_v);
    R.u1 = lp::clampd(rw + lp::clampd(uu1 - rw, P.min_w_inc, P.max_w_inc), P.min_w, P.max_w);
    R.iters = it;
    R.status = status;
    return R;
}

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lqr_control_kernel(pmp_lp_params P, pmp_lqr_params L, int n,
                                                          const double* __restrict__ s, const double* __restrict__ sd,
                                                          const double* __restrict__ ur, const double* __restrict__ vw,
                                                          double* __restrict__ u)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double s_[3] = {s[3 * i], s[3 * i + 1], s[3 * i + 2]};
    const double sd_[3] = {sd[3 * i], sd[3 * i + 1], sd[3 * i + 2]};
    const double ur_[2] = {ur[2 * i], ur[2 * i + 1]};
    double uo[2];
    lqr_control(s_, sd_, ur_, vw[2 * i], vw[2 * i + 1], P, L, uo);
    u[2 * i] = uo[0];
    u[2 * i + 1] = uo[1];
}

__global__ __launch_bounds__(kWave) void mpc_control_kernel(pmp_lp_params P, pmp_mpc_params M, int n,
                                                            const double* __restrict__ s, const double* __restrict__ sd,
                                                            const double* __restrict__ ur, double* __restrict__ up,
                                                            const double* __restrict__ vw, double* __restrict__ u,
                                                            double* __restrict__ qpH, double* __restrict__ qpg,
                                                            double* __restrict__ qplu, double* __restrict__ du,
                                                            int32_t* __restrict__ iters, int32_t* __restrict__ st)
{
    __shared__ double Hs[256];
    const int i = blockIdx.x;
    if (i >= n) return;
    const int nv = 2 * M.m;
    const double s_[3] = {s[3 * i], s[3 * i + 1], s[3 * i + 2]};
    const double sd_[3] = {sd[3 * i], sd[3 * i + 1], sd[3 * i + 2]};
    const double ur_[2] = {ur[2 * i], ur[2 * i + 1]};
    double up0 = up[2 * i], up1 = up[2 * i + 1];
    const MpcResult R = mpc_control_wave(s_, sd_, ur_, up0, up1, vw[2 * i], vw[2 * i + 1], P, M, Hs,
                                         qpH ? qpH + (size_t)i * nv * nv : nullptr, qpg ? qpg + (size_t)i * nv : nullptr,
                                         qplu ? qplu + (size_t)i * 4 * nv : nullptr, du ? du + (size_t)i * nv : nullptr);
    if (threadIdx.x == 0) {
        up[2 * i] = up0;
        up[2 * i + 1] = up1;
        u[2 * i] = R.u0;
        u[2 * i + 1] = R.u1;
        if (iters) iters[i] = R.iters;
        if (st) st[i] = R.status;
    }
}

struct TrackShared {
    double Hs[256];
    double redd[2 * kWave];
    int redi[2 * kWave];
    double la[4];
};

// One agent per wave64: `iters` iterations of LQR.plan (lqr.py:58-86) / MPC.plan (mpc.py:66-94).
template <int KIND>
__global__ __launch_bounds__(kWave) void track_kernel(pmp_lp_params P, pmp_lqr_params L, pmp_mpc_params M, int na,
                                                      double* __restrict__ state, double* __restrict__ u_p,
                                                      const double* __restrict__ goal, const double* __restrict__ path_xy,
                                                      const int32_t* __restrict__ path_off, int iters,
                                                      double* __restrict__ u_out, int32_t* __restrict__ status_out,
                                                      int32_t* __restrict__ nsteps_out, double* __restrict__ hist_pose,
                                                      int32_t* __restrict__ admm_out)
{
    __shared__ TrackShared S;
    const int a = blockIdx.x;
    const int tid = threadIdx.x;
    if (a >= na) return;
    const double* path = path_xy + 2 * (size_t)path_off[a];
    const int Pn = path_off[a + 1] - path_off[a];
    const double gl[3] = {goal[3 * a], goal[3 * a + 1], goal[3 * a + 2]};
    double st[5];
    for (int k = 0; k < 5; k++) st[k] = state[5 * a + k];
    double up0 = 0.0, up1 = 0.0;
    if (KIND == PMP_TRACK_MPC) { up0 = u_p[2 * a]; up1 = u_p[2 * a + 1]; }
    const double dt = P.dt;
    int status = 0, steps = 0, admm = 0;
    double u0 = st[3], u1 = st[4];
    for (int it = 0; it < iters; it++) {
        if (lp::reach_goal(st, gl, P)) { status = PMP_FOUND + 1; break; }
        double pt[2] = {0, 0}, theta = 0, kappa = 0;
        const int ls = lp::lookahead_block(path, Pn, st[0], st[1], st[3], P, pt, &theta, &kappa, S.redd, S.redi);
        if (tid == 0) { S.la[0] = pt[0]; S.la[1] = pt[1]; S.la[2] = theta; S.la[3] = kappa; }
        __syncthreads();
        if (ls) { status = PMP_REF_RAISES; break; }
        pt[0] = S.la[0]; pt[1] = S.la[1]; theta = S.la[2]; kappa = S.la[3];
        __syncthreads();
        // calculate velocity command (lqr.py:67-83 / mpc.py:75-91)
        double e_theta = lp::regularize_angle(st[2] - gl[2]);
        const double angreg_w = st[4];
#define ANGREG(wd) lp::clampd(angreg_w + lp::clampd((wd) - angreg_w, P.min_w_inc, P.max_w_inc), P.min_w, P.max_w)
        if (!(lp::py_hypot(gl[0] - st[0], gl[1] - st[1]) > P.goal_dist_tol)) {
            u0 = 0.0;
            u1 = fabs(e_theta) > P.rotate_tol ? ANGREG(e_theta / dt) : 0.0;
        } else {
            e_theta = lp::regularize_angle(atan2(pt[1] - st[1], pt[0] - st[0]) - st[2]);
            if (fabs(e_theta) > P.rotate_tol) {
                u0 = 0.0;
                u1 = ANGREG(e_theta / dt);
            } else {
                const double s[3] = {st[0], st[1], st[2]}, sd[3] = {pt[0], pt[1], theta};
                const double ur[2] = {st[3], st[3] * kappa};
                if (KIND == PMP_TRACK_LQR) {
                    double uo[2];
                    lqr_control(s, sd, ur, st[3], st[4], P, L, uo);
                    u0 = uo[0];
                    u1 = uo[1];
                } else {
                    const MpcResult R = mpc_control_wave(s, sd, ur, up0, up1, st[3], st[4], P, M, S.Hs, nullptr,
                                                         nullptr, nullptr, nullptr);
                    u0 = R.u0;
                    u1 = R.u1;
                    admm += R.iters;
                }
            }
        }
#undef ANGREG
        if (tid == 0 && hist_pose) {
            double* hp = hist_pose + ((size_t)a * iters + it) * 3;
            hp[0] = st[0]; hp[1] = st[1]; hp[2] = st[2];
        }
        // Robot.kinematic -> lookforward (agent.py:68-116)
        double sn, cs;
        sincos(st[2], &sn, &cs);
        const double nx = st[0] + (dt * cs) * u0, ny = st[1] + (dt * sn) * u0, nth = st[2] + dt * u1;
        st[0] = nx; st[1] = ny; st[2] = nth; st[3] = u0; st[4] = u1;
        steps++;
    }
    if (tid == 0) {
        for (int k = 0; k < 5; k++) state[5 * a + k] = st[k];
        if (KIND == PMP_TRACK_MPC) { u_p[2 * a] = up0; u_p[2 * a + 1] = up1; }
        u_out[2 * a] = u0;
        u_out[2 * a + 1] = u1;
        status_out[a] = status;
        nsteps_out[a] = steps;
        if (admm_out) admm_out[a] = admm;
    }
}

int check_mpc(pmp_ctx* ctx, const pmp_mpc_params* mp, const char* who)
{
    if (mp->m < 1 || mp->m > 8 || mp->p < 1 || mp->p > 4096 || mp->max_iter < 1 || !(mp->rho > 0) ||
        !(mp->sigma >= 0) || !(mp->alpha > 0 && mp->alpha < 2) || mp->check_every < 0 || mp->adaptive_every < 0 ||
        !(mp->adaptive_tol >= 1))
        return pmp_set_err(ctx, PMP_EINVAL, std::string(who) + ": bad pmp_mpc_params (1 <= m <= 8, p >= 1, rho > 0, 0 < alpha < 2)");
    return PMP_OK;
}

}  // namespace

extern "C" int pmp_lqr_control_batch(pmp_ctx* ctx, void* stream, const pmp_lp_params* lp, const pmp_lqr_params* lq,
                                     int n, const double* s, const double* s_d, const double* u_r,
                                     const double* robot_vw, double* u)
{
    if (!ctx) return PMP_EINVAL;
    if (!lp || !lq || n < 0) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lqr_control_batch: bad params/n");
    if (n == 0) return PMP_OK;
    if (!s || !s_d || !u_r || !robot_vw || !u) return pmp_set_err(ctx, PMP_EINVAL, "pmp_lqr_control_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(lqr_control_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *lp, *lq, n, s, s_d,
                       u_r, robot_vw, u);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

extern "C" int pmp_mpc_control_batch(pmp_ctx* ctx, void* stream, const pmp_lp_params* lp, const pmp_mpc_params* mp,
                                     int n, const double* s, const double* s_d, const double* u_r, double* u_p,
                                     const double* robot_vw, double* u, double* qp_H, double* qp_g, double* qp_lu,
                                     double* du, int32_t* admm_iters, int32_t* admm_status)
{
    if (!ctx) return PMP_EINVAL;
    if (!lp || !mp || n < 0) return pmp_set_err(ctx, PMP_EINVAL, "pmp_mpc_control_batch: bad params/n");
    if (int rc = check_mpc(ctx, mp, "pmp_mpc_control_batch")) return rc;
    if (n == 0) return PMP_OK;
    if (!s || !s_d || !u_r || !u_p || !robot_vw || !u)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_mpc_control_batch: null pointer argument");
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(mpc_control_kernel, dim3(n), dim3(kWave), 0, (hipStream_t)stream, *lp, *mp, n, s, s_d, u_r, u_p,
                       robot_vw, u, qp_H, qp_g, qp_lu, du, admm_iters, admm_status);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

extern "C" int pmp_track_step_batch(pmp_ctx* ctx, void* stream, int kind, const pmp_lp_params* lp,
                                    const pmp_lqr_params* lq, const pmp_mpc_params* mp, int na, double* state,
                                    double* u_p, const double* goal, const double* path_xy, const int32_t* path_off,
                                    int iters, double* u, int32_t* status, int32_t* n_steps, double* hist_pose,
                                    int32_t* admm_iters)
{
    if (!ctx) return PMP_EINVAL;
    if (!lp || na < 0 || iters < 1 || (kind != PMP_TRACK_LQR && kind != PMP_TRACK_MPC))
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_track_step_batch: bad kind/params/na/iters");
    if (kind == PMP_TRACK_LQR && !lq) return pmp_set_err(ctx, PMP_EINVAL, "pmp_track_step_batch: LQR needs pmp_lqr_params");
    if (kind == PMP_TRACK_MPC) {
        if (!mp || !u_p) return pmp_set_err(ctx, PMP_EINVAL, "pmp_track_step_batch: MPC needs pmp_mpc_params and u_p");
        if (int rc = check_mpc(ctx, mp, "pmp_track_step_batch")) return rc;
    }
    if (na == 0) return PMP_OK;
    if (!state || !goal || !path_xy || !path_off || !u || !status || !n_steps)
        return pmp_set_err(ctx, PMP_EINVAL, "pmp_track_step_batch: null pointer argument");
    if (!(lp->dt > 0)) return pmp_set_err(ctx, PMP_EINVAL, "pmp_track_step_batch: dt must be > 0");
    const pmp_lqr_params L = lq ? *lq : pmp_lqr_params{};
    const pmp_mpc_params M = mp ? *mp : pmp_mpc_params{};
    PMP_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    if (kind == PMP_TRACK_LQR)
        hipLaunchKernelGGL(track_kernel<PMP_TRACK_LQR>, dim3(na), dim3(kWave), 0, (hipStream_t)stream, *lp, L, M, na,
                           state, u_p, goal, path_xy, path_off, iters, u, status, n_steps, hist_pose, admm_iters);
    else
        hipLaunchKernelGGL(track_kernel<PMP_TRACK_MPC>, dim3(na), dim3(kWave), 0, (hipStream_t)stream, *lp, L, M, na,
                           state, u_p, goal, path_xy, path_off, iters, u, status, n_steps, hist_pose, admm_iters);
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
