// Batched tracking controllers for gfx950: LQR.lqrControl (local_planner/lqr.py:103-145),
// MPC.mpcControl (local_planner/mpc.py:111-214) and whole LQR.plan / MPC.plan iterations
// (lqr.py:58-86, mpc.py:66-94).
//
// Four agents per wave64, one per 16-lane DPP row (the tracking loop, the lookahead scan, the
// ADMM); an agent's scalar work runs on all 16 lanes of its row.
//
// LQR: one 3x3 Riccati update per call (the signed exit of lqr.py:134 stops it after one update
// under the reference's defaults), 2x2 inverse, K e, with the structural zeros of A and B skipped.
//
// MPC:
//  - QP assembly in closed form.  A3 = I + N with N^2 = 0 (N = column 2 of lqr/mpc's A), so
//    A3^k = I + kN and the blocks of S_u are G_n = C A5^n B5 = sum_{k<=n} A3^k B3
//    = (n+1) B3 + n(n+1)/2 N B3; S_x's block i is [I + (i+1)N | G_i].
//  - H = S_u' Qbar S_u, y = S_x x and g = (S_u' Qbar) y on the f64 MFMA (v_mfma_f64_16x16x4_f64),
//    one pass per agent of the wave: lane l holds S_u[r = 4t + l/16][col = l%16] of the t-th K-slice,
//    A = q_r * S_u, B = S_u (H) or y (g); the 3p rows of S_u are the K dimension, so one 16x16
//    accumulator tile is the whole of H.  y comes out of a 16-row block MFMA of S_x against x already
//    in the B layout of the g product.
//  - ADMM (the OSQP algorithm, unscaled), on the agent's row: lane v owns variable v and constraint
//    rows v (the cumulative-sum rows of kron(tril(1_m), I2)) and 2m+v (the identity rows).  A x is
//    a stride-2 prefix scan, A'y a stride-2 suffix scan (DPP row_shr / row_shl); the x-update
//    multiplies by an explicit inverse of H + sigma I + rho A'A (LDS, column-major) with
//    row_newbcast broadcasts of the right-hand side, built by in-place Gauss-Jordan (rebuilt only
//    when rho adapts).  The ADMM's matrix-vector products have a different matrix per agent: as
//    MFMA tiles they would fill one column in 16 (and the f64 MFMA rate is the f64 VALU rate), so
//    the matrix cores carry the GEMM-shaped assembly only.
#include <utility>

#include "localplan.h"

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// LQR.lqrControl (lqr.py:103-145) + linear/angularRegularization (local_planner.py:172-206)
// ---------------------------------------------------------------------------------------------
// Structural zeros of lqr.py's A (I + dt v [-sin, cos, 0] in column 2) and B: the products below
// skip their terms (x * 0 added to a sum changes nothing but the sign of an exact zero), which keeps
// the loops' evaluation order for every other term and a third of the registers.
__device__ constexpr bool kAnz[3][3] = {{true, false, true}, {false, true, true}, {false, false, true}};
__device__ constexpr bool kBnz[3][2] = {{true, false}, {true, false}, {false, true}};

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
#define PMP_ADD_A(acc, x, k, j) if (kAnz[k][j]) acc += (x) * A[k][j]
#define PMP_ADD_B(acc, x, k, j) if (kBnz[k][j]) acc += (x) * B[k][j]
    for (int it = 0; it < L.iters; it++) {
        double PA[3][3], PB[3][2], APA[3][3], APB[3][2], BPB[2][2], BPA[2][3], S[2][2], Si[2][2];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) { PA[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_A(PA[i][j], Pm[i][k], k, j); }
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) { PB[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_B(PB[i][j], Pm[i][k], k, j); }
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) { APA[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_A(APA[i][j], PA[k][j], k, i); }
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) { APB[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_A(APB[i][j], PB[k][j], k, i); }
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) { BPB[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_B(BPB[i][j], PB[k][j], k, i); }
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) { BPA[i][j] = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) PMP_ADD_B(BPA[i][j], PA[k][j], k, i); }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++) S[i][j] = (i == j ? L.r[i] : 0.0) + BPB[i][j];
        const double det = S[0][0] * S[1][1] - S[0][1] * S[1][0];
        Si[0][0] = S[1][1] / det; Si[0][1] = -S[0][1] / det; Si[1][0] = -S[1][0] / det; Si[1][1] = S[0][0] / det;
        double mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
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
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) { PB[i][j] = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) PMP_ADD_B(PB[i][j], Pn[i][k], k, j); }
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) { PA[i][j] = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) PMP_ADD_A(PA[i][j], Pn[i][k], k, j); }
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) { BPB[i][j] = (i == j ? L.r[i] : 0.0);
#pragma unroll
            for (int k = 0; k < 3; k++) PMP_ADD_B(BPB[i][j], PB[k][j], k, i); }
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) { BPA[i][j] = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) PMP_ADD_B(BPA[i][j], PA[k][j], k, i); }
#undef PMP_ADD_A
#undef PMP_ADD_B
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
// Rows: four agents per wave64, one per 16-lane DPP row (lanes 16r .. 16r + 15, v = lane & 15).
// Cross-lane traffic stays inside a row: row_newbcast:k broadcasts lane k of each row, row_shr /
// row_shl shift within the row (bound_ctrl: a lane with no source reads 0), row_ror rotates.  f64
// values move as two 32-bit DPP halves.
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x)
{
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true); }
template <int K> __device__ __forceinline__ double bc16(double x) { return dpp_f64<0x150 + K>(x); }  // lane K of my row

template <typename F, int... K>
__device__ __forceinline__ void for16_impl(F&& f, std::integer_sequence<int, K...>)
{
    (f(std::integral_constant<int, K>{}), ...);
}
// f(std::integral_constant<int, k>) for k = 0 .. 15, unrolled with k a constant expression
template <typename F>
__device__ __forceinline__ void for16(F&& f) { for16_impl(f, std::make_integer_sequence<int, 16>{}); }

// inclusive prefix / suffix sum over the row's lanes of the same parity (stride-2 scans): the
// cumulative-sum rows of A = [kron(tril(1_m), I2); I] and A' on them
__device__ __forceinline__ double prefix16(double t)
{
    t += dpp_f64<0x112>(t);  // row_shr:2
    t += dpp_f64<0x114>(t);
    t += dpp_f64<0x118>(t);
    return t;
}
__device__ __forceinline__ double suffix16(double t)
{
    t += dpp_f64<0x102>(t);  // row_shl:2
    t += dpp_f64<0x104>(t);
    t += dpp_f64<0x108>(t);
    return t;
}
// max over the row, in every lane of the row (rotations: exact, order-free)
__device__ __forceinline__ double max16(double t)
{
    t = fmax(t, dpp_f64<0x128>(t));  // row_ror:8
    t = fmax(t, dpp_f64<0x124>(t));
    t = fmax(t, dpp_f64<0x122>(t));
    t = fmax(t, dpp_f64<0x121>(t));
    return t;
}

// Where the ADMM keeps the inverse: registers (one row per lane, the default) or LDS (column-major,
// 16 loads per x-update, 32 fewer live VGPRs: 26.2M vs 32.7M agent-steps/s at 8192 agents on the
// same box).  A build-time switch for A/B runs (-DPMP_MPC_INV_LDS=0|1, make invlds).
#ifndef PMP_MPC_INV_LDS
#define PMP_MPC_INV_LDS 0
#endif
constexpr bool kInvLds = PMP_MPC_INV_LDS != 0;

// Minv = (H + sigma I + rho A'A)^-1, row v in this lane (rows/cols >= n are the identity).
// A'A[2k+c][2k'+c'] = [c == c'] (m - max(k, k')) + [2k+c == 2k'+c'].
// In-place Gauss-Jordan without pivoting (the matrix is SPD): at step k the pivot row goes through
// `prow` (16 doubles of LDS for the row's agent) and column k is first reset to the identity's (1 in
// the pivot row, 0 elsewhere), so one 16-entry row per lane holds [M | I]'s live columns -- the same
// operations, value for value, as eliminating on M and I side by side.  k is a run-time loop: the
// elimination keeps only its own row live (an unrolled one lets the scheduler hoist every broadcast).
__device__ __forceinline__ void build_inverse(const double* Hrow, int v, int n, int m, double sigma, double rho,
                                              double* Icol, double* prow, double (&Ireg)[16])
{
    double Aloc[16];
    double (&A)[16] = kInvLds ? Aloc : Ireg;  // the register build eliminates in place
    // opaque to the optimiser: nothing of the build is hoisted out of the ADMM loop around it (the
    // hoisted H row and per-column constants would stay live through every iteration)
    asm volatile("" : "+v"(v) : : "memory");
#pragma unroll
    for (int c = 0; c < 16; c++) {
        const bool act = v < n && c < n;
        const int kv = v >> 1, kc = c >> 1;
        const double t = ((v & 1) == (c & 1)) ? (double)(m - (kv > kc ? kv : kc)) : 0.0;
        double val = (act ? Hrow[c] : 0.0) + rho * (t + (c == v ? 1.0 : 0.0)) + (c == v ? sigma : 0.0);
        A[c] = act ? val : (c == v ? 1.0 : 0.0);
    }
#pragma unroll 1
    for (int k = 0; k < 16; k++) {
        const bool piv = v == k;
        double f = A[0];
#pragma unroll
        for (int c = 1; c < 16; c++) f = c == k ? A[c] : f;
        if (piv) {
#pragma unroll
            for (int c = 0; c < 16; c++) prow[c] = A[c];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const double inv = 1.0 / prow[k];
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const double pc = c == k ? 1.0 : prow[c];
            const double ac = c == k ? (piv ? 1.0 : 0.0) : A[c];
            const double pr = pc * inv;
            A[c] = piv ? pr : ac - f * pr;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    // the inverse, column-major for the agent (column c at Icol[16 c]): the x-update's loads of one
    // column by the row's 16 lanes are one contiguous 128 B
    if (kInvLds) {
#pragma unroll
        for (int c = 0; c < 16; c++) Icol[16 * c + v] = A[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

struct MpcResult {
    double u0, u1;  // regularised control
    int iters, status;
};

// The MPC inputs of the row's agent (mpcControl's arguments, mpc.py:111-124)
struct MpcIn {
    double s[3], sd[3], ur[2], rv, rw;
};

constexpr int kRows = 4;  // agents per wave
// LDS doubles per wave of mpc_rows: an H per row, then a pivot row per row
// (an H per row, then a pivot row per row, then an inverse per row at a 264-double stride: the
// four rows' column loads fall in different LDS bank windows)
constexpr int kInvStride = 264;
constexpr int kMpcLds = kRows * 256 + kRows * 16 + (kInvLds ? kRows * kInvStride : 0);

// MPC.mpcControl (mpc.py:111-214) for the agents of the wave's four rows, called by the whole wave
// (the MFMA needs all lanes); `need` (row-uniform) selects the rows whose agent solves now, the other
// rows' outputs are left as they are.  up0/up1 in/out.  Hs: kMpcLds doubles of LDS (one H and one pivot row per row).
// Optional outputs already offset to the row's agent.
__device__ MpcResult mpc_rows(bool need, const MpcIn& I, double& up0, double& up1, const pmp_lp_params& P,
                              const pmp_mpc_params& M, double* Hs_all, double* qpH, double* qpg, double* qplu,
                              double* duo)
{
    const int lane = lane_id();
    const int v = lane & 15, row = lane >> 4;
    const int m = M.m, n = 2 * m, p = M.p;
    const double dt = P.dt;
    double sn, cs;
    sincos(I.sd[2], &sn, &cs);
    const double a0 = -I.ur[0] * sn * dt, a1 = I.ur[0] * cs * dt;  // A[0,2], A[1,2] (mpc.py:138-139)
    const double b00 = cs * dt, b10 = sn * dt;                     // B[0,0], B[1,0] (mpc.py:143-144)
    const double e0 = I.s[0] - I.sd[0], e1 = I.s[1] - I.sd[1], e2 = I.s[2] - I.sd[2];
    const double p0 = up0, p1 = up1;
    const uint64_t needm = ballot(need);

    // ---- H = S_u' Qbar S_u + R and g = (S_u' Qbar)(S_x x) (mpc.py:181-182, the reference's association:
    //      S_u' Q first, then times the vector S_x x - Yr, Yr = 0), all three products on the f64 MFMA
    //      (v_mfma_f64_16x16x4_f64), one pass per agent of the wave over 16-row blocks of S_u / S_x:
    //       - y = S_x[16 rows] x: A = the block of S_x (lane l: row l%16, column l/16, then 4 + l/16),
    //         B = x in every column, so register t of lane l holds y[4t + l/16] -- exactly the B operand
    //         the g product needs at the block's t-th K-slice;
    //       - per K-slice (4 rows r = 4t + l/16): A = q_r S_u[r][l%16] (S_u' Qbar), B = S_u[r][l%16]
    //         into the H tile, B = y into the g tile (every column of it holds g).
    //      The agent's closed-form parameters are broadcast from its row.
    const int col = lane & 15, kq = lane >> 4;
    const int jb = col >> 1, cb = col & 1;
    const int R3 = 3 * p;
    double gv = 0.0;
#pragma unroll 1
    for (int j = 0; j < 4; j++) {
        if (!((needm >> (16 * j)) & 1ull)) continue;
        const int L0 = 16 * j;
        const double A0 = rl_f64(a0, L0), A1 = rl_f64(a1, L0), B00 = rl_f64(b00, L0), B10 = rl_f64(b10, L0);
        const double E0 = rl_f64(e0, L0), E1 = rl_f64(e1, L0), E2 = rl_f64(e2, L0);
        const double P0 = rl_f64(p0, L0), P1 = rl_f64(p1, L0);
        // x = [e_x, e_y, e_theta, u_p0, u_p1] (mpc.py:128-134): row k of the B operand, k = l/16 (+ 4)
        const double xk0 = kq == 0 ? E0 : (kq == 1 ? E1 : (kq == 2 ? E2 : P0));
        const double xk1 = kq == 0 ? P1 : 0.0;
        v4d acc = {0.0, 0.0, 0.0, 0.0}, accg = {0.0, 0.0, 0.0, 0.0};

        for (int r0 = 0; r0 < R3; r0 += 16) {
            v4d y = {0.0, 0.0, 0.0, 0.0};
            {
                // S_x's block i (rows 3i .. 3i + 2) = C A^(i+1) = [I + (i+1) N | G_i]:
                //   [1, 0, (i+1) A02, (i+1) B00, i(i+1)/2 A02 dt], [0, 1, (i+1) A12, (i+1) B10, i(i+1)/2 A12 dt],
                //   [0, 0, 1, 0, (i+1) dt]
                const int r = r0 + col;
                double s0 = 0.0, s1 = 0.0;  // S_x[r][kq], S_x[r][4 + kq]
                if (r < R3) {
                    const int i = r / 3, d = r - 3 * i;
                    const double n1 = (double)(i + 1), tri = 0.5 * (double)i * (double)(i + 1);
                    if (d == 0) {
                        s0 = kq == 0 ? 1.0 : (kq == 1 ? 0.0 : (kq == 2 ? n1 * A0 : n1 * B00));
                        s1 = kq == 0 ? (tri * A0 * dt) : 0.0;
                    } else if (d == 1) {
                        s0 = kq == 0 ? 0.0 : (kq == 1 ? 1.0 : (kq == 2 ? n1 * A1 : n1 * B10));
                        s1 = kq == 0 ? (tri * A1 * dt) : 0.0;
                    } else {
                        s0 = kq == 2 ? 1.0 : 0.0;
                        s1 = kq == 0 ? n1 * dt : 0.0;
                    }
                }
                y = __builtin_amdgcn_mfma_f64_16x16x4f64(s0, xk0, y, 0, 0, 0);
                y = __builtin_amdgcn_mfma_f64_16x16x4f64(s1, xk1, y, 0, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int r = r0 + 4 * t + kq;
                double sv = 0.0, qv = 0.0;
                if (r < R3) {
                    const int i = r / 3, d = r - 3 * i;
                    qv = d == 0 ? M.q[0] : (d == 1 ? M.q[1] : M.q[2]);
                    if (col < n && jb <= i) {
                        const int nn = i - jb;
                        const double m1 = (double)(nn + 1), tr = 0.5 * (double)nn * (double)(nn + 1);
                        if (cb == 0)
                            sv = d == 0 ? m1 * B00 : (d == 1 ? m1 * B10 : 0.0);
                        else
                            sv = d == 0 ? tr * A0 * dt : (d == 1 ? tr * A1 * dt : m1 * dt);
                    }
                }
                const double av = qv * sv;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, sv, acc, 0, 0, 0);
                accg = __builtin_amdgcn_mfma_f64_16x16x4f64(av, y[t], accg, 0, 0, 0);
            }
        }
        // g tile: register t of lane l holds g[l/16 + 4t] (every column); lane v of row j takes g[v]
        {
            const int src = 16 * (col & 3) + col;
            double gg = 0.0;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const double w = __shfl(accg[t], src);
                if ((col >> 2) == t) gg = w;
            }
            if (row == j) gv = gg;
        }
        // D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = lane/16 + 4*reg
        double* Hs = Hs_all + 256 * j;
#pragma unroll
        for (int rg = 0; rg < 4; rg++) {
            const int hr = kq + 4 * rg;
            double h = acc[rg];
            if (hr == col && hr < n) h += (hr & 1) ? M.r[1] : M.r[0];
            Hs[hr * 16 + col] = h;
        }
    }
    __syncthreads();

    MpcResult R;
    R.u0 = R.u1 = 0.0;
    R.iters = 0;
    R.status = 1;
    double x = 0.0;
    if (need) {
        const bool act = v < n;  // lanes 0..15 of the row: variable v, constraint rows v and n+v
        const int cv = v & 1;
        gv = act ? gv : 0.0;
        const double l1 = act ? (cv ? P.min_w - p1 : P.min_v - p0) : 0.0;  // U_min - U_k_1
        const double h1 = act ? (cv ? P.max_w - p1 : P.max_v - p0) : 0.0;
        const double l2 = act ? (cv ? P.min_w_inc : P.min_v_inc) : 0.0;    // dU_min
        const double h2 = act ? (cv ? P.max_w_inc : P.max_v_inc) : 0.0;
        const double* Hs = Hs_all + 256 * row;
        if (qpH)
            for (int idx = v; idx < n * n; idx += 16) qpH[idx] = Hs[(idx / n) * 16 + idx % n];
        if (qpg && act) qpg[v] = gv;
        if (qplu && act) {
            qplu[v] = l1; qplu[n + v] = l2;
            qplu[2 * n + v] = h1; qplu[3 * n + v] = h2;
        }
        // this lane's row of H stays in LDS through the ADMM (read by the inverse builds and the
        // residual checks)
        const double* Hrow = Hs + 16 * v;
        double* prow = Hs_all + kRows * 256 + 16 * row;  // the agent's pivot row
        double* Icol = Hs_all + kRows * 256 + kRows * 16 + kInvStride * row;  // the agent's inverse

        // ---- ADMM (the OSQP algorithm, unscaled), the row's agent: rows finish independently
        double rho = M.rho;
        const double sigma = M.sigma, alpha = M.alpha;
        double Ireg[16];
        build_inverse(Hrow, v, n, m, sigma, rho, Icol, prow, Ireg);
        double z1 = 0.0, z2 = 0.0, y1 = 0.0, y2 = 0.0;
        int status = 1, it = 0, cnt_c = 0, cnt_a = 0;
        while (it < M.max_iter) {
            it++;
            cnt_c++;
            cnt_a++;
            const double rinv = 1.0 / rho;
            const double w1 = act ? rho * z1 - y1 : 0.0, w2 = act ? rho * z2 - y2 : 0.0;
            const double rhs = sigma * x - gv + (suffix16(w1) + w2);
            double xt = 0.0;
            for16([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                xt += (kInvLds ? Icol[16 * c + v] : Ireg[c]) * bc16<c>(rhs);
            });
            xt = act ? xt : 0.0;
            const double zt1 = prefix16(xt);
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
            // residuals (unscaled inf norms, OSQP's termination test); H re-read here, not kept live
            asm volatile("" : : : "memory");
            const double ax1 = prefix16(x), ax2 = x;
            double hx = 0.0;
            for16([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                hx += (act && c < n ? Hrow[c] : 0.0) * bc16<c>(x);
            });
            const double aty = suffix16(y1) + y2;
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
                    build_inverse(Hrow, v, n, m, sigma, rho, Icol, prow, Ireg);
                }
            }
        }
        if (duo && act) duo[v] = x;
        const double du0 = bc16<0>(x), du1 = bc16<1>(x);
        const double uu0 = (du0 + p0) + I.ur[0], uu1 = (du1 + p1) + I.ur[1];
        up0 = uu0 - I.ur[0];
        up1 = uu1 - I.ur[1];
        R.u0 = lp::clampd(I.rv + lp::clampd(uu0 - I.rv, P.min_v_inc, P.max_v_inc), P.min_v, P.max_v);
        R.u1 = lp::clampd(I.rw + lp::clampd(uu1 - I.rw, P.min_w_inc, P.max_w_inc), P.min_w, P.max_w);
        R.iters = it;
        R.status = status;
    }
    __syncthreads();  // Hs is reused by the next call
    return R;
}

// getLookaheadPoint (local_planner.py:103-170) for the row's agent: the distance scan, the
// first-index argmin and the first-beyond-lookahead search over the row's 16 lanes (stride 16), the
// tail on every lane of the row (same inputs, same result).  Called with the whole row active.
__device__ __forceinline__ void row_best_min(double& v, int& i)
{
    // (v, i) minimum with ties to the lowest i, over the row (rotations)
#define PMP_ROW_STEP(CTRL)                                                        \
    {                                                                             \
        const double ov = dpp_f64<CTRL>(v);                                       \
        const int oi = dpp_i32<CTRL>(i);                                          \
        if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }                    \
    }
    PMP_ROW_STEP(0x128) PMP_ROW_STEP(0x124) PMP_ROW_STEP(0x122) PMP_ROW_STEP(0x121)
#undef PMP_ROW_STEP
}
__device__ inline int lookahead_row(const double* path, int P, double rx, double ry, double v, const pmp_lp_params& Pm,
                                    double* pt, double* theta, double* kappa)
{
    const int r = lane_id() & 15;
    const double L = lp::lookahead_dist(v, Pm);
    // idx_closest = dist_to_robot.index(min(dist_to_robot))
    double bd = INFINITY;
    int bi = 0x7fffffff;
#pragma unroll 1
    for (int i = r; i < P; i += 16) {
        const double d = lp::py_hypot(rx - path[2 * i], ry - path[2 * i + 1]);
        if (d < bd) { bd = d; bi = i; }  // strided in increasing i: keeps the first minimum
    }
    row_best_min(bd, bi);
    const int idx_closest = bi;
    // first i >= idx_closest with dist >= L
    int fi = 0x7fffffff;
#pragma unroll 1
    for (int i = idx_closest + r; i < P; i += 16) {
        if (lp::py_hypot(rx - path[2 * i], ry - path[2 * i + 1]) >= L) { fi = i; break; }
    }
    double fd = 0.0;
    row_best_min(fd, fi);
    const int idx_goal = fi == 0x7fffffff ? P - 1 : fi;
    return lp::lookahead_tail(path, P, rx, ry, L, idx_goal, pt, theta, kappa);
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

// four agents per wave (one per row): MPC.mpcControl for agent 4 * block + row
__global__ __launch_bounds__(kWave) void mpc_control_kernel(pmp_lp_params P, pmp_mpc_params M, int n,
                                                            const double* __restrict__ s, const double* __restrict__ sd,
                                                            const double* __restrict__ ur, double* __restrict__ up,
                                                            const double* __restrict__ vw, double* __restrict__ u,
                                                            double* __restrict__ qpH, double* __restrict__ qpg,
                                                            double* __restrict__ qplu, double* __restrict__ du,
                                                            int32_t* __restrict__ iters, int32_t* __restrict__ st)
{
    __shared__ double Hs[kMpcLds];
    const int v = threadIdx.x & 15;
    const int i = blockIdx.x * kRows + (threadIdx.x >> 4);
    const bool valid = i < n;
    const int ic = valid ? i : n - 1;  // rows past the batch read a real agent and write nothing
    const int nv = 2 * M.m;
    MpcIn I;
    for (int k = 0; k < 3; k++) { I.s[k] = s[3 * ic + k]; I.sd[k] = sd[3 * ic + k]; }
    I.ur[0] = ur[2 * ic]; I.ur[1] = ur[2 * ic + 1];
    I.rv = vw[2 * ic]; I.rw = vw[2 * ic + 1];
    double up0 = up[2 * ic], up1 = up[2 * ic + 1];
    const MpcResult R = mpc_rows(valid, I, up0, up1, P, M, Hs,
                                 (qpH && valid) ? qpH + (size_t)i * nv * nv : nullptr,
                                 (qpg && valid) ? qpg + (size_t)i * nv : nullptr,
                                 (qplu && valid) ? qplu + (size_t)i * 4 * nv : nullptr,
                                 (du && valid) ? du + (size_t)i * nv : nullptr);
    if (valid && v == 0) {
        up[2 * i] = up0;
        up[2 * i + 1] = up1;
        u[2 * i] = R.u0;
        u[2 * i + 1] = R.u1;
        if (iters) iters[i] = R.iters;
        if (st) st[i] = R.status;
    }
}

// Four agents per wave (one per row): `iters` iterations of LQR.plan (lqr.py:58-86) / MPC.plan
// (mpc.py:66-94) for agent 4 * block + row.  Control flow is per row; the MPC solve is entered by the
// whole wave with the rows that solve in this iteration flagged.
template <int KIND>
__global__ __launch_bounds__(kWave) void track_kernel(pmp_lp_params P, pmp_lqr_params L, pmp_mpc_params M, int na,
                                                      double* __restrict__ state, double* __restrict__ u_p,
                                                      const double* __restrict__ goal, const double* __restrict__ path_xy,
                                                      const int32_t* __restrict__ path_off, int iters,
                                                      double* __restrict__ u_out, int32_t* __restrict__ status_out,
                                                      int32_t* __restrict__ nsteps_out, double* __restrict__ hist_pose,
                                                      int32_t* __restrict__ admm_out)
{
    __shared__ double Hs[KIND == PMP_TRACK_MPC ? kMpcLds : 1];
    const int v = threadIdx.x & 15;
    const int ai = blockIdx.x * kRows + (threadIdx.x >> 4);
    const bool valid = ai < na;
    const int a = valid ? ai : na - 1;
    const double* path = path_xy + 2 * (size_t)path_off[a];
    const int Pn = path_off[a + 1] - path_off[a];
    const double gl[3] = {goal[3 * a], goal[3 * a + 1], goal[3 * a + 2]};
    double st[5];
    for (int k = 0; k < 5; k++) st[k] = state[5 * a + k];
    double up0 = 0.0, up1 = 0.0;
    if (KIND == PMP_TRACK_MPC) { up0 = u_p[2 * a]; up1 = u_p[2 * a + 1]; }
    const double dt = P.dt;
    int status = 0, steps = 0, admm = 0;
    bool live = valid;  // row-uniform: the agent still iterates
    double u0 = st[3], u1 = st[4];
    for (int it = 0; it < iters; it++) {
        if (!ballot(live)) break;
        bool solve = false;
        MpcIn I;
        if (live) {
            if (lp::reach_goal(st, gl, P)) {
                status = PMP_FOUND + 1;
                live = false;
            } else {
                double pt[2] = {0, 0}, theta = 0, kappa = 0;
                if (lookahead_row(path, Pn, st[0], st[1], st[3], P, pt, &theta, &kappa)) {
                    status = PMP_REF_RAISES;
                    live = false;
                } else {
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
                            I.s[0] = st[0]; I.s[1] = st[1]; I.s[2] = st[2];
                            I.sd[0] = pt[0]; I.sd[1] = pt[1]; I.sd[2] = theta;
                            I.ur[0] = st[3]; I.ur[1] = st[3] * kappa;
                            I.rv = st[3]; I.rw = st[4];
                            if (KIND == PMP_TRACK_LQR) {
                                double uo[2];
                                lqr_control(I.s, I.sd, I.ur, I.rv, I.rw, P, L, uo);
                                u0 = uo[0];
                                u1 = uo[1];
                            } else {
                                solve = true;
                            }
                        }
                    }
#undef ANGREG
                }
            }
        }
        if (KIND == PMP_TRACK_MPC) {
            if (ballot(solve)) {
                if (!solve) {  // rows not solving carry harmless inputs through the wave-wide assembly
                    for (int k = 0; k < 3; k++) { I.s[k] = 0.0; I.sd[k] = 0.0; }
                    I.ur[0] = I.ur[1] = I.rv = I.rw = 0.0;
                }
                double q0 = up0, q1 = up1;
                const MpcResult R = mpc_rows(solve, I, q0, q1, P, M, Hs, nullptr, nullptr, nullptr, nullptr);
                if (solve) {
                    up0 = q0;
                    up1 = q1;
                    u0 = R.u0;
                    u1 = R.u1;
                    admm += R.iters;
                }
            }
        }
        if (live) {
            if (v == 0 && hist_pose) {
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
    }
    if (valid && v == 0) {
        for (int k = 0; k < 5; k++) state[5 * a + k] = st[k];
        if (KIND == PMP_TRACK_MPC) { u_p[2 * a] = up0; u_p[2 * a + 1] = up1; }
        u_out[2 * a] = u0;
        u_out[2 * a + 1] = u1;
        status_out[a] = status;
        nsteps_out[a] = steps;
        if (admm_out) admm_out[a] = admm;
    }
}

// MPC.plan split at the solve, so each part keeps its own register budget (the fused loop needs the
// lookahead's and the ADMM's registers at once: 1 wave per SIMD).  Per iteration `it`:
// track_mpc_step (the kinematics of iteration it-1 for the agents that moved, then iteration it's
// reachGoal / getLookaheadPoint / rotate-or-track branch) and track_mpc_solve (mpcControl for the
// agents whose branch needs it); a last track_mpc_step (it = iters) applies the final kinematics.
// Per-agent carry between the launches: the MPC inputs (10 doubles), a flag word and the ADMM count.
enum : int { kLive = 1, kSolve = 2, kMove = 4 };
struct TrackCarry {
    double* in;    // [na][10]: s[3], sd[3], ur[2], rv, rw
    int32_t* flag;  // [na]
    int32_t* admm;  // [na]
    unsigned long long* stats;  // nullable (pmp_set_stats): [0] += QP solves
};

__global__ __launch_bounds__(kWave) void track_mpc_step(pmp_lp_params P, int na, int it, int iters,
                                                        double* __restrict__ state, const double* __restrict__ goal,
                                                        const double* __restrict__ path_xy,
                                                        const int32_t* __restrict__ path_off, double* __restrict__ u_out,
                                                        int32_t* __restrict__ status_out, int32_t* __restrict__ nsteps_out,
                                                        double* __restrict__ hist_pose, int32_t* __restrict__ admm_out,
                                                        TrackCarry C)
{
    const int v = threadIdx.x & 15;
    const int a = blockIdx.x * kRows + (threadIdx.x >> 4);
    if (a >= na) return;  // row-uniform: no cross-row work below
    const double dt = P.dt;
    double st[5];
    for (int k = 0; k < 5; k++) st[k] = state[5 * a + k];
    int flag, status, steps;
    double u0, u1;
    if (it == 0) {
        flag = kLive;
        status = steps = 0;
        u0 = st[3];
        u1 = st[4];
    } else {
        flag = C.flag[a];
        status = status_out[a];
        steps = nsteps_out[a];
        u0 = u_out[2 * a];
        u1 = u_out[2 * a + 1];
    }
    if (flag & kMove) {  // Robot.kinematic -> lookforward (agent.py:68-116) of iteration it - 1
        if (v == 0 && hist_pose) {
            double* hp = hist_pose + ((size_t)a * iters + (it - 1)) * 3;
            hp[0] = st[0]; hp[1] = st[1]; hp[2] = st[2];
        }
        double sn, cs;
        sincos(st[2], &sn, &cs);
        const double nx = st[0] + (dt * cs) * u0, ny = st[1] + (dt * sn) * u0, nth = st[2] + dt * u1;
        st[0] = nx; st[1] = ny; st[2] = nth; st[3] = u0; st[4] = u1;
        steps++;
    }
    flag &= kLive;
    double in[10];
    if (it < iters && (flag & kLive)) {
        const double* path = path_xy + 2 * (size_t)path_off[a];
        const int Pn = path_off[a + 1] - path_off[a];
        const double gl[3] = {goal[3 * a], goal[3 * a + 1], goal[3 * a + 2]};
        if (lp::reach_goal(st, gl, P)) {
            status = PMP_FOUND + 1;
            flag = 0;
        } else {
            double pt[2] = {0, 0}, theta = 0, kappa = 0;
            if (lookahead_row(path, Pn, st[0], st[1], st[3], P, pt, &theta, &kappa)) {
                status = PMP_REF_RAISES;
                flag = 0;
            } else {
                // calculate velocity command (mpc.py:75-91)
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
                        in[0] = st[0]; in[1] = st[1]; in[2] = st[2];
                        in[3] = pt[0]; in[4] = pt[1]; in[5] = theta;
                        in[6] = st[3]; in[7] = st[3] * kappa;
                        in[8] = st[3]; in[9] = st[4];
                        flag |= kSolve;
                    }
                }
#undef ANGREG
                flag |= kMove;
            }
        }
    }
    if (v == 0) {
        for (int k = 0; k < 5; k++) state[5 * a + k] = st[k];
        u_out[2 * a] = u0;
        u_out[2 * a + 1] = u1;
        status_out[a] = status;
        nsteps_out[a] = steps;
        C.flag[a] = flag;
        if (flag & kSolve)
            for (int k = 0; k < 10; k++) C.in[10 * (size_t)a + k] = in[k];
        if (it == 0) C.admm[a] = 0;
        if (it == iters && admm_out) admm_out[a] = C.admm[a];
    }
}

__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(3))) void track_mpc_solve(pmp_lp_params P, pmp_mpc_params M, int na,
                                                         double* __restrict__ u_p, double* __restrict__ u_out,
                                                         TrackCarry C)
{
    __shared__ double Hs[kMpcLds];
    const int v = threadIdx.x & 15;
    const int ai = blockIdx.x * kRows + (threadIdx.x >> 4);
    const bool valid = ai < na;
    const int a = valid ? ai : na - 1;
    const bool solve = valid && (C.flag[a] & kSolve) != 0;
    const uint64_t sm = ballot(solve && v == 0);
    if (!sm) return;  // wave-uniform
    if (C.stats && threadIdx.x == 0) atomicAdd(C.stats, (unsigned long long)__popcll(sm));
    MpcIn I;
    const double* in = C.in + 10 * (size_t)a;
    if (solve) {
        for (int k = 0; k < 3; k++) { I.s[k] = in[k]; I.sd[k] = in[3 + k]; }
        I.ur[0] = in[6]; I.ur[1] = in[7]; I.rv = in[8]; I.rw = in[9];
    } else {  // rows not solving carry harmless inputs through the wave-wide assembly
        for (int k = 0; k < 3; k++) { I.s[k] = 0.0; I.sd[k] = 0.0; }
        I.ur[0] = I.ur[1] = I.rv = I.rw = 0.0;
    }
    double up0 = u_p[2 * a], up1 = u_p[2 * a + 1];
    const MpcResult R = mpc_rows(solve, I, up0, up1, P, M, Hs, nullptr, nullptr, nullptr, nullptr);
    if (solve && v == 0) {
        u_p[2 * a] = up0;
        u_p[2 * a + 1] = up1;
        u_out[2 * a] = R.u0;
        u_out[2 * a + 1] = R.u1;
        C.admm[a] += R.iters;
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
    hipLaunchKernelGGL(mpc_control_kernel, dim3((n + kRows - 1) / kRows), dim3(kWave), 0, (hipStream_t)stream, *lp, *mp, n, s, s_d, u_r, u_p,
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
        hipLaunchKernelGGL(track_kernel<PMP_TRACK_LQR>, dim3((na + kRows - 1) / kRows), dim3(kWave), 0, (hipStream_t)stream, *lp, L, M, na,
                           state, u_p, goal, path_xy, path_off, iters, u, status, n_steps, hist_pose, admm_iters);
    else {
        // MPC: 2 iters + 1 launches (track_mpc_step / track_mpc_solve per iteration, a last step)
        TrackCarry C;
        const size_t nb = (size_t)na;
        char* scr = (char*)pmp_scratch(ctx, SCR_AUX4, nb * 80 + nb * 8 + 64);
        if (!scr) return PMP_ENOMEM;
        C.in = (double*)scr;
        C.flag = (int32_t*)(scr + nb * 80);
        C.admm = C.flag + nb;
        C.stats = ctx->stats;
        const dim3 grid((na + kRows - 1) / kRows);
        hipStream_t s = (hipStream_t)stream;
        for (int it = 0; it <= iters; it++) {
            hipLaunchKernelGGL(track_mpc_step, grid, dim3(kWave), 0, s, *lp, na, it, iters, state, goal, path_xy, path_off,
                               u, status, n_steps, hist_pose, admm_iters, C);
            if (it < iters) hipLaunchKernelGGL(track_mpc_solve, grid, dim3(kWave), 0, s, *lp, M, na, u_p, u, C);
        }
    }
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}
