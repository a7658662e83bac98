// sqp_rti_lane.hip -- batched SQP-RTI step, one wavefront lane per robot instance.
//
// Replaces the acados-generated {diff2amr,omni4amr,tric3amr}_acados_solve() call
// (src/nmpc_nav_control/NMPCNavControlDiff.cpp:142, NMPCNavControlOmni4.cpp:139, NMPCNavControlTric.cpp:146)
// for B independent instances at once. One lane owns one instance: linearisation (RK4 + forward
// sensitivities), Gauss-Newton cost, box bounds, then a Mehrotra predictor-corrector interior-point
// method whose Newton systems are solved by a Riccati recursion over the N-stage OCP-QP (no
// condensing: qp_solver_cond_N = N). Same algorithm as oracle/nmpc_oracle.c (fp64), here in fp32.
//
// Every per-stage quantity lives in a structure-of-arrays scratch buffer [stage][field][lane] so the
// 64 lanes of a wave read and write 256 contiguous bytes per field access.
//
// Mode RUN additionally fuses the wrapper pre/post of NMPCNavControl*::run():
//   pre  (NMPCNavControlDiff.cpp:87-139): x0 from pose + direct kinematics + carried ref states,
//        yref theta unwrap + padding, diff terminal-weight hack;
//   post (NMPCNavControlDiff.cpp:145-172): vel_ref_new = x0[ref] + u0*dt, inverse kinematics -> cmd,
//        carried ref states for the next tick.
#include "nmpc_kernels.hpp"

namespace nmpc {

template <class M>
struct LaneLayout {
    static constexpr int NX = M::NX, NU = M::NU, NBX = M::NBX, NBU = M::NBU, NB = NBX + NBU;
    // per-stage field offsets (floats)
    static constexpr int A = 0;
    static constexpr int Bm = A + NX * NX;
    static constexpr int LXU = Bm + NX * NU;  // Riccati factor block Lxu (NX x NU)
    static constexpr int LUU = LXU + NX * NU; // Riccati factor block Luu (NU x NU, lower)
    static constexpr int LR = LUU + NU * NU;  // Luu^{-1} (g^u + B'p) of the current rhs
    static constexpr int DU = LR + NU;
    static constexpr int DX = DU + NU;
    static constexpr int DDU = DX + NX;
    static constexpr int DDX = DDU + NU;
    static constexpr int GU = DDX + NX;
    static constexpr int GX = GU + NU;
    static constexpr int RU = GX + NX;
    static constexpr int LB = RU + NU;
    static constexpr int UB = LB + NB;
    static constexpr int TL = UB + NB;
    static constexpr int TU = TL + NB;
    static constexpr int LL = TU + NB;
    static constexpr int LU = LL + NB;
    static constexpr int DZA = LU + NB;
    static constexpr int YR = DZA + NB;  // unwrapped pose reference x, y, theta (RUN mode)
    static constexpr int NF = YR + 3;
};

template <class M>
size_t lane_scratch_floats(int N, int stride)
{
    return (size_t)(N + 1) * LaneLayout<M>::NF * stride;
}

namespace {

constexpr float kBreakdownMu = 1e-6f;
constexpr float kStatRel = 1e-5f;  // ~100 ulp of fp32
constexpr float kCompMaxRatio = 30.0f;  // largest complementarity product at exit / tol_comp (sqp_rti_team.hip)

// max that propagates NaN (fmaxf drops it)
__device__ inline float nan_max(float a, float b) { return (b > a || b != b) ? b : a; }

// Per-comp variable of stage k: comps [0, NBU) are u[idxbu], [NBU, NB) are x[idxbx].
template <class M>
__device__ inline bool comp_active(int c, int k, int N)
{
    return (c < M::NBU) ? (k < N) : (k >= 1);
}

// Forward substitution of the square-root Riccati: Du = -Luu^{-T} (Lxu' Dx + lr).
template <class M, class Lay>
__device__ inline void forward_du(const float* __restrict__ scr, int k, size_t S, const float (&Dx)[M::NX],
                                  float (&Du)[M::NU])
{
    constexpr int NX = M::NX, NU = M::NU, NF = Lay::NF;
    float w[NU];
#pragma unroll
    for (int i = 0; i < NU; i++) {
        float s = scr[((size_t)k * NF + Lay::LR + i) * S];
        if (k >= 1) {
#pragma unroll
            for (int j = 0; j < NX; j++) s += scr[((size_t)k * NF + Lay::LXU + j * NU + i) * S] * Dx[j];
        }
        w[i] = s;
    }
#pragma unroll
    for (int ii = 0; ii < NU; ii++) {
        const int i = NU - 1 - ii;
        float s = w[i];
#pragma unroll
        for (int q = i + 1; q < NU; q++) s -= scr[((size_t)k * NF + Lay::LUU + q * NU + i) * S] * Du[q];
        Du[i] = s / scr[((size_t)k * NF + Lay::LUU + i * NU + i) * S];
    }
#pragma unroll
    for (int i = 0; i < NU; i++) Du[i] = -Du[i];
}

template <class M>
__global__ __launch_bounds__(64, 1) void k_sqp_rti_lane(KParams P, KArgs a, int mode)
{
    using Lay = LaneLayout<M>;
    constexpr int NX = M::NX, NU = M::NU, NBU = M::NBU, NB = Lay::NB;
    constexpr int NF = Lay::NF;
    const int inst = blockIdx.x * blockDim.x + threadIdx.x;
    if (inst >= a.B) return;
    const int N = P.N;
    const size_t S = (size_t)a.stride;
    const size_t Bn = (size_t)a.B;
    float* __restrict__ scr = a.scratch + inst;
    float* __restrict__ xbar = a.xbar + inst;
    float* __restrict__ ubar = a.ubar + inst;
#define FLD(k, f) scr[((size_t)(k) * NF + (f)) * S]
#define XB(k, j) xbar[((size_t)(k) * NX + (j)) * S]
#define UB(k, j) ubar[((size_t)(k) * NU + (j)) * S]

    // ---- reset ({name}_acados_reset: zero iterate) -------------------------------------------------
    if (a.reset && a.reset[inst]) {
        for (int k = 0; k <= N; k++)
            for (int j = 0; j < NX; j++) XB(k, j) = 0.0f;
        for (int k = 0; k < N; k++)
            for (int j = 0; j < NU; j++) UB(k, j) = 0.0f;
    }

    // ---- x0 -----------------------------------------------------------------------------------------
    float x0[NX];
    float pose_th = 0.0f;
    if (mode == kModeRun) {
        const float pose[3] = {a.pose[inst], a.pose[Bn + inst], a.pose[2 * Bn + inst]};
        const float vel[3] = {a.vel[inst], a.vel[Bn + inst], a.vel[2 * Bn + inst]};
        const float steer = a.steer ? a.steer[inst] : 0.0f;
        x0[0] = pose[0];
        x0[1] = pose[1];
        x0[2] = pose[2];
        pose_th = pose[2];
        M::direct_kin(vel, steer, P, x0 + 3);
#pragma unroll
        for (int i = 0; i < M::NBX; i++) x0[M::idxbx(i)] = a.carried[(size_t)i * S + inst];
    } else {
#pragma unroll
        for (int j = 0; j < NX; j++) x0[j] = a.x0[(size_t)j * Bn + inst];
    }

    // yref accessor: RUN mode reads the unwrapped pose reference staged in scratch (entries >= 3 are 0,
    // SURVEY Appendix C.3); SOLVE mode reads the caller's [N+1][ny_in][B] array (entries >= ny_in are 0).
    auto yref = [&](int k, int j) -> float {
        if (mode == kModeRun) return (j < 3) ? FLD(k, Lay::YR + j) : 0.0f;
        return (j < a.ny_in) ? a.yref[((size_t)k * a.ny_in + j) * Bn + inst] : 0.0f;
    };
    if (mode == kModeRun) {
        // theta unwrap against the previous entry and padding with the last pose (NMPCNavControlDiff.cpp:104-118)
        const int len = a.traj_len ? a.traj_len[inst] : N + 1;
        float prev = pose_th, px = 0.0f, py = 0.0f;
        for (int k = 0; k <= N; k++) {
            if (k < len) {
                px = a.traj[((size_t)k * 3 + 0) * Bn + inst];
                py = a.traj[((size_t)k * 3 + 1) * Bn + inst];
                float th = a.traj[((size_t)k * 3 + 2) * Bn + inst];
                const float d = th - prev;
                if (d > kPi) th -= 2.0f * kPi;
                else if (d < -kPi) th += 2.0f * kPi;
                prev = th;
            }
            FLD(k, Lay::YR + 0) = px;
            FLD(k, Lay::YR + 1) = py;
            FLD(k, Lay::YR + 2) = prev;
        }
    }
    // terminal weight
    float We[NX];
#pragma unroll
    for (int j = 0; j < NX; j++) We[j] = (a.We) ? a.We[(size_t)j * Bn + inst] : P.We[j];
    if (mode == kModeRun && P.terminal_hack) {
        // NMPCNavControlDiff.cpp:127-139
        const bool eq = (yref(N, 0) == yref(N - 1, 0)) && (yref(N, 1) == yref(N - 1, 1)) &&
                        (yref(N, 2) == yref(N - 1, 2));
#pragma unroll
        for (int j = 0; j < 3; j++) We[j] = eq ? 100.0f * P.W[j] : P.W[j];
    }

    // ---- linearisation + QP data + IPM initial point (forward over stages) -------------------------
    const float sc = P.dt;  // cost scaling on stages 0..N-1
    float dxk[NX];
#pragma unroll
    for (int j = 0; j < NX; j++) dxk[j] = x0[j] - XB(0, j);
    int m = 0;
    for (int k = 0; k <= N; k++) {
        float xb[NX], ub[NU];
#pragma unroll
        for (int j = 0; j < NX; j++) xb[j] = XB(k, j);
#pragma unroll
        for (int j = 0; j < NX; j++) FLD(k, Lay::DX + j) = dxk[j];
        if (k < N) {
#pragma unroll
            for (int j = 0; j < NU; j++) {
                ub[j] = UB(k, j);
                FLD(k, Lay::DU + j) = 0.0f;
                FLD(k, Lay::GU + j) = sc * P.W[NX + j] * (ub[j] - yref(k, NX + j));
            }
        }
        if (k >= 1) {
#pragma unroll
            for (int j = 0; j < NX; j++)
                FLD(k, Lay::GX + j) = (k < N) ? sc * P.W[j] * (xb[j] - yref(k, j)) : We[j] * (xb[j] - yref(k, j));
        }
        // bounds and initial slacks / multipliers
#pragma unroll
        for (int c = 0; c < NB; c++) {
            if (!comp_active<M>(c, k, N)) continue;
            float lb, ubd, z;
            if (c < NBU) {
                const int v = M::idxbu(c);
                lb = P.lbu[c] - ub[v];
                ubd = P.ubu[c] - ub[v];
                z = 0.0f;
            } else {
                const int v = M::idxbx(c - NBU);
                lb = P.lbx[c - NBU] - xb[v];
                ubd = P.ubx[c - NBU] - xb[v];
                z = dxk[v];
            }
            const float tl = fmaxf(z - lb, P.thr0), tu = fmaxf(ubd - z, P.thr0);
            FLD(k, Lay::LB + c) = lb;
            FLD(k, Lay::UB + c) = ubd;
            FLD(k, Lay::TL + c) = tl;
            FLD(k, Lay::TU + c) = tu;
            FLD(k, Lay::LL + c) = P.mu0 / tl;
            FLD(k, Lay::LU + c) = P.mu0 / tu;
            m++;
        }
        if (k < N) {
            float xn[NX], A[NX][NX], Bm[NX][NU];
            rk4_sens<M>(xb, ub, P, xn, A, Bm);
            float dxn[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) {
                float s = xn[i] - XB(k + 1, i);  // b_k = phi(xbar_k, ubar_k) - xbar_{k+1}
#pragma unroll
                for (int j = 0; j < NX; j++) s += A[i][j] * dxk[j];
                dxn[i] = s;
#pragma unroll
                for (int j = 0; j < NX; j++) FLD(k, Lay::A + i * NX + j) = A[i][j];
#pragma unroll
                for (int j = 0; j < NU; j++) FLD(k, Lay::Bm + i * NU + j) = Bm[i][j];
            }
#pragma unroll
            for (int j = 0; j < NX; j++) dxk[j] = dxn[j];
        }
    }
    const float inv_m2 = (m > 0) ? 0.5f / (float)m : 0.0f;

    // ---- interior-point iterations -------------------------------------------------------------------
    int status = 0, it = 0;
    float exit_res[3] = {0.0f, 0.0f, 0.0f};
    // step length, centring target and second-order weight of the previous iteration's direction
    float alpha = 0.0f, sigma_mu = 0.0f, eta = 0.0f, mu_prev = 3.0e38f;
    for (it = 0;; it++) {
        // P1 (backward): apply previous update, residuals, adjoint pi, factorisation + predictor rhs.
        float Lp[NX][NX], pv[NX], pin[NX];
        float res_stat = 0.0f, res_ineq = 0.0f, sum_c = 0.0f, max_c = 0.0f, stat_scale = 1.0f;
        bool fail = false;
        for (int k = N; k >= 0; k--) {
            float du[NU], dx[NX];
#pragma unroll
            for (int j = 0; j < NU; j++) du[j] = (k < N) ? FLD(k, Lay::DU + j) : 0.0f;
#pragma unroll
            for (int j = 0; j < NX; j++) dx[j] = (k >= 1) ? FLD(k, Lay::DX + j) : 0.0f;
            float lamdiff_u[NU], lamdiff_x[NX], sig_u[NU], sig_x[NX], gh_u[NU], gh_x[NX];
#pragma unroll
            for (int j = 0; j < NU; j++) { lamdiff_u[j] = 0.0f; sig_u[j] = 0.0f; gh_u[j] = 0.0f; }
#pragma unroll
            for (int j = 0; j < NX; j++) { lamdiff_x[j] = 0.0f; sig_x[j] = 0.0f; gh_x[j] = 0.0f; }
            float ddu[NU], ddx[NX];
            if (it > 0) {
#pragma unroll
                for (int j = 0; j < NU; j++) ddu[j] = (k < N) ? FLD(k, Lay::DDU + j) : 0.0f;
#pragma unroll
                for (int j = 0; j < NX; j++) ddx[j] = (k >= 1) ? FLD(k, Lay::DDX + j) : 0.0f;
            }
#pragma unroll
            for (int c = 0; c < NB; c++) {
                if (!comp_active<M>(c, k, N)) continue;
                const bool isu = c < NBU;
                const int v = isu ? M::idxbu(c) : M::idxbx(c - NBU);
                const float lb = FLD(k, Lay::LB + c), ubd = FLD(k, Lay::UB + c);
                float tl = FLD(k, Lay::TL + c), tu = FLD(k, Lay::TU + c);
                float ll = FLD(k, Lay::LL + c), lu = FLD(k, Lay::LU + c);
                float z = isu ? du[v] : dx[v];
                if (it > 0) {
                    // Delta t / Delta lambda of the combined direction at the previous iterate
                    const float dz = isu ? ddu[v] : ddx[v];
                    const float dza = FLD(k, Lay::DZA + c);
                    const float rl = z - lb - tl, rr = ubd - z - tu;
                    const float dtla = dza + rl, dtua = -dza + rr;
                    const float dlla = (-ll * (tl + rl) - ll * dza) / tl;
                    const float dlua = (-lu * (tu + rr) + lu * dza) / tu;
                    const float tgl = sigma_mu - eta * dlla * dtla, tgu = sigma_mu - eta * dlua * dtua;
                    const float dtl = dz + rl, dtu = -dz + rr;
                    const float dll = (tgl - ll * (tl + rl) - ll * dz) / tl;
                    const float dlu = (tgu - lu * (tu + rr) + lu * dz) / tu;
                    tl += alpha * dtl;
                    tu += alpha * dtu;
                    ll += alpha * dll;
                    lu += alpha * dlu;
                    z += alpha * dz;
                    FLD(k, Lay::TL + c) = tl;
                    FLD(k, Lay::TU + c) = tu;
                    FLD(k, Lay::LL + c) = ll;
                    FLD(k, Lay::LU + c) = lu;
                }
                const float rl = z - lb - tl, rr = ubd - z - tu;
                res_ineq = nan_max(res_ineq, fmaxf(fabsf(rl), fabsf(rr)));
                sum_c += ll * tl + lu * tu;
                max_c = fmaxf(max_c, fmaxf(ll * tl, lu * tu));
                // predictor rhs (target 0) and barrier Hessian
                const float gh = (ll * rl) / tl + ll - (lu * rr) / tu - lu;
                const float sg = ll / tl + lu / tu;
                if (isu) { lamdiff_u[v] += ll - lu; sig_u[v] += sg; gh_u[v] += gh; }
                else { lamdiff_x[v] += ll - lu; sig_x[v] += sg; gh_x[v] += gh; }
            }
            if (it > 0) {
#pragma unroll
                for (int j = 0; j < NU; j++) du[j] += alpha * ddu[j];
#pragma unroll
                for (int j = 0; j < NX; j++) dx[j] += alpha * ddx[j];
                if (k < N) {
#pragma unroll
                    for (int j = 0; j < NU; j++) FLD(k, Lay::DU + j) = du[j];
                }
                if (k >= 1) {
#pragma unroll
                    for (int j = 0; j < NX; j++) FLD(k, Lay::DX + j) = dx[j];
                }
            }
            // stage matrices
            float A[NX][NX], Bm[NX][NU];
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NX; i++) {
#pragma unroll
                    for (int j = 0; j < NX; j++) A[i][j] = FLD(k, Lay::A + i * NX + j);
#pragma unroll
                    for (int j = 0; j < NU; j++) Bm[i][j] = FLD(k, Lay::Bm + i * NU + j);
                }
            }
            // adjoint pi_k (x-stationarity rows zero by construction) and u-stationarity residual
            float pik[NX];
            if (k >= 1) {
#pragma unroll
                for (int i = 0; i < NX; i++) {
                    const float hx = (k < N) ? sc * P.W[i] : We[i];
                    float s = hx * dx[i] + FLD(k, Lay::GX + i) - lamdiff_x[i];
                    if (k < N) {
#pragma unroll
                        for (int l = 0; l < NX; l++) s += A[l][i] * pin[l];
                    }
                    pik[i] = s;
                }
            }
            float ru[NU];
            if (k < N) {
#pragma unroll
                for (int i = 0; i < NU; i++) {
                    const float gu = FLD(k, Lay::GU + i);
                    float s = sc * P.W[NX + i] * du[i] + gu - lamdiff_u[i];
                    float bp = 0.0f;
#pragma unroll
                    for (int l = 0; l < NX; l++) bp += Bm[l][i] * pin[l];
                    s += bp;
                    ru[i] = s;
                    FLD(k, Lay::RU + i) = s;
                    res_stat = nan_max(res_stat, fabsf(s));
                    stat_scale = fmaxf(stat_scale, fmaxf(fabsf(bp), fmaxf(fabsf(gu), fabsf(lamdiff_u[i]))));
                    gh_u[i] += s;
                }
            }
            // Square-root Riccati step (HPIPM's factorised form): with P_{k+1} = L L',
            //   M = diag(H + Sigma) + (L'[B A])' (L'[B A]) = [Luu 0; Lxu Lxx] [Luu 0; Lxu Lxx]',
            // P_k = Lxx Lxx', K = -Luu^{-T} Lxu', and p_k = g^x + A'p - Lxu Luu^{-1} (g^u + B'p).
            // M is a sum of PSD terms plus a positive diagonal, so it stays PD in fp32 even when the
            // barrier weights Sigma span many decades (the explicit Schur update A'PA - S'R^{-1}S does not).
            if (k == N) {
#pragma unroll
                for (int i = 0; i < NX; i++) {
#pragma unroll
                    for (int j = 0; j < NX; j++) Lp[i][j] = 0.0f;
                    Lp[i][i] = sqrtf(fmaxf(We[i] + sig_x[i], 0.0f));
                    pv[i] = gh_x[i];
                }
            } else {
                constexpr int NV = NX + NU;
                const int nv = (k >= 1) ? NV : NU;
                float LBA[NX][NV];
#pragma unroll
                for (int i = 0; i < NX; i++)
#pragma unroll
                    for (int j = 0; j < NV; j++) {
                        float s = 0.0f;
#pragma unroll
                        for (int l = i; l < NX; l++) s += Lp[l][i] * ((j < NU) ? Bm[l][j] : A[l][j - NU]);
                        LBA[i][j] = s;
                    }
                float Mm[NV][NV];
#pragma unroll
                for (int a2 = 0; a2 < NV; a2++)
#pragma unroll
                    for (int b2 = 0; b2 <= a2; b2++) {
                        float s = 0.0f;
                        if (a2 == b2) s = (a2 < NU) ? sc * P.W[NX + a2] + sig_u[a2] : sc * P.W[a2 - NU] + sig_x[a2 - NU];
#pragma unroll
                        for (int i = 0; i < NX; i++) s += LBA[i][a2] * LBA[i][b2];
                        Mm[a2][b2] = s;
                    }
                // Cholesky (lower, in place); u pivots must be positive (R > 0), x pivots may vanish (PSD P).
#pragma unroll
                for (int j = 0; j < NV; j++) {
                    if (j >= nv) break;
                    float d = Mm[j][j];
#pragma unroll
                    for (int q = 0; q < j; q++) d -= Mm[j][q] * Mm[j][q];
                    bool zero_col = false;
                    if (j < NU) {
                        if (!(d > 0.0f)) fail = true;
                        d = sqrtf(fmaxf(d, 1e-30f));
                    } else if (!(d > 1e-10f * (1.0f + fabsf(Mm[j][j])))) {
                        zero_col = true;
                        d = 0.0f;
                    } else {
                        d = sqrtf(d);
                    }
                    Mm[j][j] = d;
                    const float id = zero_col ? 0.0f : 1.0f / d;
#pragma unroll
                    for (int i = j + 1; i < NV; i++) {
                        float s = Mm[i][j];
#pragma unroll
                        for (int q = 0; q < j; q++) s -= Mm[i][q] * Mm[j][q];
                        Mm[i][j] = s * id;
                    }
                }
                // rhs: r = g^u + B'p -> lu = Luu^{-1} r
                float lr[NU];
#pragma unroll
                for (int i = 0; i < NU; i++) {
                    float s = gh_u[i];
#pragma unroll
                    for (int l = 0; l < NX; l++) s += Bm[l][i] * pv[l];
#pragma unroll
                    for (int q = 0; q < i; q++) s -= Mm[i][q] * lr[q];
                    lr[i] = s / Mm[i][i];
                    FLD(k, Lay::LR + i) = lr[i];
                }
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j < NU; j++) FLD(k, Lay::LUU + i * NU + j) = (j <= i) ? Mm[i][j] : 0.0f;
                if (k >= 1) {
                    float pn[NX];
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        float s = gh_x[i];
#pragma unroll
                        for (int l = 0; l < NX; l++) s += A[l][i] * pv[l];
#pragma unroll
                        for (int q = 0; q < NU; q++) {
                            s -= Mm[NU + i][q] * lr[q];
                            FLD(k, Lay::LXU + i * NU + q) = Mm[NU + i][q];
                        }
                        pn[i] = s;
                    }
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        pv[i] = pn[i];
#pragma unroll
                        for (int j = 0; j < NX; j++) Lp[i][j] = (j <= i) ? Mm[NU + i][NU + j] : 0.0f;
                    }
                }
            }
            if (k >= 1) {
#pragma unroll
                for (int i = 0; i < NX; i++) pin[i] = pik[i];
            }
        }
        const float mu = sum_c * inv_m2;
        exit_res[0] = res_stat;
        exit_res[1] = res_ineq;
        exit_res[2] = mu;
        if (fail) {
            // fp32 breakdown of the factorisation (barrier weights beyond fp32 range): keep the current,
            // already updated iterate when it is well inside the central path, else report a QP failure.
            status = (mu <= kBreakdownMu && res_ineq <= P.tol_ineq * 10.0f) ? 0 : 4;
            break;
        }
        if (!(res_stat == res_stat) || !(mu == mu)) { status = 1; break; }
        // fp32 stopping rule: the u-stationarity residual is a sum of terms of size stat_scale, so it cannot
        // fall below ~kStatRel * stat_scale; and once mu is 100x below its target the iterate is final.
        const bool stat_ok = res_stat <= P.tol_stat || res_stat <= kStatRel * stat_scale;
        const bool cmax_ok = max_c <= kCompMaxRatio * P.tol_comp;
        const bool stalled = mu <= P.tol_comp && mu > 0.5f * mu_prev;  // fp32 floor (see sqp_rti_team.hip)
        if (res_ineq <= P.tol_ineq &&
            ((stat_ok && mu <= P.tol_comp && cmax_ok) || mu <= 1e-2f * P.tol_comp || (stalled && cmax_ok)))
            break;
        if (it >= P.iter_max) break;
        mu_prev = mu;

        // P2 (forward): affine direction, its maximal step and the mu_aff polynomial.
        float s1 = 0.0f, s2 = 0.0f, amax = 1e30f;
        {
            float Dx[NX];
#pragma unroll
            for (int j = 0; j < NX; j++) Dx[j] = 0.0f;
            for (int k = 0; k <= N; k++) {
                float Du[NU];
                if (k < N) forward_du<M, Lay>(scr, k, S, Dx, Du);
#pragma unroll
                for (int c = 0; c < NB; c++) {
                    if (!comp_active<M>(c, k, N)) continue;
                    const bool isu = c < NBU;
                    const int v = isu ? M::idxbu(c) : M::idxbx(c - NBU);
                    const float z = isu ? FLD(k, Lay::DU + v) : FLD(k, Lay::DX + v);
                    const float dz = isu ? Du[v] : Dx[v];
                    const float lb = FLD(k, Lay::LB + c), ubd = FLD(k, Lay::UB + c);
                    const float tl = FLD(k, Lay::TL + c), tu = FLD(k, Lay::TU + c);
                    const float ll = FLD(k, Lay::LL + c), lu = FLD(k, Lay::LU + c);
                    const float rl = z - lb - tl, rr = ubd - z - tu;
                    const float dtl = dz + rl, dtu = -dz + rr;
                    const float dll = (-ll * (tl + rl) - ll * dz) / tl;
                    const float dlu = (-lu * (tu + rr) + lu * dz) / tu;
                    amax = step_bound(amax, tl, dtl);
                    amax = step_bound(amax, tu, dtu);
                    amax = step_bound(amax, ll, dll);
                    amax = step_bound(amax, lu, dlu);
                    s1 += ll * dtl + tl * dll + lu * dtu + tu * dlu;
                    s2 += dll * dtl + dlu * dtu;
                    FLD(k, Lay::DZA + c) = dz;
                }
                if (k < N) {
                    float Dn[NX];
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        float s = 0.0f;
#pragma unroll
                        for (int j = 0; j < NX; j++) s += FLD(k, Lay::A + i * NX + j) * Dx[j];
#pragma unroll
                        for (int j = 0; j < NU; j++) s += FLD(k, Lay::Bm + i * NU + j) * Du[j];
                        Dn[i] = s;
                    }
#pragma unroll
                    for (int j = 0; j < NX; j++) Dx[j] = Dn[j];
                }
            }
        }
        const float alpha_aff = fminf(1.0f, amax);
        float sigma;
        {
            const float mu_aff = (sum_c + alpha_aff * s1 + alpha_aff * alpha_aff * s2) * inv_m2;
            float sg = (mu > 0.0f) ? mu_aff / mu : 0.0f;
            sg = fmaxf(sg, 0.0f);
            sigma = fminf(sg * sg * sg, 1.0f);
        }

        // Corrector (pass 1): target sigma*mu - alpha_aff * dlam_aff * dt_aff. Safeguard (pass 2, only if the
        // corrector step is shorter than 0.1): pure centring with target max(sigma, 0.3)*mu. Same rule as
        // oracle/nmpc_oracle.c (protects Mehrotra's method against jamming on degenerate bounds).
        for (int pass = 1; pass <= 2; pass++) {
        if (pass == 1) {
            sigma_mu = sigma * mu;
            eta = alpha_aff;
        } else {
            if (alpha >= 0.1f) break;
            sigma_mu = fmaxf(sigma, 0.3f) * mu;
            eta = 0.0f;
        }
        // P3 (backward): corrector rhs through the stored factorisation.
        {
            float p[NX];
            for (int k = N; k >= 0; k--) {
                float du[NU], dx[NX], gh_u[NU], gh_x[NX];
#pragma unroll
                for (int j = 0; j < NU; j++) {
                    du[j] = (k < N) ? FLD(k, Lay::DU + j) : 0.0f;
                    gh_u[j] = (k < N) ? FLD(k, Lay::RU + j) : 0.0f;
                }
#pragma unroll
                for (int j = 0; j < NX; j++) { dx[j] = (k >= 1) ? FLD(k, Lay::DX + j) : 0.0f; gh_x[j] = 0.0f; }
#pragma unroll
                for (int c = 0; c < NB; c++) {
                    if (!comp_active<M>(c, k, N)) continue;
                    const bool isu = c < NBU;
                    const int v = isu ? M::idxbu(c) : M::idxbx(c - NBU);
                    const float z = isu ? du[v] : dx[v];
                    const float lb = FLD(k, Lay::LB + c), ubd = FLD(k, Lay::UB + c);
                    const float tl = FLD(k, Lay::TL + c), tu = FLD(k, Lay::TU + c);
                    const float ll = FLD(k, Lay::LL + c), lu = FLD(k, Lay::LU + c);
                    const float dza = FLD(k, Lay::DZA + c);
                    const float rl = z - lb - tl, rr = ubd - z - tu;
                    const float dtla = dza + rl, dtua = -dza + rr;
                    const float dlla = (-ll * (tl + rl) - ll * dza) / tl;
                    const float dlua = (-lu * (tu + rr) + lu * dza) / tu;
                    const float tgl = sigma_mu - eta * dlla * dtla, tgu = sigma_mu - eta * dlua * dtua;
                    const float gh = -(tgl - ll * rl) / tl + ll + (tgu - lu * rr) / tu - lu;
                    if (isu) gh_u[v] += gh;
                    else gh_x[v] += gh;
                }
                if (k == N) {
#pragma unroll
                    for (int i = 0; i < NX; i++) p[i] = gh_x[i];
                } else {
                    float r[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        float s = gh_u[i];
#pragma unroll
                        for (int l = 0; l < NX; l++) s += FLD(k, Lay::Bm + l * NU + i) * p[l];
                        r[i] = s;
                    }
                    float lr[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        float s = r[i];
#pragma unroll
                        for (int q = 0; q < i; q++) s -= FLD(k, Lay::LUU + i * NU + q) * lr[q];
                        lr[i] = s / FLD(k, Lay::LUU + i * NU + i);
                        FLD(k, Lay::LR + i) = lr[i];
                    }
                    if (k >= 1) {
                        float pn[NX];
#pragma unroll
                        for (int i = 0; i < NX; i++) {
                            float s = gh_x[i];
#pragma unroll
                            for (int l = 0; l < NX; l++) s += FLD(k, Lay::A + l * NX + i) * p[l];
#pragma unroll
                            for (int q = 0; q < NU; q++) s -= FLD(k, Lay::LXU + i * NU + q) * lr[q];
                            pn[i] = s;
                        }
#pragma unroll
                        for (int i = 0; i < NX; i++) p[i] = pn[i];
                    }
                }
            }
        }

        // P4 (forward): combined direction and its step length.
        {
            float Dx[NX];
            amax = 1e30f;
#pragma unroll
            for (int j = 0; j < NX; j++) Dx[j] = 0.0f;
            for (int k = 0; k <= N; k++) {
                float Du[NU];
                if (k < N) {
                    forward_du<M, Lay>(scr, k, S, Dx, Du);
#pragma unroll
                    for (int i = 0; i < NU; i++) FLD(k, Lay::DDU + i) = Du[i];
                }
                if (k >= 1) {
#pragma unroll
                    for (int j = 0; j < NX; j++) FLD(k, Lay::DDX + j) = Dx[j];
                }
#pragma unroll
                for (int c = 0; c < NB; c++) {
                    if (!comp_active<M>(c, k, N)) continue;
                    const bool isu = c < NBU;
                    const int v = isu ? M::idxbu(c) : M::idxbx(c - NBU);
                    const float z = isu ? FLD(k, Lay::DU + v) : FLD(k, Lay::DX + v);
                    const float dz = isu ? Du[v] : Dx[v];
                    const float lb = FLD(k, Lay::LB + c), ubd = FLD(k, Lay::UB + c);
                    const float tl = FLD(k, Lay::TL + c), tu = FLD(k, Lay::TU + c);
                    const float ll = FLD(k, Lay::LL + c), lu = FLD(k, Lay::LU + c);
                    const float dza = FLD(k, Lay::DZA + c);
                    const float rl = z - lb - tl, rr = ubd - z - tu;
                    const float dtla = dza + rl, dtua = -dza + rr;
                    const float dlla = (-ll * (tl + rl) - ll * dza) / tl;
                    const float dlua = (-lu * (tu + rr) + lu * dza) / tu;
                    const float tgl = sigma_mu - eta * dlla * dtla, tgu = sigma_mu - eta * dlua * dtua;
                    const float dtl = dz + rl, dtu = -dz + rr;
                    const float dll = (tgl - ll * (tl + rl) - ll * dz) / tl;
                    const float dlu = (tgu - lu * (tu + rr) + lu * dz) / tu;
                    amax = step_bound(amax, tl, dtl);
                    amax = step_bound(amax, tu, dtu);
                    amax = step_bound(amax, ll, dll);
                    amax = step_bound(amax, lu, dlu);
                }
                if (k < N) {
                    float Dn[NX];
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        float s = 0.0f;
#pragma unroll
                        for (int j = 0; j < NX; j++) s += FLD(k, Lay::A + i * NX + j) * Dx[j];
#pragma unroll
                        for (int j = 0; j < NU; j++) s += FLD(k, Lay::Bm + i * NU + j) * Du[j];
                        Dn[i] = s;
                    }
#pragma unroll
                    for (int j = 0; j < NX; j++) Dx[j] = Dn[j];
                }
            }
            alpha = fminf(1.0f, P.tau * amax);
        }
        }  // pass
    }

    // ---- full SQP step + outputs --------------------------------------------------------------------
    if (status == 0) {
        for (int k = 0; k <= N; k++) {
#pragma unroll
            for (int j = 0; j < NX; j++) {
                const float d = (k == 0) ? x0[j] - XB(0, j) : FLD(k, Lay::DX + j);
                const float nv = XB(k, j) + d;
                XB(k, j) = (k == 0) ? x0[j] : nv;
                if (a.xtraj) a.xtraj[((size_t)k * NX + j) * Bn + inst] = (k == 0) ? x0[j] : nv;
            }
            if (k < N) {
#pragma unroll
                for (int j = 0; j < NU; j++) {
                    const float nv = UB(k, j) + FLD(k, Lay::DU + j);
                    UB(k, j) = nv;
                    if (a.utraj) a.utraj[((size_t)k * NU + j) * Bn + inst] = nv;
                }
            }
        }
    }
    float u0[NU];
#pragma unroll
    for (int j = 0; j < NU; j++) {
        u0[j] = UB(0, j);
        if (a.u0) a.u0[(size_t)j * Bn + inst] = u0[j];
    }
    if (a.x1) {
#pragma unroll
        for (int j = 0; j < NX; j++) a.x1[(size_t)j * Bn + inst] = XB(1, j);
    }
    if (a.status) a.status[inst] = status;
    if (a.qp_iter) a.qp_iter[inst] = it;
    if (a.qp_res) {
#pragma unroll
        for (int j = 0; j < 3; j++) a.qp_res[(size_t)j * Bn + inst] = exit_res[j];
    }
    if (mode == kModeRun && status == 0) {
        float r[M::NBX], cmd[3];
#pragma unroll
        for (int i = 0; i < M::NBX; i++) {
            r[i] = x0[M::idxbx(i)] + u0[i] * P.dt_ctrl;
            a.carried[(size_t)i * S + inst] = r[i];
        }
        M::inverse_kin(r, P, cmd);
        if (a.cmd) {
#pragma unroll
            for (int j = 0; j < 3; j++) a.cmd[(size_t)j * Bn + inst] = cmd[j];
        }
    }
#undef FLD
#undef XB
#undef UB
}

}  // namespace

template <class M>
hipError_t launch_sqp_rti_lane(const KParams& P, const KArgs& a, int mode, hipStream_t stream)
{
    if (a.B <= 0) return hipSuccess;
    const int block = 64;
    const int grid = (a.B + block - 1) / block;
    hipLaunchKernelGGL(k_sqp_rti_lane<M>, dim3(grid), dim3(block), 0, stream, P, a, mode);
    return hipGetLastError();
}

template hipError_t launch_sqp_rti_lane<Diff2>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_lane<Omni4>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_lane<Tric3>(const KParams&, const KArgs&, int, hipStream_t);
template size_t lane_scratch_floats<Diff2>(int, int);
template size_t lane_scratch_floats<Omni4>(int, int);
template size_t lane_scratch_floats<Tric3>(int, int);

}  // namespace nmpc
