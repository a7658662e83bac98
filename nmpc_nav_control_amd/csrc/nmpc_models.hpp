// nmpc_models.hpp -- the three robot models of the reference as device functors (fp32).
//
// Each model restates the reference's CasADi f_expl and provides the hand-written forward
// sensitivity product (the analogue of the CasADi-generated *_expl_vde_forw):
//   diff2amr  scripts/diff/diff_amr_model.py:41-60      x=[x,y,th,vl,vr,vl_ref,vr_ref] u=[dvl_ref,dvr_ref]
//   omni4amr  scripts/omni4/omni4_amr_model.py:51-73    x=[x,y,th,v1..v4,v1_ref..v4_ref] u=[dv1_ref..dv4_ref]
//   tric3amr  scripts/tric/tric_amr_model.py:43-55      x=[x,y,th,v,alpha,v_ref,alpha_ref] u=[dv_ref,dalpha_ref]
//             (cos_alpha = sin(alpha) at :45 reproduced when KParams::sin_bug != 0)
// Box-constraint index maps: scripts/{diff,omni4}/generate_c_code.py:45-55, scripts/tric/generate_c_code.py:47-57.
#pragma once

#include <hip/hip_runtime.h>

namespace nmpc {

// Uniform (per-launch) parameters: model parameters, bounds, stage weights, QP options.
// INVARIANT the team kernel relies on: dt and the model parameters p are the same for every robot of a launch, so the
// state-independent rows of [B A] (rows >= NGV of each model, Model::gmask) are bit-identical for every robot; the
// column-form M block (gconst_load, team_common.hpp) reads them from each wave's first team and applies them to all
// four. Per-robot model parameters would break this and need the row form (-DNMPC_MROW) or per-team constants;
// tests/test_gpu_split.py::test_constant_rows_per_launch checks the column form against that build.
struct KParams {
    int N;
    float dt, dt_ctrl;
    float p[3];
    float lbx[4], ubx[4], lbu[4], ubu[4];
    float W[15];   // stage weight diagonal [Q; R]
    float We[11];  // terminal weight diagonal (constructor value; diff run() may scale the pose part)
    int terminal_hack, sin_bug;
    int iter_max;
    float tol_stat, tol_ineq, tol_comp, mu0, thr0, tau;
    // IPM direction rule: 0 Mehrotra predictor-corrector, 1 one direction per iteration with centring
    // sigma = clamp((1 - alpha_prev)^2, sd_lo, sd_hi) (DESIGN.md "Algorithm and precision")
    int ipm;
    float sd_lo, sd_hi;
    // warm start of the bound multipliers from the robot's previous solve (KArgs::warm flags)
    int warm;
    float warm_kappa;
    int warm_iter_max;  // a solve that needed more IPM iterations starts the next one cold
    // infeasibility exit: multiplier threshold qp_infeas_lambda (+inf: off), scaled in the kernel by
    // max(1, max(wmax, the robot's terminal weights) / 10); wmax = the largest stage weight
    float infeas_lam, wmax;
};

enum ModelId { kDiff = 0, kOmni4 = 1, kTric = 2 };

// Column bitmask of one row of the discrete Jacobian [B A] in the team lane order (bit v: input v for v < NU,
// state v - NU above), from a pattern string ('1' = structurally nonzero). gmask(i) of a model gives its constant
// rows i >= NGV: the M block of the Riccati step multiplies them as uniform operands and skips the zeros
// (team_common.hpp m_block). tests/test_oracle.py checks every pattern against the oracle's RK4 Jacobians.
__host__ __device__ constexpr unsigned gmask_of(const char* p)
{
    unsigned m = 0;
    for (int v = 0; p[v]; v++) m |= (p[v] == '1' ? 1u : 0u) << v;
    return m;
}

struct Diff2 {
    static constexpr int ID = kDiff, NX = 7, NU = 2, NBX = 2, NBU = 2, NP = 2, NY = 9;
    // rows >= NGV of the discrete Jacobian [B A] do not depend on the state or input (theta, wheel and
    // ref rows are linear): they are computed once per launch (checked by tests/test_oracle.py)
    static constexpr int NGV = 2;
    // team kernel M block: the column form, with the input pivots one after the other (up front they cost the
    // metric config 4.4 %: profiles/r05/ab/mcol_pivots.txt)
    static constexpr bool kMcolForm = true;
    static constexpr bool kPivotsUpFront = false;
    // constant rows th, vl, vr, vl_ref, vr_ref over columns [dvl_ref dvr_ref | x y th vl vr vl_ref vr_ref]
    __host__ __device__ static constexpr unsigned gmask(int i)
    {
        return i == 2 ? gmask_of("11..11111") : i == 3 ? gmask_of("1....1.1.") : i == 4 ? gmask_of(".1....1.1")
             : i == 5 ? gmask_of("1......1.") : i == 6 ? gmask_of(".1......1") : 0u;
    }
    __host__ __device__ static constexpr int idxbx(int i) { return 5 + i; }
    __host__ __device__ static constexpr int idxbu(int i) { return i; }

    __device__ static inline void f(const float* x, const float* u, const KParams& P, float* xd)
    {
        const float ib = 1.0f / P.p[0], it = 1.0f / P.p[1];
        float s, c;
        __sincosf(x[2], &s, &c);
        const float v = 0.5f * (x[4] + x[3]);
        xd[0] = v * c;
        xd[1] = v * s;
        xd[2] = (x[4] - x[3]) * ib;
        xd[3] = it * (x[5] - x[3]);
        xd[4] = it * (x[6] - x[4]);
        xd[5] = u[0];
        xd[6] = u[1];
    }
    // dK[r][j] = sum_l Jx[r][l] S[l][j] + Ju[r][j - NX]   (NV = NX + NU columns)
    template <int NV>
    __device__ static inline void jvp(const float* x, const float (&S)[NX][NV], const KParams& P, float (&dK)[NX][NV])
    {
        const float ib = 1.0f / P.p[0], it = 1.0f / P.p[1];
        float s, c;
        __sincosf(x[2], &s, &c);
        const float v = 0.5f * (x[4] + x[3]);
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const float sw = 0.5f * (S[3][j] + S[4][j]);
            dK[0][j] = -v * s * S[2][j] + c * sw;
            dK[1][j] = v * c * S[2][j] + s * sw;
            dK[2][j] = (S[4][j] - S[3][j]) * ib;
            dK[3][j] = it * (S[5][j] - S[3][j]);
            dK[4][j] = it * (S[6][j] - S[4][j]);
            dK[5][j] = (j == NX + 0) ? 1.0f : 0.0f;
            dK[6][j] = (j == NX + 1) ? 1.0f : 0.0f;
        }
    }
    // NMPCNavControlDiff.cpp:183-187 (vel = {v, vn, w})
    __device__ static inline void direct_kin(const float* vel, float, const KParams& P, float* xv)
    {
        xv[0] = vel[0] - 0.5f * P.p[0] * vel[2];
        xv[1] = vel[0] + 0.5f * P.p[0] * vel[2];
    }
    // NMPCNavControlDiff.cpp:189-193 -> cmd {v, w, 0}
    __device__ static inline void inverse_kin(const float* r, const KParams& P, float* cmd)
    {
        cmd[0] = 0.5f * (r[1] + r[0]);
        cmd[1] = (r[1] - r[0]) / P.p[0];
        cmd[2] = 0.0f;
    }
};

struct Omni4 {
    static constexpr int ID = kOmni4, NX = 11, NU = 4, NBX = 4, NBU = 4, NP = 2, NY = 15;
    static constexpr int NGV = 2;  // x, y rows vary; theta / wheel / ref rows are linear
    static constexpr bool kMcolForm = true;  // column-form M block: +6 % (profiles/r05/ab/mcol.txt)
    static constexpr bool kPivotsUpFront = false;  // (NU = 4: chol_input_2 is for two inputs)
    // constant rows th, v1..v4, v1_ref..v4_ref over columns [dv1_ref..dv4_ref | x y th v1..v4 v1_ref..v4_ref]
    __host__ __device__ static constexpr unsigned gmask(int i)
    {
        return i == 2 ? gmask_of("1111..111111111") : i == 3 ? gmask_of("1......1...1...")
             : i == 4 ? gmask_of(".1......1...1..") : i == 5 ? gmask_of("..1......1...1.")
             : i == 6 ? gmask_of("...1......1...1") : i == 7 ? gmask_of("1..........1...")
             : i == 8 ? gmask_of(".1..........1..") : i == 9 ? gmask_of("..1..........1.")
             : i == 10 ? gmask_of("...1..........1") : 0u;
    }
    __host__ __device__ static constexpr int idxbx(int i) { return 7 + i; }
    __host__ __device__ static constexpr int idxbu(int i) { return i; }

    __device__ static inline void f(const float* x, const float* u, const KParams& P, float* xd)
    {
        const float it = 1.0f / P.p[1], iw = 1.0f / (2.0f * P.p[0]);
        float s, c;
        __sincosf(x[2], &s, &c);
        const float v = 0.25f * (x[3] - x[4] + x[5] - x[6]);
        const float vn = 0.25f * (-x[3] - x[4] + x[5] + x[6]);
        xd[0] = v * c - vn * s;
        xd[1] = v * s + vn * c;
        xd[2] = -(x[3] + x[4] + x[5] + x[6]) * iw;
#pragma unroll
        for (int i = 0; i < 4; i++) xd[3 + i] = it * (x[7 + i] - x[3 + i]);
#pragma unroll
        for (int i = 0; i < 4; i++) xd[7 + i] = u[i];
    }
    template <int NV>
    __device__ static inline void jvp(const float* x, const float (&S)[NX][NV], const KParams& P, float (&dK)[NX][NV])
    {
        const float it = 1.0f / P.p[1], iw = 1.0f / (2.0f * P.p[0]);
        float s, c;
        __sincosf(x[2], &s, &c);
        const float v = 0.25f * (x[3] - x[4] + x[5] - x[6]);
        const float vn = 0.25f * (-x[3] - x[4] + x[5] + x[6]);
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const float dv = 0.25f * (S[3][j] - S[4][j] + S[5][j] - S[6][j]);
            const float dvn = 0.25f * (-S[3][j] - S[4][j] + S[5][j] + S[6][j]);
            const float dth = S[2][j];
            dK[0][j] = dv * c - dvn * s + (-v * s - vn * c) * dth;
            dK[1][j] = dv * s + dvn * c + (v * c - vn * s) * dth;
            dK[2][j] = -(S[3][j] + S[4][j] + S[5][j] + S[6][j]) * iw;
#pragma unroll
            for (int i = 0; i < 4; i++) dK[3 + i][j] = it * (S[7 + i][j] - S[3 + i][j]);
#pragma unroll
            for (int i = 0; i < 4; i++) dK[7 + i][j] = (j == NX + i) ? 1.0f : 0.0f;
        }
    }
    // NMPCNavControlOmni4.cpp:185-192
    __device__ static inline void direct_kin(const float* vel, float, const KParams& P, float* xv)
    {
        const float hl = 0.5f * P.p[0] * vel[2];
        xv[0] = vel[0] - vel[1] - hl;
        xv[1] = -vel[0] - vel[1] - hl;
        xv[2] = vel[0] + vel[1] - hl;
        xv[3] = -vel[0] + vel[1] - hl;
    }
    // NMPCNavControlOmni4.cpp:194-200 -> cmd {v, vn, w}
    __device__ static inline void inverse_kin(const float* r, const KParams& P, float* cmd)
    {
        cmd[0] = 0.25f * (r[0] - r[1] + r[2] - r[3]);
        cmd[1] = 0.25f * (-r[0] - r[1] + r[2] + r[3]);
        cmd[2] = -(r[0] + r[1] + r[2] + r[3]) / (2.0f * P.p[0]);
    }
};

struct Tric3 {
    static constexpr int ID = kTric, NX = 7, NU = 2, NBX = 2, NBU = 2, NP = 3, NY = 9;
    static constexpr int NGV = 3;  // x, y, theta rows vary; v / alpha / ref rows are linear
    static constexpr bool kMcolForm = true;  // column-form M block: +5 % (profiles/r05/ab/mcol.txt)
    static constexpr bool kPivotsUpFront = true;  // both input pivots from the 2 x 2 block: +1.2 % (mcol_pivots.txt)
    // constant rows v, alpha, v_ref, alpha_ref over columns [dv_ref dalpha_ref | x y th v alpha v_ref alpha_ref]
    __host__ __device__ static constexpr unsigned gmask(int i)
    {
        return i == 3 ? gmask_of("1....1.1.") : i == 4 ? gmask_of(".1....1.1") : i == 5 ? gmask_of("1......1.")
             : i == 6 ? gmask_of(".1......1") : 0u;
    }
    __host__ __device__ static constexpr int idxbx(int i) { return 5 + i; }
    __host__ __device__ static constexpr int idxbu(int i) { return i; }

    __device__ static inline void f(const float* x, const float* u, const KParams& P, float* xd)
    {
        const float id = 1.0f / P.p[0], itv = 1.0f / P.p[1], ita = 1.0f / P.p[2];
        float s, c, sa, ca;
        __sincosf(x[2], &s, &c);
        __sincosf(x[4], &sa, &ca);
        const float cal = P.sin_bug ? sa : ca;  // tric_amr_model.py:45
        xd[0] = x[3] * c * cal;
        xd[1] = x[3] * s * cal;
        xd[2] = x[3] * id * sa;
        xd[3] = itv * (x[5] - x[3]);
        xd[4] = ita * (x[6] - x[4]);
        xd[5] = u[0];
        xd[6] = u[1];
    }
    template <int NV>
    __device__ static inline void jvp(const float* x, const float (&S)[NX][NV], const KParams& P, float (&dK)[NX][NV])
    {
        const float id = 1.0f / P.p[0], itv = 1.0f / P.p[1], ita = 1.0f / P.p[2];
        float s, c, sa, ca;
        __sincosf(x[2], &s, &c);
        __sincosf(x[4], &sa, &ca);
        const float cal = P.sin_bug ? sa : ca;
        const float dcal = P.sin_bug ? ca : -sa;
        const float v = x[3];
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const float dth = S[2][j], dv = S[3][j], da = S[4][j];
            dK[0][j] = -v * s * cal * dth + c * cal * dv + v * c * dcal * da;
            dK[1][j] = v * c * cal * dth + s * cal * dv + v * s * dcal * da;
            dK[2][j] = id * (sa * dv + v * ca * da);
            dK[3][j] = itv * (S[5][j] - dv);
            dK[4][j] = ita * (S[6][j] - da);
            dK[5][j] = (j == NX + 0) ? 1.0f : 0.0f;
            dK[6][j] = (j == NX + 1) ? 1.0f : 0.0f;
        }
    }
    // NMPCNavControlTric.cpp:97-98: x0[v] = measured v, x0[alpha] = steering wheel angle
    __device__ static inline void direct_kin(const float* vel, float steer, const KParams&, float* xv)
    {
        xv[0] = vel[0];
        xv[1] = steer;
    }
    // NMPCNavControlTric.cpp:161-162 -> cmd {v, alpha, 0}
    __device__ static inline void inverse_kin(const float* r, const KParams&, float* cmd)
    {
        cmd[0] = r[0];
        cmd[1] = r[1];
        cmd[2] = 0.0f;
    }
};

// One RK4 step with forward sensitivities (acados ERK default: 4 stages, 1 step, forward VDE):
// xn = phi(x, u); A = d phi / dx; B = d phi / du.
template <class M>
__device__ inline void rk4_sens(const float* x, const float* u, const KParams& P, float* xn, float (&A)[M::NX][M::NX],
                                float (&Bm)[M::NX][M::NU])
{
    constexpr int NX = M::NX, NU = M::NU, NV = NX + NU;
    const float h = P.dt;
    float k[NX], xs[NX], acc[NX];
    float S[NX][NV], dK[NX][NV], Acc[NX][NV];
#pragma unroll
    for (int i = 0; i < NX; i++) {
        xs[i] = x[i];
#pragma unroll
        for (int j = 0; j < NV; j++) S[i][j] = (i == j) ? 1.0f : 0.0f;
    }
    const float cst[4] = {0.5f, 0.5f, 1.0f, 0.0f};
    const float wgt[4] = {1.0f, 2.0f, 2.0f, 1.0f};
#pragma unroll
    for (int st = 0; st < 4; st++) {
        M::f(xs, u, P, k);
        M::template jvp<NV>(xs, S, P, dK);
#pragma unroll
        for (int i = 0; i < NX; i++) {
            acc[i] = (st == 0) ? k[i] : acc[i] + wgt[st] * k[i];
#pragma unroll
            for (int j = 0; j < NV; j++) Acc[i][j] = (st == 0) ? dK[i][j] : Acc[i][j] + wgt[st] * dK[i][j];
        }
        if (st < 3) {
            const float ch = cst[st] * h;
#pragma unroll
            for (int i = 0; i < NX; i++) {
                xs[i] = x[i] + ch * k[i];
#pragma unroll
                for (int j = 0; j < NV; j++) S[i][j] = ((i == j) ? 1.0f : 0.0f) + ch * dK[i][j];
            }
        }
    }
    const float h6 = h * (1.0f / 6.0f);
#pragma unroll
    for (int i = 0; i < NX; i++) {
        xn[i] = x[i] + h6 * acc[i];
#pragma unroll
        for (int j = 0; j < NX; j++) A[i][j] = ((i == j) ? 1.0f : 0.0f) + h6 * Acc[i][j];
#pragma unroll
        for (int j = 0; j < NU; j++) Bm[i][j] = h6 * Acc[i][NX + j];
    }
}

// RK4 without sensitivities (plant simulation of the bench harness).
template <class M>
__device__ inline void rk4(const float* x, const float* u, const KParams& P, float h, float* xn)
{
    constexpr int NX = M::NX;
    float k[NX], xs[NX], acc[NX];
#pragma unroll
    for (int i = 0; i < NX; i++) xs[i] = x[i];
    const float cst[3] = {0.5f, 0.5f, 1.0f};
    const float wgt[4] = {1.0f, 2.0f, 2.0f, 1.0f};
#pragma unroll
    for (int st = 0; st < 4; st++) {
        M::f(xs, u, P, k);
#pragma unroll
        for (int i = 0; i < NX; i++) acc[i] = (st == 0) ? k[i] : acc[i] + wgt[st] * k[i];
        if (st < 3) {
#pragma unroll
            for (int i = 0; i < NX; i++) xs[i] = x[i] + cst[st] * h * k[i];
        }
    }
#pragma unroll
    for (int i = 0; i < NX; i++) xn[i] = x[i] + h * (1.0f / 6.0f) * acc[i];
}

}  // namespace nmpc
