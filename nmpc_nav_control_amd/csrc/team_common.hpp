// team_common.hpp -- device helpers shared by the solve kernels (sqp_rti_team.hip: one 16-lane team per robot;
// sqp_rti_rowpar.hip: one wave per robot with stage-parallel phases): IPM constants, the fused fp64 DPP blocks of
// the Riccati step, the RK4 sensitivity column, lane-record access, bound directions and the step bound.
#pragma once

#include "nmpc_kernels.hpp"
#include "team_asm_gen.hpp"
#include "team_dpp.hpp"

namespace nmpc {

#ifndef NMPC_DZ_IN_RECORD
constexpr bool kDzPlane = true;
#else
constexpr bool kDzPlane = false;  // A/B: the round-2 layout, DZ a field of the lane record
#endif

constexpr bool rec_quad_major_v(int nv) { return nv > 12; }

template <class M, bool SD = false>
struct TeamRec {
    static constexpr int NX = M::NX, NU = M::NU, NV = NX + NU, NGV = M::NGV;
    // Mehrotra field order: P1's write-only outputs first (LR, LM, RU: P1 never loads them, so no record load is
    // issued into registers P1 overwrites), then the bound quad, the iterate and the rest the light sweeps read
    // (prefix [0, NL)), then the P1-only inputs (DZ, GR). P1 loads [P1L0, P1L1) and stores [0, P1S1).
    // Same-box A/B against the round-1 order (P1 rewrote a prefix it also loaded, and the compiler reused the
    // dead lanes of those loads, waiting on them): kernel ms diff N=40 B=4096 1.430 -> 1.404, omni4 1.664 ->
    // 1.655 (profiles/r02/ab/abwb.txt).
    // Single-direction order (SD, NU = 2): no sweep reads RU (the corrector's u residual) or DZA (the affine
    // direction), so they move to the end: P1 stores 2 quads instead of 3 and the forward sweep loads 3 quads
    // instead of 3.5 (same-box A/B, single-direction rule: diff N=40 B=4096 3.43 -> 3.53 M it/s, B=1024 +1.2 %,
    // tric even; the NU = 4 analogue cost omni4 1.8 %, so omni4 keeps the Mehrotra order; profiles/r02/ab/layout.txt)
    static constexpr bool L2 = SD && NU == 2;
    static constexpr int LR = 0, LM = 1;  // Luu^-1 rhs, row v of the input columns
    static constexpr int Z = L2 ? 3 : ((NU == 2) ? 8 : 6);          // QP iterate
    static constexpr int TL = (NU == 2) ? 4 : 8;                    // bound quad TL TU LL LU
    static constexpr int TU = TL + 1, LL = TL + 2, LU = TL + 3;
    static constexpr int LB = L2 ? 8 : ((NU == 2) ? 9 : 12), UB = LB + 1;  // bounds relative to the SQP iterate
    static constexpr int GV = L2 ? 10 : ((NU == 2) ? 12 : 14);      // NGV varying rows of column v of [B A]
    static constexpr int NL = GV + NGV;                             // prefix read by the light sweeps
    // combined direction, cost gradient (P1 only). DZ plane (default): the forward sweep writes one float per lane
    // and stage; in the lane record that dirtied a whole 32-byte sector per lane (8x the bytes), so DZ lives in a
    // dense plane [robot][stage][16 lanes] (64 B per team and stage, 2 sectors for 9 lanes) and its register slot
    // sits past the record's stored fields
    static constexpr int GR = kDzPlane ? NL : NL + 1;
    static constexpr int RU = L2 ? GR + 1 : LM + NU;                // u residual (corrector sweeps)
    static constexpr int DZA = L2 ? GR + 2 : Z + 1 + ((NU == 2) ? 2 : 0);  // affine direction
    static constexpr int DZ = kDzPlane ? (L2 ? GR + 3 : GR + 1) : NL;
    static constexpr int P1L0 = L2 ? Z : ((NU == 2) ? TL : Z), P1L1 = GR + 1;  // P1 loads
    static constexpr int P1S1 = L2 ? 8 : 12;                        // P1 stores [0, P1S1)
    static_assert(NU == 2 || NU == 4, "layouts for NU = 2 and 4");
    static_assert(L2 || (RU < ((NU == 2) ? TL : Z) && DZA < P1S1), "P1 store block holds RU and DZA");
    static_assert(LU < P1S1 && Z < P1S1 && LM + NU <= P1S1, "P1 store block");
    static constexpr int NF = NL, NB = NL;
    static constexpr int MAXF = (GR > RU ? GR : RU) > (DZA > DZ ? DZA : DZ) ? (GR > RU ? GR : RU) : (DZA > DZ ? DZA : DZ);
    static constexpr int RS = (MAXF + 1 + 3) / 4 * 4;  // register image of a record (dwordx4 pieces)
    // stored floats per lane record: fields [0, GR] (every kernel stores nothing past the gradient; the register
    // image may hold more: the DZ slot of the DZ plane and, in the single-direction layout, the corrector-only RU /
    // DZA). tric (NGV = 3): 16 stored against a 20-float image, 64-B instead of 80-B records
#ifndef NMPC_RSS_FULL
    static constexpr int RSS = (GR + 1 + 3) / 4 * 4;
#else
    static constexpr int RSS = RS;  // A/B: the round-3 stride (records as long as the register image)
#endif
    static constexpr int NQ = RS / 4;
    static_assert(NV <= 16, "a team holds at most 16 variables");
    static_assert(TL % 4 == 0, "bound quad aligned");
    static_assert(RSS <= RS && (kDzPlane || DZ < RSS) && (L2 || (RU < RSS && DZA < RSS)), "stored fields");
    // Split records (team kernel, single-direction layout of tric; NMPC_REC_FULL: the 64-B stage blocks for A/B): per robot a core plane [stage][NV slots][8] = LR LM[2] Z | GV[NGV] GR (pad) and a bound
    // plane [stage][NBND bounded slots][8] = TL TU LL LU | LB UB (pad), in the robot's old record region. A slot
    // without a bound keeps no bound fields in memory: its loads read the sentinel quad pair (kFar slacks and
    // bounds, zero multipliers) and its stores go to the robot's dummy pair. A sweep's stage then touches
    // 9 x 32 B of core plane (2.25 lines, stages contiguous) + 128 B of bound plane instead of 5 lines of 64-B
    // records (DESIGN.md section 3 "Record stride").
    // Taken where it wins (same-box A/B, profiles/r04/ab/split.txt): tric 3.60 -> 4.92 M it/s, mixed 4.76 -> 5.76 M
    // (the working set drops under the Infinity Cache); diff loses 1 % (issue-bound: more load instructions and
    // registers for 35 % less traffic), so diff keeps the 64-B records
    // SPLIT_OK: the layout exists for the model (diff, tric); SPLIT: tric always takes it. For diff the host picks
    // per launch (KArgs::rec_split): wide records alone on the device (the metric: -1.2 % with split planes), split
    // planes beside other resident fleets (mixed: 5.25 -> 5.76 M it/s; nmpc_batch.cpp rec_split_auto)
#ifndef NMPC_REC_FULL
    static constexpr bool SPLIT_OK = L2 && !rec_quad_major_v(NV);
    static constexpr bool SPLIT = SPLIT_OK && M::ID == kTric;
#else
    static constexpr bool SPLIT_OK = false;
    static constexpr bool SPLIT = false;
#endif
    static constexpr int NBND = NU + M::NBX;
    static constexpr int CW = 8;                 // floats per slot in either plane
    static constexpr int CS = NV * CW;           // core floats per stage
    static constexpr int BS = NBND * CW;         // bound floats per stage
    static_assert(!SPLIT_OK || (TL == 4 && LB == 8 && GV == 10 && GR == GV + NGV && NGV <= 3), "split record map");
    static_assert(!SPLIT_OK || (CS + BS) <= 16 * RSS, "split planes fit the robot's record region");
    // split planes keep no DZ / DZA field: the forward sweep's direction must live in the DZ plane
    static_assert(!SPLIT_OK || kDzPlane, "split record planes need the DZ plane (NMPC_DZ_IN_RECORD off)");
};

namespace {

constexpr float kBreakdownMuT = 1e-6f;
constexpr float kStatRelT = 1e-5f;
// largest single complementarity product at exit, relative to tol_comp: the mean (mu) alone lets one pair keep
// m * mu, which leaves a nearly active bound's multiplier at ~1e-5 and moves u0 by ~1e-3 through the weak input
// curvature R dt (DESIGN.md "Stopping rule")
constexpr float kCompMaxRatio = 30.0f;
// primal infeasibility (status 4, the wrapper's exception path, NMPCNavControl.cpp:14-23): the bound multipliers
// diverge while the bound residual cannot close. A feasible QP of this OCP keeps them at the size of its cost
// weights (max 88 over 768 bench-loop QPs with renewals, against > 1e5 by IPM iteration 13-20 for QPs made
// infeasible as the failure test does; tools/infeas_study.py); the oracle uses the same two constants
// (the multiplier threshold is nmpc_model_params.qp_infeas_lambda, 1e5 by default, scaled by the largest weight)
constexpr float kInfeasRes = 1e-3f;
constexpr float kWarmLambdaCap = 1e3f;  // largest warm-started bound multiplier
constexpr float kFar = 1e30f;  // sentinel bound / slack of unbounded slots (z + kFar - kFar == 0 in fp32)

// generated whole-block fused-DPP kernels (team_asm_gen.hpp), dispatched on the model shape
template <int NX, int NU>
__device__ __forceinline__ void pg_block(double (&acc)[NX], const double (&prow)[NX + NU], const double (&gd)[NX])
{
    if constexpr (NX == 7 && NU == 2) pg_block_7_2(acc, prow, gd);
    else pg_block_11_4(acc, prow, gd);
}
template <int NX, int NU>
__device__ __forceinline__ void mrow_pg_block(double (&acc)[NX + NU], double& md0, const double (&pg)[NX],
                                              const double (&gd)[NX])
{
    if constexpr (NX == 7 && NU == 2) mrow_pg_block_7_2(acc, md0, pg, gd);
    else mrow_pg_block_11_4(acc, md0, pg, gd);
}
// Rows of [B A] the column-form M block broadcasts across the team (m_block): the NGV state-dependent rows and
// theta's row (constant, but the densest: 7 of 9 / 13 of 15 columns, cheaper in registers as 2 more broadcast FMAs)
template <class M>
constexpr int mcol_nbc() { return M::NGV > 3 ? M::NGV : 3; }

// Constant entries of rows >= mcol_nbc of [B A] (M::gmask), identical for every robot of a launch (they depend on
// the model parameters only, tests/test_oracle.py test_constant_jacobian_rows): read once per launch from lane r of
// the wave's first team, so each is one uniform value (a scalar operand) for every lane
template <class M>
struct GConst {
    double v[M::NX][M::NX + M::NU];
};
template <class M>
__device__ __forceinline__ void gconst_load(GConst<M>& gc, const float (&gcol)[M::NX])
{
    constexpr int NX = M::NX, NV = M::NX + M::NU;
    sfor<mcol_nbc<M>(), NX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, NV>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((M::gmask(i) >> r) & 1u)
                gc.v[i][r] = (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(gcol[i]), r));
            else
                gc.v[i][r] = 0.0;
        });
    });
}

// Column j of M = D + [B A]' P [B A] on lane j (M is symmetric: its row j), lane j holding column j of P [B A] in
// pg and column j of [B A] in gd, Lr initialised with the diagonal D: the sparse constant rows (>= mcol_nbc) of
// [B A] as uniform-operand FMAs over their structural nonzeros (diff and tric 10, omni4 20), the first mcol_nbc rows
// as fused-DPP FMAs broadcasting G[i][r] from lane r (3 x NV). The row form it replaces (lane r: M[r][j] +=
// PG[i][j] from lane j times G[i][r]) needed NX x NV broadcast FMAs: diff 63 -> 37, omni4 165 -> 65.
// pivot = M[0][0] (lane 0's diagonal); NU = 2 also m11 = M[1][1] and m10 = M[0][1] (the input block, whose two
// pivots are then known at once: chol_input_2).
template <class M>
__device__ __forceinline__ void m_block(double (&Lr)[M::NX + M::NU], double& pivot, double& m11, double& m10,
                                        const double (&pg)[M::NX], const double (&gd)[M::NX], const GConst<M>& gc)
{
    constexpr int NX = M::NX, NU = M::NU, NV = NX + NU;
    static_assert(mcol_nbc<M>() == 3, "generated broadcast blocks cover three rows");
    sfor<mcol_nbc<M>(), NX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, NV>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((M::gmask(i) >> r) & 1u) Lr[r] = __builtin_fma(gc.v[i][r], pg[i], Lr[r]);
        });
    });
    if constexpr (NX == 7 && NU == 2) {
        mcol_var_block_7_2_3(Lr, pivot, m11, m10, pg, gd);
    } else {
        mcol_var_block_11_4_3(Lr, pivot, pg, gd);
        m11 = m10 = 0.0;
    }
}

// ---- fp32 split-sigma factorisation (single-direction team kernel) ---------------------------
// The fp64 factor above exists because a bounded state's barrier weight s (up to ~1e12 near the solution) enters
// P_{k+1} and cancels in the Schur complement P_k = Qxx - Qxu Quu^-1 Qux, which fp32 cannot hold. Every bounded state
// of the three models is a reference integrator: row idxbx(c) of [B A] is g = h e_{u_c} + gam e_{x_idxbx(c)} (h = dt,
// gam = 1; static_assert below), so s enters stage k as s g g'. Kept out of P (P = P~ + sum_c s_c e e'), it is added
// at the pivot of input c -- the pivot gets h^2 s, entry (x, u_c) h gam s -- and the one Schur update that cancels s,
// the diagonal (x, x), is evaluated in closed form from the s-free entries a = M[c][c], b = M[x][c], e = M[x][x]:
//     e + gam^2 s - (b + h gam s)^2 / (a + h^2 s) = [s (gam^2 a - 2 h gam b + h^2 e) + (a e - b^2)] / (a + h^2 s)
// (exact algebra, no s - s). tools/fp32_factor_study.py (variant splitsig) on 12288 dumped metric QPs:
// profiles/r06/ab/fp32_factor_study_metric.txt; the same recursion fully in fp32 leaves u0 errors up to 1.2e-3.
template <class M>
struct GConstF {
    float v[M::NX][M::NX + M::NU];
};
template <class M>
__device__ __forceinline__ void gconst_load_f(GConstF<M>& gc, const float (&gcol)[M::NX])
{
    constexpr int NX = M::NX, NV = M::NX + M::NU;
    sfor<mcol_nbc<M>(), NX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, NV>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((M::gmask(i) >> r) & 1u)
                gc.v[i][r] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gcol[i]), r));
            else
                gc.v[i][r] = 0.0f;
        });
    });
}
template <int NX, int NU>
__device__ __forceinline__ void pg_block_f(float (&acc)[NX], const float (&prow)[NX + NU], const float (&gd)[NX])
{
    if constexpr (NX == 7 && NU == 2) pg_block_f32_7_2(acc, prow, gd);
    else pg_block_f32_11_4(acc, prow, gd);
}
// m_block in fp32 (column form; pivot = M[0][0])
template <class M>
__device__ __forceinline__ void m_block_f(float (&Lr)[M::NX + M::NU], float& pivot, const float (&pg)[M::NX],
                                          const float (&gd)[M::NX], const GConstF<M>& gc)
{
    constexpr int NX = M::NX, NU = M::NU, NV = NX + NU;
    static_assert(mcol_nbc<M>() == 3, "generated broadcast blocks cover three rows");
    sfor<mcol_nbc<M>(), NX>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sfor<0, NV>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr ((M::gmask(i) >> r) & 1u) Lr[r] = __builtin_fmaf(gc.v[i][r], pg[i], Lr[r]);
        });
    });
    if constexpr (NX == 7 && NU == 2) mcol_var_block_f32_7_2_3(Lr, pivot, pg, gd);
    else mcol_var_block_f32_11_4_3(Lr, pivot, pg, gd);
}
template <int NX, int NU, int J>
__device__ __forceinline__ void chol_update_f(float (&lr)[NX + NU], float lj, float& piv)
{
    if constexpr (NX == 7 && NU == 2) chol_update_f32_7_2<J>(lr, lj, piv);
    else chol_update_f32_11_4<J>(lr, lj, piv);
}
// The input pivots of M = M~ + sum_c s_c g_c g_c' (row-distributed, lane r holds row r of M~ in Lr; pivot = M~[0][0]
// broadcast), pivots in turn. s_own: the barrier weight s_c of x_{k+1, idxbx(c)} on that state's lane (0 elsewhere).
// Leaves the input columns of the factor in Lr[0..NU) and the Schur complement P~_k in the state block. fail: a
// pivot <= 0 (or NaN).
template <class M>
__device__ __forceinline__ void chol_split_f32(float (&Lr)[M::NX + M::NU], float pivot, float s_own,
                                               const GConstF<M>& gc, int r, bool& fail)
{
    constexpr int NX = M::NX, NU = M::NU;
    sfor<0, NU>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr bool kB = j < M::NBX;
        constexpr int ib = kB ? M::idxbx(j) : 0;  // the state input j drives
        constexpr int xl = NU + ib;                // its lane
        static_assert(!kB || M::gmask(ib) == ((1u << j) | (1u << xl)), "bounded state = integrator of its input");
        float s = 0.0f, h = 0.0f, gam = 0.0f, a = 0.0f, b = 0.0f, e = 0.0f;
        if constexpr (kB) {
            h = gc.v[ib][j];
            gam = gc.v[ib][xl];
            s = bc<xl>(s_own);
            a = pivot;  // s-free entries (after the previous pivots' updates)
            b = Lr[j];  // lane xl: M[xl][j]
            e = Lr[xl]; // lane xl: M[xl][xl]
            const float hs = h * s;
            pivot = __builtin_fmaf(h, hs, pivot);
            Lr[j] += (r == j) ? h * hs : ((r == xl) ? gam * hs : 0.0f);
        }
        if (!(pivot > 0.0f)) fail = true;
        const float rd = __builtin_amdgcn_rsqf(fmaxf(pivot, 1e-30f));
        const float lj = (r >= j) ? Lr[j] * rd : 0.0f;
        Lr[j] = lj;
        chol_update_f<NX, NU, j>(Lr, lj, pivot);
        if constexpr (kB) {
            const float num = __builtin_fmaf(s, gam * gam * a - 2.0f * h * gam * b + h * h * e, a * e - b * b);
            const float den = __builtin_fmaf(h * h, s, a);
            if (r == xl) Lr[xl] = num * frcp(den);
        }
    });
}

// Right-looking Cholesky of a 2 x 2 input block held row-wise (lane r: Lr = row r of M, m00 / m11 / m10 its
// entries broadcast to every lane), leaving the Schur complement in the state block. Both pivots come from the
// block up front -- d0 = M00, d1 = M11 - M10^2 / M00 = det / M00 with det = M00 M11 - M10^2, so
// 1 / sqrt(d1) = sqrt(M00) / sqrt(det) = (M00 / sqrt(M00)) rsq(det) -- and their two rsq + Newton chains run side by
// side instead of one after the other (the second waited for the first column's update). fail: a pivot <= 0.
template <int NX>
__device__ __forceinline__ void chol_input_2(double (&Lr)[NX + 2], double m00, double m11, double m10, int r, bool& fail)
{
    const double det = __builtin_fma(m00, m11, -(m10 * m10));
    if (!(m00 > 0.0) || !(det > 0.0)) fail = true;
    const double rd0 = drsq(fmax(m00, 1e-300));
    const double rq = drsq(fmax(det, 1e-300));
    const double rd1 = (m00 * rd0) * rq;
    const double l0 = Lr[0] * rd0;
    Lr[0] = l0;
    if constexpr (NX == 7) chol_update_np_7_2_0(Lr, l0);
    const double l1 = (r >= 1) ? Lr[1] * rd1 : 0.0;
    Lr[1] = l1;
    if constexpr (NX == 7) chol_update_np_7_2_1(Lr, l1);
    static_assert(NX == 7, "generated for NX = 7 (diff, tric)");
}

template <int NX, int NU, int J>
__device__ __forceinline__ void chol_update(double (&lr)[NX + NU], double lj, double& piv)
{
    if constexpr (NX == 7 && NU == 2) chol_update_7_2<J>(lr, lj, piv);
    else chol_update_11_4<J>(lr, lj, piv);
}
template <int NX, int NU>
__device__ __forceinline__ float dot_x(float acc, float a, const float (&b)[NX])  // acc + sum_l bc_{NU+l}(a) b[l]
{
    if constexpr (NX == 7 && NU == 2) return dot_x_7_2(acc, a, b);
    else return dot_x_11_4(acc, a, b);
}
template <int NX, int NU>
__device__ __forceinline__ float dot_v(float acc, float a, const float (&b)[NX + NU])  // acc + sum_v bc_v(a) b[v]
{
    if constexpr (NX == 7 && NU == 2) return dot_v_7_2(acc, a, b);
    else return dot_v_11_4(acc, a, b);
}

// segmented-Riccati master blocks (team_asm_gen.hpp): NX x NX matrices on the state lanes NU .. NU + NX - 1
template <int NX, int NU>
__device__ __forceinline__ void mst_rowmul(double (&acc)[NX], const double (&a)[NX], const double (&b)[NX])
{
    if constexpr (NX == 7 && NU == 2) mst_rowmul_7_2(acc, a, b);
    else mst_rowmul_11_4(acc, a, b);
}
template <int NX, int NU>
__device__ __forceinline__ void mst_rowmul_lt(double (&acc)[NX], const double (&a)[NX], const double (&b)[NX])
{
    if constexpr (NX == 7 && NU == 2) mst_rowmul_lt_7_2(acc, a, b);
    else mst_rowmul_lt_11_4(acc, a, b);
}
template <int NX, int NU>
__device__ __forceinline__ void mst_rowdot(double (&acc)[NX], const double (&a)[NX], const double (&b)[NX])
{
    if constexpr (NX == 7 && NU == 2) mst_rowdot_7_2(acc, a, b);
    else mst_rowdot_11_4(acc, a, b);
}
template <int NX, int NU>
__device__ __forceinline__ void mst_rowdot_neg(double (&acc)[NX], const double (&a)[NX], const double (&b)[NX])
{
    if constexpr (NX == 7 && NU == 2) mst_rowdot_neg_7_2(acc, a, b);
    else mst_rowdot_neg_11_4(acc, a, b);
}
template <int NX, int NU, int J>
__device__ __forceinline__ void mst_chol(double (&lr)[NX], double lj, double& piv)
{
    if constexpr (NX == 7 && NU == 2) mst_chol_7_2<J>(lr, lj, piv);
    else mst_chol_11_4<J>(lr, lj, piv);
}
template <int NX, int NU, int J>
__device__ __forceinline__ void mst_trsv(double (&u)[NX], double lc, double y)
{
    if constexpr (NX == 7 && NU == 2) mst_trsv_7_2<J>(u, lc, y);
    else mst_trsv_11_4<J>(u, lc, y);
}
template <int NX, int NU>
__device__ __forceinline__ double mst_vdot(double acc, double x, const double (&a)[NX])
{
    if constexpr (NX == 7 && NU == 2) return mst_vdot_7_2(acc, x, a);
    else return mst_vdot_11_4(acc, x, a);
}

// Right-looking Cholesky of the NX x NX matrix held row-wise on the state lanes of a 16-lane row (lane NU + i: row
// i in lr, xi = i), in place: lane NU + i ends with row i of L. rdv[j] = 1 / L[j][j]. A pivot <= thr, or (rel > 0)
// <= rel x the column's original diagonal entry, is dropped (DROP: its column becomes zero, the factor of a
// positive semidefinite matrix; the relative test keeps rounding-level pivots of a nearly singular matrix from
// scaling their column by 1 / sqrt(noise)) or poisons the factor with NaN (!DROP: a breakdown the IPM's NaN test
// reports); a NaN pivot always propagates.
template <int NX, int NU, bool DROP, bool RAW_RSQ = false>
__device__ __forceinline__ void rowchol(double (&lr)[NX], double (&rdv)[NX], int xi, double thr, double rel = 0.0)
{
    double d0 = 0.0;
#pragma unroll
    for (int c = 0; c < NX; c++) d0 = (xi == c) ? lr[c] : d0;
    d0 *= rel;
    double piv = bc64<NU>(lr[0]);
    sfor<0, NX>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const double tj = fmax(thr, bc64<NU + j>(d0));
        const double rq = RAW_RSQ ? __builtin_amdgcn_rsq(piv) : drsq(piv);  // RAW_RSQ: A/B timing only
        const double rd = (piv > tj) ? rq : ((DROP && piv == piv) ? 0.0 : __builtin_nan(""));
        rdv[j] = rd;
        const double lj = (xi >= j) ? lr[j] * rd : 0.0;
        lr[j] = lj;
        if constexpr (j + 1 < NX) mst_chol<NX, NU, j>(lr, lj, piv);
    });
}

// LDS writes of this wave complete before its next LDS reads (the master's cross-lane exchanges within one wave)
__device__ __forceinline__ void lds_fence()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The segment master's step matrix Q = A (I + C A)^-1 = L (I + L' C L)^-1 L' from A = L L' (A, C >= 0; row xi of A
// in Ar, of C in Cr, on lane NU + xi of a 16-lane row), formed as Y Y', Y = L R^-T, R R' = K = I + L' C L: pivots of
// A below 1e-13 of their diagonal entry dropped, K >= I factored without pivoting. sLt: NX x NX doubles of LDS
// scratch private to the row (L' crosses lanes through it). Positive semidefinite by construction; the Woodbury
// form and a factor of C both failed numerically (tools/seg_case_study.py).
template <int NX, int NU>
__device__ __forceinline__ void mst_qform(const double (&Ar)[NX], const double (&Cr)[NX], double (&Q)[NX],
                                          double* sLt, int xi, bool is_x)
{
    double Lp[NX], Lt[NX], V[NX], K[NX], rdv[NX];
#pragma unroll
    for (int c = 0; c < NX; c++) Lp[c] = Ar[c];
    rowchol<NX, NU, true>(Lp, rdv, xi, 0.0, 1e-13);
    if (is_x) {
#pragma unroll
        for (int c = 0; c < NX; c++) sLt[xi * NX + c] = Lp[c];
    }
    lds_fence();
#pragma unroll
    for (int c = 0; c < NX; c++) {
        Lt[c] = sLt[c * NX + xi];
        V[c] = 0.0;
        K[c] = (xi == c) ? 1.0 : 0.0;
    }
    mst_rowmul_lt<NX, NU>(V, Cr, Lp);  // V = C L (L lower triangular: 28 terms)
    mst_rowmul_lt<NX, NU>(K, Lt, V);   // lower triangle of K = I + L' V
    rowchol<NX, NU, false>(K, rdv, xi, 0.5);
    sfor<0, NX>([&](auto jc) {         // Y = L R^-T (row-wise forward substitution), in place of Lp
        constexpr int j = decltype(jc)::value;
        const double y = Lp[j] * rdv[j];
        Lp[j] = y;
        if constexpr (j + 1 < NX) mst_trsv<NX, NU, j>(Lp, K[j], y);
    });
#pragma unroll
    for (int c = 0; c < NX; c++) Q[c] = 0.0;
    mst_rowdot<NX, NU>(Q, Lp, Lp);
}

template <class M>
__device__ __forceinline__ int xcomp(int xi)
{
#pragma unroll
    for (int c = 0; c < M::NBX; c++)
        if (M::idxbx(c) == xi) return c;
    return -1;
}

// Column `col` (slot convention: col < NU input col, else state col - NU) of the RK4 map's sensitivity at
// (x, u), propagated by one lane through the four stages, together with the nominal step xn.
template <class M>
__device__ __forceinline__ void rk4_column(const float* x, const float* u, const KParams& P, int col, float* xn,
                                           float* g)
{
    constexpr int NX = M::NX, NU = M::NU;
    const float h = P.dt;
    float xs[NX], k[NX], acc[NX], s0[NX], s[NX], dacc[NX];
#pragma unroll
    for (int i = 0; i < NX; i++) {
        xs[i] = x[i];
        s0[i] = (col == NU + i) ? 1.0f : 0.0f;
        s[i] = s0[i];
    }
    const float cst[3] = {0.5f, 0.5f, 1.0f};
    const float wgt[4] = {1.0f, 2.0f, 2.0f, 1.0f};
#pragma unroll
    for (int st = 0; st < 4; st++) {
        M::f(xs, u, P, k);
        float S1[NX][1], D1[NX][1];
#pragma unroll
        for (int i = 0; i < NX; i++) S1[i][0] = s[i];
        M::template jvp<1>(xs, S1, P, D1);  // Jx s (the input block of the models is [0; I] on the last NU rows)
        float dk[NX];
#pragma unroll
        for (int i = 0; i < NX; i++) dk[i] = D1[i][0];
#pragma unroll
        for (int q = 0; q < NU; q++) dk[NX - NU + q] += (col == q) ? 1.0f : 0.0f;
#pragma unroll
        for (int i = 0; i < NX; i++) {
            acc[i] = (st == 0) ? k[i] : acc[i] + wgt[st] * k[i];
            dacc[i] = (st == 0) ? dk[i] : dacc[i] + wgt[st] * dk[i];
        }
        if (st < 3) {
            const float ch = cst[st] * h;
#pragma unroll
            for (int i = 0; i < NX; i++) {
                xs[i] = x[i] + ch * k[i];
                s[i] = s0[i] + ch * dk[i];
            }
        }
    }
    const float h6 = h * (1.0f / 6.0f);
#pragma unroll
    for (int i = 0; i < NX; i++) {
        xn[i] = x[i] + h6 * acc[i];
        g[i] = s0[i] + h6 * dacc[i];
    }
}

// Record access. A lane's record is NQ quads of 4 floats, QS floats apart, in one of two stage-block layouts:
//   slot-major [slot][RS] (QS = 4): a lane's record is contiguous;
//   quad-major [quad][slot 0..15][4] (QS = 64): quad i of a team's 16 slots is 256 contiguous bytes, so a
//     dwordx4 access of a team touches 2 cache lines instead of one per two slots.
// Measured per model in same-box A/B runs (ms per tick): omni4 (15 slots, 80-B records) 2.17 slot-major ->
// 1.74 quad-major; diff 1.55 -> 1.57 and tric 4.48 -> 4.62 (9 slots) favour slot-major. RQM picks quad-major for
// teams of more than 12 slots.
template <int NV>
constexpr bool rec_quad_major()
{
    return NV > 12;
}
template <int RS, bool QM>
constexpr int rec_qs() { return QM ? 64 : 4; }  // floats between a lane's consecutive quads
template <int RS, bool QM>
constexpr int rec_lane() { return QM ? 4 : RS; }  // floats between the records of consecutive slots
template <int RS, bool QM>
constexpr int rec_off(int f) { return (f / 4) * rec_qs<RS, QM>() + f % 4; }  // offset of field f in a lane's record


// floats [F0, F1) of a record, one access per quad piece (a piece never crosses a quad)
template <int F0, int F1, int RS, bool QM>
__device__ __forceinline__ void rec_load_range(const float* p, float (&v)[RS])
{
    constexpr int QS = rec_qs<RS, QM>();
    sfor<F0 / 4, (F1 + 3) / 4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int a = (F0 > 4 * q) ? F0 : 4 * q, b = (F1 < 4 * q + 4) ? F1 : 4 * q + 4, L = b - a;
        const float* pq = p + q * QS + (a - 4 * q);
        if constexpr (L == 2 && a % 2 != 0) {  // (unaligned pair: two dword accesses)
            v[a] = pq[0];
            v[a + 1] = pq[1];
        } else if constexpr (L == 4) {
            const float4 t = *reinterpret_cast<const float4*>(pq);
            v[a] = t.x; v[a + 1] = t.y; v[a + 2] = t.z; v[a + 3] = t.w;
        } else if constexpr (L == 3) {
            const float3 t = *reinterpret_cast<const float3*>(pq);
            v[a] = t.x; v[a + 1] = t.y; v[a + 2] = t.z;
        } else if constexpr (L == 2) {
            const float2 t = *reinterpret_cast<const float2*>(pq);
            v[a] = t.x; v[a + 1] = t.y;
        } else {
            v[a] = pq[0];
        }
    });
}

template <int F0, int F1, int RS, bool QM>
__device__ __forceinline__ void rec_store_range(float* p, const float (&v)[RS])
{
    constexpr int QS = rec_qs<RS, QM>();
    sfor<F0 / 4, (F1 + 3) / 4>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int a = (F0 > 4 * q) ? F0 : 4 * q, b = (F1 < 4 * q + 4) ? F1 : 4 * q + 4, L = b - a;
        float* pq = p + q * QS + (a - 4 * q);
        if constexpr (L == 2 && a % 2 != 0) {  // (unaligned pair: two dword accesses)
            pq[0] = v[a];
            pq[1] = v[a + 1];
        } else if constexpr (L == 4) *reinterpret_cast<float4*>(pq) = make_float4(v[a], v[a + 1], v[a + 2], v[a + 3]);
        else if constexpr (L == 3) *reinterpret_cast<float3*>(pq) = make_float3(v[a], v[a + 1], v[a + 2]);
        else if constexpr (L == 2) *reinterpret_cast<float2*>(pq) = make_float2(v[a], v[a + 1]);
        else pq[0] = v[a];
    });
}

// Split records (TeamRec::SPLIT): image fields [lo, hi) <-> memory floats [m0, m0 + hi - lo) of one plane, one access
// per memory quad piece
template <int LO, int HI, int M0, int RS, bool ST>
__device__ __forceinline__ void split_piece(float* mb, float (&v)[RS])
{
    if constexpr (LO < HI) {
        constexpr int ME = M0 + (HI - LO);
        sfor<M0 / 4, (ME + 3) / 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int a = (M0 > 4 * q) ? M0 : 4 * q, b = (ME < 4 * q + 4) ? ME : 4 * q + 4, L = b - a;
            constexpr int f = LO + (a - M0);
            float* pq = mb + a;
            if constexpr (ST) {
                if constexpr (L == 4) *reinterpret_cast<float4*>(pq) = make_float4(v[f], v[f + 1], v[f + 2], v[f + 3]);
                else if constexpr (L == 2 && a % 2 == 0) *reinterpret_cast<float2*>(pq) = make_float2(v[f], v[f + 1]);
                else {
#pragma unroll
                    for (int i = 0; i < L; i++) pq[i] = v[f + i];
                }
            } else {
                if constexpr (L == 4) {
                    const float4 t = *reinterpret_cast<const float4*>(pq);
                    v[f] = t.x; v[f + 1] = t.y; v[f + 2] = t.z; v[f + 3] = t.w;
                } else if constexpr (L == 2 && a % 2 == 0) {
                    const float2 t = *reinterpret_cast<const float2*>(pq);
                    v[f] = t.x; v[f + 1] = t.y;
                } else {
#pragma unroll
                    for (int i = 0; i < L; i++) v[f + i] = pq[i];
                }
            }
        });
    }
}
template <int A, int B>
constexpr int cmax() { return A > B ? A : B; }
template <int A, int B>
constexpr int cmin() { return A < B ? A : B; }
// image [F0, F1) of a split record: core plane entry pc (LR LM Z at 0..3, GV.. GR at 4..), bound plane entry pb
// (TL TU LL LU at 0..3, LB UB at 4..5)
template <class R, int F0, int F1, int RS, bool ST>
__device__ __forceinline__ void split_access(float* pc, float* pb, float (&v)[RS])
{
    split_piece<cmax<F0, 0>(), cmin<F1, 4>(), cmax<F0, 0>(), RS, ST>(pc, v);
    split_piece<cmax<F0, 4>(), cmin<F1, 8>(), cmax<F0, 4>() - 4, RS, ST>(pb, v);
    split_piece<cmax<F0, 8>(), cmin<F1, 10>(), cmax<F0, 8>() - 4, RS, ST>(pb, v);
    split_piece<cmax<F0, R::GV>(), cmin<F1, R::GR + 1>(), cmax<F0, R::GV>() - R::GV + 4, RS, ST>(pc, v);
}
template <class R, int F0, int F1, int RS>
__device__ __forceinline__ void split_load(const float* pc, const float* pb, float (&v)[RS])
{
    split_access<R, F0, F1, RS, false>(const_cast<float*>(pc), const_cast<float*>(pb), v);
}
template <class R, int F0, int F1, int RS>
__device__ __forceinline__ void split_store(float* pc, float* pb, const float (&v)[RS])
{
    split_access<R, F0, F1, RS, true>(pc, pb, const_cast<float (&)[RS]>(v));
}

template <int RS, bool QM>
__device__ __forceinline__ void rec_store(float* p, const float (&v)[RS])
{
    rec_store_range<0, RS, RS, QM>(p, v);
}

// Newton directions of one bounded variable (lower slack tl / multiplier ll, upper tu / lu) for a step dz with
// complementarity targets tgl, tgu:  dt = dz + r (primal),  l*dt + t*dl = tg - l*t  (linearised complementarity).
struct BoundDir {
    float dtl, dtu, dll, dlu;
};
__device__ __forceinline__ BoundDir bound_dir(float dz, float rl, float rr, float tl, float tu, float ll, float lu,
                                              float itl, float itu, float tgl, float tgu)
{
    BoundDir d;
    d.dtl = dz + rl;
    d.dtu = -dz + rr;
    d.dll = (tgl - ll * (tl + rl) - ll * dz) * itl;
    d.dlu = (tgu - lu * (tu + rr) + lu * dz) * itu;
    return d;
}

// Largest step keeping v + a dv >= 0, folded into amax. t = -v / dv is a bound only for dv < 0 (v >= 0): then
// t >= +0; for dv >= 0 it is <= -0, -inf or a NaN. As unsigned integers non-negative floats keep their order and
// every negative float (and -0) is larger than +inf, so one unsigned min drops the non-bounds without a compare /
// select (same-box A/B against the branch form: diff 1.403 -> 1.398 ms, tric 4.386 -> 4.358 ms)
__device__ __forceinline__ float step_bound_r(float amax, float v, float dv)
{
    const float t = -v * frcp(dv);
    return __uint_as_float(min(__float_as_uint(amax), __float_as_uint(t)));
}

}  // namespace
}  // namespace nmpc
