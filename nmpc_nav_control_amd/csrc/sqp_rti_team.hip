// sqp_rti_team.hip -- batched SQP-RTI step, one 16-lane team (one DPP row) per robot instance.
//
// Same algorithm as sqp_rti_lane.hip and oracle/nmpc_oracle.c (RK4 + forward sensitivities, Gauss-Newton
// cost, box bounds, Mehrotra IPM with damped corrector and centring safeguard, square-root Riccati),
// mapped MI355X-first:
//   * four robots per wavefront; inside a team lane v owns QP variable v of every stage (v < NU: input,
//     NU <= v < NU+NX: state), so the stage matrix M = diag(H+Sigma) + (L'[B A])'(L'[B A]) and its Cholesky
//     factor are distributed one row per lane, and every cross-lane operand is a DPP row_newbcast
//     (no LDS, no shuffles through memory);
//   * vector reductions over the team (G * dz for the forward dynamics, mu, step bounds) are 4-step DPP
//     butterflies;
//   * the per-stage record of a team (stage matrix columns, iterate, slacks, multipliers, Riccati factor
//     columns) lives in an instance-interleaved scratch array [stage][field][team][NV], so the four teams
//     of a wave touch 4*NV*4 contiguous bytes per field; the whole working set of B=4096 diff robots at
//     N=40 is ~140 MB and stays in the 256 MB Infinity Cache between passes;
//   * the linearisation is stage-parallel: lane r integrates stages r, r+16, r+32, ...
// The IPM iteration count is per team; a wave iterates until its four teams have converged (finished
// teams take no further steps).
#include "nmpc_kernels.hpp"
#include "team_dpp.hpp"

namespace nmpc {

template <class M>
struct TeamLayout {
    static constexpr int NX = M::NX, NU = M::NU, NV = NX + NU;
    static constexpr int G = 0;  // NX fields: G[i][v] = (v < NU ? B : A)[i][v'] (column v of [B A])
    static constexpr int BV = G + NX;  // b_k[i] in slot i
    static constexpr int Z = BV + 1;   // QP iterate dz (du / dx)
    static constexpr int GR = Z + 1;   // cost gradient
    static constexpr int DZ = GR + 1;  // combined Newton direction
    static constexpr int TL = DZ + 1, TU = TL + 1, LL = TU + 1, LU = LL + 1, LB = LU + 1, UB = LB + 1;
    static constexpr int DZA = UB + 1;  // affine direction of the bounded variable
    static constexpr int LR = DZA + 1;  // Luu^{-1} (g^u + B'p) (u lanes)
    static constexpr int RU = LR + 1;   // u-stationarity residual (u lanes)
    static constexpr int YR = RU + 1;   // unwrapped pose reference (slots 0..2, run mode)
    static constexpr int LM = YR + 1;   // NU fields: row v of the stage factor, columns 0..NU-1
    static constexpr int NF = LM + NU;
};

template <class M>
size_t team_scratch_floats(int N, int stride)
{
    using Lay = TeamLayout<M>;
    return (size_t)(N + 1) * Lay::NF * stride * Lay::NV + 64;
}

namespace {

constexpr float kBreakdownMuT = 1e-6f;
constexpr float kStatRelT = 1e-5f;

template <class M>
__device__ __forceinline__ int xcomp(int xi)
{
#pragma unroll
    for (int c = 0; c < M::NBX; c++)
        if (M::idxbx(c) == xi) return c;
    return -1;
}

template <class M>
__global__ __launch_bounds__(256, 1) void k_sqp_rti_team(KParams P, KArgs a, int mode)
{
    using Lay = TeamLayout<M>;
    constexpr int NX = M::NX, NU = M::NU, NV = Lay::NV, NF = Lay::NF;
    static_assert(NV <= 16, "a team holds at most 16 variables");
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int team = gt >> 4;
    const int r = gt & 15;
    if (team >= a.B) return;  // whole DPP rows leave together
    const int N = P.N;
    const size_t S = (size_t)a.stride;  // resident state stride (capacity)
    const size_t Bn = (size_t)a.B;
    const size_t T = (size_t)a.stride;  // teams in the scratch layout
    const int inst = team;
    float* __restrict__ scr = a.scratch;
    const bool lv = r < NV;
    const bool is_u = r < NU;
    const bool is_x = lv && !is_u;
    const int xi = is_x ? r - NU : 0;
    // bound of this lane's variable (every input is bounded; states on idxbx)
    const int cx = is_x ? xcomp<M>(xi) : -1;
    const bool has_c_u = is_u;  // idxbu = all inputs in the three models
    const bool has_c_x = cx >= 0;
    const float c_lo = is_u ? P.lbu[r < 4 ? r : 0] : (has_c_x ? P.lbx[cx] : 0.0f);
    const float c_hi = is_u ? P.ubu[r < 4 ? r : 0] : (has_c_x ? P.ubx[cx] : 0.0f);
    const float sc = P.dt;
    const float h_stage = is_u ? sc * P.W[NX + r] : (is_x ? sc * P.W[xi] : 0.0f);

#define REC(k, f) scr[(((size_t)(k) * NF + (f)) * T + team) * NV + r]
#define XB(k, j) a.xbar[((size_t)(k) * NX + (j)) * S + inst]
#define UBAR(k, j) a.ubar[((size_t)(k) * NU + (j)) * S + inst]

    // ---- reset -----------------------------------------------------------------------------------------
    if (a.reset && a.reset[inst]) {
        for (int k = r; k <= N; k += 16)
            for (int j = 0; j < NX; j++) XB(k, j) = 0.0f;
        for (int k = r; k < N; k += 16)
            for (int j = 0; j < NU; j++) UBAR(k, j) = 0.0f;
    }
    __threadfence_block();

    // ---- x0 (every lane keeps the full vector) ----------------------------------------------------------
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

    // ---- references: unwrap + pad (run mode, NMPCNavControlDiff.cpp:104-118), terminal weight ----------
    bool hack_eq = false;
    if (mode == kModeRun) {
        const int len = a.traj_len ? a.traj_len[inst] : N + 1;
        float prev = pose_th, px = 0.0f, py = 0.0f, pxo = 0.0f, pyo = 0.0f, pto = 0.0f;
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
            if (r < 3) REC(k, Lay::YR) = (r == 0) ? px : (r == 1 ? py : prev);
            if (k == N - 1) { pxo = px; pyo = py; pto = prev; }
        }
        hack_eq = (px == pxo) && (py == pyo) && (prev == pto);  // NMPCNavControlDiff.cpp:127-139
    }
    // per-lane terminal weight of this lane's state
    float we_lane = 0.0f;
    if (is_x) {
        we_lane = a.We ? a.We[(size_t)xi * Bn + inst] : P.We[xi];
        if (mode == kModeRun && P.terminal_hack && xi < 3) we_lane = (hack_eq ? 100.0f : 1.0f) * P.W[xi];
    }
    // yref(k, j) for the stage-parallel linearisation
    auto yref = [&](int k, int j) -> float {
        if (mode == kModeRun) {
            if (j >= 3) return 0.0f;
            return scr[(((size_t)k * NF + Lay::YR) * T + team) * NV + j];
        }
        return (j < a.ny_in) ? a.yref[((size_t)k * a.ny_in + j) * Bn + inst] : 0.0f;
    };
    // every lane needs the terminal weights of all states for the stage-parallel gradient
    float we_all[NX];
#pragma unroll
    for (int i = 0; i < NX; i++) we_all[i] = bc16(we_lane, NU + i);
    __threadfence_block();  // YR slots written above are read by other lanes of the team (same wave) below

    // ---- P0a: stage-parallel linearisation, gradient, bounds -------------------------------------------
    for (int k = r; k <= N; k += 16) {
        float xb[NX], ub[NU];
#pragma unroll
        for (int j = 0; j < NX; j++) xb[j] = XB(k, j);
#pragma unroll
        for (int j = 0; j < NU; j++) ub[j] = (k < N) ? UBAR(k, j) : 0.0f;
        float* rec = scr + ((size_t)k * NF * T + team) * NV;  // slot base of stage k
        auto put = [&](int f, int slot, float v) { rec[(size_t)f * T * NV + slot] = v; };
        if (k < N) {
            float xn[NX], A[NX][NX], Bm[NX][NU];
            rk4_sens<M>(xb, ub, P, xn, A, Bm);
#pragma unroll
            for (int i = 0; i < NX; i++) {
#pragma unroll
                for (int v = 0; v < NU; v++) put(Lay::G + i, v, Bm[i][v]);
#pragma unroll
                for (int j = 0; j < NX; j++) put(Lay::G + i, NU + j, A[i][j]);
                put(Lay::BV, i, xn[i] - XB(k + 1, i));
            }
#pragma unroll
            for (int v = 0; v < NU; v++) {
                put(Lay::GR, v, sc * P.W[NX + v] * (ub[v] - yref(k, NX + v)));
                put(Lay::LB, v, P.lbu[v] - ub[M::idxbu(v)]);
                put(Lay::UB, v, P.ubu[v] - ub[M::idxbu(v)]);
            }
        }
        if (k >= 1) {
#pragma unroll
            for (int j = 0; j < NX; j++) {
                const float w = (k < N) ? sc * P.W[j] : we_all[j];
                put(Lay::GR, NU + j, w * (xb[j] - yref(k, j)));
            }
#pragma unroll
            for (int c = 0; c < M::NBX; c++) {
                const int j = M::idxbx(c);
                put(Lay::LB, NU + j, P.lbx[c] - xb[j]);
                put(Lay::UB, NU + j, P.ubx[c] - xb[j]);
            }
        }
    }
    __threadfence_block();  // stage records written by other lanes of the team (same wave)

    // ---- P0b: dynamics-feasible initial iterate, slacks and multipliers (forward) -----------------------
    float dxv = is_x ? x0[xi] - XB(0, xi) : 0.0f;  // this lane's state delta at the current stage
    for (int k = 0; k <= N; k++) {
        const bool valid = is_u ? (k < N) : (is_x && k >= 1);
        const float z = is_u ? 0.0f : dxv;
        if (lv) REC(k, Lay::Z) = z;
        if (valid && (has_c_u || has_c_x)) {
            const float lb = REC(k, Lay::LB), ubd = REC(k, Lay::UB);
            const float tl = fmaxf(z - lb, P.thr0), tu = fmaxf(ubd - z, P.thr0);
            REC(k, Lay::TL) = tl;
            REC(k, Lay::TU) = tu;
            REC(k, Lay::LL) = P.mu0 / tl;
            REC(k, Lay::LU) = P.mu0 / tu;
        }
        if (k < N) {
            // dx_{k+1} = A dx_k + b_k = sum over state lanes of column(A) * dx + b
            float nxt = 0.0f;
#pragma unroll
            for (int i = 0; i < NX; i++) {
                const float g = lv ? REC(k, Lay::G + i) : 0.0f;
                const float s = row_sum16(is_x ? g * z : 0.0f);
                if (i == xi) nxt = s;
            }
            const float b = is_x ? scr[(((size_t)k * NF + Lay::BV) * T + team) * NV + xi] : 0.0f;
            dxv = nxt + b;
        }
    }
    int m = 0;
#pragma unroll
    for (int c = 0; c < NU; c++) m += N;
    m += N * M::NBX;
    const float inv_m2 = 0.5f / (float)m;

    // ---- interior-point iterations ----------------------------------------------------------------------
    int status = 0, it_done = 0;
    bool done = false;
    float exit_res[3] = {0.0f, 0.0f, 0.0f};
    float alpha = 0.0f, sigma_mu = 0.0f, eta = 0.0f;
    const bool has_c_any = has_c_u || has_c_x;
    for (int it = 0;; it++) {
        // P1 (backward): update, residuals, adjoint, square-root Riccati factorisation, predictor rhs
        float Lrow[NV];  // this lane's row of the previous stage factor (state lanes carry L_{k+1})
        float pv = 0.0f, piv = 0.0f;
        float res_stat = 0.0f, res_ineq = 0.0f, sum_c = 0.0f, stat_scale = 1.0f, nanf_ = 0.0f;
        bool fail = false;
#pragma unroll
        for (int j = 0; j < NV; j++) Lrow[j] = 0.0f;
        const float a_upd = (it > 0 && !done) ? alpha : 0.0f;
        for (int k = N; k >= 0; k--) {
            const bool vu = is_u && k < N;
            const bool vx = is_x && k >= 1;
            const bool valid = vu || vx;
            float z = lv ? REC(k, Lay::Z) : 0.0f;
            const float g = valid ? REC(k, Lay::GR) : 0.0f;
            float lamdiff = 0.0f, sig = 0.0f, gh = 0.0f;
            if (valid && has_c_any) {
                const float lb = REC(k, Lay::LB), ubd = REC(k, Lay::UB);
                float tl = REC(k, Lay::TL), tu = REC(k, Lay::TU), ll = REC(k, Lay::LL), lu = REC(k, Lay::LU);
                if (a_upd > 0.0f) {
                    const float dz = REC(k, Lay::DZ), dza = REC(k, Lay::DZA);
                    const float rl = z - lb - tl, rr = ubd - z - tu;
                    const float dtla = dza + rl, dtua = -dza + rr;
                    const float dlla = (-ll * (tl + rl) - ll * dza) / tl;
                    const float dlua = (-lu * (tu + rr) + lu * dza) / tu;
                    const float tgl = sigma_mu - eta * dlla * dtla, tgu = sigma_mu - eta * dlua * dtua;
                    const float dtl = dz + rl, dtu = -dz + rr;
                    const float dll = (tgl - ll * (tl + rl) - ll * dz) / tl;
                    const float dlu = (tgu - lu * (tu + rr) + lu * dz) / tu;
                    tl += a_upd * dtl;
                    tu += a_upd * dtu;
                    ll += a_upd * dll;
                    lu += a_upd * dlu;
                    REC(k, Lay::TL) = tl;
                    REC(k, Lay::TU) = tu;
                    REC(k, Lay::LL) = ll;
                    REC(k, Lay::LU) = lu;
                }
                const float zn = (a_upd > 0.0f) ? z + a_upd * REC(k, Lay::DZ) : z;
                const float rl = zn - lb - tl, rr = ubd - zn - tu;
                res_ineq = nan_max(res_ineq, fmaxf(fabsf(rl), fabsf(rr)));
                sum_c += ll * tl + lu * tu;
                lamdiff = ll - lu;
                sig = ll / tl + lu / tu;
                gh = (ll * rl) / tl + ll - (lu * rr) / tu - lu;
            }
            if (a_upd > 0.0f && valid) {
                z += a_upd * REC(k, Lay::DZ);
                REC(k, Lay::Z) = z;
            }
            // column of [B A] of this lane (stage k < N)
            float Gc[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) Gc[i] = (k < N && lv) ? REC(k, Lay::G + i) : 0.0f;
            // adjoint: c_v = sum_l G[l][v] pi_{k+1}[l]
            float cpi = 0.0f;
            if (k < N) {
#pragma unroll
                for (int l = 0; l < NX; l++) cpi += Gc[l] * bc16(piv, NU + l);
            }
            const float hz = ((k < N) ? h_stage : we_lane) * z;
            const float base = hz + g - lamdiff + cpi;
            float ghat = gh;
            if (vu) {
                REC(k, Lay::RU) = base;
                res_stat = nan_max(res_stat, fabsf(base));
                stat_scale = fmaxf(stat_scale, fmaxf(fabsf(cpi), fmaxf(fabsf(g), fabsf(lamdiff))));
                ghat += base;
            }
            const float pi_new = vx ? base : 0.0f;
            if (!valid) ghat = 0.0f;
            if (ghat != ghat || sig != sig) nanf_ = 1.0f;
            if (k == N) {
#pragma unroll
                for (int j = 0; j < NV; j++) Lrow[j] = 0.0f;
                if (is_x) {
#pragma unroll
                    for (int j = 0; j < NX; j++)
                        if (j == xi) Lrow[NU + j] = sqrtf(fmaxf(we_lane + sig, 0.0f));
                }
                pv = is_x ? ghat : 0.0f;
            } else {
                const bool full = k >= 1;  // stage 0 has no state variables (x0 fixed)
                // LBA column v = L_{k+1}' G[:, v]; L[l][i] lives in lane NU+l at Lrow[NU+i]
                float lba[NX];
#pragma unroll
                for (int i = 0; i < NX; i++) {
                    float s = 0.0f;
#pragma unroll
                    for (int l = i; l < NX; l++) s += bc16(Lrow[NU + i], NU + l) * Gc[l];
                    lba[i] = s;
                }
                // this lane's row of M = D + LBA' LBA
                const float dg = (valid ? h_stage + sig : 1.0f);
                float Mr[NV];
#pragma unroll
                for (int b = 0; b < NV; b++) {
                    float s = (b == r) ? dg : 0.0f;
#pragma unroll
                    for (int i = 0; i < NX; i++) s += lba[i] * bc16(lba[i], b);
                    Mr[b] = s;
                }
                // Cholesky, row-distributed: Lr[j] = row r of the factor
                float Lr[NV];
#pragma unroll
                for (int j = 0; j < NV; j++) Lr[j] = 0.0f;
#pragma unroll
                for (int j = 0; j < NV; j++) {
                    if (!full && j >= NU) break;
                    float s = Mr[j];
#pragma unroll
                    for (int q = 0; q < j; q++) s -= Lr[q] * bc16(Lr[q], j);
                    const float pivot = bc16(s, j);
                    float d;
                    bool zero_col = false;
                    if (j < NU) {
                        if (!(pivot > 0.0f)) fail = true;
                        d = sqrtf(fmaxf(pivot, 1e-30f));
                    } else {
                        const float mjj = bc16(Mr[j], j);
                        zero_col = !(pivot > 1e-10f * (1.0f + fabsf(mjj)));
                        d = zero_col ? 0.0f : sqrtf(pivot);
                    }
                    if (r == j) Lr[j] = d;
                    else if (r > j) Lr[j] = zero_col ? 0.0f : s / d;
                }
                if (lv) {
#pragma unroll
                    for (int q = 0; q < NU; q++) REC(k, Lay::LM + q) = Lr[q];
                }
                // rhs: w = g^ + G' p_{k+1}; forward substitution over the input block
                float y = ghat;
#pragma unroll
                for (int l = 0; l < NX; l++) y += Gc[l] * bc16(pv, NU + l);
                float my_lr = 0.0f;
#pragma unroll
                for (int j = 0; j < NU; j++) {
                    const float lrj = bc16(y / Lr[j], j);  // valid in lane j (diagonal)
                    if (r == j) my_lr = lrj;
                    if (r > j) y -= Lr[j] * lrj;
                }
                if (is_u) REC(k, Lay::LR) = my_lr;
                pv = is_x ? y : 0.0f;
#pragma unroll
                for (int j = 0; j < NV; j++) Lrow[j] = Lr[j];
            }
            piv = pi_new;
        }
        // team reductions
        sum_c = row_sum16(lv ? sum_c : 0.0f);
        res_ineq = row_max16(lv ? res_ineq : 0.0f);
        res_stat = row_max16(lv ? res_stat : 0.0f);
        stat_scale = row_max16(stat_scale);
        nanf_ = row_max16(nanf_);
        const float mu = sum_c * inv_m2;
        if (!done) {
            exit_res[0] = res_stat;
            exit_res[1] = res_ineq;
            exit_res[2] = mu;
            bool stop = false;
            if (nanf_ > 0.0f || mu != mu) {
                status = 1;
                stop = true;
            } else if (fail) {
                status = (mu <= kBreakdownMuT && res_ineq <= P.tol_ineq * 10.0f) ? 0 : 4;
                stop = true;
            } else {
                const bool stat_ok = res_stat <= P.tol_stat || res_stat <= kStatRelT * stat_scale;
                if (res_ineq <= P.tol_ineq && ((stat_ok && mu <= P.tol_comp) || mu <= 1e-2f * P.tol_comp)) stop = true;
                if (it >= P.iter_max) stop = true;
            }
            if (stop) {
                done = true;
                it_done = it;
            }
        }
        if (__all(done)) break;

        // P2 (forward): affine direction, maximal step, mu_aff polynomial
        float s1 = 0.0f, s2 = 0.0f, amax = 1e30f;
        {
            float dx = 0.0f;
            for (int k = 0; k <= N; k++) {
                const bool vu = is_u && k < N;
                const bool vx = is_x && k >= 1;
                const bool valid = vu || vx;
                float Lr[NU];
#pragma unroll
                for (int q = 0; q < NU; q++) Lr[q] = (k < N && lv) ? REC(k, Lay::LM + q) : 0.0f;
                float du_all[NU];
                if (k < N) {
                    const float lr = is_u ? REC(k, Lay::LR) : 0.0f;
                    float w[NU];
#pragma unroll
                    for (int q = 0; q < NU; q++) w[q] = bc16(lr, q) + row_sum16(is_x ? Lr[q] * dx : 0.0f);
#pragma unroll
                    for (int qq = 0; qq < NU; qq++) {
                        const int q = NU - 1 - qq;
                        float s = w[q];
#pragma unroll
                        for (int j = q + 1; j < NU; j++) s -= bc16(Lr[q], j) * du_all[j];
                        du_all[q] = s / bc16(Lr[q], q);
                    }
#pragma unroll
                    for (int q = 0; q < NU; q++) du_all[q] = -du_all[q];
                }
                float dz = 0.0f;
#pragma unroll
                for (int q = 0; q < NU; q++)
                    if (r == q) dz = du_all[q];
                if (is_x) dz = (k >= 1) ? dx : 0.0f;
                if (valid && has_c_any) {
                    const float z = REC(k, Lay::Z);
                    const float lb = REC(k, Lay::LB), ubd = REC(k, Lay::UB);
                    const float tl = REC(k, Lay::TL), tu = REC(k, Lay::TU), ll = REC(k, Lay::LL), lu = REC(k, Lay::LU);
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
                    REC(k, Lay::DZA) = dz;
                }
                if (k < N) {
                    float nxt = 0.0f;
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        const float g = lv ? REC(k, Lay::G + i) : 0.0f;
                        const float s = row_sum16(lv ? g * dz : 0.0f);
                        if (i == xi) nxt = s;
                    }
                    dx = nxt;
                }
            }
        }
        s1 = row_sum16(lv ? s1 : 0.0f);
        s2 = row_sum16(lv ? s2 : 0.0f);
        amax = row_min16(lv ? amax : 1e30f);
        const float alpha_aff = fminf(1.0f, amax);
        float sigma;
        {
            const float mu_aff = (sum_c + alpha_aff * s1 + alpha_aff * alpha_aff * s2) * inv_m2;
            float sg = (mu > 0.0f) ? mu_aff / mu : 0.0f;
            sg = fmaxf(sg, 0.0f);
            sigma = fminf(sg * sg * sg, 1.0f);
        }

        for (int pass = 1; pass <= 2; pass++) {
            if (pass == 1) {
                sigma_mu = sigma * mu;
                eta = alpha_aff;
            } else {
                if (alpha >= 0.1f) break;
                sigma_mu = fmaxf(sigma, 0.3f) * mu;
                eta = 0.0f;
            }
            // P3 (backward): corrector rhs through the stored factorisation
            {
                float pvc = 0.0f;
                for (int k = N; k >= 0; k--) {
                    const bool vu = is_u && k < N;
                    const bool vx = is_x && k >= 1;
                    const bool valid = vu || vx;
                    float ghat = 0.0f;
                    if (valid && has_c_any) {
                        const float z = REC(k, Lay::Z);
                        const float lb = REC(k, Lay::LB), ubd = REC(k, Lay::UB);
                        const float tl = REC(k, Lay::TL), tu = REC(k, Lay::TU), ll = REC(k, Lay::LL),
                                    lu = REC(k, Lay::LU);
                        const float dza = REC(k, Lay::DZA);
                        const float rl = z - lb - tl, rr = ubd - z - tu;
                        const float dtla = dza + rl, dtua = -dza + rr;
                        const float dlla = (-ll * (tl + rl) - ll * dza) / tl;
                        const float dlua = (-lu * (tu + rr) + lu * dza) / tu;
                        const float tgl = sigma_mu - eta * dlla * dtla, tgu = sigma_mu - eta * dlua * dtua;
                        ghat = -(tgl - ll * rl) / tl + ll + (tgu - lu * rr) / tu - lu;
                    }
                    if (vu) ghat += REC(k, Lay::RU);
                    if (k == N) {
                        pvc = is_x ? ghat : 0.0f;
                    } else {
                        float y = ghat;
#pragma unroll
                        for (int l = 0; l < NX; l++) {
                            const float g = lv ? REC(k, Lay::G + l) : 0.0f;
                            y += g * bc16(pvc, NU + l);
                        }
                        float Lr[NU];
#pragma unroll
                        for (int q = 0; q < NU; q++) Lr[q] = lv ? REC(k, Lay::LM + q) : 0.0f;
                        float my_lr = 0.0f;
#pragma unroll
                        for (int j = 0; j < NU; j++) {
                            const float lrj = bc16(y / Lr[j], j);
                            if (r == j) my_lr = lrj;
                            if (r > j) y -= Lr[j] * lrj;
                        }
                        if (is_u) REC(k, Lay::LR) = my_lr;
                        pvc = is_x ? y : 0.0f;
                    }
                }
            }
            // P4 (forward): combined direction and its step length
            {
                float dx = 0.0f;
                amax = 1e30f;
                for (int k = 0; k <= N; k++) {
                    const bool vu = is_u && k < N;
                    const bool vx = is_x && k >= 1;
                    const bool valid = vu || vx;
                    float Lr[NU];
#pragma unroll
                    for (int q = 0; q < NU; q++) Lr[q] = (k < N && lv) ? REC(k, Lay::LM + q) : 0.0f;
                    float du_all[NU];
                    if (k < N) {
                        const float lr = is_u ? REC(k, Lay::LR) : 0.0f;
                        float w[NU];
#pragma unroll
                        for (int q = 0; q < NU; q++) w[q] = bc16(lr, q) + row_sum16(is_x ? Lr[q] * dx : 0.0f);
#pragma unroll
                        for (int qq = 0; qq < NU; qq++) {
                            const int q = NU - 1 - qq;
                            float s = w[q];
#pragma unroll
                            for (int j = q + 1; j < NU; j++) s -= bc16(Lr[q], j) * du_all[j];
                            du_all[q] = s / bc16(Lr[q], q);
                        }
#pragma unroll
                        for (int q = 0; q < NU; q++) du_all[q] = -du_all[q];
                    }
                    float dz = 0.0f;
#pragma unroll
                    for (int q = 0; q < NU; q++)
                        if (r == q) dz = du_all[q];
                    if (is_x) dz = (k >= 1) ? dx : 0.0f;
                    if (valid) REC(k, Lay::DZ) = dz;
                    if (valid && has_c_any) {
                        const float z = REC(k, Lay::Z);
                        const float lb = REC(k, Lay::LB), ubd = REC(k, Lay::UB);
                        const float tl = REC(k, Lay::TL), tu = REC(k, Lay::TU), ll = REC(k, Lay::LL),
                                    lu = REC(k, Lay::LU);
                        const float dza = REC(k, Lay::DZA);
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
                        float nxt = 0.0f;
#pragma unroll
                        for (int i = 0; i < NX; i++) {
                            const float g = lv ? REC(k, Lay::G + i) : 0.0f;
                            const float s = row_sum16(lv ? g * dz : 0.0f);
                            if (i == xi) nxt = s;
                        }
                        dx = nxt;
                    }
                }
                amax = row_min16(lv ? amax : 1e30f);
                alpha = fminf(1.0f, P.tau * amax);
            }
        }
    }

    // ---- full SQP step + outputs ----------------------------------------------------------------------
    if (status == 0) {
        for (int k = 0; k <= N; k++) {
            if (is_x) {
                const float nv = (k == 0) ? x0[xi] : XB(k, xi) + REC(k, Lay::Z);
                XB(k, xi) = nv;
                if (a.xtraj) a.xtraj[((size_t)k * NX + xi) * Bn + inst] = nv;
            }
            if (is_u && k < N) {
                const float nv = UBAR(k, r) + REC(k, Lay::Z);
                UBAR(k, r) = nv;
                if (a.utraj) a.utraj[((size_t)k * NU + r) * Bn + inst] = nv;
            }
        }
    }
    __threadfence_block();
    if (r == 0) {
        float u0[NU];
#pragma unroll
        for (int j = 0; j < NU; j++) {
            u0[j] = UBAR(0, j);
            if (a.u0) a.u0[(size_t)j * Bn + inst] = u0[j];
        }
        if (a.x1) {
#pragma unroll
            for (int j = 0; j < NX; j++) a.x1[(size_t)j * Bn + inst] = XB(1, j);
        }
        if (a.status) a.status[inst] = status;
        if (a.qp_iter) a.qp_iter[inst] = it_done;
        if (a.qp_res) {
#pragma unroll
            for (int j = 0; j < 3; j++) a.qp_res[(size_t)j * Bn + inst] = exit_res[j];
        }
        if (mode == kModeRun && status == 0) {
            float rr[M::NBX], cmd[3];
#pragma unroll
            for (int i = 0; i < M::NBX; i++) {
                rr[i] = x0[M::idxbx(i)] + u0[i] * P.dt_ctrl;
                a.carried[(size_t)i * S + inst] = rr[i];
            }
            M::inverse_kin(rr, P, cmd);
            if (a.cmd) {
#pragma unroll
                for (int j = 0; j < 3; j++) a.cmd[(size_t)j * Bn + inst] = cmd[j];
            }
        }
    }
#undef REC
#undef XB
#undef UBAR
}

}  // namespace

template <class M>
hipError_t launch_sqp_rti_team(const KParams& P, const KArgs& a, int mode, hipStream_t stream)
{
    if (a.B <= 0) return hipSuccess;
    const int block = 256;  // 16 teams
    const long long threads = (long long)a.B * 16;
    const int grid = (int)((threads + block - 1) / block);
    hipLaunchKernelGGL(k_sqp_rti_team<M>, dim3(grid), dim3(block), 0, stream, P, a, mode);
    return hipGetLastError();
}

template hipError_t launch_sqp_rti_team<Diff2>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_team<Omni4>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_team<Tric3>(const KParams&, const KArgs&, int, hipStream_t);
template size_t team_scratch_floats<Diff2>(int, int);
template size_t team_scratch_floats<Omni4>(int, int);
template size_t team_scratch_floats<Tric3>(int, int);

}  // namespace nmpc
