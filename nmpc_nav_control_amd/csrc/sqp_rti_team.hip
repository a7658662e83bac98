// sqp_rti_team.hip -- batched SQP-RTI step, one 16-lane team (one DPP row) per robot instance.
//
// Same algorithm as oracle/nmpc_oracle.c (RK4 + forward sensitivities, Gauss-Newton cost, box bounds,
// Mehrotra IPM with damped corrector and centring safeguard, Riccati recursion),
// mapped MI355X-first:
//   * four robots per wavefront; inside a team lane v owns QP variable v of every stage (v < NU: input,
//     NU <= v < NU+NX: state); cross-lane operands are DPP row_newbcast broadcasts, fused into the
//     multiply-accumulates (v_fmac_f32_dpp / v_fmac_f64_dpp);
//   * the stage factor is a classic Riccati step in fp64: lane NU+i carries row i of the cost-to-go Hessian
//     P_{k+1}; PG = P_{k+1}[B A] and the rows of M = D + [B A]' PG are fused fp64 DPP blocks
//     (team_asm_gen.hpp), then a right-looking Cholesky of the NU x NU input block leaves the Schur complement
//     P_k in the state block (near the solution the barrier weights of active bounds reach 1e12, and fp32
//     Schur complements cancel catastrophically). The input columns of the factor are stored in fp32 and every
//     solve with them runs in fp32 (u0 error ~1e-4 against the fp64 oracle, DESIGN.md "Algorithm and precision");
//   * rows of [B A] that do not depend on the state (model trait NGV) live in registers for the whole launch;
//     only the NGV varying rows are stored per stage;
//   * each lane's per-stage record (slacks, multipliers, iterate, directions, factor row, Jacobian column) is
//     RS contiguous floats at [team][stage][slot][RS]: one record = RS/4 dwordx4 loads, and every sweep
//     prefetches the next stage's record while the current stage computes (the ~170 MB working set of 4096
//     robots stays in the 256 MB Infinity Cache);
//   * the linearisation is column-parallel: lane v integrates the nominal RK4 step and propagates column v of
//     its sensitivity, and the initial (dynamics-feasible) iterate is simulated in the same forward pass.
// The IPM iteration count is per team; a wave iterates until its four teams have converged (finished teams
// skip their loads and stores).
#include "nmpc_kernels.hpp"
#include "team_common.hpp"
#include "path_march.hpp"

namespace nmpc {

#ifdef NMPC_STAMPS
// diagnostic build only: s_memtime at phase boundaries for the first team of the first 256 waves
constexpr int kStampIts = 64;
__device__ unsigned long long g_stamps[256][2 + 4 * kStampIts];
#define STAMP(slot)                                                                                              \
    do {                                                                                                         \
        if (r == 0 && (team & 3) == 0 && (team >> 2) < 256) g_stamps[team >> 2][(slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// fine-grained stamps inside one P1 stage body (iteration 2, stage 20)
__device__ unsigned long long g_stamps_p1[256][8];
// end of the split launches' stage-parallel P0 part (row 0 of the first robot of each group of 4)
__device__ unsigned long long g_stamps_pa[256];
// end of the corrector backward sweep (C1) of iteration it, first team of the first 256 waves
__device__ unsigned long long g_stamps_c1[256][kStampIts];
#define STAMPC1()                                                                                                \
    do {                                                                                                         \
        if (it < kStampIts && r == 0 && (team & 3) == 0 && (team >> 2) < 256)                                   \
            g_stamps_c1[team >> 2][it] = __builtin_amdgcn_s_memtime();                                           \
    } while (0)
#define STAMPF(slot)                                                                                             \
    do {                                                                                                         \
        if (it == 2 && k == 20 && r == 0 && (team & 3) == 0 && (team >> 2) < 256)                                 \
            g_stamps_p1[team >> 2][(slot)] = __builtin_amdgcn_s_memtime();                                        \
    } while (0)
#else
#define STAMP(slot) ((void)0)
#define STAMPF(slot) ((void)0)
#define STAMPC1() ((void)0)
#endif

template <class M>
size_t team_scratch_floats(int N, int stride)
{
    // the lane records [robot][stage][slot][RSS], the DZ plane [robot][stage][16], then the row-parallel kernel's
    // dummy stage blocks [256 robots][4 waves][16][RSS] and dummy DZ rows [256][4][16] (sqp_rti_rowpar.hip)
    return (size_t)stride * (N + 1) * 16 * (TeamRec<M>::RSS + 1) + (size_t)256 * 4 * 16 * (TeamRec<M>::RSS + 1) + 64;
}

namespace {
#ifndef LIGHT_D
#define LIGHT_D 4  // record buffers of the forward light sweeps (F0, F1)
#endif
#ifndef LIGHT_DC
#define LIGHT_DC LIGHT_D  // record buffers of the corrector backward sweep (C1)
#endif
#ifndef P1_D
#define P1_D 2  // record buffers of the factorisation sweep (2: ping-pong)
#endif
#ifdef NMPC_STAMPS
constexpr int kStampItsC = kStampIts;
#else
constexpr int kStampItsC = 0;
#endif

// MS: store the slack / multiplier quad only where a bound lives (launches with more waves than SIMDs, where the
// record traffic shows: tric N=60 B=8192 4.47 -> 4.39 ms; with one wave per SIMD the exec-mask switches cost
// more than the bytes save: diff N=40 B=4096 1.555 -> 1.566 ms)
// SD: one direction per IPM iteration (P1 builds the rhs with the centring target sigma mu, one forward sweep
// computes the direction, the step and the complementarity polynomial that predicts the next mu) instead of
// Mehrotra's predictor-corrector (P1 + F0 + C1 + F1 sweeps)
// zeros: the source of a cold robot's warm-start multiplier loads (load_l in P0)
__device__ float g_zero4[4];
// split records (TeamRec::SPLIT): the bound pair of a slot without a bound -- TL TU LL LU | LB UB -- as P0 writes
// it for bounded slots outside their stage range (kFar slacks and bounds, zero multipliers)
__device__ __attribute__((aligned(16))) float g_rec_sentinel[8] = {kFar, kFar, 0.0f, 0.0f, -kFar, kFar, 0.0f, 0.0f};

// MODE is a template parameter: kModeSolve, kModeRun, or kModeRunPath (run mode with the in-kernel path march,
// a.segs set). As runtime arguments their branches inside P0's stage loop (reference unwrap, yref or pose-reference
// loads, and a pose load from either LDS or global memory, i.e. a flat load) made the compiler's waits drain the
// whole memory counter, the stage's record stores and the prefetched rows included
constexpr int kModeRunPath = 2;
template <class M, bool MS, bool SD, int MODE, bool SP>
__global__ __launch_bounds__(256, 1) void k_sqp_rti_team(KParams P, KArgs a)
{
    constexpr int mode = MODE == kModeRunPath ? kModeRun : MODE;
    using R = TeamRec<M, SD>;
    constexpr int NX = M::NX, NU = M::NU, NV = R::NV, NGV = R::NGV, RS = R::RS, RSS = R::RSS;
    constexpr bool QM = rec_quad_major<NV>();
    constexpr int KS = 16 * RSS;  // floats per stage block (16 slots of RSS stored floats)
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    // split launches (a.split: small batches on an otherwise idle chip): one 256-lane block per robot. Row 0 of
    // the block is the robot's team; rows 1-15 share the stage-parallel part of P0 with it and leave.
    const int team = a.split ? (int)blockIdx.x : (gt >> 4);
    const int row = a.split ? (int)(threadIdx.x >> 4) : 0;
    const int r = gt & 15;
#ifdef NMPC_HYBRID
    // hybrid launch (A/B build): the first hyb_n[0] ranks of the order run the segmented kernel on another stream
    const int hoff = (a.hyb_role == 1) ? a.hyb_n[0] : 0;
#else
    constexpr int hoff = 0;
#endif
    if (team >= a.B - hoff) return;  // whole DPP rows leave together
    const int N = P.N;
    const size_t S = (size_t)a.stride;  // resident state stride (capacity)
    const size_t Bn = (size_t)a.B;
    const int inst = a.order ? a.order[hoff + team] : team;  // difficulty-ordered placement (schedule.hip)
    const bool lv = r < NV;
    const bool is_u = r < NU;
    const bool is_x = lv && !is_u;
    const int xi = is_x ? r - NU : 0;
    const int cx = is_x ? xcomp<M>(xi) : -1;
    const bool has_b = is_u || cx >= 0;  // bounded slot: every input (idxbu = all), states on idxbx
    const float sc = P.dt;
    // this lane's stage weight, read once: indexed by the lane, the W entries are vector loads from the kernel
    // arguments, and inside P0's loop each one waited on vmcnt(0), i.e. on the previous stage's record stores
    const float w_lane = is_u ? P.W[NX + r] : (is_x ? P.W[xi] : 0.0f);
    const float h_stage = sc * w_lane;
    float lo_b = 0.0f, hi_b = 0.0f;
#pragma unroll
    for (int q = 0; q < NU; q++)
        if (r == q) { lo_b = P.lbu[q]; hi_b = P.ubu[q]; }
#pragma unroll
    for (int c = 0; c < M::NBX; c++)
        if (cx == c) { lo_b = P.lbx[c]; hi_b = P.ubx[c]; }
    // this lane's record of stage k: tbase + k * KS
    // idle slots (r >= NV) alias slot 0's record: their (unpredicated) loads then read valid data and touch no
    // extra cache lines; they never store
    // the robot's records (indexed by the robot, not the team slot, so that they carry its multipliers to its next
    // solve whatever the placement)
    float* const tbase = a.scratch + (size_t)inst * (N + 1) * KS + (lv ? r : 0) * rec_lane<RSS, QM>();
    // every lane's own slot (idle lanes: one nobody reads), for P0's unconditional record stores
    float* const tbase_own = a.scratch + (size_t)inst * (N + 1) * KS + r * rec_lane<RSS, QM>();
    // a record nobody reads (slot 15 of the robot's stage-N block: the idle slot of every model), the target of
    // stores that lanes without work issue unconditionally
    float* const tdummy = a.scratch + (size_t)inst * (N + 1) * KS + (size_t)N * KS + 15 * rec_lane<RSS, QM>();
    // split records (R::SPLIT, TeamRec): this lane's core and bound plane entries of stage 0 (stage k: + k CS,
    // + k kb) in the robot's record region; slots without a bound (and idle slots) read the sentinel pair with
    // stride 0; the dummy pair is tdummy (past the planes)
    constexpr bool SPL = R::SPLIT_OK && SP;  // split record planes (TeamRec::SPLIT, KArgs::rec_split)
    float* const pc0 = a.scratch + (size_t)inst * (N + 1) * KS + (lv ? r : 0) * R::CW;
    float* const pb0 = has_b ? a.scratch + (size_t)inst * (N + 1) * KS + (size_t)(N + 1) * R::CS +
                                   (is_u ? r : NU + (cx >= 0 ? cx : 0)) * R::CW
                             : g_rec_sentinel;
    const int kb = has_b ? R::BS : 0;
    // this lane's DZ in the dense plane after the records: dzbase + k * 16 (every lane its own float)
    float* const dzbase = a.scratch + (size_t)a.sstride * (N + 1) * KS + (size_t)inst * (N + 1) * 16 + r;
    // IPM warm start: the bound multipliers of the robot's previous successful solve are still in its records, in
    // this launch's layout when its tag matches (nmpc_batch.h NMPC_WARM_TAG_*)
    const bool warm = P.warm && a.warm && a.warm[inst] == a.warm_tag && !(a.reset && a.reset[inst]);

#define XB(k, j) a.xbar[((size_t)(k) * NX + (j)) * S + inst]
#define UBAR(k, j) a.ubar[((size_t)(k) * NU + (j)) * S + inst]

    STAMP(0);
    // ---- reset -----------------------------------------------------------------------------------------
    if (a.reset && a.reset[inst]) {
        for (int k = r; k <= N; k += 16)
            for (int j = 0; j < NX; j++) XB(k, j) = 0.0f;
        for (int k = r; k < N; k += 16)
            for (int j = 0; j < NU; j++) UBAR(k, j) = 0.0f;
        __threadfence_block();
    }

    // ---- path-following tick (nmpc_batch_run_path): getNextNPoses in-kernel ------------------------------
    // Lane 0 of the team marches the robot's path (PathDiscretizer.cpp:14-63, path_march.hpp, fp64 without
    // contraction: bit-identical poses to k_path_discretize) and records the path parameter of each pose in the
    // team's LDS slice; the rest is padded with the path end (:58-63). The team's 16 lanes then evaluate the
    // poses 16 at a time (atan2 and all), so no lane waits in a divergent emit. A team's lanes share the wave
    // and LDS accesses of a wave retire in order, so P0 reads the poses from LDS directly afterwards.
    // LDS: path mode and split run launches: [teams][N+1] path parameters, then [teams][N+1][3] float poses
    // (split: one team); split launches then the serial P0 pass's stage inputs
    extern __shared__ double s_path[];
    constexpr bool path = MODE == kModeRunPath;  // (the launcher picks it exactly when a.segs is set)
    const bool traj_lds = path || (a.split && mode == kModeRun);
    const int nslot = a.split ? 1 : 16;
    const int tslot = a.split ? 0 : (int)(threadIdx.x >> 4);
    float* const my_traj = reinterpret_cast<float*>(s_path + nslot * (N + 1)) + (size_t)tslot * (N + 1) * 3;
    float* const s_stg = reinterpret_cast<float*>(s_path) + (traj_lds ? (size_t)nslot * (N + 1) * 5 : 0);
    if (path && row == 0) {
        double* const my_u = s_path + (size_t)tslot * (N + 1);
        const nmpc_path_segment* S = a.segs + (size_t)inst * a.seg_stride;
        const int n = a.nseg[inst];
        if (r == 0) {
            const int cnt = path_march(S, n, a.nearest_u[inst], a.period, N + 1, [&](int j, double su) { my_u[j] = su; });
            for (int j = cnt; j <= N; j++) my_u[j] = (double)n;
        }
        for (int j = r; j <= N; j += 16) {
            double px, py, pt;
            path_pose(S, n, my_u[j], a.holo, &px, &py, &pt);
            my_traj[j * 3 + 0] = (float)px;
            my_traj[j * 3 + 1] = (float)py;
            my_traj[j * 3 + 2] = (float)pt;
            if (a.traj_out) {
                a.traj_out[((size_t)j * 3 + 0) * Bn + inst] = (float)px;
                a.traj_out[((size_t)j * 3 + 1) * Bn + inst] = (float)py;
                a.traj_out[((size_t)j * 3 + 2) * Bn + inst] = (float)pt;
            }
        }
    }

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
    float x0_lane = 0.0f;
#pragma unroll
    for (int j = 0; j < NX; j++)
        if (xi == j) x0_lane = x0[j];

    // terminal weight of this lane's state (solve mode: caller's W_e; run mode: constructor W_e + diff hack)
    float we_lane = 0.0f;
    if (is_x) we_lane = (mode != kModeRun && a.We) ? a.We[(size_t)xi * Bn + inst] : P.We[xi];

    // ---- P0: linearisation (lane v: nominal step + column v), gradient, bounds, feasible initial iterate --
    // Split launches: the RK4 integrations and every global load of P0 do not depend on each other; only the
    // initial-iterate simulation (and the reference unwrap) is a recursion over the stages. The block's 16 rows
    // (4 waves) take stages row, row + 16, ... and, after a block barrier, leave each lane's stage inputs in LDS ([k][field][lane], SF
    // fields: zbar, yref entry, warm multipliers, defect b_k = xn_i - xbar_{k+1,i}, the NGV varying Jacobian
    // rows) and run-mode reference poses in row 0's pose slice; row 0 then runs the serial pass from LDS only.
    constexpr int SF = 5 + NGV;
    if (a.split) {
        const int len_a = (mode == kModeRun) ? ((a.traj_len && !path) ? a.traj_len[inst] : N + 1) : 0;
        // a stage's global inputs, loaded one stage (of this row) ahead while the current one integrates
        struct In {
            float x[NX], u[NU], y, xnext, tq;
            float2 l;
        };
        auto ld = [&](int k, In& v) {
            const int kk = k <= N ? k : N;
#pragma unroll
            for (int j = 0; j < NX; j++) v.x[j] = XB(kk, j);
            const int ku = kk < N ? kk : N - 1;
#pragma unroll
            for (int j = 0; j < NU; j++) v.u[j] = UBAR(ku, j);
            v.xnext = XB(kk < N ? kk + 1 : N, xi);
            v.y = 0.0f;
            v.tq = 0.0f;
            if (mode != kModeRun) {
                const int j = is_u ? NX + r : xi;
                v.y = (lv && j < a.ny_in) ? a.yref[((size_t)kk * a.ny_in + j) * Bn + inst] : 0.0f;
            } else if (!path && r < 3) {
                const int kt = kk < len_a ? kk : (len_a > 0 ? len_a - 1 : 0);
                v.tq = a.traj[((size_t)kt * 3 + r) * Bn + inst];
            }
            v.l = warm ? *reinterpret_cast<const float2*>(SPL ? pb0 + (size_t)kk * kb + 2
                                                              : tbase + (size_t)kk * KS + rec_off<RS, QM>(R::LL))
                       : make_float2(0.0f, 0.0f);
        };
        In cur, nxt;
        ld(row, cur);
        for (int k = row; k <= N; k += 16) {
            ld(k + 16, nxt);
            if (mode == kModeRun && !path && r < 3) my_traj[k * 3 + r] = cur.tq;
            float xn[NX], g[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) { xn[i] = 0.0f; g[i] = 0.0f; }
            float bk = 0.0f;
            if (k < N) {
                rk4_column<M>(cur.x, cur.u, P, lv ? r : NU, xn, g);
#pragma unroll
                for (int i = 0; i < NX; i++)
                    if (is_x && xi == i) bk = xn[i] - cur.xnext;
            }
            float zb = 0.0f;
#pragma unroll
            for (int j = 0; j < NU; j++)
                if (r == j) zb = cur.u[j];
#pragma unroll
            for (int j = 0; j < NX; j++)
                if (is_x && xi == j) zb = cur.x[j];
            float* const st = s_stg + (size_t)k * SF * 16 + r;
            st[0] = zb;
            st[16] = cur.y;
            st[32] = cur.l.x;
            st[48] = cur.l.y;
            st[64] = bk;
#pragma unroll
            for (int i = 0; i < NGV; i++) st[(5 + i) * 16] = g[i];
            cur = nxt;
        }
        __syncthreads();  // every row's stage inputs are in LDS
        if (row != 0) return;
#ifdef NMPC_STAMPS
        if (r == 0 && (team & 3) == 0 && (team >> 2) < 256) g_stamps_pa[team >> 2] = __builtin_amdgcn_s_memtime();
#endif
    }
    const int len = (mode == kModeRun) ? ((a.traj_len && !path) ? a.traj_len[inst] : N + 1) : 0;
    float ref_x = 0.0f, ref_y = 0.0f, ref_t = pose_th, prv_x = 0.0f, prv_y = 0.0f, prv_t = 0.0f;
    // Iterate rows are read two stages ahead (every lane of a team reads the same addresses: one request per
    // wave), the reference row likewise.
    auto load_row = [&](int k, float (&xr)[NX], float (&ur)[NU], float (&tr)[3]) {
        const int kk = k <= N ? k : N;
#pragma unroll
        for (int j = 0; j < NX; j++) xr[j] = XB(kk, j);
        const int ku = kk < N ? kk : N - 1;
#pragma unroll
        for (int j = 0; j < NU; j++) ur[j] = UBAR(ku, j);
        if (mode == kModeRun) {
            const int kt = kk < len ? kk : (len > 0 ? len - 1 : 0);
#pragma unroll
            for (int j = 0; j < 3; j++) tr[j] = path ? my_traj[kt * 3 + j] : a.traj[((size_t)kt * 3 + j) * Bn + inst];
        } else {
            tr[0] = tr[1] = tr[2] = 0.0f;
        }
    };
    float xb[NX], ub[NU], tr[3], xb1[NX], ub1[NU], tr1[3];
    load_row(0, xb, ub, tr);
    load_row(1, xb1, ub1, tr1);
    // constant rows of [B A] (rows >= NGV) from stage 0, before the sweep: lane v holds column v (gcol), lane
    // NU+xi holds row xi (grow), so the initial-iterate dynamics below need only NGV row sums
    float gcol[NX], grow[NV];
    {
        float xn0[NX], g0[NX];
        rk4_column<M>(xb, ub, P, lv ? r : NU, xn0, g0);
#pragma unroll
        for (int i = 0; i < NX; i++) gcol[i] = (lv && i >= NGV) ? g0[i] : 0.0f;
        sfor<0, NV>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            float sv = 0.0f;
#pragma unroll
            for (int i = NGV; i < NX; i++) {
                const float t = bc<v>(gcol[i]);
                if (is_x && xi == i) sv = t;
            }
            grow[v] = sv;
        });
    }
    float dx = is_x ? x0_lane - XB(0, xi) : 0.0f;  // this lane's state delta at the current stage
    float sum_c0 = 0.0f;  // complementarity of the initial point (its mean sets the first SD target)
    // warm start: the previous multipliers (LL, LU) of the stage, prefetched one stage ahead
    // (the flag selects the address, not the value: a cold team reads a zero pair. A load whose value is only
    // used under the team's warm flag is issued under that lane mask, and the compiler's waits for every later load
    // of the loop then drain the whole memory counter)
    auto load_l = [&](int k) -> float2 {
        const int kk = k <= N ? k : N;
        const float* const src = warm ? (SPL ? pb0 + (size_t)kk * kb + 2 : tbase + (size_t)kk * KS + rec_off<RS, QM>(R::LL))
                                      : g_zero4;
        return *reinterpret_cast<const float2*>(src);
    };
    // One stage of the serial pass: reference (run mode: unwrap + pad), cost gradient, bounds / slacks /
    // multipliers, the stage record, and the dynamics-feasible initial state of the next stage. Inputs: this
    // lane's iterate entry zbar, its yref entry (solve mode) or the stage's pose ref (run mode), its warm
    // multipliers, the NGV varying Jacobian rows of its column and its defect b_k.
    auto p0_body = [&](int k, float zbar, float yr_in, const float (&trk)[3], float2 lp, const float (&g)[NX],
                       float bk) __attribute__((always_inline)) {
        // stage reference of this lane: run mode unwraps + pads the pose refs (NMPCNavControlDiff.cpp:104-118),
        // entries >= 3 of yref are left at zero
        float yr = yr_in;
        if (mode == kModeRun) {
            // branch-free (selects): a divergent branch here (len is per team) made the compiler's waits at its
            // join drain the whole memory counter, the stage's record stores included
            const bool in = k < len;
            const float th = trk[2], d = th - ref_t;
            const float thu = (d > kPi) ? th - 2.0f * kPi : ((d < -kPi) ? th + 2.0f * kPi : th);
            ref_x = in ? trk[0] : ref_x;
            ref_y = in ? trk[1] : ref_y;
            ref_t = in ? thu : ref_t;
            if (k == N - 1) { prv_x = ref_x; prv_y = ref_y; prv_t = ref_t; }
            // (one select per value: the nested conditional compiled to lane-mask branches)
            float v = 0.0f;
            v = (is_x && xi == 2) ? ref_t : v;
            v = (is_x && xi == 1) ? ref_y : v;
            v = (is_x && xi == 0) ? ref_x : v;
            yr = v;
        }
        float rec[RS];
#pragma unroll
        for (int f = 0; f < RS; f++) rec[f] = 0.0f;
        const bool vu = is_u && k < N, vx = is_x && k >= 1;
        const bool valid = vu || vx;
        // gradient of the Gauss-Newton cost (stage weights scaled by dt, terminal weight unscaled). Every per-lane
        // condition of this body is a select: as lane-mask branches they cost P0 about 14 branch regions per stage
        float w = sc * w_lane;
        if (k == N) {  // (k is wave-uniform)
            float wt = we_lane;
            if (mode == kModeRun && P.terminal_hack) {  // NMPCNavControlDiff.cpp:127-139
                const bool eq = (ref_x == prv_x) && (ref_y == prv_y) && (ref_t == prv_t);
                const float wh = (eq ? 100.0f : 1.0f) * w_lane;
                const bool hk = is_x && xi < 3;
                wt = hk ? wh : wt;
                we_lane = hk ? wh : we_lane;
            }
            w = vx ? wt : w;
        }
        rec[R::GR] = valid ? w * (zbar - yr) : 0.0f;
        // iterate, bounds, slacks, multipliers
        const float z = vx ? dx : 0.0f;
        rec[R::Z] = z;
        // slots without a bound (or outside their stage range) get a sentinel bound at +-kFar with slack kFar
        // and zero multipliers: every bounded-variable expression of the sweeps then vanishes on them (r = 0,
        // Sigma = 0, no step bound), so the sweeps need no per-lane branches
        {
            const bool bd = valid && has_b;
            const float lb = lo_b - zbar, ubd = hi_b - zbar;
            const float tl = fmaxf(z - lb, P.thr0), tu = fmaxf(ubd - z, P.thr0);
            // cold: t lambda = mu0; warm: the previous multipliers, floored at kappa / t
            // (previous multipliers capped at kWarmLambdaCap: a feasible QP of this OCP ends with multipliers of
            // the size of its weights, < 1e2; a runaway value from a struggling solve would start the IPM at a huge
            // complementarity)
            // (one division per slack: with one per branch of the warm flag, a per-team value, the compiler split
            // the lanes around two division sequences)
            const float num = warm ? P.warm_kappa : P.mu0;
            const float ql = num / tl, qu = num / tu;
            const float ll0 = warm ? fmaxf(fminf(lp.x, kWarmLambdaCap), ql) : ql;
            const float lu0 = warm ? fmaxf(fminf(lp.y, kWarmLambdaCap), qu) : qu;
            rec[R::LB] = bd ? lb : -kFar;
            rec[R::UB] = bd ? ubd : kFar;
            rec[R::TL] = bd ? tl : kFar;
            rec[R::TU] = bd ? tu : kFar;
            rec[R::LL] = bd ? ll0 : 0.0f;
            rec[R::LU] = bd ? lu0 : 0.0f;
            const float c0 = ll0 * tl + lu0 * tu;
            sum_c0 += bd ? c0 : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < NGV; i++) rec[R::GV + i] = (k < N && lv) ? g[i] : 0.0f;
        // 15-slot teams (omni4): unconditional (the idle lane stores zeros / sentinels into its own unused
        // slot). A store under a lane mask may or may not be issued, so the compiler's waits for the next loads
        // drain the whole memory counter, these stores included. Same-box A/B: omni4 kernel 1.303 -> 1.256 ms;
        // diff (7 idle lanes, +78 % P0 store bytes) 1.043 -> 1.065 ms, so 9-slot teams keep the masked store
        // (profiles/r02/ab/uncond_stores.txt)
        if constexpr (NV > 12) rec_store_range<0, RSS, RS, QM>(tbase_own + (size_t)k * KS, rec);
#ifdef P0_MASKED_STORE
        else if (lv) rec_store_range<0, RSS, RS, QM>(tbase + (size_t)k * KS, rec);
#else
        // 9-slot teams: the idle lanes all store into the team's dummy record (one record's bytes, not seven)
        else if constexpr (SPL)
            split_store<R, 0, R::GR + 1, RS>(lv ? pc0 + (size_t)k * R::CS : tdummy,
                                             (lv && has_b) ? pb0 + (size_t)k * kb : tdummy + R::CW, rec);
        else rec_store_range<0, RSS, RS, QM>(lv ? tbase + (size_t)k * KS : tdummy, rec);
#endif
        if constexpr (kDzPlane) dzbase[(size_t)k * 16] = 0.0f;  // P1 of iteration 0 applies a zero step
        // dynamics-feasible initial states: dx_{k+1} = A dx_k + b_k (inputs start at du = 0, dx_0 = x0 - xbar_0);
        // row i of [B A] dz: NGV row sums over the columns + the constant rows held in grow
        if (k < N) {
            const float dzd = is_x ? dx : 0.0f;
            float nxt = dot_v<NX, NU>(0.0f, dzd, grow);
#pragma unroll
            for (int i = 0; i < NGV; i++) {
                const float sr = row_sum16(lv ? g[i] * dzd : 0.0f);
                if (xi == i) nxt = sr;
            }
            dx = is_x ? nxt + bk : 0.0f;
        }
    };
    if (a.split) {
        // split launches: every input from LDS. A loop of its own: merged with the global-load loop below, the
        // LDS values waited on vmcnt(0), i.e. on the previous stage's record stores (about one memory latency
        // per stage). Nothing is in flight past this point but the loop's own stores: the waits the compiler
        // would otherwise place inside the loop for the loads above (len, x0) wait on those stores too.
        __builtin_amdgcn_s_waitcnt(0);
        // the stage inputs are read from LDS one stage ahead (each dependent LDS read costs a round trip of the
        // one wave that runs this pass)
        struct Stg {
            float v[5], g[NGV], t[3];
        };
        auto lds_ld = [&](int k, Stg& o) {
            const int kk = k <= N ? k : N;
            const float* const st = s_stg + (size_t)kk * SF * 16 + r;
#pragma unroll
            for (int f = 0; f < 5; f++) o.v[f] = st[f * 16];
#pragma unroll
            for (int i = 0; i < NGV; i++) o.g[i] = st[(5 + i) * 16];
#pragma unroll
            for (int j = 0; j < 3; j++) o.t[j] = (mode == kModeRun) ? my_traj[kk * 3 + j] : 0.0f;
        };
        Stg cur, nxt;
        lds_ld(0, cur);
        for (int k = 0; k <= N; k++) {
            lds_ld(k + 1, nxt);
            float g[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) g[i] = (i < NGV && k < N) ? cur.g[i < NGV ? i : 0] : 0.0f;
            p0_body(k, cur.v[0], cur.v[1], cur.t, make_float2(cur.v[2], cur.v[3]), g, cur.v[4]);
            cur = nxt;
        }
    } else {
        // three row buffers used in turn (the loop unrolled by 3, compile-time buffer indices): buffer i holds stage
        // k + i while the loop is at stage k and is refilled with stage k + 3 after its body. A rotation by copies
        // (xb = xb1; xb1 = xb2) copied registers whose loads were still in flight, and each copy waited for every
        // memory operation issued before it (a full drain per stage)
        struct Row {
            float xb[NX], ub[NU], tr[3], yr;
            float2 lp;
        };
        auto load_p0 = [&](int k, Row& o) {
            load_row(k, o.xb, o.ub, o.tr);
            o.lp = load_l(k);
            o.yr = 0.0f;
            if (mode != kModeRun) {  // (unconditional load of a valid entry, then a select)
                const int kk = k <= N ? k : N;
                const int j = is_u ? NX + r : xi;
                const bool use = lv && j < a.ny_in;
                const float v = a.yref[((size_t)kk * a.ny_in + (use ? j : 0)) * Bn + inst];
                o.yr = use ? v : 0.0f;
            }
        };
        Row rw[3];
#pragma unroll
        for (int j = 0; j < NX; j++) { rw[0].xb[j] = xb[j]; rw[1].xb[j] = xb1[j]; }
#pragma unroll
        for (int j = 0; j < NU; j++) { rw[0].ub[j] = ub[j]; rw[1].ub[j] = ub1[j]; }
#pragma unroll
        for (int j = 0; j < 3; j++) { rw[0].tr[j] = tr[j]; rw[1].tr[j] = tr1[j]; }
        rw[0].lp = load_l(0);
        rw[1].lp = load_l(1);
        rw[0].yr = rw[1].yr = 0.0f;
        if (mode != kModeRun) {
            Row t0, t1;
            load_p0(0, t0);
            load_p0(1, t1);
            rw[0].yr = t0.yr;
            rw[1].yr = t1.yr;
        }
        for (int k0 = 0;; k0 += 3) {
            bool stop = false;
            sfor<0, 3>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if (stop) return;
                const int k = k0 + i;
                load_p0(k + 2, rw[(i + 2) % 3]);  // two stages ahead (clamped)
                const Row& c = rw[i];
                const Row& n1 = rw[(i + 1) % 3];
                float xn[NX], g[NX];
#pragma unroll
                for (int q = 0; q < NX; q++) { xn[q] = 0.0f; g[q] = 0.0f; }
                if (k < N) rk4_column<M>(c.xb, c.ub, P, lv ? r : NU, xn, g);
                float zbar = 0.0f;
#pragma unroll
                for (int j = 0; j < NU; j++)
                    if (r == j) zbar = c.ub[j];
#pragma unroll
                for (int j = 0; j < NX; j++)
                    if (is_x && xi == j) zbar = c.xb[j];
                float bk = 0.0f;
#pragma unroll
                for (int q = 0; q < NX; q++)
                    if (xi == q) bk = xn[q] - n1.xb[q];
                p0_body(k, zbar, c.yr, c.tr, c.lp, g, bk);
                if (k == N) stop = true;
            });
            if (stop) break;
        }
    }
    // e_r: places the diagonal D of M = D + G'PG with one multiply per entry instead of two selects (same-box
    // A/B: diff N=40 B=4096 +0.8 %, B=1024 +1.2 %, tric +0.6 %; profiles/r02/ab/onehot.txt)
    double onehot[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) onehot[j] = (r == j) ? 1.0 : 0.0;
    double gcol64[NX];
#pragma unroll
    for (int i = 0; i < NX; i++) gcol64[i] = (double)gcol[i];
#ifdef NMPC_MROW
    constexpr bool kMcol = false;  // A/B: the row form for every model
#elif defined(NMPC_MCOL_ALL)
    constexpr bool kMcol = true;  // A/B: the column form for every model
#else
    constexpr bool kMcol = M::kMcolForm;  // per model (nmpc_models.hpp)
#endif
    // -DNMPC_F32_FACTOR (A/B build): the single-direction rule factors in fp32 with the bounded states' barrier
    // weights split off (team_common.hpp chol_split_f32). As accurate as the fp64 factor (same IPM counts in the
    // closed loop, every full-batch replay green) but slower on every config, 3-10 % (profiles/r06/ab/fp32_factor.txt,
    // DESIGN.md section 5), so the product keeps the fp64 factorisation
#ifdef NMPC_F32_FACTOR
    constexpr bool kF32 = SD && kMcol;
#else
    constexpr bool kF32 = false;
#endif
    using FT = std::conditional_t<kF32, float, double>;
    GConst<M> gcs;  // the constant rows of [B A] as uniform operands of the column-form M block (m_block)
    GConstF<M> gcf;  // the same in fp32 (m_block_f32, chol_split_f32)
    if constexpr (kF32) gconst_load_f<M>(gcf, gcol);
    else if constexpr (kMcol) gconst_load<M>(gcs, gcol);
    // fp32 factor: a bounded state's barrier weight stays out of P_k (lane NU + idxbx(c), c = cx); s_next carries it
    // from stage k's body to stage k - 1's pivot of input c
    const bool split_lane = kF32 && is_x && cx >= 0;

    STAMP(1);
    // infeasibility threshold of this robot: qp_infeas_lambda scaled by its largest weight (terminal hack included)
    const float lam_thr = P.infeas_lam * fmaxf(1.0f, fmaxf(P.wmax, row_max16(is_x ? we_lane : 0.0f)) * 0.1f);
    const int m = N * NU + N * M::NBX;
    const float inv_m2 = 0.5f / (float)m;
    sum_c0 = row_sum16(lv ? sum_c0 : 0.0f);

    // dx_{k+1} (lane NU+i) = sum_v G_k[i][v] dz_v: NGV row sums over the stored columns + the constant rows
    auto dyn = [&](const float (&rc)[RS], float dzv) -> float {
        float nxt = 0.0f;
#pragma unroll
        for (int i = 0; i < NGV; i++) {
            const float s = row_sum16(lv ? rc[R::GV + i] * dzv : 0.0f);
            if (xi == i) nxt = s;
        }
        const float cr = dot_v<NX, NU>(0.0f, dzv, grow);
        return (xi >= NGV) ? cr : nxt;
    };
    // column v of [B A] at a stage (rows < NGV from the record)
    auto column = [&](const float (&rc)[RS], float (&Gc)[NX]) {
#pragma unroll
        for (int i = 0; i < NX; i++) Gc[i] = (i < NGV) ? rc[R::GV + (i < NGV ? i : 0)] : gcol[i];
    };
    // Stage sweeps k = k0, k0 + dir, ..., k1 with the next stage's record (sweep2: the next two) in flight while
    // body(k, rec) runs. The loop is unrolled by the number of register buffers, which are used in turn (no
    // copies between them), and the loads are never predicated: a conditional load or a buffer copy would make
    // the compiler move the in-flight registers, which waits for the load. Lanes that do not sweep (idle slots,
    // converged teams) re-read one fixed record instead; past k1 the pointer stays on k1.
    // P1's loads of one stage: its record fields and (DZ plane) the lane's DZ; dz points at the plane entry of
    // the stage whose record p points at (p - tbase = k KS <=> dz - dzbase = 16 k)
    auto p1_load = [&](int kk, float (&v)[RS]) {
        if constexpr (SPL) split_load<R, R::P1L0, R::P1L1, RS>(pc0 + (size_t)kk * R::CS, pb0 + (size_t)kk * kb, v);
        else rec_load_range<R::P1L0, R::P1L1, RS, QM>(tbase + (size_t)kk * KS, v);
        if constexpr (kDzPlane) v[R::DZ] = dzbase[(size_t)kk * 16];
    };
    auto sweep = [&](int k0, int k1, int dir, bool ld, auto&& body) {  // 2 buffers (compute-heavy P1)
        const int sd = ld ? dir : 0;  // stage step of this lane's loads (0: a lane that does not sweep)
        int kp = k0;
        float ra[RS], rb[RS];
        p1_load(kp, ra);
        for (int k = k0;; k += 2 * dir) {
            const int kp1 = (k == k1) ? kp : kp + sd;
            p1_load(kp1, rb);
            body(k, ra);
            if (k == k1) break;
            const int kp2 = (k + dir == k1) ? kp1 : kp1 + sd;
            p1_load(kp2, ra);
            body(k + dir, rb);
            if (k + dir == k1) break;
            kp = kp2;
        }
    };
    // D buffers: buf[i] holds stage k + i*dir while the loop is at k; after body(k + i*dir) it is refilled with
    // stage k + (i + D)*dir (clamped at k1), so D - 1 records are in flight during every body
    auto sweepd = [&](auto dc, auto f0c, auto fc, int k0, int k1, int dir, bool ld, auto&& body) {
        constexpr int D = decltype(dc)::value;
        constexpr int F0 = decltype(f0c)::value, F = decltype(fc)::value;  // floats [F0, F) this sweep reads
        const int sd = ld ? dir : 0;
        float buf[D][RS];
        int kp = k0;
        int kl = k0;
        // P1 with P1_D > 2 buffers also takes DZ from the plane (the light sweeps read only the prefix)
        auto load = [&](int kk, float (&v)[RS]) {
            if constexpr (SPL) split_load<R, F0, F, RS>(pc0 + (size_t)kk * R::CS, pb0 + (size_t)kk * kb, v);
            else rec_load_range<F0, F, RS, QM>(tbase + (size_t)kk * KS, v);
            if constexpr (kDzPlane && F == R::P1L1) v[R::DZ] = dzbase[(size_t)kk * 16];
        };
        load(kp, buf[0]);
        sfor<1, D>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            kp = (kl == k1) ? kp : kp + sd;
            kl = (kl == k1) ? kl : kl + dir;
            load(kp, buf[i]);
        });
        for (int k = k0;; k += D * dir) {
            bool stop = false;
            sfor<0, D>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if (stop) return;
                body(k + i * dir, buf[i]);
                if (k + i * dir == k1) {
                    stop = true;
                    return;
                }
                kp = (kl == k1) ? kp : kp + sd;
                kl = (kl == k1) ? kl : kl + dir;
                load(kp, buf[i]);
            });
            if (stop) break;
        }
    };
    // ---- interior-point iterations ----------------------------------------------------------------------
    int status = 0, it_done = 0;
    bool done = false;
    float exit_res[3] = {0.0f, 0.0f, 0.0f};
    float alpha = 0.0f, sigma_mu = 0.0f, eta = 0.0f, mu_prev = 3.0e38f;
    // SD: centring target of the next direction, built into P1's rhs. The first direction: sigma = sd_hi (no
    // previous step) and the initial point's mu (P0; mu0 for a cold start, where every pair has t lambda = mu0)
    float tg_rhs = P.sd_hi * sum_c0 * inv_m2;
    for (int it = 0;; it++) {
        // P1 (backward): apply the previous step, residuals, adjoint, fp64 classic Riccati factorisation,
        // predictor rhs
        FT Lrow[NV];  // lane NU+i: row i of P_{k+1} (the state block of the previous stage's M after its pivots)
#pragma unroll
        for (int j = 0; j < NV; j++) Lrow[j] = 0.0;
        float s_next = 0.0f;  // fp32 factor: the split lane's barrier weight of stage k + 1 (0 elsewhere)
        float pv = 0.0f, piv = 0.0f;
        float res_stat = 0.0f, res_ineq = 0.0f, sum_c = 0.0f, max_c = 0.0f, stat_scale = 1.0f, nanf_ = 0.0f;
        float lam_max = 0.0f;
        bool fail = false;
        const bool act = lv && !done;
        const float a_upd = (it > 0 && !done) ? alpha : 0.0f;
        // P1_D record buffers: the heavy sweep's next records are in flight for P1_D - 1 stage bodies (at four
        // waves per CU a record load from the Infinity Cache takes about one stage body)
#if P1_D > 2
        sweepd(std::integral_constant<int, P1_D>{}, std::integral_constant<int, R::P1L0>{},
               std::integral_constant<int, R::P1L1>{}, N, 0, -1, act, [&](int k, float (&rc)[RS]) {
#else
        sweep(N, 0, -1, act, [&](int k, float (&rc)[RS]) {
#endif
            STAMPF(0);
            const bool vu = is_u && k < N;
            const bool vx = is_x && k >= 1;
            const bool valid = vu || vx;
            const bool bnd = valid && has_b;
            // Branch-free: slots without a bound hold the kFar sentinel (P0), for which every bounded-variable
            // term below is 0; only the slack / multiplier step is masked (it would move lambda off zero).
            float z = rc[R::Z];
            float tl = rc[R::TL], tu = rc[R::TU], ll = rc[R::LL], lu = rc[R::LU];
            const float lb = rc[R::LB], ubd = rc[R::UB];
            {
                const float dz = rc[R::DZ];
                const float rl = z - lb - tl, rr = ubd - z - tu;
                const float itl = frcp(tl), itu = frcp(tu);
                float tgl = sigma_mu, tgu = sigma_mu;  // SD: the previous direction's target
                if constexpr (!SD) {
                    const BoundDir da = bound_dir(rc[R::DZA], rl, rr, tl, tu, ll, lu, itl, itu, 0.0f, 0.0f);
                    tgl = sigma_mu - eta * da.dll * da.dtl;
                    tgu = sigma_mu - eta * da.dlu * da.dtu;
                }
                const BoundDir d = bound_dir(dz, rl, rr, tl, tu, ll, lu, itl, itu, tgl, tgu);
                const float ab = bnd ? a_upd : 0.0f, av = valid ? a_upd : 0.0f;
                tl += ab * d.dtl;
                tu += ab * d.dtu;
                ll += ab * d.dll;
                lu += ab * d.dlu;
                z += av * dz;
                rc[R::Z] = z;
                rc[R::TL] = tl;
                rc[R::TU] = tu;
                rc[R::LL] = ll;
                rc[R::LU] = lu;
            }
            const float rl = z - lb - tl, rr = ubd - z - tu;
            const float itl = frcp(tl), itu = frcp(tu);
            res_ineq = fmaxf(res_ineq, fmaxf(fabsf(rl), fabsf(rr)));  // NaN: caught by nanf_ (ghat, sig)
            sum_c += ll * tl + lu * tu;
            max_c = fmaxf(max_c, fmaxf(ll * tl, lu * tu));
            lam_max = fmaxf(lam_max, fmaxf(ll, lu));  // 0 on the kFar-sentinel slots
            const float lamdiff = ll - lu;
            const float sig = ll * itl + lu * itu;
            // predictor rhs (zero complementarity target); SD: the centring target tg_rhs (0 on kFar slots)
            const float gh = SD ? ll * rl * itl + ll - lu * rr * itu - lu - tg_rhs * itl + tg_rhs * itu
                                : ll * rl * itl + ll - lu * rr * itu - lu;
            STAMPF(1);
            float Gc[NX];
            column(rc, Gc);
            // adjoint: c_v = sum_l G[l][v] pi_{k+1}[l]
            const float cpi = (k < N) ? dot_x<NX, NU>(0.0f, piv, Gc) : 0.0f;
            const float hz = ((k < N) ? h_stage : we_lane) * z;
            const float g = rc[R::GR];
            const float base = hz + g - lamdiff + cpi;
            rc[R::RU] = base;  // read back for the u slots only
            res_stat = fmaxf(res_stat, vu ? fabsf(base) : 0.0f);
            stat_scale = fmaxf(stat_scale, vu ? fmaxf(fabsf(cpi), fmaxf(fabsf(g), fabsf(lamdiff))) : 0.0f);
            const float ghat = valid ? (vu ? gh + base : gh) : 0.0f;
            const float pi_new = vx ? base : 0.0f;
            if (ghat != ghat || sig != sig) nanf_ = 1.0f;
            if (k == N) {
                // terminal: P_N = diag(W_e + Sigma) on the state lanes (fp32 factor: Sigma of a bounded state in
                // s_next instead)
                const FT d = is_x ? (FT)fmaxf(we_lane + (split_lane ? 0.0f : sig), 0.0f) : (FT)0.0;
#pragma unroll
                for (int j = 0; j < NV; j++) Lrow[j] = (is_x && j == r) ? d : (FT)0.0;
                s_next = split_lane ? sig : 0.0f;
                pv = is_x ? ghat : 0.0f;
            } else if constexpr (kF32) {
                // fp32 split-sigma factorisation: M~ = D~ + G' P~ G with the bounded states' barrier weights out of
                // D~ and P~ (team_common.hpp chol_split_f32 enters those of stage k + 1 at their inputs' pivots)
                float pg[NX];
#pragma unroll
                for (int i = 0; i < NX; i++) pg[i] = 0.0f;
                STAMPF(2);
                pg_block_f<NX, NU>(pg, Lrow, Gc);
                STAMPF(3);
                const float dg = valid ? h_stage + (split_lane ? 0.0f : sig) : 1.0f;
                float Lr[NV];
#pragma unroll
                for (int j = 0; j < NV; j++) Lr[j] = (j == r) ? dg : 0.0f;
                float pivot;  // = M[0][0]
                m_block_f<M>(Lr, pivot, pg, Gc, gcf);
                STAMPF(4);
                chol_split_f32<M>(Lr, pivot, s_next, gcf, r, fail);
                s_next = (split_lane && vx) ? sig : 0.0f;
                STAMPF(5);
#pragma unroll
                for (int q = 0; q < NU; q++) rc[R::LM + q] = Lr[q];
                // rhs: w = g^ + G' p_{k+1}; forward substitution over the input block (fp32)
                float y = dot_x<NX, NU>(ghat, pv, Gc);
                float my_lr = 0.0f;
                sfor<0, NU>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    const float lrj = bc<j>(y * frcp(Lr[j]));  // (y_j / L_jj) from lane j
                    if (r == j) my_lr = lrj;
                    y -= Lr[j] * lrj;
                });
                rc[R::LR] = my_lr;
                pv = is_x ? y : 0.0f;
#pragma unroll
                for (int j = 0; j < NV; j++) Lrow[j] = Lr[j];
            } else {
                double Gd[NX];
#pragma unroll
                for (int l = 0; l < NX; l++) Gd[l] = (l < NGV) ? (double)Gc[l] : gcol64[l];
                // classic Riccati in fp64: PG column v = P_{k+1} G[:, v] (P[i][l] sits in lane NU+i at Lrow[NU+l]),
                // row r of M = D + G' P G, then the right-looking row-distributed Cholesky of the input block only:
                // after the NU input pivots the state block of M holds the Schur complement
                // Qxx - Qxu Quu^-1 Qux = P_k, which the state lanes carry to the next stage
                double pg[NX];
#pragma unroll
                for (int i = 0; i < NX; i++) pg[i] = 0.0;
                STAMPF(2);
                pg_block<NX, NU>(pg, Lrow, Gd);
                STAMPF(3);
                const double dg = valid ? (double)h_stage + (double)sig : 1.0;
                double Lr[NV];
#pragma unroll
                for (int j = 0; j < NV; j++) Lr[j] = onehot[j] * dg;
                double pivot;  // = M[0][0]
                bool seq_pivots = true;
                if constexpr (kMcol) {
                    double m11, m10;
                    m_block<M>(Lr, pivot, m11, m10, pg, Gd, gcs);  // column form: uniform constant rows + 3 broadcast rows
                    STAMPF(4);
#ifdef NMPC_SEQ_PIVOTS
                    constexpr bool kPiv2 = false;  // A/B: the pivots one after the other for every model
#else
                    constexpr bool kPiv2 = M::kPivotsUpFront;
#endif
                    if constexpr (NU == 2 && kPiv2) {
                        chol_input_2<NX>(Lr, pivot, m11, m10, r, fail);  // both pivots up front
                        seq_pivots = false;
                    } else {
                        (void)m11;
                        (void)m10;
                    }
                } else {
                    mrow_pg_block<NX, NU>(Lr, pivot, pg, Gd);  // the row form (NX x NV broadcast FMAs)
                    STAMPF(4);
#ifdef NMPC_ROW_PIV2
                    if constexpr (NU == 2) {  // A/B: both input pivots up front with the row form too
                        const double m11 = bc64<1>(Lr[1]), m10 = bc64<1>(Lr[0]);
                        chol_input_2<NX>(Lr, pivot, m11, m10, r, fail);
                        seq_pivots = false;
                    }
#endif
                }
                if (seq_pivots) sfor<0, NU>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    if (!(pivot > 0.0)) fail = true;
                    const double rd = drsq(fmax(pivot, 1e-300));
                    // lane j: Lr[j] == pivot; rows r < j are the upper triangle of the stored input columns (LM)
                    const double lj = (r >= j) ? Lr[j] * rd : 0.0;
                    Lr[j] = lj;
                    chol_update<NX, NU, j>(Lr, lj, pivot);
                });
                STAMPF(5);
                float Lm[NU];
#pragma unroll
                for (int q = 0; q < NU; q++) {
                    Lm[q] = (float)Lr[q];
                    rc[R::LM + q] = Lm[q];
                }
                // rhs: w = g^ + G' p_{k+1}; forward substitution over the input block (fp32)
                float y = dot_x<NX, NU>(ghat, pv, Gc);
                float my_lr = 0.0f;
                sfor<0, NU>([&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    const float lrj = bc<j>(y * frcp(Lm[j]));  // (y_j / L_jj) from lane j
                    if (r == j) my_lr = lrj;
                    y -= Lm[j] * lrj;
                });
                rc[R::LR] = my_lr;
                pv = is_x ? y : 0.0f;
#pragma unroll
                for (int j = 0; j < NV; j++) Lrow[j] = Lr[j];
            }
            piv = pi_new;
            STAMPF(6);
#ifndef P1_MASKED_STORE
            // Unconditional stores: lanes without work (idle slots, finished teams) write a record nobody reads.
            // Under a lane mask the stores sit in a branch the wave may skip, and the compiler then placed an
            // s_waitcnt vmcnt(0) at the loop header of the ping-pong sweep (it waited for the stores just issued
            // and for the prefetch); unconditional, every wait in the loop is counted (tools/isa_waits.py)
            float* const pk = act ? tbase + (size_t)k * KS : tdummy;
            if constexpr (SPL) {
                // core quad (LR LM Z) of the sweeping lanes; the bound quad only where a bound lives
                split_store<R, 0, R::TL, RS>(act ? pc0 + (size_t)k * R::CS : tdummy, tdummy + R::CW, rc);
                split_store<R, R::TL, R::TL + 4, RS>(tdummy, (act && bnd) ? pb0 + (size_t)k * kb : tdummy + R::CW, rc);
            } else if constexpr (MS) {
                // slack / multiplier quad only where a bound lives (elsewhere it holds the constant sentinel)
                rec_store_range<R::TL, R::TL + 4, RS, QM>(bnd ? pk : tdummy, rc);
                if constexpr (R::TL > 0) rec_store_range<0, R::TL, RS, QM>(pk, rc);
                if constexpr (R::TL + 4 < R::P1S1) rec_store_range<R::TL + 4, R::P1S1, RS, QM>(pk, rc);
            } else {
                rec_store_range<0, R::P1S1, RS, QM>(pk, rc);
            }
#else
            if constexpr (MS) {
                if (act && bnd) rec_store_range<R::TL, R::TL + 4, RS, QM>(tbase + (size_t)k * KS, rc);
                if (act) {
                    if constexpr (R::TL > 0) rec_store_range<0, R::TL, RS, QM>(tbase + (size_t)k * KS, rc);
                    if constexpr (R::TL + 4 < R::P1S1) rec_store_range<R::TL + 4, R::P1S1, RS, QM>(tbase + (size_t)k * KS, rc);
                }
            } else {
                if (act) rec_store_range<0, R::P1S1, RS, QM>(tbase + (size_t)k * KS, rc);
            }
#endif
            STAMPF(7);
        });
        if (it < kStampItsC) STAMP(2 + 4 * it);
        // team reductions
        sum_c = row_sum16(lv ? sum_c : 0.0f);
        max_c = row_max16(lv ? max_c : 0.0f);
        lam_max = row_max16(lv ? lam_max : 0.0f);
        res_ineq = row_max16(lv ? res_ineq : 0.0f);
        res_stat = row_max16(lv ? res_stat : 0.0f);
        stat_scale = row_max16(stat_scale);
        nanf_ = row_max16(nanf_);
        const float failf = row_max16(fail ? 1.0f : 0.0f);
        const float mu = sum_c * inv_m2;
        if (!done) {
            exit_res[0] = res_stat;
            exit_res[1] = res_ineq;
            exit_res[2] = mu;
            bool stop = false;
            if (nanf_ > 0.0f || mu != mu) {
                status = 1;
                stop = true;
            } else if (failf > 0.0f) {
                status = (mu <= kBreakdownMuT && res_ineq <= P.tol_ineq * 10.0f) ? 0 : 4;
                stop = true;
            } else if (lam_max > lam_thr && res_ineq > kInfeasRes) {
                status = 4;  // primal infeasible: stop now instead of holding the wave for qp_iter_max iterations
                stop = true;
            } else {
                const bool stat_ok = res_stat <= P.tol_stat || res_stat <= kStatRelT * stat_scale;
                // fp32 floor: below ~1e-12 the complementarity no longer decreases and the fp32 multiplier
                // updates (Sigma ~ 1e10 times the rounding of dz) degrade stationarity, so a stalled mu that is
                // already under tol_comp ends the iteration as well
                const bool cmax_ok = max_c <= kCompMaxRatio * P.tol_comp;
                const bool stalled = mu <= P.tol_comp && mu > 0.5f * mu_prev;
                if (res_ineq <= P.tol_ineq &&
                    ((stat_ok && mu <= P.tol_comp && cmax_ok) || mu <= 1e-2f * P.tol_comp || (stalled && cmax_ok)))
                    stop = true;
                if (it >= P.iter_max) stop = true;
            }
            if (stop) {
                done = true;
                it_done = it;
            }
        }
        mu_prev = mu;
        if (__all(done)) break;

        // pass 0: affine direction (forward; stores DZA, sums s1/s2 of the mu_aff polynomial);
        // pass 1: Mehrotra corrector (backward rhs through the stored factor, then forward; stores DZ);
        // pass 2: pure-centring safeguard for teams whose pass-1 step stayed below 0.1.
        // SD: pass 1 only, without the backward sweep: P1 already built the rhs with the target tg_rhs
        float sigma = 0.0f, alpha_aff = 0.0f;
        for (int pass = SD ? 1 : 0; pass < (SD ? 2 : 3); pass++) {
            bool run = !done;
            if (SD) {
                sigma_mu = tg_rhs;
                eta = 0.0f;
            } else if (pass == 1) {
                sigma_mu = sigma * mu;
                eta = alpha_aff;
            } else if (pass == 2) {
                if (__all(done || alpha >= 0.1f)) break;
                run = run && alpha < 0.1f;
                // only the teams that take the safeguard step change their targets: the next P1 rebuilds the
                // slack / multiplier step of every team from (DZ, DZA, sigma_mu, eta)
                sigma_mu = run ? fmaxf(sigma, 0.3f) * mu : sigma_mu;
                eta = run ? 0.0f : eta;
            }
            const bool ld = lv && run;
            if (!SD && pass > 0) {
                // corrector rhs through the stored factorisation (backward)
                float pvc = 0.0f;
                sweepd(std::integral_constant<int, LIGHT_DC>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, R::NB>{}, N, 0, -1, ld, [&](int k, float (&rc)[RS]) {
                    const bool vu = is_u && k < N;
                    float ghat;
                    {  // branch-free: 0 on the kFar-sentinel slots (see P0)
                        const float z = rc[R::Z];
                        const float tl = rc[R::TL], tu = rc[R::TU], ll = rc[R::LL], lu = rc[R::LU];
                        const float rl = z - rc[R::LB] - tl, rr = rc[R::UB] - z - tu;
                        const float itl = frcp(tl), itu = frcp(tu);
                        const BoundDir da = bound_dir(rc[R::DZA], rl, rr, tl, tu, ll, lu, itl, itu, 0.0f, 0.0f);
                        const float tgl = sigma_mu - eta * da.dll * da.dtl, tgu = sigma_mu - eta * da.dlu * da.dtu;
                        ghat = -(tgl - ll * rl) * itl + ll + (tgu - lu * rr) * itu - lu;
                    }
                    ghat += vu ? rc[R::RU] : 0.0f;
                    if (k == N) {
                        pvc = is_x ? ghat : 0.0f;
                    } else {
                        float Gc[NX];
                        column(rc, Gc);
                        float y = dot_x<NX, NU>(ghat, pvc, Gc);
                        float my_lr = 0.0f;
                        sfor<0, NU>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            const float Lmj = rc[R::LM + j];
                            const float lrj = bc<j>(y * frcp(Lmj));
                            if (r == j) my_lr = lrj;
                            y -= Lmj * lrj;
                        });
                        if (ld && is_u) (SPL ? pc0[(size_t)k * R::CS] : tbase[(size_t)k * KS + rec_off<RS, QM>(R::LR)]) = my_lr;
                        rc[R::LR] = my_lr;
                        pvc = is_x ? y : 0.0f;
                    }
                });
            }
            if (pass == 1) STAMPC1();
            // forward: du from the stored factor, dz, bounded-variable directions, next-stage dx
            float amax = 1e30f, s1 = 0.0f, s2 = 0.0f;
            // body kind 0: affine pass, 1: corrector / safeguard pass, 2: SD direction (target sigma_mu without the
            // affine correction; sums the complementarity polynomial of the step) -- compile-time bodies
            auto fwd = [&](auto cc) {
            constexpr int kind = decltype(cc)::value;
            constexpr bool corr = kind != 0;
            float dxs = 0.0f;
            sweepd(std::integral_constant<int, LIGHT_D>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, R::NF>{}, 0, N, 1, ld, [&](int k, float (&rc)[RS]) {
                const bool vu = is_u && k < N;
                const bool vx = is_x && k >= 1;
                const bool valid = vu || vx;
                // NU = 2: computed at every stage and zeroed at k = N (a select): under `if (k < N)` the compiler
                // sank the first stage's LR / LM load into the branch and waited for it (and every prefetch) at once
                // (same-box: metric +0.4 %, tric +1.1 %; omni4's longer substitution lost 0.6 %, so NU = 4 keeps
                // the branch; profiles/r03/ab/f1_uncond.txt)
                float du_all[NU];
#pragma unroll
                for (int q = 0; q < NU; q++) du_all[q] = 0.0f;
                if (NU == 2 || k < N) {
                    float w[NU];
                    sfor<0, NU>([&](auto qc) {
                        constexpr int q = decltype(qc)::value;
                        w[q] = bc<q>(rc[R::LR]) + ((k > 0) ? row_sum16(is_x ? rc[R::LM + q] * dxs : 0.0f) : 0.0f);
                    });
                    sfor<0, NU>([&](auto qqc) {
                        constexpr int q = NU - 1 - decltype(qqc)::value;
                        float sq = w[q];
                        sfor<q + 1, NU>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            sq -= bc<j>(rc[R::LM + q]) * du_all[j];
                        });
                        du_all[q] = sq * frcp(bc<q>(rc[R::LM + q]));
                    });
#pragma unroll
                    for (int q = 0; q < NU; q++) du_all[q] = (k < N) ? -du_all[q] : 0.0f;
                }
                float dz = 0.0f;
#pragma unroll
                for (int q = 0; q < NU; q++)
                    if (r == q) dz = du_all[q];
                dz = is_x ? ((k >= 1) ? dxs : 0.0f) : dz;
                {  // branch-free: the kFar-sentinel slots bound no step and add nothing to s1, s2
                    const float z = rc[R::Z];
                    const float tl = rc[R::TL], tu = rc[R::TU], ll = rc[R::LL], lu = rc[R::LU];
                    const float rl = z - rc[R::LB] - tl, rr = rc[R::UB] - z - tu;
                    const float itl = frcp(tl), itu = frcp(tu);
                    float tgl = 0.0f, tgu = 0.0f;
                    if (kind == 1) {
                        const BoundDir da = bound_dir(rc[R::DZA], rl, rr, tl, tu, ll, lu, itl, itu, 0.0f, 0.0f);
                        tgl = sigma_mu - eta * da.dll * da.dtl;
                        tgu = sigma_mu - eta * da.dlu * da.dtu;
                    } else if (kind == 2) {
                        tgl = sigma_mu;
                        tgu = sigma_mu;
                    }
                    const BoundDir d = bound_dir(dz, rl, rr, tl, tu, ll, lu, itl, itu, tgl, tgu);
                    amax = step_bound_r(amax, tl, d.dtl);
                    amax = step_bound_r(amax, tu, d.dtu);
                    amax = step_bound_r(amax, ll, d.dll);
                    amax = step_bound_r(amax, lu, d.dlu);
                    if (kind == 0) {  // dll = dlu = 0 on sentinel slots at zero targets
                        s1 += ll * d.dtl + tl * d.dll + lu * d.dtu + tu * d.dlu;
                        s2 += d.dll * d.dtl + d.dlu * d.dtu;
                    } else if (kind == 2) {  // a nonzero target moves the sentinels' multipliers: bounded slots only
                        const bool bnd = valid && has_b;
                        s1 += bnd ? ll * d.dtl + tl * d.dll + lu * d.dtu + tu * d.dlu : 0.0f;
                        s2 += bnd ? d.dll * d.dtl + d.dlu * d.dtu : 0.0f;
                    }
                }
                {  // unconditional (lanes without a direction write the dummy record): a masked store here left
                   // the compiler's wait after the sweep a full drain
                    const bool st = ld && valid;
                    if (corr && kDzPlane) *(st ? dzbase + (size_t)k * 16 : tdummy) = dz;
                    else *((st && !SPL) ? tbase + (size_t)k * KS + (!corr ? rec_off<RS, QM>(R::DZA) : rec_off<RS, QM>(R::DZ))
                              : tdummy) = dz;  // (split records: single-direction only, DZ in the plane)
                }
                if (k < N) dxs = dyn(rc, valid ? dz : 0.0f);
            });
            };
            // one compiled body per pass kind: same-box A/B diff metric 1.553 -> 1.526 ms, tric 4.382 -> 4.363 ms
            if constexpr (SD) fwd(std::integral_constant<int, 2>{});
            else if (pass == 0) fwd(std::integral_constant<int, 0>{});
            else fwd(std::integral_constant<int, 1>{});
            amax = row_min16(lv ? amax : 1e30f);
            if (SD) {
                // the step, then the next direction's target: mu after the step is exactly the complementarity
                // polynomial (sum_c + a s1 + a^2 s2) / 2m; sigma = clamp((1 - a)^2, sd_lo, sd_hi)
                s1 = row_sum16(lv ? s1 : 0.0f);
                s2 = row_sum16(lv ? s2 : 0.0f);
                if (run) alpha = fminf(1.0f, P.tau * amax);
                const float mu_next = fmaxf((sum_c + alpha * s1 + alpha * alpha * s2) * inv_m2, 0.0f);
                const float om = 1.0f - alpha;
                tg_rhs = fminf(fmaxf(om * om, P.sd_lo), P.sd_hi) * mu_next;
                if (it < kStampItsC) STAMP(4 + 4 * it);
            } else if (pass == 0) {
                s1 = row_sum16(lv ? s1 : 0.0f);
                s2 = row_sum16(lv ? s2 : 0.0f);
                alpha_aff = fminf(1.0f, amax);
                const float mu_aff = (sum_c + alpha_aff * s1 + alpha_aff * alpha_aff * s2) * inv_m2;
                float sg = (mu > 0.0f) ? mu_aff / mu : 0.0f;
                sg = fmaxf(sg, 0.0f);
                sigma = fminf(sg * sg * sg, 1.0f);
                if (it < kStampItsC) STAMP(3 + 4 * it);
            } else {
                if (run) alpha = fminf(1.0f, P.tau * amax);
                if (pass == 1 && it < kStampItsC) STAMP(4 + 4 * it);
            }
        }
        if (it < kStampItsC) STAMP(5 + 4 * it);
    }

    // ---- full SQP step + outputs ----------------------------------------------------------------------
    if (status == 0) {
        // one unconditional load of z and of the iterate entry, one store per lane and stage (lanes without an
        // entry -- idle slots, u at stage N -- read and write the dummy record): under lane masks every wait in
        // this loop was a vmcnt(0), one memory round trip per stage
        // this lane's entry of stage k (clamped: stages past N repeat stage N's, read-only below)
        // (both candidate addresses computed for every lane, then selected: as a pointer choice per lane class the
        // compiler branched around each address computation, two lane-mask regions per stage)
        auto entry = [&](int k) -> float* {
            const int kk = k <= N ? k : N;
            float* const px = &XB(kk, xi);
            float* const pu = &UBAR(kk < N ? kk : N - 1, is_u ? r : 0);
            return is_x ? px : ((is_u && kk < N) ? pu : tdummy);
        };
        constexpr int EC = 8;  // stages per batch: EC loads of each kind in flight, then EC stores
        for (int k0 = 0; k0 <= N; k0 += EC) {
            float zs[EC], vs[EC];
#pragma unroll
            for (int j = 0; j < EC; j++) {
                const int kk = (k0 + j) <= N ? k0 + j : N;
                zs[j] = SPL ? pc0[(size_t)kk * R::CS + R::Z] : tbase[(size_t)kk * KS + rec_off<RS, QM>(R::Z)];
                vs[j] = *entry(k0 + j);
            }
#pragma unroll
            for (int j = 0; j < EC; j++) {
                const int k = k0 + j;
                const float nv = (is_x && k == 0) ? x0_lane : vs[j] + zs[j];
                if (k <= N) *entry(k) = nv;
            }
        }
        if (a.xtraj || a.utraj) {
            __threadfence_block();
            for (int k = 0; k <= N; k++) {
                if (is_x && a.xtraj) a.xtraj[((size_t)k * NX + xi) * Bn + inst] = XB(k, xi);
                if (is_u && k < N && a.utraj) a.utraj[((size_t)k * NU + r) * Bn + inst] = UBAR(k, r);
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
        if (a.iter_key) a.iter_key[inst] = it_done;
        // warm-start the next solve only from a solve that converged (not from one that ran to qp_iter_max)
        // and only from an easy one (P.warm_iter_max, 12 by default: warm multipliers lengthen the hard QPs)
        if (a.warm)
            a.warm[inst] = (P.warm && status == 0 && it_done < P.iter_max && it_done <= P.warm_iter_max) ? a.warm_tag : 0;
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
        } else if (mode == kModeRun && a.cmd) {
            // failed solve: the reference throws (processAcadosStatus, NMPCNavControl.cpp:14-23) and the node
            // publishes a stop command (executeNMPC catch -> Status::Error, NMPCNavControlROS.cpp:716-719); the
            // carried refs and the iterate stay as they were
#pragma unroll
            for (int j = 0; j < 3; j++) a.cmd[(size_t)j * Bn + inst] = 0.0f;
        }
    }
#undef XB
#undef UBAR
}

}  // namespace

template <class M>
hipError_t launch_sqp_rti_team(const KParams& P, const KArgs& a, int mode, hipStream_t stream)
{
    if (a.B <= 0) return hipSuccess;
    // split launches: one robot per 256-lane block, P0's stage inputs in LDS (41 KB for diff at N = 80); a
    // horizon whose inputs do not fit runs unsplit
    const size_t stg = (size_t)(P.N + 1) * 16 * (5 + M::NGV) * sizeof(float);
    const size_t split_lds = stg + (mode == kModeRun ? (sizeof(double) + 3 * sizeof(float)) * (size_t)(P.N + 1) : 0);
    KArgs as = a;
    if (as.split && split_lds > 65536) as.split = 0;
    const int block = 256;  // 16 teams, or 1 robot (split)
    const long long threads = (long long)a.B * (as.split ? 256 : 16);
    const int grid = (int)((threads + block - 1) / block);
    // path mode: each team's N+1 path parameters and reference poses in LDS (16 teams x (N+1) x (8 + 12) B,
    // 26 KB at N = 80)
    const size_t lds = as.split ? split_lds
                                : ((mode == kModeRun && a.segs) ? (sizeof(double) + 3 * sizeof(float)) * 16 * (size_t)(P.N + 1) : 0);
    if (lds > 65536) return hipErrorInvalidValue;
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(block), lds, stream, P, as); };
    // compile-time mode (the kernel's MODE parameter)
    const int km = mode != kModeRun ? kModeSolve : (a.segs ? kModeRunPath : kModeRun);
    auto pick2 = [&](auto msc, auto sdc, auto spc) {
        constexpr bool ms = decltype(msc)::value, sd = decltype(sdc)::value, sp = decltype(spc)::value;
        if (km == kModeRunPath) go(k_sqp_rti_team<M, ms, sd, kModeRunPath, sp>);
        else if (km == kModeRun) go(k_sqp_rti_team<M, ms, sd, kModeRun, sp>);
        else go(k_sqp_rti_team<M, ms, sd, kModeSolve, sp>);
    };
    // record layout: tric always split, diff per launch (a.rec_split), omni4 and Mehrotra never
    auto pick = [&](auto msc, auto sdc) {
        using R = TeamRec<M, decltype(sdc)::value>;
        if constexpr (R::SPLIT) pick2(msc, sdc, std::true_type{});
        else if constexpr (R::SPLIT_OK) {
            if (a.rec_split) pick2(msc, sdc, std::true_type{});
            else pick2(msc, sdc, std::false_type{});
        } else pick2(msc, sdc, std::false_type{});
    };
    using T = std::true_type;
    using F = std::false_type;
    if (P.ipm == 1) {
        if (a.dense) pick(T{}, T{});
        else pick(F{}, T{});
    } else if (a.dense) {
        pick(T{}, F{});
    } else {
        pick(F{}, F{});
    }
    return hipGetLastError();
}

template hipError_t launch_sqp_rti_team<Diff2>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_team<Omni4>(const KParams&, const KArgs&, int, hipStream_t);
template hipError_t launch_sqp_rti_team<Tric3>(const KParams&, const KArgs&, int, hipStream_t);
template size_t team_scratch_floats<Diff2>(int, int);
template size_t team_scratch_floats<Omni4>(int, int);
template size_t team_scratch_floats<Tric3>(int, int);

#ifdef NMPC_STAMPS
extern "C" int nmpc_debug_stamps_c1(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps_c1), sizeof(g_stamps_c1), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
extern "C" int nmpc_debug_stamps_pa(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps_pa), sizeof(g_stamps_pa), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
extern "C" int nmpc_debug_stamps_p1(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps_p1), sizeof(g_stamps_p1), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
extern "C" int nmpc_debug_stamps(unsigned long long* host, int n)
{
    const size_t bytes = sizeof(unsigned long long) * (size_t)n;
    if (bytes > sizeof(g_stamps)) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif

}  // namespace nmpc
