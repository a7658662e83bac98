// sqp_rti_rowpar.hip -- batched SQP-RTI step for small batches: one block of W wavefronts per robot (W = 4 up to
// 256 robots: one wave per SIMD of the robot's CU), the stage-independent work spread over the block's 4 W DPP rows,
// only the recursions over the horizon serial.
//
// The same single-direction IPM as k_sqp_rti_team (sqp_rti_team.hip, SD rule; DESIGN.md "Algorithm and
// precision"), the same records, warm start and stopping rule, reorganised for latency. In the team kernel one
// 16-lane team runs every stage of every sweep in turn: per IPM iteration 81 x ~350 instructions of P1 and
// 81 x ~130 of the forward sweep at N = 80, one robot's solve being the reference's whole deployment
// (NMPCNavControlROS.cpp:713 -> NMPCNavControlDiff.cpp:142). Most of that work does not depend on the
// neighbouring stage: applying the step, the slacks / multipliers, the residuals, the barrier weights and the
// rhs terms before the Riccati step (phase A), and the bound directions, the step bound and the complementarity
// polynomial after the forward recursion (phase D). Here row q of the block (lanes 16q .. 16q+15 of its wave
// q / 4; lane 16q + v owns variable v as in a team) runs those phases for stages q, q + 4 W, ..., and block
// reductions (LDS) combine the rows; the Riccati factorisation (phase B: fp64 P G, G'P G, input-block Cholesky,
// rhs) and the forward recursion of the directions (phase C) are the only stage-serial passes, and every wave
// computes them identically on its row 0 (same records, same DPP broadcasts inside the row), so no wave waits on
// another; wave 0 stores them, the other waves store to pads. The fields an IPM iteration makes and uses up stay in
// LDS (ItLds: barrier weights, rhs terms, factor columns, the direction), so only the iterate, slacks and
// multipliers are written back to the global records per iteration. P0 likewise: the RK4
// linearisation of stage k on row k mod 4 W, then the serial initial-iterate pass from LDS.
// One robot per block also makes every loop exit block-uniform (no lockstep teams).
#include "nmpc_kernels.hpp"
#include "team_common.hpp"

namespace nmpc {

// Record layout: TeamRec<M, true> (the team kernel's single-direction layout: the warm-start multipliers LL / LU
// and the record stride are shared, so a handle may alternate kernels between solves). Global memory keeps what
// outlives an IPM iteration -- the iterate Z, slacks / multipliers TL TU LL LU (phase A), bounds LB UB, Jacobian rows
// GV and gradient GR (P0) -- and the fields an iteration makes and uses up live in LDS (ItLds): SIG (barrier
// weight), C0 (h z + g - (l_lo - l_up), the stationarity term without the adjoint) and GH (the bound part of the
// rhs) from phase A for phase B, LR / LM (the factor's input columns and rhs) from phase B for phase C, DZ (the
// direction) from phase C for phases D and A. SIG / C0 / GH are register-image slots past GR only.
template <class M>
struct RowRec {
    using T = TeamRec<M, true>;
    static constexpr int NX = M::NX, NU = M::NU, NV = NX + NU, NGV = M::NGV;
    static constexpr int LR = T::LR, LM = T::LM, Z = T::Z, TL = T::TL, TU = T::TU, LL = T::LL, LU = T::LU;
    static constexpr int LB = T::LB, UB = T::UB, GV = T::GV, GR = T::GR, RS = T::RS, RSS = T::RSS;
    static constexpr int SIG = GR + 1, C0 = GR + 2, GH = GR + 3;
    static_assert(GH < RS, "phase-A fields fit the register image");
    static_assert(LM + NU <= Z && Z < TL, "LR / LM below Z");
};

// The per-iteration stage fields in LDS (RowRec): [N+1][NF][NV] floats, live slots only (lane r < NV reads / writes
// slot r; idle lanes read slot 0 and write a pad). Round 4 kept them in the global records, which cost about 1.06 KB
// of writes per robot, stage and IPM iteration at diff1024 (phase A's SIG / C0 / GH sector, phase B's LR / LM into
// the sector phase A had just written, the DZ plane): 6.3x the fetched bytes
template <class M>
struct ItLds {
    static constexpr int NU = M::NU, NV = M::NX + M::NU;
    static constexpr int SIG = 0, C0 = 1, GH = 2, LR = 3, LM = 4, DZ = 4 + NU, NF = 5 + NU;
    __host__ __device__ static constexpr size_t floats(int N) { return (size_t)(N + 1) * NF * NV; }
};

// LDS of the segmented phases (SEG, a.seg = S > 0), in floats from its base (8-byte aligned; fp64 parts at even
// offsets). Per segment q: the entry quantities of its backward sweep -- P (fp64 rows), pbar, Phi, Gam, t; per master step i: Q_i (fp64), c_i, phat_{i+1}; a transpose scratch; the
// boundary states s_q and
// costates lam_q; the lam-sensitivity Z of every stage's LR (rows of the NU input lanes).
template <class M>
struct SegLayout {
    static constexpr int NX = M::NX, NU = M::NU, NXP = (M::NX + 3) / 4 * 4;
    int SUM_P, SUM_PB, SUM_PHI, SUM_GAM, SUM_T, QS, CS, PHS, LT, XA, SL, ZL;
    __host__ __device__ explicit SegLayout(int S)
    {
        SUM_P = 0;                          // [S][NX][NX] double
        SUM_GAM = SUM_P + 2 * S * NX * NX;  // [S][NX][NX] double (fp64 sum: the dual sweep factors -Gam_0)
        SUM_PB = SUM_GAM + 2 * S * NX * NX; // [S][NX]
        SUM_PHI = SUM_PB + S * NX;          // [S][NX][NX]
        SUM_T = SUM_PHI + S * NX * NX;      // [S][NX]
        QS = (SUM_T + S * NX + 1) / 2 * 2;  // [S][NX][NX] double
        CS = QS + 2 * S * NX * NX;          // [S][NX] double
        PHS = CS + 2 * S * NX;              // [S][NX] double
        LT = PHS + 2 * S * NX;              // [2][NX][NX] double: the master rows' transpose scratch
        XA = LT + 4 * NX * NX;              // [2][NX + 1][NX] + [NX] double: Phat_m, phat_m / Shat_m, shat_m; lam_m
        SL = XA + 4 * (NX + 1) * NX + 2 * NX;  // [S + 1][2][NX]: s_q, lam_q
        ZL = SL + (S + 1) * 2 * NX;         // [N + 1][NU][NXP]
    }
    __host__ __device__ size_t floats(int N) const { return (size_t)ZL + (size_t)(N + 1) * NU * NXP; }
};

// layout of the kernel's dynamic LDS (floats): P0's stage inputs [N+1][SF][16], reference poses [N+1][3], block
// reductions [W][8], dx [N+1][16], unwrapped references [N+1][3], 64 pad floats (per-lane store targets nobody
// reads); then the IPM's per-iteration stage fields (ItLds) and (SEG) the segment area, each reusing the stage-input
// region where it fits there (P0 is done with it before the first IPM iteration, behind a block barrier)
template <class M>
struct RowLds {
    static constexpr int SF = 5 + M::NGV;
    __host__ __device__ static constexpr size_t r4(size_t f) { return (f + 3) / 4 * 4; }
    __host__ __device__ static constexpr size_t stage_floats(int N) { return (size_t)(N + 1) * SF * 16; }
    __host__ __device__ static constexpr size_t pad_off(int N) { return (size_t)(N + 1) * (16 * SF + 3 + 16 + 3) + 32; }
    __host__ __device__ static constexpr size_t base_floats(int N) { return pad_off(N) + 64; }
    __host__ __device__ static constexpr size_t it_off(int N)
    {
        return ItLds<M>::floats(N) <= stage_floats(N) ? 0 : r4(base_floats(N));
    }
    __host__ __device__ static constexpr size_t it_end(int N) { return r4(it_off(N) + ItLds<M>::floats(N)); }
    __host__ __device__ static size_t seg_off(int N, int S)
    {
        const size_t sf = SegLayout<M>(S).floats(N);
        if (it_off(N) == 0) return it_end(N) + sf <= stage_floats(N) ? it_end(N) : r4(base_floats(N));
        return it_end(N);
    }
    __host__ __device__ static size_t floats(int N, int S)
    {
        size_t end = base_floats(N) > it_end(N) ? base_floats(N) : it_end(N);
        if (S > 0) {
            const size_t se = seg_off(N, S) + SegLayout<M>(S).floats(N);
            end = se > end ? se : end;
        }
        return end;
    }
};

#ifdef NMPC_STAMPS
// diagnostic build only: s_memtime after each phase, robots 0..255, lane 0: [0] start, [1] P0a, [2] P0b, then per
// IPM iteration it: [3 + 4 it + 0..3] after phases A, B, C, D
constexpr int kRpIts = 64;
__device__ unsigned long long g_rp_stamps[256][3 + 4 * kRpIts];
#define RP_STAMP(slot)                                                                                           \
    do {                                                                                                         \
        if (tid == 0 && inst < 256 && (slot) < 3 + 4 * kRpIts) g_rp_stamps[inst][(slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
extern "C" int nmpc_debug_stamps_rowpar(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rp_stamps), sizeof(g_rp_stamps), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
// the segment master's parts, per IPM iteration (lane 0): [0] start, [1] both sweeps done, [4] join done,
// [5] both propagations done, [7] after the block barrier (slots 2, 3, 6: unused since the one-stream master)
__device__ unsigned long long g_rp_mstamps[256][kRpIts][8];
#define RP_MSTAMP(slot, lane)                                                                                    \
    do {                                                                                                         \
        if (tid == (lane) && inst < 256 && it < kRpIts) g_rp_mstamps[inst][it][(slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
extern "C" int nmpc_debug_mstamps_rowpar(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rp_mstamps), sizeof(g_rp_mstamps), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
// per master step of the backward sweep (lane 0): [it][i] after boundary step i
__device__ unsigned long long g_rp_sstamps[256][kRpIts][16];
#define RP_SSTAMP(i)                                                                                            \
    do {                                                                                                         \
        if (tid == 0 && inst < 256 && it < kRpIts && (i) < 16) g_rp_sstamps[inst][it][(i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
extern "C" int nmpc_debug_sstamps_rowpar(unsigned long long* host)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rp_sstamps), sizeof(g_rp_sstamps), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#else
#define RP_STAMP(slot) ((void)0)
#define RP_MSTAMP(slot, lane) ((void)0)
#define RP_SSTAMP(i) ((void)0)
#endif

namespace {

template <int F0, int F1, int RS, bool QM>
__device__ __forceinline__ void ld_range(const float* p, float (&v)[RS])
{
    rec_load_range<F0, F1, RS, QM>(p, v);
}

// zeros: the warm-start multiplier source of a cold robot (the flag selects the address, not the value)
__device__ __attribute__((aligned(16))) float g_rp_zero4[4];

// cross-row reductions of the wave (the four rows hold disjoint stages in the stage-parallel phases)
__device__ __forceinline__ float wave_sum_rows(float v)
{
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}
__device__ __forceinline__ float wave_max_rows(float v)
{
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float wave_min_rows(float v)
{
    v = fminf(v, __shfl_xor(v, 16));
    return fminf(v, __shfl_xor(v, 32));
}

// W waves per robot (one per SIMD): the stage-parallel phases run on all 4 W rows; every wave runs the serial
// phases (identically) and wave 0 stores their results (into LDS; the other waves store into pads).
// SEG: the horizon is cut into a.seg segments of L = N / S stages whose Riccati sweeps (phase B) and forward
// recursions (phase C) run at the same time, one segment per row, joined by a master recursion over the segment
// boundaries (DESIGN.md "Segmented Riccati"); a robot's serial chain shrinks from N + 1 stage steps to L + 1 plus S - 1
// master steps. The rhs is built in absolute form (no adjoint), so the stationarity residual of the stopping rule is
// evaluated by its own serial adjoint pass, only when the rest of the exit test already holds.
// Register bound of the segmented diff / tric instantiations: two waves per SIMD for W <= 2 (launches above 256
// robots put two robots' waves on each SIMD, tests/test_reg_usage.py), one for W = 4 (launches of at most 256 robots,
// one block per CU). Bounding the four-wave kernel to 256 registers as well (round 5) made the compiler serialise the
// master step's LDS operand loads through one register; without it the one-robot capsule takes 0.260 instead of
// 0.279 ms cold (same box, profiles/r06/ab/p0b_w4.txt). -DNMPC_W4_BOUND2 keeps round 5's bound for A/B runs.
#ifdef NMPC_W4_BOUND2
constexpr int kRowparW2Max = 4;
#else
constexpr int kRowparW2Max = 2;
#endif
template <class M, int W, bool SEG>
__global__ __launch_bounds__(64 * W, (SEG && M::NX < 10 && W <= kRowparW2Max) ? 2 : 1) void k_sqp_rti_rowpar(KParams P, KArgs a, int mode)
{
    using R = RowRec<M>;
    constexpr int NX = M::NX, NU = M::NU, NV = R::NV, NGV = R::NGV, RS = R::RS, RSS = R::RSS;
    constexpr bool QM = rec_quad_major<NV>();
    constexpr int ROWS = 4 * W;
#ifdef NMPC_HYBRID
    // hybrid launch (A/B build, role 2): block i takes the robot of rank i of the order, for the first hyb_n[0] ranks
    if (a.hyb_role == 2 && (int)blockIdx.x >= a.hyb_n[0]) return;
    const int inst = (a.hyb_role == 2) ? a.order[blockIdx.x] : (int)blockIdx.x;
#else
    const int inst = (int)blockIdx.x;
#endif
    if (inst >= a.B) return;
    const int tid = (int)threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (an SGPR: branches on it are wave-uniform)
    const int q = tid >> 4;  // row of the block: stage-parallel phases take stages q, q + ROWS, ...
    const int r = tid & 15;  // slot: variable r of the stage (as a team lane)
    const bool wr = tid < 16;  // the lanes that store the serial phases' results
    const int N = P.N;
    const size_t S = (size_t)a.stride;
    const size_t Bn = (size_t)a.B;
    const bool lv = r < NV;
    const bool is_u = r < NU;
    const bool is_x = lv && !is_u;
    const int xi = is_x ? r - NU : 0;
    const int cx = is_x ? xcomp<M>(xi) : -1;
    const bool has_b = is_u || cx >= 0;
    const float sc = P.dt;
    const float w_lane = is_u ? P.W[NX + r] : (is_x ? P.W[xi] : 0.0f);
    const float h_stage = sc * w_lane;
    float lo_b = 0.0f, hi_b = 0.0f;
#pragma unroll
    for (int j = 0; j < NU; j++)
        if (r == j) { lo_b = P.lbu[j]; hi_b = P.ubu[j]; }
#pragma unroll
    for (int c = 0; c < M::NBX; c++)
        if (cx == c) { lo_b = P.lbx[c]; hi_b = P.ubx[c]; }
    constexpr int KS = 16 * RSS;  // floats per stage block (the team kernel's layout)
    const int NR = (N + 1 + ROWS - 1) / ROWS;  // rounds of the stage-parallel phases
    float* const rbase = a.scratch + (size_t)inst * (N + 1) * KS;
    float* const tbase = rbase + (lv ? r : 0) * rec_lane<RSS, QM>();   // idle slots read slot 0
    float* const tbase_own = rbase + r * rec_lane<RSS, QM>();          // every lane's own slot
    // Stores of the serial phases: wave 0 stores (its four rows the same values to the same addresses, as one
    // row would); the other waves store into pads. Idle slots and rows past the last stage of a stage-parallel
    // phase store into tdummy (global records) or a pad (LDS).
    const bool w0 = wave == 0;
    float* const tdummy = rbase + (size_t)N * KS + 15 * rec_lane<RSS, QM>();  // nobody reads it
    const bool warm = P.warm && a.warm && a.warm[inst] == a.warm_tag && !(a.reset && a.reset[inst]);
    RP_STAMP(0);

#define XB(k, j) a.xbar[((size_t)(k) * NX + (j)) * S + inst]
#define UBAR(k, j) a.ubar[((size_t)(k) * NU + (j)) * S + inst]

    // ---- staged capsule input (one robot): host-mapped block -> device block, every thread's loads in flight
    // together (one round trip of host memory instead of a copy launch and its dispatch gap before this kernel)
    if (a.stage_in_n > 0) {
        constexpr int T = 64 * W, U = 8;
        for (int e0 = 0; e0 < a.stage_in_n; e0 += T * U) {
            float v[U];
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int e = e0 + j * T + tid;
                v[j] = a.stage_in_h[e < a.stage_in_n ? e : 0];
            }
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int e = e0 + j * T + tid;
                if (e < a.stage_in_n) a.stage_in_d[e] = v[j];
            }
        }
        __threadfence_block();
        __syncthreads();
    }

    // ---- reset ({name}_acados_reset: zero iterate) ----------------------------------------------------------
    if (a.reset && a.reset[inst]) {
        for (int e = tid; e < (N + 1) * NX; e += 64 * W) XB(e / NX, e % NX) = 0.0f;
        for (int e = tid; e < N * NU; e += 64 * W) UBAR(e / NU, e % NU) = 0.0f;
        __syncthreads();
    }

    // ---- x0 -----------------------------------------------------------------------------------------------
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
    float we_lane = 0.0f;
    if (is_x) we_lane = (mode != kModeRun && a.We) ? a.We[(size_t)xi * Bn + inst] : P.We[xi];

    // ---- P0a: RK4 linearisation of stage k on row k mod 4 -> LDS [k][field][lane] -----------------------------
    // fields: zbar, yref entry, warm multipliers (2), defect b_k, the NGV varying Jacobian rows; run mode also the
    // stage's reference pose in my_traj
    constexpr int SF = 5 + NGV;
    extern __shared__ float s_row[];
    float* const s_stg = s_row;
    float* const my_traj = s_row + (size_t)(N + 1) * SF * 16;
    float* const s_red = my_traj + (size_t)(N + 1) * 3;  // [W][8] per-wave partial reductions

    // block reductions of per-wave partials (W > 1): every wave combines the W partials in the same order, so every
    // wave holds identical values and takes identical decisions; the barrier is also the phase boundary
    auto block_combine = [&](float (&v)[6], const int (&op)[6], int n) {
        if constexpr (W == 1) {
            __syncthreads();
        } else {
            if ((tid & 63) == 0)
                for (int i = 0; i < n; i++) s_red[wave * 8 + i] = v[i];
            __syncthreads();
            for (int i = 0; i < n; i++) {
                float acc = s_red[i];
                for (int w = 1; w < W; w++) {
                    const float x = s_red[w * 8 + i];
                    acc = (op[i] == 0) ? acc + x : ((op[i] == 1) ? fmaxf(acc, x) : fminf(acc, x));
                }
                v[i] = acc;
            }
        }
    };

    const int len = (mode == kModeRun) ? (a.traj_len ? a.traj_len[inst] : N + 1) : 0;
    // a per-lane LDS slot nobody reads: the target of P0's stores for lanes / rounds without data (a store under a
    // lane mask leaves the compiler's later waits uncounted, i.e. full drains)
    float* const lpad = s_row + RowLds<M>::pad_off(N) + (tid & 63);
    // the IPM's per-iteration stage fields (ItLds): reads of idle lanes take slot 0, writes of lanes without an entry
    // go to their pad
    using IT = ItLds<M>;
    float* const it_lds = s_row + RowLds<M>::it_off(N);
    const int rv = lv ? r : 0;
    auto it_rd = [&](int k, int f) -> float { return it_lds[((size_t)k * IT::NF + f) * NV + rv]; };
    auto it_wr = [&](int k, int f, bool w) -> float* { return w ? it_lds + ((size_t)k * IT::NF + f) * NV + r : lpad; };
    // Four waves, segmented: wave 0 runs P0b's initial-iterate pass while waves 1-3 integrate the stages (P0a, rounds
    // of 12 stages), taking each round as soon as its three waves have stored it: s_cnt counts the finished
    // wave-rounds (an LDS word the block reductions leave unused). Otherwise every row integrates and P0b follows a
    // block barrier. -DNMPC_P0_NO_OVERLAP keeps the barrier for A/B runs.
#if defined(NMPC_P0_SERIAL) || defined(NMPC_P0_NO_OVERLAP)
    constexpr bool kP0Ov = false;
#else
    constexpr bool kP0Ov = W == 4 && SEG;
#endif
    constexpr int PW = kP0Ov ? 1 : 0;           // waves that skip P0a
    constexpr int PROWS = ROWS - 4 * PW;        // rows of P0a
    const int prow = q - 4 * PW;                // this row among them (wave 0: negative, unused)
    const int pnr = (N + 1 + PROWS - 1) / PROWS;  // rounds of P0a
    unsigned int* const s_cnt = reinterpret_cast<unsigned int*>(s_red + 7);
    if constexpr (W >= 2 && SEG) {  // (and phase B's counts of finished factorisation stages, s_red[15], s_red[23])
        if (tid == 0) {
            *s_cnt = 0u;
            reinterpret_cast<unsigned int*>(s_red)[15] = 0u;
            if constexpr (W == 4) reinterpret_cast<unsigned int*>(s_red)[23] = 0u;
        }
        __syncthreads();
    }
    // (wave 0, and the unwrap's wave) wait until the round holding stage k is in LDS; bounded, never a hang
    unsigned int seen = 0;
    auto wait_stage = [&](int k) {
        if constexpr (kP0Ov) {
            const int kk = k <= N ? k : N;
            const unsigned int need = (unsigned int)(W - 1) * (unsigned int)(kk / PROWS + 1);
            for (int g = 0; seen < need && g < (1 << 24); g++) {
                seen = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(s_cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (seen < need) __builtin_amdgcn_s_sleep(1);
            }
        }
    };
    if (!kP0Ov || !w0) {
        struct In {
            float x[NX], u[NU], y, xnext, tq;
            float2 l;
        };
        // every load unconditional at a valid address (values selected afterwards): a load under a lane mask or a
        // runtime condition made the compiler drain the memory counter before the round's stores
        const int jy = is_u ? NX + r : xi;
        const bool use_y = lv && jy < a.ny_in;
        auto ld = [&](int k, In& v) {
            const int kk = k <= N ? k : N;
#pragma unroll
            for (int j = 0; j < NX; j++) v.x[j] = XB(kk, j);
            const int ku = kk < N ? kk : N - 1;
#pragma unroll
            for (int j = 0; j < NU; j++) v.u[j] = UBAR(ku, j);
            v.xnext = XB(kk < N ? kk + 1 : N, xi);
            if (mode != kModeRun) {
                const float y = a.yref[((size_t)kk * a.ny_in + (use_y ? jy : 0)) * Bn + inst];
                v.y = use_y ? y : 0.0f;
                v.tq = 0.0f;
            } else {
                const int kt = kk < len ? kk : (len > 0 ? len - 1 : 0);
                v.tq = a.traj[((size_t)kt * 3 + (r < 3 ? r : 0)) * Bn + inst];
                v.y = 0.0f;
            }
            v.l = *reinterpret_cast<const float2*>(warm ? tbase + (size_t)kk * KS + rec_off<RS, QM>(R::LL) : g_rp_zero4);
        };
        // rounds j = 0 .. NR-1 (row q: stage j ROWS + q) with the next round's inputs in flight (two buffers used in
        // turn: a copy between them would wait for the load still in flight)
        auto round = [&](int j, const In& cur) {
            const int k = j * PROWS + prow;
            const bool kv = k <= N;
            if (mode == kModeRun) *((r < 3 && kv) ? my_traj + k * 3 + r : lpad) = cur.tq;
            float xn[NX], g[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) { xn[i] = 0.0f; g[i] = 0.0f; }
            float bk = 0.0f;
            if (k < N) {  // (rows past the end: k > N)
                rk4_column<M>(cur.x, cur.u, P, lv ? r : NU, xn, g);
#pragma unroll
                for (int i = 0; i < NX; i++)
                    if (is_x && xi == i) bk = xn[i] - cur.xnext;
            }
            float zb = 0.0f;
#pragma unroll
            for (int j2 = 0; j2 < NU; j2++)
                if (r == j2) zb = cur.u[j2];
#pragma unroll
            for (int j2 = 0; j2 < NX; j2++)
                if (is_x && xi == j2) zb = cur.x[j2];
            float* const st = kv ? s_stg + (size_t)k * SF * 16 + r : nullptr;
            *(kv ? st : lpad) = zb;
            *(kv ? st + 16 : lpad) = cur.y;
            *(kv ? st + 32 : lpad) = cur.l.x;
            *(kv ? st + 48 : lpad) = cur.l.y;
            *(kv ? st + 64 : lpad) = bk;
#pragma unroll
            for (int i = 0; i < NGV; i++) *(kv ? st + (5 + i) * 16 : lpad) = g[i];
        };
        // (overlap: this wave's stores of the round are in LDS, then its count)
        auto signal = [&]() {
            if constexpr (kP0Ov) {
                // LDS completes in order per wave: waiting for this wave's LDS operations is the release (a
                // workgroup-scope fence would also wait for the next round's global loads in flight)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if ((tid & 63) == 0) __hip_atomic_fetch_add(s_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        };
        In ca, cb;
        ld(prow, ca);
        for (int j = 0;; j += 2) {
            ld((j + 1) * PROWS + prow, cb);
            round(j, ca);
            signal();
            if (j + 1 >= pnr) break;
            ld((j + 2) * PROWS + prow, ca);
            round(j + 1, cb);
            signal();
            if (j + 2 >= pnr) break;
        }
    }
    // constant rows of [B A] (rows >= NGV) from stage 0 (every row, identically)
    float gcol[NX], grow[NV];
    {
        float xb0[NX], ub0[NU], xn0[NX], g0[NX];
#pragma unroll
        for (int j = 0; j < NX; j++) xb0[j] = XB(0, j);
#pragma unroll
        for (int j = 0; j < NU; j++) ub0[j] = UBAR(0, j);
        rk4_column<M>(xb0, ub0, P, lv ? r : NU, xn0, g0);
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
    if constexpr (!kP0Ov) __syncthreads();  // the stage inputs of every row are in LDS
    RP_STAMP(1);

    // ---- P0b (serial): the dynamics-feasible initial iterate dx_{k+1} = A_k dx_k + b_k on wave 0 and, in run mode,
    // the reference unwrap / padding (NMPCNavControlDiff.cpp:104-118) on the last wave, two recursions over the
    // stages; dx_k and the stage's reference pose go to LDS for P0c. Each loop body is branch-free: round 5's one
    // loop for both recursions tested the mode, the horizon end and the reference lanes in every stage (about 15
    // scalar branches per stage, 575 cycles per stage step at one robot; profiles/r06/ab/p0b_w4.txt)
    float* const s_dx = s_red + 32;                  // [N+1][16]
    float* const s_ref = s_dx + (size_t)(N + 1) * 16;  // [N+1][3]
#ifndef NMPC_P0_SERIAL
    if (w0) {
        struct Stg {
            float b, g[NGV];
        };
        auto lds_ld = [&](int k, Stg& o) {
            const int kk = k <= N ? k : N;
            const float* const st = s_stg + (size_t)kk * SF * 16 + r;
            o.b = st[64];
#pragma unroll
            for (int i = 0; i < NGV; i++) o.g[i] = st[(5 + i) * 16];
        };
        // store dx_k, then dx_{k+1} (every LDS store unconditional; rows 1-3 of wave 0 write row 0's identical values)
        float dx = is_x ? x0_lane - XB(0, xi) : 0.0f;
        auto step = [&](int k, const Stg& cur) {
            s_dx[k * 16 + r] = dx;
            const float dzd = is_x ? dx : 0.0f;
            float nx_ = dot_v<NX, NU>(0.0f, dzd, grow);
#pragma unroll
            for (int i = 0; i < NGV; i++) {
                const float sr = row_sum16(lv ? cur.g[i] * dzd : 0.0f);
                if (xi == i) nx_ = sr;
            }
            dx = is_x ? nx_ + cur.b : 0.0f;
        };
        // three buffers used in turn, loads two stages ahead (no copies: a copy waits for the LDS read in flight)
        Stg c0, c1, c2;
        wait_stage(1);
        lds_ld(0, c0);
        lds_ld(1, c1);
        for (int k = 0;; k += 3) {  // stages 0 .. N - 1
            wait_stage(k + 2);
            lds_ld(k + 2, c2);
            step(k, c0);
            if (k + 1 == N) break;
            wait_stage(k + 3);
            lds_ld(k + 3, c0);
            step(k + 1, c1);
            if (k + 2 == N) break;
            wait_stage(k + 4);
            lds_ld(k + 4, c1);
            step(k + 2, c2);
            if (k + 3 == N) break;
        }
        s_dx[N * 16 + r] = dx;
    }
    if (mode == kModeRun && wave == W - 1) {
        // (rows of the wave compute the same values; lanes 0-2 of each row store them, the rest store to a pad)
        wait_stage(N);  // (overlap: every round's reference poses)
        float ref_x = 0.0f, ref_y = 0.0f, ref_t = pose_th;
        auto ld_t = [&](int k, float (&t)[3]) {
            const int kk = k <= N ? k : N;
#pragma unroll
            for (int j = 0; j < 3; j++) t[j] = my_traj[kk * 3 + j];
        };
        auto uw = [&](int k, const float (&t)[3]) {
            const bool in = k < len;
            const float th = t[2], d = th - ref_t;
            const float thu = (d > kPi) ? th - 2.0f * kPi : ((d < -kPi) ? th + 2.0f * kPi : th);
            ref_x = in ? t[0] : ref_x;
            ref_y = in ? t[1] : ref_y;
            ref_t = in ? thu : ref_t;
            float v = ref_t;
            v = (r == 1) ? ref_y : v;
            v = (r == 0) ? ref_x : v;
            *(r < 3 ? s_ref + k * 3 + r : lpad) = v;
        };
        float t0[3], t1[3], t2[3];
        ld_t(0, t0);
        ld_t(1, t1);
        for (int k = 0;; k += 3) {  // stages 0 .. N
            ld_t(k + 2, t2);
            uw(k, t0);
            if (k == N) break;
            ld_t(k + 3, t0);
            uw(k + 1, t1);
            if (k + 1 == N) break;
            ld_t(k + 4, t1);
            uw(k + 2, t2);
            if (k + 2 == N) break;
        }
    }
#else
    // A/B only (-DNMPC_P0_SERIAL): round 5's single loop over both recursions on wave 0
    if (w0) {
        float dx = is_x ? x0_lane - XB(0, xi) : 0.0f;
        float ref_x = 0.0f, ref_y = 0.0f, ref_t = pose_th;
        struct Stg {
            float b, g[NGV], t[3];
        };
        auto lds_ld = [&](int k, Stg& o) {
            const int kk = k <= N ? k : N;
            const float* const st = s_stg + (size_t)kk * SF * 16 + r;
            o.b = st[64];
#pragma unroll
            for (int i = 0; i < NGV; i++) o.g[i] = st[(5 + i) * 16];
#pragma unroll
            for (int j = 0; j < 3; j++) o.t[j] = (mode == kModeRun) ? my_traj[kk * 3 + j] : 0.0f;
        };
        // one stage of the recursion (branch-free reference unwrap; every LDS store unconditional: lanes without
        // an entry write their pad slot, rows 1-3 of wave 0 write row 0's identical values)
        auto step = [&](int k, const Stg& cur) {
            if (mode == kModeRun) {
                const bool in = k < len;
                const float th = cur.t[2], d = th - ref_t;
                const float thu = (d > kPi) ? th - 2.0f * kPi : ((d < -kPi) ? th + 2.0f * kPi : th);
                ref_x = in ? cur.t[0] : ref_x;
                ref_y = in ? cur.t[1] : ref_y;
                ref_t = in ? thu : ref_t;
                *(r < 3 ? s_ref + k * 3 + r : lpad) = (r == 0) ? ref_x : ((r == 1) ? ref_y : ref_t);
            }
            s_dx[k * 16 + r] = dx;
            if (k < N) {
                const float dzd = is_x ? dx : 0.0f;
                float nx_ = dot_v<NX, NU>(0.0f, dzd, grow);
#pragma unroll
                for (int i = 0; i < NGV; i++) {
                    const float sr = row_sum16(lv ? cur.g[i] * dzd : 0.0f);
                    if (xi == i) nx_ = sr;
                }
                dx = is_x ? nx_ + cur.b : 0.0f;
            }
        };
        // three buffers used in turn, loads two stages ahead (no copies: a copy waits for the LDS read in flight)
        Stg c0, c1, c2;
        lds_ld(0, c0);
        lds_ld(1, c1);
        for (int k = 0;; k += 3) {
            lds_ld(k + 2, c2);
            step(k, c0);
            if (k == N) break;
            lds_ld(k + 3, c0);
            step(k + 1, c1);
            if (k + 1 == N) break;
            lds_ld(k + 4, c1);
            step(k + 2, c2);
            if (k + 2 == N) break;
        }
    }
#endif
    __syncthreads();
    RP_STAMP(2);

    // ---- P0c (stage-parallel): gradient, bounds, slacks, multipliers and the record of stage k on row k mod ROWS
    if (mode == kModeRun && P.terminal_hack && is_x && xi < 3) {  // NMPCNavControlDiff.cpp:127-139
        const bool eq = (s_ref[N * 3] == s_ref[(N - 1) * 3]) && (s_ref[N * 3 + 1] == s_ref[(N - 1) * 3 + 1]) &&
                        (s_ref[N * 3 + 2] == s_ref[(N - 1) * 3 + 2]);
        we_lane = (eq ? 100.0f : 1.0f) * w_lane;
    }
    const float lam_thr = P.infeas_lam * fmaxf(1.0f, fmaxf(P.wmax, row_max16(is_x ? we_lane : 0.0f)) * 0.1f);
    float sum_c0 = 0.0f;
    for (int j = 0; j < NR; j++) {
        const int kr = j * ROWS + q;
        const bool kv = kr <= N;
        const int k = kv ? kr : N;
        const float* const st = s_stg + (size_t)k * SF * 16 + r;
        const float zbar = st[0];
        const float yr = (mode == kModeRun) ? ((is_x && xi < 3) ? s_ref[k * 3 + xi] : 0.0f) : st[16];
        const float dxk = s_dx[k * 16 + r];
        float rec[RS];
#pragma unroll
        for (int f = 0; f < RS; f++) rec[f] = 0.0f;
        const bool vu = is_u && k < N, vx = is_x && k >= 1;
        const bool valid = vu || vx;
        const float w = vx ? ((k == N) ? we_lane : sc * w_lane) : sc * w_lane;
        rec[R::GR] = valid ? w * (zbar - yr) : 0.0f;
        const float z = vx ? dxk : 0.0f;
        rec[R::Z] = z;
        rec[R::TL] = kFar;
        rec[R::TU] = kFar;
        rec[R::LB] = -kFar;
        rec[R::UB] = kFar;
        if (valid && has_b) {
            const float lb = lo_b - zbar, ubd = hi_b - zbar;
            const float tl = fmaxf(z - lb, P.thr0), tu = fmaxf(ubd - z, P.thr0);
            rec[R::LB] = lb;
            rec[R::UB] = ubd;
            rec[R::TL] = tl;
            rec[R::TU] = tu;
            const float ll0 = warm ? fmaxf(fminf(st[32], kWarmLambdaCap), P.warm_kappa / tl) : P.mu0 / tl;
            const float lu0 = warm ? fmaxf(fminf(st[48], kWarmLambdaCap), P.warm_kappa / tu) : P.mu0 / tu;
            rec[R::LL] = ll0;
            rec[R::LU] = lu0;
            sum_c0 += kv ? ll0 * tl + lu0 * tu : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < NGV; i++) rec[R::GV + i] = (k < N && lv) ? st[(5 + i) * 16] : 0.0f;
        rec_store_range<0, RSS, RS, QM>(kv ? tbase_own + (size_t)k * KS : tdummy, rec);  // idle slots: own unused slot
    }
    {
        float v[6] = {wave_sum_rows(row_sum16(lv ? sum_c0 : 0.0f)), 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        const int op[6] = {0, 0, 0, 0, 0, 0};
        block_combine(v, op, 1);
        sum_c0 = v[0];
    }

#ifdef NMPC_ROWPAR_MCOL
    // A/B only: the column-form M block needs about 20 more registers, which pushes the segmented kernels past the
    // 256 that two waves per SIMD allow (tests/test_reg_usage.py), so the row form stays; tests/test_codegen.py
    // compiles this variant so that it keeps building
    GConst<M> gcs;  // the constant rows of [B A] as uniform operands of the M block (m_block)
    gconst_load<M>(gcs, gcol);
#endif
    const int m = N * NU + N * M::NBX;
    const float inv_m2 = 0.5f / (float)m;

    auto column = [&](const float (&rc)[RS], float (&Gc)[NX]) {
#pragma unroll
        for (int i = 0; i < NX; i++) Gc[i] = (i < NGV) ? rc[R::GV + (i < NGV ? i : 0)] : gcol[i];
    };
    auto dyn = [&](const float (&rc)[RS], float dzv) -> float {
        float nx_ = 0.0f;
#pragma unroll
        for (int i = 0; i < NGV; i++) {
            const float s = row_sum16(lv ? rc[R::GV + i] * dzv : 0.0f);
            if (xi == i) nx_ = s;
        }
        const float cr = dot_v<NX, NU>(0.0f, dzv, grow);
        return (xi >= NGV) ? cr : nx_;
    };
    // the fields of one stage each serial pass reads: the Jacobian rows GV from the global record, the rest from LDS
    // (phase B: SIG, C0, GH; phase C: LR, LM; the adjoint: C0)
    auto ld_bfields = [&](int k, float (&v)[RS]) {
        ld_range<R::GV, R::GV + NGV, RS, QM>(tbase + (size_t)k * KS, v);
        v[R::SIG] = it_rd(k, IT::SIG);
        v[R::C0] = it_rd(k, IT::C0);
        v[R::GH] = it_rd(k, IT::GH);
    };
    auto ld_cfields = [&](int k, float (&v)[RS]) {
        ld_range<R::GV, R::GV + NGV, RS, QM>(tbase + (size_t)k * KS, v);
        v[R::LR] = it_rd(k, IT::LR);
#pragma unroll
        for (int qq = 0; qq < NU; qq++) v[R::LM + qq] = it_rd(k, IT::LM + qq);
    };
    auto ld_adj = [&](int k, float (&v)[RS]) {
        ld_range<R::GV, R::GV + NGV, RS, QM>(tbase + (size_t)k * KS, v);
        v[R::C0] = it_rd(k, IT::C0);
    };
    // phase B's factor output of stage k (LR, LM) into LDS; w: this lane stores it
    auto st_lrlm = [&](int k, const float (&v)[RS], bool w) {
        *it_wr(k, IT::LR, w) = v[R::LR];
#pragma unroll
        for (int qq = 0; qq < NU; qq++) *it_wr(k, IT::LM + qq, w) = v[R::LM + qq];
    };
    // serial sweep k0 -> k1 with the next stage's fields (load(k, v)) in flight
    // (ping-pong buffers, loads never predicated: the loop is wave-uniform)
    auto serial = [&](int k0, int k1, int dir, auto&& load, auto&& body) {
        float ra[RS], rb[RS];
        load(k0, ra);
        for (int k = k0;; k += 2 * dir) {
            const int k_1 = (k == k1) ? k : k + dir;
            load(k_1, rb);
            body(k, ra);
            if (k == k1) break;
            const int k_2 = (k_1 == k1) ? k_1 : k_1 + dir;
            load(k_2, ra);
            body(k + dir, rb);
            if (k + dir == k1) break;
        }
    };

    // stage-parallel rounds j = 0 .. NR-1 (row q: stage j ROWS + q, clamped to N) with the next round's record fields
    // [F0, F1) and DZ in flight while body(j, fields, dz) runs (loads never predicated; past the last round the
    // last one is re-read)
    auto spar = [&](auto f0c, auto f1c, auto&& body) {
        constexpr int F0 = decltype(f0c)::value, F1 = decltype(f1c)::value;
        auto load = [&](int j, float (&v)[RS], float& dzv) {
            const int kr = j * ROWS + q;
            const int k = kr <= N ? kr : N;
            ld_range<F0, F1, RS, QM>(tbase + (size_t)k * KS, v);
            dzv = it_rd(k, IT::DZ);
        };
        float ra[RS], rb[RS], da, db;  // (two rounds ahead measured slower: profiles/r05/ab/spar_prefetch.txt)
        load(0, ra, da);
        for (int j = 0;; j += 2) {
            load(j + 1 < NR ? j + 1 : NR - 1, rb, db);
            body(j, ra, da);
            if (j + 1 >= NR) break;
            load(j + 2 < NR ? j + 2 : NR - 1, ra, da);
            body(j + 1, rb, db);
            if (j + 2 >= NR) break;
        }
    };

    // SEG: the segment area of the LDS (RowLds / SegLayout), and the serial adjoint pass of the stopping rule:
    // pi_k = c0_x + A_k' pi_{k+1} on the state slots, the input stationarity residual c0_u + B_k' pi_{k+1}
    const SegLayout<M> SegL(SEG ? a.seg : 1);
    float* const seg_lds = s_row + (SEG ? RowLds<M>::seg_off(N, a.seg) : 0);
    auto adjoint = [&](float& res_stat, float& cpi_max) {
        float piv = 0.0f, rs = 0.0f, cm = 0.0f;
        serial(N, 0, -1, ld_adj, [&](int k, float (&rc)[RS]) {
            const bool vu = is_u && k < N;
            const bool vx = is_x && k >= 1;
            float Gc[NX];
            column(rc, Gc);
            const float cpi = (k < N) ? dot_x<NX, NU>(0.0f, piv, Gc) : 0.0f;
            const float base = rc[R::C0] + cpi;
            rs = nan_max(rs, vu ? fabsf(base) : 0.0f);
            cm = fmaxf(cm, vu ? fabsf(cpi) : 0.0f);
            piv = vx ? base : 0.0f;
        });
        res_stat = row_max16(lv ? rs : 0.0f);
        cpi_max = row_max16(lv ? cm : 0.0f);
    };

    // ---- interior-point iterations (single-direction rule) -----------------------------------------------------
    int status = 0, it_done = 0;
    float exit_res[3] = {0.0f, 0.0f, 0.0f};
    float alpha = 0.0f, sigma_mu = 0.0f, mu_prev = 3.0e38f;
    float tg_rhs = P.sd_hi * sum_c0 * inv_m2;
    int bseg_runs = 0;  // (SEG) executions of phase B so far
    for (int it = 0;; it++) {
        // phase A (stage-parallel): apply the previous step, residuals, barrier weight, rhs terms
        const float a_upd = (it > 0) ? alpha : 0.0f;
        float res_ineq = 0.0f, sum_c = 0.0f, max_c = 0.0f, lam_max = 0.0f, sc0 = 1.0f, nanf_ = 0.0f;
        spar(std::integral_constant<int, R::Z>{}, std::integral_constant<int, R::GR + 1>{},
             [&](int j, float (&rc)[RS], float dz) {
            const int kr = j * ROWS + q;
            const bool kv = kr <= N;       // rows past the last stage redo stage N into the dummy record
            const int k = kv ? kr : N;
            const bool vu = is_u && k < N && kv;
            const bool vx = is_x && k >= 1 && kv;
            const bool valid = vu || vx;
            const bool bnd = valid && has_b;
            float z = rc[R::Z];
            float tl = rc[R::TL], tu = rc[R::TU], ll = rc[R::LL], lu = rc[R::LU];
            const float lb = rc[R::LB], ubd = rc[R::UB];
            {
                const float rl = z - lb - tl, rr = ubd - z - tu;
                const float itl = frcp(tl), itu = frcp(tu);
                dz = (it > 0) ? dz : 0.0f;  // (iteration 0 applies no step; the LDS field is not written yet)
                const BoundDir d = bound_dir(dz, rl, rr, tl, tu, ll, lu, itl, itu, sigma_mu, sigma_mu);
                const float ab = bnd ? a_upd : 0.0f, av = valid ? a_upd : 0.0f;
                tl += ab * d.dtl;
                tu += ab * d.dtu;
                ll += ab * d.dll;
                lu += ab * d.dlu;
                z += av * dz;
            }
            const float rl = z - lb - tl, rr = ubd - z - tu;
            const float itl = frcp(tl), itu = frcp(tu);
            res_ineq = fmaxf(res_ineq, kv ? fmaxf(fabsf(rl), fabsf(rr)) : 0.0f);
            sum_c += kv ? ll * tl + lu * tu : 0.0f;
            max_c = fmaxf(max_c, kv ? fmaxf(ll * tl, lu * tu) : 0.0f);
            lam_max = fmaxf(lam_max, kv ? fmaxf(ll, lu) : 0.0f);
            const float lamdiff = ll - lu;
            const float sig = ll * itl + lu * itu;
            const float gh = ll * rl * itl + ll - lu * rr * itu - lu - tg_rhs * itl + tg_rhs * itu;
            const float g = rc[R::GR];
            const float hz = ((k < N) ? h_stage : we_lane) * z;
            const float c0 = hz + g - lamdiff;
            if (vu) sc0 = fmaxf(sc0, fmaxf(fabsf(g), fabsf(lamdiff)));
            if (kv && (sig != sig || gh != gh || c0 != c0)) nanf_ = 1.0f;
            rc[R::Z] = z;
            rc[R::TL] = tl;
            rc[R::TU] = tu;
            rc[R::LL] = ll;
            rc[R::LU] = lu;
            float* const pk = (lv && kv) ? tbase + (size_t)k * KS : tdummy;
            rec_store_range<R::Z, R::LU + 1, RS, QM>(pk, rc);  // the iterate and slacks / multipliers: global
            *it_wr(k, IT::SIG, lv && kv) = sig;  // phase B's inputs: LDS
            *it_wr(k, IT::C0, lv && kv) = c0;
            *it_wr(k, IT::GH, lv && kv) = valid ? gh : 0.0f;
        });
        {
            float v[6] = {wave_sum_rows(row_sum16(lv ? sum_c : 0.0f)), wave_max_rows(row_max16(lv ? max_c : 0.0f)),
                          wave_max_rows(row_max16(lv ? lam_max : 0.0f)), wave_max_rows(row_max16(lv ? res_ineq : 0.0f)),
                          wave_max_rows(row_max16(sc0)), wave_max_rows(row_max16(nanf_))};
            const int op[6] = {0, 1, 1, 1, 1, 1};
            block_combine(v, op, 6);
            sum_c = v[0];
            max_c = v[1];
            lam_max = v[2];
            res_ineq = v[3];
            sc0 = v[4];
            nanf_ = v[5];
        }
        const float mu = sum_c * inv_m2;
        RP_STAMP(3 + 4 * it);

        // phase D's terms of stage k on this lane (kv: the stage is this row's): bound directions, the
        // fraction-to-boundary step bound and the complementarity polynomial. SEG: accumulated inside phase C as each
        // row's forward recursion produces the direction of a stage (its record fields loaded with C's), so phase D
        // is only the block reduction; -DNMPC_D_SEPARATE keeps the separate stage-parallel pass for A/B runs
#ifdef NMPC_D_SEPARATE
        constexpr bool kDinC = false;
#else
        constexpr bool kDinC = SEG;
#endif
        float amax = 1e30f, s1 = 0.0f, s2 = 0.0f;
        auto dterm = [&](int k, bool kv, const float (&rc)[RS], float dz) {
            const bool valid = kv && ((is_u && k < N) || (is_x && k >= 1));
            const bool bnd = valid && has_b;
            const float z = rc[R::Z];
            const float tl = rc[R::TL], tu = rc[R::TU], ll = rc[R::LL], lu = rc[R::LU];
            const float rl = z - rc[R::LB] - tl, rr = rc[R::UB] - z - tu;
            const float itl = frcp(tl), itu = frcp(tu);
            const BoundDir d = bound_dir(dz, rl, rr, tl, tu, ll, lu, itl, itu, sigma_mu, sigma_mu);
            if (kv) {
                amax = step_bound_r(amax, tl, d.dtl);
                amax = step_bound_r(amax, tu, d.dtu);
                amax = step_bound_r(amax, ll, d.dll);
                amax = step_bound_r(amax, lu, d.dlu);
            }
            s1 += bnd ? ll * d.dtl + tl * d.dll + lu * d.dtu + tu * d.dlu : 0.0f;
            s2 += bnd ? d.dll * d.dtl + d.dlu * d.dtu : 0.0f;
        };

        if constexpr (SEG) {
            // ---- stopping rule first (phase A's sums); the stationarity residual needs the exact adjoint, a serial
            // pass run only when the rest of the first exit clause holds (typically the last one or two iterations)
            exit_res[1] = res_ineq;
            exit_res[2] = mu;
            float res_stat = -1.0f;
            bool stop = false;
            if (nanf_ > 0.0f || mu != mu) {
                status = 1;
                stop = true;
            } else if (lam_max > lam_thr && res_ineq > kInfeasRes) {
                status = 4;
                stop = true;
            } else {
                const bool feas = res_ineq <= P.tol_ineq;
                const bool cmax_ok = max_c <= kCompMaxRatio * P.tol_comp;
                const bool stalled = mu <= P.tol_comp && mu > 0.5f * mu_prev;
                if (feas && (mu <= 1e-2f * P.tol_comp || (stalled && cmax_ok))) {
                    stop = true;
                } else if (feas && mu <= P.tol_comp && cmax_ok) {
                    float cpi_max;
                    adjoint(res_stat, cpi_max);
                    if (res_stat <= P.tol_stat || res_stat <= kStatRelT * fmaxf(sc0, cpi_max)) stop = true;
                }
                if (it >= P.iter_max) stop = true;
            }
            mu_prev = mu;
            if (stop) {
                if (res_stat < 0.0f) {
                    float cm;
                    adjoint(res_stat, cm);
                }
                exit_res[0] = res_stat;
                it_done = it;
                break;
            }

            // ---- phase B (segments in parallel, each N -> its first stage): fp64 Riccati step on the absolute
            // rhs, plus the sensitivities to the segment's free end costate lam (Phi, Z) and the lam terms of its
            // value (Gam, t). Row q takes stages [q L, (q + 1) L), the last row also the terminal stage N. Iteration
            // j = 0 initialises: the last row with the terminal P_N, p_N; the others with P = 0, p = 0, Phi = I
            const int Sg = a.seg, Ls = N / Sg;
            const bool srow = q < Sg, slast = q == Sg - 1;
            // Two or four waves and at most 4 W / 2 segments: the lam sensitivities (Phi, Z, Gam, t) of segment q run
            // on row q + 2 W (the second half of the waves), one stage behind its factorisation on row q (the first
            // half), from the factor columns LR / LM the factorisation leaves in LDS (a count per factor wave of its
            // finished stages); the factorisation's chain loses the sensitivities' ~130 instructions per stage (same
            // box: capsule -5 %, diff1024 +3.7 %, profiles/r06/ab/sens_split.txt). Otherwise each row does both.
            // -DNMPC_SENS_FUSED keeps them together for A/B runs.
#ifdef NMPC_SENS_FUSED
            constexpr bool kSensSplit = false;
#else
            constexpr bool kSensSplit = W >= 2;
#endif
            constexpr int SW = W / 2, SOFF = 4 * SW;  // factor waves [0, SW), sensitivity rows q + SOFF
            const bool ssplit = kSensSplit && Sg <= SOFF;
            double Lrow[NV];
            float pv = 0.0f, Phi[NX], tt = 0.0f, nanb = 0.0f;
            double Gam[NX];  // fp64 sum of exact fp32 products (an fp32 sum broke the dual sweep's factor of -Gam_0)
#pragma unroll
            for (int j = 0; j < NV; j++) Lrow[j] = 0.0;
#pragma unroll
            for (int c = 0; c < NX; c++) {
                Phi[c] = 0.0f;
                Gam[c] = 0.0;
            }
            bool fail = false;
            // one stage of the sensitivities: column c of Y = G' Phi_{k+1}, Z = L^-1 Y_u (uniform over the row), and
            // Phi_k = Y_x - LM Z; the value's lam terms Gam -= Z'Z, t -= Z' LR; Z to LDS for phase C
            // (column by column: the fused all-column block held 7 more accumulators live and pushed the
            // kernel past 256 registers, one wave per SIMD: diff1024 1.65 -> 1.11 M it/s)
            auto sens_step = [&](int k, bool srw, const float (&Gc)[NX], const float (&Lm)[NU], const float (&rLm)[NU],
                                 const float (&lrv)[NU]) {
                float zc[NU][NX];
                sfor<0, NX>([&](auto cc) {
                    constexpr int c = decltype(cc)::value;
                    float yc = dot_x<NX, NU>(0.0f, Phi[c], Gc);
                    sfor<0, NU>([&](auto jc) {
                        constexpr int j2 = decltype(jc)::value;
                        const float z = bc<j2>(yc * rLm[j2]);
                        zc[j2][c] = z;
                        yc -= Lm[j2] * z;
                    });
                    Phi[c] = is_x ? yc : 0.0f;
                });
                float zi[NU], zr[NX];
#pragma unroll
                for (int j2 = 0; j2 < NU; j2++) {
                    float s = 0.0f;
#pragma unroll
                    for (int c = 0; c < NX; c++) s = (xi == c) ? zc[j2][c] : s;
                    zi[j2] = s;
                }
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    double g = Gam[c];
#pragma unroll
                    for (int j2 = 0; j2 < NU; j2++) g -= (double)zi[j2] * (double)zc[j2][c];
                    Gam[c] = g;
                    float s = zc[0][c];
#pragma unroll
                    for (int j2 = 1; j2 < NU; j2++) s = (r == j2) ? zc[j2][c] : s;
                    zr[c] = s;  // input lane j: row j of Z
                }
#pragma unroll
                for (int j2 = 0; j2 < NU; j2++) tt -= zi[j2] * lrv[j2];
                if (srw && is_u) {
                    float* const zp = seg_lds + SegL.ZL + ((size_t)k * NU + r) * SegLayout<M>::NXP;
#pragma unroll
                    for (int c = 0; c < NX; c++) zp[c] = zr[c];
                }
            };
            // the segment's sensitivity summary for the master (state lanes: row xi of segment qq)
            auto store_sens = [&](int qq) {
                seg_lds[SegL.SUM_T + qq * NX + xi] = tt;
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    seg_lds[SegL.SUM_PHI + (qq * NX + xi) * NX + c] = Phi[c];
                    reinterpret_cast<double*>(seg_lds + SegL.SUM_GAM)[(qq * NX + xi) * NX + c] = Gam[c];
                }
            };
            // finished factorisation stages of factor wave w (waves 0-1), counted over the whole launch
            unsigned int* const b_cnt = reinterpret_cast<unsigned int*>(s_red + 15);  // [w * 8]
            if (4 * wave < Sg) {  // (wave-uniform) the wave holds a segment
                auto kof = [&](int j) { return srow ? (q + 1) * Ls - j : N; };
                auto bseg = [&](int j, float (&rc)[RS]) {
                    const int k = kof(j);
                    const bool vu = srow && is_u && k < N;
                    const bool vx = srow && is_x && k >= 1;
                    const bool valid = vu || vx;
                    float Gc[NX];
                    column(rc, Gc);
                    const float sig = rc[R::SIG];
                    const float ghat = valid ? rc[R::GH] + rc[R::C0] : 0.0f;
                    if (ghat != ghat) nanb = 1.0f;
                    if (j == 0) {
                        const double d = (slast && is_x) ? (double)fmaxf(we_lane + sig, 0.0f) : 0.0;
#pragma unroll
                        for (int jj = 0; jj < NV; jj++) Lrow[jj] = (is_x && jj == r) ? d : 0.0;
                        pv = (slast && is_x) ? ghat : 0.0f;
#pragma unroll
                        for (int c = 0; c < NX; c++) Phi[c] = (!slast && is_x && xi == c) ? 1.0f : 0.0f;
                        return;
                    }
                    double Gd[NX];
#pragma unroll
                    for (int l = 0; l < NX; l++) Gd[l] = (double)Gc[l];
                    double pg[NX];
#pragma unroll
                    for (int i = 0; i < NX; i++) pg[i] = 0.0;
                    pg_block<NX, NU>(pg, Lrow, Gd);
                    const double dg = valid ? (double)h_stage + (double)sig : 1.0;
                    double Lr[NV];
#pragma unroll
                    for (int jj = 0; jj < NV; jj++) Lr[jj] = (r == jj) ? dg : 0.0;
                    double pivot;
#ifdef NMPC_ROWPAR_MCOL
                    double m11, m10;  // the 2x2 input block for up-front pivots (unused: pivots in turn below)
                    m_block<M>(Lr, pivot, m11, m10, pg, Gd, gcs);
                    (void)m11;
                    (void)m10;
#else
                    mrow_pg_block<NX, NU>(Lr, pivot, pg, Gd);
#endif
                    sfor<0, NU>([&](auto jc) {
                        constexpr int j2 = decltype(jc)::value;
                        if (!(pivot > 0.0) && srow) fail = true;
                        const double rd = drsq(fmax(pivot, 1e-300));
                        const double lj = (r >= j2) ? Lr[j2] * rd : 0.0;
                        Lr[j2] = lj;
                        chol_update<NX, NU, j2>(Lr, lj, pivot);
                    });
                    float Lm[NU], rLm[NU];
#pragma unroll
                    for (int qq = 0; qq < NU; qq++) {
                        Lm[qq] = (float)Lr[qq];
                        rc[R::LM + qq] = Lm[qq];
                        rLm[qq] = frcp(Lm[qq]);
                    }
                    // rhs (absolute form): w = g^ + G' p_{k+1}, forward substitution over the input block
                    float y = dot_x<NX, NU>(ghat, pv, Gc);
                    float my_lr = 0.0f, lrv[NU];
                    sfor<0, NU>([&](auto jc) {
                        constexpr int j2 = decltype(jc)::value;
                        const float lrj = bc<j2>(y * rLm[j2]);
                        lrv[j2] = lrj;
                        if (r == j2) my_lr = lrj;
                        y -= Lm[j2] * lrj;
                    });
                    rc[R::LR] = my_lr;
                    pv = is_x ? y : 0.0f;
                    if (!ssplit) sens_step(k, srow, Gc, Lm, rLm, lrv);
#pragma unroll
                    for (int jj = 0; jj < NV; jj++) Lrow[jj] = Lr[jj];
                    st_lrlm(k, rc, lv && srow);
                    if (ssplit) {
                        // this stage's LR / LM are in LDS (LDS completes in order per wave), then its count
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if ((tid & 63) == 0)
                            __hip_atomic_fetch_add(b_cnt + wave * 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                };
                auto load = [&](int j, float (&v)[RS]) { ld_bfields(kof(j), v); };
                float ra[RS], rb[RS];
                load(0, ra);
                for (int j = 0;; j += 2) {
                    load(j + 1 <= Ls ? j + 1 : Ls, rb);
                    bseg(j, ra);
                    if (j == Ls) break;
                    load(j + 2 <= Ls ? j + 2 : Ls, ra);
                    bseg(j + 1, rb);
                    if (j + 1 == Ls) break;
                }
                // the segment's entry quantities for the master (state lanes: row xi)
                if (srow && is_x) {
                    double* const sp = reinterpret_cast<double*>(seg_lds + SegL.SUM_P) + ((size_t)q * NX + xi) * NX;
#pragma unroll
                    for (int l = 0; l < NX; l++) sp[l] = Lrow[NU + l];
                    seg_lds[SegL.SUM_PB + q * NX + xi] = pv;
                    if (!ssplit) store_sens(q);
                }
            } else if (ssplit && wave >= SW && 4 * (wave - SW) < Sg) {
                // the sensitivity rows: segment qs = q - SOFF, stage after stage as factor wave wave - SW finishes them
                const int qs = q - SOFF;
                const bool srs = qs < Sg, slast_s = qs == Sg - 1;
                auto kos = [&](int j) { return srs ? (qs + 1) * Ls - j : N; };
#pragma unroll
                for (int c = 0; c < NX; c++) Phi[c] = (srs && !slast_s && is_x && xi == c) ? 1.0f : 0.0f;
                const unsigned int base = (unsigned int)bseg_runs * (unsigned int)Ls;
                unsigned int done_f = 0;
                auto wait_f = [&](int j) {
                    const unsigned int need = base + (unsigned int)j;
                    for (int g = 0; done_f < need && g < (1 << 24); g++) {
                        done_f = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(b_cnt + (wave - SW) * 8, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                        if (done_f < need) __builtin_amdgcn_s_sleep(1);
                    }
                };
                auto sload = [&](int j, float (&v)[RS]) {
                    ld_range<R::GV, R::GV + NGV, RS, QM>(tbase + (size_t)kos(j) * KS, v);
                };
                auto sstep = [&](int j, float (&rc)[RS]) {
                    const int k = kos(j);
                    wait_f(j);
                    float Gc[NX];
                    column(rc, Gc);
                    float Lm[NU], rLm[NU], lrv[NU];
#pragma unroll
                    for (int qq = 0; qq < NU; qq++) {
                        Lm[qq] = it_rd(k, IT::LM + qq);
                        rLm[qq] = frcp(Lm[qq]);
                        lrv[qq] = it_lds[((size_t)k * IT::NF + IT::LR) * NV + qq];  // (the LR of input lane qq)
                    }
                    sens_step(k, srs, Gc, Lm, rLm, lrv);
                };
                float ra[RS], rb[RS];
                sload(1, ra);
                for (int j = 1;; j += 2) {
                    sload(j + 1 <= Ls ? j + 1 : Ls, rb);
                    sstep(j, ra);
                    if (j == Ls) break;
                    sload(j + 2 <= Ls ? j + 2 : Ls, ra);
                    sstep(j + 1, rb);
                    if (j + 1 == Ls) break;
                }
                if (srs && is_x) store_sens(qs);
            }
            bseg_runs++;
            {
                float v[6] = {wave_max_rows(row_max16(fail ? 1.0f : 0.0f)), wave_max_rows(row_max16(nanb)), 0.0f,
                              0.0f, 0.0f, 0.0f};
                const int op[6] = {1, 1, 0, 0, 0, 0};
                block_combine(v, op, 2);  // (also the barrier: every segment's summary and LR / LM are stored)
                if (v[1] > 0.0f || v[0] > 0.0f) {
                    status = (v[1] > 0.0f) ? 1 : ((mu <= kBreakdownMuT && res_ineq <= P.tol_ineq * 10.0f) ? 0 : 4);
                    float cm;
                    adjoint(res_stat, cm);
                    exit_res[0] = res_stat;
                    it_done = it;
                    break;
                }
            }
            RP_STAMP(4 + 4 * it);

            // ---- master (fp64): the two-point recursion over the segment boundaries,
            //   s_{i+1} = Phi_i' s_i + Gam_i lam_{i+1} + t_i,   lam_i = P_i s_i + pbar_i + Phi_i lam_{i+1}   (s_0 = 0),
            // solved from both ends at once and joined at boundary m = S / 2 (round 5: the chain of factorisations
            // falls from S - 1 boundary steps to max(S - 1 - m, m - 1) + 1, e.g. 7 -> 4 at N = 80, S = 8):
            //  - row 0 of wave 0, the backward sweep lam_i = Phat_i s_i + phat_i (Phat_{S-1} = P_{S-1}) down to m, with
            //    Q_i = Phat_{i+1} (I - Gam_i Phat_{i+1})^-1, Phat_i = P_i + Phi_i Q_i Phi_i', c_i = t_i + Gam_i phat_{i+1},
            //    phat_i = pbar_i + Phi_i (Q_i c_i + phat_{i+1});
            //  - row 1 of wave 0, the dual sweep s_i = -Shat_i lam_i + shat_i (Shat_1 = -Gam_0, shat_1 = t_0) up to m,
            //    Q'_i = (I + Shat_i P_i)^-1 Shat_i, Shat_{i+1} = -Gam_i + Phi_i' Q'_i Phi_i,
            //    u_i = shat_i - Q'_i (pbar_i + P_i shat_i), shat_{i+1} = t_i + Phi_i' u_i;
            //  - the join (row 0): lam_m = Q_j (shat_m - Shat_m phat_m) + phat_m, Q_j = Phat_m (I + Shat_m Phat_m)^-1,
            //    s_m = shat_m - Shat_m lam_m;
            //  - row 0 propagates s, lam forward to S - 1 (lam_{i+1} = Q_i (Phi_i' s_i + c_i) + phat_{i+1},
            //    s_{i+1} = Phi_i' s_i + Gam_i lam_{i+1} + t_i) while row 1 propagates them back to 1
            //    (s_i = u_i - Q'_i Phi_i lam_{i+1}, lam_i = P_i s_i + pbar_i + Phi_i lam_{i+1}).
            // Both sweeps are one instruction stream: a step is the same sequence of fused-DPP blocks on the two rows,
            // each row addressing its own operands (backward: C = -Gam_i, D = P_i, F = Phi_i; dual: C = P_i,
            // D = -Gam_i, F = Phi_i'), so they cost one step's issue; on two waves of a CU they slowed each other
            // down by half (profiles/r05/stamps/). Every Q (Q_i, Q'_i, Q_j) is A (I + C A)^-1 = L (I + L' C L)^-1 L'
            // with C >= 0 (mst_qform). Lane NU + r of a row holds row r of every matrix and element r of every vector.
#ifdef NMPC_SEQ_MASTER
            constexpr bool kSeqM = true;  // A/B only: the round-4 master (backward over all S - 1 boundaries, then forward)
#else
            constexpr bool kSeqM = false;
#endif
            const int mj = kSeqM ? 0 : Sg / 2;        // the join boundary (1 <= m <= S - 1)
            const int nbw = Sg - 1 - mj;              // backward-sweep steps (boundaries S - 2 .. m)
            const int ndu = kSeqM ? 0 : mj - 1;       // dual-sweep steps (boundaries 1 .. m - 1)
            const bool mrow0 = tid < 16;              // backward sweep, join, forward propagation
            const bool bwr = mrow0;                   // (row 1 of wave 0: the dual side)
            float* const sl = seg_lds + SegL.SL;
            if (Sg > 1 && wave == 0 && tid < 32) {
                const double* const sP = reinterpret_cast<const double*>(seg_lds + SegL.SUM_P);
                const double* const sG = reinterpret_cast<const double*>(seg_lds + SegL.SUM_GAM);
                double* const sQ = reinterpret_cast<double*>(seg_lds + SegL.QS);
                double* const sCv = reinterpret_cast<double*>(seg_lds + SegL.CS);
                double* const sPh = reinterpret_cast<double*>(seg_lds + SegL.PHS);
                double* const sLt = reinterpret_cast<double*>(seg_lds + SegL.LT) + (bwr ? 0 : NX * NX);
                double* const sXa = reinterpret_cast<double*>(seg_lds + SegL.XA);
                double* const sXo = sXa + (bwr ? 0 : (NX + 1) * NX);  // this row's final (X, x): Phat_m / Shat_m
                const double sgn = bwr ? -1.0 : 1.0;
                // per-row operands of boundary i: C (sign sgn) and D (sign -sgn) rows, the F row (Phi_i row or
                // column) and the vector terms a0 (t_i / pbar_i) and a1 (pbar_i / t_i)
                const double* const pC = bwr ? sG : sP;
                const double* const pD = bwr ? sP : sG;
                const int fs1 = bwr ? NX : 1, fs2 = bwr ? 1 : NX;  // F element c: Phi[i][xi * fs1 + c * fs2]
                const int a0off = bwr ? SegL.SUM_T : SegL.SUM_PB, a1off = bwr ? SegL.SUM_PB : SegL.SUM_T;
                double X[NX], x;
                {  // Phat_{S-1} = P_{S-1}, phat_{S-1} = pbar_{S-1} / Shat_1 = -Gam_0, shat_1 = t_0
                    const int i0 = bwr ? Sg - 1 : 0;
#pragma unroll
                    for (int c = 0; c < NX; c++) X[c] = -sgn * pD[((size_t)i0 * NX + xi) * NX + c];
                    x = (double)seg_lds[(bwr ? SegL.SUM_PB : SegL.SUM_T) + i0 * NX + xi];
                }
                if (is_x) {
#pragma unroll
                    for (int c = 0; c < NX; c++) sXo[xi * NX + c] = X[c];
                    sXo[NX * NX + xi] = x;
                }
                RP_MSTAMP(0, 0);
                const int ns = nbw > ndu ? nbw : ndu;
                for (int j = 0; j < ns; j++) {
                    const bool act = bwr ? (j < nbw) : (j < ndu);
                    const int i = act ? (bwr ? Sg - 2 - j : 1 + j) : 1;  // (an idle row reads boundary 1, stores nothing)
                    double Cm[NX], Q[NX];
#pragma unroll
                    for (int c = 0; c < NX; c++) Cm[c] = sgn * pC[((size_t)i * NX + xi) * NX + c];
                    mst_qform<NX, NU>(X, Cm, Q, sLt, xi, is_x);
                    // v = a0 + R x (R = Gam_i / P_i = sgn C): c_i / e_i;  w = x + sQ Q v (sQ = -sgn): phat + Q c / u_i
                    const double v = mst_vdot<NX, NU>((double)seg_lds[a0off + i * NX + xi], sgn * x, Cm);
                    const double w = mst_vdot<NX, NU>(x, -sgn * v, Q);
                    if (act && is_x) {
#pragma unroll
                        for (int c = 0; c < NX; c++) sQ[((size_t)i * NX + xi) * NX + c] = Q[c];
                        sCv[i * NX + xi] = bwr ? v : w;
                        if (bwr) sPh[i * NX + xi] = x;
                    }
                    // X' = D + F Q F', x' = a1 + F w
                    double Fr[NX], T[NX];
#pragma unroll
                    for (int c = 0; c < NX; c++) {
                        Fr[c] = (double)seg_lds[SegL.SUM_PHI + i * NX * NX + xi * fs1 + c * fs2];
                        T[c] = 0.0;
                        X[c] = -sgn * pD[((size_t)i * NX + xi) * NX + c];
                    }
                    mst_rowdot<NX, NU>(T, Q, Fr);
                    mst_rowmul<NX, NU>(X, Fr, T);
                    x = mst_vdot<NX, NU>((double)seg_lds[a1off + i * NX + xi], w, Fr);
                    if (act && is_x) {
#pragma unroll
                        for (int c = 0; c < NX; c++) sXo[xi * NX + c] = X[c];
                        sXo[NX * NX + xi] = x;
                    }
                    if (bwr) RP_SSTAMP(i);
                }
                lds_fence();  // (Q_i, c_i, u_i, phat, and both rows' final X, x in LDS)
                RP_MSTAMP(1, 0);
                // the join (row 0): lam_m, s_m
                double sv = 0.0, lam_m = 0.0;
                if (!kSeqM && bwr) {
                    double Pm[NX], Sr[NX], Q[NX];
#pragma unroll
                    for (int c = 0; c < NX; c++) {
                        Pm[c] = sXa[xi * NX + c];
                        Sr[c] = sXa[(NX + 1 + xi) * NX + c];
                    }
                    mst_qform<NX, NU>(Pm, Sr, Q, sLt, xi, is_x);
                    const double ph = sXa[NX * NX + xi], shm = sXa[(2 * NX + 1) * NX + xi];
                    const double v1 = mst_vdot<NX, NU>(shm, -ph, Sr);  // shat_m - Shat_m phat_m
                    lam_m = mst_vdot<NX, NU>(ph, v1, Q);
                    sv = mst_vdot<NX, NU>(shm, -lam_m, Sr);           // s_m = shat_m - Shat_m lam_m
                    if (is_x) {
                        sl[mj * 2 * NX + xi] = (float)sv;
                        sl[mj * 2 * NX + NX + xi] = (float)lam_m;
                        sXa[2 * (NX + 1) * NX + xi] = lam_m;  // (full precision for row 1)
                    }
                }
                lds_fence();
                RP_MSTAMP(4, 0);
                // outward propagation, both rows as one stream: z = s_i (row 0, i = m .. S - 2) / lam_{i+1} (row 1,
                // i = m - 1 .. 1);  y = F z (F = Phi_i' / Phi_i);  o = b0 + sO Q_i (y + alpha) (lam_{i+1} / s_i);
                // z' = y + beta + R o (s_{i+1} / lam_i), R = Gam_i / P_i
                double z = bwr ? sv : (kSeqM ? 0.0 : sXa[2 * (NX + 1) * NX + xi]);
                const int nfw = Sg - 1 - mj, nbp = kSeqM ? 0 : mj - 1;
                const int no = nfw > nbp ? nfw : nbp;
                const int gs1 = bwr ? 1 : NX, gs2 = bwr ? NX : 1;  // (the transposed F of the sweep)
                for (int j = 0; j < no; j++) {
                    const bool act = bwr ? (j < nfw) : (j < nbp);
                    const int i = act ? (bwr ? mj + j : mj - 1 - j) : 1;
                    double Fr[NX], Qr[NX], Rr[NX];
#pragma unroll
                    for (int l = 0; l < NX; l++) {
                        Fr[l] = (double)seg_lds[SegL.SUM_PHI + i * NX * NX + xi * gs1 + l * gs2];
                        Qr[l] = sQ[((size_t)i * NX + xi) * NX + l];
                        Rr[l] = pC[((size_t)i * NX + xi) * NX + l];
                    }
                    const double y = mst_vdot<NX, NU>(0.0, z, Fr);
                    const double cw = sCv[i * NX + xi];  // c_i (row 0) / u_i (row 1)
                    const double b0 = bwr ? sPh[i * NX + xi] : cw;
                    const double o = mst_vdot<NX, NU>(b0, bwr ? y + cw : -y, Qr);
                    const double z2 = mst_vdot<NX, NU>(y + (double)seg_lds[a0off + i * NX + xi], o, Rr);
                    if (act && is_x) {
                        const int slot = bwr ? i + 1 : i;
                        sl[slot * 2 * NX + xi] = (float)(bwr ? z2 : o);
                        sl[slot * 2 * NX + NX + xi] = (float)(bwr ? o : z2);
                    }
                    z = z2;
                }
                RP_MSTAMP(5, 0);
            }
            __syncthreads();  // the boundary states and costates
            RP_MSTAMP(7, 0);
            RP_STAMP(5 + 4 * it);

            // ---- phase C (segments in parallel, 0 -> N): row q starts at x_{qL} = s_q and takes the stored
            // factor with LR + Z lam_{q+1}; rows other than the last stop before the next segment's first stage
            sigma_mu = tg_rhs;
            // LR_k + Z_k lam_{q+1} of every stage of a segment with a free end costate, before the chain, over the
            // block's lanes. Two waves: inside phase C's chain its seven LDS operand loads serialised through one
            // register under the two-wave register bound (four dependent LDS round trips per stage in the ISA); the
            // pass takes diff1024 1.83 -> 1.88 M it/s same-box. Four waves (one per SIMD, no such bound) lose with it
            // (capsule 0.240 -> 0.248 ms cold: the chain's loads were already batched, the pass and its barrier are
            // extra), so they keep the update in the chain (profiles/r06/ab/lr_pre.txt). -DNMPC_LR_IN_C: in the
            // chain everywhere, for A/B runs
#ifdef NMPC_LR_IN_C
            constexpr bool kLrPre = false;
#else
            constexpr bool kLrPre = W == 2;
#endif
            if constexpr (kLrPre) {
                // segment by segment (0 .. S - 2), one (stage, input) pair of the segment per lane of the block
#pragma unroll 1
                for (int qs = 0; qs < Sg - 1; qs++) {
                    // lam_{qs+1} is block-uniform: scalar registers (the VGPRs are at the two-wave bound)
                    float lam[NX];
#pragma unroll
                    for (int c = 0; c < NX; c++)
                        lam[c] = __int_as_float(__builtin_amdgcn_readfirstlane(
                            __float_as_int(seg_lds[SegL.SL + (qs + 1) * 2 * NX + NX + c])));
#pragma unroll 1
                    for (int p0 = 0; p0 < Ls * NU; p0 += 64 * W) {
                        const bool act = p0 + tid < Ls * NU;
                        const int p = act ? p0 + tid : 0;
                        const int k = qs * Ls + p / NU, j = p % NU;
                        const float* const zp = seg_lds + SegL.ZL + ((size_t)k * NU + j) * SegLayout<M>::NXP;
                        float* const lrp = it_lds + ((size_t)k * IT::NF + IT::LR) * NV + j;
                        float lr = *lrp;
#pragma unroll
                        for (int c = 0; c < NX; c++) lr += zp[c] * lam[c];
                        if (act) *lrp = lr;
                    }
                }
                __syncthreads();  // the updated LR of every stage
            }
            if (4 * wave < Sg) {
                const float* const sl = seg_lds + SegL.SL;
                float lam[NX];
                float dxs = 0.0f;
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    lam[c] = (srow && !slast) ? sl[(q + 1) * 2 * NX + NX + c] : 0.0f;
                    const float s0 = (srow && q > 0) ? sl[q * 2 * NX + c] : 0.0f;
                    dxs = (is_x && xi == c) ? s0 : dxs;
                }
                auto kof = [&](int j) { return srow ? q * Ls + j : N; };
                auto cseg = [&](int j, float (&rc)[RS]) {
                    const int k = kof(j);
                    const bool live = srow && (j < Ls || slast);
                    const bool vu = is_u && k < N;
                    const bool vx = is_x && k >= 1;
                    const bool valid = live && (vu || vx);
                    float du_all[NU];
#pragma unroll
                    for (int qq = 0; qq < NU; qq++) du_all[qq] = 0.0f;
                    if (k < N) {
                        if constexpr (!kLrPre) {
                            // LR of the segment's end costate (input lane j: row j of Z_k . lam)
                            const float* const zp =
                                seg_lds + SegL.ZL + ((size_t)k * NU + (is_u ? r : 0)) * SegLayout<M>::NXP;
                            float lr = rc[R::LR];
#pragma unroll
                            for (int c = 0; c < NX; c++) lr += zp[c] * lam[c];
                            rc[R::LR] = is_u ? lr : rc[R::LR];
                        }
                        float w[NU];
                        sfor<0, NU>([&](auto qc) {
                            constexpr int qq = decltype(qc)::value;
                            w[qq] = bc<qq>(rc[R::LR]) + row_sum16(is_x ? rc[R::LM + qq] * dxs : 0.0f);
                        });
                        sfor<0, NU>([&](auto qqc) {
                            constexpr int qq = NU - 1 - decltype(qqc)::value;
                            float sq = w[qq];
                            sfor<qq + 1, NU>([&](auto jc) {
                                constexpr int j2 = decltype(jc)::value;
                                sq -= bc<j2>(rc[R::LM + qq]) * du_all[j2];
                            });
                            du_all[qq] = sq * frcp(bc<qq>(rc[R::LM + qq]));
                        });
#pragma unroll
                        for (int qq = 0; qq < NU; qq++) du_all[qq] = -du_all[qq];
                    }
                    float dz = 0.0f;
#pragma unroll
                    for (int qq = 0; qq < NU; qq++)
                        if (r == qq) dz = du_all[qq];
                    dz = is_x ? ((k >= 1) ? dxs : 0.0f) : dz;
                    dz = valid ? dz : 0.0f;
                    *it_wr(k, IT::DZ, live && lv) = dz;
                    if constexpr (kDinC) dterm(k, live, rc, dz);
                    if (k < N) dxs = dyn(rc, dz);
                };
                auto load = [&](int j, float (&v)[RS]) {
                    if constexpr (kDinC) {
                        // phase D's record fields [Z, UB] with C's Jacobian rows (one contiguous range)
                        static_assert(R::UB + 1 == R::GV && R::Z < R::GV, "D and C record fields contiguous");
                        const int k = kof(j);
                        ld_range<R::Z, R::GV + NGV, RS, QM>(tbase + (size_t)k * KS, v);
                        v[R::LR] = it_rd(k, IT::LR);
#pragma unroll
                        for (int qq = 0; qq < NU; qq++) v[R::LM + qq] = it_rd(k, IT::LM + qq);
                    } else {
                        ld_cfields(kof(j), v);
                    }
                };
                float ra[RS], rb[RS];
                load(0, ra);
                for (int j = 0;; j += 2) {
                    load(j + 1 <= Ls ? j + 1 : Ls, rb);
                    cseg(j, ra);
                    if (j == Ls) break;
                    load(j + 2 <= Ls ? j + 2 : Ls, ra);
                    cseg(j + 1, rb);
                    if (j + 1 == Ls) break;
                }
            }
            __syncthreads();  // the directions of every stage
        } else {
            // phase B (serial, N -> 0): adjoint, fp64 classic Riccati step, rhs / forward substitution
            double Lrow[NV];
    #pragma unroll
            for (int j = 0; j < NV; j++) Lrow[j] = 0.0;
            float pv = 0.0f, piv = 0.0f, res_stat = 0.0f, cpi_max = 0.0f;
            bool fail = false;
            if (!(nanf_ > 0.0f || mu != mu)) {
                serial(N, 0, -1, ld_bfields, [&](int k, float (&rc)[RS]) {
                    const bool vu = is_u && k < N;
                    const bool vx = is_x && k >= 1;
                    const bool valid = vu || vx;
                    float Gc[NX];
                    column(rc, Gc);
                    const float cpi = (k < N) ? dot_x<NX, NU>(0.0f, piv, Gc) : 0.0f;
                    const float base = rc[R::C0] + cpi;
                    res_stat = fmaxf(res_stat, vu ? fabsf(base) : 0.0f);
                    cpi_max = fmaxf(cpi_max, vu ? fabsf(cpi) : 0.0f);
                    const float sig = rc[R::SIG];
                    const float ghat = valid ? (vu ? rc[R::GH] + base : rc[R::GH]) : 0.0f;
                    const float pi_new = vx ? base : 0.0f;
                    if (ghat != ghat) nanf_ = 1.0f;
                    if (k == N) {
                        const double d = is_x ? (double)fmaxf(we_lane + sig, 0.0f) : 0.0;
    #pragma unroll
                        for (int j = 0; j < NV; j++) Lrow[j] = (is_x && j == r) ? d : 0.0;
                        pv = is_x ? ghat : 0.0f;
                    } else {
                        double Gd[NX];
    #pragma unroll
                        for (int l = 0; l < NX; l++) Gd[l] = (double)Gc[l];
                        double pg[NX];
    #pragma unroll
                        for (int i = 0; i < NX; i++) pg[i] = 0.0;
                        pg_block<NX, NU>(pg, Lrow, Gd);
                        const double dg = valid ? (double)h_stage + (double)sig : 1.0;
                        double Lr[NV];
    #pragma unroll
                        for (int j = 0; j < NV; j++) Lr[j] = (r == j) ? dg : 0.0;
                        double pivot;
#ifdef NMPC_ROWPAR_MCOL
                        double m11, m10;  // unused: pivots in turn below
                        m_block<M>(Lr, pivot, m11, m10, pg, Gd, gcs);
                        (void)m11;
                        (void)m10;
#else
                        mrow_pg_block<NX, NU>(Lr, pivot, pg, Gd);
#endif
                        sfor<0, NU>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            if (!(pivot > 0.0)) fail = true;
                            const double rd = drsq(fmax(pivot, 1e-300));
                            const double lj = (r >= j) ? Lr[j] * rd : 0.0;
                            Lr[j] = lj;
                            chol_update<NX, NU, j>(Lr, lj, pivot);
                        });
                        float Lm[NU];
    #pragma unroll
                        for (int qq = 0; qq < NU; qq++) {
                            Lm[qq] = (float)Lr[qq];
                            rc[R::LM + qq] = Lm[qq];
                        }
                        float y = dot_x<NX, NU>(ghat, pv, Gc);
                        float my_lr = 0.0f;
                        sfor<0, NU>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            const float lrj = bc<j>(y * frcp(Lm[j]));
                            if (r == j) my_lr = lrj;
                            y -= Lm[j] * lrj;
                        });
                        rc[R::LR] = my_lr;
                        pv = is_x ? y : 0.0f;
    #pragma unroll
                        for (int j = 0; j < NV; j++) Lrow[j] = Lr[j];
                        // LR, LM (wave 0's rows store the same values; the other waves and idle slots: pads)
                        st_lrlm(k, rc, lv && w0);
                    }
                    piv = pi_new;
                });
            }
            RP_STAMP(4 + 4 * it);
            res_stat = row_max16(lv ? res_stat : 0.0f);
            const float stat_scale = fmaxf(sc0, row_max16(lv ? cpi_max : 0.0f));
            nanf_ = row_max16(nanf_);
            const float failf = row_max16(fail ? 1.0f : 0.0f);
            // stopping rule of k_sqp_rti_team (DESIGN.md "Stopping rule")
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
                status = 4;
                stop = true;
            } else {
                const bool stat_ok = res_stat <= P.tol_stat || res_stat <= kStatRelT * stat_scale;
                const bool cmax_ok = max_c <= kCompMaxRatio * P.tol_comp;
                const bool stalled = mu <= P.tol_comp && mu > 0.5f * mu_prev;
                if (res_ineq <= P.tol_ineq &&
                    ((stat_ok && mu <= P.tol_comp && cmax_ok) || mu <= 1e-2f * P.tol_comp || (stalled && cmax_ok)))
                    stop = true;
                if (it >= P.iter_max) stop = true;
            }
            mu_prev = mu;
            if (stop) {
                it_done = it;
                break;
            }
            __syncthreads();  // LR / LM of every stage

            // phase C (serial, 0 -> N): the direction's input part from the stored factor, its state part from the
            // dynamics; every row the same (identical DZ stores)
            sigma_mu = tg_rhs;
            {
                float dxs = 0.0f;
                serial(0, N, 1, ld_cfields, [&](int k, float (&rc)[RS]) {
                    const bool vu = is_u && k < N;
                    const bool vx = is_x && k >= 1;
                    const bool valid = vu || vx;
                    float du_all[NU];
    #pragma unroll
                    for (int qq = 0; qq < NU; qq++) du_all[qq] = 0.0f;
                    if (k < N) {
                        float w[NU];
                        sfor<0, NU>([&](auto qc) {
                            constexpr int qq = decltype(qc)::value;
                            w[qq] = bc<qq>(rc[R::LR]) + ((k > 0) ? row_sum16(is_x ? rc[R::LM + qq] * dxs : 0.0f) : 0.0f);
                        });
                        sfor<0, NU>([&](auto qqc) {
                            constexpr int qq = NU - 1 - decltype(qqc)::value;
                            float sq = w[qq];
                            sfor<qq + 1, NU>([&](auto jc) {
                                constexpr int j = decltype(jc)::value;
                                sq -= bc<j>(rc[R::LM + qq]) * du_all[j];
                            });
                            du_all[qq] = sq * frcp(bc<qq>(rc[R::LM + qq]));
                        });
    #pragma unroll
                        for (int qq = 0; qq < NU; qq++) du_all[qq] = -du_all[qq];
                    }
                    float dz = 0.0f;
    #pragma unroll
                    for (int qq = 0; qq < NU; qq++)
                        if (r == qq) dz = du_all[qq];
                    dz = is_x ? ((k >= 1) ? dxs : 0.0f) : dz;
                    dz = valid ? dz : 0.0f;
                    *it_wr(k, IT::DZ, w0 && lv) = dz;
                    if (k < N) dxs = dyn(rc, dz);
                });
            }
            __syncthreads();  // the directions of every stage
            RP_STAMP(5 + 4 * it);
        }

        // phase D (stage-parallel unless accumulated in phase C): bound directions, fraction-to-boundary step bound,
        // complementarity polynomial, reduced over the block
        if constexpr (!kDinC) {
            spar(std::integral_constant<int, R::Z>{}, std::integral_constant<int, R::UB + 1>{},
                 [&](int j, float (&rc)[RS], float dz) {
                const int kr = j * ROWS + q;
                const bool kv = kr <= N;
                dterm(kv ? kr : N, kv, rc, dz);
            });
        }
        {
            float v[6] = {wave_min_rows(row_min16(lv ? amax : 1e30f)), wave_sum_rows(row_sum16(lv ? s1 : 0.0f)),
                          wave_sum_rows(row_sum16(lv ? s2 : 0.0f)), 0.0f, 0.0f, 0.0f};
            const int op[6] = {2, 0, 0, 0, 0, 0};
            block_combine(v, op, 3);
            amax = v[0];
            s1 = v[1];
            s2 = v[2];
        }
        alpha = fminf(1.0f, P.tau * amax);
        const float mu_next = fmaxf((sum_c + alpha * s1 + alpha * alpha * s2) * inv_m2, 0.0f);
        const float om = 1.0f - alpha;
        tg_rhs = fminf(fmaxf(om * om, P.sd_lo), P.sd_hi) * mu_next;
        RP_STAMP(6 + 4 * it);
    }

    // ---- full SQP step + outputs (row 0 stores; the other rows' entries point at the dummy record) -------------
    if (status == 0) {
        auto entry = [&](int k) -> float* {
            const int kk = k <= N ? k : N;
            return (w0 && is_x) ? &XB(kk, xi) : ((w0 && is_u && kk < N) ? &UBAR(kk, r) : tdummy);
        };
        constexpr int EC = 8;
        for (int k0 = 0; k0 <= N; k0 += EC) {
            float zs[EC], vs[EC];
#pragma unroll
            for (int j = 0; j < EC; j++) {
                const int kk = (k0 + j) <= N ? k0 + j : N;
                zs[j] = tbase[(size_t)kk * KS + rec_off<RS, QM>(R::Z)];
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
                if (wr && is_x && a.xtraj) a.xtraj[((size_t)k * NX + xi) * Bn + inst] = XB(k, xi);
                if (wr && is_u && k < N && a.utraj) a.utraj[((size_t)k * NU + r) * Bn + inst] = UBAR(k, r);
            }
        }
    }
    __threadfence_block();
    if (tid == 0) {
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
#pragma unroll
            for (int j = 0; j < 3; j++) a.cmd[(size_t)j * Bn + inst] = 0.0f;
        }
    }
    // ---- staged capsule output: device block -> host-mapped block once every output above is stored
    if (a.stage_out_n > 0) {
        __threadfence_block();
        __syncthreads();
        for (int e = tid; e < a.stage_out_n; e += 64 * W) a.stage_out_h[e] = a.stage_out_d[e];
    }
#undef XB
#undef UBAR
}

}  // namespace

template <class M>
size_t rowpar_lds_bytes(int N, int mode, int seg)
{
    (void)mode;
    return RowLds<M>::floats(N, seg) * sizeof(float);
}

template <class M>
hipError_t launch_sqp_rti_rowpar(const KParams& P, const KArgs& a, int mode, hipStream_t stream)
{
    if (a.B <= 0) return hipSuccess;
    const size_t lds = rowpar_lds_bytes<M>(P.N, mode, a.seg);
    if (lds > 163840 || P.ipm != 1 || a.segs) return hipErrorInvalidValue;  // (the host keeps every robot resident)
    // segments: N % S == 0, at most kSegMax and at most one per row of the block
    const int W = a.rowpar >= 4 ? 4 : (a.rowpar == 2 ? 2 : 1);
    if (a.seg < 0 || a.seg > kSegMax || a.seg > 4 * W || (a.seg > 0 && P.N % a.seg != 0))
        return hipErrorInvalidValue;
#ifdef NMPC_HYBRID
    const int grid = (a.hyb_role == 2) ? (a.B < a.hyb_cap ? a.B : a.hyb_cap) : a.B;
#else
    const int grid = a.B;
#endif
    // (a block above 64 KiB of LDS -- a long horizon on four waves, or omni4's wider stage fields -- asks for it)
    auto go = [&](auto kern, int threads) {
        if (lds > 65536) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, stream, P, a, mode);
        return hipGetLastError();
    };
    if (W == 4)  // four waves per robot (one per SIMD of its CU)
        return a.seg > 0 ? go(k_sqp_rti_rowpar<M, 4, true>, 256) : go(k_sqp_rti_rowpar<M, 4, false>, 256);
    if (W == 2 && a.seg > 0)  // two waves per robot above 256 robots (the default there)
        return go(k_sqp_rti_rowpar<M, 2, true>, 128);
    return a.seg > 0 ? go(k_sqp_rti_rowpar<M, 1, true>, 64) : go(k_sqp_rti_rowpar<M, 1, false>, 64);
}

#define INST(M)                                                                                                      \
    template hipError_t launch_sqp_rti_rowpar<M>(const KParams&, const KArgs&, int, hipStream_t);                   \
    template size_t rowpar_lds_bytes<M>(int, int, int);
INST(Diff2)
INST(Omni4)
INST(Tric3)
#undef INST

}  // namespace nmpc
