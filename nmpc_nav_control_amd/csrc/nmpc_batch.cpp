// nmpc_batch.cpp -- C ABI of the batched solve path (include/nmpc_amd/nmpc_batch.h).
#include "nmpc_amd/nmpc_batch.h"
#include "nmpc_amd/nmpc_path.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "nmpc_kernels.hpp"
#include "nmpc_trace.hpp"

using namespace nmpc;

struct nmpc_batch {
    nmpc_model_params prm;
    KParams kp;
    int capacity;
    int nx, nu, nbx, nbu, ny;
    float* xbar = nullptr;
    float* ubar = nullptr;
    float* carried = nullptr;
    float* scratch = nullptr;
    int sched = NMPC_SCHED_AUTO;
    int n_simd = 1024;           // SIMDs of the device (4 per CU)
    int n_cu = 256;              // CUs of the device and LDS bytes per CU (MI355X: 256, 160 KiB; read at create)
    size_t lds_per_cu = 163840;
    int split_max = 256;         // team-kernel launches of at most this many robots run one block per robot (split)
    // launches of at most this many robots (single-direction IPM, not run_path) run k_sqp_rti_rowpar (DESIGN.md
    // section 4): four waves per robot up to 256 robots; above, rowpar_w waves per robot and there only with
    // segments, all on the first wave's four rows (the second wave takes half of the stage-parallel phases; segments
    // on both waves of a SIMD's two resident waves contend: diff N = 40 B = 1024 1.15 M it/s on the team kernel ->
    // 1.57 M on one wave per robot -> 1.65 M on two, 1.52 M with 5 segments over both; profiles/r04/ab/seg.txt)
    int rowpar_max = 1024;
    int rowpar_w = 2;  // (NMPC_AMD_ROWPAR_W=1 for A/B)
    // horizon segments of the row-parallel kernel (sqp_rti_rowpar.hip SEG): -1 = chosen per launch (seg_count),
    // 0 = the serial phases B / C, S > 0 = S segments when N % S == 0 (NMPC_AMD_SEG overrides)
    int seg = -1;
    // rows that may hold a segment above 256 robots: the first wave's 4 (NMPC_AMD_SEG_ROWS = 8: both waves, A/B)
    int seg_rows = 4;
    int* iter_key = nullptr;     // [capacity] last executed IPM iterations per robot (written by the team kernel)
    int* order = nullptr;        // [capacity] team slot -> robot
    unsigned char* warm = nullptr;  // [capacity] the robot's last solve succeeded: its scratch records hold its
                                    // multipliers (IPM warm start)
    int* sorted = nullptr;       // [capacity] sort scratch
    // the team kernel's single-direction record layout (NMPC_REC_WIDE / NMPC_REC_SPLIT), fixed per handle: resolved
    // at create time from this handle alone and changed only by nmpc_batch_set_record_layout
    int rec_split = 0;
#ifdef NMPC_HYBRID
    // hybrid launch (A/B build only, -DNMPC_HYBRID, NMPC_AMD_HYBRID=H): in a team-kernel launch the robots whose last
    // IPM count was >= H (at most hybrid_cap of them, the hardest first) run the segmented row-parallel kernel (one
    // wave each) on aux, concurrently with the team kernel on the caller's stream for the rest (measured and not
    // adopted: metric 4.16 -> 3.84 M it/s at H = 12, DESIGN.md "Hybrid launch")
    int hybrid_h = 0, hybrid_cap = 1024;
    int* hyb_n = nullptr;        // [1] robots taken by the segmented part (device)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
#endif
};

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

int hip_err(hipError_t e, const char* what)
{
    if (e == hipSuccess) return NMPC_OK;
    return set_err(NMPC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

bool dims_of(int model, int* nx, int* nu, int* nbx, int* nbu, int* np)
{
    switch (model) {
    case NMPC_MODEL_DIFF2AMR: *nx = 7; *nu = 2; *nbx = 2; *nbu = 2; *np = 2; return true;
    case NMPC_MODEL_OMNI4AMR: *nx = 11; *nu = 4; *nbx = 4; *nbu = 4; *np = 2; return true;
    case NMPC_MODEL_TRIC3AMR: *nx = 7; *nu = 2; *nbx = 2; *nbu = 2; *np = 3; return true;
    default: return false;
    }
}

KParams to_kparams(const nmpc_model_params& p, int nx, int nu, int nbx, int nbu)
{
    KParams k;
    std::memset(&k, 0, sizeof(k));
    k.N = p.N;
    k.dt = (float)p.dt;
    k.dt_ctrl = (float)p.dt_ctrl;
    for (int i = 0; i < 3; i++) k.p[i] = (float)p.p[i];
    for (int i = 0; i < nbx; i++) { k.lbx[i] = (float)p.lbx[i]; k.ubx[i] = (float)p.ubx[i]; }
    for (int i = 0; i < nbu; i++) { k.lbu[i] = (float)p.lbu[i]; k.ubu[i] = (float)p.ubu[i]; }
    for (int i = 0; i < nx + nu; i++) k.W[i] = (float)p.W[i];
    for (int i = 0; i < nx; i++) k.We[i] = (float)p.W_e[i];
    k.terminal_hack = p.terminal_hack;
    k.sin_bug = p.tric_sin_bug;
    k.iter_max = p.qp_iter_max;
    k.tol_stat = (float)p.qp_tol_stat;
    k.tol_ineq = (float)p.qp_tol_ineq;
    k.tol_comp = (float)p.qp_tol_comp;
    k.mu0 = (float)p.qp_mu0;
    k.thr0 = (float)p.qp_thr0;
    k.tau = (float)p.qp_tau;
    k.ipm = p.qp_ipm;
    k.sd_lo = (float)p.qp_sigma_lo;
    k.sd_hi = (float)p.qp_sigma_hi;
    // same-box A/B overrides (tools/ab_env.py): the IPM rule and its sigma clamp
    if (const char* v = std::getenv("NMPC_AMD_IPM")) {  // single | mehrotra
        if (!std::strcmp(v, "single")) k.ipm = NMPC_IPM_SINGLE;
        else if (!std::strcmp(v, "mehrotra")) k.ipm = NMPC_IPM_MEHROTRA;
    }
    if (const char* v = std::getenv("NMPC_AMD_SIGMA_LO")) k.sd_lo = std::strtof(v, nullptr);
    if (const char* v = std::getenv("NMPC_AMD_SIGMA_HI")) k.sd_hi = std::strtof(v, nullptr);
    k.warm = p.qp_warm_start;
    k.warm_kappa = (float)p.qp_warm_kappa;
    if (const char* v = std::getenv("NMPC_AMD_WARM")) k.warm = std::atoi(v) != 0;
    if (const char* v = std::getenv("NMPC_AMD_WARM_KAPPA")) k.warm_kappa = std::strtof(v, nullptr);
    k.warm_iter_max = p.qp_warm_iter_max > 0 ? p.qp_warm_iter_max : p.qp_iter_max;
    if (const char* v = std::getenv("NMPC_AMD_WARM_ITER_MAX")) k.warm_iter_max = std::atoi(v);
    k.infeas_lam = p.qp_infeas_lambda > 0.0 ? (float)p.qp_infeas_lambda : INFINITY;
    k.wmax = 0.0f;
    for (int i = 0; i < nx + nu; i++) k.wmax = std::fmax(k.wmax, (float)p.W[i]);
    return k;
}

size_t scratch_floats(int model, int N, int stride)
{
    switch (model) {
    case NMPC_MODEL_DIFF2AMR: return team_scratch_floats<Diff2>(N, stride);
    case NMPC_MODEL_OMNI4AMR: return team_scratch_floats<Omni4>(N, stride);
    default: return team_scratch_floats<Tric3>(N, stride);
    }
}

template <class M>
hipError_t launch_m(nmpc_batch* b, const KArgs& a, int mode, hipStream_t s)
{
    if (a.rowpar) return launch_sqp_rti_rowpar<M>(b->kp, a, mode, s);
    if (a.stage_in_n > 0 || a.stage_out_n > 0) return hipErrorInvalidValue;  // (only the row-parallel kernel stages)
    return launch_sqp_rti_team<M>(b->kp, a, mode, s);
}

// Segments of the row-parallel kernel's Riccati sweeps for a horizon N on `rows` rows per robot: the divisor S of N
// (S <= rows, <= kSegMax) that minimises the robot's chain per IPM iteration, N / S stage steps of the segments'
// sweeps (backward 2.4 k + forward 1.2 k cycles) plus S - 1 master steps (5 k cycles, 1.4 stage steps; diag stamps,
// profiles/r04/stamps/); 0 (the serial phases) when no S > 1 divides N. N = 80 -> 8, N = 40 -> 5 (4 on one wave)
inline int seg_count(int N, int rows)
{
    int best = 0;
    double cost = (double)N;
    for (int S = 2; S <= rows && S <= kSegMax; S++) {
        if (N % S) continue;
        const double c = (double)N / S + 1.4 * (S - 1);
        if (c < cost) {
            cost = c;
            best = S;
        }
    }
    return best;
}

// waves per robot of a row-parallel launch of B robots (eight waves per robot up to 64 robots measured no faster:
// the one-robot phases are chains, not rounds; profiles/r05/ab/w8_rowchol2.txt)
inline int rowpar_waves(const nmpc_batch* b, int B)
{
    return B <= 256 ? 4 : b->rowpar_w;
}

// LDS a row-parallel launch of B robots may give each block: one CU's LDS shared by the ceil(B / CUs) robots each
// CU holds (one block per robot), so that every robot of the launch is resident at once. The CU count and the LDS
// per CU are the device's (hipDeviceProp_t at create: a CU-partitioned GPU has fewer CUs)
inline size_t rowpar_lds_cap(const nmpc_batch* b, int B)
{
    const int n_cu = b->n_cu > 0 ? b->n_cu : 1;
    const int per_cu = (B + n_cu - 1) / n_cu;
    return b->lds_per_cu / (size_t)(per_cu > 0 ? per_cu : 1);
}

template <class M>
bool rowpar_ok(const nmpc_batch* b, KArgs& a, int mode)
{
    if (b->kp.ipm != NMPC_IPM_SINGLE || a.segs || a.B > b->rowpar_max) return false;
    const int rows = a.B <= 256 ? 16 : b->seg_rows;  // segments: any row up to 256 robots, the first wave's above
    const size_t cap = rowpar_lds_cap(b, a.B);
    int S = b->seg >= 0 ? b->seg : seg_count(b->prm.N, rows);
    if (S > rows || S > kSegMax || (S > 0 && b->prm.N % S)) S = 0;
    if (S > 0 && rowpar_lds_bytes<M>(b->prm.N, mode, S) > cap) S = 0;
    if (a.B > 256 && S == 0 && b->seg < 0) return false;  // one wave per robot only with segments (auto)
    // above 256 robots two robots' waves share a SIMD, which needs <= 256 registers per lane: diff and tric's
    // segmented kernels take 246-250, omni4's (11 x 11 master blocks) 357 (tools/reg_usage.py), so omni4 keeps the
    // team kernel there
    if (a.B > 256 && M::NU == 4 && b->rowpar_max <= 1024) return false;
    a.seg = S;
    return rowpar_lds_bytes<M>(b->prm.N, mode, S) <= cap;
}

// Records one sweep of the team kernel touches over the handle's capacity in the wide layout (9 or 16 slots of
// 64 / 80 B per stage, plus the 64-B DZ plane entry): the measure of NMPC_REC_AUTO. diff takes the split planes when
// its own records exceed 3/4 of the 256 MB Infinity Cache. Alone on the device the metric fleet (4096 robots,
// 107 MB) keeps the wide records, 1.2 % faster there (issue-bound); a fleet beside other models (the mixed config)
// is set to SPLIT by its caller (fleet.py), where the split planes win 7 % (profiles/r04/ab/split.txt). The choice
// depends on this handle only, so no other handle can change it.
constexpr size_t kRecSplitBytes = (size_t)192 << 20;

size_t rec_footprint(const nmpc_batch* b)
{
    const size_t slots = b->prm.model == NMPC_MODEL_OMNI4AMR ? 16 : 9;  // omni4: quad-major, 16 slots of 80 B
    const size_t rec = b->prm.model == NMPC_MODEL_OMNI4AMR ? 80 : 64;
    return (size_t)b->capacity * (size_t)(b->prm.N + 1) * (slots * rec + 64);
}

int rec_layout_auto(const nmpc_batch* b)
{
    switch (b->prm.model) {
    case NMPC_MODEL_TRIC3AMR: return NMPC_REC_SPLIT;
    case NMPC_MODEL_OMNI4AMR: return NMPC_REC_WIDE;
    default: return rec_footprint(b) > kRecSplitBytes ? NMPC_REC_SPLIT : NMPC_REC_WIDE;
    }
}

// the warm-flag tag of a launch (NMPC_WARM_TAG_*): its multipliers' record layout and field order
int warm_tag_of(const nmpc_batch* b, const KArgs& a)
{
    if (b->kp.ipm != NMPC_IPM_SINGLE) return NMPC_WARM_TAG_MEHROTRA;
    return a.rec_split ? NMPC_WARM_TAG_SPLIT : NMPC_WARM_TAG_WIDE;
}

// Kernel choice, record layout and (team kernel) placement before a launch (schedule.hip); fills a.order /
// a.iter_key. Every robot's warm flag carries the tag of the layout its multipliers sit in, so a launch whose
// layout differs from a robot's last one starts that robot cold and leaves the others alone
hipError_t schedule(nmpc_batch* b, KArgs& a, int mode, hipStream_t s)
{
    a.iter_key = b->iter_key;
    a.warm = b->warm;
    switch (b->prm.model) {
    case NMPC_MODEL_DIFF2AMR: a.rowpar = rowpar_ok<Diff2>(b, a, mode); break;
    case NMPC_MODEL_OMNI4AMR: a.rowpar = rowpar_ok<Omni4>(b, a, mode); break;
    default: a.rowpar = rowpar_ok<Tric3>(b, a, mode); break;
    }
    if (a.rowpar) a.rowpar = rowpar_waves(b, a.B);  // waves per robot
    // the row-parallel kernel keeps the wide single-direction records; the team kernel the handle's layout
    a.rec_split = (!a.rowpar && b->kp.ipm == NMPC_IPM_SINGLE) ? b->rec_split : 0;
    a.warm_tag = warm_tag_of(b, a);
    if (a.rowpar) return hipSuccess;  // one robot per wave: nothing to place
    a.dense = ((a.B + 3) / 4 > b->n_simd) ? 1 : 0;  // 4 teams per wave
    // small batches leave most of the chip idle: one wave per robot, whose spare rows integrate P0's stages
    a.split = (!a.dense && a.B <= b->split_max) ? 1 : 0;
    if (a.split) return hipSuccess;  // one robot per wave: nothing to place
#ifdef NMPC_HYBRID
    // (the hybrid launch mixes the kernels in one tick: only where they share the record layout)
    if (b->hybrid_h > 0 && b->kp.ipm == NMPC_IPM_SINGLE && !a.segs && b->hyb_n && a.rec_split == 0) {
        a.hyb_role = 1;  // launch() adds the segmented part on the aux stream
        a.hyb_n = b->hyb_n;
        a.order = b->order;
        return launch_hybrid_order(b->iter_key, a.B, b->hybrid_h, b->hybrid_cap, b->order, b->hyb_n, s);
    }
#endif
    int layout = b->sched;
    if (layout == NMPC_SCHED_AUTO) layout = a.dense ? NMPC_SCHED_SORTED : NMPC_SCHED_OFF;
    if (layout == NMPC_SCHED_OFF) return hipSuccess;
    a.order = b->order;
    return launch_team_order(b->iter_key, a.B, layout, b->sorted, b->order, s);
}

#ifdef NMPC_HYBRID
template <class M>
hipError_t launch_hybrid(nmpc_batch* b, KArgs& a, int mode, hipStream_t s)
{
    // the segmented part: one wave per robot (4 rows, segments per seg_count), ranks [0, hyb_n) of the order
    KArgs g = a;
    g.hyb_role = 2;
    g.hyb_cap = b->hybrid_cap;
    g.rowpar = 1;
    g.seg = b->seg >= 0 ? b->seg : seg_count(b->prm.N, 4);
    if (g.seg > 4 || (g.seg > 0 && b->prm.N % g.seg)) g.seg = 0;
    if (rowpar_lds_bytes<M>(b->prm.N, mode, g.seg) > 65536) g.seg = 0;
    hipError_t e;
    if (!b->aux) {
        if ((e = hipStreamCreateWithFlags(&b->aux, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming)) != hipSuccess)
            return e;
    }
    if ((e = hipEventRecord(b->ev_fork, s)) != hipSuccess || (e = hipStreamWaitEvent(b->aux, b->ev_fork, 0)) != hipSuccess)
        return e;
    if ((e = launch_sqp_rti_rowpar<M>(b->kp, g, mode, b->aux)) != hipSuccess) return e;
    if ((e = launch_sqp_rti_team<M>(b->kp, a, mode, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(b->ev_join, b->aux)) != hipSuccess) return e;
    return hipStreamWaitEvent(s, b->ev_join, 0);
}
#endif

hipError_t launch(nmpc_batch* b, KArgs& a, int mode, hipStream_t s)
{
    const hipError_t e = schedule(b, a, mode, s);
    if (e != hipSuccess) return e;
#ifdef NMPC_HYBRID
    if (a.hyb_role == 1) {
        switch (b->prm.model) {
        case NMPC_MODEL_DIFF2AMR: return launch_hybrid<Diff2>(b, a, mode, s);
        case NMPC_MODEL_OMNI4AMR: return launch_hybrid<Omni4>(b, a, mode, s);
        default: return launch_hybrid<Tric3>(b, a, mode, s);
        }
    }
#endif
    switch (b->prm.model) {
    case NMPC_MODEL_DIFF2AMR: return launch_m<Diff2>(b, a, mode, s);
    case NMPC_MODEL_OMNI4AMR: return launch_m<Omni4>(b, a, mode, s);
    default: return launch_m<Tric3>(b, a, mode, s);
    }
}

__global__ void k_init_iterate(float* xbar, float* ubar, float* carried, unsigned char* warm, int B, int stride, int N,
                               int nx, int nu, int nbx, int mode)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    warm[i] = 0;  // the next solve starts its IPM cold
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx; j++)
            xbar[((size_t)k * nx + j) * stride + i] = (mode == 0 && j == 2) ? 3.14159265358979323846f : 0.0f;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu; j++) ubar[((size_t)k * nu + j) * stride + i] = 0.0f;
    // create semantics start the wrapper's x0 vel-refs at zero (the member struct is value-initialised); a reset
    // (reset_mpc -> {name}_acados_reset) leaves them, as the reference does and as the solve's reset mask does
    if (mode == 0)
        for (int j = 0; j < nbx; j++) carried[(size_t)j * stride + i] = 0.0f;
}

__global__ void k_forget_warm(unsigned char* warm, const unsigned char* mask, int B)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B && (!mask || mask[i])) warm[i] = 0;
}

int check_params(const nmpc_model_params* prm)
{
    int nx, nu, nbx, nbu, np;
    if (!prm) return set_err(NMPC_ERR_ARG, "params is NULL");
    if (!dims_of(prm->model, &nx, &nu, &nbx, &nbu, &np)) return set_err(NMPC_ERR_ARG, "unknown model id");
    if (prm->N < 1 || prm->N > 4096) return set_err(NMPC_ERR_ARG, "horizon N out of range [1, 4096]");
    if (!(prm->dt > 0.0) || !(prm->dt_ctrl > 0.0)) return set_err(NMPC_ERR_ARG, "dt must be positive");
    if (prm->qp_iter_max < 1) return set_err(NMPC_ERR_ARG, "qp_iter_max must be >= 1");
    if (prm->qp_ipm != NMPC_IPM_MEHROTRA && prm->qp_ipm != NMPC_IPM_SINGLE)
        return set_err(NMPC_ERR_ARG, "qp_ipm must be NMPC_IPM_MEHROTRA or NMPC_IPM_SINGLE");
    if (prm->qp_warm_start != 0 && prm->qp_warm_start != 1) return set_err(NMPC_ERR_ARG, "qp_warm_start must be 0 or 1");
    if (prm->qp_warm_start && !(prm->qp_warm_kappa > 0.0)) return set_err(NMPC_ERR_ARG, "qp_warm_kappa must be > 0");
    if (prm->qp_warm_iter_max < 0) return set_err(NMPC_ERR_ARG, "qp_warm_iter_max must be >= 0");
    if (!(prm->qp_infeas_lambda >= 0.0)) return set_err(NMPC_ERR_ARG, "qp_infeas_lambda must be >= 0 (0: off)");
    if (prm->qp_ipm == NMPC_IPM_SINGLE &&
        !(prm->qp_sigma_lo > 0.0 && prm->qp_sigma_lo <= prm->qp_sigma_hi && prm->qp_sigma_hi <= 1.0))
        return set_err(NMPC_ERR_ARG, "qp_sigma_lo / qp_sigma_hi need 0 < lo <= hi <= 1");
    for (int i = 0; i < nbx; i++)
        if (!(prm->lbx[i] < prm->ubx[i])) return set_err(NMPC_ERR_ARG, "state bounds need lbx < ubx");
    for (int i = 0; i < nbu; i++)
        if (!(prm->lbu[i] < prm->ubu[i])) return set_err(NMPC_ERR_ARG, "input bounds need lbu < ubu");
    for (int i = 0; i < np; i++)
        if (!(prm->p[i] > 0.0)) return set_err(NMPC_ERR_ARG, "model parameters must be positive");
    for (int i = 0; i < nu; i++)
        if (!(prm->W[nx + i] > 0.0)) return set_err(NMPC_ERR_UNSUPPORTED, "input weights R must be > 0");
    return NMPC_OK;
}

}  // namespace

extern "C" {

const char* nmpc_last_error(void) { return g_err.c_str(); }
#ifdef NMPC_HYBRID
const char* nmpc_version(void) { return "nmpc_amd 0.4 (team-per-instance DPP SQP-RTI, gfx950; A/B: hybrid launch)"; }
#else
const char* nmpc_version(void) { return "nmpc_amd 0.4 (team-per-instance DPP SQP-RTI, gfx950)"; }
#endif

int nmpc_model_dims(int model, int* nx, int* nu, int* ny, int* nbx, int* nbu, int* np)
{
    int a, b, c, d, e;
    if (!dims_of(model, &a, &b, &c, &d, &e)) return set_err(NMPC_ERR_ARG, "unknown model id");
    if (nx) *nx = a;
    if (nu) *nu = b;
    if (ny) *ny = a + b;
    if (nbx) *nbx = c;
    if (nbu) *nbu = d;
    if (np) *np = e;
    return NMPC_OK;
}

int nmpc_model_params_default(int model, int N, nmpc_model_params* prm)
{
    int nx, nu, nbx, nbu, np;
    if (!prm) return set_err(NMPC_ERR_ARG, "params is NULL");
    if (!dims_of(model, &nx, &nu, &nbx, &nbu, &np)) return set_err(NMPC_ERR_ARG, "unknown model id");
    std::memset(prm, 0, sizeof(*prm));
    prm->model = model;
    prm->N = N;
    prm->dt = 1.0 / 40.0;      // config/nmpc_nav_control_acados_models.yaml:28
    prm->dt_ctrl = 1.0 / 40.0; // config/nmpc_nav_control.yaml:4
    const double deg = M_PI / 180.0;
    // rob_wh_max_vel / rob_wh_max_ace 1.0 (nmpc_nav_control.yaml:20-21/31-32/44-45),
    // steering -45..45 deg, 15 deg/s (nmpc_nav_control.yaml:46-48)
    nmpc_model_params_set_limits(prm, 1.0, 1.0, -45.0 * deg, 45.0 * deg, 15.0 * deg);
    if (model == NMPC_MODEL_DIFF2AMR) {
        prm->p[0] = 0.270; prm->p[1] = 0.1;  // nmpc_nav_control.yaml:29-30
        const double W[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1};
        std::memcpy(prm->W, W, sizeof(W));
        prm->terminal_hack = 1;
    } else if (model == NMPC_MODEL_OMNI4AMR) {
        prm->p[0] = 0.265 + 0.270; prm->p[1] = 0.1;  // nmpc_nav_control.yaml:17-19, NMPCNavControlROS.cpp:97-99
        const double W[15] = {10, 10, 5, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1};
        std::memcpy(prm->W, W, sizeof(W));
    } else {
        prm->p[0] = 0.270; prm->p[1] = 0.1; prm->p[2] = 0.5;  // nmpc_nav_control.yaml:41-43
        const double W[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1};
        std::memcpy(prm->W, W, sizeof(W));
        prm->tric_sin_bug = 1;
    }
    for (int i = 0; i < nx; i++) prm->W_e[i] = prm->W[i];  // NMPCNavControlDiff.cpp:39-41
    prm->qp_iter_max = 50;
    prm->qp_tol_stat = 1e-4;
    prm->qp_tol_ineq = 1e-6;
    prm->qp_tol_comp = 1e-10;
    prm->qp_mu0 = 1.0;
    // initial slack floor t0 = max(z - lb, thr0): 0.25 instead of the oracle's 0.5 starts nearly active bounds
    // closer to their solution (steady-state closed loop: 8.0 -> 7.5 IPM iterations, 6 % faster ticks) while
    // the cold-start tail grows by at most 2 iterations (DESIGN.md "Algorithm and precision")
    prm->qp_thr0 = 0.25;
    prm->qp_tau = 0.995;
    // one direction per IPM iteration (P1 + one forward sweep) instead of Mehrotra's two (P1 + F0 + C1 + F1):
    // more, cheaper iterations; the slowest robot, which sets the kernel time, gets there sooner. Same-box A/B,
    // M it/s: diff N=40 B=4096 2.89 -> 3.24 (2 stream groups; 3.52 with one), B=1024 0.89 -> 1.00, tric 2.12 ->
    // 2.28, mixed 3.51 -> 3.64, omni4 2.45 -> 2.44 (profiles/r02/ab/ipm_single.txt)
    prm->qp_ipm = NMPC_IPM_SINGLE;
    prm->qp_sigma_lo = 0.01;
    prm->qp_sigma_hi = 0.5;
    // warm-started bound multipliers, floored at kappa / t: steady-state closed loop, emulator on 4096 robots of
    // real bench ticks: mean 10.9 -> 9.3 single-direction iterations, tail 22 -> 19 (DESIGN.md "Algorithm").
    // kappa per model from same-box A/B runs (profiles/r02/ab/warm.txt): diff 0.2 (as fast as 0.05, shorter
    // worst case: 29 against 39 iterations), omni4 and tric 0.01 (+7 % / +4 % against 0.05)
    prm->qp_warm_start = 1;
    prm->qp_warm_kappa = (model == NMPC_MODEL_DIFF2AMR) ? 0.2 : 0.01;
    // diff: warm start only after an easy solve. On 3 x 4096 stationary bench QPs (tools/warm_study.py, renewals
    // in the loop) warm after <= 12 iterations gives mean 8.78 / per-tick max 22, 21, 21 IPM iterations against
    // 8.60 / 30, 25, 27 for warm always and 9.38 / 22, 21, 21 for cold; same-box A/B (profiles/r03/ab/warm_iter.txt)
    // metric 3.00 -> 3.73 M it/s (cold 3.75, <= 10: 3.74, <= 16: 3.19), diff1024 0.87 -> 1.02 M. omni4 and tric
    // (kappa 0.01) lose with the rule (omni4 2.88 -> 2.47, tric 3.06 -> 2.82, mixed 4.52 -> 3.96 M): always warm
    prm->qp_warm_iter_max = (model == NMPC_MODEL_DIFF2AMR) ? 12 : 0;
    // early status-4 exit for infeasible QPs (a carried vel-ref far outside its bound): multipliers > 1e5 x the
    // weight scale with an open bound residual (tools/infeas_study.py: feasible bench QPs stay below 88)
    prm->qp_infeas_lambda = 1e5;
    return NMPC_OK;
}

int nmpc_model_params_set_limits(nmpc_model_params* prm, double v_max, double a_max, double alpha_min,
                                 double alpha_max, double dalpha_max)
{
    int nx, nu, nbx, nbu, np;
    if (!prm) return set_err(NMPC_ERR_ARG, "params is NULL");
    if (!dims_of(prm->model, &nx, &nu, &nbx, &nbu, &np)) return set_err(NMPC_ERR_ARG, "unknown model id");
    for (int i = 0; i < 4; i++) prm->lbx[i] = prm->ubx[i] = prm->lbu[i] = prm->ubu[i] = 0.0;
    for (int i = 0; i < nbx; i++) { prm->lbx[i] = -v_max; prm->ubx[i] = v_max; }
    for (int i = 0; i < nbu; i++) { prm->lbu[i] = -a_max; prm->ubu[i] = a_max; }
    if (prm->model == NMPC_MODEL_TRIC3AMR) {
        prm->lbx[1] = alpha_min;
        prm->ubx[1] = alpha_max;
        prm->lbu[1] = -dalpha_max;
        prm->ubu[1] = dalpha_max;
    }
    return NMPC_OK;
}

int nmpc_batch_create(const nmpc_model_params* prm, int capacity, nmpc_batch** out)
{
    if (!out) return set_err(NMPC_ERR_ARG, "out is NULL");
    *out = nullptr;
    int rc = check_params(prm);
    if (rc) return rc;
    if (capacity < 1) return set_err(NMPC_ERR_ARG, "capacity must be >= 1");
    nmpc_batch* b = new nmpc_batch();
    b->prm = *prm;
    b->capacity = capacity;
    int np;
    dims_of(prm->model, &b->nx, &b->nu, &b->nbx, &b->nbu, &np);
    b->ny = b->nx + b->nu;
    b->kp = to_kparams(*prm, b->nx, b->nu, b->nbx, b->nbu);
    if (const char* sv = std::getenv("NMPC_AMD_SCHED")) {  // off | auto | sorted | interleaved
        const char* names[5] = {"off", "auto", "sorted", "interleaved", "spread"};
        for (int i = 0; i < 5; i++)
            if (std::strcmp(sv, names[i]) == 0) b->sched = i;
    }
    if (const char* v = std::getenv("NMPC_AMD_SPLIT_MAX")) b->split_max = std::atoi(v);  // A/B: 0 = never split
    if (const char* v = std::getenv("NMPC_AMD_ROWPAR_MAX")) b->rowpar_max = std::atoi(v);  // A/B: 0 = never
    if (const char* v = std::getenv("NMPC_AMD_SEG")) b->seg = std::atoi(v);  // A/B: 0 = serial, S = S segments
    if (const char* v = std::getenv("NMPC_AMD_ROWPAR_W")) b->rowpar_w = std::atoi(v) == 1 ? 1 : 2;  // A/B
    if (const char* v = std::getenv("NMPC_AMD_SEG_ROWS")) b->seg_rows = std::atoi(v) == 8 ? 8 : 4;  // A/B
#ifdef NMPC_HYBRID
    if (const char* v = std::getenv("NMPC_AMD_HYBRID")) b->hybrid_h = std::atoi(v);  // A/B: 0 = off
    if (const char* v = std::getenv("NMPC_AMD_HYBRID_CAP")) b->hybrid_cap = std::atoi(v);
#endif
    const int N = prm->N;
    const size_t S = (size_t)capacity;
    hipError_t e;
    int dev = 0;
    hipDeviceProp_t props;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&props, dev) == hipSuccess &&
        props.multiProcessorCount > 0) {
        b->n_simd = 4 * props.multiProcessorCount;
        b->n_cu = props.multiProcessorCount;
        if (props.maxSharedMemoryPerMultiProcessor > 0) b->lds_per_cu = props.maxSharedMemoryPerMultiProcessor;
    }
#ifdef NMPC_HYBRID
    if ((e = hipMalloc(&b->hyb_n, sizeof(int))) != hipSuccess || (e = hipMemset(b->hyb_n, 0, sizeof(int))) != hipSuccess) {
        nmpc_batch_destroy(b);
        return hip_err(e, "hipMalloc");
    }
#endif
    if ((e = hipMalloc(&b->iter_key, sizeof(int) * S)) != hipSuccess ||
        (e = hipMalloc(&b->order, sizeof(int) * S)) != hipSuccess ||
        (e = hipMalloc(&b->sorted, sizeof(int) * S)) != hipSuccess ||
        (e = hipMemset(b->iter_key, 0, sizeof(int) * S)) != hipSuccess ||
        (e = hipMalloc(&b->warm, S)) != hipSuccess || (e = hipMemset(b->warm, 0, S)) != hipSuccess ||
        (e = hipMalloc(&b->xbar, sizeof(float) * (N + 1) * b->nx * S)) != hipSuccess ||
        (e = hipMalloc(&b->ubar, sizeof(float) * N * b->nu * S)) != hipSuccess ||
        (e = hipMalloc(&b->carried, sizeof(float) * b->nbx * S)) != hipSuccess ||
        (e = hipMalloc(&b->scratch, sizeof(float) * scratch_floats(prm->model, N, capacity))) != hipSuccess) {
        nmpc_batch_destroy(b);
        return hip_err(e, "hipMalloc");
    }
    rc = nmpc_batch_init_iterate(b, capacity, 0, nullptr);
    if (rc == NMPC_OK) rc = hip_err(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    if (rc) {
        nmpc_batch_destroy(b);
        return rc;
    }
    // the record layout: this handle's own choice (NMPC_REC_AUTO), fixed until nmpc_batch_set_record_layout
    b->rec_split = rec_layout_auto(b);
    if (const char* v = std::getenv("NMPC_AMD_REC_SPLIT"))  // A/B runs: 0 wide, 1 split (where the model has it)
        if (prm->model == NMPC_MODEL_DIFF2AMR) b->rec_split = std::atoi(v) ? NMPC_REC_SPLIT : NMPC_REC_WIDE;
    *out = b;
    return NMPC_OK;
}

int nmpc_batch_destroy(nmpc_batch* b)
{
    if (!b) return NMPC_OK;
    (void)hipFree(b->xbar);
    (void)hipFree(b->ubar);
    (void)hipFree(b->carried);
    (void)hipFree(b->scratch);
    (void)hipFree(b->iter_key);
    (void)hipFree(b->order);
    (void)hipFree(b->sorted);
    (void)hipFree(b->warm);
#ifdef NMPC_HYBRID
    (void)hipFree(b->hyb_n);
    if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
    if (b->ev_join) (void)hipEventDestroy(b->ev_join);
    if (b->aux) (void)hipStreamDestroy(b->aux);
#endif
    delete b;
    return NMPC_OK;
}

int nmpc_batch_set_params(nmpc_batch* b, const nmpc_model_params* prm)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    int rc = check_params(prm);
    if (rc) return rc;
    if (prm->model != b->prm.model || prm->N != b->prm.N)
        return set_err(NMPC_ERR_ARG, "set_params cannot change model or horizon");
    b->prm = *prm;
    b->kp = to_kparams(*prm, b->nx, b->nu, b->nbx, b->nbu);
    return NMPC_OK;
}

int nmpc_batch_get_params(const nmpc_batch* b, nmpc_model_params* prm)
{
    if (!b || !prm) return set_err(NMPC_ERR_ARG, "NULL argument");
    *prm = b->prm;
    return NMPC_OK;
}

int nmpc_batch_init_iterate(nmpc_batch* b, int B, int mode, void* stream)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (mode != 0 && mode != 1) return set_err(NMPC_ERR_ARG, "mode must be 0 (create) or 1 (reset)");
    if (B == 0) return NMPC_OK;
    hipLaunchKernelGGL(k_init_iterate, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->xbar, b->ubar,
                       b->carried, b->warm, B, b->capacity, b->prm.N, b->nx, b->nu, b->nbx, mode);
    return hip_err(hipGetLastError(), "init_iterate launch");
}

int nmpc_batch_solve(nmpc_batch* b, int B, const float* x0, const float* yref, int ny_in, const float* We,
                     const unsigned char* reset, float* u0, float* x1, float* xtraj, float* utraj, int* status,
                     int* qp_iter, float* qp_res, void* stream)
{
    const TraceRange trace("nmpc_batch_solve");
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (B == 0) return NMPC_OK;
    if (!x0 || !yref) return set_err(NMPC_ERR_ARG, "x0 and yref are required");
    if (ny_in < 1 || ny_in > b->ny) return set_err(NMPC_ERR_ARG, "ny_in out of range [1, NY]");
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = B;
    a.stride = b->capacity;
    a.sstride = b->capacity;
    a.xbar = b->xbar;
    a.ubar = b->ubar;
    a.carried = b->carried;
    a.scratch = b->scratch;
    a.x0 = x0;
    a.yref = yref;
    a.ny_in = ny_in;
    a.We = We;
    a.reset = reset;
    a.u0 = u0;
    a.x1 = x1;
    a.xtraj = xtraj;
    a.utraj = utraj;
    a.status = status;
    a.qp_iter = qp_iter;
    a.qp_res = qp_res;
    return hip_err(launch(b, a, kModeSolve, (hipStream_t)stream), "solve launch");
}

namespace {
int solve_iterate(nmpc_batch* b, int B, const float* x0, const float* yref, int ny_in, const float* We,
                  const unsigned char* reset, float* xbar, float* ubar, int ld, int* status, int* qp_iter,
                  float* qp_res, void* stream, const nmpc_stage_io* io)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (B == 0) return NMPC_OK;
    if (!x0 || !yref || !xbar || !ubar) return set_err(NMPC_ERR_ARG, "x0, yref, xbar and ubar are required");
    if (ld < B) return set_err(NMPC_ERR_ARG, "ld < B");
    if (ny_in < 1 || ny_in > b->ny) return set_err(NMPC_ERR_ARG, "ny_in out of range [1, NY]");
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = B;
    a.stride = ld;
    a.sstride = b->capacity;  // the scratch planes follow the allocation, not the caller's ld
    a.xbar = xbar;
    a.ubar = ubar;
    a.carried = b->carried;  // run mode only
    a.scratch = b->scratch;
    a.x0 = x0;
    a.yref = yref;
    a.ny_in = ny_in;
    a.We = We;
    a.reset = reset;
    a.status = status;
    a.qp_iter = qp_iter;
    a.qp_res = qp_res;
    if (io) {
        // one robot on the row-parallel kernel only (the team kernel does not stage)
        nmpc_launch_plan plan{};
        nmpc_batch_plan_ex(b, B, NMPC_PLAN_SOLVE, &plan);
        if (B != 1 || plan.kernel != 1)
            return set_err(NMPC_ERR_ARG, "staged I/O needs a one-robot row-parallel launch");
        a.stage_in_h = io->in_h;
        a.stage_in_d = io->in_d;
        a.stage_in_n = io->in_n;
        a.stage_out_h = io->out_h;
        a.stage_out_d = io->out_d;
        a.stage_out_n = io->out_n;
    }
    return hip_err(launch(b, a, kModeSolve, (hipStream_t)stream), "solve launch");
}
}  // namespace

int nmpc_batch_solve_iterate(nmpc_batch* b, int B, const float* x0, const float* yref, int ny_in, const float* We,
                             const unsigned char* reset, float* xbar, float* ubar, int ld, int* status, int* qp_iter,
                             float* qp_res, void* stream)
{
    const TraceRange trace("nmpc_batch_solve_iterate");
    return solve_iterate(b, B, x0, yref, ny_in, We, reset, xbar, ubar, ld, status, qp_iter, qp_res, stream, nullptr);
}

int nmpc_batch_solve_iterate_staged(nmpc_batch* b, const float* x0, const float* yref, int ny_in, const float* We,
                                    float* xbar, float* ubar, int* status, int* qp_iter, float* qp_res, void* stream,
                                    const nmpc_stage_io* io)
{
    const TraceRange trace("nmpc_batch_solve_iterate_staged");
    if (!io || !io->in_h || !io->in_d || !io->out_h || !io->out_d || io->in_n < 0 || io->out_n < 0)
        return set_err(NMPC_ERR_ARG, "staged I/O: host and device blocks are required");
    return solve_iterate(b, 1, x0, yref, ny_in, We, nullptr, xbar, ubar, 1, status, qp_iter, qp_res, stream, io);
}

int nmpc_batch_run(nmpc_batch* b, int B, const float* pose, const float* vel, const float* steer,
                   const float* traj, const int* traj_len, const unsigned char* reset, float* cmd, float* u0,
                   int* status, int* qp_iter, float* qp_res, void* stream)
{
    const TraceRange trace("nmpc_batch_run");
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (B == 0) return NMPC_OK;
    if (!pose || !vel || !traj) return set_err(NMPC_ERR_ARG, "pose, vel and traj are required");
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = B;
    a.stride = b->capacity;
    a.sstride = b->capacity;
    a.xbar = b->xbar;
    a.ubar = b->ubar;
    a.carried = b->carried;
    a.scratch = b->scratch;
    a.pose = pose;
    a.vel = vel;
    a.steer = steer;
    a.traj = traj;
    a.traj_len = traj_len;
    a.reset = reset;
    a.cmd = cmd;
    a.u0 = u0;
    a.status = status;
    a.qp_iter = qp_iter;
    a.qp_res = qp_res;
    return hip_err(launch(b, a, kModeRun, (hipStream_t)stream), "run launch");
}

int nmpc_batch_run_path(nmpc_batch* b, int B, const float* pose, const float* vel, const float* steer,
                        const nmpc_path_segment* segs, int seg_stride, const int* nseg, const double* nearest_u,
                        double sample_period, int is_holonomic, const unsigned char* reset, float* traj_out,
                        float* cmd, float* u0, int* status, int* qp_iter, float* qp_res, void* stream)
{
    const TraceRange trace("nmpc_batch_run_path");
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (B == 0) return NMPC_OK;
    if (!pose || !vel || !segs || !nseg || !nearest_u)
        return set_err(NMPC_ERR_ARG, "pose, vel, segs, nseg and nearest_u are required");
    if (seg_stride < 1) return set_err(NMPC_ERR_ARG, "seg_stride < 1");
    if (!(sample_period >= 0.0)) return set_err(NMPC_ERR_ARG, "sample_period must be >= 0");
    if (16 * (sizeof(double) + 3 * sizeof(float)) * (size_t)(b->prm.N + 1) > 65536)
        return set_err(NMPC_ERR_UNSUPPORTED, "horizon too long for the in-kernel path march");
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = B;
    a.stride = b->capacity;
    a.sstride = b->capacity;
    a.xbar = b->xbar;
    a.ubar = b->ubar;
    a.carried = b->carried;
    a.scratch = b->scratch;
    a.pose = pose;
    a.vel = vel;
    a.steer = steer;
    a.segs = segs;
    a.seg_stride = seg_stride;
    a.nseg = nseg;
    a.nearest_u = nearest_u;
    a.period = sample_period;
    a.holo = is_holonomic ? 1 : 0;
    a.traj_out = traj_out;
    a.reset = reset;
    a.cmd = cmd;
    a.u0 = u0;
    a.status = status;
    a.qp_iter = qp_iter;
    a.qp_res = qp_res;
    return hip_err(launch(b, a, kModeRun, (hipStream_t)stream), "run_path launch");
}

int nmpc_batch_set_kernel(nmpc_batch* b, int kernel)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (kernel != NMPC_KERNEL_TEAM) return set_err(NMPC_ERR_UNSUPPORTED, "unknown kernel (only NMPC_KERNEL_TEAM)");
    return NMPC_OK;
}

int nmpc_batch_set_schedule(nmpc_batch* b, int mode)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (mode < NMPC_SCHED_OFF || mode > NMPC_SCHED_SPREAD) return set_err(NMPC_ERR_ARG, "unknown schedule");
    b->sched = mode;
    return NMPC_OK;
}

int nmpc_batch_state(nmpc_batch* b, float** xbar, float** ubar, float** carried, int* stride)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (xbar) *xbar = b->xbar;
    if (ubar) *ubar = b->ubar;
    if (carried) *carried = b->carried;
    if (stride) *stride = b->capacity;
    return NMPC_OK;
}

int nmpc_batch_forget_warm(nmpc_batch* b, int B, const unsigned char* mask, void* stream)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (B == 0) return NMPC_OK;
    hipLaunchKernelGGL(k_forget_warm, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->warm, mask, B);
    return hip_err(hipGetLastError(), "forget_warm launch");
}

int nmpc_batch_set_record_layout(nmpc_batch* b, int layout)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (layout != NMPC_REC_AUTO && layout != NMPC_REC_WIDE && layout != NMPC_REC_SPLIT)
        return set_err(NMPC_ERR_ARG, "layout must be NMPC_REC_AUTO, NMPC_REC_WIDE or NMPC_REC_SPLIT");
    const int want = layout == NMPC_REC_AUTO ? rec_layout_auto(b) : layout;
    if ((b->prm.model == NMPC_MODEL_TRIC3AMR && want != NMPC_REC_SPLIT) ||
        (b->prm.model == NMPC_MODEL_OMNI4AMR && want != NMPC_REC_WIDE))
        return set_err(NMPC_ERR_UNSUPPORTED, "this model's team kernel has one record layout (tric split, omni4 wide)");
    b->rec_split = want;  // robots warm-started in the other layout start cold at their next solve (warm tags)
    return NMPC_OK;
}

int nmpc_batch_plan_ex(const nmpc_batch* b, int B, int mode, nmpc_launch_plan* plan)
{
    if (!b || !plan) return set_err(NMPC_ERR_ARG, "NULL argument");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range");
    if (mode != NMPC_PLAN_SOLVE && mode != NMPC_PLAN_RUN && mode != NMPC_PLAN_RUN_PATH)
        return set_err(NMPC_ERR_ARG, "mode must be NMPC_PLAN_SOLVE, NMPC_PLAN_RUN or NMPC_PLAN_RUN_PATH");
    KArgs a{};
    a.B = B;
    // run_path launches carry the path segments (a.segs), which keep them on the team kernel
    static const nmpc_path_segment kSeg{};
    if (mode == NMPC_PLAN_RUN_PATH) a.segs = &kSeg;
    const int km = mode == NMPC_PLAN_SOLVE ? kModeSolve : kModeRun;
    bool rp;
    switch (b->prm.model) {
    case NMPC_MODEL_DIFF2AMR: rp = rowpar_ok<Diff2>(b, a, km); break;
    case NMPC_MODEL_OMNI4AMR: rp = rowpar_ok<Omni4>(b, a, km); break;
    default: rp = rowpar_ok<Tric3>(b, a, km); break;
    }
    a.rowpar = rp ? 1 : 0;
    a.rec_split = (!rp && b->kp.ipm == NMPC_IPM_SINGLE) ? b->rec_split : 0;
    plan->kernel = rp ? 1 : 0;
    plan->waves_per_robot = rp ? rowpar_waves(b, B) : 0;
    plan->segments = rp ? a.seg : 0;
    plan->record_layout = a.rec_split ? NMPC_REC_SPLIT : NMPC_REC_WIDE;
    plan->warm_tag = warm_tag_of(b, a);
    plan->record_bytes = rec_footprint(b);
    return NMPC_OK;
}

int nmpc_batch_plan(const nmpc_batch* b, int B, int* kernel, int* waves_per_robot, int* segments)
{
    nmpc_launch_plan p;
    const int rc = nmpc_batch_plan_ex(b, B, NMPC_PLAN_SOLVE, &p);
    if (rc) return rc;
    if (kernel) *kernel = p.kernel;
    if (waves_per_robot) *waves_per_robot = p.waves_per_robot;
    if (segments) *segments = p.segments;
    return NMPC_OK;
}

int nmpc_batch_warm_rule(const nmpc_batch* b, int* warm, int* warm_iter_max, int* iter_max)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (warm) *warm = b->kp.warm ? 1 : 0;
    if (warm_iter_max) *warm_iter_max = b->kp.warm_iter_max;
    if (iter_max) *iter_max = b->kp.iter_max;
    return NMPC_OK;
}

int nmpc_batch_warm_state(nmpc_batch* b, unsigned char** warm, float** scratch, size_t* scratch_bytes)
{
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (warm) *warm = b->warm;
    if (scratch) *scratch = b->scratch;
    if (scratch_bytes) *scratch_bytes = sizeof(float) * scratch_floats(b->prm.model, b->prm.N, b->capacity);
    return NMPC_OK;
}

namespace {
int fleet_sim(nmpc_batch* b, int B, float* path, float* s, float* pose, float* vel, float* steer, const float* u0,
              const int* status, float* traj, int* traj_len, int advance, const nmpc_fleet_renew* renew, void* stream)
{
    const TraceRange trace("nmpc_fleet_sim_step");
    if (!b) return set_err(NMPC_ERR_ARG, "batch is NULL");
    if (B < 0 || B > b->capacity) return set_err(NMPC_ERR_ARG, "B out of range [0, capacity]");
    if (!path || !s || !pose || !vel || !traj || (advance && !u0)) return set_err(NMPC_ERR_ARG, "NULL argument");
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    switch (b->prm.model) {
    case NMPC_MODEL_DIFF2AMR:
        e = launch_fleet_sim<Diff2>(b->kp, B, b->capacity, path, s, pose, vel, steer, u0, status, b->carried, traj,
                                    traj_len, advance, renew, st);
        break;
    case NMPC_MODEL_OMNI4AMR:
        e = launch_fleet_sim<Omni4>(b->kp, B, b->capacity, path, s, pose, vel, steer, u0, status, b->carried, traj,
                                    traj_len, advance, renew, st);
        break;
    default:
        e = launch_fleet_sim<Tric3>(b->kp, B, b->capacity, path, s, pose, vel, steer, u0, status, b->carried, traj,
                                    traj_len, advance, renew, st);
        break;
    }
    return hip_err(e, "fleet_sim launch");
}
}  // namespace

int nmpc_fleet_sim_step(nmpc_batch* b, int B, const float* path, float* s, float* pose, float* vel, float* steer,
                        const float* u0, const int* status, float* traj, int* traj_len, int advance, void* stream)
{
    // without a renewal record the kernel never writes `path`
    return fleet_sim(b, B, const_cast<float*>(path), s, pose, vel, steer, u0, status, traj, traj_len, advance,
                     nullptr, stream);
}

int nmpc_fleet_sim_step_renew(nmpc_batch* b, int B, float* path, float* s, float* pose, float* vel, float* steer,
                              const float* u0, const int* status, float* traj, int* traj_len,
                              const nmpc_fleet_renew* renew, void* stream)
{
    if (!renew || !renew->ev || !renew->ttl || !renew->reset) return set_err(NMPC_ERR_ARG, "renew: NULL argument");
    if (renew->ttl_min < 1 || renew->ttl_max < renew->ttl_min) return set_err(NMPC_ERR_ARG, "renew: ttl range");
    if (const nmpc_fleet_stats* st = renew->stats)
        if (!st->qp_iter || !st->iters_sum || !st->iters_max || !st->fail_cnt || !st->hist || !st->cold_cnt ||
            !st->cold_iters || !status)
            return set_err(NMPC_ERR_ARG, "renew: stats needs every pointer and status");
    return fleet_sim(b, B, path, s, pose, vel, steer, u0, status, traj, traj_len, 1, renew, stream);
}

int nmpc_path_discretize(int B, const nmpc_path_segment* segs, int seg_stride, const int* nseg,
                         const double* nearest_u, double sample_period, int num_poses, int is_holonomic,
                         float* traj, double* traj64, void* stream)
{
    if (B < 0) return set_err(NMPC_ERR_ARG, "B < 0");
    if (B == 0) return NMPC_OK;
    if (!segs || !nseg || !nearest_u) return set_err(NMPC_ERR_ARG, "segs, nseg and nearest_u are required");
    if (seg_stride < 1) return set_err(NMPC_ERR_ARG, "seg_stride < 1");
    if (num_poses < 1 || num_poses > 8192) return set_err(NMPC_ERR_ARG, "num_poses out of range [1, 8192]");
    if (!(sample_period >= 0.0)) return set_err(NMPC_ERR_ARG, "sample_period must be >= 0");
    return hip_err(launch_path_discretize(B, segs, seg_stride, nseg, nearest_u, sample_period, num_poses,
                                          is_holonomic ? 1 : 0, traj, traj64, (hipStream_t)stream),
                   "path_discretize launch");
}

}  // extern "C"
