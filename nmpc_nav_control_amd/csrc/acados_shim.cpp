// acados_shim.cpp -- the acados-generated per-model solver ABI and the generic ocp_nlp_* setters/getters
// the reference's wrappers call, implemented on the batched MI355X solve path.
//
// Reference call sites (src/nmpc_nav_control/NMPCNavControlDiff.cpp; Omni4/Tric identical in shape):
//   create_capsule/create :10-12, update_params :44-46, constraints_model_set :49-65/:96-101,
//   cost_model_set :68-73/:121-124/:138, solve :142, nlp_out->inf_norm_res :146, ocp_nlp_get time_tot :148,
//   ocp_nlp_out_get u/x :151/:168, reset :179, free/free_capsule :78-79.
//
// A capsule keeps the acados "nlp_in" data (per-stage bounds, weights, references, parameters) and the
// warm-start iterate ("nlp_out") on the host in fp64, as the wrappers set them. solve() packs them into a
// batch of one (batch_solve() into one batch per parameter group), runs the fp32 SQP-RTI kernel and
// copies the new iterate back. Device engines are shared per (model, N) and grow on demand.
#include <hip/hip_runtime.h>

#include "nmpc_trace.hpp"
using nmpc::TraceRange;

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "nmpc_amd/nmpc_batch.h"
#include "nmpc_amd/nmpc_capsule.h"
#include "nmpc_kernels.hpp"  // nmpc_batch_solve_iterate_staged (library-internal)

struct nmpc_capsule_impl {
    int model = 0, N = 0;
    int nx = 0, nu = 0, ny = 0, nbx = 0, nbu = 0, np = 0;
    bool created = false;
    nmpc_model_params prm;           // codegen defaults + QP options
    std::vector<double> W;           // (N+1) * NY*NY col-major (stage N uses the leading NX*NX)
    std::vector<double> yref;        // (N+1) * NY (stage N uses NX)
    std::vector<double> lbx, ubx;    // (N+1) * NX: stage 0 all NX (x0 equality), stages 1..N the NBX first
    std::vector<double> lbu, ubu;    // N * NBU
    std::vector<double> p;           // (N+1) * NP
    std::vector<double> xbar, ubar;  // iterate (N+1)*NX, N*NU
    // validation cache of the stage-uniform data (W, W_e, bounds of stages >= 1, inputs, p): the wrappers set
    // them once in their constructors and only x0 and yref per tick, so solve() re-checks them only after a
    // setter touched them
    bool uniform_dirty = true, uniform_ok = false;
    std::string uniform_why;
    nmpc_model_params uniform_prm;
    std::vector<double> uniform_We;
    double time_tot = 0.0, time_lin = 0.0, time_qp = 0.0;
    int status = 5, qp_iter = 0, sqp_iter = 0;  // ACADOS_READY before the first solve
    // IPM warm start: the capsule's bound multipliers stay in the engine slot of its last solve; they are used
    // while the capsule still owns that slot, its last solve succeeded and no reset/create came in between
    std::uint64_t uid = 0;
    bool warm_ok = false;
    unsigned char warm_tag = 0;  // the record layout tag of the launch that left them (NMPC_WARM_TAG_*)
    ocp_nlp_config config;
    ocp_nlp_dims dims;
    ocp_nlp_in in;
    ocp_nlp_out out;
    ocp_nlp_solver solver;
};

namespace {

std::mutex g_mu;
std::atomic<std::uint64_t> g_next_uid{1};

// Device engine per (model, N): one batch handle plus one I/O block, on the device and pinned on the host. A call
// with n capsules packs its inputs densely ([row][n] per array) into the host block, which goes to the device in ONE
// copy; the kernel reads the iterate from the block and overwrites it with the new one in place
// (nmpc_batch_solve_iterate), next to its status / qp_iter / residual outputs, so that ONE copy brings everything
// back. Every copy is async on the launch stream and the call synchronises once.
struct Blocks {  // float offsets of the arrays inside the I/O block for n capsules
    size_t x0, We, yref, xb, ub, in_floats;  // host -> device: [0, in_floats)
    size_t ores, ost, oit, io_words;         // device -> host: [xb, io_words) (status / qp_iter are int32 words)
    Blocks(int n, int N, int nx, int nu, int ny)
    {
        x0 = 0;
        We = x0 + (size_t)nx * n;
        yref = We + (size_t)nx * n;
        xb = yref + (size_t)(N + 1) * ny * n;
        ub = xb + (size_t)(N + 1) * nx * n;
        in_floats = ub + (size_t)N * nu * n;
        ores = in_floats;
        ost = ores + (size_t)3 * n;
        oit = ost + (size_t)n;
        io_words = oit + (size_t)n;
    }
};
// Slot q of an engine keeps the scratch records (and so the bound multipliers) of the capsule that last solved
// in it. owner[q] names that capsule; dev_warm[q] mirrors the handle's device warm flag of slot q (the launch's
// NMPC_WARM_TAG_* after a successful solve, which is what the kernel leaves; kWarmUnknown = unknown), so the flags
// only travel to the device when a slot changes hands or a capsule was reset. A capsule keeps the tag of the launch
// that stored its multipliers: if its next launch takes another kernel or layout (e.g. the group grows past the
// row-parallel kernel's limit), the kernel sees the mismatch and starts that capsule cold.
constexpr unsigned char kWarmUnknown = 0xff;
struct Engine {
    nmpc_batch* batch = nullptr;
    int cap = 0;
    float *dio = nullptr, *hio = nullptr;  // the device I/O block, sized for cap capsules, and its pinned twin
    float* hio_dev = nullptr;  // hio as the device addresses it (staged one-capsule solves)
    unsigned char *dwarm = nullptr, *hwarm = nullptr;  // the handle's warm flags; pinned staging for them
    std::vector<std::uint64_t> owner;
    std::vector<unsigned char> dev_warm;
    ~Engine() { release(); }
    void release()
    {
        nmpc_batch_destroy(batch);
        batch = nullptr;
        (void)hipFree(dio); (void)hipHostFree(hio); (void)hipHostFree(hwarm);
        dio = hio = hio_dev = nullptr;
        dwarm = hwarm = nullptr;
        owner.clear();
        dev_warm.clear();
        cap = 0;
    }
};
std::map<std::pair<int, int>, std::unique_ptr<Engine>> g_engines;

void log_err(const char* what, const std::string& msg) { std::fprintf(stderr, "[nmpc_amd] %s: %s\n", what, msg.c_str()); }

// A stage index past the capsule's horizon is a caller error (e.g. a wrapper compiled against another {NAME}_N):
// log it, the caller gets -1 / 1 (acados would write out of bounds)
bool stage_ok(const nmpc_capsule_impl* c, int stage, const char* what, const char* field)
{
    if (stage >= 0 && stage <= c->N) return true;
    log_err(what, std::string(field) + ": stage " + std::to_string(stage) + " outside 0.." + std::to_string(c->N));
    return false;
}

void stage_W_diag(nmpc_capsule_impl* c, int k, const double* d, int n)
{
    double* W = c->W.data() + (size_t)k * c->ny * c->ny;
    std::fill(W, W + c->ny * c->ny, 0.0);
    for (int i = 0; i < n; i++) W[i + n * i] = d[i];
}

// Values scripts/*/generate_c_code.py bakes into the generated solver, here from a codegen descriptor
// (nmpc_codegen_default: the shipped config/nmpc_nav_control_acados_models.yaml); the wrappers overwrite p,
// bounds and W at construction time (e.g. NMPCNavControlDiff.cpp:16-73).
void codegen_defaults(nmpc_capsule_impl* c, const nmpc_codegen_desc& d)
{
    nmpc_model_params_default(c->model, c->N, &c->prm);
    c->prm.terminal_hack = 0;  // the wrappers apply it themselves through cost_model_set(N, "W")
    // a capsule is one robot whose latency is its own IPM count, so its warm start floors the multipliers for the
    // mean count (kappa 0.01; the batch default for diff, 0.2, is tuned for the slowest robot of a fleet)
    c->prm.qp_warm_kappa = 0.01;
    // acados' default, which the reference's OCP keeps (scripts/diff/generate_c_code.py:68-74 sets no
    // qp_warm_start): HPIPM starts every QP cold. ocp_nlp_solver_opts_set(.., "qp_warm_start", 2) opts in to the
    // capsule's multiplier warm start (INTEGRATION.md "Capsule semantics"; 1, acados' primal-only warm start, starts
    // cold here)
    c->prm.qp_warm_start = 0;
    // HPIPM has no infeasibility exit: a hard QP runs to qp_iter_max and acados' RTI accepts the result
    // (SURVEY Appendix B.6), so the drop-in never turns a stiff but feasible QP into the wrapper's exception
    c->prm.qp_infeas_lambda = 0.0;
    c->prm.dt = d.tf / d.N;    // uniform time steps tf / N_codegen (ocp.solver_options.tf, N_horizon)
    std::memcpy(c->prm.p, d.p, sizeof(d.p));
    std::memcpy(c->prm.lbx, d.lbx, sizeof(d.lbx));
    std::memcpy(c->prm.ubx, d.ubx, sizeof(d.ubx));
    std::memcpy(c->prm.lbu, d.lbu, sizeof(d.lbu));
    std::memcpy(c->prm.ubu, d.ubu, sizeof(d.ubu));
    const int N = c->N, nx = c->nx, nu = c->nu, ny = c->ny;
    c->W.assign((size_t)(N + 1) * ny * ny, 0.0);
    for (int k = 0; k < N; k++) stage_W_diag(c, k, d.W, ny);
    stage_W_diag(c, N, d.W_e, nx);
    c->yref.assign((size_t)(N + 1) * ny, 0.0);
    c->lbx.assign((size_t)(N + 1) * nx, 0.0);
    c->ubx.assign((size_t)(N + 1) * nx, 0.0);
    // ocp.constraints.x0 = [0, 0, pi, 0, ...] (generate_c_code.py:58-60)
    c->lbx[2] = c->ubx[2] = M_PI;
    for (int k = 1; k <= N; k++)
        for (int i = 0; i < c->nbx; i++) {
            c->lbx[(size_t)k * nx + i] = c->prm.lbx[i];
            c->ubx[(size_t)k * nx + i] = c->prm.ubx[i];
        }
    c->lbu.assign((size_t)N * c->nbu, 0.0);
    c->ubu.assign((size_t)N * c->nbu, 0.0);
    for (int k = 0; k < N; k++)
        for (int i = 0; i < c->nbu; i++) {
            c->lbu[(size_t)k * c->nbu + i] = c->prm.lbu[i];
            c->ubu[(size_t)k * c->nbu + i] = c->prm.ubu[i];
        }
    c->p.assign((size_t)(N + 1) * c->np, 0.0);
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < c->np; i++) c->p[(size_t)k * c->np + i] = c->prm.p[i];
    // iterate after create: x = x0 of the codegen, u = 0
    c->xbar.assign((size_t)(N + 1) * nx, 0.0);
    c->ubar.assign((size_t)N * nu, 0.0);
    for (int k = 0; k <= N; k++) c->xbar[(size_t)k * nx + 2] = M_PI;
}

nmpc_capsule_impl* new_impl(int model)
{
    nmpc_capsule_impl* c = new nmpc_capsule_impl();
    c->model = model;
    nmpc_model_dims(model, &c->nx, &c->nu, &c->ny, &c->nbx, &c->nbu, &c->np);
    c->config.impl = c;
    c->dims.impl = c;
    c->in.impl = c;
    c->out.impl = c;
    c->out.inf_norm_res = 0.0;
    c->out.total_cost = 0.0;
    c->out.sqp_iter = 0;
    c->solver.impl = c;
    c->uid = g_next_uid++;
    return c;
}

int impl_create(nmpc_capsule_impl* c, int N, const nmpc_codegen_desc& d)
{
    if (N < 1) return 1;
    c->N = N;
    codegen_defaults(c, d);
    c->dims.N = N;
    c->dims.nx = c->nx;
    c->dims.nu = c->nu;
    c->dims.ny = c->ny;
    c->dims.nyn = c->nx;
    c->dims.nbx = c->nbx;
    c->dims.nbu = c->nbu;
    c->dims.np = c->np;
    c->created = true;
    c->uniform_dirty = true;
    c->status = 5;
    c->warm_ok = false;
    return 0;
}

// Per-capsule packed solve input; returns false (with a message) if the capsule uses a feature the
// batched kernel does not implement.
struct Packed {
    nmpc_model_params prm;
    const double* x0 = nullptr;    // stage-0 lbx (= ubx)
    const double* yref = nullptr;  // (N+1) * NY
    const double* We = nullptr;    // NX
};

// Stage-uniform data -> kernel parameters (validated: diagonal W identical on stages 0..N-1, diagonal W_e,
// bounds and parameters identical on their stages)
bool validate_uniform(nmpc_capsule_impl* c, std::string& why)
{
    const int N = c->N, nx = c->nx, ny = c->ny;
    nmpc_model_params& prm = c->uniform_prm;
    prm = c->prm;
    const double* W0 = c->W.data();
    for (int k = 0; k < N; k++) {
        const double* Wk = c->W.data() + (size_t)k * ny * ny;
        for (int j = 0; j < ny; j++)
            for (int i = 0; i < ny; i++) {
                if (i != j && Wk[i + ny * j] != 0.0) { why = "non-diagonal W"; return false; }
                if (Wk[i + ny * j] != W0[i + ny * j]) { why = "stage-varying W"; return false; }
            }
    }
    for (int i = 0; i < ny; i++) prm.W[i] = W0[i + ny * i];
    const double* WN = c->W.data() + (size_t)N * ny * ny;
    c->uniform_We.resize(nx);
    for (int j = 0; j < nx; j++)
        for (int i = 0; i < nx; i++) {
            if (i != j && WN[i + nx * j] != 0.0) { why = "non-diagonal W_e"; return false; }
            if (i == j) c->uniform_We[i] = WN[i + nx * i];
        }
    for (int i = 0; i < c->nbx; i++) {
        prm.lbx[i] = c->lbx[(size_t)nx + i];
        prm.ubx[i] = c->ubx[(size_t)nx + i];
        for (int k = 2; k <= N; k++)
            if (c->lbx[(size_t)k * nx + i] != prm.lbx[i] || c->ubx[(size_t)k * nx + i] != prm.ubx[i]) {
                why = "stage-varying state bounds";
                return false;
            }
    }
    for (int i = 0; i < c->nbu; i++) {
        prm.lbu[i] = c->lbu[i];
        prm.ubu[i] = c->ubu[i];
        for (int k = 1; k < N; k++)
            if (c->lbu[(size_t)k * c->nbu + i] != prm.lbu[i] || c->ubu[(size_t)k * c->nbu + i] != prm.ubu[i]) {
                why = "stage-varying input bounds";
                return false;
            }
    }
    for (int i = 0; i < c->np; i++) {
        prm.p[i] = c->p[i];
        for (int k = 1; k < N; k++)
            if (c->p[(size_t)k * c->np + i] != prm.p[i]) { why = "stage-varying parameters"; return false; }
    }
    return true;
}

bool pack(nmpc_capsule_impl* c, Packed& o, std::string& why)
{
    for (int i = 0; i < c->nx; i++)
        if (c->lbx[i] != c->ubx[i]) { why = "stage-0 lbx != ubx (x0 must be an equality)"; return false; }
    if (c->uniform_dirty) {
        c->uniform_why.clear();
        c->uniform_ok = validate_uniform(c, c->uniform_why);
        c->uniform_dirty = false;
    }
    if (!c->uniform_ok) {
        why = c->uniform_why;
        return false;
    }
    o.prm = c->uniform_prm;
    o.x0 = c->lbx.data();
    o.yref = c->yref.data();
    o.We = c->uniform_We.data();
    return true;
}

// dst[r * n + q] = (float)src[q][r] for r < rows, q < n: capsule-major host data -> instance-minor staging,
// in blocks of 32 capsules (each row of a block is one 128-B line; 32 read streams)
void to_soa(float* dst, int n, size_t rows, const std::vector<const double*>& src)
{
    for (int q0 = 0; q0 < n; q0 += 32) {
        const int q1 = std::min(n, q0 + 32);
        for (size_t r = 0; r < rows; r++) {
            float* d = dst + r * n;
            for (int q = q0; q < q1; q++) d[q] = (float)src[q][r];
        }
    }
}

void from_soa(const float* srcv, int n, size_t rows, const std::vector<double*>& dst)
{
    for (int q0 = 0; q0 < n; q0 += 32) {
        const int q1 = std::min(n, q0 + 32);
        for (size_t r = 0; r < rows; r++) {
            const float* v = srcv + r * n;
            for (int q = q0; q < q1; q++)
                if (dst[q]) dst[q][r] = v[q];
        }
    }
}

bool same_params(const nmpc_model_params& a, const nmpc_model_params& b)
{
    return std::memcmp(&a, &b, sizeof(a)) == 0;
}

int ensure_engine(Engine& e, const nmpc_model_params& prm, int n, std::string& why)
{
    if (e.batch && e.cap >= n) {
        if (nmpc_batch_set_params(e.batch, &prm) != NMPC_OK) { why = nmpc_last_error(); return -1; }
        return 0;
    }
    e.release();
    int cap = 1;
    while (cap < n) cap *= 2;
    int nx, nu, ny;
    nmpc_model_dims(prm.model, &nx, &nu, &ny, nullptr, nullptr, nullptr);
    const int N = prm.N;
    if (nmpc_batch_create(&prm, cap, &e.batch) != NMPC_OK) { why = nmpc_last_error(); return -1; }
    hipError_t r = hipSuccess;
    const Blocks bl(cap, N, nx, nu, ny);
    static_assert(sizeof(int) == sizeof(float), "int32 words in the float output block");
    if ((r = hipMalloc(&e.dio, sizeof(float) * bl.io_words)) != hipSuccess ||
        (r = hipHostMalloc(&e.hio, sizeof(float) * bl.io_words)) != hipSuccess ||
        (r = hipHostMalloc(&e.hwarm, (size_t)cap)) != hipSuccess) {
        why = hipGetErrorString(r);
        e.release();
        return -1;
    }
    if ((r = hipHostGetDevicePointer(reinterpret_cast<void**>(&e.hio_dev), e.hio, 0)) != hipSuccess) e.hio_dev = nullptr;
    nmpc_batch_warm_state(e.batch, &e.dwarm, nullptr, nullptr);
    e.owner.assign(cap, 0);
    e.dev_warm.assign(cap, 0);  // nmpc_batch_create zeroes the flags
    e.cap = cap;
    return 0;
}

// Solve one group of capsules that share all uniform parameters.
void solve_group(std::vector<nmpc_capsule_impl*>& cs, std::vector<Packed>& ps, const std::vector<int>& idx)
{
    const auto t0 = std::chrono::steady_clock::now();
    nmpc_capsule_impl* c0 = cs[idx[0]];
    const int n = (int)idx.size(), N = c0->N, nx = c0->nx, nu = c0->nu, ny = c0->ny;
    auto& slot = g_engines[{c0->model, N}];
    if (!slot) slot.reset(new Engine());
    Engine& e = *slot;
    std::string why;
    auto fail_all = [&](const std::string& msg) {
        log_err("solve", msg);
        for (int i : idx) {
            cs[i]->status = 4;
            cs[i]->warm_ok = false;
        }
        for (int q = 0; q < (int)e.owner.size() && q < n; q++) {
            e.owner[q] = 0;
            e.dev_warm[q] = kWarmUnknown;
        }
    };
    {
        const TraceRange tr("capsule.engine");
        if (ensure_engine(e, ps[idx[0]].prm, n, why)) return fail_all(why);
    }
    const auto ta = std::chrono::steady_clock::now();
    const Blocks bl(n, N, nx, nu, ny);
    float *hx0 = e.hio + bl.x0, *hyref = e.hio + bl.yref, *hWe = e.hio + bl.We, *hxb = e.hio + bl.xb,
          *hub = e.hio + bl.ub;
    {
        const TraceRange tr("capsule.pack");
        std::vector<const double*> x0s(n), yrefs(n), Wes(n), xbs(n), ubs(n);
        for (int q = 0; q < n; q++) {
            const Packed& P = ps[idx[q]];
            x0s[q] = P.x0;
            yrefs[q] = P.yref;
            Wes[q] = P.We;
            xbs[q] = cs[idx[q]]->xbar.data();
            ubs[q] = cs[idx[q]]->ubar.data();
        }
        to_soa(hx0, n, nx, x0s);
        to_soa(hWe, n, nx, Wes);
        to_soa(hyref, n, (size_t)(N + 1) * ny, yrefs);
        to_soa(hxb, n, (size_t)(N + 1) * nx, xbs);
        to_soa(hub, n, (size_t)N * nu, ubs);
    }
    const auto tb = std::chrono::steady_clock::now();
    hipError_t r = hipSuccess;
    const hipStream_t st = nullptr;
    float* const dio = e.dio;
    bool flags_differ = false;
    for (int q = 0; q < n; q++) {
        const nmpc_capsule_impl* c = cs[idx[q]];
        e.hwarm[q] = (e.owner[q] == c->uid && c->warm_ok) ? c->warm_tag : 0;
        flags_differ |= e.hwarm[q] != e.dev_warm[q];
    }
    nmpc_launch_plan plan{};
    nmpc_batch_plan_ex(e.batch, n, NMPC_PLAN_SOLVE, &plan);  // the kernel of this launch, and the tag it leaves
    // One capsule on the row-parallel kernel (the reference node's case): the kernel reads the pinned input block and
    // writes the output block back itself, so the solve is one launch instead of a copy, the kernel and a copy, each
    // behind the previous one's completion (same box: profiles/r06/ab/capsule_staged.txt). NMPC_AMD_CAPSULE_STAGE=0
    // keeps the copies (A/B).
    static const bool stage_ok_env = [] {
        const char* v = std::getenv("NMPC_AMD_CAPSULE_STAGE");
        return !(v && std::atoi(v) == 0);
    }();
    const bool staged = n == 1 && plan.kernel == 1 && e.hio_dev && stage_ok_env;
    {
        const TraceRange tr("capsule.h2d");
        if (flags_differ && (r = hipMemcpyAsync(e.dwarm, e.hwarm, (size_t)n, hipMemcpyHostToDevice, st)) != hipSuccess)
            return fail_all(hipGetErrorString(r));
        if (!staged &&
            (r = hipMemcpyAsync(dio, e.hio, sizeof(float) * bl.in_floats, hipMemcpyHostToDevice, st)) != hipSuccess)
            return fail_all(hipGetErrorString(r));
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (staged) {
        const nmpc_stage_io io{e.hio_dev, dio, (int)bl.in_floats, e.hio_dev + bl.xb, dio + bl.xb,
                               (int)(bl.io_words - bl.xb)};
        if (nmpc_batch_solve_iterate_staged(e.batch, dio + bl.x0, dio + bl.yref, ny, dio + bl.We, dio + bl.xb,
                                            dio + bl.ub, reinterpret_cast<int*>(dio + bl.ost),
                                            reinterpret_cast<int*>(dio + bl.oit), dio + bl.ores, st, &io) != NMPC_OK)
            return fail_all(nmpc_last_error());
    } else if (nmpc_batch_solve_iterate(e.batch, n, dio + bl.x0, dio + bl.yref, ny, dio + bl.We, nullptr,
                                        dio + bl.xb, dio + bl.ub, n, reinterpret_cast<int*>(dio + bl.ost),
                                        reinterpret_cast<int*>(dio + bl.oit), dio + bl.ores, st) != NMPC_OK) {
        return fail_all(nmpc_last_error());
    }
    {
        const TraceRange tr("capsule.d2h_sync");  // the output copy queued behind the kernel, and the wait
        if (!staged && (r = hipMemcpyAsync(e.hio + bl.xb, dio + bl.xb, sizeof(float) * (bl.io_words - bl.xb),
                                           hipMemcpyDeviceToHost, st)) != hipSuccess)
            return fail_all(hipGetErrorString(r));
        if ((r = hipStreamSynchronize(st)) != hipSuccess) return fail_all(hipGetErrorString(r));
    }
    const float* const hres = e.hio + bl.ores;
    const int* const hst = reinterpret_cast<const int*>(e.hio + bl.ost);
    const int* const hit = reinterpret_cast<const int*>(e.hio + bl.oit);
    const auto t2 = std::chrono::steady_clock::now();
    const double tt = std::chrono::duration<double>(t2 - t0).count();
    const double tq = std::chrono::duration<double>(t2 - t1).count();
    if (std::getenv("NMPC_AMD_SHIM_TIMING"))
        std::fprintf(stderr, "[nmpc_amd] solve_group n=%d engine %.3f pack %.3f h2d %.3f solve+d2h %.3f ms\n", n,
                     std::chrono::duration<double>(ta - t0).count() * 1e3,
                     std::chrono::duration<double>(tb - ta).count() * 1e3,
                     std::chrono::duration<double>(t1 - tb).count() * 1e3, tq * 1e3);
    int rule_warm = 0, rule_wmax = 0, rule_imax = 0;
    nmpc_batch_warm_rule(e.batch, &rule_warm, &rule_wmax, &rule_imax);
    std::vector<double*> xbs(n), ubs(n);  // failed solves keep their iterate (nullptr: skipped)
    for (int q = 0; q < n; q++) {
        nmpc_capsule_impl* c = cs[idx[q]];
        c->status = hst[q];
        c->qp_iter = hit[q];
        // max of the QP's residuals at IPM exit: stationarity, bound residual, complementarity (qp_res rows 0-2; the
        // dynamics hold exactly in the dynamics-feasible IPM). acados' inf_norm_res is the NLP residual, which
        // RTI does not refresh and the reference never uses (NMPCNavControlDiff.cpp:146)
        c->out.inf_norm_res = std::fmax(std::fmax(hres[q], hres[(size_t)n + q]), hres[(size_t)2 * n + q]);
        c->sqp_iter = 1;
        c->out.sqp_iter = 1;
        c->time_tot = tt;
        c->time_qp = tq;
        c->time_lin = 0.0;
        // the kernel's epilogue rule, with the engine's effective parameters (env overrides included), so that
        // dev_warm mirrors the device flags exactly: warm && status == 0 && converged before the cap
        const bool conv = rule_warm && hst[q] == 0 && hit[q] < rule_imax && hit[q] <= rule_wmax;
        c->warm_ok = conv;
        c->warm_tag = (unsigned char)plan.warm_tag;
        e.owner[q] = c->uid;
        e.dev_warm[q] = conv ? (unsigned char)plan.warm_tag : 0;
        xbs[q] = hst[q] == 0 ? c->xbar.data() : nullptr;
        ubs[q] = hst[q] == 0 ? c->ubar.data() : nullptr;
    }
    const TraceRange tr("capsule.unpack");
    from_soa(hxb, n, (size_t)(N + 1) * nx, xbs);
    from_soa(hub, n, (size_t)N * nu, ubs);
}

int batch_solve_impl(std::vector<nmpc_capsule_impl*>& cs, int* status_out)
{
    std::lock_guard<std::mutex> lock(g_mu);
    const int n = (int)cs.size();
    std::vector<Packed> ps(n);
    std::vector<bool> done(n, false);
    for (int i = 0; i < n; i++) {
        std::string why;
        if (!cs[i] || !cs[i]->created) {
            if (cs[i]) cs[i]->status = 4;
            log_err("solve", "capsule not created");
            done[i] = true;
            continue;
        }
        if (!pack(cs[i], ps[i], why)) {
            log_err("solve", "unsupported OCP data: " + why);
            cs[i]->status = 4;
            done[i] = true;
        }
    }
    // group by (N, uniform parameters)
    for (int i = 0; i < n; i++) {
        if (done[i]) continue;
        std::vector<int> idx;
        for (int j = i; j < n; j++)
            if (!done[j] && cs[j]->N == cs[i]->N && same_params(ps[j].prm, ps[i].prm)) {
                idx.push_back(j);
                done[j] = true;
            }
        solve_group(cs, ps, idx);
    }
    int nfail = 0;
    for (int i = 0; i < n; i++) {
        const int s = cs[i] ? cs[i]->status : 4;
        if (status_out) status_out[i] = s;
        if (s != 0) nfail++;
    }
    return nfail;
}

nmpc_capsule_impl* impl_of(void* p) { return p ? static_cast<nmpc_capsule_impl*>(p) : nullptr; }

}  // namespace

// ------------------------------------------------------------------------------------------------------
// Generic acados C interface subset
// ------------------------------------------------------------------------------------------------------
extern "C" {

int ocp_nlp_constraints_model_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, ocp_nlp_out* out,
                                  int stage, const char* field, void* value)
{
    (void)config; (void)dims; (void)out;
    nmpc_capsule_impl* c = in ? impl_of(in->impl) : nullptr;
    if (!c || !c->created || !field || !value) return -1;
    if (!stage_ok(c, stage, "ocp_nlp_constraints_model_set", field)) return -1;
    const double* v = static_cast<const double*>(value);
    const int nx = c->nx;
    if (!std::strcmp(field, "lbx") || !std::strcmp(field, "ubx")) {
        std::vector<double>& dst = (field[0] == 'l') ? c->lbx : c->ubx;
        const int n = (stage == 0) ? nx : c->nbx;  // nbx0 = NX (x0), nbx = NBX on idxbx
        for (int i = 0; i < n; i++) dst[(size_t)stage * nx + i] = v[i];
        if (stage > 0) c->uniform_dirty = true;
        return 0;
    }
    if (!std::strcmp(field, "lbu") || !std::strcmp(field, "ubu")) {
        if (stage >= c->N) {
            log_err("ocp_nlp_constraints_model_set", std::string(field) + " at the terminal stage " +
                                                         std::to_string(stage) + " (inputs live on stages 0..N-1)");
            return -1;
        }
        std::vector<double>& dst = (field[0] == 'l') ? c->lbu : c->ubu;
        for (int i = 0; i < c->nbu; i++) dst[(size_t)stage * c->nbu + i] = v[i];
        c->uniform_dirty = true;
        return 0;
    }
    log_err("ocp_nlp_constraints_model_set", std::string("unsupported field ") + field);
    return -1;
}

int ocp_nlp_cost_model_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                           const char* field, void* value)
{
    (void)config; (void)dims;
    nmpc_capsule_impl* c = in ? impl_of(in->impl) : nullptr;
    if (!c || !c->created || !field || !value) return -1;
    if (!stage_ok(c, stage, "ocp_nlp_cost_model_set", field)) return -1;
    const double* v = static_cast<const double*>(value);
    const int n = (stage == c->N) ? c->nx : c->ny;
    if (!std::strcmp(field, "W")) {
        double* W = c->W.data() + (size_t)stage * c->ny * c->ny;
        std::fill(W, W + c->ny * c->ny, 0.0);
        for (int i = 0; i < n * n; i++) W[i] = v[i];  // col-major n x n
        c->uniform_dirty = true;
        return 0;
    }
    if (!std::strcmp(field, "yref")) {
        for (int i = 0; i < n; i++) c->yref[(size_t)stage * c->ny + i] = v[i];
        return 0;
    }
    log_err("ocp_nlp_cost_model_set", std::string("unsupported field ") + field);
    return -1;
}

int ocp_nlp_constraints_model_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                                  const char* field, void* value)
{
    (void)config; (void)dims;
    nmpc_capsule_impl* c = in ? impl_of(in->impl) : nullptr;
    if (!c || !c->created || !field || !value) return -1;
    if (!stage_ok(c, stage, "ocp_nlp_constraints_model_get", field)) return -1;
    double* v = static_cast<double*>(value);
    const int nx = c->nx;
    if (!std::strcmp(field, "lbx") || !std::strcmp(field, "ubx")) {
        const std::vector<double>& src = (field[0] == 'l') ? c->lbx : c->ubx;
        const int n = (stage == 0) ? nx : c->nbx;
        for (int i = 0; i < n; i++) v[i] = src[(size_t)stage * nx + i];
        return 0;
    }
    if ((!std::strcmp(field, "lbu") || !std::strcmp(field, "ubu")) && stage < c->N) {
        const std::vector<double>& src = (field[0] == 'l') ? c->lbu : c->ubu;
        for (int i = 0; i < c->nbu; i++) v[i] = src[(size_t)stage * c->nbu + i];
        return 0;
    }
    log_err("ocp_nlp_constraints_model_get", std::string("unsupported field ") + field);
    return -1;
}

int ocp_nlp_cost_model_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                           const char* field, void* value)
{
    (void)config; (void)dims;
    nmpc_capsule_impl* c = in ? impl_of(in->impl) : nullptr;
    if (!c || !c->created || !field || !value) return -1;
    if (!stage_ok(c, stage, "ocp_nlp_cost_model_get", field)) return -1;
    double* v = static_cast<double*>(value);
    const int n = (stage == c->N) ? c->nx : c->ny;
    if (!std::strcmp(field, "W")) {
        const double* W = c->W.data() + (size_t)stage * c->ny * c->ny;
        for (int i = 0; i < n * n; i++) v[i] = W[i];
        return 0;
    }
    if (!std::strcmp(field, "yref")) {
        for (int i = 0; i < n; i++) v[i] = c->yref[(size_t)stage * c->ny + i];
        return 0;
    }
    log_err("ocp_nlp_cost_model_get", std::string("unsupported field ") + field);
    return -1;
}

void ocp_nlp_out_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage, const char* field,
                     void* value)
{
    (void)config; (void)dims;
    nmpc_capsule_impl* c = out ? impl_of(out->impl) : nullptr;
    if (!c || !c->created || !field || !value || !stage_ok(c, stage, "ocp_nlp_out_get", field)) return;
    double* v = static_cast<double*>(value);
    if (!std::strcmp(field, "x")) {
        for (int i = 0; i < c->nx; i++) v[i] = c->xbar[(size_t)stage * c->nx + i];
    } else if (!std::strcmp(field, "u") && stage < c->N) {
        for (int i = 0; i < c->nu; i++) v[i] = c->ubar[(size_t)stage * c->nu + i];
    } else {
        log_err("ocp_nlp_out_get", std::string("unsupported field ") + field);
    }
}

void ocp_nlp_out_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage, const char* field,
                     void* value)
{
    (void)config; (void)dims;
    nmpc_capsule_impl* c = out ? impl_of(out->impl) : nullptr;
    if (!c || !c->created || !field || !value || !stage_ok(c, stage, "ocp_nlp_out_set", field)) return;
    const double* v = static_cast<const double*>(value);
    if (!std::strcmp(field, "x")) {
        for (int i = 0; i < c->nx; i++) c->xbar[(size_t)stage * c->nx + i] = v[i];
    } else if (!std::strcmp(field, "u") && stage < c->N) {
        for (int i = 0; i < c->nu; i++) c->ubar[(size_t)stage * c->nu + i] = v[i];
    } else {
        log_err("ocp_nlp_out_set", std::string("unsupported field ") + field);
    }
}

void ocp_nlp_get(ocp_nlp_solver* solver, const char* field, void* return_value_)
{
    nmpc_capsule_impl* c = solver ? impl_of(solver->impl) : nullptr;
    if (!c || !field || !return_value_) return;
    if (!std::strcmp(field, "time_tot")) *static_cast<double*>(return_value_) = c->time_tot;
    else if (!std::strcmp(field, "time_lin")) *static_cast<double*>(return_value_) = c->time_lin;
    else if (!std::strcmp(field, "time_qp_sol") || !std::strcmp(field, "time_qp"))
        *static_cast<double*>(return_value_) = c->time_qp;
    else if (!std::strcmp(field, "sqp_iter")) *static_cast<int*>(return_value_) = c->sqp_iter;
    else if (!std::strcmp(field, "qp_iter")) *static_cast<int*>(return_value_) = c->qp_iter;
    else if (!std::strcmp(field, "status")) *static_cast<int*>(return_value_) = c->status;
    else log_err("ocp_nlp_get", std::string("unsupported field ") + field);
}

void ocp_nlp_solver_opts_set(ocp_nlp_config* config, void* opts_, const char* field, void* value)
{
    (void)opts_;
    nmpc_capsule_impl* c = config ? impl_of(config->impl) : nullptr;
    if (!c || !field || !value) return;
    const int v = *static_cast<const int*>(value);
    if (!std::strcmp(field, "qp_warm_start")) {
        // acados / HPIPM: 0 cold, 1 warm-start the primal QP variables, 2 primal and dual. The delta-form IPM here
        // always starts its primal point from the dynamics-feasible initial iterate (there is no separate primal
        // warm start), so 0 and 1 both start cold and only 2 warm-starts the bound multipliers
        c->prm.qp_warm_start = (v == 2) ? 1 : 0;
        if (v != 2) c->warm_ok = false;
        static std::atomic<bool> told{false};
        if (v == 1 && !told.exchange(true))  // until round 5, 1 selected the multiplier warm start
            log_err("ocp_nlp_solver_opts_set", "qp_warm_start 1 (primal only) starts the QP cold here; 2 warm-starts "
                                               "the bound multipliers");
    } else if (!std::strcmp(field, "qp_iter_max") && v >= 1) {
        c->prm.qp_iter_max = v;
    } else {
        log_err("ocp_nlp_solver_opts_set", std::string("unsupported field ") + field);
    }
}

int ocp_nlp_dims_get_from_attr(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage,
                               const char* field)
{
    (void)config; (void)out;
    nmpc_capsule_impl* c = dims ? impl_of(dims->impl) : nullptr;
    if (!c || !field) return -1;
    if (!std::strcmp(field, "x")) return c->nx;
    if (!std::strcmp(field, "u")) return stage < c->N ? c->nu : 0;
    if (!std::strcmp(field, "y_ref") || !std::strcmp(field, "yref")) return stage < c->N ? c->ny : c->nx;
    return -1;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------------
// Model-generic capsule engine (include/nmpc_amd/nmpc_capsule.h). The per-model {name}_acados_* functions
// are generated by tools/generate_solver_libs.py into libacados_ocp_solver_{name}.so and forward here.
// ------------------------------------------------------------------------------------------------------
extern "C" {

int nmpc_codegen_default(int model, nmpc_codegen_desc* d)
{
    if (!d || model < 0 || model > 2) return NMPC_ERR_ARG;
    std::memset(d, 0, sizeof(*d));
    d->model = model;
    d->N = 80;  // tf_ini 2.0 s at freq 40 Hz (scripts/diff/common.py:5-9)
    d->tf = 80.0 / 40.0;
    const double deg = M_PI / 180.0;
    nmpc_model_params prm;
    nmpc_model_params_default(model, d->N, &prm);
    if (model == NMPC_MODEL_DIFF2AMR) {
        d->p[0] = 0.270; d->p[1] = 0.1;
        nmpc_model_params_set_limits(&prm, 1.0, 2.0, 0, 0, 0);
        const double w[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1}, we[7] = {1000, 1000, 500, 0, 0, 0, 0};
        std::memcpy(d->W, w, sizeof(w));
        std::memcpy(d->W_e, we, sizeof(we));
    } else if (model == NMPC_MODEL_OMNI4AMR) {
        d->p[0] = 0.535; d->p[1] = 0.1;
        nmpc_model_params_set_limits(&prm, 1.0, 1.0, 0, 0, 0);
        const double w[15] = {10, 10, 10, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1};
        std::memcpy(d->W, w, sizeof(w));
        std::memcpy(d->W_e, w, sizeof(double) * 11);
    } else {
        d->p[0] = 0.270; d->p[1] = 0.1; d->p[2] = 0.5;
        nmpc_model_params_set_limits(&prm, 1.0, 1.0, -30.0 * deg, 30.0 * deg, 120.0 * deg);
        const double w[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1}, we[7] = {1000, 1000, 500, 0, 0, 0, 0};
        std::memcpy(d->W, w, sizeof(w));
        std::memcpy(d->W_e, we, sizeof(we));
    }
    std::memcpy(d->lbx, prm.lbx, sizeof(d->lbx));
    std::memcpy(d->ubx, prm.ubx, sizeof(d->ubx));
    std::memcpy(d->lbu, prm.lbu, sizeof(d->lbu));
    std::memcpy(d->ubu, prm.ubu, sizeof(d->ubu));
    return NMPC_OK;
}

nmpc_solver_capsule* nmpc_capsule_new(int model)
{
    if (model < 0 || model > 2) return nullptr;
    nmpc_solver_capsule* cap = new nmpc_solver_capsule();
    nmpc_capsule_impl* c = new_impl(model);
    cap->impl = c;
    cap->nlp_config = &c->config;
    cap->nlp_dims = &c->dims;
    cap->nlp_in = &c->in;
    cap->nlp_out = &c->out;
    cap->nlp_solver = &c->solver;
    cap->nlp_opts = c;  // opaque: ocp_nlp_solver_opts_set finds the capsule through its config
    return cap;
}

int nmpc_capsule_delete(nmpc_solver_capsule* capsule)
{
    if (!capsule) return 1;
    delete capsule->impl;
    delete capsule;
    return 0;
}

int nmpc_capsule_create(nmpc_solver_capsule* capsule, const nmpc_codegen_desc* desc, int n_time_steps,
                        const double* new_time_steps)
{
    if (!capsule || !capsule->impl) return 1;
    nmpc_codegen_desc d;
    if (desc) {
        if (desc->model != capsule->impl->model || desc->N < 1 || !(desc->tf > 0.0)) {
            log_err("create", "codegen descriptor does not match the capsule's model");
            return 1;
        }
        d = *desc;
    } else {
        nmpc_codegen_default(capsule->impl->model, &d);
    }
    if (new_time_steps) {
        for (int k = 1; k < n_time_steps; k++)
            if (std::fabs(new_time_steps[k] - new_time_steps[0]) > 1e-12 * std::fabs(new_time_steps[0])) {
                log_err("create", "non-uniform time steps are not supported");
                return 1;
            }
        if (n_time_steps >= 1) {
            d.N = n_time_steps;
            d.tf = new_time_steps[0] * n_time_steps;
        }
    } else if (n_time_steps != d.N) {
        // as the acados template's {name}_acados_create_with_discretization: a horizon other than the baked one
        // needs its time steps (the wrappers size yref[N+1] and loop over stages by the baked {NAME}_N)
        log_err("create", "new_time_steps is NULL but the number of shooting intervals (= " +
                              std::to_string(n_time_steps) + ") differs from the number of shooting intervals (= " +
                              std::to_string(d.N) + ") during code generation: provide the time steps");
        return 1;
    }
    return impl_create(capsule->impl, n_time_steps, d);
}

int nmpc_capsule_reset(nmpc_solver_capsule* capsule, int reset_qp_solver_mem)
{
    (void)reset_qp_solver_mem;  // the only QP memory is the warm-start multipliers, dropped either way
    if (!capsule || !capsule->impl || !capsule->impl->created) return 1;
    nmpc_capsule_impl* c = capsule->impl;
    std::fill(c->xbar.begin(), c->xbar.end(), 0.0);
    std::fill(c->ubar.begin(), c->ubar.end(), 0.0);
    c->warm_ok = false;  // the next solve starts the IPM cold, like a fresh capsule
    return 0;
}

int nmpc_capsule_update_params(nmpc_solver_capsule* capsule, int stage, const double* value, int np)
{
    if (!capsule || !capsule->impl || !capsule->impl->created || !value) return 1;
    nmpc_capsule_impl* c = capsule->impl;
    if (np != c->np) {
        log_err("update_params", "np does not match the model");
        return 1;
    }
    if (!stage_ok(c, stage, "update_params", "p")) return 1;
    for (int i = 0; i < np; i++) c->p[(size_t)stage * np + i] = value[i];
    c->uniform_dirty = true;
    return 0;
}

int nmpc_capsule_solve(nmpc_solver_capsule* capsule)
{
    if (!capsule || !capsule->impl) return 4;
    static const char* const names[3] = {"diff2amr_acados_solve", "omni4amr_acados_solve", "tric3amr_acados_solve"};
    const int m = capsule->impl->model;
    const TraceRange trace(m >= 0 && m < 3 ? names[m] : "acados_solve");
    std::vector<nmpc_capsule_impl*> cs{capsule->impl};
    batch_solve_impl(cs, nullptr);
    return capsule->impl->status;
}

int nmpc_capsule_batch_solve(nmpc_solver_capsule** capsules, int* status_out, int n)
{
    if (!capsules || n < 0) return -1;
    const TraceRange trace("acados_batch_solve");
    std::vector<nmpc_capsule_impl*> cs(n);
    for (int i = 0; i < n; i++) cs[i] = capsules[i] ? capsules[i]->impl : nullptr;
    return batch_solve_impl(cs, status_out);
}

int nmpc_capsule_free(nmpc_solver_capsule* capsule)
{
    if (!capsule || !capsule->impl) return 1;
    capsule->impl->created = false;
    return 0;
}

void nmpc_capsule_print_stats(const nmpc_solver_capsule* capsule, const char* name)
{
    if (!capsule || !capsule->impl) return;
    const nmpc_capsule_impl* c = capsule->impl;
    std::printf("%s: status %d, sqp_iter %d, qp_iter %d, time_tot %.3f ms\n", name ? name : "nmpc", c->status,
                c->sqp_iter, c->qp_iter, c->time_tot * 1e3);
}

}  // extern "C"
