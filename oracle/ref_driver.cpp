// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (see nmpc_oracle.h): runs the REFERENCE's own per-model wrappers,
// src/nmpc_nav_control/NMPCNavControl{,Diff,Omni4,Tric}.cpp compiled in place from /root/reference by
// oracle/Makefile (target `ref`, outputs in oracle/_ref/ only), over ticks given on stdin, and prints what each
// run() handed to the solver and what it returned. tests/test_reference_wrappers.py compares that with the
// oracle's restatement of the same pre-/post-solve code (oc_prepare / oc_post, nmpc_oracle.c), bit for bit.
//
// Two builds of this file:
//   ref_wrappers_oracle  (-DREF_SOLVE_ORACLE): {name}_acados_solve is the fp64 oracle's SQP-RTI step (oc_sqp_rti)
//                        on the inputs the wrapper set, read back through the boundary's getters, so the whole
//                        run() -- pre-solve, solve, post-solve -- runs on the CPU;
//   ref_wrappers_device: the wrappers linked exactly as the reference's CMakeLists.txt:112-114 links them, against
//                        libacados_ocp_solver_{name}.so + libnmpc_amd.so: the reference's run() around the MI355X
//                        solve (the -m gpu test).
// The wrappers keep their capsule private, so {name}_acados_create_capsule is interposed to learn it (the real
// one is reached through dlsym(RTLD_NEXT)); every other acados call goes to the boundary unchanged.
//
// stdin (whitespace-separated):
//   <model 0|1|2> <dt> <p0> <p1> <p2> <v_max> <a_max> <alpha_min> <alpha_max> <dalpha_max> <nW> <W_diag...>
//   then any of:  R                          a new robot (a new wrapper: constructor, NMPCNavControlDiff.cpp:6-74)
//                 T <reset> <steer> <pose x y theta> <vel v vn w> <n> <n poses x y theta>
//                                            one tick: reset_mpc() if reset, setSteeringWheelAngle (tric), run()
//                 E                          end
// stdout per tick: `tick <run() returned> <status> <qp_iter>` and the lines x0 / yref / We (read back from the
// boundary after run(): stage-0 lbx, yref of stages 0..N, diag of W at stage N), xb / ub (the iterate the solve
// started from), u0 / x1 (the iterate after it), cmd, err (the exception text or -); numbers as %.17g.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "nmpc_nav_control/NMPCNavControlDiff.h"
#include "nmpc_nav_control/NMPCNavControlOmni4.h"
#include "nmpc_nav_control/NMPCNavControlTric.h"
#ifdef REF_SOLVE_ORACLE
#include "nmpc_oracle.h"
#endif

using namespace nmpc_nav_control;

namespace {

// the three generated capsule types share this layout (include/acados_solver_*.h)
typedef diff2amr_solver_capsule capsule_t;
capsule_t* g_capsule = nullptr;

template <typename F>
F real_fn(const char* name)
{
    void* f = dlsym(RTLD_NEXT, name);
    if (!f) {
        std::fprintf(stderr, "ref_driver: dlsym(%s): %s\n", name, dlerror());
        std::abort();
    }
    return reinterpret_cast<F>(f);
}

#ifdef REF_SOLVE_ORACLE
oc_params g_prm;

int oracle_solve(capsule_t* c)
{
    ocp_nlp_dims* d = c->nlp_dims;
    const int N = d->N, nx = d->nx, nu = d->nu, ny = d->ny;
    std::vector<double> x0(nx), yref((size_t)(N + 1) * ny, 0.0), WN((size_t)nx * nx), We(nx);
    std::vector<double> xb((size_t)(N + 1) * nx), ub((size_t)N * nu);
    if (ocp_nlp_constraints_model_get(c->nlp_config, d, c->nlp_in, 0, "lbx", x0.data())) return 4;
    for (int k = 0; k <= N; k++)
        if (ocp_nlp_cost_model_get(c->nlp_config, d, c->nlp_in, k, "yref", yref.data() + (size_t)k * ny)) return 4;
    if (ocp_nlp_cost_model_get(c->nlp_config, d, c->nlp_in, N, "W", WN.data())) return 4;
    for (int i = 0; i < nx; i++) We[i] = WN[(size_t)i * nx + i];
    for (int k = 0; k <= N; k++) ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, k, "x", xb.data() + (size_t)k * nx);
    for (int k = 0; k < N; k++) ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, k, "u", ub.data() + (size_t)k * nu);
    oc_params prm = g_prm;
    prm.N = N;
    oc_stats st;
    const int s = oc_sqp_rti(&prm, xb.data(), ub.data(), x0.data(), yref.data(), We.data(), &st);
    if (s == 0) {
        for (int k = 0; k <= N; k++) ocp_nlp_out_set(c->nlp_config, d, c->nlp_out, k, "x", xb.data() + (size_t)k * nx);
        for (int k = 0; k < N; k++) ocp_nlp_out_set(c->nlp_config, d, c->nlp_out, k, "u", ub.data() + (size_t)k * nu);
    }
    return s;
}
#endif

}  // namespace

// Interposed: the wrappers' capsule (NMPCNavControlDiff.cpp:10), then the boundary's own create_capsule
#define REF_INTERPOSE(name)                                                                                       \
    extern "C" name##_solver_capsule* name##_acados_create_capsule(void)                                         \
    {                                                                                                            \
        static auto real = real_fn<name##_solver_capsule* (*)(void)>(#name "_acados_create_capsule");            \
        name##_solver_capsule* c = real();                                                                       \
        g_capsule = reinterpret_cast<capsule_t*>(c);                                                             \
        return c;                                                                                                \
    }
REF_INTERPOSE(diff2amr)
REF_INTERPOSE(omni4amr)
REF_INTERPOSE(tric3amr)

#ifdef REF_SOLVE_ORACLE
extern "C" int diff2amr_acados_solve(diff2amr_solver_capsule* c) { return oracle_solve(reinterpret_cast<capsule_t*>(c)); }
extern "C" int omni4amr_acados_solve(omni4amr_solver_capsule* c) { return oracle_solve(reinterpret_cast<capsule_t*>(c)); }
extern "C" int tric3amr_acados_solve(tric3amr_solver_capsule* c) { return oracle_solve(reinterpret_cast<capsule_t*>(c)); }
#endif

namespace {

void put(const char* tag, const double* v, size_t n)
{
    std::printf("%s", tag);
    for (size_t i = 0; i < n; i++) std::printf(" %.17g", v[i]);
    std::printf("\n");
}

// The wrappers never initialise the yref entries past the pose (acados_in_.yref[i][3..NY-1], the velocity and
// input references of NMPCNavControlDiff.cpp:106-118) and pass them to the solver; construct them in zeroed memory
// so those entries are 0, as in a fresh process, instead of whatever the heap held
template <class T, class... A>
T* make_zeroed(A&&... a)
{
    void* m = ::operator new(sizeof(T));
    std::memset(m, 0, sizeof(T));
    return new (m) T(std::forward<A>(a)...);
}

double rd()
{
    double v;
    if (std::scanf("%lf", &v) != 1) throw std::runtime_error("ref_driver: truncated input");
    return v;
}

}  // namespace

int main()
{
    try {
        const int model = (int)rd();
        const double dt = rd();
        double p[3], lim[5];
        for (double& v : p) v = rd();
        for (double& v : lim) v = rd();
        const int nW = (int)rd();
        std::vector<double> W(nW);
        for (double& v : W) v = rd();
#ifdef REF_SOLVE_ORACLE
        oc_params_default(model, 80, &g_prm);
        for (int i = 0; i < 3; i++) g_prm.p[i] = p[i];
        oc_params_set_limits(&g_prm, lim[0], lim[1], lim[2], lim[3], lim[4]);
        for (int i = 0; i < nW && i < OC_NYMAX; i++) g_prm.W[i] = W[i];
        for (int i = 0; i < g_prm.nx; i++) g_prm.W_e[i] = W[i];
#endif
        std::unique_ptr<NMPCNavControl> w;
        NMPCNavControlTric* tric = nullptr;
        char op[8];
        while (std::scanf("%7s", op) == 1) {
            if (op[0] == 'E') break;
            if (op[0] == 'R') {
                w.reset();  // the previous robot's destructor frees its capsule first
                tric = nullptr;
                if (model == 0) w.reset(make_zeroed<NMPCNavControlDiff>(dt, p[0], p[1], lim[0], lim[1], W));
                else if (model == 1) w.reset(make_zeroed<NMPCNavControlOmni4>(dt, p[0], p[1], lim[0], lim[1], W));
                else {
                    tric = make_zeroed<NMPCNavControlTric>(dt, p[0], p[1], p[2], lim[0], lim[1], lim[2], lim[3], lim[4], W);
                    w.reset(tric);
                }
                continue;
            }
            if (op[0] != 'T' || !w || !g_capsule) throw std::runtime_error(std::string("ref_driver: bad op ") + op);
            const int reset = (int)rd();
            const double steer = rd();
            NMPCNavControl::Pose pose;
            pose.x = rd();
            pose.y = rd();
            pose.theta = rd();
            NMPCNavControl::Vel vel;
            vel.v = rd();
            vel.vn = rd();
            vel.w = rd();
            const int n = (int)rd();
            std::list<NMPCNavControl::Pose> traj;
            for (int j = 0; j < n; j++) {
                NMPCNavControl::Pose q;
                q.x = rd();
                q.y = rd();
                q.theta = rd();
                traj.push_back(q);
            }
            capsule_t* c = g_capsule;
            ocp_nlp_dims* d = c->nlp_dims;
            const int N = d->N, nx = d->nx, nu = d->nu, ny = d->ny;
            if (reset) w->reset_mpc();
            if (tric) tric->setSteeringWheelAngle(steer);
            std::vector<double> xb((size_t)(N + 1) * nx), ub((size_t)N * nu);
            for (int k = 0; k <= N; k++) ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, k, "x", xb.data() + (size_t)k * nx);
            for (int k = 0; k < N; k++) ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, k, "u", ub.data() + (size_t)k * nu);
            double cmd[3] = {0.0, 0.0, 0.0}, cpu_time = 0.0;
            bool ok = false;
            std::string err = "-";
            try {
                if (model == 0) {
                    NMPCNavControlDiff::CmdVelDiff cv;
                    ok = w->run(pose, vel, traj, cv, cpu_time);
                    cmd[0] = cv.v;
                    cmd[1] = cv.w;
                } else if (model == 1) {
                    NMPCNavControlOmni4::CmdVelOmni4 cv;
                    ok = w->run(pose, vel, traj, cv, cpu_time);
                    cmd[0] = cv.v;
                    cmd[1] = cv.vn;
                    cmd[2] = cv.w;
                } else {
                    NMPCNavControlTric::CmdVelTric cv;
                    ok = w->run(pose, vel, traj, cv, cpu_time);
                    cmd[0] = cv.v;
                    cmd[1] = cv.alpha;
                }
            } catch (const std::exception& e) {
                err = e.what();
                for (char& ch : err)
                    if (ch == '\n') ch = ' ';
            }
            int status = -1, qp_iter = -1;
            ocp_nlp_get(c->nlp_solver, "status", &status);
            ocp_nlp_get(c->nlp_solver, "qp_iter", &qp_iter);
            std::vector<double> x0(nx), yref((size_t)(N + 1) * ny, 0.0), WN((size_t)nx * nx), We(nx), u0(nu), x1(nx);
            ocp_nlp_constraints_model_get(c->nlp_config, d, c->nlp_in, 0, "lbx", x0.data());
            for (int k = 0; k <= N; k++) ocp_nlp_cost_model_get(c->nlp_config, d, c->nlp_in, k, "yref", yref.data() + (size_t)k * ny);
            ocp_nlp_cost_model_get(c->nlp_config, d, c->nlp_in, N, "W", WN.data());
            for (int i = 0; i < nx; i++) We[i] = WN[(size_t)i * nx + i];
            ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, 0, "u", u0.data());
            ocp_nlp_out_get(c->nlp_config, d, c->nlp_out, 1, "x", x1.data());
            std::printf("tick %d %d %d\n", ok ? 1 : 0, status, qp_iter);
            put("x0", x0.data(), x0.size());
            put("yref", yref.data(), yref.size());
            put("We", We.data(), We.size());
            put("xb", xb.data(), xb.size());
            put("ub", ub.data(), ub.size());
            put("u0", u0.data(), u0.size());
            put("x1", x1.data(), x1.size());
            put("cmd", cmd, 3);
            std::printf("err %s\n", err.c_str());
        }
        w.reset();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ref_driver: %s\n", e.what());
        return 2;
    }
    std::fflush(stdout);
    return 0;
}
