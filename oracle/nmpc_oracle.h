/*
 * nmpc_oracle.h -- CPU restatement (fp64) of the reference's per-tick NMPC solve path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (nmpc_nav_control_amd/, libnmpc_amd.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference delegates the solve to acados / HPIPM / BLASFEO and
 * CasADi-generated C (external, absent from /root/reference and from this container,
 * version unpinned -- package.xml:29 has a bare <depend>acados</depend>).  No golden
 * vectors exist in the reference.  This file restates:
 *   - the model ODEs       scripts/diff/diff_amr_model.py:41-60
 *                          scripts/omni4/omni4_amr_model.py:51-73
 *                          scripts/tric/tric_amr_model.py:43-55 (incl. cos_alpha = sin(alpha), :45)
 *   - the OCP              scripts/{diff,omni4,tric}/generate_c_code.py (cost :30-39, bounds :45-60,
 *                          options :69-74: SQP_RTI, ERK, GAUSS_NEWTON, PARTIAL_CONDENSING_HPIPM)
 *   - the wrapper logic    src/nmpc_nav_control/NMPCNavControl{Diff,Omni4,Tric}.cpp (setup, run, reset)
 *   - acados semantics     SURVEY.md Appendix B (RK4 1 step + forward VDE, cost scaled by dt on
 *                          stages 0..N-1, full-step RTI around the unshifted previous iterate, ...)
 * and is pinned only by its own independent numpy cross-checks (tests/test_oracle_*.py:
 * finite-difference Jacobians, KKT certificate of every QP solution, dense KKT re-solve).
 */
#ifndef NMPC_ORACLE_H
#define NMPC_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define OC_DIFF 0
#define OC_OMNI4 1
#define OC_TRIC 2

#define OC_NXMAX 11
#define OC_NUMAX 4
#define OC_NYMAX 15
#define OC_NBMAX 8 /* bounded components per stage: nbu + nbx (omni4: 4 + 4) */
/* IPM infeasibility exit (status 4), off by default (acados / HPIPM have none): largest bound multiplier above
 * infeas_lambda (OC_INFEAS_LAMBDA: the batched device API's default) while the bound residual is above OC_INFEAS_RES
 * (the device kernel uses the same two constants) */
#define OC_INFEAS_LAMBDA 1e5
#define OC_INFEAS_RES 1e-3

typedef struct oc_params {
    int model, N;
    int nx, nu, nbx, nbu, np, ny, nyn;
    int idxbx[4], idxbu[4];
    double dt;      /* solver time step: 1/freq of the codegen yaml (common.py:6-7) */
    double dt_ctrl; /* wrapper time step: 1/control_freq of the ROS yaml (NMPCNavControlROS.cpp:82) */
    double p[3];    /* model parameters (diff: b, tau_v; omni4: l1+l2, tau_v; tric: d, tau_v, tau_a) */
    double lbx[4], ubx[4], lbu[4], ubu[4];
    double W[OC_NYMAX];   /* stage weight diagonal, [Q_diag; R_diag] (NMPCNavControlDiff.cpp:29-38) */
    double W_e[OC_NXMAX]; /* terminal weight diagonal, initialised to Q_diag (NMPCNavControlDiff.cpp:39-41) */
    int terminal_hack;    /* diff run(): W_e pose x100 if yref[N]==yref[N-1] (NMPCNavControlDiff.cpp:127-139) */
    int tric_sin_bug;     /* tric_amr_model.py:45 cos_alpha = ca.sin(alpha); 1 = reproduce */
    /* QP interior-point options (spec of this build; see DESIGN.md "QP stopping rule") */
    int iter_max;
    double tol_stat, tol_ineq, tol_comp;
    double mu0, thr0, tau;
    /* infeasibility exit: multiplier threshold infeas_lambda * max(1, w_max / 10) (w_max: the largest stage or
     * terminal weight of the QP); 0 = off (HPIPM: run to iter_max), the default. OC_INFEAS_LAMBDA restates the
     * batched device default (nmpc_model_params_default: qp_infeas_lambda 1e5). */
    double infeas_lambda;
} oc_params;

typedef struct oc_stats {
    int status;  /* 0 success, 1 NaN detected, 4 QP failure (acados codes) */
    int qp_iter; /* executed IPM iterations */
    double res_stat, res_ineq, mu;
} oc_stats;

/* Fill defaults: dims, index maps, ROS-yaml runtime values (config/nmpc_nav_control.yaml). */
void oc_params_default(int model, int N, oc_params* prm);
/* Recompute bound vectors from the scalar limits (wrapper constructors, e.g. NMPCNavControlTric.cpp:18-29). */
void oc_params_set_limits(oc_params* prm, double v_max, double a_max, double alpha_min, double alpha_max,
                          double dalpha_max);

/* Model ODE f_expl and its Jacobians (row-major Jx[nx*nx], Ju[nx*nu]). */
void oc_model_f(const oc_params* prm, const double* x, const double* u, double* f);
void oc_model_jac(const oc_params* prm, const double* x, const double* u, double* Jx, double* Ju);
/* One RK4 step (4 stages, 1 step) with forward sensitivities A = d phi/dx, B = d phi/du (may be NULL). */
void oc_rk4(const oc_params* prm, const double* x, const double* u, double h, double* xn, double* A, double* B);

/* Delta-form OCP-QP (HPIPM convention, x_0 eliminated). Row-major stage blocks. */
typedef struct oc_qp {
    int N;
    const double* A;   /* N * nx*nx */
    const double* B;   /* N * nx*nu */
    const double* b;   /* N * nx    */
    const double* Hx;  /* (N+1) * nx (stage 0 unused) */
    const double* Hu;  /* N * nu */
    const double* gx;  /* (N+1) * nx (stage 0 unused) */
    const double* gu;  /* N * nu */
    const double* lbx; /* (N+1) * nbx (stage 0 unused) */
    const double* ubx;
    const double* lbu; /* N * nbu */
    const double* ubu;
    const double* dx0; /* nx, fixed */
} oc_qp;

typedef struct oc_qp_sol {
    double* du;     /* N * nu */
    double* dx;     /* (N+1) * nx */
    double* pi;     /* (N+1) * nx, pi[k] multiplies the dynamics x_k = ..., k = 1..N */
    double* lam_lb; /* (N+1) * OC_NBMAX, per stage [u comps; x comps] */
    double* lam_ub;
    double* t_lb;
    double* t_ub;
} oc_qp_sol;

int oc_qp_ipm(const oc_params* prm, const oc_qp* qp, oc_qp_sol* sol, oc_stats* st);

/* Build the delta-form QP of one SQP-RTI iteration around (xbar, ubar). All out arrays sized as oc_qp. */
void oc_build_qp(const oc_params* prm, const double* xbar, const double* ubar, const double* x0,
                 const double* yref, const double* We, double* A, double* B, double* b, double* Hx, double* Hu,
                 double* gx, double* gu, double* lbx, double* ubx, double* lbu, double* ubu, double* dx0);

/* One SQP-RTI iteration ({name}_acados_solve, NMPCNavControlDiff.cpp:142):
 * xbar (N+1)*nx, ubar N*nu updated in place (full step) on success.
 * yref (N+1)*ny (stage N reads its first nx entries), We nx (terminal weight diagonal). */
int oc_sqp_rti(const oc_params* prm, double* xbar, double* ubar, const double* x0, const double* yref,
               const double* We, oc_stats* st);
/* Same, also returning the QP primal-dual solution (for KKT certificate tests). sol may be NULL. */
int oc_sqp_rti_ex(const oc_params* prm, double* xbar, double* ubar, const double* x0, const double* yref,
                  const double* We, oc_stats* st, oc_qp_sol* sol);

/* Iterate initialisation: after {name}_acados_create (x = ocp.constraints.x0 = [0,0,pi,0..], u = 0;
 * generate_c_code.py:58-60) and after {name}_acados_reset (all zero). */
void oc_iterate_create(const oc_params* prm, double* xbar, double* ubar);
void oc_iterate_reset(const oc_params* prm, double* xbar, double* ubar);

/* Pre-solve of run() (NMPCNavControlDiff.cpp:87-139 and Omni4/Tric equivalents):
 * pose[3], vel[3] = {v, vn, w}, steer (tric only), traj (ntraj poses x,y,theta), carried[nbx] ref states.
 * Outputs x0[nx], yref[(N+1)*ny] (entries 3..ny-1 defined as 0), We[nx]. */
void oc_prepare(const oc_params* prm, const double* pose, const double* vel, double steer, const double* traj,
                int ntraj, const double* carried, double* x0, double* yref, double* We);
/* Post-solve of run() (NMPCNavControlDiff.cpp:145-172): cmd[3] (diff v,w,0; omni4 v,vn,w; tric v,alpha,0),
 * carried_next[nbx] = x0[idxbx] + u0*dt_ctrl. */
void oc_post(const oc_params* prm, const double* x0, const double* u0, double* cmd, double* carried_next);

/* Kinematics (a8). */
void oc_direct_kinematics(const oc_params* prm, const double* vel, double steer, double* xvel /* states 3.. */);
void oc_inverse_kinematics(const oc_params* prm, const double* refs, double* cmd);

/* Full batched tick on the CPU (the timed CPU baseline): for each instance i < B, run
 * prepare -> sqp_rti -> post. Arrays are instance-major (AoS):
 *   pose[B*3], vel[B*3], steer[B] (NULL unless tric), traj[B*(N+1)*3], ntraj[B] (NULL -> N+1),
 *   reset[B] (NULL -> none), carried[B*nbx] (in/out), xbar[B*(N+1)*nx], ubar[B*N*nu] (in/out),
 *   out: cmd[B*3], u0[B*nu], status[B], qp_iter[B]. nthreads <= 0 -> OpenMP default. */
int oc_batch_tick(const oc_params* prm, int B, const double* pose, const double* vel, const double* steer,
                  const double* traj, const int* ntraj, const unsigned char* reset, double* carried, double* xbar,
                  double* ubar, double* cmd, double* u0, int* status, int* qp_iter, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
