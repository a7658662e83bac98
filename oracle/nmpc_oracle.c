/*
 * nmpc_oracle.c -- fp64 CPU restatement of the reference's SQP-RTI solve path.
 * TEST INFRASTRUCTURE ONLY (see nmpc_oracle.h for scope, citations and the "parity unpinned" note).
 */
#include "nmpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX(r, c, ld) ((r) * (ld) + (c))

/* ------------------------------------------------------------------------------------------------ */
/* Parameters                                                                                        */
/* ------------------------------------------------------------------------------------------------ */

void oc_params_set_limits(oc_params* prm, double v_max, double a_max, double alpha_min, double alpha_max,
                          double dalpha_max)
{
    /* diff: NMPCNavControlDiff.cpp:18-22; omni4: NMPCNavControlOmni4.cpp:18-22;
     * tric: NMPCNavControlTric.cpp:18-29 (alpha bound acts on alpha_ref, idxbx = [5, 6]). */
    for (int i = 0; i < prm->nbx; i++) { prm->lbx[i] = -v_max; prm->ubx[i] = v_max; }
    for (int i = 0; i < prm->nbu; i++) { prm->lbu[i] = -a_max; prm->ubu[i] = a_max; }
    if (prm->model == OC_TRIC) {
        prm->lbx[1] = alpha_min;
        prm->ubx[1] = alpha_max;
        prm->lbu[1] = -dalpha_max;
        prm->ubu[1] = dalpha_max;
    }
}

void oc_params_default(int model, int N, oc_params* prm)
{
    memset(prm, 0, sizeof(*prm));
    prm->model = model;
    prm->N = N;
    prm->dt = 1.0 / 40.0;      /* config/nmpc_nav_control_acados_models.yaml:28 freq 40 */
    prm->dt_ctrl = 1.0 / 40.0; /* config/nmpc_nav_control.yaml:4 control_freq 40 */
    const double deg = M_PI / 180.0;
    if (model == OC_DIFF) {
        /* diff_amr_model.py:15-27, generate_c_code.py:45-55, nmpc_nav_control.yaml:28-36 */
        prm->nx = 7; prm->nu = 2; prm->nbx = 2; prm->nbu = 2; prm->np = 2;
        prm->idxbx[0] = 5; prm->idxbx[1] = 6;
        prm->idxbu[0] = 0; prm->idxbu[1] = 1;
        prm->p[0] = 0.270; prm->p[1] = 0.1;
        prm->terminal_hack = 1;
        double W[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1};
        memcpy(prm->W, W, sizeof(W));
    } else if (model == OC_OMNI4) {
        /* omni4_amr_model.py:19-33, generate_c_code.py:45-55, nmpc_nav_control.yaml:16-25
         * (yaml:22-24 misses a comma; intended values used) */
        prm->nx = 11; prm->nu = 4; prm->nbx = 4; prm->nbu = 4; prm->np = 2;
        for (int i = 0; i < 4; i++) { prm->idxbx[i] = 7 + i; prm->idxbu[i] = i; }
        prm->p[0] = 0.265 + 0.270; prm->p[1] = 0.1; /* l1 + l2, NMPCNavControlROS.cpp:97-99 */
        double W[15] = {10, 10, 5, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1};
        memcpy(prm->W, W, sizeof(W));
    } else {
        /* tric_amr_model.py:15-28, generate_c_code.py:47-57, nmpc_nav_control.yaml:39-51 */
        prm->nx = 7; prm->nu = 2; prm->nbx = 2; prm->nbu = 2; prm->np = 3;
        prm->idxbx[0] = 5; prm->idxbx[1] = 6;
        prm->idxbu[0] = 0; prm->idxbu[1] = 1;
        prm->p[0] = 0.270; prm->p[1] = 0.1; prm->p[2] = 0.5;
        prm->tric_sin_bug = 1;
        double W[9] = {10, 10, 5, 0, 0, 0, 0, 1, 1};
        memcpy(prm->W, W, sizeof(W));
    }
    prm->ny = prm->nx + prm->nu;
    prm->nyn = prm->nx;
    for (int i = 0; i < prm->nx; i++) prm->W_e[i] = prm->W[i];
    oc_params_set_limits(prm, 1.0, 1.0, -45.0 * deg, 45.0 * deg, 15.0 * deg);
    prm->iter_max = 50; /* HPIPM default iter max as used by acados */
    prm->tol_stat = 1e-8;
    prm->tol_ineq = 1e-8;
    prm->tol_comp = 1e-12;
    prm->mu0 = 1.0;
    prm->thr0 = 0.5;
    prm->tau = 0.995;
    /* acados semantics by default: HPIPM has no infeasibility exit (generate_c_code.py:69), a
     * hard QP runs to iter_max. The batched device API's early exit (nmpc_model_params.qp_infeas_lambda) is the
     * builder's own rule; a comparison against it opts in with infeas_lambda = OC_INFEAS_LAMBDA */
    prm->infeas_lambda = 0.0;
}

/* ------------------------------------------------------------------------------------------------ */
/* Models                                                                                            */
/* ------------------------------------------------------------------------------------------------ */

void oc_model_f(const oc_params* prm, const double* x, const double* u, double* f)
{
    if (prm->model == OC_DIFF) {
        /* diff_amr_model.py:42-60 */
        const double b = prm->p[0], tv = prm->p[1];
        const double v = (x[4] + x[3]) / 2.0, w = (x[4] - x[3]) / b;
        f[0] = v * cos(x[2]);
        f[1] = v * sin(x[2]);
        f[2] = w;
        f[3] = -1.0 / tv * x[3] + 1.0 / tv * x[5];
        f[4] = -1.0 / tv * x[4] + 1.0 / tv * x[6];
        f[5] = u[0];
        f[6] = u[1];
    } else if (prm->model == OC_OMNI4) {
        /* omni4_amr_model.py:52-73 */
        const double L = prm->p[0], tv = prm->p[1];
        const double v = (x[3] - x[4] + x[5] - x[6]) / 4.0;
        const double vn = (-x[3] - x[4] + x[5] + x[6]) / 4.0;
        const double w = (-x[3] - x[4] - x[5] - x[6]) / (2.0 * L);
        const double c = cos(x[2]), s = sin(x[2]);
        f[0] = v * c - vn * s;
        f[1] = v * s + vn * c;
        f[2] = w;
        for (int i = 0; i < 4; i++) f[3 + i] = -1.0 / tv * x[3 + i] + 1.0 / tv * x[7 + i];
        for (int i = 0; i < 4; i++) f[7 + i] = u[i];
    } else {
        /* tric_amr_model.py:43-55 (cos_alpha = sin(alpha) at :45 when tric_sin_bug) */
        const double d = prm->p[0], tv = prm->p[1], ta = prm->p[2];
        const double ca = prm->tric_sin_bug ? sin(x[4]) : cos(x[4]);
        const double sa = sin(x[4]);
        f[0] = x[3] * cos(x[2]) * ca;
        f[1] = x[3] * sin(x[2]) * ca;
        f[2] = x[3] / d * sa;
        f[3] = -1.0 / tv * x[3] + 1.0 / tv * x[5];
        f[4] = -1.0 / ta * x[4] + 1.0 / ta * x[6];
        f[5] = u[0];
        f[6] = u[1];
    }
}

void oc_model_jac(const oc_params* prm, const double* x, const double* u, double* Jx, double* Ju)
{
    (void)u;
    const int nx = prm->nx, nu = prm->nu;
    memset(Jx, 0, sizeof(double) * nx * nx);
    memset(Ju, 0, sizeof(double) * nx * nu);
    if (prm->model == OC_DIFF) {
        const double b = prm->p[0], tv = prm->p[1];
        const double v = (x[4] + x[3]) / 2.0, c = cos(x[2]), s = sin(x[2]);
        Jx[IDX(0, 2, nx)] = -v * s; Jx[IDX(0, 3, nx)] = 0.5 * c; Jx[IDX(0, 4, nx)] = 0.5 * c;
        Jx[IDX(1, 2, nx)] = v * c;  Jx[IDX(1, 3, nx)] = 0.5 * s; Jx[IDX(1, 4, nx)] = 0.5 * s;
        Jx[IDX(2, 3, nx)] = -1.0 / b; Jx[IDX(2, 4, nx)] = 1.0 / b;
        Jx[IDX(3, 3, nx)] = -1.0 / tv; Jx[IDX(3, 5, nx)] = 1.0 / tv;
        Jx[IDX(4, 4, nx)] = -1.0 / tv; Jx[IDX(4, 6, nx)] = 1.0 / tv;
        Ju[IDX(5, 0, nu)] = 1.0; Ju[IDX(6, 1, nu)] = 1.0;
    } else if (prm->model == OC_OMNI4) {
        const double L = prm->p[0], tv = prm->p[1];
        const double cv[4] = {0.25, -0.25, 0.25, -0.25}, cn[4] = {-0.25, -0.25, 0.25, 0.25};
        const double v = (x[3] - x[4] + x[5] - x[6]) / 4.0;
        const double vn = (-x[3] - x[4] + x[5] + x[6]) / 4.0;
        const double c = cos(x[2]), s = sin(x[2]);
        Jx[IDX(0, 2, nx)] = -v * s - vn * c;
        Jx[IDX(1, 2, nx)] = v * c - vn * s;
        for (int i = 0; i < 4; i++) {
            Jx[IDX(0, 3 + i, nx)] = cv[i] * c - cn[i] * s;
            Jx[IDX(1, 3 + i, nx)] = cv[i] * s + cn[i] * c;
            Jx[IDX(2, 3 + i, nx)] = -1.0 / (2.0 * L);
            Jx[IDX(3 + i, 3 + i, nx)] = -1.0 / tv;
            Jx[IDX(3 + i, 7 + i, nx)] = 1.0 / tv;
            Ju[IDX(7 + i, i, nu)] = 1.0;
        }
    } else {
        const double d = prm->p[0], tv = prm->p[1], ta = prm->p[2];
        const double ca = prm->tric_sin_bug ? sin(x[4]) : cos(x[4]);
        const double dca = prm->tric_sin_bug ? cos(x[4]) : -sin(x[4]);
        const double sa = sin(x[4]), dsa = cos(x[4]);
        const double c = cos(x[2]), s = sin(x[2]);
        Jx[IDX(0, 2, nx)] = -x[3] * s * ca; Jx[IDX(0, 3, nx)] = c * ca; Jx[IDX(0, 4, nx)] = x[3] * c * dca;
        Jx[IDX(1, 2, nx)] = x[3] * c * ca;  Jx[IDX(1, 3, nx)] = s * ca; Jx[IDX(1, 4, nx)] = x[3] * s * dca;
        Jx[IDX(2, 3, nx)] = sa / d; Jx[IDX(2, 4, nx)] = x[3] / d * dsa;
        Jx[IDX(3, 3, nx)] = -1.0 / tv; Jx[IDX(3, 5, nx)] = 1.0 / tv;
        Jx[IDX(4, 4, nx)] = -1.0 / ta; Jx[IDX(4, 6, nx)] = 1.0 / ta;
        Ju[IDX(5, 0, nu)] = 1.0; Ju[IDX(6, 1, nu)] = 1.0;
    }
}

/* Classic RK4 (acados ERK default: 4 stages, 1 step) with forward sensitivities: the VDE integrated with
 * the same Butcher tableau, i.e. the exact Jacobian of the discrete map. */
void oc_rk4(const oc_params* prm, const double* x, const double* u, double h, double* xn, double* A, double* B)
{
    const int nx = prm->nx, nu = prm->nu, nv = nx + nu;
    double k[4][OC_NXMAX], xs[OC_NXMAX];
    double S[OC_NXMAX * (OC_NXMAX + OC_NUMAX)];  /* d(stage input)/d[x,u], nx x nv */
    double dK[4][OC_NXMAX * (OC_NXMAX + OC_NUMAX)];
    double Jx[OC_NXMAX * OC_NXMAX], Ju[OC_NXMAX * OC_NUMAX];
    const double c[4] = {0.0, 0.5, 0.5, 1.0};
    const int sens = (A != NULL) || (B != NULL);
    for (int st = 0; st < 4; st++) {
        for (int i = 0; i < nx; i++) xs[i] = x[i] + (st ? c[st] * h * k[st - 1][i] : 0.0);
        oc_model_f(prm, xs, u, k[st]);
        if (!sens) continue;
        /* S = d xs / d[x,u] = [I 0] + c h dK[st-1] */
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nv; j++)
                S[IDX(i, j, nv)] = (i == j ? 1.0 : 0.0) + (st ? c[st] * h * dK[st - 1][IDX(i, j, nv)] : 0.0);
        oc_model_jac(prm, xs, u, Jx, Ju);
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nv; j++) {
                double acc = (j >= nx) ? Ju[IDX(i, j - nx, nu)] : 0.0;
                for (int l = 0; l < nx; l++) acc += Jx[IDX(i, l, nx)] * S[IDX(l, j, nv)];
                dK[st][IDX(i, j, nv)] = acc;
            }
    }
    for (int i = 0; i < nx; i++) xn[i] = x[i] + h / 6.0 * (k[0][i] + 2.0 * k[1][i] + 2.0 * k[2][i] + k[3][i]);
    if (!sens) return;
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < nv; j++) {
            double v = (i == j ? 1.0 : 0.0) +
                       h / 6.0 * (dK[0][IDX(i, j, nv)] + 2.0 * dK[1][IDX(i, j, nv)] + 2.0 * dK[2][IDX(i, j, nv)] +
                                  dK[3][IDX(i, j, nv)]);
            if (j < nx) { if (A) A[IDX(i, j, nx)] = v; }
            else if (B) B[IDX(i, j - nx, nu)] = v;
        }
}

/* ------------------------------------------------------------------------------------------------ */
/* QP: primal-dual interior point (Mehrotra predictor-corrector) with a Riccati recursion per Newton  */
/* system, on the N-stage OCP-QP (qp_solver_cond_N = N: no condensing).         */
/* Iterates are kept dynamics-feasible; the dynamics multipliers pi are recomputed each iteration by  */
/* the adjoint recursion so that the x-stationarity rows are zero and only the u rows carry a         */
/* residual. Same optimum as HPIPM (strictly convex QP, SURVEY Appendix B "Uniqueness").              */
/* ------------------------------------------------------------------------------------------------ */

/* max that propagates NaN (fmax drops it) */
static inline double nan_max(double a, double b) { return (b > a || b != b) ? b : a; }

typedef struct {
    int nb;               /* bounded comps at this stage */
    int var[OC_NBMAX];    /* variable index: < nu -> u[idx], else x[idx - nu] */
    double lb[OC_NBMAX], ub[OC_NBMAX];
} stage_bounds;

static inline double stage_var(const double* du, const double* dx, int nu, int v)
{
    return v < nu ? du[v] : dx[v - nu];
}

/* Cholesky of an n x n SPD matrix (row-major, lower in place). Returns 0 on failure. */
static int chol(double* M, int n)
{
    for (int j = 0; j < n; j++) {
        double d = M[IDX(j, j, n)];
        for (int k = 0; k < j; k++) d -= M[IDX(j, k, n)] * M[IDX(j, k, n)];
        if (!(d > 0.0)) return 0;
        d = sqrt(d);
        M[IDX(j, j, n)] = d;
        for (int i = j + 1; i < n; i++) {
            double s = M[IDX(i, j, n)];
            for (int k = 0; k < j; k++) s -= M[IDX(i, k, n)] * M[IDX(j, k, n)];
            M[IDX(i, j, n)] = s / d;
        }
    }
    return 1;
}

/* Solve (L L') y = r in place. */
static void chol_solve(const double* L, int n, double* r)
{
    for (int i = 0; i < n; i++) {
        double s = r[i];
        for (int k = 0; k < i; k++) s -= L[IDX(i, k, n)] * r[k];
        r[i] = s / L[IDX(i, i, n)];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = r[i];
        for (int k = i + 1; k < n; k++) s -= L[IDX(k, i, n)] * r[k];
        r[i] = s / L[IDX(i, i, n)];
    }
}

typedef struct {
    int N, nx, nu;
    double *K, *L, *kff;        /* N*nu*nx, N*nu*nu, N*nu */
    double *gu_hat, *gx_hat;    /* N*nu, (N+1)*nx */
    double *sig_u, *sig_x;      /* N*nu, (N+1)*nx diag barrier Hessian */
} ric_ws;

/* Backward Riccati. factor=1: factorise (H + Sigma) and solve; factor=0: reuse K, L for a new rhs. */
static int riccati_backward(const oc_qp* qp, ric_ws* w, int factor)
{
    const int N = w->N, nx = w->nx, nu = w->nu;
    double P[OC_NXMAX * OC_NXMAX], p[OC_NXMAX], Pn[OC_NXMAX * OC_NXMAX], pn[OC_NXMAX];
    double BP[OC_NUMAX * OC_NXMAX], AP[OC_NXMAX * OC_NXMAX], S[OC_NUMAX * OC_NXMAX];
    double R[OC_NUMAX * OC_NUMAX], r[OC_NUMAX];
    for (int i = 0; i < nx; i++) {
        for (int j = 0; j < nx; j++) P[IDX(i, j, nx)] = 0.0;
        P[IDX(i, i, nx)] = qp->Hx[N * nx + i] + w->sig_x[N * nx + i];
        p[i] = w->gx_hat[N * nx + i];
    }
    for (int k = N - 1; k >= 0; k--) {
        const double* A = qp->A + k * nx * nx;
        const double* B = qp->B + k * nx * nu;
        double* K = w->K + k * nu * nx;
        double* L = w->L + k * nu * nu;
        double* kff = w->kff + k * nu;
        /* r~ = g^u + B' p */
        for (int i = 0; i < nu; i++) {
            double s = w->gu_hat[k * nu + i];
            for (int l = 0; l < nx; l++) s += B[IDX(l, i, nu)] * p[l];
            r[i] = s;
        }
        if (factor) {
            for (int i = 0; i < nu; i++)
                for (int j = 0; j < nx; j++) {
                    double s = 0.0;
                    for (int l = 0; l < nx; l++) s += B[IDX(l, i, nu)] * P[IDX(l, j, nx)];
                    BP[IDX(i, j, nx)] = s;
                }
            for (int i = 0; i < nu; i++)
                for (int j = 0; j < nu; j++) {
                    double s = (i == j) ? qp->Hu[k * nu + i] + w->sig_u[k * nu + i] : 0.0;
                    for (int l = 0; l < nx; l++) s += BP[IDX(i, l, nx)] * B[IDX(l, j, nu)];
                    R[IDX(i, j, nu)] = s;
                }
            for (int i = 0; i < nu; i++)
                for (int j = 0; j < i; j++) {
                    double s = 0.5 * (R[IDX(i, j, nu)] + R[IDX(j, i, nu)]);
                    R[IDX(i, j, nu)] = R[IDX(j, i, nu)] = s;
                }
            if (!chol(R, nu)) return 0;
            memcpy(L, R, sizeof(double) * nu * nu);
        }
        for (int i = 0; i < nu; i++) kff[i] = -r[i];
        chol_solve(L, nu, kff);
        if (k == 0) break;
        if (factor) {
            /* S~ = B'PA, Q~ = diag(Hx + Sig) + A'PA, K = -R~^{-1} S~, P_k = Q~ + S~' K */
            for (int i = 0; i < nu; i++)
                for (int j = 0; j < nx; j++) {
                    double s = 0.0;
                    for (int l = 0; l < nx; l++) s += BP[IDX(i, l, nx)] * A[IDX(l, j, nx)];
                    S[IDX(i, j, nx)] = s;
                }
            for (int j = 0; j < nx; j++) {
                double col[OC_NUMAX];
                for (int i = 0; i < nu; i++) col[i] = -S[IDX(i, j, nx)];
                chol_solve(L, nu, col);
                for (int i = 0; i < nu; i++) K[IDX(i, j, nx)] = col[i];
            }
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < nx; j++) {
                    double s = 0.0;
                    for (int l = 0; l < nx; l++) s += A[IDX(l, i, nx)] * P[IDX(l, j, nx)];
                    AP[IDX(i, j, nx)] = s;
                }
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < nx; j++) {
                    double s = (i == j) ? qp->Hx[k * nx + i] + w->sig_x[k * nx + i] : 0.0;
                    for (int l = 0; l < nx; l++) s += AP[IDX(i, l, nx)] * A[IDX(l, j, nx)];
                    for (int l = 0; l < nu; l++) s += S[IDX(l, i, nx)] * K[IDX(l, j, nx)];
                    Pn[IDX(i, j, nx)] = s;
                }
            for (int i = 0; i < nx; i++)
                for (int j = 0; j <= i; j++) {
                    double s = 0.5 * (Pn[IDX(i, j, nx)] + Pn[IDX(j, i, nx)]);
                    P[IDX(i, j, nx)] = P[IDX(j, i, nx)] = s;
                }
        }
        /* p_k = g^x + A' p_{k+1} + K' r~ */
        for (int i = 0; i < nx; i++) {
            double s = w->gx_hat[k * nx + i];
            for (int l = 0; l < nx; l++) s += A[IDX(l, i, nx)] * p[l];
            for (int l = 0; l < nu; l++) s += K[IDX(l, i, nx)] * r[l];
            pn[i] = s;
        }
        memcpy(p, pn, sizeof(double) * nx);
    }
    return 1;
}

static void riccati_forward(const oc_qp* qp, const ric_ws* w, double* Ddu, double* Ddx)
{
    const int N = w->N, nx = w->nx, nu = w->nu;
    for (int i = 0; i < nx; i++) Ddx[i] = 0.0;
    for (int k = 0; k < N; k++) {
        const double* A = qp->A + k * nx * nx;
        const double* B = qp->B + k * nx * nu;
        const double* K = w->K + k * nu * nx;
        for (int i = 0; i < nu; i++) {
            double s = w->kff[k * nu + i];
            if (k > 0)
                for (int j = 0; j < nx; j++) s += K[IDX(i, j, nx)] * Ddx[k * nx + j];
            Ddu[k * nu + i] = s;
        }
        for (int i = 0; i < nx; i++) {
            double s = 0.0;
            for (int j = 0; j < nx; j++) s += A[IDX(i, j, nx)] * Ddx[k * nx + j];
            for (int j = 0; j < nu; j++) s += B[IDX(i, j, nu)] * Ddu[k * nu + j];
            Ddx[(k + 1) * nx + i] = s;
        }
    }
}

int oc_qp_ipm(const oc_params* prm, const oc_qp* qp, oc_qp_sol* sol, oc_stats* st)
{
    const int N = qp->N, nx = prm->nx, nu = prm->nu, NB = OC_NBMAX;
    stage_bounds* sb = (stage_bounds*)calloc(N + 1, sizeof(stage_bounds));
    int m = 0;
    for (int k = 0; k <= N; k++) {
        int c = 0;
        if (k < N)
            for (int i = 0; i < prm->nbu; i++, c++) {
                sb[k].var[c] = prm->idxbu[i];
                sb[k].lb[c] = qp->lbu[k * prm->nbu + i];
                sb[k].ub[c] = qp->ubu[k * prm->nbu + i];
            }
        if (k >= 1)
            for (int i = 0; i < prm->nbx; i++, c++) {
                sb[k].var[c] = nu + prm->idxbx[i];
                sb[k].lb[c] = qp->lbx[k * prm->nbx + i];
                sb[k].ub[c] = qp->ubx[k * prm->nbx + i];
            }
        sb[k].nb = c;
        m += c;
    }
    const double m2 = 2.0 * m;
    /* infeasibility threshold: infeas_lambda scaled by the largest stage / terminal weight (0: no such exit) */
    double wmax = 0.0;
    for (int i = 0; i < prm->ny; i++) wmax = fmax(wmax, prm->W[i]);
    for (int i = 0; i < nx; i++) wmax = fmax(wmax, qp->Hx[N * nx + i]);
    const double lam_thr = prm->infeas_lambda > 0.0 ? prm->infeas_lambda * fmax(1.0, 0.1 * wmax) : INFINITY;

    double* buf = (double*)calloc((size_t)(N + 1) * (4 * nx + 4 * nu + 4 * NB) + (size_t)N * (nu * nx + nu * nu + nu),
                                  sizeof(double));
    double* q = buf;
    ric_ws w;
    w.N = N; w.nx = nx; w.nu = nu;
    w.K = q; q += N * nu * nx;
    w.L = q; q += N * nu * nu;
    w.kff = q; q += N * nu;
    w.gu_hat = q; q += (N + 1) * nu;
    w.gx_hat = q; q += (N + 1) * nx;
    w.sig_u = q; q += (N + 1) * nu;
    w.sig_x = q; q += (N + 1) * nx;
    double* Ddu = q; q += (N + 1) * nu;
    double* Ddx = q; q += (N + 1) * nx;
    double* ru = q; q += (N + 1) * nu;
    double* pi = q; q += (N + 1) * nx;
    double* Dt_l = q; q += (N + 1) * NB;  /* affine Delta t / Delta lambda, reused for the corrector term */
    double* Dt_u = q; q += (N + 1) * NB;
    double* Dl_l = q; q += (N + 1) * NB;
    double* Dl_u = q; q += (N + 1) * NB;

    double *du = sol->du, *dx = sol->dx;
    double *tl = sol->t_lb, *tu = sol->t_ub, *ll = sol->lam_lb, *lu = sol->lam_ub;

    /* Initial point: du = 0, dx from the dynamics (feasible), slacks clipped at thr0, lambda = mu0 / t. */
    for (int i = 0; i < N * nu; i++) du[i] = 0.0;
    for (int i = 0; i < nx; i++) dx[i] = qp->dx0[i];
    for (int k = 0; k < N; k++)
        for (int i = 0; i < nx; i++) {
            double s = qp->b[k * nx + i];
            for (int j = 0; j < nx; j++) s += qp->A[k * nx * nx + IDX(i, j, nx)] * dx[k * nx + j];
            dx[(k + 1) * nx + i] = s;
        }
    for (int k = 0; k <= N; k++)
        for (int c = 0; c < sb[k].nb; c++) {
            const double z = stage_var(du + k * nu, dx + k * nx, nu, sb[k].var[c]);
            tl[k * NB + c] = fmax(z - sb[k].lb[c], prm->thr0);
            tu[k * NB + c] = fmax(sb[k].ub[c] - z, prm->thr0);
            ll[k * NB + c] = prm->mu0 / tl[k * NB + c];
            lu[k * NB + c] = prm->mu0 / tu[k * NB + c];
        }

    int status = 4, it = 0;
    double res_stat = 0.0, res_ineq = 0.0, mu = 0.0;
    const int verbose = getenv("OC_VERBOSE") != NULL;
    for (it = 0;; it++) {
        /* residuals: adjoint recursion for pi, u-stationarity, inequality residuals, mu */
        res_ineq = 0.0;
        double sum_c = 0.0, lam_max = 0.0;
        for (int k = 0; k <= N; k++)
            for (int c = 0; c < sb[k].nb; c++) {
                const double z = stage_var(du + k * nu, dx + k * nx, nu, sb[k].var[c]);
                const double rl = z - sb[k].lb[c] - tl[k * NB + c];
                const double rr = sb[k].ub[c] - z - tu[k * NB + c];
                res_ineq = nan_max(res_ineq, fmax(fabs(rl), fabs(rr)));
                sum_c += ll[k * NB + c] * tl[k * NB + c] + lu[k * NB + c] * tu[k * NB + c];
                lam_max = fmax(lam_max, fmax(ll[k * NB + c], lu[k * NB + c]));
            }
        mu = (m > 0) ? sum_c / m2 : 0.0;
        for (int k = N; k >= 1; k--) {
            for (int i = 0; i < nx; i++) {
                double s = qp->Hx[k * nx + i] * dx[k * nx + i] + qp->gx[k * nx + i];
                if (k < N)
                    for (int l = 0; l < nx; l++) s += qp->A[k * nx * nx + IDX(l, i, nx)] * pi[(k + 1) * nx + l];
                pi[k * nx + i] = s;
            }
            for (int c = 0; c < sb[k].nb; c++)
                if (sb[k].var[c] >= nu) pi[k * nx + sb[k].var[c] - nu] -= ll[k * NB + c] - lu[k * NB + c];
        }
        res_stat = 0.0;
        for (int k = 0; k < N; k++) {
            for (int i = 0; i < nu; i++) {
                double s = qp->Hu[k * nu + i] * du[k * nu + i] + qp->gu[k * nu + i];
                for (int l = 0; l < nx; l++) s += qp->B[k * nx * nu + IDX(l, i, nu)] * pi[(k + 1) * nx + l];
                ru[k * nu + i] = s;
            }
            for (int c = 0; c < sb[k].nb; c++)
                if (sb[k].var[c] < nu) ru[k * nu + sb[k].var[c]] -= ll[k * NB + c] - lu[k * NB + c];
            for (int i = 0; i < nu; i++) res_stat = nan_max(res_stat, fabs(ru[k * nu + i]));
        }
        if (!(res_stat == res_stat) || !(mu == mu)) { status = 1; break; }
        if (res_ineq <= prm->tol_ineq && ((res_stat <= prm->tol_stat && mu <= prm->tol_comp) || mu <= 1e-2 * prm->tol_comp)) {
            status = 0;
            break;
        }
        /* primal infeasibility: the bound multipliers diverge while the bound residual cannot close (a feasible
         * QP of this OCP keeps them at the size of its cost weights: max 88 over 768 bench-loop QPs against > 1e5
         * by iteration 13-20 of the infeasible ones, tools/infeas_study.py) -> QP failure, the status the
         * wrapper turns into an exception (NMPCNavControl.cpp:14-23) */
        if (lam_max > lam_thr && res_ineq > OC_INFEAS_RES) { status = 4; break; }
        if (it >= prm->iter_max) { status = 0; break; } /* max-iter tolerated in RTI */

        /* Newton solves sharing one factorisation: pass 0 predictor (affine, target 0); pass 1 Mehrotra
         * corrector, target sigma*mu - alpha_aff * dlam_aff * dt_aff (second-order term damped by the affine
         * step); pass 2 only if the corrector step is shorter than 0.1: a pure centring step with target
         * max(sigma, 0.3)*mu (safeguard against Mehrotra jamming, DESIGN.md "QP algorithm"). */
        double sigma = 0.0, alpha_aff = 1.0, alpha = 1.0;
        for (int pass = 0; pass < 3; pass++) {
            if (pass == 2 && alpha >= 0.1) break;
            const double tgt = (pass == 0) ? 0.0 : (pass == 1 ? sigma * mu : fmax(sigma, 0.3) * mu);
            const double eta = (pass == 1) ? alpha_aff : 0.0;
            /* rhs: g^ = r_z - (tgt_l - lam_l r_l)/t_l + lam_l + (tgt_u - lam_u r_u)/t_u - lam_u */
            for (int k = 0; k <= N; k++) {
                for (int i = 0; i < nu; i++) {
                    w.gu_hat[k * nu + i] = (k < N) ? ru[k * nu + i] : 0.0;
                    w.sig_u[k * nu + i] = 0.0;
                }
                for (int i = 0; i < nx; i++) { w.gx_hat[k * nx + i] = 0.0; w.sig_x[k * nx + i] = 0.0; }
                for (int c = 0; c < sb[k].nb; c++) {
                    const int j = k * NB + c;
                    const double z = stage_var(du + k * nu, dx + k * nx, nu, sb[k].var[c]);
                    const double rl = z - sb[k].lb[c] - tl[j];
                    const double rr = sb[k].ub[c] - z - tu[j];
                    const double tg_l = tgt - eta * Dl_l[j] * Dt_l[j], tg_u = tgt - eta * Dl_u[j] * Dt_u[j];
                    const double gh = -(tg_l - ll[j] * rl) / tl[j] + ll[j] + (tg_u - lu[j] * rr) / tu[j] - lu[j];
                    const double sg = ll[j] / tl[j] + lu[j] / tu[j];
                    const int v = sb[k].var[c];
                    if (v < nu) { w.gu_hat[k * nu + v] += gh; w.sig_u[k * nu + v] += sg; }
                    else { w.gx_hat[k * nx + v - nu] += gh; w.sig_x[k * nx + v - nu] += sg; }
                }
            }
            if (!riccati_backward(qp, &w, pass == 0)) { status = 4; goto done; }
            riccati_forward(qp, &w, Ddu, Ddx);
            /* Delta t, Delta lambda and the maximal step */
            double amax = 1e30;
            for (int k = 0; k <= N; k++)
                for (int c = 0; c < sb[k].nb; c++) {
                    const int j = k * NB + c;
                    const double z = stage_var(du + k * nu, dx + k * nx, nu, sb[k].var[c]);
                    const double dz = stage_var(Ddu + k * nu, Ddx + k * nx, nu, sb[k].var[c]);
                    const double rl = z - sb[k].lb[c] - tl[j];
                    const double rr = sb[k].ub[c] - z - tu[j];
                    const double tg_l = tgt - eta * Dl_l[j] * Dt_l[j], tg_u = tgt - eta * Dl_u[j] * Dt_u[j];
                    const double dtl = dz + rl, dtu = -dz + rr;
                    const double dll = (tg_l - ll[j] * (tl[j] + rl) - ll[j] * dz) / tl[j];
                    const double dlu = (tg_u - lu[j] * (tu[j] + rr) + lu[j] * dz) / tu[j];
                    if (dtl < 0.0) amax = fmin(amax, -tl[j] / dtl);
                    if (dtu < 0.0) amax = fmin(amax, -tu[j] / dtu);
                    if (dll < 0.0) amax = fmin(amax, -ll[j] / dll);
                    if (dlu < 0.0) amax = fmin(amax, -lu[j] / dlu);
                    Dt_l[j] = dtl; Dt_u[j] = dtu; Dl_l[j] = dll; Dl_u[j] = dlu;
                }
            if (pass == 0) {
                alpha_aff = fmin(1.0, amax);
                const double a = alpha_aff;
                double s = 0.0;
                for (int k = 0; k <= N; k++)
                    for (int c = 0; c < sb[k].nb; c++) {
                        const int j = k * NB + c;
                        s += (ll[j] + a * Dl_l[j]) * (tl[j] + a * Dt_l[j]) + (lu[j] + a * Dl_u[j]) * (tu[j] + a * Dt_u[j]);
                    }
                const double mu_aff = (m > 0) ? s / m2 : 0.0;
                double sig = (mu > 0.0) ? mu_aff / mu : 0.0;
                sig = sig * sig * sig;
                sigma = fmin(fmax(sig, 0.0), 1.0);
                if (verbose) fprintf(stderr, "it %d mu %.3e res_stat %.2e res_ineq %.2e alpha_aff %.3e sigma %.3e\n", it, mu, res_stat, res_ineq, a, sigma);
            } else {
                alpha = fmin(1.0, prm->tau * amax);
                if (verbose) fprintf(stderr, "   pass %d alpha %.3e\n", pass, alpha);
            }
        }
        /* update (the corrector pass left the combined direction in Ddu/Ddx/Dt/Dl) */
        for (int i = 0; i < N * nu; i++) du[i] += alpha * Ddu[i];
        for (int i = nx; i < (N + 1) * nx; i++) dx[i] += alpha * Ddx[i];
        for (int k = 0; k <= N; k++)
            for (int c = 0; c < sb[k].nb; c++) {
                const int j = k * NB + c;
                tl[j] += alpha * Dt_l[j];
                tu[j] += alpha * Dt_u[j];
                ll[j] += alpha * Dl_l[j];
                lu[j] += alpha * Dl_u[j];
            }
    }
done:
    if (sol->pi) memcpy(sol->pi, pi, sizeof(double) * (N + 1) * nx);
    if (st) {
        st->status = status;
        st->qp_iter = it;
        st->res_stat = res_stat;
        st->res_ineq = res_ineq;
        st->mu = mu;
    }
    free(buf);
    free(sb);
    return status;
}

/* ------------------------------------------------------------------------------------------------ */
/* SQP-RTI                                                                                           */
/* ------------------------------------------------------------------------------------------------ */

void oc_build_qp(const oc_params* prm, const double* xbar, const double* ubar, const double* x0,
                 const double* yref, const double* We, double* A, double* B, double* b, double* Hx, double* Hu,
                 double* gx, double* gu, double* lbx, double* ubx, double* lbu, double* ubu, double* dx0)
{
    const int N = prm->N, nx = prm->nx, nu = prm->nu, ny = prm->ny;
    const double s = prm->dt; /* cost_scaling: time step on stages 0..N-1, 1 at N */
    for (int k = 0; k < N; k++) {
        double xn[OC_NXMAX];
        oc_rk4(prm, xbar + k * nx, ubar + k * nu, prm->dt, xn, A + k * nx * nx, B + k * nx * nu);
        for (int i = 0; i < nx; i++) b[k * nx + i] = xn[i] - xbar[(k + 1) * nx + i];
        /* NONLINEAR_LS with y = [x; u]: Gauss-Newton Hessian W, gradient W (y - yref) (generate_c_code.py:30-39) */
        for (int i = 0; i < nu; i++) {
            Hu[k * nu + i] = s * prm->W[nx + i];
            gu[k * nu + i] = s * prm->W[nx + i] * (ubar[k * nu + i] - yref[k * ny + nx + i]);
        }
        for (int i = 0; i < nx; i++) {
            Hx[k * nx + i] = s * prm->W[i];
            gx[k * nx + i] = s * prm->W[i] * (xbar[k * nx + i] - yref[k * ny + i]);
        }
        for (int i = 0; i < prm->nbu; i++) {
            lbu[k * prm->nbu + i] = prm->lbu[i] - ubar[k * nu + prm->idxbu[i]];
            ubu[k * prm->nbu + i] = prm->ubu[i] - ubar[k * nu + prm->idxbu[i]];
        }
    }
    for (int i = 0; i < nx; i++) {
        Hx[N * nx + i] = We[i];
        gx[N * nx + i] = We[i] * (xbar[N * nx + i] - yref[N * ny + i]);
    }
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < prm->nbx; i++) {
            lbx[k * prm->nbx + i] = prm->lbx[i] - xbar[k * nx + prm->idxbx[i]];
            ubx[k * prm->nbx + i] = prm->ubx[i] - xbar[k * nx + prm->idxbx[i]];
        }
    for (int i = 0; i < nx; i++) dx0[i] = x0[i] - xbar[i];
}

int oc_sqp_rti_ex(const oc_params* prm, double* xbar, double* ubar, const double* x0, const double* yref,
                  const double* We, oc_stats* st, oc_qp_sol* solx)
{
    const int N = prm->N, nx = prm->nx, nu = prm->nu, nbx = prm->nbx, nbu = prm->nbu, NB = OC_NBMAX;
    size_t sz = (size_t)N * (nx * nx + nx * nu + nx + nu + nu + 2 * nbu) + (size_t)(N + 1) * (2 * nx + 2 * nbx) + nx;
    double* buf = (double*)calloc(sz, sizeof(double));
    double* q = buf;
    double *A = q; q += N * nx * nx;
    double *B = q; q += N * nx * nu;
    double *b = q; q += N * nx;
    double *Hu = q; q += N * nu;
    double *gu = q; q += N * nu;
    double *lbu = q; q += N * nbu;
    double *ubu = q; q += N * nbu;
    double *Hx = q; q += (N + 1) * nx;
    double *gx = q; q += (N + 1) * nx;
    double *lbx = q; q += (N + 1) * nbx;
    double *ubx = q; q += (N + 1) * nbx;
    double *dx0 = q;
    oc_build_qp(prm, xbar, ubar, x0, yref, We, A, B, b, Hx, Hu, gx, gu, lbx, ubx, lbu, ubu, dx0);
    oc_qp qp = {N, A, B, b, Hx, Hu, gx, gu, lbx, ubx, lbu, ubu, dx0};

    double* sbuf = NULL;
    oc_qp_sol sol;
    if (solx) sol = *solx;
    else {
        sbuf = (double*)calloc((size_t)N * nu + (size_t)(N + 1) * (2 * nx + 4 * NB), sizeof(double));
        double* r = sbuf;
        sol.du = r; r += N * nu;
        sol.dx = r; r += (N + 1) * nx;
        sol.pi = r; r += (N + 1) * nx;
        sol.lam_lb = r; r += (N + 1) * NB;
        sol.lam_ub = r; r += (N + 1) * NB;
        sol.t_lb = r; r += (N + 1) * NB;
        sol.t_ub = r;
    }
    oc_stats s0;
    int status = oc_qp_ipm(prm, &qp, &sol, &s0);
    if (status == 0) {
        for (int i = 0; i < (N + 1) * nx; i++) xbar[i] += sol.dx[i];
        for (int i = 0; i < N * nu; i++) ubar[i] += sol.du[i];
    }
    if (st) *st = s0;
    free(sbuf);
    free(buf);
    return status;
}

int oc_sqp_rti(const oc_params* prm, double* xbar, double* ubar, const double* x0, const double* yref,
               const double* We, oc_stats* st)
{
    return oc_sqp_rti_ex(prm, xbar, ubar, x0, yref, We, st, NULL);
}

void oc_iterate_create(const oc_params* prm, double* xbar, double* ubar)
{
    const int N = prm->N, nx = prm->nx, nu = prm->nu;
    for (int k = 0; k <= N; k++)
        for (int i = 0; i < nx; i++) xbar[k * nx + i] = (i == 2) ? M_PI : 0.0; /* generate_c_code.py:58-60 */
    for (int i = 0; i < N * nu; i++) ubar[i] = 0.0;
}

void oc_iterate_reset(const oc_params* prm, double* xbar, double* ubar)
{
    memset(xbar, 0, sizeof(double) * (prm->N + 1) * prm->nx);
    memset(ubar, 0, sizeof(double) * prm->N * prm->nu);
}

/* ------------------------------------------------------------------------------------------------ */
/* Wrapper pre/post (L3)                                                                             */
/* ------------------------------------------------------------------------------------------------ */

static double unwrap_angle(double current, double previous)
{
    /* NMPCNavControl.cpp:25-31 */
    double delta = current - previous;
    if (delta > M_PI) current -= 2 * M_PI;
    else if (delta < -M_PI) current += 2 * M_PI;
    return current;
}

void oc_direct_kinematics(const oc_params* prm, const double* vel, double steer, double* xv)
{
    if (prm->model == OC_DIFF) {
        /* NMPCNavControlDiff.cpp:183-187 */
        xv[0] = vel[0] - 0.5 * prm->p[0] * vel[2];
        xv[1] = vel[0] + 0.5 * prm->p[0] * vel[2];
    } else if (prm->model == OC_OMNI4) {
        /* NMPCNavControlOmni4.cpp:185-192 */
        const double hl = 0.5 * prm->p[0] * vel[2];
        xv[0] = vel[0] - vel[1] - hl;
        xv[1] = -vel[0] - vel[1] - hl;
        xv[2] = vel[0] + vel[1] - hl;
        xv[3] = -vel[0] + vel[1] - hl;
    } else {
        /* NMPCNavControlTric.cpp:97-98 */
        xv[0] = vel[0];
        xv[1] = steer;
    }
}

void oc_inverse_kinematics(const oc_params* prm, const double* r, double* cmd)
{
    if (prm->model == OC_DIFF) {
        /* NMPCNavControlDiff.cpp:189-193 */
        cmd[0] = (r[1] + r[0]) / 2.0;
        cmd[1] = (r[1] - r[0]) / prm->p[0];
        cmd[2] = 0.0;
    } else if (prm->model == OC_OMNI4) {
        /* NMPCNavControlOmni4.cpp:194-200 */
        cmd[0] = (r[0] - r[1] + r[2] - r[3]) / 4.0;
        cmd[1] = (-r[0] - r[1] + r[2] + r[3]) / 4.0;
        cmd[2] = (-r[0] - r[1] - r[2] - r[3]) / (2.0 * prm->p[0]);
    } else {
        /* NMPCNavControlTric.cpp:161-162 */
        cmd[0] = r[0];
        cmd[1] = r[1];
        cmd[2] = 0.0;
    }
}

void oc_prepare(const oc_params* prm, const double* pose, const double* vel, double steer, const double* traj,
                int ntraj, const double* carried, double* x0, double* yref, double* We)
{
    const int N = prm->N, nx = prm->nx, ny = prm->ny;
    /* x0: pose, velocity states from the kinematics, carried vel-ref states (NMPCNavControlDiff.cpp:87-94) */
    x0[0] = pose[0]; x0[1] = pose[1]; x0[2] = pose[2];
    oc_direct_kinematics(prm, vel, steer, x0 + 3);
    for (int i = 0; i < prm->nbx; i++) x0[prm->idxbx[i]] = carried[i];
    /* yref: unwrap against the previous entry, pad with the last pose (NMPCNavControlDiff.cpp:104-118) */
    double prev = pose[2];
    for (int k = 0; k <= N; k++) {
        double* y = yref + k * ny;
        for (int i = 0; i < ny; i++) y[i] = 0.0; /* entries 3..ny-1 never written by the wrapper: defined 0 */
        if (k < ntraj) {
            y[0] = traj[3 * k + 0];
            y[1] = traj[3 * k + 1];
            y[2] = unwrap_angle(traj[3 * k + 2], prev);
            prev = y[2];
        } else {
            y[0] = yref[(k - 1) * ny + 0];
            y[1] = yref[(k - 1) * ny + 1];
            y[2] = yref[(k - 1) * ny + 2];
        }
    }
    for (int i = 0; i < nx; i++) We[i] = prm->W_e[i];
    if (prm->terminal_hack) {
        /* NMPCNavControlDiff.cpp:127-139 */
        const double* a = yref + N * ny;
        const double* b = yref + (N - 1) * ny;
        const int eq = (a[0] == b[0]) && (a[1] == b[1]) && (a[2] == b[2]);
        for (int i = 0; i < 3; i++) We[i] = eq ? 100.0 * prm->W[i] : prm->W[i];
    }
}

void oc_post(const oc_params* prm, const double* x0, const double* u0, double* cmd, double* carried_next)
{
    /* vel_ref_new = x0[ref] + u0 * dt (NMPCNavControlDiff.cpp:155-157), cmd by inverse kinematics (:165),
     * carried into the next x0 (:168-172). idxbx lists the ref states, idxbu the matching inputs. */
    double r[4];
    for (int i = 0; i < prm->nbx; i++) r[i] = x0[prm->idxbx[i]] + u0[i] * prm->dt_ctrl;
    oc_inverse_kinematics(prm, r, cmd);
    for (int i = 0; i < prm->nbx; i++) carried_next[i] = r[i];
}

int oc_batch_tick(const oc_params* prm, int B, const double* pose, const double* vel, const double* steer,
                  const double* traj, const int* ntraj, const unsigned char* reset, double* carried, double* xbar,
                  double* ubar, double* cmd, double* u0, int* status, int* qp_iter, int nthreads)
{
    const int N = prm->N, nx = prm->nx, nu = prm->nu, ny = prm->ny, nbx = prm->nbx;
    int nfail = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : nfail)
#endif
    for (int i = 0; i < B; i++) {
        double x0[OC_NXMAX], We[OC_NXMAX], c[3];
        double* yref = (double*)malloc(sizeof(double) * (N + 1) * ny);
        double* xb = xbar + (size_t)i * (N + 1) * nx;
        double* ub = ubar + (size_t)i * N * nu;
        if (reset && reset[i]) oc_iterate_reset(prm, xb, ub);
        oc_prepare(prm, pose + 3 * i, vel + 3 * i, steer ? steer[i] : 0.0, traj + (size_t)i * (N + 1) * 3,
                   ntraj ? ntraj[i] : N + 1, carried + (size_t)i * nbx, x0, yref, We);
        oc_stats st;
        int s = oc_sqp_rti(prm, xb, ub, x0, yref, We, &st);
        status[i] = s;
        if (qp_iter) qp_iter[i] = st.qp_iter;
        if (s == 0) {
            oc_post(prm, x0, ub, c, carried + (size_t)i * nbx);
            for (int j = 0; j < 3; j++) cmd[3 * i + j] = c[j];
            for (int j = 0; j < nu; j++) u0[i * nu + j] = ub[j];
        } else {
            nfail++;
        }
        free(yref);
    }
    return nfail;
}
