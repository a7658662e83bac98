/*
 * acados_c/ocp_nlp_interface.h -- the subset of acados' generic NLP C interface that the reference's
 * wrappers call (include/nmpc_nav_control/NMPCNavControl.h:11), re-declared for libnmpc_amd.
 * Signatures follow acados >= v0.4 (7-argument constraints_model_set, 3-argument ocp_nlp_get;
 * SURVEY.md 8b). The structs are thin handles into the MI355X solve path; of their members only
 * ocp_nlp_out::inf_norm_res is read by the reference (NMPCNavControlDiff.cpp:146).
 */
#ifndef NMPC_AMD_OCP_NLP_INTERFACE_H
#define NMPC_AMD_OCP_NLP_INTERFACE_H

#include "acados/utils/types.h"

#ifdef __cplusplus
extern "C" {
#endif

struct nmpc_capsule_impl;

typedef struct ocp_nlp_config { struct nmpc_capsule_impl* impl; } ocp_nlp_config;
typedef struct ocp_nlp_dims {
    struct nmpc_capsule_impl* impl;
    int N;
    int nx, nu, ny, nyn, nbx, nbu, np;
} ocp_nlp_dims;
typedef struct ocp_nlp_in { struct nmpc_capsule_impl* impl; } ocp_nlp_in;
typedef struct ocp_nlp_out {
    struct nmpc_capsule_impl* impl;
    double inf_norm_res; /* max of the last QP's residuals at IPM exit (stationarity, bounds, complementarity);
                            not acados' NLP residual (INTEGRATION.md "Semantic differences") */
    double total_cost;
    int sqp_iter;
} ocp_nlp_out;
typedef struct ocp_nlp_solver { struct nmpc_capsule_impl* impl; } ocp_nlp_solver;
typedef struct ocp_nlp_plan_t ocp_nlp_plan_t;

/* fields: "lbx", "ubx" (stage 0: NX entries, equality x0; stages 1..N: NBX entries on idxbx),
 *         "lbu", "ubu" (stages 0..N-1: NBU entries). Values are copied. Returns 0, or < 0 on a bad field. */
int ocp_nlp_constraints_model_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, ocp_nlp_out* out,
                                  int stage, const char* field, void* value);
/* fields: "W" (col-major NY x NY at stages < N, NYN x NYN at N; must be diagonal), "yref" (NY / NYN). */
int ocp_nlp_cost_model_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                           const char* field, void* value);
/* Read back what the setters above stored (acados' ocp_nlp_constraints_model_get / ocp_nlp_cost_model_get):
 * the same fields and sizes ("W" as the full col-major block). Returns 0, or < 0 on a bad field or stage. Not
 * called by the reference's wrappers; tests/test_reference_wrappers.py reads the x0, yref and W_e the
 * reference's own run() set (NMPCNavControlDiff.cpp:96-139) through them. */
int ocp_nlp_constraints_model_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                                  const char* field, void* value);
int ocp_nlp_cost_model_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_in* in, int stage,
                           const char* field, void* value);
/* fields: "x" (NX doubles), "u" (NU doubles) of the current iterate. */
void ocp_nlp_out_get(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage, const char* field,
                     void* value);
/* fields: "x", "u": overwrite the warm-start iterate. */
void ocp_nlp_out_set(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage, const char* field,
                     void* value);
/* fields: "time_tot" (double, seconds), "time_lin", "time_qp_sol" (double), "sqp_iter", "qp_iter",
 *         "status" (int). */
void ocp_nlp_get(ocp_nlp_solver* solver, const char* field, void* return_value_);
/* Solver options (acados: ocp_nlp_solver_opts_set(config, capsule->nlp_opts, field, value)). Fields:
 *   "qp_warm_start" (int): 0 = HPIPM's cold start every solve (the reference's generated default and this
 *                   library's capsule default, scripts/diff/generate_c_code.py:68-74);
 *                   1 = acados' primal-only warm start, which starts cold here (the IPM has no separate primal
 *                   start: its primal point is always the dynamics-feasible initial iterate); 2 = primal and dual:
 *                   bound multipliers warm-started from the capsule's previous solve;
 *   "qp_iter_max"   (int >= 1): IPM iteration cap (50). Unknown fields are logged and ignored. */
void ocp_nlp_solver_opts_set(ocp_nlp_config* config, void* opts_, const char* field, void* value);
/* Dimension query: "x", "u", "y_ref" per stage (int). */
int ocp_nlp_dims_get_from_attr(ocp_nlp_config* config, ocp_nlp_dims* dims, ocp_nlp_out* out, int stage,
                               const char* field);

#ifdef __cplusplus
}
#endif
#endif
