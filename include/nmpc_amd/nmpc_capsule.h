/*
 * nmpc_capsule.h -- generic capsule engine behind the per-model acados solver ABI (libnmpc_amd.so), C ABI.
 *
 * acados splits a solver into the generic libacados.so (ocp_nlp_* API) and one generated
 * libacados_ocp_solver_{name}.so per model whose {name}_acados_* functions bake the codegen configuration
 * (scripts/generate_acados_libs.py:14-51 -> scripts/<geometry>/generate_c_code.py, linked at
 * CMakeLists.txt:112-114). This build keeps the split: libnmpc_amd.so holds the ocp_nlp_* API and these
 * model-generic nmpc_capsule_* functions; tools/generate_solver_libs.py turns a codegen yaml (same keys as
 * config/nmpc_nav_control_acados_models.yaml) into libacados_ocp_solver_{name}.so, whose {name}_acados_*
 * functions forward here with the baked nmpc_codegen_desc.
 */
#ifndef NMPC_AMD_NMPC_CAPSULE_H
#define NMPC_AMD_NMPC_CAPSULE_H

#include "acados_c/ocp_nlp_interface.h"

#ifdef __cplusplus
extern "C" {
#endif

/* What scripts/<geometry>/generate_c_code.py bakes into the generated solver (diff: :8-60). */
typedef struct nmpc_codegen_desc {
    int model;        /* NMPC_MODEL_* (nmpc_batch.h) */
    int N;            /* N = ceil(tf_ini / dt), dt = 1 / freq (scripts/diff/common.py:5-9) */
    double tf;        /* N * dt */
    double p[3];      /* ocp.parameter_values: diff {dist_b, tau_v}, omni4 {l1_plus_l2, tau_v},
                         tric {dist_d, tau_v, tau_a} */
    double lbx[4], ubx[4]; /* bounds of the ref states idxbx, stages 1..N (v_max; tric alpha_min/max, rad) */
    double lbu[4], ubu[4]; /* input bounds, stages 0..N-1 (a_max; tric dalpha_max, rad/s) */
    double W[15];     /* [Q_diag; R_diag] */
    double W_e[11];   /* QN_diag */
} nmpc_codegen_desc;

/* Same layout as every {name}_solver_capsule of include/acados_solver_{name}.h. */
typedef struct nmpc_solver_capsule {
    ocp_nlp_config* nlp_config;
    ocp_nlp_dims* nlp_dims;
    ocp_nlp_in* nlp_in;
    ocp_nlp_out* nlp_out;
    ocp_nlp_solver* nlp_solver;
    void* nlp_opts;
    struct nmpc_capsule_impl* impl;
} nmpc_solver_capsule;

/* The shipped codegen configuration of a model (config/nmpc_nav_control_acados_models.yaml values). */
int nmpc_codegen_default(int model, nmpc_codegen_desc* d);

nmpc_solver_capsule* nmpc_capsule_new(int model);        /* {name}_acados_create_capsule */
int nmpc_capsule_delete(nmpc_solver_capsule* capsule);   /* {name}_acados_free_capsule */
/* {name}_acados_create_with_discretization: N = n_time_steps (uniform steps tf / N; a non-NULL
 * new_time_steps must be uniform), every other default from desc (NULL: nmpc_codegen_default). */
int nmpc_capsule_create(nmpc_solver_capsule* capsule, const nmpc_codegen_desc* desc, int n_time_steps,
                        const double* new_time_steps);
int nmpc_capsule_reset(nmpc_solver_capsule* capsule, int reset_qp_solver_mem);
int nmpc_capsule_update_params(nmpc_solver_capsule* capsule, int stage, const double* value, int np);
int nmpc_capsule_solve(nmpc_solver_capsule* capsule);
/* Solve n capsules (one launch per parameter group); status_out[i] may be NULL. Returns the number of
 * capsules with a non-zero status. */
int nmpc_capsule_batch_solve(nmpc_solver_capsule** capsules, int* status_out, int n);
int nmpc_capsule_free(nmpc_solver_capsule* capsule);
void nmpc_capsule_print_stats(const nmpc_solver_capsule* capsule, const char* name);

#ifdef __cplusplus
}
#endif

#endif /* NMPC_AMD_NMPC_CAPSULE_H */
