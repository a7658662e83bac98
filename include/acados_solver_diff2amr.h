/*
 * acados_solver_diff2amr.h -- drop-in replacement of the acados-generated solver header for model
 * 'diff2amr' (included by include/nmpc_nav_control/NMPCNavControlDiff.h:4; generated in the reference by
 * scripts/generate_acados_libs.py into scripts/<model>/c_generated_code/, linked as
 * libacados_ocp_solver_diff2amr.so at CMakeLists.txt:112-114).
 * Implemented by libnmpc_amd.so on the MI355X batched SQP-RTI kernels.
 *
 * The horizon is a codegen-time constant in acados, and here: tools/generate_solver_libs.py bakes DIFF2AMR_N
 * from the codegen yaml (the in-tree default follows the shipped yaml). For another horizon regenerate the
 * library from a yaml with that tf_ini / freq, or call diff2amr_acados_create_with_discretization(capsule, n,
 * steps) with n uniform time steps (as in acados, a NULL steps vector with n != DIFF2AMR_N fails).
 */
#ifndef ACADOS_SOLVER_DIFF2AMR_H_
#define ACADOS_SOLVER_DIFF2AMR_H_

#include "acados_c/ocp_nlp_interface.h"

#define DIFF2AMR_NX     7
#define DIFF2AMR_NZ     0
#define DIFF2AMR_NU     2
#define DIFF2AMR_NP     2
#define DIFF2AMR_NBX    2
#define DIFF2AMR_NBX0   7
#define DIFF2AMR_NBU    2
#define DIFF2AMR_NBXN   2
#define DIFF2AMR_NSBX   0
#define DIFF2AMR_NSBU   0
#define DIFF2AMR_NSH    0
#define DIFF2AMR_NSG    0
#define DIFF2AMR_NS     0
#define DIFF2AMR_NG     0
#define DIFF2AMR_NGN    0
#define DIFF2AMR_NH     0
#define DIFF2AMR_NHN    0
#define DIFF2AMR_NY0    9
#define DIFF2AMR_NY     9
#define DIFF2AMR_NYN    7
#ifndef DIFF2AMR_N
#define DIFF2AMR_N      80
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct diff2amr_solver_capsule {
    /* members dereferenced by the reference wrappers (e.g. NMPCNavControlDiff.cpp:50-51,146,148) */
    ocp_nlp_config* nlp_config;
    ocp_nlp_dims* nlp_dims;
    ocp_nlp_in* nlp_in;
    ocp_nlp_out* nlp_out;
    ocp_nlp_solver* nlp_solver;
    void* nlp_opts;
    /* libnmpc_amd private state */
    struct nmpc_capsule_impl* impl;
} diff2amr_solver_capsule;

diff2amr_solver_capsule* diff2amr_acados_create_capsule(void);
int diff2amr_acados_free_capsule(diff2amr_solver_capsule* capsule);
int diff2amr_acados_create(diff2amr_solver_capsule* capsule);
int diff2amr_acados_create_with_discretization(diff2amr_solver_capsule* capsule, int n_time_steps,
                                              double* new_time_steps);
int diff2amr_acados_reset(diff2amr_solver_capsule* capsule, int reset_qp_solver_mem);
int diff2amr_acados_update_params(diff2amr_solver_capsule* capsule, int stage, double* value, int np);
int diff2amr_acados_solve(diff2amr_solver_capsule* capsule);
/* Solve N_batch capsules in one device launch per parameter group; status_out[i] (may be NULL) receives
 * each capsule's status. Returns the number of capsules with a non-zero status. */
int diff2amr_acados_batch_solve(diff2amr_solver_capsule** capsules, int* status_out, int N_batch);
int diff2amr_acados_free(diff2amr_solver_capsule* capsule);
void diff2amr_acados_print_stats(diff2amr_solver_capsule* capsule);

ocp_nlp_in* diff2amr_acados_get_nlp_in(diff2amr_solver_capsule* capsule);
ocp_nlp_out* diff2amr_acados_get_nlp_out(diff2amr_solver_capsule* capsule);
ocp_nlp_solver* diff2amr_acados_get_nlp_solver(diff2amr_solver_capsule* capsule);
ocp_nlp_config* diff2amr_acados_get_nlp_config(diff2amr_solver_capsule* capsule);
void* diff2amr_acados_get_nlp_opts(diff2amr_solver_capsule* capsule);
ocp_nlp_dims* diff2amr_acados_get_nlp_dims(diff2amr_solver_capsule* capsule);

#ifdef __cplusplus
}
#endif
#endif
