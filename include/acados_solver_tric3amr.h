/*
 * acados_solver_tric3amr.h -- drop-in replacement of the acados-generated solver header for model
 * 'tric3amr' (included by include/nmpc_nav_control/NMPCNavControlTric.h:4; generated in the reference by
 * scripts/generate_acados_libs.py into scripts/<model>/c_generated_code/, linked as
 * libacados_ocp_solver_tric3amr.so at CMakeLists.txt:112-114).
 * Implemented by libnmpc_amd.so on the MI355X batched SQP-RTI kernels.
 *
 * The horizon is a codegen-time constant in acados, and here: tools/generate_solver_libs.py bakes TRIC3AMR_N
 * from the codegen yaml (the in-tree default follows the shipped yaml). For another horizon regenerate the
 * library from a yaml with that tf_ini / freq, or call tric3amr_acados_create_with_discretization(capsule, n,
 * steps) with n uniform time steps (as in acados, a NULL steps vector with n != TRIC3AMR_N fails).
 */
#ifndef ACADOS_SOLVER_TRIC3AMR_H_
#define ACADOS_SOLVER_TRIC3AMR_H_

#include "acados_c/ocp_nlp_interface.h"

#define TRIC3AMR_NX     7
#define TRIC3AMR_NZ     0
#define TRIC3AMR_NU     2
#define TRIC3AMR_NP     3
#define TRIC3AMR_NBX    2
#define TRIC3AMR_NBX0   7
#define TRIC3AMR_NBU    2
#define TRIC3AMR_NBXN   2
#define TRIC3AMR_NSBX   0
#define TRIC3AMR_NSBU   0
#define TRIC3AMR_NSH    0
#define TRIC3AMR_NSG    0
#define TRIC3AMR_NS     0
#define TRIC3AMR_NG     0
#define TRIC3AMR_NGN    0
#define TRIC3AMR_NH     0
#define TRIC3AMR_NHN    0
#define TRIC3AMR_NY0    9
#define TRIC3AMR_NY     9
#define TRIC3AMR_NYN    7
#ifndef TRIC3AMR_N
#define TRIC3AMR_N      80
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tric3amr_solver_capsule {
    /* members dereferenced by the reference wrappers (e.g. NMPCNavControlDiff.cpp:50-51,146,148) */
    ocp_nlp_config* nlp_config;
    ocp_nlp_dims* nlp_dims;
    ocp_nlp_in* nlp_in;
    ocp_nlp_out* nlp_out;
    ocp_nlp_solver* nlp_solver;
    void* nlp_opts;
    /* libnmpc_amd private state */
    struct nmpc_capsule_impl* impl;
} tric3amr_solver_capsule;

tric3amr_solver_capsule* tric3amr_acados_create_capsule(void);
int tric3amr_acados_free_capsule(tric3amr_solver_capsule* capsule);
int tric3amr_acados_create(tric3amr_solver_capsule* capsule);
int tric3amr_acados_create_with_discretization(tric3amr_solver_capsule* capsule, int n_time_steps,
                                              double* new_time_steps);
int tric3amr_acados_reset(tric3amr_solver_capsule* capsule, int reset_qp_solver_mem);
int tric3amr_acados_update_params(tric3amr_solver_capsule* capsule, int stage, double* value, int np);
int tric3amr_acados_solve(tric3amr_solver_capsule* capsule);
/* Solve N_batch capsules in one device launch per parameter group; status_out[i] (may be NULL) receives
 * each capsule's status. Returns the number of capsules with a non-zero status. */
int tric3amr_acados_batch_solve(tric3amr_solver_capsule** capsules, int* status_out, int N_batch);
int tric3amr_acados_free(tric3amr_solver_capsule* capsule);
void tric3amr_acados_print_stats(tric3amr_solver_capsule* capsule);

ocp_nlp_in* tric3amr_acados_get_nlp_in(tric3amr_solver_capsule* capsule);
ocp_nlp_out* tric3amr_acados_get_nlp_out(tric3amr_solver_capsule* capsule);
ocp_nlp_solver* tric3amr_acados_get_nlp_solver(tric3amr_solver_capsule* capsule);
ocp_nlp_config* tric3amr_acados_get_nlp_config(tric3amr_solver_capsule* capsule);
void* tric3amr_acados_get_nlp_opts(tric3amr_solver_capsule* capsule);
ocp_nlp_dims* tric3amr_acados_get_nlp_dims(tric3amr_solver_capsule* capsule);

#ifdef __cplusplus
}
#endif
#endif
