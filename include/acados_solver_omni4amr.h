/*
 * acados_solver_omni4amr.h -- drop-in replacement of the acados-generated solver header for model
 * 'omni4amr' (included by include/nmpc_nav_control/NMPCNavControlOmni4.h:4; generated in the reference by
 * scripts/generate_acados_libs.py into scripts/<model>/c_generated_code/, linked as
 * libacados_ocp_solver_omni4amr.so at CMakeLists.txt:112-114).
 * Implemented by libnmpc_amd.so on the MI355X batched SQP-RTI kernels.
 *
 * The horizon is a codegen-time constant in acados, and here: tools/generate_solver_libs.py bakes OMNI4AMR_N
 * from the codegen yaml (the in-tree default follows the shipped yaml). For another horizon regenerate the
 * library from a yaml with that tf_ini / freq, or call omni4amr_acados_create_with_discretization(capsule, n,
 * steps) with n uniform time steps (as in acados, a NULL steps vector with n != OMNI4AMR_N fails).
 */
#ifndef ACADOS_SOLVER_OMNI4AMR_H_
#define ACADOS_SOLVER_OMNI4AMR_H_

#include "acados_c/ocp_nlp_interface.h"

#define OMNI4AMR_NX     11
#define OMNI4AMR_NZ     0
#define OMNI4AMR_NU     4
#define OMNI4AMR_NP     2
#define OMNI4AMR_NBX    4
#define OMNI4AMR_NBX0   11
#define OMNI4AMR_NBU    4
#define OMNI4AMR_NBXN   4
#define OMNI4AMR_NSBX   0
#define OMNI4AMR_NSBU   0
#define OMNI4AMR_NSH    0
#define OMNI4AMR_NSG    0
#define OMNI4AMR_NS     0
#define OMNI4AMR_NG     0
#define OMNI4AMR_NGN    0
#define OMNI4AMR_NH     0
#define OMNI4AMR_NHN    0
#define OMNI4AMR_NY0    15
#define OMNI4AMR_NY     15
#define OMNI4AMR_NYN    11
#ifndef OMNI4AMR_N
#define OMNI4AMR_N      80
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct omni4amr_solver_capsule {
    /* members dereferenced by the reference wrappers (e.g. NMPCNavControlDiff.cpp:50-51,146,148) */
    ocp_nlp_config* nlp_config;
    ocp_nlp_dims* nlp_dims;
    ocp_nlp_in* nlp_in;
    ocp_nlp_out* nlp_out;
    ocp_nlp_solver* nlp_solver;
    void* nlp_opts;
    /* libnmpc_amd private state */
    struct nmpc_capsule_impl* impl;
} omni4amr_solver_capsule;

omni4amr_solver_capsule* omni4amr_acados_create_capsule(void);
int omni4amr_acados_free_capsule(omni4amr_solver_capsule* capsule);
int omni4amr_acados_create(omni4amr_solver_capsule* capsule);
int omni4amr_acados_create_with_discretization(omni4amr_solver_capsule* capsule, int n_time_steps,
                                              double* new_time_steps);
int omni4amr_acados_reset(omni4amr_solver_capsule* capsule, int reset_qp_solver_mem);
int omni4amr_acados_update_params(omni4amr_solver_capsule* capsule, int stage, double* value, int np);
int omni4amr_acados_solve(omni4amr_solver_capsule* capsule);
/* Solve N_batch capsules in one device launch per parameter group; status_out[i] (may be NULL) receives
 * each capsule's status. Returns the number of capsules with a non-zero status. */
int omni4amr_acados_batch_solve(omni4amr_solver_capsule** capsules, int* status_out, int N_batch);
int omni4amr_acados_free(omni4amr_solver_capsule* capsule);
void omni4amr_acados_print_stats(omni4amr_solver_capsule* capsule);

ocp_nlp_in* omni4amr_acados_get_nlp_in(omni4amr_solver_capsule* capsule);
ocp_nlp_out* omni4amr_acados_get_nlp_out(omni4amr_solver_capsule* capsule);
ocp_nlp_solver* omni4amr_acados_get_nlp_solver(omni4amr_solver_capsule* capsule);
ocp_nlp_config* omni4amr_acados_get_nlp_config(omni4amr_solver_capsule* capsule);
void* omni4amr_acados_get_nlp_opts(omni4amr_solver_capsule* capsule);
ocp_nlp_dims* omni4amr_acados_get_nlp_dims(omni4amr_solver_capsule* capsule);

#ifdef __cplusplus
}
#endif
#endif
