/* acados/utils/types.h -- the subset of acados' basic types used by the reference's wrappers.
 * Thin re-declaration provided by libnmpc_amd (no acados source). Return codes follow acados
 * (external): 0 success, 1 NaN, 2 max-iter, 3 min-step, 4 QP failure, 5 ready, 6 unbounded. */
#ifndef NMPC_AMD_ACADOS_UTILS_TYPES_H
#define NMPC_AMD_ACADOS_UTILS_TYPES_H
#include <stddef.h>
typedef size_t acados_size_t;
#define ACADOS_SUCCESS 0
#define ACADOS_NAN_DETECTED 1
#define ACADOS_MAXITER 2
#define ACADOS_MINSTEP 3
#define ACADOS_QP_FAILURE 4
#define ACADOS_READY 5
#define ACADOS_UNBOUNDED 6
#endif
