/* Included by NMPCNavControl.h:12. The model functions (CasADi *_expl_ode_fun / *_expl_vde_forw in the
 * acados build) are compiled into libnmpc_amd's HIP kernels; no external-function objects are exposed. */
#ifndef NMPC_AMD_EXTERNAL_FUNCTION_INTERFACE_H
#define NMPC_AMD_EXTERNAL_FUNCTION_INTERFACE_H
#include "acados/utils/types.h"
#endif
