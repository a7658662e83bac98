/* acados/utils/print.h -- included by include/nmpc_nav_control/NMPCNavControl.h:10; nothing of it is used
 * by the reference's wrappers. Provided so the wrappers compile unchanged against libnmpc_amd. */
#ifndef NMPC_AMD_ACADOS_UTILS_PRINT_H
#define NMPC_AMD_ACADOS_UTILS_PRINT_H
#include "acados/utils/types.h"
#endif
