/* Included by NMPCNavControl.h:14; the wrappers use only the generic setters of ocp_nlp_interface.h. */
#ifndef NMPC_AMD_OCP_NLP_COST_LS_H
#define NMPC_AMD_OCP_NLP_COST_LS_H
#include "acados_c/ocp_nlp_interface.h"
#endif
