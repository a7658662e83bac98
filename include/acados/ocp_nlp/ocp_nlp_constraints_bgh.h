/* Included by NMPCNavControl.h:13; the wrappers use only the generic setters of ocp_nlp_interface.h. */
#ifndef NMPC_AMD_OCP_NLP_CONSTRAINTS_BGH_H
#define NMPC_AMD_OCP_NLP_CONSTRAINTS_BGH_H
#include "acados_c/ocp_nlp_interface.h"
#endif
