/* Included by NMPCNavControl.h:17; unused by the wrappers. */
#ifndef NMPC_AMD_BLASFEO_D_AUX_EXT_DEP_H
#define NMPC_AMD_BLASFEO_D_AUX_EXT_DEP_H
#endif
