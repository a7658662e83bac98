/* Included by NMPCNavControl.h:16; unused by the wrappers (stage blocks live on the GPU). */
#ifndef NMPC_AMD_BLASFEO_D_AUX_H
#define NMPC_AMD_BLASFEO_D_AUX_H
#endif
