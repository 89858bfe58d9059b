/*
 * zs3gpu_diag.h — diagnostics-only entry points of libzs3gpu_diag.so.
 *
 * The product library (libzs3gpu.so) compiles only the tuned default kernels and
 * the generic fallbacks and exports none of these.  The diagnostics build
 * (ZS3_DIAG=1) adds the experimental kernel variants used by the A/B scripts and the
 * variant parity tests.  Settings are per OS thread: concurrent callers never see
 * each other's choice.
 */
#ifndef ZS3GPU_DIAG_H
#define ZS3GPU_DIAG_H

#include "zs3gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Select an experimental variant of the fused kernels for the calling thread
 * (0 = tuned default; +1000 = same variant with the plain non-dyadic encode). */
int zs3_debug_set_variant(int variant);
/* Device buffer receiving per-wave stamps from the stamped variants (NULL = off),
 * for the calling thread. */
int zs3_debug_set_buffer(void* d_dbg);

#ifdef __cplusplus
}
#endif
#endif /* ZS3GPU_DIAG_H */
