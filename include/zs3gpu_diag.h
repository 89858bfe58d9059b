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
/* 1 if zs3_encode_batch accepts this batch layout (parity_bytes = m * ShardSize),
 * 0 if it returns ZS3_ERR_INVALID_ARG for it.  Host-only: no device call, so the
 * layout rules are testable without a GPU.  (The diagnostics build also accepts
 * data_stride = parity_stride = 0, its timing-only aliased runs.) */
int zs3_debug_encode_layout_ok(const void* d_data, int64_t data_stride, int64_t block_len, int64_t n_blocks,
                               const void* d_parity, int64_t parity_stride, int64_t parity_bytes);

/* Host-side phase timers of a batching queue since its creation, microseconds summed
 * over the threads that spent them (all devices of the queue): [0] submitters' lock and
 * slot reservation (backpressure included), [1] submitters' copy-in, [2] the dispatcher's
 * launch calls, [3] the completer's wait for batches, [4] waiters' wait for results,
 * [5] copy-out, [6] sum of the batches' device stream intervals, [7] their union (device
 * busy time).  Fills us[0 .. n-1]; returns the number of timers. */
int zs3_debug_queue_timers(const zs3_queue* q, double* us, int n);

#ifdef __cplusplus
}
#endif
#endif /* ZS3GPU_DIAG_H */
