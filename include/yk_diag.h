/*
 * yk_diag.h -- diagnostic entry points of libyk.so, kept out of the product boundary (yk.h).
 *
 * Parity harnesses (tools/gmd_step_diff.py) use these to copy the motion detector's internal
 * buffers in stream order; no product path calls them.  Same conventions as yk.h.
 */
#ifndef YK_DIAG_H_
#define YK_DIAG_H_

#include "yk.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics: device addresses of the last call's corners (float x, y [S][max_corners]), LK end
 * points (float x, y [S][max_corners]), status (uint8 [S][max_corners]) and corner counts
 * (int32 [S]), so a harness can copy them in stream order (tools/gmd_step_diff.py). */
int yk_gmd_debug_buffers(yk_gmd* g, void** dev_corners, void** dev_next, void** dev_status, int32_t** dev_ncorners,
                         int32_t* max_corners);
/* Diagnostics: the two gray-pyramid buffers (uint8 [S][per]) and Scharr-derivative buffers (int16 x, y
 * [S][per]) the calls alternate between; per = pixels of every level of one stream. */
int yk_gmd_debug_pyramids(yk_gmd* g, void** dev_pyr0, void** dev_pyr1, void** dev_der0, void** dev_der1, int64_t* per);
/* Diagnostics: captured forwards yk_detect_graph currently caches for this model, and the LRU
 * bound of that cache (tests/test_detector_gpu.py). */
int yk_model_graph_count(yk_model* m, int32_t* n_graphs, int32_t* cap);
/* Diagnostics: detector stores found outside every detector allocation so far (store-check build,
 * csrc/build.py YK_DEFINES=-DYK_STORE_CHECK=1); -1 from the product library. */
int yk_store_check_count(int64_t* out);
#ifdef __cplusplus
}
#endif

#endif /* YK_DIAG_H_ */
