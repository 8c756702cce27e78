/* A C host on the C ABI alone: engine file -> detector, then the tracker, for one batch of
 * frames already in device memory.  Build:
 *   gcc -O2 -I include examples/c_host.c -L yolo---small-target-recognition---kalman-trajectory-prediction_amd \
 *       -lyk -Wl,--unresolved-symbols=ignore-in-shared-libs -o c_host
 * (libyk.so resolves libamdhip64 at load time; run with LD_LIBRARY_PATH covering both). */
#include <stdio.h>
#include <stdlib.h>

#include "yk.h"

#define CHECK(x)                                                        \
  do {                                                                  \
    int rc_ = (x);                                                      \
    if (rc_) {                                                          \
      fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, yk_last_error()); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

/* frames_dev: B x H x W x 3 uint8 BGR in HBM (e.g. from a decoder writing to device memory);
 * dets_dev / counts_dev: B x 300 x 6 float32 and B int32, also device memory. */
int detect_and_track(const char* engine, const unsigned char* frames_dev, int B, float* dets_dev, int* counts_dev) {
  yk_ctx* ctx = NULL;
  yk_model* model = NULL;
  yk_tracker* trk = NULL;
  CHECK(yk_ctx_create(0, &ctx));
  CHECK(yk_model_load(ctx, engine, &model));
  yk_tracker_cfg cfg = {150, 1, 0.1, 512, 300, YK_POLICY_ENHANCED};
  CHECK(yk_tracker_create(ctx, B, &cfg, &trk));
  CHECK(yk_detect(model, frames_dev, B, 0.25f, 0.7f, 300, dets_dev, counts_dev, NULL));
  CHECK(yk_tracker_step(trk, dets_dev, YK_F32, 6, counts_dev, NULL));
  yk_track_out* rows = (yk_track_out*)malloc(sizeof(yk_track_out) * 512 * (size_t)B);
  int counts[64];
  yk_tracker_stats stats[64];
  CHECK(yk_tracker_download(trk, rows, counts, stats, NULL));
  for (int s = 0; s < B && s < 64; ++s) printf("stream %d: %d tracks\n", s, counts[s]);
  free(rows);
  yk_tracker_destroy(trk);
  yk_model_destroy(model);
  yk_ctx_destroy(ctx);
  return 0;
}
