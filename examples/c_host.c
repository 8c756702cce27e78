/* A C host on the C ABI alone: engine file -> detector, then the tracker, for one batch of
 * frames already in device memory; or the detector built by the library from a raw fp32 state
 * dict (yk_model_load_weights) with no Python step at all.  Build (library entry points only):
 *   gcc -O2 -I include -c examples/c_host.c
 * The stand-alone program (-DYK_C_HOST_MAIN: weights file + raw frames -> detections file; uses
 * the HIP runtime for device buffers), as __graft_entry__.build() makes it:
 *   gcc -O2 -std=c11 -DYK_C_HOST_MAIN -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include \
 *       examples/c_host.c -L <pkg dir> -l:libyk.so -L /opt/rocm/lib -lamdhip64 -o examples/c_host
 * (run with LD_LIBRARY_PATH covering libyk.so and libamdhip64). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
  CHECK(yk_abi_check()); /* this file's struct layouts == the loaded libyk.so's (YK_ABI_VERSION) */
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

/* Raw state-dict file (weights.save_raw): "YKWTS\0\0\0", int32
 * version 1, int32 n; per tensor: int32 name length, the name (no NUL), int32 ndim, int64
 * shape[ndim], float32 data (C order).  Little-endian. */
typedef struct {
  yk_weights w;
  yk_tensor* t;
  char** names;
  float** data;
} raw_weights;

static void free_raw_weights(raw_weights* r) {
  for (int i = 0; i < r->w.n; ++i) {
    free(r->names[i]);
    free(r->data[i]);
  }
  free(r->names);
  free(r->data);
  free(r->t);
  memset(r, 0, sizeof *r);
}

static int load_raw_weights(const char* path, raw_weights* r) {
  memset(r, 0, sizeof *r);
  FILE* f = fopen(path, "rb");
  if (!f) return 1;
  char magic[8];
  int32_t ver = 0, n = 0;
  int ok = fread(magic, 1, 8, f) == 8 && memcmp(magic, "YKWTS\0\0\0", 8) == 0 && fread(&ver, 4, 1, f) == 1 &&
           ver == 1 && fread(&n, 4, 1, f) == 1 && n >= 0 && n < 100000;
  if (ok) {
    r->t = (yk_tensor*)calloc((size_t)n + 1, sizeof(yk_tensor));
    r->names = (char**)calloc((size_t)n + 1, sizeof(char*));
    r->data = (float**)calloc((size_t)n + 1, sizeof(float*));
    ok = r->t && r->names && r->data;
  }
  for (int i = 0; ok && i < n; ++i) {
    int32_t len = 0, nd = 0;
    ok = fread(&len, 4, 1, f) == 1 && len > 0 && len < 4096;
    if (ok) {
      r->names[i] = (char*)calloc((size_t)len + 1, 1);
      ok = r->names[i] && fread(r->names[i], 1, (size_t)len, f) == (size_t)len;
    }
    ok = ok && fread(&nd, 4, 1, f) == 1 && nd >= 0 && nd <= 4;
    int64_t count = 1;
    for (int d = 0; ok && d < nd; ++d) {
      ok = fread(&r->t[i].shape[d], 8, 1, f) == 1 && r->t[i].shape[d] >= 0;
      count *= r->t[i].shape[d];
    }
    if (ok) {
      r->data[i] = (float*)malloc(sizeof(float) * (size_t)(count ? count : 1));
      ok = r->data[i] && fread(r->data[i], 4, (size_t)count, f) == (size_t)count;
    }
    r->t[i].name = r->names[i];
    r->t[i].ndim = nd;
    r->t[i].data = r->data[i];
    r->w.n = i + 1;
  }
  fclose(f);
  r->w.tensors = r->t;
  if (!ok) free_raw_weights(r);
  return ok ? 0 : 1;
}

/* The detector built by the library from a raw state dict (yk_model_load_weights), one batch. */
int detect_from_weights(const char* weights_path, char scale, int act_dtype, int frame_h, int frame_w, int imgsz,
                        const unsigned char* frames_dev, int B, float* dets_dev, int* counts_dev) {
  raw_weights rw;
  if (load_raw_weights(weights_path, &rw)) {
    fprintf(stderr, "cannot read weights file %s\n", weights_path);
    return 1;
  }
  yk_ctx* ctx = NULL;
  yk_model* model = NULL;
  int rc = yk_abi_check();
  if (!rc) rc = yk_ctx_create(0, &ctx);
  if (!rc) rc = yk_model_load_weights(ctx, &rw.w, scale, act_dtype, frame_h, frame_w, imgsz, B, &model);
  free_raw_weights(&rw);
  if (!rc) rc = yk_detect(model, frames_dev, B, 0.25f, 0.7f, 300, dets_dev, counts_dev, NULL);
  if (rc) fprintf(stderr, "detect_from_weights failed (%d): %s\n", rc, yk_last_error());
  if (model) yk_model_destroy(model);
  if (ctx) yk_ctx_destroy(ctx);
  return rc;
}

#ifdef YK_C_HOST_MAIN
#include <hip/hip_runtime_api.h>

/* c_host <weights.ykw> <scale n|s|...> <dtype 0 bf16|1 fp32|2 fp8> <H> <W> <imgsz> <frames.u8> <B> <out.bin>
 * frames.u8: B x H x W x 3 uint8 BGR; out.bin: int32 counts[B], then float32 dets[B][300][6]. */
int main(int argc, char** argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: %s weights scale dtype H W imgsz frames B out\n", argv[0]);
    return 2;
  }
  const int dtype = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]), imgsz = atoi(argv[6]), B = atoi(argv[8]);
  const size_t fbytes = (size_t)B * H * W * 3;
  unsigned char* frames = (unsigned char*)malloc(fbytes);
  FILE* f = fopen(argv[7], "rb");
  if (!frames || !f || fread(frames, 1, fbytes, f) != fbytes) {
    fprintf(stderr, "cannot read %zu frame bytes from %s\n", fbytes, argv[7]);
    return 1;
  }
  fclose(f);
  unsigned char* d_frames = NULL;
  float* d_dets = NULL;
  int* d_counts = NULL;
  if (hipMalloc((void**)&d_frames, fbytes) != hipSuccess ||
      hipMalloc((void**)&d_dets, sizeof(float) * 300 * 6 * (size_t)B) != hipSuccess ||
      hipMalloc((void**)&d_counts, sizeof(int) * (size_t)B) != hipSuccess ||
      hipMemcpy(d_frames, frames, fbytes, hipMemcpyHostToDevice) != hipSuccess) {
    fprintf(stderr, "device buffers failed\n");
    return 1;
  }
  int rc = detect_from_weights(argv[1], argv[2][0], dtype, H, W, imgsz, d_frames, B, d_dets, d_counts);
  if (rc) return 1;
  float* dets = (float*)malloc(sizeof(float) * 300 * 6 * (size_t)B);
  int* counts = (int*)malloc(sizeof(int) * (size_t)B);
  if (hipMemcpy(dets, d_dets, sizeof(float) * 300 * 6 * (size_t)B, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(counts, d_counts, sizeof(int) * (size_t)B, hipMemcpyDeviceToHost) != hipSuccess) {
    fprintf(stderr, "copy back failed\n");
    return 1;
  }
  FILE* o = fopen(argv[9], "wb");
  if (!o || fwrite(counts, sizeof(int), (size_t)B, o) != (size_t)B ||
      fwrite(dets, sizeof(float), 300 * 6 * (size_t)B, o) != 300 * 6 * (size_t)B) {
    fprintf(stderr, "cannot write %s\n", argv[9]);
    return 1;
  }
  fclose(o);
  for (int b = 0; b < B; ++b) printf("image %d: %d detections\n", b, counts[b]);
  (void)hipFree(d_frames);
  (void)hipFree(d_dets);
  (void)hipFree(d_counts);
  free(frames);
  free(dets);
  free(counts);
  return 0;
}
#endif
