// Context handling, error reporting and the engine-file loader of the C ABI (include/yk.h).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "yk_internal.h"

extern "C" {

namespace {
// Diagnostics (YK_SEGV_TRACE=1 at context creation): a SIGSEGV prints the native stack to stderr,
// then the previous handler (Python's faulthandler, or the default action) runs.
struct sigaction g_prev_segv;
void segv_trace(int sig, siginfo_t* info, void* uc) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  static const char hdr[] = "[yk] SIGSEGV native stack:\n";
  (void)!write(2, hdr, sizeof hdr - 1);
  backtrace_symbols_fd(frames, n, 2);
  if (g_prev_segv.sa_flags & SA_SIGINFO) {
    if (g_prev_segv.sa_sigaction) g_prev_segv.sa_sigaction(sig, info, uc);
  } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
    g_prev_segv.sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}
void maybe_install_segv_trace() {
  static bool done = false;
  if (done || !getenv("YK_SEGV_TRACE")) return;
  done = true;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}
}  // namespace

int yk_ctx_create(int device, yk_ctx** out) {
  YK_CHECK_ARG(out != nullptr, "yk_ctx_create: out is NULL");
  maybe_install_segv_trace();
  int n = 0;
  YK_HIP(hipGetDeviceCount(&n));
  YK_CHECK_ARG(device >= 0 && device < n, "yk_ctx_create: device index out of range");
  yk::DeviceGuard g(device);
  YK_HIP(hipFree(nullptr));  // force runtime/context initialisation on this device
  *out = new yk_ctx{device};
  return YK_OK;
}

int64_t yk_struct_size(int which) {
  switch (which) {
    case 0: return (int64_t)sizeof(yk_tracker_cfg);
    case 1: return (int64_t)sizeof(yk_tracker_stats);
    case 2: return (int64_t)sizeof(yk_track_out);
    case 3: return (int64_t)sizeof(yk_track_state);
    case 4: return (int64_t)sizeof(yk_view);
    case 5: return (int64_t)sizeof(yk_op);
    case 6: return (int64_t)sizeof(yk_model_desc);
    case 7: return (int64_t)sizeof(yk_bt_cfg);
    case 8: return (int64_t)sizeof(yk_motion);
    case 9: return (int64_t)sizeof(yk_gmd_stats);
    case 10: return (int64_t)sizeof(yk_tensor);
    case 11: return (int64_t)sizeof(yk_track_event);
    default: return -1;
  }
}

int yk_memcpy_d2h(void* host_dst, const void* dev_src, int64_t bytes) {
  YK_CHECK_ARG(host_dst && dev_src && bytes >= 0, "yk_memcpy_d2h: bad argument");
  YK_HIP(hipMemcpy(host_dst, dev_src, (size_t)bytes, hipMemcpyDeviceToHost));
  return YK_OK;
}

int yk_ctx_destroy(yk_ctx* ctx) {
  delete ctx;
  return YK_OK;
}

// Engine file (yk.h, yk_model_load): a program packed once by model.Program.export_engine, read
// and validated on the host (yk_host.cpp read_engine) before anything touches the device.
int yk_model_load(yk_ctx* ctx, const char* path, yk_model** out) {
  YK_CHECK_ARG(ctx && path && out, "yk_model_load: NULL argument");
  yk::EngineImage e;
  if (const int rc = yk::read_engine(path, e)) return rc;
  yk_model* m = nullptr;
  const int rc = yk_model_create(ctx, &e.desc, e.blob.data(), (int64_t)e.blob.size(), &m);
  if (rc != YK_OK) return rc;
  for (size_t i = 0; i < e.plan.size() / 4; ++i) {
    const int32_t* p = &e.plan[i * 4];
    const int r = yk_model_set_plan(m, p[0], e.plan_batch, p[1], p[2], p[3]);
    if (r != YK_OK) {
      yk_model_destroy(m);
      return r;
    }
  }
  *out = m;
  return YK_OK;
}

// The program built by the library (program.cpp, host only), then the model on the device.
int yk_model_load_weights(yk_ctx* ctx, const yk_weights* weights, char scale, int act_dtype, int frame_h, int frame_w,
                          int imgsz, int max_batch, yk_model** out) {
  YK_CHECK_ARG(ctx && out, "yk_model_load_weights: NULL argument");
  yk_program* p = nullptr;
  int rc = yk_program_build(weights, scale, act_dtype, frame_h, frame_w, imgsz, max_batch, 300, &p);
  if (rc != YK_OK) return rc;
  const yk_model_desc* d = nullptr;
  const void* blob = nullptr;
  int64_t bytes = 0;
  rc = yk_program_get(p, &d, &blob, &bytes);
  if (rc == YK_OK) rc = yk_model_create(ctx, d, blob, bytes, out);
  yk_program_destroy(p);
  return rc;
}

}  // extern "C"
