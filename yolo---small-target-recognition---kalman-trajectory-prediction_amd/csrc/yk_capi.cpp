// Context handling, error reporting and the engine-file loader of the C ABI (include/yk.h).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <vector>

#include "yk_internal.h"

namespace yk {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }
}  // namespace yk

extern "C" {

int yk_abi_version(void) { return YK_ABI_VERSION; }

const char* yk_last_error(void) { return yk::g_last_error.c_str(); }

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

// Engine file (yk.h, yk_model_load): a program packed once by model.Program.export_engine.
int yk_model_load(yk_ctx* ctx, const char* path, yk_model** out) {
  YK_CHECK_ARG(ctx && path && out, "yk_model_load: NULL argument");
  std::ifstream f(path, std::ios::binary);
  YK_CHECK_ARG(f.good(), std::string("yk_model_load: cannot open ") + path);
  struct Head {
    char magic[8];
    int32_t version, sizeof_desc, sizeof_op, n_bufs, n_ops, plan_batch, n_plan, pad;
    int64_t blob_bytes;
  } h{};
  f.read((char*)&h, sizeof h);
  YK_CHECK_ARG(f.good() && std::memcmp(h.magic, "YKENGINE", 8) == 0, "yk_model_load: not a YKENGINE file");
  YK_CHECK_ARG(h.version == 1, "yk_model_load: unsupported engine version");
  YK_CHECK_ARG(h.sizeof_desc == (int32_t)sizeof(yk_model_desc) && h.sizeof_op == (int32_t)sizeof(yk_op),
               "yk_model_load: engine written for another ABI (struct sizes differ)");
  YK_CHECK_ARG(h.n_bufs > 0 && h.n_bufs < (1 << 16) && h.n_ops > 0 && h.n_ops < (1 << 16) && h.blob_bytes > 0 &&
                   h.n_plan >= 0 && h.n_plan <= h.n_ops,
               "yk_model_load: corrupt engine header");
  yk_model_desc d{};
  f.read((char*)&d, sizeof d);
  std::vector<int64_t> bufs(h.n_bufs);
  std::vector<yk_op> ops(h.n_ops);
  std::vector<char> blob((size_t)h.blob_bytes);
  std::vector<int32_t> plan((size_t)h.n_plan * 4);
  f.read((char*)bufs.data(), (std::streamsize)(bufs.size() * sizeof(int64_t)));
  f.read((char*)ops.data(), (std::streamsize)(ops.size() * sizeof(yk_op)));
  f.read(blob.data(), (std::streamsize)blob.size());
  if (h.n_plan) f.read((char*)plan.data(), (std::streamsize)(plan.size() * sizeof(int32_t)));
  YK_CHECK_ARG(f.good(), "yk_model_load: truncated engine file");
  YK_CHECK_ARG(d.n_bufs == h.n_bufs && d.n_ops == h.n_ops, "yk_model_load: header / descriptor mismatch");
  d.buf_elems = bufs.data();
  d.ops = ops.data();
  yk_model* m = nullptr;
  const int rc = yk_model_create(ctx, &d, blob.data(), h.blob_bytes, &m);
  if (rc != YK_OK) return rc;
  for (int32_t i = 0; i < h.n_plan; ++i) {
    const int32_t* p = &plan[(size_t)i * 4];
    const int r = yk_model_set_plan(m, p[0], h.plan_batch, p[1], p[2], p[3]);
    if (r != YK_OK) {
      yk_model_destroy(m);
      return r;
    }
  }
  *out = m;
  return YK_OK;
}

}  // extern "C"
