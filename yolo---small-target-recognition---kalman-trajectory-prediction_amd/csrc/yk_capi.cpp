// Context handling and error reporting of the C ABI (include/yk.h).
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

int yk_ctx_create(int device, yk_ctx** out) {
  YK_CHECK_ARG(out != nullptr, "yk_ctx_create: out is NULL");
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

}  // extern "C"
