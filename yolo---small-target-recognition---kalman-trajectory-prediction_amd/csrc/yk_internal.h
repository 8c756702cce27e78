// Internal helpers shared by the libyk.so translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "../../include/yk.h"
#include "yk_host.h"

struct yk_ctx {
  int device;
};

namespace yk {

// Evaluate a HIP call; on failure record the message and return YK_ERR_HIP from the caller.
#define YK_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ::yk::set_error(std::string(#expr) + " -> " + hipGetErrorString(e_) + " (" +    \
                      __FILE__ + ":" + std::to_string(__LINE__) + ")");                \
      return YK_ERR_HIP;                                                               \
    }                                                                                  \
  } while (0)

// Bind the calling thread to the handle's device for the duration of a call.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace yk
