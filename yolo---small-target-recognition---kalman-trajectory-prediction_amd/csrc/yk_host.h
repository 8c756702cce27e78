// Host-only part of the libyk.so internals: error reporting, argument checks, and the validation
// of detector programs and engine files that arrive from outside the library (yk_model_create's
// descriptor, yk_model_load's file).  No HIP include: tests/test_asan_cpu.py builds this file and
// program.cpp with AddressSanitizer / UBSan on the CPU and feeds them corrupt inputs.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/yk.h"

namespace yk {

void set_error(const std::string& msg);
void clear_error();

#define YK_CHECK_ARG(cond, msg)      \
  do {                               \
    if (!(cond)) {                   \
      ::yk::set_error(msg);          \
      return YK_ERR_ARG;             \
    }                                \
  } while (0)

constexpr int kTabMax = 1024;       // K-chunk table entries a table-driven conv holds in LDS
constexpr int kInputCoutMax = 64;   // padded output channels of the fused input conv

// Every field of a detector program yk_model_create reads: counts and sizes within the limits the
// kernels assume, every view inside its buffer, every blob range inside the blob.  YK_OK or
// YK_ERR_ARG with yk_last_error set.
int validate_model_desc(const yk_model_desc* desc, int64_t blob_bytes);

// An engine file (yk.h, yk_model_load) read whole and checked: the header's counts against the
// file's actual size (nothing is allocated from an unchecked count), then validate_model_desc.
struct EngineImage {
  yk_model_desc desc{};
  std::vector<int64_t> buf_elems;
  std::vector<yk_op> ops;
  std::vector<char> blob;
  std::vector<int32_t> plan;  // [n_plan][4] {op, kind, nnt, npt}
  int32_t plan_batch = 0;
};
int read_engine(const char* path, EngineImage& e);

}  // namespace yk
