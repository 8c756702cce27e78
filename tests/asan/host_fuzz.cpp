// Host-side fuzz driver for the C ABI's untrusted-input parsers, built with AddressSanitizer and
// UBSan by tests/test_asan_cpu.py (no GPU, no HIP runtime: yk_host.cpp + program.cpp only).
//
//   host_fuzz engine <file>                 read_engine on a real engine file: must be accepted
//   host_fuzz engine-fuzz <file> <seed> <n> n corrupted copies (truncations, byte flips, header and
//                                           descriptor fields set to extreme values, garbage): each
//                                           must be rejected or accepted cleanly, never crash
//   host_fuzz program <weights> <n>         yk_program_build on a raw state dict (weights.save_raw):
//                                           every scale / dtype must build; then n mutated state
//                                           dicts (missing tensors, wrong ndim / shapes, NaN
//                                           weights, bad sizes) must be rejected or built cleanly
// Prints one summary line; exits non-zero on an unexpected result (sanitizer reports abort).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "yk_host.h"

namespace {

std::vector<char> slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

void spit(const std::string& path, const std::vector<char>& b) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  f.write(b.data(), (std::streamsize)b.size());
}

int engine_one(const char* path) {
  yk::EngineImage e;
  const int rc = yk::read_engine(path, e);
  if (rc != YK_OK) fprintf(stderr, "rejected: %s\n", yk_last_error());
  return rc;
}

int engine_fuzz(const char* path, unsigned seed, int n) {
  const std::vector<char> good = slurp(path);
  if (good.size() < 64) return 2;
  std::mt19937_64 rng(seed);
  const std::string tmp = std::string(path) + ".fuzz";
  const size_t head = 48, desc_end = head + sizeof(yk_model_desc);
  int accepted = 0, rejected = 0;
  const int64_t extremes[] = {0, 1, -1, 2, 7, 8, 255, 256, 65535, 65536, 0x7fffffff, -0x7fffffff - 1,
                              (int64_t)1 << 32, (int64_t)1 << 40, INT64_MAX, INT64_MIN};
  for (int it = 0; it < n; ++it) {
    std::vector<char> b = good;
    const int kind = (int)(rng() % 6);
    if (kind == 0) {  // truncation
      b.resize(rng() % good.size());
    } else if (kind == 1) {  // random byte flips anywhere in the first 64 KB
      const int flips = 1 + (int)(rng() % 8);
      for (int k = 0; k < flips; ++k) b[rng() % std::min<size_t>(b.size(), 65536)] ^= (char)(1 + rng() % 255);
    } else if (kind == 2) {  // a header / descriptor int32 field set to an extreme value
      const size_t off = (rng() % (desc_end / 4)) * 4;
      const int32_t v = (int32_t)extremes[rng() % 12];
      if (off + 4 <= b.size()) std::memcpy(&b[off], &v, 4);
    } else if (kind == 3) {  // an op field (int32 or int64) set to an extreme value
      const size_t ops_off = desc_end + 8 * (size_t)*(const int32_t*)&good[20];
      const size_t n_ops = (size_t)*(const int32_t*)&good[24];
      const size_t off = ops_off + (rng() % n_ops) * sizeof(yk_op) + (rng() % (sizeof(yk_op) / 4)) * 4;
      const int64_t v = extremes[rng() % 16];
      if (off + 8 <= b.size()) std::memcpy(&b[off], &v, (rng() & 1) ? 8 : 4);
    } else if (kind == 4) {  // a buffer size set to an extreme value
      const size_t off = desc_end + 8 * (rng() % (size_t)*(const int32_t*)&good[20]);
      const int64_t v = extremes[rng() % 16];
      if (off + 8 <= b.size()) std::memcpy(&b[off], &v, 8);
    } else {  // garbage of random length (sometimes with the magic)
      b.assign(rng() % 4096, 0);
      for (char& c : b) c = (char)rng();
      if (b.size() >= 8 && (rng() & 1)) std::memcpy(b.data(), "YKENGINE", 8);
    }
    spit(tmp, b);
    yk::EngineImage e;
    if (yk::read_engine(tmp.c_str(), e) == YK_OK) ++accepted;
    else ++rejected;
  }
  std::remove(tmp.c_str());
  printf("engine-fuzz n=%d accepted=%d rejected=%d\n", n, accepted, rejected);
  return 0;
}

struct RawWeights {
  std::vector<std::string> names;
  std::vector<yk_tensor> t;
  std::vector<std::vector<float>> data;
};

bool load_raw(const char* path, RawWeights& w) {
  const std::vector<char> b = slurp(path);
  size_t p = 0;
  auto take = [&](void* dst, size_t n) {
    if (p + n > b.size()) return false;
    std::memcpy(dst, &b[p], n);
    p += n;
    return true;
  };
  char magic[8];
  int32_t ver = 0, n = 0;
  if (!take(magic, 8) || std::memcmp(magic, "YKWTS\0\0\0", 8) || !take(&ver, 4) || ver != 1 || !take(&n, 4) || n < 0)
    return false;
  for (int i = 0; i < n; ++i) {
    int32_t len = 0, nd = 0;
    if (!take(&len, 4) || len <= 0 || len > 4096) return false;
    std::string name((size_t)len, '\0');
    if (!take(&name[0], (size_t)len) || !take(&nd, 4) || nd < 0 || nd > 4) return false;
    yk_tensor t{};
    t.ndim = nd;
    int64_t count = 1;
    for (int d = 0; d < nd; ++d) {
      if (!take(&t.shape[d], 8) || t.shape[d] < 0) return false;
      count *= t.shape[d];
    }
    std::vector<float> v((size_t)count);
    if (!take(v.data(), (size_t)count * 4)) return false;
    w.names.push_back(name);
    w.t.push_back(t);
    w.data.push_back(std::move(v));
  }
  return true;
}

// tensors pointing at their names / data (after any mutation of the vectors)
yk_weights bind(RawWeights& w) {
  for (size_t i = 0; i < w.t.size(); ++i) {
    w.t[i].name = w.names[i].c_str();
    w.t[i].data = w.data[i].data();
  }
  return yk_weights{(int32_t)w.t.size(), w.t.data()};
}

int build(const yk_weights& W, char scale, int dtype, int fh, int fw, int imgsz, int mb, int md) {
  yk_program* p = nullptr;
  const int rc = yk_program_build(&W, scale, dtype, fh, fw, imgsz, mb, md, &p);
  if (rc == YK_OK) {
    const yk_model_desc* d = nullptr;
    const void* blob = nullptr;
    int64_t bytes = 0;
    if (yk_program_get(p, &d, &blob, &bytes) != YK_OK || yk::validate_model_desc(d, bytes) != YK_OK) {
      fprintf(stderr, "built program fails validation: %s\n", yk_last_error());
      yk_program_destroy(p);
      return -100;
    }
    yk_program_destroy(p);
  }
  return rc;
}

int program_fuzz(const char* path, int n) {
  RawWeights base;
  if (!load_raw(path, base)) {
    fprintf(stderr, "cannot read %s\n", path);
    return 2;
  }
  char scale = 0;  // the scale whose channel counts the state dict has
  for (char s : {'n', 's'}) {
    RawWeights w = base;
    const int rc = build(bind(w), s, YK_ACT_F32, 512, 640, 640, 2, 300);
    if (rc == -100) return 3;
    if (rc == YK_OK) scale = s;
  }
  if (!scale) {
    fprintf(stderr, "the state dict builds at no scale: %s\n", yk_last_error());
    return 3;
  }
  // every dtype and a letterboxed frame size build and validate
  const int sizes[][3] = {{512, 640, 640}, {1080, 1920, 640}, {1024, 1280, 1280}, {375, 1242, 640}};
  for (int dt : {YK_ACT_BF16, YK_ACT_F32, YK_ACT_FP8, YK_ACT_F16})
    for (auto& sz : sizes) {
      RawWeights w = base;
      const int rc = build(bind(w), scale, dt, sz[0], sz[1], sz[2], 2, 300);
      if (rc != YK_OK) {
        fprintf(stderr, "dtype %d frame %dx%d imgsz %d: %s\n", dt, sz[1], sz[0], sz[2], yk_last_error());
        return 3;
      }
    }
  std::mt19937_64 rng(1234);
  int accepted = 0, rejected = 0;
  for (int it = 0; it < n; ++it) {
    RawWeights w = base;
    const int kind = (int)(rng() % 6);
    const size_t i = rng() % w.t.size();
    int fh = 512, fw = 640, imgsz = 640, mb = 2, md = 300, dt = YK_ACT_F32;
    char sc = scale;
    if (kind == 0) {  // a tensor missing
      w.t.erase(w.t.begin() + (long)i);
      w.names.erase(w.names.begin() + (long)i);
      w.data.erase(w.data.begin() + (long)i);
    } else if (kind == 1 || kind == 2) {  // another ndim / shape (data sized to match the claim)
      yk_tensor& t = w.t[i];
      if (kind == 1) t.ndim = (int32_t)(rng() % 5);
      int64_t count = 1;
      for (int d = 0; d < t.ndim; ++d) {
        t.shape[d] = (int64_t)(rng() % 70);
        count *= t.shape[d];
      }
      if (count > (1 << 22)) continue;
      w.data[i].assign((size_t)count, 0.5f);
    } else if (kind == 3) {  // non-finite weights
      for (float& v : w.data[i]) v = (rng() & 1) ? NAN : INFINITY;
    } else if (kind == 4) {  // sizes
      const int64_t vals[] = {-1, 0, 1, 31, 32, 33, 64, 4097, 1 << 16, 0x7fffffff};
      fh = (int)vals[rng() % 10];
      fw = (int)vals[rng() % 10];
      imgsz = (int)vals[rng() % 10];
      mb = (int)vals[rng() % 7];
      md = (int)vals[rng() % 10];
      if ((int64_t)std::abs(fh) * std::abs(fw) > (1 << 24) || (int64_t)imgsz * imgsz > (1 << 24)) continue;
    } else {  // scale / dtype codes
      sc = (char)(rng() % 128);
      dt = (int)(rng() % 6) - 1;
    }
    const int rc = build(bind(w), sc, dt, fh, fw, imgsz, mb, md);
    if (rc == -100) return 3;
    if (rc == YK_OK) ++accepted;
    else ++rejected;
  }
  printf("program-fuzz n=%d accepted=%d rejected=%d scale=%c\n", n, accepted, rejected, scale);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 3 && !std::strcmp(argv[1], "engine")) return engine_one(argv[2]) == YK_OK ? 0 : 1;
  if (argc >= 5 && !std::strcmp(argv[1], "engine-fuzz"))
    return engine_fuzz(argv[2], (unsigned)std::strtoul(argv[3], nullptr, 10), std::atoi(argv[4]));
  if (argc >= 4 && !std::strcmp(argv[1], "program")) return program_fuzz(argv[2], std::atoi(argv[3]));
  fprintf(stderr, "usage: host_fuzz engine <file> | engine-fuzz <file> <seed> <n> | program <weights> <n>\n");
  return 2;
}
