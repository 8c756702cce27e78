// Detector program builder on the C ABI: yk_program_build / yk_model_load_weights.
//
// The host half of the detection path -- what model.py Program, arch.py parse_arch,
// weights.py fused_convs and letterbox.py plan do in Python -- restated in C++ so a C / Go /
// Java host creates the detector from a raw fp32 state dict with no Python step.  The program it
// produces (yk_model_desc, ops, buffer sizes and the packed blob) is byte-identical to
// Program's (tests/test_program_cpu.py checks every byte), so the device results are too.
//
// Rules restated:
//   parse_model channel / repeat rules        nn/tasks.py:1524-1700 (yolov8-small.yaml, P2..P5)
//   Conv / C2f / Bottleneck / SPPF / Detect   nn/modules/conv.py:39-93, block.py:216-238,294-322,
//                                             470-492, head.py:26-209 (legacy v8 head)
//   fuse_conv_and_bn (eps 1e-3, float32)      utils/torch_utils.py:255-286, 488-498
//   LetterBox geometry + cv2 INTER_LINEAR     data/augment.py:1667-1744 (tables: letterbox.py)
//   scale_boxes gain / padding                utils/ops.py:105-184
// Host code only: no HIP call is made until yk_model_load_weights creates the model.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "yk_host.h"

namespace {

// ---------------------------------------------------------------- topology (arch.py YOLOV8_SMALL)
struct Row {
  int f[4];
  int nf;  // 1: f[0] (-1 = previous layer); >1: a list (Concat / Detect)
  int n;
  const char* m;
  int a0, a1, a2;  // Conv: c2, k, s; C2f: c2, shortcut; SPPF: c2, k; Upsample: scale
};
const Row kTopo[] = {
    {{-1}, 1, 1, "Conv", 32, 3, 2},          {{-1}, 1, 1, "Conv", 64, 3, 2},
    {{-1}, 1, 3, "C2f", 64, 1, 0},           {{-1}, 1, 1, "Conv", 128, 3, 2},
    {{-1}, 1, 6, "C2f", 128, 1, 0},          {{-1}, 1, 1, "Conv", 256, 3, 2},
    {{-1}, 1, 6, "C2f", 256, 1, 0},          {{-1}, 1, 1, "Conv", 512, 3, 2},
    {{-1}, 1, 3, "C2f", 512, 1, 0},          {{-1}, 1, 1, "SPPF", 512, 5, 0},
    {{-1}, 1, 1, "Upsample", 2, 0, 0},       {{-1, 6}, 2, 1, "Concat", 0, 0, 0},
    {{-1}, 1, 3, "C2f", 256, 0, 0},          {{-1}, 1, 1, "Upsample", 2, 0, 0},
    {{-1, 4}, 2, 1, "Concat", 0, 0, 0},      {{-1}, 1, 3, "C2f", 128, 0, 0},
    {{-1}, 1, 1, "Upsample", 2, 0, 0},       {{-1, 2}, 2, 1, "Concat", 0, 0, 0},
    {{-1}, 1, 3, "C2f", 64, 0, 0},           {{15}, 1, 1, "Conv", 128, 3, 2},
    {{-1, 12}, 2, 1, "Concat", 0, 0, 0},     {{-1}, 1, 3, "C2f", 256, 0, 0},
    {{-1}, 1, 1, "Conv", 256, 3, 2},         {{-1, 9}, 2, 1, "Concat", 0, 0, 0},
    {{-1}, 1, 3, "C2f", 512, 0, 0},          {{18, 15, 21, 24}, 4, 1, "Detect", 0, 0, 0},
};
constexpr int kLayers = (int)(sizeof(kTopo) / sizeof(kTopo[0]));
constexpr int kRegMax = 16;

struct Scale {
  char name;
  double depth, width;
  int max_ch;
};
const Scale kScales[] = {{'n', 0.50, 0.375, 1024}, {'s', 0.67, 0.625, 1024}, {'m', 1.00, 0.875, 768},
                         {'l', 1.33, 1.125, 512},  {'x', 1.67, 1.375, 512}};

struct Layer {
  int i;
  std::vector<int> f;
  std::string kind;
  std::vector<int> c1;
  int c2 = 0;
  int k = 1, s = 1, n = 1, pool_k = 5, up = 2, c2b = 0, c3 = 0, nc = 0;
  bool shortcut = false;
};

int make_divisible(double x, int d) { return (int)std::ceil(x / d) * d; }

// parse_arch (arch.py:113-155): parse_model's channel and repeat rules
bool parse(char scale, int nc, std::vector<Layer>& out, std::string& err) {
  const Scale* sc = nullptr;
  for (const Scale& s : kScales)
    if (s.name == scale) sc = &s;
  if (!sc) {
    err = std::string("unknown model scale '") + scale + "' (n, s, m, l or x)";
    return false;
  }
  std::vector<int> chs = {3};
  for (int i = 0; i < kLayers; ++i) {
    const Row& r = kTopo[i];
    Layer L;
    L.i = i;
    L.f.assign(r.f, r.f + r.nf);
    L.kind = r.m;
    int n = r.n;
    if (n > 1) n = std::max((int)std::nearbyint(n * sc->depth), 1);  // Python round: half to even
    auto ch = [&](int f) { return f == -1 ? chs.back() : chs[f]; };
    if (L.kind == "Conv" || L.kind == "C2f" || L.kind == "SPPF") {
      L.c1 = {ch(L.f[0])};
      int c2 = r.a0;
      if (c2 != nc) c2 = make_divisible(std::min<double>(c2, sc->max_ch) * sc->width, 8);
      L.c2 = c2;
      if (L.kind == "Conv") {
        L.k = r.a1;
        L.s = r.a2;
      } else if (L.kind == "C2f") {
        L.n = n;
        L.shortcut = r.a1 != 0;
      } else {
        L.pool_k = r.a1;
      }
    } else if (L.kind == "Upsample") {
      L.c1 = {ch(L.f[0])};
      L.c2 = L.c1[0];
      L.up = r.a0;
    } else if (L.kind == "Concat") {
      for (int f : L.f) L.c1.push_back(ch(f));
      for (int c : L.c1) L.c2 += c;
    } else {  // Detect
      for (int f : L.f) L.c1.push_back(ch(f));
      L.c2b = std::max({16, L.c1[0] / 4, kRegMax * 4});
      L.c3 = std::max(L.c1[0], std::min(nc, 100));
      L.nc = nc;
      L.c2 = kRegMax * 4 + nc;
    }
    out.push_back(L);
    if (i == 0) chs.clear();
    chs.push_back(L.c2);
  }
  return true;
}

// detect_strides (arch.py:190-210)
std::vector<int> detect_strides(const std::vector<Layer>& ar) {
  std::vector<int> st;
  for (const Layer& L : ar) {
    auto src = [&](int x) { return x == -1 ? (L.i ? st[L.i - 1] : 1) : st[x]; };
    int s;
    if (L.kind == "Conv") s = src(L.f[0]) * L.s;
    else if (L.kind == "C2f" || L.kind == "SPPF") s = src(L.f[0]);
    else if (L.kind == "Upsample") s = src(L.f[0]) / L.up;
    else if (L.kind == "Concat") s = src(L.f[0]);
    else {
      std::vector<int> out;
      for (int x : L.f) out.push_back(src(x));
      return out;
    }
    st.push_back(s);
  }
  return {};
}

// ---------------------------------------------------------------- weights (weights.py fused_convs)
struct Fused {
  std::vector<float> w;  // [c2][c1][k][k]
  std::vector<float> b;
  int c2 = 0, c1 = 0, k = 1, s = 1;
  bool act = true;
};

struct WeightsView {
  std::map<std::string, const yk_tensor*> by_name;
  const yk_tensor* get(const std::string& n, std::initializer_list<int64_t> shape, std::string& err) const {
    auto it = by_name.find(n);
    if (it == by_name.end()) {
      err = "state dict has no tensor '" + n + "'";
      return nullptr;
    }
    const yk_tensor* t = it->second;
    size_t d = 0;
    bool ok = t->data != nullptr && t->ndim == (int32_t)shape.size();
    for (int64_t v : shape) ok = ok && t->shape[d++] == v;
    if (!ok) {
      err = "tensor '" + n + "' has the wrong shape or no data";
      return nullptr;
    }
    return t;
  }
};

// fuse_conv_and_bn in float32 (weights.py:121-127): scale = g / sqrt(eps + var),
// W' = W * scale (per output row), b' = beta - g * mean / sqrt(var + eps)
bool fuse(const WeightsView& W, const std::string& p, int c1, int c2, int k, int s, bool bn, Fused& out,
          std::string& err) {
  out.c1 = c1;
  out.c2 = c2;
  out.k = k;
  out.s = s;
  out.act = bn;
  const size_t per = (size_t)c1 * k * k;
  out.w.resize((size_t)c2 * per);
  out.b.resize(c2);
  if (bn) {
    const yk_tensor* w = W.get(p + ".conv.weight", {c2, c1, k, k}, err);
    const yk_tensor* g = w ? W.get(p + ".bn.weight", {c2}, err) : nullptr;
    const yk_tensor* be = g ? W.get(p + ".bn.bias", {c2}, err) : nullptr;
    const yk_tensor* mu = be ? W.get(p + ".bn.running_mean", {c2}, err) : nullptr;
    const yk_tensor* var = mu ? W.get(p + ".bn.running_var", {c2}, err) : nullptr;
    if (!var) return false;
    const float eps = 1e-3f;
    for (int o = 0; o < c2; ++o) {
      const float sq = std::sqrt(var->data[o] + eps);
      const float scale = g->data[o] / sq;
      for (size_t j = 0; j < per; ++j) out.w[o * per + j] = w->data[o * per + j] * scale;
      out.b[o] = be->data[o] - (g->data[o] * mu->data[o]) / sq;
    }
  } else {
    const yk_tensor* w = W.get(p + ".weight", {c2, c1, k, k}, err);
    const yk_tensor* b = w ? W.get(p + ".bias", {c2}, err) : nullptr;
    if (!b) return false;
    std::copy(w->data, w->data + out.w.size(), out.w.begin());
    std::copy(b->data, b->data + c2, out.b.begin());
  }
  return true;
}

// ---------------------------------------------------------------- element conversions
uint16_t f2bf(float f) {  // torch float -> bfloat16 (round to nearest even)
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
uint8_t f2e4m3(float x) {  // float8_e4m3fn, round to nearest even, |x| <= 448 (clamped by the caller)
  const uint8_t sign = std::signbit(x) ? 0x80 : 0;
  const float a = std::fabs(x);
  if (a == 0.f) return sign;
  int ex;
  std::frexp(a, &ex);
  int e = ex - 1;  // a = 1.m * 2^e
  if (e < -6) {    // subnormal: m * 2^-9
    const int m = (int)std::nearbyint(std::ldexp(a, 9));
    return (uint8_t)(sign | m);  // m == 8 is the smallest normal, 0x08
  }
  int m = (int)std::nearbyint((std::ldexp(a, -e) - 1.f) * 8.f);
  if (m == 8) {
    m = 0;
    ++e;
  }
  return (uint8_t)(sign | ((e + 7) << 3) | m);
}

// ---------------------------------------------------------------- program (model.py Program)
struct Seg {
  int buf, c_off, c_stride, cp, cl, h, w, up;
  int lh() const { return h << up; }
  int lw() const { return w << up; }
};

struct ViewGroup {
  Seg first;
  int cp;
  std::vector<std::pair<Seg, int>> segs;
};

struct Builder {
  int dtype = YK_ACT_F32, epl = 4, align = 8, esz = 4;
  std::vector<int64_t> buf_elems;
  std::vector<yk_op> ops;
  std::vector<unsigned char> blob;
  std::map<std::string, Fused> fused;
  std::vector<int> strides;
  int n_anchors = 0;
  std::string err;

  int phys(int c) const { return (c + align - 1) / align * align; }
  int new_buf(int h, int w, int c) {
    buf_elems.push_back((int64_t)h * w * c);
    return (int)buf_elems.size() - 1;
  }
  int64_t add_blob(const void* p, size_t n) {
    const size_t off = (blob.size() + 255) / 256 * 256;
    blob.resize(off, 0);
    blob.insert(blob.end(), (const unsigned char*)p, (const unsigned char*)p + n);
    return (int64_t)off;
  }
  template <class T>
  int64_t add_blob(const std::vector<T>& v) {
    return add_blob(v.data(), v.size() * sizeof(T));
  }

  // Program.views_of (model.py:149-164)
  bool views_of(const std::vector<Seg>& segs, std::vector<ViewGroup>& views) {
    for (const Seg& s : segs) {
      if (!views.empty()) {
        ViewGroup& v = views.back();
        const Seg& f = v.first;
        if (s.buf == f.buf && s.up == f.up && s.c_off == f.c_off + v.cp && s.c_stride == f.c_stride) {
          v.segs.push_back({s, v.cp});
          v.cp += s.cp;
          continue;
        }
      }
      views.push_back(ViewGroup{s, s.cp, {{s, 0}}});
    }
    if (views.size() > 2) {
      err = "a conv may read at most two views";
      return false;
    }
    return true;
  }

  struct Packed {
    std::vector<ViewGroup> views;
    std::vector<unsigned char> packed;
    std::vector<float> bias;
    std::vector<int32_t> tab;
    int k_steps = 0, n_tiles = 0;
  };

  // Program.pack (model.py:166-216)
  bool pack(const Fused& F, const std::vector<Seg>& src, const std::vector<int>& om, int cout_p, Packed& P) {
    if (!views_of(src, P.views)) return false;
    int cin_p = 0;
    for (const auto& v : P.views) cin_p += v.cp;
    std::vector<int> im;
    int kbase = 0;
    for (const auto& v : P.views) {
      for (const auto& so : v.segs)
        for (int j = 0; j < so.first.cl; ++j) im.push_back(kbase + so.second + j);
      kbase += v.cp;
    }
    if ((int)im.size() != F.c1) {
      err = "packed input channels do not match the conv";
      return false;
    }
    const int k = F.k, K = k * k * cin_p, kstep = 4 * epl;
    P.k_steps = (K + kstep - 1) / kstep;
    P.n_tiles = (cout_p + 15) / 16;
    const size_t rows = (size_t)P.n_tiles * 16, cols = (size_t)P.k_steps * kstep;
    std::vector<float> Wp(rows * cols, 0.f);
    for (int ky = 0; ky < k; ++ky)
      for (int kx = 0; kx < k; ++kx) {
        const int tap = ky * k + kx;
        for (int o = 0; o < F.c2; ++o)
          for (int i = 0; i < F.c1; ++i)
            Wp[(size_t)om[o] * cols + (size_t)tap * cin_p + im[i]] = F.w[(((size_t)o * F.c1 + i) * k + ky) * k + kx];
      }
    std::vector<float> dq;
    if (dtype == YK_ACT_FP8) {
      dq.resize(rows);
      for (size_t r = 0; r < rows; ++r) {
        float amax = 0.f;
        for (size_t c = 0; c < cols; ++c) amax = std::max(amax, std::fabs(Wp[r * cols + c]));
        const float scale = amax > 0.f ? 448.0f / std::max(amax, 1e-30f) : 1.0f;
        dq[r] = 1.0f / scale;
        for (size_t c = 0; c < cols; ++c) Wp[r * cols + c] *= scale;
      }
    }
    // [nt][ks][kg][col][e] = Wp[nt * 16 + col][ks * kstep + kg * epl + e]
    const size_t nel = rows * cols;
    std::vector<float> ord(nel);
    size_t q = 0;
    for (int nt = 0; nt < P.n_tiles; ++nt)
      for (int ks = 0; ks < P.k_steps; ++ks)
        for (int kg = 0; kg < 4; ++kg)
          for (int col = 0; col < 16; ++col)
            for (int e = 0; e < epl; ++e) ord[q++] = Wp[((size_t)nt * 16 + col) * cols + (size_t)ks * kstep + kg * epl + e];
    P.bias.assign(rows, 0.f);
    for (int o = 0; o < F.c2; ++o) P.bias[om[o]] = F.b[o];
    if (dtype == YK_ACT_FP8) {
      P.packed.resize(nel);
      for (size_t j = 0; j < nel; ++j) P.packed[j] = f2e4m3(std::min(std::max(ord[j], -448.0f), 448.0f));
      P.bias.insert(P.bias.end(), dq.begin(), dq.end());
    } else if (dtype == YK_ACT_BF16) {
      P.packed.resize(nel * 2);
      for (size_t j = 0; j < nel; ++j) {
        const uint16_t h = f2bf(ord[j]);
        memcpy(&P.packed[2 * j], &h, 2);
      }
    } else if (dtype == YK_ACT_F16) {  // torch .half(): IEEE binary16, round to nearest even
      P.packed.resize(nel * 2);
      for (size_t j = 0; j < nel; ++j) {
        const _Float16 h = (_Float16)ord[j];
        memcpy(&P.packed[2 * j], &h, 2);
      }
    } else {
      P.packed.resize(nel * 4);
      memcpy(P.packed.data(), ord.data(), nel * 4);
    }
    const int pad = k / 2;
    for (int qq = 0; qq < K / 8; ++qq) {
      const int tap = qq * 8 / cin_p, ch = qq * 8 % cin_p;
      const int dy = tap / k - pad, dx = tap % k - pad;
      const int s = ch < P.views[0].cp ? 0 : 1;
      const int off = s == 0 ? ch : ch - P.views[0].cp;
      P.tab.push_back(((dx + 8) << 21) | ((dy + 8) << 17) | (s << 16) | off);
    }
    if (P.tab.empty()) P.tab.push_back(-1);
    return true;
  }

  static yk_view view(const Seg& s, int up) { return yk_view{s.buf, s.c_off, s.c_stride, s.h, s.w, up}; }

  // Program.conv_op (model.py:218-244)
  bool conv_op(const std::string& prefix, const std::vector<Seg>& src, const Seg& dst, const std::vector<int>& om,
               int cout_p, const Seg* res = nullptr) {
    auto it = fused.find(prefix);
    if (it == fused.end()) {
      err = "no fused weights for " + prefix;
      return false;
    }
    const Fused& F = it->second;
    Packed P;
    if (!pack(F, src, om, cout_p, P)) return false;
    yk_op op;
    memset(&op, 0, sizeof op);
    op.kind = YK_K_CONV;
    op.ksize = F.k;
    op.stride = F.s;
    op.act = F.act ? 1 : 0;
    op.n_src = (int32_t)P.views.size();
    for (size_t i = 0; i < P.views.size(); ++i) {
      op.src[i] = view(P.views[i].first, P.views[i].first.up);
      op.src_ch[i] = P.views[i].cp;
    }
    op.dst = view(dst, 0);
    op.cout = cout_p;
    if (res) {
      op.has_res = 1;
      op.res = view(*res, 0);
    }
    const int lh = src[0].lh(), lw = src[0].lw(), k = F.k, s = F.s;
    op.out_h = (lh + 2 * (k / 2) - k) / s + 1;
    op.out_w = (lw + 2 * (k / 2) - k) / s + 1;
    if (op.out_h != dst.h || op.out_w != dst.w) {
      err = "conv output size mismatch at " + prefix;
      return false;
    }
    op.k_steps = P.k_steps;
    op.n_tiles = P.n_tiles;
    op.w_off = add_blob(P.packed);
    op.b_off = add_blob(P.bias);
    op.t_off = add_blob(P.tab);
    ops.push_back(op);
    return true;
  }

  std::vector<int> iota(int n, int base = 0) {
    std::vector<int> v(n);
    for (int i = 0; i < n; ++i) v[i] = base + i;
    return v;
  }

  // Program._c2f (model.py:306-326)
  bool c2f(const Layer& L, const std::vector<Seg>& src, std::vector<Seg>& out) {
    const int c = (int)(L.c2 * 0.5), cp = phys(c), n = L.n;
    const int hh = src[0].lh(), ww = src[0].lw();
    const int Y = new_buf(hh, ww, (2 + n) * cp);
    std::vector<Seg> ys;
    for (int j = 0; j < 2 + n; ++j) ys.push_back(Seg{Y, j * cp, (2 + n) * cp, cp, c, hh, ww, 0});
    const std::string p = "model." + std::to_string(L.i);
    std::vector<int> om;
    for (int o = 0; o < 2 * c; ++o) om.push_back(o < c ? o : cp + o - c);
    if (!conv_op(p + ".cv1", src, Seg{Y, 0, (2 + n) * cp, 2 * cp, 2 * c, hh, ww, 0}, om, 2 * cp)) return false;
    const int tmp = new_buf(hh, ww, cp);
    const Seg ts{tmp, 0, cp, cp, c, hh, ww, 0};
    for (int j = 0; j < n; ++j) {
      const std::string m = p + ".m." + std::to_string(j);
      if (!conv_op(m + ".cv1", {ys[1 + j]}, ts, iota(c), cp)) return false;
      if (!conv_op(m + ".cv2", {ts}, ys[2 + j], iota(c), cp, L.shortcut ? &ys[1 + j] : nullptr)) return false;
    }
    const int c2p = phys(L.c2);
    const int ob = new_buf(hh, ww, c2p);
    const Seg dst{ob, 0, c2p, c2p, L.c2, hh, ww, 0};
    if (!conv_op(p + ".cv2", ys, dst, iota(L.c2), c2p)) return false;
    out = {dst};
    return true;
  }

  // Program._sppf (model.py:328-351)
  bool sppf(const Layer& L, const std::vector<Seg>& src, std::vector<Seg>& out) {
    const int c_ = L.c1[0] / 2, cp = phys(c_);
    const int hh = src[0].lh(), ww = src[0].lw();
    const int Z = new_buf(hh, ww, 4 * cp);
    std::vector<Seg> zs;
    for (int j = 0; j < 4; ++j) zs.push_back(Seg{Z, j * cp, 4 * cp, cp, c_, hh, ww, 0});
    const std::string p = "model." + std::to_string(L.i);
    if (!conv_op(p + ".cv1", src, zs[0], iota(c_), cp)) return false;
    if (L.pool_k != 5) {
      err = "SPPF pool size must be 5";
      return false;
    }
    yk_op op;
    memset(&op, 0, sizeof op);
    op.kind = YK_K_SPPF_POOL;
    op.n_src = 1;
    op.src[0] = yk_view{Z, 0, 4 * cp, hh, ww, 0};
    op.src_ch[0] = cp;
    op.dst = yk_view{Z, cp, 4 * cp, hh, ww, 0};
    op.cout = cp;
    op.out_h = hh;
    op.out_w = ww;
    ops.push_back(op);
    const int c2p = phys(L.c2);
    const int ob = new_buf(hh, ww, c2p);
    const Seg dst{ob, 0, c2p, c2p, L.c2, hh, ww, 0};
    if (!conv_op(p + ".cv2", zs, dst, iota(L.c2), c2p)) return false;
    out = {dst};
    return true;
  }

  // Program._detect (model.py:353-401)
  bool detect(const Layer& L, const std::vector<std::vector<Seg>>& lv) {
    const int c2b = L.c2b, c3 = L.c3, nc = L.nc;
    if (nc != 1 || c2b != 64) {
      err = "decode kernel: single class, 64 box channels";
      return false;
    }
    const int c3p = phys(c3);
    const std::string p = "model." + std::to_string(L.i);
    int anchor_off = 0;
    for (size_t li = 0; li < lv.size(); ++li) {
      const std::vector<Seg>& src = lv[li];
      const int hh = src[0].lh(), ww = src[0].lw();
      const int width = 64 + c3p;
      const int H1 = new_buf(hh, ww, width), H2 = new_buf(hh, ww, width);
      const std::string l = std::to_string(li);
      const Fused& A = fused[p + ".cv2." + l + ".0"];
      const Fused& Bc = fused[p + ".cv3." + l + ".0"];
      Fused cat;
      cat.c1 = A.c1;
      cat.c2 = A.c2 + Bc.c2;
      cat.k = 3;
      cat.s = 1;
      cat.act = true;
      cat.w = A.w;
      cat.w.insert(cat.w.end(), Bc.w.begin(), Bc.w.end());
      cat.b = A.b;
      cat.b.insert(cat.b.end(), Bc.b.begin(), Bc.b.end());
      fused[p + ".head." + l + ".0"] = cat;
      std::vector<int> om = iota(64);
      for (int o = 0; o < c3; ++o) om.push_back(64 + o);
      if (!conv_op(p + ".head." + l + ".0", src, Seg{H1, 0, width, width, 64 + c3, hh, ww, 0}, om, width)) return false;
      if (!conv_op(p + ".cv2." + l + ".1", {Seg{H1, 0, width, 64, 64, hh, ww, 0}}, Seg{H2, 0, width, 64, 64, hh, ww, 0},
                   iota(64), 64))
        return false;
      if (!conv_op(p + ".cv3." + l + ".1", {Seg{H1, 64, width, c3p, c3, hh, ww, 0}},
                   Seg{H2, 64, width, c3p, c3, hh, ww, 0}, iota(c3), c3p))
        return false;
      Packed P;
      if (!pack(fused[p + ".cv2." + l + ".2"], {Seg{H2, 0, width, 64, 64, hh, ww, 0}}, iota(64), 64, P)) return false;
      const Fused& cls = fused[p + ".cv3." + l + ".2"];
      std::vector<float> wc(c3p + 4, 0.f);
      for (int j = 0; j < c3; ++j) wc[j] = cls.w[j];
      wc[c3p] = cls.b[0];
      yk_op op;
      memset(&op, 0, sizeof op);
      op.kind = YK_K_DETECT;
      op.n_src = 1;
      op.src[0] = yk_view{H2, 0, width, hh, ww, 0};
      op.src_ch[0] = 64;
      op.dst = yk_view{H2, 0, width, hh, ww, 0};
      op.out_h = hh;
      op.out_w = ww;
      op.k_steps = P.k_steps;
      op.n_tiles = P.n_tiles;
      op.w_off = add_blob(P.packed);
      op.b_off = add_blob(P.bias);
      op.t_off = op.b_off;
      op.det_stride = strides[li];
      op.det_anchor_off = anchor_off;
      op.det_cls_off = 64;
      op.det_cls_ch = c3p;
      op.det_wc_off = add_blob(wc);
      ops.push_back(op);
      anchor_off += hh * ww;
    }
    n_anchors = anchor_off;
    return true;
  }
};

// ---------------------------------------------------------------- LetterBox (letterbox.py)
struct LbPlan {
  int in_h, in_w, top, left, new_h, new_w, mode;
  std::vector<int32_t> xofs, yofs;
  std::vector<int16_t> xw, yw;  // pairs
  double gain;
  int pad_x, pad_y;
};

void lb_coeffs(int dst, int src, bool clamp, std::vector<int32_t>& ofs, std::vector<int16_t>& w) {
  const double scale = 1.0 / ((double)dst / src);
  ofs.assign(dst, 0);
  w.assign(2 * (size_t)dst, 0);
  for (int d = 0; d < dst; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f = f - (float)s;
    if (clamp && s < 0) s = 0, f = 0.f;
    if (clamp && s + 1 >= src) s = src - 1, f = 0.f;
    const float c0 = (1.0f - f) * 2048.0f, c1 = f * 2048.0f;
    ofs[d] = s;
    w[2 * d] = (int16_t)std::min(std::max(std::nearbyint((double)c0), -32768.0), 32767.0);
    w[2 * d + 1] = (int16_t)std::min(std::max(std::nearbyint((double)c1), -32768.0), 32767.0);
  }
}

LbPlan lb_plan(int fh, int fw, int imgsz, int stride) {
  LbPlan p{};
  const double r = std::min((double)imgsz / fh, (double)imgsz / fw);
  p.new_w = (int)std::nearbyint(fw * r);
  p.new_h = (int)std::nearbyint(fh * r);
  const double dw = ((imgsz - p.new_w) % stride) / 2.0, dh = ((imgsz - p.new_h) % stride) / 2.0;
  p.top = (int)std::nearbyint(dh - 0.1);
  const int bottom = (int)std::nearbyint(dh + 0.1);
  p.left = (int)std::nearbyint(dw - 0.1);
  const int right = (int)std::nearbyint(dw + 0.1);
  p.in_h = p.new_h + p.top + bottom;
  p.in_w = p.new_w + p.left + right;
  p.mode = 0;
  if (p.new_w != fw || p.new_h != fh) {
    const double sx = 1.0 / ((double)p.new_w / fw), sy = 1.0 / ((double)p.new_h / fh);
    if (std::fabs(sx - std::nearbyint(sx)) < DBL_EPSILON && std::fabs(sy - std::nearbyint(sy)) < DBL_EPSILON &&
        std::nearbyint(sx) == 2 && std::nearbyint(sy) == 2)
      p.mode = 2;
    else
      p.mode = 1;
    lb_coeffs(p.new_w, fw, true, p.xofs, p.xw);
    lb_coeffs(p.new_h, fh, false, p.yofs, p.yw);
  }
  p.gain = std::min((double)p.in_h / fh, (double)p.in_w / fw);
  p.pad_x = (int)std::nearbyint((p.in_w - fw * p.gain) / 2 - 0.1);
  p.pad_y = (int)std::nearbyint((p.in_h - fh * p.gain) / 2 - 0.1);
  return p;
}

std::vector<int32_t> lb_table(const LbPlan& p) {
  if (p.mode == 0) return std::vector<int32_t>(4, 0);
  std::vector<int32_t> t(p.xofs);
  t.insert(t.end(), p.yofs.begin(), p.yofs.end());
  const size_t nx = p.xw.size() / 2, ny = p.yw.size() / 2;
  std::vector<int32_t> x(nx), y(ny);
  if (nx) memcpy(x.data(), p.xw.data(), nx * 4);
  if (ny) memcpy(y.data(), p.yw.data(), ny * 4);
  t.insert(t.end(), x.begin(), x.end());
  t.insert(t.end(), y.begin(), y.end());
  return t;
}

}  // namespace

struct yk_program {
  yk_model_desc desc;
  std::vector<int64_t> buf_elems;
  std::vector<yk_op> ops;
  std::vector<unsigned char> blob;
};

extern "C" {

int yk_program_build(const yk_weights* weights, char scale, int act_dtype, int frame_h, int frame_w, int imgsz,
                     int max_batch, int max_det, yk_program** out) {
  YK_CHECK_ARG(weights && out && (weights->n == 0 || weights->tensors), "yk_program_build: NULL argument");
  YK_CHECK_ARG(act_dtype == YK_ACT_BF16 || act_dtype == YK_ACT_F32 || act_dtype == YK_ACT_FP8 || act_dtype == YK_ACT_F16,
               "yk_program_build: act_dtype must be YK_ACT_BF16, YK_ACT_F32, YK_ACT_FP8 or YK_ACT_F16");
  YK_CHECK_ARG(frame_h > 0 && frame_w > 0 && imgsz >= 32 && imgsz % 32 == 0 && max_batch >= 1 && max_det >= 1,
               "yk_program_build: bad frame size, imgsz (a multiple of 32), max_batch or max_det");
  *out = nullptr;
  WeightsView W;
  for (int i = 0; i < weights->n; ++i) {
    const yk_tensor& t = weights->tensors[i];
    YK_CHECK_ARG(t.name, "yk_program_build: tensor without a name");
    W.by_name[t.name] = &t;
  }
  // nc from the class branch's last conv (Detect cv3.0.2: [nc, c3, 1, 1])
  const std::string det = "model." + std::to_string(kLayers - 1);
  auto itc = W.by_name.find(det + ".cv3.0.2.weight");
  YK_CHECK_ARG(itc != W.by_name.end() && itc->second->ndim == 4, "yk_program_build: state dict has no Detect cv3.0.2");
  const int nc = (int)itc->second->shape[0];
  std::vector<Layer> ar;
  std::string err;
  if (!parse(scale, nc, ar, err)) {
    yk::set_error("yk_program_build: " + err);
    return YK_ERR_ARG;
  }
  Builder Bd;
  Bd.dtype = act_dtype;
  Bd.esz = act_dtype == YK_ACT_F32 ? 4 : act_dtype == YK_ACT_FP8 ? 1 : 2;
  Bd.epl = 16 / Bd.esz;
  Bd.align = act_dtype == YK_ACT_FP8 ? 16 : 8;
  Bd.strides = detect_strides(ar);
  // conv_specs (arch.py:158-187) -> fused weights
  for (const Layer& L : ar) {
    const std::string p = "model." + std::to_string(L.i);
    bool ok = true;
    if (L.kind == "Conv") {
      ok = fuse(W, p, L.c1[0], L.c2, L.k, L.s, true, Bd.fused[p], err);
    } else if (L.kind == "C2f") {
      const int c = (int)(L.c2 * 0.5);
      ok = fuse(W, p + ".cv1", L.c1[0], 2 * c, 1, 1, true, Bd.fused[p + ".cv1"], err);
      for (int j = 0; ok && j < L.n; ++j) {
        const std::string m = p + ".m." + std::to_string(j);
        ok = fuse(W, m + ".cv1", c, c, 3, 1, true, Bd.fused[m + ".cv1"], err) &&
             fuse(W, m + ".cv2", c, c, 3, 1, true, Bd.fused[m + ".cv2"], err);
      }
      ok = ok && fuse(W, p + ".cv2", (2 + L.n) * c, L.c2, 1, 1, true, Bd.fused[p + ".cv2"], err);
    } else if (L.kind == "SPPF") {
      const int c_ = L.c1[0] / 2;
      ok = fuse(W, p + ".cv1", L.c1[0], c_, 1, 1, true, Bd.fused[p + ".cv1"], err) &&
           fuse(W, p + ".cv2", c_ * 4, L.c2, 1, 1, true, Bd.fused[p + ".cv2"], err);
    } else if (L.kind == "Detect") {
      for (size_t li = 0; ok && li < L.c1.size(); ++li) {
        const std::string a = p + ".cv2." + std::to_string(li), c = p + ".cv3." + std::to_string(li);
        const int x = L.c1[li];
        ok = fuse(W, a + ".0", x, L.c2b, 3, 1, true, Bd.fused[a + ".0"], err) &&
             fuse(W, a + ".1", L.c2b, L.c2b, 3, 1, true, Bd.fused[a + ".1"], err) &&
             fuse(W, a + ".2", L.c2b, 4 * kRegMax, 1, 1, false, Bd.fused[a + ".2"], err) &&
             fuse(W, c + ".0", x, L.c3, 3, 1, true, Bd.fused[c + ".0"], err) &&
             fuse(W, c + ".1", L.c3, L.c3, 3, 1, true, Bd.fused[c + ".1"], err) &&
             fuse(W, c + ".2", L.c3, nc, 1, 1, false, Bd.fused[c + ".2"], err);
      }
    }
    if (!ok) {
      yk::set_error("yk_program_build: " + err);
      return YK_ERR_ARG;
    }
  }
  const LbPlan lb = lb_plan(frame_h, frame_w, imgsz, *std::max_element(Bd.strides.begin(), Bd.strides.end()));
  // Program._build (model.py:247-304)
  std::map<int, std::vector<Seg>> outs;
  std::vector<Seg> prev;
  bool ok = true;
  for (const Layer& L : ar) {
    auto inp = [&](int f) -> std::vector<Seg> { return f == -1 ? prev : outs[f]; };
    std::vector<Seg> out;
    if (L.kind == "Conv" && L.i == 0) {
      const int k = L.k, s = L.s;
      const int oh = (lb.in_h + 2 * (k / 2) - k) / s + 1, ow = (lb.in_w + 2 * (k / 2) - k) / s + 1;
      const int cp = Bd.phys(L.c2);
      const int buf = Bd.new_buf(oh, ow, cp);
      const Fused& F = Bd.fused["model.0"];
      std::vector<float> W0((size_t)cp * 3 * k * k, 0.f), B0(cp, 0.f);
      std::copy(F.w.begin(), F.w.end(), W0.begin());
      std::copy(F.b.begin(), F.b.end(), B0.begin());
      yk_op op;
      memset(&op, 0, sizeof op);
      op.kind = YK_K_CONV_INPUT;
      op.ksize = k;
      op.stride = s;
      op.act = 1;
      op.dst = yk_view{buf, 0, cp, oh, ow, 0};
      op.cout = cp;
      op.out_h = oh;
      op.out_w = ow;
      op.w_off = Bd.add_blob(W0);
      op.b_off = Bd.add_blob(B0);
      op.t_off = op.b_off;
      Bd.ops.push_back(op);
      out = {Seg{buf, 0, cp, cp, L.c2, oh, ow, 0}};
    } else if (L.kind == "Conv") {
      const std::vector<Seg> src = inp(L.f[0]);
      const int k = L.k, s = L.s;
      const int oh = (src[0].lh() + 2 * (k / 2) - k) / s + 1, ow = (src[0].lw() + 2 * (k / 2) - k) / s + 1;
      const int cp = Bd.phys(L.c2);
      const int buf = Bd.new_buf(oh, ow, cp);
      const Seg dst{buf, 0, cp, cp, L.c2, oh, ow, 0};
      ok = Bd.conv_op("model." + std::to_string(L.i), src, dst, Bd.iota(L.c2), cp);
      out = {dst};
    } else if (L.kind == "C2f") {
      ok = Bd.c2f(L, inp(L.f[0]), out);
    } else if (L.kind == "SPPF") {
      ok = Bd.sppf(L, inp(L.f[0]), out);
    } else if (L.kind == "Upsample") {
      if (L.up != 2) {
        Bd.err = "only nn.Upsample(scale_factor=2)";
        ok = false;
      }
      for (Seg s : inp(L.f[0])) {
        s.up += 1;
        out.push_back(s);
      }
    } else if (L.kind == "Concat") {
      for (int f : L.f)
        for (const Seg& s : inp(f)) out.push_back(s);
    } else {
      std::vector<std::vector<Seg>> lv;
      for (int f : L.f) lv.push_back(inp(f));
      ok = Bd.detect(L, lv);
    }
    if (!ok) {
      yk::set_error("yk_program_build: " + Bd.err);
      return YK_ERR_ARG;
    }
    outs[L.i] = out;
    prev = out;
  }
  const int64_t rs_tab_off = Bd.add_blob(lb_table(lb));
  yk_program* p = new yk_program();
  p->buf_elems = std::move(Bd.buf_elems);
  p->ops = std::move(Bd.ops);
  p->blob = std::move(Bd.blob);
  yk_model_desc& d = p->desc;
  memset(&d, 0, sizeof d);
  d.act_dtype = act_dtype;
  d.max_batch = max_batch;
  d.frame_h = frame_h;
  d.frame_w = frame_w;
  d.in_h = lb.in_h;
  d.in_w = lb.in_w;
  d.pad_top = lb.top;
  d.pad_left = lb.left;
  d.n_anchors = Bd.n_anchors;
  d.nc = nc;
  d.max_det = max_det;
  d.n_bufs = (int32_t)p->buf_elems.size();
  d.buf_elems = p->buf_elems.data();
  d.n_ops = (int32_t)p->ops.size();
  d.ops = p->ops.data();
  d.rs_mode = lb.mode;
  d.rs_w = lb.new_w;
  d.rs_h = lb.new_h;
  d.box_pad_x = lb.pad_x;
  d.box_pad_y = lb.pad_y;
  d.box_gain = (float)lb.gain;
  d.rs_tab_off = rs_tab_off;
  // a program yk_model_create would refuse (sizes beyond the kernels' limits, e.g. max_det > 2048)
  // is refused here already, with the same message
  if (const int rc = yk::validate_model_desc(&d, (int64_t)p->blob.size())) {
    delete p;
    return rc;
  }
  *out = p;
  return YK_OK;
}

int yk_program_get(const yk_program* p, const yk_model_desc** desc, const void** blob, int64_t* blob_bytes) {
  YK_CHECK_ARG(p && desc && blob && blob_bytes, "yk_program_get: NULL argument");
  *desc = &p->desc;
  *blob = p->blob.data();
  *blob_bytes = (int64_t)p->blob.size();
  return YK_OK;
}

int yk_program_destroy(yk_program* p) {
  delete p;
  return YK_OK;
}

}  // extern "C"
