// Host-only entry points and checks of the C ABI: error state, yk_abi_version / yk_last_error, the
// detector-program validation yk_model_create runs first, and the engine-file reader of
// yk_model_load.  Built into libyk.so, and on its own (with program.cpp) under AddressSanitizer /
// UBSan by tests/test_asan_cpu.py.
#include "yk_host.h"

#include <cstring>
#include <fstream>

namespace yk {
namespace {
thread_local std::string g_last_error;

bool in_blob(int64_t off, int64_t bytes, int64_t blob) {
  return off >= 0 && bytes >= 0 && off <= blob && bytes <= blob - off;
}

// view v of a buffer, `ch` channels read or written from its c_off
bool view_ok(const yk_model_desc* d, const yk_view& v, int64_t ch) {
  if (v.buf < 0 || v.buf >= d->n_bufs) return false;
  if (v.c_stride < 1 || v.c_off < 0 || v.h < 1 || v.w < 1 || v.h > 32768 || v.w > 32768) return false;
  if (v.up != 0 && v.up != 1) return false;
  if (ch < 1 || (int64_t)v.c_off + ch > v.c_stride) return false;
  return (int64_t)v.h * v.w * v.c_stride <= d->buf_elems[v.buf];
}
}  // namespace

void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }

int validate_model_desc(const yk_model_desc* desc, int64_t blob_bytes) {
  YK_CHECK_ARG(desc, "yk_model_create: NULL argument");
  YK_CHECK_ARG(desc->n_ops > 0 && desc->ops && desc->n_bufs > 0 && desc->buf_elems, "yk_model_create: empty program");
  YK_CHECK_ARG(desc->n_ops < (1 << 16) && desc->n_bufs < (1 << 16), "yk_model_create: too many ops or buffers");
  YK_CHECK_ARG(blob_bytes > 0, "yk_model_create: empty weight blob");
  YK_CHECK_ARG(desc->max_batch >= 1 && desc->n_anchors > 0 && desc->max_det >= 1, "yk_model_create: bad sizes");
  YK_CHECK_ARG(desc->max_batch <= 4096, "yk_model_create: max_batch must be <= 4096");
  YK_CHECK_ARG(desc->nc == 1, "yk_model_create: only single-class detection heads are supported");
  YK_CHECK_ARG(desc->max_det <= 2048, "yk_model_create: max_det must be <= 2048");
  YK_CHECK_ARG(desc->act_dtype == YK_ACT_BF16 || desc->act_dtype == YK_ACT_F32 || desc->act_dtype == YK_ACT_FP8 ||
                   desc->act_dtype == YK_ACT_F16,
               "yk_model_create: bad act dtype");
  YK_CHECK_ARG(desc->frame_h >= 1 && desc->frame_w >= 1 && desc->frame_h <= 32768 && desc->frame_w <= 32768 &&
                   desc->in_h >= 1 && desc->in_w >= 1 && desc->in_h <= 32768 && desc->in_w <= 32768,
               "yk_model_create: frame / input size out of range [1, 32768]");
  YK_CHECK_ARG(desc->pad_top >= 0 && desc->pad_left >= 0 && desc->pad_top < desc->in_h && desc->pad_left < desc->in_w,
               "yk_model_create: LetterBox padding outside the input");
  YK_CHECK_ARG(desc->n_anchors <= (int64_t)desc->in_h * desc->in_w, "yk_model_create: more anchors than input pixels");
  for (int i = 0; i < desc->n_bufs; ++i)
    YK_CHECK_ARG(desc->buf_elems[i] >= 1 && desc->buf_elems[i] <= (int64_t(1) << 34),
                 "yk_model_create: buffer size out of range");
  const bool fp8 = desc->act_dtype == YK_ACT_FP8;
  for (int i = 0; i < desc->n_ops; ++i) {
    const yk_op& op = desc->ops[i];
    const std::string at = " (op " + std::to_string(i) + ", kind " + std::to_string(op.kind) + ")";
    YK_CHECK_ARG(op.kind >= YK_K_CONV_INPUT && op.kind <= YK_K_DETECT, std::string("yk_model_create: bad op kind") + at);
    YK_CHECK_ARG(op.dst.buf >= 0 && op.dst.buf < desc->n_bufs, std::string("yk_model_create: dst buffer index out of range") + at);
    YK_CHECK_ARG(op.n_src >= (op.kind == YK_K_CONV_INPUT ? 0 : 1) && op.n_src <= 2, std::string("yk_model_create: n_src") + at);
    for (int s = 0; s < op.n_src; ++s)
      YK_CHECK_ARG(op.src[s].buf >= 0 && op.src[s].buf < desc->n_bufs, std::string("yk_model_create: src buffer out of range") + at);
    YK_CHECK_ARG(op.w_off >= 0 && op.w_off < blob_bytes && op.b_off >= 0 && op.b_off < blob_bytes,
                 std::string("yk_model_create: weight offsets outside the blob") + at);
    YK_CHECK_ARG(op.out_h >= 1 && op.out_w >= 1 && op.out_h <= 32768 && op.out_w <= 32768,
                 std::string("yk_model_create: op output size out of range") + at);
    YK_CHECK_ARG((op.kind != YK_K_CONV && op.kind != YK_K_CONV_INPUT) ||
                     ((op.ksize == 1 || op.ksize == 3) && (op.stride == 1 || op.stride == 2) && (op.act == 0 || op.act == 1)),
                 std::string("yk_model_create: conv ksize must be 1 or 3, stride 1 or 2, act 0 or 1") + at);
    switch (op.kind) {
      case YK_K_CONV: {
        YK_CHECK_ARG(op.cout % 4 == 0 && op.k_steps > 0 && op.n_tiles > 0, std::string("yk_model_create: conv geometry") + at);
        YK_CHECK_ARG(op.n_tiles <= 4096 && op.k_steps <= 4096 && op.cout >= 4 && op.cout <= op.n_tiles * 16,
                     std::string("yk_model_create: conv geometry (cout within the packed tiles)") + at);
        for (int s = 0; s < op.n_src; ++s)
          YK_CHECK_ARG(op.src_ch[s] >= 1 && op.src_ch[s] <= 65536, std::string("yk_model_create: conv source channels") + at);
        YK_CHECK_ARG((int64_t)op.ksize * op.ksize * ((int64_t)op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0)) / 8 <= kTabMax,
                     std::string("yk_model_create: conv input too wide (K-chunk table > 1024 entries)") + at);
        for (int s = 0; s < op.n_src; ++s)
          YK_CHECK_ARG(view_ok(desc, op.src[s], op.src_ch[s]), std::string("yk_model_create: conv source view outside its buffer") + at);
        YK_CHECK_ARG(view_ok(desc, op.dst, op.cout) && op.dst.h == op.out_h && op.dst.w == op.out_w && op.dst.up == 0,
                     std::string("yk_model_create: conv output view outside its buffer") + at);
        YK_CHECK_ARG(!op.has_res || (view_ok(desc, op.res, op.cout) && op.res.h == op.out_h && op.res.w == op.out_w),
                     std::string("yk_model_create: residual view outside its buffer") + at);
        YK_CHECK_ARG(in_blob(op.w_off, (int64_t)op.n_tiles * op.k_steps * 64 * 16, blob_bytes) &&
                         in_blob(op.b_off, (int64_t)(fp8 ? op.n_tiles * 16 + op.cout : op.cout) * 4, blob_bytes) &&
                         in_blob(op.t_off, 0, blob_bytes),
                     std::string("yk_model_create: conv weights outside the blob") + at);
        break;
      }
      case YK_K_CONV_INPUT:
        YK_CHECK_ARG(op.ksize == 3 && op.stride <= 2, std::string("yk_model_create: the input conv must be 3x3 with stride <= 2") + at);
        YK_CHECK_ARG(op.cout >= 1 && op.cout <= kInputCoutMax,
                     std::string("yk_model_create: the input conv must have <= 64 (padded) output channels") + at);
        YK_CHECK_ARG(view_ok(desc, op.dst, op.cout) && op.dst.h == op.out_h && op.dst.w == op.out_w,
                     std::string("yk_model_create: input conv output view outside its buffer") + at);
        YK_CHECK_ARG(in_blob(op.w_off, (int64_t)op.cout * 27 * 4, blob_bytes) && in_blob(op.b_off, (int64_t)op.cout * 4, blob_bytes),
                     std::string("yk_model_create: input conv weights outside the blob") + at);
        break;
      case YK_K_SPPF_POOL:
        YK_CHECK_ARG(op.src_ch[0] >= 1 && view_ok(desc, op.src[0], 4 * (int64_t)op.src_ch[0]),
                     std::string("yk_model_create: SPPF view outside its buffer (4 concat slices)") + at);
        break;
      case YK_K_DETECT: {
        const yk_view& v = op.src[0];
        YK_CHECK_ARG(view_ok(desc, v, 1) && op.det_cls_ch >= 1 && op.det_cls_off >= 0 &&
                         (int64_t)v.c_off + op.det_cls_off + op.det_cls_ch <= v.c_stride && op.k_steps > 0 &&
                         op.k_steps <= 4096,
                     std::string("yk_model_create: Detect feature view outside its buffer") + at);
        YK_CHECK_ARG(op.det_stride >= 1 && op.det_anchor_off >= 0 &&
                         (int64_t)op.det_anchor_off + (int64_t)v.h * v.w <= desc->n_anchors,
                     std::string("yk_model_create: Detect anchors outside [0, n_anchors)") + at);
        YK_CHECK_ARG(in_blob(op.w_off, (int64_t)4 * op.k_steps * 64 * 16, blob_bytes) &&
                         in_blob(op.b_off, 64 * 4, blob_bytes) &&
                         in_blob(op.det_wc_off, ((int64_t)op.det_cls_ch + 1) * 4, blob_bytes),
                     std::string("yk_model_create: Detect weights outside the blob") + at);
        break;
      }
    }
  }
  YK_CHECK_ARG(desc->rs_mode >= 0 && desc->rs_mode <= 2, "yk_model_create: bad resize mode");
  YK_CHECK_ARG(desc->rs_mode == 0 ||
                   (desc->rs_w >= 1 && desc->rs_h >= 1 && (int64_t)desc->pad_left + desc->rs_w <= desc->in_w &&
                    (int64_t)desc->pad_top + desc->rs_h <= desc->in_h &&
                    in_blob(desc->rs_tab_off, (2 * (int64_t)desc->rs_w + 2 * (int64_t)desc->rs_h) * 4, blob_bytes) &&
                    (desc->rs_mode != 2 || (2 * (int64_t)desc->rs_w <= desc->frame_w && 2 * (int64_t)desc->rs_h <= desc->frame_h))),
               "yk_model_create: inconsistent LetterBox resize geometry");
  YK_CHECK_ARG(desc->rs_mode != 0 || ((int64_t)desc->pad_top + desc->frame_h <= desc->in_h &&
                                      (int64_t)desc->pad_left + desc->frame_w <= desc->in_w),
               "yk_model_create: the frame does not fit the network input");
  YK_CHECK_ARG(desc->box_gain > 0.f, "yk_model_create: box_gain must be > 0");
  return YK_OK;
}

int read_engine(const char* path, EngineImage& e) {
  YK_CHECK_ARG(path, "yk_model_load: NULL argument");
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  YK_CHECK_ARG(f.good(), std::string("yk_model_load: cannot open ") + path);
  const int64_t size = (int64_t)f.tellg();
  f.seekg(0);
  struct Head {
    char magic[8];
    int32_t version, sizeof_desc, sizeof_op, n_bufs, n_ops, plan_batch, n_plan, pad;
    int64_t blob_bytes;
  } h{};
  YK_CHECK_ARG(size >= (int64_t)sizeof h, "yk_model_load: not a YKENGINE file");
  f.read((char*)&h, sizeof h);
  YK_CHECK_ARG(f.good() && std::memcmp(h.magic, "YKENGINE", 8) == 0, "yk_model_load: not a YKENGINE file");
  YK_CHECK_ARG(h.version == 1, "yk_model_load: unsupported engine version");
  YK_CHECK_ARG(h.sizeof_desc == (int32_t)sizeof(yk_model_desc) && h.sizeof_op == (int32_t)sizeof(yk_op),
               "yk_model_load: engine written for another ABI (struct sizes differ)");
  YK_CHECK_ARG(h.n_bufs > 0 && h.n_bufs < (1 << 16) && h.n_ops > 0 && h.n_ops < (1 << 16) && h.blob_bytes > 0 &&
                   h.n_plan >= 0 && h.n_plan <= h.n_ops,
               "yk_model_load: corrupt engine header");
  // every section's size from the header, against the file: nothing is allocated from a count
  // the file does not back
  const int64_t fixed = (int64_t)sizeof h + (int64_t)sizeof(yk_model_desc) + (int64_t)h.n_bufs * 8 +
                        (int64_t)h.n_ops * (int64_t)sizeof(yk_op) + (int64_t)h.n_plan * 16;
  YK_CHECK_ARG(h.blob_bytes <= size - fixed, "yk_model_load: truncated engine file");
  YK_CHECK_ARG(h.blob_bytes == size - fixed, "yk_model_load: trailing bytes after the engine");
  f.read((char*)&e.desc, sizeof e.desc);
  e.buf_elems.resize(h.n_bufs);
  e.ops.resize(h.n_ops);
  e.blob.resize((size_t)h.blob_bytes);
  e.plan.resize((size_t)h.n_plan * 4);
  f.read((char*)e.buf_elems.data(), (std::streamsize)(e.buf_elems.size() * sizeof(int64_t)));
  f.read((char*)e.ops.data(), (std::streamsize)(e.ops.size() * sizeof(yk_op)));
  f.read(e.blob.data(), (std::streamsize)e.blob.size());
  if (h.n_plan) f.read((char*)e.plan.data(), (std::streamsize)(e.plan.size() * sizeof(int32_t)));
  YK_CHECK_ARG(f.good(), "yk_model_load: truncated engine file");
  YK_CHECK_ARG(e.desc.n_bufs == h.n_bufs && e.desc.n_ops == h.n_ops, "yk_model_load: header / descriptor mismatch");
  e.desc.buf_elems = e.buf_elems.data();
  e.desc.ops = e.ops.data();
  e.plan_batch = h.plan_batch;
  YK_CHECK_ARG(h.n_plan == 0 || (h.plan_batch >= 1 && h.plan_batch <= e.desc.max_batch),
               "yk_model_load: plan batch outside [1, max_batch]");
  for (int32_t i = 0; i < h.n_plan; ++i)
    YK_CHECK_ARG(e.plan[(size_t)i * 4] >= -1 && e.plan[(size_t)i * 4] < h.n_ops, "yk_model_load: plan op index out of range");
  return validate_model_desc(&e.desc, h.blob_bytes);
}

}  // namespace yk

extern "C" {

int yk_abi_version(void) { return YK_ABI_VERSION; }

const char* yk_last_error(void) { return yk::g_last_error.c_str(); }

}  // extern "C"
