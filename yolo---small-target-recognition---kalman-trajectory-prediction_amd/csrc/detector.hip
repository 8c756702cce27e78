// YOLOv8-small+P2 detector for gfx950 (MI355X): the predict() hot path as HIP kernels.
//
//   conv_input_kernel  first conv straight from uint8 BGR frames: LetterBox padding, BGR->RGB
//                      and /255 fused into the gather (engine/predictor.py:152-204,
//                      data/augment.py:1667-1744); f32 VALU (K = 27, 0.6% of the FLOPs)
//   conv_igemm_kernel  every other conv (nn/modules/conv.py:39-93, block.py C2f/Bottleneck/SPPF)
//                      as an implicit GEMM on MFMA: bf16 16x16x32 (or exact-f32 16x16x4 for the
//                      parity build).  The weights are the A operand (rows = output channels),
//                      activations the B operand (columns = pixels), so each lane ends with 4
//                      consecutive output channels of one pixel -> one 8/16-byte NHWC store.
//                      Epilogue: bias + SiLU + optional residual (Bottleneck add), written into
//                      a channel slice of the consumer's buffer (torch.cat / chunk disappear);
//                      up to two sources (Concat) with per-source nearest-upsample (nn.Upsample).
//   sppf_pool_kernel   SPPF's three chained MaxPool2d(5,1,2) = windows 5/9/13, one pass.
//   detect_kernel      Detect level: box 1x1 (MFMA) + DFL softmax-expectation + dist2bbox x stride
//                      + cls 1x1 + sigmoid + conf threshold, compacted into per-image candidate
//                      lists (nn/modules/head.py:116-187, utils/tal.py:367-391, utils/nms.py:77-123).
//   nms_kernel         per image: stable (score desc, anchor asc) sort, TorchNMS.nms greedy loop
//                      with its "no overlap -> keep all remaining" early exit (utils/nms.py:237-304),
//                      max_det cut, scale_boxes + clip_boxes (utils/ops.py:105-184).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <algorithm>
#include <array>
#include <map>
#include <tuple>
#include <vector>

#include "yk_internal.h"
#include "yk_diag.h"

// Diagnostic builds.  csrc/build.py YK_DEFINES="-DYK_DIAG=<mask>" builds libyk_diag.so with its
// own objects; the product library is always built with YK_DIAG = 0, where every bit below is off
// and the diagnostic branches are discarded at compile time.
//     1  F32S: operands used unsplit (no split VALU)      2  F32S: no weight loads
//     4  halo kernel: no weight loads                     8  halo kernel: no input staging
//    32  F32S split with scalar remainders               64  fp32 SiLU on v_exp_f32 / v_rcp_f32
//   128  two waves per SIMD for the table / halo kernels (amdgpu_waves_per_eu(2))
//   512  F32S: operands used as if stored pre-split (no split VALU, overlapping register quads)
//  1024  conv_fast: one K step of loads in flight for the large tiles instead of two (registers)
#ifndef YK_DIAG
#define YK_DIAG 0
#endif
#define YK_SPLIT_DIAG (YK_DIAG & 3)
#define YK_HALO_DIAG ((YK_DIAG >> 2) & 3)
#define YK_SPLIT_PK ((YK_DIAG & 32) == 0)
#define YK_EXACT_SILU ((YK_DIAG & 64) == 0)
#ifndef YK_FAST_WPE  // (a diagnostic build may set it: YK_DEFINES=-DYK_FAST_WPE=3)
#define YK_FAST_WPE ((YK_DIAG & 128) ? 2 : 1)
#endif
// The table-kernel tiles of at most YK_WPE_TILE fragments (NNT x NPT) with two K steps of loads in
// flight are compiled for 3 waves per SIMD (<= 168 registers) -- except the 12-fragment tile
// without a K split, which spills there, and FP8 -- the others as YK_FAST_WPE.  12 (round 6): the
// dominant <F32S, 3, 4, 4, 2> 200 -> 166 registers, 22.0 -> 21.0 us per launch, fp32 line +1 %
// (A/B x3, gpurun_out/r6d); 0 restores the round-5 allocation
#ifndef YK_WPE_TILE
#define YK_WPE_TILE 12
#endif
constexpr int fast_wpe(int nnt, int npt, int kw, int skd, bool fp8) {
  return !fp8 && nnt * npt <= YK_WPE_TILE && skd == 2 && !(kw == 1 && nnt * npt >= 12) ? 3 : YK_FAST_WPE;
}
// YK_STORE_CHECK=1 (diagnostic build): every detector-kernel store -- the conv
// epilogues (store4), detect_kernel's candidate rows, nms_kernel's outputs and global scratch --
// checks that its bytes lie inside one of the detector's own allocations (every model's arena,
// candidate / NMS buffers, letterbox canvas, and the detection buffers handed to yk_detect); a
// store outside them prints its site and address and is counted (yk_store_check_count).
#ifndef YK_STORE_CHECK
#define YK_STORE_CHECK 0
#endif

namespace yk {
namespace det {

#if YK_STORE_CHECK
constexpr int kScMax = 256;
__device__ unsigned long long sc_lo[kScMax], sc_hi[kScMax];
__device__ int sc_n;
__device__ unsigned long long sc_bad;
__device__ __noinline__ void sc_fail(const void* p, int bytes, int site) {
  const unsigned long long c = atomicAdd(&sc_bad, 1ull);
  if (c < 16) printf("[yk store check] site %d: %d bytes at %p outside every detector allocation\n", site, bytes, p);
}
__device__ __forceinline__ void sc_check(const void* p, int bytes, int site) {
  const unsigned long long a = (unsigned long long)p;
  bool ok = false;
  for (int i = 0; i < sc_n; ++i) ok = ok || (a >= sc_lo[i] && a + (unsigned long long)bytes <= sc_hi[i]);
  if (!ok) sc_fail(p, bytes, site);
}
#define YK_SC(p, bytes, site) sc_check((const void*)(p), (bytes), (site))
#else
#define YK_SC(p, bytes, site) ((void)0)
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Workgroup -> (pixel tile, channel group), XCD-aware.  The dispatcher deals workgroups (linear id,
// x fastest) round-robin to the 8 XCDs, each with its own 4 MiB L2 (MI355X_MICROARCH.md, "Workgroup
// dispatch, XCD placement").  With `on`, linear id L is mapped so that XCD L % 8 owns one contiguous
// range of work items ordered (pixel tile major, channel group minor): sibling channel groups of a
// pixel tile and neighbouring pixel tiles (the rows a 3x3 window shares) meet in one L2 instead of
// being fetched once per XCD.  Placement only: the mapping is a bijection either way.
// XCD k runs a contiguous range of (pixel block, channel group) items in pixel-major order (a
// block's channel groups on one XCD: its activations are fetched into one L2).  (Round 4: a
// channel-group-major order for the weight-heavy P5 convs cut their PMC bytes 3.73x -> 3.18x of
// algorithmic but not their time, 25.3 vs 25.8 µs; not kept.)
// The same placement for a persistent launch's item q of n (gy channel groups): item q runs on the
// workgroup q % gridDim.x, whose XCD is q % 8 when gridDim.x is a multiple of 8.
__device__ __forceinline__ int2 xcd_item(int q, int n, int gy, int on) {
  if (!on) {
    const int gx = n / gy, y = q / gx;
    return make_int2(q - y * gx, y);
  }
  const int k = q & 7, i = q >> 3, qq = n >> 3, r = n & 7;
  const int item = k * qq + (k < r ? k : r) + i;
  const int px = item / gy;
  return make_int2(px, item - px * gy);
}

__device__ __forceinline__ int2 xcd_block(int on) {
  if (!on) return make_int2(blockIdx.x, blockIdx.y);
  const int gx = gridDim.x, gy = gridDim.y, n = gx * gy;
  const int L = blockIdx.y * gx + blockIdx.x;
  const int k = L & 7, i = L >> 3, q = n >> 3, r = n & 7;
  const int item = k * q + (k < r ? k : r) + i;
  const int px = item / gy;
  return make_int2(px, item - px * gy);
}

__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// Activation storage traits.  A lane's operand fragment is always 16 bytes.
struct BF16 {
  using T = unsigned short;
  static constexpr int EPL = 8;  // k elements per lane per K-step (16x16x32: 4 groups x 8)
  static constexpr bool kExact = false;
  static constexpr bool kScaled = false;
  static constexpr bool kSplit = false;
};
// fp16 twin of BF16 (predict(half=True): the reference's model.half(), nn/autobackend.py:215):
// IEEE binary16 weights and activations on v_mfma_f32_16x16x32_f16 (the bf16 rate on gfx950),
// fp32 accumulation, the same layouts, tables and kernels.
struct F16 {
  using T = _Float16;
  static constexpr int EPL = 8;
  static constexpr bool kExact = false;
  static constexpr bool kScaled = false;
  static constexpr bool kSplit = false;
};
struct F32 {
  using T = float;
  static constexpr int EPL = 4;  // 16x16x4 issued 4x: 4 groups x 4
  static constexpr bool kExact = true;
  static constexpr bool kScaled = false;
  static constexpr bool kSplit = false;
};
// fp32 activations (the F32 build's storage, K step and tables unchanged) multiplied on the BF16
// matrix cores: every fp32 operand is split into three bf16 parts, x = x0 + x1 + x2 exactly
// (round-to-nearest-even each time: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|, and the last remainder
// has <= 8 significant bits), and the six products whose magnitude reaches 2^-16 of w.x --
// w0x0 + w0x1 + w1x0 + w1x1 + w0x2 + w2x0 -- are summed by three v_mfma_f32_16x16x32_bf16 (each
// bf16 x bf16 product is exact in f32).  What is left out (w1x2, w2x1, w2x2) is <= 2^-24 |w.x|,
// the size of one f32 rounding, so the result is fp32-grade; three 16-cycle bf16 MFMAs replace
// four 32-cycle f32 ones per K step (2.7x the matrix rate).  Weights are split once at model
// create (yk_model::wsplit), activations as they are loaded (split3).  Operand layout: an MFMA
// operand is 4 VGPRs = one dword per element e of the lane's 4, and every dword pairs two parts
// of ONE element: weights W01 = [w0(e) | w1(e)], W02 = [w0(e) | w2(e)] (32-byte fragments);
// activations X00 = [x0 | x0], X11 = [x1 | x1], X20 = [x2 | x0] (each dword one v_cvt_pk_bf16_f32
// of the element with itself or its remainder).  W01 x X00 = w0x0 + w1x0, W01 x X11 = w0x1 +
// w1x1, W02 x X20 = w0x2 + w2x0: every operand is built in place by the instruction that produces
// it, so no register copies are needed, and the three MFMA passes run over all NE x NPT
// accumulators in turn (independent accumulators back to back).
struct F32S {
  using T = float;
  static constexpr int EPL = 4;
  static constexpr bool kExact = true;
  static constexpr bool kScaled = false;
  static constexpr bool kSplit = true;
};
// OCP e4m3 (gfx950 fp8; not MI300's fnuz) activations and weights.  A 16-byte fragment holds 16
// K elements: one K step is 64 = two 16x16x32 fp8 MFMAs (bytes 0-7 and 8-15 of every lane; A and
// B use the same byte -> K slot map, so the dot product does not depend on the hardware's K
// order).  Weights carry a per-output-channel scale (bias array: [bias][dequant scale]);
// activations are unscaled e4m3, saturated to +-448 when stored.
struct FP8 {
  using T = unsigned char;
  static constexpr int EPL = 16;
  static constexpr bool kExact = false;
  static constexpr bool kScaled = true;
  static constexpr bool kSplit = false;
};

// Weight fragment of one lane and K step (A operand) and the prepared activation fragment (B
// operand): 16 bytes as loaded for every trait but F32S, whose weight fragment is the three bf16
// parts of the lane's 4 f32 weights (24 bytes: w0 | w1 in .a, w2 in .b) and whose activation
// fragment is the three bf16 parts of its 4 f32 activations (split3).
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
// F32S weight fragment (W01, W02) and activation fragment (X00, X11, X20), see F32S
struct WS2 {
  u32x4v w01, w02;
};
struct XS3 {
  u32x4v x00, x11, x20;
};
template <class Tr> struct Frag { using W = uint4; using X = uint4; static constexpr int WB = 16; };
template <> struct Frag<F32S> { using W = WS2; using X = XS3; static constexpr int WB = 32; };

template <class Tr>
__device__ __forceinline__ f32x4 mma(const uint4& w, const uint4& x, f32x4 acc);
template <>
__device__ __forceinline__ f32x4 mma<BF16>(const uint4& w, const uint4& x, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w), __builtin_bit_cast(bf16x8, x),
                                                 acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma<F16>(const uint4& w, const uint4& x, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, w), __builtin_bit_cast(f16x8, x), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma<FP8>(const uint4& w, const uint4& x, f32x4 acc) {
  const long w0 = (long)(((unsigned long long)w.y << 32) | w.x), w1 = (long)(((unsigned long long)w.w << 32) | w.z);
  const long x0 = (long)(((unsigned long long)x.y << 32) | x.x), x1 = (long)(((unsigned long long)x.w << 32) | x.z);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w0, x0, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w1, x1, acc, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf16(const u32x4v& a, const u32x4v& b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
// one split K step: per pixel fragment t (split just before its MFMAs, so one fragment's parts
// are live at a time), pass p over the NE accumulators of t, then pass p + 1
template <int NE, int NPT>
__device__ __forceinline__ void mma_split_step(const WS2* w, const uint4* xf, f32x4 (*acc)[NPT]);
template <>
__device__ __forceinline__ f32x4 mma<F32>(const uint4& w, const uint4& x, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.x), __uint_as_float(x.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.y), __uint_as_float(x.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.z), __uint_as_float(x.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.w), __uint_as_float(x.w), acc, 0, 0, 0);
  return acc;
}

// Two consecutive K steps (fragments w0/x0 of step k, w1/x1 of step k + 1) into one accumulator.
// FP8: ONE block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, K = 128 = the 32 bytes
// of the two steps' fragments of every lane) at unit E8M0 block scales (127 = 2^0), which runs
// at twice the BF16 rate per clock where the non-scaled 16x16x32 fp8 form runs at the BF16 rate
// (MI355X_MICROARCH.md, "Matrix cores").  A and B assemble their 32 bytes the same way, so the
// byte -> K-slot pairing is consistent whatever order the hardware reads K in; the per-output-
// channel dequantisation stays in the epilogue.  Other types: the two steps in order.
typedef int i32x8 __attribute__((ext_vector_type(8)));
template <class Tr>
__device__ __forceinline__ f32x4 mma2(const uint4& w0, const uint4& w1, const uint4& x0, const uint4& x1, f32x4 acc) {
  if constexpr (Tr::kScaled) {
    const i32x8 a = {(int)w0.x, (int)w0.y, (int)w0.z, (int)w0.w, (int)w1.x, (int)w1.y, (int)w1.z, (int)w1.w};
    const i32x8 b = {(int)x0.x, (int)x0.y, (int)x0.z, (int)x0.w, (int)x1.x, (int)x1.y, (int)x1.z, (int)x1.w};
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  } else {
    acc = mma<Tr>(w0, x0, acc);
    return mma<Tr>(w1, x1, acc);
  }
}

// SiLU in the conv epilogues.  The fp32 build (kExact: F32 / F32S) evaluates the reference's
// expression x / (1 + exp(-x)) with libm expf and an IEEE division (~36 VALU per value); the
// bf16 / fp8 builds use v * rcp(1 + exp(-v)) on v_exp_f32 / v_rcp_f32 (~5 VALU, a few ulp).  The
// fast form was the fp32 default for part of round 3 (+4 % on the fp32 headline,
// profiles/r03_silu_ab.txt) and reordered two equal-score detections in frame 0 of the drop-in
// driver loop (tests/test_pipeline_gpu.py), so the fp32 build keeps the exact form (YK_DIAG bit
// 64 switches fp32 to the fast form for A/B runs).
// (A reciprocal-and-correction quotient for v / (1 + expf(-v)) was checked on every float v with
// tools/micro/silu_exact.hip: it differs from the IEEE division only at v = -0 (+0 instead of -0)
// and measured no faster on the fp32 headline (5,341 vs 5,390 frames/s), so it was not kept.)
template <bool kExact>
__device__ __forceinline__ float silu(float v) {
#if YK_EXACT_SILU
  if constexpr (kExact) return v / (1.0f + expf(-v));
#endif
  return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
}

// store / load 4 consecutive channels
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
// f32 -> bf16 round-to-nearest-even with the hardware v_cvt_pk_bf16_f32 (NaN stays NaN)
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  const bf16x2 h = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, h);
}
// x = x0 + x1 + x2 exactly per element, each part bf16 (RNE); the F32S activation operands
// X00 = [x0 | x0], X11 = [x1 | x1], X20 = [x2 | x0] (one dword per element)
__device__ __forceinline__ XS3 split3(const uint4& x) {
  const unsigned u[4] = {x.x, x.y, x.z, x.w};
  XS3 o;
  if constexpr ((YK_SPLIT_DIAG & 1) != 0) {
    o.x00 = u32x4v{u[0], u[1], u[2], u[3]};
    o.x11 = u32x4v{u[1], u[2], u[3], u[0]};
    o.x20 = u32x4v{u[2], u[3], u[0], u[1]};
    return o;
  }
  if constexpr (!YK_SPLIT_PK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = __uint_as_float(u[e]);
      const unsigned d00 = pack_bf16x2(a, a);
      const float r1 = a - __uint_as_float(d00 & 0xffff0000u);
      const unsigned d11 = pack_bf16x2(r1, r1);
      const float r2 = r1 - __uint_as_float(d11 & 0xffff0000u);
      o.x00[e] = d00;
      o.x11[e] = d11;
      o.x20[e] = pack_bf16x2(r2, a);
    }
    return o;
  }
  // element pairs: the two remainders of a pair are one v_pk_add_f32 each (6 VALU per element)
#pragma unroll
  for (int e = 0; e < 4; e += 2) {
    const f32x2v a = {__uint_as_float(u[e]), __uint_as_float(u[e + 1])};
    const unsigned d00a = pack_bf16x2(a[0], a[0]), d00b = pack_bf16x2(a[1], a[1]);
    const f32x2v h0 = {__uint_as_float(d00a & 0xffff0000u), __uint_as_float(d00b & 0xffff0000u)};
    const f32x2v r1 = a - h0;
    const unsigned d11a = pack_bf16x2(r1[0], r1[0]), d11b = pack_bf16x2(r1[1], r1[1]);
    const f32x2v h1 = {__uint_as_float(d11a & 0xffff0000u), __uint_as_float(d11b & 0xffff0000u)};
    const f32x2v r2 = r1 - h1;
    o.x00[e] = d00a;
    o.x00[e + 1] = d00b;
    o.x11[e] = d11a;
    o.x11[e + 1] = d11b;
    o.x20[e] = pack_bf16x2(r2[0], a[0]);
    o.x20[e + 1] = pack_bf16x2(r2[1], a[1]);
  }
  return o;
}
template <int NE, int NPT>
__device__ __forceinline__ void mma_split_step(const WS2* w, const uint4* xf, f32x4 (*acc)[NPT]) {
  if constexpr ((YK_DIAG & 512) != 0) {  // diagnostic: operands as if stored pre-split (no split VALU)
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const u32x4v xa = u32x4v{xf[t].x, xf[t].y, xf[t].z, xf[t].w};
      const u32x4v xb = u32x4v{xf[t].z, xf[t].w, xf[t].x, xf[t].y};
#pragma unroll
      for (int i = 0; i < NE; ++i) acc[i][t] = mfma_bf16(w[i].w01, xb, acc[i][t]);
#pragma unroll
      for (int i = 0; i < NE; ++i)
        acc[i][t] = mfma_bf16(u32x4v{w[i].w01.z, w[i].w01.w, w[i].w02.x, w[i].w02.y}, xa, acc[i][t]);
#pragma unroll
      for (int i = 0; i < NE; ++i) acc[i][t] = mfma_bf16(w[i].w02, xa, acc[i][t]);
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const XS3 x = split3(xf[t]);
#pragma unroll
    for (int i = 0; i < NE; ++i) acc[i][t] = mfma_bf16(w[i].w01, x.x00, acc[i][t]);
#pragma unroll
    for (int i = 0; i < NE; ++i) acc[i][t] = mfma_bf16(w[i].w01, x.x11, acc[i][t]);
#pragma unroll
    for (int i = 0; i < NE; ++i) acc[i][t] = mfma_bf16(w[i].w02, x.x20, acc[i][t]);
  }
}


__device__ __forceinline__ void store4(unsigned short* p, const float v[4]) {
  YK_SC(p, 8, 1);
  uint2 o;
  o.x = pack_bf16x2(v[0], v[1]);
  o.y = pack_bf16x2(v[2], v[3]);
  *(uint2*)p = o;
}
__device__ __forceinline__ void store4(float* p, const float v[4]) {
  YK_SC(p, 16, 2);
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
}
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
// f32 -> f16 round-to-nearest-even (v_cvt_f16_f32), overflow to +-inf like torch's .half()
__device__ __forceinline__ void store4(_Float16* p, const float v[4]) {
  YK_SC(p, 8, 3);
  *(f16x4*)p = f16x4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
}
__device__ __forceinline__ void load4(const _Float16* p, float v[4]) {
  const f16x4 h = *(const f16x4*)p;
  v[0] = (float)h[0];
  v[1] = (float)h[1];
  v[2] = (float)h[2];
  v[3] = (float)h[3];
}
// f32 -> e4m3 with round-to-nearest-even (v_cvt_pk_fp8_f32), saturated to the finite range
__device__ __forceinline__ float sat448(float v) { return __builtin_amdgcn_fmed3f(v, -448.f, 448.f); }
__device__ __forceinline__ void store4(unsigned char* p, const float v[4]) {
  YK_SC(p, 4, 4);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat448(v[0]), sat448(v[1]), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat448(v[2]), sat448(v[3]), w, true);
  *(int*)p = w;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void load4(const unsigned char* p, float v[4]) {
  const int i = *(const int*)p;
  const f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8(i, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8(i, true);
  v[0] = lo[0];
  v[1] = lo[1];
  v[2] = hi[0];
  v[3] = hi[1];
}
// per-output-channel dequant scale of 4 consecutive channels (FP8: stored after the bias)
template <class Tr>
__device__ __forceinline__ float4 dq4(const float* bias, int n_tiles, int n0) {
  if constexpr (Tr::kScaled) return *(const float4*)(bias + n_tiles * 16 + n0);
  else return make_float4(1.f, 1.f, 1.f, 1.f);
}
__device__ __forceinline__ void load4(const unsigned short* p, float v[4]) {
  const uint2 i = *(const uint2*)p;
  v[0] = bf2f(i.x & 0xffff);
  v[1] = bf2f(i.x >> 16);
  v[2] = bf2f(i.y & 0xffff);
  v[3] = bf2f(i.y >> 16);
}
__device__ __forceinline__ void load4(const float* p, float v[4]) {
  const float4 i = *(const float4*)p;
  v[0] = i.x;
  v[1] = i.y;
  v[2] = i.z;
  v[3] = i.w;
}

struct View {
  const void* p;
  int cstride, coff, h, w, up;
};

// Indexing the kernel-argument array with a per-lane value (a.src[si]) -- or selecting between
// two of its members, which LLVM folds into a selected kernarg address -- makes the compiler
// fetch the View with vector loads and drain vmcnt before the gather, serialising every
// prefetch in flight.  uniform_view() pins each integer field in an SGPR once (readfirstlane
// breaks the link to the kernarg address) and pick_view() selects member-wise per lane.  The
// data pointer stays derived from the kernel's first source pointer (base + a uniform element
// delta), so address-space inference keeps the gathers global loads: flat loads would force
// vmcnt(0) + lgkmcnt(0) waits.
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long rfl64(long long v) {
  const unsigned lo = (unsigned)rfl((int)(unsigned long long)v);
  const unsigned hi = (unsigned)rfl((int)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ View uniform_view(const View& v) {
  View r;
  r.p = v.p;
  r.cstride = rfl(v.cstride);
  r.coff = rfl(v.coff);
  r.h = rfl(v.h);
  r.w = rfl(v.w);
  r.up = rfl(v.up);
  return r;
}
__device__ __forceinline__ View pick_view(const View& v0, const View& v1, bool second) {
  View r;
  r.p = nullptr;  // data pointer: gbase + (second ? gdelta : 0), see above
  r.cstride = second ? v1.cstride : v0.cstride;
  r.coff = second ? v1.coff : v0.coff;
  r.h = second ? v1.h : v0.h;
  r.w = second ? v1.w : v0.w;
  r.up = second ? v1.up : v0.up;
  return r;
}

// ---------------------------------------------------------------- implicit-GEMM conv
constexpr int kTsCap = 65536;  // YK_FAST_TS diagnostics: workgroups with timestamps

// Table entry of K chunk q computed arithmetically (model.py Program.pack: tap, ch =
// divmod(8q, cin); src = ch >= c0): no table load, so no memory round trip in the K loop.
__device__ __forceinline__ int chunk_entry(int q, int n_chunks, int cin, int c0, int k) {
  if (q >= n_chunks) return -1;
  const int cq = cin >> 3;
  const int tap = q / cq, c = (q - tap * cq) << 3;
  const int ky = tap / k, kx = tap - ky * k, pad = k >> 1;
  const int src = c >= c0 ? 1 : 0;
  const int ch = src ? c - c0 : c;
  return ((kx - pad + 8) << 21) | ((ky - pad + 8) << 17) | (src << 16) | ch;
}

struct ConvArgs {
  View src[2];
  int ksize, stride, pad;
  int in_h, in_w, out_h, out_w, M;
  const uint4* wpk;  // [n_tiles][k_steps][64]
  const float* bias; // [n_tiles * 16]
  const int* tab;    // per 8-channel K chunk: -1 or (dx+8)<<21 | (dy+8)<<17 | src<<16 | channel
  int k_steps, n_tiles, n_chunks;
  int c0, cin;       // K-space channels of src[0]; of both (the table is q -> (tap, channel) =
                     // divmod(8q, cin), so the K-loop kernels derive it arithmetically)
  void* dst;
  int d_cstride, d_coff, cout;
  const void* res;
  int r_cstride, r_coff;
  int act;
};

template <class Tr, int NNT, int NPT>
__global__ void __launch_bounds__(256) conv_igemm_kernel(ConvArgs a) {
  using T = typename Tr::T;
  constexpr int EPL = Tr::EPL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const int nt0 = blockIdx.y * NNT;
  const int pbase = (blockIdx.x * 4 + wave) * (16 * NPT);
  const View sv0 = uniform_view(a.src[0]), sv1 = uniform_view(a.src[1]);
  const typename Tr::T* gbase = (const typename Tr::T*)a.src[0].p;
  const long long gdelta = rfl64((const typename Tr::T*)a.src[1].p - gbase);
  if (pbase >= a.M) return;
  const int hw = a.out_h * a.out_w;
  int pb[NPT], py[NPT], px[NPT];
  bool pv[NPT];
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int p = pbase + t * 16 + col;
    pv[t] = p < a.M;
    const int pp = pv[t] ? p : 0;
    pb[t] = pp / hw;
    const int r = pp - pb[t] * hw;
    const int oy = r / a.out_w;
    const int ox = r - oy * a.out_w;
    py[t] = oy * a.stride;  // the K-chunk table carries the tap offset (ky - pad, kx - pad)
    px[t] = ox * a.stride;
  }
  f32x4 acc[NNT][NPT];
#pragma unroll
  for (int i = 0; i < NNT; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_step = [&](int ks, uint4* wf, uint4* xf) {
#pragma unroll
    for (int i = 0; i < NNT; ++i) {
      const int nt = nt0 + i < a.n_tiles ? nt0 + i : a.n_tiles - 1;
      wf[i] = a.wpk[((size_t)nt * a.k_steps + ks) * 64 + lane];
    }
    const int kel = ks * 4 * EPL + kg * EPL;
    const int q = kel >> 3, sub = kel & 7;
    const int e = chunk_entry(q, a.n_chunks, a.cin, a.c0, a.ksize);
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (e >= 0 && pv[t]) {
        const int dx = ((e >> 21) & 15) - 8, dy = ((e >> 17) & 15) - 8;
        const int si = (e >> 16) & 1, ch = e & 0xffff;
        const int iy = py[t] + dy, ix = px[t] + dx;
        if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
          const View s = pick_view(sv0, sv1, si != 0);
          const size_t off = (((size_t)pb[t] * s.h + (iy >> s.up)) * s.w + (ix >> s.up)) * s.cstride + s.coff + ch + sub;
          v = *(const uint4*)(gbase + (si ? gdelta : 0ll) + off);
        }
      }
      xf[t] = v;
    }
  };

  uint4 wf[NNT], xf[NPT], wn[NNT], xn[NPT];
  load_step(0, wf, xf);
  for (int ks = 0; ks < a.k_steps; ++ks) {
    if (ks + 1 < a.k_steps) load_step(ks + 1, wn, xn);
#pragma unroll
    for (int i = 0; i < NNT; ++i)
#pragma unroll
      for (int t = 0; t < NPT; ++t) acc[i][t] = mma<Tr>(wf[i], xf[t], acc[i][t]);
#pragma unroll
    for (int i = 0; i < NNT; ++i) wf[i] = wn[i];
#pragma unroll
    for (int t = 0; t < NPT; ++t) xf[t] = xn[t];
  }

  // epilogue: lane holds channels n0..n0+3 of pixel (pbase + t*16 + col)
#pragma unroll
  for (int i = 0; i < NNT; ++i) {
    const int nt = nt0 + i;
    if (nt >= a.n_tiles) break;
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
    const float4 bb = *(const float4*)(a.bias + n0);
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      if (!pv[t]) continue;
      const size_t p = (size_t)pbase + t * 16 + col;
      float v[4] = {acc[i][t][0] + bb.x, acc[i][t][1] + bb.y, acc[i][t][2] + bb.z, acc[i][t][3] + bb.w};
      if (a.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu<Tr::kExact>(v[j]);
      }
      if (a.res) {
        float r[4];
        load4((const T*)a.res + p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = r[j] + v[j];
      }
      store4((T*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// ---------------------------------------------------------------- split-K direct conv (low resolution)
// For the P4/P5 layers (<= 1,280 pixels per image) whole-tile workgroups are too few and their
// K loops too long: the kernel is a chain of dependent global round trips.  Here a workgroup
// owns only 16*NPT flattened output pixels x NNT*16 channels and its four waves split the K
// steps into contiguous quarters; each wave streams its weight fragments (coalesced 1 KB per
// step and n-tile, L2-resident) and gathers its input fragments straight from global memory
// with SKD steps in flight, and the four partial tiles meet in LDS before the epilogue.
constexpr int SKD = 4;  // K steps in flight per wave

template <class Tr, int NNT, int NPT>
__global__ void __launch_bounds__(256) conv_splitk_kernel(ConvArgs a) {
  using T = typename Tr::T;
  constexpr int EPL = Tr::EPL;
  __shared__ f32x4 red[4 * NNT * NPT * 64];
  const View sv0 = uniform_view(a.src[0]), sv1 = uniform_view(a.src[1]);
  const typename Tr::T* gbase = (const typename Tr::T*)a.src[0].p;
  const long long gdelta = rfl64((const typename Tr::T*)a.src[1].p - gbase);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const int nt0 = blockIdx.y * NNT;
  const int pbase = blockIdx.x * (16 * NPT);
  const int hw = a.out_h * a.out_w;
  int pb[NPT], py[NPT], px[NPT];
  bool pv[NPT];
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int p = pbase + t * 16 + col;
    pv[t] = p < a.M;
    const int pp = pv[t] ? p : 0;
    pb[t] = pp / hw;
    const int r = pp - pb[t] * hw;
    const int oy = r / a.out_w;
    const int ox = r - oy * a.out_w;
    py[t] = oy * a.stride;
    px[t] = ox * a.stride;
  }
  f32x4 acc[NNT][NPT];
#pragma unroll
  for (int i = 0; i < NNT; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_step = [&](int ks, uint4* wf, uint4* xf) {
#pragma unroll
    for (int i = 0; i < NNT; ++i) {
      const int nt = nt0 + i < a.n_tiles ? nt0 + i : a.n_tiles - 1;
      wf[i] = a.wpk[((size_t)nt * a.k_steps + ks) * 64 + lane];
    }
    const int kel = ks * 4 * EPL + kg * EPL;
    const int q = kel >> 3, sub = kel & 7;
    const int e = chunk_entry(q, a.n_chunks, a.cin, a.c0, a.ksize);
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (e >= 0 && pv[t]) {
        const int dx = ((e >> 21) & 15) - 8, dy = ((e >> 17) & 15) - 8;
        const int si = (e >> 16) & 1, ch = e & 0xffff;
        const int iy = py[t] + dy, ix = px[t] + dx;
        if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
          const View s = pick_view(sv0, sv1, si != 0);
          const size_t off = (((size_t)pb[t] * s.h + (iy >> s.up)) * s.w + (ix >> s.up)) * s.cstride + s.coff + ch + sub;
          v = *(const uint4*)(gbase + (si ? gdelta : 0ll) + off);
        }
      }
      xf[t] = v;
    }
  };

  float4 bb[NNT];  // epilogue bias, loaded up front (off the critical path)
#pragma unroll
  for (int i = 0; i < NNT; ++i) {
    const int n0 = (nt0 + i) * 16 + kg * 4;
    bb[i] = (nt0 + i < a.n_tiles && n0 < a.cout) ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int kq = (a.k_steps + 3) >> 2;
  const int k0 = wave * kq, k1 = k0 + kq < a.k_steps ? k0 + kq : a.k_steps;
  uint4 wb[SKD][NNT], xb[SKD][NPT];
#pragma unroll
  for (int d = 0; d < SKD; ++d)
    if (k0 + d < k1) load_step(k0 + d, wb[d], xb[d]);
  for (int ks = k0; ks < k1; ks += SKD) {
#pragma unroll
    for (int d = 0; d < SKD; ++d) {
      if (ks + d < k1) {
#pragma unroll
        for (int i = 0; i < NNT; ++i)
#pragma unroll
          for (int t = 0; t < NPT; ++t) acc[i][t] = mma<Tr>(wb[d][i], xb[d][t], acc[i][t]);
        if (ks + d + SKD < k1) load_step(ks + d + SKD, wb[d], xb[d]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NNT; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) red[((wave * NNT + i) * NPT + t) * 64 + lane] = acc[i][t];
  __syncthreads();
  // epilogue: wave w finishes the (i, t) fragments with (i * NPT + t) % 4 == w
#pragma unroll
  for (int i = 0; i < NNT; ++i) {
    const int nt = nt0 + i;
    if (nt >= a.n_tiles) break;
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      if (((i * NPT + t) & 3) != wave || !pv[t]) continue;
      f32x4 v4 = red[((0 * NNT + i) * NPT + t) * 64 + lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const f32x4 u = red[((w * NNT + i) * NPT + t) * 64 + lane];
        v4[0] += u[0];
        v4[1] += u[1];
        v4[2] += u[2];
        v4[3] += u[3];
      }
      const size_t p = (size_t)pbase + t * 16 + col;
      float v[4] = {v4[0] + bb[i].x, v4[1] + bb[i].y, v4[2] + bb[i].z, v4[3] + bb[i].w};
      if (a.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu<Tr::kExact>(v[j]);
      }
      if (a.res) {
        float r[4];
        load4((const T*)a.res + p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = r[j] + v[j];
      }
      store4((T*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// ---------------------------------------------------------------- LDS-tiled implicit-GEMM conv
// One workgroup = a 16-column x TH-row output tile of one image for NNT x 16 output channels.
// The input tile with its halo (all K-space channels of both sources, upsample applied) is
// staged once into LDS with an odd number of 16-byte slots per pixel (conflict-free
// ds_read_b128 for 16 consecutive pixels); weights stream through LDS in chunks of KCH K-steps
// shared by the four waves.  Wave w computes output rows [w*NPT, (w+1)*NPT) of the tile.
struct TileArgs {
  View src[2];
  int c0, cin;               // K-space channels of src[0]; total (multiple of 8)
  int ksize, stride, pad;
  int in_h, in_w, out_h, out_w;
  int tiles_x, tiles_y, tih, tiw, ps;  // tile grid per image; input tile dims; LDS pixel stride (elements)
  const uint4* wpk;
  const float* bias;
  const int* tab;
  int k_steps, n_tiles, n_chunks;
  void* dst;
  int d_cstride, d_coff, cout;
  const void* res;
  int r_cstride, r_coff;
  int act;
  int single;  // whole weight slab LDS-resident
  int xcd;     // XCD-aware workgroup placement (xcd_block)
};

template <class Tr, int NNT, int NPT, bool KSPLIT>
__global__ void __launch_bounds__(256) conv_tile_kernel(TileArgs a) {
  // KSPLIT: the four waves share one 16 x NPT output tile and split every weight chunk's K
  // steps between them (wave w takes steps w, w+4, ...); partial sums meet in LDS.  Used for
  // the low-resolution layers, where whole-tile workgroups are too few and their K loops long.
  // a.single: the whole weight slab (NNT x k_steps) is LDS-resident -- one prologue, one
  // barrier, then a K loop with no global traffic.  Otherwise weights stream in double-buffered
  // chunks of KCH steps.  The prologue issues every global load (input tile, weights, bias)
  // before the first LDS store, so a workgroup pays one memory round trip
  // instead of one per staging-loop iteration.  K-chunk table entries are computed
  // arithmetically (chunk_entry).
  using T = typename Tr::T;
  constexpr int EPL = Tr::EPL;
  constexpr int KCH = KSPLIT ? 8 : 4;
  constexpr int ROWS = KSPLIT ? NPT : 4 * NPT;  // output rows per tile
  constexpr int EU = 16 / (int)sizeof(T);   // elements per 16-byte unit
  constexpr int WU = NNT * KCH * 64;        // 16-byte weight units per chunk
  constexpr int WPT = (WU + 255) / 256;     // per thread
  constexpr int SU = 8;                     // staging loads in flight per thread
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* wl = (uint4*)smem;  // single: [NNT][k_steps][64]; else [2][NNT][KCH][64]
  const int wslab = a.single ? NNT * a.k_steps * 64 : 2 * WU;
  T* xt = (T*)(smem + (size_t)wslab * 16);  // [tih][tiw][ps]
  // K-step table [k_steps][4]: LDS element offset of each lane group's K chunk from the
  // pixel's window origin in the tile (K padding: 0, zero weights), built by the host (build_ktabs)
  int* ltab = (int*)(smem + (size_t)wslab * 16 + (((size_t)a.tih * a.tiw * a.ps * sizeof(T) + 15) & ~(size_t)15));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < a.k_steps * 4; i += 256) ltab[i] = a.tab[i];
  const int kg = lane >> 4, col = lane & 15;
  const View sv0 = uniform_view(a.src[0]), sv1 = uniform_view(a.src[1]);
  const typename Tr::T* gbase = (const typename Tr::T*)a.src[0].p;
  const long long gdelta = rfl64((const typename Tr::T*)a.src[1].p - gbase);
  const int tpi = a.tiles_x * a.tiles_y;
  const int2 blk = xcd_block(a.xcd);
  int t = blk.x;
  const int b = t / tpi;
  t -= b * tpi;
  const int ty0 = (t / a.tiles_x) * ROWS, tx0 = (t % a.tiles_x) * 16;
  const int iy0 = ty0 * a.stride - a.pad, ix0 = tx0 * a.stride - a.pad;
  const int nt0 = blk.y * NNT;
  const int wrow = KSPLIT ? 0 : wave * NPT;  // first tile row of this wave
  uint4 wreg[WPT];
  auto fetch = [&](int k0) {  // global -> registers (stays in flight over the compute)
#pragma unroll
    for (int r = 0; r < WPT; ++r) {
      const int i = tid + r * 256;
      if (i < WU) {
        const int j = i >> 6, l = i & 63;
        const int ni = j / KCH, kk = j - ni * KCH;
        const int nt = nt0 + ni < a.n_tiles ? nt0 + ni : a.n_tiles - 1;
        const int ks = k0 + kk;
        wreg[r] = ks < a.k_steps ? a.wpk[((size_t)nt * a.k_steps + ks) * 64 + l] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int r = 0; r < WPT; ++r) {
      const int i = tid + r * 256;
      if (i < WU) wl[buf * WU + i] = wreg[r];
    }
  };
  if (!a.single) fetch(0);
  // bias of this workgroup's channels (epilogue), loaded with the prologue
  float4 bb[NNT];
#pragma unroll
  for (int ni = 0; ni < NNT; ++ni) {
    const int n0 = (nt0 + ni) * 16 + kg * 4;
    bb[ni] = (nt0 + ni < a.n_tiles && n0 < a.cout) ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // ---- stage the input tile (zero outside the image = conv zero padding), SU loads in flight
  {
    const int U = a.cin / EU;
    const int total = a.tih * a.tiw * U;
    for (int base = tid; base < total; base += 256 * SU) {
      uint4 v[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = base + u * 256;
        v[u] = make_uint4(0u, 0u, 0u, 0u);
        if (i < total) {
          const int pix = i / U, uu = i - pix * U;
          const int ry = pix / a.tiw, rx = pix - ry * a.tiw;
          const int iy = iy0 + ry, ix = ix0 + rx;
          const int c = uu * EU;
          if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
            const int si = c < a.c0 ? 0 : 1;
            const View sv = pick_view(sv0, sv1, si != 0);
            const int cc = si ? c - a.c0 : c;
            v[u] = *(const uint4*)(gbase + (si ? gdelta : 0ll) +
                                   (((size_t)b * sv.h + (iy >> sv.up)) * sv.w + (ix >> sv.up)) * sv.cstride + sv.coff +
                                   cc);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = base + u * 256;
        if (i < total) {
          const int pix = i / U, uu = i - pix * U;
          *(uint4*)(xt + (size_t)pix * a.ps + uu * EU) = v[u];
        }
      }
    }
  }
  // ---- whole weight slab (single mode), SU loads in flight
  if (a.single) {
    const int ks = a.k_steps, total = NNT * ks * 64;
    for (int base = tid; base < total; base += 256 * SU) {
      uint4 v[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = base + u * 256;
        v[u] = make_uint4(0u, 0u, 0u, 0u);
        if (i < total) {
          const int ni = i / (ks * 64), r = i - ni * ks * 64;
          const int nt = nt0 + ni < a.n_tiles ? nt0 + ni : a.n_tiles - 1;
          v[u] = a.wpk[(size_t)nt * ks * 64 + r];
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = base + u * 256;
        if (i < total) wl[i] = v[u];
      }
    }
  } else {
    commit(0);
  }
  __syncthreads();
  f32x4 acc[NNT][NPT];
#pragma unroll
  for (int i = 0; i < NNT; ++i)
#pragma unroll
    for (int q = 0; q < NPT; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int s = a.stride;
  int prow[NPT];  // LDS element offset of each pixel fragment's window origin
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) prow[pt] = ((wrow + pt) * s * a.tiw + col * s) * a.ps;
  int buf = 0;
  const int kch = a.single ? a.k_steps : KCH;  // steps per chunk (= the slab row stride)
  for (int k0 = 0; k0 < a.k_steps; k0 += kch) {
    const bool more = k0 + kch < a.k_steps;
    if (more) fetch(k0 + KCH);
    const uint4* wc = wl + buf * WU;
    const int kn = a.k_steps - k0 < kch ? a.k_steps - k0 : kch;
    for (int kk = KSPLIT ? wave : 0; kk < kn; kk += KSPLIT ? 4 : 1) {
      const int e = ltab[(k0 + kk) * 4 + kg];  // K padding chunks: zero weights, finite data
      uint4 xf[NPT];
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) xf[pt] = *(const uint4*)(xt + prow[pt] + e);
#pragma unroll
      for (int ni = 0; ni < NNT; ++ni) {
        const uint4 w = wc[(ni * kch + kk) * 64 + lane];
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) acc[ni][pt] = mma<Tr>(w, xf[pt], acc[ni][pt]);
      }
    }
    if (more) commit(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // ---- split-K: sum the four waves' partial tiles through LDS (the weight buffers are free now)
  if constexpr (KSPLIT) {
    f32x4* red = (f32x4*)smem;  // [4 waves][NNT][NPT][64]
#pragma unroll
    for (int ni = 0; ni < NNT; ++ni)
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) red[((wave * NNT + ni) * NPT + pt) * 64 + lane] = acc[ni][pt];
    __syncthreads();
#pragma unroll
    for (int ni = 0; ni < NNT; ++ni)
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) {
        f32x4 v = red[((0 * NNT + ni) * NPT + pt) * 64 + lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
          const f32x4 u = red[((w * NNT + ni) * NPT + pt) * 64 + lane];
          v[0] += u[0];
          v[1] += u[1];
          v[2] += u[2];
          v[3] += u[3];
        }
        acc[ni][pt] = v;
      }
  }
  // ---- epilogue: bias + SiLU + residual, 4 consecutive channels of one pixel per lane
  // (split-K: wave w stores the (ni, pt) pairs with (ni * NPT + pt) % 4 == w)
#pragma unroll
  for (int ni = 0; ni < NNT; ++ni) {
    const int nt = nt0 + ni;
    if (nt >= a.n_tiles) break;
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      if (KSPLIT && ((ni * NPT + pt) & 3) != wave) continue;
      const int oy = ty0 + wrow + pt, ox = tx0 + col;
      if (oy >= a.out_h || ox >= a.out_w) continue;
      const size_t p = ((size_t)b * a.out_h + oy) * a.out_w + ox;
      float v[4] = {acc[ni][pt][0] + bb[ni].x, acc[ni][pt][1] + bb[ni].y, acc[ni][pt][2] + bb[ni].z,
                    acc[ni][pt][3] + bb[ni].w};
      if (a.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu<Tr::kExact>(v[j]);
      }
      if (a.res) {
        float r[4];
        load4((const T*)a.res + p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = r[j] + v[j];
      }
      store4((T*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// ---------------------------------------------------------------- table-driven implicit-GEMM conv
// The gather kernels above derive every K chunk's (tap, source, channel) and every pixel's
// address inside the K loop: ~120 VALU per K step against 4-16 MFMAs (issue-bound, measured
// SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES ~ 0.5).  Here the host precomputes, per op, one entry
// per (K step, lane group kg): {element delta from the window origin, tap | src << 4 | valid
// << 5} (model create, yk_model::ktab); the workgroup copies the op's table into LDS once.
// Each lane computes its pixels' window-origin offsets in both sources and a 9-bit tap
// validity mask once, so a K step costs one ds_read_b64, a mask test and an add per pixel
// fragment.  KW (waves per K split) 4: the four waves share one 16*NPT-pixel tile and split the
// K steps (partial tiles summed in LDS); 2: two pairs of waves, each pair one 16*NPT-pixel tile
// and half the K steps (a short split-K wave pays its prologue and exposed load latency per
// 1/4 of K, a pair per 1/2, and a launch of half as many workgroups fits the CUs in fewer
// rounds); 1: each wave owns its own 16*NPT pixels and the full K.
// SKD K steps of loads stay in flight per wave.
struct FastArgs {
  const void* arena;             // every activation buffer lives in one allocation (< kArenaMax)
  unsigned arena_bytes;
  unsigned soff0, soff1;         // byte offsets of the two source views (image b0, channel coff)
  int h0, w0, cs0, up0, h1, w1, cs1, up1;
  int stride, pad, in_h, in_w, out_h, out_w, M;
  float inv_hw, inv_w;           // 1 / (out_h * out_w), 1 / out_w (fdiv)
  const void* wblob;             // packed weights: byte offset woff, [n_tiles][k_steps][64][16 B]
  unsigned wbytes, woff;
  const float* bias;
  const int2* ktab;              // [k_steps][4] {byte delta, tap | src << 4 | valid << 5}
  int k_steps, n_tiles;
  void* dst;
  int d_cstride, d_coff, cout;
  const void* res;
  int r_cstride, r_coff;
  int act;
  int xcd;
  unsigned long long* tstamp;  // diagnostics (YK_FAST_TS): per-workgroup [start, end] wall clock
  int tstamp_cap;              // workgroups the tstamp buffer holds (3 entries each)
  // persistent form (ipw > 1): a grid of ceil(n_items / ipw) workgroups, each looping over the
  // (pixel block, channel group) items q = blockIdx.x, + gridDim.x, ... (n_cg channel groups)
  int ipw, n_items, n_cg;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Activation-arena loads use 32-bit unsigned buffer offsets (SRD num_records = the arena's bytes):
// the table / wide / halo kernels serve arenas below kArenaMax (4 GiB less 64 KiB), e.g. the
// 2.7 GiB fp32 arena of a batch-32 forward; kOOB lies past every such arena, so a masked tap's
// load returns 0 (and kOOB + 16 does not wrap)
constexpr unsigned long long kArenaMax = 0xFFFF0000ull;
constexpr unsigned kOOB = 0xFFFFFF00u;  // buffer offset past every num_records: the load returns 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const void* base, unsigned bytes) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(size_t)base);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((size_t)base >> 32));
  void* b = (void*)(((size_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// weight fragment of step ks (Frag<Tr>::WB bytes per lane, 64 lanes per step)
template <class Tr>
__device__ __forceinline__ typename Frag<Tr>::W wload(__amdgpu_buffer_rsrc_t r, unsigned voff, int ks) {
  if constexpr (Tr::kSplit) {
    WS2 w;
    if constexpr ((YK_SPLIT_DIAG & 2) != 0) {
      const unsigned c = voff ^ (unsigned)ks;
      w.w01 = u32x4v{c, c + 1u, c + 2u, c + 3u};
      w.w02 = u32x4v{c + 4u, c, c + 5u, c};
      return w;
    }
    w.w01 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, ks * 64 * 32, 0);
    w.w02 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff + 16, ks * 64 * 32, 0);
    return w;
  } else {
    return bload(r, voff, ks * 1024);
  }
}

// floor(n / d) for 0 <= n < 2^22, d >= 1, with inv = 1/d rounded up to f32 by the host:
// the f32 product is within one of the quotient, fixed by one compare.
__device__ __forceinline__ int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  q -= (q * d > n) ? 1 : 0;
  q += ((q + 1) * d <= n) ? 1 : 0;
  return q;
}

// K steps of loads each conv_fast wave keeps in flight (2 for the large register tiles: register
// budget).  8 steps for the 1- and 2-fragment tiles measured no faster than 4 (round 2).
constexpr int fast_skd(int nnt, int npt) { return nnt * npt >= 8 ? ((YK_DIAG & 1024) ? 1 : 2) : 4; }
// conv_fastw's activation slots are indexed by the step within a 4-step weight chunk: SKD | 4
constexpr int fastw_skd(int nnt, int npt) { return nnt * npt >= 8 ? 2 : 4; }

// NE = output-channel tiles this workgroup computes: NNT, or fewer for the last channel group of
// an op whose n_tiles is not a multiple of NNT (its missing tiles cost no loads and no MFMAs;
// each body is straight-line code, the dispatch is one scalar branch per workgroup).
template <class Tr, int NE, int NPT, int KW, int SKD>
__device__ __forceinline__ void conv_fast_body(const FastArgs& a, int2 blk, int nt0) {
  using T = typename Tr::T;
  constexpr int ESZ = (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool WS = KW > 1;
  int2* tab = (int2*)smem;  // [k_steps * 4]; WS: then the f32x4 reduction buffer
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, col = lane & 15;
  const int nk = a.k_steps;
  const int wg_lin = blockIdx.y * gridDim.x + blockIdx.x;
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin] = wall_clock64();
  const __amdgpu_buffer_rsrc_t xr = make_srd(a.arena, a.arena_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_srd(a.wblob, a.wbytes);
  const int hw = a.out_h * a.out_w;
  unsigned vo0[NPT], vo1[NPT], vm[NPT];
  const int pbase = (blk.x * (4 / KW) + wave / KW) * (16 * NPT);  // this wave's pixel tile
  // the lane's window origins in both sources and its 9-bit tap mask, per pixel fragment
  {
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const int p = pbase + t * 16 + col;
      const bool pv = p < a.M;
      const int pp = pv ? p : 0;
      // exact small-integer division through f32 (operands < 2^22): q = floor(n / d)
      const int b = fdiv(pp, hw, a.inv_hw);
      const int r = pp - b * hw;
      const int oy = fdiv(r, a.out_w, a.inv_w);
      const int ox = r - oy * a.out_w;
      const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
      vo0[t] = a.soff0 + (unsigned)(((b * a.h0 + (iy0 >> a.up0)) * a.w0 + (ix0 >> a.up0)) * a.cs0 * ESZ);
      vo1[t] = a.soff1 + (unsigned)(((b * a.h1 + (iy0 >> a.up1)) * a.w1 + (ix0 >> a.up1)) * a.cs1 * ESZ);
      // 9-bit tap mask = valid rows x valid columns of the 3x3 window
      const unsigned cm = ((unsigned)(ix0 >= 0 && ix0 < a.in_w)) | ((unsigned)(ix0 + 1 >= 0 && ix0 + 1 < a.in_w) << 1) |
                          ((unsigned)(ix0 + 2 >= 0 && ix0 + 2 < a.in_w) << 2);
      const unsigned m = ((iy0 >= 0 && iy0 < a.in_h) ? cm : 0u) | ((iy0 + 1 >= 0 && iy0 + 1 < a.in_h) ? cm << 3 : 0u) |
                         ((iy0 + 2 >= 0 && iy0 + 2 < a.in_h) ? cm << 6 : 0u);
      vm[t] = pv ? m : 0u;  // 1x1 convs use tap 0 = the pixel itself
    }
  }
  f32x4 acc[NE][NPT];
#pragma unroll
  for (int i = 0; i < NE; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bb[NE];
  float4 sc[NE];  // FP8 dequant scales
  unsigned wo[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int n0 = (nt0 + i) * 16 + kg * 4;
    if constexpr (!WS) {  // (WS: the epilogue loads its slots' bias / scales)
      bb[i] = (nt0 + i < a.n_tiles && n0 < a.cout) ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (Tr::kScaled) sc[i] = dq4<Tr>(a.bias, a.n_tiles, n0 < a.cout ? n0 : 0);
    }
    const int nt = nt0 + i < a.n_tiles ? nt0 + i : a.n_tiles - 1;
    wo[i] = a.woff + (unsigned)(((size_t)nt * nk * 64 + lane) * Frag<Tr>::WB);
  }
  __syncthreads();
  using WF = typename Frag<Tr>::W;
  auto issue = [&](int ks, int2 e, WF* wf, uint4* xf) {
#pragma unroll
    for (int i = 0; i < NE; ++i) wf[i] = wload<Tr>(wr, wo[i], ks);
    const unsigned tap = (unsigned)e.y & 15u;
    const bool s1 = (e.y & 16) != 0, ev = (e.y & 32) != 0;
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const bool ok = ev && ((vm[t] >> tap) & 1u);
      const unsigned off = (s1 ? vo1[t] : vo0[t]) + (unsigned)e.x;
      xf[t] = bload(xr, ok ? off : kOOB, 0);
    }
  };
  auto load_step = [&](int ks, WF* wf, uint4* xf) { issue(ks, tab[ks * 4 + kg], wf, xf); };
  // one K step's MFMAs: the activation fragments are prepared once (F32S: split into bf16 parts)
  // and used by every output-channel tile
  auto step_mma = [&](const WF* wf, const uint4* xf) {
    if constexpr (Tr::kSplit) {
      mma_split_step<NE, NPT>(wf, xf, acc);
    } else {
#pragma unroll
      for (int i = 0; i < NE; ++i)
#pragma unroll
        for (int t = 0; t < NPT; ++t) acc[i][t] = mma<Tr>(wf[i], xf[t], acc[i][t]);
    }
  };
  int k0 = 0, k1 = nk;
  if (WS) {
    const int kq = (nk + KW - 1) / KW;
    k0 = (wave % KW) * kq;
    k1 = k0 + kq < nk ? k0 + kq : nk;
  }
  WF wb[SKD][NE];
  uint4 xb[SKD][NPT];
  int ks = k0;
  if (k1 - k0 >= 2 * SKD) {
    // prologue and steady state issue the loads in the same pinned order (MFMAs of step d,
    // then step d + SKD's loads), so the waitcnt pass sees one consistent FIFO of SKD steps
#pragma unroll
    for (int d = 0; d < SKD; ++d) {
      __builtin_amdgcn_sched_barrier(0);
      load_step(k0 + d, wb[d], xb[d]);
    }
    for (; ks + 2 * SKD <= k1; ks += SKD) {
      if constexpr (Tr::kScaled) {
        // FP8: step pairs (d, d + 1) on one block-scaled K=128 MFMA, then both refills
#pragma unroll
        for (int d = 0; d < SKD; d += 2) {
          __builtin_amdgcn_sched_barrier(0);
          const int2 e0 = tab[(ks + d + SKD) * 4 + kg], e1 = tab[(ks + d + 1 + SKD) * 4 + kg];
#pragma unroll
          for (int i = 0; i < NE; ++i)
#pragma unroll
            for (int t = 0; t < NPT; ++t)
              acc[i][t] = mma2<Tr>(wb[d][i], wb[d + 1][i], xb[d][t], xb[d + 1][t], acc[i][t]);
          __builtin_amdgcn_sched_barrier(0);
          issue(ks + d + SKD, e0, wb[d], xb[d]);
          issue(ks + d + 1 + SKD, e1, wb[d + 1], xb[d + 1]);
        }
      } else {
#pragma unroll
        for (int d = 0; d < SKD; ++d) {
          __builtin_amdgcn_sched_barrier(0);
          const int2 e = tab[(ks + d + SKD) * 4 + kg];  // LDS read in flight over the MFMAs
          step_mma(wb[d], xb[d]);
          __builtin_amdgcn_sched_barrier(0);
          issue(ks + d + SKD, e, wb[d], xb[d]);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (Tr::kScaled) {
#pragma unroll
      for (int d = 0; d < SKD; d += 2)
#pragma unroll
        for (int i = 0; i < NE; ++i)
#pragma unroll
          for (int t = 0; t < NPT; ++t) acc[i][t] = mma2<Tr>(wb[d][i], wb[d + 1][i], xb[d][t], xb[d + 1][t], acc[i][t]);
    } else {
#pragma unroll
      for (int d = 0; d < SKD; ++d) step_mma(wb[d], xb[d]);
    }
    ks += SKD;
  }
  // short K ranges (the split-K waves of the low-resolution layers own 3-11 steps) and the
  // tail: up to SKD steps of loads in flight, refilled as each step's MFMAs consume them
  // (ks and k1 are wave-uniform: the guards are scalar branches)
  if (ks < k1) {
#pragma unroll
    for (int d = 0; d < SKD; ++d)
      if (ks + d < k1) load_step(ks + d, wb[d], xb[d]);
    for (; ks < k1; ks += SKD) {
      if constexpr (Tr::kScaled) {
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);  // an odd last step pairs with zeros
#pragma unroll
        for (int d = 0; d < SKD; d += 2) {
          if (ks + d < k1) {
            const bool two = ks + d + 1 < k1;
#pragma unroll
            for (int i = 0; i < NE; ++i)
#pragma unroll
              for (int t = 0; t < NPT; ++t)
                acc[i][t] = mma2<Tr>(wb[d][i], two ? wb[d + 1][i] : z, xb[d][t], two ? xb[d + 1][t] : z, acc[i][t]);
            if (ks + d + SKD < k1) load_step(ks + d + SKD, wb[d], xb[d]);
            if (two && ks + d + 1 + SKD < k1) load_step(ks + d + 1 + SKD, wb[d + 1], xb[d + 1]);
          }
        }
      } else {
#pragma unroll
        for (int d = 0; d < SKD; ++d) {
          if (ks + d < k1) {
            step_mma(wb[d], xb[d]);
            if (ks + d + SKD < k1) load_step(ks + d + SKD, wb[d], xb[d]);
          }
        }
      }
    }
  }
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin + 1] = wall_clock64();
  if constexpr (WS) {
    // partial tiles to LDS; each wave of a K-split group g (waves g KW .. g KW + KW - 1) then
    // finishes the group's (tile, fragment) slots q = KW j + (wave % KW), with the slots' bias
    // and residual loads in flight over the barrier (runtime slot indices: no acc registers
    // live in the epilogue)
    f32x4* red = (f32x4*)(smem + (((size_t)nk * 4 * 8 + 15) & ~(size_t)15));
#pragma unroll
    for (int i = 0; i < NE; ++i)
#pragma unroll
      for (int t = 0; t < NPT; ++t) red[((wave * NE + i) * NPT + t) * 64 + lane] = acc[i][t];
    constexpr int J = (NE * NPT + KW - 1) / KW;
    const int w0 = wave - wave % KW;  // the group's first wave
    float4 sb[J], ss[J];
    float rv[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = j * KW + wave % KW, i = q / NPT, t = q - i * NPT;
      const int n0 = (nt0 + i) * 16 + kg * 4, p = pbase + t * 16 + col;
      const bool ok = q < NE * NPT && nt0 + i < a.n_tiles && n0 < a.cout && p < a.M;
      sb[j] = ok ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (Tr::kScaled) ss[j] = dq4<Tr>(a.bias, a.n_tiles, ok ? n0 : 0);
      if (a.res && ok) load4((const T*)a.res + (size_t)p * a.r_cstride + a.r_coff + n0, rv[j]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = j * KW + wave % KW, i = q / NPT, t = q - i * NPT;
      const int n0 = (nt0 + i) * 16 + kg * 4, p = pbase + t * 16 + col;
      if (!(q < NE * NPT && nt0 + i < a.n_tiles && n0 < a.cout && p < a.M)) continue;
      f32x4 v4 = red[((w0 * NE + i) * NPT + t) * 64 + lane];
#pragma unroll
      for (int w = 1; w < KW; ++w) {
        const f32x4 u = red[(((w0 + w) * NE + i) * NPT + t) * 64 + lane];
        v4[0] += u[0];
        v4[1] += u[1];
        v4[2] += u[2];
        v4[3] += u[3];
      }
      float v[4] = {v4[0] + sb[j].x, v4[1] + sb[j].y, v4[2] + sb[j].z, v4[3] + sb[j].w};
      if constexpr (Tr::kScaled) {
        v[0] = v4[0] * ss[j].x + sb[j].x;
        v[1] = v4[1] * ss[j].y + sb[j].y;
        v[2] = v4[2] * ss[j].z + sb[j].z;
        v[3] = v4[3] * ss[j].w + sb[j].w;
      }
      if (a.act) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu<Tr::kExact>(v[e]);
      }
      if (a.res) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = rv[j][e] + v[e];
      }
      store4((T*)a.dst + (size_t)p * a.d_cstride + a.d_coff + n0, v);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int nt = nt0 + i;
      if (nt >= a.n_tiles) break;
      const int n0 = nt * 16 + kg * 4;
      if (n0 >= a.cout) continue;
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int p = pbase + t * 16 + col;
        if (p >= a.M) continue;
        const f32x4 v4 = acc[i][t];
        float v[4] = {v4[0] + bb[i].x, v4[1] + bb[i].y, v4[2] + bb[i].z, v4[3] + bb[i].w};
        if constexpr (Tr::kScaled) {
          v[0] = v4[0] * sc[i].x + bb[i].x;
          v[1] = v4[1] * sc[i].y + bb[i].y;
          v[2] = v4[2] * sc[i].z + bb[i].z;
          v[3] = v4[3] * sc[i].w + bb[i].w;
        }
        if (a.act) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = silu<Tr::kExact>(v[e]);
        }
        if (a.res) {
          float r[4];
          load4((const T*)a.res + (size_t)p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = r[e] + v[e];
        }
        store4((T*)a.dst + (size_t)p * a.d_cstride + a.d_coff + n0, v);
      }
    }
  }
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin + 2] = wall_clock64();
}

// Waves per SIMD the register allocation must leave room for (amdgpu_waves_per_eu): a wave of the
// large split tiles wants > 256 of the 512 unified VGPR+AGPR registers, which holds a CU to one
// 256-thread workgroup, so a launch of more workgroups than CUs runs in rounds.
// Measured (round 3, fp32 headline): 2 lets the large split tiles drop their AGPR accumulators and
// run two waves per SIMD without spills, but the headline does not move (5,279 vs 5,264 frames/s:
// those kernels are bound by the split VALU work, not by occupancy); 3 spills (-32 %).
// The op's K-step table into LDS (once per workgroup; conv_fast_body's first barrier publishes it)
__device__ __forceinline__ void fast_table_lds(const FastArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int2* tab = (int2*)smem;
  const int tid = threadIdx.x, nk = a.k_steps;
  int2 tv[2];  // <= 512 entries (nk <= 128) in one round trip
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (tid + u * 256 < nk * 4) tv[u] = a.ktab[tid + u * 256];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (tid + u * 256 < nk * 4) tab[tid + u * 256] = tv[u];
  for (int i = tid + 512; i < nk * 4; i += 256) tab[i] = a.ktab[i];
}

template <class Tr, int NNT, int NPT, int KW, int SKD>
__device__ __forceinline__ void conv_fast_item(const FastArgs& a, int2 blk) {
  const int nt0 = blk.y * NNT;
  const int rem = a.n_tiles - nt0;
  if constexpr (NNT == 1) {
    conv_fast_body<Tr, 1, NPT, KW, SKD>(a, blk, nt0);
  } else {
    if (rem >= NNT) {
      conv_fast_body<Tr, NNT, NPT, KW, SKD>(a, blk, nt0);
    } else if (rem == 1) {
      conv_fast_body<Tr, 1, NPT, KW, SKD>(a, blk, nt0);
    } else if constexpr (NNT > 2) {
      if (rem == 2 || NNT == 3)
        conv_fast_body<Tr, 2, NPT, KW, SKD>(a, blk, nt0);
      else
        conv_fast_body<Tr, (NNT > 3 ? 3 : 1), NPT, KW, SKD>(a, blk, nt0);
    }
  }
}

// One launch = every (pixel block, channel group) item of the op.  ipw = 1: one item per
// workgroup.  ipw > 1 (persistent form): ceil(items / ipw) workgroups, each
// loads the K-step table once and loops over its items; a barrier between items keeps the next
// item's LDS reduction behind this one's epilogue.
// The loop costs registers in every instantiation (the 3-waves-per-SIMD tiles spilled 28-32 B), so
// the persistent form is a build option (YK_DEFINES=-DYK_FAST_PERSIST=1, then YK_FAST_IPW=n at run
// time) for A/B runs; the product kernel is the one-item form.
#ifndef YK_FAST_PERSIST
#define YK_FAST_PERSIST 0
#endif
template <class Tr, int NNT, int NPT, int KW, int SKD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(fast_wpe(NNT, NPT, KW, SKD, Tr::kScaled)))) conv_fast_kernel(FastArgs a) {
  fast_table_lds(a);
  if (!YK_FAST_PERSIST || a.ipw <= 1) {
    conv_fast_item<Tr, NNT, NPT, KW, SKD>(a, xcd_block(a.xcd));
    return;
  }
  for (int q = blockIdx.x; q < a.n_items; q += gridDim.x) {
    conv_fast_item<Tr, NNT, NPT, KW, SKD>(a, xcd_item(q, a.n_items, a.n_cg, a.xcd));
    __syncthreads();
  }
}


// ---------------------------------------------------------------- table conv, weights shared through LDS
// conv_fast_kernel's per-wave layout (wave = NPT x 16 pixels x NNT x 16 channels, activations
// gathered straight to registers through the K-step table), but the four waves of a workgroup
// share one copy of the weight fragments: they are the same for all four waves (same channel
// group), and loading them per wave made three quarters of the workgroup's vector-memory
// instructions redundant (TA-bound: per K step NNT + NPT fragment loads per wave, against
// NPT + NNT / 4 here).  Weights stream through a two-buffer LDS ring in chunks of 4 K steps
// (4 x NNT fragments, one ds_read_b128 per fragment and lane); the chunk boundary is a raw
// s_barrier behind lgkmcnt(0) -- not __syncthreads(), whose fence would drain the activation
// loads in flight (vmcnt(0)).  Same K order and MFMA sequence per accumulator as
// conv_fast_kernel: results are bit-identical.
template <class Tr, int NNT, int NPT, int SKD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(YK_FAST_WPE))) conv_fastw_kernel(FastArgs a) {
  using T = typename Tr::T;
  constexpr int ESZ = (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nk = a.k_steps;
  int2* tab = (int2*)smem;  // [k_steps * 4]
  using WF = typename Frag<Tr>::W;
  WF* ring = (WF*)(smem + (((size_t)nk * 4 * 8 + 15) & ~(size_t)15));  // [2][4][NNT][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, col = lane & 15;
  const int2 blk = xcd_block(a.xcd);
  const int nt0 = blk.y * NNT;
  const int pbase = (blk.x * 4 + wave) * (16 * NPT);
  const int wg_lin = blockIdx.y * gridDim.x + blockIdx.x;
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin] = wall_clock64();
  for (int i = tid; i < nk * 4; i += 256) tab[i] = a.ktab[i];
  const __amdgpu_buffer_rsrc_t xr = make_srd(a.arena, a.arena_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_srd(a.wblob, a.wbytes);
  const int hw = a.out_h * a.out_w;
  unsigned vo0[NPT], vo1[NPT], vm[NPT];
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int p = pbase + t * 16 + col;
    const bool pv = p < a.M;
    const int pp = pv ? p : 0;
    const int b = fdiv(pp, hw, a.inv_hw);
    const int r = pp - b * hw;
    const int oy = fdiv(r, a.out_w, a.inv_w);
    const int ox = r - oy * a.out_w;
    const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
    vo0[t] = a.soff0 + (unsigned)(((b * a.h0 + (iy0 >> a.up0)) * a.w0 + (ix0 >> a.up0)) * a.cs0 * ESZ);
    vo1[t] = a.soff1 + (unsigned)(((b * a.h1 + (iy0 >> a.up1)) * a.w1 + (ix0 >> a.up1)) * a.cs1 * ESZ);
    const unsigned cm = ((unsigned)(ix0 >= 0 && ix0 < a.in_w)) | ((unsigned)(ix0 + 1 >= 0 && ix0 + 1 < a.in_w) << 1) |
                        ((unsigned)(ix0 + 2 >= 0 && ix0 + 2 < a.in_w) << 2);
    const unsigned m = ((iy0 >= 0 && iy0 < a.in_h) ? cm : 0u) | ((iy0 + 1 >= 0 && iy0 + 1 < a.in_h) ? cm << 3 : 0u) |
                       ((iy0 + 2 >= 0 && iy0 + 2 < a.in_h) ? cm << 6 : 0u);
    vm[t] = pv ? m : 0u;
  }
  f32x4 acc[NNT][NPT];
#pragma unroll
  for (int i = 0; i < NNT; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bb[NNT];
  float4 sc[NNT];
#pragma unroll
  for (int i = 0; i < NNT; ++i) {
    const int n0 = (nt0 + i) * 16 + kg * 4;
    bb[i] = (nt0 + i < a.n_tiles && n0 < a.cout) ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (Tr::kScaled) sc[i] = dq4<Tr>(a.bias, a.n_tiles, n0 < a.cout ? n0 : 0);
  }
  // weight staging: fragment f = wave + 4 j (j < NNT) of a chunk = (step d = f & 3, tile i = f >> 2)
  // (F32S: the 32-byte split fragment, two loads and two ring stores)
  WF wst[NNT];
  auto stage_load = [&](int c) {
#pragma unroll
    for (int j = 0; j < NNT; ++j) {
      const int f = wave + 4 * j, d = f & 3, i = f >> 2;
      const int ks = 4 * c + d;
      const int nt = nt0 + i < a.n_tiles ? nt0 + i : a.n_tiles - 1;
      const unsigned off = a.woff + (unsigned)((((size_t)nt * nk + (ks < nk ? ks : 0)) * 64 + lane) * Frag<Tr>::WB);
      wst[j] = wload<Tr>(wr, off, 0);
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NNT; ++j) {
      const int f = wave + 4 * j, d = f & 3, i = f >> 2;
      ring[((buf * 4 + d) * NNT + i) * 64 + lane] = wst[j];
    }
  };
  auto act_load = [&](int ks, uint4* xf) {
    const int2 e = tab[ks * 4 + kg];
    const unsigned tap = (unsigned)e.y & 15u;
    const bool s1 = (e.y & 16) != 0, ev = (e.y & 32) != 0;
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const bool ok = ev && ((vm[t] >> tap) & 1u);
      const unsigned off = (s1 ? vo1[t] : vo0[t]) + (unsigned)e.x;
      xf[t] = bload(xr, ok ? off : kOOB, 0);
    }
  };
  stage_load(0);
  stage_store(0);
  __syncthreads();  // the table and chunk 0 of the ring (nothing else in flight yet)
  uint4 xb[SKD][NPT];
#pragma unroll
  for (int d = 0; d < SKD; ++d)
    if (d < nk) act_load(d, xb[d]);
  const int nch = (nk + 3) >> 2;
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) stage_load(c + 1);  // in flight over this chunk's MFMAs
    const WF* wb = ring + (size_t)(c & 1) * 4 * NNT * 64;
    if constexpr (Tr::kScaled) {
      // FP8: steps (d, d + 1) of the chunk on one block-scaled K=128 MFMA (odd tail: zeros)
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int d = 0; d < 4; d += 2) {
        const int ks = 4 * c + d;
        if (ks < nk) {
          const bool two = ks + 1 < nk;
          uint4 w0[NNT], w1[NNT];
#pragma unroll
          for (int i = 0; i < NNT; ++i) {
            w0[i] = wb[(d * NNT + i) * 64 + lane];
            w1[i] = two ? wb[((d + 1) * NNT + i) * 64 + lane] : z;
          }
          uint4* x0 = xb[d % SKD];
          uint4* x1 = xb[(d + 1) % SKD];
#pragma unroll
          for (int i = 0; i < NNT; ++i)
#pragma unroll
            for (int t = 0; t < NPT; ++t) acc[i][t] = mma2<Tr>(w0[i], w1[i], x0[t], two ? x1[t] : z, acc[i][t]);
          if (ks + SKD < nk) act_load(ks + SKD, x0);
          if (two && ks + 1 + SKD < nk) act_load(ks + 1 + SKD, x1);
        }
      }
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int ks = 4 * c + d;
        if (ks < nk) {
          WF wf[NNT];
#pragma unroll
          for (int i = 0; i < NNT; ++i) wf[i] = wb[(d * NNT + i) * 64 + lane];
          // step ks's activations sit in slot ks % SKD = d % SKD (SKD divides 4): a compile-time
          // index, so the slots stay registers
          uint4* xf = xb[d % SKD];
          if constexpr (Tr::kSplit) {
            mma_split_step<NNT, NPT>(wf, xf, acc);
          } else {
#pragma unroll
            for (int i = 0; i < NNT; ++i)
#pragma unroll
              for (int t = 0; t < NPT; ++t) acc[i][t] = mma<Tr>(wf[i], xf[t], acc[i][t]);
          }
          if (ks + SKD < nk) act_load(ks + SKD, xf);
        }
      }
    }
    if (more) {
      stage_store((c + 1) & 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's ring writes landed
      __builtin_amdgcn_s_barrier();
    }
  }
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin + 1] = wall_clock64();
#pragma unroll
  for (int i = 0; i < NNT; ++i) {
    const int nt = nt0 + i;
    if (nt >= a.n_tiles) break;
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
#pragma unroll
    for (int t = 0; t < NPT; ++t) {
      const int p = pbase + t * 16 + col;
      if (p >= a.M) continue;
      const f32x4 v4 = acc[i][t];
      float v[4] = {v4[0] + bb[i].x, v4[1] + bb[i].y, v4[2] + bb[i].z, v4[3] + bb[i].w};
      if constexpr (Tr::kScaled) {
        v[0] = v4[0] * sc[i].x + bb[i].x;
        v[1] = v4[1] * sc[i].y + bb[i].y;
        v[2] = v4[2] * sc[i].z + bb[i].z;
        v[3] = v4[3] * sc[i].w + bb[i].w;
      }
      if (a.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu<Tr::kExact>(v[j]);
      }
      if (a.res) {
        float r[4];
        load4((const T*)a.res + (size_t)p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = r[j] + v[j];
      }
      store4((T*)a.dst + (size_t)p * a.d_cstride + a.d_coff + n0, v);
    }
  }
  if (a.tstamp && tid == 0 && wg_lin < a.tstamp_cap) a.tstamp[3 * wg_lin + 2] = wall_clock64();
}

inline size_t fastw_lds(int k_steps, int nnt, int wb) {
  return (((size_t)k_steps * 4 * 8 + 15) & ~(size_t)15) + (size_t)2 * 4 * nnt * 64 * wb;
}

// ---------------------------------------------------------------- persistent LDS-tiled conv (wide layers)
// For the high-resolution layers (P2/P3: 20,480 / 5,120 pixels per image) the gather kernel
// re-fetches every input pixel once per tap and every weight fragment once per wave through
// the 32 KiB L1 (L1/L2-bandwidth-bound).  Here a workgroup keeps its NNT x 16 output
// channels' whole weight slab resident in LDS, loops over 16 x 16-pixel output tiles (grid =
// resident capacity, blockIdx.y = output-channel group) and double-buffers the input tiles
// (+ halo, all K-space channels of both sources) in LDS: tile i+1's global loads are in flight
// while tile i computes.  Staging addresses are precomputed per thread (the unit pattern is
// the same for every tile); invalid pixels are buffer offsets past the arena (hardware zeros).
// Wave w computes rows 4w..4w+3 of a tile; a K step is one LDS table read, 4 + NNT
// ds_read_b128 and 4 x NNT MFMAs.
struct WideArgs {
  const void* arena;
  unsigned arena_bytes;
  unsigned soff0, soff1;
  int h0, w0, cs0, up0, h1, w1, cs1, up1;
  int c0, cin;
  int stride, pad, in_h, in_w, out_h, out_w, B;
  int tiles_x, tiles_y, tih, tiw, ps;
  const uint4* wpk;
  const float* bias;
  const int* ltab;               // [k_steps][4] LDS element offsets (K padding: 0, zero weights)
  int k_steps, n_tiles;
  void* dst;
  int d_cstride, d_coff, cout;
  const void* res;
  int r_cstride, r_coff;
  int act;
  int xcd;
  int dbg;  // diagnostics (YK_WIDE_DBG): 1 = no K loop, 2 = no epilogue stores, 4 = no staging
};

__host__ __device__ inline size_t wide_tile_bytes(int tih, int tiw, int ps, int esz) {
  return (((size_t)tih * tiw * ps * esz) + 15) & ~(size_t)15;
}
inline size_t wide_lds(int nnt, int k_steps, int tih, int tiw, int ps, int esz) {
  return (size_t)nnt * k_steps * 1024 + (size_t)((k_steps + 3) & ~3) * 16 + 2 * wide_tile_bytes(tih, tiw, ps, esz);
}

template <class Tr, int NNT, int UPT, int NW>
__global__ void __launch_bounds__(64 * NW) conv_wide_kernel(WideArgs a) {
  // NW waves per workgroup (4 or 8: one or two per SIMD, the second hides the LDS latency of
  // the first); wave w computes rows NPT*w .. NPT*w + NPT - 1 of the 16-row tile
  using T = typename Tr::T;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int EU = 16 / ESZ;
  constexpr int NTH = 64 * NW;
  constexpr int NPT = 16 / NW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nk = a.k_steps;
  uint4* wl = (uint4*)smem;                                   // [NNT][nk][64]
  int* ltab = (int*)(smem + (size_t)NNT * nk * 1024);         // [nk][4]
  T* xt0 = (T*)(smem + (size_t)NNT * nk * 1024 + (size_t)((nk + 3) & ~3) * 16);
  const size_t tbytes = wide_tile_bytes(a.tih, a.tiw, a.ps, ESZ);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, col = lane & 15;
  const int2 blk = xcd_block(a.xcd);
  const int nt0 = blk.y * NNT;
  const int nsp = a.B * a.tiles_y * a.tiles_x;
  int t = blk.x;
  if (t >= nsp) return;
  const __amdgpu_buffer_rsrc_t xr = make_srd(a.arena, a.arena_bytes);
  // resident weights + table
  for (int i = tid; i < NNT * nk * 64; i += NTH) {
    const int ni = i / (nk * 64), r = i - ni * nk * 64;
    const int nt = nt0 + ni < a.n_tiles ? nt0 + ni : a.n_tiles - 1;
    wl[i] = a.wpk[(size_t)nt * nk * 64 + r];
  }
  // table transposed to [kg][nk4] (nk4 = nk rounded up to 4; padding entries 0): a lane's four
  // consecutive K steps are one ds_read_b128
  const int nk4 = (nk + 3) & ~3;
  for (int i = tid; i < nk4 * 4; i += NTH) {
    const int g = i / nk4, ks = i - g * nk4;
    ltab[i] = ks < nk ? a.ltab[ks * 4 + g] : 0;
  }
  // per-thread staging units: packed (ry << 24 | rx << 16 | src << 15 | channel), LDS offset
  const int U = a.cin / EU;
  const int total = a.tih * a.tiw * U;
  int ud[UPT], ul[UPT];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int i = tid + j * NTH;
    ud[j] = -1;
    ul[j] = 0;
    if (i < total) {
      const int pix = i / U, uu = i - pix * U;
      const int ry = pix / a.tiw, rx = pix - ry * a.tiw;
      const int c = uu * EU;
      const int src = c >= a.c0 ? 1 : 0;
      ud[j] = (ry << 24) | (rx << 16) | (src << 15) | (src ? c - a.c0 : c);
      ul[j] = pix * a.ps + uu * EU;
    }
  }
  int prow[NPT];
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) prow[pt] = ((wave * NPT + pt) * a.stride * a.tiw + col * a.stride) * a.ps;
  float4 bb[NNT];
  float4 sc[NNT];  // FP8 dequant scales
#pragma unroll
  for (int ni = 0; ni < NNT; ++ni) {
    const int n0 = (nt0 + ni) * 16 + kg * 4;
    bb[ni] = (nt0 + ni < a.n_tiles && n0 < a.cout) ? *(const float4*)(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (Tr::kScaled) sc[ni] = dq4<Tr>(a.bias, a.n_tiles, n0 < a.cout ? n0 : 0);
  }
  const int tpi = a.tiles_y * a.tiles_x;
  uint4 st[UPT];
  auto fetch = [&](int tt) {
    const int b = tt / tpi, r = tt - b * tpi;
    const int ty = r / a.tiles_x, tx = r - ty * a.tiles_x;
    const int iy0 = ty * 16 * a.stride - a.pad, ix0 = tx * 16 * a.stride - a.pad;
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const int d = ud[j];
      const int iy = iy0 + (d >> 24), ix = ix0 + ((d >> 16) & 255);
      const bool s1 = (d >> 15) & 1;
      const int h = s1 ? a.h1 : a.h0, w = s1 ? a.w1 : a.w0, cs = s1 ? a.cs1 : a.cs0, up = s1 ? a.up1 : a.up0;
      const unsigned so = s1 ? a.soff1 : a.soff0;
      const bool ok = d >= 0 && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      const unsigned off = so + (unsigned)((((b * h + (iy >> up)) * w + (ix >> up)) * cs + (d & 0x7fff)) * ESZ);
      st[j] = bload(xr, ok ? off : kOOB, 0);
    }
  };
  auto commit = [&](T* xt) {
#pragma unroll
    for (int j = 0; j < UPT; ++j)
      if (ud[j] >= 0) *(uint4*)(xt + ul[j]) = st[j];
  };
  fetch(t);
  commit(xt0);
  __syncthreads();
  for (int it = 0;; ++it) {
    const int tn = t + gridDim.x;
    if (tn < nsp && !(a.dbg & 4)) fetch(tn);  // in flight over this tile's K loop
    const T* xt = (const T*)((const unsigned char*)xt0 + (it & 1) * tbytes);
    f32x4 acc[NNT][NPT];
#pragma unroll
    for (int ni = 0; ni < NNT; ++ni)
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) acc[ni][pt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nkl = (a.dbg & 1) ? 0 : nk;
    // four K steps per iteration: every LDS read of the group is issued before its MFMAs
    // (sched_barrier: the scheduler would otherwise sink each read to its first use)
    const int4* lt4 = (const int4*)(ltab + kg * nk4);
    int k4 = 0;
    for (; k4 + 4 <= nkl; k4 += 4) {
      const int4 e4 = lt4[k4 >> 2];
      const int ev[4] = {e4.x, e4.y, e4.z, e4.w};
      uint4 xf[4][NPT], wf[4][NNT];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
#pragma unroll
        for (int ni = 0; ni < NNT; ++ni) wf[d][ni] = wl[(ni * nk + k4 + d) * 64 + lane];
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) xf[d][pt] = *(const uint4*)(xt + prow[pt] + ev[d]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (Tr::kScaled) {  // FP8: step pairs on one block-scaled K=128 MFMA
#pragma unroll
        for (int d = 0; d < 4; d += 2)
#pragma unroll
          for (int ni = 0; ni < NNT; ++ni)
#pragma unroll
            for (int pt = 0; pt < NPT; ++pt)
              acc[ni][pt] = mma2<Tr>(wf[d][ni], wf[d + 1][ni], xf[d][pt], xf[d + 1][pt], acc[ni][pt]);
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int ni = 0; ni < NNT; ++ni)
#pragma unroll
            for (int pt = 0; pt < NPT; ++pt) acc[ni][pt] = mma<Tr>(wf[d][ni], xf[d][pt], acc[ni][pt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    for (; k4 < nkl; ++k4) {
      const int e = ltab[kg * nk4 + k4];
      uint4 xf[NPT];
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) xf[pt] = *(const uint4*)(xt + prow[pt] + e);
#pragma unroll
      for (int ni = 0; ni < NNT; ++ni) {
        const uint4 w = wl[(ni * nk + k4) * 64 + lane];
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt)
          acc[ni][pt] = Tr::kScaled ? mma2<Tr>(w, z, xf[pt], z, acc[ni][pt]) : mma<Tr>(w, xf[pt], acc[ni][pt]);
      }
    }
    // epilogue of tile t
    {
      const int b = t / tpi, r = t - b * tpi;
      const int ty = r / a.tiles_x, tx = r - ty * a.tiles_x;
      const int ox = tx * 16 + col;
#pragma unroll
      for (int ni = 0; ni < NNT; ++ni) {
        const int n0 = (nt0 + ni) * 16 + kg * 4;
        if (nt0 + ni >= a.n_tiles || n0 >= a.cout) continue;
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) {
          const int oy = ty * 16 + wave * NPT + pt;
          if (oy >= a.out_h || ox >= a.out_w) continue;
          const size_t p = ((size_t)b * a.out_h + oy) * a.out_w + ox;
          float v[4] = {acc[ni][pt][0] + bb[ni].x, acc[ni][pt][1] + bb[ni].y, acc[ni][pt][2] + bb[ni].z,
                        acc[ni][pt][3] + bb[ni].w};
          if constexpr (Tr::kScaled) {
            v[0] = acc[ni][pt][0] * sc[ni].x + bb[ni].x;
            v[1] = acc[ni][pt][1] * sc[ni].y + bb[ni].y;
            v[2] = acc[ni][pt][2] * sc[ni].z + bb[ni].z;
            v[3] = acc[ni][pt][3] * sc[ni].w + bb[ni].w;
          }
          if (a.act) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = silu<Tr::kExact>(v[j]);
          }
          if (a.res) {
            float rr[4];
            load4((const T*)a.res + p * a.r_cstride + a.r_coff + n0, rr);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = rr[j] + v[j];
          }
          if (!(a.dbg & 2) || v[0] == 12345.f) store4((T*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
        }
      }
    }
    if (tn >= nsp) break;
    commit((T*)((unsigned char*)xt0 + ((it + 1) & 1) * tbytes));
    __syncthreads();
    t = tn;
  }
}

// ---------------------------------------------------------------- halo-tile split conv (F32 build)
// The F32S body of conv_fast splits every activation fragment into its bf16 parts as it loads
// it -- once per tap and per output-channel group, so a 3x3 conv splits each element 9 times
// per group -- and that VALU work, not the matrix cores, bounds it (r03 PMC + ISA: ~4 VALU per
// v_mfma_f32_16x16x32_bf16, whose issue shadow holds 2).  Here a workgroup stages its output
// tile's input window (tile + halo) into LDS ALREADY SPLIT, 16 channels at a time, and every
// tap reads its B operands straight from there: the split runs once per staged element.
// Operand layout ("K-slot", weights built by build_wkslot): lane group kg's 8 bf16 K slots hold
// its 4 channels twice, XA = [x0(e0..3) | x1(e0..3)] and XB = [x0(e0..3) | x2(e0..3)], against
// weight fragments A1 = [w0 | w0], A2 = [w1 | w1], A3 = [w2 | w0]: A1.XA + A2.XA + A3.XB = the six
// products of F32S (w0x0 + w0x1 + w1x0 + w1x1 + w2x0 + w0x2), three MFMAs per fragment pair.
// K order: 16-channel group major, tap minor (step s = group * k*k + tap).
// LDS: two chunk buffers of 32 KiB; a chunk is one 16-channel group of the window (3x3: 8 planes
// XA / XB x kg of kHaloPx pixels x 16 B) or four of them (1x1, no halo: 32 planes of kHaloPx / 4
// pixels).  Plane bases are multiples of 256 B, so the 16 consecutive pixels of a fragment row
// fall on 16 different 4-bank groups (ds_read_b128 conflict-free).  One barrier per chunk: chunk
// c + 1's global loads are in flight over chunk c's MFMAs, then split and written to the other
// buffer.  Within a chunk each step's B operands are read one step ahead and the weight
// fragments D steps ahead (a ring of D register slots).
// Wave layout: WM = 0, the four waves split the tile's pixels (NPT fragments each) and share
// NE output-channel tiles; WM = 1, they share all NPT fragments and own NE tiles each.
struct HaloArgs {
  const void* arena;
  unsigned arena_bytes;
  unsigned soff0, soff1;  // byte offsets of the two source views (image b0, channel coff)
  int h0, w0, cs0, up0, h1, w1, cs1, up1;
  int c0, cin;
  int stride, pad, in_h, in_w, out_h, out_w;
  int tr, tc, twin, npx, tiles_x, tiles_y;  // output tile rows x cols, input window width, pixels
  int rp;  // LDS row pitch of the window (pixels): rp = tc (mod 16) (stride 1) or 2 rp = tc (mod 16)
           // (stride 2), so a fragment's 16 pixels fall on 16 consecutive 4-bank groups wherever
           // its rows break
  int hw;  // stride 2: the window's even columns are stored first (hw of them), then the odd
           // ones, so the pixels one tap reads are consecutive in LDS
  const void* wblob;  // K-slot weights: byte offset woff, [n_tiles][n_chunks * k * k][64][48 B]
  unsigned wbytes, woff;
  const float* bias;
  int n_tiles;
  void* dst;
  int d_cstride, d_coff, cout;
  const void* res;
  int r_cstride, r_coff;
  int act;
  int xcd;
};
constexpr int kHaloPx = 256;                                 // pixels per LDS plane
constexpr int kHaloPlaneB = kHaloPx * 16;                    // bytes per plane
constexpr size_t kHaloLds = (size_t)2 * 8 * kHaloPlaneB;     // 64 KiB: two workgroups per CU

struct WK3 {
  u32x4v a1, a2, a3;
};

// x = x0 + x1 + x2 per element (bf16 RNE parts, as split3), in the K-slot layout
__device__ __forceinline__ void split_kslot(const uint4& x, u32x4v& xa, u32x4v& xb) {
  const float a0 = __uint_as_float(x.x), a1 = __uint_as_float(x.y), a2 = __uint_as_float(x.z),
              a3 = __uint_as_float(x.w);
  const unsigned p0 = pack_bf16x2(a0, a1), p1 = pack_bf16x2(a2, a3);
  // the remainders of an element pair in one v_pk_add_f32
  const f32x2v ra = f32x2v{a0, a1} - f32x2v{__uint_as_float(p0 << 16), __uint_as_float(p0 & 0xffff0000u)};
  const f32x2v rb = f32x2v{a2, a3} - f32x2v{__uint_as_float(p1 << 16), __uint_as_float(p1 & 0xffff0000u)};
  const float r0 = ra[0], r1 = ra[1], r2 = rb[0], r3 = rb[1];
  const unsigned q0 = pack_bf16x2(r0, r1), q1 = pack_bf16x2(r2, r3);
  const f32x2v sa = ra - f32x2v{__uint_as_float(q0 << 16), __uint_as_float(q0 & 0xffff0000u)};
  const f32x2v sb = rb - f32x2v{__uint_as_float(q1 << 16), __uint_as_float(q1 & 0xffff0000u)};
  const float s0 = sa[0], s1 = sa[1], s2 = sb[0], s3 = sb[1];
  xa = u32x4v{p0, p1, q0, q1};
  xb = u32x4v{p0, p1, pack_bf16x2(s0, s1), pack_bf16x2(s2, s3)};
}

template <int NE, int NPT, int WM, int KS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(YK_FAST_WPE))) conv_halo_kernel(HaloArgs a) {
  constexpr int T = KS * KS;
  constexpr int CC = KS == 1 ? 4 : 1;   // 16-channel groups staged per chunk (1x1: no halo, 4 groups)
  constexpr int PXC = kHaloPx / CC;     // pixels per plane
  constexpr int PLB = PXC * 16;         // bytes per plane
  constexpr int S = CC * T;             // K steps per chunk
  constexpr int D = KS == 3 ? 3 : 2;    // weight-fragment ring: step s + D loads over step s
  constexpr int BUF = 8 * CC * PLB;     // one chunk buffer (kHaloLds / 2)
  constexpr int UPT = 4;                // staging units per thread: 1024 = 4 kg x kHaloPx per chunk
  static_assert(S % D == 0, "the ring slot of a chunk's first step is 0");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = lane >> 4, col = lane & 15;
  const int2 blk = xcd_block(a.xcd);
  const int tpi = a.tiles_x * a.tiles_y;
  const int b = blk.x / tpi, rr = blk.x - b * tpi;
  const int tyi = rr / a.tiles_x, txi = rr - tyi * a.tiles_x;
  const int oy0 = tyi * a.tr, ox0 = txi * a.tc;
  const int iy0 = oy0 * a.stride - a.pad, ix0 = ox0 * a.stride - a.pad;
  const int nt0 = (blk.y * (WM ? 4 : 1) + (WM ? wave : 0)) * NE;
  const int n_groups = (a.cin + 15) >> 4, nsteps = n_groups * T;
  const int n_chunks = (n_groups + CC - 1) / CC;
  const __amdgpu_buffer_rsrc_t xr = make_srd(a.arena, a.arena_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_srd(a.wblob, a.wbytes);
  // the lane's pixel of each fragment: LDS byte offset of its window origin in plane XA(g 0, kg)
  unsigned lb[NPT];
  int opx[NPT];  // output pixel index, -1 outside the image / tile
#pragma unroll
  for (int t = 0; t < NPT; ++t) {
    const int f = WM ? t : wave * NPT + t;
    const int q = f * 16 + col;
    const int ty = q / a.tc, tx = q - ty * a.tc;
    const bool v = q < a.tr * a.tc && oy0 + ty < a.out_h && ox0 + tx < a.out_w;
    lb[t] = (unsigned)(kg * PLB + (v ? (ty * a.stride * a.rp + tx) * 16 : 0));
    opx[t] = v ? (b * a.out_h + oy0 + ty) * a.out_w + ox0 + tx : -1;
  }
  // staging unit j of a thread: channel group kgu = (tid >> 4) & 3, window pixel px = (tid & 15)
  // + 16 (tid >> 6) (+ 64 j with one 16-channel group per chunk; with four, group j) -- the eight
  // lanes of a ds_write_b128 group write 8 consecutive pixels of one plane (conflict-free)
  const int kgu = (tid >> 4) & 3;
  unsigned sv0[UPT], sv1[UPT];
  int sl[UPT];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int px = (tid & 15) + 16 * (tid >> 6) + (CC == 1 ? 64 * j : 0);
    const int g = CC == 1 ? 0 : j;
    sl[j] = -1;
    sv0[j] = sv1[j] = kOOB;
    if (px < a.npx) {
      const int py = px / a.twin, pxx = px - py * a.twin;
      const int iy = iy0 + py, ix = ix0 + pxx;
      const int cx = a.hw ? ((pxx & 1) ? a.hw + (pxx >> 1) : (pxx >> 1)) : pxx;
      sl[j] = (g * 8 + kgu) * PLB + (py * a.rp + cx) * 16;
      if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
        sv0[j] = a.soff0 + (unsigned)(((b * a.h0 + (iy >> a.up0)) * a.w0 + (ix >> a.up0)) * a.cs0 * 4);
        sv1[j] = a.soff1 + (unsigned)(((b * a.h1 + (iy >> a.up1)) * a.w1 + (ix >> a.up1)) * a.cs1 * 4);
      }
    }
  }
  uint4 st[UPT];
  auto fetch = [&](int c) {
    if constexpr ((YK_HALO_DIAG & 2) != 0) return;  // diagnostic: no staging
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const int ch = (c * CC + (CC == 1 ? 0 : j)) * 16 + kgu * 4;
      const bool s1 = ch >= a.c0, cv = ch < a.cin;
      const unsigned o = s1 ? sv1[j] : sv0[j];
      st[j] = bload(xr, cv && o != kOOB ? o + (unsigned)((s1 ? ch - a.c0 : ch) * 4) : kOOB, 0);
    }
  };
  auto commit = [&](int buf) {
    if constexpr ((YK_HALO_DIAG & 2) != 0) return;
    unsigned char* base = smem + buf * BUF;
#pragma unroll
    for (int j = 0; j < UPT; ++j)
      if (sl[j] >= 0) {
        u32x4v xa, xb;
        split_kslot(st[j], xa, xb);
        *(u32x4v*)(base + sl[j]) = xa;
        *(u32x4v*)(base + 4 * PLB + sl[j]) = xb;
      }
  };
  unsigned wo[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int nt = nt0 + i < a.n_tiles ? nt0 + i : a.n_tiles - 1;
    wo[i] = a.woff + (unsigned)(((size_t)nt * nsteps * 64 + lane) * 48);
  }
  auto wload3 = [&](int s, WK3* w) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      if constexpr ((YK_HALO_DIAG & 1) != 0) {  // diagnostic: no weight loads
        const unsigned v = wo[i] ^ (unsigned)s;
        w[i].a1 = u32x4v{v, v + 1u, v + 2u, v + 3u};
        w[i].a2 = u32x4v{v + 4u, v, v + 5u, v};
        w[i].a3 = u32x4v{v, v + 7u, v, v + 9u};
        continue;
      }
      w[i].a1 = __builtin_amdgcn_raw_buffer_load_b128(wr, (int)wo[i], s * 64 * 48, 0);
      w[i].a2 = __builtin_amdgcn_raw_buffer_load_b128(wr, (int)wo[i] + 16, s * 64 * 48, 0);
      w[i].a3 = __builtin_amdgcn_raw_buffer_load_b128(wr, (int)wo[i] + 32, s * 64 * 48, 0);
    }
  };
  // B operands of step k of a chunk (group k / T, tap k % T) from buffer xs
  auto read_ops = [&](const unsigned char* xs, int k, u32x4v* xa, u32x4v* xb) {
    const int g = k / T, t = k - g * T;
    const int dy = t / KS, dx = t - dy * KS;
    const int cdx = a.hw ? ((dx & 1) ? a.hw + (dx >> 1) : (dx >> 1)) : dx;
    const unsigned toff = (unsigned)((dy * a.rp + cdx) * 16);
#pragma unroll
    for (int f = 0; f < NPT; ++f) {
      const unsigned char* p = xs + g * 8 * PLB + lb[f] + toff;
      xa[f] = *(const u32x4v*)p;
      xb[f] = *(const u32x4v*)(p + 4 * PLB);
    }
  };
  f32x4 acc[NE][NPT];
#pragma unroll
  for (int i = 0; i < NE; ++i)
#pragma unroll
    for (int t = 0; t < NPT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  WK3 wb[D][NE];
  u32x4v xa[2][NPT], xb[2][NPT];
  fetch(0);
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < nsteps) wload3(d, wb[d]);
  commit(0);
  __syncthreads();
  for (int c = 0; c < n_chunks; ++c) {
    const bool more = c + 1 < n_chunks;
    if (more) fetch(c + 1);  // in flight over this chunk's MFMAs
    const unsigned char* xs = smem + (c & 1) * BUF;
    const int s0 = c * S;
    read_ops(xs, 0, xa[0], xb[0]);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int s = s0 + k;
      if (s < nsteps) {  // (a 1x1 conv's last chunk may hold fewer than CC groups)
        if (k + 1 < S && s + 1 < nsteps) read_ops(xs, k + 1, xa[(k + 1) & 1], xb[(k + 1) & 1]);
        const WK3* w = wb[k % D];
        const u32x4v* ca = xa[k & 1];
        const u32x4v* cb = xb[k & 1];
#pragma unroll
        for (int f = 0; f < NPT; ++f)
#pragma unroll
          for (int i = 0; i < NE; ++i) acc[i][f] = mfma_bf16(w[i].a1, ca[f], acc[i][f]);
#pragma unroll
        for (int f = 0; f < NPT; ++f)
#pragma unroll
          for (int i = 0; i < NE; ++i) acc[i][f] = mfma_bf16(w[i].a2, ca[f], acc[i][f]);
#pragma unroll
        for (int f = 0; f < NPT; ++f)
#pragma unroll
          for (int i = 0; i < NE; ++i) acc[i][f] = mfma_bf16(w[i].a3, cb[f], acc[i][f]);
        if (s + D < nsteps) wload3(s + D, wb[k % D]);
      }
    }
    if (more) commit((c + 1) & 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int nt = nt0 + i;
    const int n0 = nt * 16 + kg * 4;
    if (nt >= a.n_tiles || n0 >= a.cout) continue;
    const float4 bb = *(const float4*)(a.bias + n0);
#pragma unroll
    for (int f = 0; f < NPT; ++f) {
      const int p = opx[f];
      if (p < 0) continue;
      float v[4] = {acc[i][f][0] + bb.x, acc[i][f][1] + bb.y, acc[i][f][2] + bb.z, acc[i][f][3] + bb.w};
      if (a.act) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu<true>(v[j]);
      }
      if (a.res) {
        float r[4];
        load4((const float*)a.res + (size_t)p * a.r_cstride + a.r_coff + n0, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = r[j] + v[j];
      }
      store4((float*)a.dst + (size_t)p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// LDS bytes of conv_fast_kernel for an op: the K-step table (+ the split-K reduction buffer).
inline size_t fast_lds(int k_steps, int nnt, int npt, int kw) {
  const size_t t = ((size_t)k_steps * 4 * 8 + 15) & ~(size_t)15;
  return t + (kw > 1 ? (size_t)4 * nnt * npt * 64 * 16 : 0);
}

// ---------------------------------------------------------------- LetterBox resize
// LetterBox (data/augment.py:1698-1729) when the frame is not at the network scale: cv2.resize
// INTER_LINEAR of the uint8 BGR frame, restated from OpenCV 4.x's fixed-point path (see
// letterbox.py for the rules), centred in an in_w x in_h canvas of 114.  One thread per output
// pixel; the first conv then reads this canvas as its frame.
struct LboxArgs {
  const unsigned char* src;  // [B][fh][fw][3]
  unsigned char* dst;        // [B][in_h][in_w][3]
  int fh, fw, in_h, in_w, top, left, rs_w, rs_h, mode, vec_end;
  const int* xofs;           // [rs_w] source column (clamped)
  const int* yofs;           // [rs_h] source row (unclamped: the fetch clips)
  const short2* xw;          // [rs_w] fixed-point weights (sum 2048)
  const short2* yw;          // [rs_h]
};

__global__ void __launch_bounds__(256) letterbox_kernel(LboxArgs a, int B) {
  const long n = (long)B * a.in_h * a.in_w;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int x = (int)(i % a.in_w);
    const long t = i / a.in_w;
    const int y = (int)(t % a.in_h), b = (int)(t / a.in_h);
    int o[3] = {114, 114, 114};
    const int ry = y - a.top, rx = x - a.left;
    if (ry >= 0 && ry < a.rs_h && rx >= 0 && rx < a.rs_w) {
      const unsigned char* S = a.src + (size_t)b * a.fh * a.fw * 3;
      if (a.mode == 2) {  // exact 2x: INTER_AREA fast path, (a + b + c + d + 2) >> 2
        const unsigned char* p0 = S + ((size_t)(2 * ry) * a.fw + 2 * rx) * 3;
        const unsigned char* p1 = p0 + (size_t)a.fw * 3;
        for (int c = 0; c < 3; ++c) o[c] = (p0[c] + p0[3 + c] + p1[c] + p1[3 + c] + 2) >> 2;
      } else {
        const int sx = a.xofs[rx], sx1 = sx + 1 < a.fw ? sx + 1 : a.fw - 1;
        const short2 aw = a.xw[rx], bw = a.yw[ry];
        const int sy = a.yofs[ry];
        const int r0 = sy < 0 ? 0 : (sy > a.fh - 1 ? a.fh - 1 : sy);
        const int r1 = sy + 1 < 0 ? 0 : (sy + 1 > a.fh - 1 ? a.fh - 1 : sy + 1);
        const unsigned char* R0 = S + (size_t)r0 * a.fw * 3;
        const unsigned char* R1 = S + (size_t)r1 * a.fw * 3;
        for (int c = 0; c < 3; ++c) {
          const int d0 = R0[sx * 3 + c] * aw.x + R0[sx1 * 3 + c] * aw.y;  // horizontal pass (exact)
          const int d1 = R1[sx * 3 + c] * aw.x + R1[sx1 * 3 + c] * aw.y;
          int v;
          if (rx * 3 + c < a.vec_end) {  // VResizeLinearVec_32s8u: v_mul_hi of (D >> 4), then >> 2
            const int t0 = ((int)(short)(d0 >> 4) * (int)bw.x) >> 16;
            const int t1 = ((int)(short)(d1 >> 4) * (int)bw.y) >> 16;
            v = (t0 + t1 + 2) >> 2;
          } else {  // FixedPtCast<int, uchar, 22>
            v = (d0 * bw.x + d1 * bw.y + (1 << 21)) >> 22;
          }
          o[c] = v < 0 ? 0 : (v > 255 ? 255 : v);
        }
      }
    }
    unsigned char* q = a.dst + (size_t)i * 3;
    q[0] = (unsigned char)o[0];
    q[1] = (unsigned char)o[1];
    q[2] = (unsigned char)o[2];
  }
}

// ---------------------------------------------------------------- first conv from uint8 frames

struct InputArgs {
  const unsigned char* frames;  // [B][fh][fw][3] BGR
  int fh, fw, pad_top, pad_left;
  int in_h, in_w, out_h, out_w, stride, ksize, pad, M;
  const float* w;  // [cout][3][k][k] fused weights (RGB channel order), f32
  const float* b;  // [cout]
  int cout;        // physical output channels (multiple of 8), weights zero-padded
  void* dst;
  int d_cstride, d_coff;
  int xcd;
};

template <class Tr>
__global__ void __launch_bounds__(256) conv_input_kernel(InputArgs a) {
  // One workgroup = a 16x16 output tile.  The frame patch it reads (3x3 taps, stride <= 2) is
  // staged once into LDS as RGB floats already divided by 255 (BGR->RGB, im /= 255, LetterBox
  // value 114 outside the frame, conv zero padding outside the network input); each thread then
  // computes one output pixel.  Weights, bias and the exact v/255 table live in LDS too:
  // loaded per output channel from global they would be a chain of dependent VMEM round trips.
  using T = typename Tr::T;
  constexpr int TI = 15 * 2 + 3;  // patch edge for stride 2 (also covers stride 1)
  __shared__ float xs[3][TI][TI + 1];
  __shared__ float ws[kInputCoutMax * 27];
  __shared__ float bs[kInputCoutMax];
  __shared__ float lut[256];
  const int tiles_x = (a.out_w + 15) / 16, tiles_y = (a.out_h + 15) / 16;
  int t = xcd_block(a.xcd).x;
  const int b = t / (tiles_x * tiles_y);
  t -= b * tiles_x * tiles_y;
  const int ty0 = (t / tiles_x) * 16, tx0 = (t % tiles_x) * 16;
  const int s = a.stride;
  const int ti = 15 * s + 3;
  const int iy0 = ty0 * s - a.pad, ix0 = tx0 * s - a.pad;
  const unsigned char* fr = a.frames + (size_t)b * a.fh * a.fw * 3;
  lut[threadIdx.x] = (float)threadIdx.x / 255.0f;  // im /= 255 (exact division, as torch)
  for (int i = threadIdx.x; i < a.cout * 27; i += 256) ws[i] = a.w[i];
  if (threadIdx.x < a.cout) bs[threadIdx.x] = a.b[threadIdx.x];
  __syncthreads();
  for (int i = threadIdx.x; i < ti * ti; i += 256) {
    const int ry = i / ti, rx = i - ry * ti;
    const int iy = iy0 + ry, ix = ix0 + rx;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
      const int fy = iy - a.pad_top, fx = ix - a.pad_left;
      if (fy >= 0 && fy < a.fh && fx >= 0 && fx < a.fw) {
        const unsigned char* px = fr + ((size_t)fy * a.fw + fx) * 3;
        v0 = lut[px[2]];
        v1 = lut[px[1]];
        v2 = lut[px[0]];
      } else {
        v0 = v1 = v2 = lut[114];
      }
    }
    xs[0][ry][rx] = v0;
    xs[1][ry][rx] = v1;
    xs[2][ry][rx] = v2;
  }
  __syncthreads();
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  const int oy = ty0 + ty, ox = tx0 + tx;
  if (oy >= a.out_h || ox >= a.out_w) return;
  float x[27];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) x[c * 9 + ky * 3 + kx] = xs[c][ty * s + ky][tx * s + kx];
  const size_t p = ((size_t)b * a.out_h + oy) * a.out_w + ox;
  T* out = (T*)a.dst + p * a.d_cstride + a.d_coff;
  const float* W = ws;
  const float* Bb = bs;
  for (int o = 0; o < a.cout; o += 4) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* w = W + (o + j) * 27;
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 27; ++q) acc += w[q] * x[q];
      v[j] = silu<Tr::kExact>(acc + Bb[o + j]);
    }
    store4(out + o, v);
  }
}

// bf16 production variant of the first conv on MFMA.  K = 3 channels x 9 taps = 27 (padded to
// one 16x16x32 K step), N = cout (<= 32: two 16-row tiles).  The uint8 pixel values are exact
// in bf16, so the staged patch holds raw values (LetterBox fill 114, conv zero padding 0) and
// the 1/255 of `im /= 255` is folded into the weights (the only rounding is the bf16 weight,
// as for every other layer).  A workgroup = a 16x16 output tile; wave w computes rows
// 4w..4w+3: per row one B fragment (8 LDS reads per lane) and two MFMAs.
template <class Tr>
__global__ void __launch_bounds__(256) conv_input_mfma_kernel(InputArgs a) {
  constexpr int TI = 15 * 2 + 3;
  constexpr int TP = TI + 1;
  __shared__ float xs[3][TI][TP];
  __shared__ float ws[32 * 27];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const int tiles_x = (a.out_w + 15) / 16, tiles_y = (a.out_h + 15) / 16;
  int t = xcd_block(a.xcd).x;
  const int b = t / (tiles_x * tiles_y);
  t -= b * tiles_x * tiles_y;
  const int ty0 = (t / tiles_x) * 16, tx0 = (t % tiles_x) * 16;
  const int s = a.stride;
  const int ti = 15 * s + 3;
  const int iy0 = ty0 * s - a.pad, ix0 = tx0 * s - a.pad;
  const unsigned char* fr = a.frames + (size_t)b * a.fh * a.fw * 3;
  for (int i = tid; i < 32 * 27; i += 256) ws[i] = i < a.cout * 27 ? a.w[i] * (1.0f / 255.0f) : 0.f;
  for (int i = tid; i < ti * ti; i += 256) {
    const int ry = i / ti, rx = i - ry * ti;
    const int iy = iy0 + ry, ix = ix0 + rx;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
      const int fy = iy - a.pad_top, fx = ix - a.pad_left;
      if (fy >= 0 && fy < a.fh && fx >= 0 && fx < a.fw) {
        const unsigned char* px = fr + ((size_t)fy * a.fw + fx) * 3;
        v0 = (float)px[2];  // BGR -> RGB
        v1 = (float)px[1];
        v2 = (float)px[0];
      } else {
        v0 = v1 = v2 = 114.f;
      }
    }
    xs[0][ry][rx] = v0;
    xs[1][ry][rx] = v1;
    xs[2][ry][rx] = v2;
  }
  __syncthreads();
  // A fragments: rows = output channels nt*16 + col, K = kg*8 + e (k = c*9 + ky*3 + kx); the
  // fp16 build rounds them to binary16 and runs the f16 MFMA (uint8 values are exact in both)
  using E = std::conditional_t<std::is_same<Tr, F16>::value, _Float16, __bf16>;
  typedef E e8 __attribute__((ext_vector_type(8)));
  e8 wa[2];
  int xoff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = kg * 8 + e;
    wa[0][e] = (E)(k < 27 ? ws[col * 27 + k] : 0.f);
    wa[1][e] = (E)(k < 27 ? ws[(16 + col) * 27 + k] : 0.f);
    const int c = k / 9, tap = k - c * 9, ky = tap / 3, kx = tap - ky * 3;
    xoff[e] = k < 27 ? (c * TI + ky) * TP + col * s + kx : -1;
  }
  const float* xsf = &xs[0][0][0];
  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int roff = (wave * 4 + r) * s * TP;
    e8 xb;
#pragma unroll
    for (int e = 0; e < 8; ++e) xb[e] = (E)(xoff[e] >= 0 ? xsf[xoff[e] + roff] : 0.f);
    if constexpr (std::is_same<Tr, F16>::value) {
      acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[0], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[1], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    } else {
      acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
  }
  const int ox = tx0 + col;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
    const float4 bb = *(const float4*)(a.b + n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oy = ty0 + wave * 4 + r;
      if (oy >= a.out_h || ox >= a.out_w) continue;
      float v[4] = {acc[nt][r][0] + bb.x, acc[nt][r][1] + bb.y, acc[nt][r][2] + bb.z, acc[nt][r][3] + bb.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = silu<false>(v[j]);
      const size_t p = ((size_t)b * a.out_h + oy) * a.out_w + ox;
      store4((typename Tr::T*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// fp32 parity build of the first conv on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32, an fmaf
// chain in f32).  The staged patch holds v / 255 (the reference's `im /= 255`, exact f32
// division, as conv_input_kernel's table), the weights stay the fused f32 weights, so every
// product and sum is f32 as in the reference's fp32 conv (summation order differs within
// rounding).  K = 27 is padded to 28 = seven K=4 MFMAs; MFMA j takes k = 4j + (lane >> 4) from
// both operands.  A workgroup = a 16x16 output tile; wave w computes rows 4w..4w+3, two
// 16-channel output tiles (cout <= 32).  Replaces conv_input_kernel's 27 LDS weight reads per
// FMA (VALU + LDS issue bound).
__global__ void __launch_bounds__(256) conv_input_f32mfma_kernel(InputArgs a) {
  constexpr int TI = 15 * 2 + 3;
  constexpr int TP = TI + 1;
  __shared__ float xs[3][TI][TP];
  __shared__ float lut[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const int tiles_x = (a.out_w + 15) / 16, tiles_y = (a.out_h + 15) / 16;
  int t = xcd_block(a.xcd).x;
  const int b = t / (tiles_x * tiles_y);
  t -= b * tiles_x * tiles_y;
  const int ty0 = (t / tiles_x) * 16, tx0 = (t % tiles_x) * 16;
  const int s = a.stride;
  const int ti = 15 * s + 3;
  const int iy0 = ty0 * s - a.pad, ix0 = tx0 * s - a.pad;
  const unsigned char* fr = a.frames + (size_t)b * a.fh * a.fw * 3;
  lut[tid] = (float)tid / 255.0f;  // im /= 255 (exact division, as torch)
  // A fragments straight from global (each lane 14 floats, read once per workgroup)
  float wa[2][7];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int k = 4 * j + kg, o = nt * 16 + col;
      wa[nt][j] = (k < 27 && o < a.cout) ? a.w[o * 27 + k] : 0.f;
    }
  __syncthreads();
  for (int i = tid; i < ti * ti; i += 256) {
    const int ry = i / ti, rx = i - ry * ti;
    const int iy = iy0 + ry, ix = ix0 + rx;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
      const int fy = iy - a.pad_top, fx = ix - a.pad_left;
      if (fy >= 0 && fy < a.fh && fx >= 0 && fx < a.fw) {
        const unsigned char* px = fr + ((size_t)fy * a.fw + fx) * 3;
        v0 = lut[px[2]];  // BGR -> RGB
        v1 = lut[px[1]];
        v2 = lut[px[0]];
      } else {
        v0 = v1 = v2 = lut[114];
      }
    }
    xs[0][ry][rx] = v0;
    xs[1][ry][rx] = v1;
    xs[2][ry][rx] = v2;
  }
  __syncthreads();
  int xoff[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int k = 4 * j + kg;
    const int c = k / 9, tap = k - c * 9, ky = tap / 3, kx = tap - ky * 3;
    xoff[j] = k < 27 ? (c * TI + ky) * TP + col * s + kx : -1;
  }
  const float* xsf = &xs[0][0][0];
  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int roff = (wave * 4 + r) * s * TP;
    acc[0][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const float xv = xoff[j] >= 0 ? xsf[xoff[j] + roff] : 0.f;
      acc[0][r] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[0][j], xv, acc[0][r], 0, 0, 0);
      acc[1][r] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[1][j], xv, acc[1][r], 0, 0, 0);
    }
  }
  const int ox = tx0 + col;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n0 = nt * 16 + kg * 4;
    if (n0 >= a.cout) continue;
    const float4 bb = *(const float4*)(a.b + n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oy = ty0 + wave * 4 + r;
      if (oy >= a.out_h || ox >= a.out_w) continue;
      float v[4] = {acc[nt][r][0] + bb.x, acc[nt][r][1] + bb.y, acc[nt][r][2] + bb.z, acc[nt][r][3] + bb.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = silu<true>(v[j]);
      const size_t p = ((size_t)b * a.out_h + oy) * a.out_w + ox;
      store4((float*)a.dst + p * a.d_cstride + a.d_coff + n0, v);
    }
  }
}

// ---------------------------------------------------------------- SPPF pooling
// slices 1..3 of the SPPF concat buffer = max over 5x5 / 9x9 / 13x13 windows of slice 0
// (MaxPool2d(5,1,2) applied 1/2/3 times; padding never wins a max).
template <class Tr>
__global__ void __launch_bounds__(256) sppf_pool_kernel(void* buf, int cstride, int coff, int C, int H, int W, int M) {
  using T = typename Tr::T;
  const int per = C / 4;  // 4-channel groups
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * per) return;
  const int p = i / per, g = i - p * per;
  const int hw = H * W, b = p / hw, r = p - b * hw, y = r / W, x = r - y * W;
  T* base = (T*)buf + (size_t)b * hw * cstride + coff + g * 4;
  float m5[4], m9[4], m13[4];
  for (int j = 0; j < 4; ++j) m5[j] = m9[j] = m13[j] = -INFINITY;
  for (int dy = -6; dy <= 6; ++dy) {
    const int yy = y + dy;
    if (yy < 0 || yy >= H) continue;
    for (int dx = -6; dx <= 6; ++dx) {
      const int xx = x + dx;
      if (xx < 0 || xx >= W) continue;
      float v[4];
      load4(base + ((size_t)yy * W + xx) * cstride, v);
      const int ad = max(abs(dy), abs(dx));
      for (int j = 0; j < 4; ++j) {
        m13[j] = fmaxf(m13[j], v[j]);
        if (ad <= 4) m9[j] = fmaxf(m9[j], v[j]);
        if (ad <= 2) m5[j] = fmaxf(m5[j], v[j]);
      }
    }
  }
  T* o = base + ((size_t)y * W + x) * cstride;
  store4(o + C, m5);
  store4(o + 2 * C, m9);
  store4(o + 3 * C, m13);
}

// One workgroup = one image x CPG channels (8, or 4 for planes of up to 2048 pixels, e.g. the P5
// map 32 x 40 at imgsz 1280): the plane is staged in LDS as f32, the 5/9/13-wide row maxima are
// formed, then the column maxima (square windows are separable), so each input element is read
// from HBM once instead of 169 times.  max is exact in any precision.
constexpr int kSppfLdsMaxHW = 1024;      // 8 channels per workgroup
constexpr int kSppfLdsMaxHW4 = 2048;     // 4 channels per workgroup
constexpr size_t kSppfLdsBytes = 128 * 1024;
template <class Tr, int CPG>
__global__ void __launch_bounds__(256) sppf_lds_kernel(void* buf, int cstride, int coff, int C, int H, int W) {
  using T = typename Tr::T;
  constexpr int IPP = CPG / 4;  // 4-channel items per pixel
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int HW = H * W, cg = C / CPG;
  const int b = blockIdx.x / cg, c0 = (blockIdx.x - b * cg) * CPG;
  float* x = (float*)smem;  // [HW][CPG]
  float* r5 = x + HW * CPG;
  float* r9 = r5 + HW * CPG;
  float* r13 = r9 + HW * CPG;
  T* base = (T*)buf + (size_t)b * HW * cstride + coff + c0;
  for (int i = threadIdx.x; i < HW * IPP; i += blockDim.x) {
    const int p = i / IPP, h = (i % IPP) * 4;
    float v[4];
    load4(base + (size_t)p * cstride + h, v);
    *(float4*)(x + p * CPG + h) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __syncthreads();
  // Window indices are clamped to the plane instead of skipped: a clamped index is the border
  // element, which lies inside the same window, and max is idempotent -- so the 13 reads of a
  // window are branch-free and issue back to back.
  for (int i = threadIdx.x; i < HW * CPG; i += blockDim.x) {
    const int p = i / CPG, c = i % CPG, yy = p / W, xx = p - yy * W;
    const float* row = x + yy * W * CPG + c;
    float v[13];
#pragma unroll
    for (int d = 0; d < 13; ++d) {
      const int u = min(max(xx + d - 6, 0), W - 1);
      v[d] = row[u * CPG];
    }
    float m5 = fmaxf(fmaxf(fmaxf(v[4], v[5]), fmaxf(v[6], v[7])), v[8]);
    float m9 = fmaxf(fmaxf(m5, fmaxf(v[2], v[3])), fmaxf(v[9], v[10]));
    float m13 = fmaxf(fmaxf(m9, fmaxf(v[0], v[1])), fmaxf(v[11], v[12]));
    r5[i] = m5;
    r9[i] = m9;
    r13[i] = m13;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HW * IPP; i += blockDim.x) {
    const int p = i / IPP, h = (i % IPP) * 4, yy = p / W, xx = p - yy * W;
    float m5[4], m9[4], m13[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m5[j] = m9[j] = m13[j] = -INFINITY;
#pragma unroll
    for (int d = 0; d < 13; ++d) {
      const int q = (min(max(yy + d - 6, 0), H - 1) * W + xx) * CPG + h;
      const float4 a13 = *(const float4*)(r13 + q);
      m13[0] = fmaxf(m13[0], a13.x); m13[1] = fmaxf(m13[1], a13.y);
      m13[2] = fmaxf(m13[2], a13.z); m13[3] = fmaxf(m13[3], a13.w);
      if (d >= 2 && d <= 10) {
        const float4 a9 = *(const float4*)(r9 + q);
        m9[0] = fmaxf(m9[0], a9.x); m9[1] = fmaxf(m9[1], a9.y);
        m9[2] = fmaxf(m9[2], a9.z); m9[3] = fmaxf(m9[3], a9.w);
      }
      if (d >= 4 && d <= 8) {
        const float4 a5 = *(const float4*)(r5 + q);
        m5[0] = fmaxf(m5[0], a5.x); m5[1] = fmaxf(m5[1], a5.y);
        m5[2] = fmaxf(m5[2], a5.z); m5[3] = fmaxf(m5[3], a5.w);
      }
    }
    T* o = base + (size_t)p * cstride + h;
    store4(o + C, m5);
    store4(o + 2 * C, m9);
    store4(o + 3 * C, m13);
  }
}

// ---------------------------------------------------------------- Detect level
struct DetArgs {
  View src;          // second-conv output: box features at src.coff, class features at cls_off
  int cls_off, cls_ch;
  const uint4* wpk;  // box 1x1 packed [4][k_steps][64]
  const float* bias; // [64]
  int k_steps;
  const float* wc;   // [cls_ch] then bias
  int stride, anchor_off, M;
  float conf;
  float* cand;       // [B][cap][6]
  int* cand_count;   // [B]
  int cap;
};

template <class Tr>
__global__ void __launch_bounds__(256) detect_kernel(DetArgs a) {
  using T = typename Tr::T;
  constexpr int EPL = Tr::EPL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane >> 4, col = lane & 15;
  const int pbase = (blockIdx.x * 4 + wave) * 16;
  if (pbase >= a.M) return;
  const int p = pbase + col;
  const bool valid = p < a.M;
  const int pp = valid ? p : a.M - 1;
  const T* px = (const T*)a.src.p + (size_t)pp * a.src.cstride;
  // box logits: 4 tiles (l, t, r, b) x 16 bins
  f32x4 acc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < a.k_steps; ++ks) {
    const int kel = ks * 4 * EPL + kg * EPL;
    const uint4 x = *(const uint4*)(px + a.src.coff + kel);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[s] = mma<Tr>(a.wpk[((size_t)s * a.k_steps + ks) * 64 + lane], x, acc[s]);
  }
  // class logit: dot product over the class features, split across the 4 lane groups
  float cl = 0.f;
  for (int c = kg * 4; c < a.cls_ch; c += 16) {
    float v[4];
    load4(px + a.cls_off + c, v);
    cl += a.wc[c] * v[0] + a.wc[c + 1] * v[1] + a.wc[c + 2] * v[2] + a.wc[c + 3] * v[3];
  }
  cl += __shfl_xor(cl, 16);
  cl += __shfl_xor(cl, 32);
  cl += a.wc[a.cls_ch];
  // DFL: softmax over 16 bins (4 per lane, 4 lane groups) -> expectation
  float d[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float v[4];
    const float4 bb = *(const float4*)(a.bias + s * 16 + kg * 4);
    const float4 sc = dq4<Tr>(a.bias, 4, s * 16 + kg * 4);
    v[0] = acc[s][0] * sc.x + bb.x;
    v[1] = acc[s][1] * sc.y + bb.y;
    v[2] = acc[s][2] * sc.z + bb.z;
    v[3] = acc[s][3] * sc.w + bb.w;
    float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float e[4], sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e[j] = Tr::kExact ? expf(v[j] - m) : __expf(v[j] - m);
      sum += e[j];
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    float ex = 0.f;
    const float rs = Tr::kExact ? 0.f : __builtin_amdgcn_rcpf(sum);  // bf16 build: v_rcp
#pragma unroll
    for (int j = 0; j < 4; ++j) ex += (float)(kg * 4 + j) * (Tr::kExact ? e[j] / sum : e[j] * rs);
    ex += __shfl_xor(ex, 16);
    ex += __shfl_xor(ex, 32);
    d[s] = ex;
  }
  if (kg != 0 || !valid) return;
  const float score = 1.0f / (1.0f + expf(-cl));
  if (!(score > a.conf)) return;
  const int hw = a.src.h * a.src.w;
  const int b = p / hw, r = p - b * hw, gy = r / a.src.w, gx = r - gy * a.src.w;
  const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f;
  // dist2bbox (xywh) * stride, then xywh2xyxy
  const float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
  const float st = (float)a.stride;
  const float cx = ((x1 + x2) / 2.0f) * st, cy = ((y1 + y2) / 2.0f) * st;
  const float w = (x2 - x1) * st, h = (y2 - y1) * st;
  const float hw2 = w / 2.0f, hh2 = h / 2.0f;
  YK_SC(&a.cand_count[b], 4, 10);
  const int slot = atomicAdd(&a.cand_count[b], 1);
  if (slot >= a.cap) return;
  float* c = a.cand + ((size_t)b * a.cap + slot) * 6;
  YK_SC(c, 24, 11);
  c[0] = cx - hw2;
  c[1] = cy - hh2;
  c[2] = cx + hw2;
  c[3] = cy + hh2;
  c[4] = score;
  c[5] = __int_as_float(a.anchor_off + r);
}

// ---------------------------------------------------------------- NMS + scale/clip
// IoU decisions must round like the reference's separate torch ops (inter = w * h rounded, then
// (area_i + area_j) - inter): no a*b+c contraction anywhere in the NMS code.
#pragma clang fp contract(off)
constexpr int NMS_NT = 512;
constexpr int NMS_LDS_N = 2048;   // candidates sorted in LDS; more -> global scratch
constexpr int NMS_MASK_N = 512;   // bitmask suppression in LDS up to this many candidates
constexpr size_t NMS_OFF_BOX = (size_t)NMS_LDS_N * 8;
constexpr size_t NMS_OFF_REM = NMS_OFF_BOX + (size_t)NMS_LDS_N * 20;
constexpr size_t NMS_OFF_MISC = NMS_OFF_REM + NMS_LDS_N;
constexpr size_t NMS_OFF_KEEP = NMS_OFF_MISC + 64;
constexpr size_t NMS_OFF_MASK = NMS_OFF_KEEP + (size_t)NMS_LDS_N * 4;
constexpr int NMS_W = NMS_MASK_N / 64;
constexpr size_t NMS_LDS = NMS_OFF_MASK + (size_t)NMS_MASK_N * NMS_W * 8 * 2;

struct NmsArgs {
  const float* cand;
  int* cand_count;
  int cap, max_nms;
  int* slot_of;                 // [B][n_anchors] anchor -> candidate slot
  unsigned long long* gkeys;    // [B][pow2 >= cap]
  float* gbox;                  // [B][cap][5]
  unsigned char* gflag;         // [B][cap]
  int n_anchors, key_cap;
  float iou;
  int max_det;
  float* dets;                  // [B][max_det][6]
  int* counts;
  float pad_x, pad_y, gain, clip_w, clip_h;
  int dbg;  // YK_NMS_DBG=1: phase times (us, s_memrealtime) in dets[b][max_det-1] (diagnostics only)
  int* keep_out;  // [B][max_det] kept rows' candidate ids (the anchor field), or NULL
  int* stat;      // [2] images that took the :291-296 early exit with boxes left, images processed
  int* err;       // device view of a host-mapped word: bit 0 = a candidate row carried an anchor
                  // outside [0, n_anchors) (the image's count is then 0); read by the host API
};

// Sort key of a candidate: ascending key = score descending (every NaN first whatever its sign
// bit, as torch's sort puts them; -0 == +0), then candidate id ascending -- the stable order of
// scores.sort(descending=True)
__device__ __forceinline__ unsigned long long nms_key(float score, int id) {
  unsigned u = __float_as_uint(score);
  if (u == 0x80000000u) u = 0u;
  if (score != score) u = 0x7fc00000u;  // canonical positive NaN: above +inf in the key order
  const unsigned m = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving float -> uint
  return ((unsigned long long)(~m) << 32) | (unsigned)id;
}
__device__ __forceinline__ void nms_flag_error(int* err) {
  __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void bitonic_sort(unsigned long long* k, int n2) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < (n2 >> 1); i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = k[lo], b = k[hi];
        if ((a > b) == up) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// the same network carrying a 32-bit payload (the candidate's slot) with each key
__device__ __forceinline__ void bitonic_sort_kv(unsigned long long* k, int* pay, int n2) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < (n2 >> 1); i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = k[lo], b = k[hi];
        if ((a > b) == up) {
          const int pa = pay[lo];
          k[lo] = b;
          k[hi] = a;
          pay[lo] = pay[hi];
          pay[hi] = pa;
        }
      }
      __syncthreads();
    }
  }
}

// bits of word `w` (candidates w*64 .. w*64+63) that lie strictly after candidate i
__device__ __forceinline__ unsigned long long after_mask(int w, int i) {
  const int base = w * 64;
  if (i < base) return ~0ull;
  if (i >= base + 63) return 0ull;
  return ~0ull << (i - base + 1);
}

// The greedy walk over precomputed masks (one wave).  Both mask rows of the picked box are read
// together, so an iteration waits on one LDS round trip.
__device__ int nms_walk(int n, int max_det, const unsigned long long* sup, const unsigned long long* ovl, int* keep,
                        int* k_out, int* early) {
  const int W = (n + 63) / 64;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned long long R = ~0ull;  // removed (or beyond n)
    if (lane < W) {
      const int rem = n - lane * 64;
      R = rem >= 64 ? 0ull : ~0ull << rem;
    }
    int k = 0, i = -1;
    while (k < max_det) {
      const unsigned long long cand = lane < W ? (~R & after_mask(lane, i)) : 0ull;
      const unsigned long long bal = __ballot(cand != 0ull);
      if (bal == 0ull) break;
      const int fl = __ffsll((long long)bal) - 1;
      // fl is wave-uniform (from a ballot): two v_readlane instead of an LDS permute
      const unsigned long long word = ((unsigned long long)__builtin_amdgcn_readlane((unsigned)(cand >> 32), fl) << 32) |
                                      __builtin_amdgcn_readlane((unsigned)cand, fl);
      i = fl * 64 + __ffsll((long long)word) - 1;
      const unsigned long long orow = lane < W ? ovl[i * NMS_W + lane] : 0ull;
      const unsigned long long srow = lane < W ? sup[i * NMS_W + lane] : 0ull;
      if (lane == 0) keep[k] = i;
      ++k;
      if (k >= max_det) break;
      const unsigned long long o = orow & ~R;
      if (__ballot(o != 0ull) == 0ull) {
        // keep every remaining candidate after i, in order
        const unsigned long long rem = lane < W ? (~R & after_mask(lane, i)) : 0ull;
        const int c = __popcll(rem);
        int incl = c;
        for (int d = 1; d < 64; d <<= 1) {
          const int v = __shfl_up(incl, d);
          if (lane >= d) incl += v;
        }
        int r = k + incl - c;
        unsigned long long bits = rem;
        while (bits) {
          const int bpos = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          if (r < max_det) keep[r] = lane * 64 + bpos;
          ++r;
        }
        const int total = __shfl(incl, 63);
        if (lane == 0 && total > 0) *early = 1;
        k = k + total < max_det ? k + total : max_det;
        break;
      }
      R |= srow;
    }
    if (lane == 0) *k_out = k;
  }
  __syncthreads();
  return *k_out;
}

// TorchNMS.nms on one image's sorted candidates as bitmasks (utils/nms.py:237-304):
// sup[i] = later boxes with !(iou <= thr), ovl[i] = later boxes with inter != 0.  One wave then
// walks the kept boxes: next kept = first candidate not yet removed; if it overlaps no remaining
// box, every remaining box is kept (the :291-296 early exit) and the walk ends.
__device__ int nms_bitmask(const float* box, int n, float thr, int max_det, unsigned long long* sup,
                           unsigned long long* ovl, int* keep, int* k_out, int* early) {
  const int W = (n + 63) / 64;
  for (int job = threadIdx.x; job < n * W; job += blockDim.x) {
    const int i = job / W, w = job - i * W;
    unsigned long long sm = 0, om = 0;
    if (w * 64 + 63 > i) {
      const float bx1 = box[i * 5], by1 = box[i * 5 + 1], bx2 = box[i * 5 + 2], by2 = box[i * 5 + 3],
                  ba = box[i * 5 + 4];
      const int j0 = w * 64;
      for (int jj = 0; jj < 64; ++jj) {
        const int j = j0 + jj;
        if (j <= i || j >= n) continue;
        const float ww = fmaxf(fminf(bx2, box[j * 5 + 2]) - fmaxf(bx1, box[j * 5]), 0.f);
        const float hh = fmaxf(fminf(by2, box[j * 5 + 3]) - fmaxf(by1, box[j * 5 + 1]), 0.f);
        const float inter = ww * hh;
        const float iou = inter / (ba + box[j * 5 + 4] - inter);
        if (inter != 0.f) om |= 1ull << jj;
        if (!(iou <= thr)) sm |= 1ull << jj;
      }
    }
    sup[i * NMS_W + w] = sm;
    ovl[i * NMS_W + w] = om;
  }
  __syncthreads();
  return nms_walk(n, max_det, sup, ovl, keep, k_out, early);
}

// TorchNMS.nms (utils/nms.py:237-304) on up to NMS_GW*64 sorted candidates by ONE wave, with no
// LDS in the loop: lane l holds columns w*64 + l (box, area, alive flag) in registers.  Each
// iteration keeps the first alive column i (ballots), fetches box i by v_readlane, and tests it
// against every alive column: all intersections zero -> keep every alive column in order and stop
// (:291-296); otherwise drop the columns with !(iou <= thr).  Work = kept x n pairs instead of the
// n^2/2 of the mask build, on one SIMD.
constexpr int NMS_GW = 4;
template <int GW>
__device__ int nms_greedy_wave(const float4* bx, const float* ar, int n, float thr, int max_det, int* keep,
                               int* k_out, int* early) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int W = (n + 63) / 64;
    float4 bj[GW];
    float aj[GW];
    bool al[GW];
#pragma unroll
    for (int w = 0; w < GW; ++w) {
      const int j = w * 64 + lane;
      al[w] = j < n;
      bj[w] = al[w] ? bx[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      aj[w] = al[w] ? ar[j] : 0.f;
    }
    int k = 0;
    while (k < max_det) {
      int i = -1;
#pragma unroll
      for (int w = 0; w < GW; ++w) {
        const unsigned long long b = __ballot(al[w]);
        if (i < 0 && b != 0ull) i = w * 64 + __ffsll((long long)b) - 1;
      }
      if (i < 0) break;
      if (lane == 0) keep[k] = i;
      ++k;
      if (k >= max_det) break;
      const int wi = i >> 6, li = i & 63;
      float4 bi = make_float4(0.f, 0.f, 0.f, 0.f);
      float ai = 0.f;
#pragma unroll
      for (int w = 0; w < GW; ++w)
        if (w == wi) {
          bi.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bj[w].x), li));
          bi.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bj[w].y), li));
          bi.z = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bj[w].z), li));
          bi.w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bj[w].w), li));
          ai = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(aj[w]), li));
          if (lane == li) al[w] = false;
        }
      bool any = false;
      bool sup[GW];
#pragma unroll
      for (int w = 0; w < GW; ++w) {
        sup[w] = false;
        if (w < W && al[w]) {
          const float ww = fmaxf(fminf(bi.z, bj[w].z) - fmaxf(bi.x, bj[w].x), 0.f);
          const float hh = fmaxf(fminf(bi.w, bj[w].w) - fmaxf(bi.y, bj[w].y), 0.f);
          const float inter = ww * hh;
          any |= inter != 0.f;
          const float iou = inter / (ai + aj[w] - inter);
          sup[w] = !(iou <= thr);
        }
      }
      if (__ballot(any) == 0ull) {
        // keep every alive column, in order
        int base = k;
#pragma unroll
        for (int w = 0; w < GW; ++w) {
          const unsigned long long b = __ballot(al[w]);
          const int r = base + __popcll(b & ((1ull << lane) - 1ull));
          if (al[w] && r < max_det) keep[r] = w * 64 + lane;
          base += __popcll(b);
        }
        if (lane == 0 && base > k) *early = 1;
        k = base < max_det ? base : max_det;
        break;
      }
#pragma unroll
      for (int w = 0; w < GW; ++w) al[w] = al[w] && !sup[w];
    }
    if (lane == 0) *k_out = k;
  }
  __syncthreads();
  return *k_out;
}

// Candidate counts up to NMS_MASK_N (the common case): the rows are read from HBM once, in one
// coalesced pass, and everything after -- sort (key + slot payload), box gather, masks, walk,
// output rows -- works on LDS copies.  Same arithmetic as the general path below.
constexpr size_t NS_PAY = (size_t)NMS_MASK_N * 8;
constexpr size_t NS_STG = NS_PAY + (size_t)NMS_MASK_N * 8;  // slot by input index, then by sorted position
constexpr size_t NS_BX = NS_STG + (size_t)NMS_MASK_N * 20;
constexpr size_t NS_AR = NS_BX + (size_t)NMS_MASK_N * 16;
constexpr size_t NS_KEEP = NS_AR + (size_t)NMS_MASK_N * 4;
constexpr size_t NS_MISC = NS_KEEP + (size_t)NMS_MASK_N * 4;
constexpr size_t NS_MASK = NS_MISC + 64;
static_assert(NS_BX % 16 == 0 && NS_MASK % 8 == 0, "NMS LDS alignment");
static_assert(NS_MASK + (size_t)NMS_MASK_N * NMS_W * 16 <= NMS_LDS, "NMS small-path LDS");

__device__ void nms_small(const NmsArgs& a, int b, int n, unsigned char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* cand = a.cand + (size_t)b * a.cap * 6;
  unsigned long long* keys = (unsigned long long*)smem;
  int* pay = (int*)(smem + NS_PAY);
  float* stg = (float*)(smem + NS_STG);
  float4* bx = (float4*)(smem + NS_BX);
  float* ar = (float*)(smem + NS_AR);
  int* keep = (int*)(smem + NS_KEEP);
  int* misc = (int*)(smem + NS_MISC);
  unsigned long long* sup = (unsigned long long*)(smem + NS_MASK);
  unsigned long long* ovl = sup + NMS_MASK_N * NMS_W;
  unsigned long long t[6], c0 = 0;
  if (a.dbg) {
    t[0] = __builtin_amdgcn_s_memrealtime();
    c0 = __builtin_amdgcn_s_memtime();
  }
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  if (tid < 16) misc[tid] = 0;  // [13] bad anchor, [14] early exit
  __syncthreads();
  for (int i = tid; i < n2; i += NMS_NT) {
    unsigned long long k = ~0ull;
    if (i < n) {
      const float2* c = (const float2*)(cand + (size_t)i * 6);  // rows are 8-byte aligned
      const float2 v01 = c[0], v23 = c[1], v45 = c[2];
      stg[i * 5 + 0] = v01.x;
      stg[i * 5 + 1] = v01.y;
      stg[i * 5 + 2] = v23.x;
      stg[i * 5 + 3] = v23.y;
      stg[i * 5 + 4] = v45.x;
      int anc = __float_as_int(v45.y);
      if (anc < 0 || anc >= a.n_anchors) {  // not a row detect_kernel / nms_load_kernel wrote
        misc[13] = 1;
        anc = i;
      }
      k = nms_key(v45.x, anc);
    }
    keys[i] = k;
  }
  __syncthreads();
  if (a.dbg) t[1] = __builtin_amdgcn_s_memrealtime();
  // rank sort: keys are unique (one candidate per anchor), so a candidate's sorted position is
  // the number of smaller keys -- no barrier stages; every lane of a wave reads the same key
  // (an LDS broadcast)
  if (tid < n) {
    const unsigned long long mine = keys[tid];
    int r = 0;
#pragma unroll 8
    for (int j = 0; j < n; ++j) r += keys[j] < mine ? 1 : 0;
    pay[NMS_MASK_N + r] = tid;  // second half of the payload area: slot at sorted position r
  }
  __syncthreads();
  if (a.dbg) t[2] = __builtin_amdgcn_s_memrealtime();
  if (n > a.max_nms) n = a.max_nms;  // nms.py:138-142
  const int* spay = pay + NMS_MASK_N;
  for (int i = tid; i < n; i += NMS_NT) {
    const int s = spay[i];
    const float x1 = stg[s * 5], y1 = stg[s * 5 + 1], x2 = stg[s * 5 + 2], y2 = stg[s * 5 + 3];
    bx[i] = make_float4(x1, y1, x2, y2);
    ar[i] = (x2 - x1) * (y2 - y1);
  }
  __syncthreads();
  int k;
  if (n <= NMS_GW * 64) {
    if (a.dbg) t[3] = __builtin_amdgcn_s_memrealtime();
    // specialised on the live word count: the unrolled word loops carry no dead blocks
    if (n <= 64) k = nms_greedy_wave<1>(bx, ar, n, a.iou, a.max_det, keep, misc + 15, misc + 14);
    else if (n <= 128) k = nms_greedy_wave<2>(bx, ar, n, a.iou, a.max_det, keep, misc + 15, misc + 14);
    else if (n <= 192) k = nms_greedy_wave<3>(bx, ar, n, a.iou, a.max_det, keep, misc + 15, misc + 14);
    else k = nms_greedy_wave<NMS_GW>(bx, ar, n, a.iou, a.max_det, keep, misc + 15, misc + 14);
    if (a.dbg) t[4] = __builtin_amdgcn_s_memrealtime();
  } else {
  // sup / ovl words: each wave holds every column box in registers (lane = column within a
  // word), then per row i one broadcast read of box i and W ballots form the row's words
  const int W = (n + 63) / 64;
  const float thr = a.iou;
  float4 bj[NMS_W];
  float aj[NMS_W];
#pragma unroll
  for (int w = 0; w < NMS_W; ++w) {
    const int j = w * 64 + lane;
    bj[w] = j < n ? bx[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    aj[w] = j < n ? ar[j] : 0.f;
  }
  for (int i = wave; i < n; i += NMS_NT / 64) {
    const float4 bi = bx[i];
    const float ai = ar[i];
    unsigned long long smw = 0ull, omw = 0ull;  // lane w keeps word w
    const int w0 = i >> 6;                       // words below hold only columns j <= i: zero
#pragma unroll
    for (int w = 0; w < NMS_W; ++w) {
      if (w >= W) break;
      if (w < w0) continue;
      const int j = w * 64 + lane;
      bool sb = false, ob = false;
      if (j > i && j < n) {
        const float ww = fmaxf(fminf(bi.z, bj[w].z) - fmaxf(bi.x, bj[w].x), 0.f);
        const float hh = fmaxf(fminf(bi.w, bj[w].w) - fmaxf(bi.y, bj[w].y), 0.f);
        const float inter = ww * hh;
        const float un = ai + aj[w] - inter;
        // iou <= thr decided on v_rcp (~1 ulp) unless within 1e-5 relative of thr; the rest (and a
        // zero or tiny union, where iou is NaN or inf) take the exact IEEE division
        const float q = inter * __builtin_amdgcn_rcpf(un);
        if (un > 1e-30f && fabsf(q - thr) > 1e-5f * thr) {
          sb = q > thr;
        } else {
          const float iou = inter / un;
          sb = !(iou <= thr);
        }
        ob = inter != 0.f;
      }
      const unsigned long long sm = __ballot(sb), om = __ballot(ob);
      if (lane == w) {
        smw = sm;
        omw = om;
      }
    }
    if (lane < W) {
      sup[i * NMS_W + lane] = smw;
      ovl[i * NMS_W + lane] = omw;
    }
  }
  __syncthreads();
  if (a.dbg) t[3] = __builtin_amdgcn_s_memrealtime();
  k = nms_walk(n, a.max_det, sup, ovl, keep, misc + 15, misc + 14);
  if (a.dbg) t[4] = __builtin_amdgcn_s_memrealtime();
  }
  if (misc[13]) k = 0;  // corrupt candidate rows: no detections, error flagged below
  // outputs: x[i] rows, then scale_boxes (x - pad) / gain and clip (ops.py:105-184)
  for (int r = tid; r < k; r += NMS_NT) {
    if (a.keep_out) {
      YK_SC(&a.keep_out[(size_t)b * a.max_det + r], 4, 20);
      a.keep_out[(size_t)b * a.max_det + r] = (int)(keys[pay[NMS_MASK_N + keep[r]]] & 0xffffffffu);
    }
    const float* c = stg + pay[NMS_MASK_N + keep[r]] * 5;
    float* o = a.dets + ((size_t)b * a.max_det + r) * 6;
    YK_SC(o, 24, 21);
    const float x1 = (c[0] - a.pad_x) / a.gain, y1 = (c[1] - a.pad_y) / a.gain;
    const float x2 = (c[2] - a.pad_x) / a.gain, y2 = (c[3] - a.pad_y) / a.gain;
    o[0] = fminf(fmaxf(x1, 0.f), a.clip_w);
    o[1] = fminf(fmaxf(y1, 0.f), a.clip_h);
    o[2] = fminf(fmaxf(x2, 0.f), a.clip_w);
    o[3] = fminf(fmaxf(y2, 0.f), a.clip_h);
    o[4] = c[4];
    o[5] = 0.f;
  }
  if (tid == 0) {
    YK_SC(&a.counts[b], 4, 22);
    a.counts[b] = k;
    if (misc[13]) nms_flag_error(a.err);
    if (a.stat) {
      atomicAdd(&a.stat[0], misc[14] && k > 0 ? 1 : 0);
      atomicAdd(&a.stat[1], 1);
    }
  }
  if (a.dbg) {
    __syncthreads();
    t[5] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      float* o = a.dets + ((size_t)b * a.max_det + a.max_det - 1) * 6;
      for (int q = 0; q < 5; ++q) o[q] = (float)(t[q + 1] - t[q]) * 0.01f;  // 100 MHz counter -> us
      o[5] = (float)n;
      o[-6] = (float)(__builtin_amdgcn_s_memtime() - c0) / ((float)(t[5] - t[0]) * 0.01f);  // core MHz
    }
  }
}

__global__ void __launch_bounds__(NMS_NT) nms_kernel(NmsArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x, tid = threadIdx.x;
  int n = a.cand_count[b];
  if (n > a.cap) n = a.cap;
  if (n <= NMS_MASK_N) {
    nms_small(a, b, n, smem);
    return;
  }
  const float* cand = a.cand + (size_t)b * a.cap * 6;
  const bool in_lds = n <= NMS_LDS_N;
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  unsigned long long* keys = in_lds ? (unsigned long long*)smem : a.gkeys + (size_t)b * a.key_cap;
  float* box = in_lds ? (float*)(smem + NMS_OFF_BOX) : a.gbox + (size_t)b * a.cap * 5;
  unsigned char* removed = in_lds ? smem + NMS_OFF_REM : a.gflag + (size_t)b * a.cap;
  int* misc = (int*)(smem + NMS_OFF_MISC);
  int* keep = (int*)(smem + NMS_OFF_KEEP);
  int* slot_of = a.slot_of + (size_t)b * a.n_anchors;
  if (tid < 16) misc[tid] = 0;  // [13] bad anchor, [14] early exit
  __syncthreads();
  // keys: (score desc, anchor asc) = the stable order (nms_key)
  for (int i = tid; i < n2; i += NMS_NT) {
    unsigned long long k = ~0ull;
    if (i < n) {
      int anc = __float_as_int(cand[i * 6 + 5]);
      if (anc < 0 || anc >= a.n_anchors) {  // not a row detect_kernel / nms_load_kernel wrote:
        misc[13] = 1;                        // never index outside slot_of; flag it
        anc = 0;
      } else {
        YK_SC(&slot_of[anc], 4, 30);
        slot_of[anc] = i;
      }
      k = nms_key(cand[i * 6 + 4], anc);
    }
    if (!in_lds) YK_SC(&keys[i], 8, 31);
    keys[i] = k;
  }
  __syncthreads();
  if (misc[13]) {
    if (tid == 0) {
      a.counts[b] = 0;
      nms_flag_error(a.err);
    }
    return;
  }
  if (n > 1) bitonic_sort(keys, n2);
  if (n > a.max_nms) n = a.max_nms;  // nms.py:138-142
  for (int i = tid; i < n; i += NMS_NT) {
    const int s = slot_of[(int)(keys[i] & 0xffffffffu)];
    const float* c = cand + (size_t)s * 6;
    const float x1 = c[0], y1 = c[1], x2 = c[2], y2 = c[3];
    if (!in_lds) {
      YK_SC(&box[i * 5], 20, 32);
      YK_SC(&removed[i], 1, 33);
    }
    box[i * 5 + 0] = x1;
    box[i * 5 + 1] = y1;
    box[i * 5 + 2] = x2;
    box[i * 5 + 3] = y2;
    box[i * 5 + 4] = (x2 - x1) * (y2 - y1);
    removed[i] = 0;
  }
  __syncthreads();
  int k = 0;
  const float thr = a.iou;
  if (n <= NMS_MASK_N) {
    unsigned long long* sup = (unsigned long long*)(smem + NMS_OFF_MASK);
    k = nms_bitmask(box, n, thr, a.max_det, sup, sup + NMS_MASK_N * NMS_W, keep, misc + 15, misc + 14);
  } else {
    for (int i = 0; i < n && k < a.max_det; ++i) {
      if (removed[i]) continue;
      if (tid == 0) keep[k] = i;
      ++k;
      const float bx1 = box[i * 5], by1 = box[i * 5 + 1], bx2 = box[i * 5 + 2], by2 = box[i * 5 + 3],
                  ba = box[i * 5 + 4];
      int any = 0;
      for (int j = i + 1 + tid; j < n; j += NMS_NT) {
        if (removed[j]) continue;
        const float w = fmaxf(fminf(bx2, box[j * 5 + 2]) - fmaxf(bx1, box[j * 5]), 0.f);
        const float h = fmaxf(fminf(by2, box[j * 5 + 3]) - fmaxf(by1, box[j * 5 + 1]), 0.f);
        if (w * h != 0.f) any = 1;
      }
      any = __syncthreads_or(any);
      if (!any) {
        // inter.sum() == 0: keep every remaining box, in order, and stop (nms.py:291-296)
        if (tid == 0 && i + 1 < n) misc[14] = 1;
        int base = k;
        for (int j0 = i + 1; j0 < n; j0 += NMS_NT) {
          const int j = j0 + tid;
          const int f = (j < n && !removed[j]) ? 1 : 0;
          const unsigned long long m = __ballot(f);
          const int lane = tid & 63, w = tid >> 6;
          if (lane == 0) misc[w] = __popcll(m);
          __syncthreads();
          int pre = 0, tot = 0;
          for (int q = 0; q < NMS_NT / 64; ++q) {
            pre += q < w ? misc[q] : 0;
            tot += misc[q];
          }
          const int r = base + pre + __popcll(m & ((1ull << lane) - 1ull));
          if (f && r < a.max_det) keep[r] = j;
          __syncthreads();
          base += tot;
        }
        k = base < a.max_det ? base : a.max_det;
        break;
      }
      for (int j = i + 1 + tid; j < n; j += NMS_NT) {
        if (removed[j]) continue;
        const float w = fmaxf(fminf(bx2, box[j * 5 + 2]) - fmaxf(bx1, box[j * 5]), 0.f);
        const float h = fmaxf(fminf(by2, box[j * 5 + 3]) - fmaxf(by1, box[j * 5 + 1]), 0.f);
        const float inter = w * h;
        const float iou = inter / (ba + box[j * 5 + 4] - inter);
        if (!(iou <= thr)) {
          if (!in_lds) YK_SC(&removed[j], 1, 34);
          removed[j] = 1;
        }
      }
      __syncthreads();
    }
  }
  __syncthreads();
  // outputs: x[i] rows, then scale_boxes (x - pad) / gain and clip (ops.py:105-184)
  for (int r = tid; r < k; r += NMS_NT) {
    const int i = keep[r];
    if (a.keep_out) {
      YK_SC(&a.keep_out[(size_t)b * a.max_det + r], 4, 35);
      a.keep_out[(size_t)b * a.max_det + r] = (int)(keys[i] & 0xffffffffu);
    }
    const int s = slot_of[(int)(keys[i] & 0xffffffffu)];
    const float* c = cand + (size_t)s * 6;
    float* o = a.dets + ((size_t)b * a.max_det + r) * 6;
    YK_SC(o, 24, 36);
    float x1 = (c[0] - a.pad_x) / a.gain, y1 = (c[1] - a.pad_y) / a.gain;
    float x2 = (c[2] - a.pad_x) / a.gain, y2 = (c[3] - a.pad_y) / a.gain;
    o[0] = fminf(fmaxf(x1, 0.f), a.clip_w);
    o[1] = fminf(fmaxf(y1, 0.f), a.clip_h);
    o[2] = fminf(fmaxf(x2, 0.f), a.clip_w);
    o[3] = fminf(fmaxf(y2, 0.f), a.clip_h);
    o[4] = c[4];
    o[5] = 0.f;
  }
  if (tid == 0) {
    YK_SC(&a.counts[b], 4, 37);
    a.counts[b] = k;
    if (a.stat) {
      atomicAdd(&a.stat[0], misc[14] && k > 0 ? 1 : 0);
      atomicAdd(&a.stat[1], 1);
    }
  }
}

// yk_nms: given boxes -> the candidate list the Detect ops would write (candidate id = row index,
// so the stable order is score desc, then input order -- torch_nms's stable sort)
__global__ void __launch_bounds__(256) nms_load_kernel(const float* rows, int row_stride, int max_rows,
                                                      const int* counts, float* cand, int* cand_count, int cap) {
  const int b = blockIdx.y;
  int n = counts[b];
  n = n < 0 ? 0 : n > max_rows ? max_rows : n;
  n = n > cap ? cap : n;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) cand_count[b] = n;
  if (i >= n) return;
  const float* r = rows + ((size_t)b * max_rows + i) * row_stride;
  float* c = cand + ((size_t)b * cap + i) * 6;
  c[0] = r[0];
  c[1] = r[1];
  c[2] = r[2];
  c[3] = r[3];
  c[4] = r[4];
  c[5] = __int_as_float(i);
}

#pragma clang fp contract(fast)

size_t nms_lds_bytes() { return NMS_LDS; }

// zero n int32 counters (one wave; n <= 64 * k handled by the loop)
__global__ void __launch_bounds__(64) zero_i32_kernel(int* p, int n) {
  for (int i = threadIdx.x; i < n; i += 64) p[i] = 0;
}

}  // namespace det
}  // namespace yk

using namespace yk::det;

// captured forwards kept per model (yk_detect_graph's LRU cache): the pipeline needs one per
// (frame buffer, detection buffer) pair, <= 2 x 4 D = 64 at D = 8
constexpr int kGraphCap = 64;

struct yk_model {
  yk_ctx* ctx = nullptr;
  yk_model_desc desc{};
  std::vector<yk_op> ops;
  std::vector<int64_t> buf_elems;
  std::vector<void*> bufs;
  char* blob = nullptr;
  float* cand = nullptr;
  int* cand_count = nullptr;
  int* slot_of = nullptr;
  unsigned long long* gkeys = nullptr;
  float* gbox = nullptr;
  unsigned char* gflag = nullptr;
  int key_cap = 0;
  float* dets = nullptr;
  int* counts = nullptr;
  int* nms_stat = nullptr;          // [2] device: NMS early exits, images (yk_model_nms_stats)
  volatile int* err_host = nullptr;  // host-mapped error word the kernels flag (nms_flag_error)
  int* err_dev = nullptr;
  // Captured forwards, keyed by the call's arguments (raw pointers: a caller that keeps handing
  // new buffers would grow the cache without bound, so it is LRU-bounded at kGraphCap entries).
  // A multi-lane graph owns the fork / join events its capture recorded (`evs`): no event is ever
  // recorded by two captures, or by a capture and an uncaptured forward.
  struct GraphEntry {
    hipGraphExec_t exec = nullptr;
    std::vector<hipEvent_t> evs;
    unsigned long long last_use = 0;
  };
  std::map<std::tuple<int, float, float, int, const void*, void*, void*>, GraphEntry> graphs;
  unsigned long long graph_clock = 0;
  const hipEvent_t* run_ev = nullptr;  // events run_dag records into (a capture's own set), or m->ev
  int plan_batch = 1;  // batch the kernel names of yk_model_op_kernel are reported for
  bool tiled = true;  // LDS-tiled conv kernel where its tile fits (YK_CONV_DIRECT=1 forces the direct kernel)
  // DAG schedule: ops run on `lanes` streams (lane 0 = the caller's stream) with event edges
  // for every cross-lane hazard; under capture this becomes a graph with parallel branches.
  // With `groups` > 1 the batch is cut into that many sub-batches, each an independent copy of
  // the DAG on its own `lanes` streams: the detector's kernels are latency-bound, so
  // independent chains overlap on the chip.
  int lanes = 1, groups = 1;
  struct Task {
    int op, grp, lane;
    std::vector<int> waits;  // producer tasks on other lanes (latest per lane)
    bool ev;                 // some later task on another lane waits on this one
  };
  std::vector<Task> tasks;
  std::vector<char> lane_used;              // lanes that run at least one task
  std::vector<hipStream_t> aux;             // lanes 1..groups*lanes-1
  hipStream_t cap = nullptr;                // graph-capture stream, kept for the model's lifetime
  std::vector<hipEvent_t> ev;               // per task + fork + joins
  // per-op conv plan chosen by yk_model_autotune (kind < 0: not tuned, use the heuristic)
  std::vector<std::array<int, 3>> tuned;    // {kind, nnt, npt}
  int tuned_batch = 0;
  // conv_fast_kernel K-step tables: one device array, per-op offsets (entries of int2)
  int2* ktab = nullptr;
  std::vector<int64_t> ktab_off;
  int* ltab = nullptr;                // conv_tile_kernel K-step tables (LDS element offsets)
  int xcd = 1;                        // YK_XCD=0: plain blockIdx order (A/B of the XCD-aware placement)
  bool input_valu = false;            // YK_INPUT_VALU=1: f32-VALU first conv in the bf16 build too
  int nms_dbg = 0;                    // YK_NMS_DBG: nms_kernel phase timing (never in production)
  int wide_dbg = 0;                   // YK_WIDE_DBG: conv_wide_kernel diagnostics (never in production)
  bool no_wide = false;               // YK_NO_WIDE=1: autotune without the LDS-resident wide kernel
  int ts_op = -1;                     // YK_FAST_TS=<op>: per-workgroup timestamps of that conv_fast op
  int fast_ipw = 1;                   // YK_FAST_IPW=<n>: conv_fast in its persistent form, n items per workgroup
  unsigned long long* ts = nullptr;   // [3 * kTsCap] start, after K loop, end (wall_clock64, 100 MHz)
  std::vector<int64_t> ltab_off;
  unsigned char* lbox = nullptr;  // letterboxed frames [max_batch][in_h][in_w][3] (resize only)
  char* arena = nullptr;      // every activation buffer (bufs[i] point into it)
  size_t arena_bytes = 0;
  size_t blob_bytes = 0;
  // F32 build: every table-kernel conv's weights split into three bf16 parts (F32S, 24-byte
  // fragments in the packed fragment order), for the split-MFMA variant (plan npt bit kSplitBit)
  char* wsplit = nullptr;
  size_t wsplit_bytes = 0;
  std::vector<int64_t> ws_off;
  // F32 build: the same weights in conv_halo_kernel's K-slot layout (build_wkslot)
  char* wkslot = nullptr;
  size_t wkslot_bytes = 0;
  std::vector<int64_t> wk_off;
  bool split_default = false;  // YK_F32_SPLIT=1: the heuristic plan uses F32S where it can
  bool autotune_split = true;  // YK_F32_SPLIT=0: autotune never picks F32S
};

namespace {

#if YK_STORE_CHECK
// (diagnostic build) the legal store ranges the kernels check against: a host copy, uploaded to
// the device table whenever it grows (never while a stream captures: callers register first)
std::vector<std::pair<unsigned long long, unsigned long long>> g_sc;
void sc_register(const void* p, size_t bytes) {
  if (!p || !bytes) return;
  const unsigned long long lo = (unsigned long long)p, hi = lo + bytes;
  for (auto& r : g_sc)
    if (r.first <= lo && hi <= r.second) return;
  if (g_sc.size() >= (size_t)kScMax) {
    fprintf(stderr, "[yk store check] range table full\n");
    return;
  }
  g_sc.push_back({lo, hi});
  std::vector<unsigned long long> l, h;
  for (auto& r : g_sc) {
    l.push_back(r.first);
    h.push_back(r.second);
  }
  const int n = (int)g_sc.size();
  (void)hipDeviceSynchronize();
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_lo), l.data(), n * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_hi), h.data(), n * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(sc_n), &n, 4);
}
#else
inline void sc_register(const void*, size_t) {}
#endif

int esz_of(int dtype) { return dtype == YK_ACT_F32 ? 4 : dtype == YK_ACT_FP8 ? 1 : 2; }  // BF16 / F16: 2
size_t act_bytes(const yk_model* m) { return (size_t)esz_of(m->desc.act_dtype); }
// trait name as rocprofv3 demangles it
const char* tr_name(int dtype) {
  return dtype == YK_ACT_F32 ? "F32" : dtype == YK_ACT_FP8 ? "FP8" : dtype == YK_ACT_F16 ? "F16" : "BF16";
}

// Base of image b0 of a buffer whose per-image extent is h x w x c_stride elements.
void* img_ptr(const yk_model* m, int buf, int h, int w, int cstride, int b0) {
  return (char*)m->bufs[buf] + (size_t)b0 * h * w * cstride * act_bytes(m);
}

View make_view(yk_model* m, const yk_view& v, int b0 = 0) {
  View o;
  o.p = img_ptr(m, v.buf, v.h, v.w, v.c_stride, b0);
  o.cstride = v.c_stride;
  o.coff = v.c_off;
  o.h = v.h;
  o.w = v.w;
  o.up = v.up;
  return o;
}

template <class Tr, int NNT>
void launch_conv_t(const ConvArgs& a, int n_tiles, hipStream_t st) {
  constexpr int NPT = 2;
  dim3 grid((a.M + 64 * NPT - 1) / (64 * NPT), (n_tiles + NNT - 1) / NNT);
  hipLaunchKernelGGL((conv_igemm_kernel<Tr, NNT, NPT>), grid, dim3(256), 0, st, a);
}

template <class Tr>
void launch_conv(const ConvArgs& a, hipStream_t st) {
  const int nt = a.n_tiles;
  if (nt <= 1) launch_conv_t<Tr, 1>(a, nt, st);
  else if (nt == 2) launch_conv_t<Tr, 2>(a, nt, st);
  else if (nt == 3 || nt == 6 || nt == 9) launch_conv_t<Tr, 3>(a, nt, st);
  else launch_conv_t<Tr, 4>(a, nt, st);
}

// Tile geometry of the LDS-tiled conv for one op (ok = false -> the direct-load kernel).
struct TilePlan {
  bool ok = false, split = false, single = false;
  int nnt = 4, npt = 1, tih = 0, tiw = 0, ps = 0, tiles_x = 0, tiles_y = 0;
  size_t lds = 0;
};
constexpr size_t kTileLdsMax = 144 * 1024;

TilePlan tile_plan_geom(const yk_op& op, int esz, int B);

// Geometry, then whether the whole weight slab fits LDS next to the input tile (one prologue,
// no chunk barriers) without costing occupancy beyond ~96 KB per workgroup.
// big_single: keep the whole weight slab LDS-resident up to the 144 KiB cap (one workgroup
// per CU, no chunk barriers), for the wide high-resolution convs.
TilePlan tile_plan(const yk_op& op, int esz, int B, bool big_single = false) {
  TilePlan t = tile_plan_geom(op, esz, B);
  if (!t.ok) return t;
  t.lds = (t.lds + 15) / 16 * 16 + (size_t)op.k_steps * 16;  // + the K-step table
  const size_t tile = (size_t)t.tih * t.tiw * t.ps * esz;
  const size_t slab = (size_t)t.nnt * op.k_steps * 1024;
  const size_t red = t.split ? (size_t)4 * t.nnt * t.npt * 64 * 16 : 0;
  const size_t lds1 = (slab > red ? slab : red) + (tile + 15) / 16 * 16 + (size_t)op.k_steps * 16;
  const size_t cap = big_single ? kTileLdsMax : t.lds > 96 * 1024 ? t.lds : 96 * 1024;
  if (lds1 <= cap && lds1 <= kTileLdsMax) {
    t.single = true;
    t.lds = lds1;
  }
  return t;
}

TilePlan tile_plan_geom(const yk_op& op, int esz, int B) {
  TilePlan t;
  const int nt = op.n_tiles;
  const int cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
  int U = cin * esz / 16;
  if ((U & 1) == 0) U += 1;  // odd number of 16-byte slots per pixel: conflict-free b128 reads
  t.ps = U * 16 / esz;
  const int s = op.stride, k = op.ksize;
  const int oh4 = (op.out_h + 3) / 4 * 4;
  const int tiles_x = (op.out_w + 15) / 16;
  // Prefer the largest whole-tile geometry (weights reused over more pixels) that gives >= 2
  // workgroups per CU.  Otherwise (low-resolution layers) use split-K tiles (the four waves
  // split K over one 16 x NPT tile), choosing the geometry with the most workgroups.
  const int nnt0 = nt <= 4 ? nt : (nt == 5 || nt == 6 || nt == 9) ? 3 : 4;
  const int cand_nnt[3] = {nnt0, nnt0 > 2 ? 2 : 0, nnt0 > 1 ? 1 : 0};
  for (int ci = 0; ci < 3; ++ci) {
    const int nnt = cand_nnt[ci];
    if (nnt <= 0) continue;
    for (int npt = 4; npt >= 1; npt >>= 1) {
      const int th = 4 * npt;
      if (npt > 1 && th > oh4) continue;
      const int tih = (th - 1) * s + k, tiw = 15 * s + k;
      const size_t lds = (size_t)2 * nnt * 4 * 1024 + (size_t)tih * tiw * t.ps * esz;
      if (lds > kTileLdsMax) continue;
      const int tiles_y = (op.out_h + th - 1) / th;
      const long wgs = (long)B * tiles_x * tiles_y * ((nt + nnt - 1) / nnt);
      if (wgs >= 512) {
        t.ok = true;
        t.nnt = nnt;
        t.npt = npt;
        t.tih = tih;
        t.tiw = tiw;
        t.lds = lds;
        t.tiles_y = tiles_y;
        t.tiles_x = tiles_x;
        return t;
      }
    }
  }
  long best = -1;
  for (int nnt = (nnt0 < 2 ? nnt0 : 2); nnt >= 1; --nnt) {
    for (int npt = 4; npt >= 1; npt >>= 1) {
      const int th = npt;
      const int tih = (th - 1) * s + k, tiw = 15 * s + k;
      const size_t red = (size_t)4 * nnt * npt * 64 * 16;
      const size_t wbytes = (size_t)2 * nnt * 8 * 1024;
      const size_t lds = (wbytes > red ? wbytes : red) + (size_t)tih * tiw * t.ps * esz;
      if (lds > kTileLdsMax) continue;
      const int tiles_y = (op.out_h + th - 1) / th;
      const long wgs = (long)B * tiles_x * tiles_y * ((nt + nnt - 1) / nnt);
      // most workgroups, then the larger tile (fewer redundant halo loads)
      if (wgs > best + best / 8) {
        best = wgs;
        t.ok = true;
        t.split = true;
        t.nnt = nnt;
        t.npt = npt;
        t.tih = tih;
        t.tiw = tiw;
        t.lds = lds;
        t.tiles_y = tiles_y;
        t.tiles_x = tiles_x;
      }
    }
  }
  return t;
}

template <class Tr, int NNT, int NPT, bool SPLIT>
void launch_tile_t(const TileArgs& a, const TilePlan& tp, int B, hipStream_t st) {
  dim3 grid(B * tp.tiles_x * tp.tiles_y, (a.n_tiles + NNT - 1) / NNT);
  hipLaunchKernelGGL((conv_tile_kernel<Tr, NNT, NPT, SPLIT>), grid, dim3(256), tp.lds, st, a);
}

template <class Tr, int NNT, bool SPLIT>
void launch_tile_n(const TileArgs& a, const TilePlan& tp, int B, hipStream_t st) {
  if (tp.npt == 4) launch_tile_t<Tr, NNT, 4, SPLIT>(a, tp, B, st);
  else if (tp.npt == 2) launch_tile_t<Tr, NNT, 2, SPLIT>(a, tp, B, st);
  else launch_tile_t<Tr, NNT, 1, SPLIT>(a, tp, B, st);
}

template <class Tr>
void launch_tile(const TileArgs& a, const TilePlan& tp, int B, hipStream_t st) {
  if (tp.split) {
    if (tp.nnt == 2) launch_tile_n<Tr, 2, true>(a, tp, B, st);
    else launch_tile_n<Tr, 1, true>(a, tp, B, st);
    return;
  }
  switch (tp.nnt) {
    case 1: launch_tile_n<Tr, 1, false>(a, tp, B, st); break;
    case 2: launch_tile_n<Tr, 2, false>(a, tp, B, st); break;
    case 3: launch_tile_n<Tr, 3, false>(a, tp, B, st); break;
    default: launch_tile_n<Tr, 4, false>(a, tp, B, st); break;
  }
}

template <class Tr, int NNT, int NPT, bool SPLIT>
void set_tile_attr() {
  (void)hipFuncSetAttribute((const void*)conv_tile_kernel<Tr, NNT, NPT, SPLIT>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTileLdsMax);
}
template <class Tr, int NNT, bool SPLIT>
void set_tile_attr_n() {
  set_tile_attr<Tr, NNT, 1, SPLIT>();
  set_tile_attr<Tr, NNT, 2, SPLIT>();
  set_tile_attr<Tr, NNT, 4, SPLIT>();
}
template <class Tr>
void set_tile_attrs_t() {
  set_tile_attr_n<Tr, 1, false>();
  set_tile_attr_n<Tr, 2, false>();
  set_tile_attr_n<Tr, 3, false>();
  set_tile_attr_n<Tr, 4, false>();
  set_tile_attr_n<Tr, 1, true>();
  set_tile_attr_n<Tr, 2, true>();
}
template <class Tr, int NNT, int NPT, int KW>
void set_fast_attr() {
  constexpr int SKD = fast_skd(NNT, NPT);
  (void)hipFuncSetAttribute((const void*)conv_fast_kernel<Tr, NNT, NPT, KW, SKD>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
}
template <class Tr, int NNT, int NPT>
void set_fastw_attr() {
  constexpr int SKD = fastw_skd(NNT, NPT);
  (void)hipFuncSetAttribute((const void*)conv_fastw_kernel<Tr, NNT, NPT, SKD>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
}
template <class Tr, int NNT, int KW>
void set_fast_attr_n() {
  set_fast_attr<Tr, NNT, 1, KW>();
  set_fast_attr<Tr, NNT, 2, KW>();
  set_fast_attr<Tr, NNT, 4, KW>();
  if constexpr (KW == 1) {
    set_fastw_attr<Tr, NNT, 1>();
    set_fastw_attr<Tr, NNT, 2>();
    set_fastw_attr<Tr, NNT, 4>();
  }
}
template <class Tr, int KW>
void set_fast_attr_w() {
  set_fast_attr_n<Tr, 1, KW>();
  set_fast_attr_n<Tr, 2, KW>();
  set_fast_attr_n<Tr, 3, KW>();
  set_fast_attr_n<Tr, 4, KW>();
}
// conv_wide_kernel instantiations that compile without spilling: with 8 waves (two per SIMD, 256
// registers each) the staging units of UPT > 12 (2 tiles) or UPT > 4 (4 tiles) spilled 12-209
// VGPRs to scratch, so those are neither built nor offered to the autotuner
constexpr bool wide_ok(int nnt, int upt, int nw) { return nw == 4 || (nnt == 2 ? upt <= 12 : upt <= 4); }
template <class Tr, int NNT, int UPT, int NW>
void set_wide_attr_u() {
  if constexpr (wide_ok(NNT, UPT, NW))
    (void)hipFuncSetAttribute((const void*)conv_wide_kernel<Tr, NNT, UPT, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}
template <class Tr, int NNT, int NW>
void set_wide_attr_w() {
  set_wide_attr_u<Tr, NNT, 4, NW>();
  set_wide_attr_u<Tr, NNT, 8, NW>();
  set_wide_attr_u<Tr, NNT, 12, NW>();
  set_wide_attr_u<Tr, NNT, 16, NW>();
}
template <class Tr, int NNT>
void set_wide_attr_n() {
  set_wide_attr_w<Tr, NNT, 4>();
  set_wide_attr_w<Tr, NNT, 8>();
}
template <int NE, int NPT>
void set_halo_attr_p() {
  (void)hipFuncSetAttribute((const void*)conv_halo_kernel<NE, NPT, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHaloLds);
  (void)hipFuncSetAttribute((const void*)conv_halo_kernel<NE, NPT, 0, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHaloLds);
  (void)hipFuncSetAttribute((const void*)conv_halo_kernel<NE, NPT, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHaloLds);
  (void)hipFuncSetAttribute((const void*)conv_halo_kernel<NE, NPT, 1, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHaloLds);
}
template <int NE>
void set_halo_attr_n() {
  set_halo_attr_p<NE, 1>();
  set_halo_attr_p<NE, 2>();
  set_halo_attr_p<NE, 4>();
}
void set_tile_attrs() {
  set_halo_attr_n<1>();
  set_halo_attr_n<2>();
  set_tile_attrs_t<BF16>();
  set_tile_attrs_t<F16>();
  set_tile_attrs_t<F32>();
  set_wide_attr_n<BF16, 2>();
  set_wide_attr_n<BF16, 4>();
  set_wide_attr_n<F16, 2>();
  set_wide_attr_n<F16, 4>();
  set_wide_attr_n<F32, 2>();
  set_wide_attr_n<F32, 4>();
  set_fast_attr_w<BF16, 1>();
  set_fast_attr_w<BF16, 2>();
  set_fast_attr_w<BF16, 4>();
  set_fast_attr_w<F16, 1>();
  set_fast_attr_w<F16, 2>();
  set_fast_attr_w<F16, 4>();
  set_fast_attr_w<F32, 1>();
  set_fast_attr_w<F32, 2>();
  set_fast_attr_w<F32, 4>();
  set_fast_attr_w<F32S, 1>();
  set_fast_attr_w<F32S, 2>();
  set_fast_attr_w<F32S, 4>();
  set_wide_attr_n<FP8, 2>();
  set_wide_attr_n<FP8, 4>();
  set_fast_attr_w<FP8, 1>();
  set_fast_attr_w<FP8, 2>();
  set_fast_attr_w<FP8, 4>();
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<FP8, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<BF16, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<F16, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<F16, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<F32, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<FP8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<BF16, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
  (void)hipFuncSetAttribute((const void*)sppf_lds_kernel<F32, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLdsBytes);
}

// Conv kernel choice for one op at batch B.
enum { CK_DIRECT = 0, CK_TILE = 1, CK_SPLITK = 2, CK_FAST = 3, CK_WIDE = 4, CK_HALO = 5 };
// CK_FAST plan npt bit: the F32 build's op runs the F32S split-MFMA body (every mode)
constexpr int kSplitBit = 64;
// CK_WIDE plan: nnt in {2, 4} (output-channel tiles per workgroup), npt unused
// CK_HALO plan (F32 build): nnt = NE in {1, 2}, npt = NPT | WM << 4 with NPT in {1, 2, 4}
// CK_FAST plan: nnt in {1, 2, 3, 4}, npt = NPT | (mode << 4) with NPT in {1, 2, 4} (launch_fast)
struct ConvPlan {
  int kind = CK_DIRECT, nnt = 0, npt = 0;
  TilePlan tp;
};

// split-K geometry: the largest fragment tile (NNT x NPT) that still gives >= 1024 workgroups
// and wastes < 25% of the n-tiles, else the one with the most workgroups.
ConvPlan splitk_plan(const yk_op& op, int B, int nnt_force = 0, int npt_force = 0) {
  static const int cand[9][2] = {{4, 4}, {4, 2}, {2, 4}, {2, 2}, {4, 1}, {1, 4}, {2, 1}, {1, 2}, {1, 1}};
  const long M = (long)B * op.out_h * op.out_w;
  const int nt = op.n_tiles;
  ConvPlan p;
  p.kind = CK_SPLITK;
  if (nnt_force) {
    p.nnt = nnt_force;
    p.npt = npt_force;
    return p;
  }
  long best = -1;
  for (auto& c : cand) {
    const int nnt = c[0], npt = c[1];
    const int groups = (nt + nnt - 1) / nnt;
    if (nnt > 1 && 4 * nt < 3 * groups * nnt) continue;
    const long wgs = (M + 16 * npt - 1) / (16 * npt) * groups;
    if (wgs >= 1024) {
      p.nnt = nnt;
      p.npt = npt;
      return p;
    }
    if (wgs > best) {
      best = wgs;
      p.nnt = nnt;
      p.npt = npt;
    }
  }
  return p;
}

// conv_wide_kernel geometry of an op: 16 x 16 output tiles, input tile 15 * s + k square,
// odd number of 16-B units per pixel; ok = fits 160 KiB of LDS with its weight slab.
struct WidePlan {
  bool ok = false;
  int tih = 0, tiw = 0, ps = 0, upt = 0;
  size_t lds = 0;
};
WidePlan wide_plan(const yk_op& op, int esz, int nnt, int nw = 4) {
  WidePlan w;
  const int cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
  if (cin % 8 || (op.ksize != 1 && op.ksize != 3)) return w;
  int U = cin * esz / 16;
  const int units = U;
  if ((U & 1) == 0) U += 1;
  w.ps = U * 16 / esz;
  w.tih = w.tiw = 15 * op.stride + op.ksize;
  const int total = w.tih * w.tiw * units;
  w.upt = (total + 64 * nw - 1) / (64 * nw);
  w.lds = wide_lds(nnt, op.k_steps, w.tih, w.tiw, w.ps, esz);
  const int ub = w.upt <= 4 ? 4 : w.upt <= 8 ? 8 : w.upt <= 12 ? 12 : 16;  // the instantiation launch_wide_n takes
  w.ok = w.upt <= 16 && w.lds <= 160 * 1024 && w.tih < 128 && wide_ok(nnt, ub, nw);
  for (int sidx = 0; sidx < op.n_src; ++sidx) w.ok = w.ok && (op.ksize == 1 || op.src[sidx].up == 0);
  return w;
}

// conv_halo_kernel tile: the output tile (tr x tc, its 16 * NF pixels row-major) whose input
// window fits a plane (kHaloPx pixels) at the least cost ~ MFMA work incl. the tile's padding
// (pixels x taps) + staging (window pixels).  Sources: 4-channel groups never straddle the two.
struct HaloPlan {
  bool ok = false;
  int tr = 0, tc = 0, twin = 0, npx = 0, tiles_x = 0, tiles_y = 0, rp = 0, hw = 0;
};
HaloPlan halo_plan(const yk_op& op, int npt, int wm) {
  HaloPlan h;
  const int k = op.ksize, s = op.stride;
  const int c0 = op.src_ch[0], cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
  if ((k != 1 && k != 3) || cin % 4 || c0 % 4 || op.out_h < 1 || op.out_w < 1) return h;
  const int px = 16 * (wm ? npt : 4 * npt);
  long best = -1;
  for (int tc = 1; tc <= op.out_w && tc <= px; ++tc) {
    const int tr = std::min(px / tc, op.out_h);
    const int twin = (tc - 1) * s + k, thin = (tr - 1) * s + k;
    int rp = twin;  // stride 1: rp = tc (mod 16); stride 2 (even tc): 2 rp = tc (mod 16)
    if (s == 1) rp = twin + (((tc - twin) % 16) + 16) % 16;
    else if (s == 2 && tc % 2 == 0) rp = twin + (((tc / 2 - twin) % 8) + 8) % 8;
    if (rp * thin > kHaloPx / (k == 1 ? 4 : 1)) continue;  // a plane (1x1: four 16-channel groups per chunk)
    const long tiles = (long)((op.out_h + tr - 1) / tr) * ((op.out_w + tc - 1) / tc);
    const long cost = tiles * (4L * k * k * px + twin * thin);
    if (best < 0 || cost < best) {
      best = cost;
      h.tr = tr;
      h.tc = tc;
      h.twin = twin;
      h.npx = twin * thin;
      h.rp = rp;
      h.hw = s == 2 ? (twin + 1) / 2 : 0;
      h.tiles_x = (op.out_w + tc - 1) / tc;
      h.tiles_y = (op.out_h + tr - 1) / tr;
    }
  }
  h.ok = best >= 0;
  return h;
}

// conv_fast_kernel geometry: the largest fragment tile (NNT x NPT) that still gives >= 1024
// workgroups (>= 4 waves per CU) and wastes < 25% of the n-tiles; the four waves split K (WS)
// when the per-wave-pixel layout would give too few workgroups.
ConvPlan fast_plan(const yk_op& op, int B) {
  static const int cand[9][2] = {{4, 4}, {4, 2}, {2, 4}, {2, 2}, {4, 1}, {1, 4}, {2, 1}, {1, 2}, {1, 1}};
  const long M = (long)B * op.out_h * op.out_w;
  const int nt = op.n_tiles;
  ConvPlan p;
  p.kind = CK_FAST;
  long best = -1;
  for (int ws = 0; ws < 2; ++ws)
    for (auto& c : cand) {
      int nnt = c[0];
      const int npt = c[1];
      if (nnt == 4 && (nt == 3 || nt == 6 || nt == 9)) nnt = 3;
      const int groups = (nt + nnt - 1) / nnt;
      if (nnt > 1 && 4 * nt < 3 * groups * nnt) continue;
      const long wgs = (M + (ws ? 16 : 64) * npt - 1) / ((ws ? 16 : 64) * npt) * groups;
      if (wgs >= 1024) {
        p.nnt = nnt;
        p.npt = npt | (ws << 4);
        return p;
      }
      if (wgs > best) {
        best = wgs;
        p.nnt = nnt;
        p.npt = npt | (ws << 4);
      }
    }
  return p;
}

ConvPlan conv_plan(const yk_model* m, const yk_op& op, int B) {
  const int esz = esz_of(m->desc.act_dtype);
  const size_t idx = (size_t)(&op - m->ops.data());
  if (idx < m->tuned.size() && m->tuned[idx][0] >= 0 && m->tuned_batch == B) {
    const auto& t = m->tuned[idx];
    if (t[0] == CK_SPLITK) return splitk_plan(op, B, t[1], t[2]);
    if (t[0] == CK_WIDE && m->ltab && m->ltab_off[idx] >= 0 && m->arena_bytes < kArenaMax &&
        wide_plan(op, esz, t[1], t[2] == 8 ? 8 : 4).ok) {
      ConvPlan p;
      p.kind = CK_WIDE;
      p.nnt = t[1];
      p.npt = t[2] == 8 ? 8 : 4;  // waves per workgroup
      return p;
    }
    if (t[0] == CK_FAST && m->ktab && m->ktab_off[idx] >= 0 && (long)B * op.out_h * op.out_w < (1L << 22)) {
      ConvPlan p;
      p.kind = CK_FAST;
      p.nnt = t[1];
      p.npt = t[2];
      if ((p.npt & kSplitBit) && !(m->wsplit && m->ws_off[idx] >= 0)) p.npt &= ~kSplitBit;
      return p;
    }
    if (t[0] == CK_HALO && m->wkslot && m->wk_off[idx] >= 0 && halo_plan(op, t[2] & 15, (t[2] >> 4) & 1).ok) {
      ConvPlan p;
      p.kind = CK_HALO;
      p.nnt = t[1];
      p.npt = t[2];
      return p;
    }
    if (t[0] == CK_TILE && m->ltab && m->ltab_off[idx] >= 0) {
      ConvPlan p;
      p.kind = CK_TILE;
      p.tp = tile_plan(op, esz, B, t[1] == 1);
      if (p.tp.ok) return p;
    }
    return ConvPlan{};
  }
  if (!m->tiled) return ConvPlan{};
  const size_t oi = (size_t)(&op - m->ops.data());
  if (m->ktab && oi < m->ktab_off.size() && m->ktab_off[oi] >= 0 && (long)B * op.out_h * op.out_w < (1L << 22)) {
    ConvPlan p = fast_plan(op, B);  // (fdiv: pixel indices < 2^22)
    if (m->split_default && m->wsplit && m->ws_off[oi] >= 0) p.npt |= kSplitBit;
    return p;
  }
  if (op.out_h * op.out_w <= 1280) return splitk_plan(op, B);
  ConvPlan p;
  p.tp = tile_plan(op, esz, B);
  p.kind = p.tp.ok && m->ltab && m->ltab_off[oi] >= 0 ? CK_TILE : CK_DIRECT;
  return p;
}

template <class Tr, int NNT, int NPT>
void launch_splitk_t(const ConvArgs& a, hipStream_t st) {
  dim3 grid((a.M + 16 * NPT - 1) / (16 * NPT), (a.n_tiles + NNT - 1) / NNT);
  hipLaunchKernelGGL((conv_splitk_kernel<Tr, NNT, NPT>), grid, dim3(256), 0, st, a);
}
template <class Tr, int NNT>
void launch_splitk_n(const ConvArgs& a, int npt, hipStream_t st) {
  if (npt == 4) launch_splitk_t<Tr, NNT, 4>(a, st);
  else if (npt == 2) launch_splitk_t<Tr, NNT, 2>(a, st);
  else launch_splitk_t<Tr, NNT, 1>(a, st);
}
template <class Tr>
void launch_splitk(const ConvArgs& a, const ConvPlan& p, hipStream_t st) {
  if (p.nnt == 4) launch_splitk_n<Tr, 4>(a, p.npt, st);
  else if (p.nnt == 2) launch_splitk_n<Tr, 2>(a, p.npt, st);
  else launch_splitk_n<Tr, 1>(a, p.npt, st);
}

template <class Tr, int NNT, int NPT, int KW>
void launch_fast_t(const FastArgs& a0, hipStream_t st) {
  constexpr int SKD = fast_skd(NNT, NPT);
  const int px = (64 / KW) * NPT;
  dim3 grid((a0.M + px - 1) / px, (a0.n_tiles + NNT - 1) / NNT);
  FastArgs a = a0;
  a.n_items = (int)(grid.x * grid.y);
  a.n_cg = (int)grid.y;
  if (YK_FAST_PERSIST && a.ipw > 1 && a.n_items > 8) {  // persistent form: a multiple of 8 workgroups (XCD placement)
    int g = (a.n_items + a.ipw - 1) / a.ipw;
    g = (g + 7) / 8 * 8;
    grid = dim3(g < a.n_items ? g : a.n_items, 1);
  } else {
    a.ipw = 1;
  }
  hipLaunchKernelGGL((conv_fast_kernel<Tr, NNT, NPT, KW, SKD>), grid, dim3(256), fast_lds(a.k_steps, NNT, NPT, KW), st,
                     a);
}
template <class Tr, int NNT, int KW>
void launch_fast_n(const FastArgs& a, int npt, hipStream_t st) {
  if (npt == 4) launch_fast_t<Tr, NNT, 4, KW>(a, st);
  else if (npt == 2) launch_fast_t<Tr, NNT, 2, KW>(a, st);
  else launch_fast_t<Tr, NNT, 1, KW>(a, st);
}
template <class Tr, int KW>
void launch_fast_w(const FastArgs& a, int nnt, int npt, hipStream_t st) {
  switch (nnt) {
    case 1: launch_fast_n<Tr, 1, KW>(a, npt, st); break;
    case 2: launch_fast_n<Tr, 2, KW>(a, npt, st); break;
    case 3: launch_fast_n<Tr, 3, KW>(a, npt, st); break;
    default: launch_fast_n<Tr, 4, KW>(a, npt, st); break;
  }
}
template <class Tr, int NNT, int NPT>
void launch_fastw_t(const FastArgs& a, hipStream_t st) {
  constexpr int SKD = fastw_skd(NNT, NPT);
  dim3 grid((a.M + 64 * NPT - 1) / (64 * NPT), (a.n_tiles + NNT - 1) / NNT);
  hipLaunchKernelGGL((conv_fastw_kernel<Tr, NNT, NPT, SKD>), grid, dim3(256), fastw_lds(a.k_steps, NNT, Frag<Tr>::WB), st,
                     a);
}
template <class Tr, int NNT>
void launch_fastw_n(const FastArgs& a, int npt, hipStream_t st) {
  if (npt == 4) launch_fastw_t<Tr, NNT, 4>(a, st);
  else if (npt == 2) launch_fastw_t<Tr, NNT, 2>(a, st);
  else launch_fastw_t<Tr, NNT, 1>(a, st);
}
template <class Tr>
void launch_fastw(const FastArgs& a, int nnt, int npt, hipStream_t st) {
  switch (nnt) {
    case 1: launch_fastw_n<Tr, 1>(a, npt, st); break;
    case 2: launch_fastw_n<Tr, 2>(a, npt, st); break;
    case 3: launch_fastw_n<Tr, 3>(a, npt, st); break;
    default: launch_fastw_n<Tr, 4>(a, npt, st); break;
  }
}
// plan.npt = NPT | mode << 4: mode 0 per-wave pixels, 1 = the four waves split K (KW 4),
// 2 = per-wave pixels with the weight fragments shared through LDS (conv_fastw_kernel),
// 3 = two pairs of waves, each pair splitting K (KW 2)
template <class Tr>
void launch_fast(const FastArgs& a, const ConvPlan& p, hipStream_t st) {
  const int mode = (p.npt >> 4) & 3;
  if (mode == 2) {
    launch_fastw<Tr>(a, p.nnt, p.npt & 15, st);
    return;
  }
  if (mode == 1) launch_fast_w<Tr, 4>(a, p.nnt, p.npt & 15, st);
  else if (mode == 3) launch_fast_w<Tr, 2>(a, p.nnt, p.npt & 15, st);
  else launch_fast_w<Tr, 1>(a, p.nnt, p.npt & 15, st);
}

template <int NE, int NPT, int WM, int KS>
void launch_halo_t(const HaloArgs& a, int B, hipStream_t st) {
  const int per = NE * (WM ? 4 : 1);
  dim3 grid(B * a.tiles_x * a.tiles_y, (a.n_tiles + per - 1) / per);
  hipLaunchKernelGGL((conv_halo_kernel<NE, NPT, WM, KS>), grid, dim3(256), kHaloLds, st, a);
}
template <int NE, int NPT, int WM>
void launch_halo_k(const HaloArgs& a, int B, int ks, hipStream_t st) {
  if (ks == 3) launch_halo_t<NE, NPT, WM, 3>(a, B, st);
  else launch_halo_t<NE, NPT, WM, 1>(a, B, st);
}
template <int NE, int NPT>
void launch_halo_w(const HaloArgs& a, int B, int wm, int ks, hipStream_t st) {
  if (wm) launch_halo_k<NE, NPT, 1>(a, B, ks, st);
  else launch_halo_k<NE, NPT, 0>(a, B, ks, st);
}
template <int NE>
void launch_halo_p(const HaloArgs& a, int B, int npt, int wm, int ks, hipStream_t st) {
  if (npt == 4) launch_halo_w<NE, 4>(a, B, wm, ks, st);
  else if (npt == 2) launch_halo_w<NE, 2>(a, B, wm, ks, st);
  else launch_halo_w<NE, 1>(a, B, wm, ks, st);
}
void launch_halo(const HaloArgs& a, int B, const ConvPlan& p, int ks, hipStream_t st) {
  const int npt = p.npt & 15, wm = (p.npt >> 4) & 1;
  if (p.nnt == 2) launch_halo_p<2>(a, B, npt, wm, ks, st);
  else launch_halo_p<1>(a, B, npt, wm, ks, st);
}

template <class Tr, int NNT, int UPT, int NW>
void launch_wide_t(const WideArgs& a, size_t lds, hipStream_t st) {
  if constexpr (!wide_ok(NNT, UPT, NW)) {
    return;  // (wide_plan never selects it)
  } else {
  const int groups = (a.n_tiles + NNT - 1) / NNT;
  const int nsp = a.B * a.tiles_y * a.tiles_x;
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu < 1) per_cu = 1;
  int gx = 256 * per_cu / groups;
  if (gx < 1) gx = 1;
  if (gx > nsp) gx = nsp;
  hipLaunchKernelGGL((conv_wide_kernel<Tr, NNT, UPT, NW>), dim3(gx, groups), dim3(64 * NW), lds, st, a);
  }
}
template <class Tr, int NNT, int NW>
void launch_wide_n(const WideArgs& a, int upt, size_t lds, hipStream_t st) {
  if (upt <= 4) launch_wide_t<Tr, NNT, 4, NW>(a, lds, st);
  else if (upt <= 8) launch_wide_t<Tr, NNT, 8, NW>(a, lds, st);
  else if (upt <= 12) launch_wide_t<Tr, NNT, 12, NW>(a, lds, st);
  else launch_wide_t<Tr, NNT, 16, NW>(a, lds, st);
}

template <class Tr>
int launch_op(yk_model* m, const yk_op& op, const uint8_t* frames, int B, float conf, hipStream_t st, int b0 = 0) {
  // images [b0, b0 + B) of the batch
  const yk_model_desc& D = m->desc;
  {
    switch (op.kind) {
      case YK_K_CONV_INPUT: {
        InputArgs a;
        // with a LetterBox resize the frames are already the letterboxed canvas (m->lbox)
        const bool rs = D.rs_mode != 0;
        a.fh = rs ? D.in_h : D.frame_h;
        a.fw = rs ? D.in_w : D.frame_w;
        a.frames = frames + (size_t)b0 * a.fh * a.fw * 3;
        a.pad_top = rs ? 0 : D.pad_top;
        a.pad_left = rs ? 0 : D.pad_left;
        a.in_h = D.in_h;
        a.in_w = D.in_w;
        a.out_h = op.out_h;
        a.out_w = op.out_w;
        a.stride = op.stride;
        a.ksize = op.ksize;
        a.pad = op.ksize / 2;
        a.M = B * op.out_h * op.out_w;
        a.w = (const float*)(m->blob + op.w_off);
        a.b = (const float*)(m->blob + op.b_off);
        a.cout = op.cout;
        a.dst = img_ptr(m, op.dst.buf, op.out_h, op.out_w, op.dst.c_stride, b0);
        a.d_cstride = op.dst.c_stride;
        a.d_coff = op.dst.c_off;
        a.xcd = m->xcd;
        const int tiles = B * ((op.out_h + 15) / 16) * ((op.out_w + 15) / 16);
        if (!Tr::kExact && op.cout <= 32 && !m->input_valu)
          hipLaunchKernelGGL(conv_input_mfma_kernel<Tr>, dim3(tiles), dim3(256), 0, st, a);
        else if (Tr::kExact && op.cout <= 32 && !m->input_valu)
          hipLaunchKernelGGL(conv_input_f32mfma_kernel, dim3(tiles), dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL(conv_input_kernel<Tr>, dim3(tiles), dim3(256), 0, st, a);
        break;
      }
      case YK_K_CONV: {
        ConvArgs a;
        for (int i = 0; i < 2; ++i) a.src[i] = make_view(m, op.src[i < op.n_src ? i : 0], b0);
        a.ksize = op.ksize;
        a.stride = op.stride;
        a.pad = op.ksize / 2;
        a.in_h = op.src[0].h << op.src[0].up;
        a.in_w = op.src[0].w << op.src[0].up;
        a.out_h = op.out_h;
        a.out_w = op.out_w;
        a.M = B * op.out_h * op.out_w;
        a.wpk = (const uint4*)(m->blob + op.w_off);
        a.bias = (const float*)(m->blob + op.b_off);
        a.tab = (const int*)(m->blob + op.t_off);
        a.k_steps = op.k_steps;
        a.n_tiles = op.n_tiles;
        a.n_chunks = op.ksize * op.ksize * (op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0)) / 8;
        a.c0 = op.src_ch[0];
        a.cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
        a.dst = img_ptr(m, op.dst.buf, op.out_h, op.out_w, op.dst.c_stride, b0);
        a.d_cstride = op.dst.c_stride;
        a.d_coff = op.dst.c_off;
        a.cout = op.cout;
        a.res = op.has_res ? img_ptr(m, op.res.buf, op.out_h, op.out_w, op.res.c_stride, b0) : nullptr;
        a.r_cstride = op.res.c_stride;
        a.r_coff = op.res.c_off;
        a.act = op.act;
        const ConvPlan cp = conv_plan(m, op, B);
        const TilePlan& tp = cp.tp;
        if (cp.kind == CK_WIDE) {
          const size_t esz = sizeof(typename Tr::T);
          const int nw = cp.npt == 8 ? 8 : 4;
          const WidePlan wp = wide_plan(op, (int)esz, cp.nnt, nw);
          WideArgs w;
          w.arena = m->arena;
          w.arena_bytes = (unsigned)m->arena_bytes;
          w.soff0 = (unsigned)(((const char*)a.src[0].p - (const char*)m->arena) + (size_t)a.src[0].coff * esz);
          w.soff1 = (unsigned)(((const char*)a.src[1].p - (const char*)m->arena) + (size_t)a.src[1].coff * esz);
          w.h0 = a.src[0].h;
          w.w0 = a.src[0].w;
          w.cs0 = a.src[0].cstride;
          w.up0 = a.src[0].up;
          w.h1 = a.src[1].h;
          w.w1 = a.src[1].w;
          w.cs1 = a.src[1].cstride;
          w.up1 = a.src[1].up;
          w.c0 = a.c0;
          w.cin = a.cin;
          w.stride = a.stride;
          w.pad = a.pad;
          w.in_h = a.in_h;
          w.in_w = a.in_w;
          w.out_h = a.out_h;
          w.out_w = a.out_w;
          w.B = B;
          w.tiles_x = (a.out_w + 15) / 16;
          w.tiles_y = (a.out_h + 15) / 16;
          w.tih = wp.tih;
          w.tiw = wp.tiw;
          w.ps = wp.ps;
          w.wpk = a.wpk;
          w.bias = a.bias;
          w.ltab = m->ltab + m->ltab_off[(size_t)(&op - m->ops.data())];
          w.k_steps = a.k_steps;
          w.n_tiles = a.n_tiles;
          w.dst = a.dst;
          w.d_cstride = a.d_cstride;
          w.d_coff = a.d_coff;
          w.cout = a.cout;
          w.res = a.res;
          w.r_cstride = a.r_cstride;
          w.r_coff = a.r_coff;
          w.act = a.act;
          w.dbg = m->wide_dbg;
          w.xcd = m->xcd;
          if (cp.nnt == 2) {
            if (nw == 8) launch_wide_n<Tr, 2, 8>(w, wp.upt, wp.lds, st);
            else launch_wide_n<Tr, 2, 4>(w, wp.upt, wp.lds, st);
          } else {
            if (nw == 8) launch_wide_n<Tr, 4, 8>(w, wp.upt, wp.lds, st);
            else launch_wide_n<Tr, 4, 4>(w, wp.upt, wp.lds, st);
          }
        } else if (cp.kind == CK_HALO) {
          if constexpr (std::is_same<Tr, F32>::value) {
            const size_t oi = (size_t)(&op - m->ops.data());
            const HaloPlan hp = halo_plan(op, cp.npt & 15, (cp.npt >> 4) & 1);
            HaloArgs h;
            h.arena = m->arena;
            h.arena_bytes = (unsigned)m->arena_bytes;
            h.soff0 = (unsigned)(((const char*)a.src[0].p - (const char*)m->arena) + (size_t)a.src[0].coff * 4);
            h.soff1 = (unsigned)(((const char*)a.src[1].p - (const char*)m->arena) + (size_t)a.src[1].coff * 4);
            h.h0 = a.src[0].h;
            h.w0 = a.src[0].w;
            h.cs0 = a.src[0].cstride;
            h.up0 = a.src[0].up;
            h.h1 = a.src[1].h;
            h.w1 = a.src[1].w;
            h.cs1 = a.src[1].cstride;
            h.up1 = a.src[1].up;
            h.c0 = a.c0;
            h.cin = a.cin;
            h.stride = a.stride;
            h.pad = a.pad;
            h.in_h = a.in_h;
            h.in_w = a.in_w;
            h.out_h = a.out_h;
            h.out_w = a.out_w;
            h.tr = hp.tr;
            h.tc = hp.tc;
            h.twin = hp.twin;
            h.npx = hp.npx;
            h.rp = hp.rp;
            h.hw = hp.hw;
            h.tiles_x = hp.tiles_x;
            h.tiles_y = hp.tiles_y;
            h.wblob = m->wkslot;
            h.wbytes = (unsigned)m->wkslot_bytes;
            h.woff = (unsigned)m->wk_off[oi];
            h.bias = a.bias;
            h.n_tiles = a.n_tiles;
            h.dst = a.dst;
            h.d_cstride = a.d_cstride;
            h.d_coff = a.d_coff;
            h.cout = a.cout;
            h.res = a.res;
            h.r_cstride = a.r_cstride;
            h.r_coff = a.r_coff;
            h.act = a.act;
            h.xcd = m->xcd;
            launch_halo(h, B, cp, op.ksize, st);
          }
        } else if (cp.kind == CK_FAST) {
          FastArgs f;
          const size_t esz = sizeof(typename Tr::T);
          f.arena = m->arena;
          f.arena_bytes = (unsigned)m->arena_bytes;
          f.soff0 = (unsigned)(((const char*)a.src[0].p - (const char*)m->arena) + (size_t)a.src[0].coff * esz);
          f.soff1 = (unsigned)(((const char*)a.src[1].p - (const char*)m->arena) + (size_t)a.src[1].coff * esz);
          f.h0 = a.src[0].h;
          f.w0 = a.src[0].w;
          f.cs0 = a.src[0].cstride;
          f.up0 = a.src[0].up;
          f.h1 = a.src[1].h;
          f.w1 = a.src[1].w;
          f.cs1 = a.src[1].cstride;
          f.up1 = a.src[1].up;
          f.wblob = m->blob;
          f.wbytes = (unsigned)m->blob_bytes;
          f.woff = (unsigned)op.w_off;
          f.stride = a.stride;
          f.pad = a.pad;
          f.in_h = a.in_h;
          f.in_w = a.in_w;
          f.out_h = a.out_h;
          f.out_w = a.out_w;
          f.M = a.M;
          f.inv_hw = 1.0f / (float)(a.out_h * a.out_w);
          f.inv_w = 1.0f / (float)a.out_w;
          f.bias = a.bias;
          f.ktab = m->ktab + m->ktab_off[(size_t)(&op - m->ops.data())];
          f.k_steps = a.k_steps;
          f.n_tiles = a.n_tiles;
          f.dst = a.dst;
          f.d_cstride = a.d_cstride;
          f.d_coff = a.d_coff;
          f.cout = a.cout;
          f.res = a.res;
          f.r_cstride = a.r_cstride;
          f.r_coff = a.r_coff;
          f.act = a.act;
          f.xcd = m->xcd;
          f.tstamp = (m->ts && (int)(&op - m->ops.data()) == m->ts_op) ? m->ts : nullptr;
          f.tstamp_cap = kTsCap;
          f.ipw = m->fast_ipw;
          if constexpr (std::is_same<Tr, F32>::value) {
            if (cp.npt & kSplitBit) {  // split-MFMA body on the bf16-split weights
              f.wblob = m->wsplit;
              f.wbytes = (unsigned)m->wsplit_bytes;
              f.woff = (unsigned)m->ws_off[(size_t)(&op - m->ops.data())];
              launch_fast<F32S>(f, cp, st);
              break;
            }
          }
          launch_fast<Tr>(f, cp, st);
        } else if constexpr (Tr::kScaled) {
          // FP8 runs only on the table-driven and wide kernels (16-channel K chunks)
          yk::set_error("yk_detect: FP8 conv op without a table/wide kernel plan");
          return YK_ERR_ARG;
        } else if (cp.kind == CK_SPLITK) {
          launch_splitk<Tr>(a, cp, st);
        } else if (cp.kind == CK_TILE) {
          TileArgs t;
          t.src[0] = a.src[0];
          t.src[1] = a.src[1];
          t.c0 = op.src_ch[0];
          t.cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
          t.ksize = a.ksize;
          t.stride = a.stride;
          t.pad = a.pad;
          t.in_h = a.in_h;
          t.in_w = a.in_w;
          t.out_h = a.out_h;
          t.out_w = a.out_w;
          t.tiles_x = tp.tiles_x;
          t.tiles_y = tp.tiles_y;
          t.tih = tp.tih;
          t.tiw = tp.tiw;
          t.ps = tp.ps;
          t.wpk = a.wpk;
          t.bias = a.bias;
          t.tab = m->ltab + m->ltab_off[(size_t)(&op - m->ops.data())];
          t.k_steps = a.k_steps;
          t.n_tiles = a.n_tiles;
          t.n_chunks = a.n_chunks;
          t.dst = a.dst;
          t.d_cstride = a.d_cstride;
          t.d_coff = a.d_coff;
          t.cout = a.cout;
          t.res = a.res;
          t.r_cstride = a.r_cstride;
          t.r_coff = a.r_coff;
          t.act = a.act;
          t.single = tp.single ? 1 : 0;
          t.xcd = m->xcd;
          launch_tile<Tr>(t, tp, B, st);
        } else {
          launch_conv<Tr>(a, st);
        }
        break;
      }
      case YK_K_SPPF_POOL: {
        const int M = B * op.src[0].h * op.src[0].w;
        const int C = op.src_ch[0];
        const int HW = op.src[0].h * op.src[0].w;
        void* pb = img_ptr(m, op.src[0].buf, op.src[0].h, op.src[0].w, op.src[0].c_stride, b0);
        if (HW <= kSppfLdsMaxHW && C % 8 == 0) {
          hipLaunchKernelGGL((sppf_lds_kernel<Tr, 8>), dim3(B * (C / 8)), dim3(256), (size_t)HW * 8 * 4 * 4, st, pb,
                             op.src[0].c_stride, op.src[0].c_off, C, op.src[0].h, op.src[0].w);
          break;
        }
        if (HW <= kSppfLdsMaxHW4 && C % 4 == 0) {
          hipLaunchKernelGGL((sppf_lds_kernel<Tr, 4>), dim3(B * (C / 4)), dim3(256), (size_t)HW * 4 * 4 * 4, st, pb,
                             op.src[0].c_stride, op.src[0].c_off, C, op.src[0].h, op.src[0].w);
          break;
        }
        const int n = M * (C / 4);
        hipLaunchKernelGGL(sppf_pool_kernel<Tr>, dim3((n + 255) / 256), dim3(256), 0, st,
                           img_ptr(m, op.src[0].buf, op.src[0].h, op.src[0].w, op.src[0].c_stride, b0),
                           op.src[0].c_stride, op.src[0].c_off, C, op.src[0].h, op.src[0].w, M);
        break;
      }
      case YK_K_DETECT: {
        DetArgs a;
        a.src = make_view(m, op.src[0], b0);
        a.cls_off = op.det_cls_off;
        a.cls_ch = op.det_cls_ch;
        a.wpk = (const uint4*)(m->blob + op.w_off);
        a.bias = (const float*)(m->blob + op.b_off);
        a.k_steps = op.k_steps;
        a.wc = (const float*)(m->blob + op.det_wc_off);
        a.stride = op.det_stride;
        a.anchor_off = op.det_anchor_off;
        a.M = B * op.src[0].h * op.src[0].w;
        a.conf = conf;
        a.cand = m->cand + (size_t)b0 * D.n_anchors * 6;
        a.cand_count = m->cand_count + b0;
        a.cap = D.n_anchors;
        hipLaunchKernelGGL(detect_kernel<Tr>, dim3((a.M + 63) / 64), dim3(256), 0, st, a);
        break;
      }
      default:
        yk::set_error("yk_detect: unknown op kind");
        return YK_ERR_ARG;
    }
  }
  return YK_OK;
}

template <class Tr>
int run_ops(yk_model* m, const uint8_t* frames, int B, float conf, hipStream_t st) {
  for (const yk_op& op : m->ops) {
    const int rc = launch_op<Tr>(m, op, frames, B, conf, st);
    if (rc != YK_OK) return rc;
  }
  return YK_OK;
}

int launch_any(yk_model* m, const yk_op& op, const uint8_t* frames, int B, float conf, hipStream_t st) {
  switch (m->desc.act_dtype) {
    case YK_ACT_F32: return launch_op<F32>(m, op, frames, B, conf, st);
    case YK_ACT_FP8: return launch_op<FP8>(m, op, frames, B, conf, st);
    case YK_ACT_F16: return launch_op<F16>(m, op, frames, B, conf, st);
    default: return launch_op<BF16>(m, op, frames, B, conf, st);
  }
}

// Name of the kernel instantiation an op launches (matches rocprofv3's demangled names).
const char* op_kernel_name(const yk_model* m, const yk_op& op) {
  const int dt = m->desc.act_dtype;
  const bool f = dt == YK_ACT_F32;
  const char* tn = tr_name(dt);  // (F32S for a split-MFMA table conv below)
  static thread_local char buf[96];
  switch (op.kind) {
    case YK_K_CONV_INPUT:
      if (!f && op.cout <= 32 && !m->input_valu) snprintf(buf, sizeof buf, "conv_input_mfma_kernel<yk::det::%s>", tn);
      else if (f && op.cout <= 32 && !m->input_valu) snprintf(buf, sizeof buf, "conv_input_f32mfma_kernel");
      else snprintf(buf, sizeof buf, "conv_input_kernel<yk::det::%s>", tn);
      return buf;
    case YK_K_SPPF_POOL:
      if (op.src[0].h * op.src[0].w <= kSppfLdsMaxHW && op.src_ch[0] % 8 == 0)
        snprintf(buf, sizeof buf, "sppf_lds_kernel<yk::det::%s, 8>", tn);
      else if (op.src[0].h * op.src[0].w <= kSppfLdsMaxHW4 && op.src_ch[0] % 4 == 0)
        snprintf(buf, sizeof buf, "sppf_lds_kernel<yk::det::%s, 4>", tn);
      else
        snprintf(buf, sizeof buf, "sppf_pool_kernel<yk::det::%s>", tn);
      return buf;
    case YK_K_DETECT: snprintf(buf, sizeof buf, "detect_kernel<yk::det::%s>", tn); return buf;
    default: break;
  }
  const ConvPlan cp = conv_plan(m, op, m->plan_batch);
  if (cp.kind == CK_WIDE) {
    const WidePlan wp = wide_plan(op, esz_of(dt), cp.nnt, cp.npt);
    const int upt = wp.upt <= 4 ? 4 : wp.upt <= 8 ? 8 : wp.upt <= 12 ? 12 : 16;
    snprintf(buf, sizeof buf, "conv_wide_kernel<yk::det::%s, %d, %d, %d>", tn, cp.nnt, upt, cp.npt);
    return buf;
  }
  if (cp.kind == CK_HALO) {
    snprintf(buf, sizeof buf, "conv_halo_kernel<%d, %d, %d, %d>", cp.nnt, cp.npt & 15, (cp.npt >> 4) & 1, op.ksize);
    return buf;
  }
  if (cp.kind == CK_FAST) {
    const int npt = cp.npt & 15, mode = (cp.npt >> 4) & 3;
    const int skd = mode == 2 ? fastw_skd(cp.nnt, npt) : fast_skd(cp.nnt, npt);
    if (cp.npt & kSplitBit) tn = "F32S";
    if (mode == 2)
      snprintf(buf, sizeof buf, "conv_fastw_kernel<yk::det::%s, %d, %d, %d>", tn, cp.nnt, npt, skd);
    else
      snprintf(buf, sizeof buf, "conv_fast_kernel<yk::det::%s, %d, %d, %d, %d>", tn, cp.nnt, npt,
               mode == 1 ? 4 : mode == 3 ? 2 : 1, skd);
    return buf;
  }
  if (cp.kind == CK_SPLITK) {
    snprintf(buf, sizeof buf, "conv_splitk_kernel<yk::det::%s, %d, %d>", tn, cp.nnt, cp.npt);
    return buf;
  }
  if (cp.kind == CK_TILE) {
    const TilePlan& tp = cp.tp;
    snprintf(buf, sizeof buf, "conv_tile_kernel<yk::det::%s, %d, %d, %s>", tn, tp.nnt, tp.npt, tp.split ? "true" : "false");
    return buf;
  }
  const int nt = op.n_tiles;
  const int nnt = nt <= 1 ? 1 : nt == 2 ? 2 : (nt == 3 || nt == 6 || nt == 9) ? 3 : 4;
  snprintf(buf, sizeof buf, "conv_igemm_kernel<yk::det::%s, %d, 2>", tn, nnt);
  return buf;
}

int launch_nms(yk_model* m, int B, float iou, int max_det, float* dets, int32_t* counts, hipStream_t st,
               int32_t* keep = nullptr);

// Buffers an op reads and writes.  The candidate list (virtual buffer n_bufs) is appended to
// with atomics by every Detect op, so Detect ops do not order against each other.
void op_access(const yk_model* m, const yk_op& op, std::vector<int>& rd, std::vector<int>& wr) {
  rd.clear();
  wr.clear();
  switch (op.kind) {
    case YK_K_CONV_INPUT: wr.push_back(op.dst.buf); break;
    case YK_K_SPPF_POOL:
      rd.push_back(op.src[0].buf);
      wr.push_back(op.src[0].buf);
      break;
    case YK_K_DETECT:
      for (int i = 0; i < op.n_src; ++i) rd.push_back(op.src[i].buf);
      wr.push_back(m->desc.n_bufs);
      break;
    default:
      for (int i = 0; i < op.n_src; ++i) rd.push_back(op.src[i].buf);
      if (op.has_res) rd.push_back(op.res.buf);
      wr.push_back(op.dst.buf);
      break;
  }
}

// List-schedule the op program onto `lanes` streams per batch group: an op continues the lane
// whose tail is its latest producer (keeps chains on one stream), else takes the lane that went
// idle first.  Groups touch disjoint images of every buffer, so they never order against each
// other; tasks are visited op-major so every group's chain advances together.
void plan_dag(yk_model* m) {
  const int n = (int)m->ops.size(), nb = m->desc.n_bufs + 1, L = m->lanes, G = m->groups;
  m->tasks.clear();
  m->lane_used.assign(G * L, 0);
  m->lane_used[0] = 1;
  std::vector<int> rd, wr;
  std::vector<std::vector<int>> last_w(G, std::vector<int>(nb, -1));
  std::vector<std::vector<std::vector<int>>> readers(G, std::vector<std::vector<int>>(nb));
  std::vector<int> tail(G * L, -1);
  for (int j = 0; j < n; ++j) {
    op_access(m, m->ops[j], rd, wr);
    for (int g = 0; g < G; ++g) {
      const int t = (int)m->tasks.size();
      std::vector<int> deps;
      for (int b : rd)
        if (last_w[g][b] >= 0) deps.push_back(last_w[g][b]);
      for (int b : wr) {
        const bool accum = b == m->desc.n_bufs;
        if (last_w[g][b] >= 0 && !accum) deps.push_back(last_w[g][b]);
        for (int r : readers[g][b]) deps.push_back(r);
      }
      int lane = -1, best = -1;
      for (int l = g * L; l < (g + 1) * L; ++l)
        for (int d : deps)
          if (tail[l] == d && d > best) best = d, lane = l;
      if (lane < 0) {
        lane = g * L;
        for (int l = g * L + 1; l < (g + 1) * L; ++l)
          if (tail[l] < tail[lane]) lane = l;
      }
      yk_model::Task task{j, g, lane, {}, false};
      std::vector<int> latest(G * L, -1);
      for (int d : deps) {
        const int dl = m->tasks[d].lane;
        if (dl != lane && d > latest[dl]) latest[dl] = d;
      }
      for (int l = 0; l < G * L; ++l)
        if (latest[l] >= 0) {
          task.waits.push_back(latest[l]);
          m->tasks[latest[l]].ev = true;
        }
      m->tasks.push_back(task);
      m->lane_used[lane] = 1;
      tail[lane] = t;
      for (int b : rd) readers[g][b].push_back(t);
      for (int b : wr) {
        if (b == m->desc.n_bufs) continue;
        last_w[g][b] = t;
        readers[g][b].clear();
      }
    }
  }
}

template <class Tr>
int run_dag(yk_model* m, const uint8_t* frames, int B, float conf, hipStream_t st) {
  const int G = m->groups, L = G * m->lanes, nt = (int)m->tasks.size();
  if (L <= 1) return run_ops<Tr>(m, frames, B, conf, st);
  int gb0[9], gbn[9];  // images of each group
  for (int g = 0, b0 = 0; g < G; ++g) {
    gbn[g] = B / G + (g < B % G ? 1 : 0);
    gb0[g] = b0;
    b0 += gbn[g];
  }
  auto lane_stream = [&](int l) { return l == 0 ? st : m->aux[l - 1]; };
  const hipEvent_t* ev = m->run_ev ? m->run_ev : m->ev.data();
  hipEvent_t fork = ev[nt];
  YK_HIP(hipEventRecord(fork, st));
  for (int l = 1; l < L; ++l)
    if (m->lane_used[l]) YK_HIP(hipStreamWaitEvent(m->aux[l - 1], fork, 0));
  for (int t = 0; t < nt; ++t) {
    const yk_model::Task& task = m->tasks[t];
    hipStream_t s = lane_stream(task.lane);
    for (int d : task.waits) YK_HIP(hipStreamWaitEvent(s, ev[d], 0));
    if (gbn[task.grp] > 0) {
      const int rc = launch_op<Tr>(m, m->ops[task.op], frames, gbn[task.grp], conf, s, gb0[task.grp]);
      if (rc != YK_OK) return rc;
    }
    if (task.ev) YK_HIP(hipEventRecord(ev[t], s));
  }
  for (int l = 1; l < L; ++l) {
    if (!m->lane_used[l]) continue;
    YK_HIP(hipEventRecord(ev[nt + l], m->aux[l - 1]));
    YK_HIP(hipStreamWaitEvent(st, ev[nt + l], 0));
  }
  return YK_OK;
}

// The network input: the frames themselves, or (LetterBox resize) the letterboxed canvas.
const uint8_t* input_frames(yk_model* m, const uint8_t* frames, int B, hipStream_t st) {
  const yk_model_desc& D = m->desc;
  if (!D.rs_mode) return frames;
  const int* t = (const int*)(m->blob + D.rs_tab_off);
  LboxArgs a;
  a.src = frames;
  a.dst = m->lbox;
  a.fh = D.frame_h;
  a.fw = D.frame_w;
  a.in_h = D.in_h;
  a.in_w = D.in_w;
  a.top = D.pad_top;
  a.left = D.pad_left;
  a.rs_w = D.rs_w;
  a.rs_h = D.rs_h;
  a.mode = D.rs_mode;
  const int W = D.rs_w * 3;  // elements per resized row: 16-byte, then 8-byte SIMD blocks
  int xv = W >= 16 ? W / 16 * 16 : 0;
  while (xv < W - 8) xv += 8;
  a.vec_end = xv;
  a.xofs = t;
  a.yofs = t + D.rs_w;
  a.xw = (const short2*)(t + D.rs_w + D.rs_h);
  a.yw = (const short2*)(t + 2 * D.rs_w + D.rs_h);
  const long n = (long)B * D.in_h * D.in_w;
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(letterbox_kernel, dim3((unsigned)g), dim3(256), 0, st, a, B);
  return m->lbox;
}

int detect_impl(yk_model* m, const uint8_t* frames, int B, float conf, float iou, int max_det, float* dets,
                int32_t* counts, hipStream_t st) {
  const yk_model_desc& D = m->desc;
  YK_CHECK_ARG(frames, "yk_detect: frames is NULL");
  YK_CHECK_ARG(B >= 1 && B <= D.max_batch, "yk_detect: batch out of range [1, max_batch]");
  YK_CHECK_ARG(conf >= 0.f && conf <= 1.f, "Invalid Confidence threshold, valid values are between 0.0 and 1.0");
  YK_CHECK_ARG(iou >= 0.f && iou <= 1.f, "Invalid IoU, valid values are between 0.0 and 1.0");
  YK_CHECK_ARG(max_det >= 0 && max_det <= D.max_det, "yk_detect: max_det exceeds the model's capacity");
  m->plan_batch = (B + m->groups - 1) / m->groups;
  if (!dets) dets = m->dets;
  if (!counts) counts = m->counts;
  // candidate counters of this forward start at 0: a kernel node, not hipMemsetAsync -- a
  // captured memset node was seen to race the detect kernels when the graph was replayed right
  // behind other work on the launch stream (stale counters -> NMS over stale slots)
  hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(64), 0, st, m->cand_count, B);
  YK_HIP(hipGetLastError());
  frames = input_frames(m, frames, B, st);
  int rc = D.act_dtype == YK_ACT_F32   ? run_dag<F32>(m, frames, B, conf, st)
           : D.act_dtype == YK_ACT_FP8 ? run_dag<FP8>(m, frames, B, conf, st)
           : D.act_dtype == YK_ACT_F16 ? run_dag<F16>(m, frames, B, conf, st)
                                       : run_dag<BF16>(m, frames, B, conf, st);
  if (rc != YK_OK) return rc;
  return launch_nms(m, B, iou, max_det, dets, counts, st);
}

int launch_nms(yk_model* m, int B, float iou, int max_det, float* dets, int32_t* counts, hipStream_t st,
               int32_t* keep) {
  const yk_model_desc& D = m->desc;
  NmsArgs a;
  a.cand = m->cand;
  a.cand_count = m->cand_count;
  a.cap = D.n_anchors;
  a.max_nms = 30000;
  a.slot_of = m->slot_of;
  a.gkeys = m->gkeys;
  a.gbox = m->gbox;
  a.gflag = m->gflag;
  a.n_anchors = D.n_anchors;
  a.key_cap = m->key_cap;
  a.iou = iou;
  a.max_det = max_det;
  a.dets = dets;
  a.counts = counts;
  a.pad_x = (float)D.box_pad_x;  // scale_boxes (utils/ops.py:123-138)
  a.pad_y = (float)D.box_pad_y;
  a.gain = D.box_gain;
  a.clip_w = (float)D.frame_w;
  a.clip_h = (float)D.frame_h;
  a.dbg = m->nms_dbg;
  a.keep_out = keep;
  a.stat = m->nms_stat;
  a.err = m->err_dev;
  hipLaunchKernelGGL(nms_kernel, dim3(B), dim3(NMS_NT), nms_lds_bytes(), st, a);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

// conv_fast_kernel tables (see FastArgs): per conv op, per (K step, lane group kg), the element
// offset of the K chunk's (tap, channel) from the pixel's window origin in its source view
// and tap | src << 4 | valid << 5.  K order = model.py Program.pack: (tap, K-space channel).
hipError_t build_ktabs(yk_model* m, bool fast) {
  const int esz = esz_of(m->desc.act_dtype);
  const int epl = 16 / esz;  // K elements per lane per K step
  if (m->arena_bytes >= kArenaMax || m->blob_bytes >= 0x7fff0000ull) fast = false;  // 32-bit offsets
  std::vector<int2> all;
  m->ktab_off.assign(m->ops.size(), -1);
  for (size_t i = 0; i < m->ops.size() && fast; ++i) {
    const yk_op& op = m->ops[i];
    if (op.kind != YK_K_CONV) continue;
    const int k = op.ksize, c0 = op.src_ch[0], cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
    bool ok = (cin % 8) == 0;
    for (int sidx = 0; sidx < op.n_src; ++sidx) ok = ok && (k == 1 || op.src[sidx].up == 0);
    if (!ok) continue;
    const int cq = cin / 8, n_chunks = k * k * cq;
    m->ktab_off[i] = (int64_t)all.size();
    for (int ks = 0; ks < op.k_steps; ++ks)
      for (int kg = 0; kg < 4; ++kg) {
        const int kel = ks * 4 * epl + kg * epl, q = kel >> 3, sub = kel & 7;
        if (q >= n_chunks) {
          all.push_back(make_int2(0, 0));
          continue;
        }
        const int tap = q / cq, c = (q - tap * cq) * 8, ky = tap / k, kx = tap - ky * k;
        const int src = c >= c0 ? 1 : 0, ch = src ? c - c0 : c;
        const yk_view& v = op.src[src < op.n_src ? src : 0];
        const int delta = ((ky * v.w + kx) * v.c_stride + ch + sub) * esz;
        const int bit = k == 3 ? ky * 3 + kx : 0;
        all.push_back(make_int2(delta, bit | (src << 4) | 32));
      }
  }
  // conv_tile_kernel: offsets inside the LDS input tile (row width 15 * stride + k pixels,
  // pixel stride ps = odd number of 16-B units >= cin, as tile_plan_geom)
  std::vector<int> lt;
  m->ltab_off.assign(m->ops.size(), -1);
  for (size_t i = 0; i < m->ops.size(); ++i) {
    const yk_op& op = m->ops[i];
    if (op.kind != YK_K_CONV) continue;
    const int k = op.ksize, cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
    if (cin % 8) continue;
    int U = cin * esz / 16;
    if ((U & 1) == 0) U += 1;
    const int ps = U * 16 / esz, tiw = 15 * op.stride + k;
    const int cq = cin / 8, n_chunks = k * k * cq;
    m->ltab_off[i] = (int64_t)lt.size();
    for (int ks = 0; ks < op.k_steps; ++ks)
      for (int kg = 0; kg < 4; ++kg) {
        const int kel = ks * 4 * epl + kg * epl, q = kel >> 3, sub = kel & 7;
        if (q >= n_chunks) {  // K padding: the packed weights are zero there, so any finite
          lt.push_back(0);    // activation works -- the window origin's first channels
          continue;
        }
        const int tap = q / cq, c = (q - tap * cq) * 8, ky = tap / k, kx = tap - ky * k;
        lt.push_back((ky * tiw + kx) * ps + c + sub);
      }
  }
  hipError_t e = hipSuccess;
  if (!lt.empty()) {
    e = hipMalloc((void**)&m->ltab, lt.size() * sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(m->ltab, lt.data(), lt.size() * sizeof(int), hipMemcpyHostToDevice);
  }
  if (all.empty() || e != hipSuccess) return e;
  e = hipMalloc((void**)&m->ktab, all.size() * sizeof(int2));
  if (e == hipSuccess) e = hipMemcpy(m->ktab, all.data(), all.size() * sizeof(int2), hipMemcpyHostToDevice);
  return e;
}

// host float -> bf16 bits, round-to-nearest-even (finite inputs)
inline unsigned short h_f2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
inline float h_bf2f(unsigned short h) {
  const unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// F32S weight fragments: the packed f32 A-operand fragments of every table-kernel conv ([n_tiles]
// [k_steps][64 lanes][4 f32], model.py Program.pack) as [n_tiles][k_steps][64][32 B]: W01 =
// [w0(e) | w1(e)] for the lane's 4 elements e, then W02 = [w0(e) | w2(e)] (bf16, low half first),
// w = w0 + w1 + w2 exactly.
hipError_t build_wsplit(yk_model* m, const char* host_blob, size_t blob_bytes) {
  m->ws_off.assign(m->ops.size(), -1);
  std::vector<unsigned short> out;
  for (size_t i = 0; i < m->ops.size(); ++i) {
    const yk_op& op = m->ops[i];
    if (op.kind != YK_K_CONV || m->ktab_off.empty() || m->ktab_off[i] < 0) continue;
    const size_t nfrag = (size_t)op.n_tiles * op.k_steps * 64;
    if ((size_t)op.w_off + nfrag * 16 > blob_bytes) continue;
    while ((out.size() * 2) % 256) out.push_back(0);  // 256-byte aligned per op
    m->ws_off[i] = (int64_t)out.size() * 2;
    const float* w = (const float*)(host_blob + op.w_off);
    for (size_t f = 0; f < nfrag; ++f) {
      unsigned short part[3][4];
      for (int e = 0; e < 4; ++e) {
        const float x = w[f * 4 + e];
        part[0][e] = h_f2bf(x);
        const float r1 = x - h_bf2f(part[0][e]);
        part[1][e] = h_f2bf(r1);
        part[2][e] = h_f2bf(r1 - h_bf2f(part[1][e]));
      }
      for (int k : {1, 2})
        for (int e = 0; e < 4; ++e) {
          out.push_back(part[0][e]);
          out.push_back(part[k][e]);
        }
    }
  }
  if (out.empty()) return hipSuccess;
  if (out.size() * 2 >= 0x7fff0000ull) {  // 32-bit buffer offsets
    m->ws_off.assign(m->ops.size(), -1);
    return hipSuccess;
  }
  m->wsplit_bytes = out.size() * 2;
  hipError_t e = hipMalloc((void**)&m->wsplit, m->wsplit_bytes);
  if (e == hipSuccess) e = hipMemcpy(m->wsplit, out.data(), m->wsplit_bytes, hipMemcpyHostToDevice);
  return e;
}

// conv_halo_kernel weights (K-slot layout, see conv_halo_kernel): per conv op with a table (its
// packed f32 fragments [n_tiles][k_steps][64 lanes][4 f32] hold W[co][tap * cin + ch] at step
// kappa / 16, lane (kappa % 16 / 4) * 16 + co % 16, element kappa % 4), the fragments of step
// s = chunk * k*k + tap as [n_tiles][steps][64][A1 | A2 | A3] (48 B): channel ch = 16 chunk +
// 4 kg + e (zero past cin), A1 = [w0(e) x4 | w0(e) x4], A2 = [w1 | w1], A3 = [w2 | w0].
hipError_t build_wkslot(yk_model* m, const char* host_blob, size_t blob_bytes) {
  m->wk_off.assign(m->ops.size(), -1);
  std::vector<unsigned short> out;
  for (size_t i = 0; i < m->ops.size(); ++i) {
    const yk_op& op = m->ops[i];
    if (op.kind != YK_K_CONV || m->ktab_off.empty() || m->ktab_off[i] < 0) continue;
    const int k = op.ksize, cin = op.src_ch[0] + (op.n_src > 1 ? op.src_ch[1] : 0);
    if ((k != 1 && k != 3) || cin % 4 || op.src_ch[0] % 4) continue;
    if ((size_t)op.w_off + (size_t)op.n_tiles * op.k_steps * 64 * 16 > blob_bytes) continue;
    const int T = k * k, nch = (cin + 15) / 16, nsteps = nch * T;
    while ((out.size() * 2) % 256) out.push_back(0);
    m->wk_off[i] = (int64_t)out.size() * 2;
    const float* w = (const float*)(host_blob + op.w_off);
    for (int nt = 0; nt < op.n_tiles; ++nt)
      for (int s = 0; s < nsteps; ++s) {
        const int c = s / T, tap = s - c * T;
        for (int lane = 0; lane < 64; ++lane) {
          const int kg = lane >> 4, col = lane & 15;
          unsigned short part[3][4];
          for (int e = 0; e < 4; ++e) {
            const int ch = 16 * c + 4 * kg + e;
            float x = 0.f;
            if (ch < cin) {
              const int kap = tap * cin + ch, ks = kap >> 4, r = kap & 15;
              x = w[(((size_t)nt * op.k_steps + ks) * 64 + (r >> 2) * 16 + col) * 4 + (r & 3)];
            }
            part[0][e] = h_f2bf(x);
            const float r1 = x - h_bf2f(part[0][e]);
            part[1][e] = h_f2bf(r1);
            part[2][e] = h_f2bf(r1 - h_bf2f(part[1][e]));
          }
          for (int e = 0; e < 4; ++e) out.push_back(part[0][e]);  // A1
          for (int e = 0; e < 4; ++e) out.push_back(part[0][e]);
          for (int e = 0; e < 4; ++e) out.push_back(part[1][e]);  // A2
          for (int e = 0; e < 4; ++e) out.push_back(part[1][e]);
          for (int e = 0; e < 4; ++e) out.push_back(part[2][e]);  // A3
          for (int e = 0; e < 4; ++e) out.push_back(part[0][e]);
        }
      }
  }
  if (out.empty()) return hipSuccess;
  if (out.size() * 2 >= 0x7fff0000ull) {  // 32-bit buffer offsets
    m->wk_off.assign(m->ops.size(), -1);
    return hipSuccess;
  }
  m->wkslot_bytes = out.size() * 2;
  hipError_t e = hipMalloc((void**)&m->wkslot, m->wkslot_bytes);
  if (e == hipSuccess) e = hipMemcpy(m->wkslot, out.data(), m->wkslot_bytes, hipMemcpyHostToDevice);
  return e;
}

// The kernels' host-mapped error word (nms_flag_error): a flagged launch made its images'
// detections empty; the next call on the model reports it (and clears it) as YK_ERR_STATE.
int take_device_error(yk_model* m) {
  if (!m->err_host || !m->err_host[0]) return YK_OK;
  m->err_host[0] = 0;
  yk::set_error("yk_detect: an earlier launch met candidate rows whose anchor index lies outside [0, n_anchors) "
                "(stale or corrupt candidate buffers); those images' detections were dropped");
  return YK_ERR_STATE;
}

void destroy_graph(yk_model::GraphEntry& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  for (hipEvent_t v : g.evs) (void)hipEventDestroy(v);
  g.exec = nullptr;
  g.evs.clear();
}

// Drop every captured forward.  A graph may still be executing (the caller's streams), so the
// device is synchronised first: hipGraphExecDestroy of a graph in flight is not defined here.
void clear_graphs(yk_model* m) {
  if (m->graphs.empty()) return;
  (void)hipDeviceSynchronize();
  for (auto& kv : m->graphs) destroy_graph(kv.second);
  m->graphs.clear();
}

hipError_t set_schedule(yk_model* m, int groups, int lanes) {
  clear_graphs(m);
  for (hipStream_t s : m->aux) (void)hipStreamDestroy(s);
  if (m->cap) (void)hipStreamDestroy(m->cap);
  m->cap = nullptr;
  for (hipEvent_t v : m->ev) (void)hipEventDestroy(v);
  m->aux.clear();
  m->ev.clear();
  m->lanes = lanes;
  m->groups = groups;
  plan_dag(m);
  hipError_t e = hipSuccess;
  for (int l = 1; l < groups * lanes && e == hipSuccess; ++l) {
    hipStream_t s;
    e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) m->aux.push_back(s);
  }
  for (size_t i = 0; i < m->tasks.size() + 1 + (size_t)groups * lanes && e == hipSuccess; ++i) {
    hipEvent_t v;
    e = hipEventCreateWithFlags(&v, hipEventDisableTiming);
    if (e == hipSuccess) m->ev.push_back(v);
  }
  return e;
}

}  // namespace

extern "C" {

int yk_model_create(yk_ctx* ctx, const yk_model_desc* desc, const void* host_blob, int64_t blob_bytes,
                    yk_model** out) {
  YK_CHECK_ARG(ctx && desc && host_blob && out, "yk_model_create: NULL argument");
  if (const int rc = yk::validate_model_desc(desc, blob_bytes)) return rc;  // (yk_host.cpp, host only)
  yk::DeviceGuard guard(ctx->device);
  auto* m = new yk_model();
  m->ctx = ctx;
  m->desc = *desc;
  m->ops.assign(desc->ops, desc->ops + desc->n_ops);
  m->buf_elems.assign(desc->buf_elems, desc->buf_elems + desc->n_bufs);
  m->desc.ops = m->ops.data();
  m->desc.buf_elems = m->buf_elems.data();
  const size_t esz = (size_t)esz_of(desc->act_dtype);
  const size_t B = desc->max_batch, A = desc->n_anchors;
  hipError_t e = hipSuccess;
  auto alloc = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes ? bytes : 16);
  };
  {
    std::vector<size_t> offs;
    size_t total = 0;
    for (int i = 0; i < desc->n_bufs; ++i) {
      offs.push_back(total);
      total += ((size_t)desc->buf_elems[i] * B * esz + 64 + 255) / 256 * 256;
    }
    alloc((void**)&m->arena, total);
    m->arena_bytes = total;
    if (m->arena) (void)hipMemset(m->arena, 0, total);
    for (int i = 0; i < desc->n_bufs; ++i) m->bufs.push_back(m->arena ? m->arena + offs[i] : nullptr);
  }
  alloc((void**)&m->blob, (size_t)blob_bytes);
  if (desc->rs_mode) alloc((void**)&m->lbox, B * (size_t)desc->in_h * desc->in_w * 3);
  m->blob_bytes = (size_t)blob_bytes;
  if (e == hipSuccess) e = hipMemcpy(m->blob, host_blob, (size_t)blob_bytes, hipMemcpyHostToDevice);
  int kc = 1;
  while (kc < (int)A) kc <<= 1;
  m->key_cap = kc;
  alloc((void**)&m->cand, B * A * 6 * sizeof(float));
  alloc((void**)&m->cand_count, B * sizeof(int));
  alloc((void**)&m->slot_of, B * A * sizeof(int));
  alloc((void**)&m->gkeys, B * (size_t)kc * sizeof(unsigned long long));
  alloc((void**)&m->gbox, B * A * 5 * sizeof(float));
  alloc((void**)&m->gflag, B * A);
  alloc((void**)&m->dets, B * desc->max_det * 6 * sizeof(float));
  alloc((void**)&m->counts, B * sizeof(int));
  alloc((void**)&m->nms_stat, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(m->counts, 0, B * sizeof(int));
  if (e == hipSuccess) e = hipMemset(m->nms_stat, 0, 2 * sizeof(int));
  if (e == hipSuccess) {
    void* h = nullptr;
    e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
      m->err_host = (volatile int*)h;
      m->err_host[0] = 0;
      e = hipHostGetDevicePointer((void**)&m->err_dev, h, 0);
    }
  }
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)nms_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)nms_lds_bytes());
  set_tile_attrs();
  if (const char* env = getenv("YK_CONV_DIRECT")) m->tiled = env[0] != '1';
  if (const char* env = getenv("YK_INPUT_VALU")) m->input_valu = env[0] == '1';
  if (const char* env = getenv("YK_XCD")) m->xcd = atoi(env);
  if (const char* env = getenv("YK_WIDE_DBG")) m->wide_dbg = atoi(env);
  if (const char* env = getenv("YK_NMS_DBG")) m->nms_dbg = atoi(env);
  if (const char* env = getenv("YK_NO_WIDE")) m->no_wide = env[0] == '1';
  if (const char* env = getenv("YK_FAST_IPW")) m->fast_ipw = atoi(env) >= 1 ? atoi(env) : 1;
  if (const char* env = getenv("YK_FAST_TS")) {
    m->ts_op = atoi(env);
    if (e == hipSuccess) e = hipMalloc((void**)&m->ts, 3 * (size_t)kTsCap * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(m->ts, 0, 3 * (size_t)kTsCap * sizeof(unsigned long long));
  }
  if (e == hipSuccess) e = build_ktabs(m, !(getenv("YK_CONV_FAST") && getenv("YK_CONV_FAST")[0] == '0'));
  if (const char* env = getenv("YK_F32_SPLIT")) {
    m->split_default = env[0] == '1';
    m->autotune_split = env[0] != '0';
  }
  if (e == hipSuccess && desc->act_dtype == YK_ACT_F32) e = build_wsplit(m, (const char*)host_blob, (size_t)blob_bytes);
  if (e == hipSuccess && desc->act_dtype == YK_ACT_F32) e = build_wkslot(m, (const char*)host_blob, (size_t)blob_bytes);
  if (e == hipSuccess && desc->act_dtype == YK_ACT_FP8)
    for (size_t i = 0; i < m->ops.size(); ++i)
      if (m->ops[i].kind == YK_K_CONV && (m->ktab_off[i] < 0 || m->ops[i].src_ch[0] % 16 ||
                                          (m->ops[i].n_src > 1 && m->ops[i].src_ch[1] % 16))) {
        yk::set_error("yk_model_create: FP8 needs every conv on the table kernel (16-channel sources, arena < 4 GiB)");
        yk_model_destroy(m);
        return YK_ERR_ARG;
      }
  if (e == hipSuccess && YK_STORE_CHECK) {
    sc_register(m->arena, m->arena_bytes);
    sc_register(m->cand, B * A * 6 * sizeof(float));
    sc_register(m->cand_count, B * sizeof(int));
    sc_register(m->slot_of, B * A * sizeof(int));
    sc_register(m->gkeys, B * (size_t)kc * sizeof(unsigned long long));
    sc_register(m->gbox, B * A * 5 * sizeof(float));
    sc_register(m->gflag, B * A);
    sc_register(m->dets, B * desc->max_det * 6 * sizeof(float));
    sc_register(m->counts, B * sizeof(int));
    sc_register(m->nms_stat, 2 * sizeof(int));
    if (m->lbox) sc_register(m->lbox, B * (size_t)desc->in_h * desc->in_w * 3);
  }
  // Default schedule: one lane (the reference's sequential op order on the caller's stream).  A
  // captured graph's parallel branches ran one after another, and the forked capture
  // is the pattern that crashed hipGraphLaunch / a capture in rounds 4-5;
  // YK_LANES=<n> selects a forked schedule for A/B runs, yk_model_set_schedule at run time.
  int lanes0 = 1;
  if (const char* env = getenv("YK_LANES")) lanes0 = atoi(env) >= 1 && atoi(env) <= 8 ? atoi(env) : 1;
  if (e == hipSuccess) e = set_schedule(m, 1, lanes0);
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_model_create: ") + hipGetErrorString(e));
    yk_model_destroy(m);
    return YK_ERR_HIP;
  }
  *out = m;
  return YK_OK;
}

int yk_model_set_lanes(yk_model* m, int lanes) {
  YK_CHECK_ARG(m && lanes >= 1 && lanes <= 8, "yk_model_set_lanes: lanes must be in [1, 8]");
  return yk_model_set_schedule(m, m->groups, lanes);
}

int yk_model_set_schedule(yk_model* m, int groups, int lanes) {
  YK_CHECK_ARG(m && lanes >= 1 && lanes <= 8 && groups >= 1 && groups <= 8 && groups * lanes <= 16,
               "yk_model_set_schedule: need 1 <= groups, lanes <= 8 and groups * lanes <= 16");
  // Several groups each fanned out over several lanes crash hipStreamEndCapture (ROCm 7.2) when
  // the schedule is captured into a graph; each combination on its own captures fine.
  YK_CHECK_ARG(groups == 1 || lanes == 1, "yk_model_set_schedule: groups > 1 needs lanes == 1");
  yk::DeviceGuard guard(m->ctx->device);
  YK_HIP(hipDeviceSynchronize());
  YK_HIP(set_schedule(m, groups, lanes));
  return YK_OK;
}

int yk_model_get_schedule(yk_model* m, int32_t* lane_of, int32_t* n_waits) {
  YK_CHECK_ARG(m && lane_of && n_waits, "yk_model_get_schedule: NULL argument");
  for (size_t i = 0; i < m->tasks.size(); ++i) {
    lane_of[i] = m->tasks[i].lane;
    n_waits[i] = (int32_t)m->tasks[i].waits.size();
  }
  return YK_OK;
}

int yk_model_destroy(yk_model* m) {
  if (!m) return YK_OK;
  yk::DeviceGuard guard(m->ctx->device);
  clear_graphs(m);
  for (hipStream_t s : m->aux) (void)hipStreamDestroy(s);
  if (m->cap) (void)hipStreamDestroy(m->cap);
  for (hipEvent_t v : m->ev) (void)hipEventDestroy(v);
  if (m->arena) (void)hipFree(m->arena);
  void* ptrs[] = {m->blob, m->cand, m->cand_count, m->slot_of, m->gkeys, m->gbox, m->gflag, m->dets, m->counts, m->ktab,
                  m->ltab, m->lbox, m->ts, m->wsplit, m->wkslot, m->nms_stat};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (m->err_host) (void)hipHostFree((void*)m->err_host);
  delete m;
  return YK_OK;
}

int yk_detect(yk_model* m, const uint8_t* frames, int batch, float conf, float iou, int max_det, float* dets,
              int32_t* counts, void* stream) {
  YK_CHECK_ARG(m, "yk_detect: NULL model");
  if (const int rc = take_device_error(m)) return rc;
  yk::DeviceGuard guard(m->ctx->device);
  if (YK_STORE_CHECK && batch >= 1) {
    sc_register(dets, (size_t)batch * max_det * 6 * sizeof(float));
    sc_register(counts, (size_t)batch * sizeof(int));
  }
  return detect_impl(m, frames, batch, conf, iou, max_det, dets, counts, (hipStream_t)stream);
}

int yk_detect_graph(yk_model* m, const uint8_t* frames, int batch, float conf, float iou, int max_det, float* dets,
                    int32_t* counts, void* stream) {
  YK_CHECK_ARG(m, "yk_detect_graph: NULL model");
  if (const int rc = take_device_error(m)) return rc;
  yk::DeviceGuard guard(m->ctx->device);
  if (YK_STORE_CHECK && batch >= 1) {  // (before any capture begins)
    sc_register(dets, (size_t)batch * max_det * 6 * sizeof(float));
    sc_register(counts, (size_t)batch * sizeof(int));
  }
  hipStream_t st = (hipStream_t)stream;
  auto key = std::make_tuple(batch, conf, iou, max_det, (const void*)frames, (void*)dets, (void*)counts);
  auto it = m->graphs.find(key);
  if (it == m->graphs.end()) {
    if (m->graphs.size() >= (size_t)kGraphCap) {  // LRU eviction (after a device sync: clear_graphs)
      auto lru = m->graphs.begin();
      for (auto j = m->graphs.begin(); j != m->graphs.end(); ++j)
        if (j->second.last_use < lru->second.last_use) lru = j;
      YK_HIP(hipDeviceSynchronize());
      destroy_graph(lru->second);
      m->graphs.erase(lru);
    }
    // a forked schedule records its fork / join events into this capture only: a fresh set, owned
    // by the graph entry (destroyed with it), never shared with another capture or with the
    // uncaptured forwards' m->ev
    yk_model::GraphEntry ent;
    if (m->groups * m->lanes > 1) {
      for (size_t i = 0; i < m->ev.size(); ++i) {
        hipEvent_t v;
        const hipError_t ee = hipEventCreateWithFlags(&v, hipEventDisableTiming);
        if (ee != hipSuccess) {
          destroy_graph(ent);
          yk::set_error(std::string("yk_detect_graph: ") + hipGetErrorString(ee));
          return YK_ERR_HIP;
        }
        ent.evs.push_back(v);
      }
    }
    // Capture stream: one per model, kept for the model's lifetime (round 4 created one per
    // capture and destroyed it after hipStreamEndCapture, and multi-lane graphs then crashed in
    // hipGraphLaunch once several models were alive; tools/graph_fork_repro.hip did not reproduce
    // that in either form).  Which stream a graph is captured on moves the launch rate through
    // the streams' hardware-queue mapping, not through the graph: capturing on the launch stream
    // (YK_CAP_STREAM=launch) or on a temporary stream (=destroy) measured 4-11 % slower on the
    // host-frame bench lines with one created stream per slot (gpurun_out/r6i: config 3
    // 4,648-4,658 vs 5,181-5,231 frames/s) and faster only with slot 0 on the legacy null stream
    // at batch 1 (r6e).  The variable is kept for A/B runs.
    const char* cm = getenv("YK_CAP_STREAM");
    const int cap_mode = cm && !strcmp(cm, "destroy") ? 1 : cm && !strcmp(cm, "launch") ? 2 : 0;
    hipStream_t cap = nullptr;
    bool cap_tmp = false;
    if (cap_mode == 2 && stream) {
      cap = (hipStream_t)stream;
    } else if (cap_mode != 0) {
      YK_HIP(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
      cap_tmp = true;
    } else {
      if (!m->cap) YK_HIP(hipStreamCreateWithFlags(&m->cap, hipStreamNonBlocking));
      cap = m->cap;
    }
    hipGraph_t g;
    const bool dbg = getenv("YK_DEBUG_GRAPH") != nullptr;
    const hipError_t be = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    if (be != hipSuccess) {
      destroy_graph(ent);
      if (cap_tmp) (void)hipStreamDestroy(cap);
      yk::set_error(std::string("yk_detect_graph: begin capture: ") + hipGetErrorString(be));
      return YK_ERR_HIP;
    }
    if (dbg) fprintf(stderr, "[yk] capture begun\n");
    m->run_ev = ent.evs.empty() ? nullptr : ent.evs.data();
    int rc = detect_impl(m, frames, batch, conf, iou, max_det, dets, counts, cap);
    m->run_ev = nullptr;
    if (dbg) fprintf(stderr, "[yk] ops recorded rc=%d\n", rc);
    hipError_t ce = hipStreamEndCapture(cap, &g);
    if (dbg) fprintf(stderr, "[yk] capture ended: %s\n", hipGetErrorString(ce));
    if (cap_tmp) (void)hipStreamDestroy(cap);
    if (rc != YK_OK || ce != hipSuccess) {
      if (ce == hipSuccess) (void)hipGraphDestroy(g);
      destroy_graph(ent);
      if (rc != YK_OK) return rc;
      yk::set_error(std::string("yk_detect_graph: capture failed: ") + hipGetErrorString(ce));
      return YK_ERR_HIP;
    }
    hipGraphExec_t ge;
    if (dbg) {
      size_t nn = 0;
      (void)hipGraphGetNodes(g, nullptr, &nn);
      fprintf(stderr, "[yk] graph nodes %zu, instantiating\n", nn);
    }
    hipError_t ie = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (dbg) fprintf(stderr, "[yk] instantiated: %s\n", hipGetErrorString(ie));
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
      destroy_graph(ent);
      yk::set_error(std::string("yk_detect_graph: instantiate failed: ") + hipGetErrorString(ie));
      return YK_ERR_HIP;
    }
    ent.exec = ge;
    it = m->graphs.emplace(key, std::move(ent)).first;
  }
  it->second.last_use = ++m->graph_clock;
  YK_HIP(hipGraphLaunch(it->second.exec, st));
  return YK_OK;
}

int yk_store_check_count(int64_t* out) {
  YK_CHECK_ARG(out, "yk_store_check_count: NULL argument");
#if YK_STORE_CHECK
  unsigned long long v = 0;
  YK_HIP(hipDeviceSynchronize());
  YK_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(sc_bad), 8));
  *out = (int64_t)v;
#else
  *out = -1;  // not a store-check build
#endif
  return YK_OK;
}

int yk_model_graph_count(yk_model* m, int32_t* n_graphs, int32_t* cap) {
  YK_CHECK_ARG(m && n_graphs && cap, "yk_model_graph_count: NULL argument");
  *n_graphs = (int32_t)m->graphs.size();
  *cap = kGraphCap;
  return YK_OK;
}

int yk_model_profile(yk_model* m, const uint8_t* frames, int batch, float conf, float iou, int max_det, int reps,
                     float* host_ms, void* stream) {
  YK_CHECK_ARG(m && frames && host_ms && reps >= 1, "yk_model_profile: bad argument");
  YK_CHECK_ARG(batch >= 1 && batch <= m->desc.max_batch, "yk_model_profile: batch out of range");
  YK_CHECK_ARG(max_det >= 1 && max_det <= m->desc.max_det, "yk_model_profile: max_det out of range");
  yk::DeviceGuard guard(m->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  m->plan_batch = batch;
  frames = input_frames(m, frames, batch, st);
  hipEvent_t e0, e1;
  YK_HIP(hipEventCreate(&e0));
  YK_HIP(hipEventCreate(&e1));
  const int n = (int)m->ops.size();
  for (int i = 0; i <= n; ++i) {
    if (i < n && m->ops[i].kind == YK_K_DETECT) YK_HIP(hipMemsetAsync(m->cand_count, 0, sizeof(int) * batch, st));
    if (i == n) YK_HIP(hipMemsetAsync(m->cand_count, 0, sizeof(int) * batch, st));
    if (i == n) {  // rebuild the candidate lists once so NMS sees a real input
      for (const yk_op& op : m->ops)
        if (op.kind == YK_K_DETECT) {
          int rc = launch_any(m, op, frames, batch, conf, st);
          if (rc != YK_OK) return rc;
        }
    }
    YK_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) {
      int rc = i < n ? launch_any(m, m->ops[i], frames, batch, conf, st)
                     : launch_nms(m, batch, iou, max_det, m->dets, m->counts, st);
      if (rc != YK_OK) return rc;
    }
    YK_HIP(hipEventRecord(e1, st));
    YK_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    YK_HIP(hipEventElapsedTime(&ms, e0, e1));
    host_ms[i] = ms / reps;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return YK_OK;
}

int yk_model_set_plan(yk_model* m, int op_index, int batch, int kind, int nnt, int npt) {
  YK_CHECK_ARG(m && op_index >= -1 && op_index < (int)m->ops.size(), "yk_model_set_plan: bad op index");
  YK_CHECK_ARG(kind >= -1 && kind <= CK_HALO, "yk_model_set_plan: kind must be -1 (heuristic), 0, 1, 2, 3, 4 or 5");
  YK_CHECK_ARG(kind != CK_HALO || (m->wkslot && (nnt == 1 || nnt == 2) &&
                                   ((npt & 15) == 1 || (npt & 15) == 2 || (npt & 15) == 4) && (npt & ~31) == 0),
               "yk_model_set_plan: halo conv (kind 5) needs the fp32 build, nnt in {1, 2}, npt in {1, 2, 4} (+16: "
               "waves split output channels)");
  YK_CHECK_ARG(kind != CK_WIDE || ((nnt == 2 || nnt == 4) && (npt == 0 || npt == 4 || npt == 8)),
               "yk_model_set_plan: wide conv nnt must be 2 or 4, npt (waves) 0, 4 or 8");
  YK_CHECK_ARG(kind != CK_FAST || (nnt >= 1 && nnt <= 4 && ((npt & 15) == 1 || (npt & 15) == 2 || (npt & 15) == 4) &&
                                   (npt & ~(kSplitBit | 63)) == 0),
               "yk_model_set_plan: table conv needs nnt in [1, 4], npt in {1, 2, 4} (+16: waves split K, +32: LDS-shared "
               "weights, +48: wave pairs split K, +64: split-bf16 MFMA)");
  YK_CHECK_ARG(kind != CK_FAST || !(npt & kSplitBit) || m->wsplit,
               "yk_model_set_plan: the split-bf16 MFMA variant (+64) needs the fp32 build");
  YK_CHECK_ARG(kind != CK_TILE || nnt == 0 || nnt == 1, "yk_model_set_plan: tiled conv nnt must be 0 or 1 (LDS-resident weights)");
  YK_CHECK_ARG(kind != CK_SPLITK || ((nnt == 1 || nnt == 2 || nnt == 4) && (npt == 1 || npt == 2 || npt == 4)),
               "yk_model_set_plan: split-K fragment tile must be nnt, npt in {1, 2, 4}");
  YK_CHECK_ARG(batch >= 1 && batch <= m->desc.max_batch, "yk_model_set_plan: batch out of range");
  if (m->tuned.size() != m->ops.size() || m->tuned_batch != batch) m->tuned.assign(m->ops.size(), {-1, 0, 0});
  m->tuned_batch = batch;
  for (int i = 0; i < (int)m->ops.size(); ++i)
    if ((op_index < 0 || i == op_index) && m->ops[i].kind == YK_K_CONV) m->tuned[i] = {kind, nnt, npt};
  clear_graphs(m);
  return YK_OK;
}

int yk_model_get_plan(yk_model* m, int32_t* plan, int32_t* batch) {
  YK_CHECK_ARG(m && plan && batch, "yk_model_get_plan: NULL argument");
  const bool have = m->tuned.size() == m->ops.size();
  *batch = have ? m->tuned_batch : 0;
  for (size_t i = 0; i < m->ops.size(); ++i)
    for (int j = 0; j < 3; ++j) plan[i * 3 + j] = have ? m->tuned[i][j] : (j == 0 ? -1 : 0);
  return YK_OK;
}

int yk_model_autotune(yk_model* m, const uint8_t* frames, int batch, float conf, int reps, void* stream) {
  YK_CHECK_ARG(m && frames && reps >= 1, "yk_model_autotune: bad argument");
  YK_CHECK_ARG(batch >= 1 && batch <= m->desc.max_batch, "yk_model_autotune: batch out of range");
  yk::DeviceGuard guard(m->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  const int n = (int)m->ops.size();
  const int bt = (batch + m->groups - 1) / m->groups;  // the batch each group's kernels run at
  m->tuned.assign(n, {-1, 0, 0});
  m->tuned_batch = bt;
  clear_graphs(m);
  int rc = detect_impl(m, frames, batch, conf, 0.7f, 1, nullptr, nullptr, st);  // valid activations
  if (rc != YK_OK) return rc;
  hipEvent_t e0, e1;
  YK_HIP(hipEventCreate(&e0));
  YK_HIP(hipEventCreate(&e1));
  const int esz = esz_of(m->desc.act_dtype);
  const bool fp8 = m->desc.act_dtype == YK_ACT_FP8;  // table/wide kernels only
  for (int i = 0; i < n; ++i) {
    const yk_op& op = m->ops[i];
    if (op.kind != YK_K_CONV) continue;
    if (op.has_res && op.res.buf == op.dst.buf && op.res.c_off == op.dst.c_off) continue;  // in place
    std::vector<std::array<int, 3>> cands;
    if (!fp8) cands.push_back({CK_DIRECT, 0, 0});
    if (!fp8 && tile_plan(op, esz, bt).ok && m->ltab && m->ltab_off[i] >= 0) {
      cands.push_back({CK_TILE, 0, 0});
      if (tile_plan(op, esz, bt, true).single && !tile_plan(op, esz, bt).single) cands.push_back({CK_TILE, 1, 0});
    }
    for (int nnt : {1, 2, 4})
      for (int npt : {1, 2, 4}) {
        if (fp8 || (nnt > 1 && 4 * op.n_tiles < 3 * ((op.n_tiles + nnt - 1) / nnt) * nnt)) continue;
        cands.push_back({CK_SPLITK, nnt, npt});
      }
    if (m->ltab && m->ltab_off[i] >= 0 && m->arena_bytes < kArenaMax && !m->no_wide)
      for (int nnt : {2, 4}) {
        if (nnt == 4 && op.n_tiles <= 2) continue;
        for (int nw : {4, 8})
          if (wide_plan(op, esz, nnt, nw).ok && (long)bt * op.out_h * op.out_w >= 4096) cands.push_back({CK_WIDE, nnt, nw});
      }
    if (m->ktab && m->ktab_off[i] >= 0 && (long)bt * op.out_h * op.out_w < (1L << 22))
      for (int mode = 0; mode < 4; ++mode)  // per-wave pixels / waves split K / LDS-shared weights / pairs split K
        for (int nnt : {1, 2, 3, 4})
          for (int npt : {1, 2, 4}) {
            if (nnt > 1 && 4 * op.n_tiles < 3 * ((op.n_tiles + nnt - 1) / nnt) * nnt) continue;
            const long px = mode == 1 ? 16 * npt : mode == 3 ? 32 * npt : 64 * npt;
            const long wgs = ((long)bt * op.out_h * op.out_w + px - 1) / px * ((op.n_tiles + nnt - 1) / nnt);
            if (wgs < 64) continue;
            cands.push_back({CK_FAST, nnt, npt | (mode << 4)});
            if (m->wsplit && m->ws_off[i] >= 0 && m->autotune_split)
              cands.push_back({CK_FAST, nnt, npt | (mode << 4) | kSplitBit});
          }
    if (m->wkslot && m->wk_off[i] >= 0 && m->autotune_split)
      for (int wm = 0; wm < 2; ++wm)
        for (int ne : {1, 2})
          for (int npt : {1, 2, 4}) {
            const int per = ne * (wm ? 4 : 1), groups = (op.n_tiles + per - 1) / per;
            if (per > 1 && 4 * op.n_tiles < 3 * groups * per) continue;
            const HaloPlan hp = halo_plan(op, npt, wm);
            if (!hp.ok || (long)bt * hp.tiles_x * hp.tiles_y * groups < 64) continue;
            cands.push_back({CK_HALO, ne, npt | (wm << 4)});
          }
    if (cands.empty()) continue;  // (FP8 without a table: yk_model_create refuses that)
    float best = 1e30f;
    std::array<int, 3> pick = {-1, 0, 0};
    for (const auto& c : cands) {
      m->tuned[i] = c;
      rc = launch_any(m, op, frames, bt, conf, st);  // warm
      if (rc != YK_OK) return rc;
      for (int trial = 0; trial < 3; ++trial) {  // min over trials: robust to clock / queue noise
        YK_HIP(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) {
          rc = launch_any(m, op, frames, bt, conf, st);
          if (rc != YK_OK) return rc;
        }
        YK_HIP(hipEventRecord(e1, st));
        YK_HIP(hipEventSynchronize(e1));
        float ms = 0.f;
        YK_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms, pick = c;
      }
    }
    m->tuned[i] = pick;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return YK_OK;
}

int yk_nms_candidates(yk_model* m, int batch, float iou, int max_det, float* dets, int32_t* counts, int32_t* keep,
                      void* stream) {
  YK_CHECK_ARG(m, "yk_nms_candidates: NULL model");
  YK_CHECK_ARG(batch >= 1 && batch <= m->desc.max_batch, "yk_nms_candidates: batch out of range [1, max_batch]");
  YK_CHECK_ARG(iou >= 0.f && iou <= 1.f, "Invalid IoU, valid values are between 0.0 and 1.0");
  YK_CHECK_ARG(max_det >= 0 && max_det <= m->desc.max_det, "yk_nms_candidates: max_det exceeds the model's capacity");
  if (const int rc = take_device_error(m)) return rc;
  yk::DeviceGuard guard(m->ctx->device);
  if (YK_STORE_CHECK) {
    sc_register(dets, (size_t)batch * max_det * 6 * sizeof(float));
    sc_register(counts, (size_t)batch * sizeof(int));
    sc_register(keep, (size_t)batch * max_det * sizeof(int));
  }
  return launch_nms(m, batch, iou, max_det, dets ? dets : m->dets, counts ? counts : m->counts, (hipStream_t)stream,
                    keep);
}

namespace yk {
namespace det {
// page-locked host -> device copy read by the device (yk_upload_pinned_async): 16 B per lane,
// grid-stride, plain loads of the host pages through their device-mapped address
// four 16-B loads in flight per lane before their stores: a read across PCIe takes microseconds,
// so a few workgroups with deep queues pull as fast as thousands with one load each
__global__ void __launch_bounds__(256) pull_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}
}  // namespace det
}  // namespace yk

int yk_upload_pinned_async(void* dev_dst, const void* host_src, size_t bytes, void* stream) {
  YK_CHECK_ARG(dev_dst && host_src && bytes % 16 == 0 && ((size_t)dev_dst & 15) == 0 && ((size_t)host_src & 15) == 0,
               "yk_upload_pinned_async: NULL pointer, or bytes / addresses not multiples of 16");
  if (bytes == 0) return YK_OK;
  hipPointerAttribute_t at;
  const hipError_t e = hipPointerGetAttributes(&at, host_src);
  if (e != hipSuccess || at.type != hipMemoryTypeHost || !at.devicePointer) {
    (void)hipGetLastError();
    yk::set_error("yk_upload_pinned_async: the source must be page-locked, device-mapped host memory");
    return YK_ERR_ARG;
  }
  const size_t n16 = bytes / 16;
  const unsigned blocks = (unsigned)std::min<size_t>((n16 + 255) / 256, 2048);
  hipLaunchKernelGGL(yk::det::pull_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (uint4*)dev_dst,
                     (const uint4*)at.devicePointer, n16);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_nms(yk_model* m, const float* dev_rows, int row_stride, int max_rows, const int32_t* dev_counts, int batch,
           float iou, int max_det, float* dets, int32_t* counts, int32_t* keep, void* stream) {
  YK_CHECK_ARG(m && dev_rows && dev_counts, "yk_nms: NULL argument");
  YK_CHECK_ARG(row_stride >= 5, "yk_nms: rows need x1 y1 x2 y2 score (row_stride >= 5)");
  YK_CHECK_ARG(max_rows >= 0 && max_rows <= m->desc.n_anchors, "yk_nms: max_rows exceeds the model's candidate capacity");
  YK_CHECK_ARG(batch >= 1 && batch <= m->desc.max_batch, "yk_nms: batch out of range [1, max_batch]");
  // every argument check and a pending device error come before nms_load_kernel overwrites the
  // model's candidate lists (which yk_model_candidates / yk_nms_candidates users may still read)
  YK_CHECK_ARG(iou >= 0.f && iou <= 1.f, "Invalid IoU, valid values are between 0.0 and 1.0");
  YK_CHECK_ARG(max_det >= 0 && max_det <= m->desc.max_det, "yk_nms: max_det exceeds the model's capacity");
  if (const int rc = take_device_error(m)) return rc;
  yk::DeviceGuard guard(m->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  if (max_rows > 0)
    hipLaunchKernelGGL(nms_load_kernel, dim3((max_rows + 255) / 256, batch), dim3(256), 0, st, dev_rows, row_stride,
                       max_rows, dev_counts, m->cand, m->cand_count, m->desc.n_anchors);
  else
    hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(64), 0, st, m->cand_count, batch);
  YK_HIP(hipGetLastError());
  return yk_nms_candidates(m, batch, iou, max_det, dets, counts, keep, stream);
}

int yk_model_nms_stats(yk_model* m, int64_t* out, int reset, void* stream) {
  YK_CHECK_ARG(m && out, "yk_model_nms_stats: NULL argument");
  yk::DeviceGuard guard(m->ctx->device);
  int h[2] = {0, 0};
  YK_HIP(hipStreamSynchronize((hipStream_t)stream));
  YK_HIP(hipMemcpy(h, m->nms_stat, sizeof h, hipMemcpyDeviceToHost));
  out[0] = h[0];
  out[1] = h[1];
  if (reset) YK_HIP(hipMemset(m->nms_stat, 0, sizeof h));
  return YK_OK;
}

int yk_model_check(yk_model* m, void* stream) {
  YK_CHECK_ARG(m, "yk_model_check: NULL model");
  yk::DeviceGuard guard(m->ctx->device);
  YK_HIP(hipStreamSynchronize((hipStream_t)stream));
  return take_device_error(m);
}

int yk_model_op_kernel(yk_model* m, int op_index, char* buf, int len) {
  YK_CHECK_ARG(m && buf && len > 0, "yk_model_op_kernel: bad argument");
  YK_CHECK_ARG(op_index >= 0 && op_index <= (int)m->ops.size(), "yk_model_op_kernel: index out of range");
  const char* nm = op_index == (int)m->ops.size() ? "nms_kernel" : op_kernel_name(m, m->ops[op_index]);
  snprintf(buf, (size_t)len, "%s", nm);
  return YK_OK;
}

int yk_model_outputs(yk_model* m, float** dets, int32_t** counts) {
  YK_CHECK_ARG(m, "yk_model_outputs: NULL model");
  if (dets) *dets = m->dets;
  if (counts) *counts = m->counts;
  return YK_OK;
}

int yk_model_candidates(yk_model* m, float** cand, int32_t** counts) {
  YK_CHECK_ARG(m, "yk_model_candidates: NULL model");
  if (cand) *cand = m->cand;
  if (counts) *counts = m->cand_count;
  return YK_OK;
}

int yk_model_buffer(yk_model* m, int buf, void** ptr) {
  YK_CHECK_ARG(m && ptr, "yk_model_buffer: NULL argument");
  YK_CHECK_ARG(buf >= -2 && buf < (int)m->bufs.size(), "yk_model_buffer: index out of range");
  if (buf == -1) {  // the letterboxed input canvas (NULL when the frames need no resize)
    *ptr = m->lbox;
    return YK_OK;
  }
  if (buf == -2) {  // YK_FAST_TS diagnostics buffer (NULL unless enabled)
    *ptr = m->ts;
    return YK_OK;
  }
  *ptr = m->bufs[buf];
  return YK_OK;
}

}  // extern "C"
