// Global camera-motion detector for gfx950 (MI355X):
// GlobalMotionDetector(method='optical_flow').detect_motion(frame) of
// camera_motion_compensation/global_motion_detector.py:67-169 for n_streams video streams per call.
//
// Per call (frames [S][H][W][3] uint8 BGR resident in HBM):
//   gray_kernel     cvtColor BGR2GRAY, fixed point (R 4899, G 9617, B 1868, >> 14)      (:79, :82)
//   pyrdown_kernel  pyramid levels 1..3 of the new frame ([1 4 6 4 1]^2 / 256, reflect-101)
//   scharr_kernel   Scharr derivatives of every level of the new frame (kept for the next call,
//                   when this frame is the "previous" one, like the stored prev_gray :93-94)
//   -- from the second frame on --
//   eig_kernel      cornerMinEigenVal(prev, blockSize 7, Sobel 3) on 32x32 tiles: Sobel
//                   responses and 7x7 box sums in exact integers through LDS, one float rounding
//                   per covariance entry, per-stream max by an ordered-bits atomicMax
//   cand_kernel     TOZERO threshold at 0.01 * max, 3x3 dilate test, interior local maxima
//                   appended as 64-bit keys (value bits, address) with wave-aggregated atomics
//   select_kernel   one workgroup per stream: keys sorted descending in LDS (bitonic, 2048 at
//                   a time; a radix select cuts larger candidate sets into windows), then the
//                   greedy minDistance-15 pass (1024 candidates tested in parallel against the
//                   kept corners, in-chunk conflicts resolved in order by one wave) to 200 corners
//   lk_kernel       pyramidal Lucas-Kanade, one wavefront per corner: the 21x21 window is 7
//                   pixels per lane in registers, window sums are exact (DPP row sums, then int64)
//   finish_kernel   the reference's numpy post-processing per stream: median, 75th percentile
//                   inliers, float32 mean / norm, thresholds, 3-vector direction consistency,
//                   GlobalMotionDetector.stats
// The OpenCV stages follow OpenCV 4.x's algorithms as restated in oracle/gmd_ref.py (cv2 itself
// is absent, so that restatement is unpinned); these kernels reproduce the restatement bit for
// bit.  Compiled with -ffp-contract=off: every float expression rounds like the C++ / numpy one.
//
// YK_GMD_SPARSE_OPTFLOW (BoT-SORT's GMC, ultralytics/trackers/utils/gmc.py:278-345) runs the same
// stages with the GMC's parameters on the half-resolution gray image -- gray_down_kernel (gray of
// each 2x2 block, then cv2.resize's INTER_AREA fast path (a+b+c+d+2) >> 2), eig_kernel<3>
// (blockSize 3), select_top_kernel (minDistance 1 keeps every local maximum: the 1000 largest keys
// in goodFeaturesToTrack order), lk_kernel -- and gmc_kernel: estimateAffinePartial2D (RANSAC with
// cv::RNG, closed-form 2-point similarity, float32 errors, RANSACUpdateNumIters; then the
// Levenberg-Marquardt refinement) restated in oracle/gmc_ref.py.  Each stream keeps its previous
// frame in the pyramid buffer sel[s]; the new frame goes to sel[s] ^ 1 and sel flips at the end of
// the call (not after a failed GMC estimate, which keeps the previous frame like the reference's
// exception path).
#include <cfloat>
#include <climits>

#include "yk_internal.h"
#include "yk_diag.h"

// Diagnostic builds (csrc/build.py YK_DEFINES="-DYK_GMD_DIAG=<mask>"; the product is 0):
//     1  lk_kernel window sums through LDS (no DPP row sums, no v_readlane)
//     2  system-scope release at the end of the pyramid / derivative producers, acquire at
//        the start of lk_kernel
//     4  lk_kernel solves every corner twice in a row, counting differing answers in info[s][0]
//     8  a second lk_kernel launch re-solves every corner and counts answers differing from the
//        first launch's in info[s][1] (the kernel template's diag bit picks the role)
//    32  the gray pyramids / derivatives in fine-grained device memory (hipDeviceMallocFinegrained)
//    64  the same in uncached device memory (hipDeviceMallocUncached)
//    16  ordering probe: every wave of the pyramid / derivative producers adds 1 to info[0][2] after
//        an agent-scope release; lk_kernel's waves check on entry that every producer wave of
//        this call has (info[0][3] counts the waves that found fewer)
#ifndef YK_GMD_DIAG
#define YK_GMD_DIAG 0
#endif

namespace yk {
namespace gmd {

constexpr int WIN = 21;                      // lk_params winSize
constexpr int WAREA = WIN * WIN;             // 441 window pixels
constexpr int NSLOT = (WAREA + 63) / 64;     // 7 window pixels per lane
constexpr int MAXC = 200;                    // feature_params maxCorners
constexpr int MAXC_G = 1000;                 // GMC feature_params maxCorners (gmc.py:78-80)
constexpr int MINDIST2 = 225;                // minDistance^2 (corners sit on integer pixels)
constexpr int MAXLV = 3;                     // lk_params maxLevel
constexpr int MAXIT = 30;                    // criteria count
constexpr double EPS2 = 0.01 * 0.01;         // criteria eps, squared by calcOpticalFlowPyrLK
constexpr int CAP = 2048;                    // candidate keys select_kernel sorts in LDS per window:
                                             // the greedy pass usually reaches maxCorners inside the
                                             // first window (round 3 sorted 16384 at once)
constexpr int NTS = 1024;                    // select_kernel threads
constexpr int MVQ = 5;                       // motion_vectors deque(maxlen=5)
constexpr float F_PI = 3.14159274101257324f;       // np.pi cast to float32 (NEP 50)
constexpr float F_2PI = 6.28318548202514648f;      // 2 * np.pi cast to float32

struct Geo {
  int W, H, levels;
  int lw[MAXLV + 1], lh[MAXLV + 1];
  long long loff[MAXLV + 1];  // offset of level l inside one stream's pyramid
  long long per;              // pyramid elements per stream
};

struct State {
  int has_prev;  // GlobalMotionDetector: a previous frame is stored (first_frame otherwise)
  int mv_len, mv_head;
  float mv[MVQ][2];
  long long total, motion_events, reset_triggers;
  float avg;
};

struct Dev {
  Geo geo;
  int S;
  unsigned char* pyr[2];   // [2][S][per] gray pyramids, ping-pong between calls
  short2* der[2];          // [2][S][per] Scharr (dx, dy) of every level
  float* eig;              // [S][H*W]
  unsigned* emax;          // [S] ordered bits of max(eig)
  unsigned long long* cand;  // [S][H*W] candidate keys
  int* ncand;              // [S]
  float2* corners;         // [S][MAXC]
  int* ncorners;           // [S]
  float2* next;            // [S][MAXC]
  unsigned char* status;   // [S][MAXC]
  State* st;               // [S]
  yk_motion* out;          // [S]
  float thr_motion, thr_reset, thr_reset_cons;
  int* sel;                // [S] pyramid buffer holding the stream's previous frame
  int mode;                // 0 GlobalMotionDetector, 1 GMC sparseOptFlow
  int maxc;                // corners per stream (MAXC / MAXC_G): stride of corners / next / status
  int W0, H0;              // input frame size (GMC: twice geo.W / geo.H)
  double* warp;            // [S][6] GMC warp
  int* info;               // [S][5] GMC diagnostics (yk_gmc_info)
  int diag_expect;         // YK_GMD_DIAG 16: producer waves launched so far, this call's included
};
// YK_GMD_DIAG 16: one count per producer wave, after its stores are released
#define GMD_PRODUCER_DONE()                                                                       \
  do {                                                                                            \
    if (YK_GMD_DIAG & 16) {                                                                       \
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");                                          \
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(g.info + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    }                                                                                             \
  } while (0)

__device__ __forceinline__ int refl(int i, int n) {  // BORDER_REFLECT_101, |overflow| < n
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}
__device__ __forceinline__ int refl_c(int i, int n) {  // refl, clamped (reads for outputs outside the image)
  i = refl(i, n);
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}
__device__ __forceinline__ unsigned ord_bits(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// Exact wave sum of per-lane int32 values whose 16-lane partial sums stay inside int32 (the LK
// window sums: |per-lane| < 2^27): butterflies within each 16-lane row on DPP (no LDS round
// trips), then the four row sums added in int64 on the scalar unit.  Wave-uniform callers only.
__device__ __forceinline__ long long wave_sum_rows(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1, 0, 3, 2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2, 3, 0, 1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror 4
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror 8
  return ((long long)__builtin_amdgcn_readlane(v, 0) + (long long)__builtin_amdgcn_readlane(v, 16)) +
         ((long long)__builtin_amdgcn_readlane(v, 32) + (long long)__builtin_amdgcn_readlane(v, 48));
}
// Diagnostic twin of wave_sum_rows: the wave's 64 values through the wave's own LDS row, every
// lane adding all of them in int64 (no DPP, no cross-lane register reads).
__device__ __forceinline__ long long wave_sum_lds(int v, int* row) {
  const int lane = threadIdx.x & 63;
  row[lane] = v;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  long long t = 0;
  for (int i = 0; i < 64; ++i) t += row[i];
  __builtin_amdgcn_wave_barrier();
  return t;
}
// The same for per-lane values < 2^28 in magnitude (LK's b1 / b2: |diff| <= 8160, |D| <= 4080, 7
// products per lane), whose 16-lane rows can leave int32: v = hi * 2^16 + lo with lo in [0, 2^16),
// both halves summed exactly by wave_sum_rows, recombined in int64.
__device__ __forceinline__ long long wave_sum_rows_wide(int v) {
  const long long h = wave_sum_rows(v >> 16);
  const long long l = wave_sum_rows(v & 0xffff);
  return h * 65536 + l;
}

// ---------------------------------------------------------------- frame ingest
__device__ __forceinline__ int gray_of(const unsigned char* p) {
  return (p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14;
}
__global__ void __launch_bounds__(256) gray_kernel(Dev g, const unsigned char* __restrict__ frames) {
  const int s = blockIdx.y, cur = g.sel[s] ^ 1;
  const long long n = (long long)g.geo.W * g.geo.H;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const unsigned char* p = frames + ((long long)s * n + i) * 3;
    g.pyr[cur][(long long)s * g.geo.per + i] = (unsigned char)gray_of(p);
    if (YK_GMD_DIAG & 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  GMD_PRODUCER_DONE();
}

// GMC: cvtColor(BGR2GRAY) then cv2.resize(gray, (W / 2, H / 2)): INTER_LINEAR at an exact 1/2
// scale is resize.cpp's INTER_AREA fast path, (a + b + c + d + 2) >> 2 of each 2x2 block
// (gmc.py:296-301; oracle/gmc_ref.py area_down2)
__global__ void __launch_bounds__(256) gray_down_kernel(Dev g, const unsigned char* __restrict__ frames) {
  const int s = blockIdx.y, cur = g.sel[s] ^ 1;
  const int W = g.geo.W, H = g.geo.H, W0 = g.W0;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < (long long)W * H) {
    const int y = (int)(i / W), x = (int)(i - (long long)y * W);
    const unsigned char* f = frames + (long long)s * W0 * g.H0 * 3;
    const unsigned char* r0 = f + ((long long)(2 * y) * W0 + 2 * x) * 3;
    const unsigned char* r1 = r0 + (long long)W0 * 3;
    const int v = gray_of(r0) + gray_of(r0 + 3) + gray_of(r1) + gray_of(r1 + 3);
    g.pyr[cur][(long long)s * g.geo.per + i] = (unsigned char)((v + 2) >> 2);
    if (YK_GMD_DIAG & 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  GMD_PRODUCER_DONE();
}

__global__ void __launch_bounds__(256) pyrdown_kernel(Dev g, int l) {
  const int s = blockIdx.z, cur = g.sel[s] ^ 1;
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int dw = g.geo.lw[l], dh = g.geo.lh[l], sw = g.geo.lw[l - 1], sh = g.geo.lh[l - 1];
  if (x < dw && y < dh) {
  const unsigned char* src = g.pyr[cur] + (long long)s * g.geo.per + g.geo.loff[l - 1];
  const int k[5] = {1, 4, 6, 4, 1};
  int xs[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) xs[j] = refl(2 * x + j - 2, sw);
  int acc = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const unsigned char* row = src + (long long)refl(2 * y + i - 2, sh) * sw;
    int r = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) r += k[j] * row[xs[j]];
    acc += k[i] * r;
  }
  g.pyr[cur][(long long)s * g.geo.per + g.geo.loff[l] + (long long)y * dw + x] = (unsigned char)((acc + 128) >> 8);
  if (YK_GMD_DIAG & 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  GMD_PRODUCER_DONE();
}

// calcSharrDeriv: vertical [3 10 3] / [-1 0 1], then horizontal [-1 0 1] / [3 10 3], reflect-101.
// Every level of every stream in one launch (blockIdx.z = stream * (levels + 1) + level; the
// grid covers level 0, smaller levels' out-of-range tiles return at once).
__global__ void __launch_bounds__(256) scharr_kernel(Dev g) {
  const int nl = g.geo.levels + 1, s = blockIdx.z / nl, l = blockIdx.z - s * nl, cur = g.sel[s] ^ 1;
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int w = g.geo.lw[l], h = g.geo.lh[l];
  if (x >= w || y >= h) return;
  const long long base = (long long)s * g.geo.per + g.geo.loff[l];
  const unsigned char* I = g.pyr[cur] + base;
  const unsigned char* r0 = I + (long long)refl(y - 1, h) * w;
  const unsigned char* r1 = I + (long long)y * w;
  const unsigned char* r2 = I + (long long)refl(y + 1, h) * w;
  const int xm = refl(x - 1, w), xp = refl(x + 1, w);
  auto t0 = [&](int c) { return (r0[c] + r2[c]) * 3 + r1[c] * 10; };
  auto t1 = [&](int c) { return r2[c] - r0[c]; };
  const int dx = t0(xp) - t0(xm);
  const int dy = (t1(xp) + t1(xm)) * 3 + t1(x) * 10;
  g.der[cur][base + (long long)y * w + x] = make_short2((short)dx, (short)dy);
  if (YK_GMD_DIAG & 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// ---------------------------------------------------------------- goodFeaturesToTrack
__global__ void clear_kernel(Dev g) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < g.S) {
    g.emax[s] = 0u;
    g.ncand[s] = 0;
  }
}

// cornerMinEigenVal on an ETS x ETS output tile: the (ETS + BS - 1)^2 Sobel-product halo (box
// radius BS / 2; the products outside the image are those of the reflected pixel, like boxFilter's
// reflect-101 border over the product image), BS-wide horizontal then vertical integer sums.  The
// gray pixels the Sobel taps of those products read -- rows / columns [o - 1, o + ETS + BS) of the
// image, each product at its reflected position with Sobel's own reflect-101 neighbours -- are
// staged in LDS once (coalesced rows), so a product costs LDS reads instead of eight global byte
// loads.  BS = 7: GlobalMotionDetector (global_motion_detector.py:49-55); 3: GMC (gmc.py:78-80).
// ETS 32 (4 outputs a thread): a quarter of the 16 x 16 tiles' workgroups, each paying the same
// load latency and barriers, and 1.4x fewer halo products per output (8 streams of 640x512 on the
// CMC line, rocprofv3: 48.8 -> 34.5 µs; results bit-identical).
constexpr int ETS = 32;
template <int BS>
__global__ void __launch_bounds__(256) eig_kernel(Dev g) {
  constexpr int R = BS / 2, PN = ETS + 2 * R, GN = PN + 2;
  __shared__ int gt[GN][GN + 1];
  __shared__ int pxx[PN][PN + 1], pxy[PN][PN + 1], pyy[PN][PN + 1];
  __shared__ int hxx[PN][ETS + 1], hxy[PN][ETS + 1], hyy[PN][ETS + 1];
  __shared__ unsigned wmax[4];
  const int s = blockIdx.z, W = g.geo.W, H = g.geo.H, tid = threadIdx.x;
  const unsigned char* img = g.pyr[g.sel[s]] + (long long)s * g.geo.per;
  const int ox = blockIdx.x * ETS - R, oy = blockIdx.y * ETS - R;
  const int gy0 = oy - 1, gx0 = ox - 1;  // LDS tile origin (image coordinates)
  for (int i = tid; i < GN * GN; i += 256) {
    const int ry = i / GN, rx = i - ry * GN;
    const int y = gy0 + ry, x = gx0 + rx;
    gt[ry][rx] = (y >= 0 && y < H && x >= 0 && x < W) ? (int)img[(long long)y * W + x] : 0;
  }
  __syncthreads();
  auto cl = [](int v) { return v < 0 ? 0 : (v > GN - 1 ? GN - 1 : v); };  // only outputs outside the image clamp
  for (int i = tid; i < PN * PN; i += 256) {
    const int ry = i / PN, rx = i - ry * PN;
    const int y = refl_c(oy + ry, H), x = refl_c(ox + rx, W);
    const int ya = cl(refl(y - 1, H) - gy0), yb = cl(y - gy0), yc = cl(refl(y + 1, H) - gy0);
    const int xm = cl(refl(x - 1, W) - gx0), xc = cl(x - gx0), xp = cl(refl(x + 1, W) - gx0);
    const int ix = (gt[ya][xp] - gt[ya][xm]) + 2 * (gt[yb][xp] - gt[yb][xm]) + (gt[yc][xp] - gt[yc][xm]);
    const int iy = (gt[yc][xm] + 2 * gt[yc][xc] + gt[yc][xp]) - (gt[ya][xm] + 2 * gt[ya][xc] + gt[ya][xp]);
    pxx[ry][rx] = ix * ix;
    pxy[ry][rx] = ix * iy;
    pyy[ry][rx] = iy * iy;
  }
  __syncthreads();
  for (int i = tid; i < PN * ETS; i += 256) {
    const int ry = i / ETS, cx = i - ry * ETS;
    int a = 0, b = 0, c = 0;
#pragma unroll
    for (int k = 0; k < BS; ++k) {
      a += pxx[ry][cx + k];
      b += pxy[ry][cx + k];
      c += pyy[ry][cx + k];
    }
    hxx[ry][cx] = a;
    hxy[ry][cx] = b;
    hyy[ry][cx] = c;
  }
  __syncthreads();
  const int tx = tid % ETS, ty0 = tid / ETS;
  unsigned m = 0u;
#pragma unroll
  for (int q = 0; q < ETS * ETS / 256; ++q) {
    const int ty = ty0 + q * (256 / ETS);
    int sxx = 0, sxy = 0, syy = 0;
#pragma unroll
    for (int k = 0; k < BS; ++k) {
      sxx += hxx[ty + k][tx];
      sxy += hxy[ty + k][tx];
      syy += hyy[ty + k][tx];
    }
    const int x = blockIdx.x * ETS + tx, y = blockIdx.y * ETS + ty;
    if (x < W && y < H) {
      constexpr double sc = 4.0 * BS * 255.0;
      const double s2 = 1.0 / (sc * sc);  // (1 / (4 * blockSize * 255))^2
      const float cxx = (float)((double)sxx * s2), cxy = (float)((double)sxy * s2), cyy = (float)((double)syy * s2);
      const float a = cxx * 0.5f, c = cyy * 0.5f, d = a - c;
      const float e = (a + c) - sqrtf(d * d + cxy * cxy);
      g.eig[(long long)s * W * H + (long long)y * W + x] = e;
      const unsigned o = ord_bits(e);
      m = o > m ? o : m;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned v = __shfl_xor(m, o);
    m = v > m ? v : m;
  }
  if ((tid & 63) == 0) wmax[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    unsigned b = wmax[0];
    for (int i = 1; i < 4; ++i) b = wmax[i] > b ? wmax[i] : b;
    // the per-stream maximum only grows: a workgroup whose maximum does not exceed a value
    // already there skips the atomic (same-address atomics per stream serialised at L2)
    if (b > __hip_atomic_load(&g.emax[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&g.emax[s], b);
  }
}

// CPX pixels per thread (a workgroup covers 256 * CPX consecutive pixels); the workgroup's
// candidates take one global atomic (per-stream counter), not one per wave.  Same-address
// atomics serialise at L2, so fewer, larger workgroups: 16 pixels a thread = 80 atomics per
// 640x512 stream (4: 320, ~33 µs for 8 streams, round 4 profile).
constexpr int CPX = 16;
__global__ void __launch_bounds__(256) cand_kernel(Dev g) {
  __shared__ int wcnt[4], wbase[4];
  const int s = blockIdx.y, W = g.geo.W, H = g.geo.H, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long HW = (long long)W * H;
  const float thr = (float)((double)unord_bits(g.emax[s]) * 0.01);  // maxVal * qualityLevel
  const float* e = g.eig + s * HW;
  auto T = [&](float v) { return v > thr ? v : 0.0f; };  // THRESH_TOZERO
  bool c[CPX];
  unsigned long long key[CPX];
  int mine = 0;
#pragma unroll
  for (int u = 0; u < CPX; ++u) {
    const long long p = ((long long)blockIdx.x * CPX + u) * 256 + tid;
    c[u] = false;
    key[u] = 0;
    if (p < HW) {
      const int y = (int)(p / W), x = (int)(p - (long long)y * W);
      if (x >= 1 && x <= W - 2 && y >= 1 && y <= H - 2) {
        const float tp = T(e[p]);
        if (tp != 0.0f) {
          float m = tp;  // dilate(3x3) of the thresholded image
#pragma unroll
          for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
              const float v = T(e[p + (long long)dy * W + dx]);
              m = v > m ? v : m;
            }
          c[u] = tp == m;
          key[u] = ((unsigned long long)ord_bits(tp) << 32) | (unsigned)p;
        }
      }
    }
    mine += c[u] ? 1 : 0;
  }
  // workgroup prefix of the candidate counts: lanes, then waves
  int incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wcnt[wave] = incl;
  __syncthreads();
  if (tid == 0) {
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    const int base = tot ? atomicAdd(&g.ncand[s], tot) : 0;
    wbase[0] = base;
    wbase[1] = base + wcnt[0];
    wbase[2] = base + wcnt[0] + wcnt[1];
    wbase[3] = base + wcnt[0] + wcnt[1] + wcnt[2];
  }
  __syncthreads();
  int o = wbase[wave] + incl - mine;
#pragma unroll
  for (int u = 0; u < CPX; ++u)
    if (c[u]) g.cand[s * HW + o++] = key[u];
}

struct SelLds {
  unsigned long long* keys;  // [CAP]
  int* ax;                   // [MAXC]
  int* ay;                   // [MAXC]
  int* cok;                  // [NTS]
  int* cx;                   // [NTS]
  int* cy;                   // [NTS]
  int* hist;                 // [NTS / 64][256]: one histogram per wave (no cross-wave atomics)
  int* misc;                 // [8]
};
__device__ __forceinline__ SelLds carve_sel(char* base) {
  SelLds L;
  L.keys = (unsigned long long*)base;
  base += sizeof(unsigned long long) * CAP;
  L.ax = (int*)base;
  base += 4 * MAXC;
  L.ay = (int*)base;
  base += 4 * MAXC;
  L.cok = (int*)base;
  base += 4 * NTS;
  L.cx = (int*)base;
  base += 4 * NTS;
  L.cy = (int*)base;
  base += 4 * NTS;
  L.hist = (int*)base;
  base += 4 * 256 * (NTS / 64);
  L.misc = (int*)base;
  return L;
}
constexpr size_t SEL_LDS = sizeof(unsigned long long) * CAP + 4 * (2 * MAXC + 3 * NTS + 256 * (NTS / 64) + 8);
enum { S_CNT = 0, S_NA = 1, S_D = 2, S_K = 3, S_REM = 4 };

// Key scans keep KU global loads in flight per thread: one workgroup per stream walks every
// candidate key of its image several times, so each scan is load-latency-bound otherwise.
constexpr int KU = 8;

// The k-th largest key among keys < U (all keys when !has_u): radix select, 8 bits a pass.  The
// candidates of one image share their top digits (similar eigenvalues), so one shared histogram
// would serialise every key of a pass on a single LDS address: each wave counts into its own.
__device__ unsigned long long kth_largest(const unsigned long long* keys, int n, unsigned long long U, bool has_u,
                                          int k, SelLds& L) {
  const int tid = threadIdx.x, wave = tid >> 6;
  constexpr int NW = NTS / 64;
  unsigned long long prefix = 0ull, mask = 0ull;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256 * NW; i += NTS) L.hist[i] = 0;
    __syncthreads();
    for (int i0 = tid; i0 < n; i0 += KU * NTS) {  // KU loads in flight, then their counts
      unsigned long long kk[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) kk[u] = i0 + u * NTS < n ? keys[i0 + u * NTS] : 0ull;
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const unsigned long long key = kk[u];
        if (i0 + u * NTS < n && (!has_u || key < U) && (key & mask) == prefix)
          atomicAdd(&L.hist[wave * 256 + ((key >> shift) & 255)], 1);
      }
    }
    __syncthreads();
    for (int i = tid; i < 256; i += NTS) {
      int c = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) c += L.hist[w * 256 + i];
      L.hist[i] = c;  // (wave 0's own count is read before this thread overwrites it)
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0, d = 255;
      for (; d > 0; --d) {
        if (acc + L.hist[d] >= k) break;
        acc += L.hist[d];
      }
      L.misc[S_D] = d;
      L.misc[S_K] = k - acc;
    }
    __syncthreads();
    const int d = L.misc[S_D];
    k = L.misc[S_K];
    prefix |= (unsigned long long)d << shift;
    mask |= 255ull << shift;
    __syncthreads();
  }
  return prefix;
}

// One workgroup per stream: std::sort by (value desc, address desc), then the greedy
// minDistance pass of goodFeaturesToTrack to maxCorners corners, in corner order.
__global__ void __launch_bounds__(NTS) select_kernel(Dev g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SelLds L = carve_sel(smem);
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W = g.geo.W;
  const long long HW = (long long)W * g.geo.H;
  const unsigned long long* keys = g.cand + s * HW;
  int n = g.ncand[s];
  if (n > HW) n = (int)HW;
  if (tid == 0) L.misc[S_NA] = 0;
  unsigned long long U = 0ull;
  bool has_u = false;
  for (;;) {
    int rem = n;
    if (has_u) {
      if (tid == 0) L.misc[S_REM] = 0;
      __syncthreads();
      int c = 0;
      for (int i0 = tid; i0 < n; i0 += KU * NTS) {
        unsigned long long kk[KU];
#pragma unroll
        for (int u = 0; u < KU; ++u) kk[u] = i0 + u * NTS < n ? keys[i0 + u * NTS] : ~0ull;
#pragma unroll
        for (int u = 0; u < KU; ++u) c += kk[u] < U ? 1 : 0;
      }
      if (c) atomicAdd(&L.misc[S_REM], c);
      __syncthreads();
      rem = L.misc[S_REM];
    }
    const bool last = rem <= CAP;
    const unsigned long long K = last ? 0ull : kth_largest(keys, n, U, has_u, CAP, L);
    if (tid == 0) L.misc[S_CNT] = 0;
    __syncthreads();
    for (int b0 = 0; b0 < n; b0 += KU * NTS) {  // gather the window [K, U)
      unsigned long long kk[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) kk[u] = b0 + u * NTS + tid < n ? keys[b0 + u * NTS + tid] : 0ull;
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const unsigned long long key = kk[u];
        const bool in = b0 + u * NTS + tid < n && (!has_u || key < U) && (last || key >= K);
        const unsigned long long mask = __ballot(in);
        if (mask) {
          const int leader = __ffsll((long long)mask) - 1;
          int b = 0;
          if (lane == leader) b = atomicAdd(&L.misc[S_CNT], __popcll(mask));
          b = __shfl(b, leader);
          if (in) L.keys[b + __popcll(mask & ((1ull << lane) - 1ull))] = key;
        }
      }
    }
    __syncthreads();
    const int m = L.misc[S_CNT];
    int P = 2;
    while (P < m) P <<= 1;
    for (int i = m + tid; i < P; i += NTS) L.keys[i] = 0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)  // bitonic sort, descending
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P; i += NTS) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const unsigned long long a = L.keys[i], b = L.keys[ixj];
            const bool desc = (i & k) == 0;
            if (desc ? a < b : a > b) {
              L.keys[i] = b;
              L.keys[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    // greedy minDistance over the sorted window, NTS candidates per chunk
    for (int base = 0; base < m; base += NTS) {
      const int na0 = L.misc[S_NA];
      if (na0 >= MAXC) break;
      const int i = base + tid;
      int ok = 0, x = 0, y = 0;
      if (i < m) {
        const unsigned a = (unsigned)(L.keys[i] & 0xffffffffull);
        y = (int)(a / (unsigned)W);
        x = (int)(a - (unsigned)y * (unsigned)W);
        ok = 1;
        for (int q = 0; q < na0; ++q) {
          const int dx = x - L.ax[q], dy = y - L.ay[q];
          if (dx * dx + dy * dy < MINDIST2) {
            ok = 0;
            break;
          }
        }
      }
      L.cok[tid] = ok;
      L.cx[tid] = x;
      L.cy[tid] = y;
      __syncthreads();
      if (wave == 0) {  // in-chunk conflicts, in sorted order
        // 64 candidates at a time (lane l holds candidate c0 + l): tested against the corners
        // this chunk accepted so far (LDS, [na0, na)), the conflicts among the 64 as one mask per
        // lane (bit j: an earlier candidate j of the block within minDistance), then the block's
        // greedy decisions on the scalar unit from those masks -- one serial step per candidate
        // that passed, instead of one broadcast-and-ballot round each.
        int na = na0;
        const int cm = m - base < NTS ? m - base : NTS;
        for (int c0 = 0; c0 < cm && na < MAXC; c0 += 64) {
          const int c = c0 + lane;
          bool okc = c < cm && L.cok[c] != 0;
          const int xl = okc ? L.cx[c] : 0, yl = okc ? L.cy[c] : 0;
          bool conflict = false;
          for (int q = na0; q < na; ++q) {
            const int dx = xl - L.ax[q], dy = yl - L.ay[q];
            conflict |= dx * dx + dy * dy < MINDIST2;
          }
          okc = okc && !conflict;
          unsigned long long mk = 0ull;
          for (int j = 0; j < 64; ++j) {
            const int dx = xl - __builtin_amdgcn_readlane(xl, j), dy = yl - __builtin_amdgcn_readlane(yl, j);
            if (j < lane && dx * dx + dy * dy < MINDIST2) mk |= 1ull << j;
          }
          const unsigned mlo = (unsigned)mk, mhi = (unsigned)(mk >> 32);
          unsigned long long todo = __ballot(okc), acc = 0ull;
          int nacc = 0;
          while (todo != 0ull && na + nacc < MAXC) {
            const int b = __ffsll((long long)todo) - 1;
            todo &= todo - 1ull;
            const unsigned long long mb = ((unsigned long long)__builtin_amdgcn_readlane(mhi, b) << 32) |
                                          (unsigned)__builtin_amdgcn_readlane(mlo, b);
            if ((mb & acc) == 0ull) {
              acc |= 1ull << b;
              ++nacc;
            }
          }
          if ((acc >> lane) & 1ull) {
            const int idx = na + __popcll(acc & ((1ull << lane) - 1ull));
            L.ax[idx] = xl;
            L.ay[idx] = yl;
          }
          na += nacc;
        }
        if (lane == 0) L.misc[S_NA] = na;
      }
      __syncthreads();
    }
    __syncthreads();
    if (L.misc[S_NA] >= MAXC || last) break;
    U = K;
    has_u = true;
  }
  __syncthreads();
  const int na = L.misc[S_NA];
  for (int i = tid; i < na; i += NTS) g.corners[s * g.maxc + i] = make_float2((float)L.ax[i], (float)L.ay[i]);
  if (tid == 0) g.ncorners[s] = na;
}

// GMC (minDistance 1): goodFeaturesToTrack's greedy pass keeps every candidate (distinct pixels are
// >= 1 apart; featureselect.cpp tests dx*dx + dy*dy < minDistance^2), so its corners are the
// MAXC_G largest keys in (value desc, address desc) order: the MAXC_G-th largest key by radix
// select, the keys >= it gathered and bitonic-sorted descending in LDS.
__global__ void __launch_bounds__(NTS) select_top_kernel(Dev g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SelLds L = carve_sel(smem);
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int W = g.geo.W;
  const long long HW = (long long)W * g.geo.H;
  const unsigned long long* keys = g.cand + s * HW;
  int n = g.ncand[s];
  if (n > HW) n = (int)HW;
  const bool all = n <= MAXC_G;
  const unsigned long long K = all ? 0ull : kth_largest(keys, n, 0ull, false, MAXC_G, L);
  if (tid == 0) L.misc[S_CNT] = 0;
  __syncthreads();
  for (int b0 = 0; b0 < n; b0 += KU * NTS) {
    unsigned long long kk[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) kk[u] = b0 + u * NTS + tid < n ? keys[b0 + u * NTS + tid] : 0ull;
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const unsigned long long key = kk[u];
      const bool in = b0 + u * NTS + tid < n && (all || key >= K);
      const unsigned long long mask = __ballot(in);
      if (mask) {
        const int leader = __ffsll((long long)mask) - 1;
        int b = 0;
        if (lane == leader) b = atomicAdd(&L.misc[S_CNT], __popcll(mask));
        b = __shfl(b, leader);
        if (in) L.keys[b + __popcll(mask & ((1ull << lane) - 1ull))] = key;
      }
    }
  }
  __syncthreads();
  const int m = L.misc[S_CNT];
  int P = 2;
  while (P < m) P <<= 1;
  for (int i = m + tid; i < P; i += NTS) L.keys[i] = 0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += NTS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = L.keys[i], b = L.keys[ixj];
          const bool desc = (i & k) == 0;
          if (desc ? a < b : a > b) {
            L.keys[i] = b;
            L.keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < m; i += NTS) {
    const unsigned a = (unsigned)(L.keys[i] & 0xffffffffull);
    const int y = (int)(a / (unsigned)W), x = (int)(a - (unsigned)y * (unsigned)W);
    g.corners[s * g.maxc + i] = make_float2((float)x, (float)y);
  }
  if (tid == 0) g.ncorners[s] = m;
}

// ---------------------------------------------------------------- calcOpticalFlowPyrLK
__device__ __forceinline__ void lk_weights(float a, float b, int& w00, int& w01, int& w10, int& w11) {
  const float sc = (float)(1 << 14);
  w00 = (int)rintf(((1.0f - a) * (1.0f - b)) * sc);
  w01 = (int)rintf((a * (1.0f - b)) * sc);
  w10 = (int)rintf(((1.0f - a) * b) * sc);
  w11 = (1 << 14) - w00 - w01 - w10;
}

// One wavefront per corner (4 corners per workgroup); all control flow is wave-uniform.
// (Staging each level's search region in LDS was measured slower: 111 -> 159 µs for 8 streams.)
// (So was a per-wave LDS copy of the 24 x 24 J pixels around the window, restaged when its integer
// position leaves the copy: 70.1 -> 87.9 µs on the CMC line, round 6.)
template <int CHECK>
__global__ void __launch_bounds__(256) lk_kernel(Dev g) {
  const int s = blockIdx.y, lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ int red_lds[(YK_GMD_DIAG & 5) ? 4 : 1][64];
  // diag 4: pass 1's per-iteration record (level, position, weights, J-sample hash), compared by pass 2
  __shared__ long long rec_lds[(YK_GMD_DIAG & 4) ? 4 : 1][(YK_GMD_DIAG & 4) ? (MAXLV + 1) * MAXIT * 3 : 1];
  long long* rec = rec_lds[(YK_GMD_DIAG & 4) ? (threadIdx.x >> 6) : 0];
  int* dred = red_lds[(YK_GMD_DIAG & 5) ? (threadIdx.x >> 6) : 0];
  int nrec = 0, first_diff = -1;
  int* red = dred;
  if (YK_GMD_DIAG & 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if ((YK_GMD_DIAG & 16) && !CHECK && (threadIdx.x & 63) == 0) {
    const int done = __hip_atomic_load(g.info + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done < g.diag_expect) {
      __hip_atomic_fetch_add(g.info + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      printf("[lk order] s %d wave %d: %d of %d producer waves done at entry\n", blockIdx.y,
             (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), done, g.diag_expect);
    }
  }
  auto wsum = [&](int v) { return (YK_GMD_DIAG & 1) ? wave_sum_lds(v, red) : wave_sum_rows(v); };
  auto wsum_wide = [&](int v) { return (YK_GMD_DIAG & 1) ? wave_sum_lds(v, red) : wave_sum_rows_wide(v); };
  if (p >= g.ncorners[s]) return;
  const int prev = g.sel[s], cur = prev ^ 1;
  const Geo& G = g.geo;
  const float2 pt = g.corners[s * g.maxc + p];
  const unsigned char* Ib = g.pyr[prev] + (long long)s * G.per;
  const short2* Db = g.der[prev] + (long long)s * G.per;
  const unsigned char* Jb = g.pyr[cur] + (long long)s * G.per;
  int wy[NSLOT], wx[NSLOT];
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    const int q = lane + 64 * k;
    wy[k] = q < WAREA ? q / WIN : -1;  // -1: no pixel in this slot
    wx[k] = q < WAREA ? q - (q / WIN) * WIN : 0;
  }
  const float half = (float)((WIN - 1) * 0.5);
  const float fs = 1.0f / (float)(1 << 20);
  float2 nxt = pt, nxt0 = pt;
  int status = 1, status0 = 1;
  // diag 4: per-lane rolling hashes of every value the pass loads (I window + derivatives, J
  // samples) and the iterations it ran, to tell a memory difference from a compute difference
  unsigned long long hI = 0, hJ = 0, hI0 = 0, hJ0 = 0;
  int nit = 0, nit0 = 0;
  // diag 4: every wave solves its corner twice in a row and counts a differing second answer
  for (int rep = 0; rep < ((YK_GMD_DIAG & 4) ? 2 : 1); ++rep) {
  if (rep == 1) {
    nxt0 = nxt;
    status0 = status;
    nxt = pt;
    status = 1;
    hI0 = hI;
    hJ0 = hJ;
    nit0 = nit;
    hI = hJ = 0;
    nit = 0;
    nrec = 0;
  }
  for (int l = G.levels; l >= 0; --l) {
    const int cols = G.lw[l], rows = G.lh[l];
    const unsigned char* I = Ib + G.loff[l];
    const short2* D = Db + G.loff[l];
    const unsigned char* J = Jb + G.loff[l];
    const float sc = (float)(1.0 / (double)(1 << l));
    const float px = pt.x * sc, py = pt.y * sc;
    float cx, cy;
    if (l == G.levels) {
      cx = px;
      cy = py;
    } else {
      cx = nxt.x * 2.0f;
      cy = nxt.y * 2.0f;
    }
    nxt = make_float2(cx, cy);
    const float qx = px - half, qy = py - half;
    const int ix = (int)floorf(qx), iy = (int)floorf(qy);
    if (ix < -WIN || ix >= cols || iy < -WIN || iy >= rows) {
      if (l == 0) status = 0;
      continue;
    }
    int w00, w01, w10, w11;
    lk_weights(qx - (float)ix, qy - (float)iy, w00, w01, w10, w11);
    int Iv[NSLOT], Dx[NSLOT], Dy[NSLOT];
    int s11 = 0, s12 = 0, s22 = 0;
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
      Iv[k] = Dx[k] = Dy[k] = 0;
      if (wy[k] >= 0) {
        const int X = ix + wx[k], Y = iy + wy[k];
        const int x0 = refl(X, cols), x1 = refl(X + 1, cols);
        const unsigned char* r0 = I + (long long)refl(Y, rows) * cols;
        const unsigned char* r1 = I + (long long)refl(Y + 1, rows) * cols;
        Iv[k] = (r0[x0] * w00 + r0[x1] * w01 + r1[x0] * w10 + r1[x1] * w11 + 256) >> 9;
        const bool ix0 = X >= 0 && X < cols, ix1 = X + 1 >= 0 && X + 1 < cols;
        const bool iy0 = Y >= 0 && Y < rows, iy1 = Y + 1 >= 0 && Y + 1 < rows;
        // (dx, dy) as one packed int32 load, 0 outside the level.  Round 4 wrote `cond ? D[i] : z`
        // with a local short2 z: the compiler turned that into a select between &D[i] and the
        // address of a stack copy of z, i.e. FLAT loads through a private-aperture pointer (8 bytes
        // of scratch).  Removing that scratch did NOT remove the run-to-run LK differences seen
        // while other kernels ran beside this one ("The camera-motion path with
        // forwards in flight": a wave re-reading the same J addresses within one launch got other
        // bytes; round 6 found no detector store outside the detector's own allocations in that
        // schedule, profiles/r06_lk_store_check_overlap.txt).  The cause is not known; the product
        // never runs these kernels beside a forward (motion windows, pipeline.py).
        const int* Dw = (const int*)D;
        const int e00 = (iy0 && ix0) ? Dw[(long long)Y * cols + X] : 0;
        const int e01 = (iy0 && ix1) ? Dw[(long long)Y * cols + X + 1] : 0;
        const int e10 = (iy1 && ix0) ? Dw[(long long)(Y + 1) * cols + X] : 0;
        const int e11 = (iy1 && ix1) ? Dw[(long long)(Y + 1) * cols + X + 1] : 0;
        auto lo = [](int e) { return (int)(short)(e & 0xffff); };  // short2.x (little endian)
        auto hi = [](int e) { return e >> 16; };                   // short2.y
        Dx[k] = (lo(e00) * w00 + lo(e01) * w01 + lo(e10) * w10 + lo(e11) * w11 + 8192) >> 14;
        Dy[k] = (hi(e00) * w00 + hi(e01) * w01 + hi(e10) * w10 + hi(e11) * w11 + 8192) >> 14;
        if (YK_GMD_DIAG & 4)
          hI = hI * 1000003ull + (unsigned long long)(unsigned)((Iv[k] * 65599 + Dx[k]) * 131 + Dy[k] + l * 7 + k);
        s11 += Dx[k] * Dx[k];
        s12 += Dx[k] * Dy[k];
        s22 += Dy[k] * Dy[k];
      }
    }
    // |Dx|, |Dy| <= 4080 (Scharr of 8-bit pixels): a lane's 7 products < 2^27, a row's 16 < 2^31
    const float A11 = (float)wsum(s11) * fs;
    const float A12 = (float)wsum(s12) * fs;
    const float A22 = (float)wsum(s22) * fs;
    const float Dd = A11 * A22 - A12 * A12;
    const float dd = A11 - A22;
    const float mine = ((A22 + A11) - sqrtf(dd * dd + (4.0f * A12) * A12)) / (float)(2 * WIN * WIN);
    if (mine < 1e-4f || Dd < FLT_EPSILON) {
      if (l == 0) status = 0;
      continue;
    }
    const float Di = 1.0f / Dd;
    int woff[NSLOT];  // the slot's pixel offset from the window origin at this level
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) woff[k] = wy[k] >= 0 ? wy[k] * cols + wx[k] : 0;
    float nx = cx - half, ny = cy - half;
    float pdx = 0.0f, pdy = 0.0f;
    for (int j = 0; j < MAXIT; ++j) {
      const int jx = (int)floorf(nx), jy = (int)floorf(ny);
      if (jx < -WIN || jx >= cols || jy < -WIN || jy >= rows) {
        if (l == 0) status = 0;
        break;
      }
      int v00, v01, v10, v11;
      lk_weights(nx - (float)jx, ny - (float)jy, v00, v01, v10, v11);
      int b1 = 0, b2 = 0;
      if (jx >= 0 && jx + WIN < cols && jy >= 0 && jy + WIN < rows) {  // window and its +1 inside
        const unsigned char* base = J + (long long)jy * cols + jx;
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) {
          if (wy[k] >= 0) {
            const unsigned char* q = base + woff[k];
            const int jv = (q[0] * v00 + q[1] * v01 + q[cols] * v10 + q[cols + 1] * v11 + 256) >> 9;
            if (YK_GMD_DIAG & 4) hJ = hJ * 1000003ull + (unsigned long long)(unsigned)(jv * 31 + j * 7 + l);
            const int diff = jv - Iv[k];
            b1 += diff * Dx[k];
            b2 += diff * Dy[k];
          }
        }
      } else {  // reflect-101 at the border
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) {
          if (wy[k] >= 0) {
            const int X = jx + wx[k], Y = jy + wy[k];
            const int x0 = refl(X, cols), x1 = refl(X + 1, cols);
            const unsigned char* r0 = J + (long long)refl(Y, rows) * cols;
            const unsigned char* r1 = J + (long long)refl(Y + 1, rows) * cols;
            const int jv = (r0[x0] * v00 + r0[x1] * v01 + r1[x0] * v10 + r1[x1] * v11 + 256) >> 9;
            if (YK_GMD_DIAG & 4) hJ = hJ * 1000003ull + (unsigned long long)(unsigned)(jv * 31 + j * 7 + l + 1000);
            const int diff = jv - Iv[k];
            b1 += diff * Dx[k];
            b2 += diff * Dy[k];
          }
        }
      }
      if (YK_GMD_DIAG & 4) {
        ++nit;
        // wave-uniform record of this iteration: position, weights, and a hash of the J samples
        const long long hj = wave_sum_lds((int)(hJ & 0x3fffffffull), dred);
        const long long r0 = ((long long)l << 48) | ((long long)(jy & 0xffff) << 16) | (jx & 0xffff);
        const long long r1 = ((long long)(v00 & 0xffff) << 32) | ((long long)(v01 & 0xffff) << 16) | (v10 & 0xffff);
        if (nrec < (MAXLV + 1) * MAXIT) {
          if (rep == 0) {
            if (lane == 0) {
              rec[nrec * 3] = r0;
              rec[nrec * 3 + 1] = r1;
              rec[nrec * 3 + 2] = hj;
            }
          } else if (first_diff < 0) {
            __builtin_amdgcn_wave_barrier();
            const long long q0 = rec[nrec * 3], q1 = rec[nrec * 3 + 1], q2 = rec[nrec * 3 + 2];
            if (q0 != r0 || q1 != r1 || q2 != hj) {
              first_diff = nrec;
              if (lane == 0)
                printf("[lk iter] s %d p %d: first differing iteration %d (level %d): pass1 pos %llx w %llx hash %llx"
                       " | pass2 pos %llx w %llx hash %llx\n", s, p, nrec, l, q0, q1, q2, r0, r1, hj);
            }
          }
        }
        ++nrec;
      }
      const float fb1 = (float)wsum_wide(b1) * fs;
      const float fb2 = (float)wsum_wide(b2) * fs;
      const float dx = (A12 * fb2 - A22 * fb1) * Di;
      const float dy = (A12 * fb1 - A11 * fb2) * Di;
      nx += dx;
      ny += dy;
      nxt = make_float2(nx + half, ny + half);
      if ((double)dx * (double)dx + (double)dy * (double)dy <= EPS2) break;
      if (j > 0 && fabs((double)(dx + pdx)) < 0.01 && fabs((double)(dy + pdy)) < 0.01) {
        nxt.x -= dx * 0.5f;
        nxt.y -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
  }
  }  // rep
  if (YK_GMD_DIAG & 4) {
    const unsigned long long dI = __ballot(hI != hI0), dJ = __ballot(hJ != hJ0);
    const bool differ = nxt.x != nxt0.x || nxt.y != nxt0.y || status != status0;
    if (lane == 0 && (differ || dI || dJ)) {
      atomicAdd(g.info + s * 5, 1);
      printf("[lk diag] s %d p %d pt (%.3f %.3f): pass1 (%.6f %.6f) st %d it %d | pass2 (%.6f %.6f) st %d it %d | "
             "I-hash lanes differ %016llx J-hash lanes differ %016llx\n",
             s, p, pt.x, pt.y, nxt0.x, nxt0.y, status0, nit0, nxt.x, nxt.y, status, nit, dI, dJ);
    }
  }
  if (CHECK && lane == 0) {  // second launch (diag 8): compare with the first launch's answer
    const float2 f = g.next[s * g.maxc + p];
    if (f.x != nxt.x || f.y != nxt.y || g.status[s * g.maxc + p] != (unsigned char)status)
      atomicAdd(g.info + s * 5 + 1, 1);
    return;
  }
  if (lane == 0) {
    g.next[s * g.maxc + p] = nxt;
    g.status[s * g.maxc + p] = (unsigned char)status;
  }
}

// ---------------------------------------------------------------- the numpy post-processing
// Stable rank of v[i] among v[0..n): its index in an ascending sort.
__device__ __forceinline__ int rank_of(const float* v, int n, int i) {
  const float x = v[i];
  int r = 0;
  for (int j = 0; j < n; ++j) r += (v[j] < x || (v[j] == x && j < i)) ? 1 : 0;
  return r;
}

// The reference's post-processing of one detect_motion call: LK results of (virtual) stream v,
// the detector state S of its stream, the record to *o.  Called by every thread of a workgroup
// (barriers inside); flip: toggle sel[v] (the per-call layout's previous-frame buffer).
__device__ void finish_one(const Dev& g, int v, State& S, yk_motion* __restrict__ o, bool flip) {
  __shared__ float vx[MAXC], vy[MAXC], sx[MAXC], sy[MAXC], dist[MAXC], sd[MAXC];
  __shared__ int wcnt[4];
  __shared__ int hv[2];
  const int tid = threadIdx.x;
  if (tid == 0) {  // read once before thread 0 sets has_prev below: every wave takes the same branch
    hv[0] = S.has_prev;
    hv[1] = g.ncorners[v];
  }
  __syncthreads();
  if (!hv[0]) {  // first frame: only stored (:77-80)
    if (tid == 0) {
      yk_motion r{};
      r.valid = 1;
      r.first_frame = 1;
      r.consistency = -1.0f;
      *o = r;
      S.has_prev = 1;
      if (flip) g.sel[v] ^= 1;  // this frame is the next call's previous one
    }
    __syncthreads();
    return;
  }
  const int n = hv[1];
  // status == 1 compaction in corner order (n <= 200 < 256 threads)
  int flag = 0;
  float mvx = 0.0f, mvy = 0.0f;
  if (tid < n && n >= 20 && g.status[v * g.maxc + tid]) {
    flag = 1;
    const float2 a = g.corners[v * g.maxc + tid], b = g.next[v * g.maxc + tid];
    mvx = b.x - a.x;  // next_points - prev_points (:140)
    mvy = b.y - a.y;
  }
  const unsigned long long bm = __ballot(flag);
  if ((tid & 63) == 0) wcnt[tid >> 6] = __popcll(bm);
  __syncthreads();
  int pos = __popcll(bm & ((1ull << (tid & 63)) - 1ull));
  int ng = 0;
  for (int w = 0; w < 4; ++w) {
    if (w < (tid >> 6)) pos += wcnt[w];
    ng += wcnt[w];
  }
  if (flag) {
    vx[pos] = mvx;
    vy[pos] = mvy;
  }
  __syncthreads();
  const bool est = n >= 20 && ng >= 10;  // (:118, :132; ng >= 10 > 8 makes :143 hold)
  float mx = 0.0f, my = 0.0f;
  if (est) {
    if (tid < ng) {
      sx[rank_of(vx, ng, tid)] = vx[tid];
      sy[rank_of(vy, ng, tid)] = vy[tid];
    }
    __syncthreads();
    if (ng & 1) {  // np.median(axis=0)
      mx = sx[ng >> 1];
      my = sy[ng >> 1];
    } else {
      mx = (sx[(ng >> 1) - 1] + sx[ng >> 1]) / 2.0f;
      my = (sy[(ng >> 1) - 1] + sy[ng >> 1]) / 2.0f;
    }
    if (tid < ng) {
      const float ex = vx[tid] - mx, ey = vy[tid] - my;
      dist[tid] = sqrtf(ex * ex + ey * ey);  // np.linalg.norm(axis=1)
    }
    __syncthreads();
    if (tid < ng) sd[rank_of(dist, ng, tid)] = dist[tid];
    __syncthreads();
  }
  if (tid == 0) {
    yk_motion r{};
    r.valid = 1;
    r.consistency = -1.0f;
    r.n_corners = n;
    r.n_tracked = n >= 20 ? ng : 0;
    if (est) {
      // np.percentile(distances, 75), linear: lerp in float32 at virtual index 0.75 * (ng - 1)
      const double vi = 0.75 * (double)(ng - 1);
      const int lo = (int)floor(vi);
      const int hi = lo + 1 < ng ? lo + 1 : ng - 1;
      const float t = (float)(vi - (double)lo);
      const float a = sd[lo], b = sd[hi], df = b - a;
      const float p75 = t >= 0.5f ? b - df * (1.0f - t) : a + df * t;
      int ni = 0;
      float gx = 0.0f, gy = 0.0f;
      for (int i = 0; i < ng; ++i)
        if (dist[i] < p75) {  // np.mean(motion_vectors[inliers], axis=0): float32, in order
          if (ni == 0) {
            gx = vx[i];
            gy = vy[i];
          } else {
            gx += vx[i];
            gy += vy[i];
          }
          ++ni;
        }
      r.n_inliers = ni;
      if (ni > 5) {
        gx = gx / (float)ni;
        gy = gy / (float)ni;
        const float mag = sqrtf(gx * gx + gy * gy);
        int pos2;  // motion_vectors.append (deque maxlen 5)
        if (S.mv_len < MVQ) {
          pos2 = S.mv_head + S.mv_len;
          if (pos2 >= MVQ) pos2 -= MVQ;
          ++S.mv_len;
        } else {
          pos2 = S.mv_head;
          S.mv_head = S.mv_head + 1 == MVQ ? 0 : S.mv_head + 1;
        }
        S.mv[pos2][0] = gx;
        S.mv[pos2][1] = gy;
        bool is_motion = mag > g.thr_motion;
        bool should_reset = mag > g.thr_reset;
        if (S.mv_len >= 3) {  // _calculate_motion_consistency(last 3) (:241-261)
          float ang[3];
          for (int k = 0; k < 3; ++k) {
            int q = S.mv_head + S.mv_len - 3 + k;
            if (q >= MVQ) q -= MVQ;
            ang[k] = (float)atan2((double)S.mv[q][1], (double)S.mv[q][0]);
          }
          float dsum = 0.0f;
          for (int k = 1; k < 3; ++k) {
            float d = fabsf(ang[k] - ang[k - 1]);
            if (d > F_PI) d = F_2PI - d;
            dsum = k == 1 ? d : dsum + d;
          }
          const float c = 1.0f - (dsum / 2.0f) / F_PI;
          const float cons = c > 0.0f ? c : 0.0f;
          r.consistency = cons;
          if (cons > 0.7f && is_motion) should_reset = should_reset || mag > g.thr_reset_cons;
        }
        r.is_motion = is_motion;
        r.should_reset = should_reset;
        r.magnitude_kind = 1;
        r.magnitude = mag;
        r.vector[0] = gx;
        r.vector[1] = gy;
      }
    }
    // GlobalMotionDetector.stats (:96-109)
    S.total += 1;
    S.motion_events += r.is_motion;
    S.reset_triggers += r.should_reset;
    S.avg = (S.avg * (float)(S.total - 1) + r.magnitude) / (float)S.total;
    *o = r;
    if (flip) g.sel[v] ^= 1;
  }
  __syncthreads();  // the shared arrays and S are reused by the caller's next call
}

__global__ void __launch_bounds__(256) finish_kernel(Dev g, yk_motion* __restrict__ out) {
  const int s = blockIdx.x;
  finish_one(g, s, g.st[s], out + s, true);
}

// Window mode (yk_gmd_detect_window): n steps of S streams as n * S virtual streams v = w S + s,
// each a (previous, new) frame pair; the post-processing steps every stream's state through its
// n records in frame order.
__global__ void __launch_bounds__(256) finish_window_kernel(Dev g, int n, int S_real, yk_motion* __restrict__ out) {
  const int s = blockIdx.x;
  for (int w = 0; w < n; ++w) finish_one(g, w * S_real + s, g.st[s], out + w * S_real + s, false);
}

// ---------------------------------------------------------------- GMC: estimateAffinePartial2D
// oracle/gmc_ref.py restates OpenCV 4.x ptsetreg.cpp / levmarq.cpp; this kernel reproduces that
// restatement operation for operation (-ffp-contract=off).  One workgroup per stream: thread 0
// runs the sequential parts (cv::RNG, the 2-point kernel, the RANSAC bookkeeping, the 4x4 LM
// solves), every thread the per-point work; sums over points use lane_sum's order (lane t adds
// points t, t + 256, ... in turn, then a pairwise tree over the 256 lanes).
constexpr int GT = 256;
constexpr unsigned long long RNG_COEFF = 4164903690ull;

__device__ __forceinline__ unsigned rng_next(unsigned long long& st) {
  st = (unsigned long long)(unsigned)st * RNG_COEFF + (unsigned)(st >> 32);
  return (unsigned)st;
}
__device__ __forceinline__ int rng_uniform(unsigned long long& st, int a, int b) {
  return a == b ? a : (int)(rng_next(st) % (unsigned)(b - a) + (unsigned)a);
}

// RANSACUpdateNumIters (pow(x, 2) of a double is x * x correctly rounded, as glibc's pow)
__device__ int ransac_update_num_iters(double p, double ep, int max_iters) {
  p = p < 0.0 ? 0.0 : (p > 1.0 ? 1.0 : p);
  ep = ep < 0.0 ? 0.0 : (ep > 1.0 ? 1.0 : ep);
  double num = 1.0 - p;
  num = num > DBL_MIN ? num : DBL_MIN;
  const double q = 1.0 - ep;
  double denom = 1.0 - q * q;
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  if (denom >= 0 || -num >= (double)max_iters * (-denom)) return max_iters;
  return (int)rint(num / denom);
}

// Cholesky solve of a 4x4 SPD system in oracle/gmc_ref.py chol_solve4's order
__device__ void chol_solve4(const double A[4][4], const double* b, double* x) {
  double L[4][4] = {};
  for (int j = 0; j < 4; ++j) {
    double sj = A[j][j];
    for (int k = 0; k < j; ++k) sj = sj - L[j][k] * L[j][k];
    L[j][j] = sj > 0.0 ? sqrt(sj) : __builtin_nan("");
    for (int i = j + 1; i < 4; ++i) {
      double si = A[i][j];
      for (int k = 0; k < j; ++k) si = si - L[i][k] * L[j][k];
      L[i][j] = si / L[j][j];
    }
  }
  double y[4];
  for (int i = 0; i < 4; ++i) {
    double si = b[i];
    for (int k = 0; k < i; ++k) si = si - L[i][k] * y[k];
    y[i] = si / L[i][i];
  }
  for (int i = 3; i >= 0; --i) {
    double si = y[i];
    for (int k = i + 1; k < 4; ++k) si = si - L[k][i] * x[k];
    x[i] = si / L[i][i];
  }
}

// lane_sum of NQ per-thread partials: red[q][GT] in LDS, pairwise tree; result in red[q][0]
template <int NQ>
__device__ __forceinline__ void tree_reduce(double (*red)[GT]) {
  for (int o = GT / 2; o >= 1; o >>= 1) {
    __syncthreads();
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < NQ; ++q) red[q][threadIdx.x] = red[q][threadIdx.x] + red[q][threadIdx.x + o];
  }
  __syncthreads();
}

enum { G_GO = 0, G_GOOD = 1, G_RECOMP = 2, G_N = 3 };

__global__ void __launch_bounds__(GT) gmc_kernel(Dev g, double* __restrict__ out) {
  __shared__ float fx[MAXC_G], fy[MAXC_G], tx[MAXC_G], ty[MAXC_G];  // tracked points; then the inliers first
  __shared__ double red[9][GT];
  __shared__ double xs[4], xds[4];  // LM parameters (a, b, tx, ty): current / trial
  __shared__ float F[6];
  __shared__ int wcnt[GT / 64], misc[8];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  State& S = g.st[s];
  double H[6] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0};
  int state = 0, npts = 0, max_good = 0, rit = 0, lit = 0;
  bool flip = true;
  // has_prev / ncorners read once, by one thread, before anything of this launch writes them: thread 0
  // sets has_prev at the end, and every wave must take the same branch (the RANSAC / LM loops below are
  // driven by LDS words only thread 0 writes)
  if (tid == 0) {
    misc[G_N] = S.has_prev;
    misc[G_N + 1] = g.ncorners[s];
  }
  __syncthreads();
  const bool have = misc[G_N] && misc[G_N + 1] > 0;  // gmc.py:306-311 (first frame / no previous keypoints)
  if (have) {
    // the points with status 1, in corner order (gmc.py:317-324)
    const int n = misc[G_N + 1];
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += GT) {
      const int i = c0 + tid;
      const int f = i < n && g.status[s * g.maxc + i] ? 1 : 0;
      const unsigned long long bm = __ballot(f);
      if (lane == 0) wcnt[wave] = __popcll(bm);
      __syncthreads();
      int pos = base + __popcll(bm & ((1ull << lane) - 1ull)), tot = 0;
      for (int w = 0; w < GT / 64; ++w) {
        pos += w < wave ? wcnt[w] : 0;
        tot += wcnt[w];
      }
      if (f) {
        const float2 a = g.corners[s * g.maxc + i], b = g.next[s * g.maxc + i];
        fx[pos] = a.x;
        fy[pos] = a.y;
        tx[pos] = b.x;
        ty[pos] = b.y;
      }
      base += tot;
      __syncthreads();
    }
    npts = base;
    state = 2;  // "not enough matching points": the identity (gmc.py:327-336)
  }
  if (have && npts > 4) {
    // ---- RANSACPointSetRegistrator::run (modelPoints 2, threshold 3, confidence 0.99, 2000 iterations)
    const float thr = (float)(3.0 * 3.0);
    unsigned long long rng = ~0ull;  // RNG((uint64)-1)
    int niters = 2000;
    double M[6] = {0, 0, 0, 0, 0, 0}, best[6] = {0, 0, 0, 0, 0, 0};
    for (;;) {
      if (tid == 0) {
        misc[G_GO] = rit < niters;
        if (rit < niters) {
          const int i0 = rng_uniform(rng, 0, npts);
          int i1 = rng_uniform(rng, 0, npts);
          while (i1 == i0) i1 = rng_uniform(rng, 0, npts);
          // AffinePartial2DEstimatorCallback::runKernel
          const double x1 = fx[i0], y1 = fy[i0], x2 = fx[i1], y2 = fy[i1];
          const double X1 = tx[i0], Y1 = ty[i0], X2 = tx[i1], Y2 = ty[i1];
          const double d = 1. / ((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2));
          const double S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2));
          const double S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2));
          const double S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2));
          const double S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2));
          M[0] = S0; M[1] = -S1; M[2] = S2; M[3] = S1; M[4] = S0; M[5] = S3;
          for (int k = 0; k < 6; ++k) F[k] = (float)M[k];
        }
      }
      __syncthreads();
      if (!misc[G_GO]) break;
      int c = 0;  // findInliers: err <= thr^2 (float32 error, computeError)
      for (int i = tid; i < npts; i += GT) {
        const float a = F[0] * fx[i] + F[1] * fy[i] + F[2] - tx[i];
        const float b = F[3] * fx[i] + F[4] * fy[i] + F[5] - ty[i];
        c += (a * a + b * b) <= thr ? 1 : 0;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
      if (lane == 0) wcnt[wave] = c;
      __syncthreads();
      if (tid == 0) {
        int good = 0;
        for (int w = 0; w < GT / 64; ++w) good += wcnt[w];
        if (good > (max_good > 1 ? max_good : 1)) {
          for (int k = 0; k < 6; ++k) best[k] = M[k];
          max_good = good;
          niters = ransac_update_num_iters(0.99, (double)(npts - good) / npts, niters);
        }
        ++rit;
      }
      __syncthreads();
    }
    if (tid == 0) {
      misc[G_GOOD] = max_good;
      for (int k = 0; k < 6; ++k) F[k] = (float)best[k];
      xs[0] = best[0];  // Hvec = (H[0], H[3], H[2], H[5]) (ptsetreg.cpp estimateAffinePartial2D)
      xs[1] = best[3];
      xs[2] = best[2];
      xs[3] = best[5];
    }
    __syncthreads();
    max_good = misc[G_GOOD];
    if (max_good <= 0) {
      state = 3;  // cv2 returns None: the identity, the previous frame kept
      flip = false;
    } else {
      state = 1;
      // compressElems: the best model's inliers first, in order (the mask recomputed from it)
      float ix[4], iy[4], jx[4], jy[4];
      int mine[4];
      const int nchunk = (npts + GT - 1) / GT;
      for (int k = 0; k < nchunk; ++k) {
        const int i = k * GT + tid;
        mine[k] = 0;
        if (i < npts) {
          ix[k] = fx[i];
          iy[k] = fy[i];
          jx[k] = tx[i];
          jy[k] = ty[i];
          const float a = F[0] * fx[i] + F[1] * fy[i] + F[2] - tx[i];
          const float b = F[3] * fx[i] + F[4] * fy[i] + F[5] - ty[i];
          mine[k] = (a * a + b * b) <= thr ? 1 : 0;
        }
      }
      __syncthreads();
      int nin = 0;
      for (int k = 0; k < nchunk; ++k) {
        const unsigned long long bm = __ballot(mine[k]);
        if (lane == 0) wcnt[wave] = __popcll(bm);
        __syncthreads();
        int pos = nin + __popcll(bm & ((1ull << lane) - 1ull)), tot = 0;
        for (int w = 0; w < GT / 64; ++w) {
          pos += w < wave ? wcnt[w] : 0;
          tot += wcnt[w];
        }
        if (mine[k]) {
          fx[pos] = ix[k];
          fy[pos] = iy[k];
          tx[pos] = jx[k];
          ty[pos] = jy[k];
        }
        nin += tot;
        __syncthreads();
      }
      // ---- LMSolverImpl::run on (a, b, tx, ty), 10 iterations, eps FLT_EPSILON
      // normal(x): J^T J, J^T r, |r|^2 and max |r| at xs, summed in lane_sum order
      auto normal = [&](const double* h) {
        double q[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = tid; i < nin; i += GT) {
          const double Mx = fx[i], My = fy[i];
          const double rx = ((h[0] * Mx - h[1] * My) + h[2]) - (double)tx[i];
          const double ry = ((h[1] * Mx + h[0] * My) + h[3]) - (double)ty[i];
          q[0] = q[0] + (Mx * Mx + My * My);
          q[1] = q[1] + Mx;
          q[2] = q[2] + My;
          q[3] = q[3] + (Mx * rx + My * ry);
          q[4] = q[4] + ((-My) * rx + Mx * ry);
          q[5] = q[5] + rx;
          q[6] = q[6] + ry;
          q[7] = q[7] + (rx * rx + ry * ry);
          q[8] = fmax(q[8], fmax(fabs(rx), fabs(ry)));
        }
        for (int k = 0; k < 9; ++k) red[k][tid] = q[k];
        for (int o = GT / 2; o >= 1; o >>= 1) {
          __syncthreads();
          if (tid < o) {
            for (int k = 0; k < 8; ++k) red[k][tid] = red[k][tid] + red[k][tid + o];
            red[8][tid] = fmax(red[8][tid], red[8][tid + o]);
          }
        }
        __syncthreads();
      };
      auto sumsq = [&](const double* h) {  // |r|^2 at h
        double q = 0.0;
        for (int i = tid; i < nin; i += GT) {
          const double Mx = fx[i], My = fy[i];
          const double rx = ((h[0] * Mx - h[1] * My) + h[2]) - (double)tx[i];
          const double ry = ((h[1] * Mx + h[0] * My) + h[3]) - (double)ty[i];
          q = q + (rx * rx + ry * ry);
        }
        red[0][tid] = q;
        tree_reduce<1>(red);
      };
      double A[4][4], v[4], D[4], Sc = 0.0, rinf = 0.0, lam = 1.0, lc = 0.75;
      const double nd = (double)nin;
      auto take = [&]() {  // thread 0: A, v, S, max |r| from the reduction
        const double sxx = red[0][0], sx = red[1][0], sy = red[2][0];
        const double a[4][4] = {{sxx, 0.0, sx, sy}, {0.0, sxx, -sy, sx}, {sx, -sy, nd, 0.0}, {sy, sx, 0.0, nd}};
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) A[i][j] = a[i][j];
        for (int k = 0; k < 4; ++k) v[k] = red[3 + k][0];
        rinf = red[8][0];
      };
      normal(xs);
      if (tid == 0) {
        take();
        Sc = red[7][0];
        for (int i = 0; i < 4; ++i) D[i] = A[i][i];
      }
      for (;;) {
        double d[4];
        if (tid == 0) {
          double Ap[4][4];
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) Ap[i][j] = A[i][j];
          for (int i = 0; i < 4; ++i) Ap[i][i] = Ap[i][i] + lam * D[i];
          chol_solve4(Ap, v, d);
          for (int k = 0; k < 4; ++k) xds[k] = xs[k] - d[k];
        }
        __syncthreads();
        sumsq(xds);
        if (tid == 0) {
          const double Sd = red[0][0];
          double temp[4];
          for (int i = 0; i < 4; ++i)
            temp[i] = (A[i][0] * d[0] + A[i][1] * d[1] + A[i][2] * d[2] + A[i][3] * d[3]) * -1.0 + 2.0 * v[i];
          const double dS = d[0] * temp[0] + d[1] * temp[1] + d[2] * temp[2] + d[3] * temp[3];
          const double R = (Sc - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1.0);
          if (R > 0.75) {
            lam *= 0.5;
            if (lam < lc) lam = 0.0;
          } else if (R < 0.25) {
            const double t = d[0] * v[0] + d[1] * v[1] + d[2] * v[2] + d[3] * v[3];
            double nu = (Sd - Sc) / (fabs(t) > DBL_EPSILON ? t : 1.0) + 2.0;
            nu = fmin(fmax(nu, 2.0), 10.0);
            if (lam == 0.0) {
              double mx = DBL_EPSILON;
              for (int i = 0; i < 4; ++i) {
                double e[4] = {0.0, 0.0, 0.0, 0.0}, c[4];
                e[i] = 1.0;
                chol_solve4(A, e, c);
                mx = fmax(mx, fabs(c[i]));
              }
              lam = lc = 1.0 / mx;
              nu *= 0.5;
            }
            lam *= nu;
          }
          misc[G_RECOMP] = Sd < Sc;
          if (Sd < Sc) {
            Sc = Sd;
            for (int k = 0; k < 4; ++k) xs[k] = xds[k];
          }
        }
        __syncthreads();
        if (misc[G_RECOMP]) {
          normal(xs);
          if (tid == 0) take();
        }
        if (tid == 0) {
          ++lit;
          double dinf = 0.0;
          for (int k = 0; k < 4; ++k) dinf = fmax(dinf, fabs(d[k]));
          misc[G_GO] = lit < 10 && dinf >= (double)FLT_EPSILON && rinf >= (double)FLT_EPSILON;
        }
        __syncthreads();
        if (!misc[G_GO]) break;
      }
      if (tid == 0) {  // H = [[a, -b, tx], [b, a, ty]], translation scaled back by the downscale 2
        H[0] = xs[0];
        H[1] = -xs[1];
        H[2] = xs[2] * 2.0;
        H[3] = xs[1];
        H[4] = xs[0];
        H[5] = xs[3] * 2.0;
      }
    }
  }
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) out[s * 6 + k] = H[k];
    int* inf = g.info + s * 5;
    inf[0] = npts;
    inf[1] = max_good;
    inf[2] = rit;
    inf[3] = lit;
    inf[4] = state;
    S.has_prev = 1;
    if (flip) g.sel[s] ^= 1;
  }
}

__global__ void state_reset_kernel(Dev g, int stats_only) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.S) return;
  State& S = g.st[s];
  if (!stats_only) {
    S.has_prev = 0;
    g.ncorners[s] = 0;
    g.sel[s] = 0;
    S.mv_len = S.mv_head = 0;
    yk_motion r{};
    r.consistency = -1.0f;
    g.out[s] = r;
  }
  S.total = S.motion_events = S.reset_triggers = 0;
  S.avg = 0.0f;
}

}  // namespace gmd
}  // namespace yk

using yk::gmd::Dev;

// Window mode (yk_gmd_detect_window): up to kWindow steps per launch sequence, as kWindow * S
// virtual streams v = w S + s.  Pyramids / derivatives of the previous frame (slot 0) and of the
// window's frames (slots 1 .. n) are laid out [slot][S][per], so the per-call kernels, run with
// pyr[0] / der[0] at slot 0 and pyr[1] / der[1] at slot 1 and every sel[v] = 0, read virtual stream
// v's previous frame from slot w and write its new one to slot w + 1; the last new frame is copied
// back to slot 0 for the next window.
constexpr int kWindow = 8;
struct GmdWindow {
  unsigned char* pyr = nullptr;  // [kWindow + 1][S][per]
  short2* der = nullptr;         // [kWindow + 1][S][per]
  float* eig = nullptr;
  unsigned* emax = nullptr;
  unsigned long long* cand = nullptr;
  int *ncand = nullptr, *ncorners = nullptr, *sel = nullptr, *info = nullptr;
  float2 *corners = nullptr, *next = nullptr;
  unsigned char* status = nullptr;
  yk_motion* out = nullptr;  // [kWindow][S]
};

struct yk_gmd {
  yk_ctx* ctx;
  Dev dev;
  long long frames;
  int calls_single = 0, calls_window = 0;  // the two layouts keep the previous frame differently
  GmdWindow win;
};

extern "C" {

int yk_gmd_create(yk_ctx* ctx, int n_streams, int height, int width, int method, yk_gmd** out) {
  YK_CHECK_ARG(ctx && out, "yk_gmd_create: NULL argument");
  YK_CHECK_ARG(n_streams >= 1 && n_streams <= 65535, "yk_gmd_create: n_streams out of range");
  YK_CHECK_ARG(height >= 32 && width >= 32 && (long long)height * width <= (1ll << 28),
               "yk_gmd_create: frame size out of range (32 .. 2^28 pixels)");
  YK_CHECK_ARG(method == YK_GMD_OPTICAL_FLOW || method == YK_GMD_FEATURE_MATCHING || method == YK_GMD_HYBRID ||
                   method == YK_GMD_SPARSE_OPTFLOW,
               "yk_gmd_create: unknown motion detection method");
  YK_CHECK_ARG(method == YK_GMD_OPTICAL_FLOW || method == YK_GMD_SPARSE_OPTFLOW,
               "yk_gmd_create: 'feature_matching' / 'hybrid' (ORB + RANSAC homography) are not built; use "
               "'optical_flow'");
  const bool gmc = method == YK_GMD_SPARSE_OPTFLOW;
  YK_CHECK_ARG(!gmc || (height % 2 == 0 && width % 2 == 0 && height >= 64 && width >= 64),
               "yk_gmd_create: GMC sparseOptFlow needs even frame sizes >= 64 (the 1/2 area downscale)");
  yk::DeviceGuard guard(ctx->device);
  auto* g = new yk_gmd{};
  g->ctx = ctx;
  Dev& d = g->dev;
  d.S = n_streams;
  d.mode = gmc ? 1 : 0;
  d.maxc = gmc ? yk::gmd::MAXC_G : yk::gmd::MAXC;
  d.W0 = width;
  d.H0 = height;
  yk::gmd::Geo& G = d.geo;
  G.W = gmc ? width / 2 : width;  // the GMC works on the downscaled gray image (gmc.py:300-301)
  G.H = gmc ? height / 2 : height;
  width = G.W;
  height = G.H;
  // buildOpticalFlowPyramid: stop before a level whose size would be <= winSize
  G.levels = 0;
  G.lw[0] = width;
  G.lh[0] = height;
  while (G.levels < yk::gmd::MAXLV) {
    const int w2 = (G.lw[G.levels] + 1) / 2, h2 = (G.lh[G.levels] + 1) / 2;
    if (w2 <= yk::gmd::WIN || h2 <= yk::gmd::WIN) break;
    ++G.levels;
    G.lw[G.levels] = w2;
    G.lh[G.levels] = h2;
  }
  long long off = 0;
  for (int l = 0; l <= G.levels; ++l) {
    G.loff[l] = off;
    off += (long long)G.lw[l] * G.lh[l];
  }
  G.per = off;
  d.thr_motion = 30.0f;
  d.thr_reset = 50.0f;
  d.thr_reset_cons = (float)(30.0 * 1.5);
  const size_t S = n_streams, HW = (size_t)width * height;
  hipError_t e = hipSuccess;
  auto A = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  auto AP = [&](void** p, size_t bytes) {  // the pyramid buffers (diag 64: uncached memory)
    if (e != hipSuccess) return;
    e = (YK_GMD_DIAG & 64)   ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached)
        : (YK_GMD_DIAG & 32) ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained)
                             : hipMalloc(p, bytes);
  };
  for (int i = 0; i < 2; ++i) {
    AP((void**)&d.pyr[i], S * G.per);
    AP((void**)&d.der[i], S * G.per * sizeof(short2));
  }
  A((void**)&d.eig, S * HW * sizeof(float));
  A((void**)&d.emax, S * sizeof(unsigned));
  A((void**)&d.cand, S * HW * sizeof(unsigned long long));
  A((void**)&d.ncand, S * sizeof(int));
  A((void**)&d.corners, S * d.maxc * sizeof(float2));
  A((void**)&d.ncorners, S * sizeof(int));
  A((void**)&d.next, S * d.maxc * sizeof(float2));
  A((void**)&d.status, S * d.maxc);
  A((void**)&d.st, S * sizeof(yk::gmd::State));
  A((void**)&d.out, S * sizeof(yk_motion));
  A((void**)&d.sel, S * sizeof(int));
  A((void**)&d.warp, S * 6 * sizeof(double));
  A((void**)&d.info, S * 5 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(d.info, 0, S * 5 * sizeof(int));
  if (e == hipSuccess) e = hipMemset(d.ncorners, 0, S * sizeof(int));
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_gmd_create: hipMalloc failed: ") + hipGetErrorString(e));
    yk_gmd_destroy(g);
    return YK_ERR_HIP;
  }
  if (hipFuncSetAttribute((const void*)yk::gmd::select_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)yk::gmd::SEL_LDS) != hipSuccess ||
      hipFuncSetAttribute((const void*)yk::gmd::select_top_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)yk::gmd::SEL_LDS) != hipSuccess)
    (void)hipGetLastError();
  int rc = yk_gmd_reset(g, nullptr);
  if (rc != YK_OK) {
    yk_gmd_destroy(g);
    return rc;
  }
  YK_HIP(hipDeviceSynchronize());
  *out = g;
  return YK_OK;
}

int yk_gmd_destroy(yk_gmd* g) {
  if (!g) return YK_OK;
  yk::DeviceGuard guard(g->ctx->device);
  Dev& d = g->dev;
  GmdWindow& w = g->win;
  void* ptrs[] = {d.pyr[0], d.pyr[1], d.der[0], d.der[1], d.eig, d.emax, d.cand, d.ncand, d.corners,
                  d.ncorners, d.next, d.status, d.st, d.out, d.sel, d.warp, d.info,
                  w.pyr, w.der, w.eig, w.emax, w.cand, w.ncand, w.ncorners, w.sel, w.info, w.corners,
                  w.next, w.status, w.out};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete g;
  return YK_OK;
}

int yk_gmd_reset(yk_gmd* g, void* stream) {
  YK_CHECK_ARG(g, "yk_gmd_reset: NULL detector");
  yk::DeviceGuard guard(g->ctx->device);
  hipLaunchKernelGGL(yk::gmd::state_reset_kernel, dim3((g->dev.S + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     g->dev, 0);
  YK_HIP(hipGetLastError());
  g->frames = 0;
  g->calls_single = g->calls_window = 0;
  return YK_OK;
}

int yk_gmd_reset_stats(yk_gmd* g, void* stream) {
  YK_CHECK_ARG(g, "yk_gmd_reset_stats: NULL detector");
  yk::DeviceGuard guard(g->ctx->device);
  hipLaunchKernelGGL(yk::gmd::state_reset_kernel, dim3((g->dev.S + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     g->dev, 1);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_gmd_set_thresholds(yk_gmd* g, double global_motion_threshold, double reset_motion_threshold) {
  YK_CHECK_ARG(g, "yk_gmd_set_thresholds: NULL detector");
  g->dev.thr_motion = (float)global_motion_threshold;
  g->dev.thr_reset = (float)reset_motion_threshold;
  g->dev.thr_reset_cons = (float)(global_motion_threshold * 1.5);
  return YK_OK;
}

// the stages both methods share: new frame's gray pyramid + derivatives, then (from the second
// frame on) corners of the previous frame and their Lucas-Kanade flow to the new one
static void gmd_front(yk_gmd* g, const uint8_t* frames, hipStream_t st) {
  Dev& d = g->dev;
  const yk::gmd::Geo& G = d.geo;
  const int S = d.S;
  const long long HW = (long long)G.W * G.H;
  if (d.mode)
    hipLaunchKernelGGL(yk::gmd::gray_down_kernel, dim3((unsigned)((HW + 255) / 256), S), dim3(256), 0, st, d, frames);
  else
    hipLaunchKernelGGL(yk::gmd::gray_kernel, dim3((unsigned)((HW + 255) / 256), S), dim3(256), 0, st, d, frames);
  if (YK_GMD_DIAG & 16) d.diag_expect += (int)((HW + 255) / 256) * S * 4;
  for (int l = 1; l <= G.levels; ++l) {
    hipLaunchKernelGGL(yk::gmd::pyrdown_kernel, dim3((G.lw[l] + 15) / 16, (G.lh[l] + 15) / 16, S), dim3(256), 0, st,
                       d, l);
    if (YK_GMD_DIAG & 16) d.diag_expect += ((G.lw[l] + 15) / 16) * ((G.lh[l] + 15) / 16) * S * 4;
  }
  hipLaunchKernelGGL(yk::gmd::scharr_kernel, dim3((G.lw[0] + 15) / 16, (G.lh[0] + 15) / 16, S * (G.levels + 1)),
                     dim3(256), 0, st, d);
  if (g->frames > 0) {
    hipLaunchKernelGGL(yk::gmd::clear_kernel, dim3((S + 255) / 256), dim3(256), 0, st, d);
    if (d.mode)
      hipLaunchKernelGGL(yk::gmd::eig_kernel<3>, dim3((G.W + yk::gmd::ETS - 1) / yk::gmd::ETS, (G.H + yk::gmd::ETS - 1) / yk::gmd::ETS, S),
                         dim3(256), 0, st, d);
    else
      hipLaunchKernelGGL(yk::gmd::eig_kernel<7>, dim3((G.W + yk::gmd::ETS - 1) / yk::gmd::ETS, (G.H + yk::gmd::ETS - 1) / yk::gmd::ETS, S),
                         dim3(256), 0, st, d);
    hipLaunchKernelGGL(yk::gmd::cand_kernel, dim3((unsigned)((HW + 256 * yk::gmd::CPX - 1) / (256 * yk::gmd::CPX)), S),
                       dim3(256), 0, st, d);
    if (d.mode)
      hipLaunchKernelGGL(yk::gmd::select_top_kernel, dim3(S), dim3(yk::gmd::NTS), yk::gmd::SEL_LDS, st, d);
    else
      hipLaunchKernelGGL(yk::gmd::select_kernel, dim3(S), dim3(yk::gmd::NTS), yk::gmd::SEL_LDS, st, d);
    hipLaunchKernelGGL(yk::gmd::lk_kernel<0>, dim3(d.maxc / 4, S), dim3(256), 0, st, d);
    if (YK_GMD_DIAG & 8) hipLaunchKernelGGL(yk::gmd::lk_kernel<1>, dim3(d.maxc / 4, S), dim3(256), 0, st, d);
  }
}

int yk_gmd_detect(yk_gmd* g, const uint8_t* frames, yk_motion* out, void* stream) {
  YK_CHECK_ARG(g && frames, "yk_gmd_detect: NULL argument");
  YK_CHECK_ARG(g->dev.mode == 0, "yk_gmd_detect: a YK_GMD_SPARSE_OPTFLOW detector computes warps (yk_gmc_apply)");
  YK_CHECK_ARG(g->calls_window == 0,
               "yk_gmd_detect: this detector's previous frame is in the window layout (yk_gmd_detect_window); "
               "yk_gmd_reset first");
  g->calls_single += 1;
  yk::DeviceGuard guard(g->ctx->device);
  const Dev& d = g->dev;
  hipStream_t st = (hipStream_t)stream;
  gmd_front(g, frames, st);
  hipLaunchKernelGGL(yk::gmd::finish_kernel, dim3(d.S), dim3(256), 0, st, d, out ? out : d.out);
  if (out) YK_HIP(hipMemcpyAsync(d.out, out, d.S * sizeof(yk_motion), hipMemcpyDeviceToDevice, st));
  YK_HIP(hipGetLastError());
  g->frames += 1;
  return YK_OK;
}

static hipError_t gmd_window_alloc(yk_gmd* g) {
  Dev& d = g->dev;
  GmdWindow& w = g->win;
  if (w.pyr) return hipSuccess;
  const size_t S = d.S, V = S * kWindow, HW = (size_t)d.geo.W * d.geo.H, per = (size_t)d.geo.per;
  hipError_t e = hipSuccess;
  auto A = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  A((void**)&w.pyr, (kWindow + 1) * S * per);
  A((void**)&w.der, (kWindow + 1) * S * per * sizeof(short2));
  A((void**)&w.eig, V * HW * sizeof(float));
  A((void**)&w.emax, V * sizeof(unsigned));
  A((void**)&w.cand, V * HW * sizeof(unsigned long long));
  A((void**)&w.ncand, V * sizeof(int));
  A((void**)&w.corners, V * d.maxc * sizeof(float2));
  A((void**)&w.ncorners, V * sizeof(int));
  A((void**)&w.next, V * d.maxc * sizeof(float2));
  A((void**)&w.status, V * d.maxc);
  A((void**)&w.sel, V * sizeof(int));
  A((void**)&w.info, V * 5 * sizeof(int));
  A((void**)&w.out, V * sizeof(yk_motion));
  if (e == hipSuccess) e = hipMemset(w.pyr, 0, (kWindow + 1) * S * per);  // (slot 0 before any frame: read, unused)
  if (e == hipSuccess) e = hipMemset(w.der, 0, (kWindow + 1) * S * per * sizeof(short2));
  if (e == hipSuccess) e = hipMemset(w.sel, 0, V * sizeof(int));
  if (e == hipSuccess) e = hipMemset(w.ncorners, 0, V * sizeof(int));
  if (e == hipSuccess) e = hipMemset(w.info, 0, V * 5 * sizeof(int));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return e;
}

// The window's device view: n steps as n * S virtual streams (see GmdWindow)
static Dev gmd_window_dev(const yk_gmd* g, int n) {
  const Dev& d = g->dev;
  const GmdWindow& w = g->win;
  const long long sp = (long long)d.S * d.geo.per;  // one slot
  Dev v = d;
  v.S = d.S * n;
  v.pyr[0] = w.pyr;
  v.pyr[1] = w.pyr + sp;
  v.der[0] = w.der;
  v.der[1] = w.der + sp;
  v.eig = w.eig;
  v.emax = w.emax;
  v.cand = w.cand;
  v.ncand = w.ncand;
  v.corners = w.corners;
  v.ncorners = w.ncorners;
  v.next = w.next;
  v.status = w.status;
  v.sel = w.sel;
  v.info = w.info;
  v.out = w.out;
  return v;  // st: the real streams' detector state (finish_window_kernel)
}

int yk_gmd_detect_window(yk_gmd* g, const uint8_t* const* frames, int n, yk_motion* out, void* stream) {
  YK_CHECK_ARG(g && frames && n >= 1, "yk_gmd_detect_window: NULL argument or n < 1");
  YK_CHECK_ARG(g->dev.mode == 0, "yk_gmd_detect_window: a YK_GMD_SPARSE_OPTFLOW detector computes warps (yk_gmc_apply)");
  YK_CHECK_ARG(g->calls_single == 0,
               "yk_gmd_detect_window: this detector's previous frame is in the per-call layout (yk_gmd_detect); "
               "yk_gmd_reset first");
  for (int i = 0; i < n; ++i) YK_CHECK_ARG(frames[i], "yk_gmd_detect_window: NULL frame pointer");
  yk::DeviceGuard guard(g->ctx->device);
  hipError_t e = gmd_window_alloc(g);
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_gmd_detect_window: hipMalloc failed: ") + hipGetErrorString(e));
    return YK_ERR_HIP;
  }
  hipStream_t st = (hipStream_t)stream;
  const Dev& d = g->dev;
  const yk::gmd::Geo& G = d.geo;
  const int S = d.S;
  const long long HW = (long long)G.W * G.H, sp = (long long)S * G.per;
  for (int c0 = 0; c0 < n; c0 += kWindow) {  // chunks of at most kWindow steps, in frame order
    const int m = n - c0 < kWindow ? n - c0 : kWindow;
    const Dev v = gmd_window_dev(g, m);
    for (int w = 0; w < m; ++w) {  // each step's gray image into slot w + 1
      Dev vw = v;
      vw.S = S;
      vw.pyr[1] = g->win.pyr + (w + 1) * sp;
      hipLaunchKernelGGL(yk::gmd::gray_kernel, dim3((unsigned)((HW + 255) / 256), S), dim3(256), 0, st, vw, frames[c0 + w]);
    }
    for (int l = 1; l <= G.levels; ++l)
      hipLaunchKernelGGL(yk::gmd::pyrdown_kernel, dim3((G.lw[l] + 15) / 16, (G.lh[l] + 15) / 16, v.S), dim3(256), 0, st,
                         v, l);
    hipLaunchKernelGGL(yk::gmd::scharr_kernel, dim3((G.lw[0] + 15) / 16, (G.lh[0] + 15) / 16, v.S * (G.levels + 1)),
                       dim3(256), 0, st, v);
    hipLaunchKernelGGL(yk::gmd::clear_kernel, dim3((v.S + 255) / 256), dim3(256), 0, st, v);
    hipLaunchKernelGGL(yk::gmd::eig_kernel<7>, dim3((G.W + yk::gmd::ETS - 1) / yk::gmd::ETS, (G.H + yk::gmd::ETS - 1) / yk::gmd::ETS, v.S),
                       dim3(256), 0, st, v);
    hipLaunchKernelGGL(yk::gmd::cand_kernel, dim3((unsigned)((HW + 256 * yk::gmd::CPX - 1) / (256 * yk::gmd::CPX)), v.S),
                       dim3(256), 0, st, v);
    hipLaunchKernelGGL(yk::gmd::select_kernel, dim3(v.S), dim3(yk::gmd::NTS), yk::gmd::SEL_LDS, st, v);
    hipLaunchKernelGGL(yk::gmd::lk_kernel<0>, dim3(d.maxc / 4, v.S), dim3(256), 0, st, v);
    yk_motion* o = out ? out + (size_t)c0 * S : g->win.out;
    hipLaunchKernelGGL(yk::gmd::finish_window_kernel, dim3(S), dim3(256), 0, st, v, m, S, o);
    // the chunk's last frame is the next chunk's (or call's) previous one
    YK_HIP(hipMemcpyAsync(g->win.pyr, g->win.pyr + m * sp, (size_t)sp, hipMemcpyDeviceToDevice, st));
    YK_HIP(hipMemcpyAsync(g->win.der, g->win.der + m * sp, (size_t)sp * sizeof(short2), hipMemcpyDeviceToDevice, st));
    // the last record of every stream is yk_gmd_outputs' "last call"
    YK_HIP(hipMemcpyAsync(d.out, o + (size_t)(m - 1) * S, S * sizeof(yk_motion), hipMemcpyDeviceToDevice, st));
  }
  YK_HIP(hipGetLastError());
  g->frames += n;
  g->calls_window += 1;
  return YK_OK;
}

int yk_gmc_apply(yk_gmd* g, const uint8_t* frames, double* warp, void* stream) {
  YK_CHECK_ARG(g && frames, "yk_gmc_apply: NULL argument");
  YK_CHECK_ARG(g->dev.mode == 1, "yk_gmc_apply: the detector was not created with YK_GMD_SPARSE_OPTFLOW");
  yk::DeviceGuard guard(g->ctx->device);
  const Dev& d = g->dev;
  hipStream_t st = (hipStream_t)stream;
  gmd_front(g, frames, st);
  hipLaunchKernelGGL(yk::gmd::gmc_kernel, dim3(d.S), dim3(yk::gmd::GT), 0, st, d, warp ? warp : d.warp);
  if (warp) YK_HIP(hipMemcpyAsync(d.warp, warp, d.S * 6 * sizeof(double), hipMemcpyDeviceToDevice, st));
  YK_HIP(hipGetLastError());
  g->frames += 1;
  return YK_OK;
}

int yk_gmc_outputs(yk_gmd* g, double** dev_warp) {
  YK_CHECK_ARG(g && dev_warp, "yk_gmc_outputs: NULL argument");
  *dev_warp = g->dev.warp;
  return YK_OK;
}

int yk_gmc_info(yk_gmd* g, int32_t* host_info, void* stream) {
  YK_CHECK_ARG(g && host_info, "yk_gmc_info: NULL argument");
  yk::DeviceGuard guard(g->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  YK_HIP(hipMemcpyAsync(host_info, g->dev.info, g->dev.S * 5 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

int yk_gmd_outputs(yk_gmd* g, yk_motion** dev_motion) {
  YK_CHECK_ARG(g && dev_motion, "yk_gmd_outputs: NULL argument");
  *dev_motion = g->dev.out;
  return YK_OK;
}

int yk_gmd_debug_buffers(yk_gmd* g, void** dev_corners, void** dev_next, void** dev_status, int32_t** dev_ncorners,
                         int32_t* max_corners) {
  YK_CHECK_ARG(g && dev_corners && dev_next && dev_status && dev_ncorners && max_corners,
               "yk_gmd_debug_buffers: NULL argument");
  *dev_corners = g->dev.corners;
  *dev_next = g->dev.next;
  *dev_status = g->dev.status;
  *dev_ncorners = g->dev.ncorners;
  *max_corners = g->dev.maxc;
  return YK_OK;
}

int yk_gmd_debug_pyramids(yk_gmd* g, void** dev_pyr0, void** dev_pyr1, void** dev_der0, void** dev_der1, int64_t* per) {
  YK_CHECK_ARG(g && dev_pyr0 && dev_pyr1 && dev_der0 && dev_der1 && per, "yk_gmd_debug_pyramids: NULL argument");
  *dev_pyr0 = g->dev.pyr[0];
  *dev_pyr1 = g->dev.pyr[1];
  *dev_der0 = g->dev.der[0];
  *dev_der1 = g->dev.der[1];
  *per = g->dev.geo.per;
  return YK_OK;
}

int yk_gmd_download(yk_gmd* g, yk_motion* host_motion, yk_gmd_stats* host_stats, void* stream) {
  YK_CHECK_ARG(g && host_motion, "yk_gmd_download: NULL argument");
  yk::DeviceGuard guard(g->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  const int S = g->dev.S;
  YK_HIP(hipMemcpyAsync(host_motion, g->dev.out, S * sizeof(yk_motion), hipMemcpyDeviceToHost, st));
  yk::gmd::State* hs = nullptr;
  if (host_stats) {
    hs = new yk::gmd::State[S];
    hipError_t e = hipMemcpyAsync(hs, g->dev.st, S * sizeof(yk::gmd::State), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      delete[] hs;
      YK_HIP(e);
    }
    for (int s = 0; s < S; ++s) {
      host_stats[s].total_detections = hs[s].total;
      host_stats[s].motion_events = hs[s].motion_events;
      host_stats[s].reset_triggers = hs[s].reset_triggers;
      host_stats[s].avg_motion_magnitude = hs[s].avg;
      host_stats[s].pad = 0;
    }
    delete[] hs;
  }
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

int yk_gmd_points(yk_gmd* g, int s, float* host_corners, float* host_next, uint8_t* host_status, int32_t* n,
                  void* stream) {
  YK_CHECK_ARG(g && host_corners && host_next && host_status && n, "yk_gmd_points: NULL argument");
  YK_CHECK_ARG(s >= 0 && s < g->dev.S, "yk_gmd_points: stream index out of range");
  yk::DeviceGuard guard(g->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  const int M = g->dev.maxc;
  YK_HIP(hipMemcpyAsync(n, g->dev.ncorners + s, sizeof(int), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_corners, g->dev.corners + (size_t)s * M, M * sizeof(float2), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_next, g->dev.next + (size_t)s * M, M * sizeof(float2), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_status, g->dev.status + (size_t)s * M, M, hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

}  // extern "C"
