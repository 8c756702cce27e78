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
//   eig_kernel      cornerMinEigenVal(prev, blockSize 7, Sobel 3) on 16x16 tiles: Sobel
//                   responses and 7x7 box sums in exact integers through LDS, one float rounding
//                   per covariance entry, per-stream max by an ordered-bits atomicMax
//   cand_kernel     TOZERO threshold at 0.01 * max, 3x3 dilate test, interior local maxima
//                   appended as 64-bit keys (value bits, address) with wave-aggregated atomics
//   select_kernel   one workgroup per stream: keys sorted descending in LDS (bitonic, 16384 at
//                   a time; a radix select cuts larger candidate sets into windows), then the
//                   greedy minDistance-15 pass (1024 candidates tested in parallel against the
//                   kept corners, in-chunk conflicts resolved in order by one wave) to 200 corners
//   lk_kernel       pyramidal Lucas-Kanade, one wavefront per corner: the 21x21 window is 7
//                   pixels per lane in registers, window sums are exact int64 wave reductions
//   finish_kernel   the reference's numpy post-processing per stream: median, 75th percentile
//                   inliers, float32 mean / norm, thresholds, 3-vector direction consistency,
//                   GlobalMotionDetector.stats
// The OpenCV stages follow OpenCV 4.x's algorithms as restated in oracle/gmd_ref.py (cv2 itself
// is absent, so that restatement is unpinned); these kernels reproduce the restatement bit for
// bit.  Compiled with -ffp-contract=off: every float expression rounds like the C++ / numpy one.
#include <cfloat>
#include <climits>

#include "yk_internal.h"

namespace yk {
namespace gmd {

constexpr int WIN = 21;                      // lk_params winSize
constexpr int WAREA = WIN * WIN;             // 441 window pixels
constexpr int NSLOT = (WAREA + 63) / 64;     // 7 window pixels per lane
constexpr int MAXC = 200;                    // feature_params maxCorners
constexpr int MINDIST2 = 225;                // minDistance^2 (corners sit on integer pixels)
constexpr int MAXLV = 3;                     // lk_params maxLevel
constexpr int MAXIT = 30;                    // criteria count
constexpr double EPS2 = 0.01 * 0.01;         // criteria eps, squared by calcOpticalFlowPyrLK
constexpr int CAP = 16384;                   // candidate keys sorted in LDS at once
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
  int has_prev;
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
};

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
__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- frame ingest
__global__ void __launch_bounds__(256) gray_kernel(Dev g, const unsigned char* __restrict__ frames, int cur) {
  const int s = blockIdx.y;
  const long long n = (long long)g.geo.W * g.geo.H;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned char* p = frames + ((long long)s * n + i) * 3;
  const int v = (p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14;
  g.pyr[cur][(long long)s * g.geo.per + i] = (unsigned char)v;
}

__global__ void __launch_bounds__(256) pyrdown_kernel(Dev g, int cur, int l) {
  const int s = blockIdx.z;
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int dw = g.geo.lw[l], dh = g.geo.lh[l], sw = g.geo.lw[l - 1], sh = g.geo.lh[l - 1];
  if (x >= dw || y >= dh) return;
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
}

// calcSharrDeriv: vertical [3 10 3] / [-1 0 1], then horizontal [-1 0 1] / [3 10 3], reflect-101.
__global__ void __launch_bounds__(256) scharr_kernel(Dev g, int cur, int l) {
  const int s = blockIdx.z;
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
}

// ---------------------------------------------------------------- goodFeaturesToTrack
__global__ void clear_kernel(Dev g) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < g.S) {
    g.emax[s] = 0u;
    g.ncand[s] = 0;
  }
}

// cornerMinEigenVal on a 16x16 output tile: the 22x22 Sobel-product halo (box radius 3; the
// products outside the image are those of the reflected pixel, like boxFilter's reflect-101
// border over the product image), 7-wide horizontal then vertical integer sums.  The gray pixels
// the Sobel taps of those products read -- rows / columns [o - 1, o + 23) of the image, each
// product at its reflected position with Sobel's own reflect-101 neighbours -- are staged in LDS
// once (coalesced rows), so a product costs LDS reads instead of eight global byte loads.
__global__ void __launch_bounds__(256) eig_kernel(Dev g, int prev) {
  __shared__ int gt[24][25];
  __shared__ int pxx[22][23], pxy[22][23], pyy[22][23];
  __shared__ int hxx[22][17], hxy[22][17], hyy[22][17];
  __shared__ unsigned wmax[4];
  const int s = blockIdx.z, W = g.geo.W, H = g.geo.H, tid = threadIdx.x;
  const unsigned char* img = g.pyr[prev] + (long long)s * g.geo.per;
  const int ox = blockIdx.x * 16 - 3, oy = blockIdx.y * 16 - 3;
  const int gy0 = oy - 1, gx0 = ox - 1;  // LDS tile origin (image coordinates)
  for (int i = tid; i < 24 * 24; i += 256) {
    const int ry = i / 24, rx = i - ry * 24;
    const int y = gy0 + ry, x = gx0 + rx;
    gt[ry][rx] = (y >= 0 && y < H && x >= 0 && x < W) ? (int)img[(long long)y * W + x] : 0;
  }
  __syncthreads();
  auto cl = [](int v) { return v < 0 ? 0 : (v > 23 ? 23 : v); };  // only outputs outside the image clamp
  for (int i = tid; i < 22 * 22; i += 256) {
    const int ry = i / 22, rx = i - ry * 22;
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
  for (int i = tid; i < 22 * 16; i += 256) {
    const int ry = i >> 4, cx = i & 15;
    int a = 0, b = 0, c = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      a += pxx[ry][cx + k];
      b += pxy[ry][cx + k];
      c += pyy[ry][cx + k];
    }
    hxx[ry][cx] = a;
    hxy[ry][cx] = b;
    hyy[ry][cx] = c;
  }
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  int sxx = 0, sxy = 0, syy = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    sxx += hxx[ty + k][tx];
    sxy += hxy[ty + k][tx];
    syy += hyy[ty + k][tx];
  }
  const int x = blockIdx.x * 16 + tx, y = blockIdx.y * 16 + ty;
  unsigned m = 0u;
  if (x < W && y < H) {
    const double s2 = 1.0 / (7140.0 * 7140.0);  // (1 / (4 * blockSize * 255))^2
    const float cxx = (float)((double)sxx * s2), cxy = (float)((double)sxy * s2), cyy = (float)((double)syy * s2);
    const float a = cxx * 0.5f, c = cyy * 0.5f, d = a - c;
    const float e = (a + c) - sqrtf(d * d + cxy * cxy);
    g.eig[(long long)s * W * H + (long long)y * W + x] = e;
    m = ord_bits(e);
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
    // already there skips the atomic (1,280 same-address atomics per stream serialised at L2)
    if (b > __hip_atomic_load(&g.emax[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&g.emax[s], b);
  }
}

// CPX pixels per thread (a workgroup covers 256 * CPX consecutive pixels); the workgroup's
// candidates take one global atomic (per-stream counter), not one per wave.
constexpr int CPX = 4;
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
  int* hist;                 // [256]
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
  base += 4 * 256;
  L.misc = (int*)base;
  return L;
}
constexpr size_t SEL_LDS = sizeof(unsigned long long) * CAP + 4 * (2 * MAXC + 3 * NTS + 256 + 8);
enum { S_CNT = 0, S_NA = 1, S_D = 2, S_K = 3, S_REM = 4 };

// The k-th largest key among keys < U (all keys when !has_u): radix select, 8 bits a pass.
__device__ unsigned long long kth_largest(const unsigned long long* keys, int n, unsigned long long U, bool has_u,
                                          int k, SelLds& L) {
  const int tid = threadIdx.x;
  unsigned long long prefix = 0ull, mask = 0ull;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += NTS) L.hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += NTS) {
      const unsigned long long key = keys[i];
      if ((!has_u || key < U) && (key & mask) == prefix) atomicAdd(&L.hist[(key >> shift) & 255], 1);
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
      for (int i = tid; i < n; i += NTS) c += keys[i] < U ? 1 : 0;
      if (c) atomicAdd(&L.misc[S_REM], c);
      __syncthreads();
      rem = L.misc[S_REM];
    }
    const bool last = rem <= CAP;
    const unsigned long long K = last ? 0ull : kth_largest(keys, n, U, has_u, CAP, L);
    if (tid == 0) L.misc[S_CNT] = 0;
    __syncthreads();
    for (int base = 0; base < n; base += NTS) {  // gather the window [K, U)
      const int i = base + tid;
      unsigned long long key = 0ull;
      bool in = false;
      if (i < n) {
        key = keys[i];
        in = (!has_u || key < U) && (last || key >= K);
      }
      const unsigned long long mask = __ballot(in);
      if (mask) {
        const int leader = __ffsll((long long)mask) - 1;
        int b = 0;
        if (lane == leader) b = atomicAdd(&L.misc[S_CNT], __popcll(mask));
        b = __shfl(b, leader);
        if (in) L.keys[b + __popcll(mask & ((1ull << lane) - 1ull))] = key;
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
        // The chunk's candidates 64 at a time in registers (lane l holds candidate c0 + l); the
        // ones that passed the test against the earlier chunks' corners are walked in order
        // through a ballot mask, and the corners accepted in this chunk stay in registers (lane
        // l, slot k holds accepted corner na0 + l + 64 k; at most MAXC < 256 of them).
        int na = na0;
        const int cm = m - base < NTS ? m - base : NTS;
        int rx[4] = {0, 0, 0, 0}, ry[4] = {0, 0, 0, 0};
        for (int c0 = 0; c0 < cm && na < MAXC; c0 += 64) {
          const int c = c0 + lane;
          const bool okc = c < cm && L.cok[c] != 0;
          const int xl = okc ? L.cx[c] : 0, yl = okc ? L.cy[c] : 0;
          unsigned long long todo = __ballot(okc);
          while (todo != 0ull && na < MAXC) {
            const int b = __ffsll((long long)todo) - 1;
            todo &= todo - 1ull;
            const int xc = __builtin_amdgcn_readlane(xl, b), yc = __builtin_amdgcn_readlane(yl, b);
            const int nin = na - na0;
            bool conflict = false;
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (lane + 64 * k < nin) {
                const int dx = xc - rx[k], dy = yc - ry[k];
                conflict |= dx * dx + dy * dy < MINDIST2;
              }
            if (__ballot(conflict) == 0ull) {
              if (lane == (nin & 63)) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                  if ((nin >> 6) == k) {
                    rx[k] = xc;
                    ry[k] = yc;
                  }
              }
              if (lane == 0) {
                L.ax[na] = xc;
                L.ay[na] = yc;
              }
              ++na;
            }
          }
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
  for (int i = tid; i < na; i += NTS) g.corners[s * MAXC + i] = make_float2((float)L.ax[i], (float)L.ay[i]);
  if (tid == 0) g.ncorners[s] = na;
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
__global__ void __launch_bounds__(256) lk_kernel(Dev g, int prev, int cur) {
  const int s = blockIdx.y, lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= g.ncorners[s]) return;
  const Geo& G = g.geo;
  const float2 pt = g.corners[s * MAXC + p];
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
  float2 nxt = pt;
  int status = 1;
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
        const short2 z = make_short2(0, 0);
        const short2 d00 = (iy0 && ix0) ? D[(long long)Y * cols + X] : z;
        const short2 d01 = (iy0 && ix1) ? D[(long long)Y * cols + X + 1] : z;
        const short2 d10 = (iy1 && ix0) ? D[(long long)(Y + 1) * cols + X] : z;
        const short2 d11 = (iy1 && ix1) ? D[(long long)(Y + 1) * cols + X + 1] : z;
        Dx[k] = (d00.x * w00 + d01.x * w01 + d10.x * w10 + d11.x * w11 + 8192) >> 14;
        Dy[k] = (d00.y * w00 + d01.y * w01 + d10.y * w10 + d11.y * w11 + 8192) >> 14;
        s11 += Dx[k] * Dx[k];
        s12 += Dx[k] * Dy[k];
        s22 += Dy[k] * Dy[k];
      }
    }
    const float A11 = (float)wave_sum64(s11) * fs;
    const float A12 = (float)wave_sum64(s12) * fs;
    const float A22 = (float)wave_sum64(s22) * fs;
    const float Dd = A11 * A22 - A12 * A12;
    const float dd = A11 - A22;
    const float mine = ((A22 + A11) - sqrtf(dd * dd + (4.0f * A12) * A12)) / (float)(2 * WIN * WIN);
    if (mine < 1e-4f || Dd < FLT_EPSILON) {
      if (l == 0) status = 0;
      continue;
    }
    const float Di = 1.0f / Dd;
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
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        if (wy[k] >= 0) {
          const int X = jx + wx[k], Y = jy + wy[k];
          const int x0 = refl(X, cols), x1 = refl(X + 1, cols);
          const unsigned char* r0 = J + (long long)refl(Y, rows) * cols;
          const unsigned char* r1 = J + (long long)refl(Y + 1, rows) * cols;
          const int jv = (r0[x0] * v00 + r0[x1] * v01 + r1[x0] * v10 + r1[x1] * v11 + 256) >> 9;
          const int diff = jv - Iv[k];
          b1 += diff * Dx[k];
          b2 += diff * Dy[k];
        }
      }
      const float fb1 = (float)wave_sum64(b1) * fs;
      const float fb2 = (float)wave_sum64(b2) * fs;
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
  if (lane == 0) {
    g.next[s * MAXC + p] = nxt;
    g.status[s * MAXC + p] = (unsigned char)status;
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

__global__ void __launch_bounds__(256) finish_kernel(Dev g, yk_motion* __restrict__ out) {
  __shared__ float vx[MAXC], vy[MAXC], sx[MAXC], sy[MAXC], dist[MAXC], sd[MAXC];
  __shared__ int wcnt[4];
  const int s = blockIdx.x, tid = threadIdx.x;
  State& S = g.st[s];
  if (!S.has_prev) {  // first frame: only stored (:77-80)
    if (tid == 0) {
      yk_motion r{};
      r.valid = 1;
      r.first_frame = 1;
      r.consistency = -1.0f;
      out[s] = r;
      S.has_prev = 1;
    }
    return;
  }
  const int n = g.ncorners[s];
  // status == 1 compaction in corner order (n <= 200 < 256 threads)
  int flag = 0;
  float mvx = 0.0f, mvy = 0.0f;
  if (tid < n && n >= 20 && g.status[s * MAXC + tid]) {
    flag = 1;
    const float2 a = g.corners[s * MAXC + tid], b = g.next[s * MAXC + tid];
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
  if (tid != 0) return;
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
  out[s] = r;
}

__global__ void state_reset_kernel(Dev g, int stats_only) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.S) return;
  State& S = g.st[s];
  if (!stats_only) {
    S.has_prev = 0;
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

struct yk_gmd {
  yk_ctx* ctx;
  Dev dev;
  int cur;
  long long frames;
};

extern "C" {

int yk_gmd_create(yk_ctx* ctx, int n_streams, int height, int width, int method, yk_gmd** out) {
  YK_CHECK_ARG(ctx && out, "yk_gmd_create: NULL argument");
  YK_CHECK_ARG(n_streams >= 1 && n_streams <= 65535, "yk_gmd_create: n_streams out of range");
  YK_CHECK_ARG(height >= 32 && width >= 32 && (long long)height * width <= (1ll << 28),
               "yk_gmd_create: frame size out of range (32 .. 2^28 pixels)");
  YK_CHECK_ARG(method == YK_GMD_OPTICAL_FLOW || method == YK_GMD_FEATURE_MATCHING || method == YK_GMD_HYBRID,
               "yk_gmd_create: unknown motion detection method");
  YK_CHECK_ARG(method == YK_GMD_OPTICAL_FLOW,
               "yk_gmd_create: 'feature_matching' / 'hybrid' (ORB + RANSAC homography) are not built; use "
               "'optical_flow'");
  yk::DeviceGuard guard(ctx->device);
  auto* g = new yk_gmd{};
  g->ctx = ctx;
  Dev& d = g->dev;
  d.S = n_streams;
  yk::gmd::Geo& G = d.geo;
  G.W = width;
  G.H = height;
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
  for (int i = 0; i < 2; ++i) {
    A((void**)&d.pyr[i], S * G.per);
    A((void**)&d.der[i], S * G.per * sizeof(short2));
  }
  A((void**)&d.eig, S * HW * sizeof(float));
  A((void**)&d.emax, S * sizeof(unsigned));
  A((void**)&d.cand, S * HW * sizeof(unsigned long long));
  A((void**)&d.ncand, S * sizeof(int));
  A((void**)&d.corners, S * yk::gmd::MAXC * sizeof(float2));
  A((void**)&d.ncorners, S * sizeof(int));
  A((void**)&d.next, S * yk::gmd::MAXC * sizeof(float2));
  A((void**)&d.status, S * yk::gmd::MAXC);
  A((void**)&d.st, S * sizeof(yk::gmd::State));
  A((void**)&d.out, S * sizeof(yk_motion));
  if (e == hipSuccess) e = hipMemset(d.ncorners, 0, S * sizeof(int));
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_gmd_create: hipMalloc failed: ") + hipGetErrorString(e));
    yk_gmd_destroy(g);
    return YK_ERR_HIP;
  }
  if (hipFuncSetAttribute((const void*)yk::gmd::select_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
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
  void* ptrs[] = {d.pyr[0], d.pyr[1], d.der[0], d.der[1], d.eig, d.emax, d.cand, d.ncand, d.corners,
                  d.ncorners, d.next, d.status, d.st, d.out};
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
  g->cur = 0;
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

int yk_gmd_detect(yk_gmd* g, const uint8_t* frames, yk_motion* out, void* stream) {
  YK_CHECK_ARG(g && frames, "yk_gmd_detect: NULL argument");
  yk::DeviceGuard guard(g->ctx->device);
  const Dev& d = g->dev;
  const yk::gmd::Geo& G = d.geo;
  hipStream_t st = (hipStream_t)stream;
  const int cur = g->cur, prev = cur ^ 1, S = d.S;
  const long long HW = (long long)G.W * G.H;
  hipLaunchKernelGGL(yk::gmd::gray_kernel, dim3((unsigned)((HW + 255) / 256), S), dim3(256), 0, st, d, frames, cur);
  for (int l = 1; l <= G.levels; ++l)
    hipLaunchKernelGGL(yk::gmd::pyrdown_kernel, dim3((G.lw[l] + 15) / 16, (G.lh[l] + 15) / 16, S), dim3(256), 0, st,
                       d, cur, l);
  for (int l = 0; l <= G.levels; ++l)
    hipLaunchKernelGGL(yk::gmd::scharr_kernel, dim3((G.lw[l] + 15) / 16, (G.lh[l] + 15) / 16, S), dim3(256), 0, st,
                       d, cur, l);
  if (g->frames > 0) {
    hipLaunchKernelGGL(yk::gmd::clear_kernel, dim3((S + 255) / 256), dim3(256), 0, st, d);
    hipLaunchKernelGGL(yk::gmd::eig_kernel, dim3((G.W + 15) / 16, (G.H + 15) / 16, S), dim3(256), 0, st, d, prev);
    hipLaunchKernelGGL(yk::gmd::cand_kernel, dim3((unsigned)((HW + 256 * yk::gmd::CPX - 1) / (256 * yk::gmd::CPX)), S),
                       dim3(256), 0, st, d);
    hipLaunchKernelGGL(yk::gmd::select_kernel, dim3(S), dim3(yk::gmd::NTS), yk::gmd::SEL_LDS, st, d);
    hipLaunchKernelGGL(yk::gmd::lk_kernel, dim3(yk::gmd::MAXC / 4, S), dim3(256), 0, st, d, prev, cur);
  }
  hipLaunchKernelGGL(yk::gmd::finish_kernel, dim3(S), dim3(256), 0, st, d, out ? out : d.out);
  if (out) YK_HIP(hipMemcpyAsync(d.out, out, S * sizeof(yk_motion), hipMemcpyDeviceToDevice, st));
  YK_HIP(hipGetLastError());
  g->cur ^= 1;
  g->frames += 1;
  return YK_OK;
}

int yk_gmd_outputs(yk_gmd* g, yk_motion** dev_motion) {
  YK_CHECK_ARG(g && dev_motion, "yk_gmd_outputs: NULL argument");
  *dev_motion = g->dev.out;
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
  const int M = yk::gmd::MAXC;
  YK_HIP(hipMemcpyAsync(n, g->dev.ncorners + s, sizeof(int), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_corners, g->dev.corners + (size_t)s * M, M * sizeof(float2), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_next, g->dev.next + (size_t)s * M, M * sizeof(float2), hipMemcpyDeviceToHost, st));
  YK_HIP(hipMemcpyAsync(host_status, g->dev.status + (size_t)s * M, M, hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

}  // extern "C"
