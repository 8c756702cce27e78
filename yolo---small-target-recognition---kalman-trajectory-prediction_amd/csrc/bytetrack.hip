// ByteTrack / BoT-SORT (ultralytics/trackers, the upstream model.track() path) on gfx950.
//
// One workgroup per video stream runs one complete BYTETracker.update()
// (ultralytics/trackers/byte_tracker.py:299-410) -- or BOTSORT's without ReID / GMC
// (bot_sort.py:156-249: KalmanFilterXYWH, BOTrack.predict zeroing both size velocities) -- on
// device-resident track state; a second, tiny launch gives the new tracks their ids from one
// counter shared by all streams (BaseTrack._count is process-global, basetrack.py:67-92).
// Checker: oracle/bytetrack_ref.py (numpy + scipy restatement of the same files).
//
// Numerics.  The 8-state filters keep F, H, Q, R, the initial P diagonal / block structured, so
// P stays four 2x2 blocks (P[c][c], P[c][c+4], P[c+4][c], P[c+4][c+4]); the products numpy
// evaluates on the full 8x8 matrices (multiply by 1 / 0, one non-zero term per element) reduce
// exactly to the block formulas below.  cho_solve on the diagonal projected covariance is
// OpenBLAS's dtrsm: multiplication by 1/sqrt(S) twice.  Dtypes follow numpy's NEP 50 rules
// (kalman_filter.py with float32 measurements): a new track's mean is the float32 array of
// initiate() until its first predict / update (mean32), BOTSORT's initial covariance is float32,
// a predict batch whose means are all float32 computes its motion noise in float32.  IoU is
// utils/metrics.py bbox_ioa(iou=True) in float32 (no FMA: -ffp-contract=off).
//
// Assignment (matching.py:20-61), both branches; the default is the one the reference takes.
// lap (use_lap=True, `lap>=0.5.12` is a hard requirement, :9-17): lapjv(extend_cost=True,
// cost_limit=thresh) solves the (n_rows + n_cols)-square problem padded with cost_limit / 2 and
// a zero dummy block, i.e. it minimises sum over matched pairs of (cost - thresh): the
// maximum-weight matching with weights thresh - cost over the pairs with cost < thresh; the
// unmatched lists are ascending (np.where).  scipy (use_lap=False): an optimal assignment of the
// full cost matrix, then the float32 threshold filter; a pair whose boxes do not overlap costs
// exactly 1, so the overlapping pairs of an optimal assignment form a maximum-weight matching of
// the overlap graph with weights 1 - cost; the unmatched lists follow CPython 3.10's frozenset
// iteration order (pyset_diff; restated and checked in oracle/pyset_order.py), which decides
// e.g. the order of new-track activation.  Either way every connected component of the edge
// graph is solved on its own (Hungarian method, one thread per component); equal-cost
// alternatives (exact ties) are this solver's choice, not lapjv's / scipy's.
#include <climits>

#include "yk_internal.h"

namespace yk {
namespace bt {

constexpr int NT = 256;
constexpr int NW = NT / 64;
enum { NEW = 0, TRACKED = 1, LOST = 2, REMOVED = 3 };

struct Slot {
  double mean[8];
  double P[16];  // per coordinate c: [4c] P[c][c], [4c+1] P[c][c+4], [4c+2] P[c+4][c], [4c+3] P[c+4][c+4]
  double Pd[64]; // dense covariance (row-major 8x8) once a GMC warp coupled x / y (dense != 0)
  int dense;
  double idx;    // detection index within its score subset (float64, the last element of the xywh row)
  float score, cls;
  int mean32;    // mean is still initiate()'s float32 array
  int state, is_activated, track_id, frame_id, start_frame, tracklet_len;
  int rm_seq;    // sequence number of the last removed_stracks append of this track (-1: none)
};

struct Hdr {
  int n_tracked, n_lost, frame_id;
  int rm_total, rm_len;  // removed_stracks: appends so far, current length (clipped to 999 past 1000)
  int n_new;             // tracks activated this step (their ids: bt_ids_kernel)
  int n_out;
  int n_overflow;  // new tracks not created because every slot was in use (0 in parity runs)
};

struct Cfg {
  float th_high, th_low, th_new, th_match;
  int max_time_lost, fuse, xywh;  // xywh: BOTSORT (KalmanFilterXYWH / BOTrack)
  int lap;                        // linear_assignment branch: 1 lap.lapjv (default), 0 scipy
  double th_match_f64;            // match_thresh as the YAML's python float (lap's cost_limit)
};

// BoT-SORT's GMC (byte_tracker.py:333-340): the step's 2x3 warp per stream, or none

struct Dev {
  Slot* slots;        // [S][T]
  Hdr* hdr;           // [S]
  int* tracked;       // [S][T] slot ids in tracked_stracks order
  int* lost;          // [S][T] slot ids in lost_stracks order
  int* newslots;      // [S][D] slots activated this step, in activation order
  int* newrow;        // [S][D] their output row (-1: not reported)
  float* cost;        // [S][T * D] cost matrix of the current assignment
  int* edges;         // [S][T * D] overlapping pairs (flat index) of the current assignment
  double* hung;       // [S][hung_stride] Hungarian work: [NT][6 (T + D + 2)] doubles, then [NT][2 T + D] ints
  size_t hung_stride;
  float* rows;        // [S][T][8] x1 y1 x2 y2 track_id score cls idx (the reference's float32 result)
  int* counts;        // [S]
  long long* ids;     // [1] the shared track id counter (BaseTrack._count)
  int T, D;
  Cfg cfg;
};

// ---------------------------------------------------------------------------- LDS
struct Lds {
  float* dtl;     // [D][4] detection tlwh (float32)
  float* dxy;     // [D][4] detection xyxy (float32)
  float* dsc;     // [D]
  float* dcl;     // [D]
  double* didx;   // [D]
  int* hi;        // [D] detections with score >= track_high_thresh, in order
  int* se;        // [D] detections with track_low < score < track_high
  int* drem;      // [D] high detections left after the first association (unmatched order)
  int* pool;      // [T] strack_pool (tracked & activated, then lost)
  int* unc;       // [T] unconfirmed
  int* rtr;       // [T] r_tracked_stracks
  float* txy;     // [T][4] xyxy (float32) of the current assignment's row tracks
  int* act;       // [T + D] activated_stracks
  int* ref;       // [T] refind_stracks
  int* lnew;      // [T] lost_stracks of this step
  int* rnew;      // [2T] removed_stracks of this step
  int* mrow;      // [T] match of each row (-1)
  int* mcol;      // [D] match of each column (-1)
  int* urow;      // [T] unmatched rows, list order
  int* ucol;      // [D] unmatched columns, list order
  int* label;     // [T + D] connected-component labels
  int* flag;      // [T + D] scratch flags
  int* ptab;      // [PTAB] CPython set table simulation
  int* misc;      // [32]
};
constexpr int PTAB = 8192;

__host__ __device__ inline size_t lds_bytes(int T, int D) {
  size_t b = 0;
  b += (size_t)D * 16 * 2 + (size_t)D * 4 * 2 + (size_t)D * 8;  // dtl dxy dsc dcl didx
  b += (size_t)D * 4 * 3;                                        // hi se drem
  b += (size_t)T * 4 * 3 + (size_t)T * 16;                       // pool unc rtr txy
  b += (size_t)(T + D) * 4 + (size_t)T * 4 * 2 + (size_t)T * 8;  // act ref lnew rnew
  b += (size_t)T * 4 + (size_t)D * 4 + (size_t)T * 4 + (size_t)D * 4;  // mrow mcol urow ucol
  b += (size_t)(T + D) * 4 * 2 + (size_t)PTAB * 4 + 32 * 4;      // label flag ptab misc
  return b + 24 * 16;  // carve() rounds each of its 24 arrays up to 16 bytes
}

__device__ Lds carve(char* p, int T, int D) {
  Lds L;
  auto take = [&](size_t bytes) {
    char* q = p;
    p += (bytes + 15) / 16 * 16;
    return q;
  };
  L.didx = (double*)take((size_t)D * 8);
  L.dtl = (float*)take((size_t)D * 16);
  L.dxy = (float*)take((size_t)D * 16);
  L.dsc = (float*)take((size_t)D * 4);
  L.dcl = (float*)take((size_t)D * 4);
  L.hi = (int*)take((size_t)D * 4);
  L.se = (int*)take((size_t)D * 4);
  L.drem = (int*)take((size_t)D * 4);
  L.pool = (int*)take((size_t)T * 4);
  L.unc = (int*)take((size_t)T * 4);
  L.rtr = (int*)take((size_t)T * 4);
  L.txy = (float*)take((size_t)T * 16);
  L.act = (int*)take((size_t)(T + D) * 4);
  L.ref = (int*)take((size_t)T * 4);
  L.lnew = (int*)take((size_t)T * 4);
  L.rnew = (int*)take((size_t)T * 8);
  L.mrow = (int*)take((size_t)T * 4);
  L.mcol = (int*)take((size_t)D * 4);
  L.urow = (int*)take((size_t)T * 4);
  L.ucol = (int*)take((size_t)D * 4);
  L.label = (int*)take((size_t)(T + D) * 4);
  L.flag = (int*)take((size_t)(T + D) * 4);
  L.ptab = (int*)take((size_t)PTAB * 4);
  L.misc = (int*)take(32 * 4);
  return L;
}
enum { Q_N = 0, Q_E, Q_CHG, Q_NC, Q_ACT, Q_REF, Q_LNEW, Q_RNEW, Q_A, Q_B, Q_WSUM = 16 };

// exclusive prefix count of flag over the workgroup
__device__ __forceinline__ int block_scan(int flag, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long m = __ballot(flag);
  const int pre = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[w] = __popcll(m);
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    base += (i < w) ? wsum[i] : 0;
    tot += wsum[i];
  }
  __syncthreads();
  total = tot;
  return base + pre;
}

// ---------------------------------------------------------------------------- boxes
// xyxy (float32) of a track from its mean: STrack.tlwh / BOTrack.tlwh then .xyxy, in the mean's
// dtype (float32 while mean32), cast to float32 (np.ascontiguousarray(..., dtype=np.float32)).
__device__ __forceinline__ void track_xyxy(const Slot& t, bool xywh, float* o) {
  if (t.mean32) {
    float r0 = (float)t.mean[0], r1 = (float)t.mean[1], r2 = (float)t.mean[2], r3 = (float)t.mean[3];
    if (!xywh) r2 = r2 * r3;
    r0 = r0 - r2 / 2.0f;
    r1 = r1 - r3 / 2.0f;
    o[0] = r0;
    o[1] = r1;
    o[2] = r2 + r0;
    o[3] = r3 + r1;
  } else {
    double r0 = t.mean[0], r1 = t.mean[1], r2 = t.mean[2], r3 = t.mean[3];
    if (!xywh) r2 = r2 * r3;
    r0 = r0 - r2 / 2.0;
    r1 = r1 - r3 / 2.0;
    o[0] = (float)r0;
    o[1] = (float)r1;
    o[2] = (float)(r2 + r0);
    o[3] = (float)(r3 + r1);
  }
}

// 1 - IoU (utils/metrics.py:23-52 bbox_ioa(iou=True), float32, eps 1e-7), then fuse_score
// (matching.py:134-157) when fuse: 1 - (1 - cost) * score.
__device__ __forceinline__ float pair_cost(const float* a, const float* b, float score, bool fuse) {
  const float iw = fmaxf(fminf(a[2], b[2]) - fmaxf(a[0], b[0]), 0.0f);
  const float ih = fmaxf(fminf(a[3], b[3]) - fmaxf(a[1], b[1]), 0.0f);
  const float inter = iw * ih;
  const float area2 = (b[2] - b[0]) * (b[3] - b[1]);
  const float area1 = (a[2] - a[0]) * (a[3] - a[1]);
  const float area = (area2 + area1) - inter;
  const float iou = inter / (area + 1e-7f);
  float c = 1.0f - iou;
  if (fuse) c = 1.0f - (1.0f - c) * score;
  return c;
}

// ---------------------------------------------------------------------------- Kalman filters
constexpr double WP = 1.0 / 20, WV = 1.0 / 160;

// KalmanFilterXYAH / XYWH.initiate (kalman_filter.py:64-96, 320-362) of a float32 measurement
__device__ void kf_initiate(Slot& t, const float* m, bool xywh) {
  for (int c = 0; c < 4; ++c) {
    t.mean[c] = (double)m[c];
    t.mean[c + 4] = 0.0;
  }
  t.mean32 = 1;
  t.dense = 0;
  const float k2 = (float)(2 * WP), k10 = (float)(10 * WV);  // python float * np.float32 -> float32
  for (int c = 0; c < 4; ++c) {
    const float ref = xywh ? ((c & 1) ? m[3] : m[2]) : m[3];
    const float sp = k2 * ref, sv = k10 * ref;
    double pp, vv;
    if (xywh) {  // all-float32 std list: np.square in float32
      pp = (double)(sp * sp);
      vv = (double)(sv * sv);
    } else {  // the python floats 1e-2 / 1e-5 make the list float64
      const double dsp = c == 2 ? 1e-2 : (double)sp, dsv = c == 2 ? 1e-5 : (double)sv;
      pp = dsp * dsp;
      vv = dsv * dsv;
    }
    t.P[4 * c + 0] = pp;
    t.P[4 * c + 1] = 0.0;
    t.P[4 * c + 2] = 0.0;
    t.P[4 * c + 3] = vv;
  }
}

// multi_predict (kalman_filter.py:165-203 / 431-470) of one track of a batch; f32: every mean
// of the batch is float32, so the motion noise is computed in float32.
__device__ void kf_predict(Slot& t, bool xywh, bool f32) {
  double q[8];
  if (f32) {
    const float wp = (float)WP, wv = (float)WV;
    float sp[4], sv[4];
    const float m2 = (float)t.mean[2], m3 = (float)t.mean[3];
    for (int c = 0; c < 4; ++c) {
      const float ref = xywh ? ((c & 1) ? m3 : m2) : m3;
      sp[c] = wp * ref;
      sv[c] = wv * ref;
    }
    if (!xywh) {
      sp[2] = 1e-2f * 1.0f;
      sv[2] = 1e-5f * 1.0f;
    }
    for (int c = 0; c < 4; ++c) {
      q[c] = (double)(sp[c] * sp[c]);
      q[c + 4] = (double)(sv[c] * sv[c]);
    }
  } else {
    double sp[4], sv[4];
    for (int c = 0; c < 4; ++c) {
      const double ref = xywh ? ((c & 1) ? t.mean[3] : t.mean[2]) : t.mean[3];
      sp[c] = WP * ref;
      sv[c] = WV * ref;
    }
    if (!xywh) {
      sp[2] = 1e-2 * 1.0;
      sv[2] = 1e-5 * 1.0;
    }
    for (int c = 0; c < 4; ++c) {
      q[c] = sp[c] * sp[c];
      q[c + 4] = sv[c] * sv[c];
    }
  }
  if (t.dense) {
    // np.dot(F, P) then .dot(F.T) (+ motion_cov): every F row / column has one or two unit
    // entries, so each product element is one rounded sum in any summation order
    for (int c = 0; c < 4; ++c) t.mean[c] = t.mean[c] + t.mean[c + 4];
    double L[64];
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) L[8 * i + j] = i < 4 ? t.Pd[8 * i + j] + t.Pd[8 * (i + 4) + j] : t.Pd[8 * i + j];
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 8; ++j) {
        const double o = j < 4 ? L[8 * i + j] + L[8 * i + j + 4] : L[8 * i + j];
        t.Pd[8 * i + j] = o + (i == j ? q[i] : 0.0);
      }
    t.mean32 = 0;
    return;
  }
  for (int c = 0; c < 4; ++c) {
    t.mean[c] = t.mean[c] + t.mean[c + 4];
    const double p = t.P[4 * c], a = t.P[4 * c + 1], b = t.P[4 * c + 2], v = t.P[4 * c + 3];
    t.P[4 * c + 0] = ((p + b) + (a + v)) + q[c];
    t.P[4 * c + 1] = (a + v) + 0.0;
    t.P[4 * c + 2] = (b + v) + 0.0;
    t.P[4 * c + 3] = v + q[c + 4];
  }
  t.mean32 = 0;
}

// Dense update (a covariance coupled by a GMC warp): project (H P H^T + R), scipy's
// cho_factor (LAPACK dpotf2 order: dot, then the column scaled by 1 / L[j][j]) and cho_solve
// (forward / backward substitution by the reciprocal diagonal), mean + innovation . K^T, and
// P - K (S K^T) (multi_dot's order for equal costs).  numpy's BLAS kernels sum in their own
// order, so this path agrees with the reference to rounding, not bit for bit (tests: 1e-6).
__device__ void kf_update_dense(Slot& t, const float* meas, const double* r) {
  double S[4][4], L[4][4] = {}, X[4][8], K[8][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) S[i][j] = t.Pd[8 * i + j] + (i == j ? r[i] : 0.0);
  for (int j = 0; j < 4; ++j) {
    double a = S[j][j];
    for (int k = 0; k < j; ++k) a = a - L[j][k] * L[j][k];
    L[j][j] = sqrt(a);
    const double il = 1.0 / L[j][j];
    for (int i = j + 1; i < 4; ++i) {
      double v = S[i][j];
      for (int k = 0; k < j; ++k) v = v - L[i][k] * L[j][k];
      L[i][j] = v * il;
    }
  }
  for (int j = 0; j < 8; ++j) {  // columns of (P H^T)^T
    double y[4];
    for (int i = 0; i < 4; ++i) {
      double v = t.Pd[8 * j + i];
      for (int k = 0; k < i; ++k) v = v - L[i][k] * y[k];
      y[i] = v * (1.0 / L[i][i]);
    }
    for (int i = 3; i >= 0; --i) {
      double v = y[i];
      for (int k = i + 1; k < 4; ++k) v = v - L[k][i] * X[k][j];
      X[i][j] = v * (1.0 / L[i][i]);
    }
  }
  for (int j = 0; j < 8; ++j)
    for (int c = 0; c < 4; ++c) K[j][c] = X[c][j];
  double inn[4];
  for (int c = 0; c < 4; ++c) inn[c] = (double)meas[c] - t.mean[c];
  for (int i = 0; i < 8; ++i) {
    double d = 0.0;
    for (int c = 0; c < 4; ++c) d = d + inn[c] * K[i][c];
    t.mean[i] = t.mean[i] + d;
  }
  double T[4][8];
  for (int a = 0; a < 4; ++a)
    for (int j = 0; j < 8; ++j) {
      double v = 0.0;
      for (int b = 0; b < 4; ++b) v = v + S[a][b] * K[j][b];
      T[a][j] = v;
    }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) {
      double v = 0.0;
      for (int a = 0; a < 4; ++a) v = v + K[i][a] * T[a][j];
      t.Pd[8 * i + j] = t.Pd[8 * i + j] - v;
    }
  t.mean32 = 0;
}

// STrack.multi_gmc (byte_tracker.py:108-125) of one track: mean = R8x8 . mean, mean[:2] += t,
// P = R8x8 . P . R8x8^T with R8x8 = kron(I4, H[:2, :2]); the covariance becomes dense (the warp
// couples x and y).  The mean's two products are rounded separately (dgemv's lanes); the
// covariance products accumulate with fma (dgemm's k loop) -- OpenBLAS's kernels, unpinned.
__device__ void kf_gmc(Slot& t, const double* Hw) {
  const double R00 = Hw[0], R01 = Hw[1], R10 = Hw[3], R11 = Hw[4];
  if (!t.dense) {
    for (int k = 0; k < 64; ++k) t.Pd[k] = 0.0;
    for (int c = 0; c < 4; ++c) {
      t.Pd[9 * c] = t.P[4 * c];
      t.Pd[8 * c + c + 4] = t.P[4 * c + 1];
      t.Pd[8 * (c + 4) + c] = t.P[4 * c + 2];
      t.Pd[9 * (c + 4)] = t.P[4 * c + 3];
    }
    t.dense = 1;
  }
  for (int p = 0; p < 4; ++p) {
    const double m0 = t.mean[2 * p], m1 = t.mean[2 * p + 1];
    t.mean[2 * p] = R00 * m0 + R01 * m1;
    t.mean[2 * p + 1] = R10 * m0 + R11 * m1;
  }
  t.mean[0] = t.mean[0] + Hw[2];
  t.mean[1] = t.mean[1] + Hw[5];
  double A[64];
  for (int p = 0; p < 4; ++p)
    for (int j = 0; j < 8; ++j) {
      const double a = t.Pd[8 * (2 * p) + j], b = t.Pd[8 * (2 * p + 1) + j];
      A[8 * (2 * p) + j] = fma(R01, b, R00 * a);
      A[8 * (2 * p + 1) + j] = fma(R11, b, R10 * a);
    }
  for (int i = 0; i < 8; ++i)
    for (int q = 0; q < 4; ++q) {
      const double a = A[8 * i + 2 * q], b = A[8 * i + 2 * q + 1];
      t.Pd[8 * i + 2 * q] = fma(b, R01, a * R00);
      t.Pd[8 * i + 2 * q + 1] = fma(b, R11, a * R10);
    }
  t.mean32 = 0;
}

// update (kalman_filter.py:205-236) with project (:135-163 / :401-429) and a float32 measurement
__device__ void kf_update(Slot& t, const float* meas, bool xywh) {
  double r[4];
  if (t.mean32) {
    const float wp = (float)WP;
    const float m2 = (float)t.mean[2], m3 = (float)t.mean[3];
    for (int c = 0; c < 4; ++c) {
      const float s = wp * (xywh ? ((c & 1) ? m3 : m2) : m3);
      if (xywh) r[c] = (double)(s * s);          // all-float32 list: squares in float32
      else r[c] = c == 2 ? 1e-1 * 1e-1 : (double)s * (double)s;  // 1e-1 makes it float64
    }
  } else {
    for (int c = 0; c < 4; ++c) {
      const double s = c == 2 && !xywh ? 1e-1 : WP * (xywh ? ((c & 1) ? t.mean[3] : t.mean[2]) : t.mean[3]);
      r[c] = s * s;
    }
  }
  if (t.dense) {
    kf_update_dense(t, meas, r);
    return;
  }
  for (int c = 0; c < 4; ++c) {
    const double p = t.P[4 * c], a = t.P[4 * c + 1], b = t.P[4 * c + 2], v = t.P[4 * c + 3];
    const double S = p + r[c];
    const double il = 1.0 / sqrt(S);  // cho_factor: sqrt(S); cho_solve: dtrsm by the reciprocal, twice
    const double kc = (p * il) * il, kv = (b * il) * il;
    const double inn = (double)meas[c] - t.mean[c];
    t.mean[c] = t.mean[c] + inn * kc;
    t.mean[c + 4] = t.mean[c + 4] + inn * kv;
    t.P[4 * c + 0] = p - kc * (S * kc);
    t.P[4 * c + 1] = a - kc * (S * kv);
    t.P[4 * c + 2] = b - kv * (S * kc);
    t.P[4 * c + 3] = v - kv * (S * kv);
  }
  t.mean32 = 0;
}

// tlwh_to_xyah / tlwh_to_xywh of a detection's float32 tlwh (byte_tracker.py:206-212, bot_sort.py:148-153)
__device__ __forceinline__ void det_measurement(const float* tl, bool xywh, float* m) {
  m[0] = tl[0] + tl[2] / 2.0f;
  m[1] = tl[1] + tl[3] / 2.0f;
  m[2] = xywh ? tl[2] : tl[2] / tl[3];
  m[3] = tl[3];
}

// ---------------------------------------------------------------------------- CPython set order
// list(frozenset(range(n)) - frozenset(excluded)) (oracle/pyset_order.py): excluded[k] != 0
// marks the excluded keys, n_ex their count.  One thread; the table lives in LDS.
__device__ int pyset_diff(int n, const int* excluded, int n_ex, int* table, int* out) {
  int cnt = 0;
  if ((n >> 2) > n_ex) {  // copy-and-discard: ascending
    for (int k = 0; k < n; ++k)
      if (!excluded[k]) out[cnt++] = k;
    return cnt;
  }
  int size = 8, mask = 7, fill = 0;
  for (int i = 0; i < size; ++i) table[i] = -1;
  for (int key = 0; key < n; ++key) {
    if (excluded[key]) continue;
    // set_add_entry (keys are distinct and non-negative: hash == key)
    size_t perturb = (size_t)key;
    int i = key & mask;
    bool done = false;
    while (!done) {
      const int probes = (i + 9 <= mask) ? 9 : 0;
      for (int j = 0; j <= probes; ++j)
        if (table[i + j] < 0) {
          table[i + j] = key;
          done = true;
          break;
        }
      if (!done) {
        perturb >>= 5;
        i = (int)(((size_t)i * 5 + 1 + perturb) & (size_t)mask);
      }
    }
    ++fill;
    if (fill * 5 >= mask * 3) {  // set_table_resize(used * 4): re-insert in table order
      int ns = 8;
      while (ns <= fill * 4) ns <<= 1;
      int m = 0;
      for (int s = 0; s < size; ++s)
        if (table[s] >= 0) out[m++] = table[s];
      size = ns;
      mask = ns - 1;
      for (int s = 0; s < size; ++s) table[s] = -1;
      for (int q = 0; q < m; ++q) {
        const int k2 = out[q];
        size_t pt = (size_t)k2;
        int ii = k2 & mask;
        while (true) {
          if (table[ii] < 0) {
            table[ii] = k2;
            break;
          }
          bool put = false;
          if (ii + 9 <= mask)
            for (int j = 1; j <= 9; ++j)
              if (table[ii + j] < 0) {
                table[ii + j] = k2;
                put = true;
                break;
              }
          if (put) break;
          pt >>= 5;
          ii = (int)(((size_t)ii * 5 + 1 + pt) & (size_t)mask);
        }
      }
    }
  }
  for (int s = 0; s < size; ++s)
    if (table[s] >= 0) out[cnt++] = table[s];
  return cnt;
}

// ---------------------------------------------------------------------------- assignment
// Hungarian method (shortest augmenting paths with potentials) on an n x m (n <= m) sub-problem;
// a(i, j) is the cost of row i, column j; writes col4row[n].  Work arrays: 6 (m + 2) doubles.
template <class A>
__device__ void hungarian(int n, int m, A a, double* w, int* col4row) {
  double* u = w;
  double* v = u + (m + 2);
  double* minv = v + (m + 2);
  int* p = (int*)(minv + (m + 2));
  int* way = p + (m + 2);
  int* used = way + (m + 2);
  for (int j = 0; j <= m; ++j) {
    u[j] = 0.0;
    v[j] = 0.0;
    p[j] = 0;
    way[j] = 0;
  }
  for (int i = 1; i <= n; ++i) {
    p[0] = i;
    int j0 = 0;
    for (int j = 0; j <= m; ++j) {
      minv[j] = INFINITY;
      used[j] = 0;
    }
    do {
      used[j0] = 1;
      const int i0 = p[j0];
      double delta = INFINITY;
      int j1 = 0;
      for (int j = 1; j <= m; ++j)
        if (!used[j]) {
          const double cur = a(i0 - 1, j - 1) - u[i0] - v[j];
          if (cur < minv[j]) {
            minv[j] = cur;
            way[j] = j0;
          }
          if (minv[j] < delta) {
            delta = minv[j];
            j1 = j;
          }
        }
      for (int j = 0; j <= m; ++j) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      j0 = j1;
    } while (p[j0] != 0);
    do {
      const int j1 = way[j0];
      p[j0] = p[j1];
      j0 = j1;
    } while (j0);
  }
  for (int j = 1; j <= m; ++j)
    if (p[j]) col4row[p[j] - 1] = j - 1;
}

// linear_assignment (matching.py:20-61) of the nr x nc matrix in C (row-major, global): mrow /
// mcol get the kept matches, urow / ucol the unmatched indices in the reference's list order;
// misc[Q_A] / misc[Q_B] their counts.  All threads call it.
//   lap branch (g.cfg.lap, the reference's default): lapjv on the extended problem (cost_limit /
//   2 per dummy pairing, 0 dummy-dummy) minimises sum over matched pairs of (cost - thresh), so
//   only pairs with cost < thresh (float64, the cost_limit's precision) are edges, a component
//   of them is solved on min(cost - thresh, 0), every assigned edge is kept, and the unmatched
//   lists are ascending (np.where).
//   scipy branch: pairs that overlap (cost < 1) are the edges, a component is solved on the
//   cost itself, the float32 `cost <= thresh` filter follows, frozenset-ordered unmatched lists.
__device__ void assign(const Dev& g, const Lds& L, float* C, int* E, double* hw, int nr, int nc, float thresh,
                       double thresh64) {
  const bool lap = g.cfg.lap != 0;
  const int tid = threadIdx.x;
  int* wsum = L.misc + Q_WSUM;
  for (int r = tid; r < nr; r += NT) L.mrow[r] = -1;
  for (int c = tid; c < nc; c += NT) L.mcol[c] = -1;
  if (tid == 0) {
    L.misc[Q_E] = 0;
    L.misc[Q_CHG] = 0;
  }
  if (nr == 0 || nc == 0) {  // cost_matrix.size == 0: tuple(range(...))
    __syncthreads();
    for (int r = tid; r < nr; r += NT) L.urow[r] = r;
    for (int c = tid; c < nc; c += NT) L.ucol[c] = c;
    if (tid == 0) {
      L.misc[Q_A] = nr;
      L.misc[Q_B] = nc;
    }
    __syncthreads();
    return;
  }
  // overlapping pairs (cost < 1) and component labels over rows [0, nr) and columns [nr, nr + nc)
  const int nn = nr + nc;
  for (int v = tid; v < nn; v += NT) L.label[v] = v;
  __syncthreads();
  for (int e = tid; e < nr * nc; e += NT)
    if (lap ? (double)C[e] < thresh64 : C[e] < 1.0f) E[atomicAdd(&L.misc[Q_E], 1)] = e;
  __syncthreads();
  const int ne = L.misc[Q_E];
  for (int it = 0; it < nn + 2; ++it) {  // min-label propagation; converges within a component's diameter
    int chg = 0;
    for (int k = tid; k < ne; k += NT) {
      const int e = E[k], r = e / nc, c = e - r * nc;
      const int a = L.label[r], b = L.label[nr + c];
      const int m = a < b ? a : b;
      if (a != m) {
        atomicMin(&L.label[r], m);
        chg = 1;
      }
      if (b != m) {
        atomicMin(&L.label[nr + c], m);
        chg = 1;
      }
    }
    __syncthreads();
    for (int v = tid; v < nn; v += NT) {  // pointer jumping
      const int l = L.label[v], ll = L.label[l];
      if (ll < l) {
        atomicMin(&L.label[v], ll);
        chg = 1;
      }
    }
    if (chg) L.misc[Q_CHG] = it + 1;
    __syncthreads();
    if (L.misc[Q_CHG] != it + 1) break;
    __syncthreads();
  }
  // components: roots are rows r with label[r] == r that have an edge (a component's minimum
  // node is a row when it has one: rows come first)
  for (int v = tid; v < nn; v += NT) L.flag[v] = 0;
  __syncthreads();
  for (int k = tid; k < ne; k += NT) {
    const int e = E[k], r = e / nc;
    L.flag[r] = 1;  // has an edge
  }
  __syncthreads();
  int ncomp = 0;
  for (int base = 0; base < nr; base += NT) {
    const int r = base + tid;
    const int root = (r < nr && L.flag[r] && L.label[r] == r) ? 1 : 0;
    int tot;
    const int pos = ncomp + block_scan(root, wsum, tot);
    if (root) L.urow[pos] = r;  // urow: scratch list of component roots
    ncomp += tot;
  }
  __syncthreads();
  // one thread per component: gather its rows / columns (ascending), solve, keep cost <= thresh
  for (int ci = tid; ci < ncomp; ci += NT) {
    const int root = L.urow[ci];
    double* w = hw + (size_t)tid * 6 * (size_t)(g.T + g.D + 2);
    int* rows = (int*)(hw + (size_t)NT * 6 * (size_t)(g.T + g.D + 2)) + (size_t)tid * (2 * g.T + g.D);
    int kr = 0, kc = 0;
    for (int r = root; r < nr; ++r)
      if (L.label[r] == root) rows[kr++] = r;
    int* cols = rows + kr;
    for (int c = 0; c < nc; ++c)
      if (L.label[nr + c] == root) cols[kc++] = c;
    int* res = cols + kc;  // [min(kr, kc)] (rows + cols + res <= 2 T + D ints per thread)
    // lap: cost - thresh where negative (an edge), else 0 (no better than both unmatched)
    auto cost = [&](int r, int c) {
      const double v = (double)C[r * nc + c];
      return lap ? fmin(v - thresh64, 0.0) : v;
    };
    auto keep = [&](int r, int c) { return lap ? (double)C[r * nc + c] < thresh64 : C[r * nc + c] <= thresh; };
    if (kr <= kc) {
      hungarian(kr, kc, [&](int i, int j) { return cost(rows[i], cols[j]); }, w, res);
      for (int i = 0; i < kr; ++i) {
        const int r = rows[i], c = cols[res[i]];
        if (keep(r, c)) {
          L.mrow[r] = c;
          L.mcol[c] = r;
        }
      }
    } else {
      hungarian(kc, kr, [&](int i, int j) { return cost(rows[j], cols[i]); }, w, res);
      for (int i = 0; i < kc; ++i) {
        const int c = cols[i], r = rows[res[i]];
        if (keep(r, c)) {
          L.mrow[r] = c;
          L.mcol[c] = r;
        }
      }
    }
  }
  __syncthreads();
  // unmatched lists: lap branch or no kept match, ascending; else frozenset order
  int nm = 0;
  for (int base = 0; base < nr; base += NT) {
    const int r = base + tid;
    int tot;
    (void)block_scan(r < nr && L.mrow[r] >= 0, wsum, tot);
    nm += tot;
  }
  for (int r = tid; r < nr; r += NT) L.flag[r] = L.mrow[r] >= 0 ? 1 : 0;
  for (int c = tid; c < nc; c += NT) L.flag[nr + c] = L.mcol[c] >= 0 ? 1 : 0;
  __syncthreads();
  if (tid == 0) {
    if (nm == 0 || lap) {  // ascending: list(np.arange) / np.where(x < 0)
      int a = 0, b = 0;
      for (int r = 0; r < nr; ++r)
        if (!L.flag[r]) L.urow[a++] = r;
      for (int c = 0; c < nc; ++c)
        if (!L.flag[nr + c]) L.ucol[b++] = c;
      L.misc[Q_A] = a;
      L.misc[Q_B] = b;
    } else {
      L.misc[Q_A] = pyset_diff(nr, L.flag, nm, L.ptab, L.urow);
      L.misc[Q_B] = pyset_diff(nc, L.flag + nr, nm, L.ptab, L.ucol);
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------- the step
// Matched pair: STrack.update (byte_tracker.py:156-183) or re_activate (:140-154).
__device__ void apply_match(Slot& t, const Lds& L, int d, int frame, bool xywh, bool* refound) {
  float m[4];
  det_measurement(&L.dtl[4 * d], xywh, m);
  const bool was_tracked = t.state == TRACKED;
  kf_update(t, m, xywh);
  if (was_tracked) t.tracklet_len += 1;
  else t.tracklet_len = 0;
  t.state = TRACKED;
  t.is_activated = 1;
  t.frame_id = frame;
  t.score = L.dsc[d];
  t.cls = L.dcl[d];
  t.idx = L.didx[d];
  *refound = !was_tracked;
}

__global__ void __launch_bounds__(NT) bt_step_kernel(Dev g, const float* __restrict__ dets, const int* __restrict__ counts,
                                                     const double* __restrict__ warp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int T = g.T, Dm = g.D;
  const Cfg& cf = g.cfg;
  const bool xywh = cf.xywh != 0;
  Lds L = carve(smem, T, Dm);
  Hdr& H = g.hdr[s];
  Slot* slots = g.slots + (size_t)s * T;
  int* tracked = g.tracked + (size_t)s * T;
  int* lost = g.lost + (size_t)s * T;
  float* C = g.cost + (size_t)s * T * Dm;
  int* E = g.edges + (size_t)s * T * Dm;
  double* hw = g.hung + (size_t)s * g.hung_stride;
  int* wsum = L.misc + Q_WSUM;

  int nd = counts[s];
  if (nd < 0) nd = 0;
  if (nd > Dm) nd = Dm;
  const int frame = H.frame_id + 1;
  const int ntr = H.n_tracked, nlo = H.n_lost;
  if (tid < 16) L.misc[tid] = 0;
  // detections: Boxes.xywh (float32), the float64 row [xywh, idx], xywh2ltwh -> float32 tlwh
  for (int d = tid; d < nd; d += NT) {
    const float* q = dets + ((size_t)s * Dm + d) * 6;
    const float x1 = q[0], y1 = q[1], x2 = q[2], y2 = q[3];
    const float cx = (x1 + x2) / 2.0f, cy = (y1 + y2) / 2.0f, w = x2 - x1, h = y2 - y1;
    float* tl = &L.dtl[4 * d];
    tl[0] = (float)((double)cx - (double)w / 2.0);
    tl[1] = (float)((double)cy - (double)h / 2.0);
    tl[2] = w;
    tl[3] = h;
    float* xy = &L.dxy[4 * d];
    xy[0] = tl[0];
    xy[1] = tl[1];
    xy[2] = tl[2] + tl[0];
    xy[3] = tl[3] + tl[1];
    L.dsc[d] = q[4];
    L.dcl[d] = q[5];
  }
  __syncthreads();
  // score subsets in detection order (byte_tracker.py:307-320); idx = position in the subset
  int nh = 0, n2 = 0;
  for (int base = 0; base < nd; base += NT) {
    const int d = base + tid;
    const float sc = d < nd ? L.dsc[d] : 0.0f;
    const int fh = (d < nd && sc >= cf.th_high) ? 1 : 0;
    const int f2 = (d < nd && sc > cf.th_low && sc < cf.th_high) ? 1 : 0;
    int th, t2;
    const int ph = nh + block_scan(fh, wsum, th);
    const int p2 = n2 + block_scan(f2, wsum, t2);
    if (fh) {
      L.hi[ph] = d;
      L.didx[d] = (double)ph;
    }
    if (f2) {
      L.se[p2] = d;
      L.didx[d] = (double)p2;
    }
    nh += th;
    n2 += t2;
  }
  // unconfirmed / activated tracked, strack_pool = joint(activated tracked, lost) (:322-330)
  int nun = 0, npool = 0;
  for (int base = 0; base < ntr; base += NT) {
    const int i = base + tid;
    const int sl = i < ntr ? tracked[i] : 0;
    const int act = i < ntr ? slots[sl].is_activated : 0;
    int tu, ta;
    const int pu = nun + block_scan(i < ntr && !act, wsum, tu);
    const int pa = npool + block_scan(i < ntr && act, wsum, ta);
    if (i < ntr) {
      if (act) L.pool[pa] = sl;
      else L.unc[pu] = sl;
    }
    nun += tu;
    npool += ta;
  }
  for (int i = tid; i < nlo; i += NT) L.pool[npool + i] = lost[i];
  npool += nlo;
  __syncthreads();
  // multi_predict (byte_tracker.py:93-106 / bot_sort.py:128-142): a batch of only float32 means
  // stays float32 for the motion noise
  {
    int any64 = 0;
    for (int i = tid; i < npool; i += NT) any64 |= slots[L.pool[i]].mean32 ? 0 : 1;
    if (any64) L.misc[Q_N] = 1;
    __syncthreads();
    const bool f32 = L.misc[Q_N] == 0;
    for (int i = tid; i < npool; i += NT) {
      Slot& t = slots[L.pool[i]];
      if (t.state != TRACKED) {
        t.mean[7] = 0.0;
        if (xywh) t.mean[6] = 0.0;
      }
      kf_predict(t, xywh, f32);
    }
  }
  __syncthreads();
  if (warp) {  // GMC (byte_tracker.py:333-340): multi_gmc(strack_pool, warp), multi_gmc(unconfirmed, warp)
    const double* Hw = warp + (size_t)s * 6;
    for (int i = tid; i < npool + nun; i += NT) kf_gmc(slots[i < npool ? L.pool[i] : L.unc[i - npool]], Hw);
    __syncthreads();
  }
  int nact = 0, nref = 0, nlnew = 0, nrnew = 0;
  // first association: strack_pool x high detections, fused IoU cost, match_thresh (:342-353)
  for (int i = tid; i < npool; i += NT) track_xyxy(slots[L.pool[i]], xywh, &L.txy[4 * i]);
  __syncthreads();
  for (int e = tid; e < npool * nh; e += NT) {
    const int r = e / nh, c = e - r * nh;
    const int d = L.hi[c];
    C[e] = pair_cost(&L.txy[4 * r], &L.dxy[4 * d], L.dsc[d], cf.fuse != 0);
  }
  __syncthreads();
  assign(g, L, C, E, hw, npool, nh, cf.th_match, cf.th_match_f64);
  int nu1 = L.misc[Q_A], nud1 = L.misc[Q_B];
  // matches in row order (linear_sum_assignment returns rows ascending)
  for (int base = 0; base < npool; base += NT) {
    const int r = base + tid;
    const int m = r < npool ? L.mrow[r] : -1;
    bool rf = false;
    if (m >= 0) apply_match(slots[L.pool[r]], L, L.hi[m], frame, xywh, &rf);
    int ta, tr;
    const int pa = nact + block_scan(m >= 0 && !rf, wsum, ta);
    const int pr = nref + block_scan(m >= 0 && rf, wsum, tr);
    if (m >= 0) {
      if (rf) L.ref[pr] = L.pool[r];
      else L.act[pa] = L.pool[r];
    }
    nact += ta;
    nref += tr;
  }
  // high detections left, in the unmatched-column order (:376)
  for (int k = tid; k < nud1; k += NT) L.drem[k] = L.hi[L.ucol[k]];
  // r_tracked_stracks: unmatched pool rows (unmatched-row order) still Tracked (:356)
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int k = 0; k < nu1; ++k) {
      const int sl = L.pool[L.urow[k]];
      if (slots[sl].state == TRACKED) L.rtr[n++] = sl;
    }
    L.misc[Q_N] = n;
  }
  __syncthreads();
  const int nrt = L.misc[Q_N];
  // second association: r_tracked x low-score detections, plain IoU cost, 0.5 (:358-368)
  for (int i = tid; i < nrt; i += NT) track_xyxy(slots[L.rtr[i]], xywh, &L.txy[4 * i]);
  __syncthreads();
  for (int e = tid; e < nrt * n2; e += NT) {
    const int r = e / n2, c = e - r * n2;
    C[e] = pair_cost(&L.txy[4 * r], &L.dxy[4 * L.se[c]], 1.0f, false);
  }
  __syncthreads();
  assign(g, L, C, E, hw, nrt, n2, 0.5f, 0.5);
  const int nu2 = L.misc[Q_A];
  for (int base = 0; base < nrt; base += NT) {
    const int r = base + tid;
    const int m = r < nrt ? L.mrow[r] : -1;
    bool rf = false;
    if (m >= 0) apply_match(slots[L.rtr[r]], L, L.se[m], frame, xywh, &rf);
    int ta, tr;
    const int pa = nact + block_scan(m >= 0 && !rf, wsum, ta);
    const int pr = nref + block_scan(m >= 0 && rf, wsum, tr);
    if (m >= 0) {
      if (rf) L.ref[pr] = L.rtr[r];
      else L.act[pa] = L.rtr[r];
    }
    nact += ta;
    nref += tr;
  }
  __syncthreads();
  // unmatched r_tracked -> mark_lost, in the unmatched order (:370-374)
  if (tid == 0) {
    for (int k = 0; k < nu2; ++k) {
      Slot& t = slots[L.rtr[L.urow[k]]];
      if (t.state != LOST) {
        t.state = LOST;
        L.lnew[nlnew++] = L.rtr[L.urow[k]];
      }
    }
    L.misc[Q_LNEW] = nlnew;
  }
  __syncthreads();
  nlnew = L.misc[Q_LNEW];
  // unconfirmed x remaining high detections, fused cost, 0.7 (:376-385)
  for (int i = tid; i < nun; i += NT) track_xyxy(slots[L.unc[i]], xywh, &L.txy[4 * i]);
  __syncthreads();
  for (int e = tid; e < nun * nud1; e += NT) {
    const int r = e / nud1, c = e - r * nud1;
    const int d = L.drem[c];
    C[e] = pair_cost(&L.txy[4 * r], &L.dxy[4 * d], L.dsc[d], cf.fuse != 0);
  }
  __syncthreads();
  assign(g, L, C, E, hw, nun, nud1, 0.7f, 0.7);
  const int nuu = L.misc[Q_A], nud3 = L.misc[Q_B];
  for (int base = 0; base < nun; base += NT) {
    const int r = base + tid;
    const int m = r < nun ? L.mrow[r] : -1;
    bool rf = false;
    if (m >= 0) apply_match(slots[L.unc[r]], L, L.drem[m], frame, xywh, &rf);
    int ta;
    const int pa = nact + block_scan(m >= 0, wsum, ta);
    if (m >= 0) L.act[pa] = L.unc[r];
    nact += ta;
  }
  __syncthreads();
  // tid 0: removals, new tracks, the new lists (sequential list semantics of :382-406)
  if (tid == 0) {
    for (int k = 0; k < nuu; ++k) {  // unconfirmed without a match -> removed
      const int sl = L.unc[L.urow[k]];
      slots[sl].state = REMOVED;
      L.rnew[nrnew++] = sl;
    }
    // free slots: not referenced by the previous lists
    for (int v = 0; v < T; ++v) L.flag[v] = 0;
    for (int i = 0; i < ntr; ++i) L.flag[tracked[i]] = 1;
    for (int i = 0; i < nlo; ++i) L.flag[lost[i]] = 1;
    int fs = 0, nnew = 0, nover = 0;
    for (int k = 0; k < nud3; ++k) {  // new tracks in the unmatched order (:386-392)
      const int d = L.drem[L.ucol[k]];
      if (L.dsc[d] < cf.th_new) continue;
      while (fs < T && L.flag[fs]) ++fs;
      if (fs >= T) {
        ++nover;
        continue;
      }
      Slot& t = slots[fs];
      L.flag[fs] = 1;
      float m[4];
      det_measurement(&L.dtl[4 * d], xywh, m);
      kf_initiate(t, m, xywh);
      t.score = L.dsc[d];
      t.cls = L.dcl[d];
      t.idx = L.didx[d];
      t.tracklet_len = 0;
      t.state = TRACKED;
      t.is_activated = frame == 1 ? 1 : 0;
      t.frame_id = frame;
      t.start_frame = frame;
      t.track_id = 0;  // bt_ids_kernel
      t.rm_seq = -1;
      g.newslots[(size_t)s * Dm + nnew] = fs;
      g.newrow[(size_t)s * Dm + nnew] = -1;
      ++nnew;
      L.act[nact++] = fs;
    }
    // lost tracks past max_time_lost -> removed (:394-397)
    for (int i = 0; i < nlo; ++i) {
      Slot& t = slots[lost[i]];
      if (frame - t.frame_id > cf.max_time_lost) {
        t.state = REMOVED;
        L.rnew[nrnew++] = lost[i];
      }
    }
    // tracked = [t in tracked if Tracked] ++ activated ++ refind (joint by id; :399-401)
    // (membership by slot: a slot is one track)
    for (int v = 0; v < T; ++v) L.flag[v] = 0;
    int nt2 = 0;
    int* ntrk = L.label;  // scratch [T + D]
    for (int i = 0; i < ntr; ++i)
      if (slots[tracked[i]].state == TRACKED) {
        ntrk[nt2++] = tracked[i];
        L.flag[tracked[i]] = 1;
      }
    for (int k = 0; k < nact; ++k)
      if (!L.flag[L.act[k]]) {
        ntrk[nt2++] = L.act[k];
        L.flag[L.act[k]] = 1;
      }
    for (int k = 0; k < nref; ++k)
      if (!L.flag[L.ref[k]]) {
        ntrk[nt2++] = L.ref[k];
        L.flag[L.ref[k]] = 1;
      }
    // lost = sub(lost, tracked) ++ lost_new, then sub(., removed_stracks of earlier steps) (:402-404)
    int* nlst = L.urow;  // scratch [T]
    int nl2 = 0;
    const int rm_lo = H.rm_total - H.rm_len;  // removed_stracks window: appends [rm_lo, rm_total)
    for (int i = 0; i < nlo; ++i)
      if (!L.flag[lost[i]]) nlst[nl2++] = lost[i];
    for (int k = 0; k < nlnew; ++k) nlst[nl2++] = L.lnew[k];
    {
      int q = 0;
      for (int i = 0; i < nl2; ++i) {
        const Slot& t = slots[nlst[i]];
        if (!(t.rm_seq >= 0 && t.rm_seq >= rm_lo)) nlst[q++] = nlst[i];
      }
      nl2 = q;
    }
    // remove_duplicate_stracks(tracked, lost) (:471-485): pairs with IoU distance < 0.15
    {
      int* fa = L.flag;   // [T]: tracked position p dropped
      int* fbl = L.ptab;  // [PTAB >= T]: lost position q dropped
      for (int p = 0; p < nt2; ++p) fa[p] = 0;
      for (int q = 0; q < nl2; ++q) fbl[q] = 0;
      for (int p = 0; p < nt2; ++p) {
        float a[4];
        track_xyxy(slots[ntrk[p]], xywh, a);
        for (int q = 0; q < nl2; ++q) {
          float b[4];
          track_xyxy(slots[nlst[q]], xywh, b);
          if (pair_cost(a, b, 1.0f, false) < 0.15f) {
            const Slot& tp = slots[ntrk[p]];
            const Slot& tq = slots[nlst[q]];
            if (tp.frame_id - tp.start_frame > tq.frame_id - tq.start_frame) fbl[q] = 1;
            else fa[p] = 1;
          }
        }
      }
      int a2 = 0;
      for (int p = 0; p < nt2; ++p)
        if (!fa[p]) tracked[a2++] = ntrk[p];
      int b2 = 0;
      for (int q = 0; q < nl2; ++q)
        if (!fbl[q]) lost[b2++] = nlst[q];
      nt2 = a2;
      nl2 = b2;
    }
    // removed_stracks.extend(removed); clip to the last 999 past 1000 (:406-408)
    for (int k = 0; k < nrnew; ++k) slots[L.rnew[k]].rm_seq = H.rm_total + k;
    H.rm_total += nrnew;
    H.rm_len += nrnew;
    if (H.rm_len > 1000) H.rm_len = 999;
    // outputs: [x.result for x in tracked if x.is_activated] (:410)
    int nout = 0;
    for (int p = 0; p < nt2; ++p) {
      const Slot& t = slots[tracked[p]];
      if (!t.is_activated) continue;
      float* row = g.rows + ((size_t)s * T + nout) * 8;
      track_xyxy(t, xywh, row);
      row[4] = (float)t.track_id;
      row[5] = t.score;
      row[6] = t.cls;
      row[7] = (float)t.idx;
      if (t.track_id == 0)  // activated this step (frame 1): bt_ids_kernel writes the id
        for (int k = 0; k < nnew; ++k)
          if (g.newslots[(size_t)s * Dm + k] == tracked[p]) g.newrow[(size_t)s * Dm + k] = nout;
      ++nout;
    }
    H.n_tracked = nt2;
    H.n_lost = nl2;
    H.frame_id = frame;
    H.n_new = nnew;
    H.n_out = nout;
    H.n_overflow += nover;
    g.counts[s] = nout;
  }
}

// BaseTrack.next_id across streams: streams in index order, each stream's new tracks in their
// activation order.
__global__ void bt_ids_kernel(Dev g, int S) {
  const int s = blockIdx.x;
  if (s >= S || threadIdx.x != 0) return;
  long long base = *g.ids;
  for (int q = 0; q < s; ++q) base += g.hdr[q].n_new;
  const int nn = g.hdr[s].n_new;
  for (int k = 0; k < nn; ++k) {
    const int sl = g.newslots[(size_t)s * g.D + k];
    const long long id = base + 1 + k;
    g.slots[(size_t)s * g.T + sl].track_id = (int)id;
    const int r = g.newrow[(size_t)s * g.D + k];
    if (r >= 0) g.rows[((size_t)s * g.T + r) * 8 + 4] = (float)id;
  }
}

__global__ void bt_ids_advance_kernel(Dev g, int S) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  long long n = 0;
  for (int q = 0; q < S; ++q) n += g.hdr[q].n_new;
  *g.ids += n;
}

__global__ void bt_reset_kernel(Dev g, int S) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < S) {
    Hdr& H = g.hdr[s];
    H = Hdr{};
    g.counts[s] = 0;
  }
  if (s == 0) *g.ids = 0;
}

}  // namespace bt
}  // namespace yk

struct yk_bt {
  yk_ctx* ctx;
  int S;
  yk_bt_cfg cfg;
  yk::bt::Dev dev;
  size_t lds;
};

extern "C" {

int yk_bt_create(yk_ctx* ctx, int n_streams, const yk_bt_cfg* cfg, yk_bt** out) {
  YK_CHECK_ARG(ctx && cfg && out, "yk_bt_create: NULL argument");
  YK_CHECK_ARG(n_streams >= 1 && n_streams <= 4096, "yk_bt_create: n_streams out of range");
  YK_CHECK_ARG(cfg->max_tracks >= 1 && cfg->max_tracks <= 1024, "yk_bt_create: max_tracks must be in [1, 1024]");
  YK_CHECK_ARG(cfg->max_dets >= 1 && cfg->max_dets <= 1024, "yk_bt_create: max_dets must be in [1, 1024]");
  YK_CHECK_ARG(cfg->kind == YK_BT_BYTETRACK || cfg->kind == YK_BT_BOTSORT, "yk_bt_create: unknown tracker kind");
  YK_CHECK_ARG(cfg->frame_rate > 0 && cfg->track_buffer >= 0, "yk_bt_create: frame_rate / track_buffer");
  const int T = cfg->max_tracks, D = cfg->max_dets;
  const size_t lds = yk::bt::lds_bytes(T, D);
  YK_CHECK_ARG(lds <= 160 * 1024, "yk_bt_create: max_tracks x max_dets exceed the 160 KiB LDS budget");
  yk::DeviceGuard guard(ctx->device);
  auto* t = new yk_bt{};
  t->ctx = ctx;
  t->S = n_streams;
  t->cfg = *cfg;
  t->lds = lds;
  yk::bt::Dev& g = t->dev;
  g.T = T;
  g.D = D;
  g.cfg.th_high = cfg->track_high_thresh;
  g.cfg.th_low = cfg->track_low_thresh;
  g.cfg.th_new = cfg->new_track_thresh;
  g.cfg.th_match = cfg->match_thresh;
  g.cfg.max_time_lost = (int)((double)cfg->frame_rate / 30.0 * (double)cfg->track_buffer);
  g.cfg.fuse = cfg->fuse_score ? 1 : 0;
  g.cfg.xywh = cfg->kind == YK_BT_BOTSORT ? 1 : 0;
  g.cfg.lap = cfg->assignment == YK_BT_SCIPY ? 0 : 1;
  g.cfg.th_match_f64 = cfg->match_thresh_f64 != 0.0 ? cfg->match_thresh_f64 : (double)cfg->match_thresh;
  const size_t S = n_streams;
  hipError_t e = hipSuccess;
  auto A = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  A((void**)&g.slots, S * T * sizeof(yk::bt::Slot));
  A((void**)&g.hdr, S * sizeof(yk::bt::Hdr));
  A((void**)&g.tracked, S * T * sizeof(int));
  A((void**)&g.lost, S * T * sizeof(int));
  A((void**)&g.newslots, S * D * sizeof(int));
  A((void**)&g.newrow, S * D * sizeof(int));
  A((void**)&g.cost, S * (size_t)T * D * sizeof(float));
  A((void**)&g.edges, S * (size_t)T * D * sizeof(int));
  g.hung_stride = (size_t)yk::bt::NT * 6 * (T + D + 2) + ((size_t)yk::bt::NT * (2 * T + D) + 1) / 2;
  A((void**)&g.hung, S * g.hung_stride * sizeof(double));
  A((void**)&g.rows, S * T * 8 * sizeof(float));
  A((void**)&g.counts, S * sizeof(int));
  A((void**)&g.ids, sizeof(long long));
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_bt_create: hipMalloc failed: ") + hipGetErrorString(e));
    yk_bt_destroy(t);
    return YK_ERR_HIP;
  }
  if (hipFuncSetAttribute((const void*)yk::bt::bt_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    (void)hipGetLastError();
  int rc = yk_bt_reset(t, nullptr);
  if (rc != YK_OK) {
    yk_bt_destroy(t);
    return rc;
  }
  YK_HIP(hipDeviceSynchronize());
  *out = t;
  return YK_OK;
}

int yk_bt_destroy(yk_bt* t) {
  if (!t) return YK_OK;
  yk::DeviceGuard guard(t->ctx->device);
  yk::bt::Dev& g = t->dev;
  void* ptrs[] = {g.slots, g.hdr, g.tracked, g.lost, g.newslots, g.newrow, g.cost, g.edges, g.hung, g.rows, g.counts, g.ids};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete t;
  return YK_OK;
}

int yk_bt_reset(yk_bt* t, void* stream) {
  YK_CHECK_ARG(t, "yk_bt_reset: NULL tracker");
  yk::DeviceGuard guard(t->ctx->device);
  hipLaunchKernelGGL(yk::bt::bt_reset_kernel, dim3((t->S + 255) / 256), dim3(256), 0, (hipStream_t)stream, t->dev, t->S);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_bt_step(yk_bt* t, const float* dets, const int32_t* counts, void* stream) {
  return yk_bt_step_warp(t, dets, counts, nullptr, stream);
}

int yk_bt_step_warp(yk_bt* t, const float* dets, const int32_t* counts, const double* warp, void* stream) {
  YK_CHECK_ARG(t && dets && counts, "yk_bt_step: NULL argument");
  YK_CHECK_ARG(!warp || t->dev.cfg.xywh, "yk_bt_step_warp: a GMC warp needs the BoT-SORT tracker");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(yk::bt::bt_step_kernel, dim3(t->S), dim3(yk::bt::NT), t->lds, st, t->dev, dets, counts, warp);
  hipLaunchKernelGGL(yk::bt::bt_ids_kernel, dim3(t->S), dim3(64), 0, st, t->dev, t->S);
  hipLaunchKernelGGL(yk::bt::bt_ids_advance_kernel, dim3(1), dim3(64), 0, st, t->dev, t->S);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_bt_outputs(yk_bt* t, float** rows, int32_t** counts) {
  YK_CHECK_ARG(t, "yk_bt_outputs: NULL tracker");
  if (rows) *rows = t->dev.rows;
  if (counts) *counts = t->dev.counts;
  return YK_OK;
}

int yk_bt_download(yk_bt* t, float* host_rows, int32_t* host_counts, void* stream) {
  YK_CHECK_ARG(t && host_counts, "yk_bt_download: NULL argument");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  YK_HIP(hipMemcpyAsync(host_counts, t->dev.counts, t->S * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  if (host_rows) {
    const size_t T = t->dev.T;
    for (int s = 0; s < t->S; ++s)
      if (host_counts[s] > 0)
        YK_HIP(hipMemcpyAsync(host_rows + s * T * 8, t->dev.rows + s * T * 8, host_counts[s] * 8 * sizeof(float),
                              hipMemcpyDeviceToHost, st));
    YK_HIP(hipStreamSynchronize(st));
  }
  return YK_OK;
}

}  // extern "C"
