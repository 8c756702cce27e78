// Batched multi-stream Kalman tracker step for gfx950 (MI355X).
//
// One workgroup per video stream runs one complete
// EnhancedMultiTargetTracker.update() (kalman/enhanced_multi_target_tracker.py:42-132):
//   predict every live track            (kalman/enhanced_aircraft_kalman_tracker.py:184-203)
//   IoU candidates, mixed f32/f64        (enhanced_multi_target_tracker.py:180-232)
//   greedy association                   (enhanced_multi_target_tracker.py:234-270)
//   update / mark_as_lost / create / delete / get_track_info
//                                        (enhanced_aircraft_kalman_tracker.py:249-405)
//
// Filter structure.  F = I + unit(i,i+4), H = [I4 0], Q, R and the initial P are all
// block-structured over the four (position_c, velocity_c) pairs, so P keeps exactly the
// 16 entries P[c][c], P[c][c+4], P[c+4][c], P[c+4][c+4].  Each track is
// therefore four independent 2x2 filters.  The arithmetic below reproduces numpy's
// evaluation order and roundings (checked bitwise against oracle/tracker_ref.py):
//   F@P@F.T + Q  -> pp' = ((p+b)+(a+v)) + q_p, pv' = a+v, vp' = b+v, vv' = v + q_v
//   K = P H^T inv(S), inv(S) = diag(1/(p+R))
//   (I-KH)@P     -> pp' = (1-Kp)*p, pv' = (1-Kp)*a, vp' = (-Kv*p)+b, vv' = (-Kv*a)+v  (unfused)
// This file is compiled with -ffp-contract=off so no FMA contraction changes a rounding.
//
// Association is the sequential greedy match over candidates ordered by (IoU desc,
// row-major pair index asc), computed in parallel as rounds of "locally dominant" pairs
// (a pair that is the best free pair of both its detection row and its track column is
// exactly the pair the sequential scan would accept).  Ties are thereby broken like a
// stable argsort; numpy's default argsort is unstable on exact ties (SURVEY §7 hard parts).
#include <climits>

#include "yk_internal.h"

namespace yk {
namespace trk {

constexpr int NT = 256;                 // threads per stream workgroup (4 waves)
constexpr int NW = NT / 64;
constexpr int VH = YK_VEL_HIST;         // velocity ring (deque maxlen=50)
constexpr int TH = YK_TRAJ_HIST;        // trajectory ring (deque maxlen=150)
constexpr int TOUT = YK_TRAJ_OUT;       // trajectory points exported per row
constexpr double kPi = 3.141592653589793;  // np.pi
constexpr int PH = 32;                  // profiling words per stream (yk_tracker_phase_ticks)

// YK_POLICY_MOTION_RESET numerics.  The reference's reset logic mixes numpy float32 and float64
// scalars with python floats; NEP 50 (numpy 2) fixes every result's dtype: a numpy scalar op a
// python float keeps the numpy dtype (the python float is cast to it), f32 op f64 is f64, and
// np.asarray of a list is float32 only when every element is a float32 scalar.  Num carries a
// value (exact in double) and that dtype.
enum { K32 = 0, K64 = 1, KPY = 2 };
struct Num {
  double v;
  int k;
};
struct ResetDetail {  // one reset_reasons entry (motion_reset_kalman_tracker.py:222-229)
  int frame, reasons;
  double value[3], conf, cons;
};

struct Slot {
  static constexpr bool kPol = true;  // carries the motion-reset state (LSlot below does not)
  double x[8];
  double P[16];  // per coordinate c: [4c+0]=P[c][c] [4c+1]=P[c][c+4] [4c+2]=P[c+4][c] [4c+3]=P[c+4][c+4]
  double vavg[2], vstd[2], direction, speed, stability, pconf;
  double vh[VH][2];
  double vang[VH];  // arctan2(vy, vx) of each velocity entry, cached at push time
  double th[TH][2];
  int age, hits, hit_streak, tsu, is_lost, lost_frames, track_num, max_lost;
  int vh_len, vh_head, th_len, th_head;
  unsigned th_cnt;  // trajectory points appended since creation (+2^20 at a history reset), mod 2^32:
                    // yk_track_out.traj_count (unsigned: a long-lived track's count wraps, defined)
  // YK_POLICY_MOTION_RESET (MotionResetKalmanTracker, motion_reset_kalman_tracker.py:28-65)
  int policy;
  int reset_count, last_reset;  // last_reset_frame: -999 at creation
  int ph_len, ph_head, bh_len, bh_head, ms_len, ms_head, dl_len, dl_head;
  int reason_count[3];
  double consistency, conf_sum, cons_sum;
  double ph[8][2];              // position_history deque(maxlen=8)
  double bh[5][4];              // bbox_history deque(maxlen=5): detection boxes
  double ms[10];                // motion_scores deque(maxlen=10)
  unsigned char ph32[8];        // entry is a float32 detection centre (else a float64 state copy)
  unsigned char mk[10];         // score dtype (K32 / K64 / KPY)
  ResetDetail dl[5];            // the last five reset_reasons entries
};

// Register copy of a Slot's scalar state, the rings left in global memory (pointer members, so
// s.vh[i][0] / s.vang[i] / s.th[i][0] read the same as on a Slot).  The enhanced per-track math
// runs on it and writes back once: on a Slot in global memory every store followed by a load of
// another field is a memory round trip in the thread's dependency chain (no alias proof).
struct LSlot {
  static constexpr bool kPol = false;
  double x[8];
  double P[16];
  double vavg[2], vstd[2], direction, speed, stability, pconf;
  double (*vh)[2];
  double* vang;
  double (*th)[2];
  int age, hits, hit_streak, tsu, is_lost, lost_frames, track_num, max_lost;
  int vh_len, vh_head, th_len, th_head;
  unsigned th_cnt;
  int policy;
};

struct Hdr {
  int n_tracks, n_free;
  yk_tracker_stats st;
  // MotionCompensatedMultiTracker's global branch (motion_compensated_multi_tracker.py:52-53)
  int dsh[10];                  // detection_stability_history deque(maxlen=10)
  int dsh_len, dsh_head;
  float gmh[20];                // global_motion_history deque(maxlen=20) ...
  unsigned char gmk[20];        // ... entry dtype: K32 (np.float32) or KPY (python float 0.0)
  int gmh_len, gmh_head;
};

struct Dev {
  Slot* slots;          // [S][T]
  Hdr* hdr;             // [S]
  int* order;           // [S][T] list position -> slot
  int* free_stack;      // [S][T]
  unsigned long long* cand_key;  // [S][C] IoU bits of candidate pairs
  int* cand_flat;                // [S][C] row-major pair index d*n + t
  yk_track_out* rows;   // [S][T]
  int* counts;          // [S]
  yk_tracker_stats* stats;  // [S]
  long long* phase;         // [S][PH] wall_clock64 at the step's phase boundaries (profiling)
  int4* items;              // [S][T] enhanced two-kernel step: {slot, det, track_num, out_row} per work item
  int2* items_vh;           // [S][T] {vh_len, vh_head} of the item's slot before the step
  int* n_items;             // [S]
  yk_track_event* events;   // [S][T] per-work-item event log (yk_tracker_set_events), or NULL
  int T, D, C;
  int max_lost, min_hits;
  double thr;
  int policy;           // yk_tracker_policy
};

// ---------------------------------------------------------------- per-track math
__device__ __forceinline__ void ring_push(double (*buf)[2], int cap, int& len, int& head, double a,
                                          double b, int* pos_out = nullptr) {
  int pos;
  if (len < cap) {
    pos = head + len;
    if (pos >= cap) pos -= cap;
    ++len;
  } else {
    pos = head;
    head = (head + 1 == cap) ? 0 : head + 1;
  }
  buf[pos][0] = a;
  buf[pos][1] = b;
  if (pos_out) *pos_out = pos;
}

__device__ __forceinline__ void state_to_bbox(const double* s, double* b) {
  // enhanced_aircraft_kalman_tracker.py:130-135
  b[0] = s[0] - s[2] / 2.0;
  b[1] = s[1] - s[3] / 2.0;
  b[2] = s[0] + s[2] / 2.0;
  b[3] = s[1] + s[3] / 2.0;
}

// bbox_to_state (kf.py:113-118) in the detection's own dtype, widened to f64.
template <typename DT>
__device__ __forceinline__ void bbox_to_state(const DT* b, double* z) {
  DT cx = (b[0] + b[2]) / DT(2);
  DT cy = (b[1] + b[3]) / DT(2);
  DT w = b[2] - b[0];
  DT h = b[3] - b[1];
  z[0] = (double)cx;
  z[1] = (double)cy;
  z[2] = (double)w;
  z[3] = (double)h;
}

template <class S>
__device__ void slot_init(S& s, const double* z, int track_num, int max_lost) {
  // AircraftKalmanTracker.__init__ (kf.py:32-101)
  for (int i = 0; i < 8; ++i) s.x[i] = 0.0;
  for (int c = 0; c < 4; ++c) {
    s.x[c] = z[c];
    s.P[4 * c + 0] = 50.0;
    s.P[4 * c + 1] = 0.0;
    s.P[4 * c + 2] = 0.0;
    s.P[4 * c + 3] = c < 2 ? 100.0 : 1.0;
  }
  s.vavg[0] = s.vavg[1] = s.vstd[0] = s.vstd[1] = 0.0;
  s.direction = s.speed = s.stability = s.pconf = 0.0;
  s.age = 0;
  s.hits = 1;
  s.hit_streak = 1;
  s.tsu = 0;
  s.is_lost = 0;
  s.lost_frames = 0;
  s.track_num = track_num;
  s.max_lost = max_lost;
  s.vh_len = s.vh_head = 0;
  s.th_len = s.th_head = 0;
  s.th_cnt = 1;
  s.policy = 0;
  ring_push(s.th, TH, s.th_len, s.th_head, z[0], z[1]);
}

template <class S>
__device__ void kf_predict(S& s) {
  // kf.py:192-201: x = F x ; P = F P F^T + Q
  const double qp[4] = {0.1, 0.1, 0.01, 0.01};
  const double qv[4] = {0.1, 0.1, 0.001, 0.001};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    s.x[c] = s.x[c] + s.x[c + 4];
    const double p = s.P[4 * c], a = s.P[4 * c + 1], b = s.P[4 * c + 2], v = s.P[4 * c + 3];
    const double app = p + b, apv = a + v;  // rows of F@P
    s.P[4 * c + 0] = (app + apv) + qp[c];
    s.P[4 * c + 1] = apv + 0.0;
    s.P[4 * c + 2] = (b + v) + 0.0;
    s.P[4 * c + 3] = v + qv[c];
  }
  s.age += 1;
  s.tsu += 1;
  ring_push(s.th, TH, s.th_len, s.th_head, s.x[0], s.x[1]);
  s.th_cnt += 1;
}

// numpy's pairwise summation for a contiguous 1-D float64 array of n <= 128 elements
// (numpy/_core/src/umath/loops_utils.h.src, pairwise_sum), the add.reduce of np.std/np.mean.
__device__ double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// Chain-friendly forms of numpy's reductions.  The guard sits on the ADDEND: x + (-0.0) == x
// exactly for every x (signed zeros, infinities and NaN included), so a masked-out element adds
// -0.0 and the accumulator's dependency chain is one v_add_f64 per element.  Loops run over the
// static ring size in chunks of 7 (inner loop unrolled, its LDS loads issued together; outer loop
// rolled, which bounds the registers).
constexpr int PW = 56;  // >= VH - 1, a multiple of 8
static_assert(VH == 50, "chunking below assumes the 50-entry velocity ring");

// np.add.reduce's pairwise summation (numpy/_core/src/umath/loops_utils.h.src, pairwise_sum) of
// f(0..n-1), n <= PW: the same additions in the same order as np_pairwise_sum.
template <class F>
__device__ __forceinline__ double np_pairwise_sum_f(F f, int n) {
  if (n < 8) {
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double v = f(i);  // unconditional: the select (not a branch) keeps the chain straight
      r += i < n ? v : -0.0;
    }
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f(j);
  const int lim = n - (n % 8);
#pragma unroll 1
  for (int i = 8; i < lim; i += 8) {
    double v[8];  // the block's operands first: one LDS round trip per block, not per element
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f(i + j);
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += v[j];
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const double v = f(lim + i);
    res += lim + i < n ? v : -0.0;
  }
  return res;
}

// The velocity history in chronological order (oldest first), as three arrays vx, vy, ang of
// n = s.vh_len entries (LDS in the step kernels); dch (>= VH - 1 entries, LDS) may alias vx.
template <class S>
__device__ void analyze_motion(S& s, const double* vx, const double* vy, const double* ang, double* dch) {
  // kf.py:137-182
  const int n = s.vh_len;
  if (n < 5) return;
  double acc0 = vx[0], acc1 = vy[0];  // np.mean(axis=0): sequential over rows
#pragma unroll 1
  for (int c = 1; c < VH; c += 7) {
    double a0[7], a1[7];  // the chunk's loads first (one LDS round trip), then the guarded addends
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      a0[u] = vx[c + u];
      a1[u] = vy[c + u];
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      acc0 += c + u < n ? a0[u] : -0.0;
      acc1 += c + u < n ? a1[u] : -0.0;
    }
  }
  const double mean[2] = {acc0 / (double)n, acc1 / (double)n};
  double d0 = vx[0] - mean[0], d1 = vy[0] - mean[1];  // np.std(axis=0), ddof=0
  double q0 = d0 * d0, q1 = d1 * d1;
#pragma unroll 1
  for (int c = 1; c < VH; c += 7) {
    double a0[7], a1[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      a0[u] = vx[c + u];
      a1[u] = vy[c + u];
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      d0 = a0[u] - mean[0];
      d1 = a1[u] - mean[1];
      const double e0 = d0 * d0, e1 = d1 * d1;
      q0 += c + u < n ? e0 : -0.0;
      q1 += c + u < n ? e1 : -0.0;
    }
  }
  const double sq[2] = {sqrt(q0 / (double)n), sqrt(q1 / (double)n)};
  s.vavg[0] = mean[0];
  s.vavg[1] = mean[1];
  s.vstd[0] = sq[0];
  s.vstd[1] = sq[1];
  s.speed = sqrt(mean[0] * mean[0] + mean[1] * mean[1]);
  s.direction = atan2(mean[1], mean[0]);
  const double speed_stab = 1.0 / (1.0 + ((0.0 + sq[0]) + sq[1]) / 2.0);
  // _calculate_direction_consistency (kf.py:165-182); n >= 5 here, so the n<3 exit is dead
  const int m = n - 1;
#pragma unroll 1
  for (int c = 0; c < m; c += 7) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = c + u;
      a[u] = ang[k < VH ? k : VH - 1];  // reads stay inside the ring (k >= m is discarded)
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int k = c + u;
      double v = a[u + 1] - a[u];
      if (!(fabs(v) < kPi)) v = v - 2.0 * kPi * (v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : v));
      dch[k] = v;  // k >= m lands on dead vx / vy entries (k < 56 <= 3 * VS - base)
    }
  }
  const double dmean = np_pairwise_sum_f([&](int k) { return dch[k]; }, m) / (double)m;
  const double dstd = sqrt(np_pairwise_sum_f(
                               [&](int k) {
                                 const double d = dch[k] - dmean;
                                 return d * d;
                               },
                               m) /
                           (double)m);
  const double dir_cons = 1.0 / (1.0 + dstd * 10.0);
  s.stability = (speed_stab + dir_cons) / 2.0;
  const double frac = (double)n / 30.0;
  s.pconf = s.stability * (1.0 < frac ? 1.0 : frac);
}

// ---------------------------------------------------------------- motion-reset policy
// camera_motion_compensation/motion_reset_kalman_tracker.py (checker: oracle/cmc_ref.py).
template <int CAP>
__device__ __forceinline__ int ring_slot(int& len, int& head) {
  int pos;
  if (len < CAP) {
    pos = head + len;
    if (pos >= CAP) pos -= CAP;
    ++len;
  } else {
    pos = head;
    head = (head + 1 == CAP) ? 0 : head + 1;
  }
  return pos;
}
template <int CAP>
__device__ __forceinline__ int ring_at(int head, int k) {
  const int i = head + k;
  return i >= CAP ? i - CAP : i;
}

__device__ __forceinline__ void ph_push(Slot& s, double a, double b, bool f32) {
  const int p = ring_slot<8>(s.ph_len, s.ph_head);
  s.ph[p][0] = a;
  s.ph[p][1] = b;
  s.ph32[p] = f32 ? 1 : 0;
}

// np.add.reduce of a 1-D contiguous array a[0..n), n <= NMAX: identity 0 + numpy's pairwise sum
// (8 accumulators from n = 8), in float32 when F = float (verified against numpy 2.2 add.reduce).
// Every loop runs to the static bound NMAX with the n-dependent part as a predicate, so after
// unrolling no private array is indexed by a run-time value (no scratch).
template <typename F, int NMAX>
__device__ __forceinline__ F np_sum_t(const double (&a)[NMAX], int n) {
  F res = F(0);
  if (NMAX < 8 || n < 8) {
#pragma unroll
    for (int i = 0; i < (NMAX < 8 ? NMAX : 7); ++i)
      if (i < n) res = res + (F)a[i];
  } else if constexpr (NMAX >= 8) {
    F r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (F)a[j];
    const int nb = n - (n % 8);  // end of the 8-wide blocks
#pragma unroll
    for (int i = 8; i + 8 <= NMAX; i += 8)
      if (i < nb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = r[j] + (F)a[i + j];
      }
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = 8; i < NMAX; ++i)
      if (i >= nb && i < n) res = res + (F)a[i];
  }
  return F(0) + res;
}

// np.mean / np.var of a python list of numpy scalars / python floats (np.asarray dtype rule)
template <int NMAX>
__device__ __forceinline__ Num np_mean_list(const Num (&a)[NMAX], int n) {
  bool f32 = true;
  double v[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    if (i < n) f32 = f32 && a[i].k == K32;
    v[i] = a[i].v;
  }
  if (f32) return Num{(double)(np_sum_t<float>(v, n) / (float)n), K32};
  return Num{np_sum_t<double>(v, n) / (double)n, K64};
}
template <int NMAX>
__device__ __forceinline__ Num np_var_list(const Num (&a)[NMAX], int n) {
  const Num m = np_mean_list(a, n);
  double d[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    if (m.k == K32) {
      const float x = (float)a[i].v - (float)m.v;
      d[i] = (double)(x * x);
    } else {
      const double x = a[i].v - m.v;
      d[i] = x * x;
    }
  }
  if (m.k == K32) return Num{(double)(np_sum_t<float>(d, n) / (float)n), K32};
  return Num{np_sum_t<double>(d, n) / (double)n, K64};
}

// numpy scalar (op) python float c: c takes the scalar's dtype (NEP 50)
__device__ __forceinline__ Num div_c(Num a, double c) {
  if (a.k == K32) return Num{(double)((float)a.v / (float)c), K32};
  return Num{a.v / c, a.k};
}
__device__ __forceinline__ Num mul_c(Num a, double c) {
  if (a.k == K32) return Num{(double)((float)a.v * (float)c), K32};
  return Num{a.v * c, a.k};
}
__device__ __forceinline__ bool gt_c(Num a, double c) { return a.k == K32 ? (float)a.v > (float)c : a.v > c; }
__device__ __forceinline__ bool lt_c(Num a, double c) { return a.k == K32 ? (float)a.v < (float)c : a.v < c; }
// python min(a, c): c only when c < a
__device__ __forceinline__ Num pymin_c(Num a, double c) { return gt_c(a, c) ? Num{c, KPY} : a; }

// a - b of two centre coordinates (float32 when both are float32)
__device__ __forceinline__ double sub_k(double a, double b, bool f32) {
  return f32 ? (double)((float)a - (float)b) : a - b;
}
// np.linalg.norm of a 2-vector = sqrt(v.dot(v)): float32 as x*x + y*y, float64 through the
// BLAS ddot, which contracts to fma(y, y, x*x) (both verified on numpy 2.2 + its OpenBLAS)
__device__ __forceinline__ Num norm2(double dx, double dy, bool f32) {
  if (f32) {
    const float x = (float)dx, y = (float)dy;
    return Num{(double)sqrtf(x * x + y * y), K32};
  }
  return Num{sqrt(fma(dy, dy, dx * dx)), K64};
}

// MotionResetKalmanTracker.__init__ on top of slot_init (:28-65): the base's position deque is
// replaced by a maxlen-8 one holding the detection centre
template <typename DT>
__device__ void cmc_init(Slot& s, const DT* b) {
  s.policy = 1;
  s.reset_count = 0;
  s.last_reset = -999;
  s.ph_len = s.ph_head = s.bh_len = s.bh_head = s.ms_len = s.ms_head = s.dl_len = s.dl_head = 0;
  s.reason_count[0] = s.reason_count[1] = s.reason_count[2] = 0;
  s.consistency = s.conf_sum = s.cons_sum = 0.0;
  const DT cx = (b[0] + b[2]) / DT(2), cy = (b[1] + b[3]) / DT(2);
  ph_push(s, (double)cx, (double)cy, sizeof(DT) == 4);
  const int p = ring_slot<5>(s.bh_len, s.bh_head);
  for (int k = 0; k < 4; ++k) s.bh[p][k] = (double)b[k];
}

// _calculate_motion_consistency (:159-172)
__device__ Num cmc_consistency(const Slot& s) {
  const int n = s.ms_len;
  if (n < 3) return Num{0.0, KPY};
  Num sc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const int i = ring_at<10>(s.ms_head, k < n ? k : 0);
    sc[k] = k < n ? Num{s.ms[i], (int)s.mk[i]} : Num{0.0, KPY};
  }
  const Num m = np_mean_list(sc, n);
  if (!(m.v > 0.0)) return Num{1.0, KPY};
  const Num v = np_var_list(sc, n);
  Num c;
  if (m.k == K32) c = Num{(double)(1.0f - (float)v.v / ((float)m.v + 0.1f)), K32};
  else c = Num{1.0 - v.v / (m.v + 0.1), K64};
  return c.v > 0.0 ? c : Num{0.0, KPY};  // python max(0.0, c)
}

// _should_reset_kalman (:174-214) with the three detectors (:86-157).  val / why: the
// reasons' values and bits (1 position jump, 2 velocity change, 4 size change).
template <typename DT>
__device__ __forceinline__ bool cmc_decide(Slot& s, const DT* b, double* val, int& why, Num& conf) {
  why = 0;
  const int since = s.age - s.last_reset;
  if (since < 15) return false;  // reset cooldown
  constexpr bool c32 = sizeof(DT) == 4;
  const DT cxd = (b[0] + b[2]) / DT(2), cyd = (b[1] + b[3]) / DT(2);
  const double cx = (double)cxd, cy = (double)cyd;
  Num f1{0.0, KPY}, f2{0.0, KPY}, f3{0.0, KPY};  // the reasons' confidence factors, appended in order
  bool b1 = false, b2 = false, b3 = false;
  // 1. position jump: the centre against the mean of the last <= 3 history entries
  if (s.ph_len >= 2) {
    const int m = s.ph_len < 3 ? s.ph_len : 3;
    int id[3];
    bool all32 = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      id[k] = ring_at<8>(s.ph_head, k < m ? s.ph_len - m + k : s.ph_len - 1);
      if (k < m) all32 = all32 && s.ph32[id[k]];
    }
    double avg[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // np.mean(axis=0): rows accumulated in order
      if (all32) {
        float acc = (float)s.ph[id[0]][j];
#pragma unroll
        for (int k = 1; k < 3; ++k)
          if (k < m) acc = acc + (float)s.ph[id[k]][j];
        avg[j] = (double)(acc / (float)m);
      } else {
        double acc = s.ph[id[0]][j];
#pragma unroll
        for (int k = 1; k < 3; ++k)
          if (k < m) acc = acc + s.ph[id[k]][j];
        avg[j] = acc / (double)m;
      }
    }
    const bool d32 = all32 && c32;
    const Num dist = norm2(sub_k(cx, avg[0], d32), sub_k(cy, avg[1], d32), d32);
    const Num sc = pymin_c(div_c(dist, 40.0), 3.0);
    const int p = ring_slot<10>(s.ms_len, s.ms_head);
    s.ms[p] = sc.v;
    s.mk[p] = (unsigned char)sc.k;
    if (gt_c(dist, 40.0)) {
      why |= 1;
      val[0] = dist.v;
      f1 = pymin_c(div_c(dist, 40.0), 2.0);
      b1 = true;
    }
  }
  // 2. velocity change: the newest step length against the mean of the two before it
  if (s.ph_len >= 3) {
    double px[4], py[4];
    bool p32[4];
    for (int k = 0; k < 3; ++k) {
      const int i = ring_at<8>(s.ph_head, s.ph_len - 3 + k);
      px[k] = s.ph[i][0];
      py[k] = s.ph[i][1];
      p32[k] = s.ph32[i] != 0;
    }
    px[3] = cx;
    py[3] = cy;
    p32[3] = c32;
    Num sp[3];
    for (int k = 1; k < 4; ++k) {
      const bool f = p32[k] && p32[k - 1];
      sp[k - 1] = norm2(sub_k(px[k], px[k - 1], f), sub_k(py[k], py[k - 1], f), f);
    }
    const Num avg = np_mean_list(sp, 2);
    const bool f = sp[2].k == K32 && avg.k == K32;
    const Num ch{fabs(sub_k(sp[2].v, avg.v, f)), f ? K32 : K64};
    if (gt_c(ch, 60.0)) {
      why |= 2;
      val[1] = ch.v;
      f2 = pymin_c(div_c(ch, 60.0), 2.0);
      b2 = true;
    }
  }
  // 3. size change against the previous detection box (the detection's dtype throughout)
  if (s.bh_len >= 2) {
    const double* q = s.bh[ring_at<5>(s.bh_head, s.bh_len - 1)];
    DT pw = (DT)q[2] - (DT)q[0], ph = (DT)q[3] - (DT)q[1];
    pw = pw < DT(1) ? DT(1) : pw;  // np.maximum(prev_size, 1.0)
    ph = ph < DT(1) ? DT(1) : ph;
    const DT r0 = (b[2] - b[0]) / pw, r1 = (b[3] - b[1]) / ph;
    const DT a0 = r0 - DT(1) < DT(0) ? DT(1) - r0 : r0 - DT(1);
    const DT a1 = r1 - DT(1) < DT(0) ? DT(1) - r1 : r1 - DT(1);
    const DT r = a1 > a0 ? a1 : a0;  // python max keeps the first on ties
    const Num rn{(double)r, c32 ? K32 : K64};
    if (gt_c(rn, 0.3)) {
      why |= 4;
      val[2] = rn.v;
      f3 = div_c(rn, 0.3);
      b3 = true;
    }
  }
  const int nf = (int)b1 + (int)b2 + (int)b3;
  if (nf == 0) return false;
  // the list [f_i for i in 1..3 if b_i], by selects (static indices)
  const Num fac[3] = {b1 ? f1 : (b2 ? f2 : f3), b1 ? (b2 ? f2 : f3) : f3, f3};
  conf = np_mean_list(fac, nf);
  const Num cons = cmc_consistency(s);
  s.consistency = cons.v;
  if (lt_c(cons, 0.3)) conf = mul_c(conf, 1.5);
  if (s.reset_count > 0 && since < 50) conf = mul_c(conf, 0.8);  // adaptive_enabled
  return conf.v > 1.0;
}

// _reset_kalman_filter (:216-259)
template <typename DT>
__device__ void cmc_reset(Slot& s, const DT* b, const double* val, int why, Num conf) {
  s.reset_count += 1;
  s.last_reset = s.age;
  ResetDetail& d = s.dl[ring_slot<5>(s.dl_len, s.dl_head)];
  d.frame = s.age;
  d.reasons = why;
  for (int k = 0; k < 3; ++k) {
    d.value[k] = (why >> k) & 1 ? val[k] : 0.0;
    s.reason_count[k] += (why >> k) & 1;
  }
  d.conf = conf.v;
  d.cons = s.consistency;
  s.conf_sum += conf.v;
  s.cons_sum += s.consistency;
  double z[4];
  bbox_to_state<DT>(b, z);
  for (int c = 0; c < 4; ++c) {
    s.x[c] = z[c];
    s.x[c + 4] = 0.0;
    s.P[4 * c + 0] = s.P[4 * c + 0] * 5.0;    // P[:4, :4] *= 5 (only the diagonal is non-zero)
    s.P[4 * c + 3] = s.P[4 * c + 3] * 100.0;  // P[4:, 4:] *= 100
  }
  s.th_len = s.th_head = 0;
  ring_push(s.th, TH, s.th_len, s.th_head, z[0], z[1]);
  s.th_cnt += 1 << 20;  // the history restarts: a host-side trajectory cache must not reuse points
  s.vh_len = s.vh_head = 0;
  s.ph_len = s.ph_head = 0;
  ph_push(s, z[0], z[1], sizeof(DT) == 4);
  s.ms_len = s.ms_head = 0;
  s.hits += 1;
  s.hit_streak += 1;
  s.tsu = 0;
}

// update() tail (:280-285): the detection centre and box join the histories
template <typename DT>
__device__ void cmc_after_update(Slot& s, const DT* b) {
  const DT cx = (b[0] + b[2]) / DT(2), cy = (b[1] + b[3]) / DT(2);
  ph_push(s, (double)cx, (double)cy, sizeof(DT) == 4);
  const int p = ring_slot<5>(s.bh_len, s.bh_head);
  for (int k = 0; k < 4; ++k) s.bh[p][k] = (double)b[k];
}

// predict() (:287-312): for 10 frames after a reset the returned box's centre is blended from
// the last history position toward the prediction (the state itself is not changed).  age: the
// track's age after that predict (assoc_kernel blends without running it: s.age + 1)
__device__ void cmc_blend(const Slot& s, double* box, int age) {
  const int since = age - s.last_reset;
  if (since >= 10 || s.ph_len == 0) return;
  const int li = ring_at<8>(s.ph_head, s.ph_len - 1);
  double w = (double)since / 10.0;
  w = 1.0 < w ? 1.0 : w;
  const double pcx = (box[0] + box[2]) / 2.0, pcy = (box[1] + box[3]) / 2.0;
  double t0, t1;
  if (s.ph32[li]) {  // python float x float32 array stays float32
    const float om = (float)(1.0 - w);
    t0 = (double)(om * (float)s.ph[li][0]);
    t1 = (double)(om * (float)s.ph[li][1]);
  } else {
    t0 = (1.0 - w) * s.ph[li][0];
    t1 = (1.0 - w) * s.ph[li][1];
  }
  const double ax = t0 + w * pcx, ay = t1 + w * pcy;
  const double sw = box[2] - box[0], sh = box[3] - box[1];
  box[0] = ax - sw / 2.0;
  box[1] = ay - sh / 2.0;
  box[2] = ax + sw / 2.0;
  box[3] = ay + sh / 2.0;
}

constexpr int VS = VH + 1;  // staged entries per array (one spare for the push onto a full ring)

// Chronological copy of the velocity history (before an update) into st[3][VS].
__device__ void stage_chrono(const Slot& s, double* st) {
  int idx = s.vh_head;
  for (int k = 0; k < s.vh_len; ++k) {
    st[k] = s.vh[idx][0];
    st[VS + k] = s.vh[idx][1];
    st[2 * VS + k] = s.vang[idx];
    idx = (idx + 1 == VH) ? 0 : idx + 1;
  }
}

// st: stage_chrono() of the slot before this update ([3][VS], LDS in the step kernel).
template <typename DT, class S>
__device__ void kf_update(S& s, const DT* box, double* st) {
  // kf.py:249-297 (recovery print omitted; the count is kept by the caller)
  s.tsu = 0;
  s.hits += 1;
  s.hit_streak += 1;
  if (s.is_lost) {
    s.is_lost = 0;
    s.lost_frames = 0;
  }
  double z[4];
  bbox_to_state<DT>(box, z);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double p = s.P[4 * c], a = s.P[4 * c + 1], b = s.P[4 * c + 2], v = s.P[4 * c + 3];
    const double y = z[c] - s.x[c];
    const double inv = 1.0 / (p + 10.0);
    const double kp = p * inv, kv = b * inv;
    s.x[c] = s.x[c] + kp * y;
    s.x[c + 4] = s.x[c + 4] + kv * y;
    const double ikh = 1.0 - kp, nkv = -kv;
    s.P[4 * c + 0] = ikh * p;
    s.P[4 * c + 1] = ikh * a;
    s.P[4 * c + 2] = nkv * p + b;
    s.P[4 * c + 3] = nkv * a + v;
  }
  int pos;
  const int len0 = s.vh_len;
  ring_push(s.vh, VH, s.vh_len, s.vh_head, s.x[4], s.x[5], &pos);
  const double ang = atan2(s.x[5], s.x[4]);
  s.vang[pos] = ang;
  // the staged chronological copy: append; a full ring drops its oldest entry (base 1)
  const int at = len0 < VH ? len0 : VH;
  st[at] = s.x[4];
  st[VS + at] = s.x[5];
  st[2 * VS + at] = ang;
  const int base = len0 < VH ? 0 : 1;
  ring_push(s.th, TH, s.th_len, s.th_head, s.x[0], s.x[1]);
  s.th_cnt += 1;
  analyze_motion(s, st + base, st + VS + base, st + 2 * VS + base, st + base);
}

template <class S>
__device__ __forceinline__ void mark_lost(S& s) {
  // kf.py:299-317
  if (!s.is_lost) {
    s.is_lost = 1;
    s.lost_frames = 0;
  }
  s.lost_frames += 1;
  s.hit_streak = 0;
}

__device__ __forceinline__ bool should_delete(const Slot& s, int max_lost) {
  // kf.py:385-405
  if (s.tsu > max_lost) return true;
  if (s.age < 5 && s.hit_streak == 0 && s.tsu > 15) return true;
  if (s.age < 10 && s.hit_streak <= 1 && s.tsu > 30) return true;
  return false;
}

// enhanced_long_term_predict(frames_ahead=k) (kf.py:205-247).  k <= 1 runs predict().
template <class S>
__device__ void long_term_predict(S& s, int k, double* box, double& conf) {
  if (k <= 1) {
    kf_predict(s);
    state_to_bbox(s.x, box);
    if constexpr (S::kPol) {
      if (s.policy) cmc_blend(s, box, s.age);  // the subclass's predict()
    }
    conf = 1.0;
    return;
  }
  // analyze_motion_pattern() is re-run by the reference here; the velocity history has
  // not changed since the last update() (which ran it), so the cached statistics are
  // identical to a recomputation.
  double st[4];
  if (s.pconf > 0.3) {
    st[0] = s.x[0] + s.vavg[0] * (double)k;
    st[1] = s.x[1] + s.vavg[1] * (double)k;
    st[2] = s.x[2];
    st[3] = s.x[3];
    const double decay = 1.0 - (double)k / (double)s.max_lost;
    conf = s.pconf * (decay > 0.1 ? decay : 0.1);
  } else {
    st[0] = s.x[0];
    st[1] = s.x[1];
    st[2] = s.x[2];
    st[3] = s.x[3];
    for (int r = 0; r < k; ++r)
      for (int c = 0; c < 4; ++c) st[c] = st[c] + s.x[c + 4];
    const double decay = 1.0 - (double)k / ((double)s.max_lost * 0.5);
    conf = decay > 0.1 ? decay : 0.1;
  }
  state_to_bbox(st, box);
}

// get_lost_prediction (kf.py:319-333)
template <class S>
__device__ void lost_prediction(S& s, double* box, double& conf) {
  if (!s.is_lost) {
    state_to_bbox(s.x, box);
    conf = 1.0;
    return;
  }
  long_term_predict(s, s.lost_frames, box, conf);
}

// get_track_info (kf.py:335-383) including quirk A (a second predict() on the first
// lost frame, via get_lost_prediction -> enhanced_long_term_predict(1)).
template <class S>
__device__ void track_info(S& s, yk_track_out& o, bool copy_traj = true) {
  double box[4];
  double conf;
  int status;
  if (s.tsu > 0) {
    status = 1;
    if (s.is_lost) {
      lost_prediction(s, box, conf);
    } else {  // short-loss branch; unreachable from update(), kept for parity
      state_to_bbox(s.x, box);
      const double decay = 1.0 - (double)s.tsu / 60.0;
      conf = decay > 0.3 ? decay : 0.3;
    }
  } else {
    status = 0;
    state_to_bbox(s.x, box);
    conf = 1.0;
  }
  o.track_num = s.track_num;
  o.status = status;
  o.age = s.age;
  o.hits = s.hits;
  o.hit_streak = s.hit_streak;
  o.time_since_update = s.tsu;
  o.is_stable_motion = s.stability > 0.5 ? 1 : 0;
  for (int i = 0; i < 4; ++i) o.bbox[i] = box[i];
  o.confidence = conf;
  o.velocity[0] = s.x[4];
  o.velocity[1] = s.x[5];
  o.motion_confidence = s.pconf;
  o.speed = s.speed;
  o.direction = s.direction;
  // MotionResetKalmanTracker.get_track_info / get_reset_statistics (:314-355).  The enhanced
  // policy never writes these fields: the rows buffer is zeroed once at creation.
  if constexpr (S::kPol) {
   if (s.policy) {
    o.reset_count = s.reset_count;
    o.frames_since_reset = s.age - s.last_reset;
    o.n_details = s.dl_len;
    for (int k = 0; k < 3; ++k) o.reason_count[k] = s.reason_count[k];
    o.motion_consistency = s.consistency;
    o.reset_confidence_sum = s.conf_sum;
    o.motion_consistency_sum = s.cons_sum;
    for (int k = 0; k < 5; ++k) {  // unused entries zeroed: a row position is reused by other tracks
      const bool u = k < s.dl_len;
      const ResetDetail& d = s.dl[ring_at<5>(s.dl_head, u ? k : 0)];
      o.details[k].frame = u ? d.frame : 0;
      o.details[k].reasons = u ? d.reasons : 0;
      for (int j = 0; j < 3; ++j) o.details[k].value[j] = u ? d.value[j] : 0.0;
      o.details[k].confidence = u ? d.conf : 0.0;
      o.details[k].motion_consistency = u ? d.cons : 0.0;
    }
   }
  }
  const int nt = s.th_len < TOUT ? s.th_len : TOUT;
  o.traj_len = nt;
  o.traj_count = (int32_t)s.th_cnt;  // two's-complement view of the mod-2^32 count
  o.reserved = 0;
  if (!copy_traj) return;  // the step kernel copies trajectories cooperatively
  int idx = s.th_head + (s.th_len - nt);
  if (idx >= TH) idx -= TH;
  for (int k = 0; k < nt; ++k) {
    o.traj[k][0] = s.th[idx][0];
    o.traj[k][1] = s.th[idx][1];
    idx = (idx + 1 == TH) ? 0 : idx + 1;
  }
  for (int k = nt; k < TOUT; ++k) o.traj[k][0] = o.traj[k][1] = 0.0;
}

// IoU of detection (DT) against a predicted track box (f64) with the reference's dtype
// propagation (enhanced_multi_target_tracker.py:200-232): python max/min
// return the winning object (ties -> the detection), f32-op-f32 stays f32.
template <typename DT>
__device__ double iou_mixed(const DT* d, const double* t) {
  // each intersection coordinate: value as double + whether it is still a DT value
  const bool tx1 = t[0] > (double)d[0];
  const bool ty1 = t[1] > (double)d[1];
  const bool tx2 = t[2] < (double)d[2];
  const bool ty2 = t[3] < (double)d[3];
  const double ix1 = tx1 ? t[0] : (double)d[0];
  const double iy1 = ty1 ? t[1] : (double)d[1];
  const double ix2 = tx2 ? t[2] : (double)d[2];
  const double iy2 = ty2 ? t[3] : (double)d[3];
  if (ix2 <= ix1 || iy2 <= iy1) return 0.0;
  // width / height: DT arithmetic when both operands are detection values
  const bool w_dt = !tx1 && !tx2, h_dt = !ty1 && !ty2;
  const double w = w_dt ? (double)(DT)(d[2] - d[0]) : ix2 - ix1;
  const double h = h_dt ? (double)(DT)(d[3] - d[1]) : iy2 - iy1;
  const double inter = (w_dt && h_dt) ? (double)((DT)w * (DT)h) : w * h;
  const DT area1 = (d[2] - d[0]) * (d[3] - d[1]);
  const double area2 = (t[2] - t[0]) * (t[3] - t[1]);
  const double uni = ((double)area1 + area2) - inter;
  if (uni <= 0.0) return 0.0;
  return inter / uni;
}

// ---------------------------------------------------------------- block helpers
// Exclusive prefix count of `flag` over the workgroup; `total` gets the block total.
template <int NTH = NT>
__device__ __forceinline__ int block_scan(int flag, int* wsum, int& total) {
  constexpr int NW = NTH / 64;
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

struct Lds {
  double* pb;                 // [T][4] predicted boxes by list position
  double* det;                // [D][4] detection boxes (exact widening of DT)
  int* det_match;             // [D] matched list position or -1
  int* trk_match;             // [T] matched detection or -1
  unsigned long long* row_max;  // [D]
  unsigned long long* col_max;  // [T]
  int* row_arg;               // [D]
  int* col_arg;               // [T]
  int* order_tmp;             // [T]
  int* misc;                  // [16]
  double* stage;              // [ch][3][VS] chronological velocity history of the tracks being updated
};

constexpr int STAGE_D = 3 * (VH + 1);   // doubles per staged track
constexpr int CH_MAX = 64;              // tracks staged per update chunk (at most)

__host__ __device__ inline size_t lds_base_bytes(int T, int D) {
  const size_t b = (size_t)T * 32 + (size_t)D * 32 + (size_t)D * 4 + (size_t)T * 4 + (size_t)D * 8 +
                   (size_t)T * 8 + (size_t)D * 4 + (size_t)T * 4 + (size_t)T * 4 + 16 * 4;
  return (b + 15) / 16 * 16;
}
// staging chunk: as many tracks as fit the 160 KiB LDS budget, up to CH_MAX
__host__ __device__ inline int stage_chunk(int T, int D) {
  const long room = (160L * 1024 - (long)lds_base_bytes(T, D)) / (STAGE_D * 8);
  return room < 1 ? 0 : room > CH_MAX ? CH_MAX : (int)room;
}
__host__ __device__ inline size_t lds_bytes(int T, int D) {
  return lds_base_bytes(T, D) + (size_t)stage_chunk(T, D) * STAGE_D * 8;
}

__device__ Lds carve(char* base, int T, int D) {
  Lds L;
  L.pb = (double*)base;
  base += (size_t)T * 32;
  L.det = (double*)base;
  base += (size_t)D * 32;
  L.row_max = (unsigned long long*)base;
  base += (size_t)D * 8;
  L.col_max = (unsigned long long*)base;
  base += (size_t)T * 8;
  L.det_match = (int*)base;
  base += (size_t)D * 4;
  L.trk_match = (int*)base;
  base += (size_t)T * 4;
  L.row_arg = (int*)base;
  base += (size_t)D * 4;
  L.col_arg = (int*)base;
  base += (size_t)T * 4;
  L.order_tmp = (int*)base;
  base += (size_t)T * 4;
  L.misc = (int*)base;
  base += 16 * 4;
  L.stage = (double*)(((size_t)base + 15) / 16 * 16);
  return L;
}

enum { M_NCAND = 0, M_ACTIVE, M_RECOVER, M_LONGTERM, M_OVERFLOW, M_RESETS, M_TRECOV, M_GRESET, M_WSUM = 8, M_TESTED = 12 };

__device__ __forceinline__ int ring_slot(int cap, int& len, int& head) {  // deque(maxlen=cap).append
  int pos;
  if (len < cap) {
    pos = head + len;
    if (pos >= cap) pos -= cap;
    ++len;
  } else {
    pos = head;
    head = head + 1 == cap ? 0 : head + 1;
  }
  return pos;
}

// MotionCompensatedMultiTracker.update's global branch up to the reset decision (:92-118),
// run by one thread: the two histories, stats['global_motion_events'], and
// _should_global_reset (:123-148) with numpy's dtypes and left-to-right sums.
__device__ bool global_branch(Hdr& H, const yk_motion* motion, int s, int n_dets) {
  H.dsh[ring_slot(10, H.dsh_len, H.dsh_head)] = n_dets;  // (:113-114)
  if (!motion || !motion[s].valid) return false;                // frame is None (:94)
  const yk_motion m = motion[s];
  const int gp = ring_slot(20, H.gmh_len, H.gmh_head);  // (:105)
  H.gmh[gp] = m.magnitude;
  H.gmk[gp] = m.magnitude_kind ? K32 : KPY;
  if (!m.should_reset) return false;
  H.st.global_motion_events += 1;  // (:107-110)
  if (H.dsh_len >= 5) {  // np.std(recent) / (np.mean(recent) + 1) > 0.5, int64 -> float64
    double c[5];
    for (int i = 0; i < 5; ++i) {
      int q = H.dsh_head + H.dsh_len - 5 + i;
      if (q >= 10) q -= 10;
      c[i] = (double)H.dsh[q];
    }
    double sum = c[0];
    for (int i = 1; i < 5; ++i) sum += c[i];
    const double mean = sum / 5.0;
    double acc = (c[0] - mean) * (c[0] - mean);
    for (int i = 1; i < 5; ++i) acc += (c[i] - mean) * (c[i] - mean);
    const double sd = sqrt(acc / 5.0);
    if (sd / (mean + 1.0) > 0.5) return true;
  }
  if (H.gmh_len >= 3) {  // np.mean(last 3) > 30.0: float32 when all three are float32 scalars
    float v[3];
    bool all32 = true;
    for (int i = 0; i < 3; ++i) {
      int q = H.gmh_head + H.gmh_len - 3 + i;
      if (q >= 20) q -= 20;
      v[i] = H.gmh[q];
      all32 = all32 && H.gmk[q] == K32;
    }
    if (all32) {
      float f = v[0];
      f += v[1];
      f += v[2];
      if (f / 3.0f > 30.0f) return true;
    } else {
      double d = (double)v[0];
      d += (double)v[1];
      d += (double)v[2];
      if (d / 3.0 > 30.0) return true;
    }
  }
  return m.magnitude > 60.0f;
}

// ---------------------------------------------------------------- the step kernel
// POL: yk_tracker_policy as a template constant, so the enhanced instantiation carries none of
// the motion-reset code (registers: 122 VGPRs, no scratch).
template <typename DT, int POL>
__global__ void __launch_bounds__(NT) step_kernel(Dev g, const DT* __restrict__ dets, int row_stride,
                                                  const int* __restrict__ counts,
                                                  const yk_motion* __restrict__ motion) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int T = g.T;
  Lds L = carve(smem, T, g.D);
  Hdr& H = g.hdr[s];
  Slot* slots = g.slots + (size_t)s * T;
  int* order = g.order + (size_t)s * T;
  int* fstack = g.free_stack + (size_t)s * T;
  int* wsum = L.misc + M_WSUM;

  if (tid == 0) g.phase[s * PH + 0] = wall_clock64();
  int Draw = counts[s];
  if (Draw < 0) Draw = 0;
  const int D = Draw < g.D ? Draw : g.D;
  int greset = 0;
  if (POL && tid == 0) greset = global_branch(H, motion, s, Draw) ? 1 : 0;
  if (tid < 8) L.misc[tid] = 0;
  const int n_old = H.n_tracks;
  int nfree_base = H.n_free;
  if (POL) {
    if (tid == 0) L.misc[M_GRESET] = greset;  // same wave as the zeroing above: program order
    __syncthreads();
    greset = L.misc[M_GRESET];
    if (greset) {  // _perform_global_reset (:150-169): trackers.clear(), slots back to the stack
      for (int i = tid; i < n_old; i += NT) fstack[nfree_base + i] = order[i];
      nfree_base += n_old;
    }
  }
  const int n = greset ? 0 : n_old;
  // load detections (rows of row_stride elements; only x1..y2 are used by the tracker)
  for (int i = tid; i < D * 4; i += NT) {
    const int d = i >> 2, k = i & 3;
    L.det[i] = (double)dets[((size_t)s * g.D + d) * row_stride + k];
  }
  for (int d = tid; d < D; d += NT) L.det_match[d] = -1;
  for (int t = tid; t < n; t += NT) L.trk_match[t] = -1;
  // Step 1: predict every live track (multi:55-58)
  for (int i = tid; i < n; i += NT) {
    Slot& sl = slots[order[i]];
    kf_predict(sl);
    state_to_bbox(sl.x, &L.pb[4 * i]);
    if (POL && sl.policy) cmc_blend(sl, &L.pb[4 * i], sl.age);
  }
  __syncthreads();
  if (tid == 0) g.phase[s * PH + 1] = wall_clock64();

  // Step 2: association (multi:61-68, 134-178)
  if (D > 0 && n > 0) {
    unsigned long long* ckey = g.cand_key + (size_t)s * g.C;
    int* cflat = g.cand_flat + (size_t)s * g.C;
    const int npair = D * n;
    for (int f = tid; f < npair; f += NT) {
      const int d = f / n, t = f - d * n;
      DT db[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) db[k] = (DT)L.det[4 * d + k];
      const double v = iou_mixed<DT>(db, &L.pb[4 * t]);
      // enhanced: iou >= thr (multi:245); motion-reset: iou > thr (motion_compensated_multi_tracker.py:260)
      if (POL ? v > g.thr : v >= g.thr) {
        const int c = atomicAdd(&L.misc[M_NCAND], 1);
        if (c < g.C) {
          ckey[c] = (unsigned long long)__double_as_longlong(v);
          cflat[c] = f;
        }
      }
    }
    __syncthreads();
    if (tid == 0) g.phase[s * PH + 2] = wall_clock64();
    int nc = L.misc[M_NCAND];
    if (nc > g.C) {
      if (tid == 0) L.misc[M_OVERFLOW] += nc - g.C;
      nc = g.C;
    }
    for (int round = 0; round <= D + 1; ++round) {
      for (int d = tid; d < D; d += NT) {
        L.row_max[d] = 0ull;
        L.row_arg[d] = INT_MAX;
      }
      for (int t = tid; t < n; t += NT) {
        L.col_max[t] = 0ull;
        L.col_arg[t] = INT_MAX;
      }
      if (tid == 0) L.misc[M_ACTIVE] = 0;
      __syncthreads();
      int local_active = 0;
      for (int c = tid; c < nc; c += NT) {
        const int f = cflat[c], d = f / n, t = f - d * n;
        if (L.det_match[d] < 0 && L.trk_match[t] < 0) {
          const unsigned long long k = ckey[c];
          atomicMax(&L.row_max[d], k);
          atomicMax(&L.col_max[t], k);
          ++local_active;
        }
      }
      if (local_active) atomicAdd(&L.misc[M_ACTIVE], local_active);
      __syncthreads();
      if (L.misc[M_ACTIVE] == 0) {
        if (tid == 0) g.phase[s * PH + 10] = round;
        break;
      }
      // among equal IoUs the enhanced tracker takes the lowest row-major pair first (stable
      // argsort), the motion-reset tracker the highest (sorted (iou, d, t) tuples, reverse)
      for (int c = tid; c < nc; c += NT) {
        const int f = cflat[c], d = f / n, t = f - d * n;
        if (L.det_match[d] < 0 && L.trk_match[t] < 0) {
          const unsigned long long k = ckey[c];
          const int rk = POL ? npair - 1 - f : f;
          if (k == L.row_max[d]) atomicMin(&L.row_arg[d], rk);
          if (k == L.col_max[t]) atomicMin(&L.col_arg[t], rk);
        }
      }
      __syncthreads();
      for (int c = tid; c < nc; c += NT) {
        const int f = cflat[c], d = f / n, t = f - d * n;
        const int rk = POL ? npair - 1 - f : f;
        if (L.row_arg[d] == rk && L.col_arg[t] == rk) {
          L.det_match[d] = t;
          L.trk_match[t] = d;
        }
      }
      __syncthreads();
    }
  }

  if (tid == 0) g.phase[s * PH + 3] = wall_clock64();
  // Steps 3-4: update matched tracks, mark the others lost (multi:71-89).  The matched
  // tracks' velocity rings (1.2 KB each) are staged into LDS CH tracks at a time by the whole
  // workgroup (coalesced 16-B loads, all in flight at once); each track's thread then runs
  // the KF update and analyze_motion_pattern's serial reductions out of LDS.
  int recov = 0, resets = 0;
  int n_upd = 0;
  for (int base = 0; base < n; base += NT) {
    const int i = base + tid;
    const int flag = (i < n && L.trk_match[i] >= 0) ? 1 : 0;
    int tot;
    const int r = n_upd + block_scan(flag, wsum, tot);
    if (flag) L.order_tmp[r] = i;
    else if (i < n) mark_lost(slots[order[i]]);
    n_upd += tot;
  }
  __syncthreads();
  const int CH = stage_chunk(T, g.D);
  for (int c0 = 0; c0 < n_upd; c0 += CH) {
    const int m = n_upd - c0 < CH ? n_upd - c0 : CH;
    for (int u = tid; u < m * VH; u += NT) {  // chronological copy of each ring
      const int j = u / VH, k = u - j * VH;
      const Slot& sl = slots[order[L.order_tmp[c0 + j]]];
      if (k < sl.vh_len) {
        int idx = sl.vh_head + k;
        if (idx >= VH) idx -= VH;
        const double2 v = *(const double2*)&sl.vh[idx][0];
        double* st = L.stage + (size_t)j * STAGE_D;
        st[k] = v.x;
        st[VS + k] = v.y;
        st[2 * VS + k] = sl.vang[idx];
      }
    }
    __syncthreads();
    if (tid < m) {
      const int i = L.order_tmp[c0 + tid];
      Slot& sl = slots[order[i]];
      const int d = L.trk_match[i];
      DT db[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) db[k] = (DT)L.det[4 * d + k];
      if (POL && sl.policy) {  // MotionResetKalmanTracker.update (:261-285)
        double val[3] = {0.0, 0.0, 0.0};
        int why = 0;
        Num conf{0.0, KPY};
        if (cmc_decide<DT>(sl, db, val, why, conf)) {
          cmc_reset<DT>(sl, db, val, why, conf);
          ++resets;
        } else {
          kf_update<DT>(sl, db, L.stage + (size_t)tid * STAGE_D);
          ph_push(sl, sl.x[0], sl.x[1], false);  // the base update's position_history append
        }
        cmc_after_update<DT>(sl, db);
      } else {
        recov += sl.is_lost ? 1 : 0;
        kf_update<DT>(sl, db, L.stage + (size_t)tid * STAGE_D);
      }
    }
    __syncthreads();
  }
  if (recov) atomicAdd(&L.misc[M_RECOVER], recov);
  if (resets) atomicAdd(&L.misc[M_RESETS], resets);
  __syncthreads();
  if (tid == 0) g.phase[s * PH + 4] = wall_clock64();

  // Step 5: new tracks for unmatched detections, ascending detection order (multi:92-101)
  int n_new_total = 0;
  const int next_num = (int)H.st.next_track_id;
  const int nfree0 = nfree_base;
  for (int base = 0; base < D; base += NT) {
    const int d = base + tid;
    const int flag = (d < D && L.det_match[d] < 0) ? 1 : 0;
    int tot;
    const int r = n_new_total + block_scan(flag, wsum, tot);
    if (flag) {
      const int pos = n + r;
      if (pos < T && r < nfree0) {
        const int slot = fstack[nfree0 - 1 - r];
        DT db[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) db[k] = (DT)L.det[4 * d + k];
        double z[4];
        bbox_to_state<DT>(db, z);
        slot_init(slots[slot], z, next_num + r, g.max_lost);
        if (POL) cmc_init<DT>(slots[slot], db);
        order[pos] = slot;
      } else {
        atomicAdd(&L.misc[M_OVERFLOW], 1);
      }
    }
    n_new_total += tot;
  }
  int n_new = n_new_total;
  if (n + n_new > T) n_new = T - n;
  if (n_new > nfree0) n_new = nfree0;
  __syncthreads();

  if (tid == 0) g.phase[s * PH + 5] = wall_clock64();
  // Step 6: delete (multi:104-113) with a stable compaction of the list
  const int n_all = n + n_new;
  int kept = 0, n_del = 0;
  for (int base = 0; base < n_all; base += NT) {
    const int i = base + tid;
    int slot = -1, keep = 0;
    if (i < n_all) {
      slot = order[i];
      keep = should_delete(slots[slot], g.max_lost) ? 0 : 1;
    }
    int tot;
    const int r = kept + block_scan(keep, wsum, tot);
    if (i < n_all) {
      if (keep) L.order_tmp[r] = slot;
    }
    kept += tot;
  }
  n_del = n_all - kept;
  __syncthreads();
  // return deleted slots to the free stack: collect them in a second pass
  {
    const int nfree_after_pop = nfree0 - n_new;
    int pushed = 0;
    for (int base = 0; base < n_all; base += NT) {
      const int i = base + tid;
      int slot = -1, del = 0;
      if (i < n_all) {
        slot = order[i];
        del = should_delete(slots[slot], g.max_lost) ? 1 : 0;
      }
      int tot;
      const int r = pushed + block_scan(del, wsum, tot);
      if (del) fstack[nfree_after_pop + r] = slot;
      // motion-reset stats['tracking_recoveries']: deleted trackers that had been reset
      if (POL && del && slots[slot].policy && slots[slot].reset_count > 0) atomicAdd(&L.misc[M_TRECOV], 1);
      pushed += tot;
    }
  }
  __syncthreads();
  for (int i = tid; i < kept; i += NT) order[i] = L.order_tmp[i];
  __syncthreads();

  if (tid == 0) g.phase[s * PH + 6] = wall_clock64();
  // Step 7: outputs in list order (multi:116-126), get_track_info may predict (quirk A).
  // Rows are filled one thread per track; the 30-point trajectories are then copied by the
  // whole workgroup, one 16-B point per thread (the ring reads are independent loads).
  const int fc = (int)H.st.frame_count + 1;
  int nout = 0, lt = 0;
  for (int base = 0; base < kept; base += NT) {
    const int i = base + tid;
    int q = 0;
    Slot* sl = nullptr;
    if (i < kept) {
      sl = &slots[order[i]];
      // the motion-reset tracker reports every live tracker (motion_compensated_multi_tracker.py:369-386)
      q = (POL || sl->hit_streak >= g.min_hits || fc <= g.min_hits || sl->is_lost) ? 1 : 0;
    }
    int tot;
    const int r = nout + block_scan(q, wsum, tot);
    if (q) {
      yk_track_out& o = g.rows[(size_t)s * T + r];
      track_info(*sl, o, false);
      if (!POL && o.status == 1 && o.time_since_update > 30) ++lt;
      L.order_tmp[r] = order[i];
    }
    nout += tot;
  }
  if (lt) atomicAdd(&L.misc[M_LONGTERM], lt);
  __syncthreads();
  for (int u = tid; u < nout * TOUT; u += NT) {
    const int r = u / TOUT, k = u - r * TOUT;
    const Slot& sl = slots[L.order_tmp[r]];
    const int nt = sl.th_len < TOUT ? sl.th_len : TOUT;
    double2 v = make_double2(0.0, 0.0);
    if (k < nt) {
      int idx = sl.th_head + (sl.th_len - nt) + k;
      if (idx >= TH) idx -= TH;
      v = make_double2(sl.th[idx][0], sl.th[idx][1]);
    }
    *(double2*)&g.rows[(size_t)s * T + r].traj[k][0] = v;
  }
  __syncthreads();
  if (tid == 0) g.phase[s * PH + 7] = wall_clock64();
  if (tid == 0) {
    H.n_tracks = kept;
    H.n_free = nfree0 - n_new + n_del;
    H.st.frame_count = fc;
    H.st.next_track_id += n_new;
    H.st.total_tracks_created += n_new;
    H.st.total_tracks_terminated += n_del + (greset ? n_old : 0);
    H.st.global_resets += greset;
    H.st.current_active_tracks = kept;
    H.st.long_term_predictions += L.misc[M_LONGTERM];
    H.st.successful_recoveries += L.misc[M_RECOVER];
    H.st.individual_resets += L.misc[M_RESETS];
    H.st.tracking_recoveries += L.misc[M_TRECOV];
    H.st.overflow += L.misc[M_OVERFLOW] + (Draw - D);
    g.counts[s] = nout;
    g.stats[s] = H.st;
  }
}

// ---------------------------------------------------------------- enhanced step across CUs
// The enhanced policy's step as two launches (one workgroup per stream left the per-track work --
// update + analyze_motion_pattern, get_track_info -- serial on S CUs):
//  assoc_kernel   one workgroup per stream: the predicted boxes (read-only, x' = F x), candidate
//                 pairs through an x-bin index of the predicted boxes, the locally-dominant greedy
//                 rounds, and every list decision of the step (kept / deleted / reported tracks,
//                 new tracks and their slots, the compacted order, the free stack, the stats).
//                 The decisions need only the counters that predict / update / mark_lost change
//                 deterministically (age, time_since_update, hit_streak, is_lost), so this kernel
//                 never waits for the per-track arithmetic.  It writes one work item per track:
//                 {slot, matched detection, new-track number (-1: existing), output row (-1: none)}.
//  tracks_kernel  ceil(T / IPB) workgroups per stream, one thread per work item: predict and
//                 update or mark_lost (kf.py:184-317), or __init__ for a new track, then
//                 get_track_info into its output row; the workgroup stages the updated tracks'
//                 velocity rings and copies the trajectories cooperatively.
// Candidate index: a pair whose x-intervals do not overlap has IoU exactly 0 in the reference's
// arithmetic (iou_mixed: ix2 <= ix1), so for a threshold > 0 only tracks whose left edge lies in
// [d.x1 - max_width - margin, d.x2 + margin] can be candidates of detection d.  Tracks are
// counting-sorted by left edge into <= NB_MAX bins (monotone bin map); the pairs in the bin range
// get the exact IoU test.  Non-finite boxes and thresholds <= 0 fall back to all pairs.

__device__ __forceinline__ void lslot_bind(LSlot& l, Slot& g) {
  l.vh = g.vh;
  l.vang = g.vang;
  l.th = g.th;
}
__device__ __forceinline__ void lslot_load(LSlot& l, Slot& g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) l.x[i] = g.x[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) l.P[i] = g.P[i];
  l.vavg[0] = g.vavg[0];
  l.vavg[1] = g.vavg[1];
  l.vstd[0] = g.vstd[0];
  l.vstd[1] = g.vstd[1];
  l.direction = g.direction;
  l.speed = g.speed;
  l.stability = g.stability;
  l.pconf = g.pconf;
  l.age = g.age;
  l.hits = g.hits;
  l.hit_streak = g.hit_streak;
  l.tsu = g.tsu;
  l.is_lost = g.is_lost;
  l.lost_frames = g.lost_frames;
  l.track_num = g.track_num;
  l.max_lost = g.max_lost;
  l.vh_len = g.vh_len;
  l.vh_head = g.vh_head;
  l.th_len = g.th_len;
  l.th_head = g.th_head;
  l.th_cnt = g.th_cnt;
  l.policy = g.policy;
  lslot_bind(l, g);
}
__device__ __forceinline__ void lslot_store(const LSlot& l, Slot& g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) g.x[i] = l.x[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) g.P[i] = l.P[i];
  g.vavg[0] = l.vavg[0];
  g.vavg[1] = l.vavg[1];
  g.vstd[0] = l.vstd[0];
  g.vstd[1] = l.vstd[1];
  g.direction = l.direction;
  g.speed = l.speed;
  g.stability = l.stability;
  g.pconf = l.pconf;
  g.age = l.age;
  g.hits = l.hits;
  g.hit_streak = l.hit_streak;
  g.tsu = l.tsu;
  g.is_lost = l.is_lost;
  g.lost_frames = l.lost_frames;
  g.track_num = l.track_num;
  g.max_lost = l.max_lost;
  g.vh_len = l.vh_len;
  g.vh_head = l.vh_head;
  g.th_len = l.th_len;
  g.th_head = l.th_head;
  g.th_cnt = l.th_cnt;
  g.policy = l.policy;
}

constexpr int NB_MAX = NT - 1;  // x bins of the candidate index (+1 for the non-finite tracks <= NT)
constexpr int IPB = 64;      // work items per tracks_kernel workgroup

struct LdsA {
  double* pb;                   // [T][4] predicted boxes by list position
  double* det;                  // [D][4]
  unsigned long long* row_max;  // [D]   (decisions: int newdet[D])
  unsigned long long* col_max;  // [T]   (decisions: int flags[T])
  double* red;                  // [3][16] per-wave index bounds
  int* det_match;               // [D]
  int* trk_match;               // [T]
  int* row_arg;                 // [D]
  int* col_arg;                 // [T]   (candidate index: tracks sorted by bin)
  int* order_tmp;               // [T]   pre-step order, then the work items' slots
  int* bins;                    // [2][NB_MAX + 1] bin starts, scatter cursors
  int* misc;                    // [32] counters; [16, 32) wave sums
  unsigned long long* ck;       // [ccap] candidate keys written by the pair walk (rest: global)
  int* cp;                      // [ccap] their pairs
  int ccap;
};
constexpr int NTA = 1024;  // assoc_kernel threads: one element per thread in most phases
constexpr int MA_WSUM = 16;

__host__ __device__ inline size_t assoc_lds_bytes(int T, int D) {
  return (size_t)T * 32 + (size_t)D * 32 + (size_t)D * 8 + (size_t)T * 8 + 48 * 8 + (size_t)D * 4 +
         (size_t)T * 4 + (size_t)D * 4 + (size_t)T * 4 + (size_t)T * 4 + 2 * (NB_MAX + 1) * 4 + 32 * 4;
}
// candidates kept in LDS: what is left of the 160 KB after the fixed arrays, at most C
constexpr size_t LDS_CU = 160 * 1024;
__host__ __device__ inline int assoc_lds_cand(int T, int D, int C) {
  const size_t b = (assoc_lds_bytes(T, D) + 7) & ~(size_t)7;
  const size_t k = b < LDS_CU ? (LDS_CU - b) / 12 : 0;
  return (int)(k < (size_t)C ? k : (size_t)C);
}
__host__ __device__ inline size_t tracks_lds_bytes() { return (size_t)IPB * STAGE_D * 8 + (size_t)IPB * 36 + 16 + 16; }

__device__ LdsA carve_a(char* base, int T, int D, int C) {
  LdsA L;
  L.pb = (double*)base;
  base += (size_t)T * 32;
  L.det = (double*)base;
  base += (size_t)D * 32;
  L.row_max = (unsigned long long*)base;
  base += (size_t)D * 8;
  L.col_max = (unsigned long long*)base;
  base += (size_t)T * 8;
  L.red = (double*)base;
  base += 48 * 8;
  L.det_match = (int*)base;
  base += (size_t)D * 4;
  L.trk_match = (int*)base;
  base += (size_t)T * 4;
  L.row_arg = (int*)base;
  base += (size_t)D * 4;
  L.col_arg = (int*)base;
  base += (size_t)T * 4;
  L.order_tmp = (int*)base;
  base += (size_t)T * 4;
  L.bins = (int*)base;
  base += 2 * (NB_MAX + 1) * 4;
  L.misc = (int*)base;
  base += 32 * 4;
  L.ccap = assoc_lds_cand(T, D, C);
  L.ck = (unsigned long long*)(((size_t)base + 7) & ~(size_t)7);
  L.cp = (int*)(L.ck + L.ccap);
  return L;
}

// exclusive prefix sum of v over the workgroup; total gets the block sum
template <int NTH>
__device__ __forceinline__ int block_excl_sum(int v, int* wsum, int& total) {
  constexpr int NW = NTH / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    base += (i < w) ? wsum[i] : 0;
    tot += wsum[i];
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

__device__ __forceinline__ int xbin(double x, double x0, double ibw, int nb) {
  const double q = (x - x0) * ibw;  // monotone in x (ibw > 0)
  return !(q > 0.0) ? 0 : (q >= (double)(nb - 1) ? nb - 1 : (int)q);
}

// Greedy association (multi:134-178) as locally-dominant rounds (header comment) over nc
// candidates {IoU bits, (d << 16) | t}; inlined once with LDS and once with global operands.
// rev: among equal IoUs the highest (d, t) first (the motion-reset tracker's reversed sort of
// (iou, d, t) tuples, motion_compensated_multi_tracker.py:262-270), else the lowest
__device__ __forceinline__ void assoc_rounds(const LdsA& L, const unsigned long long* ckey, const int* cpid, int nc,
                                             int D, int n, long long* round_out, bool rev,
                                             yk_track_event* ev = nullptr) {
  const int tid = threadIdx.x;
  for (int round = 0; round <= D + 1; ++round) {
    for (int d = tid; d < D; d += NTA) {
      L.row_max[d] = 0ull;
      L.row_arg[d] = INT_MAX;
    }
    for (int t = tid; t < n; t += NTA) {
      L.col_max[t] = 0ull;
      L.col_arg[t] = INT_MAX;
    }
    if (tid == 0) L.misc[M_ACTIVE] = 0;
    __syncthreads();
    int local_active = 0;
    for (int c = tid; c < nc; c += NTA) {
      const int f = cpid[c], d = f >> 16, t = f & 0xffff;
      if (L.det_match[d] < 0 && L.trk_match[t] < 0) {
        const unsigned long long k = ckey[c];
        atomicMax(&L.row_max[d], k);
        atomicMax(&L.col_max[t], k);
        ++local_active;
      }
    }
    if (local_active) atomicAdd(&L.misc[M_ACTIVE], local_active);
    __syncthreads();
    if (L.misc[M_ACTIVE] == 0) {
      if (tid == 0) *round_out = round;
      break;
    }
    for (int c = tid; c < nc; c += NTA) {
      const int f = cpid[c], d = f >> 16, t = f & 0xffff;
      if (L.det_match[d] < 0 && L.trk_match[t] < 0) {
        const unsigned long long k = ckey[c];
        const int rk = rev ? (INT_MAX - 1) - f : f;  // never the INT_MAX "no candidate" sentinel
        if (k == L.row_max[d]) atomicMin(&L.row_arg[d], rk);
        if (k == L.col_max[t]) atomicMin(&L.col_arg[t], rk);
      }
    }
    __syncthreads();
    for (int c = tid; c < nc; c += NTA) {
      const int f = cpid[c], d = f >> 16, t = f & 0xffff;
      const int rk = rev ? (INT_MAX - 1) - f : f;
      // (a detection or track matched in an earlier round keeps the sentinel in its arg slot:
      // only still-unmatched pairs may take this round's match)
      if (L.row_arg[d] == rk && L.col_arg[t] == rk && L.det_match[d] < 0 && L.trk_match[t] < 0) {
        L.det_match[d] = t;
        L.trk_match[t] = d;
        if (ev) ev[t].iou = __longlong_as_double((long long)ckey[c]);  // the event log's match order key
      }
    }
    __syncthreads();
  }
}

template <typename DT, int POL>
__global__ void __launch_bounds__(NTA) assoc_kernel(Dev g, const DT* __restrict__ dets, int row_stride,
                                                   const int* __restrict__ counts,
                                                   const yk_motion* __restrict__ motion) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int T = g.T;
  LdsA L = carve_a(smem, T, g.D, g.C);
  Hdr& H = g.hdr[s];
  const Slot* slots = g.slots + (size_t)s * T;
  int* order = g.order + (size_t)s * T;
  int* fstack = g.free_stack + (size_t)s * T;
  int* wsum = L.misc + MA_WSUM;
  // event log (enhanced policy only): written only when the host enabled it
  yk_track_event* evs = (!POL && g.events) ? g.events + (size_t)s * T : nullptr;

  const long long cyc0 = clock64();  // shader clock: phase[15] = cycles of this kernel (clock check)
  if (tid == 0) g.phase[s * PH + 0] = wall_clock64();
  // candidate sub-phase stamps are written only when this step has both tracks and detections:
  // clear them so phase_us never mixes a previous step's stamps in
  if (tid == 0)
    for (int k = 20; k < 23; ++k) g.phase[s * PH + k] = 0;
  int Draw = counts[s];
  if (Draw < 0) Draw = 0;
  const int D = Draw < g.D ? Draw : g.D;
  const int n_old = H.n_tracks;
  int nfree_base = H.n_free;
  int greset = 0;
  if (POL && tid == 0) greset = global_branch(H, motion, s, Draw) ? 1 : 0;
  if (tid < 16) L.misc[tid] = 0;  // counters ([16, 32): wave sums)
  if (POL) {
    __syncthreads();
    if (tid == 0) L.misc[M_GRESET] = greset;
    __syncthreads();
    greset = L.misc[M_GRESET];
    if (greset) {  // _perform_global_reset (:150-169): trackers.clear(), slots back to the stack
      for (int i = tid; i < n_old; i += NTA) fstack[nfree_base + i] = order[i];
      nfree_base += n_old;
    }
  }
  const int n = greset ? 0 : n_old;
  for (int i = tid; i < D * 4; i += NTA) {
    const int d = i >> 2, k = i & 3;
    L.det[i] = (double)dets[((size_t)s * g.D + d) * row_stride + k];
  }
  for (int d = tid; d < D; d += NTA) L.det_match[d] = -1;
  // predicted boxes: predict() (kf.py:192-201) then the bbox, without changing the slot
  double lx0 = INFINITY, lx1 = -INFINITY, lw = 0.0;
  for (int i = tid; i < n; i += NTA) {
    const int slot = order[i];
    L.order_tmp[i] = slot;
    L.trk_match[i] = -1;
    const Slot& sl = slots[slot];
    double xp[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) xp[c] = sl.x[c] + sl.x[c + 4];
    double* b = &L.pb[4 * i];
    state_to_bbox(xp, b);
    if (POL && sl.policy) cmc_blend(sl, b, sl.age + 1);  // the subclass's predict() box
    const double w = b[2] - b[0];
    if (isfinite(b[0]) && isfinite(b[2]) && isfinite(w)) {
      lx0 = fmin(lx0, b[0]);
      lx1 = fmax(lx1, b[0]);
      lw = fmax(lw, w);
    }
  }
  // the index bounds (min / max left edge, max width): per wave here, across the waves after
  // the barrier, so the reductions add no barrier; the bin counts are cleared here as well
  for (int o = 32; o > 0; o >>= 1) {
    lx0 = fmin(lx0, __shfl_xor(lx0, o));
    lx1 = fmax(lx1, __shfl_xor(lx1, o));
    lw = fmax(lw, __shfl_xor(lw, o));
  }
  if ((tid & 63) == 0) {
    L.red[tid >> 6] = lx0;
    L.red[16 + (tid >> 6)] = lx1;
    L.red[32 + (tid >> 6)] = lw;
  }
  for (int b = tid; b <= NB_MAX; b += NTA) L.bins[b] = 0;
  __syncthreads();
  if (tid == 0) g.phase[s * PH + 1] = wall_clock64();

  int nc = 0;
  if (D > 0 && n > 0) {
    unsigned long long* ckey = g.cand_key + (size_t)s * g.C;
    int* cflat = g.cand_flat + (size_t)s * g.C;
    double x0 = L.red[0], x1 = L.red[16], wmax = L.red[32];
#pragma unroll
    for (int w = 1; w < NTA / 64; ++w) {
      x0 = fmin(x0, L.red[w]);
      x1 = fmax(x1, L.red[16 + w]);
      wmax = fmax(wmax, L.red[32 + w]);
    }
    const bool index = g.thr > 0.0 && x0 <= x1;  // else every pair is tested
    if (tid == 0) g.phase[s * PH + 20] = wall_clock64();
    const int nb = n < NB_MAX ? n : NB_MAX;
    double bw = (x1 - x0) / (double)nb;
    if (!(bw > 0.0) || !isfinite(bw)) bw = 1.0;
    const double ibw = 1.0 / bw;         // bins by (x - x0) * ibw: monotone in x like the quotient
    int* bstart = L.bins;                // [nb + 1]: bin starts, [nb] = finite tracks
    int* bcur = L.bins + (NB_MAX + 1);
    int* tsorted = L.col_arg;
    int nfin = 0;
    if (index) {
      for (int i = tid; i < n; i += NTA) {
        const double* b = &L.pb[4 * i];
        const bool fin = isfinite(b[0]) && isfinite(b[2]) && isfinite(b[2] - b[0]);
        atomicAdd(&bstart[fin ? xbin(b[0], x0, ibw, nb) : nb], 1);
      }
      __syncthreads();
      int tot;
      const int v = tid <= nb ? bstart[tid] : 0;  // nb + 1 <= NTA entries
      const int ex = block_excl_sum<NTA>(v, wsum, tot);
      if (tid <= nb) {
        bstart[tid] = ex;
        bcur[tid] = ex;
      }
      __syncthreads();
      nfin = bstart[nb];
      for (int i = tid; i < n; i += NTA) {
        const double* b = &L.pb[4 * i];
        const bool fin = isfinite(b[0]) && isfinite(b[2]) && isfinite(b[2] - b[0]);
        tsorted[atomicAdd(&bcur[fin ? xbin(b[0], x0, ibw, nb) : nb], 1)] = i;
      }
      __syncthreads();
    }
    if (tid == 0) g.phase[s * PH + 21] = wall_clock64();
    // candidates (multi:180-232 over the pairs the index admits).  Detection d's pairs are the
    // tracks [k0, k0 + len) of the bin order, then the non-finite tracks; the pairs of all
    // detections are numbered by a prefix sum and every thread walks an equal slice of them
    // (one binary search for its first detection), so one wide detection cannot stall a wave.
    const double margin = 1.0 + 1e-9 * (fabs(x0) + fabs(x1) + wmax);
    int* pk0 = (int*)L.row_max;  // [D] (row_max: 8 D bytes, free until the rounds)
    int* plen = pk0 + D;         // [D]
    int* pbeg = L.row_arg;       // [D] first pair number of each detection
    const int ne = index ? n - nfin : 0;
    int total = 0;
    for (int base = 0; base < D; base += NTA) {
      const int d = base + tid;
      int cnt = 0;
      if (d < D) {
        int k0 = 0, k1 = n;  // all pairs
        if (index) {
          const double dx1 = L.det[4 * d], dx2 = L.det[4 * d + 2];
          if (isfinite(dx1) && isfinite(dx2)) {
            const double lo = (dx1 - wmax) - margin, hi = dx2 + margin;
            const int b0 = isfinite(lo) ? xbin(lo, x0, ibw, nb) : 0;
            const int b1 = isfinite(hi) ? xbin(hi, x0, ibw, nb) : nb - 1;
            k0 = bstart[b0];
            k1 = b1 >= b0 ? bstart[b1 + 1] : k0;
          } else {
            k1 = nfin;
          }
        }
        pk0[d] = k0;
        plen[d] = k1 - k0;
        cnt = k1 - k0 + ne;
      }
      int tot;
      const int ex = block_excl_sum<NTA>(cnt, wsum, tot);
      if (d < D) pbeg[d] = total + ex;
      total += tot;
    }
    __syncthreads();
    if (tid == 0) g.phase[s * PH + 22] = wall_clock64();
    {
      const int per = (total + NTA - 1) / NTA;
      int p = tid * per;
      const int pend = p + per < total ? p + per : total;
      if (p < pend) {
        int lo = 0, hi = D - 1;  // the last detection whose pairs start at or before p
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pbeg[mid] <= p) lo = mid;
          else hi = mid - 1;
        }
        int d = lo, beg = pbeg[d], k0 = pk0[d], len = plen[d];
        DT db[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) db[k] = (DT)L.det[4 * d + k];
        for (; p < pend; ++p) {
          int o = p - beg;
          while (o >= len + ne) {  // next detection with pairs
            ++d;
            beg = pbeg[d];
            k0 = pk0[d];
            len = plen[d];
#pragma unroll
            for (int k = 0; k < 4; ++k) db[k] = (DT)L.det[4 * d + k];
            o = p - beg;
          }
          const int kk = o < len ? k0 + o : nfin + (o - len);
          const int t = index ? tsorted[kk] : kk;
          const double v = iou_mixed<DT>(db, &L.pb[4 * t]);
          // enhanced: iou >= thr (multi:245); motion-reset: iou > thr (motion_compensated_multi_tracker.py:260)
          if (POL ? v > g.thr : v >= g.thr) {
            const int c = atomicAdd(&L.misc[M_NCAND], 1);
            const unsigned long long key = (unsigned long long)__double_as_longlong(v);
            const int f = (d << 16) | t;  // orders like the row-major pair index d * n + t
            if (c < L.ccap) {
              L.ck[c] = key;
              L.cp[c] = f;
            } else if (c < g.C) {
              ckey[c] = key;
              cflat[c] = f;
            }
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      g.phase[s * PH + 2] = wall_clock64();
      g.phase[s * PH + 11] = total;
      g.phase[s * PH + 12] = L.misc[M_NCAND];
      g.phase[s * PH + 13] = (long long)(isfinite(wmax) ? wmax : -1.0);
      g.phase[s * PH + 14] = n - nfin;
      g.phase[s * PH + 23] = L.ccap;  // candidates the walk's LDS area holds
    }
    nc = L.misc[M_NCAND];
    if (nc > g.C) {
      if (tid == 0) L.misc[M_OVERFLOW] += nc - g.C;
      nc = g.C;
    }
    // the rounds read the candidates from the walk's LDS area when it held them all; else the
    // LDS head joins the global tail, and the rounds read them where the boxes were (dead now)
    // when they fit there, else from global memory
    if (nc <= L.ccap) {
      assoc_rounds(L, L.ck, L.cp, nc, D, n, g.phase + s * PH + 10, POL != 0, evs);
    } else {
      for (int c = tid; c < L.ccap; c += NTA) {
        ckey[c] = L.ck[c];
        cflat[c] = L.cp[c];
      }
      __syncthreads();
      const int cap = (int)(((size_t)T * 32 + (size_t)g.D * 32) / 12);
      if (nc <= cap) {
        unsigned long long* lk = (unsigned long long*)L.pb;
        int* lp = (int*)(lk + nc);
        for (int c = tid; c < nc; c += NTA) {
          lk[c] = ckey[c];
          lp[c] = cflat[c];
        }
        __syncthreads();
        assoc_rounds(L, lk, lp, nc, D, n, g.phase + s * PH + 10, POL != 0, evs);
      } else {
        assoc_rounds(L, ckey, cflat, nc, D, n, g.phase + s * PH + 10, POL != 0, evs);
      }
    }
  } else if (tid == 0) {  // no pairs: an empty candidate phase, no rounds
    g.phase[s * PH + 2] = wall_clock64();
    g.phase[s * PH + 10] = 0;
    for (int k = 11; k < 15; ++k) g.phase[s * PH + k] = 0;
  }
  if (tid == 0) g.phase[s * PH + 3] = wall_clock64();

  // Decisions.  Post-step counters of an existing track (predict, then update or mark_lost):
  // age + 1; matched: tsu 0, hit_streak + 1, not lost; else tsu + 1, hit_streak 0, lost.
  // flags: 1 kept (not should_delete, kf.py:385-405), 2 reported (multi:116-126), 4 reported with
  // status 1 and time_since_update > 30 (long_term_predictions).
  int* flags = (int*)L.col_max;
  int* newdet = (int*)L.row_max;
  // A motion-reset update that resets the filter leaves the same counters as the plain update
  // (cmc_reset: hits + 1, hit_streak + 1, tsu 0), so the decisions hold for both policies; that
  // tracker reports every live track and counts a deleted tracker that had been reset.
  const int fc = (int)H.st.frame_count + 1;
  int recov = 0, trecov = 0;
  int2* items_vh = g.items_vh + (size_t)s * T;
  for (int i = tid; i < n; i += NTA) {
    const Slot& sl = slots[L.order_tmp[i]];
    const bool m = L.trk_match[i] >= 0;
    items_vh[i] = make_int2(sl.vh_len, sl.vh_head);
    const int age = sl.age + 1, tsu = m ? 0 : sl.tsu + 1, hs = m ? sl.hit_streak + 1 : 0;
    const bool del = tsu > g.max_lost || (age < 5 && hs == 0 && tsu > 15) || (age < 10 && hs <= 1 && tsu > 30);
    if (POL && sl.policy) {
      trecov += (del && sl.reset_count > 0) ? 1 : 0;
      flags[i] = del ? 0 : 3;
    } else {
      recov += (m && sl.is_lost) ? 1 : 0;
      const bool q = hs >= g.min_hits || fc <= g.min_hits || !m;
      flags[i] = (del ? 0 : 1) | (q ? 2 : 0) | (tsu > 30 ? 4 : 0);
      if (evs) {  // multi:104-110: removed with this time_since_update
        evs[i].list_pos = i;
        evs[i].det = L.trk_match[i];
        evs[i].deleted_tsu = del ? tsu : -1;
      }
    }
  }
  if (recov) atomicAdd(&L.misc[M_RECOVER], recov);
  if (trecov) atomicAdd(&L.misc[M_TRECOV], trecov);
  // new tracks for unmatched detections, ascending detection order (multi:92-101)
  int n_new_total = 0;
  const int next_num = (int)H.st.next_track_id;
  const int nfree0 = nfree_base;
  for (int base = 0; base < D; base += NTA) {
    const int d = base + tid;
    const int flag = (d < D && L.det_match[d] < 0) ? 1 : 0;
    int tot;
    const int r = n_new_total + block_scan<NTA>(flag, wsum, tot);
    if (flag) {
      const int pos = n + r;
      if (pos < T && r < nfree0) {
        L.order_tmp[pos] = fstack[nfree0 - 1 - r];
        newdet[r] = d;
        if (evs) {
          evs[pos].list_pos = pos;
          evs[pos].det = d;
          evs[pos].deleted_tsu = -1;
        }
        // a new track: age 0, hit_streak 1, tsu 0, not lost (kf.py:32-101)
        flags[pos] = 1 | ((POL || 1 >= g.min_hits || fc <= g.min_hits) ? 2 : 0);
      } else {
        atomicAdd(&L.misc[M_OVERFLOW], 1);
      }
    }
    n_new_total += tot;
  }
  int n_new = n_new_total;
  if (n + n_new > T) n_new = T - n;
  if (n_new > nfree0) n_new = nfree0;
  __syncthreads();  // the popped slots are read before the deleted ones are pushed
  // work items, the compacted order (kept tracks in list order), the free stack, output rows
  const int n_all = n + n_new;
  const int nfree_after_pop = nfree0 - n_new;
  int kept = 0, nout = 0, pushed = 0, lt = 0;
  int4* items = g.items + (size_t)s * T;
  for (int base = 0; base < n_all; base += NTA) {
    const int j = base + tid;
    const int f = j < n_all ? flags[j] : 0;
    const int keep = f & 1, q = (f >> 1) & keep, del = (j < n && !keep) ? 1 : 0;
    int tk, tq, td;
    const int rk = kept + block_scan<NTA>(keep, wsum, tk);
    const int rq = nout + block_scan<NTA>(q, wsum, tq);
    const int rd = pushed + block_scan<NTA>(del, wsum, td);
    if (j < n_all) {
      const int slot = L.order_tmp[j];
      if (keep) order[rk] = slot;
      if (del) fstack[nfree_after_pop + rd] = slot;
      if (q && (f & 4)) ++lt;
      items[j] = make_int4(slot, j < n ? L.trk_match[j] : newdet[j - n], j < n ? -1 : next_num + (j - n), q ? rq : -1);
    }
    kept += tk;
    nout += tq;
    pushed += td;
  }
  if (lt) atomicAdd(&L.misc[M_LONGTERM], lt);
  __syncthreads();
  if (tid == 0) {
    const long long t4 = wall_clock64();
    for (int k = 4; k < 8; ++k) g.phase[s * PH + k] = t4;
    g.phase[s * PH + 15] = clock64() - cyc0;
    g.n_items[s] = n_all;
    H.n_tracks = kept;
    H.n_free = nfree_after_pop + pushed;
    H.st.frame_count = fc;
    H.st.next_track_id += n_new;
    H.st.total_tracks_created += n_new;
    H.st.total_tracks_terminated += pushed + (greset ? n_old : 0);
    H.st.global_resets += greset;
    H.st.current_active_tracks = kept;
    H.st.long_term_predictions += L.misc[M_LONGTERM];
    H.st.successful_recoveries += L.misc[M_RECOVER];
    H.st.tracking_recoveries += L.misc[M_TRECOV];
    H.st.overflow += L.misc[M_OVERFLOW] + (Draw - D);
    g.counts[s] = nout;
    g.stats[s] = H.st;  // tracks_kernel adds the step's individual resets to both
  }
}

template <typename DT, int POL>
__global__ void __launch_bounds__(NT) tracks_kernel(Dev g, const DT* __restrict__ dets, int row_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.y, tid = threadIdx.x;
  const int base = blockIdx.x * IPB;
  const int nI = g.n_items[s];
  if (base >= nI) return;
  const int m = nI - base < IPB ? nI - base : IPB;
  double* stage = (double*)smem;                           // [IPB][STAGE_D]
  int4* it = (int4*)(smem + (size_t)IPB * STAGE_D * 8);    // [IPB]
  int2* ivh = (int2*)(it + IPB);  // [IPB] {vh_len, vh_head} before the step, then {th_len, th_head} after it
  int* lst = (int*)(ivh + IPB);   // [3][IPB] the block's items by path: update, lost, new
  int* lcnt = lst + 3 * IPB;      // [3] path counts, then [3] the step's motion-reset filter resets
  Slot* slots = g.slots + (size_t)s * g.T;
  if (blockIdx.x == 0 && tid == 0) g.phase[s * PH + 5] = wall_clock64();
  if (tid < m) {
    it[tid] = g.items[(size_t)s * g.T + base + tid];
    ivh[tid] = g.items_vh[(size_t)s * g.T + base + tid];
  }
  if (tid < 4) lcnt[tid] = 0;
  __syncthreads();
  // one path per wave (a wave runs every path its lanes take, one after the other)
  if (tid < m) {
    const int4 w = it[tid];
    const int path = w.z >= 0 ? 2 : (w.y >= 0 ? 0 : 1);
    lst[path * IPB + atomicAdd(&lcnt[path], 1)] = tid;
  }
  // chronological copy of each updated track's velocity ring (whole workgroup, independent loads)
  for (int u = tid; u < m * VH; u += NT) {
    const int j = u / VH, k = u - j * VH;
    const int4 w = it[j];
    if (w.z >= 0 || w.y < 0) continue;
    const Slot& sl = slots[w.x];
    const int2 vl = ivh[j];
    if (k < vl.x) {
      int idx = vl.y + k;
      if (idx >= VH) idx -= VH;
      const double2 v = *(const double2*)&sl.vh[idx][0];
      double* st = stage + (size_t)j * STAGE_D;
      st[k] = v.x;
      st[VS + k] = v.y;
      st[2 * VS + k] = sl.vang[idx];
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid == 0) g.phase[s * PH + 8] = wall_clock64();
  const int wv = tid >> 6, ln = tid & 63;
  const long long cw0 = clock64();
  if (POL && wv < 3 && ln < lcnt[wv]) {
    // the motion-reset tracker on the slot itself (its histories are part of the update)
    const int j = lst[wv * IPB + ln];
    const int4 w = it[j];
    Slot& sl = slots[w.x];
    DT db[4] = {DT(0), DT(0), DT(0), DT(0)};
    if (w.y >= 0) {  // (a lost track has no detection)
#pragma unroll
      for (int k = 0; k < 4; ++k) db[k] = dets[((size_t)s * g.D + w.y) * row_stride + k];
    }
    if (w.z < 0) {
      kf_predict(sl);  // the subclass's predict() blends only the returned box
      if (w.y >= 0) {  // MotionResetKalmanTracker.update (:261-285)
        double val[3] = {0.0, 0.0, 0.0};
        int why = 0;
        Num conf{0.0, KPY};
        if (sl.policy && cmc_decide<DT>(sl, db, val, why, conf)) {
          cmc_reset<DT>(sl, db, val, why, conf);
          atomicAdd(&lcnt[3], 1);
        } else {
          kf_update<DT>(sl, db, stage + (size_t)j * STAGE_D);
          if (sl.policy) ph_push(sl, sl.x[0], sl.x[1], false);  // the base update's position_history append
        }
        if (sl.policy) cmc_after_update<DT>(sl, db);
      } else {
        mark_lost(sl);
      }
    } else {
      double z[4];
      bbox_to_state<DT>(db, z);
      slot_init(sl, z, w.z, g.max_lost);
      cmc_init<DT>(sl, db);
    }
    if (w.w >= 0) track_info(sl, g.rows[(size_t)s * g.T + w.w], false);
    ivh[j] = make_int2(sl.th_len, sl.th_head);
  } else if (!POL && wv < 3 && ln < lcnt[wv]) {
    const int j = lst[wv * IPB + ln];
    const int4 w = it[j];
    Slot& gs = slots[w.x];
    LSlot sl;
    yk_track_event* ev = g.events ? g.events + (size_t)s * g.T + base + j : nullptr;
    if (w.z < 0) {
      lslot_load(sl, gs);
      const int was_lost = sl.is_lost, lost_before = sl.lost_frames;
      kf_predict(sl);  // multi:55-58
      if (w.y >= 0) {  // multi:71-80
        DT db[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) db[k] = dets[((size_t)s * g.D + w.y) * row_stride + k];
        kf_update<DT>(sl, db, stage + (size_t)j * STAGE_D);
        if (ev) {  // kf.py:264-271, multi:76-79
          ev->kind = was_lost ? YK_EV_RECOVERED : YK_EV_NONE;
          ev->lost_frames = lost_before;
        }
      } else {
        if (ev) {  // kf.py:305-314 (state after predict), multi:86-89
          ev->kind = was_lost ? YK_EV_NONE : YK_EV_LOST;
          ev->x = sl.x[0];
          ev->y = sl.x[1];
          ev->vx = sl.x[4];
          ev->vy = sl.x[5];
          ev->confidence = sl.pconf;
        }
        mark_lost(sl);  // multi:83-89
      }
      if (ev) ev->track_num = sl.track_num;
    } else {  // multi:92-101
      if (ev) {
        ev->kind = YK_EV_CREATED;
        ev->track_num = w.z;
      }
      DT db[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) db[k] = dets[((size_t)s * g.D + w.y) * row_stride + k];
      double z[4];
      bbox_to_state<DT>(db, z);
      lslot_bind(sl, gs);
      slot_init(sl, z, w.z, g.max_lost);
    }
    if (w.w >= 0) track_info(sl, g.rows[(size_t)s * g.T + w.w], false);
    lslot_store(sl, gs);
    ivh[j] = make_int2(sl.th_len, sl.th_head);
  }
  if (blockIdx.x == 0 && ln == 0 && wv < 3) g.phase[s * PH + 16 + wv] = clock64() - cw0;
  __syncthreads();
  if (POL && tid == 0 && lcnt[3]) {  // stats['individual_resets'] of this step
    atomicAdd((unsigned long long*)&g.hdr[s].st.individual_resets, (unsigned long long)lcnt[3]);
    atomicAdd((unsigned long long*)&g.stats[s].individual_resets, (unsigned long long)lcnt[3]);
  }
  if (blockIdx.x == 0 && tid == 0) g.phase[s * PH + 9] = wall_clock64();
  for (int u = tid; u < m * TOUT; u += NT) {
    const int j = u / TOUT, k = u - j * TOUT;
    const int4 w = it[j];
    if (w.w < 0) continue;
    const Slot& sl = slots[w.x];
    const int2 tl = ivh[j];  // th_len, th_head after the step
    const int nt = tl.x < TOUT ? tl.x : TOUT;
    double2 v = make_double2(0.0, 0.0);
    if (k < nt) {
      int idx = tl.y + (tl.x - nt) + k;
      if (idx >= TH) idx -= TH;
      v = *(const double2*)&sl.th[idx][0];
    }
    *(double2*)&g.rows[(size_t)s * g.T + w.w].traj[k][0] = v;
  }
  if (blockIdx.x == 0 && tid == 0) g.phase[s * PH + 6] = wall_clock64();
}

__global__ void reset_kernel(Dev g, int S) {
  const int s = blockIdx.x;
  if (s >= S) return;
  int* fstack = g.free_stack + (size_t)s * g.T;
  for (int i = threadIdx.x; i < g.T; i += blockDim.x) fstack[i] = g.T - 1 - i;  // pops 0,1,2,...
  if (threadIdx.x == 0) {
    Hdr& H = g.hdr[s];
    H.n_tracks = 0;
    H.n_free = g.T;
    H.st = yk_tracker_stats{};
    H.st.next_track_id = 1;
    H.dsh_len = H.dsh_head = H.gmh_len = H.gmh_head = 0;
    g.counts[s] = 0;
    g.stats[s] = H.st;
  }
}

// Snapshot of the live tracks of stream s in list order (dense P, rings oldest first).
__global__ void snapshot_kernel(Dev g, int s, yk_track_state* out) {
  const int n = g.hdr[s].n_tracks;
  const Slot* slots = g.slots + (size_t)s * g.T;
  const int* order = g.order + (size_t)s * g.T;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const Slot& sl = slots[order[i]];
    yk_track_state& o = out[i];
    o.track_num = sl.track_num;
    o.age = sl.age;
    o.hits = sl.hits;
    o.hit_streak = sl.hit_streak;
    o.time_since_update = sl.tsu;
    o.is_lost = sl.is_lost;
    o.lost_frames = sl.lost_frames;
    o.vel_len = sl.vh_len;
    o.traj_len = sl.th_len;
    o.max_lost_frames = sl.max_lost;
    for (int k = 0; k < 8; ++k) o.x[k] = sl.x[k];
    for (int k = 0; k < 64; ++k) o.P[k] = 0.0;
    for (int c = 0; c < 4; ++c) {
      o.P[c * 8 + c] = sl.P[4 * c + 0];
      o.P[c * 8 + c + 4] = sl.P[4 * c + 1];
      o.P[(c + 4) * 8 + c] = sl.P[4 * c + 2];
      o.P[(c + 4) * 8 + c + 4] = sl.P[4 * c + 3];
    }
    o.velocity_avg[0] = sl.vavg[0];
    o.velocity_avg[1] = sl.vavg[1];
    o.velocity_std[0] = sl.vstd[0];
    o.velocity_std[1] = sl.vstd[1];
    o.direction = sl.direction;
    o.speed = sl.speed;
    o.stability_score = sl.stability;
    o.prediction_confidence = sl.pconf;
    int idx = sl.vh_head;
    for (int k = 0; k < VH; ++k) {
      const bool v = k < sl.vh_len;
      o.vel_hist[k][0] = v ? sl.vh[idx][0] : 0.0;
      o.vel_hist[k][1] = v ? sl.vh[idx][1] : 0.0;
      idx = (idx + 1 == VH) ? 0 : idx + 1;
    }
    idx = sl.th_head;
    for (int k = 0; k < TH; ++k) {
      const bool v = k < sl.th_len;
      o.traj_hist[k][0] = v ? sl.th[idx][0] : 0.0;
      o.traj_hist[k][1] = v ? sl.th[idx][1] : 0.0;
      idx = (idx + 1 == TH) ? 0 : idx + 1;
    }
    o.reset_count = sl.policy ? sl.reset_count : 0;
    o.last_reset_frame = sl.policy ? sl.last_reset : -999;
    o.motion_consistency = sl.policy ? sl.consistency : 0.0;
  }
}

// Single-track object operations (AircraftKalmanTracker surface), one thread.
template <typename DT>
__global__ void track_op_kernel(Dev g, int s, int pos, int op, int arg, const double* in_box, double* out5,
                                yk_track_out* out_row) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Slot& sl = g.slots[(size_t)s * g.T + g.order[(size_t)s * g.T + pos]];
  double conf = 1.0;
  switch (op) {
    case YK_OP_PREDICT:
      kf_predict(sl);
      state_to_bbox(sl.x, out5);
      if (sl.policy) cmc_blend(sl, out5, sl.age);
      break;
    case YK_OP_UPDATE: {
      DT b[4];
      for (int k = 0; k < 4; ++k) b[k] = (DT)in_box[k];
      __shared__ double st[3 * VS];  // (one thread; LDS rather than a scratch array)
      stage_chrono(sl, st);
      double val[3] = {0.0, 0.0, 0.0};
      int why = 0;
      Num conf{0.0, KPY};
      if (sl.policy && cmc_decide<DT>(sl, b, val, why, conf)) {
        cmc_reset<DT>(sl, b, val, why, conf);
      } else {
        kf_update<DT>(sl, b, st);
        if (sl.policy) ph_push(sl, sl.x[0], sl.x[1], false);
      }
      if (sl.policy) cmc_after_update<DT>(sl, b);
      break;
    }
    case YK_OP_MARK_LOST:
      mark_lost(sl);
      break;
    case YK_OP_INFO:
      track_info(sl, *out_row);
      break;
    case YK_OP_LONG_TERM:
      long_term_predict(sl, arg, out5, conf);
      break;
    case YK_OP_LOST_PRED:
      lost_prediction(sl, out5, conf);
      break;
  }
  out5[4] = conf;
}

template <typename DT>
__global__ void track_create_kernel(Dev g, int s, const double* in_box, int track_num, int max_lost,
                                    int* status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Hdr& H = g.hdr[s];
  if (H.n_tracks >= g.T || H.n_free <= 0) {
    *status = 1;
    return;
  }
  const int slot = g.free_stack[(size_t)s * g.T + H.n_free - 1];
  H.n_free -= 1;
  DT b[4];
  for (int k = 0; k < 4; ++k) b[k] = (DT)in_box[k];
  double z[4];
  bbox_to_state<DT>(b, z);
  slot_init(g.slots[(size_t)s * g.T + slot], z, track_num, max_lost);
  if (g.policy) cmc_init<DT>(g.slots[(size_t)s * g.T + slot], b);
  g.order[(size_t)s * g.T + H.n_tracks] = slot;
  H.n_tracks += 1;
  *status = 0;
}

// Tracker output pushed to page-locked host memory by the device (yk_tracker_download_async): one
// workgroup per stream writes its count, its stats and only its LIVE rows (count[s] of them, known
// here and not on the host) with 8-byte stores through the host-mapped pointers -- one small
// launch instead of three copy-engine / blit transfers of every row slot.
__global__ void __launch_bounds__(256) push_out_kernel(Dev g, int S, int T, int rows_per_stream, yk_track_out* rows,
                                                       int32_t* counts, yk_tracker_stats* stats) {
  const int s = blockIdx.x;
  if (s >= S) return;
  const int c = g.counts[s];
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    counts[s] = c;
    if (stats) stats[s] = g.stats[s];
  }
  if (!rows) return;
  const int n = c < rows_per_stream ? c : rows_per_stream;
  // the live rows as one byte range spread over gridDim.y workgroups per stream: 16-byte stores when
  // both bases are 16-byte aligned (the 8-byte tail of an odd row count last), 8-byte ones otherwise
  static_assert(sizeof(yk_track_out) % 8 == 0, "8-byte row copies");
  const size_t bytes = (size_t)n * sizeof(yk_track_out);
  const yk_track_out* src = g.rows + (size_t)s * T;
  yk_track_out* dst = rows + (size_t)s * T;
  const size_t i0 = (size_t)blockIdx.y * blockDim.x + threadIdx.x, step = (size_t)gridDim.y * blockDim.x;
  if ((((size_t)src | (size_t)dst) & 15) == 0) {
    const size_t n16 = bytes / 16;
    for (size_t i = i0; i < n16; i += step) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    if (bytes % 16 && i0 == 0) ((uint2*)dst)[2 * n16] = ((const uint2*)src)[2 * n16];
  } else {
    for (size_t i = i0; i < bytes / 8; i += step) ((uint2*)dst)[i] = ((const uint2*)src)[i];
  }
}

}  // namespace trk
}  // namespace yk

using yk::trk::Dev;

struct yk_tracker {
  yk_ctx* ctx;
  int S;
  yk_tracker_cfg cfg;
  Dev dev;
  size_t lds;
  size_t lds_assoc;
  bool split;  // assoc_kernel + tracks_kernel (else one workgroup per stream: YK_TRK_SINGLE=1 / LDS)
  yk_track_state* d_snap;
  yk_track_event* d_events;  // allocated by the first yk_tracker_set_events(1)
  yk_track_out* d_row1;
  double* d_box;  // [8]: in[4], out[4]
  int* d_status;
};

extern "C" {

int yk_tracker_create(yk_ctx* ctx, int n_streams, const yk_tracker_cfg* cfg, yk_tracker** out) {
  YK_CHECK_ARG(ctx && cfg && out, "yk_tracker_create: NULL argument");
  YK_CHECK_ARG(n_streams >= 1 && n_streams <= 65535, "yk_tracker_create: n_streams out of range");
  YK_CHECK_ARG(cfg->max_tracks >= 1 && cfg->max_tracks <= 2048, "yk_tracker_create: max_tracks must be in [1, 2048]");
  YK_CHECK_ARG(cfg->max_dets >= 1 && cfg->max_dets <= 1024, "yk_tracker_create: max_dets must be in [1, 1024]");
  YK_CHECK_ARG(cfg->max_lost_frames >= 0, "yk_tracker_create: max_lost_frames must be >= 0");
  YK_CHECK_ARG(cfg->policy == YK_POLICY_ENHANCED || cfg->policy == YK_POLICY_MOTION_RESET,
               "yk_tracker_create: unknown tracker policy");
  const size_t lds = yk::trk::lds_bytes(cfg->max_tracks, cfg->max_dets);
  YK_CHECK_ARG(yk::trk::stage_chunk(cfg->max_tracks, cfg->max_dets) >= 1 && lds <= 160 * 1024,
               "yk_tracker_create: max_tracks x max_dets exceed the 160 KiB LDS budget");
  yk::DeviceGuard guard(ctx->device);
  auto* t = new yk_tracker{};
  t->ctx = ctx;
  t->S = n_streams;
  t->cfg = *cfg;
  t->lds = lds;
  Dev& g = t->dev;
  g.T = cfg->max_tracks;
  g.D = cfg->max_dets;
  g.C = cfg->max_tracks * cfg->max_dets;
  g.max_lost = cfg->max_lost_frames;
  g.min_hits = cfg->min_hits;
  g.thr = cfg->iou_threshold;
  g.policy = cfg->policy;
  const size_t S = n_streams, T = g.T;
  hipError_t e = hipSuccess;
  auto A = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  A((void**)&g.slots, S * T * sizeof(yk::trk::Slot));
  A((void**)&g.hdr, S * sizeof(yk::trk::Hdr));
  A((void**)&g.order, S * T * sizeof(int));
  A((void**)&g.free_stack, S * T * sizeof(int));
  A((void**)&g.cand_key, S * (size_t)g.C * sizeof(unsigned long long));
  A((void**)&g.cand_flat, S * (size_t)g.C * sizeof(int));
  A((void**)&g.rows, S * T * sizeof(yk_track_out));
  if (e == hipSuccess) e = hipMemset(g.rows, 0, S * T * sizeof(yk_track_out));
  A((void**)&g.counts, S * sizeof(int));
  A((void**)&g.stats, S * sizeof(yk_tracker_stats));
  A((void**)&g.items, S * T * sizeof(int4));
  A((void**)&g.items_vh, S * T * sizeof(int2));
  A((void**)&g.n_items, S * sizeof(int));
  A((void**)&g.phase, S * yk::trk::PH * sizeof(long long));
  if (e == hipSuccess) e = hipMemset(g.phase, 0, S * yk::trk::PH * sizeof(long long));
  A((void**)&t->d_snap, T * sizeof(yk_track_state));
  A((void**)&t->d_row1, sizeof(yk_track_out));
  if (e == hipSuccess) e = hipMemset(t->d_row1, 0, sizeof(yk_track_out));
  A((void**)&t->d_box, 16 * sizeof(double));
  A((void**)&t->d_status, sizeof(int));
  if (e != hipSuccess) {
    yk::set_error(std::string("yk_tracker_create: hipMalloc failed: ") + hipGetErrorString(e));
    yk_tracker_destroy(t);
    return YK_ERR_HIP;
  }
  if (hipFuncSetAttribute((const void*)yk::trk::step_kernel<float, 0>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
      hipFuncSetAttribute((const void*)yk::trk::step_kernel<double, 0>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
      hipFuncSetAttribute((const void*)yk::trk::step_kernel<float, 1>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
      hipFuncSetAttribute((const void*)yk::trk::step_kernel<double, 1>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
  }
  // enhanced policy: the two-launch step unless its LDS does not fit or YK_TRK_SINGLE=1
  t->lds_assoc = yk::trk::assoc_lds_bytes(cfg->max_tracks, cfg->max_dets);
  if (t->lds_assoc <= yk::trk::LDS_CU)
    t->lds_assoc = ((t->lds_assoc + 7) & ~(size_t)7) + (size_t)yk::trk::assoc_lds_cand(cfg->max_tracks, cfg->max_dets, g.C) * 12;
  const char* single = getenv("YK_TRK_SINGLE");
  t->split = t->lds_assoc <= 160 * 1024 && !(single && single[0] == '1');
  if (t->split) {
    const int la = (int)t->lds_assoc, lt = (int)yk::trk::tracks_lds_bytes();
    const void* ka[] = {(const void*)yk::trk::assoc_kernel<float, 0>, (const void*)yk::trk::assoc_kernel<double, 0>,
                        (const void*)yk::trk::assoc_kernel<float, 1>, (const void*)yk::trk::assoc_kernel<double, 1>};
    const void* kt[] = {(const void*)yk::trk::tracks_kernel<float, 0>, (const void*)yk::trk::tracks_kernel<double, 0>,
                        (const void*)yk::trk::tracks_kernel<float, 1>, (const void*)yk::trk::tracks_kernel<double, 1>};
    for (int i = 0; i < 4; ++i)
      if (hipFuncSetAttribute(ka[i], hipFuncAttributeMaxDynamicSharedMemorySize, la) != hipSuccess ||
          hipFuncSetAttribute(kt[i], hipFuncAttributeMaxDynamicSharedMemorySize, lt) != hipSuccess)
        (void)hipGetLastError();
  }
  int rc = yk_tracker_reset(t, nullptr);
  if (rc != YK_OK) {
    yk_tracker_destroy(t);
    return rc;
  }
  YK_HIP(hipDeviceSynchronize());
  *out = t;
  return YK_OK;
}

int yk_tracker_destroy(yk_tracker* t) {
  if (!t) return YK_OK;
  yk::DeviceGuard guard(t->ctx->device);
  Dev& g = t->dev;
  void* ptrs[] = {g.slots, g.hdr, g.order, g.free_stack, g.cand_key, g.cand_flat, g.rows,
                  g.counts, g.stats, g.items, g.items_vh, g.n_items, g.phase, t->d_events, t->d_snap, t->d_row1,
                  t->d_box, t->d_status};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete t;
  return YK_OK;
}

int yk_tracker_reset(yk_tracker* t, void* stream) {
  YK_CHECK_ARG(t, "yk_tracker_reset: NULL tracker");
  yk::DeviceGuard guard(t->ctx->device);
  hipLaunchKernelGGL(yk::trk::reset_kernel, dim3(t->S), dim3(256), 0, (hipStream_t)stream, t->dev, t->S);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_tracker_step(yk_tracker* t, const void* dets, int dtype, int row_stride, const int32_t* counts,
                    void* stream) {
  return yk_tracker_step_motion(t, dets, dtype, row_stride, counts, nullptr, stream);
}

int yk_tracker_step_motion(yk_tracker* t, const void* dets, int dtype, int row_stride, const int32_t* counts,
                           const yk_motion* motion, void* stream) {
  YK_CHECK_ARG(t && dets && counts, "yk_tracker_step: NULL argument");
  YK_CHECK_ARG(!motion || t->cfg.policy == YK_POLICY_MOTION_RESET,
               "yk_tracker_step_motion: global camera-motion input needs the YK_POLICY_MOTION_RESET policy");
  YK_CHECK_ARG(row_stride >= 4, "yk_tracker_step: row_stride must be >= 4");
  YK_CHECK_ARG(dtype == YK_F32 || dtype == YK_F64, "yk_tracker_step: dtype must be YK_F32 or YK_F64");
  yk::DeviceGuard guard(t->ctx->device);
  const bool mr = t->cfg.policy == YK_POLICY_MOTION_RESET;
  if (t->split) {
    const dim3 g2((t->dev.T + yk::trk::IPB - 1) / yk::trk::IPB, t->S);
    const size_t l2 = yk::trk::tracks_lds_bytes();
    hipStream_t st = (hipStream_t)stream;
    const yk::trk::Dev& g = t->dev;
    if (dtype == YK_F32) {
      const float* d = (const float*)dets;
      if (mr) {
        hipLaunchKernelGGL((yk::trk::assoc_kernel<float, 1>), dim3(t->S), dim3(yk::trk::NTA), t->lds_assoc, st, g, d,
                           row_stride, counts, motion);
        hipLaunchKernelGGL((yk::trk::tracks_kernel<float, 1>), g2, dim3(yk::trk::NT), l2, st, g, d, row_stride);
      } else {
        hipLaunchKernelGGL((yk::trk::assoc_kernel<float, 0>), dim3(t->S), dim3(yk::trk::NTA), t->lds_assoc, st, g, d,
                           row_stride, counts, motion);
        hipLaunchKernelGGL((yk::trk::tracks_kernel<float, 0>), g2, dim3(yk::trk::NT), l2, st, g, d, row_stride);
      }
    } else {
      const double* d = (const double*)dets;
      if (mr) {
        hipLaunchKernelGGL((yk::trk::assoc_kernel<double, 1>), dim3(t->S), dim3(yk::trk::NTA), t->lds_assoc, st, g, d,
                           row_stride, counts, motion);
        hipLaunchKernelGGL((yk::trk::tracks_kernel<double, 1>), g2, dim3(yk::trk::NT), l2, st, g, d, row_stride);
      } else {
        hipLaunchKernelGGL((yk::trk::assoc_kernel<double, 0>), dim3(t->S), dim3(yk::trk::NTA), t->lds_assoc, st, g, d,
                           row_stride, counts, motion);
        hipLaunchKernelGGL((yk::trk::tracks_kernel<double, 0>), g2, dim3(yk::trk::NT), l2, st, g, d, row_stride);
      }
    }
    YK_HIP(hipGetLastError());
    return YK_OK;
  }
  if (dtype == YK_F32) {
    if (mr)
      hipLaunchKernelGGL((yk::trk::step_kernel<float, 1>), dim3(t->S), dim3(yk::trk::NT), t->lds,
                         (hipStream_t)stream, t->dev, (const float*)dets, row_stride, counts, motion);
    else
      hipLaunchKernelGGL((yk::trk::step_kernel<float, 0>), dim3(t->S), dim3(yk::trk::NT), t->lds,
                         (hipStream_t)stream, t->dev, (const float*)dets, row_stride, counts, motion);
  } else {
    if (mr)
      hipLaunchKernelGGL((yk::trk::step_kernel<double, 1>), dim3(t->S), dim3(yk::trk::NT), t->lds,
                         (hipStream_t)stream, t->dev, (const double*)dets, row_stride, counts, motion);
    else
      hipLaunchKernelGGL((yk::trk::step_kernel<double, 0>), dim3(t->S), dim3(yk::trk::NT), t->lds,
                         (hipStream_t)stream, t->dev, (const double*)dets, row_stride, counts, motion);
  }
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_tracker_outputs(yk_tracker* t, yk_track_out** rows, int32_t** counts, yk_tracker_stats** stats) {
  YK_CHECK_ARG(t, "yk_tracker_outputs: NULL tracker");
  if (rows) *rows = t->dev.rows;
  if (counts) *counts = t->dev.counts;
  if (stats) *stats = t->dev.stats;
  return YK_OK;
}

int yk_tracker_download(yk_tracker* t, yk_track_out* host_rows, int32_t* host_counts,
                        yk_tracker_stats* host_stats, void* stream) {
  YK_CHECK_ARG(t && host_counts, "yk_tracker_download: NULL argument");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  YK_HIP(hipMemcpyAsync(host_counts, t->dev.counts, t->S * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  if (host_stats)
    YK_HIP(hipMemcpyAsync(host_stats, t->dev.stats, t->S * sizeof(yk_tracker_stats),
                          hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  if (host_rows) {
    const size_t T = t->dev.T;
    for (int s = 0; s < t->S; ++s) {
      const int c = host_counts[s];
      if (c > 0)
        YK_HIP(hipMemcpyAsync(host_rows + s * T, t->dev.rows + s * T, c * sizeof(yk_track_out),
                              hipMemcpyDeviceToHost, st));
    }
    YK_HIP(hipStreamSynchronize(st));
  }
  return YK_OK;
}

int yk_tracker_download_async(yk_tracker* t, yk_track_out* host_rows, int32_t* host_counts,
                              yk_tracker_stats* host_stats, int rows_per_stream, void* stream) {
  YK_CHECK_ARG(t && host_counts, "yk_tracker_download_async: NULL argument");
  YK_CHECK_ARG(rows_per_stream >= 0 && rows_per_stream <= t->dev.T,
               "yk_tracker_download_async: rows_per_stream out of [0, max_tracks]");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  // the device writes the host buffers itself: they must be page-locked memory mapped into the
  // device's address space; the kernel gets the device-side address of each (never a raw host one)
  void* dp[3] = {nullptr, nullptr, nullptr};
  const void* hp[3] = {host_rows, host_counts, host_stats};
  for (int i = 0; i < 3; ++i) {
    if (!hp[i] || (i == 0 && rows_per_stream == 0)) continue;
    hipPointerAttribute_t at;
    const hipError_t e = hipPointerGetAttributes(&at, hp[i]);
    if (e != hipSuccess || at.type != hipMemoryTypeHost || !at.devicePointer) {
      (void)hipGetLastError();
      yk::set_error("yk_tracker_download_async: host buffers must be page-locked, device-mapped memory");
      return YK_ERR_ARG;
    }
    dp[i] = at.devicePointer;
  }
  hipLaunchKernelGGL(yk::trk::push_out_kernel, dim3(t->S, 8), dim3(256), 0, st, t->dev, t->S, t->dev.T,
                     rows_per_stream, (yk_track_out*)dp[0], (int32_t*)dp[1], (yk_tracker_stats*)dp[2]);
  YK_HIP(hipGetLastError());
  return YK_OK;
}

int yk_tracker_snapshot(yk_tracker* t, int s, yk_track_state* host_states, int32_t* n_out, void* stream) {
  YK_CHECK_ARG(t && host_states && n_out, "yk_tracker_snapshot: NULL argument");
  YK_CHECK_ARG(s >= 0 && s < t->S, "yk_tracker_snapshot: stream index out of range");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  yk::trk::Hdr h;
  YK_HIP(hipMemcpyAsync(&h, t->dev.hdr + s, sizeof(h), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  *n_out = h.n_tracks;
  if (h.n_tracks > 0) {
    hipLaunchKernelGGL(yk::trk::snapshot_kernel, dim3((h.n_tracks + 63) / 64), dim3(64), 0, st, t->dev, s,
                       t->d_snap);
    YK_HIP(hipGetLastError());
    YK_HIP(hipMemcpyAsync(host_states, t->d_snap, h.n_tracks * sizeof(yk_track_state),
                          hipMemcpyDeviceToHost, st));
    YK_HIP(hipStreamSynchronize(st));
  }
  return YK_OK;
}

int yk_track_op(yk_tracker* t, int s, int pos, int op, int arg, const double* in_box, int dtype, double* out5,
                yk_track_out* out_row, void* stream) {
  YK_CHECK_ARG(t, "yk_track_op: NULL tracker");
  YK_CHECK_ARG(s >= 0 && s < t->S, "yk_track_op: stream index out of range");
  YK_CHECK_ARG(op >= YK_OP_PREDICT && op <= YK_OP_LOST_PRED, "yk_track_op: unknown op");
  YK_CHECK_ARG(op != YK_OP_UPDATE || in_box, "yk_track_op: update needs a box");
  YK_CHECK_ARG(dtype == YK_F32 || dtype == YK_F64, "yk_track_op: bad dtype");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  yk::trk::Hdr h;
  YK_HIP(hipMemcpyAsync(&h, t->dev.hdr + s, sizeof(h), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  YK_CHECK_ARG(pos >= 0 && pos < h.n_tracks, "yk_track_op: track position out of range");
  if (in_box) YK_HIP(hipMemcpyAsync(t->d_box, in_box, 4 * sizeof(double), hipMemcpyHostToDevice, st));
  if (dtype == YK_F32)
    hipLaunchKernelGGL(yk::trk::track_op_kernel<float>, dim3(1), dim3(64), 0, st, t->dev, s, pos, op, arg,
                       t->d_box, t->d_box + 4, t->d_row1);
  else
    hipLaunchKernelGGL(yk::trk::track_op_kernel<double>, dim3(1), dim3(64), 0, st, t->dev, s, pos, op, arg,
                       t->d_box, t->d_box + 4, t->d_row1);
  YK_HIP(hipGetLastError());
  if (out5) YK_HIP(hipMemcpyAsync(out5, t->d_box + 4, 5 * sizeof(double), hipMemcpyDeviceToHost, st));
  if (out_row) YK_HIP(hipMemcpyAsync(out_row, t->d_row1, sizeof(yk_track_out), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

int yk_track_create(yk_tracker* t, int s, const double* box, int dtype, int32_t track_num, int32_t max_lost,
                    void* stream) {
  YK_CHECK_ARG(t && box, "yk_track_create: NULL argument");
  YK_CHECK_ARG(s >= 0 && s < t->S, "yk_track_create: stream index out of range");
  YK_CHECK_ARG(dtype == YK_F32 || dtype == YK_F64, "yk_track_create: bad dtype");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  YK_HIP(hipMemcpyAsync(t->d_box, box, 4 * sizeof(double), hipMemcpyHostToDevice, st));
  if (dtype == YK_F32)
    hipLaunchKernelGGL(yk::trk::track_create_kernel<float>, dim3(1), dim3(64), 0, st, t->dev, s, t->d_box,
                       track_num, max_lost, t->d_status);
  else
    hipLaunchKernelGGL(yk::trk::track_create_kernel<double>, dim3(1), dim3(64), 0, st, t->dev, s, t->d_box,
                       track_num, max_lost, t->d_status);
  YK_HIP(hipGetLastError());
  int status = 0;
  YK_HIP(hipMemcpyAsync(&status, t->d_status, sizeof(int), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  if (status != 0) {
    yk::set_error("yk_track_create: stream is at max_tracks capacity");
    return YK_ERR_CAPACITY;
  }
  return YK_OK;
}

int yk_tracker_set_events(yk_tracker* t, int enable) {
  YK_CHECK_ARG(t, "yk_tracker_set_events: NULL tracker");
  yk::DeviceGuard guard(t->ctx->device);
  if (!enable) {
    t->dev.events = nullptr;  // the buffer stays allocated for a later enable
    return YK_OK;
  }
  if (t->cfg.policy != YK_POLICY_ENHANCED || !t->split) {
    yk::set_error("yk_tracker_set_events: the event log is written by the enhanced policy's two-launch step only");
    return YK_ERR_STATE;
  }
  if (!t->d_events) {
    const size_t bytes = (size_t)t->S * t->dev.T * sizeof(yk_track_event);
    YK_HIP(hipMalloc((void**)&t->d_events, bytes));
    YK_HIP(hipMemset(t->d_events, 0, bytes));
    YK_HIP(hipDeviceSynchronize());
  }
  t->dev.events = t->d_events;
  return YK_OK;
}

int yk_tracker_events(yk_tracker* t, int s, yk_track_event* host_events, int32_t* n_out, void* stream) {
  YK_CHECK_ARG(t && host_events && n_out, "yk_tracker_events: NULL argument");
  YK_CHECK_ARG(s >= 0 && s < t->S, "yk_tracker_events: stream index out of range");
  if (!t->dev.events) {
    yk::set_error("yk_tracker_events: the event log is off (yk_tracker_set_events)");
    return YK_ERR_STATE;
  }
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  int n = 0;
  YK_HIP(hipMemcpyAsync(&n, t->dev.n_items + s, sizeof(int), hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  if (n < 0 || n > t->dev.T) n = 0;
  if (n > 0) {
    YK_HIP(hipMemcpyAsync(host_events, t->dev.events + (size_t)s * t->dev.T, n * sizeof(yk_track_event),
                          hipMemcpyDeviceToHost, st));
    YK_HIP(hipStreamSynchronize(st));
  }
  *n_out = n;
  return YK_OK;
}

int yk_tracker_phase_ticks(yk_tracker* t, int s, int64_t* host_ticks, void* stream) {
  YK_CHECK_ARG(t && host_ticks, "yk_tracker_phase_ticks: NULL argument");
  YK_CHECK_ARG(s >= 0 && s < t->S, "yk_tracker_phase_ticks: stream index out of range");
  yk::DeviceGuard guard(t->ctx->device);
  hipStream_t st = (hipStream_t)stream;
  YK_HIP(hipMemcpyAsync(host_ticks, t->dev.phase + (size_t)s * yk::trk::PH, yk::trk::PH * sizeof(long long),
                        hipMemcpyDeviceToHost, st));
  YK_HIP(hipStreamSynchronize(st));
  return YK_OK;
}

}  // extern "C"
