/*
 * yk.h — C ABI of the MI355X-native detect-and-track hot path (libyk.so).
 *
 * The reference has no FFI: its hot path is two Python surfaces,
 *   ultralytics.YOLO.__call__/predict        (ultralytics/engine/model.py:158-188, 498-557)
 *   kalman.EnhancedMultiTargetTracker.update (kalman/enhanced_multi_target_tracker.py:42-132)
 * driven per frame by kalman/aircraft_detection_tracking.py:88-131.  This header is the
 * boundary the two Python shims of this package (and any other host: cgo, JNI, ctypes)
 * bind.  Every entry point cites the reference interface it replaces.
 *
 * Conventions
 *   - every call returns an int status (YK_OK = 0); yk_last_error() returns a
 *     thread-local message for the last failing call on the calling thread.
 *   - pointers named dev_* are device (HBM) pointers; host_* are host pointers.
 *     Callers own host buffers; handles own their device buffers.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *     No call allocates or synchronises inside a *_step / yk_detect launch, so
 *     those calls are hipGraph-capturable.
 *   - a handle is bound to one GPU and is not re-entrant (mirrors the reference
 *     predictor's threading.Lock, ultralytics/engine/predictor.py:149,304).
 */
#ifndef YK_H_
#define YK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: yk_bt_cfg gained assignment / match_thresh_f64, yk_track_state the motion-reset fields
 * (round 3).  A host built against another layout must not call in: see yk_abi_check(). */
#define YK_ABI_VERSION 3

enum yk_status {
  YK_OK = 0,
  YK_ERR_ARG = 1,      /* bad argument (reference: assert / ValueError)                */
  YK_ERR_HIP = 2,      /* HIP runtime error                                           */
  YK_ERR_CAPACITY = 3, /* a fixed capacity (max_tracks, max_dets) was exceeded         */
  YK_ERR_STATE = 4     /* call out of order (e.g. detect before a model was loaded)     */
};

enum yk_dtype { YK_F32 = 0, YK_F64 = 1 };

typedef struct yk_ctx yk_ctx;
typedef struct yk_tracker yk_tracker;
typedef struct yk_model yk_model;

/* ------------------------------------------------------------------ common */
int yk_abi_version(void);
const char* yk_last_error(void);

/* Bind a context to GPU `device` (reference: select_device, ultralytics/utils/torch_utils.py:134-245). */
int yk_ctx_create(int device, yk_ctx** out);
int yk_ctx_destroy(yk_ctx* ctx);

/* ------------------------------------------------------------------ tracker
 * Replaces kalman.EnhancedMultiTargetTracker (kalman/enhanced_multi_target_tracker.py:15-40)
 * for `n_streams` independent video streams at once (one reference tracker object per stream).
 */
typedef struct {
  int32_t max_lost_frames; /* reference default 450 (driver uses 150)            */
  int32_t min_hits;        /* reference default 3   (driver uses 1)              */
  double iou_threshold;    /* reference default 0.3 (driver uses 0.1)            */
  int32_t max_tracks;      /* capacity of live tracks per stream (<= 2048)       */
  int32_t max_dets;        /* capacity of detections per stream per frame (<= 1024) */
  int32_t policy;          /* yk_tracker_policy                                   */
} yk_tracker_cfg;

/* Tracker policy (what update() a stream runs):
 *   YK_POLICY_ENHANCED      kalman.EnhancedMultiTargetTracker (enhanced_multi_target_tracker.py)
 *   YK_POLICY_MOTION_RESET  camera_motion_compensation.MotionCompensatedMultiTracker.update(dets,
 *                           frame=None) over MotionResetKalmanTracker tracks
 *                           (motion_compensated_multi_tracker.py:77-242,
 *                           motion_reset_kalman_tracker.py:16-355): jump / velocity / size-change
 *                           Kalman resets, blended predict for 10 frames after a reset, strict
 *                           iou > thr with (iou, d, t)-descending greedy order, every live
 *                           track reported.  The global-motion branch (needs frames + optical
 *                           flow) is not part of this policy. */
enum yk_tracker_policy { YK_POLICY_ENHANCED = 0, YK_POLICY_MOTION_RESET = 1 };

/* Per-stream counters: EnhancedMultiTargetTracker.stats + frame_count/next_track_id
 * (enhanced_multi_target_tracker.py:28-38). */
typedef struct {
  int64_t frame_count;
  int64_t next_track_id;
  int64_t total_tracks_created;
  int64_t total_tracks_terminated;
  int64_t current_active_tracks;
  int64_t long_term_predictions;
  int64_t successful_recoveries;
  int64_t overflow; /* detections/tracks dropped because a capacity was hit (0 in parity runs) */
  int64_t individual_resets;   /* YK_POLICY_MOTION_RESET: stats['individual_resets']   */
  int64_t tracking_recoveries; /* YK_POLICY_MOTION_RESET: stats['tracking_recoveries'] */
  int64_t global_motion_events;/* YK_POLICY_MOTION_RESET: stats['global_motion_events'] */
  int64_t global_resets;       /* YK_POLICY_MOTION_RESET: stats['global_resets']        */
} yk_tracker_stats;

/* One output row = one reference get_track_info() dict
 * (kalman/enhanced_aircraft_kalman_tracker.py:366-383). */
#define YK_TRAJ_OUT 30
typedef struct {
  int32_t track_num;          /* track_id = "T%03d" % track_num                    */
  int32_t status;             /* 0 = 'detected', 1 = 'predicted'                   */
  int32_t age, hits, hit_streak, time_since_update; /* lost_frames == time_since_update */
  int32_t traj_len;           /* number of valid points in traj (<= 30)            */
  int32_t is_stable_motion;   /* stability_score > 0.5                             */
  double bbox[4];             /* x1, y1, x2, y2                                    */
  double confidence;
  double velocity[2];         /* x[4:6]                                            */
  double motion_confidence, speed, direction;
  double traj[YK_TRAJ_OUT][2];/* last 30 trajectory centres, oldest first          */
  /* YK_POLICY_MOTION_RESET (motion_reset_kalman_tracker.py:314-355); zero otherwise */
  int32_t reset_count, frames_since_reset;
  int32_t reason_count[3];    /* resets with a position / velocity / size reason      */
  int32_t n_details;          /* entries of details (the last min(reset_count, 5))    */
  double motion_consistency;
  double reset_confidence_sum, motion_consistency_sum; /* over every reset (f64)   */
  struct {
    int32_t frame, reasons;   /* age at the reset; bit 0 position, 1 velocity, 2 size */
    double value[3];          /* jump px, velocity change px/f, size-change ratio     */
    double confidence, motion_consistency;
  } details[5];               /* oldest first                                         */
  int32_t traj_count;         /* trajectory points appended since the track's creation (a history
                               * reset adds 2^20): traj[] advanced by the difference since a
                               * previous row of the same track, so a host can reuse its points */
  int32_t reserved;           /* 0 (written, so a row's bytes are fully defined)                     */
} yk_track_out;

/* Full filter state of one live track (AircraftKalmanTracker attributes,
 * kalman/enhanced_aircraft_kalman_tracker.py:32-101).  P is stored densely here. */
#define YK_VEL_HIST 50
#define YK_TRAJ_HIST 150
typedef struct {
  int32_t track_num, age, hits, hit_streak, time_since_update, is_lost, lost_frames;
  int32_t vel_len, traj_len, max_lost_frames;
  double x[8];
  double P[64];
  double velocity_avg[2], velocity_std[2], direction, speed, stability_score, prediction_confidence;
  double vel_hist[YK_VEL_HIST][2];   /* oldest first */
  double traj_hist[YK_TRAJ_HIST][2]; /* oldest first */
  /* motion-reset policy (MotionResetKalmanTracker attributes, motion_reset_kalman_tracker.py:
   * 50-58); 0 / -999 / 0 for the enhanced policy */
  int32_t reset_count, last_reset_frame;
  double motion_consistency;
} yk_track_state;

int yk_tracker_create(yk_ctx* ctx, int n_streams, const yk_tracker_cfg* cfg, yk_tracker** out);
int yk_tracker_destroy(yk_tracker* trk);
/* Return every stream to the freshly-constructed state (frame_count 0, next id 1). */
int yk_tracker_reset(yk_tracker* trk, void* stream);

/* One EnhancedMultiTargetTracker.update() for every stream
 * (enhanced_multi_target_tracker.py:42-132): batched predict, IoU cost matrix, greedy
 * association, update / mark_as_lost / create / delete, get_track_info().
 *   dev_dets   : n_streams x max_dets rows of `row_stride` elements of `dtype`,
 *                each row [x1, y1, x2, y2, conf, ...]; YK_F32 reproduces the reference's
 *                np.float32 detections bit for bit, YK_F64 python-float detections.
 *   dev_counts : int32[n_streams] detections per stream (clamped to max_dets; the
 *                excess is counted in stats.overflow).
 * Results stay on the device (yk_tracker_outputs) until yk_tracker_download. */
int yk_tracker_step(yk_tracker* trk, const void* dev_dets, int dtype, int row_stride,
                    const int32_t* dev_counts, void* stream);

/* Device views of the last step's results: rows[n_streams][max_tracks], counts[n_streams],
 * stats[n_streams].  Valid until the next step. */
int yk_tracker_outputs(yk_tracker* trk, yk_track_out** dev_rows, int32_t** dev_counts,
                       yk_tracker_stats** dev_stats);

/* Copy results to the host: counts and stats for every stream, then the live rows of
 * each stream into host_rows[s * max_tracks ...].  Synchronises `stream`. */
int yk_tracker_download(yk_tracker* trk, yk_track_out* host_rows, int32_t* host_counts,
                        yk_tracker_stats* host_stats, void* stream);

/* Enqueue the same transfer without waiting: one kernel on `stream` writes counts, stats and the
 * live rows of every stream (at most `rows_per_stream` of them; host_rows[s * max_tracks ...])
 * straight into the page-locked host buffers (YK_ERR_ARG for pageable memory).  Nothing is
 * synchronised: the host reads them after an event / stream sync of its own.  The per-step
 * "tracker output to the host" of a pipelined loop (bench.py). */
int yk_tracker_download_async(yk_tracker* trk, yk_track_out* host_rows, int32_t* host_counts,
                              yk_tracker_stats* host_stats, int rows_per_stream, void* stream);

/* Profiling: 32 words of stream s's last step (host_ticks holds 32).  wall_clock64 (100 MHz)
 * timestamps at the phase boundaries -- single-workgroup step: [0] start, [1] predict, [2] IoU
 * candidates, [3] greedy rounds, [4] update / mark_lost, [5] new tracks, [6] delete, [7] outputs;
 * two-launch enhanced step: [0]-[4] the association kernel (boxes, candidates, rounds, decisions),
 * [5]/[8]/[9]/[6] the first per-track workgroup (start, staged, computed, end); [10] association
 * rounds used; [11]-[15] candidate-index counters and the association kernel's shader cycles;
 * [16]-[19] shader cycles of the per-track waves (update / lost / new paths). */
int yk_tracker_phase_ticks(yk_tracker* trk, int stream_index, int64_t* host_ticks, void* stream);

/* Per-step event log of the enhanced policy: what the reference prints inside update()
 * (enhanced_multi_target_tracker.py:79,89,101,109; enhanced_aircraft_kalman_tracker.py:271,313).
 * One record per work item of the step: the tracks in list order at the start of the step
 * (list_pos 0..n-1), then the tracks created this step (list_pos n..). */
enum yk_track_event_kind { YK_EV_NONE = 0, YK_EV_RECOVERED = 1, YK_EV_LOST = 2, YK_EV_CREATED = 3 };
typedef struct {
  int32_t kind;        /* yk_track_event_kind: matched while lost / newly unmatched / new track  */
  int32_t track_num;
  int32_t list_pos;    /* position in the step's list (existing tracks first, then new ones)     */
  int32_t det;         /* matched or source detection, -1 for an unmatched track                 */
  int32_t lost_frames; /* YK_EV_RECOVERED: lost_frames before the update ("lost for N frames")    */
  int32_t deleted_tsu; /* >= 0: removed at the end of the step with this time_since_update, else -1 */
  double iou;          /* YK_EV_RECOVERED: IoU of the matched pair (the greedy match order key)  */
  double x, y, vx, vy; /* YK_EV_LOST: state after predict (lost_start_state[:2], [4:6])         */
  double confidence;   /* YK_EV_LOST: motion_analysis['prediction_confidence']                  */
} yk_track_event;

/* Turn the event log on (1) or off (0, the default: the step writes nothing extra).  Enhanced
 * policy on the two-launch step only (YK_ERR_STATE otherwise). */
int yk_tracker_set_events(yk_tracker* trk, int enable);

/* The last step's events of one stream (synchronises `stream`): host_events must hold max_tracks
 * records; *n_out receives the number of work items (every record up to it is valid, kind
 * YK_EV_NONE for a track with no event). */
int yk_tracker_events(yk_tracker* trk, int stream_index, yk_track_event* host_events, int32_t* n_out,
                      void* stream);

/* Snapshot the live tracks of one stream in list order (EnhancedMultiTargetTracker.trackers).
 * host_states must hold max_tracks entries; *n_out receives the number written. */
int yk_tracker_snapshot(yk_tracker* trk, int stream_index, yk_track_state* host_states,
                        int32_t* n_out, void* stream);

/* Device-side single-track operations on list position `pos` of stream `stream_index`,
 * for the AircraftKalmanTracker object surface (kalman/enhanced_aircraft_kalman_tracker.py):
 *   YK_OP_PREDICT      predict()                        (:184-203)  out5 <- box
 *   YK_OP_UPDATE       update(in_box)                   (:249-297)  in_box dtype as in step
 *   YK_OP_MARK_LOST    mark_as_lost()                   (:299-317)
 *   YK_OP_INFO         get_track_info()                 (:335-383)  row_out (may predict: quirk A)
 *   YK_OP_LONG_TERM    enhanced_long_term_predict(arg)  (:205-247)  out5 <- box, confidence
 *   YK_OP_LOST_PRED    get_lost_prediction()            (:319-333)  out5 <- box, confidence
 * host_in_box / host_out5 / host_row_out may be NULL when unused.  Synchronous. */
enum yk_track_op_code {
  YK_OP_PREDICT = 0,
  YK_OP_UPDATE = 1,
  YK_OP_MARK_LOST = 2,
  YK_OP_INFO = 3,
  YK_OP_LONG_TERM = 4,
  YK_OP_LOST_PRED = 5
};
int yk_track_op(yk_tracker* trk, int stream_index, int pos, int op, int arg, const double* host_in_box,
                int dtype, double* host_out5, yk_track_out* host_row_out, void* stream);

/* sizeof() of the ABI structs, for bindings that mirror them (0: yk_tracker_cfg,
 * 1: yk_tracker_stats, 2: yk_track_out, 3: yk_track_state, 4: yk_view, 5: yk_op,
 * 6: yk_model_desc, 7: yk_bt_cfg, 8: yk_motion, 9: yk_gmd_stats, 10: yk_tensor,
 * 11: yk_track_event); -1 for an unknown id. */
int64_t yk_struct_size(int which);

/* Append a new track created from a box (AircraftKalmanTracker.__init__, :23-101) to the
 * end of stream `stream_index`'s list, with the given track number. Synchronous. */
int yk_track_create(yk_tracker* trk, int stream_index, const double* host_bbox, int dtype,
                    int32_t track_num, int32_t max_lost_frames, void* stream);


/* ------------------------------------------------------------------ global camera motion
 * Replaces GlobalMotionDetector(method='optical_flow').detect_motion(frame)
 * (camera_motion_compensation/global_motion_detector.py:67-169, 241-261) for n_streams video
 * streams at once: BGR->gray, goodFeaturesToTrack(maxCorners 200, quality 0.01, minDistance 15,
 * blockSize 7) on the previous frame, pyramidal Lucas-Kanade (21x21 window, 3 levels, 30
 * iterations / eps 0.01) into the current one, then the reference's median / 75th-percentile
 * inlier mean, magnitude thresholds and 3-vector direction consistency.  The OpenCV stages
 * follow OpenCV 4.x's published algorithms (cv2 is not available to pin them).
 * 'feature_matching' and 'hybrid' (ORB + RANSAC homography) are not built.
 * YK_GMD_SPARSE_OPTFLOW is BoT-SORT's default global motion compensation instead
 * (ultralytics/trackers/utils/gmc.py:278-345, GMC(method='sparseOptFlow', downscale=2)): gray,
 * the 1/2 area downscale, goodFeaturesToTrack(1000, 0.01, 1, blockSize 3), calcOpticalFlowPyrLK
 * (21x21, maxLevel 3) from the previous frame's corners, then estimateAffinePartial2D(RANSAC) with
 * its Levenberg-Marquardt refinement; the result is a 2x3 warp per stream (yk_gmc_apply), not a
 * yk_motion.  Frames must have even width and height. */
enum yk_gmd_method { YK_GMD_OPTICAL_FLOW = 0, YK_GMD_FEATURE_MATCHING = 1, YK_GMD_HYBRID = 2,
                     YK_GMD_SPARSE_OPTFLOW = 3 };
/* One detect_motion() result (is_motion, motion_magnitude, motion_vector, should_reset). */
typedef struct {
  int32_t valid;           /* 1: the stream had a frame this step                            */
  int32_t is_motion, should_reset;
  int32_t magnitude_kind;  /* 0: the python-float 0.0 of the no-estimate returns, 1: float32  */
  float magnitude;
  float vector[2];         /* global motion vector (x, y), pixels per frame                  */
  float consistency;       /* _calculate_motion_consistency of the last 3 vectors, -1: none   */
  int32_t n_corners, n_tracked, n_inliers; /* diagnostics: corners, LK status==1, inliers     */
  int32_t first_frame;     /* 1: no previous frame yet (the detector only stored this one)   */
} yk_motion;
/* GlobalMotionDetector.stats (:58-63) */
typedef struct {
  int64_t total_detections, motion_events, reset_triggers;
  float avg_motion_magnitude;
  int32_t pad;
} yk_gmd_stats;
typedef struct yk_gmd yk_gmd;
/* Frames are height x width x 3 uint8 BGR (the decoder's / the detector's input buffer). */
int yk_gmd_create(yk_ctx* ctx, int n_streams, int height, int width, int method, yk_gmd** out);
int yk_gmd_destroy(yk_gmd* g);
/* A fresh detector for every stream (no previous frame, zero stats, empty histories). */
int yk_gmd_reset(yk_gmd* g, void* stream);
/* GlobalMotionDetector.reset_stats() (:280-288) of every stream. */
int yk_gmd_reset_stats(yk_gmd* g, void* stream);
/* global_motion_threshold / reset_motion_threshold (:38-39; set_global_motion_sensitivity,
 * motion_compensated_multi_tracker.py:353-360, divides both).  Compared in float32 like the
 * reference's float32 magnitudes. */
int yk_gmd_set_thresholds(yk_gmd* g, double global_motion_threshold, double reset_motion_threshold);
/* detect_motion() on frame s of dev_frames ([n_streams][height][width][3] uint8) for every
 * stream; results in dev_motion[n_streams] (device memory; NULL: the detector's own buffer,
 * see yk_gmd_outputs, which holds the last call's results either way).  Asynchronous on
 * `stream`. */
int yk_gmd_detect(yk_gmd* g, const uint8_t* dev_frames, yk_motion* dev_motion, void* stream);
/* n consecutive detect_motion() calls in one launch sequence: dev_frames[i] (host array of n
 * device pointers, each [n_streams][height][width][3] uint8) is step i's frame of every stream;
 * dev_motion[n][n_streams] receives the n records in frame order (NULL: a buffer of the
 * detector's own), bit for bit the n yk_gmd_detect calls' (the n frame pairs' corners and flow
 * run as n * n_streams independent problems, the post-processing steps each stream's state in
 * order).  A detector keeps its previous frame in one of two layouts: once either entry point has
 * run, the other refuses until yk_gmd_reset.  Asynchronous on `stream`. */
int yk_gmd_detect_window(yk_gmd* g, const uint8_t* const* dev_frames, int n, yk_motion* dev_motion, void* stream);
int yk_gmd_outputs(yk_gmd* g, yk_motion** dev_motion);
/* Copy the last results (and stats when host_stats != NULL) to the host; synchronous. */
int yk_gmd_download(yk_gmd* g, yk_motion* host_motion, yk_gmd_stats* host_stats, void* stream);
/* Diagnostics for parity tests: stream s's last corners (x, y), LK end points (x, y) and status
 * (host arrays of 200 entries, 1000 for YK_GMD_SPARSE_OPTFLOW); *n receives the corner count.
 * Synchronous. */
int yk_gmd_points(yk_gmd* g, int stream_index, float* host_corners, float* host_next, uint8_t* host_status,
                  int32_t* n, void* stream);

/* GMC.apply(frame) of a YK_GMD_SPARSE_OPTFLOW detector for every stream: dev_warp[n_streams][2][3]
 * float64 (device; NULL: the detector's own buffer, yk_gmc_outputs).  The first frame of a
 * stream, or one whose previous frame had no corners, gives the identity and stores the frame;
 * <= 4 tracked points give the identity; a failed estimate gives the identity and keeps the
 * previous frame (the reference's exception path, byte_tracker.py:334-338).  Asynchronous. */
int yk_gmc_apply(yk_gmd* g, const uint8_t* dev_frames, double* dev_warp, void* stream);
int yk_gmc_outputs(yk_gmd* g, double** dev_warp);
/* Per-stream diagnostics of the last yk_gmc_apply: {tracked points, RANSAC inliers, RANSAC
 * iterations, LM iterations, state (0 identity / first frame, 1 estimated, 2 too few points,
 * 3 failed)} x n_streams int32 (host).  Synchronous. */
int yk_gmc_info(yk_gmd* g, int32_t* host_info, void* stream);

/* MotionCompensatedMultiTracker.update(detections, frame) (motion_compensated_multi_tracker.py
 * :75-121): yk_tracker_step of a YK_POLICY_MOTION_RESET tracker plus the global branch --
 * global_motion_history / detection_stability_history, _should_global_reset (:123-148) and
 * _perform_global_reset (:150-169: every tracker dropped, one new tracker per detection) --
 * driven by dev_motion[n_streams] (yk_gmd_detect's output; a stream with valid == 0 had no
 * frame).  dev_motion == NULL is yk_tracker_step. */
int yk_tracker_step_motion(yk_tracker* trk, const void* dev_dets, int dtype, int row_stride,
                           const int32_t* dev_counts, const yk_motion* dev_motion, void* stream);

/* ------------------------------------------------------------------ ByteTrack / BoT-SORT
 * Replaces the upstream model.track() trackers for this path:
 * BYTETracker.update (ultralytics/trackers/byte_tracker.py:299-410) and BOTSORT.update without
 * ReID / GMC (trackers/bot_sort.py:156-249), KalmanFilterXYAH / XYWH (trackers/utils/
 * kalman_filter.py), matching.iou_distance / fuse_score / linear_assignment (trackers/utils/
 * matching.py:20-157, scipy branch).  One tracker object holds n_streams independent trackers
 * that share one track-id counter (BaseTrack._count, basetrack.py:67-92): each step, stream 0's
 * new tracks get ids first, then stream 1's, ...  Thresholds compare in float32 like the
 * reference's float32 scores. */
enum yk_bt_kind { YK_BT_BYTETRACK = 0, YK_BT_BOTSORT = 1 };
typedef struct yk_bt_cfg {
  int32_t kind;              /* yk_bt_kind (cfg tracker_type)                           */
  float track_high_thresh;   /* bytetrack.yaml / botsort.yaml defaults: 0.25           */
  float track_low_thresh;    /* 0.1                                                    */
  float new_track_thresh;    /* 0.25                                                   */
  float match_thresh;        /* 0.8                                                    */
  int32_t track_buffer;      /* 30; max_time_lost = int(frame_rate / 30 * track_buffer) */
  int32_t frame_rate;        /* 30                                                     */
  int32_t fuse_score;        /* 1                                                      */
  int32_t max_tracks;        /* tracked + lost tracks per stream (<= 1024)             */
  int32_t max_dets;          /* detections per stream and frame (<= 1024)              */
  int32_t assignment;        /* yk_bt_assignment: matching.linear_assignment's branch   */
  int32_t reserved;          /* 0                                                      */
  double match_thresh_f64;   /* match_thresh as the python float the YAML holds (the lap
                                branch's cost_limit is float64); 0 = (double)match_thresh */
} yk_bt_cfg;
/* matching.linear_assignment (trackers/utils/matching.py:20-61): YK_BT_LAP = lap.lapjv(cost,
 * extend_cost=True, cost_limit=thresh), the reference's default (use_lap=True; `lap` is a hard
 * requirement, :9-17): the maximum-weight matching with weights thresh - cost over pairs with
 * cost < thresh, unmatched lists ascending.  YK_BT_SCIPY = the scipy branch (:50-59): optimal
 * assignment of the whole matrix, then cost <= thresh, unmatched lists in frozenset order. */
enum yk_bt_assignment { YK_BT_LAP = 0, YK_BT_SCIPY = 1 };
typedef struct yk_bt yk_bt;
int yk_bt_create(yk_ctx* ctx, int n_streams, const yk_bt_cfg* cfg, yk_bt** out);
int yk_bt_destroy(yk_bt* bt);
/* BYTETracker.reset() of every stream, the shared id counter included (reset_id). */
int yk_bt_reset(yk_bt* bt, void* stream);
/* One update() of every stream.  dev_dets: [n_streams][max_dets][6] float32 rows x1 y1 x2 y2
 * conf cls (Boxes.data), dev_counts: [n_streams] rows used.  Asynchronous on `stream`. */
int yk_bt_step(yk_bt* bt, const float* dev_dets, const int32_t* dev_counts, void* stream);
/* yk_bt_step of a BoT-SORT tracker with its GMC: dev_warp[n_streams][2][3] float64 (yk_gmc_apply's
 * output for the same frames) is applied to strack_pool and the unconfirmed tracks after the
 * prediction (byte_tracker.py:333-340, STrack.multi_gmc :108-125); the covariances then become
 * dense 8x8 (tracked to rounding against numpy's BLAS, not bit for bit).  NULL: yk_bt_step. */
int yk_bt_step_warp(yk_bt* bt, const float* dev_dets, const int32_t* dev_counts, const double* dev_warp,
                    void* stream);
/* Device outputs of the last step: rows [n_streams][max_tracks][8] float32 = the reference's
 * result rows (x1 y1 x2 y2 track_id score cls idx) in tracked_stracks order; counts [n_streams]. */
int yk_bt_outputs(yk_bt* bt, float** dev_rows, int32_t** dev_counts);
/* Copy counts (and rows when host_rows != NULL) to the host; synchronises `stream`. */
int yk_bt_download(yk_bt* bt, float* host_rows, int32_t* host_counts, void* stream);

/* ------------------------------------------------------------------ detector
 * Replaces YOLO.predict() for the detection models this path uses
 * (ultralytics/engine/model.py:498-557 -> engine/predictor.py:152-387): LetterBox +
 * BGR->RGB + /255, the conv graph (nn/tasks.py:159-188), Detect decode (nn/modules/head.py
 * :116-187), non_max_suppression + TorchNMS.nms (utils/nms.py:13-304) and scale/clip
 * (utils/ops.py:105-184).  The host builds the program (parse_model rules + weight
 * packing, see arch.py / model.py); the library executes it.
 */
/* FP8: OCP e4m3 activations + weights; F16: IEEE binary16 (predict(half=True), nn/autobackend.py:215) */
enum yk_act_dtype { YK_ACT_BF16 = 0, YK_ACT_F32 = 1, YK_ACT_FP8 = 2, YK_ACT_F16 = 3 };
enum yk_op_kind {
  YK_K_CONV_INPUT = 0, /* first conv, reads uint8 BGR frames (fused letterbox/RGB//255)    */
  YK_K_CONV = 1,       /* implicit-GEMM conv (+bias, SiLU, residual, concat/upsample read)   */
  YK_K_SPPF_POOL = 2,  /* SPPF's three chained 5x5 max-pools, written as concat slices     */
  YK_K_DETECT = 3      /* Detect level: box/cls 1x1 + DFL + dist2bbox + sigmoid + threshold  */
};

typedef struct {
  int32_t buf;      /* activation buffer index                                  */
  int32_t c_off;    /* first channel of the view inside a pixel                 */
  int32_t c_stride; /* channels per pixel of the buffer                         */
  int32_t h, w;     /* stored spatial size                                      */
  int32_t up;       /* log2 nearest-upsample factor applied on read (0 or 1)    */
} yk_view;

typedef struct {
  int32_t kind;
  int32_t ksize, stride, act; /* act: 0 none, 1 SiLU                                   */
  int32_t n_src;
  yk_view src[2];
  int32_t src_ch[2];          /* physical channels of each source (multiples of 8; FP8 16) */
  yk_view dst;
  int32_t cout;               /* physical output channels written                      */
  int32_t has_res;
  yk_view res;                /* residual added after the activation (Bottleneck add)  */
  int32_t out_h, out_w;
  int32_t k_steps, n_tiles;   /* packed weights: [n_tiles][k_steps][64 lanes][16 B]    */
  int64_t w_off, b_off, t_off;/* blob offsets: packed weights, f32 bias (FP8: then f32 per-  *
                               * channel dequant scales), int32 K-chunk table             */
  /* YK_K_DETECT */
  int32_t det_stride;         /* level stride in input pixels                           */
  int32_t det_anchor_off;     /* index of this level's first anchor                     */
  int32_t det_cls_off;        /* channel offset of the class features in src[0]         */
  int32_t det_cls_ch;         /* class feature channels (physical)                      */
  int64_t det_wc_off;         /* f32 [det_cls_ch] class 1x1 weights, then f32 bias      */
} yk_op;

typedef struct {
  int32_t act_dtype;          /* yk_act_dtype                                           */
  int32_t max_batch;
  int32_t frame_h, frame_w;   /* original frame size, uint8 BGR HWC                      */
  int32_t in_h, in_w;         /* letterboxed network input size                          */
  int32_t pad_top, pad_left;  /* frame placement inside the input (LetterBox centring)  */
  int32_t n_anchors, nc, max_det;
  int32_t n_bufs;
  const int64_t* buf_elems;   /* per-image element count of each activation buffer       */
  int32_t n_ops;
  const yk_op* ops;
  /* LetterBox resize (data/augment.py:1717-1719, cv2.resize INTER_LINEAR) when the frame is not
   * at the network scale: 0 none, 1 bilinear (fixed-point), 2 exact 2x (INTER_AREA fast path).
   * The resized rs_w x rs_h image sits at (pad_left, pad_top) of the in_w x in_h input. */
  int32_t rs_mode, rs_w, rs_h;
  int32_t box_pad_x, box_pad_y; /* scale_boxes (utils/ops.py:123-126) padding and gain        */
  float box_gain;
  int64_t rs_tab_off;         /* blob: int32 xofs[rs_w], yofs[rs_h], then int16 pairs xw[rs_w][2], yw[rs_h][2] */
} yk_model_desc;

int yk_model_create(yk_ctx* ctx, const yk_model_desc* desc, const void* host_blob, int64_t blob_bytes,
                    yk_model** out);
int yk_model_destroy(yk_model* m);

/* Load a packed detector program ("engine" file) and create the model from it: what a C / Go /
 * Java host calls instead of building the program in Python.  The file is written once by
 * model.Program.export_engine (tools/export_engine.py: from an ultralytics checkpoint or a
 * state dict + the model YAML, for one frame size / dtype / max_batch, optionally with a tuned
 * conv plan).  Layout, little-endian: "YKENGINE", int32 version (1), sizeof(yk_model_desc),
 * sizeof(yk_op), n_bufs, n_ops, plan_batch, n_plan, pad, int64 blob_bytes; the yk_model_desc
 * (pointer fields ignored); int64 buf_elems[n_bufs]; yk_op ops[n_ops]; the blob; int32
 * plan[n_plan][4] = {op, kind, nnt, npt} applied with yk_model_set_plan at plan_batch. */
int yk_model_load(yk_ctx* ctx, const char* path, yk_model** out);

/* The detector program built by the library itself from a raw fp32 state dict: what
 * DetectionModel(yaml) + load_state_dict + fuse() do before predict (nn/tasks.py:1524-1700
 * parse_model channel / repeat rules of the yolov8-small P2 topology at `scale`, Conv+BN fold
 * with eps 1e-3, utils/torch_utils.py:255-286), then the lowering and weight packing of
 * model.py Program -- byte-identical to it -- for one frame size, imgsz, dtype and max_batch.
 * Host-only (no device call).  A tensor is named as in the state dict
 * ("model.2.m.0.cv1.conv.weight", "model.25.cv3.0.2.bias", ...), fp32, C-contiguous; nc is read
 * from model.25.cv3.0.2.weight.  yk_program_get's pointers stay valid until
 * yk_program_destroy. */
typedef struct {
  const char* name;
  int32_t ndim;
  int64_t shape[4];
  const float* data;
} yk_tensor;
typedef struct {
  int32_t n;
  const yk_tensor* tensors;
} yk_weights;
typedef struct yk_program yk_program;
int yk_program_build(const yk_weights* weights, char scale, int act_dtype, int frame_h, int frame_w, int imgsz,
                     int max_batch, int max_det, yk_program** out);
int yk_program_get(const yk_program* p, const yk_model_desc** desc, const void** blob, int64_t* blob_bytes);
int yk_program_destroy(yk_program* p);
/* yk_program_build (max_det 300, predict's default) + yk_model_create: the self-contained C-ABI
 * model load; examples/c_host.c shows it from a raw state-dict file. */
int yk_model_load_weights(yk_ctx* ctx, const yk_weights* weights, char scale, int act_dtype, int frame_h, int frame_w,
                          int imgsz, int max_batch, yk_model** out);

/* One predict() over `batch` frames resident in HBM (dev_frames: batch x frame_h x frame_w x 3
 * uint8 BGR).  Writes dev_dets[batch][max_det][6] = x1,y1,x2,y2,conf,cls (original-image pixels,
 * like Results.boxes.data) and dev_counts[batch].  NULL outputs use the model's own buffers
 * (yk_model_outputs).  conf/iou as in non_max_suppression (asserted in [0,1]). */
int yk_detect(yk_model* m, const uint8_t* dev_frames, int batch, float conf, float iou, int max_det,
              float* dev_dets, int32_t* dev_counts, void* stream);

/* Capture yk_detect for a fixed (batch, conf, iou, max_det, frames, outputs) into a hipGraph
 * and replay it: one graph launch per call (created on first use, cached per batch). */
int yk_detect_graph(yk_model* m, const uint8_t* dev_frames, int batch, float conf, float iou, int max_det,
                    float* dev_dets, int32_t* dev_counts, void* stream);

int yk_model_outputs(yk_model* m, float** dev_dets, int32_t** dev_counts);

/* The driver's frame in host memory -> HBM (cv2.VideoCapture.read() then model(frame),
 * kalman/aircraft_detection_tracking.py:96-100): copy `bytes` (a multiple of 16) of page-locked
 * host memory (hipHostMalloc / torch pin_memory; checked) to device memory with a kernel that
 * reads the host pages directly, on `stream`, without a host wait.  For frames below a few MiB:
 * the runtime copies small page-locked H2D transfers through the CPU synchronously (one
 * 640x512 frame held the host ~170 us), this call costs one launch; large transfers are as fast
 * through hipMemcpyAsync's DMA engine. */
int yk_upload_pinned_async(void* dev_dst, const void* host_src, size_t bytes, void* stream);

/* Pre-NMS candidates of the last yk_detect: [max_batch][n_anchors] rows of
 * {x1, y1, x2, y2, score, anchor_index (int32 bits)} in network-input pixels, unordered,
 * counts per image (parity harnesses compare them to the oracle's Detect output). */
int yk_model_candidates(yk_model* m, float** dev_cand, int32_t** dev_counts);

/* TorchNMS.nms + non_max_suppression's max_nms / max_det cut + scale_boxes / clip_boxes
 * (ultralytics/utils/nms.py:13-167, 237-304 incl. the :291-296 early exit; utils/ops.py:105-184)
 * on GIVEN boxes, through the same nms_kernel yk_detect runs after Detect.  dev_rows:
 * [batch][max_rows][row_stride] float32 rows {x1, y1, x2, y2, score, ...} in network-input
 * pixels, dev_counts: [batch] rows used.  Order among equal scores = input order (a stable sort).
 * dets / counts as yk_detect (NULL = the model's own buffers); keep (optional, [batch][max_det]):
 * the input row index of every output row.  max_rows <= n_anchors of the model.  Asynchronous. */
int yk_nms(yk_model* m, const float* dev_rows, int row_stride, int max_rows, const int32_t* dev_counts, int batch,
           float iou, int max_det, float* dets, int32_t* counts, int32_t* keep, void* stream);
/* The NMS stage alone on the model's current candidate buffers (yk_model_candidates): keep
 * gets each output row's candidate id (the anchor field). */
int yk_nms_candidates(yk_model* m, int batch, float iou, int max_det, float* dets, int32_t* counts, int32_t* keep,
                      void* stream);
/* NMS counters since the last reset: out[0] = images whose greedy loop took the :291-296 early
 * exit (no overlap with the kept box, every remaining box kept) with boxes left, out[1] = images
 * processed.  Synchronises `stream`. */
int yk_model_nms_stats(yk_model* m, int64_t* out, int reset, void* stream);
/* Synchronise `stream`, then report a device-side error flagged by an earlier launch (NMS met a
 * candidate row whose anchor index lies outside [0, n_anchors): that image's detections are
 * dropped) as YK_ERR_STATE; yk_detect / yk_detect_graph / yk_nms report it on their next call
 * without synchronising. */
int yk_model_check(yk_model* m, void* stream);

/* Per-op device time: launches every op of the program `reps` times back to back between two
 * hipEvents on `stream` and writes the average milliseconds per launch to host_ms[op]
 * (host_ms[n_ops] = the NMS kernel).  Outputs of the call are not meaningful. */
int yk_model_profile(yk_model* m, const uint8_t* dev_frames, int batch, float conf, float iou, int max_det,
                     int reps, float* host_ms, void* stream);

/* Kernel instantiation launched by op `op_index` (n_ops -> the NMS kernel), as rocprofv3
 * names it (substring of the demangled name). */
int yk_model_op_kernel(yk_model* m, int op_index, char* buf, int len);

/* Concurrency of the op program: ops are list-scheduled onto `lanes` HIP streams (1..8,
 * default 3; lane 0 is the caller's stream) with an event edge for every cross-lane buffer
 * hazard (RAW/WAR/WAW), so independent branches of the graph -- e.g. the P2 head/Detect branch
 * and the P3-P5 path after nn/tasks.py layer 15 -- overlap; yk_detect_graph captures that as
 * parallel graph branches.  Invalidates cached graphs.  No reference counterpart (the
 * reference runs nn.Module layers sequentially, nn/tasks.py:159-188). */
int yk_model_set_lanes(yk_model* m, int lanes);
/* Batch groups x lanes: the batch is cut into `groups` sub-batches (sizes differ by at most
 * one), each an independent copy of the op DAG on its own `lanes` streams, so the groups'
 * latency-bound kernel chains overlap.  groups * lanes <= 16.  Invalidates cached graphs. */
int yk_model_set_schedule(yk_model* m, int groups, int lanes);
/* Time every applicable conv kernel variant (direct, LDS-tiled, split-K x fragment tiles) for
 * each conv op on `dev_frames` (`reps` launches each, best of 3) at the batch one schedule group
 * runs (ceil(batch / groups)) and keep the fastest; later calls at that batch use the choice.  Each variant computes the same conv (fp32: the same
 * to summation order).  Invalidates cached graphs.  No reference counterpart. */
int yk_model_autotune(yk_model* m, const uint8_t* dev_frames, int batch, float conf, int reps, void* stream);
/* Force the conv kernel of one op (op_index >= 0) or of every conv op (-1) at `batch`:
 * kind -1 = heuristic, 0 = direct, 1 = LDS-tiled (falls back to direct where the tile does not
 * fit), 2 = split-K with an nnt x npt fragment tile (nnt, npt in {1, 2, 4}). */
int yk_model_set_plan(yk_model* m, int op_index, int batch, int kind, int nnt, int npt);
/* The current per-op conv plan (n_ops x {kind, nnt, npt}; kind -1 = heuristic) and the batch
 * it was tuned for (0 if none): with yk_model_set_plan, replays an autotune without re-running
 * it (e.g. under a profiler). */
int yk_model_get_plan(yk_model* m, int32_t* plan, int32_t* batch);
/* The schedule: per task (op-major: task = op * groups + group), its lane and the number of
 * cross-lane waits (arrays of n_ops * groups). */
int yk_model_get_schedule(yk_model* m, int32_t* lane_of, int32_t* n_waits);

/* Device pointer of activation buffer `buf` (debug / parity); buf = -1: the letterboxed
 * uint8 input canvas [max_batch][in_h][in_w][3] of a resizing model (NULL otherwise). */
int yk_model_buffer(yk_model* m, int buf, void** dev_ptr);

/* Synchronous device -> host copy (bindings without their own HIP runtime access). */
int yk_memcpy_d2h(void* host_dst, const void* dev_src, int64_t bytes);

/* Host-side layout check, compiled into the caller with the caller's view of the structs: 0 when
 * the loaded library has this header's ABI version and every struct size, else YK_ERR_STATE.
 * Call it once before any other entry point. */
static inline int yk_abi_check(void) {
  const int64_t want[12] = {(int64_t)sizeof(yk_tracker_cfg), (int64_t)sizeof(yk_tracker_stats),
                            (int64_t)sizeof(yk_track_out), (int64_t)sizeof(yk_track_state),
                            (int64_t)sizeof(yk_view), (int64_t)sizeof(yk_op), (int64_t)sizeof(yk_model_desc),
                            (int64_t)sizeof(yk_bt_cfg), (int64_t)sizeof(yk_motion), (int64_t)sizeof(yk_gmd_stats),
                            (int64_t)sizeof(yk_tensor), (int64_t)sizeof(yk_track_event)};
  if (yk_abi_version() != YK_ABI_VERSION) return YK_ERR_STATE;
  for (int i = 0; i < 12; ++i)
    if (yk_struct_size(i) != want[i]) return YK_ERR_STATE;
  return YK_OK;
}

#ifdef __cplusplus
}
#endif
#endif /* YK_H_ */
