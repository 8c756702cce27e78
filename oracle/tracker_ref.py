"""numpy restatement of the reference Kalman tracker (TEST ORACLE ONLY).

Follows, operation for operation, the numeric steps of
  kalman/enhanced_aircraft_kalman_tracker.py   (per-track 8-state CV filter)
  kalman/enhanced_multi_target_tracker.py      (association + lifecycle)
so that, run with the same numpy/BLAS, it produces the reference's values bit
for bit.  Console messages of the reference are reproduced only when
``verbose=True`` (they are side effects, not results).

Numeric rules that matter for parity:
  * detections arrive as np.float32 scalars (aircraft_detection_tracking.py:101-106);
    bbox->state arithmetic and the IoU keep the dtype each operand carries
    (python max/min return the winning object, f32 op f32 stays f32).
  * the filter state x / P is float64 and is advanced with numpy matmul / inv.
  * quirk A: on the first lost frame get_track_info() runs predict() again
    (enhanced_aircraft_kalman_tracker.py:216-217 via :327-333, :351-353).
"""
from __future__ import annotations

from collections import deque

import numpy as np


def _bbox_to_state(bbox):
    # enhanced_aircraft_kalman_tracker.py:103-118 -- keeps the scalar dtypes of bbox
    a, b, c, d = bbox
    return np.array([(a + c) / 2.0, (b + d) / 2.0, c - a, d - b])


def _state_to_bbox(s):
    # enhanced_aircraft_kalman_tracker.py:120-135
    cx, cy, w, h = s[:4]
    return np.array([cx - w / 2.0, cy - h / 2.0, cx + w / 2.0, cy + h / 2.0])


def _model_matrices():
    # enhanced_aircraft_kalman_tracker.py:44-71
    P = np.eye(8)
    P[:4, :4] *= 50.0
    P[4:6, 4:6] *= 100.0
    P[6:, 6:] *= 1.0
    F = np.eye(8)
    for i in range(4):
        F[i, i + 4] = 1
    H = np.zeros((4, 8))
    for i in range(4):
        H[i, i] = 1
    Q = np.eye(8)
    Q[:2, :2] *= 0.1
    Q[2:4, 2:4] *= 0.01
    Q[4:6, 4:6] *= 0.1
    Q[6:, 6:] *= 0.001
    R = np.eye(4) * 10.0
    return P, F, H, Q, R


class RefTrack:
    """One reference track (AircraftKalmanTracker semantics)."""

    def __init__(self, bbox, track_id, max_lost_frames=450, verbose=False):
        self.track_id = track_id
        self.verbose = verbose
        self.age, self.hits, self.hit_streak, self.time_since_update = 0, 1, 1, 0
        self.P, self.F, self.H, self.Q, self.R = _model_matrices()
        self.x = np.zeros(8, dtype=float)
        s0 = _bbox_to_state(bbox)
        self.x[:4] = s0
        self.trajectory_history = deque(maxlen=150)
        self.velocity_history = deque(maxlen=50)
        self.position_history = deque(maxlen=100)
        self.motion_analysis = {
            "velocity_avg": np.array([0.0, 0.0]), "velocity_std": np.array([0.0, 0.0]),
            "direction": 0.0, "speed": 0.0, "stability_score": 0.0, "prediction_confidence": 0.0,
        }
        self.is_lost, self.lost_frames = False, 0
        self.max_lost_frames = max_lost_frames
        self.lost_start_state, self.lost_start_time = None, None
        self.trajectory_history.append((s0[0], s0[1]))
        self.position_history.append(s0[:2])

    # -- motion statistics (kf.py:137-182) ---------------------------------
    def analyze_motion_pattern(self):
        n = len(self.velocity_history)
        if n < 5:
            return
        v = np.array(list(self.velocity_history))
        ma = self.motion_analysis
        ma["velocity_avg"] = np.mean(v, axis=0)
        ma["velocity_std"] = np.std(v, axis=0)
        ax, ay = ma["velocity_avg"]
        ma["speed"] = np.sqrt(ax ** 2 + ay ** 2)
        ma["direction"] = np.arctan2(ay, ax)
        speed_stab = 1.0 / (1.0 + np.mean(ma["velocity_std"]))
        ma["stability_score"] = (speed_stab + self._direction_consistency()) / 2.0
        ma["prediction_confidence"] = ma["stability_score"] * min(n / 30.0, 1.0)

    def _direction_consistency(self):
        if len(self.velocity_history) < 3:
            return 0.0
        v = np.array(list(self.velocity_history))
        ang = np.arctan2(v[:, 1], v[:, 0])
        d = np.diff(ang)
        d = np.array([c if abs(c) < np.pi else c - 2 * np.pi * np.sign(c) for c in d])
        return 1.0 / (1.0 + np.std(d) * 10)

    # -- filter steps --------------------------------------------------------
    def predict(self):
        # kf.py:184-203
        self.x = self.F @ self.x
        self.P = self.F @ self.P @ self.F.T + self.Q
        self.age += 1
        self.time_since_update += 1
        self.trajectory_history.append((self.x[0], self.x[1]))
        return _state_to_bbox(self.x)

    def long_term_predict(self, k):
        # kf.py:205-247
        if k <= 1:
            return self.predict(), 1.0
        self.analyze_motion_pattern()
        ma = self.motion_analysis
        if ma["prediction_confidence"] > 0.3:
            s = self.x.copy()
            s[0] += ma["velocity_avg"][0] * k
            s[1] += ma["velocity_avg"][1] * k
            s[2:4] = self.x[2:4]
            conf = ma["prediction_confidence"] * max(0.1, 1.0 - k / self.max_lost_frames)
        else:
            s = self.x.copy()
            for _ in range(k):
                s = self.F @ s
            conf = max(0.1, 1.0 - k / (self.max_lost_frames * 0.5))
        return _state_to_bbox(s), conf

    def update(self, bbox):
        # kf.py:249-297
        self.time_since_update = 0
        self.hits += 1
        self.hit_streak += 1
        if self.is_lost:
            lost_for = self.lost_frames
            self.is_lost, self.lost_frames = False, 0
            self.lost_start_state, self.lost_start_time = None, None
            if self.verbose:
                print(f"目标 {self.track_id} 重新检测到，丢失了 {lost_for} 帧")
        z = _bbox_to_state(bbox)
        y = z - self.H @ self.x
        S = self.H @ self.P @ self.H.T + self.R
        K = self.P @ self.H.T @ np.linalg.inv(S)
        self.x = self.x + K @ y
        self.P = (np.eye(8) - K @ self.H) @ self.P
        self.velocity_history.append(self.x[4:6].copy())
        self.position_history.append(self.x[:2].copy())
        self.trajectory_history.append((self.x[0], self.x[1]))
        self.analyze_motion_pattern()

    def mark_as_lost(self):
        # kf.py:299-317
        if not self.is_lost:
            self.is_lost, self.lost_frames = True, 0
            self.lost_start_state, self.lost_start_time = self.x.copy(), self.age
            if self.verbose:
                p, v = self.lost_start_state[:2], self.lost_start_state[4:6]
                c = self.motion_analysis.get("prediction_confidence", 0.0)
                print(f"目标 {self.track_id} 丢失 - 位置: [{p[0]:.1f}, {p[1]:.1f}], "
                      f"速度: [{v[0]:.2f}, {v[1]:.2f}], 运动置信度: {c:.2f}")
        self.lost_frames += 1
        self.hit_streak = 0

    def get_lost_prediction(self):
        # kf.py:319-333
        if not self.is_lost:
            return _state_to_bbox(self.x), 1.0
        return self.long_term_predict(self.lost_frames)

    def get_track_info(self):
        # kf.py:335-383 (dict keys and evaluation order preserved)
        predicted = self.time_since_update > 0
        if predicted:
            if self.is_lost:
                box, conf = self.get_lost_prediction()
            else:  # unreachable in the multi-target flow, kept for parity
                box = _state_to_bbox(self.x)
                conf = max(0.3, 1.0 - self.time_since_update / 60.0)
            status = "predicted"
        else:
            box, conf, status = _state_to_bbox(self.x), 1.0, "detected"
        ma = self.motion_analysis
        return {
            "track_id": self.track_id, "bbox": box, "confidence": conf, "status": status,
            "age": self.age, "hits": self.hits, "hit_streak": self.hit_streak,
            "time_since_update": self.time_since_update, "lost_frames": self.time_since_update,
            "is_lost": predicted, "trajectory": list(self.trajectory_history)[-30:],
            "velocity": self.x[4:6], "motion_confidence": ma.get("prediction_confidence", 0.0),
            "is_stable_motion": ma.get("stability_score", 0.0) > 0.5,
            "speed": ma.get("speed", 0.0), "direction": ma.get("direction", 0.0),
        }

    def should_delete(self, max_lost_frames):
        # kf.py:385-405
        if self.time_since_update > max_lost_frames:
            return True
        if self.age < 5 and self.hit_streak == 0 and self.time_since_update > 15:
            return True
        if self.age < 10 and self.hit_streak <= 1 and self.time_since_update > 30:
            return True
        return False


def ref_iou(b1, b2):
    """IoU exactly as enhanced_multi_target_tracker.py:200-232 (dtype-preserving)."""
    ax1, ay1, ax2, ay2 = b1
    bx1, by1, bx2, by2 = b2
    ix1, iy1 = max(ax1, bx1), max(ay1, by1)
    ix2, iy2 = min(ax2, bx2), min(ay2, by2)
    if ix2 <= ix1 or iy2 <= iy1:
        return 0.0
    inter = (ix2 - ix1) * (iy2 - iy1)
    union = (ax2 - ax1) * (ay2 - ay1) + (bx2 - bx1) * (by2 - by1) - inter
    if union <= 0:
        return 0.0
    return inter / union


def ref_iou_matrix_f32dets(dets, boxes):
    """The D x T matrix of ``ref_iou(det, box)`` for np.float32 detections and float64 track
    boxes, vectorised with the scalar code's exact dtype flow (a test-harness speed-up for
    large track counts; ``ref_iou`` stays the definition and tests/test_oracle_kat.py checks
    the two agree bit for bit):
      * python max(a, b) returns a (the det) unless b > a; min(a, b) unless b < a -- each
        intersection coordinate keeps its origin dtype;
      * a difference / product of two float32 operands rounds to float32, anything with a
        float64 operand is float64 (the float32 operand widens exactly);
      * area1 is float32, area2 float64; union and inter/union are float64."""
    d32 = np.asarray([[d[0], d[1], d[2], d[3]] for d in dets], dtype=np.float32).reshape(-1, 1, 4)
    b64 = np.asarray(boxes, dtype=np.float64).reshape(1, -1, 4)
    d64 = d32.astype(np.float64)
    ax1, ay1, ax2, ay2 = (d64[..., i] for i in range(4))
    bx1, by1, bx2, by2 = (b64[..., i] for i in range(4))
    tx1, ty1 = bx1 > ax1, by1 > ay1  # the track value wins max()
    tx2, ty2 = bx2 < ax2, by2 < ay2  # the track value wins min()
    ix1, iy1 = np.where(tx1, bx1, ax1), np.where(ty1, by1, ay1)
    ix2, iy2 = np.where(tx2, bx2, ax2), np.where(ty2, by2, ay2)
    empty = (ix2 <= ix1) | (iy2 <= iy1)
    with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
        # both operands from the det -> float32 arithmetic; else float64
        wx32 = d32[..., 2] - d32[..., 0]
        wy32 = d32[..., 3] - d32[..., 1]
        wx = np.where(tx1 | tx2, ix2 - ix1, wx32.astype(np.float64))
        wy = np.where(ty1 | ty2, iy2 - iy1, wy32.astype(np.float64))
        f32x = ~(tx1 | tx2)
        f32y = ~(ty1 | ty2)
        inter32 = (wx.astype(np.float32) * wy.astype(np.float32)).astype(np.float64)
        inter = np.where(f32x & f32y, inter32, wx * wy)
        area1 = ((d32[..., 2] - d32[..., 0]) * (d32[..., 3] - d32[..., 1])).astype(np.float64)
        area2 = (bx2 - bx1) * (by2 - by1)
        union = area1 + area2 - inter
        iou = np.where(empty | (union <= 0), 0.0, inter / np.where(union > 0, union, 1.0))
    return iou


def ref_greedy_assign(iou, thr, stable=False):
    """enhanced_multi_target_tracker.py:234-270.  ``stable=True`` breaks exact IoU
    ties by row-major pair index (what the HIP kernel does); the default keeps
    numpy's default argsort like the reference."""
    if iou.size == 0:
        return []
    di, ti = np.where(iou >= thr)
    if len(di) == 0:
        return []
    order = np.argsort(-iou[di, ti], kind="stable" if stable else None)
    used_d, used_t, out = set(), set(), []
    for k in order:
        d, t = di[k], ti[k]
        if d not in used_d and t not in used_t:
            out.append((d, t))
            used_d.add(d)
            used_t.add(t)
    return out


class RefMultiTracker:
    """EnhancedMultiTargetTracker semantics (enhanced_multi_target_tracker.py:4-304)."""

    def __init__(self, max_lost_frames=450, min_hits=3, iou_threshold=0.3, verbose=False,
                 stable_ties=False, fast_iou=False):
        self.trackers: list[RefTrack] = []
        self.max_lost_frames, self.min_hits, self.iou_threshold = max_lost_frames, min_hits, iou_threshold
        self.frame_count, self.next_track_id = 0, 1
        self.verbose, self.stable_ties = verbose, stable_ties
        self.fast_iou = fast_iou  # vectorised IoU (same values) for float32 detections
        self.stats = {"total_tracks_created": 0, "total_tracks_terminated": 0,
                      "current_active_tracks": 0, "long_term_predictions": 0,
                      "successful_recoveries": 0}
        # diagnostics for parity harnesses: exact IoU ties among candidate pairs, and the frames on
        # which the stable order (the HIP kernel's) and numpy's default argsort (the reference's,
        # enhanced_multi_target_tracker.py:259) pick different pairs
        self.last_iou = None
        self.tie_frames = 0
        self.tie_divergent_frames = 0
        if verbose:  # enhanced_multi_target_tracker.py:40
            print(f"增强版多目标跟踪器初始化完成 - 最大丢失容忍: {max_lost_frames}帧 ({max_lost_frames/30:.1f}秒)")

    def _associate(self, dets, boxes):
        if self.fast_iou and all(isinstance(v, np.float32) for det in dets for v in det[:4]):
            iou = ref_iou_matrix_f32dets(dets, boxes)
        else:
            iou = np.zeros((len(dets), len(boxes)))
            for d, det in enumerate(dets):
                for t, tb in enumerate(boxes):
                    iou[d, t] = ref_iou(det[:4], tb)
        self.last_iou = iou
        cand = iou[iou >= self.iou_threshold]
        pairs = ref_greedy_assign(iou, self.iou_threshold, stable=self.stable_ties)
        if cand.size != np.unique(cand).size:
            self.tie_frames += 1
            other = ref_greedy_assign(iou, self.iou_threshold, stable=not self.stable_ties)
            if sorted((int(d), int(t)) for d, t in other) != sorted((int(d), int(t)) for d, t in pairs):
                self.tie_divergent_frames += 1
        md = {p[0] for p in pairs}
        mt = {p[1] for p in pairs}
        un_d = [d for d in range(len(dets)) if d not in md]
        un_t = [t for t in range(len(boxes)) if t not in mt]
        matched = []
        for d, t in pairs:  # post-filter of :171-176 (a no-op: all pairs passed >= thr)
            if iou[d, t] >= self.iou_threshold:
                matched.append((d, t))
            else:
                un_d.append(d)
                un_t.append(t)
        return matched, un_d, un_t

    def update(self, detections):
        self.frame_count += 1
        boxes = [t.predict() for t in self.trackers]
        if len(detections) > 0 and len(self.trackers) > 0:
            matched, un_d, un_t = self._associate(detections, boxes)
        else:
            matched, un_d, un_t = [], list(range(len(detections))), list(range(len(self.trackers)))
        for d, t in matched:
            trk = self.trackers[t]
            was_lost = trk.is_lost
            trk.update(detections[d][:4])
            if was_lost:
                self.stats["successful_recoveries"] += 1
                if self.verbose:
                    print(f"跟踪器 {trk.track_id} 重新检测到，切换回检测模式")
        for t in un_t:
            trk = self.trackers[t]
            was_lost = trk.is_lost
            trk.mark_as_lost()
            if self.verbose and not was_lost:
                print(f"跟踪器 {trk.track_id} 丢失检测，切换到预测模式")
        for d in un_d:
            trk = RefTrack(detections[d][:4], f"T{self.next_track_id:03d}", self.max_lost_frames,
                           verbose=self.verbose)
            self.trackers.append(trk)
            self.next_track_id += 1
            self.stats["total_tracks_created"] += 1
            if self.verbose:
                print(f"创建新跟踪器: {trk.track_id}")
        keep = []
        for trk in self.trackers:
            if trk.should_delete(self.max_lost_frames):
                self.stats["total_tracks_terminated"] += 1
                if self.verbose:
                    print(f"删除跟踪器 {trk.track_id} - 丢失时间: {trk.time_since_update}帧")
            else:
                keep.append(trk)
        self.trackers = keep
        self.stats["current_active_tracks"] = len(keep)
        out = []
        for trk in self.trackers:
            if trk.hit_streak >= self.min_hits or self.frame_count <= self.min_hits or trk.is_lost:
                info = trk.get_track_info()
                out.append(info)
                if info["status"] == "predicted" and info["lost_frames"] > 30:
                    self.stats["long_term_predictions"] += 1
        if self.verbose and self.frame_count % 100 == 0:
            self._print_statistics()
        return out

    def _print_statistics(self):
        # enhanced_multi_target_tracker.py:272-287
        print(f"\n=== 跟踪统计 (帧 {self.frame_count}) ===")
        print(f"当前活跃轨迹: {self.stats['current_active_tracks']}")
        print(f"总创建轨迹: {self.stats['total_tracks_created']}")
        print(f"总终止轨迹: {self.stats['total_tracks_terminated']}")
        print(f"成功恢复次数: {self.stats['successful_recoveries']}")
        print(f"长期预测次数: {self.stats['long_term_predictions']}")
        for t in self.trackers:
            status = "丢失" if t.is_lost else "正常"
            confidence = t.motion_analysis.get("prediction_confidence", 0.0)
            print(f"  {t.track_id}: {status}, 年龄:{t.age}, "
                  f"命中:{t.hits}, 丢失:{t.lost_frames}, 置信度:{confidence:.2f}")

    def get_statistics(self):
        return {**self.stats, "frame_count": self.frame_count,
                "tracker_details": [{"track_id": t.track_id, "age": t.age, "hits": t.hits,
                                     "lost_frames": t.lost_frames, "is_lost": t.is_lost,
                                     "confidence": t.motion_analysis.get("prediction_confidence", 0.0)}
                                    for t in self.trackers]}
