"""numpy restatement of the camera-motion-compensation tracker variant (TEST ORACLE ONLY).

SURVEY §8f rank 1: the reference's subclasses of the hot path
  camera_motion_compensation/motion_reset_kalman_tracker.py:16-355
      MotionResetKalmanTracker(AircraftKalmanTracker): per-track jump / velocity / size-change
      detection and Kalman reset (:86-285), blended predict after a reset (:287-312),
      reset fields in get_track_info (:314-336) and get_reset_statistics (:338-355)
  camera_motion_compensation/motion_compensated_multi_tracker.py:18-394
      MotionCompensatedMultiTracker(EnhancedMultiTargetTracker).update(detections, frame=None)
      (:77-124, :176-242): strict `iou > thr`, (iou, d, t)-descending greedy match (:262-274),
      every live tracker reported (:369-386), stats total_frames / individual_resets /
      tracking_recoveries.
With a frame, update() runs the global branch (:92-121, _should_global_reset :123-148,
_perform_global_reset :150-169) on a motion detector: oracle/gmd_ref.py's restatement of
GlobalMotionDetector('optical_flow') by default, or any object with detect_motion(frame)
(the tests drive the tracker-side decision with scripted results too).

Every numpy call keeps the reference's operand dtypes, so run with the same numpy (2.x, NEP 50
scalar promotion) the values follow the reference's.  Two deliberate deviations, both outside
the arithmetic: track ids are the creation index (the reference draws ``uuid.uuid4()``), and no
console output.  numpy's ``np.linalg.norm`` of a 2-vector is ``sqrt(x.dot(x))``; its last ulp
depends on the BLAS (FMA or not), which only matters at an exact threshold crossing.
"""
from __future__ import annotations

from collections import deque

import numpy as np

from .tracker_ref import RefTrack, _state_to_bbox, ref_iou

JUMP_PX, VEL_PX, SIZE_RATIO, COOLDOWN = 40.0, 60.0, 0.3, 15


def _center(b):
    x1, y1, x2, y2 = b
    return np.array([(x1 + x2) / 2.0, (y1 + y2) / 2.0])


def _size(b):
    x1, y1, x2, y2 = b
    return np.array([x2 - x1, y2 - y1])


class RefResetTrack(RefTrack):
    """MotionResetKalmanTracker semantics on top of RefTrack."""

    def __init__(self, bbox, track_id, max_lost_frames=150):
        super().__init__(bbox, track_id, max_lost_frames)
        # the subclass replaces the base's position deque (and its first entry)
        self.position_history = deque(maxlen=8)
        self.bbox_history = deque(maxlen=5)
        self.motion_scores = deque(maxlen=10)
        self.reset_count, self.last_reset_frame = 0, -999
        self.reset_log = []
        self.adaptive_enabled = True
        self.motion_consistency = 0.0
        self.position_history.append(_center(bbox))
        self.bbox_history.append(bbox)

    # -- the three detectors (:86-157) ---------------------------------------------
    def _jump(self, c):
        if len(self.position_history) < 2:
            return False, 0.0
        avg = np.mean(list(self.position_history)[-3:], axis=0)
        dist = np.linalg.norm(c - avg)
        self.motion_scores.append(min(dist / JUMP_PX, 3.0))
        return dist > JUMP_PX, dist

    def _velocity(self, c):
        if len(self.position_history) < 3:
            return False, 0.0
        pts = list(self.position_history)[-3:] + [c]
        sp = [np.linalg.norm(pts[i] - pts[i - 1]) for i in range(1, len(pts))]
        change = abs(sp[-1] - np.mean(sp[:-1]))
        return change > VEL_PX, change

    def _size_change(self, b):
        if len(self.bbox_history) < 2:
            return False, 0.0
        ratio = _size(b) / np.maximum(_size(self.bbox_history[-1]), 1.0)
        r = max(abs(ratio[0] - 1.0), abs(ratio[1] - 1.0))
        return r > SIZE_RATIO, r

    def _consistency(self):
        if len(self.motion_scores) < 3:
            return 0.0
        sc = list(self.motion_scores)
        m = np.mean(sc)
        if m > 0:
            return max(0.0, 1.0 - np.var(sc) / (m + 0.1))
        return 1.0

    def _reset_decision(self, b):
        # :159-214
        since = self.age - self.last_reset_frame
        if since < COOLDOWN:
            return False, [], 0.0
        c = _center(b)
        reasons, factors = [], []
        j, dist = self._jump(c)
        if j:
            reasons.append(("position", dist))
            factors.append(min(dist / JUMP_PX, 2.0))
        v, change = self._velocity(c)
        if v:
            reasons.append(("velocity", change))
            factors.append(min(change / VEL_PX, 2.0))
        s, r = self._size_change(b)
        if s:
            reasons.append(("size", r))
            factors.append(r / SIZE_RATIO)
        if not factors:
            return False, reasons, 0.0
        conf = np.mean(factors)
        self.motion_consistency = self._consistency()
        if self.motion_consistency < 0.3:
            conf *= 1.5
        if self.adaptive_enabled and self.reset_count > 0 and since < 50:
            conf *= 0.8
        return conf > 1.0, reasons, conf

    def _reset(self, b, reasons, conf):
        # :216-259
        self.reset_count += 1
        self.last_reset_frame = self.age
        self.reset_log.append({"frame": self.age, "reasons": reasons, "confidence": conf,
                               "motion_consistency": self.motion_consistency})
        s = np.array([(b[0] + b[2]) / 2.0, (b[1] + b[3]) / 2.0, b[2] - b[0], b[3] - b[1]])
        self.x[:4] = s
        self.x[4:] = 0
        self.P[4:, 4:] *= 100.0
        self.P[:4, :4] *= 5.0
        c = _center(b)
        self.trajectory_history.clear()
        self.trajectory_history.append((c[0], c[1]))
        self.velocity_history.clear()
        self.position_history.clear()
        self.position_history.append(c)
        self.motion_scores.clear()
        self.hits += 1
        self.hit_streak += 1
        self.time_since_update = 0

    def update(self, bbox):
        # :261-285
        go, reasons, conf = self._reset_decision(bbox)
        if go:
            self._reset(bbox, reasons, conf)
        else:
            super().update(bbox)
        self.position_history.append(_center(bbox))
        self.bbox_history.append(bbox)

    def predict(self):
        # :287-312
        box = super().predict()
        since = self.age - self.last_reset_frame
        if since < 10 and len(self.position_history) > 0:
            last = self.position_history[-1]
            pc = _center(box)
            w = min(since / 10.0, 1.0)
            adj = (1 - w) * last + w * pc
            sz = _size(box)
            box = [adj[0] - sz[0] / 2, adj[1] - sz[1] / 2, adj[0] + sz[0] / 2, adj[1] + sz[1] / 2]
        return box

    def get_track_info(self):
        # :314-336 (the formatted motion_consistency string and status suffix included)
        info = super().get_track_info()
        since = self.age - self.last_reset_frame
        info["reset_count"] = self.reset_count
        info["frames_since_reset"] = since
        info["motion_consistency"] = f"{self.motion_consistency:.2f}"
        if self.reset_count == 0:
            suffix = ""
        elif since < 20:
            suffix = f" | 重置({since}f前)"
        elif self.reset_count == 1:
            suffix = " | 已重置1次"
        else:
            suffix = f" | 已重置{self.reset_count}次"
        info["status_suffix"] = suffix
        return info

    def get_reset_statistics(self):
        # :338-355
        if not self.reset_log:
            return {"total_resets": 0, "details": []}
        dist = {}
        for r in self.reset_log:
            for kind, _ in r["reasons"]:
                dist[kind] = dist.get(kind, 0) + 1
        return {"total_resets": self.reset_count, "reason_distribution": dist,
                "avg_confidence": np.mean([r["confidence"] for r in self.reset_log]),
                "avg_motion_consistency": np.mean([r["motion_consistency"] for r in self.reset_log]),
                "details": self.reset_log[-5:]}


def cmc_greedy(iou, thr):
    """motion_compensated_multi_tracker.py:255-274: strict `>`, candidates sorted by the
    tuple (iou, d, t) descending (exact IoU ties -> larger d first, then larger t)."""
    cand = [(iou[d, t], d, t) for d in range(iou.shape[0]) for t in range(iou.shape[1]) if iou[d, t] > thr]
    cand.sort(reverse=True)
    used_d, used_t, out = set(), set(), []
    for _, d, t in cand:
        if d not in used_d and t not in used_t:
            out.append((d, t))
            used_d.add(d)
            used_t.add(t)
    return out


class RefCMCMultiTracker:
    """MotionCompensatedMultiTracker.update(detections, frame=None) semantics."""

    def __init__(self, max_lost_frames=150, min_hits=1, iou_threshold=0.1, motion_detector=None):
        self.trackers: list[RefResetTrack] = []
        self.max_lost_frames, self.min_hits, self.iou_threshold = max_lost_frames, min_hits, iou_threshold
        self.frame_count = 0
        self.next_num = 1
        self.stats = {"total_frames": 0, "global_motion_events": 0, "global_resets": 0,
                      "individual_resets": 0, "tracking_recoveries": 0}
        self.detection_stability_history = deque(maxlen=10)
        self.global_motion_history = deque(maxlen=20)
        self.frame_motion_info = None
        if motion_detector is None:
            from .gmd_ref import RefGlobalMotionDetector
            motion_detector = RefGlobalMotionDetector()
        # anything with detect_motion(frame) -> (is_motion, magnitude, vector, should_reset)
        self.motion_detector = motion_detector

    def update(self, detections, frame=None):
        """:75-121, the global branch included (frame given -> detect_motion on it)."""
        self.frame_count += 1
        self.stats["total_frames"] += 1
        global_motion_detected = False
        if frame is not None:
            is_motion, mag, vec, should_reset = self.motion_detector.detect_motion(frame)
            self.frame_motion_info = {"is_motion": is_motion, "magnitude": mag,
                                      "vector": vec.tolist() if hasattr(vec, "tolist") else vec,
                                      "should_reset": should_reset}
            self.global_motion_history.append(mag)
            if should_reset:
                global_motion_detected = True
                self.stats["global_motion_events"] += 1
        self.detection_stability_history.append(len(detections))
        if global_motion_detected and self._should_global_reset():
            return self._perform_global_reset(detections)
        return self._standard(detections)

    def _should_global_reset(self):
        """:123-148"""
        if not self.frame_motion_info or not self.frame_motion_info["should_reset"]:
            return False
        if len(self.detection_stability_history) >= 5:
            recent = list(self.detection_stability_history)[-5:]
            if np.std(recent) / (np.mean(recent) + 1) > 0.5:
                return True
        if len(self.global_motion_history) >= 3:
            if np.mean(list(self.global_motion_history)[-3:]) > 30.0:
                return True
        return self.frame_motion_info["magnitude"] > 60.0

    def _perform_global_reset(self, detections):
        """:150-169: every tracker dropped (no recovery accounting), one new tracker per detection."""
        self.stats["global_resets"] += 1
        self.trackers = []
        for det in detections:
            self.trackers.append(RefResetTrack(det[:4], self.next_num, self.max_lost_frames))
            self.next_num += 1
        return self._results()

    def _standard(self, detections):
        """:171-233"""
        boxes = [t.predict() for t in self.trackers]
        if len(detections) > 0 and len(self.trackers) > 0:
            iou = np.zeros((len(detections), len(boxes)))
            for d, det in enumerate(detections):
                for t, tb in enumerate(boxes):
                    iou[d, t] = ref_iou(det[:4], tb)
            pairs = cmc_greedy(iou, self.iou_threshold)
            md, mt = {p[0] for p in pairs}, {p[1] for p in pairs}
            un_d = [d for d in range(len(detections)) if d not in md]
            un_t = [t for t in range(len(boxes)) if t not in mt]
        else:
            pairs, un_d, un_t = [], list(range(len(detections))), list(range(len(self.trackers)))
        resets = 0
        for d, t in pairs:
            before = self.trackers[t].reset_count
            self.trackers[t].update(detections[d][:4])
            resets += self.trackers[t].reset_count > before
        self.stats["individual_resets"] += resets
        for t in un_t:
            self.trackers[t].mark_as_lost()
        for d in un_d:
            self.trackers.append(RefResetTrack(detections[d][:4], self.next_num, self.max_lost_frames))
            self.next_num += 1
        keep = []
        for trk in self.trackers:
            if trk.should_delete(self.max_lost_frames):
                if trk.reset_count > 0:
                    self.stats["tracking_recoveries"] += 1
            else:
                keep.append(trk)
        self.trackers = keep
        return self._results()

    def _results(self):
        out = []
        for trk in self.trackers:
            info = trk.get_track_info()
            info["reset_statistics"] = trk.get_reset_statistics()
            out.append(info)
        return out
