"""ByteTrack / BoT-SORT of ultralytics/trackers restated in numpy + scipy.

TEST INFRASTRUCTURE (oracle/): the checker for the device tracker in csrc/bytetrack.hip; only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import it.

Follows, step by step and with the reference's dtypes (NEP 50 promotion: a numpy float32 scalar
op a python float stays float32; lists mixing float32 scalars and python floats become float64):
  * KalmanFilterXYAH / KalmanFilterXYWH     trackers/utils/kalman_filter.py:7-493
      initiate :64-96 / :320-362, multi_predict :165-203 / :431-470, project :135-163 / :401-429,
      update :205-236 (scipy.linalg.cho_factor / cho_solve, as the reference calls them)
  * STrack / BOTrack                         trackers/byte_tracker.py:16-237, bot_sort.py:21-153
  * BYTETracker.update and its list helpers  byte_tracker.py:299-485
  * BOTSORT without ReID                     bot_sort.py:156-249 (get_dists :227-240 with
      with_reid False is iou_distance + fuse_score); with an image, its GMC (oracle/gmc_ref.py,
      'sparseOptFlow' or 'none') and STrack.multi_gmc (byte_tracker.py:108-125, 333-340)
  * matching.iou_distance / fuse_score       trackers/utils/matching.py:64-157, with
      utils/metrics.py:23-52 bbox_ioa(iou=True) in float32
  * matching.linear_assignment (matching.py:20-61): by default the lap branch the reference
      takes (use_lap=True; `lap>=0.5.12` is a hard requirement, matching.py:9-17): lapjv's
      extended cost_limit problem (lapjv_extended; `lap` itself is not installed, so its
      problem is restated and solved exactly by scipy -- unique optima agree, equal-cost ties
      are unpinned), unmatched lists ascending.  use_lap=False keeps the scipy branch
      (:50-59): linear_sum_assignment, the threshold filter, and the unmatched lists in
      CPython's frozenset iteration order (oracle/pyset_order.py restates that order for the
      device; here the real frozensets are used).
  * Track ids: BaseTrack._count is process-global (basetrack.py:67-92): one counter shared by
    every tracker, reset by each tracker's __init__ / reset (reset_id).  IdCounter models it;
    pass one instance to all streams' trackers and step the streams in index order.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import scipy.linalg
import scipy.optimize

NEW, TRACKED, LOST, REMOVED = 0, 1, 2, 3

BYTETRACK_CFG = dict(tracker_type="bytetrack", track_high_thresh=0.25, track_low_thresh=0.1,
                     new_track_thresh=0.25, track_buffer=30, match_thresh=0.8, fuse_score=True)
BOTSORT_CFG = dict(BYTETRACK_CFG, tracker_type="botsort", gmc_method="sparseOptFlow", proximity_thresh=0.5,
                   appearance_thresh=0.8, with_reid=False, model="auto")


class IdCounter:
    """BaseTrack._count (basetrack.py:67-92)."""

    def __init__(self):
        self.count = 0

    def next_id(self):
        self.count += 1
        return self.count

    def reset(self):
        self.count = 0


class Dets:
    """The slice of ultralytics Boxes the trackers read: xyxy / conf / cls as float32 and xywh
    computed like ops.xyxy2xywh (ops.py:256-274)."""

    def __init__(self, xyxy, conf, cls):
        self.xyxy = np.asarray(xyxy, np.float32).reshape(-1, 4)
        self.conf = np.asarray(conf, np.float32).reshape(-1)
        self.cls = np.asarray(cls, np.float32).reshape(-1)

    def __len__(self):
        return len(self.conf)

    def __getitem__(self, m):
        return Dets(self.xyxy[m], self.conf[m], self.cls[m])

    @property
    def xywh(self):
        x = self.xyxy
        y = np.empty_like(x)
        y[:, 0] = (x[:, 0] + x[:, 2]) / 2
        y[:, 1] = (x[:, 1] + x[:, 3]) / 2
        y[:, 2] = x[:, 2] - x[:, 0]
        y[:, 3] = x[:, 3] - x[:, 1]
        return y


# ---------------------------------------------------------------------------- Kalman filters
_WP, _WV = 1.0 / 20, 1.0 / 160
_F = np.eye(8)
for _i in range(4):
    _F[_i, 4 + _i] = 1.0
_H = np.eye(4, 8)


def kf_initiate(kind, m):
    mean = np.r_[m, np.zeros_like(m)]
    if kind == "xyah":
        std = [2 * _WP * m[3], 2 * _WP * m[3], 1e-2, 2 * _WP * m[3],
               10 * _WV * m[3], 10 * _WV * m[3], 1e-5, 10 * _WV * m[3]]
    else:
        std = [2 * _WP * m[2], 2 * _WP * m[3], 2 * _WP * m[2], 2 * _WP * m[3],
               10 * _WV * m[2], 10 * _WV * m[3], 10 * _WV * m[2], 10 * _WV * m[3]]
    return mean, np.diag(np.square(std))


def kf_multi_predict(kind, mean, cov):
    if kind == "xyah":
        sp = [_WP * mean[:, 3], _WP * mean[:, 3], 1e-2 * np.ones_like(mean[:, 3]), _WP * mean[:, 3]]
        sv = [_WV * mean[:, 3], _WV * mean[:, 3], 1e-5 * np.ones_like(mean[:, 3]), _WV * mean[:, 3]]
    else:
        sp = [_WP * mean[:, 2], _WP * mean[:, 3], _WP * mean[:, 2], _WP * mean[:, 3]]
        sv = [_WV * mean[:, 2], _WV * mean[:, 3], _WV * mean[:, 2], _WV * mean[:, 3]]
    sqr = np.square(np.r_[sp, sv]).T
    motion = np.asarray([np.diag(sqr[i]) for i in range(len(mean))])
    mean = np.dot(mean, _F.T)
    left = np.dot(_F, cov).transpose((1, 0, 2))
    return mean, np.dot(left, _F.T) + motion


def kf_project(kind, mean, cov):
    if kind == "xyah":
        std = [_WP * mean[3], _WP * mean[3], 1e-1, _WP * mean[3]]
    else:
        std = [_WP * mean[2], _WP * mean[3], _WP * mean[2], _WP * mean[3]]
    return np.dot(_H, mean), np.linalg.multi_dot((_H, cov, _H.T)) + np.diag(np.square(std))


def kf_update(kind, mean, cov, meas):
    pm, pc = kf_project(kind, mean, cov)
    cf, lower = scipy.linalg.cho_factor(pc, lower=True, check_finite=False)
    gain = scipy.linalg.cho_solve((cf, lower), np.dot(cov, _H.T).T, check_finite=False).T
    innov = meas - pm
    return mean + np.dot(innov, gain.T), cov - np.linalg.multi_dot((gain, pc, gain.T))


# ---------------------------------------------------------------------------- tracks
class Track:
    """STrack (kind 'xyah') / BOTrack without features (kind 'xywh')."""

    def __init__(self, row, score, cls, kind):
        x = np.copy(row[:4])  # ops.xywh2ltwh (ops.py:350-363) on the float64 row, then float32
        x[0] = row[0] - row[2] / 2
        x[1] = row[1] - row[3] / 2
        self._tlwh = np.asarray(x, dtype=np.float32)
        self.kind = kind
        self.mean = self.cov = None
        self.is_activated = False
        self.score, self.cls, self.idx = score, cls, row[-1]
        self.tracklet_len = 0
        self.track_id = 0
        self.state = NEW
        self.start_frame = self.frame_id = 0

    @property
    def end_frame(self):
        return self.frame_id

    def measurement(self, tlwh):
        r = np.asarray(tlwh).copy()
        r[:2] += r[2:] / 2
        if self.kind == "xyah":
            r[2] /= r[3]
        return r

    @property
    def tlwh(self):
        if self.mean is None:
            return self._tlwh.copy()
        r = self.mean[:4].copy()
        if self.kind == "xyah":
            r[2] *= r[3]
        r[:2] -= r[2:] / 2
        return r

    @property
    def xyxy(self):
        r = self.tlwh.copy()
        r[2:] += r[:2]
        return r

    @property
    def result(self):
        return self.xyxy.tolist() + [self.track_id, self.score, self.cls, self.idx]

    def activate(self, frame_id, ids):
        self.track_id = ids.next_id()
        self.mean, self.cov = kf_initiate(self.kind, self.measurement(self._tlwh))
        self.tracklet_len = 0
        self.state = TRACKED
        if frame_id == 1:
            self.is_activated = True
        self.frame_id = self.start_frame = frame_id

    def re_activate(self, det, frame_id):
        self.mean, self.cov = kf_update(self.kind, self.mean, self.cov, self.measurement(det.tlwh))
        self.tracklet_len = 0
        self.state = TRACKED
        self.is_activated = True
        self.frame_id = frame_id
        self.score, self.cls, self.idx = det.score, det.cls, det.idx

    def update(self, det, frame_id):
        self.frame_id = frame_id
        self.tracklet_len += 1
        self.mean, self.cov = kf_update(self.kind, self.mean, self.cov, self.measurement(det.tlwh))
        self.state = TRACKED
        self.is_activated = True
        self.score, self.cls, self.idx = det.score, det.cls, det.idx


def multi_gmc(tracks, H):
    """STrack.multi_gmc (byte_tracker.py:108-125)."""
    if tracks:
        multi_mean = np.asarray([t.mean.copy() for t in tracks])
        multi_cov = np.asarray([t.cov for t in tracks])
        R = H[:2, :2]
        R8x8 = np.kron(np.eye(4, dtype=float), R)
        tr = H[:2, 2]
        for i, (mean, cov) in enumerate(zip(multi_mean, multi_cov)):
            mean = R8x8.dot(mean)
            mean[:2] += tr
            cov = R8x8.dot(cov).dot(R8x8.transpose())
            tracks[i].mean = mean
            tracks[i].cov = cov


def multi_predict(tracks, kind):
    if not tracks:
        return
    mean = np.asarray([t.mean.copy() for t in tracks])
    cov = np.asarray([t.cov for t in tracks])
    for i, t in enumerate(tracks):
        if t.state != TRACKED:
            mean[i][7] = 0
            if kind == "xywh":
                mean[i][6] = 0
    mean, cov = kf_multi_predict(kind, mean, cov)
    for i, t in enumerate(tracks):
        t.mean, t.cov = mean[i], cov[i]


# ---------------------------------------------------------------------------- matching
def bbox_iou_f32(b1, b2, eps=1e-7):
    """utils/metrics.py:23-52 bbox_ioa(iou=True) on float32 inputs."""
    a1x1, a1y1, a1x2, a1y2 = b1.T
    a2x1, a2y1, a2x2, a2y2 = b2.T
    inter = (np.minimum(a1x2[:, None], a2x2) - np.maximum(a1x1[:, None], a2x1)).clip(0) * (
        np.minimum(a1y2[:, None], a2y2) - np.maximum(a1y1[:, None], a2y1)).clip(0)
    area = (a2x2 - a2x1) * (a2y2 - a2y1)
    area = area + ((a1x2 - a1x1) * (a1y2 - a1y1))[:, None] - inter
    return inter / (area + eps)


def iou_distance(a, b):
    ious = np.zeros((len(a), len(b)), dtype=np.float32)
    if len(a) and len(b):
        ious = bbox_iou_f32(np.ascontiguousarray([t.xyxy for t in a], dtype=np.float32),
                            np.ascontiguousarray([t.xyxy for t in b], dtype=np.float32))
    return 1 - ious


def fuse_score(cost, dets):
    if cost.size == 0:
        return cost
    sim = 1 - cost
    sc = np.expand_dims(np.array([d.score for d in dets]), axis=0).repeat(cost.shape[0], axis=0)
    return 1 - sim * sc


def lapjv_extended(cost, cost_limit):
    """lap.lapjv(cost, extend_cost=True, cost_limit=cost_limit) (gatagat/lap 0.5.12, the `lap`
    the reference requires, matching.py:9-17): the (n_rows + n_cols)-square float64 problem
    whose top-left block is `cost`, every other entry cost_limit / 2 except the zero
    bottom-right block; x / y map rows / columns to their partner, -1 for a dummy.  lap's
    Jonker-Volgenant solver is replaced by scipy's exact solver on the same extended matrix:
    both return an optimum, so they agree whenever the optimum is unique; among equal-cost
    optima the choice is the solver's own (lap is not installed here: that tie rule is
    unpinned)."""
    n_rows, n_cols = cost.shape
    n = n_rows + n_cols
    ext = np.empty((n, n), dtype=np.double)
    ext[:] = cost_limit / 2.0
    ext[n_rows:, n_cols:] = 0
    ext[:n_rows, :n_cols] = cost
    r, c = scipy.optimize.linear_sum_assignment(ext)
    x = np.full(n, -1, dtype=np.int64)
    y = np.full(n, -1, dtype=np.int64)
    x[r], y[c] = c, r
    x, y = x[:n_rows], y[:n_cols]
    x[x >= n_cols] = -1
    y[y >= n_rows] = -1
    return x, y


def linear_assignment(cost, thresh, use_lap=True):
    """matching.linear_assignment (matching.py:20-61).  use_lap=True (the reference's default):
    lap.lapjv with extend_cost and cost_limit=thresh, matches in row order, unmatched lists
    ascending (np.where).  use_lap=False: the scipy branch (optimal assignment of the whole
    matrix, then the `cost <= thresh` filter, unmatched lists in frozenset order)."""
    if cost.size == 0:
        return np.empty((0, 2), dtype=int), tuple(range(cost.shape[0])), tuple(range(cost.shape[1]))
    if use_lap:
        x, y = lapjv_extended(cost, thresh)
        matches = [[ix, mx] for ix, mx in enumerate(x) if mx >= 0]
        return matches, np.where(x < 0)[0], np.where(y < 0)[0]
    x, y = scipy.optimize.linear_sum_assignment(cost)
    matches = np.asarray([[x[i], y[i]] for i in range(len(x)) if cost[x[i], y[i]] <= thresh])
    if len(matches) == 0:
        ua, ub = list(np.arange(cost.shape[0])), list(np.arange(cost.shape[1]))
    else:
        ua = list(frozenset(np.arange(cost.shape[0])) - frozenset(matches[:, 0]))
        ub = list(frozenset(np.arange(cost.shape[1])) - frozenset(matches[:, 1]))
    return matches, ua, ub


# ---------------------------------------------------------------------------- the tracker
def _joint(a, b):
    seen, out = set(), []
    for t in a:
        seen.add(t.track_id)
        out.append(t)
    for t in b:
        if t.track_id not in seen:
            seen.add(t.track_id)
            out.append(t)
    return out


def _sub(a, b):
    ids = {t.track_id for t in b}
    return [t for t in a if t.track_id not in ids]


def _remove_duplicates(a, b):
    d = iou_distance(a, b)
    pairs = np.where(d < 0.15)
    da, db = [], []
    for p, q in zip(*pairs):
        if a[p].frame_id - a[p].start_frame > b[q].frame_id - b[q].start_frame:
            db.append(q)
        else:
            da.append(p)
    return [t for i, t in enumerate(a) if i not in da], [t for i, t in enumerate(b) if i not in db]


class RefTracker:
    """BYTETracker (cfg tracker_type 'bytetrack', KalmanFilterXYAH) or BOTSORT without ReID /
    GMC (tracker_type 'botsort', KalmanFilterXYWH)."""

    def __init__(self, cfg=None, frame_rate=30, ids: IdCounter | None = None, use_lap: bool = True):
        cfg = dict(BYTETRACK_CFG if cfg is None else cfg)
        self.use_lap = bool(use_lap)
        self.args = SimpleNamespace(**cfg)
        if self.args.tracker_type == "botsort" and self.args.with_reid:
            raise NotImplementedError("BoT-SORT ReID is not restated (with_reid: False)")
        self.kind = "xywh" if self.args.tracker_type == "botsort" else "xyah"
        self.ids = ids if ids is not None else IdCounter()
        self.max_time_lost = int(frame_rate / 30.0 * self.args.track_buffer)
        self.gmc = None
        if self.kind == "xywh":  # BOTSORT.__init__ (bot_sort.py:198)
            from .gmc_ref import RefGMC

            self.gmc = RefGMC(method=getattr(self.args, "gmc_method", "sparseOptFlow"))
        self.reset()

    def reset(self):
        self.tracked, self.lost, self.removed = [], [], []
        self.frame_id = 0
        self.ids.reset()
        if self.gmc is not None:
            self.gmc.reset_params()

    def _init_track(self, dets):
        if len(dets) == 0:
            return []
        rows = np.concatenate([dets.xywh, np.arange(len(dets)).reshape(-1, 1)], axis=-1)
        return [Track(r, s, c, self.kind) for r, s, c in zip(rows, dets.conf, dets.cls)]

    def _dists(self, tracks, dets):
        d = iou_distance(tracks, dets)
        return fuse_score(d, dets) if self.args.fuse_score else d

    def update(self, results: Dets, img=None):
        a = self.args
        self.frame_id += 1
        activated, refind, lost_new, removed_new = [], [], [], []
        scores = results.conf
        keep = scores >= a.track_high_thresh
        second = (scores > a.track_low_thresh) & (scores < a.track_high_thresh)
        dets = self._init_track(results[keep])
        dets2 = self._init_track(results[second])
        unconfirmed = [t for t in self.tracked if not t.is_activated]
        tracked = [t for t in self.tracked if t.is_activated]
        pool = _joint(tracked, self.lost)
        multi_predict(pool, self.kind)
        if self.gmc is not None and img is not None:  # byte_tracker.py:333-340
            try:
                warp = self.gmc.apply(img, None)
            except Exception:
                warp = np.eye(2, 3)
            multi_gmc(pool, warp)
            multi_gmc(unconfirmed, warp)
        m, u_track, u_det = linear_assignment(self._dists(pool, dets), thresh=a.match_thresh, use_lap=self.use_lap)
        for it, idt in m:
            t = pool[it]
            if t.state == TRACKED:
                t.update(dets[idt], self.frame_id)
                activated.append(t)
            else:
                t.re_activate(dets[idt], self.frame_id)
                refind.append(t)
        r_tracked = [pool[i] for i in u_track if pool[i].state == TRACKED]
        m, u_track, _ = linear_assignment(iou_distance(r_tracked, dets2), thresh=0.5, use_lap=self.use_lap)
        for it, idt in m:
            t = r_tracked[it]
            if t.state == TRACKED:
                t.update(dets2[idt], self.frame_id)
                activated.append(t)
            else:
                t.re_activate(dets2[idt], self.frame_id)
                refind.append(t)
        for it in u_track:
            t = r_tracked[it]
            if t.state != LOST:
                t.state = LOST
                lost_new.append(t)
        dets = [dets[i] for i in u_det]
        m, u_unc, u_det = linear_assignment(self._dists(unconfirmed, dets), thresh=0.7, use_lap=self.use_lap)
        for it, idt in m:
            unconfirmed[it].update(dets[idt], self.frame_id)
            activated.append(unconfirmed[it])
        for it in u_unc:
            unconfirmed[it].state = REMOVED
            removed_new.append(unconfirmed[it])
        for i in u_det:
            t = dets[i]
            if t.score < a.new_track_thresh:
                continue
            t.activate(self.frame_id, self.ids)
            activated.append(t)
        for t in self.lost:
            if self.frame_id - t.end_frame > self.max_time_lost:
                t.state = REMOVED
                removed_new.append(t)
        self.tracked = [t for t in self.tracked if t.state == TRACKED]
        self.tracked = _joint(self.tracked, activated)
        self.tracked = _joint(self.tracked, refind)
        self.lost = _sub(self.lost, self.tracked)
        self.lost.extend(lost_new)
        self.lost = _sub(self.lost, self.removed)  # before this frame's removals are appended (quirk)
        self.tracked, self.lost = _remove_duplicates(self.tracked, self.lost)
        self.removed.extend(removed_new)
        if len(self.removed) > 1000:
            self.removed = self.removed[-999:]
        return np.asarray([t.result for t in self.tracked if t.is_activated], dtype=np.float32)
