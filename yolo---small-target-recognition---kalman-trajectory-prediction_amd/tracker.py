"""Device-backed mirror of the reference ``kalman`` package.

Reference surface (kalman/__init__.py:28-33):
  EnhancedMultiTargetTracker(max_lost_frames=450, min_hits=3, iou_threshold=0.3)
      .update(detections) -> list[dict]           enhanced_multi_target_tracker.py:42-132
      .get_statistics(), .stats, .trackers, .frame_count, .next_track_id
  AircraftKalmanTracker / EnhancedAircraftKalmanTracker(initial_bbox, track_id=None,
      max_lost_frames=450)                         enhanced_aircraft_kalman_tracker.py:7-408
  MultiTargetTracker = EnhancedMultiTargetTracker
and of the camera-motion-compensation variant:
  MotionCompensatedMultiTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
      .update(detections, frame=None)              motion_compensated_multi_tracker.py:77-242
  over MotionResetKalmanTracker tracks             motion_reset_kalman_tracker.py:16-355

All filter arithmetic, association and lifecycle run in libyk.so's HIP kernels
(csrc/tracker.hip); this module only marshals detections in and dicts out.
``MultiStreamTracker`` is the batched, device-resident fast path (one launch steps
every stream) that the benchmark and the detector pipeline use.
"""
from __future__ import annotations

import ctypes as C
import uuid
from collections import deque

import numpy as np
import torch

from . import _lib as L

_STATUS = ("detected", "predicted")


def _det_array(detections):
    """Detections -> (array[D, 4], yk dtype).  np.float32 inputs (what the reference driver
    passes, aircraft_detection_tracking.py:101-106) keep float32 semantics; python floats /
    float64 arrays keep float64 semantics, exactly as the reference's arithmetic would."""
    if isinstance(detections, torch.Tensor):
        detections = detections.detach().cpu().numpy()
    if isinstance(detections, np.ndarray):
        a = detections
        if a.size == 0:
            return np.zeros((0, 4), np.float32), L.YK_F32
        if a.ndim != 2 or a.shape[1] < 4:
            raise ValueError(f"detections must be (N, >=4), got {a.shape}")
        if a.dtype == np.float32:
            return np.ascontiguousarray(a[:, :4]), L.YK_F32
        return np.ascontiguousarray(a[:, :4], dtype=np.float64), L.YK_F64
    dets = list(detections)
    if not dets:
        return np.zeros((0, 4), np.float32), L.YK_F32
    first = dets[0][0]
    if isinstance(first, np.float32) or (isinstance(first, np.ndarray) and first.dtype == np.float32):
        return np.array([[d[0], d[1], d[2], d[3]] for d in dets], dtype=np.float32), L.YK_F32
    return np.array([[d[0], d[1], d[2], d[3]] for d in dets], dtype=np.float64), L.YK_F64


def _row_to_dict(r, track_id: str) -> dict:
    """One yk_track_out row -> the reference get_track_info() dict
    (enhanced_aircraft_kalman_tracker.py:366-383)."""
    tsu = int(r["time_since_update"])
    n = int(r["traj_len"])
    tr = r["traj"][:n]
    return {
        "track_id": track_id,
        "bbox": np.array(r["bbox"], dtype=np.float64),
        "confidence": float(r["confidence"]),
        "status": _STATUS[int(r["status"])],
        "age": int(r["age"]),
        "hits": int(r["hits"]),
        "hit_streak": int(r["hit_streak"]),
        "time_since_update": tsu,
        "lost_frames": tsu,
        "is_lost": tsu > 0,
        "trajectory": [(float(a), float(b)) for a, b in tr],
        "velocity": np.array(r["velocity"], dtype=np.float64),
        "motion_confidence": float(r["motion_confidence"]),
        "is_stable_motion": bool(r["is_stable_motion"]),
        "speed": float(r["speed"]),
        "direction": float(r["direction"]),
    }


class TrajCache:
    """Trajectory lists of the previous frame, per track, so that a frame's dicts build only the
    points the device appended since (yk_track_out.traj_count): the reference returns
    ``list(trajectory_history)[-30:]`` afresh every frame (kf.py:382), i.e. the previous list
    shifted by the one or two new centres; materialising all 30 points of every track as Python
    floats each frame was most of the drop-in tracker's host time."""

    def __init__(self):
        self.d = {}

    def lists(self, nums, counts, lens, traj):
        """nums / counts / lens: lists per row; traj: [R, 30, 2] float64 (the rows' windows)."""
        R = len(nums)
        if R == 0:
            self.d = {}
            return []
        # every row's newest point in one gather (the usual one-point advance); more than one new
        # point reads the row itself
        lp = traj[np.arange(R), np.maximum(np.asarray(lens) - 1, 0)]
        last = list(zip(lp[:, 0].tolist(), lp[:, 1].tolist()))
        out, new = [], {}
        for i in range(R):
            n, c = lens[i], counts[i]
            old = self.d.get(nums[i])
            k = -1 if old is None else (c - old[0]) % (1 << 32)  # traj_count wraps mod 2^32 on the device
            if 0 <= k <= 3 and k <= n and n == min(len(old[1]) + k, traj.shape[1]):
                if k == 0:
                    lst = old[1]
                elif k == 1:
                    lst = old[1] + [last[i]]
                else:
                    lst = old[1] + list(map(tuple, traj[i, n - k:n].tolist()))
                if len(lst) > n:
                    lst = lst[len(lst) - n:]
            else:
                lst = list(map(tuple, traj[i, :n].tolist()))
            new[nums[i]] = (c, lst)  # cached lists are never handed out (the caller may mutate its own)
            out.append(list(lst))
        self.d = new
        return out


def rows_to_dicts(rows, cache: TrajCache | None = None) -> list[dict]:
    """yk_track_out rows -> the reference get_track_info() dicts (kf.py:366-383), column-wise:
    each field is read once for all rows; the same values and types as _row_to_dict."""
    R = len(rows)
    if R == 0:
        if cache is not None:
            cache.d = {}
        return []
    nums = rows["track_num"].tolist()
    tsu = rows["time_since_update"].tolist()
    st, age, hits, hs = rows["status"].tolist(), rows["age"].tolist(), rows["hits"].tolist(), rows["hit_streak"].tolist()
    conf, mc = rows["confidence"].tolist(), rows["motion_confidence"].tolist()
    sp, di, stab = rows["speed"].tolist(), rows["direction"].tolist(), rows["is_stable_motion"].tolist()
    bb = np.array(rows["bbox"], dtype=np.float64)  # fresh per frame: the dicts' arrays are views of it
    ve = np.array(rows["velocity"], dtype=np.float64)
    lens = rows["traj_len"].tolist()
    traj = np.array(rows["traj"], dtype=np.float64)
    if cache is not None:
        trajs = cache.lists(nums, rows["traj_count"].tolist(), lens, traj)
    else:
        trajs = [list(map(tuple, traj[i, :lens[i]].tolist())) for i in range(R)]
    bbs, ves = list(bb), list(ve)  # row views, made in C
    out = []
    for i in range(R):
        k = tsu[i]
        out.append({"track_id": f"T{nums[i]:03d}", "bbox": bbs[i], "confidence": conf[i], "status": _STATUS[st[i]],
                    "age": age[i], "hits": hits[i], "hit_streak": hs[i], "time_since_update": k, "lost_frames": k,
                    "is_lost": k > 0, "trajectory": trajs[i], "velocity": ves[i], "motion_confidence": mc[i],
                    "is_stable_motion": bool(stab[i]), "speed": sp[i], "direction": di[i]})
    return out


def track_id_of(num: int) -> str:
    return f"T{int(num):03d}"


_REASONS = ("position", "velocity", "size")


def _reason_text(kind: int, value: float) -> str:
    # the reason strings of motion_reset_kalman_tracker.py:105, :134, :155
    return (f"position_jump_{value:.1f}px", f"velocity_change_{value:.1f}px/f", f"size_change_{value:.2f}")[kind]


def _reset_fields(r, info: dict) -> dict:
    """MotionResetKalmanTracker.get_track_info extras + get_reset_statistics
    (motion_reset_kalman_tracker.py:314-355) from one yk_track_out row."""
    n, since = int(r["reset_count"]), int(r["frames_since_reset"])
    info["reset_count"] = n
    info["frames_since_reset"] = since
    info["motion_consistency"] = f"{float(r['motion_consistency']):.2f}"
    if n == 0:
        info["status_suffix"] = ""
    elif since < 20:
        info["status_suffix"] = f" | 重置({since}f前)"
    elif n == 1:
        info["status_suffix"] = " | 已重置1次"
    else:
        info["status_suffix"] = f" | 已重置{n}次"
    if n == 0:
        info["reset_statistics"] = {"total_resets": 0, "details": []}
        return info
    details = []
    for d in r["details"][: int(r["n_details"])]:
        reasons = [_reason_text(k, float(d["value"][k])) for k in range(3) if (int(d["reasons"]) >> k) & 1]
        details.append({"frame": int(d["frame"]), "reasons": reasons, "confidence": float(d["confidence"]),
                        "motion_consistency": float(d["motion_consistency"])})
    info["reset_statistics"] = {
        "total_resets": n,
        "reason_distribution": {_REASONS[k]: int(r["reason_count"][k]) for k in range(3) if int(r["reason_count"][k])},
        # averages accumulated in float64 over every reset (the reference's np.mean of the
        # logged values; identical unless every logged value is a float32 scalar)
        "avg_confidence": float(r["reset_confidence_sum"]) / n,
        "avg_motion_consistency": float(r["motion_consistency_sum"]) / n,
        "details": details,
    }
    return info


class MultiStreamTracker:
    """``n_streams`` independent EnhancedMultiTargetTracker instances stepped by one
    kernel launch (one workgroup per stream).  Detections and results stay in HBM."""

    def __init__(self, n_streams: int = 1, max_lost_frames: int = 450, min_hits: int = 3,
                 iou_threshold: float = 0.3, max_tracks: int = 1024, max_dets: int = 1024,
                 device: int = 0, policy: int = L.POLICY_ENHANCED):
        self.n_streams, self.device = int(n_streams), int(device)
        self.max_lost_frames, self.min_hits, self.iou_threshold = int(max_lost_frames), int(min_hits), float(iou_threshold)
        self.max_tracks, self.max_dets = int(max_tracks), int(max_dets)
        ctx = L.context(self.device)
        self.policy = int(policy)
        cfg = L.TrackerCfg(self.max_lost_frames, self.min_hits, self.iou_threshold, self.max_tracks, self.max_dets,
                           self.policy)
        h = C.c_void_p()
        L.check(L.lib().yk_tracker_create(ctx, self.n_streams, C.byref(cfg), C.byref(h)), "yk_tracker_create")
        self._h = h
        S, T = self.n_streams, self.max_tracks
        # page-locked host mirrors: the per-frame copies are DMA transfers, not staged ones
        self._pin = {"rows": torch.zeros(S * T * L.TRACK_OUT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True),
                     "counts": torch.zeros(S, dtype=torch.int32, pin_memory=True),
                     "stats": torch.zeros(S * L.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True),
                     "in_counts": torch.zeros(S, dtype=torch.int32, pin_memory=True)}
        self.host_rows = self._pin["rows"].numpy().view(L.TRACK_OUT_DTYPE).reshape(S, T)
        self.host_counts = self._pin["counts"].numpy()
        self.host_stats = self._pin["stats"].numpy().view(L.STATS_DTYPE)
        self._pin_dets = {}
        self._pin_evt = None
        dev = torch.device("cuda", self.device)
        self._dets = {L.YK_F32: torch.zeros((S, self.max_dets, 4), dtype=torch.float32, device=dev),
                      L.YK_F64: torch.zeros((S, self.max_dets, 4), dtype=torch.float64, device=dev)}
        self._counts = torch.zeros(S, dtype=torch.int32, device=dev)

    def __del__(self):
        h = getattr(self, "_h", None)
        try:
            if h is not None and L._lib is not None:
                L.lib().yk_tracker_destroy(h)
        except Exception:  # interpreter shutdown
            pass
        self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def reset(self):
        L.check(L.lib().yk_tracker_reset(self._h, L.current_stream(self.device)), "yk_tracker_reset")

    def step_device(self, dets: torch.Tensor, counts: torch.Tensor, stream=None, motion=None):
        """dets: device tensor [S, max_dets, stride] (float32 or float64); counts: int32 [S];
        motion: device address of yk_motion[S] (BatchedMotionDetector.motion_ptr) for the
        motion-reset policy's global branch, or None (no frames)."""
        if dets.dim() != 3 or dets.shape[0] != self.n_streams or dets.shape[1] != self.max_dets or dets.shape[2] < 4:
            raise ValueError(f"dets must be [{self.n_streams}, {self.max_dets}, >=4], got {tuple(dets.shape)}")
        if not dets.is_contiguous() or not counts.is_contiguous() or counts.dtype != torch.int32:
            raise ValueError("dets / counts must be contiguous; counts int32")
        dt = {torch.float32: L.YK_F32, torch.float64: L.YK_F64}.get(dets.dtype)
        if dt is None:
            raise ValueError("dets dtype must be float32 or float64")
        st = L.current_stream(self.device) if stream is None else C.c_void_p(stream)
        L.check(L.lib().yk_tracker_step_motion(self._h, L.ptr(dets), dt, int(dets.shape[2]), L.ptr(counts),
                                               C.c_void_p(motion or 0), st), "yk_tracker_step")

    def step_host(self, per_stream_dets, motion=None):
        """Host detections (one list/array per stream) -> step.  Returns nothing; call download()."""
        arrs = [_det_array(d) for d in per_stream_dets]
        if len(arrs) != self.n_streams:
            raise ValueError("need one detection list per stream")
        dts = {a[1] for a in arrs if len(a[0])}
        dt = dts.pop() if len(dts) == 1 else (L.YK_F64 if dts else L.YK_F32)
        buf = self._dets[dt]
        pin = self._pin_dets.get(dt)
        if pin is None:
            pin = self._pin_dets[dt] = torch.zeros(buf.shape, dtype=buf.dtype, pin_memory=True)
        if self._pin_evt is not None:
            self._pin_evt.synchronize()  # the previous step's copies out of the pinned buffers are done
        host, cnt = pin.numpy(), self._pin["in_counts"].numpy()
        for s, (a, _) in enumerate(arrs):
            if len(a) > self.max_dets:
                raise L.YKError(f"{len(a)} detections exceed max_dets={self.max_dets}")
            host[s, :len(a)] = a
            cnt[s] = len(a)
        n = int(cnt.max()) if len(cnt) else 0
        if n:  # only the rows the step reads (rows past a stream's count are never read)
            buf[:, :n].copy_(pin[:, :n], non_blocking=True)
        self._counts.copy_(self._pin["in_counts"], non_blocking=True)
        self._pin_evt = torch.cuda.Event()
        self._pin_evt.record(torch.cuda.current_stream(self.device))
        self.step_device(buf, self._counts, motion=motion)

    def download(self):
        st = L.current_stream(self.device)
        L.check(L.lib().yk_tracker_download(self._h, L.ptr(self.host_rows), L.ptr(self.host_counts),
                                            L.ptr(self.host_stats), st), "yk_tracker_download")
        return self.host_rows, self.host_counts, self.host_stats

    def download_async(self, rows: torch.Tensor, counts: torch.Tensor, stats: torch.Tensor | None = None,
                       rows_per_stream: int | None = None, stream=None):
        """Enqueue counts, stats and the first rows_per_stream (default: every) rows of each stream
        into page-locked host tensors (yk_tracker_download_async); nothing waits."""
        S, T = self.n_streams, self.max_tracks
        if not (rows.is_pinned() and counts.is_pinned() and (stats is None or stats.is_pinned())):
            raise ValueError("download_async needs page-locked host tensors")
        if rows.numel() * rows.element_size() < S * T * L.TRACK_OUT_DTYPE.itemsize or counts.numel() < S:
            raise ValueError("download_async: host buffers too small")
        if stats is not None and stats.numel() * stats.element_size() < S * L.STATS_DTYPE.itemsize:
            raise ValueError("download_async: stats buffer too small")
        n = T if rows_per_stream is None else int(rows_per_stream)
        st = L.current_stream(self.device) if stream is None else C.c_void_p(stream)
        L.check(L.lib().yk_tracker_download_async(self._h, C.c_void_p(rows.data_ptr()), C.c_void_p(counts.data_ptr()),
                                                  C.c_void_p(stats.data_ptr() if stats is not None else 0), n, st),
                "yk_tracker_download_async")

    def device_outputs(self):
        rows, counts, stats = C.c_void_p(), C.c_void_p(), C.c_void_p()
        L.check(L.lib().yk_tracker_outputs(self._h, C.byref(rows), C.byref(counts), C.byref(stats)),
                "yk_tracker_outputs")
        return rows.value, counts.value, stats.value

    def set_events(self, enable: bool = True):
        """Turn the per-step event log on / off (yk_tracker_set_events; enhanced policy)."""
        L.check(L.lib().yk_tracker_set_events(self._h, int(bool(enable))), "yk_tracker_set_events")

    def events(self, stream_index: int = 0) -> np.ndarray:
        """The last step's event records of one stream (TRACK_EVENT_DTYPE, one per work item)."""
        out = np.zeros(self.max_tracks, dtype=L.TRACK_EVENT_DTYPE)
        n = C.c_int32()
        L.check(L.lib().yk_tracker_events(self._h, int(stream_index), L.ptr(out), C.byref(n),
                                          L.current_stream(self.device)), "yk_tracker_events")
        return out[: n.value].copy()

    def phase_us(self, stream_index: int = 0):
        """Per-phase device time (µs) of the last step on one stream (wall clock of the stream's
        workgroup) and the association rounds used.  Single-workgroup step: predict, candidates,
        rounds, update, create, delete, outputs.  Two-launch enhanced step: predict = predicted
        boxes, candidates = bin index + candidate pairs (pairs_tested / n_cand / max_width /
        n_nonfinite describe the index), rounds, update = the list decisions, create = the gap to
        the start of tracks_kernel's first workgroup, delete = that workgroup's duration."""
        t = np.zeros(32, np.int64)
        L.check(L.lib().yk_tracker_phase_ticks(self._h, int(stream_index), L.ptr(t), L.current_stream(self.device)),
                "yk_tracker_phase_ticks")
        names = ["predict", "candidates", "rounds", "update", "create", "delete", "outputs"]
        return {n: float(t[k + 1] - t[k]) / 100.0 for k, n in enumerate(names)} | {
            "n_rounds": int(t[10]), "pairs_tested": int(t[11]), "n_cand": int(t[12]), "max_width": int(t[13]),
            "n_nonfinite": int(t[14]), "lds_cand_cap": int(t[23]),
            "k2_stage_us": float(t[8] - t[5]) / 100.0 if t[8] else 0.0,
            "k2_compute_us": float(t[9] - t[8]) / 100.0 if t[9] else 0.0,
            "k2_traj_us": float(t[6] - t[9]) / 100.0 if t[9] else 0.0,
            "k2_wave_cycles": [int(t[16 + k]) for k in range(4)],
            "cand_sub_us": [float(t[b] - t[a]) / 100.0 for a, b in ((1, 20), (20, 21), (21, 22), (22, 2))] if t[22] else [],
            "assoc_clock_mhz": round(float(t[15]) / max(float(t[4] - t[0]) / 100.0, 1e-9), 1)}

    def snapshot(self, stream_index: int = 0) -> np.ndarray:
        out = np.zeros(self.max_tracks, dtype=L.TRACK_STATE_DTYPE)
        n = C.c_int32()
        L.check(L.lib().yk_tracker_snapshot(self._h, int(stream_index), L.ptr(out), C.byref(n),
                                            L.current_stream(self.device)), "yk_tracker_snapshot")
        return out[: n.value].copy()

    def track_op(self, stream_index, pos, op, arg=0, box=None, dtype=L.YK_F64):
        inb = None if box is None else np.ascontiguousarray(np.asarray(box, dtype=np.float64)[:4])
        out5 = np.zeros(5, np.float64)
        row = np.zeros(1, dtype=L.TRACK_OUT_DTYPE)
        L.check(L.lib().yk_track_op(self._h, int(stream_index), int(pos), int(op), int(arg), L.ptr(inb), int(dtype),
                                    L.ptr(out5), L.ptr(row), L.current_stream(self.device)), "yk_track_op")
        return out5, row[0]

    def create_track(self, stream_index, box, dtype, track_num, max_lost_frames):
        b = np.ascontiguousarray(np.asarray(box, dtype=np.float64)[:4])
        L.check(L.lib().yk_track_create(self._h, int(stream_index), L.ptr(b), int(dtype), int(track_num),
                                        int(max_lost_frames), L.current_stream(self.device)), "yk_track_create")


def event_lines(ev: np.ndarray) -> list[str]:
    """The console lines EnhancedMultiTargetTracker.update() prints for one step, from the step's
    device event records (TRACK_EVENT_DTYPE), in the reference's order: the matched tracks that
    were lost, in the greedy match order -- IoU descending, then row-major (detection) order, the
    order _solve_assignment_problem appends pairs (enhanced_multi_target_tracker.py:234-270) --
    each with AircraftKalmanTracker.update's line (enhanced_aircraft_kalman_tracker.py:271) then
    the tracker's (:79); the newly unmatched tracks in list order (mark_as_lost's line, kf.py:313,
    then :89); the new tracks in detection order (:101); the removed tracks in list order (:109)."""
    lines = []
    rec = ev[ev["kind"] == L.EV_RECOVERED]
    for r in sorted(rec, key=lambda r: (-float(r["iou"]), int(r["det"]))):
        tid = track_id_of(r["track_num"])
        lines.append(f"目标 {tid} 重新检测到，丢失了 {int(r['lost_frames'])} 帧")
        lines.append(f"跟踪器 {tid} 重新检测到，切换回检测模式")
    for r in sorted(ev[ev["kind"] == L.EV_LOST], key=lambda r: int(r["list_pos"])):
        tid = track_id_of(r["track_num"])
        lines.append(f"目标 {tid} 丢失 - 位置: [{float(r['x']):.1f}, {float(r['y']):.1f}], "
                     f"速度: [{float(r['vx']):.2f}, {float(r['vy']):.2f}], 运动置信度: {float(r['confidence']):.2f}")
        lines.append(f"跟踪器 {tid} 丢失检测，切换到预测模式")
    for r in sorted(ev[ev["kind"] == L.EV_CREATED], key=lambda r: int(r["list_pos"])):
        lines.append(f"创建新跟踪器: {track_id_of(r['track_num'])}")
    for r in sorted(ev[ev["deleted_tsu"] >= 0], key=lambda r: int(r["list_pos"])):
        lines.append(f"删除跟踪器 {track_id_of(r['track_num'])} - 丢失时间: {int(r['deleted_tsu'])}帧")
    return lines


def _box_dtype(bbox):
    a, _ = _det_array([list(bbox)[:4]])
    return a[0], (L.YK_F32 if a.dtype == np.float32 else L.YK_F64)


_F = np.eye(8)
for _i in range(4):
    _F[_i, _i + 4] = 1.0
_H = np.hstack([np.eye(4), np.zeros((4, 4))])
_Q = np.diag([0.1, 0.1, 0.01, 0.01, 0.1, 0.1, 0.001, 0.001])
_R = np.eye(4) * 10.0


class AircraftKalmanTracker:
    """One track (enhanced_aircraft_kalman_tracker.py:7-408) whose state lives in HBM.

    Constructed directly it owns a private one-track device tracker; obtained from
    ``EnhancedMultiTargetTracker.trackers`` it is a live view of that tracker's track.
    Every filter operation runs on the GPU (``yk_track_op``)."""

    state_dim, measure_dim = 8, 4
    F, H, Q, R = _F, _H, _Q, _R

    def __init__(self, initial_bbox, track_id=None, max_lost_frames=450, *, device: int = 0):
        self.track_id = track_id or str(uuid.uuid4())[:8]
        self.max_lost_frames = int(max_lost_frames)
        self._owner = MultiStreamTracker(1, max_lost_frames=self.max_lost_frames, min_hits=1, iou_threshold=0.3,
                                         max_tracks=1, max_dets=1, device=device)
        box, dt = _box_dtype(initial_bbox)
        self._dtype = dt
        self._owner.create_track(0, box, dt, -1, self.max_lost_frames)
        self._num = None  # standalone: always list position 0
        self._multi = None

    @classmethod
    def _view(cls, multi: "EnhancedMultiTargetTracker", num: int):
        self = cls.__new__(cls)
        self.track_id = track_id_of(num)
        self.max_lost_frames = multi.max_lost_frames
        self._owner = multi._core
        self._dtype = L.YK_F32
        self._num = int(num)
        self._multi = multi
        return self

    # -- location / state ------------------------------------------------------
    def _pos(self) -> int:
        if self._num is None:
            return 0
        snap = self._multi._snapshot()
        idx = np.nonzero(snap["track_num"] == self._num)[0]
        if len(idx) == 0:
            raise L.YKError(f"track {self.track_id} is no longer live")
        return int(idx[0])

    def _state(self):
        snap = self._owner.snapshot(0) if self._num is None else self._multi._snapshot()
        return snap[self._pos()]

    def _touch(self):
        if self._multi is not None:
            self._multi._snap = None

    @property
    def x(self):
        return self._state()["x"].copy()

    @property
    def P(self):
        return self._state()["P"].copy()

    def _int(name):  # noqa: N805
        return property(lambda self: int(self._state()[name]))

    age = _int("age")
    hits = _int("hits")
    hit_streak = _int("hit_streak")
    time_since_update = _int("time_since_update")
    lost_frames = _int("lost_frames")
    del _int

    @property
    def is_lost(self):
        return bool(self._state()["is_lost"])

    @property
    def velocity_history(self):
        s = self._state()
        return deque([s["vel_hist"][i].copy() for i in range(int(s["vel_len"]))], maxlen=50)

    @property
    def trajectory_history(self):
        s = self._state()
        return deque([tuple(map(float, s["traj_hist"][i])) for i in range(int(s["traj_len"]))], maxlen=150)

    @property
    def motion_analysis(self):
        s = self._state()
        return {"velocity_avg": s["velocity_avg"].copy(), "velocity_std": s["velocity_std"].copy(),
                "direction": float(s["direction"]), "speed": float(s["speed"]),
                "stability_score": float(s["stability_score"]),
                "prediction_confidence": float(s["prediction_confidence"])}

    # -- pure helpers (kf.py:103-135) -------------------------------------------
    @staticmethod
    def bbox_to_state(bbox):
        x1, y1, x2, y2 = bbox
        return np.array([(x1 + x2) / 2.0, (y1 + y2) / 2.0, x2 - x1, y2 - y1])

    @staticmethod
    def state_to_bbox(state):
        cx, cy, w, h = state[:4]
        return np.array([cx - w / 2.0, cy - h / 2.0, cx + w / 2.0, cy + h / 2.0])

    # -- filter operations (all on the device) ---------------------------------
    def predict(self):
        out, _ = self._owner.track_op(0, self._pos(), L.OP_PREDICT)
        self._touch()
        return out[:4].copy()

    def update(self, bbox):
        box, dt = _box_dtype(bbox)
        self._owner.track_op(0, self._pos(), L.OP_UPDATE, box=box, dtype=dt)
        self._touch()

    def mark_as_lost(self):
        self._owner.track_op(0, self._pos(), L.OP_MARK_LOST)
        self._touch()

    def analyze_motion_pattern(self):
        """The device recomputes the motion statistics inside every update(); the history
        cannot change in between, so an explicit call has nothing left to do."""

    def enhanced_long_term_predict(self, frames_ahead=1):
        out, _ = self._owner.track_op(0, self._pos(), L.OP_LONG_TERM, arg=int(frames_ahead))
        self._touch()
        return out[:4].copy(), float(out[4])

    def get_lost_prediction(self):
        out, _ = self._owner.track_op(0, self._pos(), L.OP_LOST_PRED)
        self._touch()
        return out[:4].copy(), float(out[4])

    def get_track_info(self):
        _, row = self._owner.track_op(0, self._pos(), L.OP_INFO)
        self._touch()
        return _row_to_dict(row, self.track_id)

    def should_delete(self, max_lost_frames):
        s = self._state()
        tsu, age, hs = int(s["time_since_update"]), int(s["age"]), int(s["hit_streak"])
        if tsu > max_lost_frames:
            return True
        if age < 5 and hs == 0 and tsu > 15:
            return True
        return age < 10 and hs <= 1 and tsu > 30


EnhancedAircraftKalmanTracker = AircraftKalmanTracker


class MotionResetKalmanTracker(AircraftKalmanTracker):
    """One motion-reset track (camera_motion_compensation/motion_reset_kalman_tracker.py:16-355)
    whose state lives in HBM, on the same device operations as the batched motion-reset policy
    (tracker.hip: cmc_decide / cmc_reset / cmc_blend): ``update(bbox)`` runs _should_reset_kalman
    (position jump against the last <= 3 centres, velocity change, size change, motion
    consistency, cooldown, adaptive factors) and either resets the filter or runs the Kalman
    update; ``predict()`` blends the box toward the last centre for 10 frames after a reset;
    ``get_track_info()`` adds reset_count / frames_since_reset / motion_consistency /
    status_suffix; ``get_reset_statistics()`` as the reference.  Constructed directly it owns a
    private one-track device tracker (policy YK_POLICY_MOTION_RESET); obtained from
    ``MotionCompensatedMultiTracker.trackers`` it is a live view of that tracker's track."""

    jump_threshold = 40.0
    velocity_threshold = 60.0
    size_change_threshold = 0.3
    reset_cooldown = 15

    def __init__(self, initial_bbox, track_id=None, max_lost_frames=150, *, device: int = 0, verbose: bool = False):
        self.track_id = track_id or str(uuid.uuid4())[:8]
        self.max_lost_frames = int(max_lost_frames)
        self._owner = MultiStreamTracker(1, max_lost_frames=self.max_lost_frames, min_hits=1, iou_threshold=0.1,
                                         max_tracks=1, max_dets=1, device=device, policy=L.POLICY_MOTION_RESET)
        box, dt = _box_dtype(initial_bbox)
        self._dtype = dt
        self._owner.create_track(0, box, dt, -1, self.max_lost_frames)
        self._num = None
        self._multi = None
        if verbose:
            print(f"🎯 运动重置跟踪器初始化: {self.track_id}")

    def _row(self):
        """get_track_info's row (OP_INFO: it may predict, quirk A, as the reference does)."""
        _, row = self._owner.track_op(0, self._pos(), L.OP_INFO)
        self._touch()
        return row

    @property
    def reset_count(self) -> int:
        return int(self._state()["reset_count"])

    @property
    def last_reset_frame(self) -> int:
        return int(self._state()["last_reset_frame"])

    @property
    def motion_consistency(self) -> float:
        return float(self._state()["motion_consistency"])

    def get_track_info(self):
        row = self._row()
        info = _reset_fields(row, _row_to_dict(row, self.track_id))
        info.pop("reset_statistics", None)
        return info

    def get_reset_statistics(self):
        row = self._row()
        return _reset_fields(row, {})["reset_statistics"]


class EnhancedMultiTargetTracker:
    """Drop-in for kalman.EnhancedMultiTargetTracker (enhanced_multi_target_tracker.py:4-304),
    one stream, executed by the batched HIP tracker kernel."""

    def __init__(self, max_lost_frames=450, min_hits=3, iou_threshold=0.3, *, max_tracks: int = 1024,
                 max_dets: int = 1024, device: int = 0, verbose: bool = False):
        self.max_lost_frames, self.min_hits, self.iou_threshold = max_lost_frames, min_hits, iou_threshold
        self.verbose = verbose
        self._core = MultiStreamTracker(1, max_lost_frames, min_hits, iou_threshold, max_tracks, max_dets, device)
        self._stats = np.zeros(1, dtype=L.STATS_DTYPE)[0]
        self._stats["next_track_id"] = 1
        self._snap = None
        self._traj = TrajCache()
        if verbose:  # the reference prints its lifecycle messages (enhanced_multi_target_tracker.py:40,79-109)
            self._core.set_events(True)
            print(f"增强版多目标跟踪器初始化完成 - 最大丢失容忍: {max_lost_frames}帧 ({max_lost_frames/30:.1f}秒)")

    @property
    def frame_count(self) -> int:
        return int(self._stats["frame_count"])

    @property
    def next_track_id(self) -> int:
        return int(self._stats["next_track_id"])

    @property
    def stats(self) -> dict:
        s = self._stats
        return {k: int(s[k]) for k in ("total_tracks_created", "total_tracks_terminated", "current_active_tracks",
                                        "long_term_predictions", "successful_recoveries")}

    def _snapshot(self):
        if self._snap is None:
            self._snap = self._core.snapshot(0)
        return self._snap

    @property
    def trackers(self) -> list:
        return [AircraftKalmanTracker._view(self, int(n)) for n in self._snapshot()["track_num"]]

    def update(self, detections):
        """One frame: list of [x1, y1, x2, y2, conf] -> list of track dicts."""
        self._core.step_host([detections])
        rows, counts, stats = self._core.download()
        self._stats = stats[0].copy()
        self._snap = None
        if int(self._stats["overflow"]):
            raise L.YKError(f"tracker capacity exceeded (max_tracks={self._core.max_tracks})")
        out = rows_to_dicts(rows[0, : int(counts[0])], self._traj)
        if self.verbose:
            for line in event_lines(self._core.events(0)):
                print(line)
            if self.frame_count % 100 == 0:
                self._print_statistics()
        return out

    def _print_statistics(self):
        s = self.stats
        print(f"\n=== 跟踪统计 (帧 {self.frame_count}) ===")
        print(f"当前活跃轨迹: {s['current_active_tracks']}")
        print(f"总创建轨迹: {s['total_tracks_created']}")
        print(f"总终止轨迹: {s['total_tracks_terminated']}")
        print(f"成功恢复次数: {s['successful_recoveries']}")
        print(f"长期预测次数: {s['long_term_predictions']}")
        for t in self._snapshot():  # enhanced_multi_target_tracker.py:282-287, list order
            status = "丢失" if t["is_lost"] else "正常"
            print(f"  {track_id_of(t['track_num'])}: {status}, 年龄:{int(t['age'])}, "
                  f"命中:{int(t['hits'])}, 丢失:{int(t['lost_frames'])}, 置信度:{float(t['prediction_confidence']):.2f}")

    def get_statistics(self):
        snap = self._snapshot()
        return {**self.stats, "frame_count": self.frame_count,
                "tracker_details": [{"track_id": track_id_of(t["track_num"]), "age": int(t["age"]),
                                     "hits": int(t["hits"]), "lost_frames": int(t["lost_frames"]),
                                     "is_lost": bool(t["is_lost"]),
                                     "confidence": float(t["prediction_confidence"])} for t in snap]}


MultiTargetTracker = EnhancedMultiTargetTracker


class MotionCompensatedMultiTracker:
    """Drop-in for camera_motion_compensation.MotionCompensatedMultiTracker
    (motion_compensated_multi_tracker.py:18-394) on the batched HIP kernels: the motion-reset
    policy of the tracker kernel (YK_POLICY_MOTION_RESET: MotionResetKalmanTracker jump /
    velocity / size-change resets, blended predict after a reset, strict iou > thr with the
    (iou, d, t)-descending greedy order, every live tracker reported with its reset fields) and,
    when ``update(detections, frame)`` gets a frame, the global branch: GlobalMotionDetector
    ('optical_flow', csrc/gmd.hip) on the frame, then _should_global_reset /
    _perform_global_reset inside the tracker step (yk_tracker_step_motion).  Track ids are
    "T%03d" of the creation index (the reference draws uuid4 strings)."""

    def __init__(self, max_lost_frames=150, min_hits=1, iou_threshold=0.1, motion_detection_method="optical_flow",
                 *, max_tracks: int = 1024, max_dets: int = 1024, device: int = 0, verbose: bool = False):
        from .motion import GlobalMotionDetector

        self.max_lost_frames, self.min_hits, self.iou_threshold = max_lost_frames, min_hits, iou_threshold
        self.motion_detection_method = motion_detection_method
        self.motion_detector = GlobalMotionDetector(motion_detection_method, device=device)
        self.global_motion_compensation = True
        self.individual_reset_enabled = True
        self.adaptive_thresholds = True
        self._core = MultiStreamTracker(1, max_lost_frames, min_hits, iou_threshold, max_tracks, max_dets, device,
                                        policy=L.POLICY_MOTION_RESET)
        self._stats = np.zeros(1, dtype=L.STATS_DTYPE)[0]
        self._stats_base = np.zeros(1, dtype=L.STATS_DTYPE)[0]
        self._snap = None
        self.detection_stability_history = deque(maxlen=10)
        self.global_motion_history = deque(maxlen=20)
        self.frame_motion_info = None
        self.current_frame = None
        self.verbose = verbose

    @property
    def frame_count(self) -> int:
        return int(self._stats["frame_count"])

    @property
    def stats(self) -> dict:
        s, b = self._stats, self._stats_base
        return {k: int(s[src]) - int(b[src]) for k, src in (
            ("total_frames", "frame_count"), ("global_motion_events", "global_motion_events"),
            ("global_resets", "global_resets"), ("individual_resets", "individual_resets"),
            ("tracking_recoveries", "tracking_recoveries"))}

    def update(self, detections, frame=None):
        """:75-121"""
        motion = None
        self.current_frame = frame
        if frame is not None and self.global_motion_compensation:
            det = self.motion_detector._detector(frame)
            det.detect_host([frame])
            motion = det.motion_ptr
        self.detection_stability_history.append(len(detections))
        self._core.step_host([detections], motion=motion)
        self._snap = None
        rows, counts, stats = self._core.download()
        self._stats = stats[0].copy()
        if int(self._stats["overflow"]):
            raise L.YKError(f"tracker capacity exceeded (max_tracks={self._core.max_tracks})")
        if motion is not None:
            from .motion import motion_tuple

            m, _ = self.motion_detector._b.download()
            is_motion, mag, vec, should_reset = motion_tuple(m[0])
            self.frame_motion_info = {"is_motion": is_motion, "magnitude": mag,
                                      "vector": vec.tolist() if hasattr(vec, "tolist") else vec,
                                      "should_reset": should_reset}
            self.global_motion_history.append(mag)
        out = []
        for r in rows[0, : int(counts[0])]:
            info = _row_to_dict(r, track_id_of(r["track_num"]))
            info = _reset_fields(r, info)
            if self.frame_motion_info:
                info["global_motion"] = self.frame_motion_info
            out.append(info)
        return out

    def _snapshot(self):
        if self._snap is None:
            self._snap = self._core.snapshot(0)
        return self._snap

    @property
    def trackers(self) -> list:
        """Live MotionResetKalmanTracker views of this tracker's tracks, in list order."""
        return [MotionResetKalmanTracker._view(self, int(n)) for n in self._snapshot()["track_num"]]

    def set_global_motion_sensitivity(self, sensitivity):
        """:353-360"""
        if 0.5 <= sensitivity <= 2.0:
            self.motion_detector.global_motion_threshold /= sensitivity
            self.motion_detector.reset_motion_threshold /= sensitivity

    def enable_adaptive_mode(self, enabled=True):
        """:345-351 (the reset trackers carry no adaptive switch; the flag is kept)"""
        self.adaptive_thresholds = enabled

    def reset_all_statistics(self):
        """:362-374"""
        self._stats_base = self._stats.copy()
        self.motion_detector.reset_stats()

    def get_comprehensive_stats(self):
        """:308-343.  The reference never appends to stats['processing_times'], so 'performance'
        is always {}."""
        rows, counts, _ = self._core.download()
        live = rows[0, : int(counts[0])]
        return {"basic": self.stats,
                "motion_detection": self.motion_detector.get_stats(),
                "performance": {},
                "trackers": {"active_trackers": int(len(live)),
                             "total_resets_by_tracker": int(live["reset_count"].sum()) if len(live) else 0},
                "motion_history_avg": np.mean(self.global_motion_history) if self.global_motion_history else 0.0}
