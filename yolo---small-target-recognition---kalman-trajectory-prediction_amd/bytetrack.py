"""ByteTrack / BoT-SORT (the upstream ultralytics model.track() trackers)
on the device: csrc/bytetrack.hip through the yk_bt_* C-ABI (include/yk.h).

Surfaces
  BYTETracker(args, frame_rate=30).update(results, img=None) -> np.ndarray[N, 8] float32
  BOTSORT(args, frame_rate=30).update(results, img=None)
      mirror ultralytics/trackers/byte_tracker.py:240-485 and bot_sort.py:156-249 (one stream;
      `results` is anything with .xyxy / .conf / .cls, e.g. Boxes.cpu().numpy()); rows are the
      reference's [x1, y1, x2, y2, track_id, score, cls, idx].
  BatchedTracker(cfg, n_streams)  many streams per launch, detections resident on the device
      ([S, max_dets, 6] float32 x1 y1 x2 y2 conf cls + [S] int32 counts), as the detect-and-track
      pipeline hands them over.
matching.linear_assignment follows its default lap branch (lap.lapjv with cost_limit, unmatched
lists ascending); use_lap=False selects the scipy branch (matching.py:50-59).
Track ids come from one counter shared by the streams of a BatchedTracker (the reference's
BaseTrack._count is process-global); separate BYTETracker objects each own a counter, like
separate processes.  BoT-SORT's ReID branch (with_reid) and its GMC (needs cv2 for every
method but 'none') are not built: requesting them raises.  There is no CPU fallback: the
library must load (YKError otherwise).
"""
from __future__ import annotations

import ctypes as C
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib as L

# cfg/trackers/bytetrack.yaml and botsort.yaml defaults
BYTETRACK_DEFAULTS = dict(tracker_type="bytetrack", track_high_thresh=0.25, track_low_thresh=0.1,
                          new_track_thresh=0.25, track_buffer=30, match_thresh=0.8, fuse_score=True)
BOTSORT_DEFAULTS = dict(BYTETRACK_DEFAULTS, tracker_type="botsort", gmc_method="sparseOptFlow",
                        proximity_thresh=0.5, appearance_thresh=0.8, with_reid=False, model="auto")


def load_tracker_cfg(source) -> SimpleNamespace:
    """A tracker config as the reference reads it (trackers/track.py:37-41): a YAML path, the
    names 'bytetrack.yaml' / 'botsort.yaml', a dict or a namespace."""
    if isinstance(source, str):
        name = source.rsplit("/", 1)[-1]
        if name in ("bytetrack.yaml", "botsort.yaml") and "/" not in source:
            d = dict(BOTSORT_DEFAULTS if name.startswith("botsort") else BYTETRACK_DEFAULTS)
        else:
            import yaml

            with open(source) as f:
                d = yaml.safe_load(f)
    elif isinstance(source, dict):
        d = dict(source)
    else:
        d = dict(vars(source))
    if d.get("tracker_type") not in ("bytetrack", "botsort"):
        raise AssertionError(f"Only 'bytetrack' and 'botsort' are supported for now, but got '{d.get('tracker_type')}'")
    base = BOTSORT_DEFAULTS if d["tracker_type"] == "botsort" else BYTETRACK_DEFAULTS
    return SimpleNamespace(**{**base, **d})


class BatchedTracker:
    """n_streams independent BYTETracker / BOTSORT states stepped by one launch."""

    def __init__(self, cfg=None, n_streams: int = 1, frame_rate: int = 30, max_tracks: int = 512,
                 max_dets: int = 512, device: int = 0, use_lap: bool = True):
        a = load_tracker_cfg(cfg if cfg is not None else dict(BYTETRACK_DEFAULTS))
        if a.tracker_type == "botsort" and getattr(a, "with_reid", False):
            raise NotImplementedError("BoT-SORT ReID (with_reid: True) is not built on the device path")
        self.args, self.S, self.device = a, int(n_streams), int(device)
        self.max_tracks, self.max_dets = int(max_tracks), int(max_dets)
        c = L.BtCfg(kind=L.BT_BOTSORT if a.tracker_type == "botsort" else L.BT_BYTETRACK,
                    track_high_thresh=float(a.track_high_thresh), track_low_thresh=float(a.track_low_thresh),
                    new_track_thresh=float(a.new_track_thresh), match_thresh=float(a.match_thresh),
                    track_buffer=int(a.track_buffer), frame_rate=int(frame_rate), fuse_score=int(bool(a.fuse_score)),
                    max_tracks=self.max_tracks, max_dets=self.max_dets,
                    assignment=L.BT_LAP if use_lap else L.BT_SCIPY, match_thresh_f64=float(a.match_thresh))
        h = C.c_void_p()
        L.check(L.lib().yk_bt_create(L.context(self.device), self.S, C.byref(c), C.byref(h)), "yk_bt_create")
        self._h = h
        self.dets = torch.zeros((self.S, self.max_dets, 6), dtype=torch.float32, device=f"cuda:{self.device}")
        self.counts = torch.zeros(self.S, dtype=torch.int32, device=f"cuda:{self.device}")
        self._rows = np.zeros((self.S, self.max_tracks, 8), np.float32)
        self._cnt = np.zeros(self.S, np.int32)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().yk_bt_destroy(h)
            except Exception:
                pass
            self._h = None

    def reset(self):
        L.check(L.lib().yk_bt_reset(self._h, L.current_stream(self.device)), "yk_bt_reset")

    def step_device(self, dets: torch.Tensor, counts: torch.Tensor):
        """One update() of every stream from device-resident detections (no host round trip)."""
        if dets.dtype != torch.float32 or dets.shape != (self.S, self.max_dets, 6) or not dets.is_contiguous():
            raise ValueError(f"dets must be a contiguous float32 tensor of shape {(self.S, self.max_dets, 6)}")
        if counts.dtype != torch.int32 or counts.shape != (self.S,):
            raise ValueError(f"counts must be an int32 tensor of shape ({self.S},)")
        L.check(L.lib().yk_bt_step(self._h, C.c_void_p(dets.data_ptr()), C.c_void_p(counts.data_ptr()),
                                   L.current_stream(self.device)), "yk_bt_step")

    def step(self, per_stream):
        """Host detections per stream (objects with .xyxy / .conf / .cls, or [n, 6] arrays)."""
        if len(per_stream) != self.S:
            raise ValueError(f"expected {self.S} streams, got {len(per_stream)}")
        buf = np.zeros((self.S, self.max_dets, 6), np.float32)
        cnt = np.zeros(self.S, np.int32)
        for s, r in enumerate(per_stream):
            a = _as_rows(r)
            if len(a) > self.max_dets:
                raise ValueError(f"stream {s}: {len(a)} detections > max_dets={self.max_dets}")
            buf[s, :len(a)] = a
            cnt[s] = len(a)
        self.dets.copy_(torch.from_numpy(buf))
        self.counts.copy_(torch.from_numpy(cnt))
        self.step_device(self.dets, self.counts)

    def download(self) -> list[np.ndarray]:
        L.check(L.lib().yk_bt_download(self._h, L.ptr(self._rows), L.ptr(self._cnt), L.current_stream(self.device)),
                "yk_bt_download")
        return [self._rows[s, :self._cnt[s]].copy() for s in range(self.S)]


def _as_rows(r) -> np.ndarray:
    if isinstance(r, np.ndarray):
        a = np.asarray(r, np.float32).reshape(-1, 6)
        return a
    xyxy = np.asarray(r.xyxy, np.float32).reshape(-1, 4)
    return np.concatenate([xyxy, np.asarray(r.conf, np.float32).reshape(-1, 1),
                           np.asarray(r.cls, np.float32).reshape(-1, 1)], axis=1)


class BYTETracker:
    """BYTETracker(args, frame_rate=30) of ultralytics/trackers/byte_tracker.py:240 on the device."""

    kind = "bytetrack"

    def __init__(self, args=None, frame_rate: int = 30, max_tracks: int = 512, max_dets: int = 1024, device: int = 0,
                 use_lap: bool = True):
        d = dict(vars(args)) if args is not None and not isinstance(args, (dict, str)) else args
        cfg = load_tracker_cfg(d if d is not None else dict(BOTSORT_DEFAULTS if self.kind == "botsort"
                                                             else BYTETRACK_DEFAULTS))
        if cfg.tracker_type != self.kind:
            cfg = SimpleNamespace(**{**vars(cfg), "tracker_type": self.kind})
        self.args = cfg
        self._b = BatchedTracker(vars(cfg), 1, frame_rate, max_tracks, max_dets, device, use_lap)
        self.frame_id = 0

    def reset(self):
        self._b.reset()
        self.frame_id = 0

    def update(self, results, img=None, feats=None) -> np.ndarray:
        if img is not None and self.kind == "botsort" and getattr(self.args, "gmc_method", "none") not in ("none", None):
            raise NotImplementedError("BoT-SORT GMC needs cv2 (absent); pass img=None or gmc_method: none")
        self.frame_id += 1
        self._b.step([results])
        return self._b.download()[0]


class BOTSORT(BYTETracker):
    """BOTSORT(args, frame_rate=30) of ultralytics/trackers/bot_sort.py:156 without ReID / GMC."""

    kind = "botsort"
