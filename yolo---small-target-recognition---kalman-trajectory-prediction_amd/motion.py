"""Global camera-motion detection on the device: csrc/gmd.hip through the yk_gmd_* C-ABI.

Surfaces
  GlobalMotionDetector(method='optical_flow').detect_motion(frame)
      mirrors camera_motion_compensation/global_motion_detector.py:11-288 for one stream:
      returns (is_motion, motion_magnitude, motion_vector, should_reset) with the reference's
      types (np.float32 magnitude and vector when estimated, 0.0 / array([0., 0.]) otherwise);
      .stats / get_stats() / reset_stats() and the threshold attributes as in the reference.
  BatchedMotionDetector(n_streams, height, width)
      one launch sequence per step for every stream, frames resident on the device
      ([S, H, W, 3] uint8 BGR, the detector pipeline's frame buffer); its device results feed
      yk_tracker_step_motion (MultiStreamTracker.step_device(..., motion=...)).
'feature_matching' and 'hybrid' (cv2 ORB + RANSAC homography) are not built: they raise.  There
is no CPU fallback: the library must load (YKError otherwise).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L


class BatchedMotionDetector:
    """n_streams GlobalMotionDetector('optical_flow') instances stepped together."""

    def __init__(self, n_streams: int, height: int, width: int, method: str = "optical_flow", device: int = 0):
        if method not in L.GMD_METHODS:
            raise ValueError(f"unknown motion detection method {method!r}")
        if method != "optical_flow":
            raise NotImplementedError(f"method {method!r} needs cv2 ORB + RANSAC findHomography; only 'optical_flow' "
                                      "is built on the device")
        self.S, self.H, self.W, self.device = int(n_streams), int(height), int(width), int(device)
        h = C.c_void_p()
        L.check(L.lib().yk_gmd_create(L.context(self.device), self.S, self.H, self.W, L.GMD_METHODS[method],
                                      C.byref(h)), "yk_gmd_create")
        self._h = h
        self.frames = torch.zeros((self.S, self.H, self.W, 3), dtype=torch.uint8, device=f"cuda:{self.device}")
        self.host_motion = np.zeros(self.S, L.MOTION_DTYPE)
        self.host_stats = np.zeros(self.S, L.GMD_STATS_DTYPE)
        dm = C.c_void_p()
        L.check(L.lib().yk_gmd_outputs(self._h, C.byref(dm)), "yk_gmd_outputs")
        self.motion_ptr = dm.value  # device yk_motion[n_streams] of the last detect

    def __del__(self):
        h = getattr(self, "_h", None)
        try:
            if h is not None and h.value and L._lib is not None:
                L.lib().yk_gmd_destroy(h)
        except Exception:
            pass
        self._h = None

    def reset(self):
        L.check(L.lib().yk_gmd_reset(self._h, L.current_stream(self.device)), "yk_gmd_reset")

    def reset_stats(self):
        L.check(L.lib().yk_gmd_reset_stats(self._h, L.current_stream(self.device)), "yk_gmd_reset_stats")

    def set_thresholds(self, global_motion_threshold: float, reset_motion_threshold: float):
        L.check(L.lib().yk_gmd_set_thresholds(self._h, float(global_motion_threshold), float(reset_motion_threshold)),
                "yk_gmd_set_thresholds")

    def detect_device(self, frames: torch.Tensor | None = None, out: int = 0):
        """detect_motion on every stream's frame (device uint8 [S, H, W, 3] BGR).  out: device
        address of a yk_motion[S] record to write instead of the detector's own (motion_ptr)."""
        f = self.frames if frames is None else frames
        if f.dtype != torch.uint8 or tuple(f.shape) != (self.S, self.H, self.W, 3) or not f.is_contiguous():
            raise ValueError(f"frames must be a contiguous uint8 tensor of shape {(self.S, self.H, self.W, 3)}")
        L.check(L.lib().yk_gmd_detect(self._h, L.ptr(f), C.c_void_p(out), L.current_stream(self.device)),
                "yk_gmd_detect")

    def detect_window(self, frames, out: int = 0):
        """detect_device on each of `frames` (a list of n device uint8 [S, H, W, 3] tensors: n
        consecutive steps) in one launch sequence (yk_gmd_detect_window): the same n records, in
        frame order, at `out` (device address of yk_motion[n][S]; 0: the detector's own buffer).
        A detector uses either this or detect_device until reset()."""
        shp = (self.S, self.H, self.W, 3)
        for f in frames:
            if f.dtype != torch.uint8 or tuple(f.shape) != shp or not f.is_contiguous():
                raise ValueError(f"frames must be contiguous uint8 tensors of shape {shp}")
        ptrs = (C.c_void_p * len(frames))(*[f.data_ptr() for f in frames])
        L.check(L.lib().yk_gmd_detect_window(self._h, ptrs, len(frames), C.c_void_p(out), L.current_stream(self.device)),
                "yk_gmd_detect_window")

    def detect_host(self, frames):
        """Host frames (one [H, W, 3] uint8 BGR array per stream)."""
        if len(frames) != self.S:
            raise ValueError(f"expected {self.S} frames, got {len(frames)}")
        a = np.stack([np.asarray(f, np.uint8) for f in frames])
        if a.shape != (self.S, self.H, self.W, 3):
            raise ValueError(f"frames must be {self.H}x{self.W}x3 uint8 BGR, got {a.shape[1:]}")
        self.frames.copy_(torch.from_numpy(a))
        self.detect_device(self.frames)

    def download(self):
        L.check(L.lib().yk_gmd_download(self._h, L.ptr(self.host_motion), L.ptr(self.host_stats),
                                        L.current_stream(self.device)), "yk_gmd_download")
        return self.host_motion, self.host_stats

    def points(self, stream_index: int = 0):
        """Last corners, LK end points and status of one stream (parity diagnostics)."""
        c = np.zeros((200, 2), np.float32)
        nx = np.zeros((200, 2), np.float32)
        st = np.zeros(200, np.uint8)
        n = C.c_int32()
        L.check(L.lib().yk_gmd_points(self._h, int(stream_index), L.ptr(c), L.ptr(nx), L.ptr(st), C.byref(n),
                                      L.current_stream(self.device)), "yk_gmd_points")
        k = n.value
        return c[:k].copy(), nx[:k].copy(), st[:k].copy()


def motion_tuple(m):
    """A yk_motion record -> detect_motion()'s (is_motion, magnitude, vector, should_reset)."""
    if int(m["magnitude_kind"]) == 1:
        return (np.bool_(m["is_motion"]), np.float32(m["magnitude"]), np.array(m["vector"], np.float32),
                np.bool_(m["should_reset"]))
    return False, 0.0, np.array([0.0, 0.0]), False


def stats_dict(st) -> dict:
    """GlobalMotionDetector.get_stats() (:263-278) from a yk_gmd_stats record."""
    n = int(st["total_detections"])
    mr = int(st["motion_events"]) / n if n else 0.0
    rr = int(st["reset_triggers"]) / n if n else 0.0
    return {"total_detections": n, "motion_events": int(st["motion_events"]),
            "reset_triggers": int(st["reset_triggers"]), "motion_detection_rate": f"{mr:.1%}",
            "reset_trigger_rate": f"{rr:.1%}", "avg_motion_magnitude": f"{float(st['avg_motion_magnitude']):.2f}px"}


class GlobalMotionDetector:
    """GlobalMotionDetector(method='optical_flow') (global_motion_detector.py:11-288), one stream."""

    def __init__(self, method: str = "optical_flow", *, device: int = 0, verbose: bool = False):
        if method not in L.GMD_METHODS:
            raise ValueError(f"unknown motion detection method {method!r}")
        if method != "optical_flow":
            raise NotImplementedError(f"method {method!r} needs cv2 ORB + RANSAC findHomography; only 'optical_flow' "
                                      "is built on the device")
        self.method, self.device = method, int(device)
        self._global_motion_threshold, self._reset_motion_threshold = 30.0, 50.0
        self.consistency_threshold = 0.7
        self._b: BatchedMotionDetector | None = None
        if verbose:
            print(f"✅ 全局运动检测器初始化完成 - 方法: {method}")

    def _detector(self, frame) -> BatchedMotionDetector:
        h, w = frame.shape[:2]
        if self._b is None:
            self._b = BatchedMotionDetector(1, h, w, self.method, self.device)
            self._b.set_thresholds(self._global_motion_threshold, self._reset_motion_threshold)
        elif (self._b.H, self._b.W) != (h, w):
            raise ValueError(f"frame size changed from {self._b.H}x{self._b.W} to {h}x{w} (calcOpticalFlowPyrLK "
                             "needs equal sizes)")
        return self._b

    @property
    def global_motion_threshold(self):
        return self._global_motion_threshold

    @global_motion_threshold.setter
    def global_motion_threshold(self, v):
        self._global_motion_threshold = v
        if self._b is not None:
            self._b.set_thresholds(self._global_motion_threshold, self._reset_motion_threshold)

    @property
    def reset_motion_threshold(self):
        return self._reset_motion_threshold

    @reset_motion_threshold.setter
    def reset_motion_threshold(self, v):
        self._reset_motion_threshold = v
        if self._b is not None:
            self._b.set_thresholds(self._global_motion_threshold, self._reset_motion_threshold)

    def detect_motion(self, frame):
        b = self._detector(frame)
        b.detect_host([frame])
        m, _ = b.download()
        return motion_tuple(m[0])

    @property
    def stats(self) -> dict:
        if self._b is None:
            return {"total_detections": 0, "motion_events": 0, "reset_triggers": 0, "avg_motion_magnitude": 0.0}
        _, st = self._b.download()
        return {"total_detections": int(st[0]["total_detections"]), "motion_events": int(st[0]["motion_events"]),
                "reset_triggers": int(st[0]["reset_triggers"]),
                "avg_motion_magnitude": float(st[0]["avg_motion_magnitude"])}

    def get_stats(self) -> dict:
        if self._b is None:
            return stats_dict(np.zeros(1, L.GMD_STATS_DTYPE)[0])
        _, st = self._b.download()
        return stats_dict(st[0])

    def reset_stats(self):
        if self._b is not None:
            self._b.reset_stats()
