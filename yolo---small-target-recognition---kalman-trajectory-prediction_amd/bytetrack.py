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
separate processes.  BoT-SORT's GMC (gmc.py): 'sparseOptFlow' (the botsort.yaml default) runs
on the device (csrc/gmd.hip yk_gmc_apply: corners, pyramidal LK, RANSAC + Levenberg-Marquardt
estimateAffinePartial2D) and its warp is applied inside the step (yk_bt_step_warp); 'none' applies
the identity, as the reference's GMC.apply returns np.eye(2, 3); 'orb' / 'sift' / 'ecc' (cv2
feature / ECC internals) raise.  The ReID branch (with_reid) is not built.  There is no CPU
fallback: the library must load (YKError otherwise).
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

    def step_device(self, dets: torch.Tensor, counts: torch.Tensor, warp: int | None = None):
        """One update() of every stream from device-resident detections (no host round trip).
        warp: device address of float64 [S][2][3] GMC warps (BoT-SORT), or None."""
        if dets.dtype != torch.float32 or dets.shape != (self.S, self.max_dets, 6) or not dets.is_contiguous():
            raise ValueError(f"dets must be a contiguous float32 tensor of shape {(self.S, self.max_dets, 6)}")
        if counts.dtype != torch.int32 or counts.shape != (self.S,):
            raise ValueError(f"counts must be an int32 tensor of shape ({self.S},)")
        L.check(L.lib().yk_bt_step_warp(self._h, C.c_void_p(dets.data_ptr()), C.c_void_p(counts.data_ptr()),
                                        C.c_void_p(warp or 0), L.current_stream(self.device)), "yk_bt_step")

    def step(self, per_stream, warp: int | None = None):
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
        self.step_device(self.dets, self.counts, warp)

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


class GMC:
    """GMC(method='sparseOptFlow' | 'none', downscale=2) of ultralytics/trackers/utils/gmc.py:48-353
    for n_streams streams on the device (yk_gmd with YK_GMD_SPARSE_OPTFLOW; created at the first
    frame, when the frame size is known).  apply(raw_frame) returns the 2x3 float64 warp like the
    reference; apply_device(frames) leaves it in HBM for the BoT-SORT step."""

    def __init__(self, method: str = "sparseOptFlow", downscale: int = 2, n_streams: int = 1, device: int = 0):
        if method not in ("sparseOptFlow", "none", None):
            raise NotImplementedError(f"GMC method {method!r} needs cv2's ORB / SIFT / ECC internals (absent); "
                                      "'sparseOptFlow' and 'none' are built")
        if method == "sparseOptFlow" and downscale != 2:
            raise NotImplementedError("GMC sparseOptFlow is built for downscale 2 (the INTER_AREA fast path)")
        self.method, self.downscale, self.S, self.device = method, max(1, downscale), int(n_streams), int(device)
        self._h = None
        self._hw = None
        dev = torch.device("cuda", self.device)
        self.identity = torch.tensor([[1.0, 0.0, 0.0, 0.0, 1.0, 0.0]] * self.S, dtype=torch.float64, device=dev)
        self.warp = torch.zeros((self.S, 6), dtype=torch.float64, device=dev)
        self.frames = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().yk_gmd_destroy(h)
            except Exception:
                pass
            self._h = None

    def reset_params(self):
        """gmc.py:347-353: forget the previous frame and keypoints."""
        if self._h is not None:
            L.check(L.lib().yk_gmd_reset(self._h, L.current_stream(self.device)), "yk_gmd_reset")

    def _frames_device(self, frames) -> torch.Tensor:
        if isinstance(frames, np.ndarray):
            frames = torch.from_numpy(np.ascontiguousarray(frames))
        if frames.dim() == 3:
            frames = frames.unsqueeze(0)
        if frames.dtype != torch.uint8 or frames.shape[0] != self.S or frames.shape[3] != 3:
            raise ValueError(f"frames must be uint8 [{self.S}, H, W, 3] BGR")
        if not frames.is_cuda:
            if self.frames is None or self.frames.shape != frames.shape:
                self.frames = torch.empty(frames.shape, dtype=torch.uint8, device=f"cuda:{self.device}")
            self.frames.copy_(frames)
            frames = self.frames
        return frames.contiguous()

    def apply_device(self, frames) -> int:
        """GMC.apply of every stream's frame (uint8 [S, H, W, 3] BGR, host or device); returns the
        device address of the float64 [S][2][3] warps."""
        if self.method != "sparseOptFlow":
            return self.identity.data_ptr()
        f = self._frames_device(frames)
        hw = (int(f.shape[1]), int(f.shape[2]))
        if hw[0] % 2 or hw[1] % 2 or min(hw) < 64:
            # the device GMC restates cv2.resize's exact-1/2 INTER_AREA fast path only; an odd or tiny
            # frame (e.g. 1242x375) would take cv2's general INTER_LINEAR path, not restated here.
            # Like the reference's identity fallbacks (gmc.py:155-158, 297-311) the warp is then the identity,
            # with one warning, instead of failing the whole track() call.
            if not getattr(self, "_warned_size", False):
                import warnings

                warnings.warn(f"GMC sparseOptFlow: frame size {hw[1]}x{hw[0]} is not even and >= 64; "
                              "using the identity warp for this stream", RuntimeWarning, stacklevel=2)
                self._warned_size = True
            return self.identity.data_ptr()
        if self._h is None or self._hw != hw:
            if self._h is not None:
                L.lib().yk_gmd_destroy(self._h)
            h = C.c_void_p()
            L.check(L.lib().yk_gmd_create(L.context(self.device), self.S, hw[0], hw[1], L.GMD_SPARSE_OPTFLOW,
                                          C.byref(h)), "yk_gmd_create")
            self._h, self._hw = h, hw
        L.check(L.lib().yk_gmc_apply(self._h, C.c_void_p(f.data_ptr()), C.c_void_p(self.warp.data_ptr()),
                                     L.current_stream(self.device)), "yk_gmc_apply")
        return self.warp.data_ptr()

    def apply(self, raw_frame, detections=None) -> np.ndarray:
        """The 2x3 warp of one frame (stream 0), float64, like the reference's GMC.apply."""
        ptr = self.apply_device(raw_frame)
        src = self.identity if ptr == self.identity.data_ptr() else self.warp
        return src[0].cpu().numpy().reshape(2, 3)

    def info(self) -> np.ndarray:
        """[S, 5]: tracked points, RANSAC inliers, RANSAC iterations, LM iterations, state."""
        out = np.zeros((self.S, 5), np.int32)
        if self._h is not None:
            L.check(L.lib().yk_gmc_info(self._h, L.ptr(out), L.current_stream(self.device)), "yk_gmc_info")
        return out

    def points(self, stream_index: int = 0):
        """(corners [n, 2], LK end points [n, 2], status [n]) of the last apply (the previous frame's
        keypoints tracked into the current one)."""
        M = 1000
        c, nx, st = np.zeros((M, 2), np.float32), np.zeros((M, 2), np.float32), np.zeros(M, np.uint8)
        n = C.c_int32()
        L.check(L.lib().yk_gmd_points(self._h, int(stream_index), L.ptr(c), L.ptr(nx), L.ptr(st), C.byref(n),
                                      L.current_stream(self.device)), "yk_gmd_points")
        return c[:n.value], nx[:n.value], st[:n.value]


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
        # BOTSORT.__init__ (bot_sort.py:198): self.gmc = GMC(method=args.gmc_method)
        self.gmc = GMC(getattr(cfg, "gmc_method", "none"), device=device) if self.kind == "botsort" else None
        self.frame_id = 0

    def reset(self):
        self._b.reset()
        if self.gmc is not None:
            self.gmc.reset_params()  # BOTSORT.reset (bot_sort.py:246-249)
        self.frame_id = 0

    def update(self, results, img=None, feats=None) -> np.ndarray:
        """byte_tracker.py:299-410: with an image, BoT-SORT applies its GMC warp (identity for
        gmc_method 'none') to the predicted pool and the unconfirmed tracks (:333-340)."""
        self.frame_id += 1
        warp = self.gmc.apply_device(img) if (self.gmc is not None and img is not None) else None
        self._b.step([results], warp)
        return self._b.download()[0]


class BOTSORT(BYTETracker):
    """BOTSORT(args, frame_rate=30) of ultralytics/trackers/bot_sort.py:156 with its GMC, without ReID."""

    kind = "botsort"
