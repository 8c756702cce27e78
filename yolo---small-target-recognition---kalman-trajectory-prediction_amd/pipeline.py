"""End-to-end detect-and-track step for S independent video streams on one GPU.

One step = the reference driver's per-frame body (kalman/aircraft_detection_tracking.py:96-109)
for every stream at once: ``model(frame)`` for S frames as one batch (yk_detect), then one
``tracker.update(detections)`` per stream (yk_tracker_step, one workgroup per stream), with
the NMS output handed to the tracker in HBM (rows [x1, y1, x2, y2, conf, cls] float32, the
reference's np.float32 detections).  The driver's ``score > 0.1`` filter (:105) is a no-op
at conf >= 0.1 and is checked, not executed.  The detector (~90 launches) replays as one
native hipGraph (yk_detect_graph); the tracker is one more launch.

``pipelined=True`` runs the tracker on its own HIP stream: detector(t+1) does not depend on
tracker state, so it starts while tracker(t) is still running.  Detections are
double-buffered; detector(t+2) waits for tracker(t) to have read its buffer.  Results are
identical to the serial order (the tracker still sees frames in order on one stream).
"""
from __future__ import annotations

import numpy as np
import torch

from . import arch as A
from . import model as M
from . import tracker as T
from . import weights as Wt


class StreamPipeline:
    def __init__(self, model_cfg: str = "yolov8s-small.yaml", n_streams: int = 8, frame_hw=(512, 640),
                 dtype: str = "bf16", weights=None, seed: int = 0, conf: float = 0.25, iou: float = 0.7,
                 max_det: int = 300, max_lost_frames: int = 150, min_hits: int = 1, iou_threshold: float = 0.1,
                 max_tracks: int = 512, device: int = 0, pipelined: bool = False, imgsz=640):
        if conf < 0.1:
            raise ValueError("conf < 0.1 would need the driver's score > 0.1 filter on the device path")
        self.S, self.device = int(n_streams), int(device)
        self.conf, self.iou, self.max_det = float(conf), float(iou), int(max_det)
        ar = A.parse_arch(A.load_model_dict(model_cfg))
        sd = weights if weights is not None else Wt.synthetic_state_dict(ar, seed)
        self.prog = M.Program(ar, sd, frame_hw[0], frame_hw[1], imgsz, self.S, dtype, self.max_det)
        self.model = M.DeviceModel(self.prog, self.device)
        self.tracker = T.MultiStreamTracker(self.S, max_lost_frames, min_hits, iou_threshold, max_tracks,
                                            self.max_det, self.device)
        dev = torch.device("cuda", self.device)
        self.frames = torch.zeros((self.S, frame_hw[0], frame_hw[1], 3), dtype=torch.uint8, device=dev)
        self._dets = torch.zeros((2, self.S, self.max_det, 6), dtype=torch.float32, device=dev)
        self._counts = torch.zeros((2, self.S), dtype=torch.int32, device=dev)
        self._k = 0  # detection buffer the next step writes
        self.pipelined = bool(pipelined)
        self.trk_stream = torch.cuda.Stream(dev) if self.pipelined else None
        self._ev_det = [torch.cuda.Event(), torch.cuda.Event()]
        self._ev_trk = [torch.cuda.Event(), torch.cuda.Event()]
        self._trk_pending = [False, False]
        self.graph = None

    @property
    def dets(self) -> torch.Tensor:
        """Detections [S, max_det, 6] of the most recent step."""
        return self._dets[self._k ^ 1]

    @property
    def counts(self) -> torch.Tensor:
        return self._counts[self._k ^ 1]

    def capture(self, tune: bool = True):
        """Autotune the conv kernels for this batch (on the current frames), then build and warm
        the detector's native hipGraph; later steps replay it."""
        if tune:
            self.model.autotune(self.frames, self.conf)
        self.graph = True
        for k in range(2):  # one graph per detection buffer
            self.model.detect(self.frames, self.conf, self.iou, self.max_det, self._dets[k], self._counts[k], graph=True)
        torch.cuda.synchronize(self.device)
        return self.graph

    def step(self):
        k = self._k
        cur = torch.cuda.current_stream(self.device)
        if self._trk_pending[k]:  # tracker(t-2) still reads buffer k
            cur.wait_event(self._ev_trk[k])
            self._trk_pending[k] = False
        self.model.detect(self.frames, self.conf, self.iou, self.max_det, self._dets[k], self._counts[k],
                          graph=bool(self.graph))
        if self.pipelined:
            self._ev_det[k].record(cur)
            self.trk_stream.wait_event(self._ev_det[k])
            with torch.cuda.stream(self.trk_stream):
                self.tracker.step_device(self._dets[k], self._counts[k])
            self._ev_trk[k].record(self.trk_stream)
            self._trk_pending[k] = True
        else:
            self.tracker.step_device(self._dets[k], self._counts[k])
        self._k ^= 1

    def sync(self):
        """Wait for every launched step (detector and tracker streams)."""
        torch.cuda.synchronize(self.device)

    def run(self, frames: torch.Tensor):
        """frames [S, H, W, 3] uint8 (device) -> one step."""
        self.frames.copy_(frames, non_blocking=True)
        self.step()

    def stats(self):
        self.sync()
        _, counts, stats = self.tracker.download()
        return counts.copy(), stats.copy()

    def flops_per_frame(self) -> int:
        return int(sum(self.prog.op_flops(1)))
