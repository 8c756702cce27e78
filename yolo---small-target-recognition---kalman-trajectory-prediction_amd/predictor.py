"""Device-backed mirror of ``ultralytics.YOLO`` for the detection predict path.

Reference surface (ultralytics/engine/model.py:82-188, 498-557; engine/results.py:240-290,
855-980): ``YOLO(model)`` from a model YAML (scale from the file name, tasks.py:1703-1740)
or a weights file; ``model(source, **kw)`` == ``model.predict(source, **kw)`` returning a
list of ``Results`` whose ``boxes.xyxy / .conf / .cls / .data`` are float32 tensors on the
model's device (so ``.cpu().numpy()`` works as in kalman/aircraft_detection_tracking.py:101-102).
Defaults follow the predictor's effective values: conf 0.25 (model.py:544), iou 0.7,
max_det 300, imgsz 640 (cfg/default.yaml).

Everything from the uint8 frame to the NMS output runs in libyk.so (csrc/detector.hip);
this module stages frames into HBM, keeps one compiled program per frame geometry and
wraps the outputs.  A per-predictor lock mirrors BasePredictor's (predictor.py:149,304).
"""
from __future__ import annotations

import os
import threading
import time

import numpy as np
import torch

from . import _lib as L
from . import arch as A
from . import model as M
from . import weights as Wt

# committed conv plans (bench.py's plans/<scale>_<W>x<H>_i<imgsz>_b<batch>_<dtype>.json): a YOLO
# engine applies the one for its geometry at batch 1 when it exists (YK_PLAN_DIR overrides)
PLAN_DIR = os.environ.get("YK_PLAN_DIR", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                      "plans"))


class _EngineIO:
    """Per-engine device / page-locked buffers of the batch path: the frames are staged through
    one pinned buffer into one device buffer, the forward replays a native hipGraph per batch size
    (yk_detect_graph; its key includes these fixed pointers), and counts come back through pinned
    memory.  Results get their own copies of the detections (the buffers are reused)."""

    def __init__(self, e: M.DeviceModel, max_batch: int, max_det: int):
        p = e.prog
        dev = torch.device("cuda", e.device)
        self.frames = torch.empty((max_batch, p.frame_h, p.frame_w, 3), dtype=torch.uint8, device=dev)
        self.host = torch.empty(self.frames.shape, dtype=torch.uint8, pin_memory=True)
        self.dets = torch.empty((max_batch, max_det, 6), dtype=torch.float32, device=dev)
        self.counts = torch.empty(max_batch, dtype=torch.int32, device=dev)
        self.host_counts = torch.empty(max_batch, dtype=torch.int32, pin_memory=True)


class Boxes:
    """engine/results.py Boxes: data (N, 6) = x1, y1, x2, y2, conf, cls."""

    def __init__(self, boxes, orig_shape):
        if boxes.ndim == 1:
            boxes = boxes[None, :]
        n = boxes.shape[-1]
        assert n in {6, 7}, f"expected 6 or 7 values but got {n}"
        self.data = boxes
        self.orig_shape = orig_shape
        self.is_track = n == 7

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return Boxes(self.data[idx], self.orig_shape)

    @property
    def shape(self):
        return self.data.shape

    @property
    def xyxy(self):
        return self.data[:, :4]

    @property
    def conf(self):
        return self.data[:, -2]

    @property
    def cls(self):
        return self.data[:, -1]

    @property
    def id(self):
        return self.data[:, -3] if self.is_track else None

    @property
    def xywh(self):
        b = self.xyxy
        return torch.cat(((b[:, :2] + b[:, 2:]) / 2, b[:, 2:] - b[:, :2]), 1)

    @property
    def xyxyn(self):
        b = self.xyxy.clone()
        b[:, [0, 2]] /= self.orig_shape[1]
        b[:, [1, 3]] /= self.orig_shape[0]
        return b

    def cpu(self):
        return Boxes(self.data.cpu(), self.orig_shape)

    def numpy(self):
        return Boxes(self.data.cpu().numpy(), self.orig_shape)

    def cuda(self):
        return Boxes(self.data.cuda(), self.orig_shape)

    def to(self, *a, **k):
        return Boxes(self.data.to(*a, **k), self.orig_shape)


class Results:
    """engine/results.py Results for detection: orig_img, orig_shape, boxes, names, path, speed."""

    def __init__(self, orig_img, path, names, boxes=None, speed=None):
        self.orig_img = orig_img
        self.orig_shape = orig_img.shape[:2]
        self.boxes = Boxes(boxes, self.orig_shape) if boxes is not None else None
        self.masks = self.probs = self.keypoints = self.obb = None
        self.speed = speed if speed is not None else {"preprocess": None, "inference": None, "postprocess": None}
        self.names = names
        self.path = path
        self.save_dir = None

    def __len__(self):
        return 0 if self.boxes is None else len(self.boxes)

    def __getitem__(self, idx):
        """Results of the indexed boxes (engine/results.py:292-307, BaseTensor.__getitem__)."""
        r = Results(self.orig_img, self.path, self.names, None, self.speed)
        r.boxes = None if self.boxes is None else self.boxes[idx]
        return r

    def update(self, boxes=None):
        """engine/results.py:327-360: new boxes, clipped to the original image (ops.clip_boxes)."""
        if boxes is not None:
            b = boxes.clone() if isinstance(boxes, torch.Tensor) else torch.as_tensor(boxes)
            h, w = self.orig_shape
            b[..., 0] = b[..., 0].clamp(0, w)
            b[..., 1] = b[..., 1].clamp(0, h)
            b[..., 2] = b[..., 2].clamp(0, w)
            b[..., 3] = b[..., 3].clamp(0, h)
            self.boxes = Boxes(b, self.orig_shape)

    def cpu(self):
        return Results(self.orig_img, self.path, self.names, None if self.boxes is None else self.boxes.data.cpu(),
                       self.speed)


class YOLO:
    """YOLO(model='yolov8s-small.yaml' | 'best.pt') -> detector executed by libyk.so.

    ``model``: a model YAML (scale from the file name, tasks.py:1703-1740) or an ultralytics
    checkpoint (``*.pt``: architecture, scale and fp16 weights read from the pickled
    DetectionModel without ultralytics and without executing the pickle, checkpoint.py).
    ``weights`` (YAML models only): None (seeded synthetic weights in the reference's shapes,
    SURVEY §8d), a state dict in the reference's naming, or a path to one saved with
    torch.save (loaded with weights_only=True).  ``dtype``: 'fp32' (the default: fp32-grade
    arithmetic with the reference's exact SiLU, so the unchanged driver gets the reference's
    decisions up to fp32 near-ties), or the explicit opt-ins
    'bf16' / 'fp8' (faster, not parity-capable: their detections differ from the reference's).
    ``predict(half=True)`` runs the fp16 build (the reference's AutoBackend(fp16=True) ->
    model.half(), nn/autobackend.py:215, engine/predictor.py:172): binary16 weights and
    activations on the f16 matrix cores, fp32 accumulation, its own engine per geometry."""

    def __init__(self, model: str = "yolov8s-small.yaml", task=None, verbose: bool = False, *, weights=None,
                 dtype: str = "fp32", device: int = 0, seed: int = 0, max_batch: int = 8):
        if task not in (None, "detect"):
            raise NotImplementedError(f"task {task!r}: only detection is on this path")
        self.ckpt_meta = None
        if str(model).endswith(".pt"):
            # ultralytics checkpoint (best.pt): the model YAML -- scale included -- comes from the
            # pickled DetectionModel itself (tasks.py:1404-1521), loaded weights_only with inert
            # stand-ins for its classes (checkpoint.py)
            if weights is not None:
                raise ValueError("give either a .pt model or weights=, not both")
            from . import checkpoint as CK

            ydict, weights, self.ckpt_meta = CK.load_checkpoint(str(model))
            self.cfg = str(model)
            self.arch = A.parse_arch(ydict)
        else:
            self.cfg = str(model)
            self.arch = A.parse_arch(A.load_model_dict(self.cfg))
        if weights is None:
            sd = Wt.synthetic_state_dict(self.arch, seed)
        elif isinstance(weights, dict):
            sd = weights
        else:
            sd = torch.load(weights, map_location="cpu", weights_only=True)
            if not isinstance(sd, dict) or not any(k.startswith("model.") for k in sd):
                raise ValueError(f"{weights}: expected a state dict with 'model.*' keys")
        self.state_dict = sd
        self.dtype, self.device, self.max_batch = dtype, int(device), int(max_batch)
        self.names = {i: f"class{i}" for i in range(self.arch.nc)}
        if self.arch.nc == 1:
            self.names = {0: "aircraft"}
        self.task = "detect"
        self.overrides = {"conf": 0.25, "iou": 0.7, "max_det": 300, "imgsz": 640}
        self._engines = {}
        self._io = {}
        self.plans = {}  # engine key -> conv plan file applied (None: the kernels' heuristic)
        self._lock = threading.Lock()
        self._staging = None

    # -- engines ------------------------------------------------------------------
    def _key(self, frame_h, frame_w, imgsz, max_det, dtype=None):
        k = (frame_h, frame_w, imgsz if isinstance(imgsz, int) else tuple(imgsz), max_det)
        return k if dtype in (None, self.dtype) else k + (dtype,)

    def engine(self, frame_h: int, frame_w: int, imgsz=640, max_det: int = 300, dtype=None) -> M.DeviceModel:
        dtype = self.dtype if dtype is None else dtype
        key = self._key(frame_h, frame_w, imgsz, max_det, dtype)
        e = self._engines.get(key)
        if e is None:
            prog = M.Program(self.arch, self.state_dict, frame_h, frame_w, imgsz, self.max_batch, dtype, max_det)
            e = M.DeviceModel(prog, self.device)
            self.plans[key] = self._apply_plan(e, prog, imgsz)
            self._engines[key] = e
            self._io[key] = _EngineIO(e, self.max_batch, max_det)
        return e

    def _apply_plan(self, e: M.DeviceModel, prog: M.Program, imgsz):
        """The committed batch-1 conv plan of this geometry (tuned kernels; held to the oracle
        chain by tests/test_bench_pipeline_gpu.py) if one exists and fits the program."""
        import json

        if not self.arch.scale or not isinstance(imgsz, int):
            return None
        dt = prog.dtype
        path = os.path.join(PLAN_DIR, f"{self.arch.scale}_{prog.frame_w}x{prog.frame_h}_i{imgsz}_b1_{dt}.json")
        if dt == "fp16" and not os.path.exists(path):
            # the fp16 build runs the bf16 build's kernels with the f16 MFMA (same shapes, same rate):
            # the committed bf16 plan is its plan too
            dt = "bf16"
            path = os.path.join(PLAN_DIR, f"{self.arch.scale}_{prog.frame_w}x{prog.frame_h}_i{imgsz}_b1_bf16.json")
        if not os.path.exists(path):
            return None
        with open(path) as f:
            pl = json.load(f)
        if pl.get("dtype", dt) != dt or len(pl.get("plan", ())) != len(prog.ops):
            return None
        e.load_plan(pl["batch"], pl["plan"])
        return path

    # -- predict --------------------------------------------------------------------
    def __call__(self, source=None, stream: bool = False, **kwargs):
        return self.predict(source, stream, **kwargs)

    def predict(self, source=None, stream: bool = False, conf=None, iou=None, imgsz=None, max_det=None,
                classes=None, agnostic_nms=False, half=False, device=None, verbose=False, batch=1, **kwargs):
        conf = self.overrides["conf"] if conf is None else conf
        iou = self.overrides["iou"] if iou is None else iou
        imgsz = self.overrides["imgsz"] if imgsz is None else imgsz
        max_det = self.overrides["max_det"] if max_det is None else max_det
        assert 0 <= conf <= 1, f"Invalid Confidence threshold {conf}, valid values are between 0.0 and 1.0"
        assert 0 <= iou <= 1, f"Invalid IoU {iou}, valid values are between 0.0 and 1.0"
        dtype = "fp16" if half else None  # AutoBackend(fp16=half): model.half() (nn/autobackend.py:215)
        if self.arch.nc != 1:
            raise NotImplementedError("only single-class detection heads are on this path")
        # nc == 1: every candidate is class 0, so non_max_suppression's class filter (utils/nms.py:128-132),
        # applied before NMS, keeps all candidates or none, and agnostic_nms (class offset c * max_wh with
        # c == 0, :144) changes nothing -- both are exact here without a kernel change.
        del agnostic_nms
        if classes is not None:
            classes = [int(c) for c in (classes if isinstance(classes, (list, tuple, set)) else [classes])]
        items = self._frames(source)
        paths = [p for p, _ in items]
        frames = [f for _, f in items]
        with self._lock:
            out = []
            for i in range(0, len(frames), self.max_batch):
                out.extend(self._predict_batch(frames[i:i + self.max_batch], conf, iou, imgsz, max_det, classes,
                                               paths[i:i + self.max_batch], dtype))
        return iter(out) if stream else out

    @staticmethod
    def _frames(source):
        """Source -> list of (path, HxWx3 uint8 BGR): ndarray(s), PIL images, image files,
        directories, globs and .npy / .y4m frame stacks (frames.py; loaders.py:309-563)."""
        from . import frames as FR

        return FR.load_source(source)

    def _predict_batch(self, frames, conf, iou, imgsz, max_det, classes, paths=None, dtype=None):
        paths = paths or [f"image{b}.jpg" for b in range(len(frames))]
        shapes = {f.shape for f in frames}
        if len(shapes) != 1:
            out = []
            for f, p in zip(frames, paths):
                out.extend(self._predict_batch([f], conf, iou, imgsz, max_det, classes, [p], dtype))
            return out
        h, w, c = frames[0].shape
        if c != 3 or frames[0].dtype != np.uint8:
            raise ValueError("frames must be uint8 HxWx3 (BGR)")
        t0 = time.perf_counter()
        md = max(max_det, 1)
        eng = self.engine(h, w, imgsz, md, dtype)
        io = self._io[self._key(h, w, imgsz, md, dtype)]
        B = len(frames)
        hb = io.host.numpy()
        for b, f in enumerate(frames):  # page-locked staging, then one DMA of the batch
            hb[b] = f
        io.frames[:B].copy_(io.host[:B], non_blocking=True)
        t1 = time.perf_counter()
        eng.detect(io.frames[:B], conf, iou, md, io.dets[:B], io.counts[:B], graph=True)
        io.host_counts[:B].copy_(io.counts[:B], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        cnt = io.host_counts[:B].tolist()
        t2 = time.perf_counter()
        res = []
        for b in range(B):
            n = min(int(cnt[b]), max_det)
            if classes is not None and 0 not in classes:
                n = 0  # the class filter ran before NMS in the reference: no candidate survives
            d = io.dets[b, :n].clone()  # the engine's buffer is reused by the next call
            res.append(Results(frames[b], paths[b], self.names, boxes=d))
        t3 = time.perf_counter()
        sp = {"preprocess": (t1 - t0) * 1e3 / B, "inference": (t2 - t1) * 1e3 / B, "postprocess": (t3 - t2) * 1e3 / B}
        for r in res:
            r.speed = sp
        return res

    # -- track (engine/model.py:559-613, trackers/track.py:18-121) ------------------------------
    def track(self, source=None, stream: bool = False, persist: bool = False, tracker="botsort.yaml", **kwargs):
        """model.track(): predict with conf defaulting to 0.1 and batch 1, then every result through
        the tracker on the device (bytetrack.hip): on_predict_start creates one tracker per call
        unless `persist` keeps the existing one (track.py:18-63, one tracker for non-stream
        sources); on_predict_postprocess_end resets it when the source path changes (unless
        persist), updates it with the result's boxes and replaces the result by the tracked subset
        with boxes [x1, y1, x2, y2, id, conf, cls] (track.py:66-100).  `tracker`: 'botsort.yaml'
        (the cfg default, with its sparseOptFlow GMC on the device) / 'bytetrack.yaml' / a YAML
        path / dict.  The frame goes to the tracker's update (track.py:93, im0s[i]) for the GMC."""
        from . import bytetrack as BT

        kwargs["conf"] = kwargs.get("conf") or 0.1
        kwargs["batch"] = kwargs.get("batch") or 1
        if not (persist and getattr(self, "trackers", None)):
            cfg = BT.load_tracker_cfg(tracker)
            kind = BT.BOTSORT if cfg.tracker_type == "botsort" else BT.BYTETracker
            self.trackers = [kind(cfg, frame_rate=30, device=self.device)]
            self.vid_path = [None]
        results = self.predict(source, stream=False, **kwargs)
        trk = self.trackers[0]
        for i, r in enumerate(results):
            vid_path = os.path.basename(str(r.path))
            if not persist and self.vid_path[0] != vid_path:
                trk.reset()
                self.vid_path[0] = vid_path
            tracks = trk.update(r.boxes.cpu().numpy(), r.orig_img)
            if len(tracks) == 0:
                continue
            idx = tracks[:, -1].astype(int)
            results[i] = r[torch.as_tensor(idx, device=r.boxes.data.device)]
            results[i].update(boxes=torch.as_tensor(tracks[:, :-1], device=r.boxes.data.device))
        return iter(results) if stream else results

    def fuse(self, verbose=True):
        return self  # Conv+BN is always fused at program build (weights.fuse_conv_bn)

    def info(self, verbose=True):
        n = sum(v.numel() for k, v in self.state_dict.items() if not k.endswith("num_batches_tracked"))
        return {"layers": len(self.arch.layers), "parameters": n, "scale": self.arch.scale}
