"""Rate of the unchanged reference driver loop on the drop-in surface.

kalman/aircraft_detection_tracking.py:88-131 per frame, through the compat packages exactly as the
driver imports them: ``results = model(frame, verbose=False)`` (batch 1, the drop-in fp32 default),
``results[0].boxes.xyxy.cpu().numpy()`` / ``.conf.cpu().numpy()``, the ``score > 0.1`` filter into a
list of [x1, y1, x2, y2, score], ``tracks = tracker.update(detections)`` (list of dicts) and the
driver's state-change bookkeeping.  Frames are host uint8 BGR arrays (what cv2.VideoCapture.read()
hands the driver), so every frame crosses PCIe as in the reference.

Reported per frame: wall ms, and the split
  pre      YOLO.predict up to the frame being in HBM (stack, H2D copy)     -- Results.speed['preprocess']
  infer    the device forward + NMS and the count read-back                -- Results.speed['inference']
  post     Results / Boxes construction                                    -- Results.speed['postprocess']
  boxes    the driver's .cpu().numpy() reads and its detection list
  tracker  EnhancedMultiTargetTracker.update (H2D, step, D2H, dicts)
  driver   the driver's state-change / status loop over the dicts
beside the oracle chain on the host cores (torch-CPU fp32 YOLOv8s+P2 + the numpy tracker, the
reference's CPU path) on a bounded sample of the same frames.

usage: python tools/dropin_bench.py [--frames 300] [--preroll 40] [--targets 40] [--cpu-frames 20]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def driver_loop(model, tracker, frames, timed_from, split):
    """The driver's per-frame body (aircraft_detection_tracking.py:96-131); returns live-track
    counts of the timed frames."""
    last, changes, live = {}, 0, []
    for i, frame in enumerate(frames):
        timed = i >= timed_from
        t0 = time.perf_counter()
        results = model(frame, verbose=False)
        t1 = time.perf_counter()
        detections = []
        if len(results) > 0 and results[0].boxes is not None:
            boxes = results[0].boxes.xyxy.cpu().numpy()
            scores = results[0].boxes.conf.cpu().numpy()
            for box, score in zip(boxes, scores):
                if score > 0.1:
                    detections.append([box[0], box[1], box[2], box[3], score])
        t2 = time.perf_counter()
        tracks = tracker.update(detections)
        t3 = time.perf_counter()
        cur = {}
        for tr in tracks:
            cur[tr["track_id"]] = tr["status"]
            if tr["track_id"] in last and last[tr["track_id"]] != tr["status"]:
                changes += 1
        last = cur
        t4 = time.perf_counter()
        if timed:
            sp = results[0].speed if len(results) else {}
            for k in ("preprocess", "inference", "postprocess"):
                split[k] += float(sp.get(k) or 0.0) / 1e3
            split["predict_call"] += t1 - t0
            split["boxes"] += t2 - t1
            split["tracker"] += t3 - t2
            split["driver"] += t4 - t3
            live.append(len(tracks))
    return live


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--preroll", type=int, default=40, help="untimed frames first (track load, warm-up)")
    ap.add_argument("--targets", type=int, default=40)
    ap.add_argument("--cpu-frames", type=int, default=20, help="timed frames of the oracle CPU chain (0: skip)")
    ap.add_argument("--dtype", default=None, help="YOLO dtype (default: the drop-in default)")
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    sys.path.insert(0, os.path.join(REPO, PKG, "compat"))
    from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker
    from ultralytics import YOLO
    sys.path.pop(0)

    n = a.preroll + a.frames
    sc = P.synth.Scene(seed=4, n_targets=a.targets, n_frames=n + 1)
    frames = [sc.frame(t) for t in range(n)]  # host uint8 BGR, as cv2 hands them over
    model = YOLO("yolov8s-small.yaml", **({"dtype": a.dtype} if a.dtype else {}))
    tracker = EnhancedMultiTargetTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    split = dict.fromkeys(("preprocess", "inference", "postprocess", "predict_call", "boxes", "tracker", "driver"), 0.0)
    # the tracker update's own phases, timed inside the same update calls (so they add up to the
    # split's "tracker" entry): H2D + step launch, download (counts / stats / rows), rows -> dicts
    T = importlib.import_module(PKG + ".tracker")
    ph = dict.fromkeys(("step_host", "download", "dicts"), 0.0)
    gate = {"on": False}

    def timed(fn, key):
        def w(*args, **kw):
            t = time.perf_counter()
            r = fn(*args, **kw)
            if gate["on"]:
                ph[key] += time.perf_counter() - t
            return r
        return w

    tracker._core.step_host = timed(tracker._core.step_host, "step_host")
    tracker._core.download = timed(tracker._core.download, "download")
    T.rows_to_dicts = timed(T.rows_to_dicts, "dicts")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    live = driver_loop(model, tracker, frames[: a.preroll], 0, dict.fromkeys(split, 0.0))
    gate["on"] = True
    live = driver_loop(model, tracker, frames[a.preroll:], 0, split)
    torch.cuda.synchronize()
    # the timed part is the frames from `preroll` on: re-time them alone
    total_split = sum(split[k] for k in ("predict_call", "boxes", "tracker", "driver"))
    fps = a.frames / total_split
    out = {"metric": "drop-in driver loop frames/s (aircraft_detection_tracking.py:88-131, batch 1, host frames)",
           "value": round(fps, 1), "unit": "frames/s", "frames": a.frames, "preroll": a.preroll,
           "dtype": model.dtype, "targets": a.targets,
           "live_tracks": {"min": int(min(live)), "mean": round(float(np.mean(live)), 1), "max": int(max(live))},
           "ms_per_frame": round(total_split * 1e3 / a.frames, 4),
           "split_ms_per_frame": {k: round(v * 1e3 / a.frames, 4) for k, v in split.items()},
           "wall_incl_preroll_s": round(time.perf_counter() - t0, 3)}
    out["tracker_split_ms_per_frame"] = {k: round(v * 1e3 / a.frames, 4) for k, v in ph.items()}
    if a.cpu_frames > 0:
        from oracle import detector_ref as D
        from oracle.tracker_ref import RefMultiTracker

        torch.set_num_threads(max(1, min(8, (os.cpu_count() or 2) - 1)))
        ar = model.arch
        layers = [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
                  for Ly in ar.layers]
        ref = D.RefDetector(layers, model.state_dict, P.arch.detect_strides(ar))
        trk = RefMultiTracker(150, 1, 0.1)
        m = min(a.cpu_frames, n)
        det_s = trk_s = 0.0
        for i in range(m + 4):
            ta = time.perf_counter()
            want, _ = D.predict(ref, [frames[i]])
            dets = [[b[0], b[1], b[2], b[3], b[4]] for b in want[0][:, :5].numpy() if b[4] > 0.1]
            tb = time.perf_counter()
            trk.update(dets)
            tc = time.perf_counter()
            if i >= 4:
                det_s += tb - ta
                trk_s += tc - tb
        out["cpu_baseline"] = {"value": round(m / (det_s + trk_s), 2), "unit": "frames/s", "kind": "port",
                               "cores": torch.get_num_threads(),
                               "split_ms_per_frame": {"detector_nms": round(det_s * 1e3 / m, 2),
                                                      "tracker": round(trk_s * 1e3 / m, 2)},
                               "sample": f"{m} frames after 4 warm-up frames of the same sequence"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
