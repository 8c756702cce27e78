#!/usr/bin/env python3
"""Driver-loop divergence probe: runs the drop-in YOLO (batch 1, committed b1 plan) on the
test_pipeline_gpu driver scene and saves every frame's detections next to the torch-CPU oracle's
(npz), so the first tracker decision that differs can be replayed on the host with the oracle
tracker (which detection, which IoU against the gate).

usage: driver_diag.py [--frames 160] [--out gpurun_out/driver_dets.npz]
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=160)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "driver_dets.npz"))
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    from test_pipeline_gpu import _driver_scene, _layers
    from oracle import detector_ref as D

    sys.path.insert(0, os.path.join(REPO, PKG, "compat"))
    from ultralytics import YOLO
    sys.path.pop(0)
    sc = _driver_scene(P, a.frames)
    frames = [sc.frame(t) for t in range(a.frames)]
    model = YOLO("yolov8s-small.yaml")
    ref = D.RefDetector(_layers(model.arch), model.state_dict, P.arch.detect_strides(model.arch))
    torch.set_num_threads(16)
    out = {}
    for t, fr in enumerate(frames):
        r = model(fr, verbose=False)[0]
        g = np.concatenate([r.boxes.xyxy.cpu().numpy(), r.boxes.conf.cpu().numpy()[:, None]], 1)
        w = D.predict(ref, [fr])[0][0][:, :5].numpy()
        out[f"gpu_{t}"] = g.astype(np.float32)
        out[f"ref_{t}"] = w.astype(np.float32)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez(a.out, **out)
    print("saved", a.out, len(frames))


if __name__ == "__main__":
    main()
