#!/usr/bin/env python3
"""Conditioning of the driver-loop test scene (tests/test_pipeline_gpu.py::_driver_scene) per
scene seed: runs the oracle chain (torch-CPU detector -> numpy RefMultiTracker(150, 1, 0.1)) and
reports the smallest association margin (tests/gpu_helpers.assign_margin) over all frames.

usage: driver_scene_margin.py [--frames 160] [--seeds 4,5,6]
"""
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
    ap.add_argument("--seeds", default="4,5,6,7")
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    from gpu_helpers import assign_margin
    from test_pipeline_gpu import _driver_scene, _layers
    from oracle import detector_ref as D
    from oracle.tracker_ref import RefMultiTracker

    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    ref = D.RefDetector(_layers(ar), sd, P.arch.detect_strides(ar))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for seed in (int(v) for v in a.seeds.split(",")):
        sc = _driver_scene(P, a.frames, seed)
        trk = RefMultiTracker(150, 1, 0.1, stable_ties=True, fast_iou=True)
        worst, at = np.inf, -1
        for t in range(a.frames):
            w = D.predict(ref, [sc.frame(t)])[0][0][:, :5].numpy()
            trk.update([[b[0], b[1], b[2], b[3], b[4]] for b in w])
            if trk.last_iou is not None:
                m = assign_margin(trk.last_iou, 0.1)
                if m < worst:
                    worst, at = m, t
        st = trk.stats
        print({"seed": seed, "min_margin": worst, "at_frame": at, "terminated": st["total_tracks_terminated"],
               "recoveries": st["successful_recoveries"]}, flush=True)


if __name__ == "__main__":
    main()
