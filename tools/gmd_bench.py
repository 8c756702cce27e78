"""Throughput of the device global camera-motion detector (csrc/gmd.hip) and of the
motion-compensated tracker step with frames (detect_motion + yk_tracker_step_motion).

Frames are synthetic camera pans (tests/gmd_helpers.py) resident in HBM; each step runs
detect_motion on one frame per stream.  Prints one JSON line per configuration:
    python tools/gmd_bench.py [--streams 1 8] [--steps 200] [--hw 512x640]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--hw", default="512x640")
    ap.add_argument("--frames", type=int, default=24)
    a = ap.parse_args()
    import importlib

    from gmd_helpers import camera_sequence

    pkg = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
    M = importlib.import_module(pkg.__name__ + ".motion")
    L = pkg._lib
    H, W = (int(v) for v in a.hw.split("x"))
    for S in a.streams:
        seqs = [camera_sequence(s, a.frames, h=H, w=W, whip_at=(a.frames // 2,))[0] for s in range(S)]
        dev = torch.from_numpy(np.stack(seqs, axis=1)).cuda()  # [F, S, H, W, 3]
        det = M.BatchedMotionDetector(S, H, W)
        ms = pkg.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=512, max_dets=64, policy=L.POLICY_MOTION_RESET)
        rng = np.random.default_rng(0)
        dets = torch.from_numpy(rng.uniform(0, 600, (S, 64, 6)).astype(np.float32)).cuda()
        dets[..., 2:4] = dets[..., 0:2] + 12
        counts = torch.full((S,), 40, dtype=torch.int32, device="cuda")
        res = {}
        for mode in ("detect_motion", "detect_motion+track"):
            for i in range(a.warmup):
                det.detect_device(dev[i % a.frames])
                if mode != "detect_motion":
                    ms.step_device(dets, counts, motion=det.motion_ptr)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for i in range(a.steps):
                det.detect_device(dev[i % a.frames])
                if mode != "detect_motion":
                    ms.step_device(dets, counts, motion=det.motion_ptr)
            e1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / a.steps
            ms_step = e0.elapsed_time(e1) / a.steps
            res[mode] = {"ms_per_step": round(ms_step, 4), "host_ms_per_step": round(wall, 4),
                         "frames_per_s": round(S * 1e3 / ms_step, 1)}
        m, st = det.download()
        print(json.dumps({"what": "global camera motion (optical_flow)", "streams": S, "hw": [H, W],
                          "steps": a.steps, **res, "corners_last": int(m[0]["n_corners"]),
                          "tracked_last": int(m[0]["n_tracked"]),
                          "motion_events_stream0": int(st[0]["motion_events"])}), flush=True)


if __name__ == "__main__":
    main()
