#!/usr/bin/env python3
"""Serial vs pipelined motion-detector records, step by step: the test_pipeline_gpu global-motion
scenario (3 streams of whip pans), the device yk_motion records of every step downloaded after a
full sync (--sync) or only at the end, printed where a pipelined run first differs from the
serial one."""
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
    from gmd_helpers import camera_sequence

    P = importlib.import_module(PKG)
    pipeline = importlib.import_module(PKG + ".pipeline")
    sync = "--sync" in sys.argv
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()
    runs = []
    for pipelined, inflight in ((False, 1), (False, 1), (True, 1), (True, 1), (True, 3)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow")
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        rec = []
        for t in range(F):
            pipe.run(frames[t])
            if sync:
                pipe.sync()
                rec.append(pipe.gmd.download()[0].copy())
        pipe.sync()
        rec.append(pipe.gmd.download()[0].copy())
        runs.append(rec)
    for j, r in enumerate(runs[1:], 1):
        for t, (a, b) in enumerate(zip(runs[0], r)):
            if a.tobytes() != b.tobytes():
                print("run", j, "step", t, "differs")
                print("  serial   ", a)
                print("  pipelined", b)
                break
        else:
            print("run", j, "identical over", len(r), "records")


if __name__ == "__main__":
    main()
