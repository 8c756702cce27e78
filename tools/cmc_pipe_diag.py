#!/usr/bin/env python3
"""Diagnose a motion-reset pipeline mismatch: the StreamPipeline(tracker_policy=1,
motion_method='optical_flow') scenario of tests/test_pipeline_gpu.py for a few frames, printing per
stream and frame the device motion record next to the oracle's detect_motion, and for every track
whose row differs: both rows, the detections near it and the oracle's IoU row.  The same detections
and device motion records are also stepped through a separate MultiStreamTracker (stride-4 host
upload), to tell the pipeline plumbing from the tracker kernels."""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def main(F=3, S=2):
    P = importlib.import_module(PKG)
    L = P._lib
    pipeline = importlib.import_module(PKG + ".pipeline")
    from oracle import detector_ref as D
    from oracle.cmc_ref import RefCMCMultiTracker
    from test_pipeline_gpu import _pan_scene

    TR = P.tracker
    seqs = [_pan_scene(90 + s, F) for s in range(S)]
    pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "fp32", seed=0, max_tracks=256,
                                   tracker_policy=1, motion_method="optical_flow")
    refs = [RefCMCMultiTracker(150, 1, 0.1) for _ in range(S)]
    side = TR.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=256, max_dets=pipe.max_det, policy=L.POLICY_MOTION_RESET)
    for t in range(F):
        fr = [seqs[s][t] for s in range(S)]
        pipe.run(torch.from_numpy(np.stack(fr)).cuda())
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        rows, counts, stats = rows.copy(), counts.copy(), stats.copy()
        motion, _ = pipe.gmd.download()
        motion = motion.copy()
        dd, dc = pipe.dets.cpu().numpy(), pipe.counts.cpu().numpy()
        mdev = torch.from_numpy(motion.view(np.uint8)).cuda()
        per = [[[b[0], b[1], b[2], b[3]] for b in dd[s, : dc[s], :4]] for s in range(S)]
        side.step_host(per, motion=mdev.data_ptr())
        srows, scounts, _ = side.download()
        for s in range(S):
            dets = [[b[0], b[1], b[2], b[3], b[4]] for b in dd[s, : dc[s], :5]]
            snap_before = [(trk.track_id, np.asarray(getattr(trk, 'x', [0]))[:4].ravel().tolist()) for trk in refs[s].trackers]
            if s == 0:  # T001's state on both sides before this update, its predict() box and IoUs
                import copy
                from oracle.tracker_ref import ref_iou
                for trk in refs[s].trackers[:1]:
                    c = copy.deepcopy(trk)
                    pb = c.predict()
                    print(f"   [{t}] oracle T{trk.track_id:03d} age {trk.age} last_reset {trk.last_reset_frame} "
                          f"x {np.asarray(trk.x).ravel().tolist()} ph {[list(map(float, v)) for v in trk.position_history]} "
                          f"pred {list(map(float, pb))}")
                    ious = [(d, float(ref_iou(dt[:4], pb))) for d, dt in enumerate(dets)]
                    print(f"   [{t}] oracle IoU>0 {[(d, round(v, 6)) for d, v in ious if v > 0]}")
                snap = pipe.tracker.snapshot(0)
                for r in snap[:1]:
                    print(f"   [{t}] device T{int(r['track_num']):03d} (after step) age {int(r['age'])} "
                          f"last_reset {int(r['last_reset_frame'])} resets {int(r['reset_count'])} x {r['x'].tolist()}")
            rb = refs[s].update(dets, fr[s])
            mi = refs[s].frame_motion_info
            print(f"== frame {t} stream {s}: dets {int(dc[s])}, device motion {motion[s]}, oracle motion {mi}")
            ours = [TR._reset_fields(r, TR._row_to_dict(r, TR.track_id_of(r["track_num"]))) for r in rows[s, : counts[s]]]
            side_rows = [TR._row_to_dict(r, TR.track_id_of(r["track_num"])) for r in srows[s, : scounts[s]]]
            print(f"   ids ours {[o['track_id'] for o in ours][:12]} oracle {[r['track_id'] for r in rb][:12]}")
            for o, so, r in zip(ours, side_rows, rb):
                if not np.allclose(np.asarray(o["bbox"], np.float64), np.asarray(r["bbox"], np.float64), rtol=1e-9, atol=1e-9):
                    print(f"   MISMATCH {o['track_id']}: ours {np.asarray(o['bbox'])} side {np.asarray(so['bbox'])} "
                          f"oracle {np.asarray(r['bbox'])} hits {o['hits']}/{r['hits']} reset {o['reset_count']}/{r['reset_count']}")
                    rbx = np.asarray(r["bbox"], np.float64)
                    near = [(d, [float(v) for v in b[:5]]) for d, b in enumerate(dets)
                            if abs(b[0] - rbx[0]) < 60 and abs(b[1] - rbx[1]) < 60]
                    print(f"     dets near: {near}")
            print(f"   oracle tracks before: {snap_before[:6]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 3))
