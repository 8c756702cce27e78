"""End-to-end GPU parity: frames in HBM -> detector -> NMS -> tracker (device hand-off),
against the oracle chain (torch-CPU detector -> numpy tracker) per stream, plus the
reference driver's loop through the compat ``ultralytics`` / ``kalman`` packages."""
import importlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, pkg
from oracle import detector_ref as D
from oracle.tracker_ref import RefMultiTracker

pytestmark = pytest.mark.gpu


def _layers(ar):
    return [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
            for Ly in ar.layers]


def _trk_dicts(P, rows, n):
    return [P.tracker._row_to_dict(r, P.tracker.track_id_of(r["track_num"])) for r in rows[:n]]


def test_stream_pipeline_fp32_matches_oracle_chain():
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 2, 10
    pipe = pipeline.StreamPipeline("yolov8-small.yaml", S, (512, 640), "fp32", seed=0, max_tracks=256)
    ar = pipe.prog.ar
    ref = D.RefDetector(_layers(ar), pipe.prog.sd, P.arch.detect_strides(ar))
    scenes = [P.synth.Scene(seed=20 + s, n_targets=20, n_frames=F) for s in range(S)]
    refs = [RefMultiTracker(150, 1, 0.1, stable_ties=True) for _ in range(S)]
    torch.set_num_threads(8)
    for t in range(F):
        fr = [sc.frame(t) for sc in scenes]
        pipe.run(torch.from_numpy(np.stack(fr)).cuda())
        rows, counts, _ = pipe.tracker.download()
        want, _ = D.predict(ref, fr)
        for s in range(S):
            dets = [[b[0], b[1], b[2], b[3], b[4]] for b in want[s][:, :5].numpy()]
            rb = refs[s].update(dets)
            ours = _trk_dicts(P, rows[s], int(counts[s]))
            assert [o["track_id"] for o in ours] == [r["track_id"] for r in rb], (t, s)
            for o, r in zip(ours, rb):
                assert (o["status"], o["age"], o["hits"], o["time_since_update"]) == \
                    (r["status"], r["age"], r["hits"], r["time_since_update"])
                np.testing.assert_allclose(o["bbox"], r["bbox"], rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(o["confidence"], r["confidence"], rtol=1e-4)


def test_reference_driver_loop_through_compat_packages(tmp_path):
    """kalman/aircraft_detection_tracking.py:58-161 with the compat imports: frames read through
    the VideoCapture-like reader (a .npy frame stack, since no codec is in the image), the
    per-frame body of :88-131, the visualizer and the VideoWriter-like sink."""
    sys.path.insert(0, os.path.join(REPO, pkg().__name__, "compat"))
    try:
        from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker
        from kalman.trajectory_visualizer import TrajectoryVisualizer
        from ultralytics import YOLO
    finally:
        sys.path.pop(0)
    P = pkg()
    FR = P.frames
    sc = P.synth.Scene(seed=4, n_targets=12, n_frames=8)
    np.save(tmp_path / "short.npy", np.stack([sc.frame(t) for t in range(8)]))
    model = YOLO("yolov8s-small.yaml")
    tracker = EnhancedMultiTargetTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    vis = TrajectoryVisualizer()
    cap = FR.VideoReader(str(tmp_path / "short.npy"))
    fps = int(cap.get(FR.CAP_PROP_FPS))
    width, height = int(cap.get(FR.CAP_PROP_FRAME_WIDTH)), int(cap.get(FR.CAP_PROP_FRAME_HEIGHT))
    out = FR.VideoWriter(str(tmp_path / "result.npy"), fps, (width, height))
    detection_frames = prediction_frames = state_changes = frame_count = 0
    last = {}
    while True:
        ret, frame = cap.read()
        if not ret:
            break
        frame_count += 1
        results = model(frame, verbose=False)
        detections = []
        if len(results) > 0 and results[0].boxes is not None:
            boxes = results[0].boxes.xyxy.cpu().numpy()
            scores = results[0].boxes.conf.cpu().numpy()
            for box, score in zip(boxes, scores):
                if score > 0.1:
                    detections.append([box[0], box[1], box[2], box[3], score])
        assert all(isinstance(v, np.float32) for d in detections for v in d)
        tracks = tracker.update(detections)
        cur = {}
        for tr in tracks:
            cur[tr["track_id"]] = tr["status"]
            if tr["track_id"] in last and last[tr["track_id"]] != tr["status"]:
                state_changes += 1
            detection_frames += tr["status"] == "detected"
            prediction_frames += tr["status"] == "predicted"
        last = cur
        frame_info = {"frame_number": frame_count, "detections": len(detections), "tracks": len(tracks),
                      "detection_frames": detection_frames, "prediction_frames": prediction_frames,
                      "state_changes": state_changes}
        vis_frame = vis.draw_tracks(frame, tracks, detections, frame_info)
        assert vis_frame.shape == frame.shape and (vis_frame != frame).any()
        out.write(vis_frame)
    cap.release()
    out.release()
    assert frame_count == 8 and detection_frames > 0
    assert tracker.frame_count == 8
    assert results[0].boxes.xyxy.is_cuda and results[0].orig_shape == (512, 640)
    assert np.load(tmp_path / "result.npy").shape == (8, 512, 640, 3)


def test_pipelined_tracker_stream_matches_serial():
    """pipelined=True (tracker(t) on its own stream, overlapping detector(t+1), double-buffered
    detections) and inflight=2/3/4 (detector graphs in flight on their own streams) give exactly the
    serial pipeline's tracker state."""
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 4, 24
    runs = []
    for pipelined, inflight in ((False, 1), (True, 1), (True, 2), (True, 3), (True, 4)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight)
        scenes = [P.synth.Scene(seed=40 + s, n_targets=16, n_frames=F) for s in range(S)]
        frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        runs.append((rows.copy(), counts.copy(), stats.copy()))
    r0, c0, s0 = runs[0]
    for r1, c1, s1 in runs[1:]:
        np.testing.assert_array_equal(c0, c1)
        np.testing.assert_array_equal(s0, s1)
        for s in range(S):
            assert r0[s][: c0[s]].tobytes() == r1[s][: c1[s]].tobytes()


def test_pipeline_with_global_motion_matches_serial():
    """StreamPipeline(tracker_policy=1, motion_method='optical_flow') -- the
    MotionCompensatedMultiTracker.update(dets, frame) loop with GlobalMotionDetector on the
    device -- gives the serial pipeline's tracker and motion-detector state when the motion
    detector reads each slot's frames on the tracker stream with forwards in flight.  The frames
    are camera pans over a textured world (tests/gmd_helpers.py) with whip pans that trigger the
    global reset branch."""
    from gmd_helpers import camera_sequence

    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()  # [F, S, H, W, 3]
    runs = []
    for pipelined, inflight in ((False, 1), (True, 1), (True, 3)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow")
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        motion, mstats = pipe.gmd.download()
        runs.append((rows.copy(), counts.copy(), stats.copy(), motion.copy(), mstats.copy()))
    r0, c0, s0, m0, ms0 = runs[0]
    assert int(ms0["reset_triggers"].sum()) > 0  # the whip pans reached the global reset branch
    for r1, c1, s1, m1, ms1 in runs[1:]:
        np.testing.assert_array_equal(c0, c1)
        np.testing.assert_array_equal(s0, s1)
        assert m0.tobytes() == m1.tobytes() and ms0.tobytes() == ms1.tobytes()
        for s in range(S):
            assert r0[s][: c0[s]].tobytes() == r1[s][: c1[s]].tobytes()
