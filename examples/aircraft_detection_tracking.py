#!/usr/bin/env python3
"""The reference driver (kalman/aircraft_detection_tracking.py:29-220) on this framework.

Same loop, same tracker settings (150, 1, 0.1), same statistics and visualizer; the only
changes are the imports (the compat packages resolve ``ultralytics`` and ``kalman`` to
libyk.so) and the frame I/O: no video codec is in this image, so the input is a ``.npy``
frame stack, an image directory / glob or a ``.y4m`` file, and the output a ``.npy`` stack
or a directory of PNGs.

    python examples/aircraft_detection_tracking.py --source frames.npy --out result.npy \\
        [--model best.pt | yolov8s-small.yaml] [--dtype fp32|bf16]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
sys.path.insert(0, os.path.join(os.path.dirname(HERE), PKG, "compat"))

from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker  # noqa: E402
from kalman.trajectory_visualizer import TrajectoryVisualizer  # noqa: E402
from ultralytics import YOLO  # noqa: E402

from kalman._pkg import sub  # noqa: E402

FR = sub("frames")
V = sub("visualize")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--model", default="yolov8s-small.yaml")
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()

    model = YOLO(a.model, dtype=a.dtype)
    tracker = EnhancedMultiTargetTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    visualizer = TrajectoryVisualizer()
    cap = FR.VideoReader(a.source)
    if not cap.isOpened():
        print(f"cannot open {a.source}")
        return 1
    fps = int(cap.get(FR.CAP_PROP_FPS))
    width, height = int(cap.get(FR.CAP_PROP_FRAME_WIDTH)), int(cap.get(FR.CAP_PROP_FRAME_HEIGHT))
    total = int(cap.get(FR.CAP_PROP_FRAME_COUNT))
    print(f"video: {width}x{height}, {fps} fps, {total} frames")
    out = FR.VideoWriter(a.out, fps, (width, height))

    frame_count = detection_frames = prediction_frames = state_changes = 0
    last_states = {}
    try:
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
            tracks = tracker.update(detections)
            current = {}
            for t in tracks:
                tid, st = t["track_id"], t["status"]
                current[tid] = st
                if tid in last_states and last_states[tid] != st:
                    state_changes += 1
                    print(f"frame {frame_count}: track {tid} {last_states[tid]} -> {st}")
                detection_frames += st == "detected"
                prediction_frames += st == "predicted"
            last_states = current
            info = {"frame_number": frame_count, "detections": len(detections), "tracks": len(tracks),
                    "detection_frames": detection_frames, "prediction_frames": prediction_frames,
                    "state_changes": state_changes}
            vis = visualizer.draw_tracks(frame, tracks, detections, info)
            if any(t["status"] == "predicted" for t in tracks):
                title, color = "AI PREDICTION MODE - Orange Boxes", (0, 165, 255)
            elif any(t["status"] == "detected" for t in tracks):
                title, color = "DETECTION MODE - Green Boxes", (0, 255, 0)
            else:
                title, color = "NO TARGETS", (255, 255, 255)
            V.put_text(vis, title, (10, 30), V.FONT_HERSHEY_SIMPLEX, 1.0, color, 3)
            out.write(vis)
            if frame_count % 50 == 0:
                print(f"progress {frame_count / max(total, 1) * 100:.1f}% ({frame_count}/{total}); "
                      f"detected {detection_frames}, predicted {prediction_frames}, changes {state_changes}")
    finally:
        cap.release()
        out.release()
    print(f"frames {frame_count}, detection frames {detection_frames}, prediction frames {prediction_frames}, "
          f"state changes {state_changes}")
    if detection_frames + prediction_frames:
        print(f"prediction share {prediction_frames / (detection_frames + prediction_frames) * 100:.1f}%")
    print(f"output: {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
