"""Repro probe: a drop-in YOLO kept alive (as a failed test's traceback keeps it) while a bf16
StreamPipeline captures its detector graphs (the r4i/r4j segfault order)."""
import faulthandler
import importlib
import os
import sys

import numpy as np
import torch

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
P = importlib.import_module(PKG)
sys.path.insert(0, os.path.join(REPO, PKG, "compat"))
from ultralytics import YOLO  # noqa: E402
from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker  # noqa: E402

sys.path.pop(0)
mode = sys.argv[1] if len(sys.argv) > 1 else "alive"
sc = P.synth.Scene(seed=4, n_targets=40, n_frames=12)
model = YOLO("yolov8s-small.yaml")
trk = EnhancedMultiTargetTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
for t in range(10):
    r = model(sc.frame(t), verbose=False)
    b, c = r[0].boxes.xyxy.cpu().numpy(), r[0].boxes.conf.cpu().numpy()
    trk.update([[x[0], x[1], x[2], x[3], s] for x, s in zip(b, c) if s > 0.1])
print("drop-in frames done", flush=True)
if mode == "free":
    del model, trk, r
    import gc
    gc.collect()
pipeline = importlib.import_module(PKG + ".pipeline")
for pipelined, inflight in ((False, 1), (True, 1), (True, 2), (True, 3), (True, 4)):
    pipe = pipeline.StreamPipeline("yolov8s-small.yaml", 4, (512, 640), "bf16", seed=0, max_tracks=256,
                                   pipelined=pipelined, inflight=inflight)
    import gc as _gc
    M_ = importlib.import_module(PKG + ".model")
    live = {k: sum(1 for o in _gc.get_objects() if type(o).__name__ == k)
            for k in ("StreamPipeline", "DeviceModel", "MultiStreamTracker", "Results", "Boxes", "Engine")}
    print("pipeline", pipelined, inflight, "built", live, torch.cuda.memory_allocated() >> 20, "MiB",
          flush=True)
    if "lanes1" in sys.argv:
        pipe.set_schedule(1, 1)
    pipe.capture(tune=False)
    print("captured", flush=True)
    for t in range(4):
        pipe.run(torch.from_numpy(np.stack([sc.frame(t)] * 4)).cuda())
    pipe.sync()
    if "gc" in sys.argv:
        import gc
        del pipe
        gc.collect()
print("ok", flush=True)
