"""Host enqueue cost per step vs device time per step (is the bench host-bound?)."""
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
pipeline = importlib.import_module(P.__name__ + ".pipeline")
import json

pipe = pipeline.StreamPipeline("yolov8s-small.yaml", 8, (512, 640), "bf16", seed=0, pipelined=True)
sc = [P.synth.Scene(seed=s, n_targets=22, n_frames=4) for s in range(8)]
fr = torch.stack([x.frames_torch(0, 2, "cuda") for x in sc], 1)
pipe.frames.copy_(fr[0])
pl = json.load(open("profiles/r01_plan.json"))
pipe.model.load_plan(pl["batch"], pl["plan"])
pipe.capture(tune=False)
for _ in range(20):
    pipe.step()
torch.cuda.synchronize()
n = 100
L = importlib.import_module(P.__name__ + "._lib")
import ctypes as C
for what in ("step", "detect_only", "graph_launch_only"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        if what == "step":
            pipe.step()
        elif what == "detect_only":
            pipe.model.detect(pipe.frames, pipe.conf, pipe.iou, pipe.max_det, pipe._dets[0], pipe._counts[0], graph=True)
        else:
            L.lib().yk_detect_graph(pipe.model._h, L.ptr(pipe.frames), 8, C.c_float(pipe.conf), C.c_float(pipe.iou), 300,
                                    L.ptr(pipe._dets[0]), L.ptr(pipe._counts[0]), L.current_stream(0))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{what}: host enqueue {1e6 * (t1 - t0) / n:.1f} us/step, wall {1e6 * (t2 - t0) / n:.1f} us/step")

# device-side step timing with events around each detect (graph) launch
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
torch.cuda.synchronize()
for e0, e1 in evs:
    e0.record()
    pipe.model.detect(pipe.frames, pipe.conf, pipe.iou, pipe.max_det, pipe._dets[0], pipe._counts[0], graph=True)
    e1.record()
torch.cuda.synchronize()
inside = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
between = [evs[i][1].elapsed_time(evs[i + 1][0]) * 1e3 for i in range(len(evs) - 1)]
print(f"graph on-stream duration {sum(inside[5:]) / len(inside[5:]):.1f} us, gap to next launch {sum(between[5:]) / len(between[5:]):.1f} us")
torch.cuda.synchronize()
for e0, e1 in evs:
    e0.record()
    pipe.model.detect(pipe.frames, pipe.conf, pipe.iou, pipe.max_det, pipe._dets[0], pipe._counts[0], graph=False)
    e1.record()
torch.cuda.synchronize()
inside = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
between = [evs[i][1].elapsed_time(evs[i + 1][0]) * 1e3 for i in range(len(evs) - 1)]
print(f"eager on-stream duration {sum(inside[5:]) / len(inside[5:]):.1f} us, gap to next launch {sum(between[5:]) / len(between[5:]):.1f} us")
pipe.model.set_schedule(1, 1)
pipe.capture(tune=False)
torch.cuda.synchronize()
for e0, e1 in evs:
    e0.record()
    pipe.model.detect(pipe.frames, pipe.conf, pipe.iou, pipe.max_det, pipe._dets[0], pipe._counts[0], graph=True)
    e1.record()
torch.cuda.synchronize()
inside = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
between = [evs[i][1].elapsed_time(evs[i + 1][0]) * 1e3 for i in range(len(evs) - 1)]
print(f"lanes=1 graph on-stream duration {sum(inside[5:]) / len(inside[5:]):.1f} us, gap {sum(between[5:]) / len(between[5:]):.1f} us")
