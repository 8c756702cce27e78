#!/usr/bin/env python3
"""Which streams the first pipeline of a process uses (each mode in a fresh process):
  null0    slot 0 on the caller's (null) stream, slots 1..3 and the tracker on pool streams (default)
  own0     every detector slot and the tracker on pool streams
  trknull  the tracker on the null stream, the four detector slots on pool streams
  trkhi    the tracker on a high-priority stream
usage: stream_map.py --mode MODE [--dtype fp32] [--steps 100]"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
pipeline = importlib.import_module(P.__name__ + ".pipeline")
ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="null0")
ap.add_argument("--dtype", default="fp32")
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--shift", type=int, default=0, help="streams created and used before the pipeline's")
a = ap.parse_args()
_dummies = [torch.cuda.Stream() for _ in range(a.shift)]
for _st in _dummies:
    with torch.cuda.stream(_st):
        torch.zeros(1, device="cuda").add_(1)
torch.cuda.synchronize()
S, H, W, F = 8, 512, 640, 40
scenes = [P.synth.Scene(seed=s, n_targets=40, n_frames=F + 1) for s in range(S)]
frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1).contiguous()
plan = json.load(open(os.path.join(REPO, "plans", f"s_640x512_i640_b8_{a.dtype}.json")))
p = pipeline.StreamPipeline("yolov8s-small.yaml", S, (H, W), a.dtype, seed=0, pipelined=True, inflight=4)
null = torch.cuda.current_stream()
if a.mode == "own0":
    p.det_streams[0] = torch.cuda.Stream()
elif a.mode == "trkhi":
    p.trk_stream = torch.cuda.Stream(priority=-1)
elif a.mode == "trknull":
    p.det_streams[0] = p.trk_stream
    p.trk_stream = null
p.set_schedule(1, 1)
for m in p.models:
    m.load_plan(plan["batch"], plan["plan"])
p.frames.copy_(frames[0])
p.capture(tune=False)
for t in range(20):
    p.run(frames[t % F])
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(a.steps):
    p.run(frames[t % F])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"mode": a.mode, "shift": a.shift, "fps": round(S * a.steps / dt, 1)}), flush=True)
