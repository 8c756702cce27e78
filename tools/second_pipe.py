#!/usr/bin/env python3
"""Why is a second StreamPipeline in one process slower?  Times config 3 (fp32, 4 in flight)
for: A fresh; B after A was deleted; C while B is still alive (idle); D after gc + empty_cache.
usage: second_pipe.py [--dtype fp32] [--steps 100]"""
import argparse
import gc
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
pipeline = importlib.import_module(P.__name__ + ".pipeline")
ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="fp32")
ap.add_argument("--steps", type=int, default=100)
a = ap.parse_args()
S, H, W = 8, 512, 640
F = 40
frames = torch.stack([torch.stack([sc.frames_torch(0, F, "cuda")[t] for sc in
                                   [P.synth.Scene(seed=s, n_targets=40, n_frames=F + 1) for s in range(S)]])
                      for t in range(F)]) if False else None
scenes = [P.synth.Scene(seed=s, n_targets=40, n_frames=F + 1) for s in range(S)]
frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1).contiguous()
plan = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plans",
                                   f"s_640x512_i640_b8_{a.dtype}.json")))


def make(streams=None):
    p = pipeline.StreamPipeline("yolov8s-small.yaml", S, (H, W), a.dtype, seed=0, pipelined=True, inflight=4)
    if streams is not None:
        p.trk_stream, p.det_streams = streams[0], streams[1]
    p.set_schedule(1, 1)
    for m in p.models:
        m.load_plan(plan["batch"], plan["plan"])
    p.frames.copy_(frames[0])
    p.capture(tune=False)
    return p


def run(p, tag):
    for t in range(20):
        p.run(frames[t % F])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.steps):
        p.run(frames[t % F])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"case": tag, "fps": round(S * a.steps / dt, 1), "ms_per_step": round(dt / a.steps * 1e3, 4)}),
          flush=True)


pa = make()
run(pa, "A fresh")
run(pa, "A again")
saved = (pa.trk_stream, list(pa.det_streams))
del pa
torch.cuda.synchronize()
torch.cuda.empty_cache()
pb = make()
run(pb, "B after A deleted")
pc = make()
run(pc, "C while B alive")
run(pb, "B again (C alive)")
del pb, pc
gc.collect()
torch.cuda.synchronize()
torch.cuda.empty_cache()
pd = make()
run(pd, "D after gc + empty_cache")
del pd
gc.collect()
pe = make(saved)
run(pe, "E with A's streams")
del pe
gc.collect()
hp = (torch.cuda.Stream(priority=-1), [None] + [torch.cuda.Stream(priority=-1) for _ in range(3)])
pf = make(hp)
run(pf, "F with fresh high-priority streams")
