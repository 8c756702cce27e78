#!/usr/bin/env python3
"""Where the host time of the host-frame bench loop goes (diagnostic): builds the bench's config-3
pipeline (heuristic plan), runs the timed loop's calls (pipe.run with next_frames, download_async)
and attributes host time to the copies (by direction), the detector graph launches, the tracker /
motion launches and the rest, per step."""
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib

PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
pipeline = importlib.import_module(PKG + ".pipeline")
lib = importlib.import_module(PKG + "._lib")

S, H, W = int(sys.argv[3]) if len(sys.argv) > 3 else 8, 512, 640
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
nbuf = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (H, W), "fp32", seed=0, device=0, pipelined=True,
                               imgsz=640, max_tracks=256, inflight=4)
pipe.set_schedule(1, 1)
pipe.capture(tune=False)
g = torch.Generator().manual_seed(0)
host = torch.randint(0, 255, (nbuf, S, H, W, 3), dtype=torch.uint8, generator=g).pin_memory()
sink = torch.empty((S, H, W, 3), dtype=torch.uint8, device="cuda")
for j in range(nbuf):  # map every page-locked page for DMA once
    sink.copy_(host[j], non_blocking=True)
torch.cuda.synchronize()
rows = torch.empty(S * 256 * lib.TRACK_OUT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
counts = torch.empty(S, dtype=torch.int32, pin_memory=True)
stats = torch.empty(S * lib.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
acc = defaultdict(int)
orig_copy = torch.Tensor.copy_


def copy_(dst, src, non_blocking=False):
    t0 = time.perf_counter_ns()
    r = orig_copy(dst, src, non_blocking)
    acc["copy " + ("d" if src.is_cuda else "h") + "2" + ("d" if dst.is_cuda else "h")] += time.perf_counter_ns() - t0
    return r


def wrap(obj, name, key):
    f = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter_ns()
        r = f(*a, **k)
        acc[key] += time.perf_counter_ns() - t0
        return r
    setattr(obj, name, w)


torch.Tensor.copy_ = copy_
for m in pipe.models:
    wrap(m, "detect", "detect (graph launch)")
wrap(pipe.tracker, "step_device", "tracker step")
wrap(pipe, "step", "pipe.step (forward + tracker enqueue)")
wrap(pipe.tracker, "download_async", "download_async")
for mode in ("warm", "host", "hbm"):
    acc.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter_ns()
    n = 8 if mode == "warm" else steps
    for t in range(n):
        if mode == "hbm":
            pipe.run(pipe.frames)
        else:
            pipe.run(host[t % nbuf], next_frames=host[(t + 1) % nbuf] if t + 1 < n else None)
            pipe.download_async(rows, counts, stats)
    t1 = time.perf_counter_ns()
    torch.cuda.synchronize()
    t2 = time.perf_counter_ns()
    if mode == "warm":
        continue
    print(f"{mode} (nbuf {nbuf}): host {(t1 - t0) / n / 1e3:8.1f} us/step, wall {(t2 - t0) / n / 1e3:8.1f} us/step", flush=True)
    for k, v in sorted(acc.items(), key=lambda x: -x[1]):
        print(f"   {k:24s} {v / n / 1e3:8.1f} us/step")
