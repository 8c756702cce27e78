"""Device ByteTrack / BoT-SORT step time vs the numpy + scipy reference restatement on the host.

usage: bt_bench.py [--streams 8] [--frames 200] [--targets 60]
Detections are pre-staged on the device for every frame; the device leg times yk_bt_step over
all streams (hipEvents), the CPU leg the oracle's update() per stream (one core, as the
reference's Python loop)."""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from bt_helpers import scenario  # noqa: E402
from oracle import bytetrack_ref as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--streams", type=int, default=8)
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--targets", type=int, default=60)
ap.add_argument("--cpu-frames", type=int, default=40)
a = ap.parse_args()
BT = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd.bytetrack")
res = {}
for kind in ("bytetrack", "botsort"):
    cfg = dict(R.BOTSORT_CFG if kind == "botsort" else R.BYTETRACK_CFG)
    S, F, D = a.streams, a.frames, 256
    seqs = [scenario(100 + s, n_targets=a.targets, n_frames=F) for s in range(S)]
    buf = np.zeros((F, S, D, 6), np.float32)
    cnt = np.zeros((F, S), np.int32)
    for f in range(F):
        for s in range(S):
            x, c, k = seqs[s][f]
            n = len(c)
            buf[f, s, :n] = np.c_[x, c, k]
            cnt[f, s] = n
    dets = torch.from_numpy(buf).cuda()
    cnts = torch.from_numpy(cnt).cuda()
    dev = BT.BatchedTracker(cfg, n_streams=S, max_tracks=512, max_dets=D)
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    warm = 20
    for f in range(warm):
        dev.step_device(dets[f], cnts[f])
    torch.cuda.synchronize()
    ev[0].record(st)
    for f in range(warm, F):
        dev.step_device(dets[f], cnts[f])
    ev[1].record(st)
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / (F - warm)
    live = [len(r) for r in dev.download()]
    # CPU reference leg
    ids = R.IdCounter()
    refs = [R.RefTracker(cfg, ids=ids) for _ in range(S)]
    t0 = time.perf_counter()
    for f in range(a.cpu_frames):
        for s in range(S):
            x, c, k = seqs[s][f]
            refs[s].update(R.Dets(x, c, k))
    cpu_ms = (time.perf_counter() - t0) * 1e3 / a.cpu_frames
    res[kind] = {"streams": S, "device_us_per_step": round(us, 1), "device_frames_per_s": round(S / (us * 1e-6), 1),
                 "cpu_ms_per_step": round(cpu_ms, 2), "cpu_frames_per_s": round(S / (cpu_ms * 1e-3), 1),
                 "reported_rows_per_stream_last": live}
print(json.dumps(res))
