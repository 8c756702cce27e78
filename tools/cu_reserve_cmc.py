#!/usr/bin/env python3
"""CMC pipeline with CUs reserved for the tracker stream: the detector slots on CU-masked HIP
streams (hipExtStreamCreateWithCUMask) that leave every (ncu / R)-th CU out, the tracker stream
(motion detector + motion-reset step) on all CUs, so its latency-bound chain never queues behind
forward workgroups.  usage: cu_reserve_cmc.py --reserve R [--dtype bf16] [--plain]"""
import argparse
import ctypes as C
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
ap.add_argument("--reserve", type=int, default=0)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--plain", action="store_true")
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
S, H, W, F, D = 8, 512, 640, 60, 4
scenes = [P.synth.Scene(seed=P.shard.stream_seed(s, S), n_targets=40, n_frames=F + 1) for s in range(S)]
frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1).contiguous()
plan = json.load(open(os.path.join(REPO, "plans", f"s_640x512_i640_b8_{a.dtype}.json")))
ncu = torch.cuda.get_device_properties(0).multi_processor_count
hip = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


def masked_stream(bits):
    words = (C.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


p = pipeline.StreamPipeline("yolov8s-small.yaml", S, (H, W), a.dtype, seed=0, pipelined=True, inflight=D,
                            max_tracks=512, tracker_policy=0 if a.plain else 1,
                            motion_method=None if a.plain else "optical_flow")
if a.reserve:
    step = ncu // a.reserve
    bits = [i for i in range(ncu) if i % step != step - 1]
    for s in range(D):
        p.det_streams[s] = masked_stream(bits)
p.set_schedule(1, 1)
for m in p.models:
    m.load_plan(plan["batch"], plan["plan"])
p.frames.copy_(frames[0])
p.capture(tune=False)
for t in range(160):  # track load
    p.run(frames[t % F])
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(a.steps):
    p.run(frames[t % F])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"reserve": a.reserve, "plain": a.plain, "dtype": a.dtype, "cus": ncu,
                  "fps": round(S * a.steps / dt, 1)}), flush=True)
