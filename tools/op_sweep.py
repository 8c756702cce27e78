#!/usr/bin/env python3
"""Per-op kernel sweep: every table / halo conv variant on the chosen ops, at the tuner's batch.

Starts from a committed plan (fp32 by default) and, for each op in --ops, sets each candidate variant in
turn (invalid ones are rejected by yk_model_set_plan and skipped) and records that op's device
time from yk_model_profile.  Prints one JSON line per op with the candidates sorted by time.

usage: op_sweep.py [--ops 3,10,22] [--batch 16] [--plan plans/s_640x512_i640_b8_fp32.json] [--dtype bf16]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="1,3,4,10,11,18,22,23,32,72,73,74")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--plan", default=os.path.join(REPO, "plans", "s_640x512_i640_b8_fp32.json"))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32", choices=("fp32", "bf16", "fp16", "fp8"))
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    M = importlib.import_module(PKG + ".model")
    L = importlib.import_module(PKG + "._lib")
    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    B = a.batch
    prog = M.Program(ar, sd, 512, 640, 640, B, a.dtype)
    dm = M.DeviceModel(prog)
    dm.set_schedule(1, 1)
    frames = torch.stack([P.synth.Scene(seed=s, n_targets=40, n_frames=2, width=640, height=512)
                          .frames_torch(0, 1, "cuda")[0] for s in range(B)]).contiguous()
    plan = json.load(open(a.plan))["plan"]
    dm.load_plan(B, plan)
    base = dm.profile(frames, reps=a.reps)
    cands = []
    for mode in range(4):
        for nnt in (1, 2, 3, 4):
            for npt in (1, 2, 4):
                for sp in (0, 64):
                    cands.append((3, nnt, npt | (mode << 4) | sp))
                    if mode == 1 and sp:  # block loop: 2 / 4 pixel blocks per workgroup
                        cands += [(3, nnt, npt | (mode << 4) | sp | nb) for nb in (128, 256)]
    for ne in (1, 2):
        for npt in (1, 2, 4):
            for wm in (0, 1):
                cands.append((5, ne, npt | (wm << 4)))
    for op in (int(v) for v in a.ops.split(",")):
        res = []
        for kind, nnt, npt in cands:
            try:
                dm.set_plan(B, kind, nnt, npt, op)
            except L.YKError:
                continue
            prof = dm.profile(frames, reps=a.reps)
            res.append((round(prof[op][3] * 1e3, 2), kind, nnt, npt, prof[op][2]))
        dm.load_plan(B, plan)
        res.sort()
        print(json.dumps({"op": op, "committed_us": round(base[op][3] * 1e3, 2), "committed": base[op][2],
                          "best": res[:8], "all": res}), flush=True)


if __name__ == "__main__":
    main()
