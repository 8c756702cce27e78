#!/usr/bin/env python3
"""Autotune the conv plan for the in-flight regime and write it as a batch-S plan.

bench.py keeps D detector forwards of batch S in flight; the per-op autotune of
yk_model_autotune times one launch at a time, where the small register tiles that expose the
most parallelism win, although under D concurrent forwards the chip is already full and the
tile that moves fewer bytes per FLOP is the faster one.  This tool tunes at batch D*S (the
work the chip sees at once, capped by the arena limit) and stores the chosen variants as the plan for batch S.

usage: tune_concurrent.py --dtype fp32 [--streams 8] [--tune-batch 16] [--out plans/...json]
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
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--tune-batch", type=int, default=16,
                    help="batch the autotune runs at (fp32: <= 16 keeps the activation arena under the 2 GiB the "
                         "table-driven kernel's 32-bit offsets address)")
    ap.add_argument("--scale", default="s")
    ap.add_argument("--hw", default="512x640")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--targets", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    M = importlib.import_module(PKG + ".model")
    H, W = (int(v) for v in a.hw.split("x"))
    Bt = a.tune_batch
    ar = P.arch.parse_arch(P.arch.load_model_dict(f"yolov8{a.scale}-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    prog = M.Program(ar, sd, H, W, a.imgsz, Bt, a.dtype)
    dm = M.DeviceModel(prog)
    dm.set_schedule(1, 1)
    frames = torch.stack([P.synth.Scene(seed=s, n_targets=a.targets, n_frames=2, width=W, height=H)
                          .frames_torch(0, 1, "cuda")[0] for s in range(Bt)]).contiguous()
    dm.autotune(frames, 0.25)
    b, plan = dm.get_plan()
    assert b == Bt, (b, Bt)
    out = a.out or os.path.join(REPO, "plans", f"{a.scale}_{W}x{H}_i{a.imgsz}_b{a.streams}_{a.dtype}.json")
    with open(out, "w") as f:
        json.dump({"batch": a.streams, "plan": plan, "dtype": a.dtype, "tuned_at_batch": Bt,
                   "workload": os.path.basename(out)}, f)
    print(json.dumps({"out": out, "tuned_at_batch": Bt, "ops": len(plan)}))


if __name__ == "__main__":
    main()
