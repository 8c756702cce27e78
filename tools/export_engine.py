#!/usr/bin/env python3
"""Pack a detector program into an engine file for yk_model_load (include/yk.h).

usage: export_engine.py --out model.ykengine [--weights best.pt | state_dict.pt | --synthetic]
                        [--yaml yolov8s-small.yaml] [--hw 512x640] [--imgsz 640] [--dtype fp32]
                        [--max-batch 8] [--plan plans/s_640x512_i640_b8_fp32.json]
A .pt ultralytics checkpoint is read without unpickling code (checkpoint.py); its own model YAML
and scale are used.  The C host then needs only libyk.so and the engine file."""
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
    ap.add_argument("--out", required=True)
    ap.add_argument("--weights", default="")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--yaml", default="yolov8s-small.yaml")
    ap.add_argument("--hw", default="512x640")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--max-batch", type=int, default=8)
    ap.add_argument("--plan", default="")
    a = ap.parse_args()
    A = importlib.import_module(PKG + ".arch")
    M = importlib.import_module(PKG + ".model")
    W = importlib.import_module(PKG + ".weights")
    if a.weights.endswith(".pt") and not a.synthetic:
        CK = importlib.import_module(PKG + ".checkpoint")
        try:
            ydict, sd, _ = CK.load_checkpoint(a.weights)
        except ValueError:  # a plain state dict saved with torch.save
            ydict, sd = A.load_model_dict(a.yaml), torch.load(a.weights, map_location="cpu", weights_only=True)
        ar = A.parse_arch(ydict)
    else:
        ar = A.parse_arch(A.load_model_dict(a.yaml))
        sd = W.synthetic_state_dict(ar, 0)
    H, Wd = (int(v) for v in a.hw.split("x"))
    prog = M.Program(ar, sd, H, Wd, a.imgsz, a.max_batch, a.dtype)
    plan, batch = None, 0
    if a.plan:
        with open(a.plan) as f:
            pl = json.load(f)
        plan, batch = pl["plan"], min(int(pl["batch"]), a.max_batch)
    prog.export_engine(a.out, plan, batch)
    print(json.dumps({"out": a.out, "bytes": os.path.getsize(a.out), "ops": len(prog.ops), "dtype": a.dtype,
                      "frame": [H, Wd], "max_batch": a.max_batch, "plan_ops": 0 if plan is None else len(plan)}))


if __name__ == "__main__":
    main()
