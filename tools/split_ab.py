#!/usr/bin/env python3
"""A/B of the F32 build's two MFMA paths on the bench workload (batch-8 forward, YOLOv8s+P2):
exact-f32 MFMA (F32) vs split-bf16 MFMA (F32S, plan npt bit 64) on the same conv plan.

Prints one JSON line: per-op device time of both (hipEvents, yk_model_profile), the sum, and
the accuracy of each against the torch-CPU oracle (max relative error of every checked layer
and of the final detections) and of split against exact.

usage: split_ab.py [--plan plans/s_640x512_i640_b8_fp32.json] [--batch 8] [--oracle-batch 2]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
SPLIT = 64


def split_plan(plan):
    """The plan with every table-kernel op (CK_FAST = 3) moved to the split-MFMA body."""
    out = []
    for kind, nnt, npt in plan:
        if kind == 3:
            npt |= SPLIT
        out.append([kind, nnt, npt])
    return out


def rel(a, b):
    a, b = torch.as_tensor(a, dtype=torch.float64), torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", default=os.path.join(REPO, "plans", "s_640x512_i640_b8_fp32.json"))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--oracle-batch", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--plan-exact", default="", help="plan of the exact leg (default: --plan with the split bit cleared)")
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    M = importlib.import_module(PKG + ".model")
    from oracle import detector_ref as D

    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    B = a.batch
    prog = M.Program(ar, sd, 512, 640, 640, B, "fp32")
    with open(a.plan) as f:
        pl = json.load(f)
    scenes = [P.synth.Scene(seed=s, n_targets=40, n_frames=2) for s in range(B)]
    frames_np = [sc.frame(0) for sc in scenes]
    ft = torch.from_numpy(np.stack(frames_np)).cuda()
    res = {}
    models = {}
    exact = [[k, n, (p & ~SPLIT) if k == 3 else p] for k, n, p in pl["plan"]]
    split = split_plan(pl["plan"])
    if a.plan_exact:  # two committed plans side by side (the split one as it is)
        with open(a.plan_exact) as f:
            exact = json.load(f)["plan"]
        split = pl["plan"]
    for name, plan in (("exact", exact), ("split", split)):
        dm = M.DeviceModel(prog)
        dm.load_plan(pl["batch"], plan)
        dets, counts = dm.detect(ft)
        torch.cuda.synchronize()
        prof = dm.profile(ft, reps=a.reps)
        res[name] = {"total_us": round(sum(p[3] for p in prof) * 1e3, 1),
                     "conv_us": round(sum(p[3] for p in prof if p[1] == 1) * 1e3, 1),
                     "ops": [(p[0], p[2], round(p[3] * 1e3, 2)) for p in prof]}
        models[name] = (dm, dets.cpu(), counts.cpu())
    # accuracy: oracle on the first oracle-batch frames
    Bo = a.oracle_batch
    layers = [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
              for Ly in ar.layers]
    ref = D.RefDetector(layers, sd, P.arch.detect_strides(ar))
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    im = D.preprocess(frames_np[:Bo], 640)
    y, _ = ref.forward(im, keep_all=True)
    want = D.non_max_suppression(y, 0.25, 0.7, 300)
    want = [D.scale_clip(p, im.shape[2:], (512, 640)) for p in want]
    acc = {}
    for name, (dm, dets, counts) in models.items():
        lay = {}
        for i in (0, 2, 4, 6, 8, 9, 12, 15, 18, 21, 24):
            lay[i] = rel(dm.layer_nchw(i, B)[:Bo], ref.outputs[i])
        box = 0.0
        same = True
        for b in range(Bo):
            n = int(counts[b])
            same = same and n == len(want[b])
            if n == len(want[b]) and n:
                box = max(box, rel(dets[b, :n, :5], want[b][:, :5]))
        acc[name] = {"layer_rel": {k: float(f"{v:.3g}") for k, v in lay.items()}, "max_layer_rel": max(lay.values()),
                     "det_counts_equal": same, "det_rel": box}
    de, ce = models["exact"][1], models["exact"][2]
    ds, cs = models["split"][1], models["split"][2]
    sv = {"counts_equal": bool((ce == cs).all()),
          "det_rel": max((rel(ds[b, :int(cs[b]), :5], de[b, :int(ce[b]), :5]) for b in range(B)
                          if int(cs[b]) == int(ce[b]) and int(ce[b])), default=0.0),
          "layer_rel": {i: float(f"{rel(models['split'][0].layer_nchw(i, B), models['exact'][0].layer_nchw(i, B)):.3g}")
                        for i in (2, 9, 15, 24)}}
    ops = [{"op": e[0], "exact_kernel": e[1], "exact_us": e[2], "split_kernel": s_[1], "split_us": s_[2]}
           for e, s_ in zip(res["exact"]["ops"], res["split"]["ops"])]
    print(json.dumps({"exact_total_us": res["exact"]["total_us"], "split_total_us": res["split"]["total_us"],
                      "exact_conv_us": res["exact"]["conv_us"], "split_conv_us": res["split"]["conv_us"],
                      "accuracy": acc, "split_vs_exact": sv, "ops": ops}))


if __name__ == "__main__":
    main()
