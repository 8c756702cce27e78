#!/usr/bin/env python3
"""Per-op device time of every halo-tile split conv variant (plan kind 5: NE x NPT x WM) against
the op's entry in a base plan, on the fp32 bench workload (batch-8 forward, YOLOv8s+P2).  One
JSON line: {op: {"base": [kind, nnt, npt, us], "halo": [[ne, npt, wm, us], ...]}}.  With YK_LIB
pointing at a YK_DIAG=4|8 build (detector.hip, "Diagnostic builds") the same sweep shows what bounds the kernel.

usage: halo_probe.py [--plan gpurun_out/.../plan.json] [--ops 72,73,76] [--reps 10]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", default=os.path.join(REPO, "plans", "s_640x512_i640_b8_fp32.json"))
    ap.add_argument("--ops", default="72,73,76,74,80,77,1,19,30,3,4,29,7")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    M = importlib.import_module(PKG + ".model")
    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    B = 8
    prog = M.Program(ar, sd, 512, 640, 640, B, "fp32")
    with open(a.plan) as f:
        base = json.load(f)["plan"]
    ft = torch.from_numpy(np.stack([P.synth.Scene(seed=s, n_targets=40, n_frames=1).frame(0) for s in range(B)])).cuda()
    dm = M.DeviceModel(prog)
    dm.load_plan(B, base)
    ops = [int(x) for x in a.ops.split(",")]

    def timed(i):
        prof = dm.profile(ft, reps=a.reps)
        return next(p[3] for p in prof if p[0] == i) * 1e3, next(p[2] for p in prof if p[0] == i)

    out = {}
    for i in ops:
        k, n, p = base[i]
        us, kern = timed(i)
        res = {"base": [k, n, p, round(us, 2), kern], "halo": []}
        for wm in (0, 1):
            for ne in (1, 2):
                for npt in (1, 2, 4):
                    try:
                        dm.set_plan(B, 5, ne, npt | (wm << 4), op=i)
                    except Exception:
                        continue
                    us, kern = timed(i)
                    if kern.startswith("conv_halo"):
                        res["halo"].append([ne, npt, wm, round(us, 2)])
        dm.set_plan(B, k, n, p, op=i)
        res["halo"].sort(key=lambda r: r[3])
        out[i] = res
        print(i, res["base"], res["halo"][:4], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
