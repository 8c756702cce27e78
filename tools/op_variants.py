"""Time every conv kernel variant on selected ops (batch 8) to see what the autotuner chooses
between.  usage: python tools/op_variants.py op [op ...]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
M = importlib.import_module(P.__name__ + ".model")
ops = [int(x) for x in sys.argv[1:]] or [1, 3, 72, 73, 74, 76]
B = 8
ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
prog = M.Program(ar, P.weights.synthetic_state_dict(ar, 0), 512, 640, 640, B, "bf16", 300)
dm = M.DeviceModel(prog, 0)
sc = P.synth.Scene(seed=0, n_targets=22, n_frames=2)
fr = sc.frames_torch(0, 1, "cuda").expand(B, -1, -1, -1).contiguous()
dm.detect(fr)
variants = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (4, 2, 4), (4, 4, 4), (4, 2, 8), (4, 4, 8)] + \
    [(3, n, p | (w << 4)) for w in (0, 1) for n in (1, 2, 3, 4) for p in (1, 2, 4)]
for o in ops:
    res = []
    for v in variants:
        try:
            dm.set_plan(B, *v, op=o)
        except Exception:
            continue
        prof = dm.profile(fr, reps=20)
        res.append((prof[o][3] * 1e3, prof[o][2], v))
    res.sort()
    print(f"op {o}: " + "  ".join(f"{k}={t:.2f}" for t, k, v in res[:6]), flush=True)
    dm.set_plan(B, -1, 0, 0, op=o)
