"""Per-op device time vs batch (autotuned per batch): separates each launch's fixed cost from
its per-frame cost.  usage: python tools/op_scaling.py [batches...]"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
M = importlib.import_module(P.__name__ + ".model")
batches = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 16]
ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
sd = P.weights.synthetic_state_dict(ar, 0)
prog = M.Program(ar, sd, 512, 640, 640, max(batches), "bf16", 300)
dm = M.DeviceModel(prog, 0)
sc = P.synth.Scene(seed=0, n_targets=22, n_frames=2)
fr = sc.frames_torch(0, 1, "cuda").expand(max(batches), -1, -1, -1).contiguous()
res = {}
for B in batches:
    dm.autotune(fr[:B])
    prof = dm.profile(fr[:B], reps=10)
    res[B] = [(k, round(ms * 1e3, 2)) for (_, _, k, ms) in prof]
    print("batch", B, "sum us", round(sum(v for _, v in res[B]), 1), flush=True)
json.dump(res, open(os.environ.get("OUT", "gpurun_out/op_scaling.json"), "w"))
