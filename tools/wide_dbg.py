"""conv_wide_kernel time on one op with parts switched off (YK_WIDE_DBG) -- diagnostics."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
M = importlib.import_module(P.__name__ + ".model")
B = 8
ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
prog = M.Program(ar, P.weights.synthetic_state_dict(ar, 0), 512, 640, 640, B, "bf16", 300)
dm = M.DeviceModel(prog, 0)
fr = P.synth.Scene(seed=0, n_targets=22, n_frames=2).frames_torch(0, 1, "cuda").expand(B, -1, -1, -1).contiguous()
dm.detect(fr)
for o in [int(x) for x in sys.argv[1:]]:
    for nnt in (2, 4):
        dm.set_plan(B, 4, nnt, 0, op=o)
        prof = dm.profile(fr, reps=20)
        print(f"dbg {os.environ.get('YK_WIDE_DBG', '0')} op {o} {prof[o][2]} {prof[o][3] * 1e3:.2f} us", flush=True)
