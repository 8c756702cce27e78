"""Per-workgroup timeline of one conv_fast op (YK_FAST_TS diagnostics): dispatch ramp (spread
of workgroup start times), workgroup duration split into prologue+K loop and reduction+epilogue,
and the tail.  usage: YK_FAST_TS=<op> python tools/wg_times.py <op> [<op> ...] (set for each op)"""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
P = importlib.import_module(PKG)
A = importlib.import_module(PKG + ".arch")
W = importlib.import_module(PKG + ".weights")
M = importlib.import_module(PKG + ".model")
L = importlib.import_module(PKG + "._lib")
op = int(os.environ["YK_FAST_TS"])
ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
B = 8
dm = M.DeviceModel(M.Program(ar, W.synthetic_state_dict(ar, 0), 512, 640, 640, B, "bf16"))
sc = P.synth.Scene(seed=0, n_targets=22, n_frames=B + 1)
ft = torch.from_numpy(np.stack([sc.frame(t) for t in range(B)])).cuda()
dm.autotune(ft, 0.25)
for _ in range(3):
    dm.detect(ft)
torch.cuda.synchronize()
ptr = C.c_void_p()
L.check(L.lib().yk_model_buffer(dm._h, -2, C.byref(ptr)), "buf")
ts = np.zeros(3 * 65536, np.uint64)
M._memcpy_d2h(ts, ptr.value)
ts = ts.reshape(-1, 3).astype(np.int64)
ts = ts[ts[:, 0] > 0]
# the buffer keeps the last launch of every workgroup index: keep the last launch's cluster
order = np.sort(ts[:, 0])
gaps = np.nonzero(np.diff(order) > 300)[0]  # > 3 us between consecutive workgroup starts
cut = order[gaps[-1] + 1] if len(gaps) else order[0]
ts = ts[ts[:, 0] >= cut]
t0 = ts[:, 0].min()
st, mid, en = (ts[:, 0] - t0) / 100.0, (ts[:, 1] - t0) / 100.0, (ts[:, 2] - t0) / 100.0  # us
prof = dm.profile(ft, reps=5)
print(f"op {op} {prof[op][2]} isolated {prof[op][3] * 1e3:.2f} us; {len(ts)} workgroups")
print(f"  start spread {st.max():.2f} us (p50 {np.median(st):.2f}); last end {en.max():.2f} us")
print(f"  per WG: total p50 {np.median(en - st):.2f} max {np.max(en - st):.2f}; prologue+K p50 {np.median(mid - st):.2f}; "
      f"reduce+epilogue p50 {np.median(en - mid):.2f}")
