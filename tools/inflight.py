"""Concurrency probe: K independent DeviceModels (own activation arenas) each replaying its
detector hipGraph on its own HIP stream, vs one model.  Answers whether independent forwards
overlap on the chip (the single graph's parallel branches do not)."""
import importlib, sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
P = importlib.import_module(PKG)
A = importlib.import_module(PKG + ".arch"); W = importlib.import_module(PKG + ".weights"); M = importlib.import_module(PKG + ".model")
ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
sd = W.synthetic_state_dict(ar, 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sc = P.synth.Scene(seed=0, n_targets=22, n_frames=B + 1)
ft = torch.from_numpy(np.stack([sc.frame(t) for t in range(B)])).cuda()
res = {}
for K in (1, 2, 3):
    models = [M.DeviceModel(M.Program(ar, sd, 512, 640, 640, B, "bf16")) for _ in range(K)]
    models[0].autotune(ft, 0.25)
    b, pl = models[0].get_plan()
    for m in models[1:]:
        m.load_plan(b, pl)
    for m in models:
        m.set_schedule(1, 1)
    streams = [torch.cuda.Stream() for _ in range(K)]
    outs = [(torch.zeros((B, 300, 6), device="cuda"), torch.zeros(B, dtype=torch.int32, device="cuda")) for _ in range(K)]
    for k in range(K):
        with torch.cuda.stream(streams[k]):
            models[k].detect(ft, 0.25, 0.7, 300, outs[k][0], outs[k][1], graph=True)
    torch.cuda.synchronize()
    n = 60
    t0 = time.perf_counter()
    for i in range(n):
        for k in range(K):
            with torch.cuda.stream(streams[k]):
                models[k].detect(ft, 0.25, 0.7, 300, outs[k][0], outs[k][1], graph=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res[K] = K * n * B / dt
    print(f"K={K} in flight: {res[K]:.0f} frames/s ({dt / n * 1e3:.3f} ms per round of {K})", flush=True)
    del models
