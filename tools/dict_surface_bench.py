"""Rate of the reference's own tracker surface: EnhancedMultiTargetTracker.update(list of
[x1, y1, x2, y2, conf]) -> list[dict] per frame (host detections in, Python dicts out), on the
device tracker vs the oracle restatement (the reference's numpy/Python loop), one stream.

usage: dict_surface_bench.py [--targets 64] [--frames 300] [--preroll 150]"""
import argparse
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle.tracker_ref import RefMultiTracker  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--targets", type=int, default=64)
ap.add_argument("--frames", type=int, default=300)
ap.add_argument("--preroll", type=int, default=150)
a = ap.parse_args()
P = importlib.import_module("yolo---small-target-recognition---kalman-trajectory-prediction_amd")
T = importlib.import_module(P.__name__ + ".tracker")
sc = P.synth.Scene(seed=5, n_targets=a.targets, n_frames=a.preroll + a.frames + 1)
dets = [sc.detections(t) for t in range(a.preroll + a.frames)]
res = {}
for name, mk in (("device", lambda: T.EnhancedMultiTargetTracker(150, 1, 0.1, max_tracks=1024)),
                 ("oracle_cpu", lambda: RefMultiTracker(150, 1, 0.1))):
    trk = mk()
    for t in range(a.preroll):
        trk.update(dets[t])
    t0 = time.perf_counter()
    n_out = 0
    for t in range(a.preroll, a.preroll + a.frames):
        out = trk.update(dets[t])
        n_out += len(out)
    dt = time.perf_counter() - t0
    live = trk.stats["current_active_tracks"]
    res[name] = {"frames_per_s": round(a.frames / dt, 1), "ms_per_frame": round(dt * 1e3 / a.frames, 3),
                 "live_tracks": int(live), "dicts_per_frame": round(n_out / a.frames, 1)}
res["speedup"] = round(res["device"]["frames_per_s"] / res["oracle_cpu"]["frames_per_s"], 2)
print(json.dumps(res))
