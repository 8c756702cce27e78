#!/usr/bin/env python3
"""Refine a conv plan by whole-pipeline throughput (the regime bench.py measures).

The autotuners time one op at a time (yk_model_autotune; tools/tune_concurrent.py at batch 16 as
a proxy for the forwards in flight), which ranks variants by latency.  bench.py's line is
throughput-bound instead: four batch-8 forwards in flight share the chip, and a variant that is
slower alone but issues fewer loads / VALU per MFMA can be the faster one there.  This tool keeps
one config-3 StreamPipeline (fp32, 8 streams, 4 forwards in flight, one lane -- bench.py's
defaults) and, for the ops with the largest isolated time, tries the variants that are within
--slack of the op's best isolated time, re-capturing the graphs and timing --steps pipelined
steps per trial; a change is kept only if it also wins the A/B re-measure.

usage: plan_refine.py [--plan plans/s_640x512_i640_b8_fp32.json] [--out gpurun_out/plan_refined.json]
                      [--ops 30] [--steps 150] [--slack 1.25]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"


def candidates():
    out = []
    for mode in range(3):
        for nnt in (1, 2, 3, 4):
            for npt in (1, 2, 4):
                out.append((3, nnt, npt | (mode << 4) | 64))
    for ne in (1, 2):
        for npt in (1, 2, 4):
            for wm in (0, 1):
                out.append((5, ne, npt | (wm << 4)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", default=os.path.join(REPO, "plans", "s_640x512_i640_b8_fp32.json"))
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "plan_refined.json"))
    ap.add_argument("--ops", type=int, default=30, help="ops tried, by isolated time")
    ap.add_argument("--steps", type=int, default=150, help="timed pipelined steps per trial")
    ap.add_argument("--slack", type=float, default=1.25, help="variants within this factor of the op's best "
                                                              "isolated time are tried")
    ap.add_argument("--max-trials", type=int, default=4, help="variants tried per op")
    a = ap.parse_args()
    P = importlib.import_module(PKG)
    pipeline = importlib.import_module(PKG + ".pipeline")
    L = importlib.import_module(PKG + "._lib")
    S, H, W, F = 8, 512, 640, 240
    dev = torch.device("cuda", 0)
    frames = torch.empty((F, S, H, W, 3), dtype=torch.uint8, device=dev)
    for s in range(S):
        sc = P.synth.Scene(seed=P.shard.stream_seed(s, S), n_targets=40, n_frames=F + 1, width=W, height=H)
        frames[:, s] = sc.frames_torch(0, F, dev)
    pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (H, W), "fp32", seed=0, pipelined=True, inflight=4,
                                   max_tracks=512)
    pipe.set_schedule(1, 1)
    plan = json.load(open(a.plan))["plan"]
    B = 8
    for m in pipe.models:
        m.load_plan(B, plan)
    pipe.frames.copy_(frames[0])
    pipe.capture(tune=False)
    t_run = [0]

    def measure(n):
        for _ in range(20):  # settle the re-captured graphs
            pipe.run(frames[t_run[0] % F])
            t_run[0] += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            pipe.run(frames[t_run[0] % F])
            t_run[0] += 1
        torch.cuda.synchronize()
        return n * S / (time.perf_counter() - t0)

    def apply(op, v):
        for m in pipe.models:
            m.set_plan(B, v[0], v[1], v[2], op)
        pipe.capture(tune=False)

    for _ in range(160 // 8):  # track load, as bench.py's pre-roll
        measure(8)
    base = np.median([measure(a.steps) for _ in range(3)])
    print(json.dumps({"start_plan": os.path.relpath(a.plan, REPO), "fps": round(base, 1)}), flush=True)
    m0 = pipe.models[0]
    prof = m0.profile(pipe.frames, reps=3)
    conv_ops = [i for i in range(len(plan)) if plan[i][0] >= 0]
    order = sorted(conv_ops, key=lambda i: -prof[i][3])[: a.ops]
    cands = candidates()
    log = []
    for op in order:
        cur = tuple(plan[op])
        # isolated time of every variant of this op (one forward at a time)
        iso = []
        for v in cands:
            try:
                for m in pipe.models:
                    m.set_plan(B, v[0], v[1], v[2], op)
            except L.YKError:
                continue
            iso.append((m0.profile(pipe.frames, reps=3)[op][3], v))
        apply(op, cur)
        if not iso:
            continue
        best_iso = min(t for t, _ in iso)
        trial = [v for t, v in sorted(iso) if t <= a.slack * best_iso and v != cur][: a.max_trials]
        best_v, best_fps = cur, measure(a.steps)
        for v in trial:
            apply(op, v)
            f = measure(a.steps)
            if f > best_fps:
                best_v, best_fps = v, f
        if best_v != cur:  # A/B re-measure: the winner against the op's current variant, twice each
            ab = {}
            for v in (cur, best_v, cur, best_v):
                apply(op, v)
                ab.setdefault(v, []).append(measure(a.steps))
            gain = np.mean(ab[best_v]) / np.mean(ab[cur])
            if gain > 1.003:
                plan[op] = list(best_v)
            else:
                best_v = cur
            rec = {"op": op, "from": list(cur), "to": list(best_v), "gain": round(float(gain), 4)}
        else:
            rec = {"op": op, "kept": list(cur)}
        apply(op, tuple(plan[op]))
        log.append(rec)
        print(json.dumps(rec), flush=True)
    final = np.median([measure(a.steps) for _ in range(3)])
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"batch": B, "plan": plan, "dtype": "fp32", "workload": "s_640x512_i640_b8_fp32.json",
                   "refined_by": "tools/plan_refine.py", "refined_from": os.path.relpath(a.plan, REPO),
                   "fps_start": round(float(base), 1), "fps_refined": round(float(final), 1)}, f)
    print(json.dumps({"out": a.out, "fps_start": round(float(base), 1), "fps_refined": round(float(final), 1),
                      "changed": sum(1 for r in log if "to" in r and r["to"] != r["from"])}), flush=True)


if __name__ == "__main__":
    main()
