#!/usr/bin/env python3
"""End-to-end detect-and-track benchmark (BASELINE.json metric).

One step = one frame of every stream on this GPU through the whole hot path
(kalman/aircraft_detection_tracking.py:96-109): uint8 BGR frame in HBM -> letterbox/normalise
-> YOLOv8s+P2 forward -> Detect decode -> NMS -> EnhancedMultiTargetTracker.update per stream,
captured as one hipGraph.  Default workload = BASELINE config 3: 8 independent 640x512 streams
per GPU (batch 8), ~64 live tracks per stream, bf16 convs.  Multi-GPU (torchrun): streams are
sharded one group per GPU with no data-path collective (weak scaling); RCCL only reduces the
end-of-run counters and the max wall time.

Prints ONE JSON line on rank 0.
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

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"

METRIC = "end-to-end frames/sec (640×512 YOLOv8s+P2, 64 tracks) at 1/2/4/8 GPUs"
PEAK = {"bf16": 2500.0, "fp32": 157.3, "fp8": 5000.0}  # dense MFMA TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK = 8000.0  # GB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 5],
                    help="BASELINE config: 2 = 640x512 batch 1, ~16 live tracks; 3 = 640x512, ~64 live tracks/stream (the metric's workload); "
                         "5 = 1280x1024 at imgsz 1280, ~256 live tracks/stream, 150-frame occlusion bursts")
    ap.add_argument("--streams", type=int, default=None,
                    help="streams (= frames per forward) per GPU (default 8; 1 for config 2)")
    ap.add_argument("--targets", type=int, default=None,
                    help="synthetic targets per stream (22 -> ~64 live tracks/stream: the planted detector plus lost-track retention)")
    ap.add_argument("--scale", default="s", choices=["n", "s"])
    ap.add_argument("--frame", default="", help="frame size WxH (e.g. 1920x1080): frames off the network scale are "
                                                 "letterboxed with the device resize; with --imgsz")
    ap.add_argument("--imgsz", type=int, default=0, help="network input size (default: the config's)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32", "fp8"],
                    help="activation/weight dtype (default: fp8 for --config 5, else bf16)")
    ap.add_argument("--frames", type=int, default=120, help="pre-rendered frames per stream (cycled)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--frame-copy", default="copy", choices=["copy", "none"],
                    help="how each step's frames reach the detector's input buffer (none: diagnostic only)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run tracker(t) on the detector's stream instead of overlapping it with detector(t+1)")
    ap.add_argument("--no-tune", action="store_true", help="skip the per-op conv kernel autotune")
    ap.add_argument("--lanes", type=int, default=None,
                    help="streams per batch group the detector's op DAG runs on (default 1 with --inflight > 1, else 3)")
    ap.add_argument("--groups", type=int, default=1, help="independent sub-batches run concurrently")
    ap.add_argument("--tracker", default="enhanced", choices=["enhanced", "motion_reset"],
                    help="tracker: kalman.EnhancedMultiTargetTracker (the driver's) or the camera_motion_compensation "
                         "MotionCompensatedMultiTracker policy (frame-free)")
    ap.add_argument("--inflight", type=int, default=3, choices=range(1, 9),
                    help="detector forwards in flight (each a batch of all streams, own graph + HIP stream)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--plan-out", default="", help="write the autotuned conv plan (json) here")
    ap.add_argument("--plan-in", default="", help="load a conv plan (json) instead of autotuning")
    ap.add_argument("--dump-ops", default="", help="write per-op device times (json) to this path")
    return ap.parse_args()


def dist_setup():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return ws, rank, local


def roofline(pipe, frames, dtype, B):
    """Per-op device times (hipEvents on the launch stream), grouped by kernel instantiation;
    the dominant one gives the roofline entry."""
    prof = pipe.model.profile(frames, pipe.conf, pipe.iou, pipe.max_det, reps=5)
    flops = pipe.prog.op_flops(B)
    by = {}
    for (i, kind, name, ms), fl in zip(prof, flops):
        d = by.setdefault(name, {"ms": 0.0, "flops": 0, "launches": 0})
        d["ms"] += ms
        d["flops"] += fl
        d["launches"] += 1
    dom = max(by, key=lambda k: by[k]["ms"])
    d = by[dom]
    avg_ms = d["ms"] / d["launches"]
    ach = d["flops"] / (d["ms"] * 1e-3) / 1e12 if d["ms"] > 0 else 0.0
    total_ms = sum(v["ms"] for v in by.values())
    return {
        "kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": PEAK[dtype], "unit": "TFLOP/s",
        "frac": round(ach / PEAK[dtype], 5), "traffic": pmc_traffic(dom), "traffic_unit": "bytes/launch", "avg_launch_us": round(avg_ms * 1e3, 2),
        "launches_per_step": d["launches"], "flops_per_launch": int(d["flops"] / d["launches"]),
        "share_of_detect_time": round(d["ms"] / total_ms, 3),
    }, by, prof


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, separate passes), or None."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            k = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    short = kernel.replace("yk::det::", "").replace("yk::trk::", "")
    v = k.get(short)
    return None if v is None else round(v["hbm_bytes_per_launch"])


def tracker_roofline(pipe, reps=20):
    """Tracker step kernel alone (events around yk_tracker_step on the launch stream); algorithmic
    bytes per track-step from SURVEY §8d (1,216 B: R+W of x and dense P, z, box)."""
    torch.cuda.synchronize()
    _, stats = pipe.stats()
    live = int(stats["current_active_tracks"].sum())
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # replay from a snapshot-free state: timing only (the tracker keeps evolving, which is fine)
    e0.record(st)
    for _ in range(reps):
        pipe.tracker.step_device(pipe.dets, pipe.counts)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    by = live * 1216
    gbps = by / (us * 1e-6) / 1e9 if us > 0 else 0.0
    return {"kernel": "step_kernel", "bound": "hbm", "avg_launch_us": round(us, 2), "live_tracks": live,
            "achieved": round(gbps, 3), "peak": HBM_PEAK, "unit": "GB/s", "frac": round(gbps / HBM_PEAK, 6)}


def cpu_baseline(P, scale, seconds, targets, seed=0, hw=(512, 640), imgsz=640, tracker="enhanced"):
    """Reference-equivalent CPU path (oracle: torch-CPU fp32 YOLOv8s+P2 + numpy tracker) on a
    bounded sample of one stream, threads as the reference's select_device: min(8, ncpu-1)."""
    from oracle import detector_ref as D
    from oracle.tracker_ref import RefMultiTracker

    threads = min(8, (os.cpu_count() or 2) - 1)
    torch.set_num_threads(threads)
    ar = P.arch.parse_arch(P.arch.load_model_dict(f"yolov8{scale}-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, seed)
    layers = [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
              for Ly in ar.layers]
    det = D.RefDetector(layers, sd, P.arch.detect_strides(ar))
    sc = P.synth.Scene(seed=seed, n_targets=targets, n_frames=400, height=hw[0], width=hw[1])
    if tracker == "motion_reset":
        from oracle.cmc_ref import RefCMCMultiTracker
        trk = RefCMCMultiTracker(150, 1, 0.1)
    else:
        trk = RefMultiTracker(150, 1, 0.1)
    n, t_total = 0, 0.0
    for t in range(400):
        f = sc.frame(t)
        t0 = time.perf_counter()
        res, _ = D.predict(det, [f], 0.25, 0.7, 300, imgsz)
        boxes = res[0][:, :4].numpy()
        scores = res[0][:, 4].numpy()
        dets = [[b[0], b[1], b[2], b[3], s] for b, s in zip(boxes, scores) if s > 0.1]
        trk.update(dets)
        dt = time.perf_counter() - t0
        if t >= 2:  # warm-up frames
            n += 1
            t_total += dt
            if t_total > seconds:
                break
    return {"value": round(n / t_total, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames of one {hw[1]}x{hw[0]} stream ({targets} targets), YOLOv8{scale}+P2 fp32 torch-CPU "
                      f"({threads} threads) + numpy {tracker} tracker, after 2 warm-up frames"}


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    ws, rank, local = dist_setup()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    P = importlib.import_module(PKG)
    from importlib import import_module

    pipeline = import_module(PKG + ".pipeline")
    if a.streams is None:
        a.streams = 1 if a.config == 2 else 8
    if a.lanes is None:
        a.lanes = 1 if a.inflight > 1 and not a.no_pipeline else 3
    if a.dtype is None:
        a.dtype = "fp8" if a.config == 5 else "bf16"
    S = a.streams
    H, W, imgsz, max_tracks = (1024, 1280, 1280, 2048) if a.config == 5 else (512, 640, 640, 512)
    if a.frame:
        W, H = (int(v) for v in a.frame.lower().split("x"))
    if a.imgsz:
        imgsz = a.imgsz
    if a.targets is None:
        a.targets = {2: 6, 3: 22, 5: 66}[a.config]
    shard = P.shard
    my_streams = shard.stream_ids(rank, ws, S)  # this GPU's block of independent streams
    pipe = pipeline.StreamPipeline(f"yolov8{a.scale}-small.yaml", S, (H, W), a.dtype, seed=0, device=local,
                                   pipelined=not a.no_pipeline, imgsz=imgsz, max_tracks=max_tracks,
                                   inflight=1 if a.no_pipeline else a.inflight,
                                   tracker_policy=1 if a.tracker == "motion_reset" else 0)
    # pre-render frames of every stream into HBM (inputs resident before the timed region)
    F = max(2, min(a.frames, a.warmup + a.steps))
    scenes = [P.synth.Scene(seed=shard.stream_seed(g, S), n_targets=a.targets, n_frames=F + 1, width=W, height=H)
              for g in my_streams]
    frames = torch.empty((F, S, H, W, 3), dtype=torch.uint8, device=dev)
    for s, sc in enumerate(scenes):
        frames[:, s] = sc.frames_torch(0, F, dev)
    torch.cuda.synchronize()
    log("frames resident; setting schedule")
    pipe.set_schedule(a.groups, a.lanes)
    pipe.frames.copy_(frames[0])
    tune = not a.no_tune
    if a.plan_in:
        with open(a.plan_in) as f:
            pl = json.load(f)
        pipe.model.load_plan(pl["batch"], pl["plan"])
        tune = False
    if not a.no_graph:
        pipe.capture(tune=tune)
    elif tune:
        pipe.model.autotune(pipe.frames, pipe.conf)
        pipe.sync_plan()
    if a.plan_out and rank == 0:
        b, pl = pipe.model.get_plan()
        with open(a.plan_out, "w") as f:
            json.dump({"batch": b, "plan": pl}, f)
    log("graph captured; warm-up")
    # warm-up
    for t in range(a.warmup):
        pipe.run(frames[t % F])
    torch.cuda.synchronize()
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(a.steps):
        if a.frame_copy == "none":
            pipe.step()
        else:
            pipe.run(frames[(a.warmup + t) % F])
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log(f"timed {a.steps} steps in {elapsed:.3f}s")
    counts, stats = pipe.stats()
    live = float(stats["current_active_tracks"].mean())
    frames_done = S * a.steps
    # PCIe-inclusive rate (host frames -> device each step): informational, never `value`
    host = frames[0].cpu().pin_memory()
    torch.cuda.synchronize()
    tp = time.perf_counter()
    n_pcie = min(20, a.steps)
    for _ in range(n_pcie):
        pipe.frames.copy_(host, non_blocking=True)
        pipe.step()
    torch.cuda.synchronize()
    pcie_fps = S * n_pcie / (time.perf_counter() - tp)
    # end-of-run exchange (RCCL): SUM of counters, MAX of wall time -- the only collective
    run, elapsed = shard.reduce_run(shard.local_counters(frames_done, stats), elapsed, dev)
    frames_done = int(run["frames"])
    live = run["current_active_tracks"] / (S * ws)
    fps = frames_done / elapsed
    rl = None
    trl = None
    if rank == 0 and not a.no_profile:
        bg = (S + a.groups - 1) // a.groups  # the batch each group's kernels run at
        rl, by_kernel, prof = roofline(pipe, frames[0][:bg], a.dtype, bg)
        trl = tracker_roofline(pipe)
        if a.dump_ops:
            flops = pipe.prog.op_flops(bg)
            with open(a.dump_ops, "w") as f:
                json.dump({"ops": [{"op": i, "kind": k, "kernel": n, "us": round(ms * 1e3, 2), "gflop": fl / 1e9}
                                   for (i, k, n, ms), fl in zip(prof, flops)], "by_kernel": by_kernel}, f, indent=1)
    log("profile done")
    cpu = None
    if rank == 0 and ws == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(P, a.scale, a.cpu_seconds, a.targets, hw=(H, W), imgsz=imgsz, tracker=a.tracker)
    if rank == 0:
        gflop = pipe.flops_per_frame() / 1e9
        out = {
            "metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "n_gpus": ws, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": f"synthetic: seeded {W}x{H} IR-like scenes rendered into HBM before timing; seeded "
                    "planted weights (no trained best.pt in the reference)",
            "config": {"workload": f"YOLOv8{a.scale}+P2 {W}x{H} (imgsz {imgsz}), {S} streams/GPU as batch {S}, "
                                   f"{a.targets} targets/stream, {a.tracker} tracker(150, 1, 0.1) (BASELINE config {a.config})",
                       "streams_per_gpu": S, "global_batch": S * ws, "parallelism": f"streams sharded over {ws} GPU(s)",
                       "graph": not a.no_graph, "tracker_overlapped": not a.no_pipeline, "autotuned": not a.no_tune, "dag_lanes": a.lanes,
                       "batch_groups": a.groups, "detector_inflight": pipe.D,
                       "live_tracks_per_stream": round(live, 1),
                       "tracks_created": int(run["total_tracks_created"]),
                       "gflop_per_frame": round(gflop, 3)},
            "network_mfma_frac": round(fps / ws * gflop / 1e3 / PEAK[a.dtype], 5),
            "pcie_inclusive_fps": round(pcie_fps * ws, 2),
            "roofline": rl, "tracker_roofline": trl, "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
