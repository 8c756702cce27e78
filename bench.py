#!/usr/bin/env python3
"""End-to-end detect-and-track benchmark (BASELINE.json metric).

One step = one frame of every stream on this GPU through the whole hot path
(kalman/aircraft_detection_tracking.py:96-109): uint8 BGR frame in HBM -> letterbox/normalise
-> YOLOv8s+P2 forward -> Detect decode -> NMS -> EnhancedMultiTargetTracker.update per stream.

Workloads (BASELINE.json configs; the default is config 3, the metric's workload):
  2  640x512, 1 stream (batch 1), bf16 convs (BASELINE names bf16), >= 16 live tracks
  3  640x512, 8 streams per GPU as one batch-8 forward, fp32 convs (the reference's
     arithmetic; bf16 reported beside it as a labelled secondary leg), >= 64 live tracks/stream
  4  640x512, ONE stream per GPU (8 GPUs x 1 stream at --gpus 8), fp32, >= 64 live tracks
  5  1280x1024 at imgsz 1280, 8 streams, fp8 convs (bf16 secondary), >= 256 live tracks/stream,
     150-frame occlusion bursts

Protocol: frames are rendered into HBM before anything is timed; the committed conv plan
(plans/*.json) is loaded instead of autotuning; an untimed tracker pre-roll of --preroll frames
(independent of --steps/--warmup) brings every stream to its steady-state track load; then
--warmup untimed steps through the timed loop's body (page-locked frames in, tracker output out)
and exactly --steps timed steps between barrier + synchronize.  The run
fails if the tracker dropped anything (stats.overflow != 0).

Multi-GPU: `torchrun --nproc-per-node N bench.py --gpus N`, or `bench.py --gpus N` alone, which
starts the N rank processes itself.  Streams are sharded one block per GPU with no data-path
collective (weak scaling); RCCL only reduces the end-of-run counters and the max wall time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"

METRIC = "end-to-end frames/sec (640×512 YOLOv8s+P2, 64 tracks) at 1/2/4/8 GPUs"
PEAK = {"bf16": 2500.0, "fp32": 157.3, "fp8": 5000.0}  # dense MFMA TFLOP/s (MI355X_MICROARCH.md)
# fp32 convs on the bf16 matrix cores (F32S bodies, halo-tile kernel): three 16x16x32 bf16 MFMAs
# per 16x16x16 fp32 block, i.e. 1/6 of the dense bf16 rate in fp32 FLOPs
PEAK_F32_ON_BF16 = PEAK["bf16"] / 6.0


def kernel_peak(kernel, dtype):
    """(peak TFLOP/s, basis) of the MFMA instruction mix a conv kernel instantiation runs."""
    if dtype == "fp32" and ("F32S" in kernel or "conv_halo_kernel" in kernel):
        return PEAK_F32_ON_BF16, "fp32 on bf16 MFMA (3-way bf16 split, 6 products): dense bf16 2,500 / 6"
    return PEAK[dtype], f"dense {dtype} MFMA"
HBM_PEAK = 8000.0  # GB/s
TRACK_STEP_BYTES = 1216  # R+W of x (8 f64) and dense P (64 f64), z, box

# BASELINE.json configs -> workload.  live_floor: the live tracks per stream the config names.
# Targets per stream are set so the steady-state LIVE track count (detected + lost-but-retained
# tracks, max_lost_frames=150) meets the floor: the planted detector's ~96-px boxes merge nearby
# targets and crossing targets churn IDs, so live tracks != targets (40 targets -> ~70-150 live).
CONFIGS = {
    2: dict(S=1, H=512, W=640, imgsz=640, max_tracks=512, targets=12, dtype="bf16", secondary="", live_floor=16),
    # tbatch (frames per stream per forward, --tbatch) x inflight (forwards in flight) x prefetch depth,
    # swept at the driver's 20 steps (gpurun_out/r6f, two runs each): fp32 T1 D4 4,914-4,938, T2 D3
    # (prefetch 4) 5,131-5,183, T2 D2 5,035-5,044, T2 D4 4,839-4,874; bf16 T1 D4 11,090-11,104, T2 D3
    # 12,384-12,527, T4 D2 11,644-11,662 frames/s
    3: dict(S=8, H=512, W=640, imgsz=640, max_tracks=512, targets=40, dtype="fp32", secondary="bf16,n:fp32", live_floor=64,
            tbatch=2, inflight=3),
    # config 4: four consecutive steps of the rank's stream per forward, four forwards in flight (20 steps:
    # 2,738-2,770 frames/s vs 2,194-2,326 at one step per forward, profiles/r06_sweeps.txt r6at)
    4: dict(S=1, H=512, W=640, imgsz=640, max_tracks=512, targets=40, dtype="fp32", secondary="", live_floor=64,
            tbatch=4, inflight=4),
    # config 5: the fp8 leg runs two steps per forward, three in flight (20 steps: 4,811-4,830 vs 4,418-4,502
    # frames/s at one step, r6av); the bf16 leg keeps one step (two steps: 3,783-3,831 vs 3,653-3,756 once its
    # 2.9 GiB batch-16 arena runs on the table kernels, r6az -- within the spread)
    5: dict(S=8, H=1024, W=1280, imgsz=1280, max_tracks=2048, targets=96, dtype="fp8", secondary="bf16",
            live_floor=256, tbatch={"fp8": 2}, inflight={"fp8": 3}),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--streams", type=int, default=None, help="streams (= frames per forward) per GPU")
    ap.add_argument("--targets", type=int, default=None, help="synthetic targets per stream")
    ap.add_argument("--scale", default="s", choices=["n", "s"])
    ap.add_argument("--frame", default="", help="frame size WxH (e.g. 1920x1080): frames off the network scale are "
                                                 "letterboxed with the device resize; with --imgsz")
    ap.add_argument("--imgsz", type=int, default=0, help="network input size (default: the config's)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32", "fp8"], help="conv dtype of the headline leg")
    ap.add_argument("--secondary", default=None,
                    help="comma list of dtypes timed after the headline leg with the same protocol (default: the "
                         "config's; 'none' to skip)")
    ap.add_argument("--preroll", type=int, default=160,
                    help="untimed tracker pre-roll frames before warm-up (steady-state track load)")
    ap.add_argument("--max-frames", type=int, default=1200, help="pre-rendered frames per stream (cycled beyond)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run tracker(t) on the detector's stream instead of overlapping it with detector(t+1)")
    ap.add_argument("--autotune", action="store_true", help="autotune the conv plan instead of loading plans/*.json")
    ap.add_argument("--lanes", type=int, default=None)
    ap.add_argument("--groups", type=int, default=1, help="independent sub-batches run concurrently")
    ap.add_argument("--tracker", default="enhanced", choices=["enhanced", "motion_reset"])
    ap.add_argument("--gmd", action="store_true",
                    help="with --tracker motion_reset: also run GlobalMotionDetector('optical_flow') on every frame "
                         "(MotionCompensatedMultiTracker.update(dets, frame)); no CPU baseline (the oracle's numpy "
                         "restatement of cv2's optical flow is not a stand-in for cv2's speed)")
    ap.add_argument("--tbatch", type=int, default=None, choices=range(1, 9),
                    help="frames per stream in one forward (temporal batching: one batch-(tbatch x streams) forward "
                         "covers tbatch consecutive steps; the tracker still steps once per frame); default: the "
                         "config's")
    ap.add_argument("--inflight", type=int, default=None, choices=range(1, 9),
                    help="detector forwards in flight (each a batch of all streams, own graph + HIP stream); "
                         "default 4")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=25.0, help="CPU-baseline sample bound (default threads)")
    ap.add_argument("--cpu-all-seconds", type=float, default=10.0, help="CPU-baseline sample bound (all cores)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--plan-out", default="", help="write the headline leg's conv plan (json) here")
    ap.add_argument("--save-plans", action="store_true", help="write every leg's conv plan to plans/<workload>.json")
    ap.add_argument("--plan-in", default="", help="conv plan (json) of the headline leg (default: plans/<workload>.json)")
    ap.add_argument("--dump-ops", default="", help="write per-op device times (json) to this path")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="upload each step's host frames on its slot stream instead of one step ahead on the copy stream")
    ap.add_argument("--prefetch-depth", type=int, default=None,
                    help="how many steps ahead the host frames are uploaded (page-locked frames >= PULL_BYTES; "
                         "default 2, 4 with --tbatch > 1: one forward's steps ahead; 2 measured +1.5-4.4 %% over 1 "
                         "at fp32, profiles/r05_inflight_lanes_sweep.txt)")
    ap.add_argument("--fw-times", action="store_true",
                    help="diagnostics: each timed forward's start / end and its tracker steps' start / end (ms from "
                         "the start of the timed region, timing events on the streams) in the line's fw_times")
    ap.add_argument("--io", default="both", choices=["both", "h2d", "d2h", "none", "stage-dev"],
                    help="diagnostics: which host copies the timed loop makes (default both: the metric's definition)")
    a = ap.parse_args()
    if a.inflight is None:
        # the config's (config 3: 3 with two frames per forward, the CMC lines too: motion windows of
        # three batch-16 forwards, bf16 9,004 vs 8,208 frames/s for four forwards of one step, fp32
        # 4,420 vs 4,429, profiles/r06_sweeps.txt r6aa), else 4
        cfg = CONFIGS[a.config]
        a.inflight = 4 if a.no_pipeline else by_dtype(cfg.get("inflight", 4), a.dtype or cfg["dtype"], 4)
    return a


def by_dtype(v, dtype, default):
    """A CONFIGS schedule entry: one value, or a {dtype: value} map (default for other dtypes)."""
    return v.get(dtype, default) if isinstance(v, dict) else v


# ---------------------------------------------------------------------------- ranks
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (one per GPU) like
    torch.distributed.run does, before this process touches any GPU; exit with the first
    non-zero child status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


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


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()


# ---------------------------------------------------------------------------- measurement helpers
def roofline(pipe, frames, dtype, B):
    """Per-op device times of one forward at a time (hipEvents on the launch stream, `reps`
    back-to-back launches per op), grouped by kernel instantiation; the dominant one gives the
    roofline entry.  Returns (entry, by_kernel, per-op list, [t0_ns, t1_ns] of the pass)."""
    # two untimed passes first: the clocks the GPU settles at under load, not the ones it comes
    # back with after the host-side gap since the timed region (tools/profile_repeat.py: the
    # dominant kernel 32.2 / 29.6 / 28.6 / 28.2 us over four back-to-back passes)
    for _ in range(2):
        pipe.model.profile(frames, pipe.conf, pipe.iou, pipe.max_det, reps=5)
    t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    prof = pipe.model.profile(frames, pipe.conf, pipe.iou, pipe.max_det, reps=5)
    t1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    flops = pipe.prog.op_flops(B)
    by = {}
    for (i, kind, name, ms), fl in zip(prof, flops):
        d = by.setdefault(name, {"ms": 0.0, "flops": 0, "launches": 0})
        d["ms"] += ms
        d["flops"] += fl
        d["launches"] += 1
    conv = {k: v for k, v in by.items() if v["flops"] > 0}
    dom = max(conv, key=lambda k: conv[k]["ms"])
    d = by[dom]
    avg_ms = d["ms"] / d["launches"]
    ach = d["flops"] / (d["ms"] * 1e-3) / 1e12 if d["ms"] > 0 else 0.0
    total_ms = sum(v["ms"] for v in by.values())
    peak, basis = kernel_peak(dom, dtype)
    return {
        "kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
        "frac": round(ach / peak, 5), "peak_basis": basis, "frac_of_dtype_mfma_peak": round(ach / PEAK[dtype], 5),
        "traffic": pmc_traffic(dom, dtype), "traffic_unit": "bytes/launch",
        "avg_launch_us": round(avg_ms * 1e3, 2), "launches_per_step": d["launches"],
        "flops_per_launch": int(d["flops"] / d["launches"]), "share_of_detect_time": round(d["ms"] / total_ms, 3),
        "timing": "hipEvents around 5 back-to-back launches of each op, one forward at a time, after two untimed passes",
    }, by, prof, [t0, t1]


def decode_nms_rooflines(pipe, prof, dtype, B):
    """HBM rooflines of the decode and NMS kernels (north_star: "Kalman/NMS HBM-GB/s fractions of
    peak"), from the same per-op hipEvent pass as the conv roofline.  Algorithmic bytes per SURVEY
    §8(d): decode reads the Detect head's 65 fp32 logits per anchor (64 DFL box bins + 1 class),
    65 * A * 4 B per image, summed over the four detect_kernel launches of a forward (one per
    stride; detect_kernel fuses the head's last 1x1 convs, so its real input is the (64 + c3)
    features per anchor: `traffic` from the PMC passes); NMS reads the candidate rows that passed
    the confidence threshold (6 f32 each) and writes the kept rows (<= 300 x 6 x 4 B per image),
    counted from this forward's own candidate and detection counts."""
    det = [(name, ms) for (i, kind, name, ms) in prof if "detect_kernel" in name]
    nms = [(name, ms) for (i, kind, name, ms) in prof if name.startswith("nms_kernel")]
    A = int(pipe.prog.n_anchors)
    _, cand_n = pipe.model.candidates(B)
    kept = np.zeros(pipe.prog.max_batch, np.int32)
    P = importlib.import_module(PKG)
    P.model._memcpy_d2h(kept, pipe.model.counts_ptr)
    out = {}
    if det:
        ms = sum(m for _, m in det)
        by = 65 * A * 4 * B
        gbps = by / (ms * 1e-3) / 1e9
        out["detect_roofline"] = {
            "kernel": det[0][0], "bound": "hbm", "achieved": round(gbps, 2), "peak": HBM_PEAK, "unit": "GB/s",
            "frac": round(gbps / HBM_PEAK, 5), "algorithmic_bytes_per_forward": by, "launches_per_step": len(det),
            "avg_launch_us": round(ms / len(det) * 1e3, 2), "us_per_forward": round(ms * 1e3, 2),
            "traffic": pmc_traffic(det[0][0], dtype), "traffic_unit": "bytes/launch (PMC, mean over the 4 strides)",
            "bytes_basis": "SURVEY §8(d): 65 logits x A anchors x 4 B per image, A = %d, batch %d" % (A, B)}
    if nms:
        ms = sum(m for _, m in nms)
        n_in, n_out = int(cand_n[:B].sum()), int(kept[:B].sum())
        by = (n_in + n_out) * 6 * 4
        gbps = by / (ms * 1e-3) / 1e9
        out["nms_roofline"] = {
            "kernel": nms[0][0], "bound": "hbm", "achieved": round(gbps, 3), "peak": HBM_PEAK, "unit": "GB/s",
            "frac": round(gbps / HBM_PEAK, 6), "algorithmic_bytes_per_launch": by, "launches_per_step": len(nms),
            "avg_launch_us": round(ms / len(nms) * 1e3, 2), "candidates_in": n_in, "detections_out": n_out,
            "traffic": pmc_traffic(nms[0][0], dtype), "traffic_unit": "bytes/launch",
            "bytes_basis": "SURVEY §8(d): candidate rows read + kept rows written, 6 x f32 each, batch %d" % B}
    return out


def pmc_traffic(kernel, dtype):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py: FETCH_SIZE + WRITE_SIZE, separate passes), or None."""
    for path in (os.path.join(REPO, "profiles", f"pmc_traffic_{dtype}.json"),
                 os.path.join(REPO, "profiles", "pmc_traffic.json")):
        try:
            with open(path) as f:
                k = json.load(f)["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        short = kernel.replace("yk::det::", "").replace("yk::trk::", "")
        v = k.get(short)
        if v is not None:
            return round(v["hbm_bytes_per_launch"])
    return None


def tracker_roofline(pipe, reps=20):
    """Tracker step kernel alone (events around yk_tracker_step on the launch stream); algorithmic
    bytes per track-step from SURVEY §8d (1,216 B)."""
    torch.cuda.synchronize()
    _, stats = pipe.stats()
    live = int(stats["current_active_tracks"].sum())
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        pipe.tracker.step_device(pipe.dets, pipe.counts)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    by = live * TRACK_STEP_BYTES
    gbps = by / (us * 1e-6) / 1e9 if us > 0 else 0.0
    return {"kernel": "assoc_kernel + tracks_kernel", "bound": "hbm", "avg_launch_us": round(us, 2), "live_tracks": live,
            "achieved": round(gbps, 3), "peak": HBM_PEAK, "unit": "GB/s", "frac": round(gbps / HBM_PEAK, 6)}


def tbatch_of(a, cfg, dtype) -> int:
    """Frames per stream in one forward (temporal batching); 1 without forwards in flight."""
    tb = a.tbatch if a.tbatch is not None else by_dtype(cfg.get("tbatch", 1), dtype, 1)
    if a.no_pipeline or a.inflight < 2:
        tb = 1
    return tb


def plan_path(a, dtype, S, W, H, imgsz):
    return os.path.join(REPO, "plans", f"{a.scale}_{W}x{H}_i{imgsz}_b{S}_{dtype}.json")


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------- CPU baseline
def _cpu_quota() -> int:
    """CPUs this process may use: affinity, capped by a cgroup v2 cpu.max quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(P, scale, S, targets, hw, imgsz, tracker, threads, seconds, warm_frames=10, max_frames=300):
    """Reference-equivalent CPU path (the oracle: torch-CPU fp32 YOLOv8+P2 incl. NMS with the
    TorchNMS quirk + the numpy tracker with its Python IoU loop) on the same workload shape:
    S frames per forward (one frame per stream) and S trackers stepped one after another, as
    BASELINE.md's protocol says; time.perf_counter around each whole step (detector / NMS /
    tracker split recorded), >= `warm_frames` warm-up frames, then up to `max_frames` frames or
    `seconds` of timed steps, whichever comes first."""
    from oracle import detector_ref as D
    from oracle.tracker_ref import RefMultiTracker

    torch.set_num_threads(threads)
    ar = P.arch.parse_arch(P.arch.load_model_dict(f"yolov8{scale}-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    layers = [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
              for Ly in ar.layers]
    det = D.RefDetector(layers, sd, P.arch.detect_strides(ar))
    warm_steps = -(-warm_frames // S)
    max_steps = warm_steps + max(1, -(-max_frames // S))
    scenes = [P.synth.Scene(seed=s, n_targets=targets, n_frames=max_steps + 1, height=hw[0], width=hw[1])
              for s in range(S)]
    frames = [sc.frames_torch(0, max_steps, "cpu").numpy() for sc in scenes]
    if tracker == "motion_reset":
        from oracle.cmc_ref import RefCMCMultiTracker
        trks = [RefCMCMultiTracker(150, 1, 0.1) for _ in range(S)]
    else:
        trks = [RefMultiTracker(150, 1, 0.1) for _ in range(S)]
    step_ms, split = [], np.zeros(3)
    t_total = 0.0
    for t in range(max_steps):
        batch = [frames[s][t] for s in range(S)]
        t0 = time.perf_counter()
        with torch.no_grad():
            im = D.preprocess(batch, imgsz)
            y, _ = det.forward(im)
            t1 = time.perf_counter()
            out = D.non_max_suppression(y, 0.25, 0.7, 300)
            res = [D.scale_clip(p, im.shape[2:], batch[0].shape[:2]) for p in out]
        t2 = time.perf_counter()
        for s in range(S):
            boxes = res[s][:, :4].numpy()
            scores = res[s][:, 4].numpy()
            trks[s].update([[b[0], b[1], b[2], b[3], c] for b, c in zip(boxes, scores) if c > 0.1])
        t3 = time.perf_counter()
        if t >= warm_steps:
            step_ms.append((t3 - t0) * 1e3)
            split += (t1 - t0, t2 - t1, t3 - t2)
            t_total += t3 - t0
            if t_total > seconds:
                break
    n = len(step_ms)
    live = float(np.mean([len(tr.trackers) for tr in trks]))
    per_frame = np.asarray(step_ms) / S
    return {"value": round(n * S / t_total, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "median_ms_per_frame": round(float(np.median(per_frame)), 3),
            "p90_ms_per_frame": round(float(np.percentile(per_frame, 90)), 3),
            "split_ms_per_frame": {"detector": round(split[0] / (n * S) * 1e3, 3), "nms": round(split[1] / (n * S) * 1e3, 3),
                                   "tracker": round(split[2] / (n * S) * 1e3, 3)},
            "live_tracks_per_stream": round(live, 1),
            "sample": f"{n} timed steps x {S} frames ({S} stream(s) of {hw[1]}x{hw[0]}, {targets} targets each; one "
                      f"batch-{S} forward + {S} numpy {tracker} trackers per step) after {warm_steps * S} warm-up "
                      f"frames; YOLOv8{scale}+P2 fp32 torch-CPU, {threads} threads"}


# ---------------------------------------------------------------------------- one timed leg
def run_leg(a, P, cfg, dtype, frames, dev, local, rank, ws, headline):
    pipeline = importlib.import_module(PKG + ".pipeline")
    S, H, W, imgsz = cfg["S"], cfg["H"], cfg["W"], cfg["imgsz"]
    F = frames.shape[0]
    lanes = a.lanes if a.lanes is not None else 1  # (the model's default schedule: one lane)
    tb = tbatch_of(a, cfg, dtype)
    pipe = pipeline.StreamPipeline(f"yolov8{a.scale}-small.yaml", S, (H, W), dtype, seed=0, device=local,
                                   pipelined=not a.no_pipeline, imgsz=imgsz, max_tracks=cfg["max_tracks"],
                                   inflight=1 if a.no_pipeline else a.inflight,
                                   tracker_policy=1 if a.tracker == "motion_reset" else 0,
                                   motion_method="optical_flow" if a.gmd else None, frames_per_forward=tb)
    pipe.set_schedule(a.groups, lanes)
    pipe.frames.copy_(frames[0])
    plan_src, parity = "heuristic", None
    pth = (a.plan_in if (headline and a.plan_in) else plan_path(a, dtype, (tb * S + a.groups - 1) // a.groups, W, H, imgsz))
    tune = a.autotune
    if not tune and os.path.exists(pth):
        with open(pth) as f:
            pl = json.load(f)
        if len(pl["plan"]) != len(pipe.prog.ops):
            raise SystemExit(f"conv plan {pth} has {len(pl['plan'])} ops, the program {len(pipe.prog.ops)}: "
                             "regenerate it with --autotune --plan-out")
        for m in pipe.models:
            m.load_plan(pl["batch"], pl["plan"])
        plan_src = os.path.relpath(pth, REPO)
        # the plan's chain-parity record: near-tie flips / order ties of this plan over the
        # 1,280-stream-frame oracle chain, asserted by tests/test_bench_pipeline_gpu.py
        parity = pl.get("parity")
    elif not tune:
        log(f"no committed conv plan at {pth}: autotuning")
        tune = True
    if tune:
        plan_src = "autotuned at run time"
    if not a.no_graph:
        pipe.capture(tune=tune)
    elif tune:
        pipe.model.autotune(pipe.forward_frames, pipe.conf)
        pipe.sync_plan()
    for out_path in ([a.plan_out] if headline and a.plan_out else []) + ([pth] if a.save_plans else []):
        if rank == 0:
            b, pl = pipe.model.get_plan()
            os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
            with open(out_path, "w") as f:
                json.dump({"batch": b, "plan": pl, "dtype": dtype, "workload": os.path.basename(pth)}, f)
    # the metric runs from the frame in host memory to the tracker output.  The
    # timed steps' frames wait in page-locked host memory (the driver's decoded frames); every
    # step copies its S frames host -> HBM on the slot's stream in front of the forward that reads
    # them, and enqueues the tracker output (counts, stats, every row) device -> host behind the
    # tracker step.  Both copies are inside the timed region.  The host buffers are set up before
    # the pre-roll and warm-up, so the warm-up steps run right before the timed ones: a GPU left
    # idle for the tens of ms those page-locked allocations and staging copies take comes back at
    # lower clocks (the per-op profile pass: the dominant kernel 32 us after a 0.5 s pause, 28 us
    # after three back-to-back passes, tools/profile_repeat.py).
    n_pre = a.preroll
    t_first = n_pre + a.warmup
    n_host = min(a.steps, F)
    host = torch.empty((n_host,) + tuple(frames.shape[1:]), dtype=torch.uint8, pin_memory=True)
    for j in range(n_host):
        host[j].copy_(frames[(t_first + j) % F])
    # the warm-up steps' own frames, also in page-locked memory: the warm-up runs the timed loop's
    # body (host frames uploaded ahead, tracker output pushed back), so the copy engines and their
    # page mappings are in use right before the timed steps (a warm-up from HBM frames left the
    # first timed forward waiting 2.4 ms for its uploads at bf16, r6ai)
    n_warm = min(a.warmup, F)
    host_w = torch.empty((max(n_warm, 1),) + tuple(frames.shape[1:]), dtype=torch.uint8, pin_memory=True)
    for j in range(n_warm):
        host_w[j].copy_(frames[(n_pre + j) % F])
    # a video driver's decode buffers are long-lived and already DMA-mapped: one untimed upload of
    # each host frame (the first DMA from a fresh page-locked page costs its mapping)
    sink = torch.empty_like(frames[0])
    for j in range(n_host):
        sink.copy_(host[j], non_blocking=True)
    for j in range(n_warm):
        sink.copy_(host_w[j], non_blocking=True)
    torch.cuda.synchronize()
    del sink
    n_rows = pipe.tracker.n_streams * pipe.tracker.max_tracks
    out_rows = torch.empty(n_rows * P._lib.TRACK_OUT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
    out_counts = torch.empty(S, dtype=torch.int32, pin_memory=True)
    out_stats = torch.empty(S * P._lib.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
    h2d, d2h = a.io in ("both", "h2d", "stage-dev"), a.io in ("both", "d2h")
    if a.io == "stage-dev":  # diagnostics: the host path's copy-stream structure, frames from HBM
        host = frames[t_first:t_first + n_host].clone() if t_first + n_host <= F else host.to(dev)
        host_w = frames[n_pre:n_pre + n_warm].clone() if n_pre + n_warm <= F else host_w.to(dev)
    io_side = None if h2d else torch.cuda.Stream(dev)
    big = host[0].numel() >= pipe.PULL_BYTES or a.io == "stage-dev"
    depth = a.prefetch_depth if a.prefetch_depth is not None else (4 if tb > 1 else 2)
    ahead = depth if pipe.D > 1 and big and not a.no_prefetch else 0

    def steps(hbuf, n, t_dev):
        """n steps of the timed loop's body on page-locked frames hbuf[t % len] (from HBM, frame
        t_dev + t, without --io h2d); returns the host time spent enqueueing."""
        ns = 0
        for t in range(n):
            h0 = time.perf_counter_ns()
            if h2d:  # the next steps' frames are uploaded while this step runs (decode-ahead driver)
                pipe.run(hbuf[t % len(hbuf)])
                for u in range(t + 1 + pipe.n_prefetched, min(t + 1 + ahead, n)):
                    pipe.prefetch(hbuf[u % len(hbuf)])
            else:  # (frames from HBM: issued from a created stream, see the HBM-resident pass below)
                with torch.cuda.stream(io_side):
                    pipe.run(frames[(t_dev + t) % F])
            if d2h:
                pipe.download_async(out_rows, out_counts, out_stats)
            ns += time.perf_counter_ns() - h0
        return ns

    # untimed pre-roll (steady-state track load, independent of --steps/--warmup), then the
    # warm-up through the timed loop's body.  The ranks line up first, so they finish the warm-up
    # together and none idles long at the barrier before the timed steps (the same clock drop as
    # above)
    barrier(ws)
    for t in range(n_pre):
        pipe.run(frames[t % F])
    steps(host_w[:n_warm], n_warm, n_pre)
    pipe.flush()
    _, st0 = pipe.stats()
    live_start = st0["current_active_tracks"].astype(np.float64)
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    if a.fw_times:
        ev_t0 = torch.cuda.Event(enable_timing=True)
        ev_t0.record()
        pipe.fw_events = []
    host_ns = steps(host, a.steps, t_first)
    pipe.flush()  # (motion windows: the last partial wave's motion + tracker steps, inside the timing)
    torch.cuda.synchronize()
    barrier(ws)
    elapsed = time.perf_counter() - t0
    fw_times = None
    if a.fw_times:
        fw_times = [[round(ev_t0.elapsed_time(e), 3) if e is not None else None for e in evs] for evs in pipe.fw_events]
        pipe.fw_events = None
    w1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    log(f"{dtype}: timed {a.steps} steps (host frames in, tracker output out) in {elapsed:.4f}s")
    counts, stats = pipe.stats()
    # the host copy of the last step's output is the tracker's own
    rows_dev, _, _ = pipe.tracker.download()
    rows_host = out_rows.numpy().view(P._lib.TRACK_OUT_DTYPE).reshape(S, -1)
    if d2h and not np.array_equal(out_counts.numpy(), counts) or d2h and any(
            rows_host[s, :counts[s]].tobytes() != rows_dev[s, :counts[s]].tobytes() for s in range(S)):
        raise SystemExit("bench: the per-step tracker output copied to the host differs from the tracker's")
    # informational: the same steps with the frames already resident in HBM and no output copy.
    # Issued from a created stream: run() orders a device source behind the caller's current stream,
    # and on the legacy null stream that wait would also order it behind every other blocking stream
    # (the forwards in flight), serialising the steps
    torch.cuda.synchronize()
    barrier(ws)
    side = torch.cuda.Stream(dev)
    th = time.perf_counter()
    with torch.cuda.stream(side):
        for t in range(a.steps):
            pipe.run(frames[(t_first + a.steps + t) % F])
        pipe.flush()
    torch.cuda.synchronize()
    barrier(ws)
    hbm_elapsed = time.perf_counter() - th
    frames_done = S * a.steps
    overflow = int(stats["overflow"].sum())
    shard = P.shard
    local_c = shard.local_counters(frames_done, stats)
    local_c["live_min_start"] = float(live_start.min())
    devices = shard.gather_devices(shard.device_identity(dev))  # raises unless one rank per GPU
    run, elapsed_max = shard.reduce_run(local_c, elapsed, dev)
    _, hbm_max = shard.reduce_run({"frames": float(frames_done)}, hbm_elapsed, dev)
    fps = run["frames"] / elapsed_max
    gflop = pipe.flops_per_frame() / 1e9
    leg = {"dtype": dtype, "value": round(fps, 2), "ms_per_step": round(elapsed_max / a.steps * 1e3, 4),
           "hbm_resident_fps": round(run["frames"] / max(hbm_max, 1e-12), 2),
           "host_enqueue_ms_per_step": round(host_ns / a.steps / 1e6, 4),
           "network_mfma_frac": round(fps / ws * gflop / 1e3 / PEAK[dtype], 5),
           "live_tracks_per_stream": round(run["current_active_tracks"] / (S * ws), 1),
           "live_tracks_per_stream_min_at_start": int(live_start.min()),
           "overflow": int(run["overflow"]), "tracks_created": int(run["total_tracks_created"]),
           "conv_plan": plan_src, "conv_plan_parity": parity, "window_monotonic_ns": [w0, w1],
           "frames_per_forward": tb,
           "rank_devices": devices}
    if fw_times is not None:
        leg["fw_times"] = fw_times
    if overflow:
        log(f"tracker overflow on this rank: {overflow} detections/tracks dropped")
    if rank == 0 and not a.no_profile:
        bg = (tb * S + a.groups - 1) // a.groups  # images per forward (per batch group)
        rl, by_kernel, prof, win = roofline(pipe, frames[0].repeat(tb, 1, 1, 1)[:bg].contiguous(), dtype, bg)
        rl["window_monotonic_ns"] = win
        leg["roofline"] = rl
        leg.update(decode_nms_rooflines(pipe, prof, dtype, bg))
        leg["tracker_roofline"] = tracker_roofline(pipe)
        if headline and a.dump_ops:
            flops = pipe.prog.op_flops(bg)
            with open(a.dump_ops, "w") as f:
                json.dump({"ops": [{"op": i, "kind": k, "kernel": n, "us": round(ms * 1e3, 2), "gflop": fl / 1e9}
                                   for (i, k, n, ms), fl in zip(prof, flops)], "by_kernel": by_kernel}, f, indent=1)
    leg["gflop_per_frame"] = round(gflop, 3)
    del pipe
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return leg


def cpu_baseline_seconds(a, rank, ws):
    """Sample bound of the CPU baseline this rank runs, or 0: rank 0 only, after every rank's
    timed region; at N > 1 a shorter sample (<= 10 s; the other ranks are idle by then), so a
    scaling line carries the same baseline beside it.  None with --no-cpu-baseline or --gmd."""
    if rank != 0 or a.no_cpu_baseline or a.gmd:
        return 0
    return a.cpu_seconds if ws == 1 else min(a.cpu_seconds, 10.0)


def leg_argv(argv, dtype, scale=None):
    """bench.py's own arguments for a secondary leg: the same workload and protocol, `dtype` as
    the only leg (and `scale`, if given, as the model scale), no CPU baseline, no plan / op-dump
    outputs, one process (no --gpus)."""
    skip = {"--dtype", "--secondary", "--dump-ops", "--plan-in", "--plan-out", "--gpus"} | ({"--scale"} if scale else set())
    out, i = [], 0
    while i < len(argv):
        t = argv[i]
        key = t.split("=", 1)[0]
        if key in skip:
            i += 1 if "=" in t else 2
            continue
        if key in ("--no-cpu-baseline", "--save-plans"):
            i += 1
            continue
        out.append(t)
        i += 1
    return out + ["--dtype", dtype, "--secondary", "none", "--no-cpu-baseline"] + (["--scale", scale] if scale else [])


def run_leg_subprocess(spec):
    """One more leg (same workload and protocol, another conv dtype -- "bf16" -- or another model
    scale and dtype -- "n:fp32", the reference's trained scale) as its own bench.py process;
    returns its leg dict.  Only used at world size 1 (secondary legs)."""
    scale, dtype = spec.split(":") if ":" in spec else (None, spec)
    cmd = [sys.executable, os.path.abspath(__file__)] + leg_argv(sys.argv[1:], dtype, scale)
    r = subprocess.run(cmd, capture_output=True, text=True)
    sys.stderr.write(r.stderr)
    if r.returncode != 0:
        raise SystemExit(f"secondary leg {spec} failed (exit {r.returncode})")
    d = json.loads(r.stdout.strip().splitlines()[-1])
    c = d["config"]
    leg = {"dtype": dtype, "workload": c["workload"], "value": d["value"], "ms_per_step": d["ms_per_step"],
           "network_mfma_frac": d["network_mfma_frac"], "live_tracks_per_stream": c["live_tracks_per_stream"],
           "live_tracks_per_stream_min_at_start": c["live_tracks_per_stream_min_at_start"],
           "overflow": c["tracker_overflow"], "tracks_created": c["tracks_created"], "conv_plan": c["conv_plan"],
           "process": "own", "gflop_per_frame": c["gflop_per_frame"], "hbm_resident_fps": d.get("hbm_resident_fps"),
           "frames_per_forward": c.get("frames_per_forward", 1)}
    for k in ("roofline", "detect_roofline", "nms_roofline", "tracker_roofline"):
        if d.get(k) is not None:
            leg[k] = d[k]
    return leg


def main():
    a = parse()
    if a.gmd and a.tracker != "motion_reset":
        raise SystemExit("--gmd needs --tracker motion_reset")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus))
    ws, rank, local = dist_setup()
    if ws != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ws}: launch one process per GPU")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    P = importlib.import_module(PKG)
    cfg = dict(CONFIGS[a.config])
    if a.streams is not None:
        cfg["S"] = a.streams
    if a.targets is not None:
        cfg["targets"] = a.targets
    if a.frame:
        cfg["W"], cfg["H"] = (int(v) for v in a.frame.lower().split("x"))
    if a.imgsz:
        cfg["imgsz"] = a.imgsz
    dtype = a.dtype or cfg["dtype"]
    sec = cfg["secondary"] if a.secondary is None else ("" if a.secondary == "none" else a.secondary)
    secondary = [d for d in sec.split(",") if d and d != dtype and d != f"{a.scale}:{dtype}"] if ws == 1 else []
    S, H, W = cfg["S"], cfg["H"], cfg["W"]
    shard = P.shard
    my_streams = shard.stream_ids(rank, ws, S)  # this GPU's block of independent streams
    # pre-render every stream's frames into HBM (inputs resident before anything is timed)
    F = min(a.max_frames, a.preroll + a.warmup + a.steps)
    frames = torch.empty((F, S, H, W, 3), dtype=torch.uint8, device=dev)
    for s, g in enumerate(my_streams):
        sc = P.synth.Scene(seed=shard.stream_seed(g, S), n_targets=cfg["targets"], n_frames=F + 1, width=W, height=H)
        frames[:, s] = sc.frames_torch(0, F, dev)
    torch.cuda.synchronize()
    log(f"{F} frames x {S} streams resident; headline leg {dtype}, secondary {secondary or 'none'}")
    head = run_leg(a, P, cfg, dtype, frames, dev, local, rank, ws, headline=True)
    del frames
    # each secondary leg runs in a fresh process: a second StreamPipeline in the same process
    # measured 10-25 % slower on either dtype (bf16 12,313 as the first leg vs 9,742 as the
    # second; fp32 4,877 vs 4,323) -- its new HIP streams land on different hardware queues
    # (tools/second_pipe.py: the second pipeline is as fast as the first on the first one's streams)
    legs = [run_leg_subprocess(d) for d in secondary]
    cpu = None
    cpu_s = cpu_baseline_seconds(a, rank, ws)
    if cpu_s:
        ncpu = os.cpu_count() or 2
        ref_threads = max(1, min(8, ncpu - 1))  # the reference's select_device for CPU
        cpu = cpu_baseline(P, a.scale, S, cfg["targets"], (H, W), cfg["imgsz"], a.tracker, ref_threads, cpu_s)
        n_all = _cpu_quota()
        if ws == 1 and n_all != ref_threads and a.cpu_all_seconds > 0:
            allc = cpu_baseline(P, a.scale, S, cfg["targets"], (H, W), cfg["imgsz"], a.tracker, n_all,
                                a.cpu_all_seconds)
            cpu["all_cores"] = {k: allc[k] for k in ("value", "cores", "median_ms_per_frame", "p90_ms_per_frame",
                                                     "split_ms_per_frame", "sample")}
        cpu["host_cpus"] = {"os.cpu_count": ncpu, "usable": n_all}
    if rank == 0:
        ok_floor = head["live_tracks_per_stream_min_at_start"] >= cfg["live_floor"]
        out = {
            "metric": METRIC, "value": head["value"], "unit": "frames/s", "n_gpus": ws, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype,
            "data": f"synthetic: seeded {W}x{H} IR-like scenes ({cfg['targets']} targets/stream, occlusion bursts) "
                    "rendered into HBM before timing; seeded planted weights (no trained best.pt in the reference)",
            "config": {"workload": f"YOLOv8{a.scale}+P2 {W}x{H} (imgsz {cfg['imgsz']}), {S} stream(s)/GPU as batch {S}"
                                   + (f" ({head['frames_per_forward']} consecutive steps per forward: batch "
                                      f"{head['frames_per_forward'] * S})" if head["frames_per_forward"] > 1 else "")
                                   + f", {a.tracker} tracker(150, 1, 0.1), BASELINE config {a.config}",
                       "frames_per_forward": head["frames_per_forward"],
                       "baseline_config": a.config, "streams_per_gpu": S, "global_batch": S * ws,
                       "parallelism": f"streams sharded over {ws} GPU(s), no data-path collective",
                       "targets_per_stream": cfg["targets"], "tracker_preroll_frames": a.preroll,
                       "live_tracks_per_stream": head["live_tracks_per_stream"],
                       "live_tracks_per_stream_min_at_start": head["live_tracks_per_stream_min_at_start"],
                       "live_tracks_floor": cfg["live_floor"], "live_tracks_floor_met": ok_floor,
                       "tracker_overflow": head["overflow"], "tracks_created": head["tracks_created"],
                       "conv_plan": head["conv_plan"], "conv_plan_parity": head["conv_plan_parity"],
                       "graph": not a.no_graph, "tracker_overlapped": not a.no_pipeline,
                       "detector_inflight": a.inflight, "gflop_per_frame": head["gflop_per_frame"],
                       "rank_devices": head["rank_devices"],
                       "global_motion": "optical_flow" if a.gmd else None},
            "network_mfma_frac": head["network_mfma_frac"],
            "hbm_resident_fps": head["hbm_resident_fps"], "host_enqueue_ms_per_step": head["host_enqueue_ms_per_step"],
            "timed_region": "frames in page-locked host memory -> H2D on the slot stream -> forward -> NMS -> tracker "
                            "-> tracker output (counts, stats, rows) D2H, every step; hbm_resident_fps: the same steps "
                            "with the frames already in HBM and no output copy (informational)",
            "roofline": head.get("roofline"), "detect_roofline": head.get("detect_roofline"),
            "nms_roofline": head.get("nms_roofline"), "tracker_roofline": head.get("tracker_roofline"),
            "cpu_baseline": cpu,
            "secondary": [{k: v for k, v in leg.items() if k != "window_monotonic_ns"} for leg in legs],
            "timed_window_monotonic_ns": head["window_monotonic_ns"],
        }
        if "fw_times" in head:
            out["fw_times"] = head["fw_times"]
        print(json.dumps(out), flush=True)
    bad = head["overflow"] or any(leg["overflow"] for leg in legs)
    if ws > 1:
        import torch.distributed as dist

        barrier(ws)  # rank 0's CPU baseline ran after the timed region
        dist.destroy_process_group()
    if bad:
        log("FAIL: the tracker dropped detections/tracks (stats.overflow != 0); results would diverge from the reference")
        sys.exit(3)


if __name__ == "__main__":
    main()
