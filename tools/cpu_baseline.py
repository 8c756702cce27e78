#!/usr/bin/env python3
"""BASELINE.md's CPU-baseline protocol, every config row, on this host's cores.

The reference-equivalent CPU path is the oracle (oracle/detector_ref.py torch-CPU fp32 +
oracle/tracker_ref.py numpy, Python IoU loop as in the reference): the reference's own Python
cannot be run.  Per row: 10 warm-up frames, then 300 timed frames (time.perf_counter
around each whole step: detector / NMS / tracker split), median and p90 ms/frame, frames/s; with
torch.set_num_threads(min(8, os.cpu_count() - 1)) as the reference's select_device does
(ultralytics/utils/torch_utils.py:241-242) and with all usable cores.

Rows (BASELINE.json configs):
  1  640x512, 1 stream, 4 targets            (CPU plumbing; scale s, and scale n)
  2  640x512, 1 stream, B=1, 12 targets
  3  640x512, 8 streams: one batch-8 forward + 8 trackers per step, 40 targets/stream
  4  640x512, 1 stream (the per-GPU unit of config 4; x8 streams is not parallelised on CPU)
  5  1280x1024 at imgsz 1280, 8 streams, 96 targets/stream

Usage: python tools/cpu_baseline.py [--rows 1,2,3,4,5] [--frames 300] [--out file.json]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import platform
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

ROWS = {
    1: dict(scale="s", S=1, targets=4, hw=(512, 640), imgsz=640),
    "1n": dict(scale="n", S=1, targets=4, hw=(512, 640), imgsz=640),
    2: dict(scale="s", S=1, targets=12, hw=(512, 640), imgsz=640),
    3: dict(scale="s", S=8, targets=40, hw=(512, 640), imgsz=640),
    4: dict(scale="s", S=1, targets=40, hw=(512, 640), imgsz=640),
    5: dict(scale="s", S=8, targets=96, hw=(1024, 1280), imgsz=1280),
}


def host_info():
    info = {"os.cpu_count": os.cpu_count(), "usable_cpus": bench._cpu_quota(), "platform": platform.platform()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)")
        info["lscpu"] = {k.strip(): v.strip() for k, v in (l.split(":", 1) for l in out.splitlines() if ":" in l)
                         if k.strip() in keep}
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,1n,2,3,4,5")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--seconds", type=float, default=1e9, help="optional bound per row")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    P = importlib.import_module(bench.PKG)
    ncpu = os.cpu_count() or 2
    ref_threads = max(1, min(8, ncpu - 1))
    all_threads = bench._cpu_quota()
    out = {"protocol": "10 warm-up frames + up to {} timed frames per row; perf_counter per whole step".format(a.frames),
           "host": host_info(), "rows": {}}
    for key in a.rows.split(","):
        r = ROWS[int(key) if key.isdigit() else key]
        res = {}
        for label, th in (("reference_threads", ref_threads), ("all_cores", all_threads)):
            if label == "all_cores" and th == ref_threads:
                continue
            t0 = time.time()
            res[label] = bench.cpu_baseline(P, r["scale"], r["S"], r["targets"], r["hw"], r["imgsz"], "enhanced", th,
                                            a.seconds, warm_frames=10, max_frames=a.frames)
            print(f"[cpu_baseline] row {key} {label} ({th} threads): {res[label]['value']} frames/s, "
                  f"median {res[label]['median_ms_per_frame']} ms, {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
        out["rows"][key] = {"workload": r, **res}
    js = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)


if __name__ == "__main__":
    main()
