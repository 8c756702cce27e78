#!/usr/bin/env python3
"""Where the driver-length timed window goes: fill, steady state and drain of the in-flight
pipeline, from one rocprofv3 trace (kernel + memory-copy) of `bench.py`.

usage: fill_profile.py <trace dir> <bench.json> [--bin-us 250]

The timed window is bench.py's `timed_window_monotonic_ns` (the same host clock as rocprofv3's
stamps, checked by rocprof_window.py).  Output (json):
  first_kernel_us / last_kernel_end_us   offsets of the first yk:: kernel and of the last kernel
                                         end inside the window (host enqueue + upload latency at
                                         the start, the drain's host tail at the end)
  forwards     per forward (conv_input_f32mfma_kernel .. nms_kernel on one queue): start, end and
               latency, relative to the window start
  bins         per --bin-us slice of the window: busy fraction (union of kernel intervals) and mean
               kernel concurrency (summed kernel time / slice), H2D / D2H bytes that started in it
  phases       the same two figures over the fill (window start .. the third forward's start), the
               steady part and the drain (the last forward's start .. window end)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def union(iv, t0, t1):
    iv = sorted((max(s, t0), min(e, t1)) for s, e in iv if e > t0 and s < t1)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None:
            cs, ce = s, e
        elif s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    return busy


def slice_stats(ker, t0, t1):
    iv = [(s, e) for s, e, _, _ in ker]
    tot = sum(max(0, min(e, t1) - max(s, t0)) for s, e in iv)
    return {"us": round((t1 - t0) / 1e3, 1), "busy": round(union(iv, t0, t1) / max(1, t1 - t0), 3),
            "concurrency": round(tot / max(1, t1 - t0), 3)}


def main():
    d, bench = sys.argv[1], sys.argv[2]
    bin_us = float(sys.argv[sys.argv.index("--bin-us") + 1]) if "--bin-us" in sys.argv else 250.0
    with open(bench) as f:
        b = json.loads(f.read().strip().splitlines()[-1])
    t0, t1 = b["timed_window_monotonic_ns"]
    ker = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"].split("(")[0].replace("void ", ""),
                  x.get("Queue_Id", "")) for x in load(d, "*kernel_trace.csv") if "yk::" in x["Kernel_Name"])
    cp = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x.get("Direction", ""), int(x.get("Size", 0) or 0))
                for x in load(d, "*memory_copy_trace.csv"))
    win = [k for k in ker if t0 <= k[0] < t1]
    if not win:
        print(json.dumps({"error": "no kernels inside the timed window (clock domains?)"}))
        return
    # forwards: a conv_input kernel opens one on its queue, that queue's next nms_kernel closes it
    fw, open_ = [], {}
    for s, e, n, q in win:
        if "conv_input" in n:
            open_[q] = s
        elif "nms_kernel" in n and q in open_:
            st = open_.pop(q)
            fw.append({"start_us": round((st - t0) / 1e3, 1), "end_us": round((e - t0) / 1e3, 1),
                       "latency_us": round((e - st) / 1e3, 1), "queue": q})
    fw.sort(key=lambda r: r["start_us"])
    bins = []
    step = int(bin_us * 1e3)
    for a in range(t0, t1, step):
        z = min(a + step, t1)
        r = slice_stats(win, a, z)
        r["at_us"] = round((a - t0) / 1e3, 1)
        r["h2d_mb"] = round(sum(c[3] for c in cp if a <= c[0] < z and "HOST_TO_DEVICE" in c[2].upper()) / 1e6, 2)
        r["d2h_mb"] = round(sum(c[3] for c in cp if a <= c[0] < z and "DEVICE_TO_HOST" in c[2].upper()) / 1e6, 2)
        bins.append(r)
    phases = {}
    if len(fw) >= 4:
        f3 = t0 + int(fw[2]["start_us"] * 1e3)
        fl = t0 + int(fw[-1]["start_us"] * 1e3)
        phases = {"fill": slice_stats(win, t0, f3), "steady": slice_stats(win, f3, fl), "drain": slice_stats(win, fl, t1)}
    out = {"bench": {k: b.get(k) for k in ("value", "ms_per_step", "steps", "dtype")},
           "window_us": round((t1 - t0) / 1e3, 1),
           "first_kernel_us": round((win[0][0] - t0) / 1e3, 1),
           "last_kernel_end_us": round((max(k[1] for k in win) - t0) / 1e3, 1),
           "whole": slice_stats(win, t0, t1), "phases": phases, "forwards": fw, "bins": bins}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
