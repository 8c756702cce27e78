#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace of `bench.py` to the bench's own windows and summarise it.

usage: rocprof_window.py <run_kernel_trace.csv> <bench.json> [--steps K]

bench.py reports CLOCK_MONOTONIC nanoseconds around its timed region
(`timed_window_monotonic_ns`) and around the headline leg's per-op profile pass
(`roofline.window_monotonic_ns`).  rocprofv3 stamps kernels in nanoseconds of the same
host clock domain; the tool checks that by counting the records inside each window (a clock
mismatch leaves the windows empty and is reported as such).

Output (json):
  timed    per-kernel calls / avg / total us of the `yk::` kernels that STARTED inside the timed
           window, calls and device time per step, the union of busy time, and the window length
  profile  the same for the per-op profile pass (one forward at a time, 5 back-to-back launches
           of each op): its average duration of the bench's dominant kernel is the number the
           bench's `roofline.avg_launch_us` (hipEvents) must agree with
  check    dominant-kernel avg (profile window) vs roofline.avg_launch_us, and
           avg x launches/step (timed window) vs ms_per_step
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("yk::det::", "").replace("yk::trk::", "")
    return n.strip()


def summarise(rows, t0, t1, steps=None):
    sel = [r for r in rows if t0 <= r[0] < t1]
    by = defaultdict(lambda: [0, 0.0])
    for s, e, n in sel:
        by[n][0] += 1
        by[n][1] += (e - s) / 1e3
    iv = sorted((s, e) for s, e, _ in sel)
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
    out = {"records": len(sel), "window_us": round((t1 - t0) / 1e3, 1), "busy_union_us": round(busy / 1e3, 1),
           "kernels": {k: {"calls": c, "avg_us": round(t / c, 3), "total_us": round(t, 1)}
                       for k, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1])}}
    if steps:
        out["steps"] = steps
        for k, v in out["kernels"].items():
            v["calls_per_step"] = round(v["calls"] / steps, 2)
            v["us_per_step"] = round(v["total_us"] / steps, 2)
    return out


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    with open(bench) as f:
        b = json.loads(f.read().strip().splitlines()[-1])
    rows = []
    with open(trace) as f:
        for x in csv.DictReader(f):
            if "yk::" in x["Kernel_Name"]:
                rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), short(x["Kernel_Name"])))
    rows.sort()
    tw = b["timed_window_monotonic_ns"]
    pw = (b.get("roofline") or {}).get("window_monotonic_ns")
    res = {"bench": {k: b[k] for k in ("value", "ms_per_step", "dtype", "steps")},
           "trace_span_ns": [rows[0][0], rows[-1][1]] if rows else None,
           "timed": summarise(rows, tw[0], tw[1], b["steps"])}
    if pw:
        res["profile"] = summarise(rows, pw[0], pw[1])
    rl = b.get("roofline") or {}
    dom = short(rl.get("kernel", ""))
    chk = {"dominant_kernel": dom, "bench_avg_launch_us": rl.get("avg_launch_us"), "bench_frac": rl.get("frac")}
    if pw and dom in res["profile"]["kernels"]:
        p = res["profile"]["kernels"][dom]
        chk["rocprof_profile_window_avg_us"] = p["avg_us"]
        if rl.get("avg_launch_us"):
            chk["avg_ratio_rocprof_over_bench"] = round(p["avg_us"] / rl["avg_launch_us"], 4)
        if rl.get("flops_per_launch") and rl.get("peak"):
            chk["frac_from_rocprof"] = round(rl["flops_per_launch"] / (p["avg_us"] * 1e-6) / 1e12 / rl["peak"], 5)
    if dom in res["timed"]["kernels"]:
        t = res["timed"]["kernels"][dom]
        chk["timed_window_avg_us"] = t["avg_us"]
        chk["timed_avg_x_launches_per_step_us"] = round(t["avg_us"] * t["calls_per_step"], 1)
        chk["ms_per_step_us"] = round(b["ms_per_step"] * 1e3, 1)
    res["check"] = chk
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
