"""Host-frame loop vs HBM-resident loop from ONE rocprofv3 trace of bench.py (kernel + memory-copy
trace): bench runs preroll + warmup steps, then the timed host loop, then the HBM-resident loop of
the same length, so forwards [pre, pre + steps) and [pre + steps, pre + 2 steps) (in nms_kernel
order) are the two windows.  Per window: span, GPU busy union, mean kernel concurrency, forward
latency (first kernel -> nms_kernel on its queue), the forward-to-forward interval per queue, and the
copies that fall inside it.
usage: io_timeline.py <dir with *_kernel_trace.csv, *_memory_copy_trace.csv> <pre> <steps>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(pattern):
    f = glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True)
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


ker = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"], x.get("Queue_Id", ""))
       for x in load("*kernel_trace.csv")]
ker.sort()
cp = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x.get("Direction", ""), int(x.get("Size", 0) or 0))
      for x in load("*memory_copy_trace.csv")]
cp.sort()
nms = [r for r in ker if "nms_kernel" in r[2]]
steps = int(sys.argv[3])
pre = len(nms) - 2 * steps if sys.argv[2] == "auto" else int(sys.argv[2])  # (the two loops end the trace)


def window(name, a, b):
    t0 = nms[a - 1][1]
    t1 = nms[b - 1][1]
    seg = [r for r in ker if t0 <= r[0] < t1]
    iv = sorted((r[0], min(r[1], t1)) for r in seg)
    u, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            u += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    u += ce - cs
    tot = sum(e - s for s, e in iv)
    span = t1 - t0
    # per queue: forward latency and the interval between consecutive forwards' ends
    byq = defaultdict(list)
    for r in seg:
        byq[r[3]].append(r)
    lat, ends = [], defaultdict(list)
    for q, rs in byq.items():
        start = None
        for r in rs:
            if "nms_kernel" in r[2]:
                if start is not None:
                    lat.append(r[1] - start)
                ends[q].append(r[1])
                start = None
            elif start is None and "yk::det" in r[2]:
                start = r[0]
    gaps = [b2 - a2 for q in ends for a2, b2 in zip(ends[q], ends[q][1:])]
    cps = [c for c in cp if t0 <= c[0] < t1]
    print(f"{name}: {b - a} forwards, span {span / 1e3:.1f} us = {span / 1e3 / (b - a):.1f} us/forward, "
          f"busy {u / span:.3f}, concurrency {tot / span:.2f} (busy-time {tot / max(u, 1):.2f})")
    print(f"   queues {sorted((q, len(rs)) for q, rs in byq.items())}")
    if lat:
        lat.sort()
        print(f"   forward latency us: mean {sum(lat) / len(lat) / 1e3:.1f}  p50 {lat[len(lat) // 2] / 1e3:.1f}"
              f"  p90 {lat[int(len(lat) * .9)] / 1e3:.1f}")
    if gaps:
        gaps.sort()
        print(f"   same-queue forward interval us: mean {sum(gaps) / len(gaps) / 1e3:.1f}  p50 {gaps[len(gaps) // 2] / 1e3:.1f}")
    if cps:
        dirs = defaultdict(list)
        for c in cps:
            dirs[c[2]].append(c)
        for d, cs2 in dirs.items():
            du = sorted(c[1] - c[0] for c in cs2)
            print(f"   copies {d}: {len(cs2)}, {sum(c[3] for c in cs2) / len(cs2) / 1e6:.2f} MB mean, "
                  f"duration mean {sum(du) / len(du) / 1e3:.1f} us p90 {du[int(len(du) * .9)] / 1e3:.1f}")


window("host-frame loop", pre + 1, pre + steps)
window("HBM-resident loop", pre + steps + 1, pre + 2 * steps)
