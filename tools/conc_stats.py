"""Concurrency summary of a rocprofv3 kernel trace (csv): over the last `frac` of the run, the
time-weighted number of yk kernels in flight, the idle fraction, and per-kernel-name mean
durations in situ.  usage: conc_stats.py run_kernel_trace.csv [frac]"""
import csv
import sys
from collections import defaultdict

rows = []
for x in csv.DictReader(open(sys.argv[1])):
    n = x["Kernel_Name"]
    if "yk::" in n or "nms_kernel" in n:
        rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), n.split("(")[0].replace("void ", "")))
rows.sort()
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3  # > 1: the last `frac` kernels
t_end = rows[-1][1]
t_beg = rows[int(len(rows) * (1 - frac)) if frac <= 1 else len(rows) - int(frac)][0]
seg = [r for r in rows if r[0] >= t_beg]
ev = []
for s, e, _ in seg:
    ev.append((s, 1))
    ev.append((e, -1))
ev.sort()
busy = idle = weighted = 0
cur = 0
last = ev[0][0]
hist = defaultdict(int)
for t, d in ev:
    dt = t - last
    if cur == 0:
        idle += dt
    else:
        busy += dt
        weighted += dt * cur
    hist[cur] += dt
    cur += d
    last = t
span = ev[-1][0] - ev[0][0]
print(f"kernels {len(seg)} span {span/1e3:.1f} us  idle {idle/span:.3f}  mean in flight (busy) {weighted/max(busy,1):.2f}")
print("time share by #in flight:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
dur = defaultdict(list)
for s, e, n in seg:
    dur[n].append(e - s)
tot = sum(sum(v) for v in dur.values())
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:12]:
    print(f"{sum(v)/tot:6.3f} {len(v):6d} {sum(v)/len(v)/1e3:8.2f} us  {n[:70]}")
