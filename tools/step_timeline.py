"""Timeline of one detector graph replay from a rocprofv3 kernel trace: span, busy union,
gaps between consecutive kernels.  usage: step_timeline.py <kernel_trace.csv> [k-th step from end]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for x in csv.DictReader(f):
        if "yk::" in x["Kernel_Name"]:
            nm = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("yk::det::", "")
            rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), nm))
rows.sort()
nms = [i for i, r in enumerate(rows) if "nms_kernel" in r[2]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
seg = rows[nms[-k - 1] + 1:nms[-k] + 1]
t0 = seg[0][0]
t1 = max(r[1] for r in seg)
iv = sorted((r[0], r[1]) for r in seg if "step_kernel" not in r[2])
u = 0
cs, ce = iv[0]
gaps = []
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        gaps.append(s - ce)
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"kernels {len(seg)} span {(t1 - t0) / 1e3:.1f} us, busy union {u / 1e3:.1f} us, "
      f"sum {sum(r[1] - r[0] for r in seg) / 1e3:.1f} us, gaps {len(gaps)} total {sum(gaps) / 1e3:.1f} us, "
      f"max gap {max(gaps + [0]) / 1e3:.1f} us")
if "-v" in sys.argv:
    for r in seg:
        print(f"{(r[0] - t0) / 1e3:8.2f} {(r[1] - r[0]) / 1e3:7.2f} {r[2][:70]}")
