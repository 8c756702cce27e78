"""All kernels (any name) between the end of one detector step and the start of the next."""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for x in csv.DictReader(f):
        rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"][:80], x.get("Queue_Id", "")))
rows.sort()
nms = [i for i, r in enumerate(rows) if "nms_kernel" in r[2]]
i = nms[-6]
t0 = rows[i][0]
for r in rows[i:i + 12]:
    print(f"{(r[0] - t0) / 1e3:9.2f} {(r[1] - r[0]) / 1e3:8.2f} q{r[3]} {r[2]}")
