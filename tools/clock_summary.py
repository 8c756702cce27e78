#!/usr/bin/env python3
"""Effective clock per yk kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace run:
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so clock = value / 8 / duration (MI355X_MICROARCH.md,
'DVFS give-back').  usage: clock_summary.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
rows = [r for p in cc for r in csv.DictReader(open(p))]
agg = collections.defaultdict(list)
for r in rows:
    if "yk::" not in r["Kernel_Name"] or r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    n = re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["Kernel_Name"])).replace("yk::det::", "")
    dur = None
    if r.get("End_Timestamp") and r.get("Start_Timestamp"):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg[n].append((float(r["Counter_Value"]), dur))
print("kernel  n  mean_us  clock_GHz(GRBM_GUI_ACTIVE/8/dur)")
for n, v in sorted(agg.items(), key=lambda kv: -sum((x[1] or 0) for x in kv[1])):
    v = [x for x in v if x[1]]
    if not v:
        continue
    us = sum(x[1] for x in v) / len(v) * 1e6
    clk = sum(x[0] / 8 / x[1] for x in v) / len(v) / 1e9
    print(f"{n[:60]:60s} {len(v):4d} {us:8.1f} {clk:6.3f}")
