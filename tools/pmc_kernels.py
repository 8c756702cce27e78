#!/usr/bin/env python3
"""Per-kernel average of every PMC counter in rocprofv3 counter_collection CSVs (yk kernels).
usage: pmc_kernels.py <csv> [<csv> ...]"""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        continue
    for r in rows:
        if "yk::" not in r["Kernel_Name"]:
            continue
        n = re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["Kernel_Name"])).replace("yk::det::", "").replace("yk::trk::", "")
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    d = {k: sum(v) / len(v) for k, v in cs.items()}
    line = f"{n[:58]:58s} n={len(next(iter(cs.values())))}"
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        line += "  wait %.2f inst_stall %.2f active %.2f" % (d.get("SQ_WAIT_ANY", 0) / wc, d.get("SQ_WAIT_INST_ANY", 0) / wc,
                                                            d.get("SQ_ACTIVE_INST_ANY", 0) / wc)
    if d.get("SQ_BUSY_CYCLES"):
        line += "  mfma_busy/busy %.2f" % (d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / d["SQ_BUSY_CYCLES"])
    line += "  " + " ".join(f"{k}={v:.4g}" for k, v in sorted(d.items()))
    print(line)
