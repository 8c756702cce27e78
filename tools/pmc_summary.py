#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

Corrections (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Each counter comes from its own pass.

usage: pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        if "yk::" not in r["Kernel_Name"]:
            continue  # benchmark set-up kernels (torch frame rendering, copies)
        name = re.sub(r"^void ", "", r["Kernel_Name"])
        name = re.sub(r"\(.*$", "", name).replace("yk::det::", "").replace("yk::trk::", "")
        agg[name].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main(fetch_csv, write_csv, out):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = sum(f[k]) / len(f[k]) * 2.0 if f.get(k) else None
        wb = sum(w[k]) / len(w[k]) if w.get(k) else None
        res[k] = {"launches_fetch": len(f.get(k, [])), "launches_write": len(w.get(k, [])),
                  "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); FETCH x2 (gfx950)",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
