#!/bin/bash
# PMC passes + kernel trace over the fp32 headline with a given conv plan: MFMA busy, LDS wait /
# bank conflicts and the effective clock (GRBM_GUI_ACTIVE / 8 / wall) per kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${PMC_DIR:-pmchalo}
mkdir -p $O
P=${PLAN:-plans/exp/s_640x512_i640_b8_fp32_r3i.json}
B="bench.py --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline --no-profile --plan-in $P"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u $B > /dev/null 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p1 -o run -- python3 -u $B > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $O/p2 -o run -- python3 -u $B > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
python3 tools/pmc_kernels.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv > $O/summary.txt
cp $O/kt/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || true
python3 - "$O" <<'PY'
import csv, sys, collections
O = sys.argv[1]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f"{O}/kt/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if "conv_" in n:
        dur[n.split("(")[0].replace("void ", "").replace("yk::det::", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
grb = collections.defaultdict(list)
for r in csv.DictReader(open(f"{O}/p2/run_counter_collection.csv")):
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "conv_" in r["Kernel_Name"]:
        grb[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("yk::det::", "")].append(float(r["Counter_Value"]))
for n in sorted(dur, key=lambda k: -sum(dur[k])):
    us = sum(dur[n]) / len(dur[n])
    g = sum(grb.get(n, [0])) / max(1, len(grb.get(n, [0])))
    print(f"{n[:60]:60s} n={len(dur[n]):4d} avg_us={us:8.2f} clock_GHz={g / 8 / (us * 1e3) if us else 0:.2f}")
PY
rm -rf $O/p1 $O/p2 $O/kt
head -12 $O/summary.txt
