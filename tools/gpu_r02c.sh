#!/bin/bash
# SPPF (LDS, 4/8 channels per workgroup) + fp8 parity, config 5 re-measured, and per-workgroup
# timelines of fp32 conv ops under the committed plan (tools/wg_times.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02c
mkdir -p $O
true
true
for op in 3 10 72 73; do
  YK_FAST_TS=$op YK_DTYPE=fp32 YK_PLAN=plans/s_640x512_i640_b8_fp32.json timeout -k 10 200 python -u tools/wg_times.py > $O/wg_$op.txt 2>&1; rc=$?; [ $rc -le 1 ] || { echo "wg $op rc $rc"; tail -20 $O/wg_$op.txt; exit 1; }
  cat $O/wg_$op.txt
done
timeout -k 10 400 python -u bench.py --config 5 --no-cpu-baseline --dump-ops $O/ops_c5.json > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -20 $O/bench_c5.err; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --inflight 1 --no-cpu-baseline > $O/bench_c5_if1.json 2> $O/bench_c5_if1.err || { echo "c5 if1 failed"; tail -20 $O/bench_c5_if1.err; exit 1; }
python3 - <<'PY'
import json
for n in ("c5", "c5_if1"):
    d = json.load(open(f"gpurun_out/r02c/bench_{n}.json"))
    print(n, d["value"], d["dtype"], d["ms_per_step"], d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"],
          [(s["dtype"], s["value"], s["network_mfma_frac"]) for s in d["secondary"]])
PY
