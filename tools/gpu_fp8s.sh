#!/bin/bash
# Block-scaled fp8 MFMA: parity tests, then config 5 (fp8 vs bf16) with three and one forwards
# in flight, plans re-tuned.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fp8s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_detector_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --config 5 --autotune --save-plans --no-cpu-baseline --dump-ops $O/ops_c5.json > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -20 $O/bench_c5.err; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --inflight 1 --no-cpu-baseline > $O/bench_c5_if1.json 2> $O/bench_c5_if1.err || { echo "c5 if1 failed"; tail -20 $O/bench_c5_if1.err; exit 1; }
cp plans/s_1280x1024_i1280_b8_*.json $O/
python3 - <<'PY'
import json
for n in ("c5", "c5_if1"):
    d = json.load(open(f"gpurun_out/fp8s/bench_{n}.json"))
    print(n, d["value"], d["dtype"], d["ms_per_step"], d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"],
          [(s["dtype"], s["value"], s["network_mfma_frac"]) for s in d["secondary"]])
PY
