#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fastw
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_detector_gpu.py -x -q -k "fastw or variants" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/tune_concurrent.py --dtype fp32 --tune-batch 16 --out $O/plan_c16.json > $O/tune16.log 2>&1 || { tail -20 $O/tune16.log; exit 1; }
timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --autotune --plan-out $O/plan_iso.json --dump-ops $O/ops_iso.json > $O/bench_iso.json 2> $O/bench_iso.err || { tail -20 $O/bench_iso.err; exit 1; }
timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline --plan-in $O/plan_c16.json --dump-ops $O/ops_c16.json > $O/bench_c16.json 2> $O/bench_c16.err || { tail -20 $O/bench_c16.err; exit 1; }
timeout -k 10 200 python -u bench.py --secondary none --no-cpu-baseline --plan-in plans/s_640x512_i640_b8_fp32.json > $O/bench_old.json 2> $O/bench_old.err || { tail -20 $O/bench_old.err; exit 1; }
python3 - <<'PY'
import json
for n in ("old", "iso", "c16"):
    d = json.load(open(f"gpurun_out/fastw/bench_{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
for n in ("iso", "c16"):
    o = json.load(open(f"gpurun_out/fastw/ops_{n}.json"))
    print(n, "op sum", round(sum(x["us"] for x in o["ops"]), 1), "fastw ops", sum("fastw" in x["kernel"] for x in o["ops"]))
PY
