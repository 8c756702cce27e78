#!/bin/bash
# conv_fast load-pipeline depth: fp32 headline bench + isolated per-op times (committed plan)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/skd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_detector_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py --secondary none --no-cpu-baseline --dump-ops $O/ops_fp32.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/skd/bench.json"))
print(d["value"], d["ms_per_step"], d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
PY
