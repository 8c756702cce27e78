#!/bin/bash
# FP8 build check: fp8 parity tests, the bf16/fp32 detector suite, config-5 bench (fp8 and bf16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fp8
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_detector_fp8_gpu.py tests/test_detector_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --steps 40 --dump-ops $O/ops5.json > $O/bench5.json 2> $O/bench5.err || { tail -20 $O/bench5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench5.json'));print('fp8 c5', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --config 5 --dtype bf16 --no-cpu-baseline --steps 40 > $O/bench5b.json 2> $O/bench5b.err || { tail -20 $O/bench5b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench5b.json'));print('bf16 c5', d['value'], d['ms_per_step'])"
