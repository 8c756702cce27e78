#!/bin/bash
# fast SiLU in the fp32 epilogues: parity (fp32 layers, exact bench pipeline, golden) + headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/silu
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_detector_gpu.py tests/test_bench_pipeline_gpu.py tests/test_golden_gpu.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --secondary none --no-cpu-baseline --dump-ops $O/ops_fp32.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['network_mfma_frac'], d['roofline']['kernel'], d['roofline']['frac'])"
