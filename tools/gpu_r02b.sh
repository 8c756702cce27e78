#!/bin/bash
# Round-2 step B: new parity tests (exact bench pipeline vs oracle chain, config-5 tracker leg,
# golden fixtures) and the bench line with the committed conv plans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_bench_pipeline_gpu.py tests/test_golden_gpu.py tests/test_tracker_gpu.py -x -v -s --timeout 900 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|assert" $O/tests.log | head -40; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|BENCH_PIPELINE|CONFIG5" $O/tests.log
timeout -k 10 400 python -u bench.py --dump-ops $O/ops.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
