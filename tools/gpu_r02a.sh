#!/bin/bash
# Round-2 step A: autotune + save the conv plans of config 3 (fp32 headline, bf16 secondary),
# the new bench line, then the new parity tests (exact bench pipeline vs oracle chain, config-5
# tracker leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02a
mkdir -p $O plans
timeout -k 10 400 python -u bench.py --autotune --save-plans --no-cpu-baseline --dump-ops $O/ops.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cp plans/*.json $O/ 2>/dev/null
timeout -k 10 1200 python -u -m pytest tests/test_bench_pipeline_gpu.py tests/test_tracker_gpu.py -x -v -s --timeout 900 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed|BENCH_PIPELINE|CONFIG5" $O/tests.log
