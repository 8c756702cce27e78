#!/bin/bash
# GPU round check: parity tests, one bench line, a rocprofv3 kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --dump-ops gpurun_out/ops.json > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --steps 50 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "rocprof failed"; tail -30 gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof -name '*stats*'
