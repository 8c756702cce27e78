#!/bin/bash
# rocprofv3 kernel trace of the bench command with the committed conv plans (no autotune), then
# the trace cut to the bench's timed window and per-op profile window (tools/rocprof_window.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/trace
mkdir -p $O
ARGS="${BENCH_ARGS:---steps 50 --secondary none --no-cpu-baseline}"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o run -- python3 -u bench.py $ARGS > $O/bench.json 2> $O/bench.err || { echo "trace failed"; tail -30 $O/bench.err; exit 1; }
python3 tools/rocprof_window.py $O/raw/run_kernel_trace.csv $O/bench.json > $O/window.json || { echo "window failed"; exit 1; }
rm -f $O/raw/run_kernel_trace.csv
cat $O/window.json | head -80
