#!/bin/bash
# Bench + rocprofv3 evidence for profiles/: kernel-trace stats of the bench command (same conv
# plan as the bench, no autotune launches in the trace) and HBM traffic PMC passes (one block of
# counters per pass, MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
ARGS="${BENCH_ARGS:-}"
timeout -k 10 400 python -u bench.py $ARGS --plan-out $O/plan.json --dump-ops $O/ops.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u bench.py $ARGS --plan-in $O/plan.json --steps 50 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -30 $O/trace_bench.err; exit 1; }
cat $O/trace_bench.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u bench.py $ARGS --plan-in $O/plan.json --steps 5 --warmup 2 --no-cpu-baseline --no-profile > /dev/null 2> $O/pmc_fetch.err || { echo "pmc fetch failed"; tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u bench.py $ARGS --plan-in $O/plan.json --steps 5 --warmup 2 --no-cpu-baseline --no-profile > /dev/null 2> $O/pmc_write.err || { echo "pmc write failed"; tail -20 $O/pmc_write.err; exit 1; }
find $O -name '*.csv' | xargs ls -la
