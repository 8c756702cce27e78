#!/bin/bash
# Bench + rocprofv3 evidence for profiles/: kernel-trace stats of the bench command (same conv
# plan as the bench, no autotune launches in the trace) and HBM traffic PMC passes (one block of
# counters per pass, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Large raw CSVs are reduced to
# summaries on the box (gpurun copies back at most 64 MiB).
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
python3 tools/step_timeline.py $O/trace/run_kernel_trace.csv 5 -v > $O/step_timeline.txt || true
rm -f $O/trace/run_kernel_trace.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u bench.py $ARGS --plan-in $O/plan.json --steps 5 --warmup 2 --no-cpu-baseline --no-profile > /dev/null 2> $O/pmc_fetch.err || { echo "pmc fetch failed"; tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u bench.py $ARGS --plan-in $O/plan.json --steps 5 --warmup 2 --no-cpu-baseline --no-profile > /dev/null 2> $O/pmc_write.err || { echo "pmc write failed"; tail -20 $O/pmc_write.err; exit 1; }
python3 tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/pmc_traffic.json
rm -f $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv
find $O -type f | xargs ls -la
