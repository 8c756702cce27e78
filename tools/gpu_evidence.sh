#!/bin/bash
# Round-end evidence for profiles/: default bench (config 3: fp32 headline + bf16 secondary,
# CPU baseline), rocprofv3 kernel trace (+ --stats) of the same workload cut to the bench's
# windows, HBM PMC passes (fp32 and bf16 builds), config 2 / 4 / 5 lines -- all on the committed
# conv plans (no autotune).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${EVIDENCE_DIR:-final}
mkdir -p $O
timeout -k 10 400 python -u bench.py --dump-ops $O/ops_c3.json > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -20 $O/bench_c3.err; exit 1; }
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u bench.py --steps 50 --secondary none --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -20 $O/trace_bench.err; exit 1; }
python3 tools/rocprof_window.py $O/trace/run_kernel_trace.csv $O/trace_bench.json > $O/trace_window.json || exit 1
rm -f $O/trace/run_kernel_trace.csv
echo "trace ok"
for DTY in fp32 bf16; do
  B="bench.py --dtype $DTY --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline --no-profile"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$DTY -o run -- python3 -u $B > /dev/null 2> $O/pmc_fetch_$DTY.err || { echo "pmc fetch failed"; tail -5 $O/pmc_fetch_$DTY.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$DTY -o run -- python3 -u $B > /dev/null 2> $O/pmc_write_$DTY.err || { echo "pmc write failed"; tail -5 $O/pmc_write_$DTY.err; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_fetch_$DTY/run_counter_collection.csv $O/pmc_write_$DTY/run_counter_collection.csv $O/pmc_traffic_$DTY.json
  rm -f $O/pmc_fetch_$DTY/run_counter_collection.csv $O/pmc_write_$DTY/run_counter_collection.csv
done
echo "pmc ok"
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo "c4 failed"; tail -20 $O/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo "c2 failed"; tail -20 $O/bench_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --no-cpu-baseline --dump-ops $O/ops_c5.json > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -20 $O/bench_c5.err; exit 1; }
python3 - <<'PY'
import json, os
for n in ("c3", "c4", "c2", "c5"):
    d = json.load(open(f"gpurun_out/{os.environ.get('EVIDENCE_DIR', 'final')}/bench_{n}.json"))
    print(n, d["value"], d["dtype"], d["ms_per_step"], d["config"]["live_tracks_per_stream"], d["config"]["live_tracks_per_stream_min_at_start"],
          d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["traffic"], [(s["dtype"], s["value"]) for s in d["secondary"]])
PY
