#!/bin/bash
# GPU driver (one gpurun call runs a list of steps).  STEPS (space separated) picks what runs, in order:
#   pytest   the whole -m gpu suite
#   bench    the default bench line (committed plan) with --dump-ops
#   tune     concurrent autotune of the fp32 plan (all kernel kinds incl. split / halo) -> plan_tuned.json
#   btuned   bench on plan_tuned.json
#   trace    rocprofv3 kernel trace + stats of the default bench, cut to the timed window
#   pmc      FETCH_SIZE / WRITE_SIZE passes of the fp32 build
#   cmc      the camera-motion-compensation bench line (motion-reset tracker + global motion)
#   diag     tools/cmc_pipe_diag.py
#   wg       per-workgroup timelines of conv ops $WG_OPS (tools/wg_times.py, committed fp32 plan)
#   libab    fp32 bench on each library variant in $LIBS (YK_LIB)
#   c4plan   config-4 bench with its run-time autotuned plan written to plan_c4.json
#   c4tune   config-4 plan tuned over every kernel kind vs the committed one
#   smoke    __graft_entry__.smoke()
#   sweep    bench at detector in-flight depths $SWEEP (default 3 5 6)
#   ab       tools/split_ab.py: committed (split / halo) plan vs the round-2 exact-f32 plan, accuracy vs the oracle
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r4}
mkdir -p $O
PLAN=${PLAN:-}
BARGS=${BARGS:-}
for s in ${STEPS:-pytest bench}; do
  case $s in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --maxfail=3 --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
      tail -2 $O/pytest_gpu.log ;;
    bench)
      timeout -k 10 400 python -u bench.py ${PLAN:+--plan-in $PLAN} $BARGS --dump-ops $O/ops.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    tune)
      timeout -k 10 600 python -u tools/tune_concurrent.py --dtype fp32 --tune-batch ${TUNE_BATCH:-16} --out $O/plan_tuned.json > $O/tune.log 2>&1 || { echo "tune failed"; tail -20 $O/tune.log; exit 1; }
      tail -1 $O/tune.log ;;
    btuned)
      timeout -k 10 300 python -u bench.py --steps 100 --secondary none --no-cpu-baseline --plan-in $O/plan_tuned.json --dump-ops $O/ops_tuned.json > $O/bench_tuned.json 2> $O/bench_tuned.err || { echo "bench tuned failed"; tail -20 $O/bench_tuned.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_tuned.json')); print('tuned', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u bench.py ${PLAN:+--plan-in $PLAN} --steps 50 --secondary none --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -20 $O/trace_bench.err; exit 1; }
      python3 tools/rocprof_window.py $O/trace/run_kernel_trace.csv $O/trace_bench.json > $O/trace_window.json || exit 1
      rm -f $O/trace/run_kernel_trace.csv
      echo "trace ok" ;;
    pmc)
      B="bench.py ${PLAN:+--plan-in $PLAN} --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline --no-profile"
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u $B > /dev/null 2> $O/pmc_fetch.err || { echo "pmc fetch failed"; tail -5 $O/pmc_fetch.err; exit 1; }
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u $B > /dev/null 2> $O/pmc_write.err || { echo "pmc write failed"; tail -5 $O/pmc_write.err; exit 1; }
      python3 tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/pmc_traffic.json
      rm -f $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv
      echo "pmc ok" ;;
    cmc)
      timeout -k 10 300 python -u bench.py --tracker motion_reset --gmd --secondary none --no-cpu-baseline > $O/bench_cmc.json 2> $O/bench_cmc.err || { echo "bench cmc failed"; tail -20 $O/bench_cmc.err; exit 1; }
      cat $O/bench_cmc.json ;;
    diag)
      timeout -k 10 300 python -u tools/cmc_pipe_diag.py 3 > $O/cmc_diag.txt 2> $O/cmc_diag.err || { echo "diag failed"; tail -20 $O/cmc_diag.err; exit 1; }
      grep -v "^   oracle tracks" $O/cmc_diag.txt | head -60 ;;
    ab)
      timeout -k 10 300 python -u tools/split_ab.py --plan plans/s_640x512_i640_b8_fp32.json --plan-exact plans/exp/s_640x512_i640_b8_fp32_exact_r2.json > $O/split_ab.json 2> $O/split_ab.err || { echo "ab failed"; tail -20 $O/split_ab.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/split_ab.json')); print({k: d[k] for k in ('exact_total_us','split_total_us')}, json.dumps(d['accuracy']), d['split_vs_exact'])" ;;
    sweep)
      for D in ${SWEEP:-3 5 6}; do
        timeout -k 10 200 python -u bench.py --steps 100 --secondary none --no-cpu-baseline --no-profile --inflight $D > $O/bench_if$D.json 2> $O/bench_if$D.err || { echo "sweep $D failed"; tail -20 $O/bench_if$D.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/bench_if$D.json')); print('inflight $D', d['value'], d['ms_per_step'])"
      done ;;
    wg)
      for op in ${WG_OPS:-10 32 72}; do
        YK_FAST_TS=$op YK_DTYPE=fp32 YK_PLAN=plans/s_640x512_i640_b8_fp32.json timeout -k 10 120 python -u tools/wg_times.py > $O/wg_$op.txt 2> $O/wg_$op.err || { echo "wg $op failed"; tail -10 $O/wg_$op.err; exit 1; }
        cat $O/wg_$op.txt
      done ;;
    libab)
      # bench (fp32 headline, no bf16 leg) on each library variant in $LIBS (libyk*.so names in the package)
      for L in ${LIBS:-libyk.so}; do
        YK_LIB=$PWD/yolo---small-target-recognition---kalman-trajectory-prediction_amd/$L timeout -k 10 200 python -u bench.py --steps 100 --secondary none --no-cpu-baseline $BARGS --dump-ops $O/ops_$L.json > $O/bench_$L.json 2> $O/bench_$L.err || { echo "bench $L failed"; tail -20 $O/bench_$L.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
      done ;;
    graphkeep)
      timeout -k 10 120 tools/_graph_fork_repro keep 8 4 > $O/graph_keep.log 2>&1; rc=$?; tail -2 $O/graph_keep.log; [ $rc -eq 0 ] || { echo "graph repro keep rc=$rc"; exit 1; } ;;
    graphdestroy)
      timeout -k 10 120 tools/_graph_fork_repro destroy 8 4 > $O/graph_destroy.log 2>&1; rc=$?; tail -2 $O/graph_destroy.log; echo "graph repro destroy rc=$rc"; [ $rc -eq 0 ] || exit 1 ;;
    lanes)
      timeout -k 10 300 python -u tools/graph_lanes_repro.py alive > $O/graph_lanes.log 2>&1 || { echo "graph_lanes_repro failed"; tail -20 $O/graph_lanes.log; exit 1; }
      tail -2 $O/graph_lanes.log ;;
    stepdiff)
      timeout -k 10 600 python -u tools/gmd_step_diff.py --inflight ${SD_INFLIGHT:-6} --reps ${SD_REPS:-10} > $O/stepdiff.log 2>&1 || { echo "stepdiff failed"; tail -20 $O/stepdiff.log; exit 1; }
      tail -15 $O/stepdiff.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
      tail -3 $O/smoke.txt ;;
    c4plan)
      timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --steps 100 --plan-out $O/plan_c4.json > $O/bench_c4.json 2> $O/bench_c4.err || { echo "c4 failed"; tail -20 $O/bench_c4.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['config']['conv_plan'])" ;;
    c4tune)
      # config 4 (one stream per GPU): concurrent autotune at batch $TUNE_BATCH (default 4 = four forwards of
      # batch 1 in flight) over every kernel kind, then config-4 benches on the committed and the tuned plan
      timeout -k 10 600 python -u tools/tune_concurrent.py --dtype fp32 --streams 1 --tune-batch ${TUNE_BATCH:-4} --out $O/plan_c4_tuned.json > $O/tune_c4.log 2>&1 || { echo "tune c4 failed"; tail -20 $O/tune_c4.log; exit 1; }
      for P in plans/s_640x512_i640_b1_fp32.json $O/plan_c4_tuned.json; do
        timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --steps 200 --plan-in $P > $O/bench_c4_$(basename $P) 2> $O/bench_c4.err || { echo "c4 bench failed"; tail -20 $O/bench_c4.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/bench_c4_$(basename $P)')); print('c4', '$P', d['value'], d['ms_per_step'], d['roofline']['kernel'])"
      done ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
done
