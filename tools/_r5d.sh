set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=yolo---small-target-recognition---kalman-trajectory-prediction_amd
O=gpurun_out/r5d; mkdir -p $O
YK_LIB=$PWD/$P/libyk_lkD.so timeout -k 10 300 python -u tools/gmd_step_diff.py --inflight 6 --reps 4 > $O/sd_D.log 2>&1 || { echo D failed; tail $O/sd_D.log; exit 1; }
grep -E "lk diag|runs differ" $O/sd_D.log | head -40
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tr -o run -- python3 -u bench.py --secondary none --no-cpu-baseline --no-profile --io both --steps 30 --warmup 5 --preroll 20 > $O/bench_tr.json 2> $O/bench_tr.err || { echo trace failed; tail $O/bench_tr.err; exit 1; }
ls $O/tr
head -5 $O/tr/run_memory_copy_stats.csv 2>/dev/null
