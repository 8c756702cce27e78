set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=yolo---small-target-recognition---kalman-trajectory-prediction_amd
O=gpurun_out/r5c; mkdir -p $O
YK_LIB=$PWD/$P/libyk_lkC.so timeout -k 10 300 python -u tools/gmd_step_diff.py --inflight 6 --reps 6 > $O/sd_C.log 2>&1 || { echo C failed; tail $O/sd_C.log; exit 1; }
grep -E "mismatch|runs differ" $O/sd_C.log
for io in none h2d d2h both; do
  timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-profile --io $io > $O/bench_$io.json 2> $O/bench_$io.err || { echo bench $io failed; tail $O/bench_$io.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$io.json')); print('$io', d['value'], d['hbm_resident_fps'], d['ms_per_step'])"
done
