set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=yolo---small-target-recognition---kalman-trajectory-prediction_amd
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u tools/gmd_step_diff.py --inflight 6 --reps 10 > $O/sd_prod.log 2>&1 || { echo prod failed; tail $O/sd_prod.log; exit 1; }
tail -1 $O/sd_prod.log
YK_LIB=$PWD/$P/libyk_lkA.so timeout -k 10 300 python -u tools/gmd_step_diff.py --inflight 6 --reps 10 > $O/sd_A.log 2>&1 || { echo A failed; tail $O/sd_A.log; exit 1; }
tail -1 $O/sd_A.log
YK_LIB=$PWD/$P/libyk_lkB.so timeout -k 10 300 python -u tools/gmd_step_diff.py --inflight 6 --reps 10 > $O/sd_B.log 2>&1 || { echo B failed; tail $O/sd_B.log; exit 1; }
tail -1 $O/sd_B.log
timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('graph', d['value'], d['hbm_resident_fps'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-graph --no-profile > $O/bench_ng.json 2> $O/bench_ng.err || { echo bench ng failed; tail $O/bench_ng.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_ng.json')); print('nograph', d['value'], d['hbm_resident_fps'], d['ms_per_step'])"
timeout -k 10 300 python -u tools/op_sweep.py --ops 3,10,22,32 --batch 8 > $O/op_sweep.json 2> $O/op_sweep.err || { echo sweep failed; tail $O/op_sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/op_sweep.json'):
    d=json.loads(l); print({k:(v if not isinstance(v,list) else v[:6]) for k,v in d.items()})
"
timeout -k 10 600 python -u -m pytest tests/test_detector_gpu.py tests/test_predictor_gpu.py tests/test_gmc_gpu.py -x -v --timeout 200 --timeout-method thread -k "fp16 or predict or gmc" > $O/pytest_fp16.log 2>&1 || { echo pytest fp16 failed; grep -E "FAILED|Error|assert" $O/pytest_fp16.log | head -20; exit 1; }
tail -2 $O/pytest_fp16.log
