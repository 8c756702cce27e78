set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_detector_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
for v in 1 0 1; do
  YK_XCD=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --dump-ops gpurun_out/ab/ops_xcd$v.json > gpurun_out/ab/b$v.json 2> gpurun_out/ab/b$v.err || { tail -20 gpurun_out/ab/b$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab/b$v.json'));print('xcd $v', d['value'], d['ms_per_step'])"
done
