#!/bin/bash
# New golden GPU tests (global motion, ByteTrack) + the camera-motion-compensation variant bench
# + the global-motion detector rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_golden_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for d in fp32 bf16; do
  timeout -k 10 300 python -u bench.py --tracker motion_reset --gmd --dtype $d --secondary none > $O/b_$d.json 2> $O/b_$d.err || { tail -20 $O/b_$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$d.json'));print('$d', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python -u tools/gmd_bench.py > $O/gmd.txt 2>&1 || { tail -5 $O/gmd.txt; exit 1; }
tail -2 $O/gmd.txt | cut -c1-300
