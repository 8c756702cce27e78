#!/bin/bash
# two-launch tracker step: parity tests, then phases on config 3 / 5 (split vs single workgroup)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/trk2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tracker_gpu.py tests/test_cmc_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/trk_phases.py --config 3 > $O/c3.txt 2>&1 || { echo "c3 failed"; tail -20 $O/c3.txt; exit 1; }
grep -v amdgpu $O/c3.txt | head -3; tail -3 $O/c3.txt
tail -2 $O/tests.log
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/trk_phases.py --config 5 > $O/c5.txt 2>&1 || { echo "c5 failed"; tail -20 $O/c5.txt; exit 1; }
grep -v amdgpu $O/c5.txt | head -3; tail -3 $O/c5.txt
tail -2 $O/tests.log
tail -2 $O/tests.log
