#!/bin/bash
# device ByteTrack / BoT-SORT parity against the oracle
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/bt
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bytetrack_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -40 $O/tests.log
exit $rc
