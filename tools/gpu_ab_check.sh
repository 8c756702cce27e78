#!/bin/bash
# Conv parity tests on the new build, then an A/B of scratch/libyk_old.so vs the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_detector_gpu.py tests/test_detector_fp8_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
BENCH_ARGS="${BENCH_ARGS:---secondary none}" bash tools/ab_lib.sh
