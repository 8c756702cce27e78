#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bt
timeout -k 10 300 python -u tools/bt_bench.py > gpurun_out/bt/bench.json 2> gpurun_out/bt/bench.err || { tail -20 gpurun_out/bt/bench.err; exit 1; }
cat gpurun_out/bt/bench.json
