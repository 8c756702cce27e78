#!/bin/bash
# Round-2 re-entry check at HEAD: whole GPU suite, smoke, default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 400 python -u bench.py --dump-ops $O/ops.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
