#!/bin/bash
# inflight=2 check: pipeline parity tests, bench with 1 vs 2 detector graphs in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/inf
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in ${ARGSETS:-"--inflight 1" "--inflight 2" "--inflight 3" "--inflight 4"}; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-profile $args > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$n.json'));print('$args', d['value'], d['ms_per_step'], d['config']['live_tracks_per_stream'])"
done
