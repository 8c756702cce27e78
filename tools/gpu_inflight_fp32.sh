#!/bin/bash
# fp32 headline leg at several detector forwards in flight (committed plan, no CPU baseline / profile).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/infl
mkdir -p $O
for rep in 1 2; do
for d in ${DEPTHS:-2 3 4 5 6}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-profile --secondary none --inflight $d > $O/b$d.json 2> $O/b$d.err || { echo "bench inflight $d failed"; tail -20 $O/b$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$d.json'));print('inflight $d', d['value'], d['ms_per_step'])"
done
done
