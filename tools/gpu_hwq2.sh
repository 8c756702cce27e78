#!/bin/bash
# Fewer hardware queues per process vs detector forwards in flight (fp32 headline leg only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/hwq2
mkdir -p $O
for q in 1 2 3 4; do
  for d in 2 4 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-profile --secondary none --inflight $d > $O/q${q}_d$d.json 2> $O/q${q}_d$d.err || { tail -5 $O/q${q}_d$d.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/q${q}_d$d.json'));print('hwq $q inflight $d fp32', d['value'])"
  done
done
