#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) vs detector forwards in flight:
# each StreamPipeline uses D detector streams + a tracker stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/hwq
mkdir -p $O
for q in 4 8 16; do
  for d in 4 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-profile --inflight $d > $O/q${q}_d$d.json 2> $O/q${q}_d$d.err || { tail -5 $O/q${q}_d$d.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/q${q}_d$d.json'));print('hwq $q inflight $d fp32', d['value'], 'bf16 sec', d['secondary'][0]['value'])"
  done
done
