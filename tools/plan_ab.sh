#!/bin/bash
# fp32 headline A/B of two conv plans on one box, alternating A B A B A B (bench.py --plan-in).
# usage: PLAN_A=... PLAN_B=... OUT_DIR=... bash tools/plan_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT_DIR:-r4planab}
mkdir -p $O
for i in 1 2 3; do
  for P in A B; do
    F=$([ $P = A ] && echo $PLAN_A || echo $PLAN_B)
    timeout -k 10 300 python -u bench.py --plan-in $F --secondary none --no-cpu-baseline --no-profile > $O/$P$i.json 2> $O/$P$i.err || { echo "bench $P$i failed"; tail -20 $O/$P$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$P$i.json')); print('$P$i', d['value'])"
  done
done
