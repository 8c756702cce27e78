#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sched
for g in "1 3" "2 1" "2 3" "4 1"; do
  set -- $g
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --groups $1 --lanes $2 > gpurun_out/sched/b_$1_$2.json 2> gpurun_out/sched/b_$1_$2.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sched/b_$1_$2.json'));print('groups $1 lanes $2', d['value'], d['ms_per_step'])"
done
