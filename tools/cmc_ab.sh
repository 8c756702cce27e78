#!/bin/bash
# CMC line against the plain line in one GPU call: bf16 plain and bf16 CMC (motion-reset tracker +
# global motion detector) bench lines.  OUT_DIR under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT_DIR:-r4cmc}
mkdir -p $O
for V in plain cmc; do
  A="--dtype ${DTYPE:-bf16} --secondary none --no-cpu-baseline"
  [ $V = cmc ] && A="$A --tracker motion_reset --gmd"
  timeout -k 10 300 python -u bench.py $A > $O/bench_$V.json 2> $O/bench_$V.err || { echo "bench $V failed"; tail -20 $O/bench_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$V.json')); print('$V', d['value'], d['ms_per_step'])"
done
