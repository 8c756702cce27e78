#!/bin/bash
# CMC line A/B in one GPU call: bf16 plain and bf16 CMC (motion-reset + GMD) bench lines with the
# tracker stream at default and at high priority (YK_TRK_PRIORITY).  OUT_DIR under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT_DIR:-r4cmc}
mkdir -p $O
for P in 0 1; do
  for V in plain cmc; do
    A="--dtype bf16 --secondary none --no-cpu-baseline"
    [ $V = cmc ] && A="$A --tracker motion_reset --gmd"
    YK_TRK_PRIORITY=$P timeout -k 10 300 python -u bench.py $A > $O/bench_${V}_p$P.json 2> $O/bench_${V}_p$P.err || { echo "bench $V p$P failed"; tail -20 $O/bench_${V}_p$P.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${V}_p$P.json')); print('$V prio=$P', d['value'], d['ms_per_step'])"
  done
done
