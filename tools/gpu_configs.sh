#!/bin/bash
# Bench lines for the BASELINE configs other than the default (config 3), plus the host CPU
# description BENCH.md records next to the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/configs
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1; python3 -c "import os; print('os.cpu_count', os.cpu_count())" >> $O/lscpu.txt
for c in ${CONFIGS:-2 5}; do
  timeout -k 10 400 python -u bench.py --config $c ${BENCH_ARGS:-} > $O/config$c.json 2> $O/config$c.err || { echo "config $c failed"; tail -30 $O/config$c.err; exit 1; }
  cat $O/config$c.json
done
