#!/bin/bash
# A/B of two libyk.so builds on one box: per-op sums and bench lines, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab
mkdir -p $O
NEW=yolo---small-target-recognition---kalman-trajectory-prediction_amd/libyk.so
for rep in 1 2; do
  for v in old new; do
    L=$([ $v = old ] && echo scratch/libyk_old.so || echo $NEW)
    YK_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --dump-ops $O/ops_$v.json ${BENCH_ARGS:-} > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_$v.json'));o=json.load(open('$O/ops_$v.json'))['ops'];print('$v', d['value'], d['ms_per_step'], 'opsum', round(sum(x['us'] for x in o),1))"
  done
done
