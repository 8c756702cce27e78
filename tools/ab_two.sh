#!/bin/bash
# A/B of scratch/libyk_old.so vs scratch/libyk_new.so (bench lines only, alternating).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab2
mkdir -p $O
for rep in 1 2 3; do
  for v in old new; do
    YK_LIB=$PWD/scratch/libyk_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --dump-ops $O/ops_$v.json ${BENCH_ARGS:---secondary none} > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_$v.json'));o=json.load(open('$O/ops_$v.json'))['ops'];print('$v', d['value'], d['ms_per_step'], 'opsum', round(sum(x['us'] for x in o),1))"
  done
done
