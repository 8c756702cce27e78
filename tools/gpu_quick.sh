#!/bin/bash
# Parity suite subset + one bench line with per-op times (iteration loop on the GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_detector_gpu.py} ${TESTK:+-k "$TESTK"} -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dump-ops $O/ops.json ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'])"
python3 -c "
import json;d=json.load(open('$O/ops.json'))['ops']
print('sum', round(sum(o['us'] for o in d),1)); [print(o['op'], o['kernel'][:40], o['us']) for o in d if o['kind'] != 1]"
