#!/bin/bash
# The round's secondary bench lines in one GPU call: BASELINE configs 2, 4 (per-rank leg), 5, the CMC
# variant (fp32 and bf16) and the drop-in driver loop (tools/dropin_bench.py).  OUT_DIR under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT_DIR:-r4lines}
mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python -u "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -20 $O/$n.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d.get('value'), d.get('ms_per_step', d.get('ms_per_frame')))"; }
run c2 bench.py --config 2 --no-cpu-baseline
run c4 bench.py --config 4 --no-cpu-baseline
run c5 bench.py --config 5 --no-cpu-baseline
run cmc_fp32 bench.py --tracker motion_reset --gmd --secondary none --no-cpu-baseline
run cmc_bf16 bench.py --tracker motion_reset --gmd --dtype bf16 --secondary none --no-cpu-baseline
run dropin tools/dropin_bench.py --frames 300
