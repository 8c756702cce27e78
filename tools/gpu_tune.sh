#!/bin/bash
# A/B: bench with the committed plan vs a plan tuned at batch TB (in-flight proxy), dtype DT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/tune_${DT:-fp32}
mkdir -p $O
DTY=${DT:-fp32}
PLAN=plans/s_640x512_i640_b8_${DTY}.json
timeout -k 10 300 python -u tools/tune_concurrent.py --dtype $DTY --tune-batch ${TB:-16} --out $O/plan_conc.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
for i in 1 2; do
timeout -k 10 200 python -u bench.py --dtype $DTY --secondary none --no-cpu-baseline --plan-in $PLAN > $O/bench_iso_$i.json 2> $O/bench_iso.err || { tail -20 $O/bench_iso.err; exit 1; }
timeout -k 10 200 python -u bench.py --dtype $DTY --secondary none --no-cpu-baseline --plan-in $O/plan_conc.json --dump-ops $O/ops_conc.json > $O/bench_conc_$i.json 2> $O/bench_conc.err || { tail -20 $O/bench_conc.err; exit 1; }
done
python3 - <<PY
import json
for n in ("iso_1", "conc_1", "iso_2", "conc_2"):
    d = json.load(open(f"$O/bench_{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["network_mfma_frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
PY
