#!/bin/bash
# Config 5 (1280x1024 at imgsz 1280): plans tuned at batch TB (in-flight proxy) for fp8 and bf16,
# A/B against the committed plans on the bench's config-5 legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/tune_c5
mkdir -p $O
for DTY in fp8 bf16; do
  timeout -k 10 400 python -u tools/tune_concurrent.py --dtype $DTY --hw 1024x1280 --imgsz 1280 --targets 96 --tune-batch ${TB:-16} --out $O/plan_$DTY.json > $O/tune_$DTY.log 2>&1 || { tail -20 $O/tune_$DTY.log; exit 1; }
done
for i in 1 2; do
  for DTY in fp8 bf16; do
    timeout -k 10 300 python -u bench.py --config 5 --dtype $DTY --secondary none --no-cpu-baseline --no-profile > $O/old_${DTY}_$i.json 2> $O/old.err || { tail -20 $O/old.err; exit 1; }
    timeout -k 10 300 python -u bench.py --config 5 --dtype $DTY --secondary none --no-cpu-baseline --no-profile --plan-in $O/plan_$DTY.json > $O/new_${DTY}_$i.json 2> $O/new.err || { tail -20 $O/new.err; exit 1; }
    python3 -c "import json;a=json.load(open('$O/old_${DTY}_$i.json'));b=json.load(open('$O/new_${DTY}_$i.json'));print('$DTY', 'old', a['value'], 'new', b['value'])"
  done
done
