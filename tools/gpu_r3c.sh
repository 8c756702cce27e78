set -o pipefail
O=gpurun_out/${OUT_DIR:-r3c}; mkdir -p $O
timeout -k 10 400 python -u tools/tune_concurrent.py --dtype fp32 --out $O/plan_split.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
[ -n "${SKIP_BASE:-}" ] || { timeout -k 10 300 python -u bench.py --steps 100 --secondary none --no-cpu-baseline --dump-ops $O/ops_base.json > $O/bench_base.json 2> $O/bench_base.err || { tail -20 $O/bench_base.err; exit 1; }; }
timeout -k 10 300 python -u bench.py --steps 100 --secondary none --no-cpu-baseline --plan-in $O/plan_split.json --dump-ops $O/ops_split.json > $O/bench_split.json 2> $O/bench_split.err || { tail -20 $O/bench_split.err; exit 1; }
python3 -c "
import json
for n in ('base','split'):
  try:
    d=json.load(open('$O/bench_'+n+'.json')); print(n, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])
  except Exception as e: print(n, e)
"
