#!/bin/bash
# Bench lines: config 3 with the motion-reset tracker (+ CPU baseline), config 5 (fp8) and config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 300 python -u bench.py --tracker motion_reset > $O/cmc.json 2> $O/cmc.err || { tail -20 $O/cmc.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cmc.json'));print('cmc', d['value'], d['ms_per_step'], d['config']['live_tracks_per_stream'], d['cpu_baseline'])"
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['network_mfma_frac'])"
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c2.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
