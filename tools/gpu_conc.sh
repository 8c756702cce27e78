#!/bin/bash
# Kernel-trace of bench with batch groups (concurrency check between independent chains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/conc
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/g2 -o run -- python3 -u bench.py --groups 2 --lanes 1 --steps 30 --warmup 5 --no-cpu-baseline --no-profile --no-tune > $O/g2.json 2> $O/g2.err || { tail -20 $O/g2.err; exit 1; }
python3 - <<'PY'
import csv
rows=[]
for x in csv.DictReader(open('gpurun_out/conc/g2/run_kernel_trace.csv')):
    if 'yk::' in x['Kernel_Name'] or 'nms_kernel' in x['Kernel_Name']:
        rows.append((int(x['Start_Timestamp']), int(x['End_Timestamp']), x['Kernel_Name'][:50], x.get('Queue_Id', x.get('Stream_Id','?'))))
rows.sort()
# take a window in the last third
seg = rows[len(rows)*2//3: len(rows)*2//3 + 200]
t0 = seg[0][0]
for r in seg[:120]:
    print((r[0]-t0)//1000, (r[1]-t0)//1000, r[3], r[2])
PY
