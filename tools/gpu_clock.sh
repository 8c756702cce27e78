#!/bin/bash
# Effective shader clock per conv kernel (GRBM_GUI_ACTIVE / 8 / kernel duration; one counter pass
# with the kernel trace) on the fp32 headline's per-op profile pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/clock
mkdir -p $O
B="bench.py --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/p -o run -- python3 -u $B > /dev/null 2> $O/p.err || { tail -5 $O/p.err; exit 1; }
python3 tools/clock_summary.py $O/p > $O/summary.txt
rm -f $O/p/*counter_collection.csv $O/p/*kernel_trace.csv
cat $O/summary.txt | head -40
