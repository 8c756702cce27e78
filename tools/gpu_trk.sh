#!/bin/bash
# tracker step phases on the config-3 and config-5 workloads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/trk
mkdir -p $O
timeout -k 10 300 python -u tools/trk_phases.py --config 3 > $O/c3.txt 2>&1 || { echo "c3 failed"; tail -20 $O/c3.txt; exit 1; }
cat $O/c3.txt
timeout -k 10 400 python -u tools/trk_phases.py --config 5 --frames 200 > $O/c5.txt 2>&1 || { echo "c5 failed"; tail -20 $O/c5.txt; exit 1; }
cat $O/c5.txt
