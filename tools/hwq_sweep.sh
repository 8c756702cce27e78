#!/bin/bash
# Hardware-queue sweep: bench lines at GPU_MAX_HW_QUEUES = 4 (HIP's default) / 8 / 16 and several
# forwards in flight.  With D detector streams plus the tracker stream, D + 1 > 4 streams share
# four hardware queues and the work of two streams on one queue runs in submission order.
# OUT_DIR under gpurun_out/; CASES = "Q:D:dtype[:cmc]" list.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT_DIR:-r4hwq}
mkdir -p $O
for C in ${CASES:-4:4:fp32 8:4:fp32 4:4:fp32 8:4:fp32 8:6:fp32 16:6:fp32}; do
  IFS=: read Q D T X <<< "$C"
  A="--dtype $T --inflight $D --secondary none --no-cpu-baseline --no-profile"
  [ "$X" = cmc ] && A="$A --tracker motion_reset --gmd"
  N=$O/bench_q${Q}_d${D}_${T}${X:+_$X}
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u bench.py $A >> $N.json 2>> $N.err || { echo "bench $C failed"; tail -20 $N.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$N.json').read().strip().splitlines()[-1]); print('$C', d['value'], d['ms_per_step'])"
done
