#!/bin/bash
# SQ / TA counters of the fp32 headline's conv kernels (one counter block per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${PMC_DIR:-pmcsq}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o -E "\b(SQ|TA|TD|TCP)_[A-Z0-9_]+" $O/counters.txt | sort -u > $O/counter_names.txt || true
B="bench.py --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline --no-profile ${BENCH_EXTRA:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU --output-format csv -d $O/p1 -o run -- python3 -u $B > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d $O/p2 -o run -- python3 -u $B > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; echo "p2 failed"; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/p3 -o run -- python3 -u $B > /dev/null 2> $O/p3.err || { tail -5 $O/p3.err; echo "p3 failed"; }
python3 tools/pmc_kernels.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv $O/p3/run_counter_collection.csv > $O/summary.txt
rm -f $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv $O/p3/run_counter_collection.csv
cat $O/summary.txt | head -60
