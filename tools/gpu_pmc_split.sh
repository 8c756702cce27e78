#!/bin/bash
# PMC passes over the F32S (split) conv kernels of the fp32 headline, on the product library and
# on the YK_DIAG=3 build (csrc/build.py YK_DEFINES=-DYK_DIAG=3 YK_OUT=...libyk_diag3.so: no split VALU, no weight loads): where the split kernel's time goes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${PMC_DIR:-pmcsplit}
mkdir -p $O
P=${PLAN:-plans/exp/s_640x512_i640_b8_fp32_split_r3c.json}
B="bench.py --steps 5 --warmup 2 --preroll 4 --secondary none --no-cpu-baseline --no-profile --plan-in $P"
L=yolo---small-target-recognition---kalman-trajectory-prediction_amd
for v in "" 3; do
  export YK_LIB=$PWD/$L/libyk${v:+_diag$v}.so
  D=$O/v$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $D/p1 -o run -- python3 -u $B > /dev/null 2> $D.p1.err || { tail -5 $D.p1.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM --output-format csv -d $D/p2 -o run -- python3 -u $B > /dev/null 2> $D.p2.err || { tail -5 $D.p2.err; exit 1; }
  python3 tools/pmc_kernels.py $D/p1/run_counter_collection.csv $D/p2/run_counter_collection.csv > $D.summary.txt
  rm -rf $D/p1 $D/p2
  head -8 $D.summary.txt
done
