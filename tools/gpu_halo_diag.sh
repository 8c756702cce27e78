# halo-tile split conv: per-op variant sweep on the product library and the YK_HALO_DIAG builds
# (1 no weight loads, 2 no staging, 4 no LDS operand reads)
set -o pipefail
O=gpurun_out/halodiag; mkdir -p $O
P=${PLAN:-plans/exp/s_640x512_i640_b8_fp32_r3h.json}
OPS=${OPS:-72,73,76,80,30}
for v in "" 1 2 4; do
  L=yolo---small-target-recognition---kalman-trajectory-prediction_amd/libyk${v:+_hd$v}.so
  [ -f "$L" ] || continue
  YK_LIB=$PWD/$L timeout -k 10 200 python -u tools/halo_probe.py --plan $P --ops $OPS > $O/probe$v.log 2> $O/probe$v.err || { tail -20 $O/probe$v.err; exit 1; }
  echo "== $v"; grep -v "^{" $O/probe$v.log
done
