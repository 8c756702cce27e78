# split-kernel bottleneck diagnostics: exact vs split A/B on the product library and on the
# YK_SPLIT_DIAG builds (1 no split VALU, 2 no weight loads, 3 neither)
set -o pipefail
O=gpurun_out/diag; mkdir -p $O
P=${PLAN:-plans/exp/s_640x512_i640_b8_fp32_split_r3c.json}
for v in "" 1 2 3; do
  L=yolo---small-target-recognition---kalman-trajectory-prediction_amd/libyk${v:+_diag$v}.so
  YK_LIB=$PWD/$L timeout -k 10 240 python -u tools/split_ab.py --plan $P > $O/ab$v.json 2> $O/ab$v.err || { tail -20 $O/ab$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab$v.json'));print('$v',d['exact_total_us'],d['split_total_us'],d['exact_conv_us'],d['split_conv_us'])"
done
