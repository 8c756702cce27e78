set -o pipefail
O=gpurun_out/r3h; mkdir -p $O
export YK_LIB=$PWD/yolo---small-target-recognition---kalman-trajectory-prediction_amd/libyk_fastsilu.so
timeout -k 10 300 python -u tools/split_ab.py --plan plans/s_640x512_i640_b8_fp32.json --plan-exact plans/exp/s_640x512_i640_b8_fp32_exact_r2.json > $O/split_ab_fastsilu.json 2> $O/split_ab.err || { tail -20 $O/split_ab.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/split_ab_fastsilu.json')); print(json.dumps(d['accuracy']))"
timeout -k 10 900 python -u -m pytest tests/test_bench_pipeline_gpu.py -k fp32 -v -rP --timeout 800 --timeout-method thread > $O/chain_fastsilu.log 2>&1 || { grep -E "FAILED|Error|assert" $O/chain_fastsilu.log | head -20; exit 1; }
grep -E "passed|BENCH_PIPELINE" $O/chain_fastsilu.log | cut -c1-400
